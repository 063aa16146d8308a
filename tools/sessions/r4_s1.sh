#!/bin/bash
# Round 4, session 1: the multi-device host path (ZCRC_DEVICES=0,0), the sp16
# near-ring inflate test, the deflated preload modes, then
# the whole GPU suite, smoke and the default bench; split-borrow (worktree
# ablibs/borrow) validated and timed beside main.
# A step that fails a test goes on; a fault, abort or time limit ends the call.
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r4s1; mkdir -p $O
step() {  # step <log> <seconds> cmd...
  local log=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$log 2>&1
  local rc=$?
  echo "$log rc=$rc" >> $O/steps.txt
  if [ $rc -ge 124 ]; then echo "stopping after $log (rc $rc)" >> $O/steps.txt; exit $rc; fi
  return 0
}
PYT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
step pytest_new.log 600 $PYT tests/test_gpu_multidevice.py tests/test_gpu_inflate_split.py tests/test_gpu_preload.py -k "multidevice or logical or bad_device or sp16 or deflated"
step pytest_gpu.log 900 $PYT tests -m gpu
step smoke.log 120 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench_default.jsonl 400 python3 bench.py
step preload_inflate.jsonl 600 python3 tools/bench_preload_inflate.py --sizes 1,16,64,256 --reps 3
step bench_one_main.jsonl 300 python3 tools/bench_inflate_one.py --sizes 1,4,16,64 --reps 5 --no-serial
cd ablibs/borrow
step borrow_pytest_split.log 500 $PYT tests/test_gpu_inflate_split.py
step bench_one_borrow.jsonl 300 python3 tools/bench_inflate_one.py --sizes 1,4,16,64 --reps 5 --no-serial
