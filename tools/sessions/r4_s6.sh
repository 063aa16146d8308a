#!/bin/bash
# Round 4, session 6: split-plan tile size A/B (plan_probe: 8/4/2/1 buffers
# per thread), then session 2's inflate measurements: f4 at the call site
# (preloadram_now loop on deflated entries: zlib + reference CRC vs drop-in
# vs GPU inflate, same run), the single-entry inflate bench, and the
# split-borrow worktree (ablibs/borrow) validated and timed beside it.
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r4s6; mkdir -p $O
fault_stop() { if grep -qi "illegal\|memory access fault\|Aborted\|core dumped" "$O/$1"; then echo "fault in $1: stopping" >> $O/steps.txt; exit 9; fi; }
step() {
  local log=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$log 2>&1
  local rc=$?
  echo "$log rc=$rc" >> $O/steps.txt
  if [ $rc -ge 124 ]; then echo "stopping after $log (rc $rc)" >> $O/steps.txt; exit $rc; fi
  fault_stop $log
  return 0
}
step plan_c4.jsonl 60 tools/plan_probe 100000 0 50 3
step plan_z1m.jsonl 60 tools/plan_probe 1000000 0 50 2
step plan_u16k.jsonl 60 tools/plan_probe 65536 16384 50 2
step plan_big4m.jsonl 60 tools/plan_probe 4200000 0 20 2
PYT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
step preload_inflate.jsonl 600 python3 tools/bench_preload_inflate.py --sizes 1,16,64,256 --reps 3
step bench_one_main.jsonl 300 python3 tools/bench_inflate_one.py --sizes 1,4,16,64 --reps 5 --no-serial
cd ablibs/borrow
step borrow_pytest_split.log 500 $PYT tests/test_gpu_inflate_split.py
step bench_one_borrow.jsonl 300 python3 tools/bench_inflate_one.py --sizes 1,4,16,64 --reps 5 --no-serial
