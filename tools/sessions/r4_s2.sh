#!/bin/bash
# Round 4, session 2: f4 at the call site (the preloadram_now loop on
# deflated entries: zlib + reference CRC vs drop-in vs GPU inflate, same
# run), the single-entry inflate bench, and split-borrow (worktree
# ablibs/borrow) validated and timed beside it.
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r4s2; mkdir -p $O
step() {
  local log=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$log 2>&1
  local rc=$?
  echo "$log rc=$rc" >> $O/steps.txt
  if [ $rc -ge 124 ]; then echo "stopping after $log (rc $rc)" >> $O/steps.txt; exit $rc; fi
  return 0
}
PYT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
step preload_inflate.jsonl 600 python3 tools/bench_preload_inflate.py --sizes 1,16,64,256 --reps 3
step bench_one_main.jsonl 300 python3 tools/bench_inflate_one.py --sizes 1,4,16,64 --reps 5 --no-serial
cd ablibs/borrow
step borrow_pytest_split.log 500 $PYT tests/test_gpu_inflate_split.py
step bench_one_borrow.jsonl 300 python3 tools/bench_inflate_one.py --sizes 1,4,16,64 --reps 5 --no-serial
