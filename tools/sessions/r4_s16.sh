#!/bin/bash
# Round 4, session 16: every workgroup takes its share of the split plan's
# small list first (ZCRC_AB_FLAGS=16, A/B): parity with it on, c4_probe, the
# bench line with and without, interleaved.
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r4s16; mkdir -p $O
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
PYT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
step pytest_spread.log 600 env ZCRC_AB_FLAGS=16 $PYT tests/test_gpu_parity.py tests/test_gpu_small_kernel.py -k "config4 or dynamic_part or split_plan or mixed or random"
step c4_probe.txt 300 tools/c4_probe 4 20
for r in 1 2; do
  step bench_base_$r.jsonl 300 python3 bench.py --no-cpu-baseline
  step bench_spread_$r.jsonl 300 env ZCRC_AB_FLAGS=16 python3 bench.py --no-cpu-baseline
done
