#!/bin/bash
# Round 4, session 12: the split plan's small-list workgroups join the batch
# kernel's dynamic part once their list is done.  Focused GPU tests (join and
# not), c4_probe (join / no join / small-list weights), the bench line
# without the CPU baseline, then the full suite.
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r4s12; mkdir -p $O
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
step pytest_focus.log 600 $PYT tests/test_gpu_parity.py tests/test_gpu_small_kernel.py -k "config4 or dynamic_part or split_plan or mixed or random or concurrent or graph"
step c4_probe.txt 300 tools/c4_probe 4 20
step bench_nocpu.jsonl 300 python3 bench.py --no-cpu-baseline
step c4_probe_after.txt 200 tools/c4_probe 2 20
step pytest_gpu.log 900 $PYT tests -m gpu
