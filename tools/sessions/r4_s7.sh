#!/bin/bash
# Round 4, session 7: split-plan tiles by batch size, the ZCRC_DYN_TAIL knob
# and the merged split-borrow inflate -- focused GPU tests, then the full
# suite; c4_probe (tail half units), c2_probe (per-buffer priorities by
# progress / none).  Stops at the first sign of a fault.
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r4s7; mkdir -p $O
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
step pytest_focus.log 600 $PYT tests/test_gpu_small_kernel.py tests/test_gpu_inflate_split.py tests/test_gpu_parity.py -k "split_plan or config4 or dynamic_part or inflate or per_buffer or fused"
step c4_probe.txt 240 tools/c4_probe 4 20
step c2_probe.txt 120 tools/c2_probe 48
step pytest_gpu.log 900 $PYT tests -m gpu
