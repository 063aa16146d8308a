#!/bin/bash
# Round 4, session 10: the three-input-xor braid step (bitop3, two-word
# stream state) in the batch kernel and the small body, grain-table split
# shifts, per-buffer form 15.  Focused GPU tests; c4_probe (old shift A/B)
# and c2_probe; bench (no CPU baseline) and small batches, new library
# against the pre-bitop3 build (ablibs/prebit), interleaved; the full suite.
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r4s10; mkdir -p $O
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
step pytest_focus.log 600 $PYT tests/test_gpu_parity.py tests/test_gpu_small_kernel.py -k "single_large or dynamic_part or config4 or config2 or config1 or per_buffer or fused or split_plan or beyond or lengths or small"
step c4_probe.txt 300 tools/c4_probe 4 20
step c2_probe.txt 120 tools/c2_probe 48
for r in 1 2; do
  step bench_new_$r.jsonl 300 python3 bench.py --no-cpu-baseline
  step bench_prebit_$r.jsonl 300 python3 tools/run_with_lib.py ablibs/prebit/zipsfs_amd/libzcrc.so bench.py --no-cpu-baseline
  step small_new_$r.jsonl 300 python3 tools/small_batches.py 10 1024,4096,8192
  step small_prebit_$r.jsonl 300 python3 tools/run_with_lib.py ablibs/prebit/zipsfs_amd/libzcrc.so tools/small_batches.py 10 1024,4096,8192
done
step pytest_gpu.log 900 $PYT tests -m gpu
