#!/bin/bash
# Round 4, session 3: the small body's x^-8 byte table and the split plan's
# direct mode (parity, then small device batches A/B: the build before both,
# ablibs/pre; this build with ZCRC_SMALL_DIRECT=0; this build, interleaved).
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r4s3; mkdir -p $O
step() {
  local log=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$log 2>&1
  local rc=$?
  echo "$log rc=$rc" >> $O/steps.txt
  if [ $rc -ge 124 ]; then echo "stopping after $log (rc $rc)" >> $O/steps.txt; exit $rc; fi
  return 0
}
PYT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
step pytest_small.log 600 $PYT tests/test_gpu_small_kernel.py tests/test_gpu_parity.py
for r in 1 2; do
  step small_pre_$r.jsonl 300 python3 tools/run_with_lib.py ablibs/pre/zipsfs_amd/libzcrc.so tools/small_batches.py 10 1024,2048,3000,4096
  step small_nodirect_$r.jsonl 300 env ZCRC_SMALL_DIRECT=0 python3 tools/small_batches.py 10 1024,2048,3000,4096
  step small_new_$r.jsonl 300 python3 tools/small_batches.py 10 1024,2048,3000,4096
done
