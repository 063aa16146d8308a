#!/bin/bash
# Round 4, session 1: the multi-device host path (ZCRC_DEVICES=0,0), the sp16
# near-ring inflate test, the per-buffer round-4 form and
# the medium-before-big split plan (parity, then same-box A/B: c2_probe for
# config 2, ZCRC_BIG_MIN for config 4), the whole GPU suite, smoke and the
# default bench.  A step that fails a test goes on; a fault, abort or time
# limit ends the call.
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
step pytest_new.log 600 $PYT tests/test_gpu_multidevice.py tests/test_gpu_inflate_split.py tests/test_gpu_preload.py tests/test_gpu_parity.py tests/test_gpu_small_kernel.py -k "multidevice or logical or bad_device or sp16 or deflated or per_buffer or fused or split_plan or config"
step pytest_gpu.log 900 $PYT tests -m gpu
step c2_probe.txt 120 tools/c2_probe 48
step ab_c4_bigmin.jsonl 400 bash tools/ab_env.sh $O/ab_c4_bigmin_rows.jsonl 4 3 20 - ZCRC_BIG_MIN=1099511627776
step smoke.log 120 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench_default.jsonl 400 python3 bench.py
