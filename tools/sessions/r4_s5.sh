#!/bin/bash
# Round 4, session 5: the host inflate without per-call hipMallocAsync (the
# C harness's second gpu_inflate call read stale input and once faulted in
# session 1 / s4), then the suite, c2_probe (round-3 / round-4 / kPB=5 forms)
# and the small-batch A/B (x^-8 table, direct mode).  Stops at the first
# sign of a fault.
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r4s5; mkdir -p $O
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
gcc -O1 -Wall -I zipsfs_amd -I include tests/dropin/preload_main.c -o $O/pm -L zipsfs_amd -lzcrc -Wl,-rpath,$PWD/zipsfs_amd -pthread -ldl -lz
python3 -c "
import sys; sys.path.insert(0,'tests')
import inflate_streams as S, zlib
d=S.PAYLOADS['text'](1<<20,17); open('$O/e17.deflate','wb').write(S.deflate(d,6)); open('$O/e17.crc','w').write('%08x %d'%(zlib.crc32(d),len(d)))"
read CRC USIZE < $O/e17.crc
step harness_text17.log 200 env ZCRC_SPLIT_TRACE=1 ZCRC_PRELOAD_DEFLATED=$USIZE $O/pm $O/e17.deflate $CRC 5 gpu_inflate
PYT="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
step pytest_focus.log 600 $PYT tests/test_gpu_preload.py tests/test_gpu_inflate.py tests/test_gpu_inflate_split.py tests/test_gpu_small_kernel.py tests/test_gpu_parity.py -k "deflated or inflate or zip or direct or split_plan or strided or per_buffer or fused"
step pytest_gpu.log 900 $PYT tests -m gpu
step c4_probe_first.txt 240 tools/c4_probe 2 20
step c2_probe.txt 120 tools/c2_probe 48
for r in 1 2; do
  step small_pre_$r.jsonl 300 python3 tools/run_with_lib.py ablibs/pre/zipsfs_amd/libzcrc.so tools/small_batches.py 10 1024,2048,3000,4096
  step small_nodirect_$r.jsonl 300 env ZCRC_SMALL_DIRECT=0 python3 tools/small_batches.py 10 1024,2048,3000,4096
  step small_new_$r.jsonl 300 python3 tools/small_batches.py 10 1024,2048,3000,4096
done
step c4_probe.txt 240 tools/c4_probe 4 20
