#!/bin/bash
# Round 3, session 8: DPP wave scans and folds (GPU suite; A/B against the
# same sources with shuffles: small batches, configs 2/3/4); plan probe; the
# drop-in with staged launches reading the pinned copy over PCIe.
set -e -o pipefail
O=gpurun_out/r3s8; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
for args in "100000 0" "1048576 1024" "262144 4096" "65536 16384"; do
  timeout -k 10 60 tools/plan_probe $args 50 >> $O/plan_probe.jsonl
done
timeout -k 10 300 python3 tools/small_batches.py 10 > $O/small_batches_dpp.jsonl
timeout -k 10 300 python3 tools/run_with_lib.py ablibs/predpp/zipsfs_amd/libzcrc.so tools/small_batches.py 10 > $O/small_batches_predpp.jsonl
for c in 4 2 3; do
  timeout -k 10 900 tools/ab_libs.sh $O/ab_dpp_c$c.jsonl $c 2 20 zipsfs_amd/libzcrc.so ablibs/predpp/zipsfs_amd/libzcrc.so
done
gcc -O1 -Wall -I zipsfs_amd -I include tests/dropin/preload_main.c -o /tmp/preload_main -L zipsfs_amd -lzcrc \
    -Wl,-rpath,$PWD/zipsfs_amd -pthread -ldl
for mib in 16 64 256; do
  python3 -c "import sys; sys.path.insert(0,'.'); from oracle import oracle as o; o.payload($mib<<20, 41).tofile('/tmp/e$mib.bin'); print('%08x' % o.payload_crc($mib<<20, 41))" > /tmp/e$mib.crc
  ZCRC_TRACE_HOST=1 timeout -k 10 180 /tmp/preload_main /tmp/e$mib.bin $(cat /tmp/e$mib.crc) 9 none dropin > $O/preload_${mib}_sdma.jsonl 2> $O/preload_${mib}_sdma_trace.txt
  ZCRC_STAGE_ZEROCOPY=1 ZCRC_TRACE_HOST=1 timeout -k 10 180 /tmp/preload_main /tmp/e$mib.bin $(cat /tmp/e$mib.crc) 9 none dropin > $O/preload_${mib}_zc.jsonl 2> $O/preload_${mib}_zc_trace.txt
done
