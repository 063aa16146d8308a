#!/bin/bash
# Round 3, session 9: GPU suite (zero-copy staging by default) and the
# stream tests with zero-copy stream pieces; the preload table with SDMA vs
# zero-copy stream pieces; host-resident rates 1-32 threads, zero-copy vs
# SDMA staging; plan probe.
set -e -o pipefail
O=gpurun_out/r3s9; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
ZCRC_STREAM_ZEROCOPY=1 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_stream.py tests/test_gpu_host_pool.py tests/test_gpu_preload.py -m gpu -x -v --timeout 300 --timeout-method thread -k "stream or pool or preload" > $O/pytest_stream_zc.log 2>&1
gcc -O1 -Wall -I zipsfs_amd -I include tests/dropin/preload_main.c -o /tmp/preload_main -L zipsfs_amd -lzcrc \
    -Wl,-rpath,$PWD/zipsfs_amd -pthread -ldl
for mib in 16 64 256; do
  python3 -c "import sys; sys.path.insert(0,'.'); from oracle import oracle as o; o.payload($mib<<20, 41).tofile('/tmp/e$mib.bin'); print('%08x' % o.payload_crc($mib<<20, 41))" > /tmp/e$mib.crc
  timeout -k 10 180 /tmp/preload_main /tmp/e$mib.bin $(cat /tmp/e$mib.crc) 7 none dropin stream stream_reg > $O/preload_${mib}_sdma.jsonl
  ZCRC_STREAM_ZEROCOPY=1 timeout -k 10 180 /tmp/preload_main /tmp/e$mib.bin $(cat /tmp/e$mib.crc) 7 none dropin stream stream_reg > $O/preload_${mib}_zc.jsonl
done
timeout -k 10 300 python3 tools/host_threads.py > $O/host_threads_zc.json
ZCRC_STAGE_ZEROCOPY=0 timeout -k 10 300 python3 tools/host_threads.py > $O/host_threads_sdma.json
for args in "100000 0" "1048576 1024" "65536 16384"; do
  timeout -k 10 60 tools/plan_probe $args 50 >> $O/plan_probe.jsonl
done
