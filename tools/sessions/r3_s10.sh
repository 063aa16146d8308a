#!/bin/bash
# Round 3, session 10: GPU suite (zero-copy streams by default); the preload
# table; config-2 per-buffer timeline (c2_probe); default bench.
set -e -o pipefail
O=gpurun_out/r3s10; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
gcc -O1 -Wall -I zipsfs_amd -I include tests/dropin/preload_main.c -o /tmp/preload_main -L zipsfs_amd -lzcrc \
    -Wl,-rpath,$PWD/zipsfs_amd -pthread -ldl
for kib in 4 1024 16384 65536 262144; do
  python3 -c "import sys; sys.path.insert(0,'.'); from oracle import oracle as o; o.payload($kib<<10, 41).tofile('/tmp/e$kib.bin'); print('%08x' % o.payload_crc($kib<<10, 41))" > /tmp/e$kib.crc
  ZCRC_REF_LIB=$PWD/oracle/_ref/libref_cg_crc32_O0.so timeout -k 10 180 /tmp/preload_main /tmp/e$kib.bin $(cat /tmp/e$kib.crc) 7 none dropin stream stream_reg ref > $O/preload_$kib.jsonl
done
timeout -k 10 120 tools/c2_probe 20 > $O/c2_probe.txt 2>&1
timeout -k 10 400 python3 bench.py > $O/bench_default.jsonl 2> $O/bench_default.err
