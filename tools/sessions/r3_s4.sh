#!/bin/bash
# Round 3, session 4: GPU suite; preload harness per size with the phase
# trace (slots warmed at creation, registered last chunk waits for its DMA);
# small_body noinline experiment (kernel A/B on config 3, tree A/B on
# configs 3/4); default bench with the CPU-baseline thread sweep.
set -e -o pipefail
O=gpurun_out/r3s4; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
gcc -O1 -Wall -I zipsfs_amd -I include tests/dropin/preload_main.c -o /tmp/preload_main -L zipsfs_amd -lzcrc \
    -Wl,-rpath,$PWD/zipsfs_amd -pthread -ldl
for kib in 4 1024 16384 65536 262144; do
  python3 -c "import sys; sys.path.insert(0,'.'); from oracle import oracle as o; o.payload($kib<<10, 41).tofile('/tmp/e$kib.bin'); print('%08x' % o.payload_crc($kib<<10, 41))" > /tmp/e$kib.crc
  ZCRC_TRACE_HOST=1 ZCRC_REF_LIB=$PWD/oracle/_ref/libref_cg_crc32_O0.so timeout -k 10 180 /tmp/preload_main /tmp/e$kib.bin $(cat /tmp/e$kib.crc) 7 none dropin stream stream_reg ref > $O/preload_$kib.jsonl 2> $O/preload_${kib}_trace.txt
done
for b in WT_noinl r1_noinl r1_WT WT_noinl; do
  timeout -k 10 120 ablibs/ab/crc_ab_$b 65536 1048576 10 > $O/crc_ab_$b.txt 2>&1 || true
  cat $O/crc_ab_$b.txt | tail -1
done
timeout -k 10 900 tools/ab_trees.sh $O/ab_noinl_c4.jsonl 4 3 20 . ablibs/noinl
timeout -k 10 900 tools/ab_trees.sh $O/ab_noinl_c3.jsonl 3 2 20 . ablibs/noinl
timeout -k 10 400 python3 bench.py > $O/bench_default.jsonl 2> $O/bench_default.err
