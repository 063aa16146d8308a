#!/bin/bash
# Round 3, session 17: the one-barrier per-buffer mode without preload.
# Full GPU suite, A/B against 8cbf5c7, bench configs 2 and default.
set -e -o pipefail
O=gpurun_out/s17; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1
for shape in "4096 65536 40" "4096 16384 40" "1000 65536 40" "4096 4096 40" "4096 1024 40" "4096 0 20"; do
  timeout -k 10 120 tools/crc_ab_fused $shape >> $O/crc_ab_fused.txt 2>&1
done
timeout -k 10 120 tools/c2_probe 20 > $O/c2_probe.txt 2>&1
for i in 1 2 3; do timeout -k 10 200 python3 bench.py --config 2 --steps 200 --warmup 20 >> $O/bench_c2.jsonl 2>> $O/bench.err; done
