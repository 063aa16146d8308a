#!/bin/bash
# Round 3, session 15: per-buffer mode with one barrier (braid built in
# registers, decision flags in the combine tables' zero words).  GPU suite of
# the one-launch paths, A/B against 8cbf5c7 (tools/crc_ab_fused) and
# preload on/off (crc_ab_fused_np: A = no preload), c2_probe, bench config 2.
set -e -o pipefail
O=gpurun_out/s15; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_small_kernel.py > $O/pytest_parity.log 2>&1
for shape in "4096 65536 40" "4096 16384 40" "1000 65536 40" "4096 1024 40" "4096 0 20" "2048 65537 20"; do
  timeout -k 10 120 tools/crc_ab_fused $shape >> $O/crc_ab_fused.txt 2>&1
done
for shape in "4096 65536 40" "4096 16384 40" "4096 1024 40"; do
  timeout -k 10 120 tools/crc_ab_fused_np $shape >> $O/crc_ab_fused_np.txt 2>&1
done
timeout -k 10 120 tools/c2_probe 20 > $O/c2_probe.txt 2>&1
for i in 1 2 3; do timeout -k 10 200 python3 bench.py --config 2 --steps 200 --warmup 20 >> $O/bench_c2.jsonl 2>> $O/bench.err; done
