#!/bin/bash
# Round 3, session 19/20: per-buffer mode variants against fc529b5 (s20: the preload
# barrier waits only for the combine-table loads) against fc529b5.
set -e -o pipefail
O=gpurun_out/s20; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_small_kernel.py > $O/pytest_parity.log 2>&1
for shape in "4096 65536 40" "4096 16384 40" "1000 65536 40" "4096 4096 40" "4096 1024 40" "4096 0 20" "2048 65537 20"; do
  timeout -k 10 120 tools/crc_ab_fused $shape >> $O/crc_ab_fused.txt 2>&1
done
timeout -k 10 180 tools/c2_probe 20 > $O/c2_probe.txt 2>&1
