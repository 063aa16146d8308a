#!/bin/bash
# Round 3, session 22: repeat the s21 A/B on 4 KiB and 64 KiB shapes (noise check)
set -e -o pipefail
O=gpurun_out/s22; mkdir -p $O
for shape in "4096 4096 60" "4096 65536 60" "4096 4096 60" "4096 16384 60" "4096 4096 60" "4096 65536 60"; do
  timeout -k 10 120 tools/crc_ab_fused $shape >> $O/crc_ab_fused.txt 2>&1
done
