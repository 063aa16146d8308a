#!/bin/bash
# Round 4: does config 3's step depend on how long the GPU has been busy
# (clock ramp on a cold box)?  Fresh bench processes, config 3 only, warmup
# 3 vs 100 steps, alternating, starting cold; GPU clocks between.
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r4warm; mkdir -p $O
i=0
for w in 3 100 3 100 3; do
  i=$((i+1))
  (rocm-smi --showclocks > $O/clocks_$i.txt 2>&1 || true)
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-secondary --warmup $w > $O/bench_${i}_w$w.jsonl 2>&1; echo "bench_${i}_w$w rc=$?" >> $O/steps.txt
done
