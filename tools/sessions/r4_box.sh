#!/bin/bash
# Round 4: does config 3's per-box spread follow the box's pure-read rate?
# c2_probe (pure reads in the CRC kernel's shapes, nt) and config 3's bench
# step on the same box, twice.
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r4box_$(date +%H%M%S); mkdir -p $O
for i in 1 2; do
  timeout -k 10 120 tools/c2_probe 24 > $O/c2_probe_$i.txt 2>&1; echo "c2_probe_$i rc=$?" >> $O/steps.txt
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-secondary > $O/bench_$i.jsonl 2>&1; echo "bench_$i rc=$?" >> $O/steps.txt
done
