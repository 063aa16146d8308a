#!/bin/bash
# Round 4: config 3's per-box spread against a 64 GiB pure read on the same
# box (tools/hbm_probe: grid-stride and wave-contiguous, nt and not), twice.
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r4box2_$(date +%H%M%S); mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 tools/hbm_probe 64 3 > $O/hbm_probe_$i.txt 2>&1; echo "hbm_probe_$i rc=$?" >> $O/steps.txt
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-secondary > $O/bench_$i.jsonl 2>&1; echo "bench_$i rc=$?" >> $O/steps.txt
done
