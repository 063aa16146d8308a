#!/bin/bash
# Round 4: the default bench line on whatever box this lands on (box spread
# of the committed tree), with the GPU's clocks before and after.
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r4bench_$(date +%H%M%S); mkdir -p $O
(rocm-smi --showclocks > $O/clocks_before.txt 2>&1 || true)
timeout -k 10 400 python3 bench.py > $O/bench_default.jsonl 2> $O/bench_default.err; echo "bench rc=$?" >> $O/steps.txt
(rocm-smi --showclocks > $O/clocks_after.txt 2>&1 || true)
