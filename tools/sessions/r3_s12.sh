#!/bin/bash
# Round 3, session 12: per-buffer prologue phases (lengths arrival stamp);
# the drop-in's host/GPU crossover with zero-copy staging.
set -e -o pipefail
O=gpurun_out/r3s12; mkdir -p $O
timeout -k 10 120 tools/c2_probe 20 > $O/c2_probe.txt 2>&1
timeout -k 10 300 python3 tools/dropin_crossover.py > $O/dropin_crossover.json 2> $O/dropin_crossover.err
