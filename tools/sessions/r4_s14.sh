#!/bin/bash
# Round 4, session 14 (research for the next round): pure-read cost of short
# pieces with 2-4 groups in flight, restarting or carrying the pipeline
# across pieces (tools/piece_probe).
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r4s14; mkdir -p $O
timeout -k 10 120 tools/piece_probe 5 > $O/piece_probe.txt 2>&1; echo "piece_probe rc=$?" >> $O/steps.txt
