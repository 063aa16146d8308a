#!/bin/bash
# Round 3, session 1: GPU suite (with the new config-5 tests), smoke, and the
# same-box A/B of the round-1 tree (9a6b3f0) against HEAD on configs 3, 2, 4.
set -e -o pipefail
O=gpurun_out/r3s1; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 900 tools/ab_trees.sh $O/ab_c3.jsonl 3 3 20 ablibs/r1 .
timeout -k 10 600 tools/ab_trees.sh $O/ab_c2.jsonl 2 2 50 ablibs/r1 .
timeout -k 10 600 tools/ab_trees.sh $O/ab_c4.jsonl 4 2 20 ablibs/r1 .
