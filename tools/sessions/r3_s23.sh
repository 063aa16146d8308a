#!/bin/bash
# Round 3, session 23 (fresh container): GPU suite, smoke and the default bench
# of the rebuilt tree.
set -e -o pipefail
O=gpurun_out/s23; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python3 bench.py > $O/bench_default.jsonl 2> $O/bench_default.err
