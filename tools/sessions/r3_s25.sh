#!/bin/bash
# Round 3, session 25 (s24 rerun after a test fix): block-parallel single-stream inflate (zcrc_inflate_split.hip)
# -- the batched inflate suite (element-generic ring), the new split tests,
# then single-entry timings; then the GPU suite, smoke and default bench.
set -e -o pipefail
O=gpurun_out/s25; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_inflate_split.py -x -v --timeout 120 --timeout-method thread > $O/pytest_split.log 2>&1
timeout -k 10 300 python3 -u tools/bench_inflate_one.py --sizes 1,16,64 --reps 5 > $O/bench_inflate_one.jsonl 2> $O/bench_inflate_one.err
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python3 bench.py > $O/bench_default.jsonl 2> $O/bench_default.err
