#!/bin/bash
# Round 3, session 40: in-place pointer jumping with per-window skip flags.
# Split parity first, then the whole GPU suite, smoke, the default bench, the
# single-entry inflate bench and its kernel trace.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s40; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_inflate_split.py -x -v --timeout 120 --timeout-method thread > $O/pytest_split.log 2>&1
timeout -k 10 300 python3 tools/bench_inflate_one.py --sizes 1,4,16,64 --reps 5 --no-serial > $O/bench_one.jsonl 2> $O/bench_one.err
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 tools/bench_inflate_one.py --sizes 1,4,16,64 --reps 3 --no-serial > $O/bench_kt.jsonl 2> $O/bench_kt.err
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python3 bench.py > $O/bench_default.jsonl 2> $O/bench_default.err
