#!/bin/bash
# Round 3, session 39: parts only for small streams (<= resident / 4 chunks):
# split parity, single-entry bench (with the one-wave column), kernel trace.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s39; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_inflate_split.py -x -v --timeout 120 --timeout-method thread > $O/pytest_split.log 2>&1
timeout -k 10 300 python3 tools/bench_inflate_one.py --sizes 1,4,16,64 --reps 5 > $O/bench_one.jsonl 2> $O/bench_one.err
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 tools/bench_inflate_one.py --sizes 1,4,16,64 --reps 3 --no-serial > $O/bench_kt.jsonl 2> $O/bench_kt.err
