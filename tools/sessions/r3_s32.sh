#!/bin/bash
# Round 3, session 32: chunk-owned regions split among parts -- trace of a
# 1 MiB text and spectrum entry, parity, single-entry bench, kernel trace.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s32; mkdir -p $O
timeout -k 10 120 python3 tools/sessions/trace_split_one.py > $O/trace.out 2> $O/trace.err
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_inflate_split.py -x -v --timeout 120 --timeout-method thread > $O/pytest_split.log 2>&1
timeout -k 10 300 python3 tools/bench_inflate_one.py --sizes 1,4,16,64 --reps 5 --no-serial > $O/bench.jsonl 2> $O/bench.err
for k in text spectrum; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$k -o run -- python3 tools/bench_inflate_one.py --kinds $k --sizes 1,16,64 --reps 3 --no-serial > $O/bench_$k.jsonl 2> $O/bench_$k.err
done
