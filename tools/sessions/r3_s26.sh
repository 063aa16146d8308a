#!/bin/bash
# Round 3, session 26: per-kernel breakdown of the block-parallel inflate
# (rocprofv3 kernel trace of tools/bench_inflate_one.py, no one-wave runs).
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s26; mkdir -p $O
for k in text spectrum; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$k -o run -- python3 tools/bench_inflate_one.py --kinds $k --sizes 1,16,64 --reps 3 --no-serial > $O/bench_$k.jsonl 2> $O/bench_$k.err
done
