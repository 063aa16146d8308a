#!/bin/bash
# Round 3, session 34: where the finder's time goes (ZCRC_SPLIT_FIND_TIMING:
# 1 = quick filter only, 2 = staging only; candidates then none, the serial
# fall-back decodes) -- kernel traces of 1 MiB text and spectrum entries.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s34; mkdir -p $O
for t in 0 1 2; do
  ZCRC_SPLIT_FIND_TIMING=$t timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$t -o run -- python3 tools/bench_inflate_one.py --sizes 1 --reps 2 --no-serial > $O/bench_$t.jsonl 2> $O/bench_$t.err
done
