#!/bin/bash
# Round 3, session 29: split inflate with pointer-jumping windows instead of the tails walk;
# word-window finder and the residency chunk rule: parity, then the kernel
# trace of the single-entry bench.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s29; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_inflate_split.py -x -v --timeout 120 --timeout-method thread > $O/pytest_split.log 2>&1
for k in text spectrum; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$k -o run -- python3 tools/bench_inflate_one.py --kinds $k --sizes 1,16,64 --reps 3 --no-serial > $O/bench_$k.jsonl 2> $O/bench_$k.err
done
for r in 16 32; do
  ZCRC_SPLIT_RING=$r timeout -k 10 300 python3 tools/bench_inflate_one.py --sizes 1,4,16,64 --reps 5 --no-serial > $O/bench_ring$r.jsonl 2> $O/bench_ring$r.err
done
