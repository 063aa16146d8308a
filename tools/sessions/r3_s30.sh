#!/bin/bash
# Round 3, session 30: split inflate with parts (a chunk's first block cut
# into items started at probed token boundaries, per-token landing): parity,
# then the single-entry bench with parts on (default) and off, and a kernel
# trace of the default.
set -e -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s30; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_inflate_split.py -x -v --timeout 120 --timeout-method thread > $O/pytest_split.log 2>&1
for p in 0 1; do
  ZCRC_SPLIT_PARTS=$p timeout -k 10 300 python3 tools/bench_inflate_one.py --sizes 1,4,16,64 --reps 5 --no-serial > $O/bench_parts$p.jsonl 2> $O/bench_parts$p.err
done
for k in text spectrum; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$k -o run -- python3 tools/bench_inflate_one.py --kinds $k --sizes 1,16,64 --reps 3 --no-serial > $O/bench_$k.jsonl 2> $O/bench_$k.err
done
