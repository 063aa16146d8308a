#!/bin/bash
# Round 3, session 33: the whole GPU suite, smoke and the default bench on the
# current tree (split inflate with parts), plus the batched inflate bench
# (the serial kernels share zcrc_inflate_impl.h with the split decoder).
set -e -o pipefail
O=gpurun_out/s33; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python3 bench.py > $O/bench_default.jsonl 2> $O/bench_default.err
timeout -k 10 300 python3 tools/bench_inflate.py --entries 4096 --kind mixed --reps 3 --no-cpu > $O/bench_inflate_mixed.jsonl 2> $O/bench_inflate_mixed.err
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/bench_inflate_one.py --sizes 1,4,16,64 --reps 5 --no-serial > $O/bench_one.jsonl 2> $O/bench_one.err
for k in text spectrum; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$k -o run -- python3 tools/bench_inflate_one.py --kinds $k --sizes 1,16 --reps 3 --no-serial > $O/bench_$k.jsonl 2> $O/bench_$k.err
done
