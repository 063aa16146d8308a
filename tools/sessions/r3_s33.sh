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
