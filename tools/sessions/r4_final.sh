#!/bin/bash
# Round 4, closing evidence for the committed tree: GPU suite, smoke,
# rocprofv3 kernel stats + PMC (FETCH_SIZE, WRITE_SIZE, SQ) for configs 3, 2
# and 4 (tools/collect_profiles.sh), the default bench line and uniform
# small device batches.  Stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4final; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
for c in 3 2 4; do
  timeout -k 10 900 bash tools/collect_profiles.sh $O $c > $O/collect_c$c.log 2>&1 || exit 1$c
done
timeout -k 10 400 python3 bench.py > $O/bench_default.jsonl 2> $O/bench_default.err || exit 3
timeout -k 10 300 python3 tools/small_batches.py 10 1024,2048,3000,4096,8192,16384 > $O/small_batches.jsonl 2> $O/small_batches.err || exit 4
