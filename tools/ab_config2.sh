#!/bin/bash
# Same-box A/B of library builds on config 2 (measurement tooling): runs
# bench.py --config 2 against each .so in turn, ROUNDS times interleaved,
# one JSON line per run into OUT.   tools/ab_config2.sh OUT ROUNDS LIB...
set -e -o pipefail
OUT=$1; ROUNDS=$2; shift 2
: > "$OUT"
for r in $(seq "$ROUNDS"); do
  for lib in "$@"; do
    line=$(timeout -k 10 120 python3 tools/bench_with_lib.py "$lib" --config 2 --no-cpu-baseline --steps 50 | tail -n1)
    python3 -c "import json,sys; d=json.loads(sys.argv[2]); print(json.dumps({'lib': sys.argv[1], 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_ms': d['roofline']['avg_kernel_ms']}))" "$lib" "$line" >> "$OUT"
  done
done
