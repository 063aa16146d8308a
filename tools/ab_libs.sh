#!/bin/bash
# Same-box A/B of library builds (measurement tooling): runs bench.py
# --config CONFIG against each .so in turn, ROUNDS times interleaved, one
# JSON line per run into OUT.   tools/ab_libs.sh OUT CONFIG ROUNDS STEPS LIB...
set -e -o pipefail
OUT=$1; CONFIG=$2; ROUNDS=$3; STEPS=$4; shift 4
: > "$OUT"
for r in $(seq "$ROUNDS"); do
  for lib in "$@"; do
    # shellcheck disable=SC2086
    line=$(timeout -k 10 180 python3 tools/bench_with_lib.py "$lib" --config "$CONFIG" --no-cpu-baseline --steps "$STEPS" \
      ${AB_BENCH_ARGS:-} | tail -n1)
    python3 -c "import json,sys; d=json.loads(sys.argv[3]); print(json.dumps({'lib': sys.argv[1], 'config': int(sys.argv[2]), 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_ms': d['roofline']['avg_kernel_ms'], 'parity': d.get('parity')}))" "$lib" "$CONFIG" "$line" >> "$OUT"
  done
done
