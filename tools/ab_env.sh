#!/bin/bash
# Same-box A/B of environment settings (measurement tooling): runs bench.py
# --config CONFIG once per setting, ROUNDS times interleaved, one JSON line
# per run into OUT.      tools/ab_env.sh OUT CONFIG ROUNDS STEPS "VAR=a" "VAR=b" ...
# ("-" = the defaults)
set -e -o pipefail
OUT=$1; CONFIG=$2; ROUNDS=$3; STEPS=$4; shift 4
: > "$OUT"
for r in $(seq "$ROUNDS"); do
  for setting in "$@"; do
    if [ "$setting" = - ]; then envs=(); else envs=("$setting"); fi
    line=$(env "${envs[@]}" timeout -k 10 180 python3 bench.py --config "$CONFIG" --no-cpu-baseline --no-secondary --steps "$STEPS" | tail -n1)
    python3 -c "import json,sys; d=json.loads(sys.argv[3]); print(json.dumps({'env': sys.argv[1], 'config': int(sys.argv[2]), 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_ms': d['roofline']['avg_kernel_ms'], 'parity': d.get('parity')}))" "$setting" "$CONFIG" "$line" >> "$OUT"
  done
done
