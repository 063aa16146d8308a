#!/bin/bash
# Same-box A/B of whole source trees (measurement tooling): runs each tree's
# own bench.py --config CONFIG in turn, ROUNDS times interleaved, one JSON
# line per run into OUT.   tools/ab_trees.sh OUT CONFIG ROUNDS STEPS TREE...
# (a TREE is a directory holding bench.py and its built zipsfs_amd/libzcrc.so,
# e.g. `git archive <rev> | tar -x -C ablibs/<name>` + make -C zipsfs_amd/csrc)
set -e -o pipefail
OUT=$1; CONFIG=$2; ROUNDS=$3; STEPS=$4; shift 4
: > "$OUT"
for r in $(seq "$ROUNDS"); do
  for tree in "$@"; do
    extra=""
    grep -q -- "--no-secondary" "$tree/bench.py" && extra="--no-secondary"
    line=$(cd "$tree" && timeout -k 10 240 python3 bench.py --config "$CONFIG" --no-cpu-baseline $extra --steps "$STEPS" | tail -n1)
    python3 -c "import json,sys; d=json.loads(sys.argv[3]); print(json.dumps({'tree': sys.argv[1], 'round': int(sys.argv[4]), 'config': int(sys.argv[2]), 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_ms': d['roofline']['avg_kernel_ms'], 'parity': d.get('parity')}))" "$tree" "$CONFIG" "$line" "$r" >> "$OUT"
    tail -n1 "$OUT"
  done
done
