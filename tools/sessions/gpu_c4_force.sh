# tools/gpu_c4_force.sh -- config 4 with the split plan forced (small-list
# weights) vs auto, and the split-plan GPU tests (writes gpurun_out/c4f/)
set -o pipefail
O=gpurun_out/c4f
mkdir -p $O
true
for r in 1 2; do
  for w in 14 20 28; do
    ZCRC_SMALL=2 ZCRC_SMALL_COST=$w timeout -k 10 300 python -u bench.py --config 4 --steps 20 --warmup 3 --no-cpu-baseline > $O/force_w${w}_$r.jsonl 2> $O/ef_$r || exit 2
  done
  timeout -k 10 300 python -u bench.py --config 4 --steps 20 --warmup 3 --no-cpu-baseline > $O/auto_$r.jsonl 2> $O/ea_$r || exit 3
done
