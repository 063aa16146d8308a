# tools/gpu_small_session3.sh -- config 3 A/B of the split path, alternating (writes gpurun_out/sk3/)
set -o pipefail
O=gpurun_out/sk3
mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-secondary > $O/c3_small1_$r.jsonl 2> $O/err1_$r || exit 2
  ZCRC_SMALL=0 timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --no-secondary > $O/c3_small0_$r.jsonl 2> $O/err0_$r || exit 3
done
