# tools/gpu_small_session3.sh -- A/B of the device split plan on the bench
# configs, alternating (writes gpurun_out/sk3/)
set -o pipefail
O=gpurun_out/sk3
mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/b_small1_$r.jsonl 2> $O/err1_$r || exit 2
  ZCRC_SMALL=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/b_small0_$r.jsonl 2> $O/err0_$r || exit 3
done
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof4 -o run --output-format csv -- python3 $R/bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline > $R/$O/prof4.log 2>&1 || exit 5
