# tools/gpu_small_session3.sh -- split-plan GPU tests, then A/B of the device
# split plan on the bench configs, alternating (writes gpurun_out/sk3/)
set -o pipefail
O=gpurun_out/sk3
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_small_kernel.py > $O/tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/b_small1_$r.jsonl 2> $O/err1_$r || exit 2
  ZCRC_SMALL=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/b_small0_$r.jsonl 2> $O/err0_$r || exit 3
done
