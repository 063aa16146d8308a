# tools/gpu_small_session.sh -- measurement session for the small-buffer
# kernel (run on the GPU box from the repo root; writes gpurun_out/sk/)
set -o pipefail
O=gpurun_out/sk
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_small_kernel.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $O/bench_small1.jsonl 2> $O/bench_small1.err || exit 2
ZCRC_SMALL=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_small0b.jsonl 2> $O/bench_small0b.err || exit 3
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_small1b.jsonl 2> $O/bench_small1b.err || exit 3
ZCRC_SMALL=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_small0.jsonl 2> $O/bench_small0.err || exit 4
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof4 -o run --output-format csv -- python3 $R/bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline > $R/$O/prof4.log 2>&1 || exit 5
