set -o pipefail
O=gpurun_out/r2ad
mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench_default.jsonl 2> $O/bench_default.err || exit 1
timeout -k 10 300 python -u bench.py --gpus 2 --dist-backend gloo --buffers-per-gpu 32768 --steps 5 --warmup 2 > $O/spawn2_gloo.jsonl 2> $O/spawn2_gloo.err || exit 2
