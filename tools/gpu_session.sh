set -o pipefail
O=gpurun_out/r2v
mkdir -p $O
export TMPDIR=/tmp
for shape in "4096 65536 40" "100000 0 20" "16384 1048576 10" "1048576 1024 20" "262144 4096 20" "65536 16384 20"; do
  timeout -k 10 200 tools/crc_ab $shape >> $O/crc_ab.txt 2>&1 || exit 1
done
timeout -k 10 200 tools/small_probe 10 > $O/small_probe.txt 2>&1 || exit 2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 3
for c in 2 3 4; do
  timeout -k 10 300 python -u bench.py --config $c --steps 30 --warmup 5 --no-cpu-baseline >> $O/bench.jsonl 2>> $O/bench.err || exit 4
done
for c in 2 3 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c$c -o run -- python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_c$c.log 2>&1 || exit 5
done
