set -e
B="python -u tools/bench_inflate.py --entries 1024 --reps 2 --no-cpu"
for k in text spectrum; do
  timeout -k 10 100 $B --kind $k >> gpurun_out/abl.jsonl
  timeout -k 10 100 $B --kind $k --lib tools/abl_NOLIT.so >> gpurun_out/abl.jsonl
  timeout -k 10 100 $B --kind $k --lib tools/abl_NOCOPY.so >> gpurun_out/abl.jsonl
done
