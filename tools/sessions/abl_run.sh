#!/bin/bash
# Inflate ablations (measurement tooling, run on the GPU box from the repo
# root): builds made by hand with -DZI_ABL_NOLIT / -DZI_ABL_NOCOPY into
# tools/abl_*.so (see zcrc_inflate.hip) timed against the product library on
# text and spectrum payloads.  Output: gpurun_out/abl.jsonl.
set -e
B="python -u tools/bench_inflate.py --entries 1024 --reps 2 --no-cpu"
for k in text spectrum; do
  timeout -k 10 100 $B --kind $k >> gpurun_out/abl.jsonl
  for v in tools/abl_*.so; do
    [ -f "$v" ] && timeout -k 10 100 $B --kind $k --lib "$v" >> gpurun_out/abl.jsonl
  done
done
