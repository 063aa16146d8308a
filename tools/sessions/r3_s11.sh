#!/bin/bash
# Round 3, session 11: per-buffer prologue with the decision's lengths
# loaded first (c2_probe timeline; config 2 A/B against the previous build);
# GPU suite.
set -e -o pipefail
O=gpurun_out/r3s11; mkdir -p $O
timeout -k 10 120 tools/c2_probe 20 > $O/c2_probe.txt 2>&1
timeout -k 10 900 tools/ab_libs.sh $O/ab_c2.jsonl 2 4 200 zipsfs_amd/libzcrc.so ablibs/prev/zipsfs_amd/libzcrc.so
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
