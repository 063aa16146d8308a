#!/bin/bash
# Round 3, session 16: per-buffer timeline with and without the preload
# (tools/c2_probe, c2_probe_np built with -DZCRC_PERBUF_PRELOAD=0).
set -e -o pipefail
O=gpurun_out/s16; mkdir -p $O
timeout -k 10 120 tools/c2_probe 20 > $O/c2_probe.txt 2>&1
timeout -k 10 120 tools/c2_probe_np 20 > $O/c2_probe_np.txt 2>&1
timeout -k 10 120 tools/c2_probe 20 > $O/c2_probe_2.txt 2>&1
