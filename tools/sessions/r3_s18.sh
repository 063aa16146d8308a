#!/bin/bash
# Round 3, session 18: config-2 shape probes (pure reads in the per-buffer
# mapping, rotated start, no priorities) beside the CRC kernels.
set -e -o pipefail
O=gpurun_out/s18; mkdir -p $O
timeout -k 10 180 tools/c2_probe 20 > $O/c2_probe.txt 2>&1
timeout -k 10 180 tools/c2_probe 20 > $O/c2_probe_2.txt 2>&1
