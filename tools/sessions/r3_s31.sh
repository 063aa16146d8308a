#!/bin/bash
# Round 3, session 31: why the text chain fails with parts (ZCRC_SPLIT_TRACE)
set -e -o pipefail
O=gpurun_out/s31; mkdir -p $O
timeout -k 10 120 python3 tools/sessions/trace_split_one.py > $O/trace.out 2> $O/trace.err
