#!/bin/bash
# Round 4, session 18: per-buffer form 16 (combine tables after the first
# barrier, a second barrier in front of the fold) against the product's 15.
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r4s18; mkdir -p $O
for i in 1 2; do
  timeout -k 10 150 tools/c2_probe 48 > $O/c2_probe_$i.txt 2>&1; rc=$?
  echo "c2_probe_$i rc=$rc" >> $O/steps.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
