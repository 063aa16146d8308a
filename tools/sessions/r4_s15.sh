#!/bin/bash
# Round 4, session 15 (research for the next round): which of config 4's
# buffer classes streams below config 3's rate?  c4_probe on all / big /
# medium / no-small subsets and on ~13 GB of 1 MiB buffers.
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r4s15; mkdir -p $O
for c in uniform1m all big nosmall medium uniform1m; do
  timeout -k 10 200 tools/c4_probe 2 20 $c > $O/c4_$c.txt 2>&1; rc=$?
  echo "c4_$c rc=$rc" >> $O/steps.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
