#!/bin/bash
# Round 4, session 17 (research): what does the dynamic units' range-search
# latency cost config 4?  c4_probe with the search done twice, serially
# (ab_flags 32), against once; all buffers and the 1 MiB reference.
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r4s17; mkdir -p $O
for c in all uniform1m; do
  timeout -k 10 200 tools/c4_probe 3 20 $c > $O/c4_$c.txt 2>&1; rc=$?
  echo "c4_$c rc=$rc" >> $O/steps.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
done
