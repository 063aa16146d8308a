#!/bin/bash
# Round 3, session 13: rocprofv3 evidence for the current kernel sources
# (kernel trace + stats, FETCH_SIZE, WRITE_SIZE, SQ counters in separate
# passes) for configs 3, 2, 4 -> profiles/r03/final/.
set -e -o pipefail
O=profiles/r03/final; mkdir -p $O
for c in 3 2 4; do
  timeout -k 10 1000 tools/collect_profiles.sh $O $c
done
