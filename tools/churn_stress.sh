#!/bin/bash
# Repeated runs of tests/dropin/stream_churn.c under several settings, to
# find what an intermittent mismatch depends on (measurement tooling; run on
# the GPU box from the repo root).  A run that reports mismatches (exit 1) is
# recorded and the next one starts; any other failure (abort, fault, time
# limit) ends the script.
#
#   tools/churn_stress.sh OUTDIR REPS "label|ENV=V ...|parts|rounds|threads" ...
set -o pipefail
O=$1; REPS=$2; shift 2
mkdir -p "$O"
exe="$O/stream_churn"
gcc -O1 -Wall -Werror -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude tests/dropin/stream_churn.c -o "$exe" \
  -Lzipsfs_amd -lzcrc -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,"$PWD/zipsfs_amd" -pthread -lz || exit 3
for spec in "$@"; do
  IFS='|' read -r label envs parts rounds threads <<< "$spec"
  for r in $(seq "$REPS"); do
    # shellcheck disable=SC2086
    env $envs STREAM_CHURN_PARTS="$parts" timeout -k 10 240 "$exe" "$rounds" "$threads" \
      > "$O/$label.$r.out" 2> "$O/$label.$r.err"
    rc=$?
    echo "$label rep $r rc=$rc $(tail -n1 "$O/$label.$r.out")" | tee -a "$O/summary.txt"
    sed 's/^/    /' "$O/$label.$r.err" | head -8 | tee -a "$O/summary.txt"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  done
done
