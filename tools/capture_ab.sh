#!/bin/bash
# Do the scratch reaper's trims invalidate graph captures another thread has
# open in global mode?  tests/dropin/destroy_release.c "capture" against
# libzcrc with ZCRC_SCRATCH_CACHE_MIB=1 (~30 trims during the loop) and 2048
# (no trims).  ($2 = another build's directory, e.g. one whose reaper thread
# switched itself to relaxed capture mode: profiles/r06/s10)
# Output: one JSON line per run into $1.
set -o pipefail
OUT=${1:-gpurun_out/capture_ab.jsonl}
mkdir -p "$(dirname "$OUT")"
: > "$OUT"
ALT=${2:-}
for v in trims nobudget ${ALT:+alt}; do
  d=zipsfs_amd; [ $v = alt ] && d=$ALT
  mib=1; [ $v = nobudget ] && mib=2048  # nobudget: the reaper never trims
  gcc -O1 -Wall -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude tests/dropin/destroy_release.c \
    -o /tmp/dr_$v -L$d -lzcrc -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,$PWD/$d -pthread -lz || exit 1
  line=$(ZCRC_SCRATCH_CACHE_MIB=$mib timeout -k 10 120 /tmp/dr_$v capture 3.5 2>$(dirname "$OUT")/dr_$v.err | tail -n1)
  rc=$?
  echo "{\"lib\": \"$v\", \"rc\": $rc, \"result\": ${line:-null}}" >> "$OUT"
  [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ] && exit $rc
done
exit 0
