#!/bin/bash
# Round 4, session 8: claim-counter throughput (atomic_probe), per-buffer
# register-group depth A/B (c2_probe 104/204/105), and HEAD's config-2 PMC
# (collect_profiles.sh: kernel stats, FETCH/WRITE, SQ incl. LDS conflicts).
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r4s8; mkdir -p $O
fault_stop() { if grep -qi "illegal\|memory access fault\|Aborted\|core dumped" "$O/$1"; then echo "fault in $1: stopping" >> $O/steps.txt; exit 9; fi; }
step() {
  local log=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$log 2>&1
  local rc=$?
  echo "$log rc=$rc" >> $O/steps.txt
  if [ $rc -ge 124 ]; then echo "stopping after $log (rc $rc)" >> $O/steps.txt; exit $rc; fi
  fault_stop $log
  return 0
}
step atomic12.txt 60 tools/atomic_probe 12
step atomic24.txt 60 tools/atomic_probe 24
step c2_probe.txt 120 tools/c2_probe 48
step collect_c2.log 600 bash tools/collect_profiles.sh $O/prof 2
