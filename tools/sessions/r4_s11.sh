#!/bin/bash
# Round 4, session 11: why does bench.py's config-4 step (secondary, after
# config 3 and 2 in the same process) read ~2.5% above c4_probe's?  Config 4
# alone in a fresh bench process, c4_probe, the default bench line, c4_probe
# again; then config 2 alone.
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r4s11; mkdir -p $O
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
step bench_c4_alone_1.jsonl 200 python3 bench.py --config 4 --steps 20 --no-cpu-baseline --no-secondary
step c4_probe_1.txt 200 tools/c4_probe 2 20
step bench_default_1.jsonl 300 python3 bench.py --no-cpu-baseline
step c4_probe_2.txt 200 tools/c4_probe 2 20
step bench_c4_alone_2.jsonl 200 python3 bench.py --config 4 --steps 20 --no-cpu-baseline --no-secondary
step bench_c2_alone.jsonl 200 python3 bench.py --config 2 --steps 200 --no-cpu-baseline --no-secondary
step bench_default_2.jsonl 300 python3 bench.py --no-cpu-baseline
