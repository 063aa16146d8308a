#!/bin/bash
# Round 3, session 2: bisect of the config-3 slowdown over round-2 trees
# (same box, interleaved), config-2 step with/without per-launch HIP events
# (+ kernel traces for the inter-launch gaps), host registration probe.
set -e -o pipefail
O=gpurun_out/r3s2; mkdir -p $O
timeout -k 10 120 tools/reg_probe 3 > $O/reg_probe.jsonl 2>&1
timeout -k 10 1200 tools/ab_trees.sh $O/bisect_c3.jsonl 3 2 20 ablibs/r1 ablibs/bfefb3c ablibs/8e121b5 ablibs/ee983f1 ablibs/58086df ablibs/6887c22 ablibs/65795a2 ablibs/7ef436a .
for r in 1 2 3; do
  timeout -k 10 120 python3 bench.py --config 2 --no-cpu-baseline --steps 200 | tail -n1 > $O/c2_events_$r.json
  ZCRC_BENCH_NO_EVENTS=1 timeout -k 10 120 python3 bench.py --config 2 --no-cpu-baseline --steps 200 | tail -n1 > $O/c2_noevents_$r.json
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ZCRC_BENCH_NO_EVENTS=1 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/kt_c2_noev -- python3 bench.py --config 2 --no-cpu-baseline --steps 200 > $O/kt_c2_noev.log 2>&1
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/kt_c2_ev -- python3 bench.py --config 2 --no-cpu-baseline --steps 200 > $O/kt_c2_ev.log 2>&1
