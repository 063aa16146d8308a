#!/bin/bash
# Collect the rocprofv3 evidence behind bench.py's roofline object
# (measurement tooling; run on the GPU box from the repo root):
#
#     tools/collect_profiles.sh <out_dir> [config]
#
# Four separate profiler runs of the same bench command, as the MI355X guide's
# HBM/rocprofv3 section prescribes (counters never share a run with traces):
#   1. --kernel-trace --stats        per-kernel durations (must agree with the
#                                    HIP-event average bench.py reports)
#   2. --pmc FETCH_SIZE              HBM read bytes (gfx950: x 2 x 1024)
#   3. --pmc WRITE_SIZE              HBM write bytes (KiB)
#   4. --pmc SQ_* GRBM_GUI_ACTIVE    instruction mix, LDS conflicts, clock
# then tools/pmc_summary.py folds them into <out_dir>/pmc_summary_config<C>.json.
# Each step has its own time limit and the chain stops at the first failure.
set -e -o pipefail
OUT=${1:?usage: collect_profiles.sh <out_dir> [config]}
CFG=${2:-3}
export TMPDIR=/tmp
W=gpurun_out/prof_c${CFG}
mkdir -p "$OUT" "$W"
BENCH=(python3 bench.py --config "$CFG" --steps 5 --warmup 1 --no-cpu-baseline --no-secondary --no-read-ceiling
       --host-resident-gib 0)

timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$W/kt" -o bench -- "${BENCH[@]}" > "$W/kt.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$W/fetch" -o bench -- "${BENCH[@]}" > "$W/fetch.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$W/write" -o bench -- "${BENCH[@]}" > "$W/write.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
  SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d "$W/sq" -o bench -- "${BENCH[@]}" > "$W/sq.log" 2>&1

python3 tools/pmc_summary.py "$W/kt" "$W/fetch" "$W/write" "$W/sq" "$OUT/pmc_summary_config${CFG}.json" > /dev/null
cp "$(find "$W/kt" -name '*kernel_stats.csv' | head -1)" "$OUT/rocprof_kernel_stats_config${CFG}.csv"
grep '^{"metric"' "$W/kt.log" | tail -1 > "$OUT/rocprof_bench_config${CFG}.jsonl"
echo "profiles for config $CFG in $OUT"
