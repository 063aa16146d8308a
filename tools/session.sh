#!/bin/bash
# One parameterised GPU-session runner (replaces round 3-4's one-off
# tools/sessions/*.sh).  Run on the GPU box from the repo
# root through gpurun:
#
#     tools/session.sh <name> <step> [<step> ...]
#
# Steps (each under its own time limit, the chain stops at the first failure,
# logs in gpurun_out/<name>/):
#   pytest                 the whole -m gpu suite
#   pytest:<k-expr>        -m gpu -k <k-expr>
#   smoke                  __graft_entry__.smoke()
#   bench                  the default bench line (what the driver runs)
#   bench:<args>           bench.py <args> (commas stand for spaces)
#   profiles:<cfg>         tools/collect_profiles.sh for config <cfg>
#   small                  uniform small device batches (tools/small_batches.py)
#   probe:<tool>:<args>    a built tools/<tool> binary (commas for spaces)
#   py:<script>:<args>     python3 <script> <args> (commas for spaces)
#   kt:<script>:<args>     the same under rocprofv3 --kernel-trace --stats
#                          (csv under gpurun_out/<name>/kt<step>/)
#   ab:<config>:<rounds>:<steps>:<lib>,<lib>...  tools/ab_libs.sh (bench.py per
#                          library build, interleaved; no secondaries, ceiling
#                          or host-resident line) into gpurun_out/<name>/ab_<config>.jsonl
#   churn:<reps>,<spec>... tools/churn_stress.sh (specs "label|ENV=V|parts|rounds|threads")
#   export:<VAR>=<value>   set an environment variable for the steps after it
#   unset:<VAR>            remove it again
set -o pipefail
export TMPDIR=/tmp
NAME=${1:?usage: session.sh <name> <step>...}
shift
O=gpurun_out/$NAME
mkdir -p "$O"
# heartbeat: a slow but healthy step (the first import torch on a fresh box,
# a quiet test) must not read as a hang; every step keeps its own time limit
( while sleep 30; do date +%T >> "$O/heartbeat"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
n=0
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%:*}
  arg=${step#*:}
  [ "$arg" = "$step" ] && arg=""
  log="$O/$(printf %02d $n)_${kind}.log"
  echo "[$n] $step -> $log" | tee -a "$O/steps.txt"
  case "$kind" in
    pytest)
      if [ -n "$arg" ]; then
        timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread \
          -k "$arg" > "$log" 2>&1
      else
        timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
          > "$log" 2>&1
      fi ;;
    smoke)
      timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$log" 2>&1 ;;
    bench)
      # shellcheck disable=SC2086
      timeout -k 10 600 python3 -u bench.py ${arg//,/ } > "$log" 2> "$log.err" ;;
    profiles)
      timeout -k 10 900 bash tools/collect_profiles.sh "$O" "${arg:-3}" > "$log" 2>&1 ;;
    small)
      timeout -k 10 300 python3 tools/small_batches.py 10 1024,2048,3000,4096,8192,16384 > "$log" 2> "$log.err" ;;
    probe)
      tool=${arg%%:*}; targs=${arg#*:}; [ "$targs" = "$arg" ] && targs=""
      # shellcheck disable=SC2086
      timeout -k 10 300 "tools/$tool" ${targs//,/ } > "$log" 2>&1 ;;
    py)
      script=${arg%%:*}; pargs=${arg#*:}; [ "$pargs" = "$arg" ] && pargs=""
      # shellcheck disable=SC2086
      timeout -k 10 600 python3 -u "$script" ${pargs//,/ } > "$log" 2>&1 ;;
    kt)
      script=${arg%%:*}; pargs=${arg#*:}; [ "$pargs" = "$arg" ] && pargs=""
      # shellcheck disable=SC2086
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt$n" -o kt -- \
        python3 -u "$script" ${pargs//,/ } > "$log" 2>&1 ;;
    ab)
      IFS=: read -r cfg rounds steps libs <<< "$arg"
      # shellcheck disable=SC2086
      AB_BENCH_ARGS="--no-secondary --no-read-ceiling --host-resident-gib 0" timeout -k 10 1000 \
        bash tools/ab_libs.sh "$O/ab_$cfg.jsonl" "$cfg" "$rounds" "$steps" ${libs//,/ } > "$log" 2>&1 ;;
    churn)
      # shellcheck disable=SC2086
      timeout -k 10 1100 bash tools/churn_stress.sh "$O/churn$n" ${arg//,/ } > "$log" 2>&1 ;;
    export)
      export "${arg?}"; echo "    $arg" >> "$O/steps.txt"; continue ;;
    unset)
      unset "${arg?}"; continue ;;
    *)
      echo "unknown step $step" | tee -a "$O/steps.txt"; exit 90 ;;
  esac
  rc=$?
  echo "    rc=$rc" | tee -a "$O/steps.txt"
  if [ $rc -ne 0 ]; then
    tail -30 "$log"
    exit $rc
  fi
  tail -2 "$log"
done
