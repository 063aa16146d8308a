# tools/gpu_final_session.sh -- PMC + kernel-trace evidence for configs 3, 2, 4
# and the default bench line (run on the GPU box from the repo root; writes
# gpurun_out/final_small/)
set -o pipefail
O=gpurun_out/final_small
mkdir -p $O
for c in 3; do
  timeout -k 10 900 bash tools/collect_profiles.sh $O $c > $O/collect_c$c.log 2>&1 || exit $c
done
true
