set -o pipefail
O=profiles/r02/final
mkdir -p $O gpurun_out/r2z
for c in 2 3 4; do
  timeout -k 10 900 bash tools/collect_profiles.sh $O $c > gpurun_out/r2z/collect_c$c.log 2>&1 || exit $c
done
