# tools/gpu_final_session.sh -- the round's closing evidence on one box:
# GPU suite, smoke, rocprofv3 kernel stats + PMC traffic for configs 3, 2, 4
# (tools/collect_profiles.sh), then the default bench line (run on the GPU
# box from the repo root; writes gpurun_out/final_small/)
set -o pipefail
O=gpurun_out/final_small
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 2
for c in 3 2 4; do
  timeout -k 10 900 bash tools/collect_profiles.sh $O $c > $O/collect_c$c.log 2>&1 || exit 1$c
done
