# tools/gpu_small_session.sh -- GPU suite, smoke and the small-batch table
# (run on the GPU box from the repo root; writes gpurun_out/sk/)
set -o pipefail
O=gpurun_out/sk
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/small_batches.py 10 > $O/small_batches.jsonl 2> $O/small_batches.err || exit 3
