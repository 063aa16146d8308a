set -o pipefail
O=gpurun_out/r2y
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_host_pool.py -x -q --timeout 120 --timeout-method thread -k "stream or pool" > $O/stream_tests.log 2>&1 || exit 1
ZCRC_PRELOAD_TABLE=$O/preload_table.jsonl timeout -k 10 400 python -u -m pytest tests/test_gpu_preload.py -q --timeout 300 --timeout-method thread > $O/preload.log 2>&1 || exit 2
timeout -k 10 200 python -u tools/host_threads.py > $O/host_threads.json 2> $O/host_threads.err || exit 3
