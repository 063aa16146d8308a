set -o pipefail
O=gpurun_out/r2m
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_pool.py tests/test_gpu_preload.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "pool or stream_objects or preload or extract or zip_verify or dropin or stream or growth" > $O/new_tests.log 2>&1 || exit 1
ZCRC_PRELOAD_TABLE=$O/preload_table.jsonl timeout -k 10 300 python -u -m pytest tests/test_gpu_preload.py -q --timeout 200 --timeout-method thread > $O/preload.log 2>&1 || exit 2
timeout -k 10 200 python -u tools/host_threads.py > $O/host_threads.json 2> $O/host_threads.err || exit 3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 4
