set -o pipefail
O=gpurun_out/r2ae
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_host_pool.py tests/test_gpu_dropin.py -x -v -s --timeout 300 --timeout-method thread > $O/pool_tests.log 2>&1 || exit 1
