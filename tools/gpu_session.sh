set -o pipefail
O=gpurun_out/r2af
mkdir -p $O
for shape in "4096 65536 40" "100000 0 20" "16384 1048576 10" "1048576 1024 20" "262144 4096 20"; do
  timeout -k 10 200 tools/crc_ab $shape >> $O/crc_ab.txt 2>&1 || exit 1
done
timeout -k 10 200 tools/c2_probe 48 > $O/c2_probe.txt 2>&1 || exit 2
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/parity.log 2>&1 || exit 3
