set -o pipefail
O=gpurun_out/r2aa
mkdir -p $O
export TMPDIR=/tmp
for u in 65536 131072 262144 1048576; do
  ZCRC_DYN_UNIT=$u timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$u -o b -- python3 bench.py --config 4 --steps 3 --warmup 1 --no-cpu-baseline > $O/fetch_$u.log 2>&1 || exit 1
done
