# tools/gpu_small_prof.sh -- the small-batch table, then rocprofv3 kernel
# trace and HBM counters of the small-buffer paths on uniform 4 KiB batches,
# on one box (writes gpurun_out/sprof/)
set -o pipefail
R=$PWD
O=$R/gpurun_out/sprof
mkdir -p $O
timeout -k 10 300 python -u tools/small_batches.py 10 > $O/small_batches.jsonl 2> $O/small_batches.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/tools/small_uniform.py 4096 10 > $O/kt.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $R/tools/small_uniform.py 4096 3 > $O/fetch.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $R/tools/small_uniform.py 4096 3 > $O/write.log 2>&1 || exit 4
