#!/bin/bash
# Round 3, session 5: new split plan (coalesced count + ballot-ranked
# scatter): GPU suite incl. the plan-vs-model test, uniform small batches and
# configs 3/4 against the previous plan's library, plan kernel durations, and
# the drop-in's slowest queueing call per staged call.
set -e -o pipefail
O=gpurun_out/r3s5; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python3 tools/small_batches.py 10 > $O/small_batches_new.jsonl
timeout -k 10 300 python3 tools/run_with_lib.py ablibs/oldplan/zipsfs_amd/libzcrc.so tools/small_batches.py 10 > $O/small_batches_old.jsonl
timeout -k 10 600 tools/ab_libs.sh $O/ab_plan_c4.jsonl 4 3 20 zipsfs_amd/libzcrc.so ablibs/oldplan/zipsfs_amd/libzcrc.so
timeout -k 10 600 tools/ab_libs.sh $O/ab_plan_c3.jsonl 3 2 20 zipsfs_amd/libzcrc.so ablibs/oldplan/zipsfs_amd/libzcrc.so
gcc -O1 -Wall -I zipsfs_amd -I include tests/dropin/preload_main.c -o /tmp/preload_main -L zipsfs_amd -lzcrc \
    -Wl,-rpath,$PWD/zipsfs_amd -pthread -ldl
for mib in 64 256; do
  python3 -c "import sys; sys.path.insert(0,'.'); from oracle import oracle as o; o.payload($mib<<20, 41).tofile('/tmp/e$mib.bin'); print('%08x' % o.payload_crc($mib<<20, 41))" > /tmp/e$mib.crc
  ZCRC_TRACE_HOST=1 timeout -k 10 180 /tmp/preload_main /tmp/e$mib.bin $(cat /tmp/e$mib.crc) 9 dropin > $O/preload_$mib.jsonl 2> $O/preload_${mib}_trace.txt
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -- python3 bench.py --config 4 --no-cpu-baseline > $O/prof_c4.log 2>&1
