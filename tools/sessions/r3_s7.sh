#!/bin/bash
# Round 3, session 7: GPU suite (16-B small-list descriptors, prefix guard,
# prewarm's staged calls); the preload table; small batches against the
# previous plan; plan probe; kernel trace of the 1 KiB / 4 KiB device path.
set -e -o pipefail
O=gpurun_out/r3s7; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
gcc -O1 -Wall -I zipsfs_amd -I include tests/dropin/preload_main.c -o /tmp/preload_main -L zipsfs_amd -lzcrc \
    -Wl,-rpath,$PWD/zipsfs_amd -pthread -ldl
for kib in 4 1024 16384 65536 262144; do
  python3 -c "import sys; sys.path.insert(0,'.'); from oracle import oracle as o; o.payload($kib<<10, 41).tofile('/tmp/e$kib.bin'); print('%08x' % o.payload_crc($kib<<10, 41))" > /tmp/e$kib.crc
  ZCRC_TRACE_HOST=1 ZCRC_REF_LIB=$PWD/oracle/_ref/libref_cg_crc32_O0.so timeout -k 10 180 /tmp/preload_main /tmp/e$kib.bin $(cat /tmp/e$kib.crc) 7 none dropin stream stream_reg ref > $O/preload_$kib.jsonl 2> $O/preload_${kib}_trace.txt
done
timeout -k 10 300 python3 tools/small_batches.py 10 > $O/small_batches_new.jsonl
timeout -k 10 300 python3 tools/run_with_lib.py ablibs/oldplan/zipsfs_amd/libzcrc.so tools/small_batches.py 10 > $O/small_batches_old.jsonl
for args in "100000 0" "1048576 1024" "262144 4096" "65536 16384"; do
  timeout -k 10 60 tools/plan_probe $args 50 >> $O/plan_probe.jsonl
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_small -- python3 tools/small_batches.py 10 1024,4096 > $O/prof_small.log 2>&1
