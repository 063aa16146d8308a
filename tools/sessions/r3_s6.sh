#!/bin/bash
# Round 3, session 6 (second form): the drop-in's blocking H2D (HIP runtime
# log around it); plan probe; kernel A/B of the prefix guard and of the
# descriptor windows; kernel trace of the 1 KiB device path; GPU suite.
set -e -o pipefail
O=gpurun_out/r3s6; mkdir -p $O
gcc -O1 -Wall -I zipsfs_amd -I include tests/dropin/preload_main.c -o /tmp/preload_main -L zipsfs_amd -lzcrc \
    -Wl,-rpath,$PWD/zipsfs_amd -pthread -ldl
python3 -c "import sys; sys.path.insert(0,'.'); from oracle import oracle as o; o.payload(64<<20, 41).tofile('/tmp/e64.bin'); print('%08x' % o.payload_crc(64<<20, 41))" > /tmp/e64.crc
ZCRC_PRELOAD_REUSE=1 ZCRC_TRACE_HOST=1 timeout -k 10 180 /tmp/preload_main /tmp/e64.bin $(cat /tmp/e64.crc) 9 dropin > $O/preload_64_reuse.jsonl 2> $O/preload_64_reuse_trace.txt
AMD_LOG_LEVEL=4 ZCRC_TRACE_HOST=1 timeout -k 10 180 /tmp/preload_main /tmp/e64.bin $(cat /tmp/e64.crc) 4 dropin > $O/preload_64_amdlog.jsonl 2> $O/preload_64_amdlog.txt
for args in "100000 0" "1048576 1024" "262144 4096" "65536 16384"; do
  timeout -k 10 60 tools/plan_probe $args 50 >> $O/plan_probe.jsonl
done
for args in "65536 1048576 10" "100000 0 10" "262144 4096 10" "1048576 1024 10"; do
  echo "== guard $args" >> $O/crc_ab_guard.txt
  timeout -k 10 120 ablibs/ab/crc_ab_noguard_guard $args >> $O/crc_ab_guard.txt 2>&1
  echo "== nowin $args" >> $O/crc_ab_nowin.txt
  timeout -k 10 120 ablibs/ab/crc_ab_WT_nowin $args >> $O/crc_ab_nowin.txt 2>&1
done
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_small1k -- python3 tools/small_batches.py 10 1024,4096 > $O/prof_small1k.log 2>&1
