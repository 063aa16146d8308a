#!/bin/bash
# Round 3, session 3: GPU suite (registered/pageable streams, prewarm, the
# preload harness with the no-CRC and registered modes), the drop-in hold
# time per phase (ZCRC_TRACE_HOST), same-process kernel A/B of the round-1
# kernel against each round-2 revision on config 3, the default bench with
# the region-event kernel timing, and its rocprofv3 kernel trace.
set -e -o pipefail
O=gpurun_out/r3s3; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
gcc -O1 -Wall -I zipsfs_amd -I include tests/dropin/preload_main.c -o /tmp/preload_main -L zipsfs_amd -lzcrc \
    -Wl,-rpath,$PWD/zipsfs_amd -pthread -ldl
for mib in 16 64 256; do
  python3 -c "import sys; sys.path.insert(0,'.'); from oracle import oracle as o; o.payload($mib<<20, 41).tofile('/tmp/e$mib.bin'); print('%08x' % o.payload_crc($mib<<20, 41))" > /tmp/e$mib.crc
  ZCRC_TRACE_HOST=1 ZCRC_REF_LIB=$PWD/oracle/_ref/libref_cg_crc32_O0.so timeout -k 10 120 /tmp/preload_main /tmp/e$mib.bin $(cat /tmp/e$mib.crc) 5 none dropin stream stream_reg > $O/preload_$mib.jsonl 2> $O/preload_${mib}_trace.txt
done
for b in bfefb3c 8e121b5 ee983f1 58086df 6887c22 WT; do
  timeout -k 10 120 ablibs/ab/crc_ab_r1_$b 65536 1048576 10 > $O/crc_ab_r1_$b.txt 2>&1
done
timeout -k 10 300 python3 bench.py > $O/bench_default.jsonl 2> $O/bench_default.err
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_default -- python3 bench.py --no-cpu-baseline > $O/prof_default.log 2>&1
