#!/bin/bash
# Round 3, session 6: the drop-in's blocking H2D (per-call trace, with and
# without a fresh segment per repetition); kernel trace of the 1 KiB device
# path (plan kernels, gaps, batch kernel with the small list).
set -e -o pipefail
O=gpurun_out/r3s6; mkdir -p $O
gcc -O1 -Wall -I zipsfs_amd -I include tests/dropin/preload_main.c -o /tmp/preload_main -L zipsfs_amd -lzcrc \
    -Wl,-rpath,$PWD/zipsfs_amd -pthread -ldl
for mib in 64 256; do
  python3 -c "import sys; sys.path.insert(0,'.'); from oracle import oracle as o; o.payload($mib<<20, 41).tofile('/tmp/e$mib.bin'); print('%08x' % o.payload_crc($mib<<20, 41))" > /tmp/e$mib.crc
  ZCRC_TRACE_HOST=1 timeout -k 10 180 /tmp/preload_main /tmp/e$mib.bin $(cat /tmp/e$mib.crc) 9 dropin > $O/preload_$mib.jsonl 2> $O/preload_${mib}_trace.txt
  ZCRC_PRELOAD_REUSE=1 ZCRC_TRACE_HOST=1 timeout -k 10 180 /tmp/preload_main /tmp/e$mib.bin $(cat /tmp/e$mib.crc) 9 dropin > $O/preload_${mib}_reuse.jsonl 2> $O/preload_${mib}_reuse_trace.txt
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_small1k -- python3 tools/small_batches.py 10 1024,4096 > $O/prof_small1k.log 2>&1
