#!/bin/bash
# Round 4, last check of the committed tree: the host inflate / preload /
# multi-device GPU tests after the buffer-retention change, the full suite,
# smoke.
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r4last; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
