#!/bin/bash
# Strip zcrc_batch_kernel.h (from a git revision, or the working tree with
# "WT") down to a body that tools/crc_ab.hip can include inside its own
# namespace (measurement tooling).   tools/ab/make_body.sh <rev|WT> <out.h>
set -e -o pipefail
REV=$1
OUT=$2
if [ "$REV" = WT ]; then SRC=$(cat "$(dirname "$0")/../../zipsfs_amd/csrc/zcrc_batch_kernel.h"); else SRC=$(git show "$REV":zipsfs_amd/csrc/zcrc_batch_kernel.h); fi
printf '%s\n' "$SRC" | grep -v '^#pragma once' | grep -v '^#include "zcrc_' | grep -v '^namespace zcrc {' | grep -v '^}  // namespace zcrc' > "$OUT"
