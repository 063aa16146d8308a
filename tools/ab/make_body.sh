#!/bin/bash
# Strip zcrc_batch_kernel.h (from a git revision, or the working tree with
# "WT") down to a body that tools/crc_ab.hip can include inside its own
# namespace (measurement tooling).   tools/ab/make_body.sh <rev|WT> <out.h>
# When the kernel includes zcrc_small_kernel.h (round 2+), that body follows.
set -e -o pipefail
REV=$1
OUT=$2
CSRC="$(dirname "$0")/../../zipsfs_amd/csrc"
src() { if [ "$REV" = WT ]; then cat "$CSRC/$1"; else git show "$REV":zipsfs_amd/csrc/"$1"; fi; }
strip() { grep -v '^#pragma once' | grep -v '^#include "zcrc_' | grep -v '^namespace zcrc {' | grep -v '^}  // namespace zcrc'; }
SRC=$(src zcrc_batch_kernel.h)
printf '%s\n' "$SRC" | strip > "$OUT"
if printf '%s\n' "$SRC" | grep -q '^#include "zcrc_small_kernel.h"'; then
  src zcrc_small_kernel.h | strip >> "$OUT"
fi
