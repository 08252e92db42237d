#!/bin/bash
# Build liblsmck.so of a commit (or of the work tree: "WT") into
# lsm_storage_engine_amd/ab/<name>.so for same-box A/B runs (tools/gpu_ab_libs.sh),
# with the stream kernel's diagnostic ablations (crc_ablate 2, 4..10) compiled in.
#   [EXTRA=-DFLAG] tools/build_ab.sh <name> <commit|WT>
set -e
NAME=$1; REV=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
D=/tmp/lsmck_ab_$NAME
rm -rf $D; mkdir -p $D
if [ "$REV" = WT ]; then
  cp -r $ROOT/include $D/; mkdir -p $D/lsm_storage_engine_amd; cp -r $ROOT/lsm_storage_engine_amd/csrc $D/lsm_storage_engine_amd/
  rm -rf $D/lsm_storage_engine_amd/csrc/build
else
  git -C $ROOT archive $REV include lsm_storage_engine_amd/csrc | tar -x -C $D
fi
mkdir -p $ROOT/lsm_storage_engine_amd/ab
make -s -j8 -C $D/lsm_storage_engine_amd/csrc EXTRA="-DLSMCK_AB_ABLATIONS -DLSMCK_DIAG $EXTRA" OUT=$ROOT/lsm_storage_engine_amd/ab/$NAME.so $ROOT/lsm_storage_engine_amd/ab/$NAME.so 2>&1 | grep -v hip-link || true
ls -la $ROOT/lsm_storage_engine_amd/ab/$NAME.so
