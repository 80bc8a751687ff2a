#!/bin/bash
# Build an A/B variant of libvstyler.so: scripts/build_diag.sh <name> <source.hip> "<-D flags>"
# -> video-styler_amd/vstyler/lib/diag_<name>/libvstyler.so (only <source> recompiled with the flags;
# load it with VSTYLER_LIB=... ; diagnostic builds are never the product library)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
N=$1; SRC=$2; FL=$3
OBJ=$R/build/diag_$N
mkdir -p $OBJ
cp -p $R/build/obj/*.o $OBJ/
rm -f $OBJ/${SRC%.hip}.o
make -s -C $R/video-styler_amd/csrc OUT_DIR=$R/video-styler_amd/vstyler/lib/diag_$N OBJ_DIR=$OBJ EXTRA="$FL" \
  $R/video-styler_amd/vstyler/lib/diag_$N/libvstyler.so
