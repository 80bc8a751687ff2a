#!/bin/bash
# Build libvstyler variants (EXTRA flag sets) into build/var_<name>/ for same-box A/B timing.
# usage: scripts/build_variants.sh name1="-DFOO" name2="-DBAR -DBAZ" ...
set -e
R=$(cd $(dirname $0)/.. && pwd)
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  make -C $R/video-styler_amd/csrc -j8 OUT_DIR=$R/build/var_$name OBJ_DIR=$R/build/var_${name}_obj EXTRA="$flags" > /dev/null
  echo "built $name ($flags)"
done
