#!/bin/bash
# Build libvstyler variants into tests/probes/var/<name>/ (git-ignored .so files that travel with
# gpurun) for same-box A/B runs with scripts/ab_probe.sh.
#   scripts/build_probe_variants.sh name1="-DFOO" name2="-DBAR" ...
set -e
R=$(cd $(dirname $0)/.. && pwd)
rm -rf $R/tests/probes/var
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  make -C $R/video-styler_amd/csrc -j8 OUT_DIR=$R/tests/probes/var/$name OBJ_DIR=$R/build/pvar_${name}_obj EXTRA="$flags" > /dev/null
  echo "built $name ($flags)"
done
