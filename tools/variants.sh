#!/bin/bash
# Build librtx.so measurement variants under c-raytracer_amd/lib/var/<name>/ (git-ignored, they
# travel to the GPU box): tools/variants.sh name:"-DFLAG=1 -DOTHER=2" ...  (clears old variants)
set -eu
cd "$(dirname "$0")/../c-raytracer_amd"
rm -rf lib/var
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  make -s rtx LIB=lib/var/$name EXTRA="$flags" > /tmp/var_$name.log 2>&1 || { tail -20 /tmp/var_$name.log; exit 1; }
  find lib/var/$name -name '*.o' -delete
  echo "built $name ($flags)"
done
