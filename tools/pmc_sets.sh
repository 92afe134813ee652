#!/bin/bash
# PMC passes over k_shadow for several builds: tools/pmc_sets.sh <tag> <lib-variant|main>...
# Counter sets in $SETS ("name:C1 C2 ...;name2:..."); each pass is one rocprofv3 --pmc run of
# one bench frame (kernel trace off).  Stops at the first timeout/signal.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
python3 tools/standins.py scene5 scene6 > /dev/null
SETS=${SETS:-"sq:SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS"}
for v in "$@"; do
  if [ "$v" = main ]; then lib=""; else lib=$PWD/c-raytracer_amd/lib/var/$v/librtx.so; fi
  IFS=';' read -ra sets <<< "$SETS"
  for s in "${sets[@]}"; do
    name=${s%%:*}; ctrs=${s#*:}
    echo "=== $v $name ($(date +%T))"
    RTX_LIBRTX=$lib timeout -k 10 600 rocprofv3 --pmc $ctrs -d "$OUT/${v}_$name" -o run --output-format csv -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-count --no-post ${PMCARGS:-} > "$OUT/${v}_$name.log" 2>&1
    rc=$?; echo "=== rc=$rc"; tail -2 "$OUT/${v}_$name.log"
    if [ $rc -ge 124 ]; then exit $rc; fi
  done
done
