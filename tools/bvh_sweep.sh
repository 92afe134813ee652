#!/bin/bash
# Shadow-pass time vs BVH builder parameters (RTX_BVH_LEAF / _CT / _CI), one frame each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; mkdir -p "$OUT"; export TMPDIR=/tmp
python3 tools/standins.py scene5 > /dev/null
shift
for cfg in "$@"; do  # leaf:ct:ci
  IFS=: read -r L T I <<< "$cfg"
  echo "=== leaf=$L ct=$T ci=$I"
  RTX_BVH_LEAF=$L RTX_BVH_CT=$T RTX_BVH_CI=$I timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-post > "$OUT/bvh_${L}_${T}_${I}.log" 2>&1
  rc=$?; echo "rc=$rc"; if [ $rc -ge 124 ]; then exit $rc; fi
done
