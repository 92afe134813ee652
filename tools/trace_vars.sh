#!/bin/bash
# k_trace variants on scene6 2160p -n 128 and scene5 1080p -n 64 (one frame each after a warmup);
# stops at the first failing step.  usage: tools/trace_vars.sh <tag> <variant>...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1; shift; mkdir -p "$OUT"; export TMPDIR=/tmp
python3 tools/standins.py scene5 scene6 > /dev/null
for v in "$@"; do
  for sc in scene6 scene5; do
    if [ $sc = scene6 ]; then args="--scene scene6 --width 3840 --height 2160 --spp 128"; else args=""; fi
    RTX_LIBRTX=$PWD/c-raytracer_amd/lib/var/$v/librtx.so timeout -k 10 300 python3 bench.py $args --steps 1 --warmup 1 \
      --no-cpu-baseline --no-count --no-post > "$OUT/${sc}_$v.log" 2>&1
    rc=$?; echo "$sc $v rc=$rc $(grep -o '"trace_ms": [0-9.]*' "$OUT/${sc}_$v.log")"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
