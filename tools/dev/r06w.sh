# round-6: walks starting at the root children the point's cones meet (RTX_SH_ROOTSKIP): the cull
# tests on that build, then k_shadow with and without it
set -u
mkdir -p gpurun_out/r06w
RTX_LIBRTX=$PWD/c-raytracer_amd/lib/var/rs1/librtx.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_cull.py -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06w/culltests_rs1.log 2>&1 || { tail -30 gpurun_out/r06w/culltests_rs1.log; exit 1; }
tail -3 gpurun_out/r06w/culltests_rs1.log
VARS="rs0 rs1" bash tools/gpu_round.sh r06w variants || exit $?
echo done-r06w
