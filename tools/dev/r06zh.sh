# round-6: the cone cull on the lane-slot path (RTX_SH_SLOTCULL): its tests, then scene6 and scene5
# with and without it
set -u
mkdir -p gpurun_out/r06zh
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_cull.py tests/test_gpu_slots.py -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06zh/tests.log 2>&1 || { tail -30 gpurun_out/r06zh/tests.log; exit 1; }
tail -2 gpurun_out/r06zh/tests.log
VARS="sc0 sc1" bash tools/gpu_round.sh r06zh s6var variants || exit $?
echo done-r06zh
