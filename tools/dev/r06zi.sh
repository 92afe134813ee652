# round-6: the lane-slot cull as a runtime option (RTX_OPT_SHADOW_CULL 2, default 1): its tests, and
# scene6 / scene5 with the code present but the option at its default, against the build without it
set -u
mkdir -p gpurun_out/r06zi
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_cull.py tests/test_gpu_slots.py -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06zi/tests.log 2>&1 || { tail -30 gpurun_out/r06zi/tests.log; exit 1; }
tail -2 gpurun_out/r06zi/tests.log
VARS="sc0 rt" bash tools/gpu_round.sh r06zi s6var variants || exit $?
echo done-r06zi
