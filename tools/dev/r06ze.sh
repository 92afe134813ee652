# round-6: the cull and group suites after the readback moved to the context's stream
set -u
mkdir -p gpurun_out/r06ze
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_cull.py tests/test_gpu_group.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06ze/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r06ze/tests.log; exit $rc
