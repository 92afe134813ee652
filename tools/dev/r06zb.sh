# round-6: the cone around the emitter itself (sphere radius / triangle circumsphere) instead of its
# world box's sphere: the cull and frame suites, then the bench frame
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06zb; mkdir -p $OUT; export TMPDIR=/tmp
python3 tools/standins.py scene5 scene6 > /dev/null
run() { local name=$1 to=$2; shift 2; echo "=== $name"; timeout -k 10 $to "$@" > $OUT/$name.log 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -3 $OUT/$name.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
run culltests 600 python3 -u -m pytest tests/test_gpu_cull.py -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider
run ptests 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_frame.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider
run bench 600 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-post --verbose
echo done-r06zb
