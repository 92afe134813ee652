# round-6: the lane-slot cone cull in its own kernel instance (PATH 3, RTX_OPT_SHADOW_CULL 2): the
# cull / slot / frame suites; scene6 and scene5 at the default; scene5 in 16-lane slots with and
# without the slot cull
set -u
OUT=gpurun_out/r06zj; mkdir -p $OUT
python3 tools/standins.py scene5 scene6 > /dev/null
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_cull.py tests/test_gpu_slots.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 600 python3 bench.py --scene scene6 --width 3840 --height 2160 --spp 128 --steps 1 --warmup 1 --no-cpu-baseline --no-post --no-count > $OUT/s6.log 2>&1 || exit $?
timeout -k 10 600 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-post --no-count > $OUT/s5.log 2>&1 || exit $?
timeout -k 10 600 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-post --no-count --shadow-slot 16 > $OUT/s5_slot16.log 2>&1 || exit $?
timeout -k 10 600 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-post --no-count --shadow-slot 16 --cull-slots > $OUT/s5_slot16_cull.log 2>&1 || exit $?
echo done-r06zj
