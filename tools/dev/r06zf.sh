# round-6 final source: the driver's own bench command, and the default command twice more (spread)
set -u
OUT=gpurun_out/r06zf; mkdir -p $OUT
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver_cmd.log 2>&1 || exit $?
tail -1 $OUT/bench_driver_cmd.log | cut -c1-200
for k in 1 2; do timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-post > $OUT/bench_rep$k.log 2>&1 || exit $?; done
echo done-r06zf
