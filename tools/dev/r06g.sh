# round-6: attenuation formed before the walk (one float across it) against variants, scene5 and scene6,
# counting renders of both configs (leaf rounds, stack spills), PMC write/fetch of the product build
set -u
bash tools/gpu_round.sh r06g variants s6var || exit $?
timeout -k 10 600 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-post --verbose > gpurun_out/r06g/count_s5.log 2>&1 || exit $?
timeout -k 10 600 python3 bench.py --scene scene6 --width 3840 --height 2160 --spp 128 --steps 1 --warmup 1 --no-cpu-baseline --no-post --verbose > gpurun_out/r06g/count_s6.log 2>&1 || exit $?
SETS="w:WRITE_SIZE;f:FETCH_SIZE" bash tools/pmc_sets.sh r06g_s5 main || exit $?
PMCARGS="--scene scene6 --width 3840 --height 2160 --spp 128" SETS="w:WRITE_SIZE;f:FETCH_SIZE" bash tools/pmc_sets.sh r06g_s6 main || exit $?
echo done-r06g
