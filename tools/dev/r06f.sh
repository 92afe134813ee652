# round-6: the spill-free walk (lane-stack addresses formed at use) against its variants, scene5 and
# scene6, then the WRITE_SIZE / FETCH_SIZE of the product build on both scenes
set -u
bash tools/gpu_round.sh r06f variants s6var || exit $?
SETS="w:WRITE_SIZE;f:FETCH_SIZE" bash tools/pmc_sets.sh r06f_s5 main || exit $?
PMCARGS="--scene scene6 --width 3840 --height 2160 --spp 128" SETS="w:WRITE_SIZE;f:FETCH_SIZE" bash tools/pmc_sets.sh r06f_s6 main || exit $?
echo done-r06f
