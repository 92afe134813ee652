# round-6: k_shadow split by packet layout (one register allocation each): GPU tests, variants on both
# scenes, and the product build's WRITE_SIZE / FETCH_SIZE on both scenes
set -u
bash tools/gpu_round.sh r06i tests variants s6var || exit $?
SETS="w:WRITE_SIZE;f:FETCH_SIZE" bash tools/pmc_sets.sh r06i_s5 main || exit $?
PMCARGS="--scene scene6 --width 3840 --height 2160 --spp 128" SETS="w:WRITE_SIZE;f:FETCH_SIZE" bash tools/pmc_sets.sh r06i_s6 main || exit $?
echo done-r06i
