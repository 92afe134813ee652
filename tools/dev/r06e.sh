# round-6 measurement pass: GPU tests, the far-cull variants on scene5 / scene6, and the WRITE_SIZE /
# FETCH_SIZE split of k_shadow (base, no walk, no leaf tests) on both scenes
set -u
VARS="base farlin0 farlin2" bash tools/gpu_round.sh r06e tests variants s6var || exit $?
SETS="w:WRITE_SIZE;f:FETCH_SIZE" bash tools/pmc_sets.sh r06e_s5 base nowalk noleaf || exit $?
PMCARGS="--scene scene6 --width 3840 --height 2160 --spp 128" SETS="w:WRITE_SIZE;f:FETCH_SIZE" bash tools/pmc_sets.sh r06e_s6 base nowalk noleaf || exit $?
echo done-r06e
