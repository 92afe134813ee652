# round-6: k_shadow's PMC passes on the final source (scene5, scene6), and scene6 with 64-lane
# packets (the cone cull's reach there)
set -u
bash tools/gpu_round.sh r06v pmcf pmcw pmcv pmcta pmcsum || exit $?
S6="--scene scene6 --width 3840 --height 2160 --spp 128"
PMCARGS="$S6" PMCKEY=scene6_3840x2160_n128_g1 bash tools/gpu_round.sh r06v6 pmcf pmcw pmcv pmcta pmcsum || exit $?
SLOTS="64" bash tools/gpu_round.sh r06v6s s6slot || exit $?
echo done-r06v
