# round-6 final source (slot-cull instance): k_shadow's PMC passes (scene5, scene6)
set -u
bash tools/gpu_round.sh r06zk pmcf pmcw pmcv pmcta pmcsum || exit $?
S6="--scene scene6 --width 3840 --height 2160 --spp 128"
PMCARGS="$S6" PMCKEY=scene6_3840x2160_n128_g1 bash tools/gpu_round.sh r06zk6 pmcf pmcw pmcv pmcta pmcsum || exit $?
echo done-r06zk
