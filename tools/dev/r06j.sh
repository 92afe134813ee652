# round-6 final PMC of k_shadow (source as committed): scene5 bench frame and scene6 configs[4], the
# fetch / write / VALU-issue / texture-path passes and the summary (profiles/pmc_k_shadow.json), then
# the VALU passes of the one-leaf-per-round build on scene6
set -u
bash tools/gpu_round.sh r06j pmcf pmcw pmcv pmcta pmcsum || exit $?
S6="--scene scene6 --width 3840 --height 2160 --spp 128"
PMCARGS="$S6" PMCKEY=scene6_3840x2160_n128_g1 bash tools/gpu_round.sh r06j6 pmcf pmcw pmcv pmcta pmcsum || exit $?
PMCARGS="$S6" VARS="l2d2off" bash tools/gpu_round.sh r06j6v pmcvars || exit $?
echo done-r06j
