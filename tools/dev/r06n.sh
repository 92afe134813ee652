# round-6: the group tests with the RCCL self-exchange transport, then k_shadow's PMC passes on
# the committed source (scene5 and scene6) for profiles/pmc_k_shadow.json
set -u
bash tools/gpu_round.sh r06n grouptests || exit $?
grep -q "rccl_self.*PASSED" gpurun_out/r06n/grouptests.log || exit 5
bash tools/gpu_round.sh r06n pmcf pmcw pmcv pmcta pmcsum || exit $?
S6="--scene scene6 --width 3840 --height 2160 --spp 128"
PMCARGS="$S6" PMCKEY=scene6_3840x2160_n128_g1 bash tools/gpu_round.sh r06n6 pmcf pmcw pmcv pmcta pmcsum || exit $?
echo done-r06n
