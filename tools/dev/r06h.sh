# round-6: who writes k_shadow's WRITE_SIZE on scene6 (vector-memory write instructions beside it)
set -u
S6="--scene scene6 --width 3840 --height 2160 --spp 128"
PMCARGS="$S6" SETS="w:WRITE_SIZE;s:SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INSTS_SMEM SQ_INSTS_VMEM_RD" bash tools/pmc_sets.sh r06h_s6 main nowalk noleaf slotfold0 || exit $?
SETS="s:SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INSTS_SMEM SQ_INSTS_VMEM_RD" bash tools/pmc_sets.sh r06h_s5 main || exit $?
PMCARGS="$S6" SETS="t:TCP_TCC_WRITE_REQ_sum TA_FLAT_WRITE_WAVEFRONTS_sum" bash tools/pmc_sets.sh r06h_s6t main || exit $?
echo done-r06h
