# round-6: the cone cull's point read apart from light_sample's: k_shadow time and WRITE_SIZE
set -u
bash tools/gpu_round.sh r06t benchq pmcw || exit $?
python3 tools/pmc_table.py gpurun_out/r06t/pmc_write > gpurun_out/r06t/pmcw_table.log 2>&1
echo done-r06t
