set -u
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/dev/dropin_debug.py > gpurun_out/dropin_debug.log 2>&1; echo "dropin rc=$?"
timeout -k 10 300 python3 tools/dev/count_deltas.py > gpurun_out/count_deltas.log 2>&1; echo "deltas rc=$?"
bash tools/gpu_round.sh r06d tests benchq variants s6var
