# round-6: the walk's tuning re-checked after the cone cull (scene5): deferred-round trigger,
# deferred queue depth, visit order, and the work-queue grab
set -u
VARS="base d48 tq3 so1" bash tools/gpu_round.sh r06za variants || exit $?
GRABS="1024 2048 8192" bash tools/gpu_round.sh r06za grabs || exit $?
echo done-r06za
