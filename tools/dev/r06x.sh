# round-6 final: the GPU suite and smoke on the final source, the default bench (its PMC record now
# matches the source), and the no-walk build's k_shadow (everything but the tree walks)
set -u
bash tools/gpu_round.sh r06x smoke tests bench nowalk || exit $?
echo done-r06x
