set -o pipefail
bash tools/gpu_run.sh test || exit 1
PREV=ab_objs/r3 OBJS="ab_objs/hoist.hsaco" AB_CFGS="c4 c2 c3 stress" ROUNDS=2 bash tools/gpu_run.sh ab || exit 1
