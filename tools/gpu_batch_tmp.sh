set -o pipefail
PREV=ab_objs/r3 OBJS="ab_objs/nodiv.hsaco ab_objs/hoist.hsaco" AB_CFGS="c4 c2" ROUNDS=3 bash tools/gpu_run.sh ab || exit 1
OBJS="ab_objs/hoist.hsaco" bash tools/gpu_run.sh pmcab || exit 1
