# round-4 working batch: tests; A/B of the tree against round 3 and against the previous
# commit's kernel (without the fast divisions) under this tree's host (G = 4); the 8-way sweep
# with the default partition; the stats build's phases
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_run.sh test || exit 1
PREV=ab_objs/r3 OBJS="ab_objs/nodeal.hsaco" AB_CFGS="c4" ROUNDS=3 bash tools/gpu_run.sh ab || exit 1
SWEEP_REPS=2 WORLDS=2,4,8 bash tools/gpu_run.sh sweep || exit 1
bash tools/gpu_run.sh phases || exit 1
