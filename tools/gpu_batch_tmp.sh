set -o pipefail
bash tools/gpu_run.sh test profile || exit 1
SWEEP_REPS=1 WORLDS=2,4,8 bash tools/gpu_run.sh sweep || exit 1
bash tools/gpu_run.sh phases || exit 1
