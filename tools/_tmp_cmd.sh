set -o pipefail
WORLDS=8 SWEEP_REPS=2 SWEEP_ENVS="VCRT_WORK_ORDER=costtail" bash tools/gpu_run.sh sweep
