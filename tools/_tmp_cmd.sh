set -o pipefail
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "occupancy_cap or cost_order" > gpurun_out/occ_test.log 2>&1 || { tail -30 gpurun_out/occ_test.log; exit 1; }
tail -1 gpurun_out/occ_test.log
timeout -k 10 300 python tools/ab.py default default@VCRT_WORK_ORDER=cost --spp 1024 --rounds 3 --frames 3 > gpurun_out/c4cost.json &&
timeout -k 10 300 python tools/ab.py default default@VCRT_WORK_ORDER=cost --spp 256 --rounds 4 --frames 4 > gpurun_out/c3cost.json &&
WORLDS=8 SWEEP_REPS=2 SWEEP_ENVS="VCRT_WORK_ORDER=cost" bash tools/gpu_run.sh sweep
