set -o pipefail
bash tools/gpu_run.sh test || exit 1
A="--scene three --width 800 --height 450 --spp 64 --depth 8 --frames 40 --rounds 4"
timeout -k 10 250 python tools/ab.py default default@VCRT_WORK_ORDER=static default@VCRT_MAX_BLOCKS_PER_CU=6 $A > gpurun_out/c2final.json &&
CFGS=c2 bash tools/gpu_run.sh bench &&
VCRT_DEBUG_STATS=2 timeout -k 10 100 python tools/wave_times.py ab_objs/wt.hsaco --scene three --width 800 --height 450 --spp 64 --depth 8 --worlds 1 > gpurun_out/wt_c2c.json
