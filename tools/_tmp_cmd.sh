set -o pipefail
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "occupancy_cap or cost_order" > gpurun_out/occ_test.log 2>&1 || { tail -30 gpurun_out/occ_test.log; exit 1; }
tail -2 gpurun_out/occ_test.log
A="--scene three --width 800 --height 450 --spp 64 --depth 8 --frames 40 --rounds 4"
timeout -k 10 200 python tools/ab.py default default@VCRT_WORK_ORDER=static default@VCRT_MAX_BLOCKS_PER_CU=5 default@VCRT_MAX_BLOCKS_PER_CU=5,VCRT_WORK_ORDER=static default@VCRT_MAX_BLOCKS_PER_CU=4 $A > gpurun_out/c2occ.json &&
timeout -k 10 100 python tools/cost_map.py ab_objs/costmap.hsaco gpurun_out/cost_c2.npy --scene three --width 800 --height 450 --spp 64 --depth 8 &&
VCRT_DEBUG_STATS=2 VCRT_WORK_ORDER=static timeout -k 10 100 python tools/wave_times.py ab_objs/wt.hsaco --scene three --width 800 --height 450 --spp 64 --depth 8 --worlds 1 > gpurun_out/wt_c2.json
