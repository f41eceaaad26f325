set -o pipefail
A="--scene three --width 800 --height 450 --spp 64 --depth 8 --frames 40 --rounds 4"
timeout -k 10 200 python tools/ab.py default default@VCRT_MAX_BLOCKS_PER_CU=5 default@VCRT_MAX_BLOCKS_PER_CU=4 default@VCRT_MAX_BLOCKS_PER_CU=3 default@desc.accumulate_tail=16,desc.accumulate_tail_chunk=4 default@VCRT_MAX_BLOCKS_PER_CU=5,desc.accumulate_tail=16,desc.accumulate_tail_chunk=4 $A > gpurun_out/c2occ.json &&
timeout -k 10 200 python tools/ab.py default default@VCRT_MAX_BLOCKS_PER_CU=4 --spp 1024 --rounds 2 --frames 2 > gpurun_out/c4occ.json
