# C5 kernel placement A/B (run on the GPU box from the repo root): the flat scan with its tables
# in global memory (vcrt_trace_cull_flat_global) against the boxes in LDS
# (vcrt_trace_cull_flat_boxes, VCRT_CULL_LANE_TABLES=boxes); same bits required.
#   short: the stress scene at 4K, 64 spp, depth 50 (tools/ab.py, interleaved rounds)
#   full:  bench.py --config c5 with each placement
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S="--scene stress4096 --width 3840 --height 2160 --spp 64 --depth 50 --frames 2"
timeout -k 10 300 python tools/ab.py default default@VCRT_CULL_LANE_TABLES=boxes --rounds 2 $S \
  > gpurun_out/c5_ab.txt 2>&1 || { cat gpurun_out/c5_ab.txt; exit 1; }
grep round gpurun_out/c5_ab.txt
if [ -n "$FULL" ]; then
  timeout -k 10 200 python bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c5_global.json 2> gpurun_out/c5_global.err || exit 1
  VCRT_CULL_LANE_TABLES=boxes timeout -k 10 200 python bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c5_boxes.json 2> gpurun_out/c5_boxes.err || exit 1
  cat gpurun_out/c5_global.json gpurun_out/c5_boxes.json
fi
echo c5_done
