set -o pipefail
timeout -k 10 300 python tools/ab.py default default@desc.accumulate_chunk=32 default@desc.accumulate_chunk=16,VCRT_FETCH_MIN=8,VCRT_FETCH_WAIT=2 --spp 256 --rounds 4 --frames 3 > gpurun_out/c3k.json &&
PMC_CFG=c3 bash tools/gpu_run.sh trafficab
