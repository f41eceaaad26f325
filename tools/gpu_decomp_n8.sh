# Where the 8-way shard time goes at C4: the full frame with the N = 8 partition (K = 16, tail
# 128 x 4, and without the tail), then wave start / drain / end times (tools/wave_times.py) of
# the -DVCRT_WAVE_END_TIMES build in ab_objs/wt.hsaco (EXTRA=-DVCRT_WAVE_END_TIMES tools/mkab.sh wt).
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 200 python tools/shard_sweep.py --spp 1024 --worlds 8 --chunk 16 --tail 128 --tail-chunk 4 > gpurun_out/d_k16t.json 2>/dev/null &&
timeout -k 10 200 python tools/shard_sweep.py --spp 1024 --worlds 8 --chunk 16 --tail -1 > gpurun_out/d_k16n.json 2>/dev/null &&
VCRT_DEBUG_STATS=2 timeout -k 10 200 python tools/wave_times.py ab_objs/wt.hsaco --worlds 1,8 --ranks 2 > gpurun_out/d_wt.txt 2>&1 &&
cat gpurun_out/d_k16t.json gpurun_out/d_k16n.json gpurun_out/d_wt.txt
