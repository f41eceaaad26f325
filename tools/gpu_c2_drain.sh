# C2 (three-material, 800x450, 64 spp, depth 8): wave start / drain / end times of the
# diagnostics build (ab_objs/wt.hsaco: EXTRA=-DVCRT_WAVE_END_TIMES tools/mkab.sh wt), then the
# product kernel's time over chunk sizes, tails and workgroups per CU (render_once, 6 frames).
set -o pipefail
export TMPDIR=/tmp
C2="--scene three --width 800 --height 450 --spp 64 --depth 8"
VCRT_DEBUG_STATS=2 timeout -k 10 120 python tools/wave_times.py ab_objs/wt.hsaco $C2 --worlds 1 --ranks 1 > gpurun_out/c2_wt.txt 2>&1 || exit 1
VCRT_DEBUG_STATS=2 timeout -k 10 120 python tools/wave_times.py ab_objs/wt.hsaco $C2 --worlds 1 --ranks 1 --chunk 16 >> gpurun_out/c2_wt.txt 2>&1 || exit 1
VCRT_DEBUG_STATS=2 timeout -k 10 120 python tools/wave_times.py ab_objs/wt.hsaco $C2 --worlds 1 --ranks 1 --chunk 8 >> gpurun_out/c2_wt.txt 2>&1 || exit 1
cat gpurun_out/c2_wt.txt
for cfg in "--chunk 0" "--chunk 8" "--chunk 16" "--chunk 32" "--chunk 64" "--chunk 32 --tail 16 --tail-chunk 4" "--chunk 32 --tail 32 --tail-chunk 8" "--chunk 16 --tail 16 --tail-chunk 4" "--blocks-per-cu 4" "--blocks-per-cu 5" "--blocks-per-cu 3"; do
  timeout -k 10 120 python tools/render_once.py $C2 --frames 6 $cfg > gpurun_out/c2_r.json 2>/dev/null || exit 1
  python -c "
import json,sys; d=json.load(open('gpurun_out/c2_r.json')); ks=sorted(s['kernel_ms'] for s in d[1:])
print('$cfg'.ljust(40), 'K', d[-1]['accumulate_chunk'], 'tail', d[-1]['accumulate_tail'], d[-1]['accumulate_tail_chunk'], 'grid', d[-1]['grid_blocks'], 'ring', d[-1].get('ring_entries'), 'ms min %.3f med %.3f' % (ks[0], ks[len(ks)//2]))"
done
