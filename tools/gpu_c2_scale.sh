# C2 at 4x and 16x the samples (spp 256, 1024): does the kernel time scale with the work (a
# throughput limit) or keep a fixed tail? Plus wave lifetimes at spp 256 (ab_objs/wt.hsaco).
set -o pipefail
export TMPDIR=/tmp
for spp in 64 256 1024; do
  timeout -k 10 120 python tools/render_once.py --scene three --width 800 --height 450 --depth 8 --spp $spp --frames 4 > gpurun_out/c2s.json 2>/dev/null || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/c2s.json')); ks=sorted(s['kernel_ms'] for s in d[1:])
print('spp $spp K', d[-1]['accumulate_chunk'], 'tail', d[-1]['accumulate_tail'], 'ms min %.3f' % ks[0], 'Msps %.0f' % (d[-1]['samples']/ks[0]/1e3), 'segments', d[-1]['segments'])"
done
VCRT_DEBUG_STATS=2 timeout -k 10 120 python tools/wave_times.py ab_objs/wt.hsaco --scene three --width 800 --height 450 --spp 256 --depth 8 --worlds 1 --ranks 1 2>/dev/null || exit 1
