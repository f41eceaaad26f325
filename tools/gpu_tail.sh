set -o pipefail
for c in 8 16; do for w in 1 8; do
VCRT_DEBUG_STATS=1 timeout -k 10 120 python tools/render_once.py --spp 1024 --chunk $c --world $w --rank 0 > gpurun_out/tail_${c}_$w.json || exit 1
python -c "
import json; st=json.load(open('gpurun_out/tail_${c}_$w.json')); d=st['debug']
print('chunk $c world $w kernel_ms %.2f  end spread (last-first) %.3f ms  mean-end to last %.3f ms' % (st['kernel_ms'], (d[4]-d[5])/1e5, (d[4]-d[6]*256/d[7])/1e5))"
done; done
