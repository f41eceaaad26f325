# Per-rank kernel time of the 8-way (and 1-GPU) C4 frame for several code objects and chunk
# sizes: OBJS="default ab_objs/x.hsaco ..." KS="16 32 64" bash tools/gpu_tail_sweep.sh
set -o pipefail
mkdir -p gpurun_out
for k in ${KS:-16 32 64}; do
  for o in ${OBJS:-default}; do
    co=""; [ "$o" != default ] && co="--code-object $o"
    timeout -k 10 200 python tools/shard_sweep.py --chunk $k --worlds ${WORLDS:-8} $co > gpurun_out/ts.json 2>/dev/null || exit 1
    python3 -c "
import json; r = json.load(open('gpurun_out/ts.json'))
print('K=$k', '$o', 'full %.2f' % r['full_ms'], ' '.join('N=%s max %.2f sum %.1f' % (k[5:], v['max_ms'], v['sum_ms']) for k, v in r.items() if k.startswith('world')))"
  done
done
