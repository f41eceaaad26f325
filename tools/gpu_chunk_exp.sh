# Chunk-size sensitivity (full frame, bench config) and the N=8 per-rank shard timings.
set -o pipefail
mkdir -p gpurun_out
for c in 8 16 32; do timeout -k 10 120 python tools/render_once.py --spp 1024 --chunk $c > gpurun_out/full_c$c.json || exit 1; done
timeout -k 10 300 python tools/shard_sweep.py --worlds 8 > gpurun_out/sweep8.json 2>/dev/null || exit 1
for c in 8 16 32; do python -c "import json;d=json.load(open('gpurun_out/full_c$c.json'));print('chunk', $c, 'kernel_ms %.1f resolve_ms %.2f Msps %.0f' % (d['kernel_ms'], d['resolve_ms'], d['msamples_per_s']))"; done
cat gpurun_out/sweep8.json
