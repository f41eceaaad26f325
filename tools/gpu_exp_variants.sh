# Timing-only experiments (images differ): cost of the canonical sin and of correctly rounded
# div/sqrt, by swapping in code objects built without them (tools: lib/variants/exp_*.hsaco).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/render_once.py --spp 256 --frames 2 > gpurun_out/x_base.json || exit 1
for v in fastsin fastdiv fastboth; do
  timeout -k 10 120 python tools/render_once.py --spp 256 --frames 2 --code-object vulkancomputeraytracing_amd/lib/variants/exp_$v.hsaco > gpurun_out/x_$v.json || exit 1
done
for v in base fastsin fastdiv fastboth; do python -c "import json;d=json.load(open('gpurun_out/x_$v.json'))[-1];print('$v', 'kernel_ms %.2f Msps %.0f segs %d' % (d['kernel_ms'], d['msamples_per_s'], d['segments']))"; done
