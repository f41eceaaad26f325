# Experiment batch: parity, kernel-variant sweep with diagnostics, full bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest_failed; exit 1; }
R="python tools/render_once.py --spp 256 --frames 2"
out=gpurun_out/sweep.jsonl; : > $out
for cfg in "lds|--variant 1" "smem|--variant 2" "smem_noslp|--variant 2 --code-object vulkancomputeraytracing_amd/lib/variants/noslp.hsaco" "smem_c16|--variant 2 --chunk 16" "smem_c64|--variant 2 --chunk 64" "smem_c256|--variant 2 --chunk 256" "smem_b6|--variant 2 --blocks-per-cu 6" "smem_b8|--variant 2 --blocks-per-cu 8"; do
  name=${cfg%%|*}; args=${cfg#*|}
  for env in "VCRT_DEBUG_STATS=0" "VCRT_DEBUG_STATS=1"; do
    line=$(env $env timeout -k 10 180 $R $args 2>/dev/null | tail -1) || { echo "{\"name\": \"$name\", \"env\": \"$env\", \"failed\": true}" >> $out; exit 1; }
    echo "{\"name\": \"$name\", \"env\": \"$env\", \"r\": $line}" >> $out
  done
done
timeout -k 10 300 python bench.py --steps 2 --warmup 1 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
echo all_done
