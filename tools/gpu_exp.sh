# Experiment batch (round 1): microbenchmark, parity, kernel-variant sweep with diagnostics.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/microbench_valu > gpurun_out/microbench_valu.txt 2>&1 || exit 1
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest_failed; exit 1; }
R="python tools/render_once.py --spp 64 --frames 2"
out=gpurun_out/sweep.jsonl; : > $out
for cfg in "lds|--variant 1" "smem|--variant 2" "lds_noslp|--variant 1 --code-object vulkancomputeraytracing_amd/lib/variants/noslp.hsaco" "smem_noslp|--variant 2 --code-object vulkancomputeraytracing_amd/lib/variants/noslp.hsaco" "lds_b4|--variant 1 --blocks-per-cu 4" "smem_b8|--variant 2 --blocks-per-cu 8"; do
  name=${cfg%%|*}; args=${cfg#*|}
  for env in "VCRT_DEBUG_STATS=0" "VCRT_DEBUG_STATS=1" "VCRT_DEBUG_STATS=1 VCRT_WORK_ORDER=reverse"; do
    line=$(env $env timeout -k 10 180 $R $args 2>/dev/null | tail -1) || { echo "{\"name\": \"$name\", \"env\": \"$env\", \"failed\": true}" >> $out; exit 1; }
    echo "{\"name\": \"$name\", \"env\": \"$env\", \"r\": $line}" >> $out
  done
done
echo all_done
