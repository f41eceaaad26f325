# Experiment batch: parity, sharding-coherence sweep, bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest_failed; exit 1; }
R="python tools/render_once.py --spp 256 --frames 2"
out=gpurun_out/sweep.jsonl; : > $out
for cfg in "full|" "r0w8s1|--rank 0 --world 8 --stripe 1" "r0w8s16|--rank 0 --world 8 --stripe 16" "r0w8s8|--rank 0 --world 8 --stripe 8" "r3w8s1|--rank 3 --world 8 --stripe 1" "stress_smem|--scene stress4096 --width 960 --height 540 --spp 16 --depth 50 --variant 2" "stress_lds|--scene stress4096 --width 960 --height 540 --spp 16 --depth 50 --variant 1"; do
  name=${cfg%%|*}; args=${cfg#*|}
  line=$(VCRT_DEBUG_STATS=1 timeout -k 10 180 $R $args 2>/dev/null | tail -1) || { echo "{\"name\": \"$name\", \"env\": \"\", \"failed\": true}" >> $out; exit 1; }
  echo "{\"name\": \"$name\", \"env\": \"stats\", \"r\": $line}" >> $out
done
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
echo all_done
