# The queue's last blocks in quarters (split_blocks, VCRT_SPLIT_BLOCKS): the parity suite on the
# new build, then A/B of ab_objs/base.hsaco (before) against the package's code object at
# several split counts on C2, C3 and C4 8-way shards; C2 wave lifetimes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
C2="--scene three --width 800 --height 450 --spp 64 --depth 8"
timeout -k 10 150 python tools/ab.py ab_objs/base.hsaco default@VCRT_SPLIT_BLOCKS=0 default default@VCRT_SPLIT_BLOCKS=3000 default@VCRT_SPLIT_BLOCKS=12000 --rounds 3 --frames 6 $C2 > gpurun_out/abs_c2.json 2>&1 || { cat gpurun_out/abs_c2.json; exit 1; }
timeout -k 10 200 python tools/ab.py ab_objs/base.hsaco default@VCRT_SPLIT_BLOCKS=0 default default@VCRT_SPLIT_BLOCKS=12000 --rounds 2 --spp 256 > gpurun_out/abs_c3.json 2>&1 || { cat gpurun_out/abs_c3.json; exit 1; }
VCRT_DEBUG_STATS=2 timeout -k 10 120 python tools/wave_times.py ab_objs/wt.hsaco $C2 --worlds 1 --ranks 1 > gpurun_out/abs_wt.txt 2>/dev/null || exit 1
cat gpurun_out/abs_wt.txt
for sb in 0 -; do
  if [ "$sb" = "-" ]; then unset VCRT_SPLIT_BLOCKS; else export VCRT_SPLIT_BLOCKS=$sb; fi
  timeout -k 10 200 python tools/shard_sweep.py --spp 1024 --worlds 8 > gpurun_out/abs_n8_$sb.json 2>/dev/null || exit 1
  echo "split $sb"; tail -3 gpurun_out/abs_n8_$sb.json
done
