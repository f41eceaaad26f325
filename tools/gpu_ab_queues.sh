# Eight work queues (one per XCD) against the single counter: the parity suite on the new build,
# then A/B of ab_objs/base.hsaco (single queue) against the package's code object on C2, C3,
# C4 and the C4 8-way shards, and the stress scene.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
C2="--scene three --width 800 --height 450 --spp 64 --depth 8"
timeout -k 10 150 python tools/ab.py ab_objs/base.hsaco default --rounds 3 --frames 6 $C2 > gpurun_out/abq_c2.json 2>&1 || { cat gpurun_out/abq_c2.json; exit 1; }
timeout -k 10 200 python tools/ab.py ab_objs/base.hsaco default --rounds 2 --spp 256 > gpurun_out/abq_c3.json 2>&1 || { cat gpurun_out/abq_c3.json; exit 1; }
timeout -k 10 200 python tools/ab.py ab_objs/base.hsaco default --rounds 2 --spp 1024 > gpurun_out/abq_c4.json 2>&1 || { cat gpurun_out/abq_c4.json; exit 1; }
timeout -k 10 200 python tools/ab.py ab_objs/base.hsaco default --rounds 2 --scene stress4096 --width 3840 --height 2160 --spp 32 --depth 50 > gpurun_out/abq_c5.json 2>&1 || { cat gpurun_out/abq_c5.json; exit 1; }
for rep in 1 2; do
  timeout -k 10 200 python tools/shard_sweep.py --spp 1024 --worlds 8 --code-object ab_objs/base.hsaco > gpurun_out/abq_n8_base_$rep.json 2>/dev/null || exit 1
  timeout -k 10 200 python tools/shard_sweep.py --spp 1024 --worlds 8 > gpurun_out/abq_n8_new_$rep.json 2>/dev/null || exit 1
  echo "base"; tail -1 gpurun_out/abq_n8_base_$rep.json; echo "new"; tail -1 gpurun_out/abq_n8_new_$rep.json
done
