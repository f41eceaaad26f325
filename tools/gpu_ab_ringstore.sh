# Ring entries that took every chunk of their pixel store instead of adding atomically
# (kFlagRingStore): the parity suite on the new build, then A/B of ab_objs/base.hsaco (HEAD
# before the change) against ab_objs/new.hsaco on C2, C3 and the stress scene, and C2's wave
# end times.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 120 python tools/ab.py ab_objs/base.hsaco ab_objs/new.hsaco --rounds 3 --frames 6 --scene three --width 800 --height 450 --spp 64 --depth 8 > gpurun_out/ab_c2.json 2>&1 || { cat gpurun_out/ab_c2.json; exit 1; }
timeout -k 10 200 python tools/ab.py ab_objs/base.hsaco ab_objs/new.hsaco --rounds 2 --spp 256 > gpurun_out/ab_c3.json 2>&1 || { cat gpurun_out/ab_c3.json; exit 1; }
timeout -k 10 200 python tools/ab.py ab_objs/base.hsaco ab_objs/new.hsaco --rounds 2 --scene stress4096 --width 3840 --height 2160 --spp 32 --depth 50 > gpurun_out/ab_c5.json 2>&1 || { cat gpurun_out/ab_c5.json; exit 1; }
timeout -k 10 120 python bench.py --config c2 > gpurun_out/bench_c2_new.json 2>/dev/null || exit 1
cat gpurun_out/ab_c2.json gpurun_out/ab_c3.json gpurun_out/ab_c5.json gpurun_out/bench_c2_new.json
