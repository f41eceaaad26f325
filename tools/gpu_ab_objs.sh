# A/B timing of code objects against the package's own build (run on the GPU box from the repo
# root): OBJS="ab_objs/a.hsaco ab_objs/b.hsaco" [STRESS=1] [C2=1] bash tools/gpu_ab_objs.sh
# tools/ab.py renders each configuration with every object in interleaved rounds and requires
# bit-identical images. C4 workload (1080p, 1024 spp, depth 10), the stress scene at 4K 64 spp
# depth 50, and the C2 workload (three-material, 800x450, 64 spp, depth 8).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${ROUNDS:-3}
timeout -k 10 400 python tools/ab.py default $OBJS --rounds $R --spp 1024 --frames 2 \
  > gpurun_out/ab_c4.txt 2>&1 || { cat gpurun_out/ab_c4.txt; exit 1; }
grep round gpurun_out/ab_c4.txt
if [ -n "$STRESS" ]; then
  timeout -k 10 400 python tools/ab.py default $OBJS --rounds 2 --scene stress4096 --width 3840 \
    --height 2160 --spp 64 --depth 50 --frames 2 > gpurun_out/ab_c5.txt 2>&1 || { cat gpurun_out/ab_c5.txt; exit 1; }
  grep round gpurun_out/ab_c5.txt
fi
if [ -n "$C2" ]; then
  timeout -k 10 200 python tools/ab.py default $OBJS --rounds 3 --scene three --width 800 \
    --height 450 --spp 64 --depth 8 --frames 20 > gpurun_out/ab_c2.txt 2>&1 || { cat gpurun_out/ab_c2.txt; exit 1; }
  grep round gpurun_out/ab_c2.txt
fi
echo ab_done
