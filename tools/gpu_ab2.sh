# Parity suite of the current tree, the flat-pass stats, then A/B timing of exp/ab/base.hsaco vs
# exp/ab/new.hsaco on the final scene (1080p 256 spp) and the stress scene (4K 32 spp depth 50).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
bash tools/gpu_phases.sh > gpurun_out/phases.txt 2>&1 || { cat gpurun_out/phases.txt; exit 1; }
tail -3 gpurun_out/phases.txt
timeout -k 10 200 python tools/ab.py exp/ab/base.hsaco exp/ab/new.hsaco --rounds 3 > gpurun_out/ab_f.json 2>&1 || { cat gpurun_out/ab_f.json; exit 1; }
timeout -k 10 200 python tools/ab.py exp/ab/base.hsaco exp/ab/new.hsaco --rounds 2 --scene stress4096 --width 3840 --height 2160 --spp 32 --depth 50 > gpurun_out/ab_s.json 2>&1 || { cat gpurun_out/ab_s.json; exit 1; }
cat gpurun_out/ab_f.json gpurun_out/ab_s.json
