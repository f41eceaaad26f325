# Parity suite of the current tree, then A/B timing of every code object in exp/ab/ on the final
# scene (1080p 256 spp); images must be bit-identical.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/ab.py exp/ab/*.hsaco --rounds ${ROUNDS:-2} ${ABARGS} > gpurun_out/ab_f.json 2>&1 || { cat gpurun_out/ab_f.json; exit 1; }
grep -E 'round|same_bits|sha' gpurun_out/ab_f.json
