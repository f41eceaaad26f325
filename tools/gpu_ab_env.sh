# Parity suite, then A/B timing of an environment switch ($ABVAR, values $ABVALS) with the
# current build, alternating processes: final scene 1080p 256 spp and the stress scene 4K 32 spp.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
S="--scene stress4096 --width 3840 --height 2160 --spp 32 --depth 50"
for i in 1 2; do for v in ${ABVALS:-0 1}; do
  env $ABVAR=$v timeout -k 10 120 python tools/ab.py default --rounds 1 > gpurun_out/abe.json 2>&1 || { cat gpurun_out/abe.json; exit 1; }
  echo "final $ABVAR=$v $(grep -o '"msamples_per_s": [0-9.]*' gpurun_out/abe.json) $(grep -o '"sha": "[0-9a-f]*"' gpurun_out/abe.json)"
done; done
for v in ${ABVALS:-0 1}; do
  env $ABVAR=$v timeout -k 10 120 python tools/ab.py default --rounds 1 $S > gpurun_out/abe.json 2>&1 || { cat gpurun_out/abe.json; exit 1; }
  echo "stress $ABVAR=$v $(grep -o '"msamples_per_s": [0-9.]*' gpurun_out/abe.json) $(grep -o '"sha": "[0-9a-f]*"' gpurun_out/abe.json)"
done
