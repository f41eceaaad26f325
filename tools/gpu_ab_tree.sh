# A/B of the current tree against the build in ab_objs/prev (an earlier commit, any ABI; made by
#   git archive REV | tar -x -C ab_objs/prev && make -C ab_objs/prev/vulkancomputeraytracing_amd)
# plus the code objects / env settings in $OBJS (tools/ab.py syntax, loaded by the current tree).
# Parity tests of the current tree first (unless NOTEST=1), then alternating single-process
# timing runs on the C4 workload (1080p 1024 spp) and, with STRESS=1, the stress scene (4K 32 spp
# depth 50). Every line prints Msamples/s and the image digest; digests must agree per config.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -1 gpurun_out/pytest_gpu.log
fi
run() {  # tag, env prefix, ab.py args
  local tag=$1; shift
  timeout -k 10 120 "$@" > gpurun_out/abt.json 2>&1 || { cat gpurun_out/abt.json; exit 1; }
  echo "$tag $(grep -o '"msamples_per_s": [0-9.]*' gpurun_out/abt.json | head -1) $(grep -o '"sha": "[0-9a-f]*"' gpurun_out/abt.json | head -1)"
}
C4="--spp 1024 --frames 2"
S="--scene stress4096 --width 3840 --height 2160 --spp 32 --depth 50 --frames 2"
for i in ${ROUNDS:-1 2}; do
  run "prev c4" env VCRT_PKG_ROOT=${PREV:-ab_objs/prev} python tools/ab.py default --rounds 1 $C4
  run "new c4" python tools/ab.py default --rounds 1 $C4
  for o in $OBJS; do run "$o c4" python tools/ab.py $o --rounds 1 $C4; done
done
if [ -n "$STRESS" ]; then
  for i in ${STRESS_ROUNDS:-1}; do
    run "prev stress" env VCRT_PKG_ROOT=${PREV:-ab_objs/prev} python tools/ab.py default --rounds 1 $S
    run "new stress" python tools/ab.py default --rounds 1 $S
    for o in $OBJS; do run "$o stress" python tools/ab.py $o --rounds 1 $S; done
  done
fi
if [ -n "$C2" ]; then
  C2A="--scene three --width 800 --height 450 --spp 64 --depth 8 --frames 20"
  for i in 1 2 3; do
    run "prev c2" env VCRT_PKG_ROOT=${PREV:-ab_objs/prev} python tools/ab.py default --rounds 1 $C2A
    run "new c2" python tools/ab.py default --rounds 1 $C2A
    for o in $OBJS; do run "$o c2" python tools/ab.py $o --rounds 1 $C2A; done
  done
fi
echo ab_done
