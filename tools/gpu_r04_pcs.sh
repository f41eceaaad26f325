# Round 4, first GPU call: GPU tests of the tree, the A/B against round 3 (ab_objs/r3) and the
# static-first fetch (ab_objs/sf.hsaco), then PC sampling of the product flat kernel (final
# scene, 1080p, 64 spp, 4 frames) for the VALU attribution.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
PREV=ab_objs/r3 OBJS=ab_objs/sf.hsaco C2=1 bash tools/gpu_ab_tree.sh || exit $?
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic \
  --pc-sampling-unit cycles --pc-sampling-interval 65536 -d "$R/gpurun_out/pcs" -o pcs \
  --output-format csv -- python3 tools/render_once.py --spp 64 --frames 4 > gpurun_out/pcs.log 2>&1
rc=$?
echo "stochastic rc=$rc"
tail -5 gpurun_out/pcs.log
if [ $rc -ne 0 ]; then
  case $rc in 124|137|134|139) exit $rc;; esac
  timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap \
    --pc-sampling-unit time --pc-sampling-interval 50 -d "$R/gpurun_out/pcs_ht" -o pcs \
    --output-format csv -- python3 tools/render_once.py --spp 64 --frames 4 > gpurun_out/pcs_ht.log 2>&1
  rc=$?
  echo "host_trap rc=$rc"
  tail -5 gpurun_out/pcs_ht.log
  [ $rc -eq 0 ] || exit $rc
fi
find gpurun_out/pcs* -type f | head -20
