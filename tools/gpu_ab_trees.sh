# Alternating single-process timing runs of several package trees (each built in place, any ABI):
#   TREES="ab_objs/prev ab_objs/pad ." bash tools/gpu_ab_trees.sh
# on the C4 workload (1080p 1024 spp) and, with STRESS=1, the stress scene (4K 32 spp depth 50).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
C4="--spp 1024 --frames 2"
S="--scene stress4096 --width 3840 --height 2160 --spp 32 --depth 50 --frames 2"
run() {  # tag, tree, args
  local tag=$1 tree=$2; shift 2
  VCRT_PKG_ROOT=$tree timeout -k 10 120 python tools/ab.py default --rounds 1 "$@" > gpurun_out/abt.json 2>&1 || { cat gpurun_out/abt.json; exit 1; }
  echo "$tag $(grep -o '"msamples_per_s": [0-9.]*' gpurun_out/abt.json | head -1) $(grep -o '"sha": "[0-9a-f]*"' gpurun_out/abt.json | head -1)"
}
for i in ${ROUNDS:-1 2}; do
  for t in $TREES; do run "$t c4" $t $C4; done
done
if [ -n "$STRESS" ]; then
  for i in 1 2; do for t in $TREES; do run "$t stress" $t $S; done; done
fi
echo ab_done
