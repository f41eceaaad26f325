# Build the tracer code object of the working tree (or of a git revision) into ab_objs/NAME.hsaco
# for tools/ab.py A/B timing:  bash tools/mkab.sh NAME [REV]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1
REV=$2
SRC=$ROOT/vulkancomputeraytracing_amd/csrc
INC=$ROOT/include
if [ -n "$REV" ]; then
  T=$(mktemp -d)
  git -C "$ROOT" archive "$REV" vulkancomputeraytracing_amd/csrc include | tar -x -C "$T"
  SRC=$T/vulkancomputeraytracing_amd/csrc
  INC=$T/include
fi
mkdir -p "$ROOT/ab_objs"
/opt/rocm/bin/hipcc --genco --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math \
  -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -munsafe-fp-atomics \
  $EXTRA -I"$INC" -I"$SRC" "$SRC/tracer.hip" -o "$ROOT/ab_objs/$NAME.hsaco"
echo "$ROOT/ab_objs/$NAME.hsaco"
