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
# the Makefile's recipe: two code-generation parts (VCRT_PART), linked into one code object
L=/opt/rocm/lib/llvm/bin
W=$(mktemp -d)
for part in 1 2; do
  /opt/rocm/bin/hipcc --cuda-device-only -emit-llvm -c --offload-arch=gfx950 -O3 -std=c++17 \
    -ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt \
    -fno-gpu-flush-denormals-to-zero -munsafe-fp-atomics $EXTRA -I"$INC" -I"$SRC" \
    -I/opt/rocm/include -DVCRT_PART=$part "$SRC/tracer.hip" -o "$W/p$part.bc"
done
$L/llc -mtriple=amdgcn-amd-amdhsa -mcpu=gfx950 -O3 -filetype=obj -amdgpu-use-amdgpu-trackers=1 $LLC_EXTRA1 \
  $LLC_EXTRA "$W/p1.bc" -o "$W/p1.o"
$L/llc -mtriple=amdgcn-amd-amdhsa -mcpu=gfx950 -O3 -filetype=obj $LLC_EXTRA $LLC_EXTRA2 "$W/p2.bc" -o "$W/p2.o"
$L/ld.lld -shared "$W/p1.o" "$W/p2.o" -o "$ROOT/ab_objs/$NAME.hsaco"
rm -rf "$W"
echo "$ROOT/ab_objs/$NAME.hsaco"
