# Export a git revision's package into ab_objs/NAME and build it there, for A/B timing across
# host-side changes:  bash tools/mkab_tree.sh NAME REV ; then on the GPU box
#   VCRT_PKG_ROOT=ab_objs/NAME python tools/ab.py default ...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1
REV=$2
D=$ROOT/ab_objs/$NAME
rm -rf "$D" && mkdir -p "$D"
git -C "$ROOT" archive "$REV" vulkancomputeraytracing_amd include | tar -x -C "$D"
make -s -C "$D/vulkancomputeraytracing_amd" -j8 all >/dev/null
echo "$D"
