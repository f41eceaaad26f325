# C2 wave lifetime histograms (diagnostics build ab_objs/wt.hsaco) at K = 32, K = 8 and 3
# workgroups per CU.
set -o pipefail
export TMPDIR=/tmp
C2="--scene three --width 800 --height 450 --spp 64 --depth 8 --worlds 1 --ranks 1"
for x in "" "--chunk 8" "--blocks-per-cu 3"; do
  VCRT_DEBUG_STATS=2 timeout -k 10 120 python tools/wave_times.py ab_objs/wt.hsaco $C2 $x 2>/dev/null || exit 1
done
