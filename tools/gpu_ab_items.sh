# A/B of the current tree against ab_objs/$PREV (tools/mkab_tree.sh) where item costs show: the
# C3 frame (256 spp) and C4's 8-way shards rendered in turn (tools/shard_sweep.py), alternating
# processes, $REPS times.
set -o pipefail
mkdir -p gpurun_out
for i in $(seq 1 ${REPS:-2}); do
  for t in prev new; do
    if [ $t = prev ]; then E="VCRT_PKG_ROOT=ab_objs/$PREV"; else E="X=1"; fi
    env $E timeout -k 10 200 python tools/shard_sweep.py --spp 256 --worlds 8 > gpurun_out/sw_c3_$t.json 2>/dev/null || exit 1
    env $E timeout -k 10 200 python tools/shard_sweep.py --spp 1024 --worlds 8 > gpurun_out/sw_c4_$t.json 2>/dev/null || exit 1
    python - "$t" <<'PY'
import json, sys
t = sys.argv[1]
a = json.load(open(f"gpurun_out/sw_c3_{t}.json")); b = json.load(open(f"gpurun_out/sw_c4_{t}.json"))
print(t, "c3 full %.2f w8 max %.2f | c4 full %.2f w8 max %.2f" % (
    a["full_ms"], a["world8"]["max_ms"], b["full_ms"], b["world8"]["max_ms"]))
PY
  done
done
