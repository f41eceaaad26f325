# A/B of two package trees (ab_objs/A vs the working tree), interleaved rounds:
#   bash tools/gpu_ab_trees.sh A [ab.py args]
set -o pipefail
A=$1; shift
for r in 1 2; do
  VCRT_PKG_ROOT=ab_objs/$A timeout -k 10 300 python tools/ab.py default --rounds 1 "$@" > gpurun_out/abt_${A}_$r.json 2>&1 || exit 1
  timeout -k 10 300 python tools/ab.py default --rounds 1 "$@" > gpurun_out/abt_cur_$r.json 2>&1 || exit 1
done
python - "$A" <<'PY'
import json, sys
a = sys.argv[1]
def load(tag, r):
    txt = open(f"gpurun_out/abt_{tag}_{r}.json").read()
    return json.loads(txt[txt.index("{"):])["results"]["default"]
for tag in (a, "cur"):
    runs = [load(tag, r) for r in (1, 2)]
    print(tag, round(max(x["msamples_per_s"] for x in runs)), {x["sha"] for x in runs})
PY
