# Accumulation chunk K at the C4 workload: the full frame on one GPU, and the N-way shards
# rendered rank by rank (strong-scaling estimate), for K in $KS (default 16 32 64) and N in
# $WORLDS (default 2,4,8).
set -o pipefail
mkdir -p gpurun_out
KS=${KS:-"16 32 64"}
WORLDS=${WORLDS:-"2,4,8"}
for k in $KS; do
  timeout -k 10 300 python tools/shard_sweep.py --chunk $k --worlds $WORLDS > gpurun_out/sweep_k$k.json 2>/dev/null || exit 1
done
KS="$KS" python - <<'PY'
import json, os
for k in os.environ["KS"].split():
    r = json.load(open(f"gpurun_out/sweep_k{k}.json"))
    for key in sorted(x for x in r if x.startswith("world")):
        w = r[key]
        print(f"K={int(k):4d} full {r['full_ms']:.1f} ms  {key}: max {w['max_ms']:.2f} "
              f"sum {w['sum_ms']:.1f} ideal_eff {w['ideal_efficiency']:.3f} per-rank {w['per_rank_ms']}")
PY
