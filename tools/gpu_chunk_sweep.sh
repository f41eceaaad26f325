# Accumulation chunk K at the C4 workload: the full frame on one GPU, and the 8-way shards
# rendered rank by rank (strong-scaling estimate), for K = 16 .. 256.
set -o pipefail
mkdir -p gpurun_out
for k in 8 16 32; do
  timeout -k 10 300 python tools/shard_sweep.py --chunk $k --worlds 8 > gpurun_out/sweep_k$k.json 2>/dev/null || exit 1
done
python - <<'PY'
import json
for k in (8, 16, 32):
    r = json.load(open(f"gpurun_out/sweep_k{k}.json"))
    w = r["world8"]
    print(f"K={k:4d} full {r['full_ms']:.1f} ms  N=8 max {w['max_ms']:.2f} sum {w['sum_ms']:.1f} "
          f"ideal_eff {w['ideal_efficiency']:.3f}")
PY
