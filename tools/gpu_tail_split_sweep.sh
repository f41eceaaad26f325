# The tail partition at the C4 workload: head chunk K (0 = default rule), the last T samples of
# every pixel in chunks of KT handed out after the head (accumulate_tail / _chunk: T = 0 and
# KT = 0 the rule, T = -1 none); full frame and N-way shards rendered rank by rank, for each
# "K:T:KT" in $TAILS, $REPS times interleaved.
set -o pipefail
mkdir -p gpurun_out
TAILS=${TAILS:-"0:-1:0 0:0:0"}
WORLDS=${WORLDS:-"8"}
REPS=${REPS:-2}
for rep in $(seq 1 $REPS); do
  for c in $TAILS; do
    IFS=: read -r k t kt <<< "$c"
    timeout -k 10 300 python tools/shard_sweep.py --spp ${SPP:-1024} --chunk $k --tail $t --tail-chunk $kt \
      --worlds $WORLDS > gpurun_out/tail_${k}_${t}_${kt}_r$rep.json 2>/dev/null || exit 1
    echo "rep $rep $c done"
  done
done
TAILS="$TAILS" REPS=$REPS python - <<'PY'
import json, os
for c in os.environ["TAILS"].split():
    k, t, kt = c.split(":")
    rs = [json.load(open(f"gpurun_out/tail_{k}_{t}_{kt}_r{i}.json"))
          for i in range(1, int(os.environ["REPS"]) + 1)]
    line = f"K {int(k):3d} tail {int(t):4d} K_tail {int(kt):3d}  full {rs[0]['full_partition']} " + " ".join(
        f"{r['full_ms']:.2f}" for r in rs)
    for key in sorted(x for x in rs[0] if x.startswith("world")):
        line += f"  {key} (K={rs[0][key]['chunk']}, tail={rs[0][key]['tail']}) max " + " ".join(
            f"{r[key]['max_ms']:.2f}" for r in rs)
    print(line)
PY
