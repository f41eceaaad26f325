# C2 (three spheres, 800x450, 64 spp, depth 8): head chunk K and tail (T, KT) settings, best
# kernel ms of 10 frames each, two interleaved rounds; "K:T:KT" in $CFGS (T = -1: no tail).
set -o pipefail
mkdir -p gpurun_out
CFGS=${CFGS:-"16:-1:0 16:16:4 16:16:2 32:16:4 32:32:4 8:-1:0"}
for rep in 1 2; do
  for c in $CFGS; do
    IFS=: read -r k t kt <<< "$c"
    timeout -k 10 60 python tools/render_once.py --scene three --width 800 --height 450 --spp 64 \
      --depth 8 --chunk $k --tail $t --tail-chunk $kt --frames 10 > gpurun_out/c2t_${k}_${t}_${kt}_$rep.json 2>/dev/null || exit 1
  done
done
CFGS="$CFGS" python - <<'PY'
import json, os
for c in os.environ["CFGS"].split():
    k, t, kt = c.split(":")
    best = [min(s["kernel_ms"] for s in json.load(open(f"gpurun_out/c2t_{k}_{t}_{kt}_{r}.json")))
            for r in (1, 2)]
    st = json.load(open(f"gpurun_out/c2t_{k}_{t}_{kt}_1.json"))[-1]
    print(f"K {st['accumulate_chunk']:3d} tail {st['accumulate_tail']:3d} x {st['accumulate_tail_chunk']:2d}"
          f"  kernel ms {best[0]:.3f} {best[1]:.3f}")
PY
