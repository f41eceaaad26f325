# Culled-scan diagnostics (VCRT_DEBUG_STATS kernels), per wave-iteration: groups tested (union
# for CULL, exact passes for CULL_LANE), bound tests, per-lane need (mean, wave max) and, for
# CULL_LANE, candidate-root passes.
set -o pipefail
mkdir -p gpurun_out
export VCRT_DEBUG_STATS=1
for v in 3 4; do
timeout -k 10 120 python tools/render_once.py --spp 64 --variant $v > gpurun_out/cs_final_v$v.json || exit 1
timeout -k 10 120 python tools/render_once.py --spp 8 --depth 50 --scene stress4096 --variant $v > gpurun_out/cs_stress_v$v.json || exit 1
done
python - <<'PY'
import json
for f in ("final", "stress"):
  for v in (3, 4):
    st = json.load(open(f"gpurun_out/cs_{f}_v{v}.json"))
    d = st["debug"]
    print(f, v, "wave-iters", d[0], "lanes/iter %.1f" % (d[1] / d[0]),
          "groups/iter %.1f" % (st["group_tests"] / d[0]),
          "bounds/iter %.1f" % (st["bound_tests"] / d[0]),
          ("lane need mean %.2f" % (d[2] / d[1])) if v == 3 else ("cand passes/iter %.2f" % (d[2] / d[0])),
          "wave max lane need %.2f" % (d[3] / d[0]))
PY
