# Culled-scan diagnostics (VCRT_DEBUG_STATS kernels): per wave-iteration union of groups tested
# vs per-lane group need (mean and wave max).
set -o pipefail
mkdir -p gpurun_out
export VCRT_DEBUG_STATS=1
timeout -k 10 120 python tools/render_once.py --spp 64 --variant 3 > gpurun_out/cs_final.json || exit 1
timeout -k 10 120 python tools/render_once.py --spp 8 --depth 50 --scene stress4096 --variant 3 > gpurun_out/cs_stress.json || exit 1
python - <<'PY'
import json
for f in ("final", "stress"):
    st = json.load(open(f"gpurun_out/cs_{f}.json"))
    d = st["debug"]
    print(f, "wave-iters", d[0], "lanes/iter %.1f" % (d[1] / d[0]),
          "union groups/iter %.1f" % (st["group_tests"] / d[0]),
          "bounds/iter %.1f" % (st["bound_tests"] / d[0]),
          "lane need mean %.2f" % (d[2] / d[1]), "wave max lane need %.2f" % (d[3] / d[0]))
PY
