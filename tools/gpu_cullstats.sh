# Culled-scan diagnostics: wave-union vs per-lane group need (VCRT_DEBUG_STATS kernels).
set -o pipefail
mkdir -p gpurun_out
export VCRT_DEBUG_STATS=1
for lab in t line; do
  co=""; [ $lab = line ] && co="--code-object vulkancomputeraytracing_amd/lib/variants/cull_line_only.hsaco"
  timeout -k 10 120 python tools/render_once.py --spp 64 --variant 3 $co > gpurun_out/cs_final_$lab.json || exit 1
  timeout -k 10 120 python tools/render_once.py --spp 8 --depth 50 --scene stress4096 --variant 3 $co > gpurun_out/cs_stress_$lab.json || exit 1
done
python - <<'PY'
import json
for f in ("final", "stress"):
    for lab in ("t", "line"):
        st = json.load(open(f"gpurun_out/cs_{f}_{lab}.json"))
        d = st["debug"]
        print(f, lab, "wave-iters", d[0], "lanes/iter %.1f" % (d[1] / d[0]),
              "union groups/iter %.1f" % (st["group_tests"] / d[0]),
              "bounds/iter %.1f" % (st["bound_tests"] / d[0]),
              "lane need/lane-seg %.2f" % (d[2] / d[1]))
PY
