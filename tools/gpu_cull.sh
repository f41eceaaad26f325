# Culled-scan check on the GPU box: parity tests first, then timings against the linear scan.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest_failed; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
for v in 2 3; do
  timeout -k 10 120 python tools/render_once.py --spp 256 --frames 2 --variant $v > gpurun_out/cull_final_v$v.json || exit 1
  timeout -k 10 120 python tools/render_once.py --spp 16 --depth 50 --scene stress4096 --frames 2 --variant $v > gpurun_out/cull_stress_v$v.json || exit 1
done
python - <<'PY'
import json
for f in ("final", "stress"):
    for v in (2, 3):
        st = json.load(open(f"gpurun_out/cull_{f}_v{v}.json"))[-1]
        print(f, v, "Msps %.0f" % st["msamples_per_s"], "kernel_ms %.2f" % st["kernel_ms"],
              "segs", st["segments"], "groups", st["group_tests"], "bounds", st["bound_tests"])
PY
echo all_done
