# Quick GPU loop: the parity suite, then 1080p 256 spp timings of the variants in $QV (default 4 5).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest_failed; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for v in ${QV:-4 5}; do timeout -k 10 120 python tools/render_once.py --spp 256 --frames 3 --variant $v > gpurun_out/q_$v.json || exit 1; done
if [ -n "$QSTRESS" ]; then
  for v in ${QV:-4 5}; do timeout -k 10 200 python tools/render_once.py --width 3840 --height 2160 --spp 32 --depth 50 --scene stress4096 --frames 2 --variant $v > gpurun_out/qs_$v.json || exit 1; done
fi
QV="${QV:-4 5}" python - <<'PY'
import json, os
for pre in ("q", "qs"):
    for v in os.environ["QV"].split():
        f = f"gpurun_out/{pre}_{v}.json"
        if not os.path.exists(f):
            continue
        for st in json.load(open(f)):
            w = st["segments"] / 64
            print(pre, v, "Msps %.0f" % st["msamples_per_s"], "kernel_ms %.2f" % st["kernel_ms"],
                  "grid", st["grid_blocks"], "lds", st["lds_bytes"],
                  "groups/wi %.2f bounds/wi %.2f" % (st["group_tests"] / w, st["bound_tests"] / w))
PY
