set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest_failed; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for v in 4 5; do timeout -k 10 120 python tools/render_once.py --spp 256 --frames 3 --variant $v > gpurun_out/q_$v.json || exit 1; done
python - <<'PY'
import json
for v in (4,5):
    for st in json.load(open(f"gpurun_out/q_{v}.json")):
        print(v, "Msps %.0f" % st["msamples_per_s"], "kernel_ms %.2f" % st["kernel_ms"], "grid", st["grid_blocks"], "lds", st["lds_bytes"])
PY
