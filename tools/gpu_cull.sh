# Culled-scan check on the GPU box: parity tests first, then timings against the linear scan.
#   VARIANTS="label=path.hsaco ..." also times variant 3 from those code objects.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_gpu.log 2>&1 || { echo pytest_failed; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
run() {  # label variant extra-args...
  local lab=$1 v=$2; shift 2
  timeout -k 10 120 python tools/render_once.py --spp 256 --frames 2 --variant $v "$@" > gpurun_out/cull_final_$lab.json || return 1
  timeout -k 10 120 python tools/render_once.py --width 3840 --height 2160 --spp 32 --depth 50 --scene stress4096 --frames 2 --variant $v "$@" > gpurun_out/cull_stress_$lab.json || return 1
}
run smem 2 && run cull 3 && run lane 4 && run flat 5 || exit 1
VCRT_CULL_LANE_TABLES=global run lane_global 4 || exit 1
labs="smem cull lane flat lane_global"
for lv in $VARIANTS; do run "${lv%%=*}" ${VARIANT_ID:-3} --code-object "${lv#*=}" || exit 1; labs="$labs ${lv%%=*}"; done
LABS="$labs" python - <<'PY'
import json, os
for f in ("final", "stress"):
    for lab in os.environ["LABS"].split():
        st = json.load(open(f"gpurun_out/cull_{f}_{lab}.json"))[-1]
        print(f, lab, "Msps %.0f" % st["msamples_per_s"], "kernel_ms %.2f" % st["kernel_ms"],
              "segs", st["segments"], "groups", st["group_tests"], "bounds", st["bound_tests"],
              "lds", st["lds_bytes"], "block", st["block_threads"], "grid", st["grid_blocks"])
PY
echo all_done
