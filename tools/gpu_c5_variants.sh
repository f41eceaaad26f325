# C5 stress scene (4100 spheres, 3840x2160, depth 50): the culled kernels compared on 1 GPU at
# 64 spp (a 4096-spp frame takes ~4 s per variant); images must be bit-identical across variants.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 5 4 3; do
  for t in auto lds global; do
    [ "$v" = 3 ] && [ "$t" != auto ] && continue
    VCRT_CULL_LANE_TABLES=$t timeout -k 10 200 python tools/render_once.py --scene stress4096 \
      --width 3840 --height 2160 --spp 64 --depth 50 --variant $v --frames 2 \
      > gpurun_out/c5_v${v}_${t}.json || exit 1
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/c5_v*.json")):
    st = json.load(open(f))[-1]
    print(f, "variant", st["kernel_variant"], "lds", st["tables_in_lds"], "block", st["block_threads"],
          "grid", st["grid_blocks"], "kernel_ms %.1f" % st["kernel_ms"],
          "Msamples/s %.0f" % st["msamples_per_s"], "segments", st["segments"])
PY
