for k in 0 4 16 64; do
  timeout -k 10 60 python tools/render_once.py --scene three --width 800 --height 450 --spp 64 --depth 8 --chunk $k --frames 5 > gpurun_out/c2_k$k.json 2>/dev/null || exit 1
done
python - <<'PY'
import json
for k in (0, 4, 16, 64):
    st = json.load(open(f"gpurun_out/c2_k{k}.json"))[-1]
    print(k, st["accumulate_chunk"], st["kernel"], "kernel %.3f ms resolve %.3f frame %.3f" % (st["kernel_ms"], st["resolve_ms"], st["frame_ms"]), "grid", st["grid_blocks"])
PY
