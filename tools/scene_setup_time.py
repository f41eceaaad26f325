"""Host time of a renderer's scene set-up (vcrt_begin + vcrt_set_scene: culling tables, camera-ray
lists, uploads) for the final scene at 1080p and the stress scene at 4K; VCRT_HOST_THREADS sets
the list builders' threads."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vulkancomputeraytracing_amd as vc  # noqa: E402

out = {}
for name, w, h in (("final", 1920, 1080), ("stress4096", 3840, 2160)):
    best = None
    for _ in range(3):
        t = time.perf_counter()
        r = vc.Renderer(vc.RenderDesc(width=w, height=h, samples_per_pixel=1, device=0), name)
        dt = time.perf_counter() - t
        r.close()
        best = dt if best is None else min(best, dt)
    out[name] = round(best * 1e3, 1)
print(json.dumps({"threads": os.environ.get("VCRT_HOST_THREADS", "auto"), "setup_ms": out}))
