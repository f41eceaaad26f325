"""One-off: host overhead per vcrt_draw_next_frame on a tiny frame."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import vulkancomputeraytracing_amd as vc
for scene, w, h, spp in (("three", 16, 16, 8), ("final", 16, 16, 8)):
    desc = vc.RenderDesc(width=w, height=h, samples_per_pixel=spp, max_depth=8, device=0)
    with vc.Renderer(desc, scene) as r:
        for _ in range(50):
            r.draw_next_frame()
        t = time.perf_counter()
        n = 500
        ks = 0.0
        for _ in range(n):
            r.draw_next_frame()
            ks += r.frame_times()[0]
        dt = (time.perf_counter() - t) / n
        st = r.stats()
        print(scene, f"per draw {dt*1e6:.1f} us, kernel {ks/n*1e3:.1f} us, resolve {st['resolve_ms']*1e3:.1f} us, kernel {st['kernel']}")
