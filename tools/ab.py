"""A/B timing of tracer code objects on one configuration: each code object renders the same
frames in turn (interleaved rounds), and the images must be bit-identical to the first one's.

  python tools/ab.py exp/base.hsaco exp/new.hsaco [--spp 256] [--rounds 2] [--scene final]
"""
import argparse
import hashlib
import json
import os
import sys

# VCRT_PKG_ROOT: import the package (and its libvcrt.so) from another tree, e.g. a build of an
# earlier commit, to compare across ABI changes (one tree per process)
sys.path.insert(0, os.environ.get("VCRT_PKG_ROOT",
                                  os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import vulkancomputeraytracing_amd as vc  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("objects", nargs="+", help="code objects, or 'default' for the package's own; "
                   "OBJ@VAR=VALUE,... sets environment variables for that object's renders, "
                   "and OBJ@desc.FIELD=VALUE a RenderDesc field (e.g. desc.accumulate_quantum=8)")
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--spp", type=int, default=256)
    p.add_argument("--depth", type=int, default=10)
    p.add_argument("--scene", default="final")
    p.add_argument("--variant", type=int, default=0)
    p.add_argument("--frames", type=int, default=2)
    p.add_argument("--rounds", type=int, default=2)
    a = p.parse_args()
    best = {o: None for o in a.objects}
    digest = {}
    for rnd in range(a.rounds):
        for obj in a.objects:
            path, _, env = obj.partition("@")
            fields = {}
            for kv in filter(None, env.split(",")):
                k, _, v = kv.partition("=")
                if k.startswith("desc."):
                    fields[k[5:]] = int(v)
                else:
                    os.environ[k] = v
            desc = vc.RenderDesc(width=a.width, height=a.height, samples_per_pixel=a.spp,
                                 max_depth=a.depth, kernel_variant=a.variant, device=0,
                                 code_object_path=None if path == "default" else path, **fields)
            with vc.Renderer(desc, a.scene) as r:
                for _ in range(a.frames):
                    r.draw_next_frame()
                    st = r.stats()
                    ms = st["kernel_ms"]
                    if best[obj] is None or ms < best[obj]["kernel_ms"]:
                        best[obj] = {"kernel_ms": ms,
                                     "msamples_per_s": st["samples"] / (ms * 1e3),
                                     "segments": st["segments"],
                                     "group_tests": st["group_tests"],
                                     "bound_tests": st["bound_tests"],
                                     "ring_entries": st["ring_entries"]}
                if rnd == 0:
                    digest[obj] = hashlib.sha256(r.read_framebuffer().tobytes()).hexdigest()[:16]
            for kv in filter(None, env.split(",")):
                if not kv.startswith("desc."):
                    os.environ.pop(kv.partition("=")[0], None)
            print(f"round {rnd} {obj}: {best[obj]['msamples_per_s']:.0f} Msamples/s", flush=True)
    ref = digest[a.objects[0]]
    out = {o: dict(best[o], sha=digest[o], same_bits=digest[o] == ref) for o in a.objects}
    print(json.dumps({"config": vars(a), "results": out}, indent=1))
    # objects that change a desc field (e.g. the accumulation quantum) may change the image
    if not all(v["same_bits"] for o, v in out.items() if "desc." not in o):
        sys.exit(3)


if __name__ == "__main__":
    main()
