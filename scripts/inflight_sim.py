"""Frames in flight: D independent frame contexts (own buffers, constants, framebuffer) on D HIP
streams, frames dealt round-robin, so frame i+1's prepass and primary phase can fill the CUs
that frame i's tail leaves idle. Times rank r's share of an N-way tile-cyclic frame.
Usage: python scripts/inflight_sim.py [--depth 2] [--ns 1,8]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--max-steps", type=int, default=512)
    ap.add_argument("--ao", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--depths", default="1,2,3")
    ap.add_argument("--ns", default="1,8")
    a = ap.parse_args()
    import torch
    import gpgpuraytrace_amd as G
    W, H = a.width, a.height
    ctx = []
    for _ in range(max(int(x) for x in a.depths.split(","))):
        dev = G.DeviceFactory.construct(G.DeviceAPI.HIP, W, H, gpu=0)
        ter = G.Terrain(dev, "nomadplains", max_steps=a.max_steps, ao_samples=a.ao)
        ter.create()
        assert ter.reload()
        ter.set_camera(G.Camera(W, H))
        ter.set_time_of_day(0.3)
        s = torch.cuda.Stream()
        dev.set_stream(s.cuda_stream)
        ter.update_shaders()
        ctx.append((dev, ter))
    res = {}
    for depth in [int(x) for x in a.depths.split(",")]:
        for n in [int(x) for x in a.ns.split(",")]:
            worst = 0.0
            for r in range(n):
                def frame(i):
                    dev, ter = ctx[i % depth]
                    ter.render_device(r, n)
                    dev.present()
                for i in range(2 * depth):
                    frame(i)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i in range(a.steps):
                    frame(i)
                torch.cuda.synchronize()
                worst = max(worst, (time.perf_counter() - t0) / a.steps * 1e3)
            res[(depth, n)] = worst
            print(json.dumps({"depth": depth, "n": n, "worst_frame_ms": round(worst, 4),
                              "ceiling_vs_depth1_n1": round(res.get((1, 1), worst) / worst, 3)}), flush=True)
    for dev, _ in ctx:
        dev.destroy()


if __name__ == "__main__":
    main()
