"""Predict multi-GPU strong scaling on one GPU: time rank r's share of an N-way tile-cyclic frame.

For each N in 1,2,4,8 and each rank r < N, render_device(r, N) is timed over K frames (HIP events
via the device's kernel timer + wall clock). The frame time of an N-GPU run is bounded below by
max_r(t(r, N)) + the gather, so the ratio t(0,1) / max_r t(r,N) is the scaling ceiling.
Usage: python scripts/shard_sim.py [--config c3] [--steps 10]
"""
import argparse
import ctypes as C
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
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--ns", default="1,2,4,8")
    a = ap.parse_args()
    import torch
    import gpgpuraytrace_amd as G
    W, H = a.width, a.height
    dev = G.DeviceFactory.construct(G.DeviceAPI.HIP, W, H, gpu=0)
    ter = G.Terrain(dev, "nomadplains", max_steps=a.max_steps, ao_samples=a.ao)
    ter.create()
    assert ter.reload()
    ter.set_camera(G.Camera(W, H))
    ter.set_time_of_day(0.3)
    stream = torch.cuda.current_stream()
    dev.set_stream(stream.cuda_stream)
    ter.update_shaders()
    out = {}
    for n in [int(x) for x in a.ns.split(",")]:
        per = []
        for r in range(n):
            for _ in range(2):
                ter.render_device(r, n)
            torch.cuda.synchronize()
            G.lib().rt_device_set_profiling(dev._h, 1)
            G.lib().rt_device_kernel_time(dev._h, None, None)
            t0 = time.perf_counter()
            for _ in range(a.steps):
                ter.render_device(r, n)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / a.steps * 1e3
            kms, kn = C.c_double(), C.c_int()
            G.lib().rt_device_kernel_time(dev._h, C.byref(kms), C.byref(kn))
            per.append({"rank": r, "frame_ms": round(dt, 4), "tracescreen_ms": round(kms.value / max(1, kn.value), 4)})
        worst = max(p["frame_ms"] for p in per)
        out[n] = {"worst_frame_ms": worst, "ranks": per}
        print(json.dumps({"n": n, "worst_frame_ms": worst, "ranks": per}), flush=True)
    base = out[min(out)]["worst_frame_ms"]
    print(json.dumps({"scaling_ceiling": {n: round(base / v["worst_frame_ms"], 3) for n, v in out.items()}}), flush=True)
    dev.destroy()


if __name__ == "__main__":
    main()
