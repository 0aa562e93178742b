"""The reference's frame loop (Terrain::render, then IDevice::present) on one device, timed: the C3 workload
at 1920x1080 (512-step cap, 1 AO ray), --frames frames after 3 warm-up frames.  Under `rocprofv3
--kernel-trace` the launches' timeline shows where a serial frame's time goes (scripts/serial_timeline.py).
Usage: python scripts/serial_loop.py [--frames 20] [--defer K] [--reserve N]"""
import argparse
import os
import sys
import time

os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")  # as bench.py
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--defer", type=int, default=0,
                    help="0: the plain device; K >= 1: RT_DEVICE_DEFERRED with K frames to a launch")
    ap.add_argument("--reserve", type=int, default=0,
                    help="rt_device_reserve_cus: the trace kernel leaves N CUs free (for the prepass stream's kernel)")
    a = ap.parse_args()
    import gpgpuraytrace_amd as G
    W, H = a.width, a.height
    dev = G.DeviceFactory.construct(G.DeviceAPI.HIP, W, H, deferred=a.defer > 0)
    if a.defer > 0:
        dev.defer_batch(a.defer)
    if a.reserve:
        dev.reserve_cus(a.reserve)
    ter = G.Terrain(dev, "nomadplains", max_steps=512, ao_samples=1)
    ter.create()
    assert ter.reload()
    ter.set_camera(G.Camera(W, H))
    ter.set_time_of_day(0.3)
    for _ in range(3):
        ter.render_device()
        dev.present()
    dev.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.frames):
        ter.render_device()
        dev.present()
    dev.synchronize()
    print(f"serial{'' if a.defer == 0 else f' (deferred, {a.defer} frames to a launch)'}"
          f"{f', {a.reserve} CUs reserved' if a.reserve else ''}: "
          f"{(time.perf_counter() - t0) / a.frames * 1e3:.4f} ms/frame", flush=True)
    dev.destroy()


if __name__ == "__main__":
    main()
