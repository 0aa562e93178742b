"""One-frame-at-a-time C3 renders (rt_terrain_render, one stream) with the segment tail forced off,
on, or left to the launch heuristic; ms per frame over --frames frames after a warm-up.
usage: python3 scripts/single_frame_ab.py [frames]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import gpgpuraytrace_amd as G  # noqa: E402

W, H = 1920, 1080
n = int(sys.argv[1]) if len(sys.argv) > 1 else 24
for rep in range(2):
    for seg in (None, False, True):
        dev = G.DeviceFactory.construct(G.DeviceAPI.HIP, W, H, gpu=0, seg_tail=seg)
        ter = G.Terrain(dev, "nomadplains", max_steps=512, ao_samples=1)
        ter.create()
        assert ter.reload()
        ter.set_camera(G.Camera(W, H))
        ter.set_time_of_day(0.3)
        for _ in range(3):
            ter.render_device()
        dev.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            ter.render_device()
            dev.present()
        dev.synchronize()
        dt = (time.perf_counter() - t0) / n
        print("seg_tail=%-5s %.4f ms per frame" % (seg, dt * 1e3), flush=True)
        dev.destroy()
