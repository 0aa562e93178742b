"""Single frames (B=1, 3 in flight) along a moving camera against the same frames with a fixed
camera: what per-frame constant uploads cost when the frame ring overlaps frames.

  python3 scripts/moving_single.py [--frames 48] [--lookahead 0|1] [--batch 1]

The two modes render different frames (the path moves into cheaper views), so compare a mode with
itself across builds or settings (profiles/r03/moving_single/: old_* = every camera move also
re-uploaded the 2 KiB gradient table, new_* = only the 812 B constant block; same within noise).
With a moving camera the ahead prepass (--lookahead 1) prepasses stale cameras and
rt_terrain_trace_ahead runs the prepass again: 2.56-2.59 vs 2.32-2.41 ms per frame.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["GPU_MAX_HW_QUEUES"] = "8"  # as bench.py


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=48)
    ap.add_argument("--lookahead", type=int, default=1)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--depth", type=int, default=3)
    a = ap.parse_args()
    import numpy as np
    import torch
    import gpgpuraytrace_amd as G
    W, H = 1920, 1080
    eu = G.camera.INITIAL_ROTATION_EULER
    base = G.Camera(W, H, euler=eu)
    path = [G.Camera(W, H, position=base.position + i * 2.0 * np.asarray(base.front, float),
                     euler=(eu[0], eu[1] + 0.01 * i, eu[2])) for i in range(a.frames)]
    out = {"env_cp_dma": os.environ.get("GPU_CP_DMA_COPY_SIZE"), "batch": a.batch, "lookahead": a.lookahead}
    for mode in ("fixed", "moving", "fixed", "moving"):
        ring = G.FrameRing(W, H, depth=a.depth, batch=a.batch, camera=base, time_of_day=0.3, max_steps=512,
                           ao_samples=1, lookahead=bool(a.lookahead) and a.batch >= 1)

        def run(n0, n):
            for j in range(n0, n0 + n, a.batch):
                if mode == "moving":
                    for (_, ter), cam in zip(ring.group(), path[j:j + a.batch]):
                        ter.set_camera(cam)
                        ter.update_terrain()
                ring.render_batch(ahead=j + a.batch < n0 + n)
        run(0, a.depth * a.batch)
        ring.synchronize()
        t0 = time.perf_counter()
        run(0, a.frames)
        ring.synchronize()
        dt = time.perf_counter() - t0
        ring.destroy()
        out.setdefault(mode, []).append(round(dt / a.frames * 1e3, 4))
        torch.cuda.synchronize()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
