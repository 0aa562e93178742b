"""Per-frame work counts of the C3 frame (instrumented kernels): steps per ray kind, noise3d
per step.  Usage: python scripts/frame_stats.py [--max-steps 512 --ao 1]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--max-steps", type=int, default=512)
    ap.add_argument("--ao", type=int, default=1)
    a = ap.parse_args()
    import gpgpuraytrace_amd as G
    dev = G.DeviceFactory.construct(G.DeviceAPI.HIP, a.width, a.height, stats=True)
    ter = G.Terrain(dev, "nomadplains", max_steps=a.max_steps, ao_samples=a.ao)
    ter.create()
    assert ter.reload()
    ter.set_camera(G.Camera(a.width, a.height))
    ter.set_time_of_day(0.3)
    ter.update_shaders()
    ter.camera_compute.run(2, 2, 1)
    pre = dev.stats(reset=True)
    ter.render_device()
    st = dev.stats(reset=True)
    px = a.width * a.height
    steps = st["primary_steps"] + st["shadow_steps"] + st["ao_steps"]
    out = {"prepass": pre, "frame": st, "primary_steps_per_pixel": st["primary_steps"] / px,
           "shadow_steps_per_hit": st["shadow_steps"] / max(1, st["hits"]),
           "ao_steps_per_hit": st["ao_steps"] / max(1, st["hits"]),
           "step_share": {k: round(st[k] / steps, 3) for k in ("primary_steps", "shadow_steps", "ao_steps")},
           "noise3d_per_step": (st["noise_calls"] - pre["noise_calls"]) / steps}
    print(json.dumps(out, indent=1))
    dev.destroy()


if __name__ == "__main__":
    main()
