"""Noise lane utilisation of an instrumented C3 batch (default 12 frames, as bench.py), split by
k_trace work kind.  Run once per diagnostic build: RT_LIB_VARIANT=<name> loads
_build/librt_hip_<name>.so (make variant NAME=.. FLAGS="-DRT_COUNT_PHASE=K": 1 primary units, 2 long
shadow/AO rays, 3 shading batches; -DRT_COUNT_PHASE=99 -DRT_COUNT_LONG_STEPS=1|2|3: live lanes per
long-ray step, all / unit queue drained / not drained), or none (all noise).
usage: python3 scripts/phase_util.py [frames]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import with_variant  # noqa: E402

with_variant.apply()
import gpgpuraytrace_amd as G  # noqa: E402
from gpgpuraytrace_amd import engine as E  # noqa: E402

W, H = 1920, 1080
B = int(sys.argv[1]) if len(sys.argv) > 1 else 12
devs, ters = [], []
for _ in range(B):
    dev = G.DeviceFactory.construct(G.DeviceAPI.HIP, W, H, gpu=0, stats=True)
    ter = G.Terrain(dev, "nomadplains", max_steps=512, ao_samples=1)
    ter.create()
    assert ter.reload()
    ter.set_camera(G.Camera(W, H))
    ter.set_time_of_day(0.3)
    devs.append(dev)
    ters.append(ter)


def total():
    s = [d.stats(reset=True) for d in devs]
    return sum(x["noise_calls"] for x in s), sum(x["noise_wave_iters"] for x in s)


for t in ters:
    t.update_shaders()
    t.camera_compute.run(2, 2, 1)
pc, pw = total()  # the prepass alone (B frames)
E.render_batch(ters) if B > 1 else ters[0].render_device()
for d in devs:
    d.synchronize()
c, w = total()
calls, waves = c - pc, w - pw
print("%-8s B=%d noise %d  wave-iterations %d  lane utilisation %.4f" % (
    os.environ.get("RT_LIB_VARIANT", "all"), B, calls, waves, calls / (64.0 * waves) if waves else 0.0))
for d in devs:
    d.destroy()

if os.environ.get("RT_LIB_VARIANT") == "lh":  # live lanes per primary march step (RT_LIVE_HIST build)
    import ctypes as C
    h = (C.c_ulonglong * 65)()
    G.lib().rt_debug_live_hist(h, 1)  # cumulative over both renders above (the prepass adds none)
    tot = sum(h)
    lost = sum((64 - i) * n for i, n in enumerate(h))
    print("primary wave-steps %d, mean live %.2f / 64" % (tot, sum(i * n for i, n in enumerate(h)) / max(1, tot)))
    acc = 0
    for lo in range(0, 64, 8):
        n = sum(h[lo + 1:lo + 9])
        l = sum((64 - i) * h[i] for i in range(lo + 1, lo + 9))
        acc += l
        print("  live %2d-%2d: %5.1f%% of steps, %5.1f%% of idle lane-steps" % (lo + 1, lo + 8, 100.0 * n / tot, 100.0 * l / max(1, lost)))
