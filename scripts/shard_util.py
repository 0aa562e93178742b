"""Work and lane utilisation of rank 0's share of an N-way sharded C3 batch against the whole
batch (instrumented kernels): does a rank's k_trace at N = 8 do 1/8 of the N = 1 work, at the same
noise lane utilisation?  With a diagnostic build (RT_LIB_VARIANT, -DRT_COUNT_PHASE=k) the noise
counts are one work kind's (phase_util.py's kinds).
usage: python3 scripts/shard_util.py [frames] [N,...]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import with_variant  # noqa: E402

with_variant.apply()
import gpgpuraytrace_amd as G  # noqa: E402
from gpgpuraytrace_amd import engine as E  # noqa: E402

W, H = 1920, 1080
B = int(sys.argv[1]) if len(sys.argv) > 1 else 10
NS = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,8").split(",")]
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
KEYS = ("primary_steps", "shadow_steps", "ao_steps", "hits", "noise_calls", "noise_wave_iters")


def total():
    s = [d.stats(reset=True) for d in devs]
    return {k: sum(x[k] for x in s) for k in KEYS + ("prepass_steps",)}


base = None
for n in NS:
    for t in ters:
        t.update_shaders()
        t.camera_compute.run(2, 2, 1)
    pre = total()  # the prepass alone
    E.render_batch(ters, 0, n)
    for d in devs:
        d.synchronize()
    tr = total()
    row = {k: tr[k] - (pre[k] if k != "prepass_steps" else 0) for k in KEYS}
    util = row["noise_calls"] / (64.0 * row["noise_wave_iters"]) if row["noise_wave_iters"] else 0.0
    if base is None:
        base = row
    rel = {k: round(row[k] * n / base[k], 4) if base[k] else None for k in KEYS}
    print("%s B=%d N=%d rank 0: %s  lane utilisation %.4f  (x N / N=1: %s)" % (
        os.environ.get("RT_LIB_VARIANT", "") or "all", B, n, row, util, rel), flush=True)
for d in devs:
    d.destroy()
