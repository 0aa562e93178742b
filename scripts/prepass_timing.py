"""Standalone time of a batch's camerarays prepass (rt_terrain_prepass_batch of all B frames into
one CameraResults buffer), alone on the GPU: the latency a rank pays between two k_traces at N > 1
(DESIGN.md section 7).  HIP events around R back-to-back prepasses on the batch's stream.
usage: [RT_LIB_VARIANT=name] python3 scripts/prepass_timing.py [B ...]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import with_variant  # noqa: E402

with_variant.apply()
import torch  # noqa: E402

import gpgpuraytrace_amd as G  # noqa: E402
from gpgpuraytrace_amd import engine as E  # noqa: E402

W, H = 1920, 1080
for B in [int(x) for x in sys.argv[1:]] or [1, 2, 4, 10, 12]:
    ring = E.FrameRing(W, H, depth=1, gpu=0, theme="nomadplains", camera=G.Camera(W, H), time_of_day=0.3,
                       max_steps=512, ao_samples=1, batch=B)
    ters = [t for _, t in ring.slots[:B]]
    buf = torch.zeros(B * 1024 * 4, dtype=torch.float32, device="cuda:0")
    torch.cuda.synchronize()
    stream = torch.cuda.ExternalStream(ring.slots[0][0].stream(), device="cuda:0")
    for _ in range(3):
        E.prepass_batch(ters, 0, B, buf.data_ptr())
    ring.synchronize()
    R = 20
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(R):
        E.prepass_batch(ters, 0, B, buf.data_ptr())
    e1.record(stream)
    e1.synchronize()
    print("%-8s B=%2d prepass %.4f ms" % (os.environ.get("RT_LIB_VARIANT", "product"), B, e0.elapsed_time(e1) / R),
          flush=True)
    ring.destroy()
