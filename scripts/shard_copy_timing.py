"""Rank 0's per-batch unpack at N GPUs, timed on one GPU: (N-1) x B shards of 1920x1080 frames
(rotated shards, parallel.BatchPlan offsets) through one rt_shard_unpack call per shard (the
round-2 sequence) against one rt_shard_unpack_batch launch, both on the batch's stream, plus the
pack of a rank's B frames the same two ways.  HIP events on that stream; medians of 20 repeats.
usage: python scripts/shard_copy_timing.py [world ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gpgpuraytrace_amd as G  # noqa: E402
from gpgpuraytrace_amd import engine as E  # noqa: E402
from gpgpuraytrace_amd import parallel as P  # noqa: E402

W, H, B = 1920, 1080, 12


def timed(stream, fn, reps=20):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(stream):
            a.record()
            fn()
            b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[len(ts) // 2]


def main():
    worlds = [int(x) for x in sys.argv[1:]] or [2, 4, 8]
    devs = [G.DeviceFactory.construct(G.DeviceAPI.HIP, W, H) for _ in range(B)]
    for d in devs[1:]:
        d.set_stream(devs[0].stream())  # a FrameRing slot group: one stream per batch
    stream = torch.cuda.ExternalStream(devs[0].stream(), device="cuda:0")
    for world in worlds:
        plan = P.BatchPlan(W, H, B, world)
        gathered = [torch.zeros(plan.packed_bytes(), dtype=torch.uint8, device="cuda:0") for _ in range(world)]
        ups = plan.unpacks()
        packs = plan.packs(0)

        def unpack_each():
            for src, f, s, off in ups:
                E.shard_unpack(devs[f], s, world, gathered[src].data_ptr() + off)

        def unpack_batch():
            E.shard_unpack_batch([devs[f] for _, f, _, _ in ups], [s for _, _, s, _ in ups], world,
                                 [gathered[src].data_ptr() + off for src, _, _, off in ups])

        def pack_each():
            for f, s, off in packs:
                E.shard_pack(devs[f], s, world, gathered[0].data_ptr() + off)

        def pack_batch():
            E.shard_pack_batch([devs[f] for f, _, _ in packs], [s for _, s, _ in packs], world,
                               [gathered[0].data_ptr() + off for _, _, off in packs])

        for fn in (unpack_each, unpack_batch, pack_each, pack_batch):
            fn()
        torch.cuda.synchronize()
        mb = len(ups) * plan.max_bytes / 2**20
        print(f"N={world} B={B}: unpack {len(ups)} shards ({mb:.0f} MiB): {timed(stream, unpack_each):.3f} ms "
              f"one call each, {timed(stream, unpack_batch):.3f} ms batched; pack {len(packs)}: "
              f"{timed(stream, pack_each):.3f} ms each, {timed(stream, pack_batch):.3f} ms batched", flush=True)
    for d in devs[1:]:
        d.destroy()
    devs[0].destroy()


if __name__ == "__main__":
    main()
