"""Predict multi-GPU strong scaling of frame batches on one GPU: for each N and each rank r < N,
time rank r's share (tile-cyclic, rt_terrain_render_batch(.., r, N)) of B-frame batches with D
batches in flight (engine.FrameRing(depth=D, batch=B)), steady state.  The N-GPU frame time is
bounded below by max_r of these (plus the gather), so t(N=1) / max_r t(r, N) is the ceiling.
Usage: python scripts/batch_shard_sim.py [--batches 1,4,8] [--depth 2] [--ns 1,2,4,8]
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
    ap.add_argument("--frames", type=int, default=24, help="frames timed per (B, N, rank)")
    ap.add_argument("--batches", default="1,4,8")
    ap.add_argument("--depth", type=int, default=2)
    ap.add_argument("--ns", default="1,2,4,8")
    ap.add_argument("--ranks", default="all", help="'all' or 'first' (rank 0 only: quick)")
    ap.add_argument("--split-prepass", type=int, default=0,
                    help="1: rank r runs only its ceil(B/N) frames' prepass (bench.py --split-prepass; the "
                         "all-gather is not simulated: the other frames' CameraResults come from a full prepass "
                         "run once before timing)")
    a = ap.parse_args()
    import torch
    import gpgpuraytrace_amd as G
    W, H = a.width, a.height
    cam = G.Camera(W, H)
    base = None
    for B in [int(x) for x in a.batches.split(",")]:
        ring = G.FrameRing(W, H, depth=a.depth, batch=B, camera=cam, time_of_day=0.3, max_steps=a.max_steps,
                           ao_samples=a.ao)
        bufs = []
        for g in range(a.depth):
            ters = [t for _, t in ring.slots[g * B:(g + 1) * B]]
            bufs.append(torch.zeros(B * 1024 * 4, dtype=torch.float32, device="cuda:0"))
            G.engine.prepass_batch(ters, 0, B, bufs[g].data_ptr())
        torch.cuda.synchronize()

        def step(r, n):
            if not a.split_prepass or n == 1:
                ring.render_batch(r, n, present=False)
                return
            g = (ring.frame // B) % ring.depth
            ters = [t for _, t in ring.slots[g * B:(g + 1) * B]]
            chunk = -(-B // n)
            G.engine.prepass_batch(ters, min(r * chunk, B), max(0, min(B - r * chunk, chunk)), bufs[g].data_ptr())
            G.engine.trace_batch(ters, r, n, bufs[g].data_ptr())
            ring.frame += B
        for n in [int(x) for x in a.ns.split(",")]:
            worst, per = 0.0, []
            for r in (range(n) if a.ranks == "all" else [0]):
                for _ in range(2 * a.depth):
                    step(r, n)
                torch.cuda.synchronize()
                nb = max(1, a.frames // B)
                t0 = time.perf_counter()
                for _ in range(nb):
                    step(r, n)
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) / (nb * B) * 1e3
                per.append(round(ms, 4))
                worst = max(worst, ms)
            if base is None:
                base = worst
            print(json.dumps({"batch": B, "depth": a.depth, "split_prepass": a.split_prepass, "n": n, "worst_frame_ms": round(worst, 4),
                              "ceiling_vs_first": round(base / worst, 3), "ranks_ms": per}), flush=True)
        ring.destroy()


if __name__ == "__main__":
    main()
