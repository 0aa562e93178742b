"""Predict multi-GPU strong scaling of frame batches on one GPU: for each N and each rank r < N,
time rank r's share (tile-cyclic, rt_terrain_render_batch(.., r, N)) of B-frame batches with D
batches in flight (engine.FrameRing(depth=D, batch=B)), steady state.  The N-GPU frame time is
bounded below by max_r of these (plus the gather), so t(N=1) / max_r t(r, N) is the ceiling.
Usage: python scripts/batch_shard_sim.py [--batches 1,4,8] [--depth 2] [--ns 1,2,4,8]

--barrier-model: the split prepass's all-gather couples the ranks every batch.
Per rank and batch, one batch at a time on the card (synchronised), it times the rank's prepass
chunk P_r(b), the full B-frame prepass P(b) and the rank's trace T_r(b) (setTargetDepths +
tracescreen of its shard), and models
  recompute (no collective before the trace):  max_r sum_b (P(b) + T_r(b))
  split, no barrier (the earlier, optimistic reading):     max_r sum_b (P_r(b) + T_r(b))
  split + all-gather barrier:  sum_b [max_r (T_r(b-1) + P_r(b)) + L]
(rank r's prepass chunk of batch b runs when its trace of batch b-1 ends, since k_trace holds every
CU; batch b's trace starts on every rank once the slowest rank's chunk is in and the all-gather,
L = --gather-us, has run), each divided by the frames.
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
    ap.add_argument("--barrier-model", action="store_true")
    ap.add_argument("--no-prepass", action="store_true",
                    help="diagnostic bound for a prepass fused into the previous batch's trace: every batch traces "
                         "from CameraResults computed once before timing (rt_terrain_trace_batch), no prepass "
                         "in the timed loop")
    ap.add_argument("--lookahead", type=int, default=0,
                    help="1: FrameRing(lookahead=True), each batch's prepass queued on the GPU's side stream before "
                         "the previous batch's trace (rt_terrain_prepass_ahead); 0 (bench.py's default): in line")
    ap.add_argument("--hw-queues", type=int, default=8,
                    help="GPU_MAX_HW_QUEUES for this process (bench.py sets 8; 0 = leave the environment's)")
    ap.add_argument("--extra-streams", type=int, default=0,
                    help="diagnostic: K torch streams kept busy-free but alive (HW queue sharing study)")
    ap.add_argument("--gather-us", type=float, default=40.0,
                    help="modelled all-gather latency per batch (16 KiB per frame over xGMI)")
    ap.add_argument("--transport-us", type=float, default=0.0,
                    help="N > 1: after each batch, on its stream, bench.py's transport as a stand-in: the rank's "
                         "rt_shard_pack_batch, a one-block spin kernel of this many us for the RCCL gather (it "
                         "needs a CU like RCCL's kernels do; 200 us ~ rank 0 receiving 7 x 10 frames' shards "
                         "over xGMI), and rank 0's rt_shard_unpack_batch of the other ranks' (N-1) x B shards")
    ap.add_argument("--transport-model", choices=["local", "coupled"], default="local",
                    help="with --transport-us: local = every rank's stand-in spins --transport-us on its own; coupled "
                         "= rank 0's receive stand-in (after its batch's trace, on the batch stream) spins "
                         "--transport-us and stores when it started, and rank r > 0's send stand-in holds its CU "
                         "until rank 0's receive of that batch started plus --transport-us (rank 0 runs first; the "
                         "ranks' timed regions are aligned at their start): a peer's send waits for rank 0's "
                         "receive, which queues behind rank 0's other-batch trace kernel")
    ap.add_argument("--direct-pack", type=int, default=1,
                    help="N > 1: ranks > 0 render their shards straight into the packed buffer "
                         "(rt_terrain_render_batch_packed, bench.py's default) and nobody packs; 0: render + "
                         "rt_shard_pack_batch on every rank (round 4)")
    ap.add_argument("--gate", type=int, default=0,
                    help="with --transport-us: each batch's prepass (rt_terrain_prepass_batch) is queued at once, its "
                         "trace (rt_terrain_trace_batch) after an event recorded behind the previous batch's pack, "
                         "so the previous batch's finish and pack run before this k_trace takes the CUs and its "
                         "gather finds a CU beside it")
    ap.add_argument("--reserve-cus", type=int, default=0,
                    help="N > 1: the trace kernels of the ranks below (--reserve-ranks) leave this many CUs free "
                         "(rt_device_reserve_cus), so rank 0's receive need not wait for its other-batch trace")
    ap.add_argument("--reserve-ranks", choices=["first", "all"], default="first")
    a = ap.parse_args()
    if a.hw_queues:
        os.environ["GPU_MAX_HW_QUEUES"] = str(a.hw_queues)  # before HIP starts (torch below)
    if a.barrier_model:
        return barrier_model(a)
    import torch
    import gpgpuraytrace_amd as G
    W, H = a.width, a.height
    extra = [torch.cuda.Stream(device="cuda:0") for _ in range(a.extra_streams)]
    for st in extra:  # each stream runs one op, so it holds its hardware queue
        with torch.cuda.stream(st):
            torch.zeros(1, device="cuda:0").add_(1)
    torch.cuda.synchronize()
    cam = G.Camera(W, H)
    base = None
    for B in [int(x) for x in a.batches.split(",")]:
        ring = G.FrameRing(W, H, depth=a.depth, batch=B, camera=cam, time_of_day=0.3, max_steps=a.max_steps,
                           ao_samples=a.ao, lookahead=bool(a.lookahead) and not a.split_prepass)
        bufs = []
        for g in range(a.depth):
            ters = [t for _, t in ring.slots[g * B:(g + 1) * B]]
            bufs.append(torch.zeros(B * 1024 * 4, dtype=torch.float32, device="cuda:0"))
            G.engine.prepass_batch(ters, 0, B, bufs[g].data_ptr())
        torch.cuda.synchronize()

        plan_n = {}

        def plan_for(n):
            from gpgpuraytrace_amd import parallel as P
            if n not in plan_n:
                plan = P.BatchPlan(W, H, B, n)
                plan_n[n] = (plan, [torch.zeros(plan.packed_bytes(), dtype=torch.uint8, device="cuda:0")
                                    for _ in range(a.depth)])
                torch.cuda.synchronize()
            return plan_n[n]

        # coupled model: rank 0's receive starts (100 MHz GPU clock, per timed batch) and each pass's t0
        clock = torch.zeros(64, dtype=torch.int64, device="cuda:0")  # [0] t0 of the pass, [1 + i] rank 0's recv i
        recv_off = {}  # n -> [rank 0's receive start of timed batch i - its t0] (ticks)
        trace_end_ms = {}  # n -> [rank 0's trace end of timed batch i - the pass's start] (ms, HIP events)
        xfer_ticks = int(a.transport_us * 100)  # 100 MHz

        trace_end = {}  # timed batch i -> a timing event recorded on its stream right after its trace (rank 0)

        def transport(r, n, i):
            """i: the timed batch's index (-1: warm-up)"""
            if r == 0 and i >= 0 and n > 1:
                g = ((ring.frame - B) // B) % ring.depth
                ev = torch.cuda.Event(enable_timing=True)
                ev.record(torch.cuda.ExternalStream(ring.slots[g * B][0].stream(), device="cuda:0"))
                trace_end[i] = ev
            if n == 1 or a.transport_us <= 0:
                return
            plan, packed = plan_for(n)
            g = ((ring.frame - B) // B) % ring.depth  # the batch just queued
            grp = ring.slots[g * B:(g + 1) * B]
            devs = [d for d, _ in grp]
            base = packed[g].data_ptr()
            if not a.direct_pack:
                items = plan.packs(r)
                G.engine.shard_pack_batch([devs[f] for f, _, _ in items], [s for _, s, _ in items], n,
                                          [base + off for _, _, off in items])
            stream = devs[0].stream()
            with torch.cuda.stream(torch.cuda.ExternalStream(stream, device="cuda:0")):
                if a.gate:
                    gate[0] = torch.cuda.Event()
                    gate[0].record()
                if a.transport_model == "local" or i < 0:
                    torch.cuda._sleep(int(a.transport_us * 2400))  # clock64 ticks ~2.4 per ns (tests: 50e6 ~ 20 ms)
                elif r == 0:  # the receive: stamped, then the transfer time
                    G.lib().rt_debug_spin(stream, None, 0, xfer_ticks, clock.data_ptr() + 8 * (1 + i))
                else:  # the send: holds its CU until rank 0's receive of this batch started, plus the transfer
                    G.lib().rt_debug_spin(stream, clock.data_ptr(), recv_off[n][i], xfer_ticks, None)
            if r == 0:
                ups = plan.unpacks()
                G.engine.shard_unpack_batch([devs[f] for _, f, _, _ in ups], [s for _, _, s, _ in ups], n,
                                            [base + off for _, _, _, off in ups])

        def step(r, n, ahead=True, i=-1):
            step_(r, n, ahead)
            transport(r, n, i)

        gate = [None]

        def step_(r, n, ahead=True):
            if a.gate and n > 1 and not a.split_prepass and not a.no_prepass:
                g = (ring.frame // B) % ring.depth
                grp = ring.slots[g * B:(g + 1) * B]
                ters = [t for _, t in grp]
                G.engine.prepass_batch(ters, 0, B, bufs[g].data_ptr())
                if gate[0] is not None:
                    grp[0][0].wait_event(gate[0].cuda_event)
                G.engine.trace_batch(ters, r, n, bufs[g].data_ptr())
                ring.frame += B
                return
            if a.no_prepass:
                g = (ring.frame // B) % ring.depth
                G.engine.trace_batch([t for _, t in ring.slots[g * B:(g + 1) * B]], r, n, bufs[g].data_ptr())
                ring.frame += B
                return
            if a.direct_pack and n > 1 and r > 0 and not a.split_prepass and not ring.lookahead:
                plan, packed = plan_for(n)
                g = (ring.frame // B) % ring.depth
                G.engine.render_batch_packed([t for _, t in ring.slots[g * B:(g + 1) * B]], r, n,
                                             packed[g].data_ptr(), plan.max_bytes)
                ring.frame += B
                return
            if not a.split_prepass or n == 1:
                ring.render_batch(r, n, present=False, ahead=ahead)
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
                res = a.reserve_cus if n > 1 and (r == 0 or a.reserve_ranks == "all") else 0
                for d, _ in ring.slots:
                    d.reserve_cus(res)
                for i in range(2 * a.depth):  # (lookahead: no ahead prepass across the timed region's edges)
                    step(r, n, ahead=i + 1 < 2 * a.depth)
                torch.cuda.synchronize()
                nb = max(1, a.frames // B)
                G.lib().rt_debug_spin(None, None, 0, 0, clock.data_ptr())  # the pass's t0 (GPU clock)
                ev0 = torch.cuda.Event(enable_timing=True)
                ev0.record()
                trace_end.clear()
                t0 = time.perf_counter()
                for i in range(nb):
                    step(r, n, ahead=i + 1 < nb, i=i)
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) / (nb * B) * 1e3
                if r == 0 and n > 1 and a.transport_model == "coupled" and a.transport_us > 0:
                    c = clock.cpu().tolist()
                    recv_off[n] = [max(0, c[1 + i] - c[0]) for i in range(nb)]
                if r == 0 and n > 1:
                    trace_end_ms[n] = [round(ev0.elapsed_time(trace_end[i]), 4) for i in sorted(trace_end)]
                per.append(round(ms, 4))
                worst = max(worst, ms)
            if base is None:
                base = worst
            print(json.dumps({"batch": B, "depth": a.depth, "split_prepass": a.split_prepass, "no_prepass": a.no_prepass,
                              "transport_us": a.transport_us, "transport_model": a.transport_model,
                              "direct_pack": a.direct_pack, "gate": a.gate,
                              **({"rank0_recv_start_ms": [round(x / 1e5, 4) for x in recv_off[n]]} if n in recv_off else {}),
                              **({"rank0_trace_end_ms": trace_end_ms[n]} if n in trace_end_ms else {}),
                              "reserve_cus": a.reserve_cus, "reserve_ranks": a.reserve_ranks,
                              "lookahead": int(ring.lookahead), "n": n, "worst_frame_ms": round(worst, 4),
                              "ceiling_vs_first": round(base / worst, 3), "ranks_ms": per}), flush=True)
        ring.destroy()


def barrier_model(a):
    import torch
    import gpgpuraytrace_amd as G
    W, H = a.width, a.height
    cam = G.Camera(W, H)

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3

    for B in [int(x) for x in a.batches.split(",")]:
        ring = G.FrameRing(W, H, depth=1, batch=B, camera=cam, time_of_day=0.3, max_steps=a.max_steps,
                           ao_samples=a.ao)
        ters = [t for _, t in ring.slots[:B]]
        buf = torch.zeros(B * 1024 * 4, dtype=torch.float32, device="cuda:0")
        nb = max(2, a.frames // B)
        for n in [int(x) for x in a.ns.split(",")]:
            chunk = -(-B // n)
            P, Pr, T = [], [], []  # P[b], Pr[r][b], T[r][b] in ms
            for r in range(n):
                lo, cnt = min(r * chunk, B), max(0, min(B - r * chunk, chunk))
                pr, tr = [], []
                for b in range(nb + 1):  # the first batch warms up
                    if r == 0:
                        p = timed(lambda: G.engine.prepass_batch(ters, 0, B, buf.data_ptr()))
                        if b:
                            P.append(p)
                    else:
                        G.engine.prepass_batch(ters, 0, B, buf.data_ptr())
                    p = timed(lambda: G.engine.prepass_batch(ters, lo, cnt, buf.data_ptr())) if cnt else 0.0
                    t = timed(lambda: G.engine.trace_batch(ters, r, n, buf.data_ptr()))
                    if b:
                        pr.append(p)
                        tr.append(t)
                Pr.append(pr)
                T.append(tr)
            frames = nb * B
            recompute = max(sum(P[b] + T[r][b] for b in range(nb)) for r in range(n)) / frames
            split_free = max(sum(Pr[r][b] + T[r][b] for b in range(nb)) for r in range(n)) / frames
            L = a.gather_us / 1e3 if n > 1 else 0.0
            # batch 0's chunk starts at time 0 on every rank; batch b's chunk after the rank's trace of b-1
            split_barrier = (max(Pr[r][0] for r in range(n)) + L
                             + sum(max(T[r][b - 1] + Pr[r][b] for r in range(n)) + L for b in range(1, nb))
                             + max(T[r][nb - 1] for r in range(n))) / frames
            print(json.dumps({"batch": B, "n": n, "batches": nb, "gather_us": a.gather_us,
                              "ms_per_frame": {"recompute": round(recompute, 4), "split_no_barrier": round(split_free, 4),
                                               "split_barrier": round(split_barrier, 4)},
                              "prepass_full_ms": round(sum(P) / len(P), 4),
                              "prepass_chunk_ms": [round(sum(x) / len(x), 4) for x in Pr],
                              "trace_ms": [round(sum(x) / len(x), 4) for x in T],
                              "trace_spread_ms": [round(max(x) - min(x), 4) for x in T]}), flush=True)
        ring.destroy()


if __name__ == "__main__":
    main()
