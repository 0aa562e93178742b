#!/usr/bin/env python3
"""bench.py -- Mray/s + ms/frame at 1920x1080 on 1..8 MI355X (BASELINE.json metric).

A "step" is one frame of the hot path: camerarays prepass -> setTargetDepths
(on the GPU) -> tracescreen (primary march + normal + colour + shadow march + sky
[+ AO]) over the whole frame, nomadplains landscape, noise seed 300 (MSVC rand),
camera reset pose, time of day 0.3, AA 1.

Default workload = BASELINE.json configs[2] ("C3", the config the 1920x1080 metric
is quoted on): 1920x1080, 512-step primary cap + one shadow ray per hit + one
"1-bounce AO" ray per hit (both build extensions; the AO
definition is rt_shader.h ao_dir / oracle ambient_occlusion).  --config ref runs the
reference semantics (uncapped march, no AO); c2 / c5 are the other GPU configs.

N>1: the frame's 32x32-pixel tiles are dealt tile-cyclically over the ranks (strong
scaling: the frame is fixed), each rank packs its tiles and one RCCL gather to rank 0
assembles the frame, which rank 0 unpacks into its framebuffer.

Frames in flight (--frames-in-flight, default 2): the timed loop deals frames round-robin
over D complete frame contexts, each on its own HIP stream (engine.FrameRing), so frame
i+1's prepass and primary phase fill the CUs that frame i's ray tail leaves idle.  Every
frame is still computed in full; value / ms_per_step are the steady-state frame rate, and
config.frame_latency_ms is the one-frame-at-a-time time of the same frame.

Prints ONE JSON line on rank 0 (driver contract), with "roofline" for the dominant
kernel (tracescreen, timed by HIP events on its own stream in a pass with one frame in
flight, so launches do not overlap) and "cpu_baseline" (the C oracle on a bounded row
sample, rank 0 at N=1 only).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mray/s + ms/frame at 1920×1080, 1/2/4/8 MI355X; % HBM roofline"
FLOPS_PER_NOISE3D = 88          # algorithmic work unit
PEAK_FP32_VECTOR_TFLOPS = 157.3 # MI355X_MICROARCH.md chip table (vector FP32, = FP32 MFMA dense)
PEAK_HBM_GBS = 8000.0
# BASELINE.json configs (GPU ones): resolution, primary step cap, AO rays per hit
CONFIGS = {
    "c2": {"width": 1280, "height": 720, "max_steps": 256, "ao": 0,
           "name": "C2: 1280x720, 256-step primary + 1 shadow ray"},
    "c3": {"width": 1920, "height": 1080, "max_steps": 512, "ao": 1,
           "name": "C3: 1920x1080, 512-step primary + shadow + 1-bounce AO"},
    "c5": {"width": 3840, "height": 2160, "max_steps": 1024, "ao": 4,
           "name": "C5: 3840x2160, 1024-step primary + shadow + 4 AO samples"},
    "ref": {"width": 1920, "height": 1080, "max_steps": 0, "ao": 0,
            "name": "1920x1080, reference semantics (uncapped march, shadow, no AO)"},
}

# what one tracescreen launch (the HIP-event-timed region) runs, per RT_PIPELINE
TRACESCREEN_KERNELS = {"split": "tracescreen = k_order + k_trace + k_shade_pre + k_shadow + k_finish",
                       "staged": "tracescreen = k_order + k_primary + k_shade_pre + k_shadow + k_finish",
                       "refill": "tracescreen = k_march + k_shade_pre + k_shadow + k_finish",
                       "mega": "tracescreen = k_tracescreen"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--landscape", default="nomadplains")
    ap.add_argument("--pose", choices=["reset", "lookdown"], default="reset")
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c3",
                    help="BASELINE.json config preset (resolution, step cap, AO rays); explicit flags override")
    ap.add_argument("--max-steps", type=int, default=None, help="primary-march cap (build extension); 0 = reference")
    ap.add_argument("--ao", type=int, default=None, help="AO rays per primary hit (build extension); 0 = off")
    ap.add_argument("--frames-in-flight", type=int, default=2,
                    help="frame contexts (HIP streams) kept in flight; 1 = one frame at a time (with --batch B: "
                         "batches of B frames in flight)")
    ap.add_argument("--batch", type=int, default=12,
                    help="frames per rt_terrain_render_batch launch sequence (1..16); the timed loop renders whole "
                         "batches (steps rounded up to a multiple)")
    ap.add_argument("--split-prepass", type=int, default=1,
                    help="N>1: each rank runs the prepass of B/N frames of a batch and one all-gather shares them "
                         "(0 = every rank runs every frame's prepass)")
    ap.add_argument("--graph", type=int, default=None,
                    help="1 = every slot replays its frame as captured hipGraphs (RT_DEVICE_GRAPH), 0 = direct "
                         "launches; default: on for c5 (BASELINE's hipGraph-captured frame loop), off otherwise")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verify", action="store_true",
                    help="after the timed loop rank 0 checks every assembled frame of the last batch against a "
                         "whole-frame render on one device (RGBA8, bit for bit); adds config.verify")
    ap.add_argument("--cpu-row-step", type=int, default=1)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "r01", "traffic.json"),
                    help="PMC-derived HBM bytes per tracescreen launch (from rocprofv3 --pmc), if present")
    a = ap.parse_args()
    preset = CONFIGS[a.config]
    for key in ("width", "height", "max_steps", "ao"):
        if getattr(a, key) is None:
            setattr(a, key, preset[key])
    if a.graph is None:
        a.graph = 1 if a.config == "c5" else 0
    return a


def cpu_baseline(consts, landscape, max_steps, ao, row_step, threads):
    """Oracle (scalar C restatement, OpenMP over rows) on a bounded row sample of the same frame."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import oracle_lib as O
    nz = O.noise_tables()
    fr = O.make_frame(consts, landscape=O.LANDSCAPES[landscape], max_steps=max_steps,
                      rows=(0, consts["height"], row_step), threads=threads, ao=ao)
    import ctypes as C
    cr = np.zeros(1024 * 4, np.float32)
    cd = np.zeros(1024 * 2, np.float32)
    st = O.Stats()
    t0 = time.perf_counter()
    O.lib().ro_camerarays(C.byref(nz), C.byref(fr), O._fp(cr), C.byref(st))
    O.lib().ro_set_target_depths(O._fp(cr), O._fp(cd))
    O.lib().ro_tracescreen(C.byref(nz), C.byref(fr), O._fp(cd), None, None, None, C.byref(st))
    dt = time.perf_counter() - t0
    s = st.as_dict()
    rays = s["primary_rays"] + s["primary_hits"] + s["ao_rays"] + 1024
    return {"value": round(rays / dt / 1e6, 4), "unit": "Mray/s", "cores": threads,
            "kind": "port",
            "sample": f"oracle/rt_oracle.c, prepass + rows 0::{row_step} of the {consts['width']}x{consts['height']} "
                      f"frame ({s['primary_rays']} primary + {s['primary_hits']} shadow + {s['ao_rays']} AO + "
                      f"1024 prepass rays, {dt:.1f} s, {threads} OpenMP threads)"}


def main():
    a = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the N>1 path on one GPU (RT_BENCH_SAME_GPU=1: every rank on cuda:0, with
    # RT_DIST_BACKEND=gloo: collectives staged through host memory); the default is RCCL
    backend = os.environ.get("RT_DIST_BACKEND", "nccl")
    if os.environ.get("RT_BENCH_SAME_GPU") == "1":
        local = 0
    if world > 1:
        dist.init_process_group(backend)
    torch.cuda.set_device(local)

    def all_gather(out, mine, group):
        if backend == "nccl":
            dist.all_gather_into_tensor(out, mine, group=group)
            return
        parts = [torch.empty(mine.numel(), dtype=mine.dtype) for _ in range(world)]
        dist.all_gather(parts, mine.cpu(), group=group)
        out.copy_(torch.cat(parts).to(out.device))

    def gather(t, outs):
        if backend == "nccl":
            dist.gather(t, outs if rank == 0 else None, dst=0)
            return
        lst = [torch.empty(t.numel(), dtype=t.dtype) for _ in range(world)] if rank == 0 else None
        dist.gather(t.cpu(), lst, dst=0)
        if rank == 0:
            for o, part in zip(outs, lst):
                o.copy_(part.to(o.device))

    import gpgpuraytrace_amd as G
    from gpgpuraytrace_amd import engine as E

    euler = G.camera.INITIAL_ROTATION_EULER if a.pose == "reset" else G.camera.LOOKDOWN_ROTATION_EULER
    W, H = a.width, a.height

    def make(stats):
        dev = G.DeviceFactory.construct(G.DeviceAPI.HIP, W, H, gpu=local, stats=stats)
        if dev is None:
            raise RuntimeError("device create failed: " + G.lib().rt_last_error().decode())
        ter = G.Terrain(dev, a.landscape, max_steps=a.max_steps, ao_samples=a.ao)
        ter.create()
        if not ter.reload():
            raise RuntimeError("shader load failed: " + G.lib().rt_last_error().decode())
        ter.set_camera(G.Camera(W, H, euler=euler))
        ter.set_time_of_day(0.3)
        return dev, ter

    # --- instrumented frame (untimed): exact ray and noise3d counts of this frame ---
    sdev, ster = make(stats=True)
    ster.update_shaders()
    ster.camera_compute.run(2, 2, 1)
    pre = sdev.stats(reset=True)
    ster.render_device(rank if world > 1 else 0, world)
    full = sdev.stats(reset=True)
    sdev.synchronize()
    shard_noise = full["noise_calls"] - pre["noise_calls"]
    # a batch's frame f traces shard (rank + f) % world (per-frame rotation): its launch's noise count
    B = max(1, min(16, a.batch))
    per_shard = {rank % world if world > 1 else 0: shard_noise}
    if world > 1 and B > 1:
        for s in {(rank + f) % world for f in range(B)} - set(per_shard):
            ster.camera_compute.run(2, 2, 1)
            pre = sdev.stats(reset=True)
            ster.render_device(s, world)
            per_shard[s] = sdev.stats(reset=True)["noise_calls"] - pre["noise_calls"]
        sdev.synchronize()
    batch_noise = (sum(per_shard[(rank + f) % world] for f in range(B)) if world > 1 and B > 1
                   else B * shard_noise)
    # whole-frame counts (all shards) for the ray total
    if world > 1:
        ster.render_device(0, 1)
        whole = sdev.stats(reset=True)
    else:
        whole = full
    hits = whole["hits"]
    rays_per_frame = W * H + hits + hits * a.ao + 1024
    sdev.destroy()

    # --- timed: D frames in flight (FrameRing: one full frame context + HIP stream per slot) ---
    camera = G.Camera(W, H, euler=euler)
    ring = E.FrameRing(W, H, depth=a.frames_in_flight, gpu=local, theme=a.landscape, camera=camera,
                       time_of_day=0.3, max_steps=a.max_steps, ao_samples=a.ao, graph=bool(a.graph), batch=B)
    packed, gathered = {}, {}
    if world > 1:
        nb = [E.shard_bytes(ring.slots[0][0], r, world) for r in range(world)]
        maxb = max(nb)
        for g in range(ring.depth):  # one packed buffer per batch slot: the batch's B shards back to back
            packed[g] = torch.zeros(B * maxb, dtype=torch.uint8, device=f"cuda:{local}")
            if rank == 0:
                gathered[g] = [torch.zeros(B * maxb, dtype=torch.uint8, device=f"cuda:{local}") for _ in range(world)]
        group_streams = [torch.cuda.ExternalStream(ring.slots[g * B][0].stream(), device=f"cuda:{local}")
                         for g in range(ring.depth)]
        # split prepass: rank r runs the prepass of frames [r*chunk, (r+1)*chunk) of each batch and
        # one all-gather (its own communicator, so it never queues behind the frame gathers)
        # hands every rank all B frames' CameraResults before its trace
        chunk = -(-B // world)
        pre_group = dist.new_group(backend=backend) if a.split_prepass else None
        cam_bufs = [torch.zeros(world * chunk * 1024 * 4, dtype=torch.float32, device=f"cuda:{local}")
                    for _ in range(ring.depth)]

    def batch_step():
        g = (ring.frame // B) % ring.depth
        if world > 1 and a.split_prepass:
            group = ring.slots[g * B:(g + 1) * B]
            ters = [t for _, t in group]
            devs = [d for d, _ in group]
            first = min(rank * chunk, B)  # ranks past the batch's last frame (B < world * chunk) run none
            E.prepass_batch(ters, first, min(B - first, chunk), cam_bufs[g].data_ptr())
            with torch.cuda.stream(group_streams[g]):
                mine = cam_bufs[g][rank * chunk * 4096:(rank + 1) * chunk * 4096]
                all_gather(cam_bufs[g], mine, pre_group)
            E.trace_batch(ters, rank, world, cam_bufs[g].data_ptr())
            ring.frame += B
        else:
            devs = ring.render_batch(rank if world > 1 else 0, world, present=world == 1)
        if world > 1:
            # one gather per batch rides on the batch's stream, so the other batches keep running
            with torch.cuda.stream(group_streams[g]):
                # (a batch's devices share its stream: FrameRing)
                for f, dev in enumerate(devs):
                    E.shard_pack(dev, (rank + f) % world, world, packed[g].data_ptr() + f * maxb)  # frame f: shard (rank + f) % world
                gather(packed[g], gathered[g] if rank == 0 else None)
                if rank == 0:
                    for r in range(1, world):
                        for f, dev in enumerate(devs):
                            E.shard_unpack(dev, (r + f) % world, world, gathered[g][r].data_ptr() + f * maxb)
            for dev in devs:
                dev.present()

    n_batches = -(-a.steps // B)
    frames_timed = n_batches * B
    for _ in range(-(-a.warmup // B) + ring.depth):
        batch_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n_batches):
        batch_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0

    verify = None
    if a.verify and rank == 0:
        # the last timed batch's frames, assembled from every rank's shards, against one whole frame
        g_last = ((ring.frame // B) - 1) % ring.depth
        vdev, vter = make(stats=False)
        vter.render_device(0, 1)
        want = vdev.readback()
        vdev.destroy()
        verify = all(np.array_equal(d.readback(), want) for d, _ in ring.slots[g_last * B:(g_last + 1) * B])

    # --- roofline pass: the same batches one at a time on slot group 0 (launches do not overlap),
    # HIP events around every tracescreen launch on the stream it runs on; also the latency ---
    group0 = ring.slots[:B]
    dev0 = group0[0][0]
    ring.set_profiling(True)
    ring.kernel_time()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(n_batches):
        E.render_batch([t for _, t in group0], rank if world > 1 else 0, world)
        for d, _ in group0:
            d.present()
    for d, _ in group0:
        d.synchronize()
    latency_ms = (time.perf_counter() - t1) / n_batches * 1e3
    kms, kn = ring.kernel_time()
    ring.set_profiling(False)
    k_avg_ms = kms / max(1, kn)  # one launch = a batch of B frames
    if world > 1:
        t = torch.tensor([elapsed, latency_ms], dtype=torch.float64,
                         device=f"cuda:{local}" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, latency_ms = float(t[0].item()), float(t[1].item())

    ms_per_frame = elapsed / frames_timed * 1e3
    value = rays_per_frame * frames_timed / elapsed / 1e6
    achieved = batch_noise * FLOPS_PER_NOISE3D / (k_avg_ms * 1e-3) / 1e12
    traffic = None
    if os.path.exists(a.traffic_json):
        try:
            with open(a.traffic_json) as f:
                tj = json.load(f)
            key = f"{W}x{H}_{a.landscape}_{a.pose}_ms{a.max_steps}_ao{a.ao}_b{B}"
            traffic = tj.get(key, {}).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    if rank == 0:
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "Mray/s", "n_gpus": world, "steps": frames_timed,
            "warmup": a.warmup, "ms_per_step": round(ms_per_frame, 4), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic: procedural nomadplains terrain, noise seed 300 (MSVC rand), fixed camera",
            "config": {
                "workload": f"{CONFIGS[a.config]['name'] if (W, H, a.max_steps, a.ao) == tuple(CONFIGS[a.config][k] for k in ('width', 'height', 'max_steps', 'ao')) else 'custom'}; "
                            f"{W}x{H} {a.landscape} frame ({a.pose} pose), camerarays prepass + device "
                            f"setTargetDepths + tracescreen (primary + normal + colour + shadow + sky"
                            f"{f' + {a.ao} AO ray(s) per hit' if a.ao else ''}), "
                            f"{'uncapped march (reference semantics)' if a.max_steps == 0 else f'{a.max_steps}-step primary cap'}",
                "width": W, "height": H, "landscape": a.landscape, "pose": a.pose, "aa_samples": 1,
                "max_steps": a.max_steps, "ao_samples": a.ao, "rays_per_frame": rays_per_frame, "primary_rays": W * H,
                "shadow_rays": hits, "ao_rays": hits * a.ao, "prepass_rays": 1024,
                "hit_fraction": round(hits / (W * H), 4),
                "noise3d_per_frame_tracescreen": shard_noise if world == 1 else None,
                "parallelism": "single GPU" if world == 1 else (
                    f"tile-cyclic 32x32 shards x{world} + RCCL gather per batch"
                    + (" + prepass split over ranks (RCCL all-gather of CameraResults)" if a.split_prepass else "")),
                "frames_in_flight": a.frames_in_flight * B,
                "batch": B,
                "frame_loop": "hipGraph replay per slot (prepass graph + tracescreen graph)" if a.graph
                              else "direct launches",
                "frame_latency_ms": round(latency_ms, 4),  # one batch of B frames at a time
                **({"verify": "frames equal a whole-frame render" if verify else "MISMATCH"}
                   if verify is not None else {}),
            },
            "roofline": {
                "bound": "valu", "achieved": round(achieved, 3), "peak": PEAK_FP32_VECTOR_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / PEAK_FP32_VECTOR_TFLOPS, 4), "traffic": traffic,
                "kernel": TRACESCREEN_KERNELS.get(os.environ.get("RT_PIPELINE", "split"), TRACESCREEN_KERNELS["split"]),
                "kernel_avg_ms": round(k_avg_ms, 4), "kernel_launches": kn,
                "timing": "HIP events per launch on its stream, one batch in flight (the last "
                          f"{kn} tracescreen launches of the run; one launch = {B} frames)",
                "work_unit": f"{FLOPS_PER_NOISE3D} FP32 flop per noise3d x {batch_noise} noise3d per launch ({B} "
                             f"frame(s); frame f traces shard (rank + f) % world)",
                "note": "FP32 vector-ALU bound (no MFMA-shaped or HBM-bound work); gfx950 vector FP32 peak "
                        "= FP32 dense matrix peak = 157.3 TFLOP/s",
            },
        }
        if world == 1 and not a.no_cpu_baseline:
            consts = G.frame_constants(W, H, euler=euler)
            threads = a.cpu_threads or min(16, os.cpu_count() or 1)
            out["cpu_baseline"] = cpu_baseline(consts, a.landscape, a.max_steps, a.ao, a.cpu_row_step, threads)
        print(json.dumps(out), flush=True)
    ring.destroy()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
