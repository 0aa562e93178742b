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

Frames are rendered in BATCHES (rt_terrain_render_batch: one launch sequence traces B frames)
with D batches in flight (engine.FrameRing).  Exactly --steps frames are timed: the steps are
split into ceil(steps / B) batches of near-equal size.  Every frame is computed in full and
independently; value / ms_per_step are the steady-state frame rate; config.frame_latency_ms is
one batch at a time, config.single_frame one frame per launch sequence (B = 1) with three frames
in flight, config.single_frame_serial the reference's frame loop (render + present, one frame per call)
on one device, config.single_frame_deferred the same loop on an RT_DEVICE_DEFERRED device (each render
launches the previous frame's trace with its own prepass inside it), config.moving_camera
the timed loop's batching over --steps distinct frames of a camera path, config.sustained the
timed loop's batches back to back for ~5 s (rates per ~1 s window: clocks under a long load), and
(C3) config.ref_semantics the same machinery at the reference's own semantics (uncapped, no AO).

N>1: the frame's 32x32-pixel tiles are dealt tile-cyclically over the ranks (strong
scaling: the frame is fixed); parallel.BatchPlan / run_batch hold the per-batch sequence
(every rank's prepass of the batch -- with --lookahead 1 queued one batch ahead on a side stream
-- or with --split-prepass 1 a B/N share + CameraResults all-gather; shard rotation, pack, one
RCCL gather to rank 0, unpack), which tests/test_dist.py drives with host ops over gloo.  With
lookahead the timed region holds exactly the prepasses of its own batches: the last warm-up
batch and the last timed batch queue no ahead prepass.

Prints ONE JSON line on rank 0 (driver contract), with "roofline" for the dominant
kernel (tracescreen, timed by HIP events on its own stream in a pass with one batch in
flight, so launches do not overlap) and "cpu_baseline" (the C oracle on the host cores, rank 0
at N=1 only; its frame is also compared with the GPU's: config.parity).
"""
import argparse
import json
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# One hardware queue per busy stream, set before HIP starts: the frame ring's
# slot-group streams, the ahead-prepass side stream, torch's and RCCL's.  With HIP's default of 4,
# two busy streams share a queue and the batches the ring overlaps run one after the other
# (profiles/r03/hw_queues.md: one-rank shard simulation at N=8, one extra stream alive,
# 0.397 -> 0.430 ms/frame; 8 queues: 0.398).
# (RT_BENCH_HW_QUEUES overrides the count for A/B runs)
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("RT_BENCH_HW_QUEUES", "8")

# A/B runs only: RT_BENCH_GATED=1 renders with RT_DEVICE_GATED (the gated launch: the prepass inside the trace
# kernel) instead of the default prepass launch before the trace
GATED = os.environ.get("RT_BENCH_GATED") == "1"
METRIC = "Mray/s + ms/frame at 1920×1080, 1/2/4/8 MI355X; % HBM roofline"
FLOPS_PER_NOISE3D = 88          # algorithmic work unit
PEAK_FP32_VECTOR_TFLOPS = 157.3 # MI355X_MICROARCH.md chip table (vector FP32, = FP32 MFMA dense)
# BASELINE.json configs (GPU ones): resolution, primary step cap, AO rays per hit, and the
# CPU baseline's row samples (all host cores: parity + value; one thread: single_thread)
CONFIGS = {
    "c1": {"width": 256, "height": 256, "max_steps": 64, "ao": 0, "cpu_rows": 1, "cpu_rows_1t": 1, "batch": 24,
           "name": "C1: 256x256, 64-step primary + shadow (the reference's CPU-scale plumbing case)"},
    "c2": {"width": 1280, "height": 720, "max_steps": 256, "ao": 0, "cpu_rows": 1, "cpu_rows_1t": 8,
           "name": "C2: 1280x720, 256-step primary + 1 shadow ray"},
    "c3": {"width": 1920, "height": 1080, "max_steps": 512, "ao": 1, "cpu_rows": 1, "cpu_rows_1t": 16,
           "name": "C3: 1920x1080, 512-step primary + shadow + 1-bounce AO"},
    "c5": {"width": 3840, "height": 2160, "max_steps": 1024, "ao": 4, "cpu_rows": 8, "cpu_rows_1t": 128,
           "name": "C5: 3840x2160, 1024-step primary + shadow + 4 AO samples"},
    "ref": {"width": 1920, "height": 1080, "max_steps": 0, "ao": 0, "cpu_rows": 1, "cpu_rows_1t": 16,
            "name": "1920x1080, reference semantics (uncapped march, shadow, no AO)"},
}
TRACESCREEN_KERNELS = "tracescreen = k_order + k_trace + k_finish"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=24, help="frames timed (exactly)")
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
                    help="batches (slot groups, one HIP stream each) kept in flight; 1 = one batch at a time")
    ap.add_argument("--batch", type=int, default=None,
                    help="max frames per rt_terrain_render_batch launch sequence (1..24; default 12, and 24 at 8 ranks or "
                         "more or for C1 whose 256x256 frames underfill the chip at 12: 855-871 against 703 Mray/s, "
                         "DESIGN.md section 5); "
                         "the --steps frames are split into ceil(steps / batch) batches of near-equal size")
    ap.add_argument("--split-prepass", type=int, default=0,
                    help="N>1: 1 = each rank runs the prepass of B/N frames of a batch and an all-gather shares "
                         "them (a second collective and a cross-rank barrier per batch); 0 (default, SURVEY 8e and "
                         "north_star's single gather) = every rank runs every frame's prepass.  The barrier model "
                         "(scripts/batch_shard_sim.py --barrier-model, profiles/r03/batch_shard_barrier.log) puts "
                         "the split's gain at <= 2%% (N=8)")
    ap.add_argument("--lookahead", type=int, default=0,
                    help="1 = the timed loop queues the next batch's prepass on the GPU's side stream before this "
                         "batch's trace (rt_terrain_prepass_ahead, DESIGN.md section 7); 0 (default) = each batch's "
                         "prepass in line on its slot group's stream (measured 0.6%% faster at B=12: "
                         "profiles/r03/hw_queues.md).  config.single_frame always runs it (B=1: +1.3%%)")
    ap.add_argument("--direct-pack", type=int, default=1,
                    help="N>1, in-line prepass: 1 (default) = ranks > 0 render their shards straight into the packed "
                         "gather buffer (rt_terrain_render_batch_packed, no pack launch) and rank 0 packs nothing; "
                         "0 = render, then rt_shard_pack_batch (round 4)")
    ap.add_argument("--graph", type=int, default=None,
                    help="1 = every slot replays its frame as captured hipGraphs (RT_DEVICE_GRAPH), 0 = direct "
                         "launches; default: on for c5 (BASELINE's hipGraph-captured frame loop), off otherwise")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-companions", action="store_true",
                    help="skip config.single_frame / config.ref_semantics (extra timed passes)")
    ap.add_argument("--sustained-s", type=float, default=5.0,
                    help="N=1 companion config.sustained: the timed loop's batches back to back for about this "
                         "many seconds (0 = skip)")
    ap.add_argument("--verify", action="store_true",
                    help="after the timed loop rank 0 checks every assembled frame of the last batch against a "
                         "whole-frame render on one device (RGBA8, bit for bit); adds config.verify (always on "
                         "at N>1)")
    ap.add_argument("--cpu-row-step", type=int, default=None, help="CPU baseline (all cores): every n-th row")
    ap.add_argument("--cpu-threads", type=int, default=0, help="CPU baseline threads (0 = the host's share)")
    ap.add_argument("--traffic", choices=["pmc", "off"], default="pmc",
                    help="pmc (N=1): measure roofline.traffic in this run, two rocprofv3 --pmc passes (FETCH_SIZE, "
                         "WRITE_SIZE) over one B-frame tracescreen launch in child processes; off: null")
    ap.add_argument("--traffic-child", action="store_true", help=argparse.SUPPRESS)
    a = ap.parse_args()
    preset = CONFIGS[a.config]
    for key in ("width", "height", "max_steps", "ao"):
        if getattr(a, key) is None:
            setattr(a, key, preset[key])
    if a.batch is None:
        # 12; 24 from 8 ranks on, where a 12-frame batch leaves each rank 1.5 frames of trace per launch and its
        # prepass, tail and gather dominate: the N = 8 coupled shard model 0.4327 -> 0.4189 ms/frame at 20 frames
        # (N = 2 / 4 prefer 12; N = 1 equal; profiles/r06/batch_by_ranks.md)
        ranks = int(os.environ.get("WORLD_SIZE", a.gpus))
        a.batch = preset.get("batch", 24 if ranks >= 8 else 12)
    if a.graph is None:
        a.graph = 1 if a.config == "c5" else 0
    if a.lookahead and a.graph:
        ap.error("--lookahead runs the prepass on a side stream: not with --graph 1")
    if a.cpu_row_step is None:
        a.cpu_row_step = preset["cpu_rows"]
    if a.steps < 1:
        ap.error("--steps must be >= 1")
    return a


def host_threads():
    """The CPU share this process may use: OMP_NUM_THREADS where the launcher sets it (16 on
    the GPU box), else the affinity mask."""
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        return int(env)
    return len(os.sched_getaffinity(0))


def batch_sizes(steps, batch):
    """ceil(steps / batch) batches of near-equal size summing to exactly `steps`."""
    n = -(-steps // batch)
    base, extra = divmod(steps, n)
    return [base + (1 if i < extra else 0) for i in range(n)]


def cpu_baseline(consts, landscape, max_steps, ao, row_step, row_step_1t, threads, gpu_rgba32f, gpu_rgba8,
                 timed_frames):
    """Oracle (scalar C restatement, OpenMP over rows) on the host cores: (1) all `threads` on
    rows 0::row_step (the reported value; its pixels are compared with the GPU's: the frames the
    timed loop rendered, `timed_frames` = [(label, rgba8)], and the instrumented whole frame's
    float32 colour), (2) one thread on rows 0::row_step_1t."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import oracle_lib as O
    nz = O.noise_tables()
    land = O.LANDSCAPES[landscape]

    def timed(rows, nthreads):
        fr = O.make_frame(consts, landscape=land, max_steps=max_steps, rows=rows, threads=nthreads, ao=ao)
        t0 = time.perf_counter()
        rgba, rgba8, _, _, s = O.render_rows(nz, fr)
        dt = time.perf_counter() - t0
        rays = s["primary_rays"] + s["primary_hits"] + s["ao_rays"] + 1024
        return rgba, rgba8, s, rays, dt

    H, W = consts["height"], consts["width"]
    rgba, rgba8, s, rays, dt = timed((0, H, row_step), threads)
    _, _, s1, rays1, dt1 = timed((0, H, row_step_1t), 1)
    sl = slice(0, H, row_step)
    a, b = gpu_rgba32f[sl], rgba[sl]
    same_bits = bool(np.all((a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))))
    timed = {label: bool(np.array_equal(img[sl], rgba8[sl])) for label, img in timed_frames}
    parity = {
        "oracle": "oracle/rt_oracle.c (CPU restatement of the HLSL; D3D path not runnable here)",
        "rows": f"0::{row_step} of {H} ({len(range(0, H, row_step)) * W} pixels per frame)",
        # the frames the timed loop itself rendered (RGBA8 framebuffers read back after the timed region)
        "timed_frames_rgba8_equal": timed,
        "timed_frames_all_equal": all(timed.values()),
        # the instrumented whole frame (float32 output enabled, same kernels' instrumented build)
        "whole_frame_rgba32f_bitexact": same_bits,
        "whole_frame_max_abs_delta_rgba32f": float(np.max(np.abs(a.astype(np.float64) - b.astype(np.float64))))
        if a.size else 0.0,
        "whole_frame_rgba8_equal": bool(np.array_equal(gpu_rgba8[sl], rgba8[sl])),
        "tolerance": "bit-exact (north_star bound: 1e-4 per channel; profiles/r03/parity_sensitivity.md bounds "
                     "the oracle's own arithmetic conventions)",
    }
    out = {"value": round(rays / dt / 1e6, 4), "unit": "Mray/s", "cores": threads, "kind": "port",
           "host_cpus": os.cpu_count(),
           "sample": f"oracle/rt_oracle.c, prepass + rows 0::{row_step} of the {W}x{H} frame "
                     f"({s['primary_rays']} primary + {s['primary_hits']} shadow + {s['ao_rays']} AO + 1024 "
                     f"prepass rays, {dt:.1f} s, {threads} OpenMP threads = this process's CPU share "
                     f"(OMP_NUM_THREADS / affinity) of the host's {os.cpu_count()})",
           "single_thread": {"value": round(rays1 / dt1 / 1e6, 4), "unit": "Mray/s", "cores": 1,
                             "sample": f"prepass + rows 0::{row_step_1t} ({rays1} rays, {dt1:.1f} s, 1 thread)"}}
    return out, parity


TRAFFIC_KERNELS = ("k_order", "k_trace", "k_finish")


def instrumented_kernel(name):
    """The STATS instantiations (k_trace<L, true, ...>, k_camerarays_group<true, ...>): not the timed path."""
    return re.match(r"k_trace<\d+, true|k_camerarays_group<true", name) is not None


def traffic_child(a):
    """--traffic-child: what the PMC passes profile: two B-frame batches, one in flight (the first
    warms up; the second is the launch measured)."""
    import gpgpuraytrace_amd as G
    from gpgpuraytrace_amd import engine as E
    euler = G.camera.INITIAL_ROTATION_EULER if a.pose == "reset" else G.camera.LOOKDOWN_ROTATION_EULER
    B = max(1, min(24, a.batch))
    ring = E.FrameRing(a.width, a.height, gated=GATED, depth=1, theme=a.landscape, camera=G.Camera(a.width, a.height, euler=euler),
                       time_of_day=0.3, max_steps=a.max_steps, ao_samples=a.ao, graph=bool(a.graph), batch=B)
    for _ in range(2):
        ring.render_batch()
    ring.synchronize()
    ring.destroy()


def measure_traffic(a, B):
    """HBM bytes of one B-frame tracescreen launch, measured now: rocprofv3 --pmc FETCH_SIZE and
    --pmc WRITE_SIZE (separate passes: the two do not fit the 4 TCC slots of one) over
    `bench.py --traffic-child` child processes (children, never an exec of this GPU process), the
    uninstrumented tracescreen kernels of the second (measured) launch, 2 * FETCH_SIZE + WRITE_SIZE
    (MI355X_MICROARCH.md HBM: gfx950 FETCH_SIZE tallies half the bytes of these loads;
    profiles/r02/hbm_counter_calibration.txt).  Returns (bytes or None, note)."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None, "rocprofv3 not found"
    work = tempfile.mkdtemp(prefix="bench_traffic_", dir="/tmp")
    child = [sys.executable, os.path.abspath(__file__), "--traffic-child", "--config", a.config, "--width", str(a.width),
             "--height", str(a.height), "--landscape", a.landscape, "--pose", a.pose, "--max-steps", str(a.max_steps),
             "--ao", str(a.ao), "--batch", str(B), "--graph", str(a.graph)]
    env = dict(os.environ, TMPDIR="/tmp")
    kib = {}
    try:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            out = os.path.join(work, counter)
            r = subprocess.run([prof, "--pmc", counter, "--output-format", "csv", "-d", out, "-o", "run", "--"] + child,
                               cwd="/tmp", env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=180)
            if r.returncode != 0:
                return None, f"rocprofv3 --pmc {counter} rc={r.returncode}: {r.stderr.decode(errors='replace')[-200:]}"
            per = {}
            for f in glob.glob(out + "/**/*counter_collection.csv", recursive=True):
                for row in csv.DictReader(open(f)):
                    name = row["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
                    key = (int(row["Dispatch_Id"]), name)
                    per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
            orders = sorted(d for d, n in per if n.startswith("k_order"))
            if len(orders) < 2:
                return None, f"rocprofv3 --pmc {counter}: {len(orders)} tracescreen launches in the trace"
            last = orders[len(orders) // 2]  # k_order of the second (measured) launch; one workgroup per frame
            kib[counter] = sum(v for (d, n), v in per.items()
                               if d >= last and n.startswith(TRAFFIC_KERNELS) and not instrumented_kernel(n))
    except (subprocess.TimeoutExpired, OSError, KeyError, ValueError) as e:
        return None, f"traffic pass failed: {type(e).__name__}: {e}"
    finally:
        shutil.rmtree(work, ignore_errors=True)
    return int((2.0 * kib["FETCH_SIZE"] + kib["WRITE_SIZE"]) * 1024), (
        f"measured in this run: rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE passes over one {B}-frame launch "
        f"({' + '.join(TRAFFIC_KERNELS)}), 2 * FETCH_SIZE + WRITE_SIZE = {2 * kib['FETCH_SIZE'] / 1024:.1f} + "
        f"{kib['WRITE_SIZE'] / 1024:.1f} MiB")


def stream_capturing(stream):
    """hipStreamIsCapturing on a torch stream (bench.py's timed-region check): True while a hipGraph
    capture is active on it."""
    import ctypes
    global _HIP
    if _HIP is None:
        _HIP = ctypes.CDLL("libamdhip64.so")
        _HIP.hipStreamIsCapturing.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
    st = ctypes.c_int(0)
    rc = _HIP.hipStreamIsCapturing(ctypes.c_void_p(stream.cuda_stream), ctypes.byref(st))
    if rc != 0:
        raise RuntimeError(f"hipStreamIsCapturing failed: {rc}")
    return st.value == 1  # hipStreamCaptureStatusActive


_HIP = None


def progress(rank, msg):
    """One progress line on stderr (the JSON line stays alone on stdout)."""
    print(f"[bench rank {rank}] {msg}", file=sys.stderr, flush=True)


def launch_ranks(a):
    """`python bench.py --gpus N` (N > 1) outside a torch.distributed launcher: run the same command
    under `torch.distributed.run` (one rank per GPU, rendezvous on 127.0.0.1) as a CHILD process,
    before this process touches the GPU, and exit with its code."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    progress(0, f"--gpus {a.gpus} without a launcher: starting {a.gpus} ranks under torch.distributed.run")
    return subprocess.call(cmd)


def main():
    a = parse()
    if a.traffic_child:
        return traffic_child(a)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(a)
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != a.gpus:
        progress(int(os.environ.get("RANK", "0")), f"note: --gpus {a.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}; "
                 "the run uses WORLD_SIZE ranks")
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
    if os.environ.get("RT_BENCH_WATCHDOG"):  # diagnostics: every rank's Python stack every N s on stderr
        import faulthandler
        faulthandler.dump_traceback_later(int(os.environ["RT_BENCH_WATCHDOG"]), repeat=True)
    # the rank's GPU first: RCCL's communicator and the barrier's device follow the current device
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group(backend)

    import gpgpuraytrace_amd as G
    from gpgpuraytrace_amd import engine as E
    from gpgpuraytrace_amd import parallel as P

    euler = G.camera.INITIAL_ROTATION_EULER if a.pose == "reset" else G.camera.LOOKDOWN_ROTATION_EULER
    W, H = a.width, a.height
    sizes = batch_sizes(a.steps, max(1, min(24, a.batch)))
    B = sizes[0]
    n_full = sum(1 for s in sizes if s == B)

    def make(stats, max_steps=a.max_steps, ao=a.ao, float_output=False):
        dev = G.DeviceFactory.construct(G.DeviceAPI.HIP, W, H, gpu=local, stats=stats, float_output=float_output,
                                        gated=GATED)
        if dev is None:
            raise RuntimeError("device create failed: " + G.lib().rt_last_error().decode())
        ter = G.Terrain(dev, a.landscape, max_steps=max_steps, ao_samples=ao)
        ter.create()
        if not ter.reload():
            raise RuntimeError("shader load failed: " + G.lib().rt_last_error().decode())
        ter.set_camera(G.Camera(W, H, euler=euler))
        ter.set_time_of_day(0.3)
        return dev, ter

    def frame_counts(max_steps, ao, keep_frame=False, batch_stats=True):
        """Instrumented frames (untimed): (1) one batch of B frames exactly as the timed loop traces
        it on this rank (rt_terrain_render_batch, rotated shards): its tracescreen noise3d and the
        wave iterations of that noise (SIMD lane utilisation); (2) one whole frame: hits, rays,
        noise per frame and (keep_frame) its pixels."""
        out = {"batch_noise": None, "noise_lane_util": None, "prepass_noise": None}
        if batch_stats:
            devs, ters = [], []
            for _ in range(B):
                d, t = make(stats=True, max_steps=max_steps, ao=ao)
                devs.append(d)
                ters.append(t)

            def total():
                st = [d.stats(reset=True) for d in devs]
                return sum(x["noise_calls"] for x in st), sum(x["noise_wave_iters"] for x in st)

            for t in ters:
                t.update_shaders()
                t.camera_compute.run(2, 2, 1)
            pc, pw = total()  # the prepass alone; render_batch runs it again
            if B > 1:
                E.render_batch(ters, rank if world > 1 else 0, world)
            else:
                ters[0].render_device(rank if world > 1 else 0, world)
            for d in devs:
                d.synchronize()
            c, w = total()
            out["batch_noise"], out["noise_lane_util"] = c - pc, (c - pc) / (64.0 * (w - pw)) if w > pw else None
            out["prepass_noise"] = pc
            for d in devs:
                d.destroy()
        sdev, ster = make(stats=True, max_steps=max_steps, ao=ao, float_output=keep_frame)
        ster.update_shaders()
        ster.camera_compute.run(2, 2, 1)
        pre = sdev.stats(reset=True)
        ster.render_device(0, 1)
        whole = sdev.stats(reset=True)
        img = (sdev.readback_float(), sdev.readback()) if keep_frame else None
        sdev.destroy()
        hits = whole["hits"]
        out.update({"frame_noise": whole["noise_calls"] - pre["noise_calls"], "hits": hits,
                    "rays": W * H + hits + hits * ao + 1024, "img": img})
        return out

    want_cpu = rank == 0 and world == 1 and not a.no_cpu_baseline
    progress(rank, f"instrumented batch of {B} + whole frame")
    counts = frame_counts(a.max_steps, a.ao, keep_frame=want_cpu)
    progress(rank, "counts done")
    rays_per_frame, hits = counts["rays"], counts["hits"]

    # --- timed: batches of B frames, D batches in flight (FrameRing slot groups) ---
    camera = G.Camera(W, H, euler=euler)
    ring = E.FrameRing(W, H, gated=GATED, depth=a.frames_in_flight, gpu=local, theme=a.landscape, camera=camera,
                       time_of_day=0.3, max_steps=a.max_steps, ao_samples=a.ao, graph=bool(a.graph), batch=B)
    plan = P.BatchPlan(W, H, B, world, split_prepass=a.split_prepass, lookahead=a.lookahead,
                       direct_pack=bool(a.direct_pack))
    coll = P.Collectives(dist, backend, rank, world)
    dev_str = f"cuda:{local}"
    # a batch's devices share its stream (FrameRing): every op of a batch rides on it
    bufs = {g: {"stream": torch.cuda.ExternalStream(ring.slots[g * B][0].stream(), device=dev_str)}
            for g in range(ring.depth)}
    if world > 1:
        pre_group = dist.new_group(backend=backend) if plan.split_prepass else None
        for g in range(ring.depth):
            bufs[g].update({
                "packed": torch.zeros(plan.packed_bytes(), dtype=torch.uint8, device=dev_str),
                "gathered": [torch.zeros(plan.packed_bytes(), dtype=torch.uint8, device=dev_str)
                             for _ in range(world)] if rank == 0 else None,
                "cams": torch.zeros(plan.camera_floats(), dtype=torch.float32, device=dev_str),
            })
        # the fills ran on torch's stream; the batches' streams are non-blocking (no implicit order):
        # every slot group's stream waits for them through the C-ABI's event handoff (ABI 6), no host
        # synchronisation
        filled = torch.cuda.Event()
        filled.record(torch.cuda.current_stream())
        for g in range(ring.depth):
            ring.slots[g * B][0].wait_event(filled.cuda_event)

    class DeviceOps:
        """run_batch's actions on this GPU: HIP kernels through the C-ABI, RCCL collectives."""

        def __init__(self, n):
            self.g = (ring.frame // B) % ring.depth
            self.group = ring.group(n)
            self.ters = [t for _, t in self.group]
            self.devs = [d for d, _ in self.group]
            self.b = bufs.get(self.g)

        def prepass(self, first, count):
            E.prepass_batch(self.ters, first, count, self.b["cams"].data_ptr())

        def all_gather_cameras(self):
            with torch.cuda.stream(self.b["stream"]):
                coll.all_gather(self.b["cams"], self.b["cams"][plan.camera_slice(rank)], pre_group)

        def trace(self):
            E.trace_batch(self.ters, rank, world, self.b["cams"].data_ptr())

        def render(self):
            E.render_batch(self.ters, rank if world > 1 else 0, world)

        def render_packed(self, items):
            # frame f's shard at base + f * max_bytes (items' offsets): the gather's send buffer, written by the
            # trace kernels themselves
            assert [off for _, _, off in items] == [plan.pack_offset(f) for f, _, _ in items]
            E.render_batch_packed(self.ters, rank, world, self.b["packed"].data_ptr(), plan.max_bytes)

        def prepass_ahead(self):
            if self.g not in ahead:
                E.prepass_ahead(self.ters)
            ahead.discard(self.g)

        def prepass_ahead_next(self):
            nxt = (self.g + 1) % ring.depth
            if nxt != self.g:
                E.prepass_ahead([t for _, t in ring.slots[nxt * B:(nxt + 1) * B]])
                ahead.add(nxt)

        def trace_ahead(self):
            E.trace_ahead(self.ters, rank if world > 1 else 0, world)

        def pack_batch(self, items):
            base = self.b["packed"].data_ptr()
            E.shard_pack_batch([self.devs[f] for f, _, _ in items], [s for _, s, _ in items], world,
                               [base + off for _, _, off in items])

        def gather(self):
            with torch.cuda.stream(self.b["stream"]):
                coll.gather(self.b["packed"], self.b["gathered"])

        def unpack_batch(self, items):
            g = self.b["gathered"]
            E.shard_unpack_batch([self.devs[f] for _, f, _, _ in items], [s for _, _, s, _ in items], world,
                                 [g[src].data_ptr() + off for src, _, _, off in items])

        def present(self):
            for d in self.devs:
                d.present()

    timed_marks, timed_t0 = [], []  # per timed batch: run_batch's phase marks (HIP events) and its stream's t0
    capturing_marks = []  # marks recorded while their stream was capturing a hipGraph (expected: none)
    ahead = set()  # slot groups whose prepass is queued ahead (plan.lookahead)

    def batch_step(n, timed=False, ahead_next=True):
        ops = DeviceOps(n)
        mark = None
        if timed:
            marks, stream = [], ops.b["stream"]

            def mark(name):
                if stream_capturing(stream):
                    capturing_marks.append((len(timed_marks) - 1, name))
                ev = torch.cuda.Event(enable_timing=True)
                ev.record(stream)
                marks.append((name, ev))
            timed_marks.append(marks)
            timed_t0.append(t0_events[ops.g])
        P.run_batch(plan, rank, ops, frames=n, mark=mark, ahead_next=ahead_next)
        ring.frame += B

    progress(rank, "warmup")
    n_warm = -(-a.warmup // B) + ring.depth
    for i in range(n_warm):
        batch_step(B, ahead_next=i + 1 < n_warm)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    progress(rank, f"timed: {len(sizes)} batches")
    # the timed region's start on every batch stream (the phase marks' time base)
    t0_events = []
    for g in range(ring.depth):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(bufs[g]["stream"])
        t0_events.append(ev)
    captures_before = sum(d.graph_info()[0] for d, _ in ring.slots)
    t0 = time.perf_counter()
    for i, n in enumerate(sizes):
        batch_step(n, timed=True, ahead_next=i + 1 < len(sizes))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    graph_captures_timed = sum(d.graph_info()[0] for d, _ in ring.slots) - captures_before
    for d, _ in ring.slots:  # a dropped k_trace queue push (never expected) fails the run
        d.check()

    # this rank's phases of the timed batches (HIP events on each batch's stream, from the common
    # start barrier), read NOW: the events were recorded on the ring's streams, and HIP's event
    # queries look at the stream an event was recorded on -- read after ring.destroy() (as in round 3)
    # they touched destroyed streams, the likely source of the hipErrorCapturedEvent seen at C1 / C5
    # (no capture runs in the timed region: graph_captures_in_timed_region, marks_on_capturing_stream)
    names = {id(ev): f"batch {b} mark '{nm}'" for b, mk in enumerate(timed_marks) for nm, ev in mk}
    names.update({id(ev): f"t0 of slot group {g}" for g, ev in enumerate(t0_events)})

    def event_ms(x, y):
        """HIP event pair -> ms; a refused pair fails the run, naming the pair"""
        try:
            return x.elapsed_time(y)
        except Exception as e:  # noqa: BLE001
            raise RuntimeError(f"phase marks: HIP refused elapsed_time({names.get(id(x))} -> {names.get(id(y))}): "
                               f"{e}; graph captures in the timed region: {graph_captures_timed}, marks recorded "
                               f"on a capturing stream: {capturing_marks}") from e

    phases = P.phase_summary(timed_marks, event_ms, t0=timed_t0)
    capture_check = {"graph_captures_in_timed_region": graph_captures_timed,
                     "marks_on_capturing_stream": len(capturing_marks)}

    progress(rank, f"timed done ({elapsed * 1e3:.1f} ms)")
    # the timed loop's own output: the first and last frame of its last batch (rank 0 holds every
    # frame whole: at N>1 assembled from all ranks' shards), read back now, before any other pass
    # reuses the slots; N=1 compares them with the oracle (config.parity), N>1 with a whole-frame
    # render on one device (config.verify)
    g_last = ((ring.frame // B) - 1) % ring.depth
    last = ring.slots[g_last * B:g_last * B + sizes[-1]]
    timed_frames = []
    if rank == 0:
        for f in sorted({0, len(last) - 1}):
            timed_frames.append((f"batch {len(sizes) - 1} frame {f}", last[f][0].readback()))
    verify = None
    if (a.verify or world > 1) and rank == 0:
        # the last timed batch's frames, assembled from every rank's shards, against one whole frame
        vdev, vter = make(stats=False)
        vter.render_device(0, 1)
        want = vdev.readback()
        vdev.destroy()
        verify = []
        for f, (d, _) in enumerate(last):
            bad = np.any(d.readback() != want, axis=-1)
            if bad.any():  # which tiles (and so which shards) came out wrong
                ty, tx = np.nonzero(bad)
                tiles = sorted({int(t) for t in (ty // 32) * ((W + 31) // 32) + tx // 32})
                verify.append({"frame": f, "pixels": int(bad.sum()), "tiles": len(tiles),
                               "shards": sorted({t % world for t in tiles}), "first_tiles": tiles[:8]})

    # --- roofline pass: full batches one at a time on slot group 0 (launches do not overlap),
    # HIP events around every tracescreen launch on the stream it runs on; also the latency ---
    group0 = ring.slots[:B]
    progress(rank, "roofline pass")
    ring.set_profiling(True)
    ring.kernel_time()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for i in range(n_full):
        E.render_batch([t for _, t in group0], rank if world > 1 else 0, world)
        for d, _ in group0:
            d.present()
        progress(rank, f"roofline batch {i + 1}/{n_full} queued")
    for d, _ in group0:
        d.synchronize()
    progress(rank, "roofline pass done")
    latency_ms = (time.perf_counter() - t1) / n_full * 1e3
    kms, kn = ring.kernel_time()
    ring.set_profiling(False)
    k_avg_ms = kms / max(1, kn)  # one launch = a batch of B frames

    # --- companions (N=1): frames rendered one per launch sequence (B = 1) ---
    companions = {}
    if world == 1 and not a.no_companions:
        d0, ter0 = group0[0]
        torch.cuda.synchronize()
        ts = time.perf_counter()
        for _ in range(a.steps):
            ter0.render_device()
            d0.present()
        d0.synchronize()
        dt_serial = time.perf_counter() - ts
        # the same loop on an RT_DEVICE_DEFERRED device (ABI 9): each render launches the previous frame's
        # trace with its own frame's prepass inside it
        # (and with 2 frames to a deferred launch, rt_device_defer_batch)
        dt_deferred, deferred_fused = {}, {}
        for kdef in (1, 2):
            ddev = E.DeviceFactory.construct(E.DeviceAPI.HIP, W, H, gpu=local, deferred=True)
            ddev.defer_batch(kdef)
            dter = E.Terrain(ddev, a.landscape, max_steps=a.max_steps, ao_samples=a.ao)
            dter.create()
            assert dter.reload(), G.lib().rt_last_error()
            dter.set_camera(camera)
            dter.set_time_of_day(0.3)
            for _ in range(4):
                dter.render_device()
                ddev.present()
            ddev.synchronize()
            f0 = ddev.deferred_fused()
            ts = time.perf_counter()
            for _ in range(a.steps):
                dter.render_device()
                ddev.present()
            ddev.synchronize()
            dt_deferred[kdef] = time.perf_counter() - ts
            deferred_fused[kdef] = ddev.deferred_fused() - f0
            ddev.destroy()
    ring.destroy()
    if world == 1 and not a.no_companions:
        # B = 1 with three frames in flight (D3D11's default maximum frame latency, the reference
        # frame loop's own queue depth): each frame is its own prepass -> k_order -> k_trace ->
        # k_finish on its slot's stream, and the next frame's prepass overlaps this one's tail
        sring = E.FrameRing(W, H, gated=GATED, depth=3, gpu=local, theme=a.landscape, camera=camera, time_of_day=0.3,
                            max_steps=a.max_steps, ao_samples=a.ao, batch=1, lookahead=True)
        for i in range(sring.depth + 1):
            sring.render_batch(ahead=i < sring.depth)
        sring.synchronize()
        ts = time.perf_counter()
        for i in range(a.steps):
            sring.render_batch(ahead=i + 1 < a.steps)
        sring.synchronize()
        dt = time.perf_counter() - ts
        sring.destroy()
        ps = W * H + hits + 1024  # primary + shadow (+ prepass), as config.primary_plus_shadow_mrays
        companions["single_frame"] = {
            "value": round(rays_per_frame * a.steps / dt / 1e6, 3), "unit": "Mray/s",
            "ms_per_frame": round(dt / a.steps * 1e3, 4),
            "primary_plus_shadow_mrays": round(ps * a.steps / dt / 1e6, 3),
            "how": f"B=1 (one frame per launch sequence), 3 frames in flight on 3 streams, each frame's "
                   f"prepass queued one frame ahead on the side stream (rt_terrain_prepass_ahead), {a.steps} frames"}
        companions["single_frame_serial"] = {
            "value": round(rays_per_frame * a.steps / dt_serial / 1e6, 3), "unit": "Mray/s",
            "ms_per_frame": round(dt_serial / a.steps * 1e3, 4),
            "primary_plus_shadow_mrays": round(ps * a.steps / dt_serial / 1e6, 3),
            "how": f"rt_terrain_render + rt_device_present, one frame per call on one device and its stream (B=1; "
                   f"each frame's prepass on the device's prepass stream behind the previous frame's k_order, "
                   f"overlapping that frame's trace tail), {a.steps} frames"}
        for kdef, key in ((1, "single_frame_deferred"), (2, "single_frame_deferred2")):
            companions[key] = {
                "value": round(rays_per_frame * a.steps / dt_deferred[kdef] / 1e6, 3), "unit": "Mray/s",
                "ms_per_frame": round(dt_deferred[kdef] / a.steps * 1e3, 4),
                "primary_plus_shadow_mrays": round(ps * a.steps / dt_deferred[kdef] / 1e6, 3),
                "fused_prepasses": deferred_fused[kdef],
                "how": (f"the same loop on an RT_DEVICE_DEFERRED device (ABI 9): each rt_terrain_render launches the "
                        f"previous frame's setTargetDepths + trace with its own frame's prepass inside that trace "
                        f"kernel, the last frame by rt_device_synchronize (a frame under 1280x720 pixels renders as "
                        f"without the flag: fused_prepasses 0), {a.steps} frames") if kdef == 1 else
                       (f"the same loop on an RT_DEVICE_DEFERRED device tracing 2 frames to a launch "
                        f"(rt_device_defer_batch(2)): every second rt_terrain_render launches the two oldest queued "
                        f"frames' setTargetDepths + trace with the next two frames' prepasses inside it; every frame "
                        f"in full, the intermediate ones into frame slots (a DISCARD swap chain), {a.steps} frames")}

    if world == 1 and not a.no_companions and a.config == "c3" and (a.max_steps, a.ao) == (512, 1):
        rc = frame_counts(0, 0, batch_stats=False)
        rring = E.FrameRing(W, H, gated=GATED, depth=a.frames_in_flight, gpu=local, theme=a.landscape, camera=camera,
                            time_of_day=0.3, max_steps=0, ao_samples=0, batch=B, lookahead=bool(a.lookahead))
        for i in range(rring.depth + 1):
            rring.render_batch(ahead=i < rring.depth)
        rring.synchronize()
        ts = time.perf_counter()
        for i, n in enumerate(sizes):
            rring.render_batch(frames=n, ahead=i + 1 < len(sizes))
        rring.synchronize()
        dt = time.perf_counter() - ts
        rring.destroy()
        companions["ref_semantics"] = {
            "value": round(rc["rays"] * a.steps / dt / 1e6, 3), "unit": "Mray/s",
            "ms_per_frame": round(dt / a.steps * 1e3, 4), "rays_per_frame": rc["rays"],
            "how": "--config ref: the same frames and batching, uncapped march (tracing.hlsl:68), no AO"}

    if world == 1 and not a.no_companions:
        # a moving camera: every frame of the run distinct (the eye advances 2 units per frame along
        # the view direction and the yaw turns 0.01 rad per frame), batched exactly like the timed
        # loop; rays counted per frame by an instrumented render of each camera, and the run's last
        # frame compared with that render (RGBA8, bit for bit)
        base = G.Camera(W, H, euler=euler)
        path = [G.Camera(W, H, position=base.position + i * 2.0 * np.asarray(base.front, float),
                         euler=(euler[0], euler[1] + 0.01 * i, euler[2])) for i in range(a.steps)]
        cdev, cter = make(stats=True)
        path_rays, want_last = 0, None
        for i, cam in enumerate(path):
            cter.set_camera(cam)
            cter.update_terrain()
            cter.render_device(0, 1)
            path_rays += W * H + cdev.stats(reset=True)["hits"] * (1 + a.ao) + 1024
            if i + 1 == len(path):
                want_last = cdev.readback()
        cdev.destroy()
        mring = E.FrameRing(W, H, gated=GATED, depth=a.frames_in_flight, gpu=local, theme=a.landscape, camera=camera,
                            time_of_day=0.3, max_steps=a.max_steps, ao_samples=a.ao, batch=B)

        def path_batch(first, n):
            for (_, ter), cam in zip(mring.group(n), path[first:first + n]):
                ter.set_camera(cam)
                ter.update_terrain()
            return mring.render_batch(frames=n)
        for i in range(mring.depth + 1):  # warm-up over the path's first batches
            path_batch((i * B) % max(1, a.steps - B + 1), min(B, a.steps))
        mring.synchronize()
        ts, first = time.perf_counter(), 0
        for n in sizes:
            devs = path_batch(first, n)
            first += n
        mring.synchronize()
        dt = time.perf_counter() - ts
        last_ok = bool(np.array_equal(devs[-1].readback(), want_last))
        mring.destroy()
        companions["moving_camera"] = {
            "value": round(path_rays / dt / 1e6, 3), "unit": "Mray/s", "ms_per_frame": round(dt / a.steps * 1e3, 4),
            "rays_per_frame_mean": round(path_rays / a.steps), "last_frame_rgba8_equal": last_ok,
            "how": f"{a.steps} distinct frames (eye +2 units and yaw +0.01 rad per frame), the timed loop's "
                   f"batches {sizes}, cameras written into each slot group before its batch; the last frame "
                   f"against an instrumented single-frame render of its camera"}

    if world == 1 and not a.no_companions and a.sustained_s > 0:
        # sustained rate: the timed loop's batches back to back for ~--sustained-s seconds (clocks and
        # power under a long load), a HIP event after every batch on its stream, read once at the end
        n_sus = max(2, int(a.sustained_s * 1e3 / (elapsed / a.steps * 1e3 * B) + 0.5))
        uring = E.FrameRing(W, H, gated=GATED, depth=a.frames_in_flight, gpu=local, theme=a.landscape, camera=camera,
                            time_of_day=0.3, max_steps=a.max_steps, ao_samples=a.ao, batch=B)
        for _ in range(uring.depth + 1):
            uring.render_batch()
        uring.synchronize()
        ev0 = torch.cuda.Event(enable_timing=True)
        ev0.record(torch.cuda.ExternalStream(uring.slots[0][0].stream(), device=f"cuda:{local}"))
        ends = []
        for _ in range(n_sus):
            g = (uring.frame // B) % uring.depth
            uring.render_batch()
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(torch.cuda.ExternalStream(uring.slots[g * B][0].stream(), device=f"cuda:{local}"))
            ends.append(ev)
        uring.synchronize()
        t_end = [ev0.elapsed_time(ev) for ev in ends]  # ms from the start, per batch
        uring.destroy()
        total = max(t_end)
        # rates over windows of ~1 s (batch ends in order of completion; with two batches in flight
        # the ends come in pairs, so a window is counted to +-1 batch, ~3% of a 1 s window)
        t_sorted, wins, last_t, last_n = sorted(t_end), [], 0.0, 0
        for i, t in enumerate(t_sorted):
            if t - last_t >= 1000.0 or (i + 1 == len(t_sorted) and t - last_t >= 750.0):
                wins.append(rays_per_frame * B * (i + 1 - last_n) / ((t - last_t) * 1e-3) / 1e6)
                last_t, last_n = t, i + 1
        companions["sustained"] = {
            "value": round(rays_per_frame * B * n_sus / (total * 1e-3) / 1e6, 3), "unit": "Mray/s",
            "seconds": round(total * 1e-3, 3), "frames": n_sus * B,
            "window_mrays": [round(w, 1) for w in wins],
            "how": f"the timed loop's {B}-frame batches back to back for ~{a.sustained_s:g} s "
                   f"({a.frames_in_flight} in flight), HIP event per batch; windows of ~1 s"}

    # this rank's tracescreen launch time with its phases; rank 0 reports every rank's (config.per_rank)
    phases.update({"rank": rank, "tracescreen_kernel_ms": round(k_avg_ms, 4)})
    per_rank = [phases]
    if world > 1:
        t = torch.tensor([elapsed, latency_ms], dtype=torch.float64, device=dev_str if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, latency_ms = float(t[0].item()), float(t[1].item())
        per_rank = [None] * world
        dist.all_gather_object(per_rank, phases)

    ms_per_frame = elapsed / a.steps * 1e3
    value = rays_per_frame * a.steps / elapsed / 1e6
    # the timed launch's noise3d: tracescreen's, plus (RT_BENCH_GATED=1: the gated launch, nomadplains) the
    # batch's prepass rays, which then run inside the same trace kernel
    gated = GATED and a.landscape == "nomadplains"
    batch_noise = counts["batch_noise"] + (counts["prepass_noise"] if gated else 0)
    achieved = batch_noise * FLOPS_PER_NOISE3D / (k_avg_ms * 1e-3) / 1e12
    traffic, traffic_how = None, "not measured (N>1: a rank's launch traces a shard; or --traffic off)"
    if world == 1 and a.traffic == "pmc":
        progress(rank, "traffic: rocprofv3 FETCH_SIZE / WRITE_SIZE passes")
        traffic, traffic_how = measure_traffic(a, B)
        progress(rank, f"traffic: {traffic}")

    if rank == 0:
        preset = CONFIGS[a.config]
        named = (W, H, a.max_steps, a.ao) == tuple(preset[k] for k in ("width", "height", "max_steps", "ao"))
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "Mray/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms_per_frame, 4), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic: procedural nomadplains terrain, noise seed 300 (MSVC rand), fixed camera",
            "config": {
                "workload": f"{preset['name'] if named else 'custom'}; "
                            f"{W}x{H} {a.landscape} frame ({a.pose} pose), camerarays prepass + device "
                            f"setTargetDepths + tracescreen (primary + normal + colour + shadow + sky"
                            f"{f' + {a.ao} AO ray(s) per hit' if a.ao else ''}), "
                            f"{'uncapped march (reference semantics)' if a.max_steps == 0 else f'{a.max_steps}-step primary cap'}",
                "width": W, "height": H, "landscape": a.landscape, "pose": a.pose, "aa_samples": 1,
                "max_steps": a.max_steps, "ao_samples": a.ao, "rays_per_frame": rays_per_frame, "primary_rays": W * H,
                "shadow_rays": hits, "ao_rays": hits * a.ao, "prepass_rays": 1024,
                "primary_plus_shadow_mrays": round((W * H + hits + 1024) * a.steps / elapsed / 1e6, 3),
                "hit_fraction": round(hits / (W * H), 4),
                "noise3d_per_frame_tracescreen": counts["frame_noise"],
                # the timed batch's noise3d lane-calls / (64 x their wave iterations): SIMD lane
                # utilisation of the noise work, counted by the instrumented kernels
                "noise_lane_utilisation": round(counts["noise_lane_util"], 4) if counts["noise_lane_util"] else None,
                "noise_lane_utilisation_scope": "instrumented (STATS) kernels, which take the product's code paths "
                                                "(the primary segment tail included: RT_STATS_PRIMARY_SEG)",
                "parallelism": "single GPU" if world == 1 else (
                    f"tile-cyclic 32x32 shards x{world} (rotated per frame) + RCCL gather per batch"
                    + (" (shards rendered straight into the packed send buffer)" if plan.direct_pack else "")
                    + (" + prepass split over ranks (RCCL all-gather of CameraResults)" if plan.split_prepass
                       else "")),
                "batch": B, "batches": sizes, "batches_in_flight": a.frames_in_flight,
                "hip_hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
                "frame_loop": "hipGraph replay per slot (prepass graph + tracescreen graph)" if a.graph
                              else "direct launches" + (", each batch's prepass queued one batch ahead on the GPU's "
                                                        "side stream (rt_terrain_prepass_ahead)" if plan.lookahead else ""),
                "frame_latency_ms": round(latency_ms, 4),  # one batch of B frames at a time
                # per rank: mean / max ms per timed batch of each run_batch phase on the batch's stream
                # (prepass, all_gather, trace, pack, gather, unpack; waits for the other batch in flight
                # included), each batch's trace start from the common start barrier, and the rank's
                # tracescreen launch (roofline pass); trace_start_skew_ms = per batch max - min over ranks
                "per_rank": per_rank,
                "timed_capture_check": capture_check,
                **({"trace_start_skew_ms": P.start_skew(per_rank)} if world > 1 else {}),
                **companions,
                **({"verify": f"all {sizes[-1]} frames of the last timed batch equal a whole-frame render on one "
                              f"device" if not verify else {"MISMATCH": verify}}
                   if verify is not None else {}),
            },
            "roofline": {
                "bound": "valu", "achieved": round(achieved, 3), "peak": PEAK_FP32_VECTOR_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / PEAK_FP32_VECTOR_TFLOPS, 4), "traffic": traffic,
                "traffic_how": traffic_how,
                **({"traffic_per_frame_vs_rgba8": round(traffic / B / (W * H * 4), 2)} if traffic else {}),
                "kernel": TRACESCREEN_KERNELS + (" (the gated launch: the prepass runs inside k_trace)" if gated else ""), "kernel_avg_ms": round(k_avg_ms, 4), "kernel_launches": kn,
                "timing": "HIP events per launch on its stream, one batch in flight (the last "
                          f"{kn} tracescreen launches of the run; one launch = {B} frames)",
                "work_unit": f"{FLOPS_PER_NOISE3D} FP32 flop per noise3d x {batch_noise} noise3d per launch ({B} "
                             f"frame(s); frame f traces shard (rank + f) % world"
                             + (f"; incl. their {counts['prepass_noise']} prepass noise3d: the gated launch runs the "
                                "prepass inside the trace kernel)" if gated else ")"),
                "note": "FP32 vector-ALU bound (no MFMA-shaped or HBM-bound work); gfx950 vector FP32 peak "
                        "= FP32 dense matrix peak = 157.3 TFLOP/s",
            },
        }
        if want_cpu:
            consts = G.frame_constants(W, H, euler=euler)
            threads = a.cpu_threads or host_threads()
            img32, img8 = counts["img"]
            out["cpu_baseline"], out["config"]["parity"] = cpu_baseline(
                consts, a.landscape, a.max_steps, a.ao, a.cpu_row_step, preset["cpu_rows_1t"], threads, img32, img8,
                timed_frames)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
