"""k_trace per-wave timeline (debug build: make -C gpgpuraytrace_amd/csrc trace).

Renders rank r of an N-way shard (default the whole frame) with the trace library and
reports, from the last k_trace launch: the spread of wave end times, what the
last-finishing waves spent their time on, and the per-SIMD load.
Usage: RT_LIB_VARIANT=trace python scripts/wave_trace.py [--n 8 --rank 0]
"""
import argparse
import ctypes as C
import os
import sys

os.environ.setdefault("RT_LIB_VARIANT", "trace")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import with_variant  # noqa: E402

with_variant.apply()

F = 28


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--max-steps", type=int, default=512)
    ap.add_argument("--ao", type=int, default=1)
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--batch", type=int, default=1, help="frames per launch (rt_terrain_render_batch)")
    a = ap.parse_args()
    import numpy as np
    import gpgpuraytrace_amd as G
    W, H = 1920, 1080
    devs, ters = [], []
    for _ in range(a.batch):
        d = G.DeviceFactory.construct(G.DeviceAPI.HIP, W, H, gpu=0)
        t = G.Terrain(d, "nomadplains", max_steps=a.max_steps, ao_samples=a.ao)
        t.create()
        assert t.reload()
        t.set_camera(G.Camera(W, H))
        t.set_time_of_day(0.3)
        devs.append(d)
        ters.append(t)
    dev = devs[0]
    for _ in range(3):
        if a.batch > 1:
            G.engine.render_batch(ters, a.rank, a.n)
        else:
            ters[0].render_device(a.rank, a.n)
    for d in devs:
        d.synchronize()
    L = G.lib()
    L.rt_debug_wave_trace.argtypes = [C.c_void_p, C.c_int]
    nw = 256 * 16
    buf = np.zeros(nw * F, np.uint64)
    assert L.rt_debug_wave_trace(buf.ctypes.data, nw) == F
    t = buf.reshape(nw, F).astype(np.int64)
    slot = np.nonzero(t[:, 0] > 0)[0]
    t = t[t[:, 0] > 0]
    t0 = t[:, 0].min()
    us = lambda x: x * 0.01  # 100 MHz realtime clock -> us
    beg, end = us(t[:, 0] - t0), us(t[:, 1] - t0)
    print(f"waves {len(t)}  span {end.max():.1f} us  begin spread {beg.max():.1f} us")
    for q in (50, 90, 99, 100):
        print(f"  end p{q}: {np.percentile(end, q):.1f} us")
    tot = lambda c: us(t[:, c])
    print(f"mean per wave: unit {tot(2).mean():.1f} us ({t[:, 5].mean():.2f} units), shade {tot(3).mean():.1f} us "
          f"({t[:, 6].mean():.2f}), long {tot(4).mean():.1f} us ({t[:, 7].mean():.2f}), idle {tot(9).mean():.1f} us")
    order = np.argsort(-end)[:a.top]
    print("last waves: end  units(us,n)  shade(us,n)  long(us,n)  last-unit-end  idle  hw_id  xcc  iters  long-rays  "
          "max-long-iters  max-primary-iters")
    for i in order:
        r = t[i]
        print(f"  {end[i]:8.1f}  {us(r[2]):8.1f},{r[5]:3d}  {us(r[3]):8.1f},{r[6]:3d}  {us(r[4]):8.1f},{r[7]:3d}  "
              f"{us(r[8] - t0) if r[8] else 0:8.1f}  {us(r[9]):7.1f}  {r[10]:#010x}  {r[11]}  {r[12]}  {r[13]}  "
              f"{r[14]}  {r[16]}")
    # the gated launch's prepass tasks (fields 21, 22: task time, last task end)
    tw = t[:, 21] > 0
    if tw.any():
        print(f"prepass tasks: {tw.sum()} waves, task time mean {tot(21)[tw].mean():.1f} max {tot(21)[tw].max():.1f} us; "
              f"last task end p50 {np.percentile(us(t[tw, 22] - t0), 50):.1f} max {us(t[tw, 22] - t0).max():.1f} us")
    # long-ray march latency: segment jobs (fields 23-25: time, jobs, loop steps = the job's longest ray) and
    # lane-refill long-ray batches (26, 27: loop steps, time), per loop step
    sj, ss, lst, lt = t[:, 24].sum(), t[:, 25].sum(), t[:, 26].sum(), t[:, 27].sum()
    if sj:
        print(f"segment jobs: {sj}, {us(t[:, 23].sum()) / sj:.1f} us per job, {ss / sj:.1f} steps per job, "
              f"{us(t[:, 23].sum()) / max(ss, 1):.3f} us per step")
    if lst:
        print(f"lane-refill long-ray loops: {lst} steps, {us(lt) / lst:.3f} us per step")
    # per SIMD busy (unit+shade+long) from hw_id: simd [5:4], cu [11:8], sh [12], se [15:13], + xcc
    hw = t[:, 10]
    simd = (hw >> 4) & 3
    key = (t[:, 11] << 16) | (((hw >> 8) & 0xFF) << 2) | simd
    busy = tot(2) + tot(3) + tot(4)
    sums = {}
    for k_, b in zip(key, busy):
        sums[k_] = sums.get(k_, 0.0) + b
    v = np.array(list(sums.values()))
    print(f"per-SIMD busy (sum over its waves): mean {v.mean():.1f} us  max {v.max():.1f} us  p99 {np.percentile(v, 99):.1f}")
    # when each SIMD's last wave left, and each SIMD's live-wave count over time: the launch's tail
    last = {}
    for k_, e in zip(key, end):
        last[k_] = max(last.get(k_, 0.0), e)
    le = np.array(sorted(last.values()))
    span = end.max()
    print(f"SIMD idle-after-last-wave: p10 {np.percentile(le, 10):.1f}  p50 {np.percentile(le, 50):.1f}  "
          f"p90 {np.percentile(le, 90):.1f}  max {span:.1f} us; SIMD-time after its last wave = "
          f"{(span - le).sum() / (len(le) * span):.2%} of the launch")
    print(f"wave-slot time after the wave left = {(span - end).sum() / (len(end) * span):.2%} of the launch")
    # longest single activity
    print(f"longest single unit (wave total/units, max): {(tot(2) / np.maximum(t[:, 5], 1)).max():.1f} us")
    # per block: when the unit queue ran dry for it (first wave to see it), its backlog then
    # (long rays, hits), and when its last wave left
    blk = slot // 16
    rows = []
    for b in np.unique(blk):
        m = blk == b
        dr = t[m, 18]
        seen = dr > 0
        if not seen.any():
            continue
        i0 = np.argmin(np.where(seen, dr, np.iinfo(np.int64).max))
        rows.append((us(dr[i0] - t0), t[m, 19][i0], t[m, 20][i0], end[m].max()))
    if rows:
        r = np.array(rows, float)
        print(f"blocks: drain seen p50 {np.percentile(r[:, 0], 50):.1f} us (p10 {np.percentile(r[:, 0], 10):.1f}, "
              f"p90 {np.percentile(r[:, 0], 90):.1f}); block end p50 {np.percentile(r[:, 3], 50):.1f}, max "
              f"{r[:, 3].max():.1f} us")
        print(f"  backlog at drain: long rays p50 {np.percentile(r[:, 1], 50):.0f} p90 {np.percentile(r[:, 1], 90):.0f} "
              f"max {r[:, 1].max():.0f}; hits p50 {np.percentile(r[:, 2], 50):.0f} max {r[:, 2].max():.0f}")
        late = np.argsort(-r[:, 3])[:8]
        print("  last blocks: end  drain-seen  long-backlog  hit-backlog")
        for i in late:
            print(f"    {r[i, 3]:8.1f}  {r[i, 0]:8.1f}  {r[i, 1]:6.0f}  {r[i, 2]:6.0f}")
        c = np.corrcoef(r[:, 1] + r[:, 2], r[:, 3] - r[:, 0])[0, 1] if len(r) > 2 else 0.0
        print(f"  corr(backlog, end - drain) = {c:.2f}")
    for d in devs:
        d.destroy()


if __name__ == "__main__":
    main()
