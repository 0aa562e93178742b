// rt_kernels.h -- host-side launch interface of the HIP kernels.
#pragma once

#include <hip/hip_runtime.h>

#include "rt_types.h"

// work counters (one 128-byte block, zeroed by k_order before every k_trace: the unit queue, then one
// first-unit counter per wave slot of a k_trace block), then the device's sticky flags (zeroed at
// device creation and by rt_device_check only): a k_trace queue push that would exceed its bound
// raises a flag instead of storing (rt_spill_caps)
// RT_CTR_GATE / RT_CTR_SCAN: the gated launch's prepass task counter and its tile scan's start (GatedPrepass)
enum { RT_CTR_PRIMARY = 0, RT_CTR_FIRST = 1, RT_CTR_GATE = 24, RT_CTR_SCAN = 25 };
#define RT_CTR_BYTES 128
#define RT_QUEUE_BYTES 192
enum { RT_FLAG_HIT_OVERFLOW = 1u, RT_FLAG_SPILL_OVERFLOW = 2u, RT_FLAG_PREPASS_TIMEOUT = 4u };

// A frame batch: up to RT_MAX_BATCH frames of one resolution, landscape and shard traced by
// one sequence of launches (rt_terrain_render_batch).  Each frame keeps its own constant
// block (camera, sun), CameraResults, CellDistance and framebuffer; the kernels find them
// through this table in device memory.  A single frame is a batch of one.
#define RT_MAX_BATCH 24
struct FrameTable {
    const RtConsts* k[RT_MAX_BATCH];    // tracescreen's constant block
    const RtConsts* kcam[RT_MAX_BATCH]; // camerarays' constant block (its own cbuffers)
    float4* cam[RT_MAX_BATCH];   // CameraResults, float4[1024]
    float2* cells[RT_MAX_BATCH]; // CellDistance, float2[1024]
    uint32_t* out8[RT_MAX_BATCH];
    float4* out32[RT_MAX_BATCH]; // may be null
};

// The NEXT batch's camerarays prepass fused into this batch's k_trace (nomadplains):
// `tasks` tasks of 8 rays (RT_PREPASS_LPR lanes per ray) of the frames of `ft` (their camerarays constant
// blocks kcam, their CameraResults cam), taken from ctl[0]; a finished wave stores its rays' CameraResults
// (sc1; one whole 128-B line per 8-ray wave) and adds its rays to ctl[1]; that batch's k_order waits for ctl[1] to reach
// its rays (frames x 1024) before it reads them.  tasks == 0: none.
#define RT_FUSE_RAYS_PER_TASK 8
#define RT_FUSE_TASKS_PER_FRAME (RT_CAMERA_RES * RT_CAMERA_RES / RT_FUSE_RAYS_PER_TASK)
struct FusedPrepass {
    const FrameTable* ft;
    uint32_t* ctl;
    uint32_t tasks;
};

// The batch's OWN camerarays prepass inside its k_trace (the gated launch, nomadplains; DESIGN.md
// section 7): `tasks` = frames x RT_FUSE_TASKS_PER_FRAME tasks of 8 rays, taken first by the waves
// (top priority), each storing its 8 CameraResults as one whole 128-B line (sc1) and then, per frame
// (RT_GATE_WORDS words at gate + f * RT_GATE_WORDS, zeroed by k_order), setting its bit in the frame's
// task mask (words 0-3; task = ray row * 4 + ray column / 8) and adding 8 to the frame's ray counter
// (word RT_GATE_CTR; the task that completes the frame derives the frame's CellDistance and flags it in
// word RT_GATE_CTR + 1).  Units are claimed by tile (claims[i]: units of order entry i taken) in k_order's
// longest-first order from the tiles whose cells' prepass rays (the 5x5 neighbourhoods setTargetDepths
// reads) are in, so units start while the prepass's long rays still march.  tasks == 0: off (the prepass
// ran before; cells from k_order).
#define RT_GATE_WORDS 256 // per frame: the task mask (words 0-3), the ray counter and the cells flag on a line of
#define RT_GATE_CTR 32    // their own, the per-task wave counters (words 128-255)
#define RT_GATE_TASKS 128
// lanes per prepass ray in k_trace's prepass tasks (a task's 8 rays are marched by 8 / (64 / LPR) waves):
// 8 = one wave per task, 3 rounds of the 18 octave values per step.  32 (one round, 4 waves per task) was
// measured slower inside k_trace: the rays' latency there is set by the units sharing their SIMDs
// (profiles/r05/gated_ab.md)
#ifndef RT_PREPASS_LPR
#define RT_PREPASS_LPR 8
#endif
struct GatedPrepass {
    uint32_t* gate;   // RT_MAX_BATCH x RT_GATE_WORDS
    uint32_t* claims; // per order entry (tile of the batch): its units claimed so far
    uint32_t tasks;
    // RT_DEVICE_DEBUG_GATE_STRESS (diagnostic): 1 = every wave first reads its frames' previous CellDistance with
    // plain loads (the CU's L1 then holds lines the frame's last task rewrites), 2 = that task waits ~200 us
    // before it stores CellDistance (more units start from CameraResults, the rest read the flagged cells late)
    uint32_t debug;
};

struct RtLaunch {
    hipStream_t stream;
    int landscape;
    const RtConsts* consts;   // device copy of the constant block
    const uint32_t* perm2d;   // device texPerm2D (128*128 texels)
    const float4* grad;       // device CBNoise.permGradients (128 float4)
    RtStats* stats;           // nullptr = uninstrumented kernels
    uint32_t* queue;          // RT_CTR_BYTES of device work counters
    int num_cus;              // compute units (persistent grid size)
    // per-sample buffers, rt_split_samples() entries per frame (sample t, see rt_kernels.hip)
    float4* samples;          // saturated colour of hit samples (written by S, read by R)
    // k_trace's per-block queues in HBM, consumed by the same block; capacities per block
    // (rt_spill_caps: the bound on a block's queued work)
    float4* hitq;             // hit queue: primary hit records (1 float4, 3 with fog), hit_cap per block
    float4* spill_long;       // long-ray records (3 float4) the LDS ring cannot hold, long_spill_cap per block
    uint32_t hit_cap, long_spill_cap;
    int cells_from_cam;       // k_order derives CellDistance from CameraResults (setTargetDepths) first
    int small_rings;          // diagnostic (RT_DEVICE_DEBUG_SMALL_RINGS): k_trace's LDS long ring holds 64 entries, its fin pool 8
    int fit;                  // hit pixels finish in k_trace (aa 1, <= 1 AO ray, no float output; UnitMap::fit)
    float4* fin;              // 3 float4 per sample: shading inputs a long shadow ray needs to finish
    float4* finpool;          // the same per block in a pool of RT_FIN_SLOTS slots of 3 float4 (fin is the fallback)
    float4* cpool;            // per block RT_AO_POOL_SLOTS colours: a multi-AO hit's colour for its last AO ray (fitm)
    int fitm;                 // hit pixels without a long shadow finish in k_trace with >= 2 AO rays (UnitMap::fitm)
    uint32_t* aocc;           // per sample: occluded AO rays (AO extension), a byte each, 4 per word
    int ao_samples;           // AO rays per primary hit (0 = off)
    int aa;                   // AA samples per pixel
    uint32_t* order;          // k_order's tile order (rt_split_samples/1024 entries per frame)
    uint64_t* hitmask;        // per 8x8 unit and AA sample: the primary hits' ballot (k_trace -> k_finish)
    const FrameTable* frames; // device table of the batch's frames
    FrameTable frames_host;   // the same pointers on the host
    uint32_t n_frames;        // frames in the batch (1..RT_MAX_BATCH)
    hipEvent_t after_order;   // recorded after k_order when set (its read of CameraResults is done)
    FusedPrepass fuse_next;   // the next batch's prepass, run inside this k_trace (tasks 0: none); k_order zeroes its ctl
    const uint32_t* wait_ctl; // this batch's prepass ran inside the previous k_trace: k_order waits for wait_ctl[1]
    uint32_t wait_total;      //   to reach this many rays
    hipEvent_t after_order_fuse; // recorded after k_order when set: fuse_next's counters are zeroed (its batch's
                                 // own k_order, on another stream, polls them only after this event)
    uint32_t* host_flag;      // host-mapped word of the GPU: k_order stores RT_FLAG_PREPASS_TIMEOUT there when its
                              // wait for a fused prepass times out (every later C-ABI call on the GPU fails)
    GatedPrepass gated;       // this batch's prepass inside its own k_trace (tasks 0: off)
    int packed;               // frames.out8[f] are packed shard buffers (UnitMap::packed; no float output)
};

void rt_launch_camerarays(const RtLaunch& a, float4* camera_results);
// the prepass of every frame of a.frames (-> CameraResults); with a.cells_from_cam the
// tracescreen launch derives CellDistance from them first (setTargetDepths, in k_order)
void rt_launch_camerarays_batch(const RtLaunch& a);
// Trace the region [off, off+ext) in 32x32-pixel tiles of every frame of a.frames (cells and
// outputs from the table), tile-cyclic sharding: a single frame traces the tiles t (row-major
// over the region) with t % tile_stride == tile_first; in a batch of n > 1 frames with
// tile_stride > 1, frame f traces shard (tile_first + f) % tile_stride (per-frame rotation).
void rt_launch_tracescreen(const RtLaunch& a, uint32_t off_x, uint32_t off_y, uint32_t ext_x, uint32_t ext_y,
                           uint32_t tile_first, uint32_t tile_stride);

#define RT_TILE 32
#define RT_FIN_SLOTS 1536 // k_trace's fin pool slots per block
#define RT_AO_POOL_SLOTS 256 // k_trace's AO counter slots per block (LDS) and their colours (cpool)
// k_trace's queue capacities per block (1024 threads = 16 waves): the hit queue and the long-ray
// spill stack.  A wave starts a primary unit only while fewer than 64 hits are queued and starts
// shading only while fewer than 128 long rays are (k_trace's work priority), so a block never
// queues more than 64 + 16 * 64 * aa hits or 128 + 16 * 64 * (1 + ao) long rays plus 16 compaction
// hand-backs of < 64: the rings cannot fill.
inline void rt_spill_caps(int aa, int ao, uint32_t* hits, uint32_t* longs)
{
    *hits = 64u * (uint32_t)aa * 17u + 64u;
    *longs = 64u * 16u * (uint32_t)(ao + 2) + 256u;
}
// samples the split pipeline addresses for a w x h frame: whole 32x32 tiles x AA
inline size_t rt_split_samples(int w, int h, int aa)
{
    return (size_t)((w + RT_TILE - 1) / RT_TILE) * ((h + RT_TILE - 1) / RT_TILE) * RT_TILE * RT_TILE * (size_t)aa;
}
inline size_t rt_shard_tiles(int w, int h, int rank, int count)
{
    size_t tx = (size_t)(w + RT_TILE - 1) / RT_TILE, ty = (size_t)(h + RT_TILE - 1) / RT_TILE, total = tx * ty;
    return total > (size_t)rank ? (total - (size_t)rank + (size_t)count - 1) / (size_t)count : 0;
}
// RGBA8 framebuffer -> BGRX rows (RecorderWinAPI::write's swizzle), dst pitch in uint32 words
void rt_launch_bgrx(hipStream_t s, const uint32_t* fb, uint32_t* dst, int w, int h, int pitch_words);
// Shard transport jobs of one launch (a kernel argument: 2.5 KiB): job j copies shard shard[j]
// of the w x h framebuffer fb[j] to packed[j] (pack != 0: 1024 px per tile, tiles ascending) or back.
#define RT_SHARD_JOBS 128
struct ShardJobs {
    uint32_t* fb[RT_SHARD_JOBS];
    uint32_t* packed[RT_SHARD_JOBS];
    int shard[RT_SHARD_JOBS];
};
void rt_launch_shard_copy(hipStream_t s, const ShardJobs& jobs, int n, int w, int h, int count, int pack);

// diagnostics (primitive-level parity tests)
void rt_launch_debug_math(hipStream_t s, int op, const float* a, const float* b, float* y, int n);
void rt_launch_debug_noise(const RtLaunch& a, const float* xyz, float* out, int n, int density);
void rt_launch_debug_sky(const RtLaunch& a, const float* dirs, float* out, int n);
void rt_launch_debug_spin(hipStream_t s, const unsigned long long* base, unsigned long long until_ticks,
                          unsigned long long ticks, unsigned long long* stamp);
