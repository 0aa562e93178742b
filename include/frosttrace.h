/*
 * frosttrace.h -- C-ABI drop-in boundary of the MI355X-native terrain ray-marcher.
 *
 * Every entry point replaces one call of the reference engine's dispatch-and-
 * readback surface (paths relative to /root/reference/gpuraytrace):
 *
 *   IDevice         Factories/IDevice.h:16-54, DeviceFactory.cpp:6-29
 *   ICompute        Factories/ICompute.h:16-59 (implemented by Adapters/ComputeDirect3D.cpp)
 *   IShaderVariable Graphics/IShaderVariable.h:7-40 (ShaderVariableDirect3D.cpp:195-202)
 *   IShaderArray    Graphics/IShaderVariable.h:42-61 (UAVBufferD3D :92-193, StructuredBufferD3D :204-281)
 *   ITexture        Factories/ITexture.h:38-63 (TextureDirect3D.cpp:40-164)
 *   VFS::addPath    Common/VFS.h (landscape selection, Terrain.cpp:23)
 *
 * Conventions: plain C types only; opaque handles; functions return RT_OK (0) or
 * a negative RT_ERR_* code and set a thread-local message (rt_last_error()).
 * Lookups that the reference answers with nullptr (missing variable/array)
 * return NULL here too.  All GPU work is enqueued on the device's HIP stream;
 * calls that hand data to the host (rt_array_map, rt_device_readback*) block.
 */
#ifndef FROSTTRACE_H
#define FROSTTRACE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 9

enum {
    RT_OK = 0,
    RT_ERR_INVALID = -1,    /* bad handle / argument */
    RT_ERR_HIP = -2,        /* HIP runtime error (message carries hipGetErrorString) */
    RT_ERR_NOT_FOUND = -3,  /* unknown shader file / entry / landscape */
    RT_ERR_UNSUPPORTED = -4,/* operation the reference also rejects (e.g. map on an SRV array) */
    RT_ERR_STATE = -5       /* e.g. run() before create()/swap(), missing texture */
};

/* DeviceDirect3D.cpp:113-126 swap-chain format R8G8B8A8_UNORM is always
 * produced; RT_DEVICE_FLOAT_OUTPUT additionally keeps the pre-quantisation
 * float4 colour (texOut's float4 value, tracescreen.hlsl:75) for parity. */
enum {
    RT_DEVICE_FLOAT_OUTPUT = 1u,
    RT_DEVICE_STATS = 2u,
    RT_DEVICE_GRAPH = 4u,
    /* 8u, 16u: retired in ABI 6 (ABI <= 5 RT_DEVICE_SEG_TAIL_OFF / _ON, no effect since ABI 4);
     * rt_device_create rejects them, as every unknown flag */
    RT_DEVICE_DEBUG_SMALL_RINGS = 32u,
    RT_DEVICE_DEBUG_WITHHOLD_FUSE = 64u,
    RT_DEVICE_GATED = 128u,
    RT_DEVICE_DEBUG_GATE_STRESS = 512u,
    RT_DEVICE_DEFERRED = 1024u,
    RT_DEVICE_DEBUG_DEFER_SMALL = 2048u
};
/* RT_DEVICE_GRAPH: rt_terrain_render / rt_terrain_render_feed capture the frame's launches
 * into two hipGraphs (prepass + setTargetDepths, tracescreen) on first use and replay them
 * every frame; a changed launch argument (shader swap, buffers, shard, stats) re-captures.
 * No reference counterpart (the D3D frame loop re-records its dispatches every frame).
 * RT_DEVICE_DEBUG_SMALL_RINGS (ABI 4, diagnostic): the trace kernel's per-CU LDS long-ray ring holds
 * 64 entries instead of 570 and its fin pool 8 slots instead of 1536, so queued long rays take the
 * per-block spill rings in HBM and most long shadows the fin[t] fallback (the parity tests run
 * frames through those paths); same bits, slower.
 * RT_DEVICE_GATED (ABI 7, opt-in): a full nomadplains render this device leads (rt_terrain_render /
 * _batch, not the camera feed, not the instrumented RT_DEVICE_STATS kernels) is ONE gated launch: the
 * trace kernel runs the batch's prepass rays first and starts each 8x8 unit as soon as the prepass rays
 * its cells' setTargetDepths reads are in; the frame's last prepass task writes its CellDistance.  Same
 * bits as the default sequence (the camerarays prepass as its own launch, then setTargetDepths and the
 * trace).  Measured slower on MI355X (prepass rays that share their SIMDs with
 * units march 2-3x slower than alone), so it is not the default.
 * RT_DEVICE_DEBUG_WITHHOLD_FUSE (ABI 7, diagnostic): a trace this device leads that would run the next
 * batch's fused prepass (rt_terrain_trace_ahead) runs none of its tasks, so that batch's bounded wait
 * times out: the fail-safe's test (rt_device_check below).
 * RT_DEVICE_DEBUG_GATE_STRESS (ABI 8, diagnostic, with RT_DEVICE_GATED): the gated launch's cross-CU hand-off of a
 * frame's CellDistance under stress -- every trace wave first reads the frame's previous CellDistance with
 * plain loads (its CU's L1 holds lines that the frame's last prepass task then rewrites) and that task waits
 * ~200 us before it stores them, so units read the flagged cells late, on CUs whose L1 holds the old ones.
 * RT_DEVICE_DEFERRED (ABI 9): deferred submission for the one-frame-per-call loop.  rt_terrain_render queues
 * its frame's prepass (or has it queued) and uploads both constant blocks, but its setTargetDepths + trace are
 * launched by the NEXT rt_terrain_render, whose own frame's prepass then runs inside that trace kernel
 * (nomadplains, a trace that has tiles, the same noise tables): a D3D driver's batching of a frame's
 * dispatches until the next submission, without a prepass launch that waits for the trace's CUs.  Every other
 * call that launches on, reads, waits on or reconfigures the device -- rt_device_flush, _synchronize,
 * _readback*, _stats*, _kernel_time, _set_stream, _wait_event, _record_event, _check, _framebuffer, _stream,
 * _destroy, rt_device_present while recording, any other render, prepass or shard call, a map / unmap / write
 * or device pointer of its arrays, a compute run / swap / destroy / set_texture, a texture init / destroy,
 * rt_device_defer_batch -- launches a pending
 * frame first.  rt_device_present without a recorder launches nothing (there is no display): a caller that
 * reads the framebuffer through its own stream calls rt_device_flush or rt_device_record_event first.  Same
 * bits as without the flag.  At one frame to a launch (the default; rt_device_defer_batch), a device of fewer than
 * 1280 x 720 pixels renders every frame as without the flag: its trace is shorter than the prepass it would carry
 * (profiles/r06/deferred.md).
 * RT_DEVICE_DEBUG_DEFER_SMALL (ABI 9, diagnostic, with RT_DEVICE_DEFERRED): the one-frame deferral at every frame
 * size, so that tests run it on small frames. */

/* ITexture.h:7-33 enum values */
enum { RT_TEXTURE_1D = 0, RT_TEXTURE_2D = 1, RT_TEXTURE_3D = 2 };
enum { RT_FORMAT_UNKNOWN = 0, RT_FORMAT_R8G8B8A8_SNORM = 1, RT_FORMAT_R8G8B8A8_UNORM = 2, RT_FORMAT_R8G8B8A8_UINT = 3 };

typedef struct rt_device_s* rt_device;
typedef struct rt_compute_s* rt_compute;
typedef struct rt_texture_s* rt_texture;
typedef struct rt_variable_s* rt_variable;
typedef struct rt_array_s* rt_array;
typedef struct rt_recorder_s* rt_recorder;

typedef struct {
    unsigned long long primary_steps; /* traceRay iterations, primary rays */
    unsigned long long shadow_steps;  /* traceRay iterations, shadow rays */
    unsigned long long prepass_steps; /* traceRay iterations, camerarays */
    unsigned long long hits;          /* primary hits == shadow rays */
    unsigned long long noise_calls;   /* noise3d evaluations (BASELINE.md algorithmic work unit) */
    unsigned long long ao_steps;      /* traceRay iterations, AO rays (build extension RT_AO_SAMPLES) */
    unsigned long long noise_wave_iters; /* wave64 iterations of the noise3d evaluations outside the prepass
                                          * (noise_calls / (64 * this) = SIMD lane utilisation of the
                                          * noise work; ABI 2) */
} rt_stats;

/* ---- diagnostics ---- */
const char* rt_last_error(void);
int rt_abi_version(void);

/* ---- VFS (Common/VFS.cpp:19-31; Terrain.cpp:23 adds "Media/<landscape>") ----
 * The most recently added "Media/<name>" path selects the landscape whose
 * shaders rt_compute_create() loads (nomadplains, testing, simple, greenrocks). */
int rt_vfs_add_path(const char* path);
int rt_vfs_clear(void);

/* ---- IDevice ----
 * rt_device_create  <- DeviceFactory::construct + DeviceDirect3D::create (DeviceDirect3D.cpp:77-227):
 *                      `ordinal` is the -g adapter index (:128-141), width/height the window size.
 * rt_device_present <- IDevice::present (DeviceDirect3D.cpp:234-257): frame boundary.
 * rt_device_flush   <- IDevice::flush (DeviceDirect3D.cpp:259-262).
 * rt_device_readback<- the present() staging readback (:244-256): RGBA8 rows, `row_pitch` bytes apart. */
int rt_device_create(int ordinal, int width, int height, unsigned flags, rt_device* out);
void rt_device_destroy(rt_device dev);
int rt_device_present(rt_device dev);
int rt_device_flush(rt_device dev);
int rt_device_synchronize(rt_device dev);
int rt_device_readback(rt_device dev, void* dst, size_t row_pitch);
int rt_device_readback_float(rt_device dev, float* dst); /* W*H*4 floats, needs RT_DEVICE_FLOAT_OUTPUT */
/* rt_device_readback_bgrx <- the recorder's readback (DeviceDirect3D.cpp:242-256) with
 * RecorderWinAPI::write's pixel conversion (RecorderWinAPI.cpp:244-253) done on the GPU:
 * rows of W uint32 (B, G, R, 0) = MFVideoFormat_RGB32, `row_pitch` bytes apart. */
int rt_device_readback_bgrx(rt_device dev, void* dst, size_t row_pitch);
int rt_device_size(rt_device dev, int* width, int* height);
void* rt_device_framebuffer(rt_device dev);       /* device pointer, W*H uint32 RGBA8 */
void* rt_device_stream(rt_device dev);            /* hipStream_t */
/* NULL = the device's own stream.  Devices' own streams are reference-counted: a device that
 * borrows another device's stream keeps it alive, so the owner may be destroyed first (its stream
 * is destroyed with its last user).  A stream no device created (the caller's) must outlive every
 * device using it: rt_device_destroy synchronizes the stream its device uses. */
int rt_device_set_stream(rt_device dev, void* hip_stream);
/* (ABI 4) devices currently holding `hip_stream` (its owner while alive + its borrowers); 0 for a
 * stream no live device created. */
int rt_stream_refs(void* hip_stream);
int rt_device_stats(rt_device dev, rt_stats* out, int reset); /* needs RT_DEVICE_STATS */
/* (ABI 4) the same with the caller's struct size: writes min(size, sizeof(rt_stats)) bytes, so a
 * caller built against an older, shorter rt_stats is never written past its struct. */
int rt_device_stats_sized(rt_device dev, rt_stats* out, size_t size, int reset);
/* HIP-event timing of the dominant kernel (tracescreen) on the device stream:
 * enable, then rt_device_kernel_time returns the summed elapsed ms and launch count
 * since the last call (synchronises). */
int rt_device_set_profiling(rt_device dev, int enable);
int rt_device_kernel_time(rt_device dev, double* total_ms, int* launches);
/* RT_DEVICE_GRAPH bookkeeping: graphs captured and graph launches since device creation. */
int rt_device_graph_info(rt_device dev, unsigned long long* captures, unsigned long long* launches);
/* (ABI 7) Counters of the renders a device led: RT_INFO_GATED_LAUNCHES = renders whose prepass ran inside
 * their trace kernel (the gated launch), RT_INFO_PREPASS_LAUNCHES = renders with a prepass launch of
 * their own, RT_INFO_PRESTREAM_RENDERS = those of them whose prepass ran on the device's prepass stream
 * (rt_terrain_render with a frame in flight).  No reference counterpart (the tests check which sequence
 * ran). */
/* (ABI 9) RT_INFO_DEFERRED_FUSED: RT_DEVICE_DEFERRED renders whose prepass ran inside the previous frame's
 * trace kernel. */
enum { RT_INFO_GATED_LAUNCHES = 0, RT_INFO_PREPASS_LAUNCHES = 1, RT_INFO_PRESTREAM_RENDERS = 2, RT_INFO_DEFERRED_FUSED = 3 };
int rt_device_info(rt_device dev, int key, unsigned long long* out);
/* (ABI 8) The trace kernel of the renders this device leads launches (CUs - n) persistent blocks instead of
 * one per CU (0 <= n < CUs; default 0), so n CUs stay free beside it for another stream's kernels -- a
 * collective's (RCCL's receive on rank 0 at N > 1, which otherwise queues behind the other batch's trace
 * until its tail) or a transport copy.  Same bits.  No reference counterpart. */
int rt_device_reserve_cus(rt_device dev, int n);
/* (ABI 9) An RT_DEVICE_DEFERRED device traces `frames` (1..4; default 1) frames to a launch: each rt_terrain_render
 * of the whole frame (shard 0 of 1) snapshots its frame's constant blocks into a frame slot of the device (its own
 * CameraResults, CellDistance and framebuffers) and queues it; every frames-th render launches the oldest
 * `frames` queued frames' setTargetDepths + trace as one batch, with the next `frames` frames' prepasses inside
 * that trace kernel.  A flush (the calls listed under RT_DEVICE_DEFERRED) launches everything queued; its last
 * frame writes the device's framebuffers and the compute pair's CellDistance and CameraResults, the others write
 * their slots (scratch: the reference's DISCARD swap chain never shows a frame that was not presented to a
 * reader).  Same bits per frame.  Changing it launches what is queued.  No reference counterpart (the D3D
 * runtime queues up to three frames). */
int rt_device_defer_batch(rt_device dev, int frames);
/* (ABI 6) Stream handoff without a host synchronisation.  `hip_event` is a hipEvent_t the caller
 * owns (a C++ host's, or torch.cuda.Event.cuda_event).  rt_device_wait_event: the work the device
 * queues from now on waits for the event -- e.g. buffers the caller filled on its own stream, then
 * recorded the event there (rt_shard_unpack's source, the split prepass's gathered CameraResults).
 * rt_device_record_event: records the event after everything queued on the device so far; the
 * caller's stream waits for it (hipStreamWaitEvent) before it reads the device's outputs.  The
 * device streams are non-blocking, so without one of these (or a host synchronisation) a caller's
 * stream and a device's run in no order.  No reference counterpart (D3D11 orders one immediate
 * context implicitly). */
int rt_device_wait_event(rt_device dev, void* hip_event);
int rt_device_record_event(rt_device dev, void* hip_event);
/* (ABI 6) Queue-overflow check: k_trace's per-block queues (hit stack, long-ray spill ring) are
 * bounded by its work priorities (rt_spill_caps); a push that would exceed a bound is not stored and
 * raises a sticky flag on the device instead of overwriting queued work.  rt_device_check
 * synchronises the device stream and returns RT_ERR_STATE (the message names the queue) if any
 * flag was raised since the last check, clearing it; RT_OK otherwise.
 * (ABI 7) Fail-safe of the fused prepass (rt_terrain_trace_ahead): when a batch's bounded wait for
 * its prepass rays times out (0.5 s; never expected), its frames may be wrong.  The kernel then also
 * sets a host-mapped word of its GPU, and from then on every call that launches on, synchronises or
 * reads a device of that GPU (rt_terrain_*, rt_compute_run, rt_device_present / synchronize /
 * readback*, rt_array_map, rt_shard_*) returns RT_ERR_STATE, until rt_device_check on a device of
 * that GPU reports and clears it.  A host that follows the reference's call sequence and never calls
 * rt_device_check therefore cannot read such a frame silently. */
int rt_device_check(rt_device dev);

/* ---- ITexture (IDevice::createTexture + ITexture::create(dims, fmt, w, h, data, binding, cpu)) ---- */
int rt_texture_create(rt_device dev, rt_texture* out);
int rt_texture_init(rt_texture tex, int dimensions, int format, int width, int height, const void* data,
                    int binding, int cpu_access);
void rt_texture_destroy(rt_texture tex);

/* ---- ICompute ----
 * rt_compute_create     <- IDevice::createCompute (DeviceDirect3D.cpp:264-267)
 * rt_compute_load       <- ICompute::create(directory, file, entry, ThreadSize, macros)
 *                          (ComputeDirect3D.cpp:403-465).  Files: "tracescreen.hlsl",
 *                          "camerarays.hlsl"; macros RECORDING, AA_SAMPLES and the build
 *                          extension RT_MAX_STEPS.  A failed load keeps the previous shader.
 * rt_compute_swap       <- ICompute::swap (:508-528): 1 if a new shader became current;
 *                          invalidates the handles from rt_compute_get_*.
 * rt_compute_run        <- ICompute::run (:530-581): dispatch (dx,dy,dz) groups of the
 *                          compiled thread size; silent no-op without a current shader.
 * rt_compute_set_texture<- ICompute::setTexture (:583-614), borrowed (not owned).
 * rt_compute_get_*      <- getVariable/getArray/getBuffer by reflected name (NULL if absent;
 *                          getBuffer is always NULL, as the reference's CBuffer=0 mask makes it). */
int rt_compute_create(rt_device dev, rt_compute* out);
void rt_compute_destroy(rt_compute cs);
int rt_compute_load(rt_compute cs, const char* directory, const char* file, const char* entry, int tx, int ty, int tz,
                    const char* const* macro_names, const char* const* macro_values, int n_macros);
int rt_compute_swap(rt_compute cs);
int rt_compute_run(rt_compute cs, unsigned dispatch_x, unsigned dispatch_y, unsigned dispatch_z);
int rt_compute_set_texture(rt_compute cs, int stage, rt_texture tex);
int rt_compute_thread_size(rt_compute cs, int* x, int* y, int* z);
rt_variable rt_compute_get_variable(rt_compute cs, const char* name);
rt_array rt_compute_get_array(rt_compute cs, const char* name);
void* rt_compute_get_buffer(rt_compute cs, const char* name);

/* ---- IShaderVariable ---- write copies exactly the reflected size (cbuffer shadow, uploaded lazily on run) */
int rt_variable_write(rt_variable var, const void* data);
size_t rt_variable_size(rt_variable var);
const char* rt_variable_name(rt_variable var);

/* ---- IShaderArray ----
 * create: allocate `elements` x reflected stride.  UAV arrays (CameraResults): map = blocking
 * device->host copy, unmap = host->device copy back; write unsupported.  SRV arrays
 * (CellDistance): write = full upload; map/unmap unsupported.  As UAVBufferD3D/StructuredBufferD3D. */
int rt_array_create(rt_array arr, unsigned elements);
void* rt_array_map(rt_array arr);
int rt_array_unmap(rt_array arr);
int rt_array_write(rt_array arr, const void* data);
size_t rt_array_stride(rt_array arr);
void* rt_array_device_pointer(rt_array arr);

/* ---- Terrain::render without the host round trip (Terrain.cpp:105-136) ----
 * Runs camera_cs (prepass) -> setTargetDepths on the device (Terrain.cpp:398-439) ->
 * screen_cs over the whole screen, all enqueued on the device stream.  Equivalent to the
 * reference sequence run(2,2,1); CameraResults map/unmap; setTargetDepths; CellDistance
 * write; tiled run(...).  With shard_count > 1 only screen tiles t (32x32 pixels,
 * row-major tile index) with t % shard_count == shard_rank are traced.
 * Frames in flight (ABI 7, same bits): from a device's second consecutive rt_terrain_render on,
 * the prepass runs on the device's own prepass stream, ordered after the previous frame's
 * setTargetDepths (the last reader of CameraResults) and before this frame's setTargetDepths, so it
 * overlaps the previous frame's trace; the device stream stays the order a host sees (synchronise,
 * readbacks, events).  Any other call that touches the device's arrays or launches on it (a batch, the
 * feed, an ahead prepass, rt_compute_run, rt_array_unmap / write, a stream change, rt_device_wait_event)
 * makes the next render prepass in line.  A host writing CameraResults through rt_array_device_pointer on its own
 * must synchronise first.  Not for RT_DEVICE_GRAPH, RT_DEVICE_STATS or RT_DEVICE_GATED devices. */
int rt_terrain_render(rt_compute camera_cs, rt_compute screen_cs, int shard_rank, int shard_count);
/* rt_terrain_render_feed: rt_terrain_render that also hands the frame's 1024 CameraResults
 * (camerarays.hlsl:12-21, Terrain::getCameraView) to the host as soon as the prepass ends,
 * without waiting for tracescreen -- the feed of Flyby::fly (Gameplay/Flyby.cpp:26-196, which
 * reads the previous frame's view).  rt_terrain_feed_wait blocks until that copy has landed and
 * copies it (1024 x float4: hit xyz, depth) to `camera_results`. */
int rt_terrain_render_feed(rt_compute camera_cs, rt_compute screen_cs, int shard_rank, int shard_count);
int rt_terrain_feed_wait(rt_compute camera_cs, float* camera_results);
/* rt_terrain_render_batch: rt_terrain_render for n (1..24; 16 before ABI 6) frames at once -- frame i is
 * (camera_cs[i], screen_cs[i]), each with its own constants (camera, sun), CameraResults,
 * CellDistance and device framebuffer.  All frames must share one GPU, resolution,
 * landscape, macro set and noise tables.  Every frame's prepass runs in one launch, and one
 * tracescreen launch traces all frames' units frame-major, so one frame's last rays overlap
 * the next frame's units instead of idling the GPU.  Enqueued on the stream of frame 0's
 * device with frame 0's device buffers and counters; streams of frames on other devices
 * wait for the batch.  No reference counterpart (the reference renders one frame per
 * Terrain::render); each frame's pixels equal its rt_terrain_render frame bit for bit.
 * Sharded (shard_count > 1, n > 1): frame i traces shard (shard_rank + i) % shard_count, a
 * per-frame rotation that evens out the ranks' work; rt_shard_pack/unpack frame i with that
 * shard index. */
int rt_terrain_render_batch(const rt_compute* camera_cs, const rt_compute* screen_cs, int n, int shard_rank,
                            int shard_count);
/* (ABI 7) rt_terrain_render_batch of a shard (shard_count >= 2) whose pixels go straight to a packed
 * device buffer instead of the framebuffers: frame i's shard at dst_device + i * frame_stride, in
 * rt_shard_pack's layout (its k-th tile at k * 4 KiB, rows of 32 pixels).  The trace kernels store there
 * directly, so a rank's batch needs no rt_shard_pack_batch launch before its gather (the pack queued
 * behind the other batch in flight; parallel.run_batch's direct pack).  RGBA8-only devices
 * (RT_ERR_UNSUPPORTED with RT_DEVICE_FLOAT_OUTPUT); the framebuffers are not written. */
int rt_terrain_render_batch_packed(const rt_compute* camera_cs, const rt_compute* screen_cs, int n, int shard_rank,
                                   int shard_count, void* dst_device, size_t frame_stride);
/* The same batch in two phases, for a prepass split across ranks (one process per GPU):
 * rt_terrain_prepass_batch runs the camerarays prepass of frames [first, first + count) only
 * and writes frame f's 1024 CameraResults to camera_out + f * 1024 float4 (a device buffer of
 * n * 16 KiB); the ranks' shares are then exchanged with one all-gather of that buffer, and
 * rt_terrain_trace_batch runs setTargetDepths + tracescreen of all n frames from camera_in
 * (the gathered buffer), copying each frame's results into its CameraResults array too.
 * The prepass is deterministic, so the frames equal rt_terrain_render_batch's bit for bit. */
int rt_terrain_prepass_batch(const rt_compute* camera_cs, const rt_compute* screen_cs, int n, int first, int count,
                             void* camera_out);
int rt_terrain_trace_batch(const rt_compute* camera_cs, const rt_compute* screen_cs, int n, int shard_rank,
                           int shard_count, const void* camera_in);
/* (ABI 5) The prepass one batch ahead, for a stream of batches (FrameRing(lookahead=True),
 * parallel.run_batch): rt_terrain_prepass_ahead queues the batch's camerarays prepass (into each
 * frame's CameraResults) on the GPU's side stream -- one per GPU, created on first use -- after
 * the last setTargetDepths of the batches screen_cs[0]'s device leads (their last read of those
 * arrays).  Issued before the previous batch's trace, it gets CUs before that trace's persistent
 * kernel holds them all.  rt_terrain_trace_ahead then runs setTargetDepths + tracescreen of the
 * batch after that prepass; for frames the pending prepass did not cover (other computes, more
 * frames, or camera constants written since) it renders the full batch (rt_terrain_render_batch)
 * instead, so the frames always equal rt_terrain_render_batch's bit for bit.  One ahead prepass
 * per leading device at a time (RT_ERR_STATE otherwise); not on RT_DEVICE_GRAPH devices.
 * No reference counterpart (Terrain::render runs its prepass in line, Terrain.cpp:105-136). */
int rt_terrain_prepass_ahead(const rt_compute* camera_cs, const rt_compute* screen_cs, int n);
int rt_terrain_trace_ahead(const rt_compute* camera_cs, const rt_compute* screen_cs, int n, int shard_rank,
                           int shard_count);
/* Tile-cyclic shard transport: pack this rank's tiles from the framebuffer into a
 * contiguous device buffer (RGBA8, 32x32-pixel tiles in tile order), or unpack a rank's
 * packed tiles into the framebuffer.  Byte counts from rt_shard_bytes. */
size_t rt_shard_bytes(rt_device dev, int shard_rank, int shard_count);
int rt_shard_pack(rt_device dev, int shard_rank, int shard_count, void* dst_device);
int rt_shard_unpack(rt_device dev, int shard_rank, int shard_count, const void* src_device);
/* The same for n frames in one launch (ABI 3): job i packs shard shard_ranks[i] of devs[i]'s
 * framebuffer into dst_device[i] (or unpacks src_device[i] into it).  Every device has the same
 * size; the launch runs on devs[0]'s stream, and devices on other streams are ordered around it
 * (their earlier work before, their later work after).  A batch's root unpacks its (N-1) x B
 * shards with one call (parallel.run_batch) instead of one launch each. */
int rt_shard_pack_batch(const rt_device* devs, const int* shard_ranks, int shard_count, void* const* dst_device,
                        int n);
int rt_shard_unpack_batch(const rt_device* devs, const int* shard_ranks, int shard_count,
                          const void* const* src_device, int n);

/* ---- host helpers (Noise.cpp:39-94, Camera.cpp, Terrain.cpp:285-311) ----
 * rt_noise_generate: the engine's noise tables; rand_kind 0 = MSVC CRT rand (the
 * reference's shipping platform), 1 = glibc rand.  perm2d: 128*128*4 bytes,
 * grad: 128*4 floats. */
int rt_noise_generate(uint32_t seed, int rand_kind, uint8_t* perm2d, float* grad);
/* Terrain::setTargetDepths (Terrain.cpp:398-439) on the host: CameraResults float4[1024] ->
 * CellDistance float2[1024], for engines that keep the reference's readback round trip. */
int rt_terrain_set_target_depths(const float* camera_results, float* cell_distance);

/* ---- diagnostics (primitive-level parity tests; no reference counterpart) ----
 * rt_debug_math: device evaluation of the numeric primitives of DESIGN.md §Numerics
 *   (op 0 exp2, 1 log2, 2 exp, 3 sin, 4 cos, 5 sqrt, 6 rcp, 7 rsqrt, 8 pow, 9 max,
 *   10 min, 11 pow for x >= 0); host arrays of n floats (b may be NULL for unary ops).
 *   op 12 sweeps the nomadplains octave-count estimate over the n floats whose bit
 *   patterns follow bits(a[0]) and writes 3 uint32 to out: unflagged estimates that differ
 *   from the exact count, flagged estimates, patterns swept.
 * rt_debug_noise: noise3d (density = 0, noise.hlsl:153-179) or the compute's landscape
 *   getDensity (density = 1) at n points (xyz interleaved), with the compute's
 *   current tables and constants. */
int rt_debug_math(rt_device dev, int op, const float* a, const float* b, float* out, int n);
int rt_debug_noise(rt_compute cs, const float* xyz, float* out, int n, int density);
/* rt_debug_sky (ABI 4): the sky of n view directions (xyz interleaved) with the compute's current
 *   constants (Eye, SunDirection) and tables: 7 floats per direction, getRayleighMieColor's
 *   (mie.rgb, rayleigh.rgb) (sky.hlsl:83-137) and getSpaceColor (sky.hlsl:26-36). */
int rt_debug_sky(rt_compute cs, const float* dirs, float* out, int n);
/* rt_debug_spin (ABI 7, scripts/batch_shard_sim.py's coupled transport model): one 64-thread workgroup
 *   on `hip_stream` that stores the GPU's 100 MHz clock at its start to *stamp_device (if not NULL), waits
 *   until *base_device + until_ticks (base_device a stamp an earlier spin stored; NULL: no wait), then
 *   spins `ticks` more -- the CU a collective's kernel holds while it waits for its peer and transfers. */
int rt_debug_spin(void* hip_stream, const unsigned long long* base_device, unsigned long long until_ticks,
                  unsigned long long ticks, unsigned long long* stamp_device);
/* rt_debug_defer_slot (ABI 9, tests): the device pointers of frame slot `slot` of an RT_DEVICE_DEFERRED device
 *   tracing K >= 2 frames to a launch (rt_device_defer_batch): its RGBA8 framebuffer, CameraResults (1024
 *   float4) and CellDistance (1024 float2), where a queued frame that was not a flush's last one wrote them.
 *   Frame i of a sequence that started with an empty queue takes slot i % (2K).  RT_ERR_INVALID for a slot
 *   never used. */
int rt_debug_defer_slot(rt_device dev, int slot, void** fb8, void** camera_results, void** cell_distance);

/* ---- IRecorder (Factories/IRecorder.h; RecorderWinAPI.cpp; RecorderFactory.cpp) ----
 * rt_recorder_create   <- RecorderFactory::construct(device, frameRate, fixedSpeed) + create():
 *                         attaches to the device (DeviceDirect3D::setRecorder, :229-232).  The
 *                         Media Foundation WMV sink (:80, "output.wmv") becomes a raw-video sink:
 *                         `path` (default "output.rgb32") receives the frames as raw
 *                         MFVideoFormat_RGB32 rows (B, G, R, 0), `path`.txt one line per sample
 *                         "frame sample_time duration" in 100 ns units (IMFSample time stamps).
 * rt_recorder_start    <- IRecorder::start + BeginWriting (:205-216)
 * rt_recorder_stop     <- IRecorder::stop + Finalize (:218-224); no start after it (as the sink writer)
 * rt_recorder_write    <- RecorderWinAPI::write(frame, stride) on host RGBA8 rows (:226-279)
 * rt_device_present    writes the frame to an attached, recording recorder (DeviceDirect3D.cpp:242-256),
 *                      with the swizzle on the GPU.
 * rt_recorder_set_frame_time: Timer::getConstant() the next sample uses when !fixed_speed (:264-269). */
int rt_recorder_create(rt_device dev, int frame_rate, int fixed_speed, const char* path, rt_recorder* out);
int rt_recorder_start(rt_recorder rec);
int rt_recorder_stop(rt_recorder rec);
int rt_recorder_is_recording(rt_recorder rec);
int rt_recorder_set_frame_time(rt_recorder rec, float seconds);
int rt_recorder_write(rt_recorder rec, const void* frame, int stride);
int rt_recorder_info(rt_recorder rec, unsigned long long* frames, unsigned long long* next_sample_time,
                     unsigned long long* frame_duration);
void rt_recorder_destroy(rt_recorder rec);

/* ---- VariableManager (Common/VariableManager.{h,cpp}; main.cpp:99 `-m`) ----
 * The live-tweak TCP protocol (VariableManager.cpp:76-83): on connect the server sends every
 * registered variable as [1][name len:1][name][type len:1][type][size:2 LE][data]; a clear sends
 * [2]; the client writes a variable as [name len:1][name][data] (an unknown name closes the
 * connection).  Registered variables are the members of cbuffers named 'X...' (XTweakable's
 * SunDirection, tracing.hlsl:6-9); a write updates the compute's cbuffer shadow, uploaded on the
 * next launch.  As in ComputeDirect3D::create (:408, :188-197) every rt_compute_load clears the
 * registry and registers its own shader's variables -- so after Terrain::reload (tracescreen, then
 * camerarays, which has no 'X' cbuffer) the registry is empty, as in the reference.
 * rt_varmgr_register_compute (not in the reference) re-registers one compute's variables and
 * sends them to a connected client.  port <= 0 means 10666; bind_address NULL = 127.0.0.1. */
int rt_varmgr_start(int port, const char* bind_address);
int rt_varmgr_stop(void);
int rt_varmgr_count(void);
int rt_varmgr_register_compute(rt_compute cs);

#ifdef __cplusplus
}
#endif
#endif
