// rt_runtime.cpp -- implementation of the C-ABI in include/frosttrace.h.
//
// Mirrors the reference's D3D11 adapter semantics (Adapters/ComputeDirect3D.cpp,
// Adapters/ShaderVariableDirect3D.cpp, Adapters/DeviceDirect3D.cpp,
// Adapters/TextureDirect3D.cpp) on HIP: a compute object owns a "shader" (here: a
// precompiled gfx950 kernel family selected by file + landscape + macros) with
// reflected cbuffer variables whose CPU shadows are uploaded lazily on run(),
// structured/UAV arrays, and borrowed textures.  swap() replaces the current
// shader and invalidates its variables, exactly as the reference does.
#include <hip/hip_runtime.h>

#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/frosttrace.h"
#include "rt_kernels.h"
#include "rt_math.h"
#include "rt_noise.h"

// RT_DEVICE_DEFERRED with one frame to a launch: frames of fewer pixels render as without the flag (at 256x256 the
// fused prepass outlasts the frame's trace: 0.642 against 0.585 ms a frame; neutral at 1280x720)
#define RT_DEFER_FUSE_MIN_PIXELS ((size_t)1280 * 720)

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess) return fail(RT_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

std::mutex g_vfs_mu;
std::vector<std::string> g_vfs;

int landscape_from_vfs()
{
    std::lock_guard<std::mutex> lk(g_vfs_mu);
    static const char* names[] = {"nomadplains", "testing", "simple", "greenrocks"};
    for (auto it = g_vfs.rbegin(); it != g_vfs.rend(); ++it) { // VFS.cpp:19-31 searches newest first
        for (int l = 0; l < RT_NUM_LANDSCAPES; ++l) {
            std::string n = names[l];
            const std::string& p = *it;
            if (p.size() >= n.size() && p.compare(p.size() - n.size(), n.size(), n) == 0) return l;
        }
        if (it->find("benchmark") != std::string::npos) return -2; // Media/benchmark/terrain.hlsl:39-40 does not compile
    }
    return RT_NOMADPLAINS; // main.cpp:87 default landscape
}

// Pinned staging buffer whose reuse waits for the previous async copy.
struct Staging {
    void* host = nullptr;
    size_t bytes = 0;
    hipEvent_t ev = nullptr;
    bool pending = false;
    ~Staging()
    {
        if (ev) (void)hipEventDestroy(ev);
        if (host) (void)hipHostFree(host);
    }
    int upload(hipStream_t s, void* dst, const void* src, size_t n)
    {
        if (n > bytes) {
            if (pending) HIP_TRY(hipEventSynchronize(ev));
            if (host) HIP_TRY(hipHostFree(host));
            HIP_TRY(hipHostMalloc(&host, n));
            bytes = n;
            pending = false;
        }
        if (!ev) HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        if (pending) HIP_TRY(hipEventSynchronize(ev));
        memcpy(host, src, n);
        HIP_TRY(hipMemcpyAsync(dst, host, n, hipMemcpyHostToDevice, s));
        HIP_TRY(hipEventRecord(ev, s));
        pending = true;
        return RT_OK;
    }
};

} // namespace

// ---------------------------------------------------------------------------
struct rt_device_s {
    int ordinal = 0, width = 0, height = 0;
    unsigned flags = 0;
    // own_stream: created with the device; stream: the one it launches on (own, or borrowed via
    // rt_device_set_stream); both are reference-counted in the stream registry below
    hipStream_t own_stream = nullptr, stream = nullptr;
    uint32_t* fb8 = nullptr;
    float4* fb32 = nullptr;
    RtStats* stats = nullptr;
    float4* scratch_cam = nullptr; // camera results for rt_terrain_render when the compute has none
    uint32_t* queue = nullptr;     // persistent-kernel work counters (RT_CTR_BYTES)
    int num_cus = 256;
    int reserve_cus = 0;           // CUs the trace kernel leaves free (rt_device_reserve_cus)
    float4* samples = nullptr;     // per-sample buffers, sized for samples_cap samples
    float4* hitq = nullptr;       // k_trace's per-block hit queues and long-ray spill stacks (rt_spill_caps per block)
    float4* spill_long = nullptr;
    size_t hitq_n = 0, spill_long_n = 0; // records allocated (all blocks)
    uint32_t* order = nullptr;
    uint64_t* hitmask = nullptr; // per unit and AA sample: the primary-hit ballot (k_trace -> k_finish)
    float4* fin = nullptr;
    float4* finpool = nullptr; // k_trace's per-block fin pools (RT_FIN_SLOTS slots of 3 float4 per block)
    float4* cpool = nullptr;   // k_trace's per-block AO colour pools (RT_AO_POOL_SLOTS float4 per block)
    uint32_t* gate = nullptr;  // the gated launch (GatedPrepass): per frame task flags + ray counter
    uint32_t* claims = nullptr; //   and the units claimed per tile of the batch's order
    uint32_t* aocc = nullptr;
    size_t samples_cap = 0;
    // dominant-kernel timing (rt_device_set_profiling)
    bool profiling = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pool;
    size_t ev_used = 0;
    // RT_DEVICE_GRAPH: rt_terrain_render replays two captured graphs per frame, the prepass
    // (camerarays + setTargetDepths) and tracescreen, re-captured when any launch argument changes
    struct FrameGraph {
        std::vector<uint64_t> key;
        hipGraphExec_t exec = nullptr;
    } graph_pre, graph_trace;
    unsigned long long graph_captures = 0, graph_launches = 0;
    // renders this device led: gated launches (prepass inside the trace) and prepass launches (rt_device_info)
    unsigned long long gated_launches = 0, prepass_launches = 0, prestream_renders = 0, deferred_fused = 0;
    // RT_DEVICE_DEFERRED: the last rt_terrain_render's frame, its prepass queued (or run inside the trace before)
    // and both constant blocks up, whose setTargetDepths + trace are not launched yet: the next rt_terrain_render
    // launches them with its own frame's prepass fused into that trace; any other call that launches on, reads
    // or reconfigures the device launches them first (defer_flush)
    struct Deferred {
        struct rt_compute_s* cam = nullptr;
        struct rt_compute_s* scr = nullptr;
        int rank = 0, count = 1;
        bool pending = false;
    } defer;
    // RT_DEVICE_DEFERRED with rt_device_defer_batch(K >= 2): frames are traced K to a launch.  Each render takes a
    // frame slot (its constant blocks snapshotted there, its own CameraResults, CellDistance and framebuffers)
    // and queues it; every K-th render launches the oldest K queued frames' setTargetDepths + trace as one batch,
    // with the next K frames' prepasses fused into that trace kernel.  A flush launches everything queued; its
    // last frame writes the device's framebuffers and the API's CellDistance / CameraResults.
    struct FrameSlot {
        RtConsts hk{}, hkcam{};             // the frame's tracescreen and camerarays blocks, as at its render
        const RtConsts* dk = nullptr;       // where they went up (in the launch block of its prepass)
        const RtConsts* dkcam = nullptr;
        float4* cam = nullptr;   // its CameraResults
        float2* cells = nullptr; // its CellDistance
        uint32_t* fb8 = nullptr; // its framebuffers (scratch: only a flush's last frame is read)
        float4* fb32 = nullptr;
        ~FrameSlot()
        {
            for (void* p : {(void*)cam, (void*)cells, (void*)fb8, (void*)fb32})
                if (p) (void)hipFree(p);
        }
    };
    std::vector<std::unique_ptr<FrameSlot>> slots;
    // one upload per deferred launch: the frame tables it reads and the constant blocks of the frames whose
    // prepass it runs (a ring of 3: a block's frames are traced by the next launch, so a block is rewritten
    // three launches later, in stream order behind both)
    struct LaunchBlock {
        FrameTable ft, nx;
        RtConsts k[4], kcam[4];
    };
    LaunchBlock* blocks = nullptr;
    Staging block_stage[3];
    int block_next = 0;
    int defer_k = 1;         // frames per deferred launch (1: the Deferred path above)
    int slot_next = 0;
    std::deque<int> dq;      // queued frames' slots, oldest first; the first dq_pre have their prepass done
    int dq_pre = 0;
    struct rt_compute_s *dq_cam = nullptr, *dq_scr = nullptr;
    // frame tables (rt_kernels.h FrameTable): the batch's, and the split prepass's frame subset
    struct DevTable {
        FrameTable* d = nullptr;
        FrameTable last{};
        bool valid = false;
        Staging staging;
    } table, pre_table, fuse_table;
    hipEvent_t sync_ev = nullptr; // orders this device's stream against a batch on another device
    // rt_terrain_prepass_ahead, for batches led by this device: ev_order follows its last k_order
    // (the last read of the frames' CameraResults), ev_ahead the ahead prepass on the GPU's side
    // stream; ahead_cams are that prepass's frames (a trace of another batch prepasses again)
    hipEvent_t ev_order = nullptr, ev_ahead = nullptr;
    bool order_recorded = false, ahead_pending = false;
    std::vector<const void*> ahead_cams;
    // every device whose frames a pending ahead prepass writes (the lead included): its CameraResults
    // are not read -- by a render this device leads, or a map -- before ev_ahead_in
    hipEvent_t ev_ahead_in = nullptr;
    bool ahead_in_pending = false;
    // rt_terrain_render's own prepass stream (round 5): frame i+1's prepass waits for frame i's k_order
    // (ev_order) only, so it runs in frame i's trace tail instead of after it; ev_pre orders the trace
    // after it.  serial_ok: the last render this device led was such a render (nothing but k_order and
    // the trace read its CameraResults since)
    hipStream_t pre_stream = nullptr;
    hipEvent_t ev_pre = nullptr;
    bool serial_ok = false;
    // the prepass of the batch this device leads fused into another batch's k_trace (FusedPrepass):
    // STAGED = constants and frame table uploaded by rt_terrain_prepass_ahead, waiting for a trace to
    // take it; FUSED = a k_trace runs it (ev_fuser_done follows that launch).  fctl: its task / ray
    // counters (zeroed by the fusing batch's k_order, polled by this batch's k_order)
    enum { FUSE_NONE = 0, FUSE_STAGED = 1, FUSE_FUSED = 2 };
    int fuse_state = FUSE_NONE, fuse_n = 0;
    uint32_t* fctl = nullptr;
    std::vector<rt_device_s*> fuse_devs; // the devices of its frames
    hipEvent_t ev_fuser_done = nullptr;
    // recorded after the fusing launch's k_order, which zeroes fctl: this batch's own k_order (its poll of
    // fctl) waits for it, so it can never pass on the previous fused round's count
    hipEvent_t ev_fuse_order = nullptr;
    // output path: BGRX staging for the recorder / rt_device_readback_bgrx (allocated on first use)
    uint32_t* bgrx = nullptr;
    struct rt_recorder_s* recorder = nullptr; // DeviceDirect3D::recorder (setRecorder), not owned
    // children (IDevice::createCompute / createTexture); destroyed with the device
    std::vector<struct rt_compute_s*> computes;
    std::vector<struct rt_texture_s*> textures;
    ~rt_device_s();
};

static int recorder_capture(rt_recorder r);
static void recorder_detach(rt_recorder r);
static int defer_flush(rt_device d);

namespace {
// Work on stream s that touches device d's frames (their CameraResults) comes after a pending ahead
// prepass that writes them (rt_terrain_prepass_ahead, on the GPU's side stream).
int ahead_wait(rt_device_s* d, hipStream_t s)
{
    if (!d->ahead_in_pending) return 0;
    const hipError_t e = hipStreamWaitEvent(s, d->ev_ahead_in, 0);
    if (e != hipSuccess) return (int)e;
    d->ahead_in_pending = false;
    return 0;
}

// bracket one tracescreen launch with a pair of events when profiling is on
struct KernelTimer {
    rt_device_s* d;
    hipEvent_t stop = nullptr;
    explicit KernelTimer(rt_device_s* dev) : d(dev)
    {
        if (!d->profiling) return;
        if (d->ev_used == d->ev_pool.size()) {
            hipEvent_t a, b;
            if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return;
            d->ev_pool.emplace_back(a, b);
        }
        auto& pr = d->ev_pool[d->ev_used++];
        (void)hipEventRecord(pr.first, d->stream);
        stop = pr.second;
    }
    ~KernelTimer()
    {
        if (stop) (void)hipEventRecord(stop, d->stream);
    }
};
} // namespace

struct rt_texture_s {
    rt_device dev = nullptr;
    int dims = 0, fmt = 0, w = 0, h = 0;
    uint32_t* data = nullptr;
    uint64_t hash = 0; // FNV-1a of the texels (frame batches check that they share the noise)
};

struct Shader;

struct rt_variable_s {
    std::string name;
    int cbuf = 0, offset = 0, size = 0;
    Shader* owner = nullptr;
};

struct rt_array_s {
    std::string name;
    int stride = 0;
    bool uav = false;
    unsigned elements = 0;
    void* dev_ptr = nullptr;
    std::vector<uint8_t> host;
    Shader* owner = nullptr;
    rt_device dev = nullptr;
    Staging staging;
};

enum { KIND_CAMERARAYS = 0, KIND_TRACESCREEN = 1 };
enum { CB_XTWEAK = 0, CB_FRAME = 1, CB_PERM = 2, CB_NOISE = 3, CB_DISPATCH = 4, CB_COUNT = 5 };
static const int kCbSize[CB_COUNT] = {12, 84, 80, 2048, 8};

struct Shader;
static void varmgr_forget(Shader* s);
static void varmgr_clear();
static void varmgr_register(Shader* s);
static std::mutex g_cb_mu; // cbuffer shadows: written by the live-tweak thread (VariableManager) and the API

struct Shader {
    int kind = KIND_TRACESCREEN;
    int landscape = RT_NOMADPLAINS;
    int aa = 1, recording = 0, max_steps = 0, ao = 0;
    int tx = 16, ty = 16, tz = 1;
    bool has_cb[CB_COUNT] = {};
    std::vector<uint8_t> cb[CB_COUNT];
    bool cb_dirty = true;
    bool grad_dirty = true; // CBNoise (permGradients) changed: its own upload, not one per camera move
    std::vector<std::unique_ptr<rt_variable_s>> vars;
    std::vector<std::unique_ptr<rt_array_s>> arrays;
    rt_texture textures[16] = {};
    // device-side state
    RtConsts host_consts{};
    RtConsts* d_consts = nullptr;
    float4* d_grad = nullptr;
    Staging consts_staging, grad_staging;

    ~Shader()
    {
        varmgr_forget(this);
        if (d_consts) (void)hipFree(d_consts);
        if (d_grad) (void)hipFree(d_grad);
        for (auto& a : arrays)
            if (a->dev_ptr) (void)hipFree(a->dev_ptr);
    }
    void add_var(const char* n, int cbuf, int off, int size)
    {
        auto v = std::make_unique<rt_variable_s>();
        v->name = n;
        v->cbuf = cbuf;
        v->offset = off;
        v->size = size;
        v->owner = this;
        vars.push_back(std::move(v));
    }
    void add_array(const char* n, int stride, bool uav, rt_device dev)
    {
        auto a = std::make_unique<rt_array_s>();
        a->name = n;
        a->stride = stride;
        a->uav = uav;
        a->owner = this;
        a->dev = dev;
        arrays.push_back(std::move(a));
    }
    rt_array_s* array(const char* n)
    {
        for (auto& a : arrays)
            if (a->name == n) return a.get();
        return nullptr;
    }
};

struct rt_compute_s {
    rt_device dev = nullptr;
    Shader* shader = nullptr;
    Shader* new_shader = nullptr;
    // camera feed (rt_terrain_render_feed): pinned copy of CameraResults + the event after it
    float4* feed_host = nullptr;
    hipEvent_t feed_ev = nullptr;
    bool feed_pending = false;
    ~rt_compute_s()
    {
        delete shader;
        delete new_shader;
        if (feed_ev) (void)hipEventDestroy(feed_ev);
        if (feed_host) (void)hipHostFree(feed_host);
    }
};

namespace {

float rd_f(const std::vector<uint8_t>& b, int off)
{
    float f;
    memcpy(&f, b.data() + off, 4);
    return f;
}

// Build the constant block from the cbuffer shadows (tracing.hlsl:6-41,
// sky.hlsl:1-16/:74-80, landscape color constants, antialiasing.hlsl:9-49).
void build_consts(const Shader& s, const rt_device_s& dev, RtConsts& k)
{
    memset(&k, 0, sizeof(k));
    const auto& fr = s.cb[CB_FRAME];
    const auto& pm = s.cb[CB_PERM];
    const auto& xt = s.cb[CB_XTWEAK];
    for (int i = 0; i < 4; ++i) k.eye[i] = s.has_cb[CB_FRAME] ? rd_f(fr, 4 * i) : 0.0f;
    // column_major cbuffer packing: HLSL M[r][c] = mem[c*4 + r]
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) k.view_inverse[4 * r + c] = s.has_cb[CB_FRAME] ? rd_f(fr, 16 + 4 * (4 * c + r)) : 0.0f;
    k.screen[0] = s.has_cb[CB_PERM] ? rd_f(pm, 0) : 0.0f;
    k.screen[1] = s.has_cb[CB_PERM] ? rd_f(pm, 4) : 0.0f;
    float proj[16];
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) proj[4 * r + c] = s.has_cb[CB_PERM] ? rd_f(pm, 16 + 4 * (4 * c + r)) : 0.0f;
    k.proj11 = proj[0];
    k.proj22 = proj[5];
    k.rcp_w = rtm::rcp(k.screen[0]);
    k.rcp_h = rtm::rcp(k.screen[1]);
    for (int i = 0; i < 3; ++i) k.sun[i] = s.has_cb[CB_XTWEAK] ? rd_f(xt, 4 * i) : 0.0f;

    k.step_factor = s.recording ? 1.001f : 1.009f;
    k.one_minus_step_factor = (float)(1.0 - (double)k.step_factor);
    k.density_factor = s.recording ? 0.15f : 0.35f;
    k.min_limit = (float)((double)0.02f * (double)0.03f);
    for (int n = 1; n <= RT_NP_OCTAVES; ++n) {
        float S = rtm::pow(1.96f, (float)n);
        k.np_scale[n] = S;
        k.np_scale_y[n] = S * 0.35f;
        k.np_rcp[n] = rtm::rcp(S);
    }
    k.np_expo = 0.68f + 0.1f;
    for (int n = 1; n <= RT_COL_OCTAVES; ++n) {
        float S = rtm::pow(2.03f, (float)n);
        k.col_scale[n] = S;
        k.col_rcp[n] = rtm::rcp(S);
    }
    switch (s.landscape) {
    case RT_TESTING: k.albedo[0] = 0.6f; k.albedo[1] = 0.5f; k.albedo[2] = 0.3f; k.albedo[3] = 0.1f; break;
    case RT_GREENROCKS: k.albedo[0] = 0.6f; k.albedo[1] = 0.7f; k.albedo[2] = 0.3f; k.albedo[3] = 0.1f; break;
    default:
        k.albedo[0] = (float)(193.0 / 255.0);
        k.albedo[1] = (float)(131.0 / 255.0);
        k.albedo[2] = (float)(92.0 / 255.0);
        k.albedo[3] = 0.2f;
        break;
    }
    const float shc[3] = {0.08f, 0.12f, 0.14f};
    for (int i = 0; i < 3; ++i) {
        k.shadow_color[i] = shc[i];
        k.one_minus_shadow[i] = (float)(1.0 - (double)shc[i]);
    }
    k.rcp200 = rtm::rcp(200.0f);

    // sky.hlsl constants (folded in double, rounded once)
    const double wl[3] = {0.650f, 0.570f, 0.475f};
    const double kr = 0.003f, km = 0.0025f, pi = 3.14159265f, eSun = 12.0f;
    float outerRadius = (float)(200.0 * (double)1.025f);
    float fScale = (float)(1.0 / ((double)outerRadius - 200.0));
    float sos = (float)((double)fScale / (double)0.19f);
    float fKrESun = (float)(eSun * kr), fKmESun = (float)(eSun * km);
    float fKr4PI = (float)(kr * 4.0 * pi), fKm4PI = (float)(km * 4.0 * pi);
    for (int i = 0; i < 3; ++i) {
        float wl4 = (float)std::pow(wl[i], 4.0);
        float inv = (float)(1.0 / (double)wl4);
        k.sky_att[i] = (float)((double)inv * (double)fKr4PI + (double)fKm4PI);
        k.sky_mie_k[i] = (float)((double)inv * (double)fKrESun);
    }
    k.sky_km_esun = fKmESun;
    float g = -0.99f, g2 = g * g;
    k.sky_mie_a = (float)(1.5 * ((1.0 - (double)g2) / (2.0 + (double)g2)));
    k.sky_one_plus_g2 = (float)(1.0 + (double)g2);
    k.sky_two_g = (float)(2.0 * (double)g);
    k.sky_rcp_samples = (float)(1.0 / 3.0);
    k.sky_fscale = fScale;
    k.sky_sos = sos;
    // eye-dependent (getRayleighMieColor prologue, sky.hlsl:88-100)
    float camHeight = rtm::fma(k.eye[1], 0.001f, 200.0f);
    camHeight = rtm::max(camHeight, 0.0f);
    k.sky_dist_to_top = outerRadius - camHeight;
    k.sky_start[0] = k.eye[0] * 0.001f;
    k.sky_start[1] = camHeight;
    k.sky_start[2] = k.eye[2] * 0.001f;
    rtm::f3 sn = rtm::normalize(rtm::mk(k.sky_start[0], k.sky_start[1], k.sky_start[2]));
    k.sky_start_n[0] = sn.x;
    k.sky_start_n[1] = sn.y;
    k.sky_start_n[2] = sn.z;
    k.sky_depth0 = rtm::exp(sos * (200.0f - camHeight));

    static const float off1[1][2] = {{0, 0}};
    static const float off2[2][2] = {{4, 4}, {-4, -4}};
    static const float off4[4][2] = {{-2, -6}, {6, -2}, {-6, 2}, {2, 6}};
    static const float off8[8][2] = {{1, -3}, {-1, 3}, {5, 1}, {-3, -5}, {-5, 5}, {-7, -1}, {3, 7}, {7, -7}};
    static const float off16[16][2] = {{1, 1}, {-1, 3}, {-3, 2}, {4, -1}, {-5, -2}, {2, 5}, {5, 3}, {3, -5},
                                       {-2, 6}, {0, -7}, {-4, -6}, {-6, 4}, {-8, 0}, {7, -4}, {6, 7}, {-7, -8}};
    const float(*offs)[2] = off1;
    switch (s.aa) {
    case 2: offs = off2; break;
    case 4: offs = off4; break;
    case 8: offs = off8; break;
    case 16: offs = off16; break;
    default: break;
    }
    for (int a = 0; a < s.aa; ++a) {
        k.aa_off[a][0] = offs[a][0] * (1.0f / 16.0f);
        k.aa_off[a][1] = offs[a][1] * (1.0f / 16.0f);
    }
    k.aa_samples = s.aa;
    k.landscape = s.landscape;
    k.max_steps = s.max_steps;
    k.ao_samples = s.kind == KIND_TRACESCREEN ? s.ao : 0;
    k.width = dev.width;
    k.height = dev.height;
}

int sync_shader(rt_device dev, Shader* s)
{
    if (!s->d_consts) HIP_TRY(hipMalloc(&s->d_consts, sizeof(RtConsts)));
    if (!s->d_grad) HIP_TRY(hipMalloc(&s->d_grad, 128 * sizeof(float4)));
    std::lock_guard<std::mutex> lk(g_cb_mu);
    if (s->cb_dirty) {
        // cbuffer shadows -> device (ConstantBufferD3D::update on run, ShaderVariableDirect3D.cpp:59-66)
        build_consts(*s, *dev, s->host_consts);
        int rc = s->consts_staging.upload(dev->stream, s->d_consts, &s->host_consts, sizeof(RtConsts));
        if (rc) return rc;
        s->cb_dirty = false;
    }
    if (s->grad_dirty) {
        int rc = s->grad_staging.upload(dev->stream, s->d_grad, s->cb[CB_NOISE].data(), 128 * sizeof(float4));
        if (rc) return rc;
        s->grad_dirty = false;
    }
    return RT_OK;
}

// The GPU's host-mapped flag word (one per GPU ordinal, allocated on first use): k_order stores
// RT_FLAG_PREPASS_TIMEOUT there when its bounded wait for a fused prepass gives up, so the frames of
// that batch may be wrong.  Every C-ABI call that launches on or reads from a device of that GPU checks
// it (host_flag_check) and fails with RT_ERR_STATE until rt_device_check clears it: a host that follows
// the reference's call sequence and never calls rt_device_check still cannot read such a frame.
std::mutex g_host_flag_mu;
std::map<int, std::pair<uint32_t*, uint32_t*>> g_host_flags; // ordinal -> (host pointer, device pointer)

uint32_t* host_flag_device(int ordinal)
{
    std::lock_guard<std::mutex> lk(g_host_flag_mu);
    auto it = g_host_flags.find(ordinal);
    if (it != g_host_flags.end()) return it->second.second;
    void* h = nullptr;
    void* dptr = nullptr;
    if (hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return nullptr;
    if (hipHostGetDevicePointer(&dptr, h, 0) != hipSuccess) {
        (void)hipHostFree(h);
        return nullptr;
    }
    std::memset(h, 0, 64);
    g_host_flags[ordinal] = {(uint32_t*)h, (uint32_t*)dptr};
    return (uint32_t*)dptr;
}

uint32_t host_flag_read(int ordinal, bool clear)
{
    std::lock_guard<std::mutex> lk(g_host_flag_mu);
    auto it = g_host_flags.find(ordinal);
    if (it == g_host_flags.end()) return 0;
    volatile uint32_t* w = it->second.first;
    const uint32_t v = *w;
    if (clear) *w = 0;
    return v;
}

int host_flag_check(rt_device d)
{
    if (d && host_flag_read(d->ordinal, false))
        return fail(RT_ERR_STATE, "GPU %d: a k_order wait for a fused prepass timed out; frames traced since may be "
                    "wrong (rt_device_check reports and clears it)", d->ordinal);
    return RT_OK;
}

RtLaunch make_launch(rt_device dev, Shader* s)
{
    RtLaunch a;
    a.stream = dev->stream;
    a.landscape = s->landscape;
    a.consts = s->d_consts;
    a.perm2d = s->textures[0] ? s->textures[0]->data : nullptr;
    a.grad = s->d_grad;
    a.stats = (dev->flags & RT_DEVICE_STATS) ? dev->stats : nullptr;
    a.queue = dev->queue;
    a.num_cus = dev->num_cus - dev->reserve_cus;
    a.samples = dev->samples;
    a.order = dev->order;
    a.hitmask = dev->hitmask;
    a.hitq = dev->hitq;
    a.spill_long = dev->spill_long;
    rt_spill_caps(s->aa, s->ao, &a.hit_cap, &a.long_spill_cap);
    a.cells_from_cam = 0;
    a.small_rings = (dev->flags & RT_DEVICE_DEBUG_SMALL_RINGS) ? 1 : 0;
    a.fit = 0;
    a.fin = dev->fin;
    a.finpool = dev->finpool;
    a.cpool = dev->cpool;
    a.fitm = 0;
    a.aocc = dev->aocc;
    a.ao_samples = s->ao;
    a.aa = s->aa;
    a.frames = dev->table.d;
    a.frames_host = FrameTable{};
    a.n_frames = 1;
    a.after_order = nullptr;
    a.fuse_next = FusedPrepass{nullptr, nullptr, 0u};
    a.wait_ctl = nullptr;
    a.wait_total = 0;
    a.after_order_fuse = nullptr;
    a.host_flag = host_flag_device(dev->ordinal);
    a.gated = GatedPrepass{nullptr, nullptr, 0u, 0u};
    a.packed = 0;
    return a;
}

// a frame table the kernels read (uploaded only when its contents change)
int upload_frames(rt_device dev, rt_device_s::DevTable& t, const FrameTable& ft)
{
    if (!t.d) HIP_TRY(hipMalloc(&t.d, sizeof(FrameTable)));
    if (t.valid && memcmp(&ft, &t.last, sizeof(FrameTable)) == 0) return RT_OK;
    const int rc = t.staging.upload(dev->stream, t.d, &ft, sizeof(FrameTable));
    if (rc) return rc;
    t.last = ft;
    t.valid = true;
    return RT_OK;
}

int check_texture(Shader* s)
{
    rt_texture t = s->textures[0];
    if (!t || !t->data) return fail(RT_ERR_STATE, "texture stage 0 (texPerm2D) not bound");
    if (t->w != 128 || t->h != 128 || t->fmt != RT_FORMAT_R8G8B8A8_UINT)
        return fail(RT_ERR_UNSUPPORTED, "texPerm2D must be a 128x128 R8G8B8A8_UINT texture");
    return RT_OK;
}

// Per-sample buffers: per AA sample of every whole 32x32 tile, one shaded colour (16 B; 12 B used
// with one sample per pixel), the shading inputs of a long shadow ray (48 B; 32 B used without
// fog), an AO occlusion count (1 B) and a hit bit (the 64-lane ballot per 8x8 unit and AA sample).
// Per block (one per CU): k_trace's hit stack (hit records of up to 48 B) and long-ray spill stack
// (48 B records), rt_spill_caps records each, and its fin pool (RT_FIN_SLOTS records of up to 48 B).
int ensure_split_buffers(rt_device dev, int aa, int ao, int n_frames)
{
    uint32_t hcap, lcap;
    rt_spill_caps(aa, ao, &hcap, &lcap);
    const size_t hq_need = (size_t)dev->num_cus * hcap, ls_need = (size_t)dev->num_cus * lcap;
    if (hq_need > dev->hitq_n || ls_need > dev->spill_long_n) {
        HIP_TRY(hipStreamSynchronize(dev->stream));
        if (dev->hitq) HIP_TRY(hipFree(dev->hitq));
        if (dev->spill_long) HIP_TRY(hipFree(dev->spill_long));
        if (dev->finpool) HIP_TRY(hipFree(dev->finpool));
        if (dev->cpool) HIP_TRY(hipFree(dev->cpool));
        dev->cpool = nullptr;
        dev->hitq = nullptr;
        dev->spill_long = nullptr;
        dev->finpool = nullptr;
        dev->hitq_n = dev->spill_long_n = 0;
        HIP_TRY(hipMalloc(&dev->hitq, hq_need * 3 * sizeof(float4)));
        HIP_TRY(hipMalloc(&dev->spill_long, ls_need * 3 * sizeof(float4)));
        HIP_TRY(hipMalloc(&dev->finpool, (size_t)dev->num_cus * RT_FIN_SLOTS * 3 * sizeof(float4)));
        HIP_TRY(hipMalloc(&dev->cpool, (size_t)dev->num_cus * RT_AO_POOL_SLOTS * sizeof(float4)));
        if (!dev->gate) HIP_TRY(hipMalloc(&dev->gate, (size_t)RT_MAX_BATCH * RT_GATE_WORDS * sizeof(uint32_t)));
        dev->hitq_n = hq_need;
        dev->spill_long_n = ls_need;
    }
    size_t need = rt_split_samples(dev->width, dev->height, aa) * (size_t)n_frames;
    if (need <= dev->samples_cap) return RT_OK;
    HIP_TRY(hipStreamSynchronize(dev->stream));
    if (dev->samples) HIP_TRY(hipFree(dev->samples));
    if (dev->order) HIP_TRY(hipFree(dev->order));
    if (dev->hitmask) HIP_TRY(hipFree(dev->hitmask));
    if (dev->fin) HIP_TRY(hipFree(dev->fin));
    if (dev->aocc) HIP_TRY(hipFree(dev->aocc));
    dev->fin = nullptr;
    dev->aocc = nullptr;
    dev->samples = nullptr;
    dev->order = nullptr;
    dev->hitmask = nullptr;
    dev->samples_cap = 0;
    HIP_TRY(hipMalloc(&dev->samples, need * sizeof(float4)));
    HIP_TRY(hipMalloc(&dev->fin, need * 3 * sizeof(float4)));
    // AO counts, a byte per sample (ao_count): zero once here; k_finish clears what it reads
    HIP_TRY(hipMalloc(&dev->aocc, (need + 3) / 4 * sizeof(uint32_t)));
    HIP_TRY(hipMemsetAsync(dev->aocc, 0, (need + 3) / 4 * sizeof(uint32_t), dev->stream));
    HIP_TRY(hipMalloc(&dev->order, rt_split_samples(dev->width, dev->height, 1) / 64 * RT_MAX_BATCH * sizeof(uint32_t)));
    HIP_TRY(hipMalloc(&dev->hitmask, need / 64 * sizeof(uint64_t)));
    if (dev->claims) HIP_TRY(hipFree(dev->claims));
    HIP_TRY(hipMalloc(&dev->claims, rt_split_samples(dev->width, dev->height, 1) / 1024 * RT_MAX_BATCH * sizeof(uint32_t)));
    dev->samples_cap = need;
    return RT_OK;
}

} // namespace

// ===========================================================================
extern "C" {

const char* rt_last_error(void) { return g_err.c_str(); }
int rt_abi_version(void) { return RT_ABI_VERSION; }

int rt_vfs_add_path(const char* path)
{
    if (!path) return fail(RT_ERR_INVALID, "null path");
    std::lock_guard<std::mutex> lk(g_vfs_mu);
    g_vfs.emplace_back(path);
    return RT_OK;
}
int rt_vfs_clear(void)
{
    std::lock_guard<std::mutex> lk(g_vfs_mu);
    g_vfs.clear();
    return RT_OK;
}

// ---- device ---------------------------------------------------------------
// ---- stream ownership ------------------------------------------------------
// A device's own stream may be lent to other devices (rt_device_set_stream: FrameRing's slot
// groups share one stream per batch).  The registry counts the devices using each own stream
// (its owner while alive, plus its borrowers); the stream is destroyed when the count drops to
// zero, so an owner destroyed before its borrowers leaves them a live stream (and nothing
// synchronizes or launches on a destroyed one).  Streams the caller passes in that no device
// created (e.g. a torch stream) are not tracked: the caller keeps them alive.
namespace {
std::mutex g_stream_mu;
std::map<hipStream_t, int> g_stream_refs;

void stream_ref(hipStream_t s)
{
    std::lock_guard<std::mutex> lk(g_stream_mu);
    auto it = g_stream_refs.find(s);
    if (it != g_stream_refs.end()) ++it->second;
}

// drop one reference; the last one destroys the stream (after draining it)
void stream_unref(hipStream_t s)
{
    bool last = false;
    {
        std::lock_guard<std::mutex> lk(g_stream_mu);
        auto it = g_stream_refs.find(s);
        if (it == g_stream_refs.end()) return;
        if (--it->second == 0) {
            g_stream_refs.erase(it);
            last = true;
        }
    }
    if (last) {
        (void)hipStreamSynchronize(s);
        (void)hipStreamDestroy(s);
    }
}

// rt_terrain_prepass_ahead's side stream: one per GPU, shared by every batch on it (the ahead
// prepasses run one after another, like the batches), created on first use and kept for the
// process (devices come and go; the stream carries no state of theirs past its work)
std::map<int, hipStream_t> g_ahead_streams;

// lead devices whose batch is STAGED for fusing, per GPU, oldest first
std::map<int, std::vector<rt_device_s*>> g_fuse_staged;

void fuse_forget(rt_device_s* d)
{
    std::lock_guard<std::mutex> lk(g_stream_mu);
    auto& v = g_fuse_staged[d->ordinal];
    v.erase(std::remove(v.begin(), v.end(), d), v.end());
}

hipStream_t ahead_stream(int ordinal, bool create)
{
    std::lock_guard<std::mutex> lk(g_stream_mu);
    auto it = g_ahead_streams.find(ordinal);
    if (it != g_ahead_streams.end()) return it->second;
    hipStream_t s = nullptr;
    if (!create || hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return nullptr;
    return g_ahead_streams[ordinal] = s;
}
} // namespace

rt_device_s::~rt_device_s()
{
    (void)hipSetDevice(ordinal);
    fuse_forget(this);
    if (fuse_state == FUSE_FUSED && ev_fuser_done) (void)hipEventSynchronize(ev_fuser_done); // it writes our frames
    if (stream) (void)hipStreamSynchronize(stream); // the stream in use is alive: a reference is held
    if (hipStream_t side = ahead_stream(ordinal, false)) (void)hipStreamSynchronize(side); // ahead prepasses
    if (pre_stream) { // rt_terrain_render's prepasses
        (void)hipStreamSynchronize(pre_stream);
        (void)hipStreamDestroy(pre_stream);
    }
    for (auto* c : computes) delete c;              // children die with their device
    for (auto* t : textures) {
        if (t->data) (void)hipFree(t->data);
        delete t;
    }
    for (void* p : {(void*)fb8, (void*)fb32, (void*)stats, (void*)scratch_cam, (void*)queue, (void*)samples,
                    (void*)hitq, (void*)finpool, (void*)cpool, (void*)gate, (void*)claims, (void*)order, (void*)hitmask, (void*)spill_long, (void*)fin, (void*)aocc,
                    (void*)bgrx, (void*)table.d, (void*)pre_table.d, (void*)fuse_table.d, (void*)fctl, (void*)blocks})
        if (p) (void)hipFree(p);
    if (recorder) recorder_detach(recorder); // the recorder outlives its device: it stops capturing
    if (graph_pre.exec) (void)hipGraphExecDestroy(graph_pre.exec);
    if (graph_trace.exec) (void)hipGraphExecDestroy(graph_trace.exec);
    for (hipEvent_t e : {sync_ev, ev_order, ev_ahead, ev_ahead_in, ev_fuser_done, ev_fuse_order, ev_pre})
        if (e) (void)hipEventDestroy(e);
    for (auto& pr : ev_pool) {
        (void)hipEventDestroy(pr.first);
        (void)hipEventDestroy(pr.second);
    }
    if (stream && stream != own_stream) stream_unref(stream); // a borrowed stream
    if (own_stream) stream_unref(own_stream);                 // destroyed here unless lent out
}

int rt_device_create(int ordinal, int width, int height, unsigned flags, rt_device* out)
{
    if (!out || width <= 0 || height <= 0) return fail(RT_ERR_INVALID, "bad device arguments");
    *out = nullptr;
    const unsigned known = RT_DEVICE_FLOAT_OUTPUT | RT_DEVICE_STATS | RT_DEVICE_GRAPH | RT_DEVICE_DEBUG_SMALL_RINGS |
                           RT_DEVICE_DEBUG_WITHHOLD_FUSE | RT_DEVICE_GATED | RT_DEVICE_DEBUG_GATE_STRESS |
                           RT_DEVICE_DEFERRED | RT_DEVICE_DEBUG_DEFER_SMALL;
    if (flags & ~known) return fail(RT_ERR_INVALID, "unknown device flags 0x%x (8 and 16 were retired in ABI 6)", flags & ~known);
    int n = 0;
    HIP_TRY(hipGetDeviceCount(&n));
    if (ordinal < 0 || ordinal >= n) return fail(RT_ERR_INVALID, "GPU ordinal %d out of range (%d devices)", ordinal, n);
    HIP_TRY(hipSetDevice(ordinal));
    // from here on every early return frees what was made (the destructor)
    auto d = std::make_unique<rt_device_s>();
    d->ordinal = ordinal;
    d->width = width;
    d->height = height;
    d->flags = flags;
    HIP_TRY(hipStreamCreateWithFlags(&d->own_stream, hipStreamNonBlocking));
    {
        std::lock_guard<std::mutex> lk(g_stream_mu);
        g_stream_refs[d->own_stream] = 1;
    }
    d->stream = d->own_stream;
    HIP_TRY(hipMalloc(&d->fb8, (size_t)width * height * 4));
    HIP_TRY(hipMemset(d->fb8, 0, (size_t)width * height * 4));
    if (flags & RT_DEVICE_FLOAT_OUTPUT) {
        HIP_TRY(hipMalloc(&d->fb32, (size_t)width * height * 16));
        HIP_TRY(hipMemset(d->fb32, 0, (size_t)width * height * 16));
    }
    HIP_TRY(hipMalloc(&d->stats, sizeof(RtStats)));
    HIP_TRY(hipMemset(d->stats, 0, sizeof(RtStats)));
    HIP_TRY(hipMalloc(&d->scratch_cam, 1024 * sizeof(float4)));
    HIP_TRY(hipMalloc(&d->queue, RT_QUEUE_BYTES));
    HIP_TRY(hipMemset(d->queue, 0, RT_QUEUE_BYTES)); // the counters are reset per launch, the flags here
    HIP_TRY(hipMalloc(&d->fctl, 16));
    HIP_TRY(hipMemset(d->fctl, 0, 16));
    HIP_TRY(hipDeviceGetAttribute(&d->num_cus, hipDeviceAttributeMultiprocessorCount, ordinal));
    *out = d.release();
    return RT_OK;
}

void rt_device_destroy(rt_device d)
{
    if (d) (void)defer_flush(d); // a pending frame is traced (the destructor then drains the stream)
    delete d;
}

int rt_stream_refs(void* hip_stream)
{
    std::lock_guard<std::mutex> lk(g_stream_mu);
    auto it = g_stream_refs.find((hipStream_t)hip_stream);
    return it == g_stream_refs.end() ? 0 : it->second;
}

int rt_device_present(rt_device d)
{
    if (!d) return fail(RT_ERR_INVALID, "null device");
    HIP_TRY(hipGetLastError());
    if (int rc = host_flag_check(d)) return rc;
    // DeviceDirect3D.cpp:242-256: while recording, the frame goes to the recorder
    if (d->recorder && rt_recorder_is_recording(d->recorder) == 1) {
        if (int rc = defer_flush(d)) return rc;
        return recorder_capture(d->recorder);
    }
    return RT_OK;
}

int rt_device_flush(rt_device d)
{
    if (!d) return fail(RT_ERR_INVALID, "null device");
    // HIP submits at launch; flush launches a deferred frame (RT_DEVICE_DEFERRED) and surfaces asynchronous
    // launch errors.
    if (int rc = defer_flush(d)) return rc;
    HIP_TRY(hipGetLastError());
    return RT_OK;
}

int rt_device_synchronize(rt_device d)
{
    if (!d) return fail(RT_ERR_INVALID, "null device");
    if (int rc = defer_flush(d)) return rc;
    HIP_TRY(hipStreamSynchronize(d->stream));
    return host_flag_check(d);
}

int rt_device_readback(rt_device d, void* dst, size_t row_pitch)
{
    if (!d || !dst) return fail(RT_ERR_INVALID, "bad readback arguments");
    if (row_pitch == 0) row_pitch = (size_t)d->width * 4;
    if (row_pitch < (size_t)d->width * 4) return fail(RT_ERR_INVALID, "row pitch smaller than a row");
    if (int rc = defer_flush(d)) return rc;
    HIP_TRY(hipMemcpy2DAsync(dst, row_pitch, d->fb8, (size_t)d->width * 4, (size_t)d->width * 4, d->height,
                             hipMemcpyDeviceToHost, d->stream));
    HIP_TRY(hipStreamSynchronize(d->stream));
    return host_flag_check(d);
}

// GPU swizzle into the device BGRX buffer (rt_launch_bgrx), on the device stream
static int device_bgrx(rt_device d)
{
    if (!d->bgrx) HIP_TRY(hipMalloc(&d->bgrx, (size_t)d->width * d->height * 4));
    rt_launch_bgrx(d->stream, d->fb8, d->bgrx, d->width, d->height, d->width);
    HIP_TRY(hipGetLastError());
    return RT_OK;
}

int rt_device_readback_bgrx(rt_device d, void* dst, size_t row_pitch)
{
    if (!d || !dst) return fail(RT_ERR_INVALID, "bad readback arguments");
    if (row_pitch == 0) row_pitch = (size_t)d->width * 4;
    if (row_pitch < (size_t)d->width * 4) return fail(RT_ERR_INVALID, "row pitch smaller than a row");
    if (int rc = defer_flush(d)) return rc;
    if (int rc = device_bgrx(d)) return rc;
    HIP_TRY(hipMemcpy2DAsync(dst, row_pitch, d->bgrx, (size_t)d->width * 4, (size_t)d->width * 4, d->height,
                             hipMemcpyDeviceToHost, d->stream));
    HIP_TRY(hipStreamSynchronize(d->stream));
    return host_flag_check(d);
}

int rt_device_readback_float(rt_device d, float* dst)
{
    if (!d || !dst) return fail(RT_ERR_INVALID, "bad readback arguments");
    if (!d->fb32) return fail(RT_ERR_STATE, "device created without RT_DEVICE_FLOAT_OUTPUT");
    if (int rc = defer_flush(d)) return rc;
    HIP_TRY(hipMemcpyAsync(dst, d->fb32, (size_t)d->width * d->height * 16, hipMemcpyDeviceToHost, d->stream));
    HIP_TRY(hipStreamSynchronize(d->stream));
    return host_flag_check(d);
}

int rt_device_size(rt_device d, int* w, int* h)
{
    if (!d) return fail(RT_ERR_INVALID, "null device");
    if (w) *w = d->width;
    if (h) *h = d->height;
    return RT_OK;
}

// (the caller reads or enqueues behind the frame: a deferred one is launched first)
void* rt_device_framebuffer(rt_device d)
{
    if (!d || defer_flush(d)) return nullptr;
    return (void*)d->fb8;
}
void* rt_device_stream(rt_device d)
{
    if (!d || defer_flush(d)) return nullptr;
    return (void*)d->stream;
}

int rt_device_set_stream(rt_device d, void* s)
{
    if (!d) return fail(RT_ERR_INVALID, "null device");
    hipStream_t want = s ? (hipStream_t)s : d->own_stream;
    if (want == d->stream) return RT_OK;
    if (int rc = defer_flush(d)) return rc; // a pending frame goes on the stream it was queued behind
    if (want != d->own_stream) stream_ref(want);             // borrow (tracked if another device owns it)
    if (d->stream != d->own_stream) stream_unref(d->stream); // return the previous loan
    d->stream = want;
    d->serial_ok = false;
    return RT_OK;
}

int rt_device_stats_sized(rt_device d, rt_stats* out, size_t size, int reset)
{
    if (!d || !out) return fail(RT_ERR_INVALID, "bad arguments");
    if (int rc = defer_flush(d)) return rc;
    RtStats h;
    HIP_TRY(hipMemcpyAsync(&h, d->stats, sizeof(h), hipMemcpyDeviceToHost, d->stream));
    HIP_TRY(hipStreamSynchronize(d->stream));
    rt_stats v{};
    v.primary_steps = h.primary_steps;
    v.shadow_steps = h.shadow_steps;
    v.prepass_steps = h.prepass_steps;
    v.hits = h.hits;
    v.noise_calls = h.noise_calls;
    v.ao_steps = h.ao_steps;
    v.noise_wave_iters = h.noise_waves;
    std::memcpy(out, &v, size < sizeof(v) ? size : sizeof(v));
    if (reset) HIP_TRY(hipMemsetAsync(d->stats, 0, sizeof(RtStats), d->stream));
    return RT_OK;
}

int rt_device_stats(rt_device d, rt_stats* out, int reset) { return rt_device_stats_sized(d, out, sizeof(rt_stats), reset); }

int rt_device_set_profiling(rt_device d, int enable)
{
    if (!d) return fail(RT_ERR_INVALID, "null device");
    d->profiling = enable != 0;
    return RT_OK;
}

int rt_device_kernel_time(rt_device d, double* total_ms, int* launches)
{
    if (!d) return fail(RT_ERR_INVALID, "null device");
    if (int rc = defer_flush(d)) return rc;
    HIP_TRY(hipStreamSynchronize(d->stream));
    double tot = 0.0;
    for (size_t i = 0; i < d->ev_used; ++i) {
        float ms = 0.0f;
        HIP_TRY(hipEventElapsedTime(&ms, d->ev_pool[i].first, d->ev_pool[i].second));
        tot += ms;
    }
    if (total_ms) *total_ms = tot;
    if (launches) *launches = (int)d->ev_used;
    d->ev_used = 0;
    return RT_OK;
}

int rt_debug_spin(void* hip_stream, const unsigned long long* base_device, unsigned long long until_ticks,
                  unsigned long long ticks, unsigned long long* stamp_device)
{
    rt_launch_debug_spin((hipStream_t)hip_stream, base_device, until_ticks, ticks, stamp_device);
    HIP_TRY(hipGetLastError());
    return RT_OK;
}

int rt_device_info(rt_device d, int key, unsigned long long* out)
{
    if (!d || !out) return fail(RT_ERR_INVALID, "bad arguments");
    switch (key) {
    case RT_INFO_GATED_LAUNCHES: *out = d->gated_launches; return RT_OK;
    case RT_INFO_PREPASS_LAUNCHES: *out = d->prepass_launches; return RT_OK;
    case RT_INFO_PRESTREAM_RENDERS: *out = d->prestream_renders; return RT_OK;
    case RT_INFO_DEFERRED_FUSED: *out = d->deferred_fused; return RT_OK;
    default: return fail(RT_ERR_INVALID, "unknown rt_device_info key %d", key);
    }
}

int rt_device_reserve_cus(rt_device d, int n)
{
    if (!d) return fail(RT_ERR_INVALID, "null device");
    if (n < 0 || n >= d->num_cus) return fail(RT_ERR_INVALID, "reserve 0..%d CUs, not %d", d->num_cus - 1, n);
    d->reserve_cus = n;
    return RT_OK;
}

int rt_debug_defer_slot(rt_device d, int slot, void** fb8, void** camera_results, void** cell_distance)
{
    if (!d || slot < 0 || slot >= (int)d->slots.size() || !d->slots[slot]->cam) return fail(RT_ERR_INVALID, "no frame slot %d", slot);
    if (int rc = defer_flush(d)) return rc;
    const rt_device_s::FrameSlot& f = *d->slots[slot];
    if (fb8) *fb8 = f.fb8;
    if (camera_results) *camera_results = f.cam;
    if (cell_distance) *cell_distance = f.cells;
    return RT_OK;
}

int rt_device_defer_batch(rt_device d, int frames)
{
    if (!d) return fail(RT_ERR_INVALID, "null device");
    if (frames < 1 || frames > 4) return fail(RT_ERR_INVALID, "1..4 frames per deferred launch, not %d", frames);
    if (!(d->flags & RT_DEVICE_DEFERRED)) return fail(RT_ERR_STATE, "rt_device_defer_batch needs RT_DEVICE_DEFERRED");
    if (frames == d->defer_k) return RT_OK;
    if (int rc = defer_flush(d)) return rc;
    d->defer_k = frames;
    d->slot_next = 0;
    return RT_OK;
}

int rt_device_graph_info(rt_device d, unsigned long long* captures, unsigned long long* launches)
{
    if (!d) return fail(RT_ERR_INVALID, "null device");
    if (captures) *captures = d->graph_captures;
    if (launches) *launches = d->graph_launches;
    return RT_OK;
}

// ---- textures -------------------------------------------------------------
int rt_device_wait_event(rt_device d, void* ev)
{
    if (!d || !ev) return fail(RT_ERR_INVALID, "null device or event");
    if (int rc = defer_flush(d)) return rc; // a pending frame was asked for before the caller's event
    HIP_TRY(hipSetDevice(d->ordinal));
    HIP_TRY(hipStreamWaitEvent(d->stream, (hipEvent_t)ev, 0));
    // every later launch waits for the caller's event, the prepass-stream prepass of rt_terrain_render
    // included: the next render prepasses in line on d->stream (which now waits), so it neither reads
    // inputs the caller is still writing nor overwrites CameraResults the caller's stream still reads
    d->serial_ok = false;
    return RT_OK;
}

int rt_device_record_event(rt_device d, void* ev)
{
    if (!d || !ev) return fail(RT_ERR_INVALID, "null device or event");
    if (int rc = defer_flush(d)) return rc;
    HIP_TRY(hipSetDevice(d->ordinal));
    HIP_TRY(hipEventRecord((hipEvent_t)ev, d->stream));
    return RT_OK;
}

int rt_device_check(rt_device d)
{
    if (!d) return fail(RT_ERR_INVALID, "null device");
    if (int rc = defer_flush(d)) return rc;
    HIP_TRY(hipSetDevice(d->ordinal));
    HIP_TRY(hipStreamSynchronize(d->stream));
    uint32_t flags = 0;
    HIP_TRY(hipMemcpy(&flags, reinterpret_cast<char*>(d->queue) + RT_CTR_BYTES, 4, hipMemcpyDeviceToHost));
    flags |= host_flag_read(d->ordinal, true); // the GPU's fail-safe word (a timeout on another device's batch)
    if (!flags) return RT_OK;
    HIP_TRY(hipMemset(reinterpret_cast<char*>(d->queue) + RT_CTR_BYTES, 0, 4));
    return fail(RT_ERR_STATE, "device flags 0x%x:%s%s%s", flags,
                (flags & RT_FLAG_HIT_OVERFLOW) ? " k_trace hit stack overflow (a push past rt_spill_caps' bound was dropped)" : "",
                (flags & RT_FLAG_SPILL_OVERFLOW) ? " k_trace long-ray spill stack overflow" : "",
                (flags & RT_FLAG_PREPASS_TIMEOUT) ? " k_order timed out waiting for a fused prepass" : "");
}

int rt_texture_create(rt_device d, rt_texture* out)
{
    if (!d || !out) return fail(RT_ERR_INVALID, "bad arguments");
    auto t = new rt_texture_s();
    t->dev = d;
    d->textures.push_back(t);
    *out = t;
    return RT_OK;
}

int rt_texture_init(rt_texture t, int dims, int fmt, int w, int h, const void* data, int binding, int cpu)
{
    (void)binding;
    (void)cpu;
    if (!t || !data || w <= 0) return fail(RT_ERR_INVALID, "bad texture arguments");
    if (int rc = defer_flush(t->dev)) return rc; // a pending frame reads the texels it replaces
    if (dims != RT_TEXTURE_2D) return fail(RT_ERR_UNSUPPORTED, "only 2D textures are used on the hot path");
    if (fmt == RT_FORMAT_UNKNOWN) return fail(RT_ERR_UNSUPPORTED, "unknown texture format");
    if (t->data) HIP_TRY(hipFree(t->data));
    size_t bytes = (size_t)w * h * 4;
    HIP_TRY(hipMalloc(&t->data, bytes));
    HIP_TRY(hipMemcpy(t->data, data, bytes, hipMemcpyHostToDevice));
    uint64_t hsh = 0xcbf29ce484222325ull;
    for (size_t i = 0; i < bytes; ++i) hsh = (hsh ^ ((const uint8_t*)data)[i]) * 0x100000001b3ull;
    t->hash = hsh;
    t->dims = dims;
    t->fmt = fmt;
    t->w = w;
    t->h = h;
    return RT_OK;
}

void rt_texture_destroy(rt_texture t)
{
    if (!t) return;
    (void)defer_flush(t->dev);
    auto& v = t->dev->textures;
    v.erase(std::remove(v.begin(), v.end(), t), v.end());
    if (t->data) (void)hipFree(t->data);
    delete t;
}

// ---- compute --------------------------------------------------------------
int rt_compute_create(rt_device d, rt_compute* out)
{
    if (!d || !out) return fail(RT_ERR_INVALID, "bad arguments");
    auto c = new rt_compute_s();
    c->dev = d;
    d->computes.push_back(c);
    *out = c;
    return RT_OK;
}

void rt_compute_destroy(rt_compute c)
{
    if (!c) return;
    (void)defer_flush(c->dev);
    (void)hipStreamSynchronize(c->dev->stream);
    auto& v = c->dev->computes;
    v.erase(std::remove(v.begin(), v.end(), c), v.end());
    delete c;
}

int rt_compute_load(rt_compute c, const char* directory, const char* file, const char* entry, int tx, int ty, int tz,
                    const char* const* mn, const char* const* mv, int n)
{
    (void)directory;
    if (!c || !file) return fail(RT_ERR_INVALID, "bad arguments");
    varmgr_clear(); // ComputeDirect3D.cpp:408: every create clears the live-tweak registry (and tells the client)
    if (entry && strcmp(entry, "CSMain") != 0) return fail(RT_ERR_NOT_FOUND, "entry point %s not found", entry);
    std::string f = file;
    int kind;
    if (f == "tracescreen.hlsl") kind = KIND_TRACESCREEN;
    else if (f == "camerarays.hlsl") kind = KIND_CAMERARAYS;
    else return fail(RT_ERR_NOT_FOUND, "shader file %s not found", file);
    int land = landscape_from_vfs();
    if (land == -2) return fail(RT_ERR_NOT_FOUND, "benchmark landscape does not compile (terrain.hlsl:39-40)");
    if (tx <= 0 || ty <= 0 || tz <= 0 || tx * ty * tz > 1024)
        return fail(RT_ERR_INVALID, "thread group %dx%dx%d exceeds 1024 threads", tx, ty, tz);
    auto s = std::make_unique<Shader>();
    s->kind = kind;
    s->landscape = land;
    s->tx = tx;
    s->ty = ty;
    s->tz = tz;
    for (int i = 0; i < n; ++i) {
        if (!mn || !mv || !mn[i] || !mv[i]) continue;
        std::string k = mn[i], v = mv[i];
        if (k == "RECORDING") s->recording = atoi(v.c_str()) != 0;
        else if (k == "AA_SAMPLES") {
            int aa = atoi(v.c_str());
            if (aa != 1 && aa != 2 && aa != 4 && aa != 8 && aa != 16)
                return fail(RT_ERR_INVALID, "Unsupported AA sample count (antialiasing.hlsl:47)");
            s->aa = aa;
        } else if (k == "RT_MAX_STEPS") s->max_steps = std::max(0, atoi(v.c_str()));
        else if (k == "RT_AO_SAMPLES") {
            int ao = atoi(v.c_str());
            if (ao < 0 || ao > 16) return fail(RT_ERR_INVALID, "RT_AO_SAMPLES must be 0..16");
            s->ao = ao;
        }
    }
    // Reflection (what fxc reports for these shaders; tracing.hlsl:6-22, noise.hlsl:130-133,
    // tracescreen.hlsl:8-14, camerarays.hlsl:3).
    if (kind == KIND_TRACESCREEN) {
        s->has_cb[CB_XTWEAK] = s->has_cb[CB_FRAME] = s->has_cb[CB_PERM] = s->has_cb[CB_NOISE] = s->has_cb[CB_DISPATCH] = true;
        s->add_var("SunDirection", CB_XTWEAK, 0, 12);
        s->add_var("ThreadOffset", CB_DISPATCH, 0, 8);
        s->add_array("CellDistance", 8, false, c->dev);
    } else {
        s->has_cb[CB_FRAME] = s->has_cb[CB_PERM] = s->has_cb[CB_NOISE] = true;
        s->add_array("CameraResults", 16, true, c->dev);
    }
    s->add_var("Eye", CB_FRAME, 0, 16);
    s->add_var("ViewInverse", CB_FRAME, 16, 64);
    s->add_var("Time", CB_FRAME, 80, 4);
    s->add_var("ScreenSize", CB_PERM, 0, 8);
    s->add_var("Projection", CB_PERM, 16, 64);
    s->add_var("permGradients", CB_NOISE, 0, 2048);
    for (int i = 0; i < CB_COUNT; ++i)
        if (s->has_cb[i]) s->cb[i].assign(kCbSize[i], 0); // ConstantBufferD3D zero-fills (ShaderVariableDirect3D.cpp:10-11)
    varmgr_register(s.get()); // ComputeDirect3D.cpp:188-197: variables of 'X' cbuffers
    delete c->new_shader;
    c->new_shader = s.release();
    return RT_OK;
}

int rt_compute_swap(rt_compute c)
{
    if (!c) return fail(RT_ERR_INVALID, "null compute");
    if (!c->new_shader) return 0;
    if (int rc = defer_flush(c->dev)) return rc;
    if (c->shader) {
        (void)hipStreamSynchronize(c->dev->stream); // kernels may still read the old shader's buffers
        delete c->shader;
    }
    c->shader = c->new_shader;
    c->new_shader = nullptr;
    return 1;
}

int rt_compute_thread_size(rt_compute c, int* x, int* y, int* z)
{
    if (!c) return fail(RT_ERR_INVALID, "null compute");
    Shader* s = c->shader ? c->shader : c->new_shader;
    if (!s) return fail(RT_ERR_STATE, "no shader");
    if (x) *x = s->tx;
    if (y) *y = s->ty;
    if (z) *z = s->tz;
    return RT_OK;
}

rt_variable rt_compute_get_variable(rt_compute c, const char* name)
{
    if (!c || !c->shader || !name) return nullptr;
    for (auto& v : c->shader->vars)
        if (v->name == name) return v.get();
    return nullptr;
}

rt_array rt_compute_get_array(rt_compute c, const char* name)
{
    if (!c || !c->shader || !name) return nullptr;
    return c->shader->array(name);
}

void* rt_compute_get_buffer(rt_compute c, const char* name)
{
    (void)c;
    (void)name;
    return nullptr; // ComputeDirect3D.cpp:138-141: CBuffer == 0 masks every resource out
}

int rt_compute_set_texture(rt_compute c, int stage, rt_texture t)
{
    if (!c || stage < 0 || stage >= 16) return fail(RT_ERR_INVALID, "bad arguments");
    if (!c->shader) return fail(RT_ERR_STATE, "no current shader");
    if (c->shader->textures[stage] != t)
        if (int rc = defer_flush(c->dev)) return rc;
    c->shader->textures[stage] = t;
    return RT_OK;
}

int rt_compute_run(rt_compute c, unsigned dx, unsigned dy, unsigned dz)
{
    if (!c) return fail(RT_ERR_INVALID, "null compute");
    Shader* s = c->shader;
    if (!s) return RT_OK; // ComputeDirect3D.cpp:532
    rt_device dev = c->dev;
    int rc = host_flag_check(dev);
    if (rc) return rc;
    if ((rc = defer_flush(dev))) return rc;
    dev->serial_ok = false; // a dispatch of its own (reads / writes the arrays on the stream)
    rc = check_texture(s);
    if (rc) return rc;
    rc = sync_shader(dev, s);
    if (rc) return rc;
    if (s->kind == KIND_TRACESCREEN && (rc = ensure_split_buffers(dev, s->aa, s->ao, 1))) return rc;
    RtLaunch a = make_launch(dev, s);
    if (dz == 0) return RT_OK;
    if (s->kind == KIND_CAMERARAYS) {
        rt_array_s* cr = s->array("CameraResults");
        if (!cr->dev_ptr || cr->elements < 1024) return fail(RT_ERR_STATE, "CameraResults not created with 1024 elements");
        uint32_t ex = std::min<uint64_t>((uint64_t)dx * s->tx, RT_CAMERA_RES);
        uint32_t ey = std::min<uint64_t>((uint64_t)dy * s->ty, RT_CAMERA_RES);
        if (ex == RT_CAMERA_RES && ey == RT_CAMERA_RES) {
            rt_launch_camerarays(a, (float4*)cr->dev_ptr);
        } else {
            // partial prepass dispatch: trace into scratch, copy the covered cells
            rt_launch_camerarays(a, dev->scratch_cam);
            HIP_TRY(hipMemcpy2DAsync(cr->dev_ptr, RT_CAMERA_RES * 16, dev->scratch_cam, RT_CAMERA_RES * 16, ex * 16, ey,
                                     hipMemcpyDeviceToDevice, dev->stream));
        }
    } else {
        rt_array_s* cd = s->array("CellDistance");
        if (!cd->dev_ptr || cd->elements < 1024) return fail(RT_ERR_STATE, "CellDistance not created with 1024 elements");
        uint32_t off[2];
        memcpy(off, s->cb[CB_DISPATCH].data(), 8);
        uint64_t ex = (uint64_t)dx * s->tx, ey = (uint64_t)dy * s->ty;
        ex = std::min<uint64_t>(ex, dev->width > (int)off[0] ? dev->width - off[0] : 0);
        ey = std::min<uint64_t>(ey, dev->height > (int)off[1] ? dev->height - off[1] : 0);
        FrameTable ft{};
        ft.k[0] = s->d_consts;
        ft.cells[0] = (float2*)cd->dev_ptr;
        ft.out8[0] = dev->fb8;
        ft.out32[0] = dev->fb32;
        if ((rc = upload_frames(dev, dev->table, ft))) return rc;
        a.frames = dev->table.d;
        a.frames_host = ft;
        KernelTimer kt(dev);
        rt_launch_tracescreen(a, off[0], off[1], (uint32_t)ex, (uint32_t)ey, 0, 1);
    }
    HIP_TRY(hipGetLastError());
    return RT_OK;
}

// ---- variables / arrays ---------------------------------------------------
int rt_variable_write(rt_variable v, const void* data)
{
    if (!v || !data) return fail(RT_ERR_INVALID, "bad arguments");
    Shader* s = v->owner;
    std::lock_guard<std::mutex> lk(g_cb_mu);
    uint8_t* dst = s->cb[v->cbuf].data() + v->offset;
    if (!memcmp(dst, data, v->size)) return RT_OK; // unchanged: no upload (and an ahead prepass stays current)
    memcpy(dst, data, v->size);
    if (v->cbuf != CB_DISPATCH) s->cb_dirty = true; // ThreadOffset is a launch argument
    if (v->cbuf == CB_NOISE) s->grad_dirty = true;
    return RT_OK;
}
size_t rt_variable_size(rt_variable v) { return v ? (size_t)v->size : 0; }
const char* rt_variable_name(rt_variable v) { return v ? v->name.c_str() : nullptr; }

int rt_array_create(rt_array a, unsigned elements)
{
    if (!a || elements == 0) return fail(RT_ERR_INVALID, "bad arguments");
    if (a->dev_ptr) return fail(RT_ERR_STATE, "array %s already created", a->name.c_str()); // UAVBufferD3D::create
    size_t bytes = (size_t)elements * a->stride;
    HIP_TRY(hipMalloc(&a->dev_ptr, bytes));
    HIP_TRY(hipMemset(a->dev_ptr, 0, bytes));
    a->elements = elements;
    if (a->uav) a->host.assign(bytes, 0);
    return RT_OK;
}

void* rt_array_map(rt_array a)
{
    if (!a) {
        fail(RT_ERR_INVALID, "null array");
        return nullptr;
    }
    if (!a->uav) {
        fail(RT_ERR_UNSUPPORTED, "map not supported on SRV array %s", a->name.c_str());
        return nullptr;
    }
    if (!a->dev_ptr) {
        fail(RT_ERR_STATE, "array %s not created", a->name.c_str());
        return nullptr;
    }
    if (defer_flush(a->dev)) return nullptr;
    hipStream_t s = a->dev->stream;
    if (ahead_wait(a->dev, s) != 0 ||
        hipMemcpyAsync(a->host.data(), a->dev_ptr, a->host.size(), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
        fail(RT_ERR_HIP, "map readback failed");
        return nullptr;
    }
    if (host_flag_check(a->dev)) return nullptr;
    return a->host.data();
}

int rt_array_unmap(rt_array a)
{
    if (!a) return fail(RT_ERR_INVALID, "null array");
    if (!a->uav) return fail(RT_ERR_UNSUPPORTED, "unmap not supported on SRV array %s", a->name.c_str());
    if (!a->dev_ptr) return fail(RT_ERR_STATE, "array not created");
    if (int rc = defer_flush(a->dev)) return rc;
    a->dev->serial_ok = false; // the upload is ordered on the stream only: the next render prepasses in line
    return a->staging.upload(a->dev->stream, a->dev_ptr, a->host.data(), a->host.size());
}

int rt_array_write(rt_array a, const void* data)
{
    if (!a || !data) return fail(RT_ERR_INVALID, "bad arguments");
    if (a->uav) return fail(RT_ERR_UNSUPPORTED, "write not supported on UAV array %s", a->name.c_str());
    if (!a->dev_ptr) return fail(RT_ERR_STATE, "array %s not created", a->name.c_str());
    if (int rc = defer_flush(a->dev)) return rc;
    a->dev->serial_ok = false;
    return a->staging.upload(a->dev->stream, a->dev_ptr, data, (size_t)a->elements * a->stride);
}

size_t rt_array_stride(rt_array a) { return a ? (size_t)a->stride : 0; }
void* rt_array_device_pointer(rt_array a) // (the caller reads it behind the frame: a deferred one is launched first)
{
    if (!a || defer_flush(a->dev)) return nullptr;
    return a->dev_ptr;
}

// ---- Terrain::render on the device -------------------------------------------
// PH_STAGE (rt_terrain_prepass_ahead, fused): upload the camerarays constants and the frame table a
// fusing k_trace reads, launch nothing.  PH_KEEP (with PH_TRACE; RT_DEVICE_DEFERRED): upload no constant
// block -- the frame's went up when it was rendered, and the host copies may hold the next frame's since
enum { PH_PRE = 1, PH_TRACE = 2, PH_STAGE = 4, PH_KEEP = 8 };
// the tracescreen launch's fused-prepass roles (FusedPrepass): the next batch's prepass it runs, and
// the wait of its k_order for this batch's prepass that the previous k_trace ran
struct TraceFuse {
    FusedPrepass next{nullptr, nullptr, 0u};
    hipEvent_t next_after_order = nullptr; // recorded after this launch's k_order (it zeroes next.ctl)
    const uint32_t* wait_ctl = nullptr;
    uint32_t wait_total = 0;
};
static int terrain_render_batch(const rt_compute* cams, const rt_compute* scrs, int n, int shard_rank,
                                int shard_count, bool feed, int phases = PH_PRE | PH_TRACE, int first = 0,
                                int count = -1, float4* camera_out = nullptr, const float4* camera_in = nullptr,
                                const TraceFuse* fuse = nullptr, uint8_t* packed_dst = nullptr,
                                size_t packed_stride = 0);

// Terrain::render (Terrain.cpp:105-136), one frame per call on the device's stream.  Frame i+1's
// camerarays prepass needs only frame i's k_order to be done (the last reader of CameraResults): on the
// device's own prepass stream it waits for that k_order (ev_order, recorded between k_order and k_trace)
// and so runs in frame i's trace tail, where the persistent k_trace's blocks retire, instead of after
// the whole frame; the trace waits for it (ev_pre).  Same launches, same bits.  The first frame, and a
// frame after anything else read this device's CameraResults on its stream (a feed render, an ahead or
// fused prepass, a batch), prepass in line; so do the instrumented, graph and gated devices.
static int deferred_render(rt_device d, rt_compute cam, rt_compute scr, int shard_rank, int shard_count);
static int serial_render(rt_device d, rt_compute cam, rt_compute scr, int shard_rank, int shard_count);

int rt_terrain_render(rt_compute cam, rt_compute scr, int shard_rank, int shard_count)
{
    rt_device d = (cam && scr && scr->dev && cam->dev == scr->dev) ? scr->dev : nullptr;
    if (d && (d->flags & RT_DEVICE_DEFERRED)) return deferred_render(d, cam, scr, shard_rank, shard_count);
    return serial_render(d, cam, scr, shard_rank, shard_count);
}

static int serial_render(rt_device d, rt_compute cam, rt_compute scr, int shard_rank, int shard_count)
{
    const bool plain = d && !(d->flags & (RT_DEVICE_GRAPH | RT_DEVICE_STATS | RT_DEVICE_GATED)) && d->stream &&
                       !d->ahead_pending && !d->ahead_in_pending && d->fuse_state == rt_device_s::FUSE_NONE;
    if (!plain) {
        if (d) d->serial_ok = false;
        return terrain_render_batch(&cam, &scr, 1, shard_rank, shard_count, false);
    }
    if (int rc0 = host_flag_check(d)) return rc0;
    HIP_TRY(hipSetDevice(d->ordinal));
    if (!d->ev_order) HIP_TRY(hipEventCreateWithFlags(&d->ev_order, hipEventDisableTiming));
    if (!(d->serial_ok && d->order_recorded)) {
        int rc = terrain_render_batch(&cam, &scr, 1, shard_rank, shard_count, false); // records ev_order
        d->serial_ok = rc == RT_OK;
        return rc;
    }
    if (!d->pre_stream) HIP_TRY(hipStreamCreateWithFlags(&d->pre_stream, hipStreamNonBlocking));
    if (!d->ev_pre) HIP_TRY(hipEventCreateWithFlags(&d->ev_pre, hipEventDisableTiming));
    HIP_TRY(hipStreamWaitEvent(d->pre_stream, d->ev_order, 0));
    hipStream_t main = d->stream;
    d->stream = d->pre_stream; // the prepass-only call uploads the camerarays constants and launches there
    int rc = terrain_render_batch(&cam, &scr, 1, 0, 1, false, PH_PRE);
    d->stream = main;
    if (rc) {
        d->serial_ok = false;
        return rc;
    }
    HIP_TRY(hipEventRecord(d->ev_pre, d->pre_stream));
    HIP_TRY(hipStreamWaitEvent(main, d->ev_pre, 0));
    rc = terrain_render_batch(&cam, &scr, 1, shard_rank, shard_count, false, PH_TRACE);
    d->serial_ok = rc == RT_OK;
    if (rc == RT_OK) { // a render with a prepass launch (rt_device_info), on the prepass stream
        ++d->prepass_launches;
        ++d->prestream_renders;
    }
    return rc;
}

int rt_terrain_render_feed(rt_compute cam, rt_compute scr, int shard_rank, int shard_count)
{
    if (cam && cam->dev) cam->dev->serial_ok = false; // its CameraResults copy follows the prepass
    return terrain_render_batch(&cam, &scr, 1, shard_rank, shard_count, true);
}

int rt_terrain_feed_wait(rt_compute cam, float* camera_results)
{
    if (!cam || !camera_results) return fail(RT_ERR_INVALID, "bad arguments");
    if (!cam->feed_pending) return fail(RT_ERR_STATE, "no camera feed pending (rt_terrain_render_feed)");
    HIP_TRY(hipEventSynchronize(cam->feed_ev));
    memcpy(camera_results, cam->feed_host, 1024 * sizeof(float4));
    cam->feed_pending = false;
    return RT_OK;
}

extern "C++" {
namespace {
// every value a captured launch bakes in: pointers, sizes and modes
void key_launch(std::vector<uint64_t>& k, const RtLaunch& a)
{
    const uint64_t v[] = {(uint64_t)(uintptr_t)a.stream, (uint64_t)a.landscape, (uint64_t)(uintptr_t)a.consts,
                          (uint64_t)(uintptr_t)a.perm2d, (uint64_t)(uintptr_t)a.grad, (uint64_t)(uintptr_t)a.stats,
                          (uint64_t)(uintptr_t)a.queue, (uint64_t)a.num_cus, (uint64_t)(uintptr_t)a.hitmask,
                          (uint64_t)(uintptr_t)a.samples, (uint64_t)(uintptr_t)a.hitq,
                          (uint64_t)(uintptr_t)a.spill_long, (uint64_t)a.hit_cap, (uint64_t)a.long_spill_cap,
                          (uint64_t)a.cells_from_cam, (uint64_t)a.small_rings, (uint64_t)a.fit, (uint64_t)a.fitm, (uint64_t)(uintptr_t)a.fin, (uint64_t)(uintptr_t)a.finpool, (uint64_t)(uintptr_t)a.cpool,
                          (uint64_t)(uintptr_t)a.aocc, (uint64_t)a.ao_samples, (uint64_t)a.aa,
                          (uint64_t)(uintptr_t)a.order, (uint64_t)(uintptr_t)a.frames, (uint64_t)a.n_frames,
                          (uint64_t)(uintptr_t)a.gated.gate, (uint64_t)(uintptr_t)a.gated.claims, (uint64_t)a.gated.tasks,
                          (uint64_t)a.packed};
    k.insert(k.end(), std::begin(v), std::end(v));
}

// Replay g (capturing `launches` on dev->stream first when its key changed).  Stream
// capture records the same launches the direct path issues, so a replay is the same work.
template <class F>
int graph_run(rt_device dev, rt_device_s::FrameGraph& g, std::vector<uint64_t>&& key, F launches)
{
    if (!g.exec || g.key != key) {
        if (g.exec) HIP_TRY(hipGraphExecDestroy(g.exec));
        g.exec = nullptr;
        g.key.clear();
        hipGraph_t graph = nullptr;
        HIP_TRY(hipStreamBeginCapture(dev->stream, hipStreamCaptureModeThreadLocal));
        launches();
        const hipError_t launch_err = hipGetLastError();
        const hipError_t end_err = hipStreamEndCapture(dev->stream, &graph);
        if (launch_err != hipSuccess || end_err != hipSuccess) {
            if (graph) (void)hipGraphDestroy(graph);
            return fail(RT_ERR_HIP, "graph capture failed: %s",
                        hipGetErrorString(launch_err != hipSuccess ? launch_err : end_err));
        }
        const hipError_t inst_err = hipGraphInstantiate(&g.exec, graph, nullptr, nullptr, 0);
        (void)hipGraphDestroy(graph);
        if (inst_err != hipSuccess) {
            g.exec = nullptr;
            return fail(RT_ERR_HIP, "graph instantiate failed: %s", hipGetErrorString(inst_err));
        }
        g.key = std::move(key);
        ++dev->graph_captures;
    }
    HIP_TRY(hipGraphLaunch(g.exec, dev->stream));
    ++dev->graph_launches;
    return RT_OK;
}
} // namespace
} // extern "C++"

namespace {
// every shader of a batch traces frame 0's noise tables: they must hold the same bytes
bool same_tables(const Shader* a, const Shader* b)
{
    return a->textures[0]->hash == b->textures[0]->hash && a->cb[CB_NOISE] == b->cb[CB_NOISE];
}

void key_frames(std::vector<uint64_t>& k, const FrameTable& ft)
{
    const uint64_t* w = reinterpret_cast<const uint64_t*>(&ft);
    k.insert(k.end(), w, w + sizeof(FrameTable) / sizeof(uint64_t));
}

// A validated batch: its frame table, the device it runs on (frame 0's: stream, buffers,
// counters) and whether frames live on other devices.
struct Batch {
    FrameTable ft{};
    rt_device dev = nullptr;
    const Shader* s0 = nullptr;
    bool others = false;
};

// Check the n (camerarays, tracescreen) pairs, upload their constants, build the frame table
// and order the other frames' device streams before the batch.
int batch_begin(const rt_compute* cams, const rt_compute* scrs, int n, Batch& b, bool sync_cam = true,
                bool sync_scr = true)
{
    if (!cams || !scrs || n < 1 || n > RT_MAX_BATCH) return fail(RT_ERR_INVALID, "a batch holds 1..%d frames", RT_MAX_BATCH);
    int rc;
    for (int f = 0; f < n; ++f) {
        rt_compute cam = cams[f], scr = scrs[f];
        if (!cam || !scr || cam->dev != scr->dev) return fail(RT_ERR_INVALID, "computes must share a device");
        if (!cam->shader || !scr->shader) return fail(RT_ERR_STATE, "both computes need a current shader (swap)");
        if (cam->shader->kind != KIND_CAMERARAYS || scr->shader->kind != KIND_TRACESCREEN)
            return fail(RT_ERR_INVALID, "expected (camerarays, tracescreen)");
        if ((rc = check_texture(cam->shader)) || (rc = check_texture(scr->shader))) return rc;
        rt_device d = scr->dev;
        const Shader* s = scr->shader;
        if (f == 0) {
            b.dev = d;
            b.s0 = s;
        } else if (d->ordinal != b.dev->ordinal || d->width != b.dev->width || d->height != b.dev->height ||
                   s->landscape != b.s0->landscape || s->aa != b.s0->aa || s->ao != b.s0->ao ||
                   s->max_steps != b.s0->max_steps || s->recording != b.s0->recording ||
                   cam->shader->recording != cams[0]->shader->recording || !same_tables(s, b.s0) ||
                   !same_tables(cam->shader, b.s0)) {
            return fail(RT_ERR_INVALID, "frame %d: a batch needs one GPU, resolution, landscape, macro set and noise", f);
        }
        // a prepass-only call uploads the camerarays constants only: the tracescreen block may still be
        // read by this device's previous trace, which another stream can be running
        if ((sync_cam && (rc = sync_shader(d, cam->shader))) || (sync_scr && (rc = sync_shader(d, scr->shader))))
            return rc;
        rt_array_s* cr = cam->shader->array("CameraResults");
        rt_array_s* cd = scr->shader->array("CellDistance");
        if (!cd->dev_ptr || cd->elements < 1024) return fail(RT_ERR_STATE, "CellDistance not created with 1024 elements");
        b.ft.k[f] = scr->shader->d_consts;
        b.ft.kcam[f] = cam->shader->d_consts;
        b.ft.cam[f] = (cr->dev_ptr && cr->elements >= 1024) ? (float4*)cr->dev_ptr : d->scratch_cam;
        b.ft.cells[f] = (float2*)cd->dev_ptr;
        b.ft.out8[f] = d->fb8;
        b.ft.out32[f] = d->fb32;
    }
    // frames on other devices: their pending work (constant uploads, readbacks of the
    // framebuffer) precedes the batch on its stream
    for (int f = 1; f < n; ++f) {
        rt_device d = scrs[f]->dev;
        if (d == b.dev) continue;
        b.others = true;
        if (!d->sync_ev) HIP_TRY(hipEventCreateWithFlags(&d->sync_ev, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(d->sync_ev, d->stream));
        HIP_TRY(hipStreamWaitEvent(b.dev->stream, d->sync_ev, 0));
    }
    return RT_OK;
}

// the other frames' devices see their frames complete in their own stream order
int batch_end(const rt_compute* scrs, int n, Batch& b)
{
    HIP_TRY(hipGetLastError());
    if (!b.others) return RT_OK;
    rt_device dev = b.dev;
    if (!dev->sync_ev) HIP_TRY(hipEventCreateWithFlags(&dev->sync_ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(dev->sync_ev, dev->stream));
    for (int f = 1; f < n; ++f)
        if (scrs[f]->dev != dev) HIP_TRY(hipStreamWaitEvent(scrs[f]->dev->stream, dev->sync_ev, 0));
    return RT_OK;
}

} // namespace

// Terrain::render (Terrain.cpp:105-136) for n frames at once: every frame's prepass and
// setTargetDepths in one launch each, then one tracescreen over all frames' units
// (frame-major), on frame 0's device stream and buffers.  Frames on other devices (a
// FrameRing's slots) are ordered around the batch with events.  Phases: PRE = prepass,
// TRACE = setTargetDepths + tracescreen; `first`/`count` select the prepass frames,
// camera_out / camera_in redirect CameraResults through a contiguous device buffer
// (n x 1024 float4) for the split prepass of rt_terrain_prepass_batch / rt_terrain_trace_batch.
static int terrain_render_batch(const rt_compute* cams, const rt_compute* scrs, int n, int shard_rank,
                                int shard_count, bool feed, int phases, int first, int count, float4* camera_out,
                                const float4* camera_in, const TraceFuse* fuse, uint8_t* packed_dst,
                                size_t packed_stride)
{
    if (shard_count < 1 || shard_rank < 0 || shard_rank >= shard_count) return fail(RT_ERR_INVALID, "bad shard");
    if (feed && n != 1) return fail(RT_ERR_INVALID, "the camera feed is per frame");
    if (scrs && n >= 1 && scrs[0] && scrs[0]->dev)
        if (int rc0 = host_flag_check(scrs[0]->dev)) return rc0;
    for (int f = 0; scrs && f < n && f < RT_MAX_BATCH; ++f) // a deferred frame of these devices goes first
        if (scrs[f] && scrs[f]->dev)
            if (int rc0 = defer_flush(scrs[f]->dev)) return rc0;
    if (cams && scrs && n >= 1 && n <= RT_MAX_BATCH && scrs[0] && scrs[0]->dev) {
        // a pending ahead prepass writes these frames' CameraResults: it comes before anything this
        // call queues, the constant uploads of batch_begin included (they rewrite the block the
        // side-stream prepass reads)
        rt_device lead = scrs[0]->dev;
        for (int f = 0; f < n; ++f)
            if (scrs[f] && scrs[f]->dev && ahead_wait(scrs[f]->dev, lead->stream) != 0)
                return fail(RT_ERR_HIP, "waiting for the ahead prepass failed");
        // a full render prepasses in line: the lead's pending ahead prepass is superseded
        if (lead->ahead_pending && phases != PH_PRE && phases != PH_STAGE) lead->ahead_pending = false;
        if ((phases & PH_PRE) && lead->fuse_state != rt_device_s::FUSE_NONE) { // so is a staged / fused one
            fuse_forget(lead);
            lead->fuse_state = rt_device_s::FUSE_NONE;
        }
    }
    for (int f = 0; scrs && f < n && f < RT_MAX_BATCH; ++f) // rt_terrain_render re-arms its own renders
        if (scrs[f] && scrs[f]->dev) scrs[f]->dev->serial_ok = false;
    int rc;
    Batch b;
    const bool keep = (phases & PH_KEEP) != 0;
    phases &= ~PH_KEEP;
    if ((rc = batch_begin(cams, scrs, n, b, !keep && (phases & (PH_PRE | PH_STAGE)) != 0, !keep && (phases & PH_TRACE) != 0)))
        return rc;
    rt_device dev = b.dev;
    FrameTable& ft = b.ft;
    if (count < 0) count = n;
    // an empty range is valid anywhere: a rank past the last frame of a split prepass (B < N * chunk)
    if (count > n || (count > 0 && (first < 0 || first > n - count))) return fail(RT_ERR_INVALID, "bad prepass frame range");
    const bool graphs = (dev->flags & RT_DEVICE_GRAPH) && dev->stream != nullptr && phases == (PH_PRE | PH_TRACE);
    // gathered prepass results: the table reads them, and each frame's CameraResults array
    // receives its copy (Terrain::getCameraView stays valid) once the trace is queued, so the
    // copies do not delay it
    float4* cam_copy[RT_MAX_BATCH] = {};
    if (camera_in) {
        for (int f = 0; f < n; ++f) {
            const float4* src = camera_in + (size_t)f * 1024;
            if (ft.cam[f] != scrs[f]->dev->scratch_cam) cam_copy[f] = ft.cam[f];
            ft.cam[f] = const_cast<float4*>(src);
        }
    }
    if (phases == PH_STAGE) { // the frames' camerarays constants (above) and the table a fusing k_trace reads
        if ((rc = upload_frames(dev, dev->fuse_table, ft))) return rc;
        return batch_end(scrs, n, b);
    }
    if (phases == PH_PRE) {
        // the prepass of frames [first, first + count) only, on its own table
        if (count == 0) return batch_end(scrs, n, b);
        RtLaunch la_cam = make_launch(dev, cams[0]->shader);
        FrameTable sub{};
        for (int i = 0; i < count; ++i) {
            sub.k[i] = ft.k[first + i];
            sub.kcam[i] = ft.kcam[first + i];
            sub.cam[i] = camera_out ? camera_out + (size_t)(first + i) * 1024 : ft.cam[first + i];
        }
        if ((rc = upload_frames(dev, dev->pre_table, sub))) return rc;
        la_cam.frames = dev->pre_table.d;
        la_cam.frames_host = sub;
        la_cam.n_frames = (uint32_t)count;
        rt_launch_camerarays_batch(la_cam);
        return batch_end(scrs, n, b);
    }
    if ((rc = ensure_split_buffers(dev, b.s0->aa, b.s0->ao, n))) return rc;
    RtLaunch la_cam = make_launch(dev, cams[0]->shader), la_scr = make_launch(dev, scrs[0]->shader);
    if (packed_dst) { // rt_terrain_render_batch_packed: frame f's shard pixels straight into its packed buffer
        for (int f = 0; f < n; ++f) {
            if (ft.out32[f]) return fail(RT_ERR_UNSUPPORTED, "packed output: RGBA8-only devices (no RT_DEVICE_FLOAT_OUTPUT)");
            ft.out8[f] = reinterpret_cast<uint32_t*>(packed_dst + (size_t)f * packed_stride);
        }
        la_scr.packed = 1;
    }
    // The gated launch (GatedPrepass; opt-in, RT_DEVICE_GATED): a full nomadplains
    // render runs its prepass inside its own k_trace, and each unit starts once the prepass rays its cells
    // read are in, instead of a latency-bound prepass launch the whole trace waits for.  Measured slower
    // (the prepass rays march 2-3x slower beside the units), so off by default.  Not for the instrumented
    // kernels (their prepass counts stay separate), the camera feed (it wants the CameraResults before the
    // trace), a trace from gathered CameraResults or a fused prepass.
    const bool gated = phases == (PH_PRE | PH_TRACE) && !feed && !camera_in &&
                       (!fuse || (fuse->wait_ctl == nullptr && fuse->next.ctl == nullptr)) &&
                       b.s0->landscape == RT_NOMADPLAINS &&
                       (dev->flags & RT_DEVICE_GATED) && !(dev->flags & RT_DEVICE_STATS);
    if (gated)
        la_scr.gated = GatedPrepass{dev->gate, dev->claims, (uint32_t)n * (uint32_t)RT_FUSE_TASKS_PER_FRAME,
                                    (dev->flags & RT_DEVICE_DEBUG_GATE_STRESS) ? 3u : 0u};
    // rt_terrain_prepass_ahead: ev_order follows the last read of the frames' CameraResults -- k_order's,
    // or with the gated launch k_trace's (recorded after the trace below)
    if (!graphs && dev->ev_order && !gated) {
        la_scr.after_order = dev->ev_order;
        dev->order_recorded = true;
    }
    if ((rc = upload_frames(dev, dev->table, ft))) return rc;
    la_cam.frames = la_scr.frames = dev->table.d;
    la_cam.frames_host = la_scr.frames_host = ft;
    la_cam.n_frames = la_scr.n_frames = (uint32_t)n;
    // setTargetDepths runs at the start of the tracescreen launch (k_order), from the CameraResults; the
    // gated launch's k_order orders the units by the frames' previous CellDistance instead (scheduling
    // only: each unit derives its cells' brackets from this frame's rays, and the frame's last prepass
    // task writes its CellDistance)
    la_scr.cells_from_cam = gated ? 0 : 1;
    if (fuse) {
        la_scr.fuse_next = fuse->next;
        la_scr.after_order_fuse = fuse->next_after_order;
        la_scr.wait_ctl = fuse->wait_ctl;
        la_scr.wait_total = fuse->wait_total;
    }
    // one sample per pixel, at most one AO ray and no float output: hit pixels finish where their last
    // ray ends (k_trace), not through a per-sample colour and k_finish
    la_scr.fit = b.s0->aa == 1 && b.s0->ao <= 1;
    // (the colour pool packs frame << 23 | pixel: frames of < 2^23 pixels)
    la_scr.fitm = b.s0->aa == 1 && b.s0->ao >= 2 && (size_t)dev->width * (size_t)dev->height < ((size_t)1 << 23);
    for (int f = 0; f < n; ++f) {
        la_scr.fit = la_scr.fit && ft.out32[f] == nullptr;
        la_scr.fitm = la_scr.fitm && ft.out32[f] == nullptr;
    }
    auto pre = [&] {
        if ((phases & PH_PRE) && !gated) rt_launch_camerarays_batch(la_cam);
    };
    if (gated) ++dev->gated_launches;
    else if (phases & PH_PRE) ++dev->prepass_launches;
    if (graphs && !gated) {
        // the constant / table uploads stay outside: they precede the replay on this stream
        std::vector<uint64_t> kp;
        key_launch(kp, la_cam);
        key_frames(kp, ft);
        if ((rc = graph_run(dev, dev->graph_pre, std::move(kp), pre))) return rc;
    } else {
        pre();
    }
    if (feed) {
        // Flyby's view of this frame, on the host as soon as the prepass is done
        rt_compute cam = cams[0];
        if (!cam->feed_host) HIP_TRY(hipHostMalloc(&cam->feed_host, 1024 * sizeof(float4)));
        if (!cam->feed_ev) HIP_TRY(hipEventCreateWithFlags(&cam->feed_ev, hipEventDisableTiming));
        HIP_TRY(hipMemcpyAsync(cam->feed_host, ft.cam[0], 1024 * sizeof(float4), hipMemcpyDeviceToHost, dev->stream));
        HIP_TRY(hipEventRecord(cam->feed_ev, dev->stream));
        cam->feed_pending = true;
    }
    auto trace = [&] {
        rt_launch_tracescreen(la_scr, 0, 0, (uint32_t)dev->width, (uint32_t)dev->height, (uint32_t)shard_rank,
                              (uint32_t)shard_count);
    };
    {
        KernelTimer kt(dev);
        if (graphs) {
            std::vector<uint64_t> kt_key;
            key_launch(kt_key, la_scr);
            key_frames(kt_key, ft);
            const uint64_t extra[] = {(uint64_t)dev->width, (uint64_t)dev->height, (uint64_t)shard_rank,
                                      (uint64_t)shard_count};
            kt_key.insert(kt_key.end(), std::begin(extra), std::end(extra));
            if ((rc = graph_run(dev, dev->graph_trace, std::move(kt_key), trace))) return rc;
        } else {
            trace();
        }
    }
    if (gated && !graphs && dev->ev_order) { // k_trace read (and wrote) the frames' CameraResults
        HIP_TRY(hipEventRecord(dev->ev_order, dev->stream));
        dev->order_recorded = true;
    }
    for (int f = 0; f < n; ++f)
        if (cam_copy[f])
            HIP_TRY(hipMemcpyAsync(cam_copy[f], camera_in + (size_t)f * 1024, 1024 * sizeof(float4),
                                   hipMemcpyDeviceToDevice, dev->stream));
    return batch_end(scrs, n, b);
}

int rt_terrain_render_batch(const rt_compute* cams, const rt_compute* scrs, int n, int shard_rank, int shard_count)
{
    return terrain_render_batch(cams, scrs, n, shard_rank, shard_count, false);
}

// RT_DEVICE_DEFERRED: launch the device's pending frame (its setTargetDepths + trace; its prepass and constant
// blocks are queued already) with nothing fused.  Every call that launches on, reads or reconfigures the
// device calls this first.
static int defer_flush_batch(rt_device d);
static int deferred_render_batch(rt_device d, rt_compute cam, rt_compute scr);

static int defer_flush_one(rt_device d)
{
    if (!d->defer.pending) return RT_OK;
    const rt_device_s::Deferred p = d->defer;
    d->defer.pending = false;
    return terrain_render_batch(&p.cam, &p.scr, 1, p.rank, p.count, false, PH_TRACE | PH_KEEP);
}

static int defer_flush(rt_device d)
{
    if (!d) return RT_OK;
    if (!d->dq.empty()) return defer_flush_batch(d); // (a device has frames queued one way or the other, not both)
    return defer_flush_one(d);
}

// rt_terrain_render on an RT_DEVICE_DEFERRED device (Terrain.cpp:105-136, one frame per call).  The frame's
// setTargetDepths + trace wait for the next call; that call launches them with ITS frame's prepass run inside
// the trace kernel by the waves that finish their first unit (FusedPrepass; on the same stream, so this
// frame's k_order, launched later behind that whole kernel, needs no wait).  The prepass then rides on the
// trace's throughput instead of a latency-bound launch that gets CUs only as the trace retires (the plain
// path's ~0.2-0.3 ms per frame, profiles/r06/swap_chain.md).  Stream order keeps every buffer safe:
//   [camerarays constants of frame i+1] [k_order i: reads CameraResults] [k_trace i: frame i+1's prepass
//   writes CameraResults; reads only frame i's tracescreen constants] [tracescreen constants of frame i+1]
// (the prepass kernels are the only readers of the camerarays block).  Anything else falls back to a flush
// and the full render.
static int deferred_render(rt_device d, rt_compute cam, rt_compute scr, int shard_rank, int shard_count)
{
    if (shard_count < 1 || shard_rank < 0 || shard_rank >= shard_count) return fail(RT_ERR_INVALID, "bad shard");
    const bool np = cam->shader && scr->shader && cam->shader->landscape == RT_NOMADPLAINS &&
                    scr->shader->landscape == RT_NOMADPLAINS;
    const bool plain = np && d->stream && !(d->flags & (RT_DEVICE_GRAPH | RT_DEVICE_STATS | RT_DEVICE_GATED)) &&
                       !d->ahead_pending && !d->ahead_in_pending && d->fuse_state == rt_device_s::FUSE_NONE;
    if (!plain) {
        if (int rc = defer_flush(d)) return rc;
        return terrain_render_batch(&cam, &scr, 1, shard_rank, shard_count, false);
    }
    if (int rc0 = host_flag_check(d)) return rc0;
    HIP_TRY(hipSetDevice(d->ordinal));
    if (d->defer_k >= 2 && shard_count == 1 && same_tables(cam->shader, scr->shader)) {
        if (int rc = defer_flush_one(d)) return rc; // (a K = 1 frame pending: traced alone first)
        return deferred_render_batch(d, cam, scr);
    }
    if (int rc = defer_flush_batch(d)) return rc; // (frames queued for a batch, then a sharded render: they go first)
    if ((size_t)d->width * (size_t)d->height < RT_DEFER_FUSE_MIN_PIXELS && !(d->flags & RT_DEVICE_DEBUG_DEFER_SMALL)) {
        // a small frame's trace is shorter than the prepass it would carry (profiles/r06/deferred.md): it renders
        // as without the flag, its prepass on the prepass stream in the previous frame's trace tail
        if (int rc = defer_flush(d)) return rc;
        return serial_render(d, cam, scr, shard_rank, shard_count);
    }
    const rt_device_s::Deferred p = d->defer;
    // the pending frame's trace must run a k_trace (a single frame's shard past the last tile launches none)
    // with the noise tables this prepass reads
    // (the trace loads its noise tables from the pending frame's tracescreen gradients, which are up to date on the
    // device unless a later write dirtied them)
    const bool fuse = p.pending && p.scr->shader && p.scr->shader->landscape == RT_NOMADPLAINS &&
                      !p.scr->shader->grad_dirty && same_tables(cam->shader, p.scr->shader) &&
                      (size_t)p.rank < rt_shard_tiles(d->width, d->height, 0, 1);
    if (!fuse) {
        if (int rc = defer_flush(d)) return rc;
        // this frame's prepass in line (its camerarays constants go up with it)
        if (int rc = terrain_render_batch(&cam, &scr, 1, 0, 1, false, PH_PRE)) return rc;
        ++d->prepass_launches; // (a render with a prepass launch, rt_device_info)
    } else {
        Batch b; // this frame's camerarays constants (only the prepass kernels read that block)
        if (int rc = batch_begin(&cam, &scr, 1, b, true, false)) return rc;
        FrameTable sub{};
        sub.k[0] = b.ft.k[0];
        sub.kcam[0] = b.ft.kcam[0];
        sub.cam[0] = b.ft.cam[0];
        if (int rc = upload_frames(d, d->fuse_table, sub)) return rc;
        TraceFuse tf;
        tf.next = FusedPrepass{d->fuse_table.d, d->fctl, (uint32_t)RT_FUSE_TASKS_PER_FRAME};
        d->defer.pending = false;
        if (int rc = terrain_render_batch(&p.cam, &p.scr, 1, p.rank, p.count, false, PH_TRACE | PH_KEEP, 0, -1,
                                          nullptr, nullptr, &tf))
            return rc;
        ++d->deferred_fused;
    }
    // this frame's tracescreen constants (and noise gradients), behind the trace that read the previous frame's
    if (int rc = sync_shader(d, scr->shader)) return rc;
    d->defer = rt_device_s::Deferred{cam, scr, shard_rank, shard_count, true};
    return RT_OK;
}

// ---- RT_DEVICE_DEFERRED, K frames to a launch (rt_device_defer_batch) ----
// frame slot i of the device (made on first use)
static int slot_get(rt_device d, int i, rt_device_s::FrameSlot** out)
{
    while ((int)d->slots.size() <= i) d->slots.emplace_back(new rt_device_s::FrameSlot());
    rt_device_s::FrameSlot& f = *d->slots[i];
    if (!f.cam) {
        const size_t px = (size_t)d->width * d->height;
        HIP_TRY(hipMalloc(&f.cam, 1024 * sizeof(float4)));
        HIP_TRY(hipMalloc(&f.cells, 1024 * sizeof(float2)));
        HIP_TRY(hipMalloc(&f.fb8, px * 4));
        if (d->fb32) HIP_TRY(hipMalloc(&f.fb32, px * 16));
    }
    *out = &f;
    return RT_OK;
}

// the next launch block: the frames' tables and the constant blocks of the m frames from queue position `from`
// (their prepass runs in this launch), uploaded in one copy; those frames' constants are read from there on
static int block_upload(rt_device d, rt_device_s::LaunchBlock& hb, int from, int m, rt_device_s::LaunchBlock** out)
{
    if (!d->blocks) HIP_TRY(hipMalloc(&d->blocks, 3 * sizeof(rt_device_s::LaunchBlock)));
    const int b = d->block_next;
    d->block_next = (b + 1) % 3;
    rt_device_s::LaunchBlock* db = d->blocks + b;
    for (int i = 0; i < m; ++i) {
        rt_device_s::FrameSlot& f = *d->slots[d->dq[from + i]];
        hb.k[i] = f.hk;
        hb.kcam[i] = f.hkcam;
        f.dk = db->k + i;
        f.dkcam = db->kcam + i;
        hb.nx.k[i] = f.dk;
        hb.nx.kcam[i] = f.dkcam;
        hb.nx.cam[i] = f.cam;
    }
    if (int rc = d->block_stage[b].upload(d->stream, db, &hb, sizeof(hb))) return rc;
    *out = db;
    return RT_OK;
}

// launch the first n of the queued frames (their prepass done): setTargetDepths + one trace over the n frames
// (the shard is the whole frame), with the prepasses of the next m queued frames fused into it (FusedPrepass on
// the same stream: the next launch's k_order comes after this whole kernel).  last: the n-th frame is the
// flush's last, so it writes the device's framebuffers and the API's CellDistance; its CameraResults are
// copied to the API's array behind the trace.
static int batch_trace(rt_device d, int n, int m, bool last)
{
    rt_compute cam = d->dq_cam, scr = d->dq_scr;
    Shader* s = scr->shader;
    rt_device_s::LaunchBlock hb{};
    FrameTable& ft = hb.ft;
    for (int i = 0; i < n; ++i) {
        rt_device_s::FrameSlot& f = *d->slots[d->dq[i]];
        const bool out = last && i == n - 1;
        ft.k[i] = f.dk;
        ft.kcam[i] = f.dkcam;
        ft.cam[i] = f.cam;
        ft.cells[i] = out ? (float2*)s->array("CellDistance")->dev_ptr : f.cells;
        ft.out8[i] = out ? d->fb8 : f.fb8;
        ft.out32[i] = out ? d->fb32 : f.fb32;
    }
    if (int rc = ensure_split_buffers(d, s->aa, s->ao, n)) return rc;
    rt_device_s::LaunchBlock* db = nullptr;
    if (int rc = block_upload(d, hb, n, m, &db)) return rc;
    RtLaunch a = make_launch(d, s);
    a.consts = ft.k[0];
    a.frames = &db->ft;
    a.frames_host = ft;
    a.n_frames = (uint32_t)n;
    a.cells_from_cam = 1;
    if (m > 0) {
        a.fuse_next = FusedPrepass{&db->nx, d->fctl, (uint32_t)m * (uint32_t)RT_FUSE_TASKS_PER_FRAME};
        d->deferred_fused += (unsigned long long)m;
    }
    // (as terrain_render_batch: hit pixels finish in k_trace with one sample, <= 1 AO ray and no float output)
    a.fit = s->aa == 1 && s->ao <= 1 && !d->fb32;
    a.fitm = s->aa == 1 && s->ao >= 2 && !d->fb32 && (size_t)d->width * (size_t)d->height < ((size_t)1 << 23);
    {
        KernelTimer kt(d);
        rt_launch_tracescreen(a, 0, 0, (uint32_t)d->width, (uint32_t)d->height, 0u, 1u);
    }
    if (last) {
        rt_array_s* cr = cam->shader->array("CameraResults");
        if (cr && cr->dev_ptr && cr->elements >= 1024)
            HIP_TRY(hipMemcpyAsync(cr->dev_ptr, ft.cam[n - 1], 1024 * sizeof(float4), hipMemcpyDeviceToDevice, d->stream));
    }
    HIP_TRY(hipGetLastError());
    for (int i = 0; i < n; ++i) d->dq.pop_front();
    d->dq_pre = m;
    return RT_OK;
}

// the standalone prepass of the first n queued frames (nothing queued before them runs a trace to fuse it into)
static int batch_prepass(rt_device d, int n)
{
    rt_device_s::LaunchBlock hb{};
    rt_device_s::LaunchBlock* db = nullptr;
    if (int rc = block_upload(d, hb, 0, n, &db)) return rc;
    RtLaunch a = make_launch(d, d->dq_cam->shader);
    a.consts = hb.nx.kcam[0];
    a.frames = &db->nx;
    a.frames_host = hb.nx;
    a.n_frames = (uint32_t)n;
    rt_launch_camerarays_batch(a);
    HIP_TRY(hipGetLastError());
    ++d->prepass_launches;
    d->dq_pre = n;
    return RT_OK;
}

// launch every queued frame, K to a launch, the last into the device's own buffers
static int defer_flush_batch(rt_device d)
{
    const int K = d->defer_k;
    while (!d->dq.empty()) {
        if (d->dq_pre == 0)
            if (int rc = batch_prepass(d, std::min<int>(K, (int)d->dq.size()))) return rc;
        const int n = d->dq_pre, m = std::min<int>(K, (int)d->dq.size() - n);
        if (int rc = batch_trace(d, n, m, (int)d->dq.size() == n)) {
            d->dq.clear();
            d->dq_pre = 0;
            return rc;
        }
    }
    return RT_OK;
}

// rt_terrain_render with K >= 2 frames to a deferred launch: queue this frame (its constant blocks snapshotted in
// its slot); the K-th queued frame beyond a launch-ready group launches that group with this group's prepasses
// fused.  Slots are reused by stream order: a slot's buffers are next written by launches behind the one that
// read them.
static int deferred_render_batch(rt_device d, rt_compute cam, rt_compute scr)
{
    const int K = d->defer_k;
    Shader *sc = cam->shader, *ss = scr->shader;
    d->serial_ok = false; // (its launches read the device's CameraResults: a later serial render prepasses in line)
    // another compute pair, or new noise tables: what is queued goes first, then the tables go up
    if (!d->dq.empty() && (cam != d->dq_cam || scr != d->dq_scr || sc->grad_dirty || ss->grad_dirty))
        if (int rc = defer_flush_batch(d)) return rc;
    if (d->dq.empty()) {
        if (int rc = check_texture(sc)) return rc;
        if (int rc = check_texture(ss)) return rc;
        rt_array_s* cd = ss->array("CellDistance");
        if (!cd || !cd->dev_ptr || cd->elements < 1024) return fail(RT_ERR_STATE, "CellDistance not created with 1024 elements");
        if (int rc = sync_shader(d, sc)) return rc; // the noise gradients (and the shaders' own blocks) up
        if (int rc = sync_shader(d, ss)) return rc;
        d->dq_cam = cam;
        d->dq_scr = scr;
    }
    const int slot = d->slot_next;
    d->slot_next = (d->slot_next + 1) % (2 * K);
    rt_device_s::FrameSlot* f = nullptr;
    if (int rc = slot_get(d, slot, &f)) return rc;
    {
        std::lock_guard<std::mutex> lk(g_cb_mu); // (a snapshot: they go up with the launch that runs its prepass)
        build_consts(*sc, *d, f->hkcam);
        build_consts(*ss, *d, f->hk);
    }
    f->dk = f->dkcam = nullptr;
    d->dq.push_back(slot);
    if (d->dq_pre == 0 && (int)d->dq.size() == K) return batch_prepass(d, K); // the first group: nothing to ride on
    if (d->dq_pre == K && (int)d->dq.size() == 2 * K) return batch_trace(d, K, K, false);
    return RT_OK;
}

int rt_terrain_render_batch_packed(const rt_compute* cams, const rt_compute* scrs, int n, int shard_rank,
                                   int shard_count, void* dst_device, size_t frame_stride)
{
    if (!dst_device || shard_count < 2) return fail(RT_ERR_INVALID, "packed output: a device buffer and shard_count >= 2");
    if (cams && scrs && n >= 1 && scrs[0] && scrs[0]->dev) {
        const rt_device d = scrs[0]->dev;
        size_t need = 0;
        for (int f = 0; f < n; ++f) { // frame f traces shard (rank + f) % count (rotation, n > 1)
            const int sh = n > 1 ? (shard_rank + f) % shard_count : shard_rank;
            need = std::max(need, rt_shard_tiles(d->width, d->height, sh, shard_count) * RT_TILE * RT_TILE * 4);
        }
        if (frame_stride < need || frame_stride % 16) return fail(RT_ERR_INVALID, "packed output: frame_stride %zu < %zu bytes "
                                                                   "or not 16-byte aligned", frame_stride, need);
    }
    return terrain_render_batch(cams, scrs, n, shard_rank, shard_count, false, PH_PRE | PH_TRACE, 0, -1, nullptr,
                                nullptr, nullptr, (uint8_t*)dst_device, frame_stride);
}

int rt_terrain_prepass_batch(const rt_compute* cams, const rt_compute* scrs, int n, int first, int count,
                             void* camera_out)
{
    return terrain_render_batch(cams, scrs, n, 0, 1, false, PH_PRE, first, count, (float4*)camera_out);
}

int rt_terrain_trace_batch(const rt_compute* cams, const rt_compute* scrs, int n, int shard_rank, int shard_count,
                           const void* camera_in)
{
    if (!camera_in) return fail(RT_ERR_INVALID, "camera_in: the batch's gathered CameraResults");
    return terrain_render_batch(cams, scrs, n, shard_rank, shard_count, false, PH_TRACE, 0, -1, nullptr,
                                (const float4*)camera_in);
}

// The prepass one batch ahead.  For nomadplains on uninstrumented devices the
// batch is STAGED: its camerarays constants and a frame table go up on the GPU's side stream (after the
// last k_order of the batches this device leads: the last read of the CameraResults and of the
// constants), and the next trace on this GPU (rt_terrain_trace_ahead of another batch) runs its
// prepass inside that trace's persistent k_trace (FusedPrepass): the rays ride on that kernel's
// throughput instead of a latency-bound launch that waits for its CUs.  Otherwise the prepass itself
// is queued on the side stream, issued before the previous batch's trace so that it takes CUs before
// that trace's k_trace holds them all.
int rt_terrain_prepass_ahead(const rt_compute* cams, const rt_compute* scrs, int n)
{
    if (!cams || !scrs || n < 1 || n > RT_MAX_BATCH) return fail(RT_ERR_INVALID, "a batch holds 1..%d frames", RT_MAX_BATCH);
    for (int f = 0; f < n; ++f)
        if (!cams[f] || !scrs[f] || cams[f]->dev != scrs[f]->dev) return fail(RT_ERR_INVALID, "computes must share a device");
    rt_device lead = scrs[0]->dev;
    if (int rc0 = host_flag_check(lead)) return rc0;
    for (int f = 0; f < n; ++f)
        if (int rc0 = defer_flush(scrs[f]->dev)) return rc0;
    if (lead->flags & RT_DEVICE_GRAPH) return fail(RT_ERR_STATE, "the ahead prepass runs on a side stream: not with RT_DEVICE_GRAPH");
    if (lead->ahead_pending) return fail(RT_ERR_STATE, "a prepass is already ahead for this device's batch: trace it first");
    if (lead->fuse_state == rt_device_s::FUSE_FUSED && lead->ev_fuser_done) {
        // an earlier fused prepass of this device's frames that no trace consumed: it still writes them
        HIP_TRY(hipStreamWaitEvent(lead->stream, lead->ev_fuser_done, 0));
    }
    fuse_forget(lead);
    lead->fuse_state = rt_device_s::FUSE_NONE;
    HIP_TRY(hipSetDevice(lead->ordinal));
    hipStream_t side = ahead_stream(lead->ordinal, true);
    if (!side) return fail(RT_ERR_HIP, "side stream");
    if (!lead->ev_order) HIP_TRY(hipEventCreateWithFlags(&lead->ev_order, hipEventDisableTiming));
    if (!lead->ev_ahead) HIP_TRY(hipEventCreateWithFlags(&lead->ev_ahead, hipEventDisableTiming));
    // before the first recorded k_order: after everything queued so far
    if (!lead->order_recorded) {
        HIP_TRY(hipEventRecord(lead->ev_order, lead->stream));
        lead->order_recorded = true;
    }
    HIP_TRY(hipStreamWaitEvent(side, lead->ev_order, 0));
    const Shader* s0 = scrs[0]->shader;
    const bool fuse = s0 && s0->landscape == RT_NOMADPLAINS && !(lead->flags & RT_DEVICE_STATS);
    // the batch's devices upload their constants and launch on the side stream for this call
    std::vector<std::pair<rt_device, hipStream_t>> saved;
    for (int f = 0; f < n; ++f) {
        rt_device d = scrs[f]->dev;
        bool seen = false;
        for (auto& p : saved) seen |= p.first == d;
        if (!seen) {
            saved.emplace_back(d, d->stream);
            d->stream = side;
        }
    }
    int rc = terrain_render_batch(cams, scrs, n, 0, 1, false, fuse ? PH_STAGE : PH_PRE, 0, n, nullptr);
    for (auto& p : saved) p.first->stream = p.second;
    if (rc) return rc;
    HIP_TRY(hipEventRecord(lead->ev_ahead, side));
    lead->ahead_pending = true;
    lead->ahead_cams.assign(cams, cams + n);
    lead->fuse_devs.clear();
    for (auto& p : saved) { // every device whose frames it writes or stages (not the lead alone)
        rt_device d = p.first;
        if (!d->ev_ahead_in) HIP_TRY(hipEventCreateWithFlags(&d->ev_ahead_in, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(d->ev_ahead_in, side));
        d->ahead_in_pending = true;
        lead->fuse_devs.push_back(d);
    }
    if (fuse) {
        lead->fuse_state = rt_device_s::FUSE_STAGED;
        lead->fuse_n = n;
        std::lock_guard<std::mutex> lk(g_stream_mu);
        g_fuse_staged[lead->ordinal].push_back(lead);
    }
    return RT_OK;
}

// setTargetDepths + tracescreen of a batch whose prepass rt_terrain_prepass_ahead queued or staged:
// after the side-stream prepass, or (fused) with k_order waiting for the rays the previous k_trace
// computed; a batch that was staged but never fused prepasses in line; without one (or for other
// frames, or after a camera constant changed since) the full render_batch.  In every case the
// oldest batch staged on this GPU by another device is fused into this launch's k_trace.
int rt_terrain_trace_ahead(const rt_compute* cams, const rt_compute* scrs, int n, int shard_rank, int shard_count)
{
    if (!cams || !scrs || n < 1 || n > RT_MAX_BATCH || !scrs[0] || !scrs[0]->shader) return fail(RT_ERR_INVALID, "a batch holds 1..%d frames", RT_MAX_BATCH);
    rt_device lead = scrs[0]->dev;
    if (int rc0 = host_flag_check(lead)) return rc0;
    for (int f = 0; f < n; ++f)
        if (scrs[f] && scrs[f]->dev)
            if (int rc0 = defer_flush(scrs[f]->dev)) return rc0;
    HIP_TRY(hipSetDevice(lead->ordinal));
    bool ahead = lead->ahead_pending && (size_t)n <= lead->ahead_cams.size();
    for (int f = 0; ahead && f < n; ++f)
        ahead = cams[f] == lead->ahead_cams[f] && cams[f]->shader && !cams[f]->shader->cb_dirty;
    TraceFuse tf;
    int phases = PH_PRE | PH_TRACE;
    const int state = lead->fuse_state;
    if (ahead && state == rt_device_s::FUSE_FUSED) {
        // the previous k_trace ran this batch's prepass: k_order polls its ray counter, so the frames'
        // devices need not wait for that whole kernel (their ahead_in event follows it).  The poll comes
        // after the fusing launch's k_order, which zeroed the counter (otherwise a k_order on
        // this stream could run first and pass on the previous fused round's count)
        HIP_TRY(hipStreamWaitEvent(lead->stream, lead->ev_fuse_order, 0));
        tf.wait_ctl = lead->fctl;
        tf.wait_total = (uint32_t)lead->fuse_n * (uint32_t)(RT_CAMERA_RES * RT_CAMERA_RES);
        for (rt_device d : lead->fuse_devs) d->ahead_in_pending = false;
        phases = PH_TRACE;
    } else if (ahead && state == rt_device_s::FUSE_NONE) {
        HIP_TRY(hipStreamWaitEvent(lead->stream, lead->ev_ahead, 0)); // the side-stream prepass
        phases = PH_TRACE;
    }
    // (STAGED and never fused, or not covered: the full render, in line; a fused prepass this call does
    // not use is waited for through the frames' ahead_in events, before anything is uploaded)
    fuse_forget(lead);
    lead->fuse_state = rt_device_s::FUSE_NONE;
    lead->ahead_pending = false;
    // the next batch: the oldest staged by another device of this GPU that can share this k_trace (its
    // landscape, noise tables and frame size)
    rt_device z = nullptr;
    const Shader* s0 = scrs[0]->shader;
    // only a launch that runs k_trace can take it: a single-frame (or unrotated) shard past the last tile
    // launches nothing (launch_split_l), and a batch fused there would wait for tasks no kernel runs
    // 
    const size_t frame_tiles = rt_shard_tiles(lead->width, lead->height, 0, 1);
    const bool runs_trace = (n > 1 && shard_count > 1) || (size_t)shard_rank < frame_tiles;
    if (runs_trace && s0->landscape == RT_NOMADPLAINS && !(lead->flags & (RT_DEVICE_STATS | RT_DEVICE_GRAPH))) {
        std::lock_guard<std::mutex> lk(g_stream_mu);
        auto& v = g_fuse_staged[lead->ordinal];
        for (auto it = v.begin(); it != v.end(); ++it) {
            rt_device c = *it;
            const rt_compute cz = c->ahead_cams.empty() ? nullptr : (rt_compute)c->ahead_cams[0];
            if (c == lead || c->width != lead->width || c->height != lead->height || !cz || !cz->shader ||
                cz->shader->landscape != RT_NOMADPLAINS || !same_tables(cz->shader, s0))
                continue;
            z = c;
            v.erase(it);
            break;
        }
    }
    if (z) {
        // its staged constants and table are up, and its previous k_order (the last poll of its counters,
        // which this launch's k_order zeroes) is done
        HIP_TRY(hipStreamWaitEvent(lead->stream, z->ev_ahead, 0));
        // (diagnostic RT_DEVICE_DEBUG_WITHHOLD_FUSE on the fusing device: no task runs, the counters are still
        // zeroed, so z's k_order times out -- the fail-safe's test)
        const uint32_t tasks = (lead->flags & RT_DEVICE_DEBUG_WITHHOLD_FUSE)
                                   ? 0u : (uint32_t)z->fuse_n * (uint32_t)RT_FUSE_TASKS_PER_FRAME;
        tf.next = FusedPrepass{z->fuse_table.d, z->fctl, tasks};
        if (!z->ev_fuse_order) HIP_TRY(hipEventCreateWithFlags(&z->ev_fuse_order, hipEventDisableTiming));
        tf.next_after_order = z->ev_fuse_order;
    }
    int rc = terrain_render_batch(cams, scrs, n, shard_rank, shard_count, false, phases, 0, -1, nullptr, nullptr, &tf);
    if (z) {
        if (rc) { // not launched: z stays staged (prepasses in line when traced)
            std::lock_guard<std::mutex> lk(g_stream_mu);
            g_fuse_staged[z->ordinal].insert(g_fuse_staged[z->ordinal].begin(), z);
            return rc;
        }
        if (!z->ev_fuser_done) HIP_TRY(hipEventCreateWithFlags(&z->ev_fuser_done, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(z->ev_fuser_done, lead->stream));
        z->fuse_state = rt_device_s::FUSE_FUSED;
        for (rt_device d : z->fuse_devs) { // a render of z's frames that does not use the fused prepass waits for it
            HIP_TRY(hipEventRecord(d->ev_ahead_in, lead->stream));
            d->ahead_in_pending = true;
        }
    }
    return rc;
}

size_t rt_shard_bytes(rt_device d, int rank, int count)
{
    if (!d || count < 1 || rank < 0 || rank >= count) return 0;
    size_t tiles = rt_shard_tiles(d->width, d->height, rank, count);
    return tiles * RT_TILE * RT_TILE * 4;
}

// n (device, shard, buffer) jobs in launches of up to RT_SHARD_JOBS on devs[0]'s stream; devices on
// other streams are ordered around them with events (their earlier work first, their later work after)
static int shard_copy(const rt_device* devs, const int* shards, int count, void* const* bufs, int n, int pack)
{
    if (!devs || !shards || !bufs || n < 0 || count < 1) return fail(RT_ERR_INVALID, "bad arguments");
    if (n == 0) return RT_OK;
    rt_device d0 = devs[0];
    if (d0 && host_flag_check(d0)) return RT_ERR_STATE;
    for (int i = 0; i < n; ++i) {
        if (!devs[i] || !bufs[i] || shards[i] < 0 || shards[i] >= count) return fail(RT_ERR_INVALID, "bad arguments");
        if (int rc = defer_flush(devs[i])) return rc; // the pending frame is what the shard copy reads or overwrites
        if (devs[i]->width != d0->width || devs[i]->height != d0->height)
            return fail(RT_ERR_INVALID, "shard batch: devices differ in size");
    }
    auto order = [&](rt_device from, rt_device to) -> int {
        if (!from->sync_ev) HIP_TRY(hipEventCreateWithFlags(&from->sync_ev, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(from->sync_ev, from->stream));
        HIP_TRY(hipStreamWaitEvent(to->stream, from->sync_ev, 0));
        return RT_OK;
    };
    int rc;
    for (int i = 1; i < n; ++i)
        if (devs[i]->stream != d0->stream && (rc = order(devs[i], d0))) return rc;
    ShardJobs jobs;
    for (int b = 0; b < n; b += RT_SHARD_JOBS) {
        const int m = n - b < RT_SHARD_JOBS ? n - b : RT_SHARD_JOBS;
        for (int j = 0; j < m; ++j) {
            jobs.fb[j] = devs[b + j]->fb8;
            jobs.packed[j] = (uint32_t*)bufs[b + j];
            jobs.shard[j] = shards[b + j];
        }
        rt_launch_shard_copy(d0->stream, jobs, m, d0->width, d0->height, count, pack);
    }
    HIP_TRY(hipGetLastError());
    bool others = false;
    for (int i = 1; i < n; ++i) others |= devs[i]->stream != d0->stream;
    if (others) {
        if (!d0->sync_ev) HIP_TRY(hipEventCreateWithFlags(&d0->sync_ev, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(d0->sync_ev, d0->stream));
        for (int i = 1; i < n; ++i)
            if (devs[i]->stream != d0->stream) HIP_TRY(hipStreamWaitEvent(devs[i]->stream, d0->sync_ev, 0));
    }
    return RT_OK;
}

int rt_shard_pack(rt_device d, int rank, int count, void* dst)
{
    return shard_copy(&d, &rank, count, &dst, 1, 1);
}

int rt_shard_unpack(rt_device d, int rank, int count, const void* src)
{
    void* p = const_cast<void*>(src);
    return shard_copy(&d, &rank, count, &p, 1, 0);
}

int rt_shard_pack_batch(const rt_device* devs, const int* shard_ranks, int shard_count, void* const* dst_device, int n)
{
    return shard_copy(devs, shard_ranks, shard_count, dst_device, n, 1);
}

int rt_shard_unpack_batch(const rt_device* devs, const int* shard_ranks, int shard_count,
                          const void* const* src_device, int n)
{
    return shard_copy(devs, shard_ranks, shard_count, const_cast<void* const*>(src_device), n, 0);
}

int rt_noise_generate(uint32_t seed, int rand_kind, uint8_t* perm2d, float* grad)
{
    if (!perm2d || !grad) return fail(RT_ERR_INVALID, "null output");
    if (rand_kind != 0 && rand_kind != 1) return fail(RT_ERR_INVALID, "rand_kind must be 0 (MSVC) or 1 (glibc)");
    rt_noise::generate(seed, rand_kind, perm2d, grad);
    return RT_OK;
}

} // extern "C"

// ---- host-side Terrain helpers (engine code that stays on the CPU in the
// reference's flow; used by the compatibility render path) ----------------
namespace {
float host_depth(const float* cr, int x, int y)
{
    if (x < 0) x = 0;
    if (x >= RT_CAMERA_RES) x = RT_CAMERA_RES - 1;
    if (y < 0) y = 0;
    if (y >= RT_CAMERA_RES) y = RT_CAMERA_RES - 1;
    return cr[(y * RT_CAMERA_RES + x) * 4 + 3];
}
float host_depth_interp(const float* cr, int x, int y)
{
    if (x < 0) { float m = host_depth(cr, x + 1, y); float d = host_depth(cr, x + 2, y) - m; return m - d; }
    if (x >= RT_CAMERA_RES) { float m = host_depth(cr, x - 1, y); float d = host_depth(cr, x - 2, y) - m; return m - d; }
    if (y < 0) { float m = host_depth(cr, x, y + 1); float d = host_depth(cr, x, y + 2) - m; return m - d; }
    if (y >= RT_CAMERA_RES) { float m = host_depth(cr, x, y - 1); float d = host_depth(cr, x, y - 2) - m; return m - d; }
    return host_depth(cr, x, y);
}
} // namespace

extern "C" int rt_terrain_set_target_depths(const float* cr, float* cells)
{
    // Terrain.cpp:398-439 (Terrain::getDepth/getDepthInterp :356-396)
    if (!cr || !cells) return fail(RT_ERR_INVALID, "null arguments");
    for (int x = 0; x < RT_CAMERA_RES * RT_CAMERA_RES; ++x) {
        int xpos = x % RT_CAMERA_RES, ypos = x / RT_CAMERA_RES;
        float dmin = host_depth_interp(cr, xpos, ypos);
        float dmax = dmin;
        for (int xp = -2; xp <= 2; ++xp)
            for (int yp = -2; yp <= 2; ++yp) {
                float d = host_depth_interp(cr, xpos + xp, ypos + yp);
                dmin = std::min(d, dmin);
                dmax = std::max(d, dmax);
            }
        dmin = dmin * 0.96f - 0.01f;
        dmax = dmax * 1.22f + 0.4f;
        dmin = std::max(RT_CAMERA_NEAR, dmin);
        dmax = std::min(RT_CAMERA_FAR, dmax);
        cells[2 * x] = dmin;
        cells[2 * x + 1] = dmax;
    }
    return RT_OK;
}

// ---- diagnostics ------------------------------------------------------------
extern "C" int rt_debug_math(rt_device d, int op, const float* a, const float* b, float* y, int n)
{
    if (!d || !a || !y || n <= 0) return fail(RT_ERR_INVALID, "bad arguments");
    float *da = nullptr, *db = nullptr, *dy = nullptr;
    if (op == 12) {
        // octave-count sweep over n bit patterns from bits(a[0]): 3 counters out
        HIP_TRY(hipMalloc(&da, 4));
        HIP_TRY(hipMalloc(&dy, 12));
        HIP_TRY(hipMemcpy(da, a, 4, hipMemcpyHostToDevice));
        HIP_TRY(hipMemset(dy, 0, 12));
        rt_launch_debug_math(d->stream, op, da, da, dy, n);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipStreamSynchronize(d->stream));
        HIP_TRY(hipMemcpy(y, dy, 12, hipMemcpyDeviceToHost));
        HIP_TRY(hipFree(da));
        HIP_TRY(hipFree(dy));
        return RT_OK;
    }
    size_t bytes = (size_t)n * 4;
    HIP_TRY(hipMalloc(&da, bytes));
    HIP_TRY(hipMalloc(&db, bytes));
    HIP_TRY(hipMalloc(&dy, bytes));
    HIP_TRY(hipMemcpy(da, a, bytes, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(db, b ? b : a, bytes, hipMemcpyHostToDevice));
    rt_launch_debug_math(d->stream, op, da, db, dy, n);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(d->stream));
    HIP_TRY(hipMemcpy(y, dy, bytes, hipMemcpyDeviceToHost));
    HIP_TRY(hipFree(da));
    HIP_TRY(hipFree(db));
    HIP_TRY(hipFree(dy));
    return RT_OK;
}

// Evaluate noise3d (density = 0) or the compute's landscape getDensity (density = 1)
// at n points with the compute's current tables and constants.
extern "C" int rt_debug_noise(rt_compute c, const float* xyz, float* out, int n, int density)
{
    if (!c || !c->shader || !xyz || !out || n <= 0) return fail(RT_ERR_INVALID, "bad arguments");
    rt_device dev = c->dev;
    int rc;
    if ((rc = check_texture(c->shader)) || (rc = sync_shader(dev, c->shader))) return rc;
    float *dx = nullptr, *dy = nullptr;
    HIP_TRY(hipMalloc(&dx, (size_t)n * 12));
    HIP_TRY(hipMalloc(&dy, (size_t)n * 4));
    HIP_TRY(hipMemcpyAsync(dx, xyz, (size_t)n * 12, hipMemcpyHostToDevice, dev->stream));
    rt_launch_debug_noise(make_launch(dev, c->shader), dx, dy, n, density);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(out, dy, (size_t)n * 4, hipMemcpyDeviceToHost, dev->stream));
    HIP_TRY(hipStreamSynchronize(dev->stream));
    HIP_TRY(hipFree(dx));
    HIP_TRY(hipFree(dy));
    return RT_OK;
}

extern "C" int rt_debug_sky(rt_compute c, const float* dirs, float* out, int n)
{
    if (!c || !c->shader || !dirs || !out || n <= 0) return fail(RT_ERR_INVALID, "bad arguments");
    rt_device dev = c->dev;
    int rc;
    if ((rc = check_texture(c->shader)) || (rc = sync_shader(dev, c->shader))) return rc;
    float *dx = nullptr, *dy = nullptr;
    HIP_TRY(hipMalloc(&dx, (size_t)n * 12));
    HIP_TRY(hipMalloc(&dy, (size_t)n * 28));
    HIP_TRY(hipMemcpyAsync(dx, dirs, (size_t)n * 12, hipMemcpyHostToDevice, dev->stream));
    rt_launch_debug_sky(make_launch(dev, c->shader), dx, dy, n);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(out, dy, (size_t)n * 28, hipMemcpyDeviceToHost, dev->stream));
    HIP_TRY(hipStreamSynchronize(dev->stream));
    HIP_TRY(hipFree(dx));
    HIP_TRY(hipFree(dy));
    return RT_OK;
}

// ---------------------------------------------------------------------------
// IRecorder / RecorderWinAPI (Factories/IRecorder.h, Adapters/RecorderWinAPI.cpp) over a
// raw-video sink: Media Foundation's WMV sink writer does not exist here, so the frames
// are appended as raw MFVideoFormat_RGB32 (B, G, R, 0) rows to `path` (ffmpeg reads it as
// -f rawvideo -pix_fmt bgr0 -s WxH -r <rate>) and every sample's time stamp and duration
// (100 ns units, IMFSample::SetSampleTime/SetSampleDuration) go to `path`.txt.
struct rt_recorder_s {
    rt_device dev = nullptr;
    int width = 0, height = 0, frame_rate = 0;
    bool fixed_speed = true;
    bool recording = false, begun = false, finalized = false;
    std::string path;
    FILE* video = nullptr;
    FILE* index = nullptr;
    uint64_t rt_start = 0, rt_duration = 0; // RecorderWinAPI::rtStart / rtDuration
    float frame_time = 0.0f;                 // Timer::getConstant() of the frame being written
    uint64_t frames = 0;
    uint32_t* host = nullptr;                // pinned W*H*4 staging (swapStaging's role)
    std::vector<uint32_t> conv;              // CPU conversion buffer of rt_recorder_write (pBuffer's role)
    ~rt_recorder_s()
    {
        if (video) fclose(video);
        if (index) fclose(index);
        if (host) (void)hipHostFree(host);
        if (dev && dev->recorder == this) dev->recorder = nullptr; // ~RecorderWinAPI: setRecorder(nullptr)
    }
};

static void recorder_detach(rt_recorder r) { r->dev = nullptr; }

static int recorder_sample(rt_recorder r, const uint32_t* bgrx)
{
    // RecorderWinAPI.cpp:264-274: fixed speed = 1/frameRate per frame, else the frame's
    // own time in float (10000000.0f * modifier, truncated)
    uint64_t dur = r->rt_duration;
    if (!r->fixed_speed) dur = (uint64_t)(10000000.0f * r->frame_time);
    const size_t n = (size_t)r->width * r->height;
    if (fwrite(bgrx, 4, n, r->video) != n) return fail(RT_ERR_STATE, "recorder: short write to %s", r->path.c_str());
    fprintf(r->index, "%llu %llu %llu\n", (unsigned long long)r->frames, (unsigned long long)r->rt_start,
            (unsigned long long)dur);
    r->rt_start += dur;
    r->frames++;
    return RT_OK;
}

static int recorder_capture(rt_recorder r)
{
    if (!r->begun || r->finalized) return fail(RT_ERR_STATE, "recorder: write outside BeginWriting/Finalize");
    rt_device d = r->dev;
    if (int rc = device_bgrx(d)) return rc;
    HIP_TRY(hipMemcpyAsync(r->host, d->bgrx, (size_t)d->width * d->height * 4, hipMemcpyDeviceToHost, d->stream));
    HIP_TRY(hipStreamSynchronize(d->stream));
    // the fail-safe word after the sync: a fused-prepass timeout raised by this frame's own k_order
    // (asynchronous to rt_device_present's check) keeps the possibly wrong frame out of the video
    if (int rc = host_flag_check(d)) return rc;
    return recorder_sample(r, r->host);
}

int rt_recorder_create(rt_device d, int frame_rate, int fixed_speed, const char* path, rt_recorder* out)
{
    if (!d || !out || frame_rate <= 0) return fail(RT_ERR_INVALID, "bad recorder arguments");
    *out = nullptr;
    auto r = std::make_unique<rt_recorder_s>();
    r->dev = d;
    r->width = d->width;
    r->height = d->height;
    r->frame_rate = frame_rate;
    r->fixed_speed = fixed_speed != 0;
    r->path = path && *path ? path : "output.rgb32"; // RecorderWinAPI.cpp:80 "output.wmv"
    r->video = fopen(r->path.c_str(), "wb");
    if (!r->video) return fail(RT_ERR_STATE, "recorder: cannot open %s", r->path.c_str());
    r->index = fopen((r->path + ".txt").c_str(), "w");
    if (!r->index) {
        fclose(r->video);
        return fail(RT_ERR_STATE, "recorder: cannot open %s.txt", r->path.c_str());
    }
    fprintf(r->index, "# rgb32 (B,G,R,0) %dx%d @ %d fps; frame sample_time duration (100 ns units)\n", r->width,
            r->height, frame_rate);
    // MFFrameRateToAverageTimePerFrame(frameRate, 1): 10^7 / rate 100-ns units (exact for 25 fps)
    r->rt_start = 0;
    r->rt_duration = 10000000ull / (uint64_t)frame_rate;
    HIP_TRY(hipSetDevice(d->ordinal));
    HIP_TRY(hipHostMalloc(&r->host, (size_t)d->width * d->height * 4));
    d->recorder = r.get(); // RecorderWinAPI.cpp:199 setRecorder(this)
    *out = r.release();
    return RT_OK;
}

int rt_recorder_start(rt_recorder r)
{
    if (!r) return fail(RT_ERR_INVALID, "null recorder");
    r->recording = true; // IRecorder::start
    if (r->finalized) return fail(RT_ERR_STATE, "recorder: BeginWriting after Finalize");
    r->begun = true;
    return RT_OK;
}

int rt_recorder_stop(rt_recorder r)
{
    if (!r) return fail(RT_ERR_INVALID, "null recorder");
    r->recording = false; // IRecorder::stop, then Finalize
    if (!r->begun || r->finalized) return RT_OK;
    r->finalized = true;
    if (fflush(r->video) != 0 || fflush(r->index) != 0) return fail(RT_ERR_STATE, "recorder: flush failed");
    return RT_OK;
}

int rt_recorder_is_recording(rt_recorder r) { return r && r->recording ? 1 : 0; }

int rt_recorder_set_frame_time(rt_recorder r, float seconds)
{
    if (!r) return fail(RT_ERR_INVALID, "null recorder");
    r->frame_time = seconds;
    return RT_OK;
}

int rt_recorder_write(rt_recorder r, const void* frame, int stride)
{
    if (!r || !frame || stride < r->width * 4) return fail(RT_ERR_INVALID, "bad recorder write arguments");
    if (!r->begun || r->finalized) return fail(RT_ERR_STATE, "recorder: write outside BeginWriting/Finalize");
    // RecorderWinAPI.cpp:244-253 on host memory, as the interface receives it
    r->conv.resize((size_t)r->width * r->height);
    for (int y = 0; y < r->height; ++y) {
        const uint32_t* row = reinterpret_cast<const uint32_t*>(static_cast<const char*>(frame) + (size_t)y * stride);
        uint32_t* o = r->conv.data() + (size_t)y * r->width;
        for (int x = 0; x < r->width; ++x) {
            const uint32_t dwc = row[x];
            o[x] = (dwc & 0x0000FF00u) | (dwc & 0x000000FFu) << 16 | (dwc & 0x00FF0000u) >> 16;
        }
    }
    return recorder_sample(r, r->conv.data());
}

int rt_recorder_info(rt_recorder r, unsigned long long* frames, unsigned long long* next_sample_time,
                     unsigned long long* frame_duration)
{
    if (!r) return fail(RT_ERR_INVALID, "null recorder");
    if (frames) *frames = r->frames;
    if (next_sample_time) *next_sample_time = r->rt_start;
    if (frame_duration) *frame_duration = r->rt_duration;
    return RT_OK;
}

void rt_recorder_destroy(rt_recorder r)
{
    if (!r) return;
    if (r->recording) (void)rt_recorder_stop(r);
    delete r;
}

// ---------------------------------------------------------------------------
// VariableManager (Common/VariableManager.{h,cpp}): the live-tweak TCP protocol on a thread.
//   server -> client: [1][nlen:1][name][tlen:1][type][size:2 LE][data]   add
//                     [2]                                                 remove all
//   client -> server: [nlen:1][name][data: the variable's size]          write
// Variables are the members of cbuffers whose name starts with 'X' (XTweakable.SunDirection,
// tracing.hlsl:6-9); a write lands in the owning shader's cbuffer shadow and marks it dirty
// (ComputeDirect3D::onVariableChangedCallback, :212-216), so the next launch uploads it.
// Unlike the reference (which writes the shadow from its network thread unlocked), shadow
// writes take g_cb_mu.  bind_address defaults to the loopback interface (the reference binds
// INADDR_ANY).
namespace {
struct VarEntry {
    std::string name, type;
    int size = 0, cbuf = 0, offset = 0;
    Shader* owner = nullptr;
};
std::vector<VarEntry> g_vars; // under g_cb_mu
std::atomic<int> g_client{-1};
int g_listener = -1;
std::thread g_net;
std::atomic<bool> g_running{false};

void send_all_bytes(int fd, const void* p, size_t n)
{
    const char* c = static_cast<const char*>(p);
    while (n) {
        ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
        if (k <= 0) return;
        c += k;
        n -= (size_t)k;
    }
}

void send_variable(int fd, const VarEntry& v) // VariableManager.cpp:89-111
{
    std::vector<uint8_t> m;
    m.push_back(1);
    m.push_back((uint8_t)v.name.size());
    m.insert(m.end(), v.name.begin(), v.name.end());
    m.push_back((uint8_t)v.type.size());
    m.insert(m.end(), v.type.begin(), v.type.end());
    const uint16_t len = (uint16_t)v.size;
    m.push_back((uint8_t)(len & 0xff));
    m.push_back((uint8_t)(len >> 8));
    const uint8_t* d = v.owner->cb[v.cbuf].data() + v.offset;
    m.insert(m.end(), d, d + len);
    send_all_bytes(fd, m.data(), m.size());
}

bool read_bytes(int fd, void* out, size_t n) // VariableManager.cpp:47-72
{
    char* c = static_cast<char*>(out);
    while (n) {
        ssize_t k = ::recv(fd, c, n, 0);
        if (k <= 0) return false;
        c += k;
        n -= (size_t)k;
    }
    return true;
}

void net_loop() // VariableManager.cpp:124-188
{
    while (g_running.load()) {
        int fd = ::accept(g_listener, nullptr, nullptr);
        if (fd < 0) {
            if (!g_running.load()) break;
            continue;
        }
        {
            std::lock_guard<std::mutex> lk(g_cb_mu);
            g_client.store(fd);
            for (auto& v : g_vars) send_variable(fd, v); // sendAllVariables on connect
        }
        for (;;) {
            uint8_t nlen = 0;
            if (!read_bytes(fd, &nlen, 1)) break;
            std::string name(nlen, '\0');
            if (nlen && !read_bytes(fd, &name[0], nlen)) break;
            int size = -1;
            {
                std::lock_guard<std::mutex> lk(g_cb_mu);
                for (auto& v : g_vars)
                    if (v.name == name) {
                        size = v.size;
                        break;
                    }
            }
            if (size < 0) break; // "Var not found": the reference closes the client
            std::vector<uint8_t> data((size_t)size);
            if (size && !read_bytes(fd, data.data(), (size_t)size)) break;
            std::lock_guard<std::mutex> lk(g_cb_mu);
            for (auto& v : g_vars)
                if (v.name == name && v.size == size) {
                    memcpy(v.owner->cb[v.cbuf].data() + v.offset, data.data(), (size_t)size);
                    v.owner->cb_dirty = true;
                    if (v.cbuf == CB_NOISE) v.owner->grad_dirty = true;
                    break;
                }
        }
        {
            std::lock_guard<std::mutex> lk(g_cb_mu);
            g_client.store(-1);
        }
        ::close(fd);
    }
}
} // namespace

static void varmgr_clear() // VariableManager::clear: tell the client, drop every variable
{
    std::lock_guard<std::mutex> lk(g_cb_mu);
    const int fd = g_client.load();
    if (fd >= 0) {
        const uint8_t two = 2;
        send_all_bytes(fd, &two, 1);
    }
    g_vars.clear();
}

static void varmgr_register(Shader* s)
{
    if (!s->has_cb[CB_XTWEAK]) return;
    std::lock_guard<std::mutex> lk(g_cb_mu);
    for (auto& v : s->vars) {
        if (v->cbuf != CB_XTWEAK) continue;
        VarEntry e;
        e.name = v->name;
        e.type = v->size == 12 ? "float3" : v->size == 16 ? "float4" : v->size == 8 ? "float2" : "float";
        e.size = v->size;
        e.cbuf = v->cbuf;
        e.offset = v->offset;
        e.owner = s;
        g_vars.push_back(e);
    }
}

static void varmgr_forget(Shader* s)
{
    std::lock_guard<std::mutex> lk(g_cb_mu);
    g_vars.erase(std::remove_if(g_vars.begin(), g_vars.end(), [s](const VarEntry& e) { return e.owner == s; }),
                 g_vars.end());
}

extern "C" {

int rt_varmgr_start(int port, const char* bind_address)
{
    if (g_running.load()) return fail(RT_ERR_STATE, "variable manager already running");
    if (port <= 0 || port > 65535) port = 10666; // VariableManager.cpp:131
    int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) return fail(RT_ERR_STATE, "socket failed");
    int one = 1;
    (void)setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    if (inet_pton(AF_INET, bind_address && *bind_address ? bind_address : "127.0.0.1", &a.sin_addr) != 1) {
        ::close(fd);
        return fail(RT_ERR_INVALID, "bad bind address");
    }
    if (::bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || ::listen(fd, 5) != 0) {
        ::close(fd);
        return fail(RT_ERR_STATE, "bind/listen on port %d failed", port); // LOGERROR "bind"
    }
    g_listener = fd;
    g_running.store(true);
    g_net = std::thread(net_loop);
    return RT_OK;
}

int rt_varmgr_stop(void)
{
    if (!g_running.load()) return RT_OK;
    g_running.store(false);
    ::shutdown(g_listener, SHUT_RDWR);
    {
        std::lock_guard<std::mutex> lk(g_cb_mu);
        const int c = g_client.load();
        if (c >= 0) ::shutdown(c, SHUT_RDWR);
    }
    if (g_net.joinable()) g_net.join();
    ::close(g_listener);
    g_listener = -1;
    return RT_OK;
}

int rt_varmgr_count(void)
{
    std::lock_guard<std::mutex> lk(g_cb_mu);
    return (int)g_vars.size();
}

int rt_varmgr_register_compute(rt_compute c)
{
    if (!c) return fail(RT_ERR_INVALID, "null compute");
    Shader* s = c->new_shader ? c->new_shader : c->shader;
    if (!s) return fail(RT_ERR_STATE, "no shader");
    varmgr_forget(s);
    varmgr_register(s);
    std::lock_guard<std::mutex> lk(g_cb_mu);
    const int fd = g_client.load();
    if (fd >= 0)
        for (auto& v : g_vars)
            if (v.owner == s) send_variable(fd, v);
    return RT_OK;
}

} // extern "C"
