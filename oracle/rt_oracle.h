/*
 * rt_oracle.h -- TEST INFRASTRUCTURE, NOT PRODUCT CODE.
 *
 * CPU restatement of the reference hot path (camerarays -> setTargetDepths ->
 * tracescreen -> traceRay -> getDensity -> noise3d, shading, shadow ray, sky) of
 * MadrMan/gpgpuraytrace.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker.  The product
 * path (gpgpuraytrace_amd/) never links or calls it.
 *
 * Parity status: the noise tables are pinned by the reference's own
 * gpuraytrace/Graphics/Noise.cpp (built from /root/reference by oracle/Makefile
 * into oracle/_ref/, glibc rand) plus the MSVC-rand values recorded in SURVEY.md
 * §8c.  The HLSL itself cannot be compiled or run here (no fxc/dxc/D3D), so the
 * shader arithmetic is a restatement of the HLSL semantics with the evaluation
 * rules listed in rt_oracle.c ("parity unpinned" beyond the tables and the
 * analytic known-answer tests in tests/).
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { RO_NOMADPLAINS = 0, RO_TESTING = 1, RO_SIMPLE = 2, RO_GREENROCKS = 3 };
enum { RO_RAND_MSVC = 0, RO_RAND_GLIBC = 1 };

/* Noise tables (Graphics/Noise.cpp:39-94). */
typedef struct {
    uint8_t perm2d[128 * 128 * 4]; /* texPerm2D, texel (x,y) at (x + y*128)*4 */
    float grad[128 * 4];           /* CBNoise.permGradients[128] (xyzw, w = 0) */
    int32_t perm[128];             /* Noise::permutations */
} ro_noise;

/* Frame constants as the shaders see them (tracing.hlsl:6-22). Matrices are the
 * HLSL matrices M[row][col] (element _rc == m[(r-1)*4 + (c-1)]), i.e. the
 * DirectXMath row-vector matrices (the host uploads their transpose, which the
 * column_major cbuffer packing turns back into M). */
typedef struct {
    int32_t width, height;        /* CBPermanent.ScreenSize */
    int32_t landscape;            /* RO_* */
    int32_t aa_samples;           /* AA_SAMPLES macro: 1,2,4,8,16 */
    int32_t recording;            /* RECORDING macro (tracing.hlsl:35-41) */
    int32_t max_steps;            /* build extension: cap on primary-march iterations, 0 = unbounded (reference) */
    float eye[4];                 /* CBFrame.Eye */
    float view_inverse[16];       /* CBFrame.ViewInverse (HLSL matrix) */
    float projection[16];         /* CBPermanent.Projection (HLSL matrix) */
    float sun[3];                 /* XTweakable.SunDirection */
    int32_t row_begin, row_end, row_step; /* tracescreen rows to evaluate (CPU-baseline subsample) */
    int32_t threads;              /* OpenMP threads, <=0 = all */
    int32_t ao_samples;           /* build extension (BASELINE configs C3/C5): AO rays per primary hit, 0 = off */
} ro_frame;

typedef struct {
    uint64_t noise3d_calls;   /* every noise3d evaluation (algorithmic work unit) */
    uint64_t prepass_steps;   /* traceRay iterations in camerarays */
    uint64_t primary_steps;   /* traceRay iterations of primary rays */
    uint64_t shadow_steps;    /* traceRay iterations of shadow rays */
    uint64_t primary_rays;
    uint64_t primary_hits;    /* = shadow rays */
    uint64_t density_calls;
    uint64_t ao_steps;        /* traceRay iterations of AO rays (build extension) */
    uint64_t ao_rays;
} ro_stats;

/* ---- tables ---- */
void ro_noise_generate(ro_noise* out, uint32_t seed, int rand_kind);

/* ---- numeric primitives (exported for the GPU primitive-parity tests) ---- */
float ro_exp2(float x);
float ro_log2(float x);
float ro_pow(float x, float y);
float ro_exp(float x);
float ro_sin(float x);
float ro_cos(float x);
float ro_max(float a, float b);
float ro_min(float a, float b);
void ro_batch_unary(int op, const float* x, float* y, int64_t n);   /* op: 0 exp2 1 log2 2 exp 3 sin 4 cos 5 sqrt 6 rcp 7 rsqrt */
void ro_batch_binary(int op, const float* a, const float* b, float* y, int64_t n); /* op: 0 pow 1 max 2 min */

/* ---- hot-path functions ---- */
float ro_noise3d(const ro_noise* nz, float x, float y, float z);
void ro_noise3d_batch(const ro_noise* nz, const float* xyz, float* out, int64_t n);
float ro_get_density(const ro_noise* nz, const ro_frame* fr, float x, float y, float z);
void ro_get_density_batch(const ro_noise* nz, const ro_frame* fr, const float* xyz, float* out, int64_t n);

/* camerarays.hlsl:12-21 -> CameraResults float4[1024] */
void ro_camerarays(const ro_noise* nz, const ro_frame* fr, float* camera_results, ro_stats* st);
/* same, plus the per-cell traceRay iteration count (steps_out may be NULL) */
void ro_camerarays_steps(const ro_noise* nz, const ro_frame* fr, float* camera_results, float* steps_out,
                         ro_stats* st);
/* Terrain.cpp:356-439 -> CellDistance float2[1024] */
void ro_set_target_depths(const float* camera_results, float* cell_distance);
/* tracescreen.hlsl:50-76 for rows [row_begin,row_end) step row_step.  Outputs
 * are full-frame arrays (W*H) indexed by pixel; rows not evaluated are left
 * untouched.  Any output pointer may be NULL. */
void ro_tracescreen(const ro_noise* nz, const ro_frame* fr, const float* cell_distance,
                    float* rgba32f, uint8_t* rgba8, float* primary_steps, ro_stats* st);
/* The same with each pixel's shadow + AO march iterations in secondary_steps (W*H, may be NULL). */
void ro_tracescreen2(const ro_noise* nz, const ro_frame* fr, const float* cell_distance, float* rgba32f,
                     uint8_t* rgba8, float* primary_steps, float* secondary_steps, ro_stats* st);
/* Whole frame: prepass + depths + tracescreen. */
void ro_render_frame(const ro_noise* nz, const ro_frame* fr, float* camera_results, float* cell_distance,
                     float* rgba32f, uint8_t* rgba8, float* primary_steps, ro_stats* st);

/* Sky of n view directions (dirs xyz interleaved) under fr's Eye / SunDirection: 7 floats per
 * direction, getRayleighMieColor (mie.rgb, rayleigh.rgb; sky.hlsl:83-137) and getSpaceColor
 * (sky.hlsl:26-36).  Known-answer tests (SURVEY 8c iv) check it against a float64 restatement. */
void ro_sky(const ro_noise* nz, const ro_frame* fr, const float* dirs, float* out, int64_t n);

/* Output path: RecorderWinAPI::write's conversion of the R8G8B8A8
 * backbuffer rows (RecorderWinAPI.cpp:244-253) into MFVideoFormat_RGB32 DWORDs, and the
 * sample time stamps it sets (:264-274, rtDuration from MFFrameRateToAverageTimePerFrame,
 * :197).  frame_times[i] = Timer::getConstant() of frame i (used when !fixed_speed). */
void ro_bgrx(const uint8_t* frame, int width, int height, int stride, uint32_t* out);
void ro_sample_times(int frame_rate, int fixed_speed, const float* frame_times, int n, uint64_t* sample_time,
                     uint64_t* duration);

#ifdef __cplusplus
}
#endif
#endif
