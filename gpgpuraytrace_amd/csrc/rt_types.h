// rt_types.h -- plain-data types shared by host runtime and kernels.
#pragma once

#include <stdint.h>

enum { RT_NOMADPLAINS = 0, RT_TESTING = 1, RT_SIMPLE = 2, RT_GREENROCKS = 3, RT_NUM_LANDSCAPES = 4 };

#define RT_CAMERA_RES 32       // tracing.hlsl:1 CAMERA_SIZE, Flyby.h:6 CAMERA_VIEW_RES
#define RT_CAMERA_NEAR 0.01f   // tracing.hlsl:3
#define RT_CAMERA_FAR 5000.0f  // tracing.hlsl:4
#define RT_NP_OCTAVES 17       // nomadplains FBM: detail = max(18 - dist^0.33, 2) with dist >= 0.01 -> N <= 17
#define RT_COL_OCTAVES 20      // nomadplains colour FBM (color.hlsl:31); simple's dynamic one stays below 16

// Per-frame constant block.  Built on the host from the cbuffer shadows the
// engine writes through IShaderVariable::write (CBFrame, CBPermanent,
// XTweakable) plus compile-time derived values; uploaded once per change.
struct RtConsts {
    // CBFrame (tracing.hlsl:11-16)
    float eye[4];
    float view_inverse[16]; // HLSL matrix M[r][c] at [4r+c]
    // CBPermanent (tracing.hlsl:18-22)
    float screen[2];
    float proj11, proj22;
    float rcp_w, rcp_h;
    // XTweakable
    float sun[3];
    // tracing.hlsl:32-41 (RECORDING-dependent, folded)
    float step_factor, one_minus_step_factor, density_factor, min_limit;
    // FBM octave tables (pow(LUCAN, N) under R5)
    float np_scale[RT_NP_OCTAVES + 1];   // 1.96^N
    float np_scale_y[RT_NP_OCTAVES + 1]; // 1.96^N * 0.35
    float np_rcp[RT_NP_OCTAVES + 1];     // rcp(1.96^N)
    float np_expo;                       // 0.68f + 0.1f
    float col_scale[RT_COL_OCTAVES + 1]; // 2.03^N
    float col_rcp[RT_COL_OCTAVES + 1];
    float albedo[4];                     // landscape base colour (rgb, a)
    float shadow_color[3], one_minus_shadow[3];
    float rcp200;
    // sky.hlsl constants (folded) and per-frame eye-dependent terms
    float sky_dist_to_top, sky_start[3], sky_start_n[3], sky_depth0, sky_rcp_samples, sky_fscale, sky_sos;
    float sky_att[3], sky_mie_k[3], sky_km_esun, sky_mie_a, sky_two_g, sky_one_plus_g2;
    // antialiasing.hlsl: offsets already divided by 16
    float aa_off[16][2];
    int32_t aa_samples;
    int32_t landscape;
    int32_t max_steps; // build extension (0 = unbounded, reference semantics)
    int32_t ao_samples; // build extension: AO rays per primary hit (0 = off, reference semantics)
    int32_t width, height;
    int32_t pad[3];
};

// Frame-level statistics written by the instrumented kernels.
struct RtStats {
    unsigned long long primary_steps;
    unsigned long long shadow_steps;
    unsigned long long prepass_steps;
    unsigned long long hits;
    unsigned long long noise_calls;
    unsigned long long ao_steps;
    unsigned long long noise_waves; // wave iterations of the noise3d evaluations (not the prepass's)
};
