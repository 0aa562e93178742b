/*
 * prepass_band_study.c -- DIAGNOSTIC (not product, not the checker): can speculative multi-sample
 * marching shorten the camerarays prepass rays?  A march sample whose density d lies in [-5, 0]
 * makes the next step the plain unit step (stepmult = 1 + pow(0, df) = 1, tracing.hlsl:92), so the
 * next sample's position is known before d is; elsewhere it depends on d.  This records, per prepass
 * ray (camerarays.hlsl:12-21 through the oracle's trace_ray), which samples are in that band.
 * Built and driven by tests/tools/prepass_band_study.py, which includes the oracle's own source.
 */
#define RO_STUDY 1
#include "../../oracle/rt_oracle.c"

static uint8_t g_flags[1 << 22];
static int64_t g_n = 0;
static int32_t g_start[2048];
static int g_rays = 0;
int64_t pp_n(void) { return g_n; }
const uint8_t* pp_flags(void) { return g_flags; }
int pp_rays(void) { return g_rays; }
const int32_t* pp_starts(void) { return g_start; }
void pp_reset(void) { g_n = 0; g_rays = 0; }

static void ro_study_sample(ctx* c, f3 p, float d, int calcfog, int skiprefine, int max_steps, int iters,
                            float dist, float enddist, float step, float lastStep)
{
    (void)c; (void)p; (void)max_steps; (void)dist; (void)step; (void)lastStep;
    if (!(skiprefine && !calcfog && enddist > 1000.0f)) return; /* the prepass's marches only */
    if (iters == 1 && g_rays < 2048) g_start[g_rays++] = (int32_t)g_n;
    if (g_n < (int64_t)sizeof(g_flags)) g_flags[g_n++] = (uint8_t)((d >= -5.0f && d <= 0.0f) ? 1 : 0);
}
