/*
 * skip_study.c -- DIAGNOSTIC (not product, not the checker): how many nomadplains FBM octaves a
 * march sample could leave unevaluated without changing any result bit.
 *
 * A march step needs the exact density d only (a) when d < -5 (the step multiplier
 * pow(|d + 5|, 0.35), tracing.hlsl:92) and (b) at a primary ray's last sample when it is a hit
 * (RayResult.density feeds getNormal, tracing.hlsl:107-116).  Otherwise only the sign of d and
 * whether d >= -5 matter.  After k of the n octaves of terrain.hlsl:20-24 the unevaluated rest is
 * bounded by NB * sum_{N>k} 1/S_N (|noise3d| <= NB); pushing that interval through
 * pow(|30 s + 1| * 35, 0.78), the terraces and the floor lift (terrain.hlsl:26-38) bounds d.
 * Per sample this records (n, k_need): the octaves evaluated now and the fewest that decide the
 * step.  Built by tests/tools/skip_study.py, which includes the oracle's own source.
 */
#define RO_STUDY 1
#include "../../oracle/rt_oracle.c"

#include <stdio.h>

static float g_nb = 1.0f;          /* bound on |noise3d| */
static float g_margin = 0.02f;     /* absolute margin in density units (+ relative below) */

typedef struct { uint8_t* v; int64_t n, cap; } buf8;
static void b_push(buf8* b, uint8_t x, uint8_t y)
{
    if (b->n + 2 > b->cap) {
        b->cap = b->cap ? b->cap * 2 : 256;
        b->v = (uint8_t*)realloc(b->v, (size_t)b->cap);
    }
    b->v[b->n++] = x;
    b->v[b->n++] = y;
}

static buf8* g_pix = NULL;        /* primary samples per pixel */
static int64_t g_npix = 0;
#define ST_THREADS 256
static buf8 g_long[4][ST_THREADS];  /* kind 0 prepass, 1 shadow, 2 AO, 3 unused */
static double g_check_err = 0.0;   /* |d recomputed - d| (sanity) */

void st_config(float nb, float margin, int64_t npix)
{
    g_nb = nb;
    g_margin = margin;
    for (int64_t i = 0; i < g_npix; ++i) free(g_pix[i].v);
    free(g_pix);
    g_npix = npix;
    g_pix = (buf8*)calloc((size_t)npix, sizeof(buf8));
    for (int k = 0; k < 4; ++k)
        for (int t = 0; t < ST_THREADS; ++t) { free(g_long[k][t].v); g_long[k][t].v = NULL; g_long[k][t].n = g_long[k][t].cap = 0; }
    g_check_err = 0.0;
}

int64_t st_pixel_len(int64_t i) { return g_pix[i].n; }
const uint8_t* st_pixel_data(int64_t i) { return g_pix[i].v; }
int64_t st_long_len(int kind, int t) { return g_long[kind][t].n; }
const uint8_t* st_long_data(int kind, int t) { return g_long[kind][t].v; }
double st_check_err(void) { return g_check_err; }

static void ro_study_sample(ctx* c, f3 p, float d, int calcfog, int skiprefine, int max_steps, int iters,
                            float dist, float enddist, float step, float lastStep)
{
    (void)dist; (void)enddist; (void)lastStep;
    if (c->fr->landscape != RO_NOMADPLAINS) return;
    ctx cc = *c; /* keep the caller's counters */
    float dd = ro_max(len3(sub3(p, cc.eye)), 0.01f);
    float detail = ro_max(18.0f - ro_pow(dd, 0.33f), 2.0f);
    f3 p1 = scale3(p, 0.4f);
    f3 q0 = scale3(p1, 0.006f);
    float sk[24], rc[24];
    int n = 0;
    float s = 0.0f;
    sk[0] = 0.0f;
    for (int N = 1; (float)N <= detail; ++N) {
        float S = fbm_scale(1.96f, N);
        float nv = noise3d(&cc, q0.x * S, q0.y * (S * 0.35f), q0.z * S);
        s = fmaf(nv, rcp(S), s);
        sk[N] = s;
        rc[N] = rcp(S);
        n = N;
    }
    float steep = sat((noise3d(&cc, p1.x * 0.007138f, p1.z * 0.007138f, 0.0f) - 0.2f) * 6.0f) * 7.5f;
    float floorsize = steep * 1.8f, T = 0.0f;
    const float hs[4] = {13.0f, 16.0f, 19.0f, 22.0f};
    for (int i = 0; i < 4; ++i) { float t = sat((p1.y - hs[i]) * steep); T += (t * t) * floorsize; }
    float L = ro_pow(sat((-p1.y + 10.0f) * 1.6f), 1.5f) * 19.0f;
    /* sanity: the full sum reproduces d */
    {
        float sp = ro_pow(fabsf(fmaf(s, 30.0f, 1.0f)) * 35.0f, 0.78f);
        double e = fabs((double)(-p.y + (sp - T + L)) - (double)d);
        if (e > g_check_err) {
#pragma omp critical
            if (e > g_check_err) g_check_err = e;
        }
    }
    int kind; /* 0 primary, 1 prepass, 2 shadow, 3 AO */
    if (!skiprefine) kind = 0;
    else if (calcfog) kind = 2;
    else kind = (enddist > 1000.0f) ? 1 : 3;
    int final_if_hit = !(step * 0.3f > cc.min_limit) || (max_steps > 0 && iters >= max_steps);
    int k_need = n;
    for (int k = 0; k <= n; ++k) {
        double tail = 0.0;
        for (int N = k + 1; N <= n; ++N) tail += (double)rc[N];
        tail *= (double)g_nb;
        double slo = (double)sk[k] - tail, shi = (double)sk[k] + tail;
        double alo = 30.0 * slo + 1.0, ahi = 30.0 * shi + 1.0;
        double mlo, mhi;
        if (alo <= 0.0 && ahi >= 0.0) { mlo = 0.0; mhi = fmax(-alo, ahi); }
        else { mlo = fmin(fabs(alo), fabs(ahi)); mhi = fmax(fabs(alo), fabs(ahi)); }
        double plo = pow(mlo * 35.0, 0.78), phi = pow(mhi * 35.0, 0.78);
        double m = (double)g_margin + 1e-4 * phi;
        double dlo = -(double)p.y + plo - T + L - m, dhi = -(double)p.y + phi - T + L + m;
        int band = dhi < 0.0 && dlo > -5.0;
        int pos = dlo > 0.0 && (skiprefine || !final_if_hit);
        if (band || pos) { k_need = k; break; }
    }
    if (kind == 0) {
        if (c->study_pixel >= 0 && c->study_pixel < g_npix) b_push(&g_pix[c->study_pixel], (uint8_t)n, (uint8_t)k_need);
    } else {
        int t = 0;
#ifdef _OPENMP
        t = omp_get_thread_num();
#endif
        if (t < ST_THREADS) b_push(&g_long[kind - 1][t], (uint8_t)n, (uint8_t)k_need);
    }
}
