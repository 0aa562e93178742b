// rt_noise.cpp -- see rt_noise.h.
#include "rt_noise.h"

namespace rt_noise {
namespace {

// The two CRT rand() implementations the engine can meet: MSVC's 15-bit LCG
// (the reference ships for Windows) and glibc's additive-feedback TYPE_3 generator.
class CrtRand {
public:
    CrtRand(uint32_t seed, int kind) : kind_(kind)
    {
        if (kind_ == RAND_MSVC) {
            lcg_ = seed;
            return;
        }
        int32_t r0 = (int32_t)(seed == 0 ? 1 : seed);
        uint32_t s[344];
        int64_t prev = r0;
        s[0] = (uint32_t)r0;
        for (int i = 1; i < 31; ++i) {
            int64_t w = (16807LL * prev) % 2147483647LL;
            if (w < 0) w += 2147483647LL;
            s[i] = (uint32_t)w;
            prev = w;
        }
        for (int i = 31; i < 34; ++i) s[i] = s[i - 31];
        for (int i = 34; i < 344; ++i) s[i] = s[i - 31] + s[i - 3];
        for (int i = 0; i < 34; ++i) ring_[i] = s[310 + i];
    }

    int next()
    {
        if (kind_ == RAND_MSVC) {
            lcg_ = lcg_ * 214013u + 2531011u;
            return (int)((lcg_ >> 16) & 0x7fffu);
        }
        uint32_t v = ring_[(pos_ + 3) % 34] + ring_[(pos_ + 31) % 34];
        ring_[pos_] = v;
        pos_ = (pos_ + 1) % 34;
        return (int)(v >> 1);
    }

private:
    int kind_;
    uint32_t lcg_ = 0;
    uint32_t ring_[34] = {};
    int pos_ = 0;
};

// Perlin's improved-noise gradient set, in the engine's order.
const float kGrad[16][3] = {{1, 1, 0}, {-1, 1, 0}, {1, -1, 0}, {-1, -1, 0}, {1, 0, 1}, {-1, 0, 1},
                            {1, 0, -1}, {-1, 0, -1}, {0, 1, 1}, {0, -1, 1}, {0, 1, -1}, {0, -1, -1},
                            {1, 1, 0}, {0, -1, 1}, {-1, 1, 0}, {0, -1, -1}};

} // namespace

void generate(uint32_t seed, int rand_kind, uint8_t* perm2d, float* grad)
{
    const int N = 128;
    int perm[N];
    for (int i = 0; i < N; ++i) perm[i] = i;
    CrtRand rng(seed, rand_kind);
    for (int i = 0; i < N; ++i) {
        int j = rng.next() % N;
        int t = perm[i];
        perm[i] = perm[j];
        perm[j] = t;
    }
    auto P = [&](int i) { return perm[i % N]; };
    for (int y = 0; y < N; ++y) {
        for (int x = 0; x < N; ++x) {
            uint8_t* texel = perm2d + (x + y * N) * 4;
            int a = P(x) + y, b = P(x + 1) + y;
            texel[0] = (uint8_t)P(a);
            texel[1] = (uint8_t)P(a + 1);
            texel[2] = (uint8_t)P(b);
            texel[3] = (uint8_t)P(b + 1);
        }
    }
    for (int i = 0; i < N; ++i) {
        const float* g = kGrad[perm[i] % 16];
        grad[4 * i + 0] = g[0];
        grad[4 * i + 1] = g[1];
        grad[4 * i + 2] = g[2];
        grad[4 * i + 3] = 0.0f;
    }
}

} // namespace rt_noise
