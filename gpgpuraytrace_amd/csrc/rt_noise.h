// rt_noise.h -- host-side noise-table generator (the engine's Noise::generate,
// Graphics/Noise.cpp:39-94): a 128-entry permutation shuffled with the CRT's
// rand(), the 128x128 RGBA8 perm2D lattice texture and the 128 x float4
// gradient table (Ken Perlin's 16 improved-noise gradients).
#pragma once

#include <stdint.h>

namespace rt_noise {

enum { RAND_MSVC = 0, RAND_GLIBC = 1 };

// perm2d: 128*128*4 bytes (texel (x,y) at (x + y*128)*4), grad: 128*4 floats.
void generate(uint32_t seed, int rand_kind, uint8_t* perm2d, float* grad);

} // namespace rt_noise
