// puct_common.h — pieces shared by the PUCT searches (chess_puct.hip, c4_puct.hip; SURVEY
// §8 a21, no reference counterpart): the counter-based Dirichlet draws of the root noise and
// wave-wide reductions.  Included by exactly those translation units.
#pragma once
#include <hip/hip_runtime.h>

#include "counter_rng.h"

namespace zc {
namespace {

__device__ __forceinline__ float u01(uint32_t x) { return ((float)(x >> 8) + 0.5f) * (1.0f / 16777216.0f); }

// Gamma(alpha, 1) by Marsaglia-Tsang (alpha < 1 via Gamma(alpha + 1) * U^(1/alpha)); the
// draws of (game, move j) in the game's search number sno come from Philox counters
// (j, attempt | sno << 6, game, tag).
__device__ float gamma_draw(float alpha, uint2 key, uint32_t game, uint32_t j, uint32_t sno) {
    const bool boost = alpha < 1.0f;
    const float a = boost ? alpha + 1.0f : alpha;
    const float d = a - 1.0f / 3.0f, cc = 1.0f / sqrtf(9.0f * d);
    float g = 0.0f;
    for (uint32_t att = 0; att < 64; ++att) {
        const uint4 r = philox(make_uint4(j, att | (sno << 6), game, 0x6A09E667u), key);
        // Box-Muller normal from two uniforms
        const float z = sqrtf(-2.0f * logf(u01(r.x))) * cospif(2.0f * u01(r.y));
        const float v1 = 1.0f + cc * z;
        if (v1 <= 0.0f) continue;
        const float v = v1 * v1 * v1, u = u01(r.z);
        if (logf(u) < 0.5f * z * z + d - d * v + d * logf(v)) {
            g = d * v;
            if (boost) g *= powf(u01(r.w), 1.0f / alpha);
            break;
        }
    }
    return g;
}

// The game's search number: the counter word of its noise and temperature sample.
template <class Params>
__device__ __forceinline__ uint32_t search_number(const Params &p, int gl) {
    return p.search_no ? (uint32_t)__builtin_amdgcn_readfirstlane(p.search_no[gl]) : 0u;
}

__device__ __forceinline__ double wave_sum_d(double x) {
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    return x;
}
__device__ __forceinline__ float wave_max_f(float x) {
    for (int o = 32; o > 0; o >>= 1) x = fmaxf(x, __shfl_xor(x, o));
    return x;
}
__device__ __forceinline__ float wave_sum_f(float x) {
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    return x;
}

}  // namespace
}  // namespace zc
