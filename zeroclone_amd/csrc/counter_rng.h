// Counter-based and small-state random generators for the paths that are NOT tied to the
// reference's CPython MT19937 stream (the PUCT extension's Dirichlet noise and sampling, and
// the Connect4 search's Philox rollout mode).  Both are pinned in tests/ by their published
// known-answer vectors (Random123 philox4x32-10; xoshiro128** from state {1, 2, 3, 4}).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace zc {
namespace {

// Philox4x32-10 (Salmon et al., SC'11): 10 rounds of the 4x32 Philox S-box over counter c
// with key k (Weyl-incremented per round).
__device__ __forceinline__ uint4 philox(uint4 c, uint2 k) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.x, p1 = (uint64_t)0xCD9E8D57u * c.z;
        const uint32_t h0 = (uint32_t)(p0 >> 32), l0 = (uint32_t)p0, h1 = (uint32_t)(p1 >> 32), l1 = (uint32_t)p1;
        c = make_uint4(h1 ^ c.y ^ k.x, l1, h0 ^ c.w ^ k.y, l0);
        k.x += 0x9E3779B9u;
        k.y += 0xBB67AE85u;
    }
    return c;
}

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

// xoshiro128** (Blackman & Vigna): one 32-bit draw per step from 128 bits of lane state.
struct Xoshiro128 {
    uint32_t s0, s1, s2, s3;
    __device__ __forceinline__ uint32_t next() {
        const uint32_t r = rotl32(s1 * 5u, 7) * 9u;
        const uint32_t t = s1 << 9;
        s2 ^= s0;
        s3 ^= s1;
        s1 ^= s2;
        s0 ^= s3;
        s2 ^= t;
        s3 = rotl32(s3, 11);
        return r;
    }
};

}  // namespace
}  // namespace zc
