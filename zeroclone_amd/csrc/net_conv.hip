// net_conv.hip — the value network's residual tower on gfx950 matrix cores.
//
// ValueNetwork (models/chess_value/network.py:24-45) with BatchNorm folded into the
// convolutions (zeroclone_amd/nets.py) is 17 conv3x3 layers of 128 channels on tiny boards
// (8x8 chess, 6x7 Connect4) plus a pooled linear head.  Each layer is an implicit GEMM
//   D[cout][pixel] = sum_{tap, cin} Wt[tap][cout][cin] * X[pixel shifted by tap][cin]
// with M = 128 output channels, N = the pixels of a tile of boards, K = 9 taps x cin, on
// v_mfma_f32_32x32x16_f16.  Activations are NHWC fp16 (a pixel's channels contiguous).
//
// Two forms (bit-identical results; tools/ab_conv.py): the default half-tile kernel below
// (128-pixel tiles, 70 KB of LDS, two workgroups per CU) and this one (ZC_CONV_IMPL=tile).
// One workgroup = 4 waves = one tile of BPW boards (<= 256 pixels; 4 chess boards, 6
// Connect4 boards).  The tile's input pixels are staged ONCE in LDS (rows padded by 16 B so
// the 32 lanes reading 32 pixels hit different banks); the 9 shifted views of a tap are
// just different LDS rows (zero outside the board), so no im2col ever touches HBM.  The
// weights of one tap (128 x cin) sit in one of two LDS buffers; the next tap's weights are
// fetched into registers while the current tap computes.  Wave w owns all 128 channels x
// 64 pixels (4 x 2 MFMA tiles): per 16-deep k-step it reads 4 weight and 2 activation
// fragments (ds_read_b128) for 8 MFMAs, 0.75 KB of LDS per MFMA.  The epilogue adds the
// folded-BN bias, the residual and ReLU in fp32 and stores 4 channels (8 B) per lane per
// row group.
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "zc_internal.h"

#ifdef ZC_CONV_STAMP
// diagnostic build only: per wave of conv3x3_stream_kernel, {HW_ID, XCC_ID, start, tile
// staged, main loop done, end} (s_memtime), read by tools/conv_phases.py
__device__ uint64_t g_conv_stamp[1 << 20];
extern "C" int zc_debug_conv_stamps(void *host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_conv_stamp), (size_t)n * sizeof(uint64_t)) == hipSuccess ? 0 : -1;
}
#define CSTAMP(k) const uint64_t cst_##k = __builtin_amdgcn_s_memtime()
#else
#define CSTAMP(k)
#endif

namespace zc {
namespace {
#ifndef ZC_TOWER_STAMP
#define ZC_TOWER_STAMP 0  // diagnostic build: per-phase s_memtime cycles of the fused tower's waves
#endif
#if ZC_TOWER_STAMP
__device__ unsigned long long g_tower_stamp[4];  // MFMA loop, epilogue, barrier wait, whole kernel
#endif

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef float f16x __attribute__((ext_vector_type(16)));
typedef float f4x __attribute__((ext_vector_type(4)));

constexpr int kCout = 128;
constexpr int kTilePix = 256;

template <int H, int W, int BPW, int CIN>
__global__ __launch_bounds__(256) void conv3x3_kernel(int nboards, const _Float16 *__restrict__ in,
                                                      const _Float16 *__restrict__ wt, const float *__restrict__ bias,
                                                      const _Float16 *__restrict__ res, _Float16 *__restrict__ out,
                                                      int relu) {
    constexpr int HW = H * W;
    constexpr int PIX = BPW * HW;
    static_assert(PIX <= kTilePix, "tile too large");
    constexpr int LD = CIN + 8;                // padded LDS row, halves
    constexpr int C8 = CIN / 8;
    constexpr int WCH = kCout * C8 / 256;      // 16-byte weight chunks per thread per tap
    constexpr int NI = kTilePix * C8 / 256;    // 16-byte input chunks per thread
    extern __shared__ __attribute__((aligned(16))) _Float16 lds[];
    _Float16 *const sin = lds;                         // [kTilePix + 1][LD]; the last row is zero
    _Float16 *const swb = lds + (kTilePix + 1) * LD;  // [2][kCout][LD]: weights of even / odd taps

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int b0 = blockIdx.x * BPW;
    const int npix = min(BPW, nboards - b0) * HW;
    const h8 zero = {0, 0, 0, 0, 0, 0, 0, 0};
    h8 wpre[WCH];
    {
        // stage the tile's input and tap 0's weights: every load in flight before the first
        // LDS store
        h8 v[NI];
#pragma unroll
        for (int q = 0; q < NI; ++q) {
            const int i = tid + q * 256, row = i / C8, c8 = i - row * C8;
            v[q] = row < npix ? *(const h8 *)(in + ((size_t)b0 * HW + row) * CIN + c8 * 8) : zero;
        }
#pragma unroll
        for (int q = 0; q < WCH; ++q) {
            const int i = tid + q * 256, row = i / C8, c8 = i - row * C8;
            wpre[q] = *(const h8 *)(wt + (size_t)row * CIN + c8 * 8);
        }
#pragma unroll
        for (int q = 0; q < NI; ++q) {
            const int i = tid + q * 256, row = i / C8, c8 = i - row * C8;
            *(h8 *)(sin + row * LD + c8 * 8) = v[q];
        }
        if (tid < C8) *(h8 *)(sin + kTilePix * LD + tid * 8) = zero;  // the off-board row
#pragma unroll
        for (int q = 0; q < WCH; ++q) {
            const int i = tid + q * 256, row = i / C8, c8 = i - row * C8;
            *(h8 *)(swb + row * LD + c8 * 8) = wpre[q];
        }
    }

    // wave w: all 128 output channels x pixels [64w, 64w+64) (2 tiles of 32)
    const int r = lane & 31, hh = lane >> 5;
    int pb[2], py[2], px[2];
    bool pv[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const int P = wave * 64 + t * 32 + r;
        pv[t] = P < npix;
        pb[t] = P / HW;
        const int rem = P - pb[t] * HW;
        py[t] = rem / W;
        px[t] = rem - py[t] * W;
    }
    f16x acc[4][2];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int k = 0; k < 16; ++k) acc[m][t][k] = 0.0f;

    for (int tap = 0; tap < 9; ++tap) {
        __syncthreads();  // this tap's weights (and, at tap 0, the input tile) are in LDS
        if (tap + 1 < 9) {
#pragma unroll
            for (int q = 0; q < WCH; ++q) {
                const int i = tid + q * 256, row = i / C8, c8 = i - row * C8;
                wpre[q] = *(const h8 *)(wt + ((size_t)(tap + 1) * kCout + row) * CIN + c8 * 8);
            }
        }
        const _Float16 *sw = swb + (tap & 1) * kCout * LD;
        const int dy = tap / 3 - 1, dx = tap % 3 - 1;
        const _Float16 *xb[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int sy = py[t] + dy, sx = px[t] + dx;
            const bool sv = pv[t] && (unsigned)sy < (unsigned)H && (unsigned)sx < (unsigned)W;
            xb[t] = sin + (sv ? pb[t] * HW + sy * W + sx : kTilePix) * LD + hh * 8;  // off-board: zeros
        }
        const _Float16 *wa = sw + r * LD + hh * 8;
        // software-pipelined k loop: the fragments of step kc+1 are read from LDS while the
        // 8 MFMAs of step kc run (one wave per SIMD has nobody else to hide LDS latency)
        h8 a[4], x[2], an[4], xn[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) x[t] = *(const h8 *)(xb[t]);
#pragma unroll
        for (int m = 0; m < 4; ++m) a[m] = *(const h8 *)(wa + m * 32 * LD);
#pragma unroll
        for (int kc = 0; kc < CIN / 16; ++kc) {
            if (kc + 1 < CIN / 16) {
#pragma unroll
                for (int t = 0; t < 2; ++t) xn[t] = *(const h8 *)(xb[t] + (kc + 1) * 16);
#pragma unroll
                for (int m = 0; m < 4; ++m) an[m] = *(const h8 *)(wa + m * 32 * LD + (kc + 1) * 16);
            }
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int t = 0; t < 2; ++t)
                    acc[m][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[m], x[t], acc[m][t], 0, 0, 0);
            if (kc + 1 < CIN / 16) {
                // interleave: one LDS read of step kc+1 behind each MFMA of step kc
#pragma unroll
                for (int q = 0; q < 6; ++q) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
                }
                __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);      // the last 2 MFMAs
#pragma unroll
                for (int m = 0; m < 4; ++m) a[m] = an[m];
#pragma unroll
                for (int t = 0; t < 2; ++t) x[t] = xn[t];
            }
        }
        if (tap + 1 < 9) {
            _Float16 *dst = swb + ((tap + 1) & 1) * kCout * LD;
#pragma unroll
            for (int q = 0; q < WCH; ++q) {
                const int i = tid + q * 256, row = i / C8, c8 = i - row * C8;
                *(h8 *)(dst + row * LD + c8 * 8) = wpre[q];
            }
        }
    }

    // epilogue: D[cout][pixel], pixel = lane & 31, cout rows (reg&3) + 8*(reg>>2) + 4*hh.
    // All residual loads are issued before any is used.
    h4 rv[2][4][4];
    if (res) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int P = min(wave * 64 + t * 32 + r, max(npix - 1, 0));
            const size_t orow = ((size_t)b0 * HW + P) * kCout;
#pragma unroll
            for (int m = 0; m < 4; ++m)
#pragma unroll
                for (int g = 0; g < 4; ++g) rv[t][m][g] = *(const h4 *)(res + orow + m * 32 + 8 * g + 4 * hh);
        }
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const int P = wave * 64 + t * 32 + r;
        const size_t orow = ((size_t)b0 * HW + P) * kCout;
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int co = m * 32 + 8 * g + 4 * hh;
                const float4 bb = *(const float4 *)(bias + co);
                float v0 = acc[m][t][4 * g + 0] + bb.x, v1 = acc[m][t][4 * g + 1] + bb.y;
                float v2 = acc[m][t][4 * g + 2] + bb.z, v3 = acc[m][t][4 * g + 3] + bb.w;
                if (res) {
                    v0 += (float)rv[t][m][g][0];
                    v1 += (float)rv[t][m][g][1];
                    v2 += (float)rv[t][m][g][2];
                    v3 += (float)rv[t][m][g][3];
                }
                if (relu) {
                    v0 = fmaxf(v0, 0.0f);
                    v1 = fmaxf(v1, 0.0f);
                    v2 = fmaxf(v2, 0.0f);
                    v3 = fmaxf(v3, 0.0f);
                }
                h4 o;
                o[0] = (_Float16)v0;
                o[1] = (_Float16)v1;
                o[2] = (_Float16)v2;
                o[3] = (_Float16)v3;
                if (P < npix) *(h4 *)(out + orow + co) = o;
            }
    }
}

// Half-tile form: 128-pixel tiles with ONE weight buffer, 70 KB of LDS, so two workgroups
// share a CU and one's staging, barriers and epilogue run under the other's MFMAs.  Its
// epilogue goes through LDS so that the residual loads and output stores cover whole
// 256-byte pixel rows (3-7 % per layer over per-fragment 16-byte pieces).  Wave w
// owns output channels [64 (w & 1), +64) x pixels [64 (w >> 1), +64) (2 x 2 MFMA tiles).
// Per tap: the next tap's weights are fetched into registers during the MFMAs, then
// barrier -> store -> barrier.  Same accumulation order as conv3x3_kernel (bit-identical).
constexpr int kHalfPix = 128;
constexpr size_t kHalfEpiBytes = (size_t)kHalfPix * (kCout + 4) * sizeof(float);  // the epilogue's fp32 tile

template <int H, int W, int BPW, int CIN>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) void conv3x3_half_kernel(int nboards, const _Float16 *__restrict__ in,
                                                              const _Float16 *__restrict__ wt,
                                                              const float *__restrict__ bias,
                                                              const _Float16 *__restrict__ res,
                                                              _Float16 *__restrict__ out, int relu) {
    constexpr int HW = H * W;
    constexpr int PIX = BPW * HW;
    static_assert(PIX <= kHalfPix, "tile too large");
    constexpr int LD = CIN + 8;
    constexpr int C8 = CIN / 8;
    constexpr int WCH = kCout * C8 / 256;
    constexpr int NI = kHalfPix * C8 / 256;
    extern __shared__ __attribute__((aligned(16))) _Float16 lds[];
    _Float16 *const sin = lds;                         // [kHalfPix + 1][LD]; the last row is zero
    _Float16 *const sw = lds + (kHalfPix + 1) * LD;   // [kCout][LD]: the current tap's weights

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int b0 = blockIdx.x * BPW;
    const int npix = min(BPW, nboards - b0) * HW;
    const h8 zero = {0, 0, 0, 0, 0, 0, 0, 0};
    h8 wpre[WCH];
    {
        h8 v[NI];
        const _Float16 *src = in + (size_t)b0 * HW * CIN;
#pragma unroll
        for (int q = 0; q < NI; ++q) {
            const int i = tid + q * 256, row = i / C8, c8 = i - row * C8;
            const h8 t = *(const h8 *)(src + min(row, npix - 1) * CIN + c8 * 8);
            v[q] = row < npix ? t : zero;
        }
#pragma unroll
        for (int q = 0; q < WCH; ++q) {
            const int i = tid + q * 256, row = i / C8, c8 = i - row * C8;
            wpre[q] = *(const h8 *)(wt + (size_t)row * CIN + c8 * 8);
        }
#pragma unroll
        for (int q = 0; q < NI; ++q) {
            const int i = tid + q * 256, row = i / C8, c8 = i - row * C8;
            *(h8 *)(sin + row * LD + c8 * 8) = v[q];
        }
        if (tid < C8) *(h8 *)(sin + kHalfPix * LD + tid * 8) = zero;  // the off-board row
#pragma unroll
        for (int q = 0; q < WCH; ++q) {
            const int i = tid + q * 256, row = i / C8, c8 = i - row * C8;
            *(h8 *)(sw + row * LD + c8 * 8) = wpre[q];
        }
    }

    const int r = lane & 31, hh = lane >> 5;
    const int m0 = 2 * (wave & 1), p0 = 64 * (wave >> 1);
    int pb[2], py[2], px[2];
    bool pv[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const int P = p0 + t * 32 + r;
        pv[t] = P < npix;
        pb[t] = P / HW;
        const int rem = P - pb[t] * HW;
        py[t] = rem / W;
        px[t] = rem - py[t] * W;
    }
    f16x acc[2][2];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int k = 0; k < 16; ++k) acc[m][t][k] = 0.0f;

    for (int tap = 0; tap < 9; ++tap) {
        __syncthreads();  // this tap's weights (and, at tap 0, the input tile) are in LDS
        if (tap + 1 < 9) {
#pragma unroll
            for (int q = 0; q < WCH; ++q) {
                const int i = tid + q * 256, row = i / C8, c8 = i - row * C8;
                wpre[q] = *(const h8 *)(wt + ((size_t)(tap + 1) * kCout + row) * CIN + c8 * 8);
            }
        }
        const int dy = tap / 3 - 1, dx = tap % 3 - 1;
        const _Float16 *xb[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int sy = py[t] + dy, sx = px[t] + dx;
            const bool sv = pv[t] && (unsigned)sy < (unsigned)H && (unsigned)sx < (unsigned)W;
            xb[t] = sin + (sv ? pb[t] * HW + sy * W + sx : kHalfPix) * LD + hh * 8;  // off-board: zeros
        }
        const _Float16 *wa = sw + (m0 * 32 + r) * LD + hh * 8;
        h8 a[2], x[2], an[2], xn[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) x[t] = *(const h8 *)(xb[t]);
#pragma unroll
        for (int m = 0; m < 2; ++m) a[m] = *(const h8 *)(wa + m * 32 * LD);
#pragma unroll
        for (int kc = 0; kc < CIN / 16; ++kc) {
            if (kc + 1 < CIN / 16) {
#pragma unroll
                for (int t = 0; t < 2; ++t) xn[t] = *(const h8 *)(xb[t] + (kc + 1) * 16);
#pragma unroll
                for (int m = 0; m < 2; ++m) an[m] = *(const h8 *)(wa + m * 32 * LD + (kc + 1) * 16);
            }
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int t = 0; t < 2; ++t)
                    acc[m][t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[m], x[t], acc[m][t], 0, 0, 0);
            if (kc + 1 < CIN / 16) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
                }
#pragma unroll
                for (int m = 0; m < 2; ++m) a[m] = an[m];
#pragma unroll
                for (int t = 0; t < 2; ++t) x[t] = xn[t];
            }
        }
        if (tap + 1 < 9) {
            __syncthreads();  // every wave is done with this tap's weights
#pragma unroll
            for (int q = 0; q < WCH; ++q) {
                const int i = tid + q * 256, row = i / C8, c8 = i - row * C8;
                *(h8 *)(sw + row * LD + c8 * 8) = wpre[q];
            }
        }
    }

    // epilogue through LDS: the fp32 tile is transposed to [pixel][cout] (rows padded by 4
    // floats) so that bias, residual, ReLU and the fp16 store run on whole 256-byte output
    // rows, 16 lanes per pixel — coalesced residual loads and stores instead of 16-byte
    // pieces of 32 different rows per instruction.  Same fp32 operations in the same order.
    constexpr int SL = kCout + 4;
    // (the launch sizes the LDS for this tile too: kHalfEpiBytes)
    float *const sacc = (float *)lds;
    __syncthreads();  // every wave is done with the input tile and the weights
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int P = p0 + t * 32 + r, co = (m0 + m) * 32 + 8 * g + 4 * hh;
                *(float4 *)(sacc + P * SL + co) =
                    make_float4(acc[m][t][4 * g + 0], acc[m][t][4 * g + 1], acc[m][t][4 * g + 2], acc[m][t][4 * g + 3]);
            }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kHalfPix * (kCout / 8) / 256; ++q) {
        const int i = tid + q * 256, P = i >> 4, c0 = (i & 15) * 8;
        if (P < npix) {
            const size_t o = ((size_t)b0 * HW + P) * kCout + c0;
            h8 rv8;
            if (res) rv8 = *(const h8 *)(res + o);
            const float4 a0 = *(const float4 *)(sacc + P * SL + c0), a1 = *(const float4 *)(sacc + P * SL + c0 + 4);
            const float4 b0v = *(const float4 *)(bias + c0), b1v = *(const float4 *)(bias + c0 + 4);
            float v[8] = {a0.x + b0v.x, a0.y + b0v.y, a0.z + b0v.z, a0.w + b0v.w,
                          a1.x + b1v.x, a1.y + b1v.y, a1.z + b1v.z, a1.w + b1v.w};
            h8 ov;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                if (res) v[e] += (float)rv8[e];
                if (relu) v[e] = fmaxf(v[e], 0.0f);
                ov[e] = (_Float16)v[e];
            }
            *(h8 *)(out + o) = ov;
        }
    }
}


// ---- the swizzled activation layout (the 16x16x32 form, EPI = 3): unpadded 256-byte rows
// (128 halfs, sixteen 16-byte chunks) whose chunk c sits at c ^ hsw(row).  hsw depends on
// row & 7 only (so a zero row, 8 of them, stands for any row of its class) and was chosen
// (an exhaustive search over the XOR-linear maps) so that every LDS access of the tower is
// conflict-free on gfx950's banking (MI355X_MICROARCH §LDS):
//   - the MFMA B operand (ds_read_b128, lane (pixel l & 15, k-chunk l >> 4), rows shifted by
//     any tap offset): each lane group's 16 chunks land on 16 distinct bank quads;
//   - the epilogue, in 8-consecutive-channel form (permlane16_swap, as tower_epilogue16_swap):
//     the residual ds_read_b128 and the ds_write_b128 (8 aligned rows, one chunk) alike;
//   - the value head's and the output copy's row reads, the input staging's stores.
// Only the policy 1x1 conv's 32-pixel reads stay 2-way (once per tower).  The padded layout it
// replaces (144-half rows) left the epilogue's ds_write_b64 4-way and its residual reads 2-way.
constexpr int kSwzLD = kCout;
__device__ __forceinline__ int hsw(int row) { return (int)((0xAE9D7340u >> ((row & 7) << 2)) & 15u); }
__device__ __forceinline__ int swz(int row, int chunk) { return row * kSwzLD + ((chunk ^ hsw(row)) << 3); }
template <int NT> constexpr size_t tower_lds_swz() { return (size_t)(64 * NT + 8) * kSwzLD * sizeof(_Float16); }

// One layer's MFMA loop in the 16x16x32 form: each wave its 32 output channels (two 16-row
// M tiles) x the tile's pixels as NN 16-pixel N tiles, k-steps of 32 channels.  Lane l takes
// pixel l & 15 of each N tile and k-chunk q = l >> 4; the weight fragments come from the same
// packed stream as tower_mfma's (lane l of M tile m reads the 8 halfs of fragment row
// 16 m + (l & 15), k 8 q .. 8 q + 7: wa already holds the lane's offset), one tap ahead.
#ifndef ZC_TOWER_DIAG
#define ZC_TOWER_DIAG 0  // diagnostic builds (wrong outputs, timing only; tools/tower_diag_libs.sh): 1 = no weight
                         // reloads, 2 = no B reloads, 4 = every layer reads layer 1's weights, 8 = every weight
                         // load of a wave reads its first fragment (L1-resident)
#endif
template <int H, int W, int NN, int KC, int KCN, int LD, int ZERO, int ZR, int NA>
__device__ __forceinline__ void tower_mfma16(const _Float16 *lds, int src, const _Float16 *wa, const _Float16 *wn,
                                             h8 (&a)[NA], int l16, const int (&pyx)[NN], int q,
                                             f4x (&acc)[2][NN]) {
    constexpr int J = KC / 2, JN = KCN / 2;
    auto rows = [&](int tap, const _Float16 *(&xb)[NN]) {
        const int dy = tap / 3 - 1, dx = tap % 3 - 1;
#pragma unroll
        for (int n = 0; n < NN; ++n) {
            const int sy = (pyx[n] >> 8) + dy, sx = (pyx[n] & 255) + dx;
            const bool sv = (unsigned)sy < (unsigned)H && (unsigned)sx < (unsigned)W;
            const int row = l16 + (n * 16 + dy * W + dx);  // pixel n * 16 + l16, shifted by the tap
            xb[n] = lds + (sv ? src + row : ZERO + (row & (ZR - 1))) * LD + q * 8;
        }
    };
    const _Float16 *xb[NN];
    rows(0, xb);
    h8 x[NN], xn[NN];
#pragma unroll
    for (int n = 0; n < NN; ++n) x[n] = *(const h8 *)(xb[n]);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
        const _Float16 *xbn[NN];
        if (tap + 1 < 9) rows(tap + 1, xbn);
#pragma unroll
        for (int j = 0; j < J; ++j) {
            if (ZC_TOWER_DIAG & 2) {
#pragma unroll
                for (int n = 0; n < NN; ++n) xn[n] = x[n];
            } else if (j + 1 < J) {
#pragma unroll
                for (int n = 0; n < NN; ++n) xn[n] = *(const h8 *)(xb[n] + (j + 1) * 32);
            } else if (tap + 1 < 9) {
#pragma unroll
                for (int n = 0; n < NN; ++n) xn[n] = *(const h8 *)(xbn[n]);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int n = 0; n < NN; ++n)
#pragma unroll
                for (int m = 0; m < 2; ++m)
                    acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[2 * j + m], x[n], acc[m][n], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int m = 0; m < 2; ++m) {
                if (ZC_TOWER_DIAG & 1) break;
                if (ZC_TOWER_DIAG & 8) a[2 * j + m] = *(const h8 *)(wa + (size_t)(__builtin_amdgcn_readfirstlane(m * 0)));
                else if (tap + 1 < 9) a[2 * j + m] = *(const h8 *)(wa + (size_t)((tap + 1) * KC + 2 * j) * 2048 + m * 128);
                else if (JN == J && wn) a[2 * j + m] = *(const h8 *)(wn + (size_t)(2 * j) * 2048 + m * 128);
            }
#pragma unroll
            for (int n = 0; n < NN; ++n) x[n] = xn[n];
        }
        if (tap + 1 < 9) {
#pragma unroll
            for (int n = 0; n < NN; ++n) xb[n] = xbn[n];
        }
    }
    if (JN != J && wn && !(ZC_TOWER_DIAG & 1)) {
#pragma unroll
        for (int j = 0; j < JN; ++j)
#pragma unroll
            for (int m = 0; m < 2; ++m) a[2 * j + m] = *(const h8 *)(wn + (size_t)(2 * j) * 2048 + m * 128);
    }
}

// tower_mfma16 on the swizzled layout: the same MFMAs in the same order; lane (pixel l16,
// k-chunk q) of N tile n reads chunk 4 j + q of its row at (4 j + q) ^ hsw(row) — the row's
// chunk offset for j = 0 XOR 64 j bytes (hsw of the tap-shifted row does not depend on n).
template <int H, int W, int NN, int KC, int KCN, int ZERO, int NA>
__device__ __forceinline__ void tower_mfma16_swz(const _Float16 *lds, int src, const _Float16 *wa, const _Float16 *wn,
                                                 h8 (&a)[NA], int l16, const int (&pyx)[NN], int q,
                                                 f4x (&acc)[2][NN]) {
    constexpr int J = KC / 2, JN = KCN / 2;
    auto rows = [&](int tap, int (&xo)[NN]) {
        const int dy = tap / 3 - 1, dx = tap % 3 - 1;
        const int qh = (q ^ hsw(l16 + dy * W + dx)) << 3;  // the same for every N tile (16 n = 0 mod 8)
#pragma unroll
        for (int n = 0; n < NN; ++n) {
            const int sy = (pyx[n] >> 8) + dy, sx = (pyx[n] & 255) + dx;
            const bool sv = (unsigned)sy < (unsigned)H && (unsigned)sx < (unsigned)W;
            const int row = l16 + (n * 16 + dy * W + dx);
            xo[n] = (sv ? src + row : ZERO + (row & 7)) * kSwzLD + qh;
        }
    };
    int xo[NN];
    rows(0, xo);
    h8 x[NN], xn[NN];
#pragma unroll
    for (int n = 0; n < NN; ++n) x[n] = *(const h8 *)(lds + xo[n]);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
        int xon[NN];
        if (tap + 1 < 9) rows(tap + 1, xon);
#pragma unroll
        for (int j = 0; j < J; ++j) {
            if (j + 1 < J) {
#pragma unroll
                for (int n = 0; n < NN; ++n) xn[n] = *(const h8 *)(lds + (xo[n] ^ ((j + 1) * 32)));
            } else if (tap + 1 < 9) {
#pragma unroll
                for (int n = 0; n < NN; ++n) xn[n] = *(const h8 *)(lds + xon[n]);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int n = 0; n < NN; ++n)
#pragma unroll
                for (int m = 0; m < 2; ++m)
                    acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[2 * j + m], x[n], acc[m][n], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int m = 0; m < 2; ++m) {
                if (tap + 1 < 9) a[2 * j + m] = *(const h8 *)(wa + (size_t)((tap + 1) * KC + 2 * j) * 2048 + m * 128);
                else if (JN == J && wn) a[2 * j + m] = *(const h8 *)(wn + (size_t)(2 * j) * 2048 + m * 128);
            }
#pragma unroll
            for (int n = 0; n < NN; ++n) x[n] = xn[n];
        }
        if (tap + 1 < 9) {
#pragma unroll
            for (int n = 0; n < NN; ++n) xo[n] = xon[n];
        }
    }
    if (JN != J && wn) {
#pragma unroll
        for (int j = 0; j < JN; ++j)
#pragma unroll
            for (int m = 0; m < 2; ++m) a[2 * j + m] = *(const h8 *)(wn + (size_t)(2 * j) * 2048 + m * 128);
    }
}

// Streamed-weight form (zc_net_conv3x3_packed_async): wave w owns output channels
// [32 w, +32) x all 128 pixels of the tile (4 MFMA tiles).  The weights are pre-packed so
// that every A fragment (32 channels x 16 k of one tap) is one contiguous 1-KB piece, 16 B
// per lane in MFMA operand order (pack_conv_weight_kernel); each wave streams its own
// fragments from L2 straight into registers one tap ahead, so the LDS holds only the input
// tile and the main loop has no barrier and no weight restaging.  WPE = waves per SIMD:
// at 3 the fp32 epilogue tile goes through LDS in two 64-pixel halves, so three
// workgroups fit a CU.  Same accumulation order as the other forms (bit-identical).
template <int H, int W, int BPH, int CIN, int WPE, int MF = 32>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void conv3x3_stream_kernel(
    int nboards, const _Float16 *__restrict__ in, const _Float16 *__restrict__ wp, const float *__restrict__ bias,
    const _Float16 *__restrict__ res, _Float16 *__restrict__ out, int relu) {
    constexpr int HW = H * W;
    constexpr int PIX = BPH * HW;
    static_assert(PIX <= kHalfPix, "tile too large");
    // MF = 16: the 16x16x32 MFMA form (tower_mfma16; rows of CIN + 16 halfs, 8 (mod 64) dwords x
    // an odd number, keep its operand reads conflict-free)
    constexpr int LD = MF == 16 ? CIN + 16 : CIN + 8;
    constexpr int C8 = CIN / 8;
    constexpr int KC = CIN / 16;
    constexpr int NI = kHalfPix * C8 / 256;
    CSTAMP(0);
    extern __shared__ __attribute__((aligned(16))) _Float16 lds[];
    // [kHalfPix + 16][LD]: the tile, then 16 zero rows.  An off-board pixel reads the zero
    // row in the bank class of the row it would have read, so the 16 lanes of a read group
    // stay on 16 different bank quads (one shared zero row cost a 2-way conflict at edges).
    _Float16 *const sin = lds;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int b0 = blockIdx.x * BPH;
    const int npix = min(BPH, nboards - b0) * HW;
    const h8 zero = {0, 0, 0, 0, 0, 0, 0, 0};
    const int r = lane & 31, hh = lane >> 5;
    const int l16 = lane & 15, q4 = lane >> 4;
    // fragment (tap, kc) of this wave: wp + ((tap * KC + kc) * 4 + wave) * 512 + lane * 8 (MF = 16:
    // lane l reads row 16 m + (l & 15), k-chunk l >> 4 of the same stream)
    const _Float16 *const wa =
        MF == 16 ? wp + (size_t)wave * 512 + (size_t)((q4 & 1) * 32 + l16) * 8 + (size_t)(q4 >> 1) * 2048
                 : wp + (size_t)wave * 512 + lane * 8;
    h8 a[KC];
    if constexpr (MF == 16) {
#pragma unroll
        for (int j = 0; j < KC / 2; ++j)
#pragma unroll
            for (int m = 0; m < 2; ++m) a[2 * j + m] = *(const h8 *)(wa + (size_t)(2 * j) * 2048 + m * 128);
    } else {
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) a[kc] = *(const h8 *)(wa + (size_t)kc * 2048);
    }
    {
        h8 v[NI];
        const _Float16 *src = in + (size_t)b0 * HW * CIN;
#pragma unroll
        for (int q = 0; q < NI; ++q) {
            const int i = tid + q * 256, row = i / C8, c8 = i - row * C8;
            const h8 t = *(const h8 *)(src + min(row, npix - 1) * CIN + c8 * 8);
            v[q] = row < npix ? t : zero;
        }
#pragma unroll
        for (int q = 0; q < NI; ++q) {
            const int i = tid + q * 256, row = i / C8, c8 = i - row * C8;
            *(h8 *)(sin + row * LD + c8 * 8) = v[q];
        }
        for (int z = tid; z < 16 * C8; z += 256) *(h8 *)(sin + (kHalfPix + z / C8) * LD + (z % C8) * 8) = zero;
    }
    f16x acc[MF == 16 ? 1 : 4];
    f4x acc16[2][MF == 16 ? 8 : 1];
    if constexpr (MF == 16) {
        int pyx16[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            const int P = t * 16 + l16;
            const int pb = P / HW, rem = P - pb * HW, py = rem / W;
            pyx16[t] = (P < npix ? py << 8 : 64 << 8) | (rem - py * W);
#pragma unroll
            for (int m = 0; m < 2; ++m) acc16[m][t] = f4x{0.0f, 0.0f, 0.0f, 0.0f};
        }
        __syncthreads();  // the input tile is in LDS
        tower_mfma16<H, W, 8, KC, KC, LD, kHalfPix, 16>(lds, 0, wa, nullptr, a, l16, pyx16, q4, acc16);
    }
    if constexpr (MF != 16) {
    // per MFMA pixel tile t: the pixel's LDS row and its (y, x) packed as y << 8 | x (a pixel
    // beyond the tile gets y = 64: every shifted view of it is off the board)
    int prow[4], pyx[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        const int P = t * 32 + r;
        const int pb = P / HW, rem = P - pb * HW, py = rem / W;
        prow[t] = P;
        pyx[t] = (P < npix ? py << 8 : 64 << 8) | (rem - py * W);
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int k = 0; k < 16; ++k) acc[t][k] = 0.0f;
    __syncthreads();  // the input tile is in LDS
    CSTAMP(1);

#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
        const int dy = tap / 3 - 1, dx = tap % 3 - 1;
        const _Float16 *xb[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int sy = (pyx[t] >> 8) + dy, sx = (pyx[t] & 255) + dx;
            const bool sv = (unsigned)sy < (unsigned)H && (unsigned)sx < (unsigned)W;
            const int row = prow[t] + dy * W + dx;
            xb[t] = sin + (sv ? row : kHalfPix + (row & 15)) * LD + hh * 8;
        }
        h8 x[4], xn[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) x[t] = *(const h8 *)(xb[t]);
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
            // the next k-step's four fragment reads go out before this step's MFMAs, pinned
            // there, so they land under the MFMAs (left alone, the compiler pairs every read
            // with its consumer and waits on it)
            if (kc + 1 < KC) {
#pragma unroll
                for (int t = 0; t < 4; ++t) xn[t] = *(const h8 *)(xb[t] + (kc + 1) * 16);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[kc], x[t], acc[t], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            // a ring: this fragment's register now fetches the same k-step of the next tap
            if (tap + 1 < 9) a[kc] = *(const h8 *)(wa + (size_t)((tap + 1) * KC + kc) * 2048);
            if (kc + 1 < KC) {
#pragma unroll
                for (int t = 0; t < 4; ++t) x[t] = xn[t];
            }
        }
    }

    }
    // epilogue through LDS (as in the half form): fp32 [pixel][cout] rows, then bias,
    // residual, ReLU and the fp16 store on whole 256-byte output rows; NP pixels per pass
    constexpr int SL = kCout + 4;
    constexpr int NP = WPE >= 3 ? 64 : 128;
    CSTAMP(2);
    float *const sacc = (float *)lds;
#pragma unroll
    for (int h0 = 0; h0 < kHalfPix; h0 += NP) {
        __syncthreads();  // the input tile / the previous pass is no longer read
        if constexpr (MF == 16) {
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                if (t * 16 < h0 || t * 16 >= h0 + NP) continue;
#pragma unroll
                for (int m = 0; m < 2; ++m) {
                    const int P = t * 16 + l16 - h0, co = wave * 32 + 16 * m + 4 * q4;
                    *(float4 *)(sacc + P * SL + co) = make_float4(acc16[m][t][0], acc16[m][t][1], acc16[m][t][2],
                                                                  acc16[m][t][3]);
                }
            }
        } else {
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                if (t * 32 < h0 || t * 32 >= h0 + NP) continue;
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int P = t * 32 + r - h0, co = wave * 32 + 8 * g + 4 * hh;
                    *(float4 *)(sacc + P * SL + co) =
                        make_float4(acc[t][4 * g + 0], acc[t][4 * g + 1], acc[t][4 * g + 2], acc[t][4 * g + 3]);
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < NP * (kCout / 8) / 256; ++q) {
            const int i = tid + q * 256, Pl = i >> 4, c0 = (i & 15) * 8, P = h0 + Pl;
            if (P < npix) {
                const size_t o = ((size_t)b0 * HW + P) * kCout + c0;
                h8 rv8;
                if (res) rv8 = *(const h8 *)(res + o);
                const float4 a0 = *(const float4 *)(sacc + Pl * SL + c0), a1 = *(const float4 *)(sacc + Pl * SL + c0 + 4);
                const float4 b0v = *(const float4 *)(bias + c0), b1v = *(const float4 *)(bias + c0 + 4);
                float v[8] = {a0.x + b0v.x, a0.y + b0v.y, a0.z + b0v.z, a0.w + b0v.w,
                              a1.x + b1v.x, a1.y + b1v.y, a1.z + b1v.z, a1.w + b1v.w};
                h8 ov;
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    if (res) v[e] += (float)rv8[e];
                    if (relu) v[e] = fmaxf(v[e], 0.0f);
                    ov[e] = (_Float16)v[e];
                }
                *(h8 *)(out + o) = ov;
            }
        }
    }
#ifdef ZC_CONV_STAMP
    CSTAMP(3);
    if (lane == 0 && (blockIdx.x * 4 + wave) * 6 + 6 <= (1 << 20)) {
        uint64_t *d = g_conv_stamp + (size_t)(blockIdx.x * 4 + wave) * 6;
        d[0] = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));   // HW_ID
        d[1] = __builtin_amdgcn_s_getreg(20 | (0 << 6) | (15 << 11));  // XCC_ID
        d[2] = cst_0;
        d[3] = cst_1;
        d[4] = cst_2;
        d[5] = cst_3;
    }
#endif
}

// Fused tower (zc_net_tower_async): the stem and every residual block of one tile of boards
// in ONE workgroup, the activations resident in LDS from the input planes to the tower's
// output — no HBM round trip between layers (a layer-by-layer launch moves ~1.6 GB of
// activations per 32768 boards per layer and stalls each workgroup on its load and store
// phases).  The MFMA loop is the streamed-weight form's (each wave its 32 output channels x
// the tile's 128 pixels, fragments from L2 one tap ahead, activation reads one k-step ahead);
// the epilogue goes straight from the accumulators into the next layer's input buffer:
//   layer 0 (stem)        buf1 (input planes) -> buf0
//   layer 2k+1 (conv1)    buf0 (x)            -> buf1 (h)
//   layer 2k+2 (conv2)    buf1 (h)            -> buf0 (x := relu(conv + bias + x), in place:
//                          each output pixel reads only its own residual, and no wave reads x
//                          during conv2)
// with one barrier per layer.  LDS: buf0 [128][136], 16 zero rows, buf1 [128][136] (73,984
// B; two workgroups per CU).  Off-board taps of either buffer read the shared zero rows, in
// the bank class of the row they would have read.  Every value is computed with the same
// operations in the same order as the layer-by-layer packed form: bit-identical outputs
// (tests/test_gpu_net.py).
constexpr int kTowerLD = kCout + 8;
// NT pixel MFMA tiles (32 pixels each) per wave; PG pixel groups of 4 waves per workgroup
// (the 4 waves of a group split the 128 output channels; the groups split the pixels): buffer
// rows TP = 32 NT PG.  With PG = 2 the two waves that own the same output channels load the
// same weight fragments at about the same time, so the second load is served by the CU's
// vector L1 instead of L2.
// MF = 16 (the 16x16x32 MFMA form, tower_mfma16): rows of 144 halfs (72 dwords: the operand's
// four 16-byte k-chunks per pixel row land on distinct banks in every ds_read_b128 lane group)
// and 8 zero rows (the bank class of a row is its index mod 8)
template <int MF> constexpr int tower_ld() { return MF == 16 ? kCout + 16 : kTowerLD; }
template <int MF> constexpr int tower_zr() { return MF == 16 ? 8 : 16; }
template <int NT, int PG = 1> constexpr int tower_zero() { return 32 * NT * PG; }       // first zero row
template <int NT, int PG = 1, int MF = 32> constexpr int tower_buf1() {                 // buf1's first row
    return 32 * NT * PG + tower_zr<MF>();
}
template <int NT, int PG = 1, int MF = 32> constexpr size_t tower_lds() {
    return (size_t)(64 * NT * PG + tower_zr<MF>()) * tower_ld<MF>() * sizeof(_Float16);
}


// One layer's MFMA loop: acc[t] += sum over taps and k of W * X (X from the LDS buffer at
// row `src`).  a[0..KC) holds the layer's tap-0 fragments on entry; on exit it holds the
// next layer's (KCN fragments from wn, when wn != nullptr and KCN == KC: in the ring at the
// last tap; otherwise loaded after the loop).
template <int H, int W, int NT, int KC, int KCN, int PG = 1>
__device__ __forceinline__ void tower_mfma(const _Float16 *lds, int src, const _Float16 *wa, const _Float16 *wn,
                                           h8 (&a)[8], const int (&prow)[NT], const int (&pyx)[NT], int hh,
                                           f16x (&acc)[NT]) {
    // tap `tap`'s activation rows of the 4 pixel tiles (off-board: a zero row)
    auto rows = [&](int tap, const _Float16 *(&xb)[NT]) {
        const int dy = tap / 3 - 1, dx = tap % 3 - 1;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int sy = (pyx[t] >> 8) + dy, sx = (pyx[t] & 255) + dx;
            const bool sv = (unsigned)sy < (unsigned)H && (unsigned)sx < (unsigned)W;
            const int row = prow[t] + dy * W + dx;
            xb[t] = lds + (sv ? src + row : tower_zero<NT, PG>() + (row & 15)) * kTowerLD + hh * 8;
        }
    };
    const _Float16 *xb[NT];
    rows(0, xb);
    h8 x[NT], xn[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) x[t] = *(const h8 *)(xb[t]);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
        // the next tap's rows: its first fragments are read during this tap's last k-step
        const _Float16 *xbn[NT];
        if (tap + 1 < 9) rows(tap + 1, xbn);
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
            if (kc + 1 < KC) {
#pragma unroll
                for (int t = 0; t < NT; ++t) xn[t] = *(const h8 *)(xb[t] + (kc + 1) * 16);
            } else if (tap + 1 < 9) {
#pragma unroll
                for (int t = 0; t < NT; ++t) xn[t] = *(const h8 *)(xbn[t]);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[kc], x[t], acc[t], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            if (tap + 1 < 9) a[kc] = *(const h8 *)(wa + (size_t)((tap + 1) * KC + kc) * 2048);
            else if (KCN == KC && wn) a[kc] = *(const h8 *)(wn + (size_t)kc * 2048);
#pragma unroll
            for (int t = 0; t < NT; ++t) x[t] = xn[t];
        }
        if (tap + 1 < 9) {
#pragma unroll
            for (int t = 0; t < NT; ++t) xb[t] = xbn[t];
        }
    }
    if (KCN != KC && wn) {
#pragma unroll
        for (int kc = 0; kc < KCN; ++kc) a[kc] = *(const h8 *)(wn + (size_t)kc * 2048);
    }
}

// acc + bias (+ the residual already in dst), ReLU, fp16 -> dst rows (the stream form's
// epilogue arithmetic, per lane: 4 channels x one pixel per store)
template <int NT>
__device__ __forceinline__ void tower_epilogue(_Float16 *dst, const float4 (&bv)[4], bool res, int npix, int wave,
                                               int r, int hh, const f16x (&acc)[NT], int pbase = 0) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const int P = pbase + t * 32 + r;
        if (P >= npix) continue;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int co = wave * 32 + 8 * g + 4 * hh;
            h4 *const o = (h4 *)(dst + P * kTowerLD + co);
            float v[4] = {acc[t][4 * g + 0] + bv[g].x, acc[t][4 * g + 1] + bv[g].y, acc[t][4 * g + 2] + bv[g].z,
                          acc[t][4 * g + 3] + bv[g].w};
            if (res) {
                const h4 rv = *o;
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] += (float)rv[e];
            }
            h4 ov;
#pragma unroll
            for (int e = 0; e < 4; ++e) ov[e] = (_Float16)fmaxf(v[e], 0.0f);
            *o = ov;
        }
    }
}

// tower_epilogue for the 16x16x32 form: lane (pixel l & 15 of N tile n, q = l >> 4) holds
// channels wave * 32 + 16 m + 4 q .. + 3; the same per-element arithmetic
template <int NN>
__device__ __forceinline__ void tower_epilogue16(_Float16 *dst, const float4 (&bv)[2], bool res, int npix, int wave,
                                                 int l16, int q, const f4x (&acc)[2][NN]) {
    constexpr int LD = tower_ld<16>();
#pragma unroll
    for (int n = 0; n < NN; ++n) {
        const int P = n * 16 + l16;
        if (P >= npix) continue;
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            h4 *const o = (h4 *)(dst + P * LD + wave * 32 + 16 * m + 4 * q);
            float v[4] = {acc[m][n][0] + bv[m].x, acc[m][n][1] + bv[m].y, acc[m][n][2] + bv[m].z,
                          acc[m][n][3] + bv[m].w};
            if (res) {
                const h4 rv = *o;
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] += (float)rv[e];
            }
            h4 ov;
#pragma unroll
            for (int e = 0; e < 4; ++e) ov[e] = (_Float16)fmaxf(v[e], 0.0f);
            *o = ov;
        }
    }
}

// tower_epilogue16 with the residual layer's reads issued together (one wait for all 16
// instead of a read-wait-add chain per 4 channels), no per-tile branch when the tile is full
// and the residual switch resolved per layer (RES): the same per-element arithmetic.
template <int NN, bool RES, bool CHECK>
__device__ __forceinline__ void tower_epilogue16_batch(_Float16 *dst, const float4 (&bv)[2], int npix, int wave,
                                                       int l16, int q, const f4x (&acc)[2][NN]) {
    constexpr int LD = tower_ld<16>();
    _Float16 *const base = dst + l16 * LD + wave * 32 + 4 * q;
    h4 rv[2][NN];
    if constexpr (RES) {
#pragma unroll
        for (int n = 0; n < NN; ++n) {
            const int P = CHECK ? min(n * 16 + l16, npix - 1) - l16 : n * 16;  // a valid row to read
#pragma unroll
            for (int m = 0; m < 2; ++m) rv[m][n] = *(const h4 *)(base + P * LD + 16 * m);
        }
    }
#pragma unroll
    for (int n = 0; n < NN; ++n) {
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            float v[4] = {acc[m][n][0] + bv[m].x, acc[m][n][1] + bv[m].y, acc[m][n][2] + bv[m].z,
                          acc[m][n][3] + bv[m].w};
            if constexpr (RES) {
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] += (float)rv[m][n][e];
            }
            h4 ov;
#pragma unroll
            for (int e = 0; e < 4; ++e) ov[e] = (_Float16)fmaxf(v[e], 0.0f);
            if (!CHECK || n * 16 + l16 < npix) *(h4 *)(base + n * 16 * LD + 16 * m) = ov;
        }
    }
}

template <int NN>
__device__ __forceinline__ void tower_epilogue16b(_Float16 *dst, const float4 (&bv)[2], bool res, int npix, int wave,
                                                  int l16, int q, const f4x (&acc)[2][NN]) {
    if (npix >= NN * 16) {
        if (res) tower_epilogue16_batch<NN, true, false>(dst, bv, npix, wave, l16, q, acc);
        else tower_epilogue16_batch<NN, false, false>(dst, bv, npix, wave, l16, q, acc);
    } else {
        if (res) tower_epilogue16_batch<NN, true, true>(dst, bv, npix, wave, l16, q, acc);
        else tower_epilogue16_batch<NN, false, true>(dst, bv, npix, wave, l16, q, acc);
    }
}

// tower_epilogue16 with whole 16-byte stores: the per-element arithmetic in the MFMA layout
// (residual read per 4 channels, as there), then one v_permlane16_swap per dword hands lane
// (pixel, q) the 8 consecutive channels wave * 32 + 16 (q & 1) + 8 (q >> 1) .. + 7 of its
// pixel (rows 0 / 2 keep M tile 0 and take the next row's, rows 1 / 3 the M tile 1 halves):
// 8 ds_write_b128 per layer and wave instead of 16 ds_write_b64, 2-way instead of 4-way on
// the 72-dword rows.  Every lane takes part in the swaps; only the store is predicated.
template <int NN>
__device__ __forceinline__ void tower_epilogue16_swap(_Float16 *dst, const float4 (&bv)[2], bool res, int npix,
                                                      int wave, int l16, int q, const f4x (&acc)[2][NN]) {
    constexpr int LD = tower_ld<16>();
    const int co8 = wave * 32 + 16 * (q & 1) + 8 * (q >> 1);
    h4 rv[2][NN];  // the residual, every read issued before the first use
    if (res) {
#pragma unroll
        for (int n = 0; n < NN; ++n)
#pragma unroll
            for (int m = 0; m < 2; ++m)
                rv[m][n] = *(const h4 *)(dst + min(n * 16 + l16, npix - 1) * LD + wave * 32 + 16 * m + 4 * q);
    }
#pragma unroll
    for (int n = 0; n < NN; ++n) {
        const int P = n * 16 + l16;
        uint32_t pk[2][2];
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            float v[4] = {acc[m][n][0] + bv[m].x, acc[m][n][1] + bv[m].y, acc[m][n][2] + bv[m].z,
                          acc[m][n][3] + bv[m].w};
            if (res) {
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] += (float)rv[m][n][e];
            }
            h4 ov;
#pragma unroll
            for (int e = 0; e < 4; ++e) ov[e] = (_Float16)fmaxf(v[e], 0.0f);
            __builtin_memcpy(pk[m], &ov, 8);
        }
        const auto s0 = __builtin_amdgcn_permlane16_swap(pk[0][0], pk[1][0], false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(pk[0][1], pk[1][1], false, false);
        if (P < npix) *(uint4 *)(dst + P * LD + co8) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
    }
}

// The epilogue on the swizzled layout: the fp32 accumulators are first handed over by
// v_permlane16_swap (4 per N tile) so that lane (pixel l16, q) holds the 8 consecutive
// channels co8 = wave * 32 + 16 (q & 1) + 8 (q >> 1) .. + 7 of its pixel — one chunk — and the
// residual read, + bias, + residual, ReLU, fp16 and the store are whole 16-byte chunks
// (conflict-free, see hsw).  Per element the arithmetic of tower_epilogue16: bit-identical.
// bv8: this lane's 8 bias values (channels co8 ..).
template <int NN, bool RES, bool CHECK>
__device__ __forceinline__ void tower_epilogue16_swz(_Float16 *dst, const float (&bv8)[8], int npix, int wave, int l16,
                                                     int q, const f4x (&acc)[2][NN]) {
    const int c8 = wave * 4 + 2 * (q & 1) + (q >> 1);  // the lane's chunk (co8 / 8)
    h8 rv[NN];
    if constexpr (RES) {
#pragma unroll
        for (int n = 0; n < NN; ++n) {
            const int P = CHECK ? min(n * 16 + l16, npix - 1) : n * 16 + l16;  // a valid row to read
            rv[n] = *(const h8 *)(dst + swz(P, c8));
        }
    }
#pragma unroll
    for (int n = 0; n < NN; ++n) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[0][n][e]), __float_as_uint(acc[1][n][e]),
                                                             false, false);
            v[e] = __uint_as_float(sw[0]);
            v[4 + e] = __uint_as_float(sw[1]);
        }
        h8 ov;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            float y = v[e] + bv8[e];
            if constexpr (RES) y += (float)rv[n][e];
            ov[e] = (_Float16)fmaxf(y, 0.0f);
        }
        const int P = n * 16 + l16;
        if (!CHECK || P < npix) *(h8 *)(dst + swz(P, c8)) = ov;
    }
}

template <int NN>
__device__ __forceinline__ void tower_epilogue16s(_Float16 *dst, const float (&bv8)[8], bool res, int npix, int wave,
                                                  int l16, int q, const f4x (&acc)[2][NN]) {
    if (npix >= NN * 16) {
        if (res) tower_epilogue16_swz<NN, true, false>(dst, bv8, npix, wave, l16, q, acc);
        else tower_epilogue16_swz<NN, false, false>(dst, bv8, npix, wave, l16, q, acc);
    } else {
        if (res) tower_epilogue16_swz<NN, true, true>(dst, bv8, npix, wave, l16, q, acc);
        else tower_epilogue16_swz<NN, false, true>(dst, bv8, npix, wave, l16, q, acc);
    }
}

// The policy head's 1x1 conv (PolicyValueNetwork.policy[0..2]: 128 -> 32 channels, BN folded,
// ReLU) on the tower's output while it is still in LDS (tower_policy): pw = the folded
// weights as 32x32x16 MFMA A fragments [8 k-steps][64 lanes][8] (lane = output channel
// lane % 32, k = 16 kc + 8 (lane / 32) + e), pb [32] fp32 bias; out [n * H * W][32] fp16.
struct TowerPolicy {
    const _Float16 *pw;  // [mblocks][8 k-steps][64 lanes][8] fp16 A fragments
    const float *pb;     // [32 * mblocks]
    _Float16 *out;       // [n][hw][32 * mblocks]
    int head_raw;        // test switch (ZC_HEAD_RAW=1): the value head writes its pre-tanh sum
    int mblocks;         // output channels / 32 (1: the 128 -> 32 conv; 2: the 128 -> 64 logit conv)
    int relu;            // ReLU on the outputs (the linear-head network's conv) or not (logits)
};

template <int H, int W, int BPH, int CIN0, int NT, int WPE, int PG = 1, int MF = 32, int EPI = 0>
__global__ __launch_bounds__(256 * PG) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void tower_kernel(
    int nboards, int nconv, const _Float16 *__restrict__ in, const _Float16 *__restrict__ wall,
    const float *__restrict__ ball, _Float16 *__restrict__ out, const float *__restrict__ fcw, float fcb,
    double *__restrict__ values, TowerPolicy pol) {
    constexpr int HW = H * W;
    static_assert(BPH * HW <= 32 * NT * PG, "tile too large");
    static_assert(MF == 32 || (MF == 16 && PG == 1), "the 16x16x32 form has one pixel group");
    constexpr int TP = 32 * NT * PG;
    constexpr int NTH = 256 * PG;   // threads
    constexpr int KC0 = CIN0 / 16;
    constexpr bool SWZ = EPI == 3;  // the swizzled layout (hsw): unpadded rows, chunk c at c ^ hsw(row)
    static_assert(!SWZ || (MF == 16 && PG == 1), "the swizzled layout is the 16x16x32 form's");
    constexpr int LD = SWZ ? kSwzLD : tower_ld<MF>(), ZR = tower_zr<MF>(), BUF1 = tower_buf1<NT, PG, MF>();
    constexpr int NP = MF == 16 ? 2 * NT : NT;  // pixel tiles per wave (16 or 32 pixels)
    constexpr size_t kW0 = (size_t)9 * CIN0 * kCout, kW = (size_t)9 * kCout * kCout;  // halfs per layer
    extern __shared__ __attribute__((aligned(16))) _Float16 lds[];
    const int tid = threadIdx.x, lane = tid & 63, wave = (tid >> 6) & 3, pg = tid >> 8;
    const int pbase = pg * 32 * NT;   // this wave's first pixel of the tile
    const int b0 = blockIdx.x * BPH;
    const int npix = min(BPH, nboards - b0) * HW;
    const h8 zero = {0, 0, 0, 0, 0, 0, 0, 0};
    const int r = lane & 31, hh = lane >> 5;
    const int l16 = lane & 15, q4 = lane >> 4;  // the 16x16x32 form's pixel / k-chunk
    // this wave's fragments, layer 0 (MF = 16: lane l reads row 16 m + (l & 15), k-chunk l >> 4
    // of the same packed stream)
    const _Float16 *const wl0 =
        MF == 16 ? wall + (size_t)wave * 512 + (size_t)((q4 & 1) * 32 + l16) * 8 + (size_t)(q4 >> 1) * 2048
                 : wall + (size_t)wave * 512 + lane * 8;
    h8 a[8];
    if constexpr (MF == 16) {
#pragma unroll
        for (int j = 0; j < KC0 / 2; ++j)
#pragma unroll
            for (int m = 0; m < 2; ++m) a[2 * j + m] = *(const h8 *)(wl0 + (size_t)(2 * j) * 2048 + m * 128);
    } else {
#pragma unroll
        for (int kc = 0; kc < KC0; ++kc) a[kc] = *(const h8 *)(wl0 + (size_t)kc * 2048);
    }
    {
        constexpr int C8 = CIN0 / 8;
        const _Float16 *src = in + (size_t)b0 * HW * CIN0;
#pragma unroll
        for (int q = 0; q < (TP * C8 + NTH - 1) / NTH; ++q) {
            const int i = tid + q * NTH, row = i / C8, c8 = i - row * C8;
            if (row >= TP) break;
            const h8 t = *(const h8 *)(src + min(row, npix - 1) * CIN0 + c8 * 8);
            *(h8 *)(lds + (SWZ ? swz(BUF1 + row, c8) : (BUF1 + row) * LD + c8 * 8)) = row < npix ? t : zero;
        }
        for (int z = tid; z < ZR * LD / 8; z += NTH)
            *(h8 *)(lds + tower_zero<NT, PG>() * LD + z * 8) = zero;
    }
    int prow[NP], pyx[NP];
#pragma unroll
    for (int t = 0; t < NP; ++t) {
        const int P = MF == 16 ? t * 16 + l16 : pbase + t * 32 + r;
        const int pb = P / HW, rem = P - pb * HW, py = rem / W;
        prow[t] = P;
        pyx[t] = (P < npix ? py << 8 : 64 << 8) | (rem - py * W);
    }
    __syncthreads();  // the input tile and the zero rows are in LDS
#if ZC_TOWER_STAMP
    uint64_t st_mfma = 0, st_epi = 0, st_bar = 0;
    const uint64_t st_k0 = __builtin_amdgcn_s_memtime();
#endif
    // layer l: src -> dst, then a barrier (dst complete before layer l+1 reads it; dst was
    // layer l-1's src, which every wave finished reading before the previous barrier)
    auto layer = [&](int l, auto kc_tag) {
        constexpr int KC = decltype(kc_tag)::value;
        // per-lane pixel coordinates re-derived inside the layer (opaque to the compiler), so
        // that the 36 tap addresses are not hoisted out of the layer loop into registers
        const int src = (l & 1) ? 0 : BUF1, dst = (l & 1) ? BUF1 : 0;
        const _Float16 *const wa = l == 0 ? wl0 : wl0 + kW0 + (size_t)((ZC_TOWER_DIAG & 4) ? 0 : l - 1) * kW;
        const _Float16 *const wn = l + 1 < nconv ? wl0 + kW0 + (size_t)((ZC_TOWER_DIAG & 4) ? 0 : l) * kW : nullptr;  // layer l+1's
        if constexpr (MF == 16) {
            int py16[NP];  // (the pixel rows are l16 + 16 t: nothing to carry)
#pragma unroll
            for (int t = 0; t < NP; ++t) {
                py16[t] = pyx[t];
                __asm__ volatile("" : "+v"(py16[t]));
            }
            f4x acc[2][NP];
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int t = 0; t < NP; ++t) acc[m][t] = f4x{0.0f, 0.0f, 0.0f, 0.0f};
            if constexpr (SWZ) {
                const float *bp = ball + (size_t)l * kCout + wave * 32 + 16 * (q4 & 1) + 8 * (q4 >> 1);
                const float4 b0 = *(const float4 *)bp, b1 = *(const float4 *)(bp + 4);
                const float bv8[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
                tower_mfma16_swz<H, W, NP, KC, 8, tower_zero<NT>()>(lds, src, wa, wn, a, l16, py16, q4, acc);
                tower_epilogue16s<NP>(lds + dst * LD, bv8, l >= 2 && !(l & 1), npix, wave, l16, q4, acc);
                __syncthreads();
                return;
            }
            float4 bv[2];
#pragma unroll
            for (int m = 0; m < 2; ++m) bv[m] = *(const float4 *)(ball + (size_t)l * kCout + wave * 32 + 16 * m + 4 * q4);
#if ZC_TOWER_STAMP
            __builtin_amdgcn_sched_barrier(0);
            const uint64_t ts0 = __builtin_amdgcn_s_memtime();
            __builtin_amdgcn_sched_barrier(0);
#endif
            tower_mfma16<H, W, NP, KC, 8, LD, tower_zero<NT>(), ZR>(lds, src, wa, wn, a, l16, py16, q4, acc);
#if ZC_TOWER_STAMP
            __builtin_amdgcn_sched_barrier(0);
            const uint64_t ts1 = __builtin_amdgcn_s_memtime();
            __builtin_amdgcn_sched_barrier(0);
            st_mfma += ts1 - ts0;
#endif
            if constexpr (EPI == 1)
                tower_epilogue16_swap<NP>(lds + dst * LD, bv, l >= 2 && !(l & 1), npix, wave, l16, q4, acc);
            else if constexpr (EPI == 2)
                tower_epilogue16<NP>(lds + dst * LD, bv, l >= 2 && !(l & 1), npix, wave, l16, q4, acc);
            else
                tower_epilogue16b<NP>(lds + dst * LD, bv, l >= 2 && !(l & 1), npix, wave, l16, q4, acc);
#if ZC_TOWER_STAMP
            __builtin_amdgcn_sched_barrier(0);
            const uint64_t ts2 = __builtin_amdgcn_s_memtime();
            __builtin_amdgcn_sched_barrier(0);
            st_epi += ts2 - ts1;
            __syncthreads();
            __builtin_amdgcn_sched_barrier(0);
            st_bar += __builtin_amdgcn_s_memtime() - ts2;
            __builtin_amdgcn_sched_barrier(0);
            return;
#endif
        } else {
            int pr[NT], py[NT];
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                pr[t] = prow[t];
                py[t] = pyx[t];
                __asm__ volatile("" : "+v"(pr[t]), "+v"(py[t]));
            }
            f16x acc[NT];
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int k = 0; k < 16; ++k) acc[t][k] = 0.0f;
            float4 bv[4];  // this wave's bias slice, in flight during the MFMA loop
#pragma unroll
            for (int g = 0; g < 4; ++g) bv[g] = *(const float4 *)(ball + (size_t)l * kCout + wave * 32 + 8 * g + 4 * hh);
            tower_mfma<H, W, NT, KC, 8, PG>(lds, src, wa, wn, a, pr, py, hh, acc);
            tower_epilogue(lds + dst * LD, bv, l >= 2 && !(l & 1), npix, wave, r, hh, acc, pbase);
        }
        __syncthreads();
    };
    layer(0, std::integral_constant<int, KC0>{});
    for (int l = 1; l < nconv; ++l) layer(l, std::integral_constant<int, 8>{});
#if ZC_TOWER_STAMP
    if (lane == 0) {
        atomicAdd(&g_tower_stamp[0], (unsigned long long)st_mfma);
        atomicAdd(&g_tower_stamp[1], (unsigned long long)st_epi);
        atomicAdd(&g_tower_stamp[2], (unsigned long long)st_bar);
        atomicAdd(&g_tower_stamp[3], (unsigned long long)(__builtin_amdgcn_s_memtime() - st_k0));
    }
#endif
    // the tower's output is the last layer's dst (buf0, nconv odd)
    if (values) {
        // the value head on it, one wave per board: value_head_kernel's arithmetic in its
        // order (lane l sums channels 8 (l & 15) .. +8 over pixels l / 16, +4, ...), from LDS
        const int c0 = (lane & 15) * 8;
        for (int bi = wave + 4 * pg; bi < npix / HW; bi += 4 * PG) {
            const _Float16 *act = lds + bi * HW * LD + c0;
            float sum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
            for (int p = lane >> 4; p < HW; p += 4) {
                const h8 v = *(const h8 *)(SWZ ? lds + swz(bi * HW + p, lane & 15) : act + p * LD);
#pragma unroll
                for (int e = 0; e < 8; ++e) sum[e] += (float)v[e];
            }
            float d = 0.f;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                float t = sum[e] + __shfl_xor(sum[e], 16);
                t += __shfl_xor(t, 32);
                d += t * fcw[c0 + e];
            }
            d /= (float)HW;
            for (int o = 8; o > 0; o >>= 1) d += __shfl_xor(d, o);
            if (lane == 0) values[b0 + bi] = pol.head_raw ? (double)(d + fcb) : (double)tanhf(d + fcb);
        }
    }
    if (pol.out) {
        // the 1x1 conv: wave (pg, wave) takes pixel tiles wave, wave + 4, ... of its group (32
        // pixels each); per block of 32 output channels 8 MFMAs over the 128 channels, + bias,
        // ReLU (the linear head's conv) or not (the convolutional head's logits), fp16 ->
        // [pixel][32 * mblocks]
        const int nout = 32 * pol.mblocks;
        for (int mb = 0; mb < pol.mblocks; ++mb) {
            h8 pa[8];
#pragma unroll
            for (int kc = 0; kc < 8; ++kc) pa[kc] = *(const h8 *)(pol.pw + (((size_t)mb * 8 + kc) * 64 + lane) * 8);
            float4 pbv[4];
#pragma unroll
            for (int g = 0; g < 4; ++g) pbv[g] = *(const float4 *)(pol.pb + 32 * mb + 8 * g + 4 * hh);
            const bool relu = pol.relu != 0;
            for (int t = wave; t < NT; t += 4) {
                const int P = pbase + t * 32 + r;
                f16x acc;
#pragma unroll
                for (int k = 0; k < 16; ++k) acc[k] = 0.0f;
#pragma unroll
                for (int kc = 0; kc < 8; ++kc) {
                    const h8 x = *(const h8 *)(lds + (SWZ ? swz(P, 2 * kc + hh) : P * LD + kc * 16 + hh * 8));
                    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(pa[kc], x, acc, 0, 0, 0);
                }
                if (P < npix) {
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const float bb[4] = {pbv[g].x, pbv[g].y, pbv[g].z, pbv[g].w};
                        h4 ov;
#pragma unroll
                        for (int e = 0; e < 4; ++e) {  // logits (relu = 0): no floor, a NaN stays a NaN
                            const float y = acc[4 * g + e] + bb[e];
                            ov[e] = (_Float16)(relu ? fmaxf(y, 0.0f) : y);
                        }
                        *(h4 *)(pol.out + ((size_t)b0 * HW + P) * nout + 32 * mb + 8 * g + 4 * hh) = ov;
                    }
                }
            }
        }
    }
    if (out) {  // -> HBM, whole 256-byte rows
#pragma unroll
        for (int q = 0; q < TP * (kCout / 8) / NTH; ++q) {
            const int i = tid + q * NTH, P = i >> 4, c0 = (i & 15) * 8;
            if (P < npix)
                *(h8 *)(out + ((size_t)b0 * HW + P) * kCout + c0) =
                    *(const h8 *)(lds + (SWZ ? swz(P, i & 15) : P * LD + c0));
        }
    }
}

// A/B and test switches of the network launches.  Read from the environment ONCE, when the
// library loads (ZC_TOWER_MF, ZC_TOWER_EPI, ZC_HEAD_RAW), and changed afterwards only through
// zc_debug_net_switch — a product process never re-reads the environment per launch.
struct NetSwitches {
    int tower_mf, tower_epi, head_raw;
};
int env_switch(const char *name, int dflt, int (*parse)(const char *)) {
    const char *e = getenv(name);
    return e ? parse(e) : dflt;
}
NetSwitches g_net_sw = {
    env_switch("ZC_TOWER_MF", 0, [](const char *e) { return !strcmp(e, "32") ? 32 : !strcmp(e, "16") ? 16 : 0; }),
    env_switch("ZC_TOWER_EPI", 0, [](const char *e) { return e[0] >= '0' && e[0] <= '3' && !e[1] ? e[0] - '0' : 0; }),
    env_switch("ZC_HEAD_RAW", 0, [](const char *e) { return !strcmp(e, "1") ? 1 : 0; })};

int tower_epi() {  // 1 = the 16x16x32 form's epilogue with 16-byte stores,
                  // 2 = the per-tile read-wait-add epilogue (before the batched one)
    return g_net_sw.tower_epi;
}

template <int H, int W, int BPH, int NT, int WPE, int PG = 1, int MF = 32>
void launch_tower(int n, int nconv, const void *in, const void *wall, const float *ball, void *out, const float *fcw,
                  float fcb, double *values, TowerPolicy pol, hipStream_t s) {
    if constexpr (MF == 16) {
        if (tower_epi() == 1) {
            hipLaunchKernelGGL((tower_kernel<H, W, BPH, 32, NT, WPE, PG, MF, 1>), dim3((n + BPH - 1) / BPH),
                               dim3(256 * PG), (tower_lds<NT, PG, MF>()), s, n, nconv, (const _Float16 *)in,
                               (const _Float16 *)wall, ball, (_Float16 *)out, fcw, fcb, values, pol);
            return;
        }
        if (tower_epi() == 2) {
            hipLaunchKernelGGL((tower_kernel<H, W, BPH, 32, NT, WPE, PG, MF, 2>), dim3((n + BPH - 1) / BPH),
                               dim3(256 * PG), (tower_lds<NT, PG, MF>()), s, n, nconv, (const _Float16 *)in,
                               (const _Float16 *)wall, ball, (_Float16 *)out, fcw, fcb, values, pol);
            return;
        }
        if (tower_epi() == 3) {
            hipLaunchKernelGGL((tower_kernel<H, W, BPH, 32, NT, WPE, PG, MF, 3>), dim3((n + BPH - 1) / BPH),
                               dim3(256 * PG), (tower_lds_swz<NT>()), s, n, nconv, (const _Float16 *)in,
                               (const _Float16 *)wall, ball, (_Float16 *)out, fcw, fcb, values, pol);
            return;
        }
    }
    hipLaunchKernelGGL((tower_kernel<H, W, BPH, 32, NT, WPE, PG, MF>), dim3((n + BPH - 1) / BPH),
                           dim3(256 * PG), (tower_lds<NT, PG, MF>()), s, n, nconv, (const _Float16 *)in,
                           (const _Float16 *)wall, ball, (_Float16 *)out, fcw, fcb, values, pol);
}


// [9][kCout][cin] -> the stream form's fragments: packed[((tap * KC + kc) * 4 + mb) * 512 +
// lane * 8 + e] = w[tap][mb * 32 + lane % 32][kc * 16 + 8 * (lane / 32) + e].
__global__ void pack_conv_weight_kernel(int cin, const _Float16 *__restrict__ w, _Float16 *__restrict__ packed) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;  // one 8-half piece
    const int KC = cin / 16;
    if (i >= 9 * KC * 4 * 64) return;
    const int lane = i & 63, mb = (i >> 6) & 3, kc = (i >> 8) % KC, tap = (i >> 8) / KC;
    const int row = mb * 32 + (lane & 31), k0 = kc * 16 + 8 * (lane >> 5);
    *(h8 *)(packed + (size_t)i * 8) = *(const h8 *)(w + ((size_t)tap * kCout + row) * cin + k0);
}

// planes [n][cin][H*W] (state_to_tensor layout, fp16) -> NHWC [n][H*W][cpad], zero padded.
__global__ void planes_to_nhwc_kernel(int n, int cin, int hw, int cpad, const _Float16 *__restrict__ planes,
                                      _Float16 *__restrict__ out) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= (int64_t)n * hw) return;
    const int i = (int)(g / hw), p = (int)(g - (int64_t)i * hw);
    const _Float16 *src = planes + (size_t)i * cin * hw + p;
    h8 *o = (h8 *)(out + g * cpad);  // cpad is a multiple of 8: 16-byte stores
    for (int c8 = 0; c8 < cpad / 8; ++c8) {
        h8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int c = c8 * 8 + e;
            v[e] = c < cin ? src[(size_t)c * hw] : (_Float16)0.0f;
        }
        o[c8] = v;
    }
}

// head (network.py:37-42): global average pool -> Linear(128, 1) -> tanh, in fp32; one wave
// per position.  Lane l reads 16-byte pieces (channels 8 (l & 15) .. +8) of pixels l / 16,
// +4, +8, ..., so every load instruction covers four whole 256-byte pixel rows; the four
// pixel groups are then summed across lanes.  Writes the fp64 value the backup takes.
__global__ __launch_bounds__(256) void value_head_kernel(int n, int hw, const _Float16 *__restrict__ act,
                                                         const float *__restrict__ fcw, float fcb,
                                                         double *__restrict__ values, int raw) {
    const int i = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int lane = threadIdx.x & 63;
    if (i >= n) return;
    const int c0 = (lane & 15) * 8;
    const _Float16 *a = act + (size_t)i * hw * kCout + c0;
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int p = lane >> 4; p < hw; p += 4) {
        const h8 v = *(const h8 *)(a + (size_t)p * kCout);
#pragma unroll
        for (int e = 0; e < 8; ++e) s[e] += (float)v[e];
    }
    float d = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        float t = s[e] + __shfl_xor(s[e], 16);
        t += __shfl_xor(t, 32);
        d += t * fcw[c0 + e];
    }
    d /= (float)hw;
    for (int o = 8; o > 0; o >>= 1) d += __shfl_xor(d, o);
    if (lane == 0) values[i] = raw ? (double)(d + fcb) : (double)tanhf(d + fcb);
}

// head_raw = 1 (tests only): the value head returns its pre-tanh sum, so the pooled Linear
// can be checked exactly against float64 on integer networks
int head_raw() { return g_net_sw.head_raw; }

int conv_impl() {  // ZC_CONV_IMPL=tile: 256-pixel tiles for every layer; default: half tiles for 128 planes
    static const int v = [] {
        const char *e = getenv("ZC_CONV_IMPL");
        return e && !strcmp(e, "tile") ? 0 : 1;
    }();
    return v;
}

// The MFMA form (zc_debug_net_switch("tower_mf", ...) between launches, so an A/B can alternate in one process): the fused tower
// runs the 16x16x32 form (+9 % over 32x32x16 at the power-held clock, outputs bit-identical:
// profiles/r04_ab_tower_mf.log) unless ZC_TOWER_MF=32; the packed per-layer conv keeps the
// 32x32x16 form at three workgroups per CU unless ZC_TOWER_MF=16
int tower_mf() { return g_net_sw.tower_mf == 32 ? 32 : 16; }
int stream_mf() { return g_net_sw.tower_mf == 16 ? 16 : 32; }

int stream_wpe() {  // ZC_CONV_WPE=2: the packed form at two workgroups per CU (default 3)
    static const int v = [] {
        const char *e = getenv("ZC_CONV_WPE");
        return e && !strcmp(e, "2") ? 2 : 3;
    }();
    return v;
}

template <int H, int W, int BPH, int CIN>
void launch_stream(int n, const void *in, const void *wp, const float *bias, const void *res, void *out, int relu,
                   hipStream_t s) {
    const size_t tile = (size_t)(kHalfPix + 16) * (CIN + 8) * sizeof(_Float16);
    if (stream_mf() == 16) {
        const size_t tile16 = (size_t)(kHalfPix + 16) * (CIN + 16) * sizeof(_Float16);
        hipLaunchKernelGGL((conv3x3_stream_kernel<H, W, BPH, CIN, 2, 16>), dim3((n + BPH - 1) / BPH), dim3(256),
                           std::max(tile16, kHalfEpiBytes), s, n, (const _Float16 *)in, (const _Float16 *)wp, bias,
                           (const _Float16 *)res, (_Float16 *)out, relu);
    } else if (stream_wpe() == 2)
        hipLaunchKernelGGL((conv3x3_stream_kernel<H, W, BPH, CIN, 2>), dim3((n + BPH - 1) / BPH), dim3(256),
                           std::max(tile, kHalfEpiBytes), s, n, (const _Float16 *)in, (const _Float16 *)wp, bias,
                           (const _Float16 *)res, (_Float16 *)out, relu);
    else
        hipLaunchKernelGGL((conv3x3_stream_kernel<H, W, BPH, CIN, 3>), dim3((n + BPH - 1) / BPH), dim3(256),
                           std::max(tile, kHalfEpiBytes / 2), s, n, (const _Float16 *)in, (const _Float16 *)wp, bias,
                           (const _Float16 *)res, (_Float16 *)out, relu);
}

template <int H, int W, int BPW, int BPH, int CIN>
void launch_conv(int n, const void *in, const void *wt, const float *bias, const void *res, void *out, int relu,
                 hipStream_t s) {
    if (conv_impl() == 1 && CIN >= 64) {  // the 32-plane stem runs faster on 256-pixel tiles
        const size_t lds = std::max((size_t)(kHalfPix + 1 + kCout) * (CIN + 8) * sizeof(_Float16), kHalfEpiBytes);
        hipLaunchKernelGGL((conv3x3_half_kernel<H, W, BPH, CIN>), dim3((n + BPH - 1) / BPH), dim3(256), lds, s, n,
                           (const _Float16 *)in, (const _Float16 *)wt, bias, (const _Float16 *)res, (_Float16 *)out,
                           relu);
    } else {
        const size_t lds = (size_t)(kTilePix + 1 + 2 * kCout) * (CIN + 8) * sizeof(_Float16);
        hipLaunchKernelGGL((conv3x3_kernel<H, W, BPW, CIN>), dim3((n + BPW - 1) / BPW), dim3(256), lds, s, n,
                           (const _Float16 *)in, (const _Float16 *)wt, bias, (const _Float16 *)res, (_Float16 *)out,
                           relu);
    }
}

}  // namespace
#if ZC_TOWER_STAMP
extern "C" int zc_debug_tower_stamps(unsigned long long *host, int clear) {
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_tower_stamp), sizeof(unsigned long long) * 4) != hipSuccess) return 1;
    if (clear) {
        static unsigned long long zeros[4];
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_tower_stamp), zeros, sizeof(zeros)) != hipSuccess) return 1;
    }
    return 0;
}
#endif

bool launch_net_conv3x3(int n, int h, int w, int cin, const void *in, const void *wt, const float *bias,
                        const void *res, void *out, int relu, hipStream_t s) {
    if (h == 8 && w == 8 && cin == 128) launch_conv<8, 8, 4, 2, 128>(n, in, wt, bias, res, out, relu, s);
    else if (h == 8 && w == 8 && cin == 32) launch_conv<8, 8, 4, 2, 32>(n, in, wt, bias, res, out, relu, s);
    else if (h == 6 && w == 7 && cin == 128) launch_conv<6, 7, 6, 3, 128>(n, in, wt, bias, res, out, relu, s);
    else if (h == 6 && w == 7 && cin == 32) launch_conv<6, 7, 6, 3, 32>(n, in, wt, bias, res, out, relu, s);
    else return false;
    return true;
}

bool launch_net_conv3x3_packed(int n, int h, int w, int cin, const void *in, const void *wp, const float *bias,
                               const void *res, void *out, int relu, hipStream_t s) {
    if (h == 8 && w == 8 && cin == 128) launch_stream<8, 8, 2, 128>(n, in, wp, bias, res, out, relu, s);
    else if (h == 8 && w == 8 && cin == 32) launch_stream<8, 8, 2, 32>(n, in, wp, bias, res, out, relu, s);
    else if (h == 6 && w == 7 && cin == 128) launch_stream<6, 7, 3, 128>(n, in, wp, bias, res, out, relu, s);
    else if (h == 6 && w == 7 && cin == 32) launch_stream<6, 7, 3, 32>(n, in, wp, bias, res, out, relu, s);
    else return false;
    return true;
}

bool launch_net_tower(int n, int h, int w, int cin0, int nconv, const void *in, const void *wall, const float *ball,
                      void *out, const float *fcw, float fcb, double *values, const void *pw, const float *pb,
                      void *pout, hipStream_t s, int pol_channels, int pol_relu) {
    if (cin0 != 32 || nconv < 1 || !(nconv & 1)) return false;
    if (pout && pol_channels != 32 && pol_channels != 64) return false;
    const TowerPolicy pol{(const _Float16 *)pw, pb, (_Float16 *)pout, head_raw(), pol_channels / 32, pol_relu ? 1 : 0};
    // 128-pixel tiles at two workgroups per CU; 64-pixel tiles (one chess board) at 3 or 4
    // workgroups per CU measured 10 % slower (tools/ab_tower.py)
#ifndef ZC_TOWER_PG
#define ZC_TOWER_PG 1
#endif
#if ZC_TOWER_PG == 2
    if (h == 8 && w == 8) launch_tower<8, 8, 4, 4, 2, 2>(n, nconv, in, wall, ball, out, fcw, fcb, values, pol, s);
    else if (h == 6 && w == 7) launch_tower<6, 7, 6, 4, 2, 2>(n, nconv, in, wall, ball, out, fcw, fcb, values, pol, s);
#else
    if (tower_mf() == 16) {
        if (h == 8 && w == 8) launch_tower<8, 8, 2, 4, 2, 1, 16>(n, nconv, in, wall, ball, out, fcw, fcb, values, pol, s);
        else if (h == 6 && w == 7) launch_tower<6, 7, 3, 4, 2, 1, 16>(n, nconv, in, wall, ball, out, fcw, fcb, values, pol, s);
        else return false;
    } else if (h == 8 && w == 8) launch_tower<8, 8, 2, 4, 2>(n, nconv, in, wall, ball, out, fcw, fcb, values, pol, s);
    else if (h == 6 && w == 7) launch_tower<6, 7, 3, 4, 2>(n, nconv, in, wall, ball, out, fcw, fcb, values, pol, s);
#endif
    else return false;
    return true;
}

bool launch_net_pack_conv_weight(int cin, const void *w, void *packed, hipStream_t s) {
    if (cin != 32 && cin != 128) return false;
    const int n = 9 * (cin / 16) * 4 * 64;
    hipLaunchKernelGGL(pack_conv_weight_kernel, dim3((n + 255) / 256), dim3(256), 0, s, cin, (const _Float16 *)w,
                       (_Float16 *)packed);
    return true;
}

void launch_net_planes_to_nhwc(int n, int cin, int hw, int cpad, const void *planes, void *out, hipStream_t s) {
    const int64_t total = (int64_t)n * hw;
    hipLaunchKernelGGL(planes_to_nhwc_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, n, cin, hw, cpad,
                       (const _Float16 *)planes, (_Float16 *)out);
}

void launch_net_value_head(int n, int hw, const void *act, const float *fcw, float fcb, double *values, hipStream_t s) {
    hipLaunchKernelGGL(value_head_kernel, dim3((unsigned)(((int64_t)n * 64 + 255) / 256)), dim3(256), 0, s, n, hw,
                       (const _Float16 *)act, fcw, fcb, values, head_raw());
}

}  // namespace zc

namespace zc {
// zc_debug_net_switch (engine.hip): false for an unknown name or value
bool net_switch(const char *name, int value, int *old) {
    int *slot = nullptr;
    bool ok = false;
    if (name && !strcmp(name, "tower_mf")) {
        slot = &g_net_sw.tower_mf;
        ok = value == 0 || value == 16 || value == 32;
    } else if (name && !strcmp(name, "tower_epi")) {
        slot = &g_net_sw.tower_epi;
        ok = value >= 0 && value <= 3;
    } else if (name && !strcmp(name, "head_raw")) {
        slot = &g_net_sw.head_raw;
        ok = value == 0 || value == 1;
    }
    if (!slot || !ok) return false;
    if (old) *old = *slot;
    *slot = value;
    return true;
}
}  // namespace zc
