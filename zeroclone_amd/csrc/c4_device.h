// c4_device.h — device-side building blocks shared by the Connect4 search kernels
// (c4_search.hip: fused rollout search; c4_ext.hip: stepwise search with caller values).
// Included by exactly those translation units; everything is internal to each of them.
#pragma once
#include <math.h>

#include "c4_order_table.h"
#include "zc_internal.h"

namespace zc {
namespace {

__constant__ uint32_t d_order[128] = {ZC_C4_ORDER_LIST};

constexpr uint32_t kRingMask = kRingWords - 1;
constexpr uint64_t kBottom = 0x0000040810204081ull;  // bit 7c: bottom cell of column c
constexpr uint64_t kFull = kBottom * 0x3Full;        // the 42 playable cells
constexpr uint64_t kTop = kBottom << 5;              // top playable cell of each column
// LDS tables: move-list order[128] u32, then sel[128][8] u8 (the r-th set bit of a 7-bit mask)
constexpr int kTabBytes = 128 * 4 + 128 * 8;

// Untried moves of a node (record +4 / Fresh.u): bit i (i < 7) set while move i of the
// node's move list is untried; bits 28..31 = number of moves.  The reference keeps the
// untried INDICES in list order and lets random.choice pick the r-th (mcts.cpp:67-72); the
// r-th remaining index is the r-th set bit of the mask (one ballot over lanes 0..6).
__device__ __forceinline__ uint32_t untried_init(uint32_t n) { return ((1u << n) - 1u) | (n << 28); }
__device__ __forceinline__ uint32_t untried_count(uint32_t u) { return (uint32_t)__popc(u & 0x7Fu); }

// Fill the LDS tables (whole workgroup): s_order = d_order; sel[m][r] = position of the r-th
// set bit of m (7 when m has fewer), right after s_order.
__device__ __forceinline__ void load_tables(uint32_t *s_order) {
    for (int i = (int)threadIdx.x; i < 128; i += blockDim.x) s_order[i] = d_order[i];
    uint8_t *const s_sel = (uint8_t *)(s_order + 128);
    for (int i = (int)threadIdx.x; i < 1024; i += blockDim.x) {
        const uint32_t m = (uint32_t)i >> 3, r = (uint32_t)i & 7u;
        uint32_t c = 0, pos = 7;
        for (uint32_t b = 0; b < 7; ++b)
            if ((m >> b) & 1u) {
                if (c == r) {
                    pos = b;
                    break;
                }
                ++c;
            }
        s_sel[i] = (uint8_t)pos;
    }
}
__device__ __forceinline__ const uint8_t *sel_table(const uint32_t *s_order) { return (const uint8_t *)(s_order + 128); }
constexpr int kWin = 64;                             // RNG window: one word per lane
// LDS bytes after the leaves' paths: select_flush stores a path with all 64 lanes, so the
// last leaf's lanes >= kMaxDepth land here
constexpr int kPathSpill = 2 * (64 - kMaxDepth) + 24;

// ------------------------------------------------------------------ wave helpers
__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint64_t uni64(uint64_t x) {
    return ((uint64_t)uni((uint32_t)(x >> 32)) << 32) | (uint64_t)uni((uint32_t)x);
}
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
// lane-wise select by a wave mask in SGPRs: bit `lane` of m set -> b, else a (or 0)
__device__ __forceinline__ uint32_t mask_sel(uint64_t m, uint32_t a, uint32_t b) {
    uint32_t r;
    __asm__("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
    return r;
}
__device__ __forceinline__ uint32_t mask_sel0(uint64_t m, uint32_t b) {
    uint32_t r;
    __asm__("v_cndmask_b32 %0, 0, %1, %2" : "=v"(r) : "v"(b), "s"(m));
    return r;
}
// x + 1 in the lanes of wave mask m (the mask as the add's carry-in)
__device__ __forceinline__ uint32_t add_in_mask(uint32_t x, uint64_t m) {
    uint32_t r;
    uint64_t co;
    __asm__("v_addc_co_u32_e64 %0, %1, 0, %2, %3" : "=v"(r), "=s"(co) : "v"(x), "s"(m));
    return r;
}
__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {  // set bits of m in lanes below this one
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Wait for x's load here.  Stores and loads share gfx950's in-order vector-memory counter, so
// a load still in flight where two paths join makes the compiler's wait at the join (vmcnt(0))
// also drain every store issued since — on the path that never loaded anything.  Waiting on
// the loading path itself keeps the other path free of it.
template <class T>
__device__ __forceinline__ void vmem_ready(T &x) {
    asm volatile("" : "+v"(x));
}

__device__ __forceinline__ void wave_mem_order() {
    // Same-wave hand-offs through memory (one lane stores, another loads) are ordered by
    // program order on gfx950 (wavefront scope needs no cache action); this only stops the
    // compiler from moving memory operations across the point.
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

template <int CTRL>
__device__ __forceinline__ int dpp(int x) {
    return __builtin_amdgcn_mov_dpp(x, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ double dpp(double x) {
    const int lo = dpp<CTRL>(__double2loint(x));
    const int hi = dpp<CTRL>(__double2hiint(x));
    return __hiloint2double(hi, lo);
}

// First maximum over lanes 0..7 (ties -> lower slot), as mcts.cpp:55-58 (`v > best_val`,
// scanning slots in order).  Three DPP steps inside each 8-lane half row: xor 1, xor 2,
// mirror; afterwards every lane of the half row holds the winner.
template <class T>
__device__ __forceinline__ void argmax_step(T &v, int &i, T ov, int oi) {
    if (ov > v || (ov == v && oi < i)) {
        v = ov;
        i = oi;
    }
}
template <class T>
__device__ __forceinline__ void argmax8(T &v, int &i) {
    argmax_step(v, i, dpp<0xB1>(v), dpp<0xB1>(i));    // quad_perm [1,0,3,2]
    argmax_step(v, i, dpp<0x4E>(v), dpp<0x4E>(i));    // quad_perm [2,3,0,1]
    argmax_step(v, i, dpp<0x141>(v), dpp<0x141>(i));  // row_half_mirror
}

// The same first maximum for the walk's UCT scores: the maximum over lanes 0..7 by three DPP
// v_max_f64 steps (no index carried, no per-step branch: the compare-and-swap form compiled to
// exec-mask juggling, ~8 SALU per step), then the first slot holding it from one ballot.  The
// scores are finite or -inf (never NaN), and a slot holding the maximum compares equal to it,
// so this is the strict `>` scan of mcts.cpp:55-58 (+0 and -0 compare equal there too).
// Returns the maximum; *first = the lowest slot k < 8 with v == max.
__device__ __forceinline__ double max8_first(double v, int *first) {
    double m = v;
    m = fmax(m, dpp<0xB1>(m));   // quad_perm [1,0,3,2]
    m = fmax(m, dpp<0x4E>(m));   // quad_perm [2,3,0,1]
    m = fmax(m, dpp<0x141>(m));  // row_half_mirror
    *first = __builtin_ctzll((__ballot(v == m) & 0xFFull) | 0x100ull);
    return m;
}

// ------------------------------------------------------------------ Connect4 bitboards
__device__ __forceinline__ uint64_t drop_bit(uint64_t occ, int col) {
    // c4_backend.play_move (:14-23): lowest empty row of `col`; a full column drops nothing.
    const int s = 7 * col;
    return (occ + (1ull << s)) & (0x3Full << s);
}

__device__ __forceinline__ int legal_mask(uint64_t occ) {
    // c4_backend.get_legal_moves (:49-50): column c is legal while its top cell is empty.
    // Gather bit 7c -> bit c with one multiply: the 49 partial products t_c * 2^(56-6i) land
    // on distinct bit positions (7c - 6i is injective on 0..6 x 0..6), so nothing carries
    // and bits 56..62 of the product are exactly t_0..t_6.
    const uint64_t t = (~occ & kTop) >> 5;  // bit 7c
    return (int)((t * 0x0104104104100000ull) >> 56) & 0x7F;
}

__device__ __forceinline__ bool has_four(uint64_t b) {
    // c4_backend.check_win (:25-44) for one token: any horizontal, vertical or diagonal run.
    uint64_t m = b & (b >> 7);
    uint64_t r = m & (m >> 14);
    m = b & (b >> 1);
    r |= m & (m >> 2);
    m = b & (b >> 6);
    r |= m & (m >> 12);
    m = b & (b >> 8);
    r |= m & (m >> 16);
    return r != 0;
}

// ------------------------------------------------------------------ CPython MT19937
__device__ __forceinline__ uint32_t temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

// The game's stream lives in a ring of RAW MT words x[p] (absolute position p, slot
// p % kRingWords).  The recurrence x[p] = x[p-227] ^ twist(x[p-624], x[p-623]) regenerates
// it kChunk words at a time, all lanes in parallel (every input is >= 227 words older).
// Three 64-word windows sit in registers: wt (tempered, the window holding the next word),
// wn (tempered, the one after) and wx (raw, in flight from the ring), so a 64-word view
// starting at ANY position of wt is two lane permutes away (rng_view).
struct Rng {
    uint32_t *ring;
    uint32_t base;   // low 32 bits of the absolute position at the search's start (use0)
    int32_t wrel;    // window start - use0 (a multiple of 64 in absolute terms; may be < 0)
    uint32_t off;    // next word to consume = window start + off, off in [0, 128)
    int32_t grel;    // words generated so far - use0
    uint32_t wt;     // tempered x[window start + lane]
    uint32_t wn;     // tempered x[window start + 64 + lane]
    uint32_t wx;     // raw x[window start + 128 + lane], in flight until the window advances
    __device__ __forceinline__ int32_t use() const { return wrel + (int32_t)off; }  // relative to use0
    __device__ __forceinline__ uint32_t slot(int32_t rel) const { return (base + (uint32_t)rel) & kRingMask; }
    __device__ __forceinline__ uint32_t cur() const { return wt; }
};

__device__ __forceinline__ int32_t rng_generate(uint32_t *ring, uint32_t base, int32_t grel, int32_t target) {
    const uint32_t lane = lane_id();
    constexpr int K = kChunk / 64;
    while (grel < target) {
        // every input of the chunk is >= 227 words older than any output: load all, then store
        uint32_t a[K], b[K], m[K];
        const uint32_t p0 = base + (uint32_t)grel + lane;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t p = p0 + 64u * k;
            a[k] = ring[(p - 624) & kRingMask];
            b[k] = ring[(p - 623) & kRingMask];
            m[k] = ring[(p - 227) & kRingMask];
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t p = p0 + 64u * k;
            const uint32_t y = (a[k] & 0x80000000u) | (b[k] & 0x7fffffffu);
            ring[p & kRingMask] = m[k] ^ (y >> 1) ^ ((b[k] & 1u) ? 0x9908b0dfu : 0u);
        }
        grel += kChunk;
        wave_mem_order();
    }
    return grel;
}

__device__ __forceinline__ void rng_fill(Rng &r, int32_t target) {
    if (r.grel < target) r.grel = rng_generate(r.ring, r.base, r.grel, target);
}

// use0 / gen0: absolute positions (words consumed / generated) from the game's rngpos.
__device__ __forceinline__ void rng_open(Rng &r, uint32_t *ring, uint64_t use0, uint64_t gen0) {
    r.ring = ring;
    r.base = (uint32_t)use0;
    r.grel = (int32_t)(gen0 - use0);
    r.off = (uint32_t)use0 & (uint32_t)(kWin - 1);
    r.wrel = -(int32_t)r.off;
    rng_fill(r, r.wrel + 3 * kWin);
    r.wt = temper(r.ring[r.slot(r.wrel + (int32_t)lane_id())]);
    r.wn = temper(r.ring[r.slot(r.wrel + kWin + (int32_t)lane_id())]);
    r.wx = r.ring[r.slot(r.wrel + 2 * kWin + (int32_t)lane_id())];
    vmem_ready(r.wx);
}

// Move the windows on by 64 words (precondition: off >= 64).
__device__ __forceinline__ void rng_advance(Rng &r) {
    r.wrel += kWin;
    r.off -= (uint32_t)kWin;
    r.wt = r.wn;
    r.wn = temper(r.wx);
    if (r.grel < r.wrel + 3 * kWin) rng_fill(r, r.wrel + 3 * kWin);
    r.wx = r.ring[r.slot(r.wrel + 2 * kWin + (int32_t)lane_id())];
    vmem_ready(r.wx);  // once per 64 words, instead of at every later join
}

// The 64 tempered words from the next unconsumed one on: lane l = word off + l of the
// window (precondition: off < 64).
template <class R>
__device__ __forceinline__ uint32_t rng_view(const R &r) {
    const uint32_t j = lane_id() + r.off;
    const int idx = (int)(j << 2);  // ds_bpermute reads the lane from address bits 7:2 only
    const uint32_t a = (uint32_t)__builtin_amdgcn_ds_bpermute(idx, (int)r.wt);
    const uint32_t b = (uint32_t)__builtin_amdgcn_ds_bpermute(idx, (int)r.wn);
    return j < 64u ? a : b;
}

// rngpos after the search: {use0 + use(), use0 + grel}
__device__ __forceinline__ void rng_close(const Rng &r, uint64_t use0, uint64_t *rngpos) {
    rngpos[0] = use0 + (uint64_t)(int64_t)r.use();
    rngpos[1] = use0 + (uint64_t)(int64_t)r.grel;
}

// ------------------------------------------------------------------ the stream in LDS
// The fused search (c4_search_kernel) keeps its game's stream in a 1024-word LDS ring
// instead of the HBM ring: the recurrence runs one 64-word step per window advance, lane l
// generating x[W + 128 + l] (W = the new window start) from inputs read one advance earlier
// (x[p-624], x[p-623], x[p-227] are all older than W + 128 - 163, so they are known a whole
// window ahead), and the new raw word is the new `wx` itself — no HBM traffic and no
// memory wait on the chain.  Invariant: words [W - 832, W + 192) are in the ring.
// The HBM ring is the hand-over format to every other kernel and to zc_rng_get_state: the
// kernel loads its game's last 1024 words at the start and, at the end, writes back the
// words [min(U & ~63, block start, G' - 624), G') (U = next word, block = the 624-word block
// holding word U-1, G' = words generated, at least that block's end) — what rng_open,
// zc_rng_get_state and the recurrence read.
constexpr int kLRingWords = 1024;
constexpr uint32_t kLRingMask = kLRingWords - 1;
constexpr int kLRingBytes = kLRingWords * 4;

struct LRng {
    uint32_t *lds;   // this wave's ring: raw x[p] at slot p % 1024
    uint32_t base;   // low 32 bits of the absolute position at the search's start (use0)
    int32_t wrel;    // window start - use0
    uint32_t off;    // next word to consume = window start + off, off in [0, 128)
    int32_t hrel;    // words [.., use0 + hrel) were in the ring at the start (hrel >= 192 - off)
    // the two tempered windows stay in their registers: wa/wb hold x[W + lane] and
    // x[W + 64 + lane] when ph == 0, the other way round when ph == 64 (an advance overwrites
    // the older one in place and flips ph: no register rotation, so no loop-carried copies)
    uint32_t wa, wb, ph;
    __device__ __forceinline__ uint32_t cur() const { return ph ? wb : wa; }  // tempered x[W + lane]
    uint32_t wx;     // raw x[W + 128 + lane]
    uint32_t ia, ib, im;  // raw x[p-624], x[p-623], x[p-227] for p = W + 192 + lane (the next step)
    __device__ __forceinline__ int32_t use() const { return wrel + (int32_t)off; }
    __device__ __forceinline__ uint32_t slot(int32_t rel) const { return (base + (uint32_t)rel) & kLRingMask; }
};

__device__ __forceinline__ uint32_t mt_twist(uint32_t a, uint32_t b, uint32_t m) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return m ^ (y >> 1) ^ ((b & 1u) ? 0x9908b0dfu : 0u);
}

__device__ __forceinline__ void lrng_prefetch(LRng &r) {
    const int32_t p = r.wrel + 192 + (int32_t)lane_id();
    r.ia = r.lds[r.slot(p - 624)];
    r.ib = r.lds[r.slot(p - 623)];
    r.im = r.lds[r.slot(p - 227)];
}

// Generate absolute words [g, end) in the ring, 64 at a time (every input is >= 227 older).
__device__ __forceinline__ void lrng_generate_abs(uint32_t *lds, uint64_t g, uint64_t end) {
    const uint32_t lane = lane_id();
    for (; g < end; g += 64) {
        const uint32_t p = (uint32_t)g + lane;
        const uint32_t a = lds[(p - 624) & kLRingMask], b = lds[(p - 623) & kLRingMask],
                       m = lds[(p - 227) & kLRingMask];
        if (g + lane < end) lds[p & kLRingMask] = mt_twist(a, b, m);
        wave_mem_order();
    }
}

// use0 / gen0: absolute positions (words consumed / generated) from the game's rngpos.
// Words already generated (and the seeded block 0..623, which no recurrence produces) are
// kept: an advance inside them re-reads the ring instead of generating (hrel).
__device__ __forceinline__ void lrng_open(LRng &r, uint32_t *lds, const uint32_t *ring, uint64_t use0, uint64_t gen0) {
    const uint32_t lane = lane_id();
    r.lds = lds;
    r.base = (uint32_t)use0;
    r.off = (uint32_t)use0 & (uint32_t)(kWin - 1);
    r.wrel = -(int32_t)r.off;
    const uint64_t w0 = use0 - r.off, target = w0 + 192;
    // the ring can take every word up to gen0 when gen0 - w0 <= 960 (always after this
    // kernel's own close: <= 879); an HBM kernel's lookahead may go further, and then its
    // ring is valid throughout, so the words past the first window are generated again
    const uint64_t g = gen0 <= w0 + 960 ? gen0 : (target < 624 ? 624 : target);
    for (uint32_t i = lane; i < (uint32_t)kLRingWords; i += 64) {
        const uint32_t p = (uint32_t)g - (uint32_t)kLRingWords + i;
        lds[p & kLRingMask] = ring[p & kRingMask];
    }
    wave_mem_order();
    lrng_generate_abs(lds, g, target);
    r.hrel = (int32_t)(g - use0);
    r.wa = temper(lds[r.slot(r.wrel + (int32_t)lane)]);
    r.wb = temper(lds[r.slot(r.wrel + kWin + (int32_t)lane)]);
    r.ph = 0;
    r.wx = lds[r.slot(r.wrel + 2 * kWin + (int32_t)lane)];
    lrng_prefetch(r);
}

// rng_view for the LDS stream: the window holding word off + l is wa or wb by ph
__device__ __forceinline__ uint32_t rng_view(const LRng &r) {
    const uint32_t j = lane_id() + r.off;
    const int idx = (int)(j << 2);
    const uint32_t a = (uint32_t)__builtin_amdgcn_ds_bpermute(idx, (int)r.wa);
    const uint32_t b = (uint32_t)__builtin_amdgcn_ds_bpermute(idx, (int)r.wb);
    return (j ^ r.ph) < 64u ? a : b;
}

// Move the windows on by 64 words (precondition: off >= 64); one recurrence step.
__device__ __forceinline__ void rng_advance(LRng &r) {
    r.wrel += kWin;
    r.off -= (uint32_t)kWin;
    const uint32_t t = temper(r.wx);  // the new second window replaces the old first one
    if (r.ph) r.wb = t;
    else r.wa = t;
    r.ph ^= 64u;
    const int32_t p = r.wrel + 128 + (int32_t)lane_id();
    uint32_t x = mt_twist(r.ia, r.ib, r.im);
    if (r.wrel + 128 < r.hrel) {  // only inside the seeded block: words already in the ring
        const uint32_t old = r.lds[r.slot(p)];
        x = p < r.hrel ? old : x;
    }
    r.lds[r.slot(p)] = x;
    r.wx = x;
    lrng_prefetch(r);
}

// Consume w words without reading them (the walk-replay diagnostic: a flush's recorded
// rollout words), window by window.
__device__ __forceinline__ void lrng_skip(LRng &r, uint32_t w) {
    r.off += w;
    while (r.off >= (uint32_t)kWin) rng_advance(r);
}

// Write the stream back to the game's HBM ring and rngpos (see above).
__device__ __forceinline__ void lrng_close(const LRng &r, uint32_t *ring, uint64_t use0, uint64_t *rngpos) {
    const uint32_t lane = lane_id();
    const uint64_t U = use0 + (uint64_t)(int64_t)r.use();
    uint64_t G = use0 + (uint64_t)(int64_t)max(r.wrel + 192, r.hrel);
    const uint64_t blk = U ? (U - 1) / 624 : 0;
    const uint64_t bend = (blk + 1) * 624;
    wave_mem_order();
    if (G < bend) {
        lrng_generate_abs(r.lds, G, bend);
        G = bend;
    }
    // what rng_open reads (the window of U), what zc_rng_get_state reads (U-1's block) and
    // what the recurrence reads next (the last 624 words); at most 815 words
    const uint64_t wu = U & ~(uint64_t)(kWin - 1);
    uint64_t start = wu < blk * 624 ? wu : blk * 624;
    start = start < G - 624 ? start : G - 624;
    for (uint64_t q = start + lane; q < G; q += 64) ring[(uint32_t)q & kRingMask] = r.lds[(uint32_t)q & kLRingMask];
    if (lane == 0) {
        rngpos[0] = U;
        rngpos[1] = G;
    }
}

// random._randbelow_with_getrandbits(n), 1 <= n < 2**31: k = n.bit_length(); draw
// getrandbits(k) = word >> (32-k) until < n.  All window words are tested at once; the
// first accepted one (in stream order) is the draw, and everything before it is consumed.
template <class R>
__device__ __forceinline__ uint32_t rng_below(R &r, uint32_t n) {
    const uint32_t sh = (uint32_t)__clz(n);
    const uint32_t lane = lane_id();
    for (;;) {
        if (r.off >= (uint32_t)kWin) rng_advance(r);
        const uint32_t v = r.cur() >> sh;
        // one compare: words before `off` get bit 31 set (never < n)
        const uint64_t bal = __ballot((v | ((lane - r.off) & 0x80000000u)) < n);
        if (bal) {
            const int f = __builtin_ctzll(bal);
            r.off = (uint32_t)f + 1;
            return (uint32_t)__builtin_amdgcn_readlane((int)v, f);
        }
        r.off = kWin;
    }
}

// random.choice(untried) of an expansion (policy_functions.py:12 with the untried list in
// list order, mcts.cpp:67-72): rng_below(n) as above, but every lane also looks up row[v]
// (row = sel[untried mask]: the v-th untried move) for its own candidate word, so the move
// index of the accepted draw is a readlane of that lookup (n <= 7, so v < 8).
template <class R>
__device__ __forceinline__ uint32_t rng_below_pick(R &r, uint32_t n, const uint8_t *row) {
    const uint32_t sh = (uint32_t)__clz(n);
    const uint32_t lane = lane_id();
    for (;;) {
        if (r.off >= (uint32_t)kWin) rng_advance(r);
        const uint32_t v = r.cur() >> sh;
        const uint32_t pick = row[v & 7u];
        const uint64_t bal = __ballot((v | ((lane - r.off) & 0x80000000u)) < n);
        if (bal) {
            const int f = __builtin_ctzll(bal);
            r.off = (uint32_t)f + 1;
            return (uint32_t)__builtin_amdgcn_readlane((int)pick, f);
        }
        r.off = kWin;
    }
}

// Per-search counters, accumulated in lane 0 of VGPRs (off the scalar unit, no SGPRs).
struct Counters {
    int32_t expansions = 0, depth_sum = 0, plies = 0, blocks = 0;
    __device__ __forceinline__ void add(int32_t &c, int32_t v) { c += (lane_id() == 0) ? v : 0; }
};

// A pending leaf, kept in LDS between the phases of a flush.
struct Leaf {
    uint64_t p0, p1;  // stones of 'X' / 'O'
    uint32_t meta;    // node | depth << 16 | turn << 24 | legal mask << 25
    int32_t val;      // rollout value from the leaf's side to move
    uint32_t ow;      // d_order[legal mask]: the move-list order word (saves the rollout a lookup)
    uint32_t pad;
};

// LDS copy of a node created in the current flush.  During selection the node lives only
// here; its HBM record is written in one coalesced batch when the flush's leaves are chosen.
struct Fresh {
    uint32_t u;       // untried word (record +4)
    uint32_t ow;      // packed move-list columns (record +12)
    uint32_t link;    // parent | pact << 16 | depth << 24 (record +8)
    uint32_t lmask;   // legal-column mask of the node's position
    int32_t na;       // the edge INTO this node: Na (backup accumulates here, LDS atomics)
    int32_t w;        //                          Wa
    uint32_t pad1, pad2;
    uint16_t ch[8];   // children (record +16)
};
static_assert(sizeof(Fresh) == 48, "Fresh is three 16-byte LDS slots");

// ------------------------------------------------------------------ node records
struct Tree {
    uint8_t *nodes;  // this game's records
    __device__ __forceinline__ uint8_t *rec(int nd) const { return nodes + (size_t)nd * kRecBytes; }
    __device__ __forceinline__ uint32_t *hdr(int nd) const { return (uint32_t *)rec(nd); }
    __device__ __forceinline__ uint16_t *child(int nd) const { return (uint16_t *)(rec(nd) + 16); }
    __device__ __forceinline__ int32_t *na(int nd) const { return (int32_t *)(rec(nd) + 32); }
    // +64: stepwise search: Wa in fp64 (q); rollout search: Wa as int32 (w).  Either way Qa
    // is formed as Wa / Na when read — the IEEE quotient mcts.cpp:95 stores
    __device__ __forceinline__ double *q(int nd) const { return (double *)(rec(nd) + 64); }
    __device__ __forceinline__ int32_t *w(int nd) const { return (int32_t *)(rec(nd) + 64); }
};

// Node(state, legal_moves, parent, idx) (mcts.cpp:23-34): all moves untried, in list order.
// Lanes 0..7 write slot `lane`; lane 0 writes the header.
__device__ __forceinline__ void node_init(const Tree &t, int nd, int parent, int pact, int depth, uint32_t ow) {
    const uint32_t lane = lane_id();
    const uint32_t n = (ow >> 24) & 15u;
    if (lane == 0) {
        uint4 h;
        h.x = 0;                                                                 // N
        h.y = untried_init(n);                                                   // untried, #moves
        h.z = (uint32_t)(parent & 0xFFFF) | ((uint32_t)(pact & 0xFF) << 16) | ((uint32_t)depth << 24);
        h.w = ow;
        *(uint4 *)t.rec(nd) = h;
    }
    if (lane < kSlots) {
        t.child(nd)[lane] = 0xFFFF;
        t.na(nd)[lane] = 0;
        t.q(nd)[lane] = 0.0;  // Wa (either form) = 0
    }
}

__device__ __forceinline__ bool valid_state(uint64_t p0, uint64_t p1, int turn) {
    if ((p0 & p1) || ((p0 | p1) & ~kFull) || (turn & ~1)) return false;
    const uint64_t occ = p0 | p1;
#pragma unroll
    for (int c = 0; c < 7; ++c) {
        const uint64_t col = (occ >> (7 * c)) & 0x3Full;
        if (col & (col + 1)) return false;  // stones must stack from the bottom
    }
    return true;
}

// ------------------------------------------------------------------ phase stamps (diagnostic)
template <bool ON>
struct Stamp {
    uint64_t ph[kPhases];
    uint64_t t;
    __device__ __forceinline__ Stamp() : t(ON ? __builtin_amdgcn_s_memtime() : 0) {
        for (int i = 0; i < kPhases; ++i) ph[i] = 0;
    }
    __device__ __forceinline__ void mark(int k) {
        if (ON) {
            const uint64_t now = __builtin_amdgcn_s_memtime();
            ph[k] += now - t;
            t = now;
        }
    }
};

using ConstDouble = const __attribute__((address_space(4))) double;

// ------------------------------------------------------------------ selection of one flush
// What a flush's selection leaves behind for its backup and publish steps.
struct FlushSel {
    int f0;          // first node created in this flush
    int x0node, d0;  // X0: where the first walk stopped, and its depth
    uint32_t ppath;  // lane l (l <= d0): level l of root..X0 = node | slot << 16
    bool x0_dirty;   // X0 expanded during the flush (its record must be rewritten)
    uint32_t x_u, x_ch;  // X0's untried word / child slot `lane & 7` as last seen
    // select_flush_plan2 only (planned = true): the fresh nodes are the draws 0..D-1; bit j of
    // Sm: draw j is a chain node's first draw; bit j of Z: draw j created the next chain node
    bool planned = false;
    int D = 0;
    uint64_t Sm = 0, Z = 0;
};

// The walk from the root over HBM records (select, mcts.cpp:47-63): the UCT child (first
// maximum, +inf for an unvisited edge) until a node with untried moves or without children.
// QW = false: the record's +64 slots hold Wa as int32 (rollout search: values are +-1/0);
// QW = true:  they hold Wa in fp64 (stepwise search).  Q = Wa / Na is formed here — the same
//             IEEE quotient mcts.cpp:95 stores, so the UCT inputs are bit-identical.
struct WalkEnd {
    int node, depth, turn;
    uint64_t b0, b1;     // the node's position
    uint32_t pathv;      // lane l (l <= depth): level l of the path = node | slot << 16
    uint32_t u, ow, ch;  // the node's record (ch: slot lane & 7)
};
template <bool QW>
__device__ __forceinline__ WalkEnd walk_hbm(const Tree &t, ConstDouble *logtab, uint64_t rp0, uint64_t rp1,
                                            int rturn, int done, double c, int &status) {
    const uint32_t lane = lane_id();
    const uint32_t k = lane & 7u;
    int node = 0, depth = 0, turn = rturn, nN = done;  // nN = N(node) = Na of its in-edge
    uint64_t b0 = rp0, b1 = rp1;
    uint32_t pathv = (lane == 0) ? 0x00FF0000u : 0u;
    uint32_t u, ow, ch;  // the current node's record (ch: slot k)
    for (;;) {  // the first walk: select (mcts.cpp:47-63) over HBM records
        const uint8_t *R = t.rec(node);
        const uint4 h = *(const uint4 *)R;
        ch = ((const uint16_t *)(R + 16))[k];
        const int32_t na = ((const int32_t *)(R + 32))[k];
        // Wa: fp64 (QW) or int32 (rollout search)
        const double qw = QW ? ((const double *)(R + 64))[k] : (double)((const int32_t *)(R + 64))[k];
        const double lg = logtab[nN];  // log(N), glibc values tabulated on the host
        u = uni(h.y);
        ow = uni(h.w);
        if (untried_count(u)) break;  // untried moves left: expand here
        if (depth >= kMaxDepth - 2) {  // unreachable (a C4 tree is <= 42 deep); never spin
            status = ZC_STATUS_INTERNAL;
            u = 0;
            break;
        }
        const uint32_t nm = u >> 28;
        const bool valid = k < nm && ch != 0xFFFF;
        int best;
        // slots k < nm (a scalar mask) with a child and no visit: masks ANDed, no per-lane bool
        const uint64_t unvisited = ((1ull << nm) - 1ull) & __ballot(ch != 0xFFFF) & __ballot(na == 0) & 0xFFull;
        if (unvisited) {  // +inf beats everything; first such slot
            best = __builtin_ctzll(unvisited);
        } else {
            // UCT (mcts.cpp:41-45) = fma(c, sqrt(log(N)/Na), Qa), first max in slot order
            const double q = valid ? qw / (double)na : 0.0;
            const double v = valid ? fma(c, sqrt(lg / (double)na), q) : -INFINITY;
#ifndef ZC_MAX8
#define ZC_MAX8 1  // 0: the compare-and-swap argmax8 (A/B runs)
#endif
            int bi;
            if (ZC_MAX8) {
                const double mx = max8_first(v, &bi);
                if ((__ballot(mx == -INFINITY) & 1ull) != 0) break;  // no child: terminal leaf
            } else {
                double vv = v;
                bi = (int)k;
                argmax8(vv, bi);
                if ((__ballot(vv == -INFINITY) & 1ull) != 0) break;
                bi = uni(bi);
            }
            best = bi;
        }
        const int nxt = __builtin_amdgcn_readlane((int)ch, best);
        nN = __builtin_amdgcn_readlane(na, best);
        const uint64_t bit = drop_bit(b0 | b1, (int)((ow >> (3 * best)) & 7u));
        if (turn) b1 |= bit; else b0 |= bit;
        turn ^= 1;
        node = nxt;
        ++depth;
        if (lane == (uint32_t)depth) pathv = (uint32_t)node | ((uint32_t)best << 16);
    }
    return WalkEnd{node, depth, turn, b0, b1, pathv, u, ow, ch};
}

// select + expand of the nb leaves of one flush (mcts.cpp:129-147), shared by the fused
// rollout search and the stepwise search.
//
// No backup happens inside a flush, so (1) the UCT path from the root to the node X0 where
// the flush's first walk stops is shared by every leaf of the flush (each walk resumes where
// the previous one expanded, always at or below X0), and (2) every node below X0 is created
// in this flush ("fresh": id >= f0, Na = W = 0 on every edge).  The reference's walk from a
// node without untried moves takes the first child with the largest UCT; an unvisited child
// scores +inf, so below X0 that is simply the lowest slot holding a fresh child — no
// arithmetic, no HBM.  Fresh nodes live in LDS (`fresh`) until the caller publishes them.
// Leaf j goes to leaves[j] (board, node, depth, turn, legal mask) and its path (node ids of
// levels 0..depth) to paths[j][*] (paths = nullptr: not recorded; the fresh part of a path is
// also the chain of parent links in `fresh`).  QW: as walk_hbm.
template <bool QW, bool STAMP, class RNG>
__device__ __forceinline__ void select_flush(const Tree &t, Fresh *fresh, Leaf *leaves, uint16_t *paths,
                                             const uint32_t *s_order, ConstDouble *logtab,
                                             RNG &rng, Counters &cn, Stamp<STAMP> &stamp, int &nnodes, int &status,
                                             uint64_t rp0, uint64_t rp1, int rturn, int done, int nb, double c,
                                             FlushSel &fs) {
    const uint32_t lane = lane_id();
    const uint32_t k = lane & 7u;  // child slot handled by this lane (lanes 8.. mirror 0..7)
    const int f0 = nnodes;
    for (int i = (int)lane; i < nb; i += 64) {  // fresh slots: no children, zero in-edge counters
        fresh[i].na = 0;
        fresh[i].w = 0;
        *(uint4 *)fresh[i].ch = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
    }
    WalkEnd we = walk_hbm<QW>(t, logtab, rp0, rp1, rturn, done, c, status);
    int node = we.node, depth = we.depth, turn = we.turn;
    uint64_t b0 = we.b0, b1 = we.b1;
    uint32_t pathv = we.pathv, u = we.u, ow = we.ow, ch = we.ch;
    int cmask = legal_mask(b0 | b1);  // legal columns of the current node
    const int x0node = node;
    bool x0_dirty = false;
    uint32_t x_u = u, x_ch = ch;
    fs.f0 = f0;
    fs.x0node = x0node;
    fs.d0 = depth;
    fs.ppath = pathv;
    stamp.mark(1);

    // The rest of the flush, a node at a time.  Below X0 the walks take the lowest slot
    // holding a fresh child and a node is left only once it has no untried move, so the
    // flush visits a chain of nodes X0 = N0, N1, ... and at each one expands m = min(#untried,
    // leaves left) moves in a row: m random.choice draws over m, m-1, ... remaining moves
    // (count-sequence known in advance), then the next node is N's child in its lowest slot.
    // The draws are a scalar chain over ONE 64-word view (the accepted word of each draw is
    // the first word after the previous one with (w >> (32-k)) < n); the children and their
    // leaves are then built lane-parallel (lane i = the i-th draw), and the walk into the next
    // node reads the child from those lanes — no LDS round trip, no per-leaf scalar work.
    // ul: the node's untried list (move indices in list order, 3 bits each; random.choice's
    // r-th element, erased in place as mcts.cpp:67-72 does).
    constexpr uint32_t kIdentList = 0x1AC688u;  // 0, 1, ..., 6
    uint32_t ul = 0;
    {
        uint32_t c = 0;
        for (uint32_t bb = 0; bb < 7; ++bb)
            if ((u >> bb) & 1u) ul |= bb << (3 * c++);
    }
    int bulk0 = 0;          // first node id of the last bulk (the children of `node`)
    uint32_t invl = 0;      // lane k: 8 | i when slot k of `node` was expanded by draw i of that bulk
    uint32_t c_low = 0, c_lmask = 0;  // lane i: child i's order word / legal mask
    int j = 0;
    while (j < nb) {
        const uint32_t cnt = untried_count(u);
        if (cnt == 0) {
            const uint64_t fm = ((1ull << (u >> 28)) - 1ull) & __ballot(ch != 0xFFFF) & __ballot((int)ch >= f0) & 0xFFull;
            if (!fm) {  // no child at all: terminal, every remaining leaf of the flush is this node
                const uint32_t meta = (uint32_t)node | ((uint32_t)depth << 16) | ((uint32_t)turn << 24) |
                                      ((uint32_t)cmask << 25);
                for (int i = (int)lane; j + i < nb; i += 64) leaves[j + i] = Leaf{b0, b1, meta, 0, ow, 0};
                if (paths)
                    for (int jj = j; jj < nb; ++jj) paths[jj * kMaxDepth + lane] = (uint16_t)pathv;
                j = nb;
                wave_mem_order();
                break;
            }
            const int s = __builtin_ctzll(fm);
            const int i = __builtin_amdgcn_readlane((int)invl, s) & 7;
            const int child = bulk0 + i;
            if (node == x0node) {  // leaving X0 for good (walks never go back up)
                x_u = u;
                x_ch = ch;
            }
            const uint64_t bit = drop_bit(b0 | b1, (int)((ow >> (3 * s)) & 7u));
            if (turn) b1 |= bit; else b0 |= bit;
            turn ^= 1;
            ++depth;
            if (lane == (uint32_t)depth) pathv = (uint32_t)child | ((uint32_t)s << 16);
            node = child;
            ow = (uint32_t)__builtin_amdgcn_readlane((int)c_low, i);
            cmask = __builtin_amdgcn_readlane((int)c_lmask, i);
            u = untried_init((ow >> 24) & 15u);
            ul = kIdentList;
            ch = 0xFFFF;
            stamp.mark(2);
            continue;
        }
        // ---- m draws (random.choice over cnt, cnt-1, ... untried moves)
        const int m = min((int)cnt, nb - j);
        uint32_t rr = 0;  // lane i < m: draw i's value r (the index into the untried list then)
        {
            int done = 0;
            for (;;) {  // one 64-word view per pass
                if (rng.off >= (uint32_t)kWin) rng_advance(rng);
                const uint32_t w = rng_view(rng);  // lane l: word off + l
                const int rem = m - done;
                // acceptance masks of the next (up to 7) draws, n = cnt - done - i: independent
                // of each other, issued back to back
                uint64_t A[7];
#pragma unroll
                for (int i = 0; i < 7; ++i) {
                    const uint32_t n = (uint32_t)max((int)cnt - done - i, 1);
                    A[i] = __ballot((w >> __clz(n)) < n);
                }
                // the draws, a branch-free scalar chain: each takes the lowest accepted word
                // after the last one (lb = acc & -acc); a draw without one zeroes `gt`, and with
                // it every later draw of the view
                uint64_t gt = ~0ull, F = 0;  // lanes after the last accepted word; accepted words
#pragma unroll
                for (int i = 0; i < 7; ++i) {
                    const uint64_t acc = (i < rem ? A[i] : 0ull) & gt;
                    const uint64_t lb = acc & (0ull - acc);
                    F |= lb;
                    gt = 0ull - (lb << 1);
                }
                const int nd = __popcll(F);
                const int f = 63 - __clzll(F | 1ull);  // the last accepted word (F != 0 when nd > 0)
                // lane-parallel: accepted word l is draw di = done + (accepted words below it);
                // its value goes to lane di (a forward permute; lanes outside [done, done + nd)
                // keep theirs)
                const uint32_t di = (uint32_t)done + mbcnt64(F);
                const uint32_t rl = w >> __clz(max((int)cnt - (int)di, 1));
                const uint32_t got = (uint32_t)__builtin_amdgcn_ds_permute((int)(mask_sel(F, 63u, di) << 2), (int)rl);
                rr = mask_sel(((1ull << nd) - 1ull) << done, rr, got);  // lanes done .. done + nd - 1
                done += nd;
                if (done < m) {  // the view ran out: all of it is consumed
                    rng.off += (uint32_t)kWin;
                    continue;
                }
                rng.off += (uint32_t)f + 1u;
                break;
            }
        }
        // draw i's position in the untried list as it was before the bulk (the erase of
        // mcts.cpp:72 undone all at once, a Lehmer code: later draws skip the earlier picks)
        // (step i compares with draw i's own r: lane i is only adjusted by the later steps i' < i)
        uint32_t pl = rr;
        uint32_t rpick[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) rpick[i] = (uint32_t)__builtin_amdgcn_readlane((int)rr, i);
#pragma unroll
        for (int i = 5; i >= 0; --i) {
            const uint64_t later = ((1ull << m) - 1ull) & ~((2ull << i) - 1ull);  // lanes i+1 .. m-1
            pl = add_in_mask(pl, __ballot(pl >= rpick[i]) & later);
        }
        const uint32_t mi_l = (ul >> (3 * (pl & 7u))) & 7u;  // lane i < m: draw i's move index
        // the expanded slots (OR over lanes 0..7, DPP) and, in lane k, the draw that took slot k
        uint32_t slotbit = (int)lane < m ? 1u << mi_l : 0u;
        slotbit |= (uint32_t)dpp<0xB1>((int)slotbit);
        slotbit |= (uint32_t)dpp<0x4E>((int)slotbit);
        slotbit |= (uint32_t)dpp<0x141>((int)slotbit);
        const uint32_t ucl = uni(slotbit);
        const uint32_t sent = (uint32_t)__builtin_amdgcn_ds_permute((int)(((int)lane < m ? mi_l : 63u) << 2),
                                                                     (int)(8u | lane));
        invl = (ucl >> (lane & 7u)) & 1u ? sent : 0u;
        u &= ~ucl;
        // ---- the m children and their leaves, lane i = draw i
        {
            const uint32_t mi = mi_l;
            const int col = (int)((ow >> (3 * mi)) & 7u);
            const uint64_t bit = drop_bit(b0 | b1, col);
            const bool filled = (bit & kTop) != 0;
            c_lmask = (uint32_t)cmask & ~(filled ? (1u << col) : 0u);
            c_low = ow;
            if ((int)lane < m && filled) c_low = s_order[c_lmask];
            const int ldepth = depth + 1;
            const uint32_t leaf = (uint32_t)nnodes + lane;
            if ((int)lane < m) {
                *(uint4 *)&fresh[leaf - (uint32_t)f0] =
                    make_uint4(untried_init((c_low >> 24) & 15u), c_low,
                               (uint32_t)node | (mi << 16) | ((uint32_t)ldepth << 24), c_lmask);
                const uint64_t l0 = turn ? b0 : (b0 | bit), l1 = turn ? (b1 | bit) : b1;
                leaves[j + (int)lane] = Leaf{l0, l1,
                                             leaf | ((uint32_t)ldepth << 16) | ((uint32_t)(turn ^ 1) << 24) | (c_lmask << 25),
                                             0, c_low, 0};
            }
            // leaf j+i's path: the walk's path plus the new node (all 64 lanes store: lanes
            // >= kMaxDepth spill into the next leaf's path, written after this, or the spill bytes)
            if (paths)
                for (int i = 0; i < m; ++i)
                    paths[(j + i) * kMaxDepth + lane] = (uint16_t)(lane == (uint32_t)ldepth ? (uint32_t)(nnodes + i) : pathv);
            // the node's new children
            const uint32_t pk = lane < 8 ? invl : 0u;
            if (pk & 8u) ch = (uint32_t)nnodes + (pk & 7u);
            if (node >= f0) {  // the node's copy in LDS
                if (lane == 0) fresh[node - f0].u = u;
                if (lane < 8 && (pk & 8u)) fresh[node - f0].ch[k] = (uint16_t)ch;
            } else {
                x0_dirty = true;  // X0 itself: written back when the flush is published
            }
            wave_mem_order();
        }
        bulk0 = nnodes;
        nnodes += m;
        j += m;
        stamp.mark(3);
    }
    if (node == x0node) {
        x_u = u;
        x_ch = ch;
    }
    // the flush's expansions = its fresh nodes; their depths summed lane-parallel (bit-sliced
    // ballots) instead of per expansion on the chain
    {
        const int nf = nnodes - f0;
        int dsum = 0;
        for (int base = 0; base < nf; base += 64) {
            const int i = base + (int)lane;
            const uint32_t d = i < nf ? fresh[i].link >> 24 : 0u;
#pragma unroll
            for (int bit = 0; bit < 6; ++bit) dsum += __popcll(__ballot((d >> bit) & 1u)) << bit;
        }
        cn.add(cn.expansions, nf);
        cn.add(cn.depth_sum, dsum);
    }
    fs.x0_dirty = x0_dirty;
    fs.x_u = x_u;
    fs.x_ch = x_ch;
}

}  // namespace
}  // namespace zc
