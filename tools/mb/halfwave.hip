// halfwave.hip — measured A/B of the Connect4 rollout loop: ONE game per wave (the product's
// c4_rollouts, zeroclone_amd/csrc/c4_search.hip) against TWO games per wave, lanes 0-31 and
// 32-63 (DESIGN §9's half-wave design), on the rollout phase alone — 78 %
// of the headline kernel's time (extra.phases.share.rollout).
//
// Workload: G games, each with its own CPython MT19937 stream (the words from position 624 of
// init_genrand(seed + g), as after random.seed), rolls out F flushes x 32 leaves in order
// (value_functions.py:35-45 per leaf, mcts.cpp:112-127 per flush), the leaves being positions
// of seeded random play (0..30 stones; some already won, some full).  Both kernels must give
// every leaf the same value and leave every stream at the same position (bit-exact); then each
// is timed with HIP events.  Occupancy is the headline's: the full-wave kernel runs G waves
// (4 games per workgroup, 16 waves per CU at G = 4096), the half-wave one G / 2 waves.
//
// The half-wave form, per block of plies, per half h (its own game):
//   * a 32-word view of its stream (its own LDS ring, 32-word windows in the half's lanes);
//   * acceptance ballot, per-half ply index (mbcnt minus the lower half's count), a 32-lane
//     prefix sum of per-column nibble counters (5 DPP steps: the 64-lane scan without the
//     row_bcast:31 step that would cross halves);
//   * the block end per half (first fill / the cap / the last accepted word) from the two
//     32-bit halves of each ballot, the first fill absorbed per half (re-drawn under the new
//     legal set; the order word of the legal set minus one column from a 7-lane table per
//     half instead of the full-wave kernel's 49-lane pair table);
//   * the win test on the compacted plies: ply q of half h to lane 32h + (q & 1) * 16 + q / 2
//     (one forward permute), a 16-lane prefix OR per row, and every row testing all four
//     directions (the full-wave kernel tests two per row on a copied half);
//   * each half's rollout ends on its own; a half then takes its next leaf (or idles once its
//     32 leaves are done) while the other half goes on.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math \
//        -I include -o tools/mb/halfwave tools/mb/halfwave.hip      (tools/mb/build_halfwave.sh)
// Run:   tools/mb/halfwave [games] [flushes] [reps]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../../zeroclone_amd/csrc/c4_search.hip"

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

namespace hw {
using namespace zc;

struct LeafIn {  // one leaf as the host builds it
    uint64_t p0, p1;
    uint32_t turn, pad;
};

constexpr int kLeaves = 32;          // leaves per flush (batch_size 32)
constexpr int kGames = 4;            // games per full-wave workgroup (one wave each)
constexpr int kRingBytes = 4096;     // LDS ring per game (1024 words)
constexpr int kLeafBytes = kLeaves * (int)sizeof(Leaf);

__device__ __forceinline__ void make_leaf(Leaf &o, const LeafIn &in, const uint32_t *s_order) {
    o.p0 = in.p0;
    o.p1 = in.p1;
    const int lm = legal_mask(in.p0 | in.p1);
    o.meta = (in.turn << 24) | ((uint32_t)lm << 25);
    o.ow = s_order[lm];
    o.val = 0;
}

// ------------------------------------------------------------------ full wave (the product)
__global__ __launch_bounds__(64 * kGames) void full_kernel(const uint32_t *rings, const LeafIn *leaves, int G, int F,
                                                           int32_t *vals, int64_t *uses) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t *s_order = (uint32_t *)smem;
    load_tables(s_order);
    __syncthreads();
    const int wave = (int)(threadIdx.x >> 6);
    const int g = (int)blockIdx.x * kGames + wave;
    if (g >= G) return;
    uint8_t *mine = smem + kTabBytes + wave * (kRingBytes + kLeafBytes);
    uint32_t *ring = (uint32_t *)mine;
    Leaf *L = (Leaf *)(mine + kRingBytes);
    const uint32_t lane = lane_id();
    LRng r;
    lrng_open(r, ring, rings + (size_t)g * kRingWords, 624, 624);
    Counters cn;
    for (int f = 0; f < F; ++f) {
        if (lane < (uint32_t)kLeaves) make_leaf(L[lane], leaves[((size_t)g * F + f) * kLeaves + lane], s_order);
        wave_mem_order();
        c4_rollouts(L, kLeaves, r, s_order, cn);
        wave_mem_order();
        if (lane < (uint32_t)kLeaves) vals[((size_t)g * F + f) * kLeaves + lane] = L[lane].val;
        wave_mem_order();
    }
    if (lane == 0) uses[g] = 624 + (int64_t)r.use();
}

// ------------------------------------------------------------------ half wave
// Per-lane values that are uniform within each half ("half-uniform") carry each game's state;
// per-half decisions read the two 32-bit halves of the ballots on the scalar unit.
__device__ __forceinline__ uint32_t hsel(uint32_t lo, uint32_t hi) {  // lanes < 32: lo, else hi
    return mask_sel(0xFFFFFFFFull, hi, lo);
}
__device__ __forceinline__ uint32_t ffs32(uint32_t m) { return m ? (uint32_t)__builtin_ctz(m) : 32u; }

// The stream of one half's game: an LDS ring of 1024 raw words (as LRng), 32-word windows.
struct HRng {
    uint32_t *lds;   // this half's ring (per lane)
    uint32_t base;   // use0 (low bits)
    int32_t wrel;    // window start - use0
    uint32_t off;    // next word = window start + off, off in [0, 64)
    uint32_t wa, wb, ph;  // tempered x[W + l], x[W + 32 + l] (by ph), l = lane & 31
    uint32_t wx;          // raw x[W + 64 + l]
    uint32_t ia, ib, im;  // inputs of x[W + 96 + l]
    __device__ __forceinline__ uint32_t slot(int32_t rel) const { return (base + (uint32_t)rel) & kLRingMask; }
};

__device__ __forceinline__ void hrng_prefetch(HRng &r) {
    const int32_t p = r.wrel + 96 + (int32_t)(lane_id() & 31u);
    r.ia = r.lds[r.slot(p - 624)];
    r.ib = r.lds[r.slot(p - 623)];
    r.im = r.lds[r.slot(p - 227)];
}

// use0 = gen0 (a fresh stream: the words are generated from the seeded block on)
__device__ void hrng_open(HRng &r, uint32_t *lds, const uint32_t *ring, uint32_t use0) {
    const uint32_t l = lane_id() & 31u;
    r.lds = lds;
    r.base = use0;
    r.off = use0 & 31u;
    r.wrel = -(int32_t)r.off;
    for (uint32_t i = l; i < (uint32_t)kLRingWords; i += 32) {
        const uint32_t p = use0 - (uint32_t)kLRingWords + i;
        lds[p & kLRingMask] = ring[p & kRingMask];
    }
    wave_mem_order();
    const uint32_t target = use0 - r.off + 96;
    for (uint32_t g = use0; g < target; g += 32) {
        const uint32_t p = g + l;
        const uint32_t a = lds[(p - 624) & kLRingMask], b = lds[(p - 623) & kLRingMask], m = lds[(p - 227) & kLRingMask];
        if (p < target) lds[p & kLRingMask] = mt_twist(a, b, m);
        wave_mem_order();
    }
    r.wa = temper(lds[r.slot(r.wrel + (int32_t)l)]);
    r.wb = temper(lds[r.slot(r.wrel + 32 + (int32_t)l)]);
    r.ph = 0;
    r.wx = lds[r.slot(r.wrel + 64 + (int32_t)l)];
    hrng_prefetch(r);
}

__device__ __forceinline__ uint32_t hrng_view(const HRng &r) {  // lane l: word off + (l & 31) of its game
    const uint32_t lane = lane_id();
    const uint32_t j = (lane & 31u) + r.off;
    const int idx = (int)(((lane & 32u) | (j & 31u)) << 2);
    const uint32_t a = (uint32_t)__builtin_amdgcn_ds_bpermute(idx, (int)r.wa);
    const uint32_t b = (uint32_t)__builtin_amdgcn_ds_bpermute(idx, (int)r.wb);
    return (j ^ r.ph) < 32u ? a : b;
}

__device__ __forceinline__ void hrng_advance(HRng &r) {  // precondition off >= 32 (lanes of advancing halves)
    r.wrel += 32;
    r.off -= 32u;
    const uint32_t t = temper(r.wx);
    if (r.ph) r.wb = t;
    else r.wa = t;
    r.ph ^= 32u;
    const int32_t p = r.wrel + 64 + (int32_t)(lane_id() & 31u);
    const uint32_t x = mt_twist(r.ia, r.ib, r.im);
    r.lds[r.slot(p)] = x;
    r.wx = x;
    hrng_prefetch(r);
}

// Inclusive prefix sum within each 32-lane half (the 64-lane scan_add32 without row_bcast:31).
__device__ __forceinline__ uint32_t scan_add_half(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
    return x;
}

__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l); }
// lane (lane & 32) + k of v: a per-half readlane (k half-uniform)
__device__ __forceinline__ uint32_t hpick(uint32_t v, uint32_t k) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((lane_id() & 32u) + k) << 2), (int)v);
}
__device__ __forceinline__ uint64_t hpick64(uint64_t v, uint32_t k) {
    return ((uint64_t)hpick((uint32_t)(v >> 32), k) << 32) | hpick((uint32_t)v, k);
}

// Rollout state of one half's current leaf (half-uniform values)
struct HState {
    uint64_t me, op;   // side to move / last mover stones
    uint32_t hp;       // column heights, 4 bits per column
    int32_t room, room0;
    uint32_t mask, ow, owt, n, sh;  // legal set, its order word, the 7-lane table, count, shift
    int32_t j;         // the half's current leaf
};

// Take the half's next leaf that needs plies: won or full leaves get their value at once.
// Runs on the lanes of the halves that call it.  Returns false (in those lanes) when the half
// has no leaf left.
__device__ bool h_next_leaf(HState &s, Leaf *L, int nb, const uint32_t *s_order) {
    const uint32_t lane = lane_id();
    for (;;) {
        if (s.j >= nb) return false;
        const Leaf &lf = L[s.j];
        const uint32_t lm = lf.meta;
        const uint32_t tn = (lm >> 24) & 1u;
        const uint64_t x0 = lf.p0, x1 = lf.p1;
        const uint64_t op = tn ? x0 : x1;
        const int room0 = has_four(op) ? -2 : 41 - __popcll(x0 | x1);
        if (room0 < 0) {  // won by the last mover (-1) or a full board (0)
            if ((lane & 31u) == 0) L[s.j].val = room0 == -2 ? -1 : 0;
            ++s.j;
            continue;
        }
        s.me = tn ? x1 : x0;
        s.op = op;
        const uint64_t oc = x0 | x1;
        uint32_t hp = 0;
        for (int c = 0; c < 7; ++c) hp |= (uint32_t)__popcll((oc >> (7 * c)) & 0x3Full) << (4 * c);
        s.hp = hp;
        s.room = s.room0 = room0;
        s.mask = lm >> 25;
        s.ow = lf.ow;
        s.n = (s.ow >> 24) & 15u;
        s.sh = (uint32_t)__builtin_clz(s.n);
        const uint32_t c = lane & 31u;
        s.owt = c < 7u ? s_order[s.mask & ~(1u << c)] : 0u;
        return true;
    }
}

__device__ void rollouts_pair(Leaf *LA, Leaf *LB, int nb, HRng &r, const uint32_t *s_order) {
    const uint32_t lane = lane_id();
    const uint32_t H = lane >> 5;
    const uint32_t c5 = lane & 31u;
    const bool even_row = (lane & 16u) == 0;  // rows 0 (lanes 0-15, 32-47): the block's first mover
    Leaf *L = H ? LB : LA;
    HState s;
    s.j = 0;
    bool act = h_next_leaf(s, L, nb, s_order);
    // per-half activity as wave masks: lanes of active halves
    uint64_t actm = __ballot(act);
    while (actm) {
        const bool aA = (uint32_t)actm != 0u, aB = (actm >> 32) != 0ull;
        // the view (an empty one — probability 2^-32 per half — is consumed whole)
        if (act && r.off >= 32u) hrng_advance(r);
        uint32_t wv = hrng_view(r);
        uint32_t v = wv >> s.sh;
        uint64_t A = __ballot(v < s.n) & actm;
        while (__builtin_expect((aA && (uint32_t)A == 0u) || (aB && (A >> 32) == 0ull), 0)) {
            const bool empty = act && (H ? (A >> 32) == 0ull : (uint32_t)A == 0u);
            if (empty) {
                r.off += 32u;
                hrng_advance(r);
            }
            wv = hrng_view(r);
            v = wv >> s.sh;
            A = __ballot(v < s.n) & actm;
        }
        const uint32_t cap = (uint32_t)min(s.room, 30);
        const uint32_t nlo = (uint32_t)__popc((uint32_t)A), nhi = (uint32_t)__popc((uint32_t)(A >> 32));
        uint32_t qk = mbcnt(A) - (H ? nlo : 0u);
        uint32_t col = (s.ow >> (3 * v)) & 7u;
        uint32_t one = mask_sel0(A, 1u << (4 * col));
        uint32_t sc = scan_add_half(one);
        uint32_t row = ((sc - one + s.hp) >> (4 * col)) & 15u;
        uint32_t nacc = hsel(nlo, nhi);
        uint64_t F = __ballot(row == 5u);
        uint64_t E0 = A & (F | __ballot(qk >= min(cap, nacc - 1u)));
        uint32_t l0A = ffs32((uint32_t)E0), l0B = ffs32((uint32_t)(E0 >> 32));
        const uint64_t Gm = A & F & __ballot(qk < cap);
        const bool absA = aA && ffs32((uint32_t)Gm) == l0A;
        const bool absB = aB && ffs32((uint32_t)(Gm >> 32)) == l0B;
        uint32_t lfA = 64u, lfB = 64u, cfA = 0u, cfB = 0u;
        if (absA || absB) {
            uint64_t low = 0ull;
            uint32_t ow2A = 0u, ow2B = 0u;
            if (absA) {
                lfA = l0A;
                cfA = rl(col, lfA);
                ow2A = rl(s.owt, cfA);
                low |= (2ull << lfA) - 1ull;
            } else {
                low |= 0xFFFFFFFFull;
            }
            if (absB) {
                lfB = l0B;
                cfB = rl(col, 32u + lfB);
                ow2B = rl(s.owt, 32u + cfB);
                low |= ((2ull << lfB) - 1ull) << 32;
            } else {
                low |= 0xFFFFFFFF00000000ull;
            }
            const uint32_t ow2 = hsel(ow2A, ow2B);
            const uint32_t n2 = (ow2 >> 24) & 15u;
            const uint32_t v2 = wv >> __clz(n2 | 1u);
            A = (A & low) | (__ballot(v2 < n2) & ~low & actm);
            const uint32_t mlo = (uint32_t)__popc((uint32_t)A);
            qk = mbcnt(A) - (H ? mlo : 0u);
            col = mask_sel(low, (ow2 >> (3 * v2)) & 7u, col);
            one = mask_sel0(A, 1u << (4 * col));
            sc = scan_add_half(one);
            row = ((sc - one + s.hp) >> (4 * col)) & 15u;
            nacc = hsel(mlo, (uint32_t)__popc((uint32_t)(A >> 32)));
            F = (__ballot(row == 5u) & ~low) | (F & ~(absA ? 0xFFFFFFFFull : 0ull) & ~(absB ? 0xFFFFFFFF00000000ull : 0ull));
            E0 = A & (F | __ballot(qk >= min(cap, nacc - 1u)));
            l0A = ffs32((uint32_t)E0);
            l0B = ffs32((uint32_t)(E0 >> 32));
        }
        // the win test on the compacted plies
        const uint32_t cq = ((qk & 1u) << 4) | ((qk >> 1) & 15u);
        const uint32_t dest = (lane & 32u) | mask_sel(A, 31u, cq);
        const uint32_t b = __umul24(col, 7u) + row;
        const uint32_t pl = (uint32_t)__builtin_amdgcn_ds_permute((int)(dest << 2), (int)b);
        const uint64_t bit = 1ull << (pl & 63u);
        uint32_t blo = (uint32_t)bit, bhi = (uint32_t)(bit >> 32);
        scan_or16x2(blo, bhi);
        const uint64_t mine = ((uint64_t)bhi << 32) | blo;
        const uint64_t bd = (even_row ? s.me : s.op) | mine;
        uint64_t m = bd & (bd >> 1), f4 = m & (m >> 2);
        m = bd & (bd >> 7);
        f4 |= m & (m >> 14);
        m = bd & (bd >> 6);
        f4 |= m & (m >> 12);
        m = bd & (bd >> 8);
        f4 |= m & (m >> 16);
        const uint64_t W = __ballot(f4 != 0ull);
        const uint32_t Wh = hsel((uint32_t)W, (uint32_t)(W >> 32));
        const uint64_t Ew = A & __ballot(((Wh >> cq) & 1u) != 0u);
        const uint32_t ewA = ffs32((uint32_t)Ew), ewB = ffs32((uint32_t)(Ew >> 32));
        const uint32_t endA = min(ewA, l0A), endB = min(ewB, l0B);
        const bool winA = ewA <= l0A, winB = ewB <= l0B;
        const uint32_t eplyA = aA ? rl(qk, endA) : 0u, eplyB = aB ? rl(qk, 32u + endB) : 0u;
        const uint32_t endl = hsel(endA, endB), eply = hsel(eplyA, eplyB);
        const bool win = H ? winB : winA;
        if (act) {
            r.off += endl + 1u;
            s.room -= (int32_t)eply + 1;
        }
        const bool done = act && (win || s.room < 0);
        if (act && !done) {
            // the rollout goes on (off the common path): both sides' stones after ply eply,
            // the heights, and the legal set after the block's fills
            const uint64_t s1 = hpick64(mine, eply >> 1);          // first mover through ply 2 (eply / 2)
            const uint64_t s2 = hpick64(mine, (eply + 31u) >> 1);  // second mover through the odd plies <= eply
            const uint64_t a2 = s.me | s1;
            const uint64_t b2 = s.op | (eply ? s2 : 0ull);
            const bool odd = eply & 1u;
            s.me = odd ? a2 : b2;
            s.op = odd ? b2 : a2;
            s.hp += hpick(sc, endl);
            const uint32_t lf = H ? lfB : lfA, cf = H ? cfB : cfA;
            const bool fa = endl >= lf;
            const bool fe = ((F >> ((lane & 32u) + endl)) & 1ull) != 0ull;
            const uint32_t ce = fe ? hpick(col, endl) : cf;
            const uint32_t ca = fa ? cf : ce;
            if (fa | fe) {
                s.mask &= ~((1u << ca) | (1u << ce));
                s.ow = s_order[s.mask];
                s.owt = c5 < 7u ? s_order[s.mask & ~(1u << c5)] : 0u;
            }
            s.n = (s.ow >> 24) & 15u;
            s.sh = (uint32_t)__builtin_clz(s.n);
        }
        if (done) {
            if (c5 == 0) L[s.j].val = win ? (((s.room0 - s.room) & 1) ? 1 : -1) : 0;
            ++s.j;
            act = h_next_leaf(s, L, nb, s_order);
        }
        actm = __ballot(act);
    }
}

__global__ __launch_bounds__(64 * kGames) void half_kernel(const uint32_t *rings, const LeafIn *leaves, int G, int F,
                                                           int32_t *vals, int64_t *uses) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t *s_order = (uint32_t *)smem;
    load_tables(s_order);
    __syncthreads();
    const int wave = (int)(threadIdx.x >> 6);
    const int g0 = ((int)blockIdx.x * kGames + wave) * 2;  // this wave's two games: g0 (lanes 0-31), g0 + 1
    if (g0 >= G) return;
    const uint32_t lane = lane_id();
    const uint32_t H = lane >> 5;
    const int g = g0 + (int)H;
    uint8_t *mine = smem + kTabBytes + wave * 2 * (kRingBytes + kLeafBytes);
    uint32_t *ring = (uint32_t *)(mine + H * kRingBytes);
    Leaf *LA = (Leaf *)(mine + 2 * kRingBytes), *LB = LA + kLeaves;
    HRng r;
    hrng_open(r, ring, rings + (size_t)g * kRingWords, 624);
    for (int f = 0; f < F; ++f) {
        make_leaf((H ? LB : LA)[lane & 31u], leaves[((size_t)g * F + f) * kLeaves + (lane & 31u)], s_order);
        wave_mem_order();
        rollouts_pair(LA, LB, kLeaves, r, s_order);
        wave_mem_order();
        vals[((size_t)g * F + f) * kLeaves + (lane & 31u)] = (H ? LB : LA)[lane & 31u].val;
        wave_mem_order();
    }
    if ((lane & 31u) == 0) uses[g] = 624 + (int64_t)(r.wrel + (int32_t)r.off);
}
}  // namespace hw

// ------------------------------------------------------------------ host
static void mt_init(uint32_t *mt, uint32_t seed) {  // init_genrand
    mt[0] = seed;
    for (int i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
}

static bool four(uint64_t b) {
    uint64_t m = b & (b >> 7), r = m & (m >> 14);
    m = b & (b >> 1);
    r |= m & (m >> 2);
    m = b & (b >> 6);
    r |= m & (m >> 12);
    m = b & (b >> 8);
    r |= m & (m >> 16);
    return r != 0;
}

int main(int argc, char **argv) {
    const int G = argc > 1 ? atoi(argv[1]) : 4096;
    const int F = argc > 2 ? atoi(argv[2]) : 25;
    const int reps = argc > 3 ? atoi(argv[3]) : 5;
    using hw::LeafIn;
    std::vector<uint32_t> rings((size_t)G * zc::kRingWords, 0u);
    for (int g = 0; g < G; ++g) mt_init(&rings[(size_t)g * zc::kRingWords], 1000u + (uint32_t)g);
    std::vector<LeafIn> leaves((size_t)G * F * hw::kLeaves);
    std::mt19937 rng(7);
    for (auto &lf : leaves) {  // seeded random play: 0..30 plies, stopping at a win or a full board
        uint64_t s[2] = {0, 0};
        int t = 0;
        const int plies = (int)(rng() % 31u);
        for (int k = 0; k < plies; ++k) {
            const uint64_t occ = s[0] | s[1];
            int cols[7], nc = 0;
            for (int c = 0; c < 7; ++c)
                if (!((occ >> (7 * c + 5)) & 1ull)) cols[nc++] = c;
            if (!nc) break;
            const int c = cols[rng() % (uint32_t)nc];
            s[t] |= (occ + (1ull << (7 * c))) & (0x3Full << (7 * c));
            t ^= 1;
            if (four(s[t ^ 1])) break;
        }
        lf = LeafIn{s[0], s[1], (uint32_t)t, 0u};
    }
    uint32_t *d_rings;
    LeafIn *d_leaves;
    int32_t *d_vals[2];
    int64_t *d_uses[2];
    CK(hipMalloc(&d_rings, rings.size() * 4));
    CK(hipMalloc(&d_leaves, leaves.size() * sizeof(LeafIn)));
    CK(hipMemcpy(d_rings, rings.data(), rings.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_leaves, leaves.data(), leaves.size() * sizeof(LeafIn), hipMemcpyHostToDevice));
    for (int k = 0; k < 2; ++k) {
        CK(hipMalloc(&d_vals[k], leaves.size() * 4));
        CK(hipMalloc(&d_uses[k], (size_t)G * 8));
        CK(hipMemset(d_vals[k], 0x7F, leaves.size() * 4));
    }
    const size_t lds_full = zc::kTabBytes + hw::kGames * (hw::kRingBytes + hw::kLeafBytes);
    const size_t lds_half = zc::kTabBytes + hw::kGames * 2 * (hw::kRingBytes + hw::kLeafBytes);
    const int blocks_full = (G + hw::kGames - 1) / hw::kGames, blocks_half = (G / 2 + hw::kGames - 1) / hw::kGames;
    auto run = [&](int k) {
        if (k == 0)
            hipLaunchKernelGGL(hw::full_kernel, dim3(blocks_full), dim3(64 * hw::kGames), lds_full, 0, d_rings,
                               d_leaves, G, F, d_vals[0], d_uses[0]);
        else
            hipLaunchKernelGGL(hw::half_kernel, dim3(blocks_half), dim3(64 * hw::kGames), lds_half, 0, d_rings,
                               d_leaves, G, F, d_vals[1], d_uses[1]);
        CK(hipGetLastError());
    };
    run(0);
    run(1);
    CK(hipDeviceSynchronize());
    std::vector<int32_t> v0(leaves.size()), v1(leaves.size());
    std::vector<int64_t> u0(G), u1(G);
    CK(hipMemcpy(v0.data(), d_vals[0], v0.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(v1.data(), d_vals[1], v1.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(u0.data(), d_uses[0], G * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(u1.data(), d_uses[1], G * 8, hipMemcpyDeviceToHost));
    size_t bad_v = 0, bad_u = 0, first = (size_t)-1;
    long long wins = 0, draws = 0;
    for (size_t i = 0; i < v0.size(); ++i) {
        if (v0[i] != v1[i]) {
            ++bad_v;
            if (first == (size_t)-1) first = i;
        }
        wins += v0[i] != 0;
        draws += v0[i] == 0;
    }
    for (int g = 0; g < G; ++g) bad_u += u0[g] != u1[g];
    long long words = 0;
    for (int g = 0; g < G; ++g) words += u0[g] - 624;
    printf("games %d, flushes %d, leaves %zu: value mismatches %zu, stream-position mismatches %zu "
           "(decisive %lld, draws %lld, words consumed %lld)\n",
           G, F, v0.size(), bad_v, bad_u, wins, draws, words);
    if (bad_v) {
        const size_t g = first / ((size_t)F * hw::kLeaves);
        printf("first mismatch: leaf %zu (game %zu): full %d half %d; uses %lld vs %lld\n", first, g, v0[first],
               v1[first], (long long)u0[g], (long long)u1[g]);
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int rep = 0; rep < reps; ++rep) {
        float ms[2];
        for (int k = 0; k < 2; ++k) {
            CK(hipEventRecord(e0, 0));
            run(k);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms[k], e0, e1));
        }
        printf("rep %d: full wave %.3f ms, half wave %.3f ms (%.3fx)\n", rep, ms[0], ms[1], ms[0] / ms[1]);
    }
    return (bad_v || bad_u) ? 2 : 0;
}
