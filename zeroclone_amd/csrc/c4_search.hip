// c4_search.hip — batched Connect4 UCT search for gfx950 (MI355X).
//
// Replaces engine/mcts/src/mcts.cpp:102-160 (get_move) together with the callbacks it makes
// for c4_backend (engine/games/connect4/c4_backend.py), Policy('random')
// (engine/policy_functions.py:10-12) and Value('random_rollout')
// (engine/value_functions.py:35-45), for thousands of games per launch.
//
// Execution model: ONE GAME PER WAVE.  A game's search is a strictly serial chain (every
// random number comes from one CPython MT19937 stream, consumed in the reference's order),
// so the chip is filled with games, not with work from inside one game: 4096 games are
// 4096 waves, 16 per CU.  Inside a wave all control flow is wave-uniform, the game state
// (board, stream position, node counter) lives in SGPRs and runs on the scalar unit, and
// the 64 lanes take the parts that are parallel:
//   - selection: lane k scores child slot k (UCT in fp64, exactly mcts.cpp:41-45) and a
//     DPP reduction picks the first maximum;
//   - RNG: lane k holds word wbase+k of a 64-word window of the stream, so a
//     random.choice draw (with its rejection loop) is one ballot;
//   - rollouts: a block of plies is simulated at once, one ply per lane (c4_rollouts);
//   - backup: lane l updates tree level l of the leaf's path (all levels at once);
//   - stream refill: the MT recurrence is regenerated 192 words at a time.
// The whole move (every flush of `batch_size` leaves) runs in one launch; games never
// synchronise with each other.
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
constexpr int kTabBytes = 128 * 4 + 128 * 8;  // LDS tables: move-list order[128], select[128][8]

// Untried moves of a node (record +4 / Fresh.u): bit i (i < 7) set while move i of the
// node's move list is untried; bits 28..31 = number of moves.  The reference keeps the
// untried INDICES in list order and lets random.choice pick the r-th (mcts.cpp:67-72); the
// r-th remaining index is the r-th set bit of the mask (table sel[mask][r]).
__device__ __forceinline__ uint32_t untried_init(uint32_t n) { return ((1u << n) - 1u) | (n << 28); }
__device__ __forceinline__ uint32_t untried_count(uint32_t u) { return (uint32_t)__popc(u & 0x7Fu); }

// Fill the LDS tables (whole wave): s_order = d_order, s_sel[m*8 + r] = r-th set bit of m.
__device__ __forceinline__ void load_tables(uint32_t *s_order, uint8_t *s_sel) {
    for (int i = (int)threadIdx.x; i < 128; i += blockDim.x) s_order[i] = d_order[i];
    for (int i = (int)threadIdx.x; i < 1024; i += blockDim.x) {
        const uint32_t m = (uint32_t)i >> 3, r = (uint32_t)i & 7u;
        uint32_t x = m, c = 0, bitpos = 7;
        for (uint32_t b = 0; b < 7; ++b)
            if ((x >> b) & 1u) {
                if (c == r) { bitpos = b; break; }
                ++c;
            }
        s_sel[i] = (uint8_t)bitpos;
    }
}
constexpr int kWin = 64;                             // RNG window: one word per lane

// ------------------------------------------------------------------ wave helpers
__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint64_t uni64(uint64_t x) {
    return ((uint64_t)uni((uint32_t)(x >> 32)) << 32) | (uint64_t)uni((uint32_t)x);
}
__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

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
struct Rng {
    uint32_t *ring;
    uint32_t base;   // low 32 bits of the absolute position at the search's start (use0)
    int32_t wrel;    // window start - use0 (a multiple of 64 in absolute terms; may be < 0)
    uint32_t off;    // next word to consume = window start + off, off in [0, 64]
    int32_t grel;    // words generated so far - use0
    uint32_t wt;     // tempered x[window start + lane]
    uint32_t wn;     // raw x[window start + 64 + lane], in flight until the window advances
    __device__ __forceinline__ int32_t use() const { return wrel + (int32_t)off; }  // relative to use0
    __device__ __forceinline__ uint32_t slot(int32_t rel) const { return (base + (uint32_t)rel) & kRingMask; }
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
    rng_fill(r, r.wrel + 2 * kWin);
    r.wt = temper(r.ring[r.slot(r.wrel + (int32_t)lane_id())]);
    r.wn = r.ring[r.slot(r.wrel + kWin + (int32_t)lane_id())];
}

__device__ __forceinline__ void rng_advance(Rng &r) {
    r.wrel += kWin;
    r.off = 0;
    r.wt = temper(r.wn);
    if (r.grel < r.wrel + 2 * kWin) rng_fill(r, r.wrel + 2 * kWin);
    r.wn = r.ring[r.slot(r.wrel + kWin + (int32_t)lane_id())];
}

// rngpos after the search: {use0 + use(), use0 + grel}
__device__ __forceinline__ void rng_close(const Rng &r, uint64_t use0, uint64_t *rngpos) {
    rngpos[0] = use0 + (uint64_t)(int64_t)r.use();
    rngpos[1] = use0 + (uint64_t)(int64_t)r.grel;
}

// random._randbelow_with_getrandbits(n), 1 <= n <= 7: k = n.bit_length(); draw
// getrandbits(k) = word >> (32-k) until < n.  All window words are tested at once; the
// first accepted one (in stream order) is the draw, and everything before it is consumed.
__device__ __forceinline__ uint32_t rng_below(Rng &r, uint32_t n) {
    const uint32_t sh = (uint32_t)__clz(n);
    const uint32_t lane = lane_id();
    for (;;) {
        if (r.off >= (uint32_t)kWin) rng_advance(r);
        const uint32_t v = r.wt >> sh;
        const uint64_t bal = __ballot(lane >= r.off && v < n);
        if (bal) {
            const int f = __builtin_ctzll(bal);
            r.off = (uint32_t)f + 1;
            return (uint32_t)__builtin_amdgcn_readlane((int)v, f);
        }
        r.off = kWin;
    }
}

// Per-search counters, accumulated in lane 0 of VGPRs (off the scalar unit, no SGPRs).
struct Counters {
    int32_t expansions = 0, depth_sum = 0, plies = 0, blocks = 0;
    __device__ __forceinline__ void add(int32_t &c, int32_t v) { c += (lane_id() == 0) ? v : 0; }
};

// ------------------------------------------------------------------ random rollouts
// A pending leaf, kept in LDS between the phases of a flush.
struct Leaf {
    uint64_t p0, p1;  // stones of 'X' / 'O'
    uint32_t meta;    // node | depth << 16 | turn << 24 | legal mask << 25
    int32_t val;      // rollout value from the leaf's side to move
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

__device__ __forceinline__ uint64_t readlane64(uint64_t x, int l) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(x >> 32), l) << 32) |
           (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)x, l);
}

__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {  // set bits of m in lanes below this one
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Inclusive prefix SUM over the 64 lanes (same DPP pattern as scan_or32).
__device__ __forceinline__ uint32_t scan_add32(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);
    return x;
}

// Inclusive prefix OR over the 64 lanes (DPP: row_shr 1,2,4,8, then row_bcast 15 / 31).
__device__ __forceinline__ uint32_t scan_or32(uint32_t x) {
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);
    return x;
}
__device__ __forceinline__ uint64_t scan_or(uint64_t x) {
    return ((uint64_t)scan_or32((uint32_t)(x >> 32)) << 32) | (uint64_t)scan_or32((uint32_t)x);
}

// Value.random_rollout (value_functions.py:35-45) for the nb pending leaves of one flush, in
// pending order (value.batch: mcts.cpp:118).  Per leaf, from the side to move `turn`:
//   while not check_win(s) and not check_draw(s): s = play(s, choice(list(legal(s))))
//   win -> -1 if the side to move at the end (the loser) is the leaf's side to move, else +1
// check_win looks at the LAST mover only (c4_backend.py:27, tokens[1 - turn]).
//
// Plies are simulated a BLOCK at a time.  While the legal set is unchanged (no column has
// filled), the draws are exactly the window words w with (w >> (32-k)) < n, in stream
// order — so one ballot yields the moves of every ply the window covers.  Lane k (an
// accepted word) is ply q_k = #accepted lanes below it; its stone's row is the column
// height plus #earlier accepted lanes in the same column; prefix-OR scans over the lanes
// build each player's stones after every ply, and every lane tests check_win / full board
// / column filled for ITS ply.  The first lane with an event ends the block (a fill changes
// the legal set, so the next block restarts from the following word).
__device__ void c4_rollouts(Leaf *L, int nb, Rng &rng, const uint32_t *s_order, Counters &cn) {
    const uint32_t lane = lane_id();
    for (int j = 0; j < nb; ++j) {
        const uint64_t x0 = uni64(L[j].p0);
        const uint64_t x1 = uni64(L[j].p1);
        const uint32_t lm = uni(L[j].meta);
        const int tn = (int)((lm >> 24) & 1u);
        uint64_t me = tn ? x1 : x0;  // side to move
        uint64_t op = tn ? x0 : x1;  // last mover
        int val = 0;
        int q = 0;  // plies played in this rollout
        if (has_four(op)) {
            val = -1;
        } else if ((me | op) != kFull) {
            int mask = (int)(lm >> 25);
            uint32_t ow = uni(s_order[mask]);
            uint32_t n = (ow >> 24) & 15u;
            int stones = __popcll(me | op);
            for (;;) {
                if (rng.off >= (uint32_t)kWin) rng_advance(rng);
                const uint32_t v = rng.wt >> __clz(n);
                const bool acc = lane >= rng.off && v < n;
                const uint64_t A = __ballot(acc);
                if (!A) {
                    rng.off = kWin;
                    continue;
                }
                cn.add(cn.blocks, 1);
                const uint32_t qk = mbcnt(A);                    // this lane's ply in the block
                const uint32_t col = (ow >> (3 * (v & 7u))) & 7u;  // its column (if accepted)
                // earlier plies in the same column: 4-bit per-column counters, prefix-summed
                // (a nibble can only overflow past 15 plies in one column, i.e. after that
                // column filled — beyond the block's first event, so never read)
                const uint32_t one = acc ? (1u << (4 * col)) : 0u;
                const uint32_t same = ((scan_add32(one) - one) >> (4 * col)) & 15u;
                const uint64_t occ = me | op;
                const uint32_t h0 = (uint32_t)__popcll((occ >> (7 * col)) & 0x3Full);
                const uint32_t row = min(h0 + same, 6u);
                const uint64_t bit = acc ? (1ull << (7 * col + row)) : 0ull;
                const bool even = (qk & 1u) == 0;
                const uint64_t E = scan_or(even ? bit : 0ull);  // stones of the block's first mover
                const uint64_t O = scan_or(even ? 0ull : bit);  // stones of the other side
                const bool win = has_four(even ? (me | E) : (op | O));
                const bool full = stones + (int)qk + 1 == 42;
                const uint64_t W = __ballot(acc && win);
                const uint64_t EV = W | __ballot(acc && (full || row == 5));
                const int kend = EV ? __builtin_ctzll(EV) : 63 - __builtin_clzll(A);
                const int np = __builtin_amdgcn_readlane((int)qk, kend) + 1;  // plies in this block
                const uint64_t a2 = me | readlane64(E, kend);
                const uint64_t b2 = op | readlane64(O, kend);
                if (np & 1) {
                    me = b2;
                    op = a2;
                } else {
                    me = a2;
                    op = b2;
                }
                q += np;
                stones += np;
                rng.off = EV ? (uint32_t)kend + 1 : (uint32_t)kWin;
                if (!EV) continue;
                if ((W >> kend) & 1ull) {  // the ply's mover completed four
                    val = (q & 1) ? 1 : -1;
                    break;
                }
                if (stones >= 42) {  // check_draw: board full
                    val = 0;
                    break;
                }
                // a column filled: the legal set (and its CPython order) changes
                mask &= ~(1 << __builtin_amdgcn_readlane((int)col, kend));
                ow = uni(s_order[mask]);
                n = (ow >> 24) & 15u;
            }
        }
        if (lane == 0) L[j].val = val;
        cn.add(cn.plies, q);
    }
}

// ------------------------------------------------------------------ node records
struct Tree {
    uint8_t *nodes;  // this game's records
    int32_t *W;      // this game's W rows
    __device__ __forceinline__ uint8_t *rec(int nd) const { return nodes + (size_t)nd * kRecBytes; }
    __device__ __forceinline__ uint32_t *hdr(int nd) const { return (uint32_t *)rec(nd); }
    __device__ __forceinline__ uint16_t *child(int nd) const { return (uint16_t *)(rec(nd) + 16); }
    __device__ __forceinline__ int32_t *na(int nd) const { return (int32_t *)(rec(nd) + 32); }
    __device__ __forceinline__ double *q(int nd) const { return (double *)(rec(nd) + 64); }
    __device__ __forceinline__ int32_t *w(int nd) const { return W + (size_t)nd * kSlots; }
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
        t.q(nd)[lane] = 0.0;
        t.w(nd)[lane] = 0;
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

// ------------------------------------------------------------------ the search kernel
// STAMP = diagnostic build: lane 0 adds s_memtime deltas per phase into p.a.phase[g][0..7] =
// {rng generation at flush start, first walk of a flush, resumed walks, expansion + leaf
//  bookkeeping, rollouts, backup, -, -}.
template <bool STAMP>
__global__ __launch_bounds__(kBlock) void c4_search_kernel(SearchParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t s_dyn[];
    // LDS: tables (order[128] u32, sel[128][8] u8), fresh[bs] (48 B), leaves[bs] (24 B),
    //      paths[bs][kMaxDepth] (u16 node ids)
    uint32_t *const s_order = (uint32_t *)s_dyn;
    uint8_t *const s_sel = s_dyn + 512;
    Fresh *const fresh = (Fresh *)(s_dyn + kTabBytes);
    Leaf *const leaves = (Leaf *)(s_dyn + kTabBytes + sizeof(Fresh) * (size_t)p.bs);
    uint16_t *const paths = (uint16_t *)(s_dyn + kTabBytes + (sizeof(Fresh) + sizeof(Leaf)) * (size_t)p.bs);
    load_tables(s_order, s_sel);
    __syncthreads();
    // log(N) table read through the constant address space: uniform index -> scalar loads,
    // which do not sit in the vector-memory counter the walk and the RNG window wait on.
    const __attribute__((address_space(4))) double *logtab =
        (const __attribute__((address_space(4))) double *)p.a.logtab;

    const uint32_t lane = lane_id();
    const uint32_t k = lane & 7u;  // child slot handled by this lane (lanes 8.. mirror 0..7)
    const int gl = blockIdx.x;     // game within this call (one wave per game)
    if (gl >= p.n_games) return;
    const int g = p.game_ids ? uni(p.game_ids[gl]) : p.first_game + gl;

    {
        const zc_c4_state root = p.roots[gl];
        const uint64_t rp0 = uni64(root.stones[0]), rp1 = uni64(root.stones[1]);
        const int rturn = uni(root.turn);
        if (!valid_state(rp0, rp1, rturn) || legal_mask(rp0 | rp1) == 0) {
            if (lane == 0) {
                zc_game_stats st{};
                st.status = valid_state(rp0, rp1, rturn) ? ZC_STATUS_NO_MOVES : ZC_STATUS_BAD_STATE;
                p.out_stats[gl] = st;
                p.out_move[gl] = -1;
            }
            if (lane < 7) p.out_na[(size_t)gl * 7 + lane] = 0;
            return;
        }
    }

    const Arena &a = p.a;
    const Tree t{a.nodes + (size_t)g * p.M * kRecBytes, a.W + (size_t)g * p.M * kSlots};

    Rng rng;
    rng_open(rng, a.ring + (size_t)g * kRingWords, uni64(a.rngpos[2 * (size_t)g]), uni64(a.rngpos[2 * (size_t)g + 1]));
    Counters cn;
    int status = 0;

    {
        const zc_c4_state root = p.roots[gl];
        node_init(t, 0, 0xFFFF, 0xFF, 0, uni(s_order[legal_mask(uni64(root.stones[0]) | uni64(root.stones[1]))]));
    }
    int nnodes = 1;
    wave_mem_order();

    uint64_t ph[kPhases] = {};
    uint64_t tstamp = STAMP ? __builtin_amdgcn_s_memtime() : 0;
#define ZC_STAMP(k_)                                         \
    if (STAMP) {                                             \
        const uint64_t now_ = __builtin_amdgcn_s_memtime();  \
        ph[k_] += now_ - tstamp;                             \
        tstamp = now_;                                       \
    }
    for (int done = 0; done < p.sims;) {
        const int nb = min(p.bs, p.sims - done);
        rng_fill(rng, rng.use() + kLookahead);
        ZC_STAMP(0)

        // ---- selection + expansion of nb leaves (mcts.cpp:129-147) -------------------------
        // No backup happens inside a flush, so (1) the UCT path from the root to the node X0
        // where the flush's first walk stops is shared by every leaf of the flush (each walk
        // resumes where the previous one expanded, always at or below X0), and (2) every node
        // below X0 is created in this flush ("fresh": id >= f0, Na = Q = 0 on every edge).
        // The reference's walk from a node without untried moves takes the first child with
        // the largest UCT; an unvisited child scores +inf, so below X0 that is simply the
        // lowest slot holding a fresh child — no arithmetic, no HBM.  Fresh nodes live in
        // LDS until the flush is published.  Lane l holds level l of the current path.
        const int f0 = nnodes;
        for (int i = (int)lane; i < nb; i += 64) {  // fresh slots: no children, zero in-edge counters
            fresh[i].na = 0;
            fresh[i].w = 0;
            *(uint4 *)fresh[i].ch = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
        }
        // the root position, re-read every flush rather than held in registers
        const zc_c4_state root = p.roots[gl];
        int node = 0, depth = 0, turn = uni(root.turn), nN = done;  // nN = N(node) = Na of its in-edge
        uint64_t b0 = uni64(root.stones[0]), b1 = uni64(root.stones[1]);
        uint32_t pathv = (lane == 0) ? 0x00FF0000u : 0u;
        uint32_t u, ow, ch;  // the current node's record (ch: slot k)
        for (;;) {  // the first walk: select (mcts.cpp:47-63) over HBM records
            const uint8_t *R = t.rec(node);
            const uint4 h = *(const uint4 *)R;
            ch = ((const uint16_t *)(R + 16))[k];
            const int32_t na = ((const int32_t *)(R + 32))[k];
            const double q = ((const double *)(R + 64))[k];
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
            const uint64_t unvisited = __ballot(valid && na == 0) & 0xFFull;
            if (unvisited) {  // +inf beats everything; first such slot
                best = __builtin_ctzll(unvisited);
            } else {
                // UCT (mcts.cpp:41-45) = fma(c, sqrt(log(N)/Na), Qa), first max in slot order
                double v = valid ? fma(p.c, sqrt(lg / (double)na), q) : -INFINITY;
                int bi = (int)k;
                argmax8(v, bi);
                if ((__ballot(v == -INFINITY) & 1ull) != 0) break;  // no child: terminal leaf
                best = uni(bi);
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
        int cmask = legal_mask(b0 | b1);      // legal columns of the current node
        const int x0node = node, d0 = depth;  // X0: shared by every leaf of this flush
        const uint32_t ppath = pathv;         // root .. X0 (lanes 0..d0)
        bool x0_dirty = false;
        uint32_t x_u = u, x_ch = ch;          // X0's record as last seen (written back if dirty)
        ZC_STAMP(1)

        for (int j = 0; j < nb; ++j) {
            // resume at `node` (fully described by u, ow, ch, cmask in registers)
            for (;;) {
                if (untried_count(u)) break;  // untried moves: expand here
                const uint64_t fm = __ballot(k < (u >> 28) && ch != 0xFFFF && (int)ch >= f0) & 0xFFull;
                if (!fm) break;               // no child at all: terminal, re-queued as its own leaf
                const int s = __builtin_ctzll(fm);
                const int child = __builtin_amdgcn_readlane((int)ch, s);
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
                const uint4 fh = *(const uint4 *)&fresh[child - f0];  // u, ow, link, lmask
                u = uni(fh.x);
                ow = uni(fh.y);
                cmask = uni((int)fh.w);
                ch = fresh[child - f0].ch[k];
            }
            ZC_STAMP(2)
            int leaf = node, ldepth = depth, lturn = turn, lmask = cmask;
            uint64_t l0 = b0, l1 = b1;
            const uint32_t cnt = untried_count(u);
            if (cnt) {  // expand (mcts.cpp:65-78): policy = random.choice(untried)
                const uint32_t r = rng_below(rng, cnt);
                const int mi = (int)uni((uint32_t)s_sel[(u & 0x7Fu) * 8u + r]);
                u &= ~(1u << mi);
                const int col = (int)((ow >> (3 * mi)) & 7u);
                const uint64_t bit = drop_bit(b0 | b1, col);
                if (turn) l1 |= bit; else l0 |= bit;
                lturn = turn ^ 1;
                leaf = nnodes++;
                ldepth = depth + 1;
                if (bit & kTop) lmask &= ~(1 << col);  // the column just filled
                const uint32_t low_ = uni(s_order[lmask]);
                if (k == (uint32_t)mi) ch = (uint32_t)leaf;
                if (node < f0) x0_dirty = true;  // X0 itself: written back when the flush is published
                if (lane == 0) {
                    // Node(state, legal_moves) (mcts.cpp:23-34): all moves untried, no children
                    *(uint4 *)&fresh[leaf - f0] =
                        make_uint4(untried_init((low_ >> 24) & 15u), low_,
                                   (uint32_t)node | ((uint32_t)mi << 16) | ((uint32_t)ldepth << 24), (uint32_t)lmask);
                    if (node >= f0) fresh[node - f0].u = u;  // the parent's copy in LDS
                }
                if (node >= f0 && lane == (uint32_t)mi) fresh[node - f0].ch[mi] = (uint16_t)leaf;
                cn.add(cn.expansions, 1);
                cn.add(cn.depth_sum, ldepth);
            }
            // the leaf's path: the walk's path plus the new node (the next walk resumes at `node`)
            const uint32_t lpath = (cnt && lane == (uint32_t)ldepth) ? (uint32_t)leaf : pathv;
            if (lane == 0) {
                leaves[j].p0 = l0;
                leaves[j].p1 = l1;
                leaves[j].meta = (uint32_t)leaf | ((uint32_t)ldepth << 16) | ((uint32_t)lturn << 24) |
                                 ((uint32_t)lmask << 25);
            }
            if (lane < (uint32_t)kMaxDepth) paths[j * kMaxDepth + lane] = (uint16_t)lpath;
            wave_mem_order();
            ZC_STAMP(3)
        }
        if (node == x0node) {
            x_u = u;
            x_ch = ch;
        }

        // ---- value.batch: random rollouts in pending order (mcts.cpp:112-124) ---------------
        c4_rollouts(leaves, nb, rng, s_order, cn);
        wave_mem_order();
        ZC_STAMP(4)

        // ---- backprop of the whole flush (mcts.cpp:80-100, :124-125) ------------------------
        // Leaf j adds Na += 1 and Wa -= v_j * (-1)^(d_j - l) on the edge into level l of its
        // path, l = 1..d_j.  Integer adds commute, so the flush is applied as a sum:
        //   levels 1..d0 (root -> X0, on every path): Na += nb, Wa -= (-1)^l * S with
        //     S = sum_j v_j (-1)^d_j — one read-modify-write per level, all levels at once;
        //   levels > d0 (fresh nodes): LDS atomics into the fresh node's in-edge counters,
        //     written to HBM with the fresh records below.
        // Node::N is not stored: it equals Na of the in-edge (root: leaves flushed so far).
        int S = 0;
        for (int base = 0; base < nb; base += 64) {
            const int jj = base + (int)lane;
            int sv = 0;
            if (jj < nb) {
                const int v = leaves[jj].val;
                sv = ((leaves[jj].meta >> 16) & 1u) ? -v : v;
            }
            S += __popcll(__ballot(sv > 0)) - __popcll(__ballot(sv < 0));
        }
        for (int j = 0; j < nb; ++j) {
            const uint32_t meta = uni(leaves[j].meta);
            const int d = (int)((meta >> 16) & 0xFFu);
            const int v = uni(leaves[j].val);
            if (lane > (uint32_t)d0 && lane <= (uint32_t)d) {
                const int fi = (int)paths[j * kMaxDepth + lane] - f0;
                const int vl = ((d - (int)lane) & 1) ? -v : v;
                atomicAdd(&fresh[fi].na, 1);
                atomicAdd(&fresh[fi].w, -vl);
            }
        }
        if (lane >= 1 && lane <= (uint32_t)d0) {
            const int par = __shfl((int)(ppath & 0xFFFFu), (int)lane - 1);
            const int act = (int)(ppath >> 16);
            const int dw = (lane & 1u) ? S : -S;  // Wa -= (-1)^l * S
            const int32_t na1 = t.na(par)[act] + nb;
            const int32_t w1 = t.w(par)[act] + dw;
            t.na(par)[act] = na1;
            t.w(par)[act] = w1;
            t.q(par)[act] = (double)w1 / (double)na1;  // Qa = Wa / Na
        }
        wave_mem_order();
        ZC_STAMP(5)

        // ---- publish: X0's changes and every fresh node, in coalesced stores ------------------
        if (x0_dirty) {
            if (lane == 0) t.hdr(x0node)[1] = x_u;
            if (lane < kSlots) {
                t.child(x0node)[lane] = (uint16_t)x_ch;
                if (x_ch != 0xFFFF && (int)x_ch >= f0) {  // edge into a fresh child
                    const int32_t na = fresh[x_ch - f0].na, w = fresh[x_ch - f0].w;
                    t.na(x0node)[lane] = na;
                    t.w(x0node)[lane] = w;
                    t.q(x0node)[lane] = (double)w / (double)na;
                }
            }
        }
        {
            const int nf = nnodes - f0;
            for (int base = 0; base < nf * 8; base += 64) {
                const int idx = base + (int)lane;
                if (idx < nf * 8) {
                    const int r = idx >> 3, slot = idx & 7;
                    const Fresh &F = fresh[r];
                    const uint16_t c = F.ch[slot];
                    int32_t na = 0, w = 0;
                    if (c != 0xFFFF) {
                        na = fresh[c - f0].na;
                        w = fresh[c - f0].w;
                    }
                    uint8_t *R = t.rec(f0 + r);
                    if (slot == 0) *(uint4 *)R = make_uint4(0u, F.u, F.link, F.ow);
                    ((uint16_t *)(R + 16))[slot] = c;
                    ((int32_t *)(R + 32))[slot] = na;
                    ((double *)(R + 64))[slot] = na ? (double)w / (double)na : 0.0;
                    t.w(f0 + r)[slot] = w;
                }
            }
        }
        wave_mem_order();
        ZC_STAMP(6)
        done += nb;
    }
#undef ZC_STAMP
    if (STAMP && lane == 0)
        for (int k_ = 0; k_ < kPhases; ++k_) a.phase[kPhases * (size_t)g + k_] += (int64_t)ph[k_];

    // ---- best move: first max of child N over the root's move list (mcts.cpp:150-157) ----
    const uint32_t u = uni(t.hdr(0)[1]);
    const uint32_t ow = uni(t.hdr(0)[3]);
    const uint32_t nm = u >> 28;
    int bv = (k < nm) ? t.na(0)[k] : -1;
    int bi = (int)k;
    argmax8(bv, bi);
    const int best = uni(bi);
    if (lane < 7) {  // visits per column
        int pos = -1;
        for (uint32_t s = 0; s < nm; ++s)
            if (((ow >> (3 * s)) & 7u) == lane) pos = (int)s;
        p.out_na[(size_t)gl * 7 + lane] = pos >= 0 ? t.na(0)[pos] : 0;
    }
    if (lane == 0) {
        p.out_move[gl] = (int)((ow >> (3 * best)) & 7u);
        zc_game_stats st{};
        st.status = status;
        st.expansions = cn.expansions;
        st.depth_sum = cn.depth_sum;
        st.leaves = p.sims;
        st.rollout_plies = cn.plies;
        st.rollout_blocks = cn.blocks;
        st.rng_words = rng.use();
        p.out_stats[gl] = st;
        rng_close(rng, a.rngpos[2 * (size_t)g], a.rngpos + 2 * (size_t)g);
    }
}

// ------------------------------------------------------------------ small kernels
__global__ __launch_bounds__(kBlock) void c4_rollout_debug_kernel(Arena a, int first_game, int n,
                                                                  const zc_c4_state *states, int32_t *out_value,
                                                                  int64_t *out_words) {
    __shared__ Leaf s_leaf[1];
    __shared__ uint32_t s_order[128];
    __shared__ uint8_t s_sel[1024];
    load_tables(s_order, s_sel);
    __syncthreads();
    const uint32_t lane = lane_id();
    const int gl = blockIdx.x;
    if (gl >= n) return;
    const int g = first_game + gl;
    Rng rng;
    const uint64_t use0 = uni64(a.rngpos[2 * (size_t)g]);
    rng_open(rng, a.ring + (size_t)g * kRingWords, use0, uni64(a.rngpos[2 * (size_t)g + 1]));
    const zc_c4_state s = states[gl];
    if (lane == 0) {
        s_leaf[0].p0 = s.stones[0];
        s_leaf[0].p1 = s.stones[1];
        s_leaf[0].meta = ((uint32_t)s.turn << 24) | ((uint32_t)legal_mask(s.stones[0] | s.stones[1]) << 25);
    }
    wave_mem_order();
    Counters cn;
    c4_rollouts(s_leaf, 1, rng, s_order, cn);
    wave_mem_order();
    if (lane == 0) {
        out_value[gl] = s_leaf[0].val;
        out_words[gl] = rng.use();
        rng_close(rng, use0, a.rngpos + 2 * (size_t)g);
    }
}

// Value('random_rollout').batch: n states rolled out IN ORDER on one game's stream.
__global__ __launch_bounds__(kBlock) void c4_rollout_seq_kernel(Arena a, int g, int n, const zc_c4_state *states,
                                                                int32_t *out_value, int64_t *out_words) {
    __shared__ Leaf s_leaf[kBlock];
    __shared__ uint32_t s_order[128];
    __shared__ uint8_t s_sel[1024];
    load_tables(s_order, s_sel);
    __syncthreads();
    const uint32_t lane = lane_id();
    Rng rng;
    const uint64_t use0 = uni64(a.rngpos[2 * (size_t)g]);
    rng_open(rng, a.ring + (size_t)g * kRingWords, use0, uni64(a.rngpos[2 * (size_t)g + 1]));
    Counters cn;
    for (int base = 0; base < n; base += kBlock) {
        const int cnt = min(kBlock, n - base);
        if ((int)lane < cnt) {
            const zc_c4_state s = states[base + lane];
            s_leaf[lane].p0 = s.stones[0];
            s_leaf[lane].p1 = s.stones[1];
            s_leaf[lane].meta = ((uint32_t)s.turn << 24) | ((uint32_t)legal_mask(s.stones[0] | s.stones[1]) << 25);
        }
        wave_mem_order();
        rng_fill(rng, rng.use() + kLookahead);
        c4_rollouts(s_leaf, cnt, rng, s_order, cn);
        wave_mem_order();
        if ((int)lane < cnt) out_value[base + lane] = s_leaf[lane].val;
        wave_mem_order();
    }
    if (lane == 0) {
        out_words[0] = rng.use();
        rng_close(rng, use0, a.rngpos + 2 * (size_t)g);
    }
}

__global__ void c4_play_kernel(int n, zc_c4_state *states, const int32_t *moves, int32_t *results, int reset) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int col = moves[i];
    if (col < 0 || col > 6) {
        results[i] = ZC_C4_ONGOING;
        return;
    }
    zc_c4_state s = states[i];
    const int turn = s.turn & 1;
    s.stones[turn] |= drop_bit(s.stones[0] | s.stones[1], col);
    s.turn = turn ^ 1;
    int r = ZC_C4_ONGOING;
    if (has_four(s.stones[turn])) r = s.turn * 2 - 1;  // Engine._evaluate: check_win -> turn*2-1
    else if ((s.stones[0] | s.stones[1]) == kFull) r = 0;
    if (reset && r != ZC_C4_ONGOING) s = zc_c4_state{{0, 0}, 0, 0};
    states[i] = s;
    results[i] = r;
}

__global__ void uct_debug_kernel(int n, const double *logn, const int32_t *na, const double *q, double c,
                                 double *out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = na[i] == 0 ? INFINITY : fma(c, sqrt(logn[i] / (double)na[i]), q[i]);
}

}  // namespace

size_t c4_search_lds_bytes(int bs) {
    return kTabBytes + (sizeof(Leaf) + sizeof(Fresh) + sizeof(uint16_t) * kMaxDepth) * (size_t)bs;
}

void launch_c4_search(const SearchParams &p, hipStream_t s) {
    const size_t lds = c4_search_lds_bytes(p.bs);
    if (p.stamp)
        hipLaunchKernelGGL(c4_search_kernel<true>, dim3(p.n_games), dim3(kBlock), lds, s, p);
    else
        hipLaunchKernelGGL(c4_search_kernel<false>, dim3(p.n_games), dim3(kBlock), lds, s, p);
}

void launch_c4_rollout_debug(const Arena &a, int M, int first_game, int n, const zc_c4_state *states,
                             int32_t *out_value, int64_t *out_words, hipStream_t s) {
    (void)M;
    hipLaunchKernelGGL(c4_rollout_debug_kernel, dim3(n), dim3(kBlock), 0, s, a, first_game, n, states, out_value,
                       out_words);
}

void launch_c4_rollout_seq(const Arena &a, int game, int n, const zc_c4_state *states, int32_t *out_value,
                           int64_t *out_words, hipStream_t s) {
    hipLaunchKernelGGL(c4_rollout_seq_kernel, dim3(1), dim3(kBlock), 0, s, a, game, n, states, out_value, out_words);
}

void launch_c4_play(int n, zc_c4_state *states, const int32_t *moves, int32_t *results, int reset, hipStream_t s) {
    hipLaunchKernelGGL(c4_play_kernel, dim3((n + 255) / 256), dim3(256), 0, s, n, states, moves, results, reset);
}

void launch_uct_debug(int n, const double *logn, const int32_t *na, const double *q, double c, double *out,
                      hipStream_t s) {
    hipLaunchKernelGGL(uct_debug_kernel, dim3((n + 255) / 256), dim3(256), 0, s, n, logn, na, q, c, out);
}

}  // namespace zc
