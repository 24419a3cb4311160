// c4_search.hip — batched Connect4 UCT search for gfx950 (MI355X).
//
// Replaces engine/mcts/src/mcts.cpp:102-160 (get_move) together with the callbacks it makes
// for c4_backend (engine/games/connect4/c4_backend.py), Policy('random')
// (engine/policy_functions.py:10-12) and Value('random_rollout')
// (engine/value_functions.py:35-45), for thousands of games per launch.
//
// Execution model.  A game is owned by a group of 8 lanes (8 games per wave64, one wave per
// workgroup); the whole search of a move — every flush of `batch_size` leaves — runs inside
// one launch, so games never synchronise with each other.  Inside a group all lanes follow
// the same control flow; the lanes split the per-node work (lane k owns child slot k, tree
// level l is backed up by lane l % 8, the RNG window holds word wbase+k in lane k) and agree
// through ballots / shuffles.  Every random number is drawn from the game's own CPython
// MT19937 stream in the reference's order, so results are bit-identical to the reference.
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
constexpr uint32_t kIdentDigits = 0 | (1u << 3) | (2u << 6) | (3u << 9) | (4u << 12) | (5u << 15) | (6u << 18);

// ------------------------------------------------------------------ Connect4 bitboards
__device__ __forceinline__ uint64_t drop_bit(uint64_t occ, int col) {
    // c4_backend.play_move (:14-23): lowest empty row of `col`; a full column drops nothing.
    const int s = 7 * col;
    return (occ + (1ull << s)) & (0x3Full << s);
}

__device__ __forceinline__ int legal_mask(uint64_t occ) {
    // c4_backend.get_legal_moves (:49-50): column c is legal while its top cell is empty.
    const uint64_t t = (~occ & kTop) >> 5;  // bit 7c
    int m = 0;
#pragma unroll
    for (int c = 0; c < 7; ++c) m |= (int)((t >> (6 * c)) & (1ull << c));
    return m;
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

// ------------------------------------------------------------------ group primitives
__device__ __forceinline__ unsigned group_ballot(bool p, int gbase) {
    return (unsigned)((__ballot(p) >> gbase) & 0xFFull);
}

// First maximum over the group (ties -> lower slot), as mcts.cpp:55-58 (`v > best_val`).
__device__ __forceinline__ void group_argmax(double &v, int &i) {
#pragma unroll
    for (int off = 1; off < kGroup; off <<= 1) {
        const double ov = __shfl_xor(v, off);
        const int oi = __shfl_xor(i, off);
        if (ov > v || (ov == v && oi < i)) {
            v = ov;
            i = oi;
        }
    }
}

__device__ __forceinline__ void group_argmax_int(int &v, int &i) {
#pragma unroll
    for (int off = 1; off < kGroup; off <<= 1) {
        const int ov = __shfl_xor(v, off);
        const int oi = __shfl_xor(i, off);
        if (ov > v || (ov == v && oi < i)) {
            v = ov;
            i = oi;
        }
    }
}

__device__ __forceinline__ void wave_mem_order() {
    // Same-wave hand-offs through memory (one lane stores, another loads) are ordered by
    // program order on gfx950 (wavefront scope needs no cache action); this only stops the
    // compiler from moving memory operations across the point.
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
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
// it 224 words at a time, all lanes in parallel (every input is >= 227 words older).
struct Rng {
    uint32_t *ring;
    uint64_t use;    // next word to consume
    uint64_t gen;    // words generated so far
    uint64_t wbase;  // window start (multiple of 8); use in [wbase, wbase + 8]
    uint32_t wt;     // tempered x[wbase + sub]
    uint32_t wn;     // tempered x[wbase + 8 + sub]
};

__device__ __noinline__ uint64_t rng_generate(uint32_t *ring, uint64_t gen, uint64_t target, int sub) {
    while (gen < target) {
#pragma unroll 4
        for (int i = sub; i < kChunk; i += kGroup) {
            const uint64_t p = gen + (uint64_t)i;
            const uint32_t a = ring[(p - 624) & kRingMask];
            const uint32_t b = ring[(p - 623) & kRingMask];
            const uint32_t m = ring[(p - 227) & kRingMask];
            const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
            ring[p & kRingMask] = m ^ (y >> 1) ^ ((b & 1u) ? 0x9908b0dfu : 0u);
        }
        gen += kChunk;
        wave_mem_order();
    }
    return gen;
}

__device__ __forceinline__ void rng_fill(Rng &r, uint64_t target, int sub) {
    if (r.gen < target) r.gen = rng_generate(r.ring, r.gen, target, sub);
}

__device__ __forceinline__ void rng_open(Rng &r, uint32_t *ring, uint64_t use, uint64_t gen, int sub) {
    r.ring = ring;
    r.use = use;
    r.gen = gen;
    r.wbase = use & ~7ull;
    rng_fill(r, r.wbase + 16, sub);
    r.wt = temper(r.ring[(r.wbase + sub) & kRingMask]);
    r.wn = temper(r.ring[(r.wbase + 8 + sub) & kRingMask]);
}

// random._randbelow_with_getrandbits(n), 1 <= n <= 7: k = n.bit_length(); draw
// getrandbits(k) = word >> (32-k) until < n.  The 8 window words are tested at once; the
// first accepted one (in stream order) is the draw, and everything before it is consumed.
__device__ __forceinline__ uint32_t rng_below(Rng &r, uint32_t n, int sub, int gbase) {
    const int sh = __clz(n);
    for (;;) {
        if (r.use >= r.wbase + 8) {
            r.wbase += 8;
            r.wt = r.wn;
            if (r.gen < r.wbase + 16) rng_fill(r, r.wbase + 16, sub);
            r.wn = temper(r.ring[(r.wbase + 8 + sub) & kRingMask]);
        }
        const uint32_t v = r.wt >> sh;
        const unsigned off = (unsigned)(r.use - r.wbase);
        const unsigned bal = group_ballot(((unsigned)sub >= off) && (v < n), gbase);
        if (bal) {
            const int f = __ffs(bal) - 1;
            r.use = r.wbase + (uint64_t)f + 1;
            return (uint32_t)__shfl((int)v, gbase + f);
        }
        r.use = r.wbase + 8;
    }
}

// ------------------------------------------------------------------ random rollout
// Value.random_rollout (value_functions.py:35-45) from the side to move `turn`:
//   while not check_win(s) and not check_draw(s): s = play(s, choice(list(legal(s))))
//   win -> -1 if the side to move at the end (the loser) is the leaf's side to move, else +1
// check_win looks at the LAST mover only (c4_backend.py:27, tokens[1 - turn]).
__device__ int c4_rollout(uint64_t p0, uint64_t p1, int turn, Rng &rng, const uint32_t *s_order, int sub,
                          int gbase, int64_t &plies) {
    uint64_t me = turn ? p1 : p0;   // side to move
    uint64_t op = turn ? p0 : p1;   // last mover
    uint64_t occ = me | op;
    int mask = legal_mask(occ);
    uint32_t ow = s_order[mask];
    int parity = 0;
    for (;;) {
        if (has_four(op)) return parity ? 1 : -1;
        if (occ == kFull) return 0;
        const uint32_t r = rng_below(rng, (ow >> 24) & 15u, sub, gbase);
        const int col = (int)((ow >> (3 * r)) & 7u);
        const uint64_t bit = drop_bit(occ, col);
        if (!bit) return 0;  // unreachable for valid states; guarantees termination
        const uint64_t moved = me | bit;
        me = op;
        op = moved;
        occ |= bit;
        parity ^= 1;
        ++plies;
        if (bit & kTop) {  // column just filled: the legal set (and its order) changes
            mask &= ~(1 << col);
            ow = s_order[mask];
        }
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
__device__ __forceinline__ void node_init(const Tree &t, int nd, int parent, int pact, int depth, uint32_t ow,
                                          int sub) {
    const uint32_t n = (ow >> 24) & 15u;
    if (sub == 0) {
        uint4 h;
        h.x = 0;                                                         // N
        h.y = (kIdentDigits & ((1u << (3 * n)) - 1u)) | (n << 24) | (n << 28);  // untried, #moves
        h.z = (uint32_t)(parent & 0xFFFF) | ((uint32_t)(pact & 0xFF) << 16) | ((uint32_t)depth << 24);
        h.w = ow;
        *(uint4 *)t.rec(nd) = h;
    }
    t.child(nd)[sub] = 0xFFFF;
    t.na(nd)[sub] = 0;
    t.q(nd)[sub] = (sub == 7) ? -INFINITY : 0.0;  // slot 7 = log(N) = log(0)
    t.w(nd)[sub] = 0;
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
__global__ __launch_bounds__(kBlock) void c4_search_kernel(SearchParams p) {
    __shared__ uint32_t s_order[128];
    for (int i = threadIdx.x; i < 128; i += kBlock) s_order[i] = d_order[i];
    __syncthreads();

    const int lane = threadIdx.x & 63;
    const int sub = lane & (kGroup - 1);
    const int gbase = lane & ~(kGroup - 1);
    const int gl = blockIdx.x * (kBlock / kGroup) + (threadIdx.x / kGroup);  // game within call
    if (gl >= p.n_games) return;                                            // whole group leaves
    const int g = p.first_game + gl;                                          // engine game

    const zc_c4_state root = p.roots[gl];
    const uint64_t rp0 = root.stones[0], rp1 = root.stones[1];
    const int rturn = root.turn;
    zc_game_stats st{};
    if (!valid_state(rp0, rp1, rturn) || legal_mask(rp0 | rp1) == 0) {
        if (sub == 0) {
            st.status = valid_state(rp0, rp1, rturn) ? ZC_STATUS_NO_MOVES : ZC_STATUS_BAD_STATE;
            p.out_stats[gl] = st;
            p.out_move[gl] = -1;
        }
        if (sub < 7) p.out_na[(size_t)gl * 7 + sub] = 0;
        return;
    }

    const Arena &a = p.a;
    Tree t{a.nodes + (size_t)g * p.M * kRecBytes, a.W + (size_t)g * p.M * kSlots};
    uint32_t *const path0 = a.path + (size_t)g * p.max_batch * kMaxDepth;
    uint64_t *const pstate = a.pstate + (size_t)g * p.max_batch * 2;
    uint32_t *const pmeta = a.pmeta + (size_t)g * p.max_batch;
    int32_t *const pval = a.pval + (size_t)g * p.max_batch;

    Rng rng;
    const uint64_t use0 = a.rngpos[2 * (size_t)g];
    rng_open(rng, a.ring + (size_t)g * kRingWords, use0, a.rngpos[2 * (size_t)g + 1], sub);

    node_init(t, 0, 0xFFFF, 0xFF, 0, s_order[legal_mask(rp0 | rp1)], sub);
    int nnodes = 1;
    int64_t plies = 0;
    wave_mem_order();

    for (int done = 0; done < p.sims;) {
        const int nb = min(p.bs, p.sims - done);
        rng_fill(rng, rng.use + kLookahead, sub);

        // ---- selection + expansion of nb leaves (mcts.cpp:129-147) -------------------------
        // Within a flush no backup happens, so UCT scores on the path above the node that
        // was just expanded cannot change: leaf j+1's walk resumes there (exactly the walk
        // the reference repeats from the root).
        int xnode = 0, xdepth = 0, xturn = rturn;
        uint64_t x0 = rp0, x1 = rp1;
        for (int j = 0; j < nb; ++j) {
            uint32_t *const pj = path0 + (size_t)j * kMaxDepth;
            int node = xnode, depth = xdepth, turn = xturn;
            uint64_t b0 = x0, b1 = x1;
            if (j == 0) {
                if (sub == 0) pj[0] = 0x00FF0000u;
            } else {
                const uint32_t *pp = pj - kMaxDepth;
                for (int l = sub; l <= depth; l += kGroup) pj[l] = pp[l];
            }
            uint32_t u, ow;
            for (;;) {  // select (mcts.cpp:47-63)
                const uint32_t *h = t.hdr(node);
                u = h[1];
                ow = h[3];
                if ((u >> 24) & 15u) break;  // untried moves left: expand here
                if (depth >= kMaxDepth - 2) {  // unreachable (a C4 tree is <= 42 deep); never spin
                    st.status = ZC_STATUS_INTERNAL;
                    u = 0;
                    break;
                }
                const int nm = (int)(u >> 28);
                const uint16_t ch = t.child(node)[sub];
                const int32_t na = t.na(node)[sub];
                const double q = t.q(node)[sub];
                const double lg = t.q(node)[7];
                // UCT (mcts.cpp:41-45) = fma(c, sqrt(log(N)/Na), Qa); unvisited -> +inf
                double v = (sub < nm && ch != 0xFFFF)
                               ? (na == 0 ? INFINITY : fma(p.c, sqrt(lg / (double)na), q))
                               : -INFINITY;
                int bi = sub;
                group_argmax(v, bi);
                if (v == -INFINITY) break;  // no child at all: terminal node is its own leaf
                const int nxt = __shfl((int)ch, gbase + bi);
                const uint64_t bit = drop_bit(b0 | b1, (int)((ow >> (3 * bi)) & 7u));
                if (turn) b1 |= bit; else b0 |= bit;
                turn ^= 1;
                node = nxt;
                ++depth;
                if (sub == (depth & (kGroup - 1))) pj[depth] = (uint32_t)node | ((uint32_t)bi << 16);
            }
            // the walk ends here; leaf j+1 resumes from this node
            xnode = node;
            xdepth = depth;
            xturn = turn;
            x0 = b0;
            x1 = b1;
            int leaf = node;
            const uint32_t cnt = (u >> 24) & 15u;
            if (cnt) {  // expand (mcts.cpp:65-78): policy = random.choice(untried)
                const uint32_t r = rng_below(rng, cnt, sub, gbase);
                const uint32_t digits = u & 0x1FFFFFu;
                const int mi = (int)((digits >> (3 * r)) & 7u);
                const uint32_t low = (1u << (3 * r)) - 1u;
                const uint32_t rest = (digits & low) | ((digits >> 3) & ~low & 0x1FFFFFu);
                if (sub == 0) t.hdr(node)[1] = rest | ((cnt - 1u) << 24) | (u & 0xF0000000u);
                const uint64_t bit = drop_bit(b0 | b1, (int)((ow >> (3 * mi)) & 7u));
                if (turn) b1 |= bit; else b0 |= bit;
                turn ^= 1;
                leaf = nnodes++;
                ++depth;
                node_init(t, leaf, node, mi, depth, s_order[legal_mask(b0 | b1)], sub);
                if (sub == mi) t.child(node)[mi] = (uint16_t)leaf;
                if (sub == (depth & (kGroup - 1))) pj[depth] = (uint32_t)leaf | ((uint32_t)mi << 16);
                st.expansions += 1;
                st.depth_sum += depth;
            }
            if (sub == 0) {
                pstate[2 * j] = b0;
                pstate[2 * j + 1] = b1;
                pmeta[j] = (uint32_t)leaf | ((uint32_t)depth << 16) | ((uint32_t)turn << 24);
            }
            wave_mem_order();
        }

        // ---- value.batch: random rollouts in pending order (mcts.cpp:112-124) ---------------
        for (int j = 0; j < nb; ++j) {
            const uint32_t meta = pmeta[j];
            const int v = c4_rollout(pstate[2 * j], pstate[2 * j + 1], (int)(meta >> 24), rng, s_order, sub, gbase,
                                     plies);
            if (sub == 0) pval[j] = v;
        }
        wave_mem_order();

        // ---- backprop in pending order (mcts.cpp:80-100, :124-125) --------------------------
        // Level l of every path is handled by lane l % 8; a node's level never changes, so
        // every read-modify-write of a given word stays in one lane, in leaf order.
        for (int j = 0; j < nb; ++j) {
            const uint32_t *pj = path0 + (size_t)j * kMaxDepth;
            const int d = (int)((pmeta[j] >> 16) & 0xFFu);
            const int v = pval[j];
            for (int l = sub; l <= d; l += kGroup) {
                const uint32_t e = pj[l];
                const int nd = (int)(e & 0xFFFFu);
                const int vl = ((d - l) & 1) ? -v : v;
                uint32_t *h = t.hdr(nd);
                const uint32_t n1 = h[0] + 1u;
                h[0] = n1;
                t.q(nd)[7] = a.logtab[n1];
                if (l > 0) {
                    const int par = (int)(pj[l - 1] & 0xFFFFu);
                    const int act = (int)(e >> 16);
                    const int32_t na1 = t.na(par)[act] + 1;
                    const int32_t w1 = t.w(par)[act] - vl;  // Wa -= result
                    t.na(par)[act] = na1;
                    t.w(par)[act] = w1;
                    t.q(par)[act] = (double)w1 / (double)na1;  // Qa = Wa / Na
                }
            }
            wave_mem_order();
        }
        st.leaves += nb;
        done += nb;
    }

    // ---- best move: first max of child N over the root's move list (mcts.cpp:150-157) ----
    const uint32_t u = t.hdr(0)[1];
    const uint32_t ow = t.hdr(0)[3];
    const int nm = (int)(u >> 28);
    const int na = (sub < nm) ? t.na(0)[sub] : -1;
    int bv = na, bi = sub;
    group_argmax_int(bv, bi);
    int pos = 0;
    bool found = false;
    for (int k = 0; k < nm; ++k)
        if ((int)((ow >> (3 * k)) & 7u) == sub) { pos = k; found = true; }
    const int na_col = __shfl(na, gbase + pos);
    if (sub < 7) p.out_na[(size_t)gl * 7 + sub] = found ? na_col : 0;
    if (sub == 0) {
        p.out_move[gl] = (int)((ow >> (3 * bi)) & 7u);
        st.rollout_plies = plies;
        st.rng_words = (int64_t)(rng.use - use0);
        p.out_stats[gl] = st;
        a.rngpos[2 * (size_t)g] = rng.use;
        a.rngpos[2 * (size_t)g + 1] = rng.gen;
    }
}

// ------------------------------------------------------------------ self-test kernels
__global__ __launch_bounds__(kBlock) void c4_rollout_debug_kernel(Arena a, int first_game, int n,
                                                                  const zc_c4_state *states, int32_t *out_value,
                                                                  int64_t *out_words) {
    __shared__ uint32_t s_order[128];
    for (int i = threadIdx.x; i < 128; i += kBlock) s_order[i] = d_order[i];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int sub = lane & (kGroup - 1);
    const int gbase = lane & ~(kGroup - 1);
    const int gl = blockIdx.x * (kBlock / kGroup) + (threadIdx.x / kGroup);
    if (gl >= n) return;
    const int g = first_game + gl;
    Rng rng;
    const uint64_t use0 = a.rngpos[2 * (size_t)g];
    rng_open(rng, a.ring + (size_t)g * kRingWords, use0, a.rngpos[2 * (size_t)g + 1], sub);
    const zc_c4_state s = states[gl];
    int64_t plies = 0;
    const int v = c4_rollout(s.stones[0], s.stones[1], s.turn, rng, s_order, sub, gbase, plies);
    if (sub == 0) {
        out_value[gl] = v;
        out_words[gl] = (int64_t)(rng.use - use0);
        a.rngpos[2 * (size_t)g] = rng.use;
        a.rngpos[2 * (size_t)g + 1] = rng.gen;
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
    if (has_four(s.stones[turn])) r = s.turn * 2 - 1;   // check_win: the side that just moved
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

void launch_c4_search(const SearchParams &p, hipStream_t s) {
    const int per_block = kBlock / kGroup;
    const int blocks = (p.n_games + per_block - 1) / per_block;
    hipLaunchKernelGGL(c4_search_kernel, dim3(blocks), dim3(kBlock), 0, s, p);
}

void launch_c4_rollout_debug(const Arena &a, int M, int first_game, int n, const zc_c4_state *states,
                             int32_t *out_value, int64_t *out_words, hipStream_t s) {
    (void)M;
    const int per_block = kBlock / kGroup;
    hipLaunchKernelGGL(c4_rollout_debug_kernel, dim3((n + per_block - 1) / per_block), dim3(kBlock), 0, s, a,
                       first_game, n, states, out_value, out_words);
}

void launch_c4_play(int n, zc_c4_state *states, const int32_t *moves, int32_t *results, int reset, hipStream_t s) {
    hipLaunchKernelGGL(c4_play_kernel, dim3((n + 255) / 256), dim3(256), 0, s, n, states, moves, results, reset);
}

void launch_uct_debug(int n, const double *logn, const int32_t *na, const double *q, double c, double *out,
                      hipStream_t s) {
    hipLaunchKernelGGL(uct_debug_kernel, dim3((n + 255) / 256), dim3(256), 0, s, n, logn, na, q, c, out);
}

}  // namespace zc
