// chess_tree.h — the chess search tree on the device (zc_internal.h ChessNode + SoA child
// slots) and the wave-level helpers shared by the UCT search (chess_search.hip) and the
// PUCT search (chess_puct.hip).  Included by exactly those translation units.
#pragma once
#include <hip/hip_runtime.h>

#ifndef ZC_CHESS_STAMP
#define ZC_CHESS_STAMP 0  // diagnostic build: per-game s_memtime cycles per phase (tools/chess_stamps.py)
#endif
#if ZC_CHESS_STAMP
// [game of the launch][kCStamps]: walk, policy + erase, apply_move, create_node, values, backup,
// select flush (whole), whole search, legal_moves_check, material, node writes,
// inside legal_moves_check: emission, copy, legality, bit view + check; then inside policy +
// erase: the cached path, the node fields + lazy generation, the untried / move loads, the
// pick + erase, and the count of cached expansions; the leader's wait for the helper, the
// leaf records, the flush's stream open + close.  A region adds
// its cycles to the workgroup's LDS copy with a no-return LDS atomic (no wait on the chain);
// the kernel folds the LDS copy into the global table once at its end (CSTAMP_FLUSH).
namespace zc {
namespace {
constexpr int kCStamps = 24;
__device__ uint64_t g_chess_stamp[4096 * kCStamps];
__shared__ uint64_t s_chess_stamp[kCStamps];
}  // namespace
}  // namespace zc
#define CSTAMP_T(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define CSTAMP_ADD(k, t0)                                                                          \
    do {                                                                                           \
        const uint64_t now_ = __builtin_amdgcn_s_memtime();                                        \
        if (__lane_id() == 0)                                                                      \
            __hip_atomic_fetch_add(&::zc::s_chess_stamp[(k)], now_ - (t0), __ATOMIC_RELAXED,       \
                                   __HIP_MEMORY_SCOPE_WORKGROUP);                                  \
    } while (0)
#define CSTAMP_COUNT(k)                                                                            \
    do {                                                                                           \
        if (__lane_id() == 0)                                                                      \
            __hip_atomic_fetch_add(&::zc::s_chess_stamp[(k)], (uint64_t)1, __ATOMIC_RELAXED,       \
                                   __HIP_MEMORY_SCOPE_WORKGROUP);                                  \
    } while (0)
#define CSTAMP_INIT()                                                                              \
    do {                                                                                           \
        if (__lane_id() < ::zc::kCStamps) ::zc::s_chess_stamp[__lane_id()] = 0;                    \
    } while (0)
#define CSTAMP_FLUSH()                                                                             \
    do {                                                                                           \
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");                                     \
        if (__lane_id() < ::zc::kCStamps && blockIdx.x < 4096)                                     \
            ::zc::g_chess_stamp[blockIdx.x * ::zc::kCStamps + __lane_id()] += ::zc::s_chess_stamp[__lane_id()]; \
    } while (0)
#else
#define CSTAMP_T(v)
#define CSTAMP_ADD(k, t0)
#define CSTAMP_COUNT(k)
#define CSTAMP_INIT()
#define CSTAMP_FLUSH()
#endif
#define CDEV_T(v) CSTAMP_T(v)
#define CDEV_ADD(k, t0) CSTAMP_ADD(k, t0)

#include "c4_device.h"
#include "chess_device.h"

namespace zc {
namespace {

using chessdev::ChessScratch;

struct CTree {
    ChessNode *nodes;
    uint16_t *mv;
    uint8_t *ut;
    uint16_t *ch;
    int32_t *na;
    double *w;
    float *pr;
    int64_t S;
};

__device__ __forceinline__ CTree ctree(const ChessParams &p, int g) {
    const ChessArena &a = p.ca;
    const size_t so = (size_t)g * (size_t)a.S;
    return CTree{a.nodes + (size_t)g * p.M, a.mv + so, a.ut + so, a.ch + so, a.na + so, a.w + so,
                 a.prior ? a.prior + so : nullptr, a.S};
}

enum : int { cNodes = 0, cSlots = 1, cStatus = 2, cNb = 3, cExp = 4, cDepth = 5, cUse0 = 6, cHpNode = 8 };

struct CLds {
    ChessScratch s;
    zc_chess_state st;  // staging: the position of the node being created
};

__device__ __forceinline__ void wave_sync_mem() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

// Node(state, get_legal_moves(state), parent, idx) (mcts.cpp:23-34) for the position in
// L.st, in two parts: create_node_gen generates the legal moves (into L.s.legal), the check flag
// of a position without moves and the material; create_node_commit takes the next `n` slots
// and writes the moves (all untried, no children) and the node record.  The generation is the
// expensive part and touches nothing but L, so another wave can run it (chess_search.hip's
// helper wave) while the leader generates another node.
struct NodeGen {
    int n;
    int check;
    int32_t mat;
    int lazy;  // 1: the position has legal moves, not generated yet (legal_moves_probe); NodeGen{n, check, mat}: 0
};

// ChessNode::nmoves of a lazy node (nu = 1: the walk stops there, and its first expansion
// generates the list: chess_search.hip generate_lazy)
constexpr uint16_t kChessLazy = 0xFFFF;

// The child of the position in `stw` (lanes 0..17: its zc_chess_state words) by move m, into
// L.st, and its generation, with the child's squares kept in registers (one LDS round trip
// fewer than staging the parent in L.st and applying the move there).
template <bool PROBE = false>
__device__ __forceinline__ NodeGen create_child_gen(CLds &L, uint32_t stw, uint32_t m) {
    const uint32_t lane = lane_id();
    uint32_t w16;
    const uint32_t x = chessdev::apply_move_regs(stw, m, w16);
    L.st.board[lane] = (uint8_t)x;
    if (lane == 16) ((uint32_t *)&L.st)[16] = w16;
    if (lane == 17) ((uint32_t *)&L.st)[17] = stw;
    wave_sync_mem();
    bool check, lazy = false;
    CSTAMP_T(cs8);
    const int n = PROBE ? chessdev::legal_moves_probe(L.st.board, x, (int)(w16 & 0xFFu), L.s.legal, L.s.pseudo,
                                                      L.s.region, check, lazy)
                        : chessdev::legal_moves_check(L.st.board, x, (int)(w16 & 0xFFu), L.s.legal, L.s.pseudo,
                                                      L.s.region, check);
    CSTAMP_ADD(8, cs8);
    CSTAMP_T(cs9);
    const int32_t mat = chessdev::material(x);
    CSTAMP_ADD(9, cs9);
    return NodeGen{n, check ? 1 : 0, mat, lazy ? 1 : 0};
}

__device__ __forceinline__ NodeGen create_node_gen(CLds &L) {
    const uint32_t lane = lane_id();
    const uint32_t sq = L.st.board[lane];
    L.s.board[lane] = (uint8_t)sq;
    wave_sync_mem();
    const int turn = uni((int)L.st.turn);
    bool check;
    CSTAMP_T(cs8);
    const int n = chessdev::legal_moves_check(L.s.board, turn, L.s.legal, L.s.pseudo, L.s.region, check);
    CSTAMP_ADD(8, cs8);
    CSTAMP_T(cs9);
    const int32_t mat = chessdev::material(sq);
    CSTAMP_ADD(9, cs9);
    return NodeGen{n, check ? 1 : 0, mat};
}

// The slot range of a node of gen.n moves: its base (the next free slot) and the move count it
// keeps (0 when the list overflowed or the slots ran out: ZC_STATUS_CAPACITY).
__device__ __forceinline__ int create_node_take(const CTree &t, NodeGen gen, int &slots, int &status) {
    if (gen.lazy) return 0;  // no list, no slots until its first expansion
    int n = gen.n;
    if (n < 0) {
        status = ZC_STATUS_CAPACITY;
        n = 0;
    }
    const int base = slots;
    if ((int64_t)base + n > t.S) {
        status = ZC_STATUS_CAPACITY;
        n = 0;
    }
    slots = base + n;
    return n;
}

__device__ __forceinline__ void create_node_commit(const CTree &t, const CLds &L, NodeGen gen, int id, int parent,
                                                   int pact, int depth, int &slots, int &status) {
    const uint32_t lane = lane_id();
    CSTAMP_T(cs10);
    const int base = slots;
    const int n = create_node_take(t, gen, slots, status);
    for (int j = (int)lane; j < n; j += 64) {
        t.mv[base + j] = L.s.legal[j];
        t.ut[base + j] = (uint8_t)j;
        t.ch[base + j] = 0xFFFF;
        t.na[base + j] = 0;
        t.w[base + j] = 0.0;
    }
    ChessNode *N = &t.nodes[id];
    if (lane < 18) ((uint32_t *)&N->st)[lane] = ((const uint32_t *)&L.st)[lane];
    if (lane == 0) {
        N->base = (uint32_t)base;
        N->nmoves = gen.lazy ? kChessLazy : (uint16_t)n;
        N->nu = gen.lazy ? (uint16_t)1 : (uint16_t)n;
        N->parent = (uint16_t)parent;
        N->pact = (uint16_t)pact;
        N->depth = (uint16_t)depth;
        N->material = (int16_t)gen.mat;
        N->check = gen.check ? 1 : 0;
        N->evaluated = 0;
    }
    wave_sync_mem();
    CSTAMP_ADD(10, cs10);
}

__device__ void create_node(const CTree &t, CLds &L, int id, int parent, int pact, int depth, int &slots, int &status) {
    const NodeGen gen = create_node_gen(L);
    create_node_commit(t, L, gen, id, parent, pact, depth, slots, status);
}

__device__ __forceinline__ void argmax64(double &v, int &i) {
    for (int o = 32; o > 0; o >>= 1) {
        const double ov = __shfl_xor(v, o);
        const int oi = __shfl_xor(i, o);
        if (ov > v || (ov == v && oi < i)) {
            v = ov;
            i = oi;
        }
    }
}

// The r-th set position (in index order) of a predicate over [0, n), 64 per pass.
template <class Pred>
__device__ __forceinline__ int nth_true(int n, uint32_t r, Pred pred) {
    const uint32_t lane = lane_id();
    for (int b = 0; b < n; b += 64) {
        const int j = b + (int)lane;
        const uint64_t m = __ballot(j < n && pred(j));
        const uint32_t c = (uint32_t)__popcll(m);
        if (r < c) {
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            const uint64_t hit = __ballot(((m >> lane) & 1ull) && rank == r);
            return b + __builtin_ctzll(hit);
        }
        r -= c;
    }
    return -1;
}

}  // namespace
}  // namespace zc
