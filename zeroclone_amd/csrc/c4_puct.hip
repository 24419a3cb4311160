// c4_puct.hip — AlphaZero-style PUCT search for Connect4 on gfx950 (SURVEY.md §8 a21 on the
// target game).  The reference has no counterpart: its search is plain UCT with one-at-a-
// time expansion and random rollouts (engine/mcts/src/mcts.cpp:41-78), its network plugin a
// value net only (engine/value_functions.py:61-99).  This extension keeps the reference's
// game rules (engine/games/connect4/c4_backend.py: legal moves in CPython set order,
// check_win on the last mover, check_draw on a full board), its flush protocol and the
// leaf value convention, and changes the search to the chess PUCT form (chess_puct.hip):
//
//   select  a = first argmax  Q(a) + c_puct * P(a) * sqrt(sum_b N(b)) / (1 + N(a)),
//           Q(a) = W(a) / N(a) (0 when N(a) = 0); the walk stops at an edge without a child
//           (the child is created and is the leaf), at a terminal position (four in a row
//           for the last mover, or a full board) or at a node still waiting for its
//           evaluation; virtual loss on every edge walked (N += 1, W -= 1) until backup;
//   backup  per leaf in pending order: a first evaluation sets the node's priors = softmax
//           of the policy head's 7 column logits over the legal columns (Dirichlet(alpha)
//           noise of weight eps at the root, Philox keyed by (seed, game)); every edge then
//           takes W += 1 - r with r = the leaf value, alternating in sign (N already
//           counted); a terminal leaf's value is -1 (the side to move has lost) or 0;
//   root    flush 0 evaluates the root alone.
//
// Node = one 192-byte record, slot k (a move, in the node's move-list order) in lane k:
// everything a selection step reads is one coalesced load per field.  One wave per game.
// Specification in executable form: oracle/puct_ref.py (C4Rules).
#include <hip/hip_fp16.h>

#include "c4_device.h"
#include "puct_common.h"

namespace zc {
namespace {

static_assert(sizeof(C4PNode) == 192, "C4PNode is 192 bytes");

enum : int { pNodes = 0, pStatus = 1, pNb = 2, pExp = 3, pDepth = 4 };

__device__ __forceinline__ C4PNode *pnodes(const C4PuctParams &p, int g) { return p.nodes + (size_t)g * p.M; }

// flushes: 0 = the root alone, then batches of bs
__device__ __forceinline__ int pflush_leaves(const C4PuctParams &p, int f) {
    if (f == 0) return 1;
    return max(0, min(p.bs, p.sims - 1 - (f - 1) * p.bs));
}

// Node(state): move list in CPython set order (c4_backend.get_legal_moves), none at a
// terminal position (the last mover has four, or the board is full).
__device__ __forceinline__ void pnode_init(C4PNode *N, uint64_t s0, uint64_t s1, int turn, int parent, int pact,
                                           int depth) {
    const uint32_t lane = lane_id();
    const uint64_t occ = s0 | s1;
    const bool won = has_four(turn ? s0 : s1);  // check_win: the last mover's stones
    const int lm = legal_mask(occ);
    const uint32_t ow = d_order[lm];
    const int nm = (won || occ == kFull) ? 0 : (int)((ow >> 24) & 15u);
    if (lane == 0) {
        N->s0 = s0;
        N->s1 = s1;
        N->order = ow;
        N->turn = (uint8_t)turn;
        N->nmoves = (uint8_t)nm;
        N->evaluated = 0;
        N->won = won ? 1 : 0;
        N->parent = (uint16_t)parent;
        N->pact = (uint8_t)pact;
        N->depth = (uint8_t)depth;
    }
    if (lane < kSlots) {
        N->child[lane] = 0xFFFF;
        N->na[lane] = 0;
        N->pr[lane] = 0.0f;
        N->w[lane] = 0.0;
    }
}

__global__ __launch_bounds__(64) void c4_puct_begin_kernel(C4PuctParams p) {
    const int gl = blockIdx.x;
    if (gl >= p.n_games) return;
    const int g = p.first_game + gl;
    const zc_c4_state root = p.roots[gl];
    const uint64_t s0 = uni64(root.stones[0]), s1 = uni64(root.stones[1]);
    const int turn = uni(root.turn);
    int32_t *ctl = p.ctl + (size_t)g * kCtlWords;
    int status = 0;
    if (!valid_state(s0, s1, turn)) {
        status = ZC_STATUS_BAD_STATE;
    } else {
        C4PNode *N = pnodes(p, g);
        pnode_init(N, s0, s1, turn, 0xFFFF, 0xFF, 0);
        wave_mem_order();
        if (uni((int)N->nmoves) == 0) status = ZC_STATUS_NO_MOVES;
    }
    if (lane_id() == 0) {
        ctl[pNodes] = 1;
        ctl[pStatus] = status;
        ctl[pNb] = 0;
        ctl[pExp] = 0;
        ctl[pDepth] = 0;
    }
}

// One PUCT walk + expansion; returns the leaf and its depth, the edges of its path in lanes
// 1..depth of pathv (node | slot << 16).  Applies the virtual loss on every edge it takes.
__device__ int c4_puct_walk(const C4PuctParams &p, C4PNode *T, int &nnodes, int &status, int &ldepth,
                            uint32_t &pathv, Counters &cn) {
    const uint32_t lane = lane_id();
    const uint32_t k = lane & 7u;
    int node = 0, depth = 0;
    pathv = 0;
    for (;;) {
        C4PNode *N = &T[node];
        const int nm = uni((int)N->nmoves);
        if (nm == 0 || !uni((int)N->evaluated)) break;  // terminal, or a leaf still pending
        if (depth >= kMaxDepth - 2) {  // unreachable (a Connect4 game is <= 42 plies)
            status = ZC_STATUS_INTERNAL;
            break;
        }
        const bool valid = (int)k < nm;
        const int32_t na = valid ? N->na[k] : 0;
        const double wk = valid ? N->w[k] : 0.0;
        const float pk = valid ? N->pr[k] : 0.0f;
        const uint32_t chk = valid ? (uint32_t)N->child[k] : 0xFFFFu;  // with the others: no dependent load after the argmax
        // sum_b N(b): lanes 0..7 (integers: exact in any order)
        int tot = (lane < 8u) ? na : 0;
        tot += dpp<0xB1>(tot);
        tot += dpp<0x4E>(tot);
        tot += dpp<0x141>(tot);
        const double sq = sqrt((double)uni(tot));
        const double q = na > 0 ? wk / (double)na : 0.0;
        double v = valid ? q + p.c * (double)pk * sq / (double)(1 + na) : -INFINITY;
        int bi = (int)k;
        argmax8(v, bi);
        const int best = uni(bi);
        if (lane == 0) {  // virtual loss: one visit lost by this node's mover
            N->na[best] = N->na[best] + 1;
            N->w[best] = N->w[best] - 1.0;
        }
        ++depth;
        if (lane == (uint32_t)depth) pathv = (uint32_t)node | ((uint32_t)best << 16);
        const int child = (int)(uint32_t)__builtin_amdgcn_readlane((int)chk, best);
        if (child != 0xFFFF) {
            node = child;
            continue;
        }
        // expand the edge: the child position (c4_backend.play_move), its move list
        const int id = nnodes;
        if (id >= p.M) {
            status = ZC_STATUS_CAPACITY;
            break;
        }
        ++nnodes;
        const uint64_t s0 = uni64(N->s0), s1 = uni64(N->s1);
        const int turn = uni((int)N->turn);
        const int col = (int)((uni(N->order) >> (3 * best)) & 7u);
        const uint64_t bit = drop_bit(s0 | s1, col);
        pnode_init(&T[id], turn ? s0 : s0 | bit, turn ? s1 | bit : s1, turn ^ 1, node, best, depth);
        if (lane == 0) N->child[best] = (uint16_t)id;
        cn.add(cn.expansions, 1);
        cn.add(cn.depth_sum, depth);
        wave_mem_order();
        node = id;
        break;
    }
    ldepth = depth;
    return node;
}

__global__ __launch_bounds__(64) void c4_puct_select_kernel(C4PuctParams p) {
    const int gl = blockIdx.x;
    if (gl >= p.n_games) return;
    const int g = p.first_game + gl;
    C4PNode *T = pnodes(p, g);
    int32_t *ctl = p.ctl + (size_t)g * kCtlWords;
    const uint32_t lane = lane_id();
    int status = uni(ctl[pStatus]);
    int nb = status ? 0 : pflush_leaves(p, p.flush);
    int nnodes = uni(ctl[pNodes]);
    uint32_t *paths = p.paths + (size_t)g * p.max_batch * kMaxDepth;
    uint32_t *meta = p.meta + (size_t)g * p.max_batch;
    Counters cn;
    for (int j = 0; j < nb && !status; ++j) {
        int d = 0;
        uint32_t pathv = 0;
        const int leaf = p.flush == 0 ? 0 : c4_puct_walk(p, T, nnodes, status, d, pathv, cn);
        if (lane < (uint32_t)kMaxDepth) paths[(size_t)j * kMaxDepth + lane] = pathv;
        if (lane == 0) meta[j] = (uint32_t)leaf | ((uint32_t)d << 16);
    }
    if (status) nb = 0;
    wave_mem_order();
    if (lane == 0) {
        ctl[pNodes] = nnodes;
        ctl[pStatus] = status;
        ctl[pNb] = nb;
        ctl[pExp] += cn.expansions;
        ctl[pDepth] += cn.depth_sum;
        if (p.counts) p.counts[gl] = nb;
    }
    // the pending flush's leaves: states, and state_to_tensor planes (c4_backend.py:52-61:
    // [2][6][7], plane 0 = the side to move's stones, row 0 = top = bit row 5 - r)
    const size_t obase = (size_t)gl * p.bs;
    for (int j = (int)lane; j < nb; j += 64) {
        const C4PNode *N = &T[meta[j] & 0xFFFFu];
        if (p.leaves) {
            zc_c4_state s;
            s.stones[0] = N->s0;
            s.stones[1] = N->s1;
            s.turn = N->turn;
            s.reserved = 0;
            p.leaves[obase + j] = s;
        }
    }
    if (p.planes) {
        for (int idx = (int)lane; idx < nb * 84; idx += 64) {
            const int j = idx / 84, e = idx - j * 84;
            const int pl = e / 42, cell = e - pl * 42;
            const int r = cell / 7, col = cell - r * 7;
            const C4PNode *N = &T[meta[j] & 0xFFFFu];
            const uint64_t stones = (pl == (int)N->turn) ? N->s0 : N->s1;
            const float v = (float)((stones >> (7 * col + 5 - r)) & 1ull);
            const size_t o = (obase + j) * 84 + e;
            if (p.planes_f16) ((__half *)p.planes)[o] = __float2half(v);
            else ((float *)p.planes)[o] = v;
        }
    }
}

__global__ __launch_bounds__(64) void c4_puct_backup_kernel(C4PuctParams p) {
    const int gl = blockIdx.x;
    if (gl >= p.n_games) return;
    const int g = p.first_game + gl;
    C4PNode *T = pnodes(p, g);
    const int32_t *ctl = p.ctl + (size_t)g * kCtlWords;
    const uint32_t lane = lane_id();
    const int nb = uni(ctl[pNb]);
    if (uni(ctl[pStatus]) || nb == 0) return;
    const uint32_t *paths = p.paths + (size_t)g * p.max_batch * kMaxDepth;
    const uint32_t *meta = p.meta + (size_t)g * p.max_batch;
    const uint2 key = make_uint2((uint32_t)p.seed, (uint32_t)(p.seed >> 32));
    for (int j = 0; j < nb; ++j) {
        const uint32_t mt = uni(meta[j]);
        const int node = (int)(mt & 0xFFFFu), d = (int)(mt >> 16);
        C4PNode *N = &T[node];
        const int nm = uni((int)N->nmoves);
        const size_t li = (size_t)gl * (p.leaf_rows ? p.leaf_rows : p.bs) + j;
        double v;
        if (nm == 0) {
            v = uni((int)N->won) ? -1.0 : 0.0;  // the side to move has lost / a full board
        } else {
            v = __hiloint2double(uni(__double2hiint(p.values[li])), uni(__double2loint(p.values[li])));
            if (!uni((int)N->evaluated)) {
                // priors: softmax of the column logits over the node's legal columns, in
                // move-list order (slot k = lane k)
                const bool valid = lane < (uint32_t)nm;
                const uint32_t col = (uni(N->order) >> (3 * (lane & 7u))) & 7u;
                float lg = -INFINITY;
                if (valid)
                    lg = p.logits_f16 ? __half2float(((const __half *)p.logits)[li * 7 + col])
                                      : ((const float *)p.logits)[li * 7 + col];
                const float mx = wave_max_f(lg);
                const float e = valid ? expf(lg - mx) : 0.0f;
                const float sum = wave_sum_f(e);
                float pr = e / sum;
                if (node == 0 && p.dir_eps > 0.0f) {  // Dirichlet(alpha) noise on the root priors
                    const float gm = valid ? gamma_draw(p.dir_alpha, key, (uint32_t)g, lane, search_number(p, gl)) : 0.0f;
                    const float gs = wave_sum_f(gm);
                    pr = (1.0f - p.dir_eps) * pr + p.dir_eps * (gs > 0.0f ? gm / gs : 0.0f);
                }
                if (valid) N->pr[lane] = pr;
                if (lane == 0) N->evaluated = 1;
            }
        }
        wave_mem_order();
        // backup with the virtual loss undone: W += 1 - r on the edge into level l
        if (lane >= 1 && lane <= (uint32_t)d) {
            const uint32_t e = paths[(size_t)j * kMaxDepth + lane];
            C4PNode *P = &T[e & 0xFFFFu];
            const int s = (int)(e >> 16);
            const double r = ((d - (int)lane) & 1) ? -v : v;
            P->w[s] = P->w[s] + 1.0 - r;
        }
        wave_mem_order();
    }
}

__global__ __launch_bounds__(64) void c4_puct_end_kernel(C4PuctParams p) {
    const int gl = blockIdx.x;
    if (gl >= p.n_games) return;
    const int g = p.first_game + gl;
    const C4PNode *R = pnodes(p, g);
    const int32_t *ctl = p.ctl + (size_t)g * kCtlWords;
    const uint32_t lane = lane_id();
    const uint32_t k = lane & 7u;
    const int status = uni(ctl[pStatus]);
    const int nm = status ? 0 : uni((int)R->nmoves);
    const uint32_t ow = status ? 0u : uni(R->order);
    const int32_t na = (int)k < nm ? R->na[k] : -1;
    if (lane < 7) {  // visits and priors per column
        int pos = -1;
        for (int s = 0; s < nm; ++s)
            if ((int)((ow >> (3 * s)) & 7u) == (int)lane) pos = s;
        p.out_na[(size_t)gl * 7 + lane] = pos >= 0 ? R->na[pos] : 0;
        if (p.out_prior) p.out_prior[(size_t)gl * 7 + lane] = pos >= 0 ? R->pr[pos] : 0.0f;
    }
    int best = -1;
    if (nm > 0) {
        if (p.temperature <= 0.0f) {  // most visits, first maximum in move-list order
            int bv = na, bi = (int)k;
            argmax8(bv, bi);
            best = uni(bi);
        } else {  // sample proportional to Na^(1/T): inverse CDF over the moves in order
            double tot = 0.0;
            for (int j = 0; j < nm; ++j) tot += pow((double)uni(R->na[j]), 1.0 / (double)p.temperature);
            const uint4 r = philox(make_uint4((uint32_t)g, 0x5BE0CD19u, search_number(p, gl), 0),
                                   make_uint2((uint32_t)p.seed, (uint32_t)(p.seed >> 32)));
            const double target = (double)u01(r.x) * tot;
            double run = 0.0;
            best = nm - 1;
            for (int j = 0; j < nm; ++j) {
                run += pow((double)uni(R->na[j]), 1.0 / (double)p.temperature);
                if (run > target) {
                    best = j;
                    break;
                }
            }
        }
    }
    if (lane == 0) {
        if (p.search_no) p.search_no[gl] = (int32_t)(search_number(p, gl) + 1);
        p.out_move[gl] = best >= 0 ? (int)((ow >> (3 * best)) & 7u) : -1;
        zc_game_stats st{};
        st.status = status;
        st.expansions = ctl[pExp];
        st.depth_sum = ctl[pDepth];
        st.leaves = p.sims;
        p.out_stats[gl] = st;
    }
}

}  // namespace

void launch_c4_puct_begin(const C4PuctParams &p, hipStream_t s) {
    hipLaunchKernelGGL(c4_puct_begin_kernel, dim3(p.n_games), dim3(64), 0, s, p);
}
void launch_c4_puct_select(const C4PuctParams &p, hipStream_t s) {
    hipLaunchKernelGGL(c4_puct_select_kernel, dim3(p.n_games), dim3(64), 0, s, p);
}
void launch_c4_puct_backup(const C4PuctParams &p, hipStream_t s) {
    hipLaunchKernelGGL(c4_puct_backup_kernel, dim3(p.n_games), dim3(64), 0, s, p);
}
void launch_c4_puct_end(const C4PuctParams &p, hipStream_t s) {
    hipLaunchKernelGGL(c4_puct_end_kernel, dim3(p.n_games), dim3(64), 0, s, p);
}

}  // namespace zc
