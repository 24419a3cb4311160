// chess_puct.hip — AlphaZero-style PUCT search for chess on gfx950 (SURVEY.md §8 a21, config
// C5: a policy + value network, Dirichlet root noise).  The reference has no counterpart
// (its search is plain UCT with one-at-a-time expansion, mcts.cpp:41-78); this extension
// reuses its tree, rules and flush protocol and changes the selection rule:
//
//   select  a = first argmax  Q(a) + c_puct * P(a) * sqrt(sum_b N(b)) / (1 + N(a)),
//           Q(a) = W(a) / N(a) (0 when N(a) = 0), P from the policy head of the node's own
//           evaluation; the walk stops at an edge without a child (the child is created and
//           is the leaf), at a terminal node, or at a node still waiting for its evaluation;
//   virtual loss: every edge of a pending leaf's path counts as one visit lost by the
//           parent's mover (N += 1, W -= 1) until the flush is backed up, so the leaves of a
//           flush spread over the tree instead of repeating one path;
//   backup  per leaf in pending order: the node's priors = softmax of the policy logits over
//           its legal moves (first evaluation only), then each edge undoes its virtual loss
//           and takes the value (W += 1 - r, N already counted), r alternating in sign;
//           a terminal leaf's value is -1 (side to move mated) or 0 (no moves otherwise);
//   root    flush 0 evaluates the root alone; its priors get Dirichlet(alpha) noise with
//           weight eps, drawn with a counter-based Philox4x32-10 stream keyed by (seed, game).
//
// Launches (one wave per game): begin (root node), select (flush f's leaves, planes),
// backup (priors + values), end (move by visits or temperature sampling, visit counts).
#include <hip/hip_fp16.h>

#include "chess_tree.h"
#include "puct_common.h"

namespace zc {
namespace {

// meta[j] bit 31: leaf j's walk created its node (its moves are generated after the walks)
constexpr uint32_t kMetaCreated = 0x80000000u;

// flushes: 0 = the root alone, then batches of bs
__device__ __forceinline__ int flush_leaves(const ChessParams &p, int f) {
    if (f == 0) return 1;
    return max(0, min(p.bs, p.sims - 1 - (f - 1) * p.bs));
}

// One PUCT walk + expansion; returns the leaf, its depth, and the edge slots of its path
// in lanes 1..depth of pathv.  Applies the virtual loss on every edge it takes.
//
// The expansion is DEFERRED: the new node gets its id, position, parent, depth and
// `evaluated = 0` here — everything a later walk of the same flush looks at (it stops at a node
// not yet evaluated) — and *created is set; its legal moves are generated after the flush's
// walks, every created node of every game in parallel (puct_expand_kernel, one wave each), and
// committed in creation order (puct_commit_kernel: slot ranges by a prefix sum over the
// creation order, i.e. exactly the ranges the serial create_node would have taken).  Nothing
// reads a node's moves before its first backup, so the tree is the serial one.
__device__ int puct_walk(const ChessParams &p, const CTree &t, CLds &L, int &nnodes, int &slots, int &status,
                         int &ldepth, uint32_t &pathv, Counters &cn, bool &created) {
    const uint32_t lane = lane_id();
    int node = 0, depth = 0;
    pathv = 0;
    for (;;) {
        ChessNode *N = &t.nodes[node];
        const int nm = uni((int)N->nmoves);
        if (nm == 0 || !uni((int)N->evaluated)) break;  // terminal, or a leaf still pending
        if (depth >= kChessPath - 2) {
            status = ZC_STATUS_CAPACITY;
            break;
        }
        const uint32_t base = uni(N->base);
        // ONE round of loads per level: every child slot's N, W, P and child id (up to four
        // 64-slot chunks, registers), issued together; the sum of N, the scores and the child
        // pointer then come from registers (round 4 read N twice and the child once more:
        // three dependent global round trips per level).  Same arithmetic in the same order.
        int32_t na_r[4];
        double w_r[4];
        float pr_r[4];
        uint32_t ch_r[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int j = q * 64 + (int)lane;
            na_r[q] = 0;
            w_r[q] = 0.0;
            pr_r[q] = 0.0f;
            ch_r[q] = 0xFFFFu;
            if (q * 64 < nm && j < nm) {
                na_r[q] = t.na[base + j];
                w_r[q] = t.w[base + j];
                pr_r[q] = t.pr[base + j];
                ch_r[q] = t.ch[base + j];
            }
        }
        double tot = 0.0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int j = q * 64 + (int)lane;
            if (q * 64 < nm) tot += j < nm ? (double)na_r[q] : 0.0;
        }
        const double sq = sqrt(wave_sum_d(tot));
        double bv = -INFINITY;
        int bi = 0x7FFFFFFF;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int j = q * 64 + (int)lane;
            if (q * 64 < nm && j < nm) {
                const int32_t na = na_r[q];
                const double qv = na > 0 ? w_r[q] / (double)na : 0.0;
                const double u = p.c * (double)pr_r[q] * sq / (double)(1 + na);
                const double v = qv + u;
                if (v > bv) {
                    bv = v;
                    bi = j;
                }
            }
        }
        argmax64(bv, bi);
        const int best = uni(bi);
        const uint32_t s = base + (uint32_t)best;
        const int bq = best >> 6;
        const uint32_t chv = bq == 0 ? ch_r[0] : bq == 1 ? ch_r[1] : bq == 2 ? ch_r[2] : ch_r[3];
        const int child = (int)(uint32_t)__builtin_amdgcn_readlane((int)chv, best & 63);
        if (lane == 0) {  // virtual loss: one visit lost by this node's mover
            t.na[s] += 1;
            t.w[s] -= 1.0;
        }
        ++depth;
        if (lane == (uint32_t)depth) pathv = s;
        if (child != 0xFFFF) {
            node = child;
            continue;
        }
        // expand the edge: the child position, its legal moves, no priors yet
        const uint32_t m = uni((uint32_t)t.mv[s]);
        if (lane < 18) ((uint32_t *)&L.st)[lane] = ((const uint32_t *)&N->st)[lane];
        wave_sync_mem();
        chessdev::apply_move_wave(L.st, m);
        wave_sync_mem();
        const int id = nnodes++;
        if (id >= p.M) {
            status = ZC_STATUS_CAPACITY;
            break;
        }
        ChessNode *C = &t.nodes[id];  // the record without its moves (puct_commit_kernel adds them)
        if (lane < 18) ((uint32_t *)&C->st)[lane] = ((const uint32_t *)&L.st)[lane];
        if (lane == 0) {
            C->base = 0;
            C->nmoves = 0;
            C->nu = 0;
            C->parent = (uint16_t)node;
            C->pact = (uint16_t)best;
            C->depth = (uint16_t)depth;
            C->evaluated = 0;
            t.ch[s] = (uint16_t)id;
        }
        created = true;
        cn.add(cn.expansions, 1);
        cn.add(cn.depth_sum, depth);
        wave_sync_mem();
        node = id;
        break;
    }
    ldepth = depth;
    return node;
}

__global__ __launch_bounds__(64) void puct_begin_kernel(ChessParams p) {
    __shared__ CLds L;
    const int gl = blockIdx.x;
    if (gl >= p.n_games) return;
    const int g = p.first_game + gl;
    const CTree t = ctree(p, g);
    int32_t *ctl = p.ca.ctl + (size_t)g * kCtlWords;
    const uint32_t lane = lane_id();
    if (lane < 18) {
        const uint32_t w = ((const uint32_t *)&p.roots[gl])[lane];
        ((uint32_t *)&L.st)[lane] = w;
        ((uint32_t *)&p.ca.roots[g])[lane] = w;
    }
    wave_sync_mem();
    int slots = 0, status = 0;
    create_node(t, L, 0, 0xFFFF, 0xFFFF, 0, slots, status);
    if (!status && uni((int)t.nodes[0].nmoves) == 0) status = ZC_STATUS_NO_MOVES;
    if (lane == 0) {
        ctl[cNodes] = 1;
        ctl[cSlots] = slots;
        ctl[cStatus] = status;
        ctl[cNb] = 0;
        ctl[cExp] = 0;
        ctl[cDepth] = 0;
    }
}

__global__ __launch_bounds__(64) void puct_select_kernel(ChessParams p) {
    __shared__ CLds L;
    const int gl = blockIdx.x;
    if (gl >= p.n_games) return;
    const int g = p.first_game + gl;
    const CTree t = ctree(p, g);
    int32_t *ctl = p.ca.ctl + (size_t)g * kCtlWords;
    const uint32_t lane = lane_id();
    int status = uni(ctl[cStatus]);
    int nb = status ? 0 : flush_leaves(p, p.flush);
    int nnodes = uni(ctl[cNodes]), slots = uni(ctl[cSlots]);
    uint32_t *paths = p.ca.paths + (size_t)g * p.max_batch * kChessPath;
    uint32_t *meta = p.ca.meta + (size_t)g * p.max_batch;
    Counters cn;
    int j = 0;
    for (; j < nb && !status; ++j) {
        int d = 0;
        uint32_t pathv = 0;
        bool created = false;
        const int leaf = p.flush == 0 ? 0 : puct_walk(p, t, L, nnodes, slots, status, d, pathv, cn, created);
        if (lane < (uint32_t)kChessPath) paths[(size_t)j * kChessPath + lane] = pathv;
        if (lane == 0) meta[j] = (uint32_t)leaf | ((uint32_t)d << 16) | (created ? kMetaCreated : 0u);
    }
    if (status) nb = 0;
    wave_sync_mem();
    if (lane == 0) {
        ctl[cNodes] = nnodes;
        ctl[cStatus] = status;
        ctl[cNb] = nb;
        ctl[cExp] += cn.expansions;
        ctl[cDepth] += cn.depth_sum;
        if (p.counts) p.counts[gl] = nb;
    }
    const size_t obase = (size_t)gl * p.bs;
    for (int k = 0; k < nb; ++k) {
        const ChessNode *N = &t.nodes[uni(meta[k]) & 0xFFFFu];  // (the position is in the record already)
        if (p.leaves && lane < 18) ((uint32_t *)&p.leaves[obase + k])[lane] = ((const uint32_t *)&N->st)[lane];
        if (p.planes) {
            const uint32_t pc = N->st.board[lane];
            const char pieces[12] = {'P', 'N', 'B', 'R', 'Q', 'K', 'p', 'n', 'b', 'r', 'q', 'k'};
            int which = -1;
            for (int q = 0; q < 12; ++q)
                if (pc == (uint8_t)pieces[q]) {
                    which = q;
                    break;
                }
            const int turn = N->st.turn, castle = N->st.castle;
            if (p.planes_f16 == 2) {  // ZC_F16_NHWC32: lane = square, its 32 channels (17 planes, zeros)
                typedef _Float16 h8_t __attribute__((ext_vector_type(8)));
                h8_t v8[4];
#pragma unroll
                for (int q = 0; q < 32; ++q) {
                    float v = 0.0f;
                    if (q < 12) v = q == which ? 1.0f : 0.0f;
                    else if (q == 12) v = turn == 0 ? 1.0f : 0.0f;
                    else if (q < 17) v = (castle >> (q - 13)) & 1 ? 1.0f : 0.0f;
                    v8[q >> 3][q & 7] = (_Float16)v;
                }
                h8_t *o = (h8_t *)((_Float16 *)p.planes + ((obase + k) * 64 + lane) * 32);
#pragma unroll
                for (int c = 0; c < 4; ++c) o[c] = v8[c];
            } else {
                for (int q = 0; q < 17; ++q) {
                    float v;
                    if (q < 12) v = q == which ? 1.0f : 0.0f;
                    else if (q == 12) v = turn == 0 ? 1.0f : 0.0f;
                    else v = (castle >> (q - 13)) & 1 ? 1.0f : 0.0f;
                    const size_t o = ((obase + k) * 17 + q) * 64 + lane;
                    if (p.planes_f16) ((__half *)p.planes)[o] = __float2half(v);
                    else ((float *)p.planes)[o] = v;
                }
            }
        }
    }
}

// The deferred expansions of a flush, one wave per (leaf, game) whose walk created a node: its
// legal moves (order, capture values, the check flag of a position without moves: create_node's
// generation) into the per-leaf scratch.
__global__ __launch_bounds__(64) void puct_expand_kernel(ChessParams p) {
    __shared__ CLds L;
    const int j = blockIdx.x, gl = blockIdx.y;
    if (gl >= p.n_games) return;
    const int g = p.first_game + gl;
    const int32_t *ctl = p.ca.ctl + (size_t)g * kCtlWords;
    if (j >= uni(ctl[cNb])) return;
    const uint32_t mt = uni(p.ca.meta[(size_t)g * p.max_batch + j]);
    if (!(mt & kMetaCreated)) return;
    const CTree t = ctree(p, g);
    const uint32_t lane = lane_id();
    const ChessNode *C = &t.nodes[mt & 0xFFFFu];
    if (lane < 18) ((uint32_t *)&L.st)[lane] = ((const uint32_t *)&C->st)[lane];
    wave_sync_mem();
    const NodeGen gen = create_node_gen(L);
    const size_t x = (size_t)g * p.max_batch + j;
    uint16_t *xm = p.ca.xmv + x * ZC_CHESS_MAX_MOVES;
    for (int k = (int)lane; k < gen.n; k += 64) xm[k] = L.s.legal[k];
    if (lane == 0) {
        p.ca.xinfo[2 * x] = gen.n;
        p.ca.xinfo[2 * x + 1] = (int32_t)(((uint32_t)gen.mat & 0xFFFFu) | ((uint32_t)gen.check << 16));
    }
}

// ... and their commit, one wave per (leaf, game) again: the node's slot range is the slots in
// use before the flush plus the move counts of the nodes created before it in this flush
// (create_node_take's arithmetic, capacity included), then create_node_commit's writes.  The
// last created node of the game publishes the new slot count.
__global__ __launch_bounds__(64) void puct_commit_kernel(ChessParams p) {
    const int j = blockIdx.x, gl = blockIdx.y;
    if (gl >= p.n_games) return;
    const int g = p.first_game + gl;
    int32_t *ctl = p.ca.ctl + (size_t)g * kCtlWords;
    const int nb = uni(ctl[cNb]);
    if (j >= nb) return;
    const uint32_t *meta = p.ca.meta + (size_t)g * p.max_batch;
    const uint32_t mt = uni(meta[j]);
    if (!(mt & kMetaCreated)) return;
    const CTree t = ctree(p, g);
    const uint32_t lane = lane_id();
    const size_t x0 = (size_t)g * p.max_batch;
    // the move counts of the nodes created before this one (leaves i < j), and whether a node
    // was created after it (leaves j < i < nb)
    int before = 0;
    bool later = false;
    for (int b = 0; b < nb; b += 64) {
        const int i = b + (int)lane;
        const bool cr = i < nb && (meta[min(i, nb - 1)] & kMetaCreated);
        if (cr && i < j) before += max(p.ca.xinfo[2 * (x0 + i)], 0);
        later |= cr && i > j;
    }
    for (int o = 32; o > 0; o >>= 1) before += __shfl_xor(before, o);
    const bool last = __ballot(later) == 0ull;
    const int slots0 = uni(ctl[cSlots]);
    int n = uni(p.ca.xinfo[2 * (x0 + j)]);
    const uint32_t mc = (uint32_t)uni(p.ca.xinfo[2 * (x0 + j) + 1]);
    const int base = slots0 + before;
    int status = 0;
    if (n < 0) {
        status = ZC_STATUS_CAPACITY;
        n = 0;
    }
    if ((int64_t)base + n > t.S) {
        status = ZC_STATUS_CAPACITY;
        n = 0;
    }
    const uint16_t *xm = p.ca.xmv + (x0 + j) * ZC_CHESS_MAX_MOVES;
    for (int k = (int)lane; k < n; k += 64) {
        t.mv[base + k] = xm[k];
        t.ut[base + k] = (uint8_t)k;
        t.ch[base + k] = 0xFFFF;
        t.na[base + k] = 0;
        t.w[base + k] = 0.0;
    }
    ChessNode *C = &t.nodes[mt & 0xFFFFu];
    if (lane == 0) {
        C->base = (uint32_t)base;
        C->nmoves = (uint16_t)n;
        C->nu = (uint16_t)n;
        C->material = (int16_t)(mc & 0xFFFFu);
        C->check = (mc >> 16) & 1u;
        if (status) ctl[cStatus] = status;
        if (last) ctl[cSlots] = base + n;  // the flush's last created node
    }
}

__global__ __launch_bounds__(64) void puct_backup_kernel(ChessParams p) {
    const int gl = blockIdx.x;
    if (gl >= p.n_games) return;
    const int g = p.first_game + gl;
    const CTree t = ctree(p, g);
    const int32_t *ctl = p.ca.ctl + (size_t)g * kCtlWords;
    const uint32_t lane = lane_id();
    const int nb = uni(ctl[cNb]);
    if (uni(ctl[cStatus]) || nb == 0) return;
    const uint32_t *paths = p.ca.paths + (size_t)g * p.max_batch * kChessPath;
    const uint32_t *meta = p.ca.meta + (size_t)g * p.max_batch;
    const uint2 key = make_uint2((uint32_t)p.seed, (uint32_t)(p.seed >> 32));
    for (int j = 0; j < nb; ++j) {
        const uint32_t mt = uni(meta[j]);
        const int node = (int)(mt & 0xFFFFu), d = (int)((mt >> 16) & 0xFFu);
        ChessNode *N = &t.nodes[node];
        const int nm = uni((int)N->nmoves);
        const size_t li = (size_t)gl * (p.leaf_rows ? p.leaf_rows : p.bs) + j;
        double v;
        if (nm == 0) {
            v = uni((int)N->check) ? -1.0 : 0.0;  // checkmated side to move / no moves
        } else {
            v = __hiloint2double(uni(__double2hiint(p.values[li])), uni(__double2loint(p.values[li])));
            if (!uni((int)N->evaluated)) {
                // priors: softmax of the logits of this node's legal moves (from*64 + to)
                const uint32_t base = uni(N->base);
                float lg[4];
                float mx = -INFINITY;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int k = q * 64 + (int)lane;
                    lg[q] = -INFINITY;
                    if (k < nm) {
                        const uint32_t m = t.mv[base + k];
                        const size_t o = li * 4096 + (m & 63u) * 64 + ((m >> 6) & 63u);
                        lg[q] = p.logits_f16 ? __half2float(((const __half *)p.logits)[o]) : ((const float *)p.logits)[o];
                        mx = fmaxf(mx, lg[q]);
                    }
                }
                mx = wave_max_f(mx);
                float e[4], sum = 0.0f;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    e[q] = q * 64 + (int)lane < nm ? expf(lg[q] - mx) : 0.0f;
                    sum += e[q];
                }
                sum = wave_sum_f(sum);
                float pr[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) pr[q] = e[q] / sum;
                if (node == 0 && p.dir_eps > 0.0f) {
                    // Dirichlet(alpha) noise on the root priors
                    float gm[4], gs = 0.0f;
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int k = q * 64 + (int)lane;
                        gm[q] = k < nm ? gamma_draw(p.dir_alpha, key, (uint32_t)g, (uint32_t)k, search_number(p, gl)) : 0.0f;
                        gs += gm[q];
                    }
                    gs = wave_sum_f(gs);
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        pr[q] = (1.0f - p.dir_eps) * pr[q] + p.dir_eps * (gs > 0.0f ? gm[q] / gs : 0.0f);
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int k = q * 64 + (int)lane;
                    if (k < nm) t.pr[base + k] = pr[q];
                }
                if (lane == 0) N->evaluated = 1;
            }
        }
        wave_sync_mem();
        // backup with the virtual loss undone: W += 1 - r on the edge into level l
        if (lane >= 1 && lane <= (uint32_t)d) {
            const uint32_t s = paths[(size_t)j * kChessPath + lane];
            const double r = ((d - (int)lane) & 1) ? -v : v;
            t.w[s] = t.w[s] + 1.0 - r;
        }
        wave_sync_mem();
    }
}

__global__ __launch_bounds__(64) void puct_end_kernel(ChessParams p) {
    const int gl = blockIdx.x;
    if (gl >= p.n_games) return;
    const int g = p.first_game + gl;
    const CTree t = ctree(p, g);
    const int32_t *ctl = p.ca.ctl + (size_t)g * kCtlWords;
    const uint32_t lane = lane_id();
    const int status = uni(ctl[cStatus]);
    const ChessNode *R = &t.nodes[0];
    const int nm = status == ZC_STATUS_NO_MOVES ? 0 : uni((int)R->nmoves);
    const uint32_t base = uni(R->base);
    for (int j = (int)lane; j < ZC_CHESS_MAX_MOVES; j += 64) {
        p.out_na[(size_t)gl * ZC_CHESS_MAX_MOVES + j] = j < nm ? t.na[base + j] : 0;
        if (p.out_prior) p.out_prior[(size_t)gl * ZC_CHESS_MAX_MOVES + j] = j < nm ? t.pr[base + j] : 0.0f;
    }
    int best = -1;
    if (nm > 0) {
        if (p.temperature <= 0.0f) {  // most visits, first maximum
            int bv = -1, bi = 0x7FFFFFFF;
            for (int b = 0; b < nm; b += 64) {
                const int j = b + (int)lane;
                if (j < nm && t.na[base + j] > bv) {
                    bv = t.na[base + j];
                    bi = j;
                }
            }
            for (int o = 32; o > 0; o >>= 1) {
                const int ov = __shfl_xor(bv, o), oi = __shfl_xor(bi, o);
                if (ov > bv || (ov == bv && oi < bi)) {
                    bv = ov;
                    bi = oi;
                }
            }
            best = uni(bi);
        } else {  // sample proportional to Na^(1/T): inverse CDF over the moves in order
            double tot = 0.0;
            for (int b = 0; b < nm; b += 64) {
                const int j = b + (int)lane;
                tot += j < nm ? pow((double)t.na[base + j], 1.0 / (double)p.temperature) : 0.0;
            }
            tot = wave_sum_d(tot);
            const uint4 r = philox(make_uint4((uint32_t)g, 0x5BE0CD19u, search_number(p, gl), 0),
                                   make_uint2((uint32_t)p.seed, (uint32_t)(p.seed >> 32)));
            const double target = (double)u01(r.x) * tot;
            double run = 0.0;
            best = nm - 1;
            for (int j = 0; j < nm; ++j) {  // serial scan in move order (<= 256 steps, once per move)
                run += pow((double)uni(t.na[base + j]), 1.0 / (double)p.temperature);
                if (run > target) {
                    best = j;
                    break;
                }
            }
        }
    }
    if (lane == 0) {
        if (p.search_no) p.search_no[gl] = (int32_t)(search_number(p, gl) + 1);
        p.out_move[gl] = (best >= 0 && !status) ? t.mv[base + best] : (uint16_t)0xFFFF;
        zc_game_stats st{};
        st.status = status;
        st.expansions = ctl[cExp];
        st.depth_sum = ctl[cDepth];
        st.leaves = p.sims;
        p.out_stats[gl] = st;
    }
}

}  // namespace

void launch_chess_puct_begin(const ChessParams &p, hipStream_t s) {
    hipLaunchKernelGGL(puct_begin_kernel, dim3(p.n_games), dim3(64), 0, s, p);
}
void launch_chess_puct_select(const ChessParams &p, hipStream_t s) {
    hipLaunchKernelGGL(puct_select_kernel, dim3(p.n_games), dim3(64), 0, s, p);
    if (p.flush > 0) {  // flush 0 evaluates the root alone: nothing is created
        hipLaunchKernelGGL(puct_expand_kernel, dim3(p.bs, p.n_games), dim3(64), 0, s, p);
        hipLaunchKernelGGL(puct_commit_kernel, dim3(p.bs, p.n_games), dim3(64), 0, s, p);
    }
}
void launch_chess_puct_backup(const ChessParams &p, hipStream_t s) {
    hipLaunchKernelGGL(puct_backup_kernel, dim3(p.n_games), dim3(64), 0, s, p);
}
void launch_chess_puct_end(const ChessParams &p, hipStream_t s) {
    hipLaunchKernelGGL(puct_end_kernel, dim3(p.n_games), dim3(64), 0, s, p);
}

}  // namespace zc
