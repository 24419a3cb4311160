// c4_ext.hip — stepwise Connect4 search: mcts.get_move (engine/mcts/src/mcts.cpp:102-160)
// with the flush (:112-127) handed to the caller, so any value function — a neural network
// on the same GPU (Value('network_*'), engine/value_functions.py:61-99) or a Python
// Value.batch — evaluates the pending leaves.
//
// Same execution model as the rollout search (one game per wave, c4_device.h), split at the
// flush into launches that keep the game's state in HBM between them:
//   begin  : root record, control words                               (mcts.cpp:104-108)
//   select : nb walks + expansions (select_flush), fresh nodes published, leaves exported
//            as states and as state_to_tensor planes                 (mcts.cpp:129-147)
//   backup : the flush's values applied in pending order, Wa in fp64 (mcts.cpp:80-100,
//            :118-125) — subtractions per edge in exactly the reference's order
//   end    : first max of child N, visits per column, counters       (mcts.cpp:150-157)
#include <hip/hip_fp16.h>

#include "c4_device.h"

namespace zc {
namespace {

__device__ __forceinline__ uint32_t mbcnt_lo(uint64_t m) {  // set bits of m in lanes below this one
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ Tree ext_tree(const ExtParams &p, int g) {
    return Tree{p.a.nodes + (size_t)g * p.M * kRecBytes};
}

__global__ __launch_bounds__(kBlock) void c4_ext_begin_kernel(ExtParams p) {
    const uint32_t lane = lane_id();
    const int gl = blockIdx.x;
    if (gl >= p.n_games) return;
    const int g = p.first_game + gl;
    const zc_c4_state root = p.roots[gl];
    const uint64_t rp0 = uni64(root.stones[0]), rp1 = uni64(root.stones[1]);
    const int rturn = uni(root.turn);
    int status = 0;
    if (!valid_state(rp0, rp1, rturn)) status = ZC_STATUS_BAD_STATE;
    else if (legal_mask(rp0 | rp1) == 0) status = ZC_STATUS_NO_MOVES;
    int32_t *ctl = p.a.ext_ctl + (size_t)g * kCtlWords;
    const uint64_t use0 = p.a.rngpos[2 * (size_t)g];
    if (lane == 0) {
        p.a.ext_roots[g] = root;
        ctl[kCtlNodes] = 1;
        ctl[kCtlF0] = 0;
        ctl[kCtlD0] = 0;
        ctl[kCtlNb] = 0;
        ctl[kCtlStatus] = status;
        ctl[kCtlExp] = 0;
        ctl[kCtlDepth] = 0;
        ctl[kCtlUse0] = (int32_t)(uint32_t)use0;
        ctl[kCtlUse0 + 1] = (int32_t)(uint32_t)(use0 >> 32);
    }
    if (!status) node_init(ext_tree(p, g), 0, 0xFFFF, 0xFF, 0, uni(d_order[legal_mask(rp0 | rp1)]));
}

__global__ __launch_bounds__(kBlock) void c4_ext_select_kernel(ExtParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t s_dyn[];
    uint32_t *const s_order = (uint32_t *)s_dyn;
    Fresh *const fresh = (Fresh *)(s_dyn + kTabBytes);
    Leaf *const leaves = (Leaf *)(s_dyn + kTabBytes + sizeof(Fresh) * (size_t)p.bs);
    uint16_t *const paths = (uint16_t *)(s_dyn + kTabBytes + (sizeof(Fresh) + sizeof(Leaf)) * (size_t)p.bs);
    load_tables(s_order);
    __syncthreads();
    ConstDouble *logtab = (ConstDouble *)p.a.logtab;

    const uint32_t lane = lane_id();
    const int gl = blockIdx.x;
    if (gl >= p.n_games) return;
    const int g = p.first_game + gl;
    const Arena &a = p.a;
    int32_t *ctl = a.ext_ctl + (size_t)g * kCtlWords;
    int status = uni(ctl[kCtlStatus]);
    if (status) {
        if (lane == 0) {
            ctl[kCtlNb] = 0;
            if (p.counts) p.counts[gl] = 0;
        }
        return;
    }
    const Tree t = ext_tree(p, g);
    const int done = p.flush * p.bs;
    const int nb = min(p.bs, p.sims - done);
    int nnodes = uni(ctl[kCtlNodes]);

    Rng rng;
    const uint64_t use_now = uni64(a.rngpos[2 * (size_t)g]);
    rng_open(rng, a.ring + (size_t)g * kRingWords, use_now, uni64(a.rngpos[2 * (size_t)g + 1]));
    Counters cn;
    Stamp<false> stamp;
    FlushSel fs;
    const zc_c4_state root = a.ext_roots[g];
    select_flush<true, false>(t, fresh, leaves, paths, s_order, logtab, rng, cn, stamp, nnodes, status,
                              uni64(root.stones[0]), uni64(root.stones[1]), uni(root.turn), done, nb, p.c, fs);
    const int f0 = fs.f0;

    // publish: X0's untried word and children, then every fresh node (Na = 0, Wa = 0.0)
    if (fs.x0_dirty) {
        if (lane == 0) t.hdr(fs.x0node)[1] = fs.x_u;
        if (lane < kSlots) t.child(fs.x0node)[lane] = (uint16_t)fs.x_ch;
    }
    const int nf = nnodes - f0;
    for (int idx = (int)lane; idx < nf * 8; idx += 64) {
        const int r = idx >> 3, slot = idx & 7;
        const Fresh &F = fresh[r];
        uint8_t *R = t.rec(f0 + r);
        if (slot == 0) *(uint4 *)R = make_uint4(0u, F.u, F.link, F.ow);
        ((uint16_t *)(R + 16))[slot] = F.ch[slot];
        ((int32_t *)(R + 32))[slot] = 0;
        ((double *)(R + 64))[slot] = 0.0;
    }

    // the pending flush: leaf records for backup, states and planes for the caller
    const size_t lbase = (size_t)g * p.max_batch;
    const size_t obase = (size_t)gl * p.bs;
    for (int j = (int)lane; j < nb; j += 64) {
        const Leaf L = leaves[j];
        a.ext_meta[lbase + j] = L.meta;
        if (p.leaves) {
            zc_c4_state s;
            s.stones[0] = L.p0;
            s.stones[1] = L.p1;
            s.turn = (int32_t)((L.meta >> 24) & 1u);
            s.reserved = 0;
            p.leaves[obase + j] = s;
        }
    }
    for (int idx = (int)lane; idx < nb * kMaxDepth; idx += 64)
        a.ext_paths[lbase * kMaxDepth + idx] = paths[idx];
    if (p.planes) {
        // c4_backend.state_to_tensor (c4_backend.py:52-61): [2][6][7], plane 0 = stones of the
        // side to move, plane 1 = the opponent's; row 0 = top (bit row 5 - r)
        for (int idx = (int)lane; idx < nb * 84; idx += 64) {
            const int j = idx / 84, e = idx - j * 84;
            const int pl = e / 42, cell = e - pl * 42;
            const int r = cell / 7, col = cell - r * 7;
            const Leaf &L = leaves[j];
            const int tn = (int)((L.meta >> 24) & 1u);
            const uint64_t stones = (pl == tn) ? L.p0 : L.p1;  // pl 0 & turn 0 -> X, ...
            const float v = (float)((stones >> (7 * col + 5 - r)) & 1ull);
            const size_t o = (obase + j) * 84 + e;
            if (p.planes_f16) ((__half *)p.planes)[o] = __float2half(v);
            else ((float *)p.planes)[o] = v;
        }
    }
    wave_mem_order();
    if (lane == 0) {
        ctl[kCtlNodes] = nnodes;
        ctl[kCtlF0] = f0;
        ctl[kCtlD0] = fs.d0;
        ctl[kCtlNb] = nb;
        ctl[kCtlStatus] = status;
        ctl[kCtlExp] += cn.expansions;
        ctl[kCtlDepth] += cn.depth_sum;
        if (p.counts) p.counts[gl] = nb;
        rng_close(rng, use_now, a.rngpos + 2 * (size_t)g);
    }
    if (lane <= (uint32_t)fs.d0) ctl[kCtlPath + lane] = (int32_t)fs.ppath;
}

__global__ __launch_bounds__(kBlock) void c4_ext_backup_kernel(ExtParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t s_dyn[];
    double *const fw = (double *)s_dyn;             // [bs] Wa of each fresh node's in-edge
    int32_t *const fna = (int32_t *)(fw + p.bs);    // [bs] Na
    const uint32_t lane = lane_id();
    const int gl = blockIdx.x;
    if (gl >= p.n_games) return;
    const int g = p.first_game + gl;
    const Arena &a = p.a;
    const int32_t *ctl = a.ext_ctl + (size_t)g * kCtlWords;
    const int status = uni(ctl[kCtlStatus]);
    const int nb = uni(ctl[kCtlNb]);
    if (status || nb == 0) return;
    const Tree t = ext_tree(p, g);
    const int f0 = uni(ctl[kCtlF0]), d0 = uni(ctl[kCtlD0]), nf = uni(ctl[kCtlNodes]) - f0;
    for (int i = (int)lane; i < nf; i += 64) {
        fw[i] = 0.0;
        fna[i] = 0;
    }
    // lane l in 1..d0 owns the prefix edge into level l (shared by every leaf of the flush)
    const bool pre = lane >= 1 && lane <= (uint32_t)d0;
    int par = 0, act = 0;
    int32_t na = 0;
    double w = 0.0;
    if (pre) {
        par = ctl[kCtlPath + lane - 1] & 0xFFFF;
        act = (int)((uint32_t)ctl[kCtlPath + lane] >> 16);
        na = t.na(par)[act];
        w = t.q(par)[act];
    }
    wave_mem_order();
    const size_t lbase = (size_t)g * p.max_batch;
    const double *vals = p.values + (size_t)gl * p.bs;
    for (int j = 0; j < nb; ++j) {
        const uint32_t meta = uni(a.ext_meta[lbase + j]);
        const int d = (int)((meta >> 16) & 0xFFu);
        const double v = __hiloint2double(uni(__double2hiint(vals[j])), uni(__double2loint(vals[j])));
        if (lane >= 1 && lane <= (uint32_t)d) {
            // backprop (mcts.cpp:86-96): the edge into level l gets Wa -= (-1)^(d-l) * v
            const double r = ((d - (int)lane) & 1) ? -v : v;
            if (lane <= (uint32_t)d0) {
                w -= r;
                na += 1;
            } else {
                const int fi = (int)a.ext_paths[(lbase + j) * kMaxDepth + lane] - f0;
                fw[fi] -= r;
                fna[fi] += 1;
            }
        }
    }
    wave_mem_order();
    if (pre) {
        t.na(par)[act] = na;
        t.q(par)[act] = w;
    }
    for (int i = (int)lane; i < nf; i += 64) {
        const uint32_t link = t.hdr(f0 + i)[2];
        const int fp = (int)(link & 0xFFFFu), fa = (int)((link >> 16) & 0xFFu);
        t.na(fp)[fa] = fna[i];
        t.q(fp)[fa] = fw[i];
    }
}

__global__ __launch_bounds__(kBlock) void c4_ext_end_kernel(ExtParams p) {
    const uint32_t lane = lane_id();
    const uint32_t k = lane & 7u;
    const int gl = blockIdx.x;
    if (gl >= p.n_games) return;
    const int g = p.first_game + gl;
    const Arena &a = p.a;
    const int32_t *ctl = a.ext_ctl + (size_t)g * kCtlWords;
    const int status = uni(ctl[kCtlStatus]);
    zc_game_stats st{};
    st.status = status;
    if (status == ZC_STATUS_NO_MOVES || status == ZC_STATUS_BAD_STATE) {
        if (lane == 0) {
            p.out_stats[gl] = st;
            p.out_move[gl] = -1;
        }
        if (lane < 7) p.out_na[(size_t)gl * 7 + lane] = 0;
        return;
    }
    const Tree t = ext_tree(p, g);
    const uint32_t u = uni(t.hdr(0)[1]);
    const uint32_t ow = uni(t.hdr(0)[3]);
    const uint32_t nm = u >> 28;
    int bv = (k < nm) ? t.na(0)[k] : -1;
    int bi = (int)k;
    argmax8(bv, bi);
    const int best = uni(bi);
    if (lane < 7) {
        int pos = -1;
        for (uint32_t s = 0; s < nm; ++s)
            if (((ow >> (3 * s)) & 7u) == lane) pos = (int)s;
        p.out_na[(size_t)gl * 7 + lane] = pos >= 0 ? t.na(0)[pos] : 0;
    }
    if (lane == 0) {
        p.out_move[gl] = (int)((ow >> (3 * best)) & 7u);
        const uint64_t use0 = (uint64_t)(uint32_t)ctl[kCtlUse0] | ((uint64_t)(uint32_t)ctl[kCtlUse0 + 1] << 32);
        st.expansions = ctl[kCtlExp];
        st.depth_sum = ctl[kCtlDepth];
        st.leaves = p.sims;
        st.rng_words = (int64_t)(a.rngpos[2 * (size_t)g] - use0);
        p.out_stats[gl] = st;
    }
}

// ---- host-policy search (zc_c4_hp_*, the §8(b) fallback for any policy callable) --------
// One game, one simulation at a time: walk (select over the HBM tree, fresh children of the
// pending flush included — their edges have Na = 0, so UCT takes them first exactly as in
// mcts.cpp:41-45), the caller's policy picks among the untried moves, expand.  The pending
// flush is kept in the stepwise search's format (ctl F0 / D0 / path, ext_paths, ext_meta),
// so zc_c4_ext_backup applies it.
__global__ __launch_bounds__(kBlock) void c4_hp_walk_kernel(ExtParams p) {
    const uint32_t lane = lane_id();
    const int g = p.first_game;
    const Arena &a = p.a;
    int32_t *ctl = a.ext_ctl + (size_t)g * kCtlWords;
    int status = uni(ctl[kCtlStatus]);
    zc_c4_hp_node *out = p.hp_node;
    if (status) {
        if (lane == 0) {
            out->node = -1;
            out->n_untried = 0;
            out->depth = 0;
        }
        return;
    }
    const Tree t = ext_tree(p, g);
    const zc_c4_state root = a.ext_roots[g];
    const WalkEnd we = walk_hbm<true>(t, (ConstDouble *)a.logtab, uni64(root.stones[0]), uni64(root.stones[1]),
                                      uni(root.turn), p.flush * p.bs, p.c, status);
    const size_t lbase = (size_t)g * p.max_batch;
    if (lane <= (uint32_t)we.depth) a.ext_paths[(lbase + p.hp_leaf) * kMaxDepth + lane] = (uint16_t)we.pathv;
    if (p.hp_leaf == 0) {  // the flush's X0: its prefix path is every leaf's (backup)
        if (lane <= (uint32_t)we.depth) ctl[kCtlPath + lane] = (int32_t)we.pathv;
        if (lane == 0) {
            ctl[kCtlD0] = we.depth;
            ctl[kCtlF0] = ctl[kCtlNodes];
        }
    }
    const uint32_t cnt = status ? 0u : untried_count(we.u);
    // the untried moves' columns in list order: bit l of the untried word is move l
    const bool in = lane < 7 && ((we.u >> lane) & 1u);
    const uint32_t rank = mbcnt_lo(__ballot(in));
    if (in) out->untried[rank] = (int32_t)((we.ow >> (3 * lane)) & 7u);
    if (lane < 7 && lane >= cnt) out->untried[lane] = -1;
    if (lane == 0) {
        out->state.stones[0] = we.b0;
        out->state.stones[1] = we.b1;
        out->state.turn = we.turn;
        out->state.reserved = 0;
        out->node = we.node;
        out->n_untried = (int32_t)cnt;
        out->depth = we.depth;
        ctl[kCtlHpNode] = we.node;
        ctl[kCtlHpNode + 1] = we.depth | (we.turn << 8);
        ctl[kCtlHpNode + 2] = (int32_t)(uint32_t)we.b0;
        ctl[kCtlHpNode + 3] = (int32_t)(uint32_t)(we.b0 >> 32);
        ctl[kCtlHpNode + 4] = (int32_t)(uint32_t)we.b1;
        ctl[kCtlHpNode + 5] = (int32_t)(uint32_t)(we.b1 >> 32);
        ctl[kCtlStatus] = status;
    }
}

__global__ __launch_bounds__(kBlock) void c4_hp_expand_kernel(ExtParams p) {
    const uint32_t lane = lane_id();
    const int g = p.first_game;
    const Arena &a = p.a;
    int32_t *ctl = a.ext_ctl + (size_t)g * kCtlWords;
    if (uni(ctl[kCtlStatus])) return;
    const Tree t = ext_tree(p, g);
    const int node = uni(ctl[kCtlHpNode]);
    const int dt = uni(ctl[kCtlHpNode + 1]);
    const int depth = dt & 0xFF, turn = (dt >> 8) & 1;
    const uint64_t b0 = (uint64_t)(uint32_t)uni(ctl[kCtlHpNode + 2]) | ((uint64_t)(uint32_t)uni(ctl[kCtlHpNode + 3]) << 32);
    const uint64_t b1 = (uint64_t)(uint32_t)uni(ctl[kCtlHpNode + 4]) | ((uint64_t)(uint32_t)uni(ctl[kCtlHpNode + 5]) << 32);
    const uint32_t u = uni(t.hdr(node)[1]);
    const uint32_t ow = uni(t.hdr(node)[3]);
    const uint32_t cnt = untried_count(u);
    int nnodes = uni(ctl[kCtlNodes]);
    int leaf = node, ldepth = depth, lturn = turn;
    uint64_t l0 = b0, l1 = b1;
    if (cnt) {
        if (p.hp_index < 0 || p.hp_index >= (int)cnt) {
            if (lane == 0) ctl[kCtlStatus] = ZC_STATUS_INTERNAL;
            return;
        }
        // expand (mcts.cpp:65-78): the hp_index-th untried move in list order
        const bool in = lane < 7 && ((u >> lane) & 1u);
        const uint32_t rank = mbcnt_lo(__ballot(in));
        const int mi = __builtin_ctzll(__ballot(in && rank == (uint32_t)p.hp_index));
        const int col = (int)((ow >> (3 * mi)) & 7u);
        const uint64_t bit = drop_bit(b0 | b1, col);
        if (turn) l1 |= bit; else l0 |= bit;
        lturn = turn ^ 1;
        ldepth = depth + 1;
        leaf = nnodes++;
        node_init(t, leaf, node, mi, ldepth, uni(d_order[legal_mask(l0 | l1)]));
        if (lane == 0) {
            t.hdr(node)[1] = u & ~(1u << mi);
            t.child(node)[mi] = (uint16_t)leaf;
            a.ext_paths[((size_t)g * p.max_batch + p.hp_leaf) * kMaxDepth + ldepth] = (uint16_t)leaf;
            ctl[kCtlExp] += 1;
            ctl[kCtlDepth] += ldepth;
        }
    }
    if (lane == 0) {
        const uint32_t lmask = (uint32_t)legal_mask(l0 | l1);
        a.ext_meta[(size_t)g * p.max_batch + p.hp_leaf] =
            (uint32_t)leaf | ((uint32_t)ldepth << 16) | ((uint32_t)lturn << 24) | (lmask << 25);
        if (p.leaves) {
            zc_c4_state s;
            s.stones[0] = l0;
            s.stones[1] = l1;
            s.turn = lturn;
            s.reserved = 0;
            p.leaves[0] = s;
        }
        ctl[kCtlNodes] = nnodes;
        ctl[kCtlNb] = p.hp_leaf + 1;
    }
}

}  // namespace

void launch_c4_hp_walk(const ExtParams &p, hipStream_t s) {
    hipLaunchKernelGGL(c4_hp_walk_kernel, dim3(1), dim3(kBlock), 0, s, p);
}

void launch_c4_hp_expand(const ExtParams &p, hipStream_t s) {
    hipLaunchKernelGGL(c4_hp_expand_kernel, dim3(1), dim3(kBlock), 0, s, p);
}

void launch_c4_ext_begin(const ExtParams &p, hipStream_t s) {
    hipLaunchKernelGGL(c4_ext_begin_kernel, dim3(p.n_games), dim3(kBlock), 0, s, p);
}

void launch_c4_ext_select(const ExtParams &p, hipStream_t s) {
    hipLaunchKernelGGL(c4_ext_select_kernel, dim3(p.n_games), dim3(kBlock), c4_search_lds_bytes(p.bs), s, p);
}

void launch_c4_ext_backup(const ExtParams &p, hipStream_t s) {
    const size_t lds = (sizeof(double) + sizeof(int32_t)) * (size_t)p.bs;
    hipLaunchKernelGGL(c4_ext_backup_kernel, dim3(p.n_games), dim3(kBlock), lds, s, p);
}

void launch_c4_ext_end(const ExtParams &p, hipStream_t s) {
    hipLaunchKernelGGL(c4_ext_end_kernel, dim3(p.n_games), dim3(kBlock), 0, s, p);
}

}  // namespace zc
