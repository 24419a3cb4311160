// chess_search.hip — batched chess tree search for gfx950: mcts.get_move
// (engine/mcts/src/mcts.cpp:102-160) with the chess backend (chess.hip rules), Policy('random')
// or Policy('immediate_value') (engine/policy_functions.py:10-20) on each game's CPython
// MT19937 stream, and either Value('crude_chess_score') evaluated in the kernel
// (engine/value_functions.py:48-55; configs/crude_chess.yaml) or values supplied by the
// caller at every flush (the network modes, value_functions.py:61-99; configs/chess_value.yaml).
//
// One game per wave.  The tree lives in HBM (zc_internal.h ChessNode + SoA child slots);
// every node keeps its position, so selection never replays moves.  Lanes take:
//   - the UCT scan: up to 256 child slots, 64 per pass, fp64 fma(c, sqrt(log N / Na), Q)
//     with the reference's first-maximum rule (a butterfly argmax over the wave);
//   - node creation: the legal-move generator of chess_device.h (one square per lane);
//   - the policy's candidate filter and the untried-list erase;
//   - backup: lane l updates the edge into level l of the leaf's path.
// Backups are applied leaf by leaf in pending order, so every Wa receives its fp64
// subtractions in the reference's order.
#include <hip/hip_fp16.h>

#include "chess_tree.h"

namespace zc {
namespace {

// Where the previous simulation of the same flush stopped.  No backup happens inside a
// flush, so every decision above that node is unchanged and the next walk from the root
// would arrive there again: it resumes there (the C4 search's flush structure,
// c4_device.h::select_flush).  Below it every child created in this flush has Na == 0
// (+inf), so the resumed walk takes first-unvisited slots, as the full walk would.
// While that node still has untried moves (and at most 64), the next walk stops there again
// and expands it: its untried list, moves and position stay in registers (`cached`), so
// the simulation reads nothing of it from memory.
struct Resume {
    int node = 0, depth = 0, nN = 0;
    uint32_t pathv = 0;
    bool valid = false;
    bool cached = false;
    int nu = 0, utv = 0;        // untried count; lane i: untried entry i
    uint32_t base = 0, mvv = 0;  // first slot; lane i: the move of untried entry i
    uint32_t stw = 0;            // lanes 0..17: the node's position (zc_chess_state words)
};

// select (mcts.cpp:47-63) from `node` down: the UCT child (first maximum, +inf for an
// unvisited edge) until a node with untried moves or without moves; lane l of pathv gets the
// slot of the edge into level l.
__device__ __forceinline__ void chess_walk(const ChessParams &p, const CTree &t, ConstDouble *logtab, int &node,
                                           int &depth, int &nN, uint32_t &pathv, int &status) {
    const uint32_t lane = lane_id();
    for (;;) {  // select (mcts.cpp:47-63)
        const ChessNode *N = &t.nodes[node];
        const uint32_t base = uni(N->base);
        const int nm = uni((int)N->nmoves), nu = uni((int)N->nu);
        if (nu > 0 || nm == 0) break;
        if (depth >= kChessPath - 2) {
            status = ZC_STATUS_CAPACITY;
            break;
        }
        const double lg = logtab[nN];
        int first_unv = 0x7FFFFFFF;
        double bv = -INFINITY;
        int bi = 0x7FFFFFFF;
        int chv = 0xFFFF, nav = 0;  // this lane's slot of the last pass (nm <= 64: the only one)
        for (int b = 0; b < nm; b += 64) {
            const int j = b + (int)lane;
            bool valid = false;
            int32_t na = 0;
            double w = 0.0;
            if (j < nm) {
                chv = t.ch[base + j];
                valid = chv != 0xFFFF;
                na = t.na[base + j];
                w = t.w[base + j];
            }
            nav = na;
            const uint64_t unv = __ballot(valid && na == 0);
            if (unv && first_unv == 0x7FFFFFFF) first_unv = b + __builtin_ctzll(unv);
            if (valid && na > 0) {
                // UCT (mcts.cpp:41-45): fma(c, sqrt(log(N)/Na), Qa), Qa = Wa / Na (:95)
                const double v = fma(p.c, sqrt(lg / (double)na), w / (double)na);
                if (v > bv) {
                    bv = v;
                    bi = j;
                }
            }
        }
        int best;
        if (first_unv != 0x7FFFFFFF) {
            best = first_unv;
        } else {
            argmax64(bv, bi);
            if (bi == 0x7FFFFFFF) break;  // no child at all (cannot happen with nu == 0, nm > 0)
            best = uni(bi);
        }
        int nxt;
        if (nm <= 64) {  // the chosen slot is still in a lane's registers
            nxt = __builtin_amdgcn_readlane(chv, best);
            nN = __builtin_amdgcn_readlane(nav, best);
        } else {
            nxt = uni((int)t.ch[base + best]);
            nN = uni(t.na[base + best]);
        }
        ++depth;
        if (lane == (uint32_t)depth) pathv = base + (uint32_t)best;
        node = nxt;
    }
}

// One simulation's decision (mcts.cpp:129-147) before its child exists: the walk (or the
// resumed one), and when the node it stops at has untried moves, the policy's pick among them
// and the untried list's erase.  midx < 0: no expansion (the leaf is `node` itself).
struct Expansion {
    int node;        // the expanded node X (or the leaf, midx < 0)
    int depth;       // its depth
    uint32_t pathv;  // lane l: the slot of the edge into level l of X's path
    int midx;        // the expanded slot of X, or -1
    uint32_t m;      // its move
    uint32_t stw;    // lanes 0..17: X's position (zc_chess_state words)
    uint32_t base;   // X's first slot
};

#ifndef ZC_CHESS_LAZY
#define ZC_CHESS_LAZY 1  // 1: crude-search nodes are created with a legal-move probe only (A/B: 0)
#endif

// The first expansion of a lazy node (created by create_child_gen<true>): its position into
// L.st, the full get_legal_moves, and the node's move list committed as create_node_commit
// would have at its creation (slots taken now, all moves untried, no children).  Returns the
// list's length (nu == nmoves from here on) and its first slot in `base`.
__device__ __forceinline__ int generate_lazy(const CTree &t, CLds &L, ChessNode *N, int &slots, int &status,
                                             uint32_t &base) {
    const uint32_t lane = lane_id();
    if (lane < 18) ((uint32_t *)&L.st)[lane] = ((const uint32_t *)&N->st)[lane];
    wave_sync_mem();
    const NodeGen gen = create_node_gen(L);
    const int b = slots;
    const int n = create_node_take(t, gen, slots, status);
    for (int j = (int)lane; j < n; j += 64) {
        t.mv[b + j] = L.s.legal[j];
        t.ut[b + j] = (uint8_t)j;
        t.ch[b + j] = 0xFFFF;
        t.na[b + j] = 0;
        t.w[b + j] = 0.0;
    }
    if (lane == 0) {
        N->base = (uint32_t)b;
        N->nmoves = (uint16_t)n;
        N->nu = (uint16_t)n;
    }
    wave_sync_mem();
    base = (uint32_t)b;
    return n;
}

__device__ __forceinline__ Expansion sim_front(const ChessParams &p, const CTree &t, ConstDouble *logtab, Rng &rng, int done,
                               int &status, Resume &rs, CLds &L, int &slots) {
    const uint32_t lane = lane_id();
    int node = 0, depth = 0, nN = done;
    uint32_t pathv = 0;
    if (rs.valid) {
        node = rs.node;
        depth = rs.depth;
        nN = rs.nN;
        pathv = rs.pathv;
    }
    CSTAMP_T(cs0);
    if (!rs.cached) chess_walk(p, t, logtab, node, depth, nN, pathv, status);
    CSTAMP_ADD(0, cs0);
    CSTAMP_T(cs1);
    ChessNode *N = &t.nodes[node];
    const bool hit = rs.cached;
    int nu = hit ? rs.nu : uni((int)N->nu);
    uint32_t lazy_base = 0;
    bool lazy_gen = false;
    if (ZC_CHESS_LAZY && !hit && nu > 0 && !status && uni((int)N->nmoves) == (int)kChessLazy) {
        nu = generate_lazy(t, L, N, slots, status, lazy_base);
        lazy_gen = true;
    }
    if (hit) CSTAMP_COUNT(20);
    if (!hit) CSTAMP_ADD(17, cs1);
    CSTAMP_T(cs18);
    rs.node = node;
    rs.depth = depth;
    rs.nN = nN;
    rs.pathv = pathv;
    rs.valid = true;
    rs.cached = false;
    if (nu == 0 || status) return Expansion{node, depth, pathv, -1, 0u, 0u, 0u};

    // expand (mcts.cpp:65-78): the policy picks among the untried moves, in untried order.
    // The node's position is fetched now, under the policy's memory traffic.
    uint32_t stw = rs.stw;
    if (!hit) {
        stw = lane < 18 ? ((const uint32_t *)&N->st)[lane] : 0u;
        vmem_ready(stw);
    }
    const uint32_t base = hit ? rs.base : lazy_gen ? lazy_base : uni(N->base);
    int local, midx;
    uint32_t m;
    if (nu <= 64) {
        // untried entry and move of lane i, read once: the policy, the erase and the chosen
        // move all come out of these registers
        int utv;
        uint32_t mvv;
        if (hit) {
            utv = rs.utv;
            mvv = rs.mvv;
        } else {
            utv = lane < (uint32_t)nu ? (int)t.ut[base + lane] : 0;
            mvv = lane < (uint32_t)nu ? (uint32_t)t.mv[base + utv] : 0u;
            vmem_ready(mvv);
            CSTAMP_ADD(18, cs18);
        }
        CSTAMP_T(cs19);
        CSTAMP_T(cs22);
        if (p.policy == 1) {
            // Policy('immediate_value') (policy_functions.py:14-17): random.choice over the
            // untried moves whose capture value >= max - policy_freedom
            // the maximum capture value (4 bits) of the untried moves, bit by bit from the top
            // with ballots instead of a cross-lane shuffle reduction (nu >= 1 here)
            // A capture value is one of 0, 1, 3, 5, 9 (chess_device.h capval): one ballot per
            // value, all independent, give the maximum and the candidates at once (ok: the
            // classes that pass `value >= max - freedom` for each maximum, ChessParams::cls_ok)
            const uint32_t cv = mvv >> 12;
            const bool in = lane < (uint32_t)nu;
            const uint64_t B1 = __ballot(in && cv == 1u), B3 = __ballot(in && cv == 3u);
            const uint64_t B5 = __ballot(in && cv == 5u), B9 = __ballot(in && cv == 9u);
            const uint64_t B0 = __ballot(in) & ~(B1 | B3 | B5 | B9);
            const int top = B9 ? 4 : B5 ? 3 : B3 ? 2 : B1 ? 1 : 0;
            const uint32_t ok = (p.cls_ok >> (5 * top)) & 31u;
            const uint64_t cm = ((ok & 1u) ? B0 : 0ull) | ((ok & 2u) ? B1 : 0ull) | ((ok & 4u) ? B3 : 0ull) |
                                ((ok & 8u) ? B5 : 0ull) | ((ok & 16u) ? B9 : 0ull);
            const uint32_t r = rng_below(rng, (uint32_t)__popcll(cm));
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(cm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)cm, 0u));
            local = __builtin_ctzll(__ballot(((cm >> lane) & 1ull) && rank == r));
        } else {
            local = (int)rng_below(rng, (uint32_t)nu);  // Policy('random'): random.choice(untried)
        }
        if (hit) CSTAMP_ADD(22, cs22);
        CSTAMP_T(cs23);
        midx = __builtin_amdgcn_readlane(utv, local);
        m = (uint32_t)__builtin_amdgcn_readlane((int)mvv, local);
        // untried.erase(begin + local): entry i takes entry i + 1
        const int nxt = dpp<0x130>(utv);  // wave_shl:1, lane l reads lane l + 1
        const uint32_t nmv = (uint32_t)dpp<0x130>((int)mvv);
        const bool moved = (int)lane >= local;
        if (moved && (int)lane < nu - 1) t.ut[base + lane] = (uint8_t)nxt;
        rs.cached = nu > 1;  // the next walk stops here again
        rs.nu = nu - 1;
        rs.utv = moved ? nxt : utv;
        rs.mvv = moved ? nmv : mvv;
        rs.base = base;
        rs.stw = stw;
        if (!hit) CSTAMP_ADD(19, cs19);
        if (hit) CSTAMP_ADD(23, cs23);
    } else {
        if (p.policy == 1) {
            int best = -1;
            for (int b = 0; b < nu; b += 64) {
                const int i = b + (int)lane;
                int v = -1;
                if (i < nu) v = (int)(t.mv[base + t.ut[base + i]] >> 12);
                for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
                best = max(best, v);
            }
            const double thr = (double)best - p.freedom;
            auto cand = [&](int i) { return (double)(t.mv[base + t.ut[base + i]] >> 12) >= thr; };
            uint32_t k = 0;
            for (int b = 0; b < nu; b += 64) {
                const int i = b + (int)lane;
                k += (uint32_t)__popcll(__ballot(i < nu && cand(i)));
            }
            const uint32_t r = rng_below(rng, k);
            local = nth_true(nu, r, cand);
        } else {
            local = (int)rng_below(rng, (uint32_t)nu);
        }
        midx = uni((int)t.ut[base + local]);
        // untried.erase(begin + local): shift the tail down, 64 entries per pass (each pass
        // reads entries the previous pass has not overwritten)
        for (int b = local; b < nu - 1; b += 64) {
            const int i = b + (int)lane;
            uint8_t v = 0;
            if (i < nu - 1) v = t.ut[base + i + 1];
            wave_sync_mem();
            if (i < nu - 1) t.ut[base + i] = v;
        }
        m = uni((uint32_t)t.mv[base + midx]);
    }
    if (lane == 0) N->nu = (uint16_t)(nu - 1);
    CSTAMP_ADD(1, cs1);
    if (hit) CSTAMP_ADD(16, cs1);
    return Expansion{node, depth, pathv, midx, m, stw, base};
}

// The hand-off between a search workgroup's leader wave and its helper wave (LDS): when two
// consecutive simulations of a flush expand the same node (the cached case: no backup inside a
// flush, so the second walk stops where the first did), the leader posts the second child's
// parent position and move; the helper plays the move and generates the child's legal moves
// while the leader does the same for the first child.  The leader then commits both children
// in simulation order (node ids, slots), so the tree, the stream and every output are those of
// the one-wave search.  The hand-offs are plain LDS accesses ordered by the barriers (a volatile
// one is a flat store whose wait drains all the wave's global stores).  Letting the helper also
// write the second child, with a join before every walk, measured within 1 % of this
// (profiles/r05_ab_chess_variants.log): the two waves are about balanced.
struct Helper {
    CLds L;
    NodeGen gen;
    int cmd;           // 1: generate; 2: exit
    uint32_t stw[18];  // the parent's position (zc_chess_state words) ...
    uint32_t m;        // ... and the move to play
};

__device__ void helper_loop(Helper &h) {
    const uint32_t lane = lane_id();
    for (;;) {
        __syncthreads();  // a command is posted
        if (uni(h.cmd) != 1) return;  // plain LDS accesses: the barriers order them
        const uint32_t stw = lane < 18 ? h.stw[lane] : 0u;
        const NodeGen gen = create_child_gen<ZC_CHESS_LAZY != 0>(h.L, stw, uni(h.m));
        if (lane == 0) h.gen = gen;
        __syncthreads();  // the generated child is in h
    }
}

__device__ __forceinline__ void helper_exit(Helper *h) {
    if (!h) return;
    if (lane_id() == 0) h->cmd = 2;
    __syncthreads();
}

// The child of expansion e in L (generated: gen), committed as node `child` (mcts.cpp:74-76).
__device__ __forceinline__ void commit_child(const CTree &t, const CLds &L, NodeGen gen, const Expansion &e, int child,
                                             int &slots, int &status, Counters &cn) {
    create_node_commit(t, L, gen, child, e.node, e.midx, e.depth + 1, slots, status);
    if (lane_id() == 0) t.ch[e.base + (uint32_t)e.midx] = (uint16_t)child;
    cn.add(cn.expansions, 1);
    cn.add(cn.depth_sum, e.depth + 1);
    wave_sync_mem();
}

__device__ __forceinline__ void root_init(const ChessParams &p, const CTree &t, CLds &L, int gl, int g, int32_t *ctl) {
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
    const uint64_t use0 = p.a.rngpos[2 * (size_t)g];
    if (lane == 0) {
        ctl[cNodes] = 1;
        ctl[cSlots] = slots;
        ctl[cStatus] = status;
        ctl[cNb] = 0;
        ctl[cExp] = 0;
        ctl[cDepth] = 0;
        ctl[cUse0] = (int32_t)(uint32_t)use0;
        ctl[cUse0 + 1] = (int32_t)(uint32_t)(use0 >> 32);
    }
    wave_sync_mem();
}

// first max of child N over the root's moves (mcts.cpp:150-155): the slot index, or
// 0x7FFFFFFF when the root has no child
__device__ __forceinline__ int best_root_slot(const CTree &t, int nm, uint32_t base) {
    const uint32_t lane = lane_id();
    int bv = -1, bi = 0x7FFFFFFF;
    for (int b = 0; b < nm; b += 64) {
        const int j = b + (int)lane;
        if (j < nm && t.ch[base + j] != 0xFFFF) {
            const int na = t.na[base + j];
            if (na > bv) {
                bv = na;
                bi = j;
            }
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const int ov = __shfl_xor(bv, o), oi = __shfl_xor(bi, o);
        if (ov > bv || (ov == bv && oi < bi)) {
            bv = ov;
            bi = oi;
        }
    }
    return uni(bi);
}

__device__ __forceinline__ void finish(const ChessParams &p, const CTree &t, int gl, int g, const int32_t *ctl) {
    const uint32_t lane = lane_id();
    const int status = uni(ctl[cStatus]);
    const ChessNode *R = &t.nodes[0];
    const int nm = status == ZC_STATUS_NO_MOVES ? 0 : uni((int)R->nmoves);
    const uint32_t base = uni(R->base);
    const int bi = best_root_slot(t, nm, base);
    for (int j = (int)lane; j < ZC_CHESS_MAX_MOVES; j += 64)
        p.out_na[(size_t)gl * ZC_CHESS_MAX_MOVES + j] = j < nm ? t.na[base + j] : 0;
    if (lane == 0) {
        p.out_move[gl] = (bi != 0x7FFFFFFF && !status) ? t.mv[base + bi] : (uint16_t)0xFFFF;
        zc_game_stats st{};
        st.status = status;
        st.expansions = ctl[cExp];
        st.depth_sum = ctl[cDepth];
        st.leaves = p.sims;
        const uint64_t use0 = (uint64_t)(uint32_t)ctl[cUse0] | ((uint64_t)(uint32_t)ctl[cUse0 + 1] << 32);
        st.rng_words = (int64_t)(p.a.rngpos[2 * (size_t)g] - use0);
        p.out_stats[gl] = st;
    }
}

// select + expand of one flush; leaf records to the arena (meta, paths).  Returns nb.
// With a helper wave (h != nullptr), two consecutive expansions of the same node generate their
// children's legal moves in parallel (Helper).
__device__ __forceinline__ int chess_select_flush(const ChessParams &p, const CTree &t, CLds &L, ConstDouble *logtab, int g, int32_t *ctl,
                            int done, int nb, Helper *h = nullptr) {
    const uint32_t lane = lane_id();
    int nnodes = uni(ctl[cNodes]), slots = uni(ctl[cSlots]), status = uni(ctl[cStatus]);
    Rng rng;
    const uint64_t use_now = uni64(p.a.rngpos[2 * (size_t)g]);
    rng_open(rng, p.a.ring + (size_t)g * kRingWords, use_now, uni64(p.a.rngpos[2 * (size_t)g + 1]));
    Counters cn;
    uint32_t *paths = p.ca.paths + (size_t)g * p.max_batch * kChessPath;
    uint32_t *meta = p.ca.meta + (size_t)g * p.max_batch;
    int j = 0;
    Resume rs;
    auto record = [&](int leaf, int d, uint32_t pathv) {
        if (lane < (uint32_t)kChessPath) paths[(size_t)j * kChessPath + lane] = pathv;
        if (lane == 0) meta[j] = (uint32_t)leaf | ((uint32_t)d << 16);
        ++j;
    };
    auto leaf_path = [&](const Expansion &e) { return lane == (uint32_t)(e.depth + 1) ? e.base + (uint32_t)e.midx : e.pathv; };
    while (j < nb && !status) {
        const Expansion a = sim_front(p, t, logtab, rng, done, status, rs, L, slots);
        if (a.midx < 0 || status) {  // no expansion: the walk's end is the leaf
            record(a.node, a.depth, a.pathv);
            continue;
        }
        // the next simulation expands the same node (its untried moves are still cached):
        // take its pick now and let the helper generate its child
        // Only where a cannot run out of capacity on nodes or slots: b's sim_front erases b's
        // move from the node's untried list, which a failing a could not undo, so near the
        // arena's end the two run one at a time, as the one-wave search does (a position with
        // more than ZC_CHESS_MAX_MOVES legal moves, the one failure left, is unreachable chess).
        const bool pair = h != nullptr && rs.cached && j + 1 < nb && nnodes + 2 <= p.M &&
                          (int64_t)slots + 2 * ZC_CHESS_MAX_MOVES <= t.S;
        Expansion b{};
        const Rng rng_a = rng;  // the stream after a's draw: restored when a ends the flush
        if (pair) {
            b = sim_front(p, t, logtab, rng, done, status, rs, L, slots);
            if (lane < 18) h->stw[lane] = b.stw;
            if (lane == 0) {
                h->m = b.m;
                h->cmd = 1;
            }
            __syncthreads();  // the helper starts on b's child
        }
        const int ida = nnodes++;
        if (ida >= p.M) status = ZC_STATUS_INTERNAL;
        CSTAMP_T(cs3);
        // play_move + Node(...) (mcts.cpp:74-76); its legal moves generated on its first expansion
        const NodeGen ga = create_child_gen<ZC_CHESS_LAZY != 0>(L, a.stw, a.m);
        if (!status) commit_child(t, L, ga, a, ida, slots, status, cn);
        CSTAMP_ADD(3, cs3);
        record(ida, a.depth + 1, leaf_path(a));
        if (pair) {
            CSTAMP_T(cs21);
            __syncthreads();  // b's child is generated
            CSTAMP_ADD(21, cs21);
            if (status) {  // a ended the flush (a list past ZC_CHESS_MAX_MOVES): b's draw is not consumed
                rng = rng_a;
                break;
            }
            const int idb = nnodes++;
            if (idb >= p.M) status = ZC_STATUS_INTERNAL;
            if (!status) commit_child(t, h->L, h->gen, b, idb, slots, status, cn);
            record(idb, b.depth + 1, leaf_path(b));
        }
    }
    j = min(j, nb);
    wave_sync_mem();
    if (lane == 0) {
        ctl[cNodes] = nnodes;
        ctl[cSlots] = slots;
        ctl[cStatus] = status;
        ctl[cNb] = status ? 0 : nb;
        ctl[cExp] += cn.expansions;
        ctl[cDepth] += cn.depth_sum;
        rng_close(rng, use_now, p.a.rngpos + 2 * (size_t)g);
    }
    wave_sync_mem();
    return status ? 0 : nb;
}

__device__ __forceinline__ void chess_backup_flush(const ChessParams &p, const CTree &t, int g, const int32_t *ctl, const double *vals,
                             int nb) {
    const uint32_t *paths = p.ca.paths + (size_t)g * p.max_batch * kChessPath;
    const uint32_t *meta = p.ca.meta + (size_t)g * p.max_batch;
    const uint32_t lane = lane_id();
    if (nb <= 0) return;
    // leaf j + 1's record is loaded while leaf j's edges are updated: the only dependent
    // memory round trip left per leaf is its edges' read-modify-write
    uint32_t mn = meta[0], sn = paths[lane];
    for (int j = 0; j < nb; ++j) {
        const int d = (int)(uni(mn) >> 16);
        const uint32_t s = sn;
        if (j + 1 < nb) {
            mn = meta[j + 1];
            sn = paths[(size_t)(j + 1) * kChessPath + lane];
        }
        const double v = __hiloint2double(uni(__double2hiint(vals[j])), uni(__double2loint(vals[j])));
        // backprop (mcts.cpp:80-100): Na += 1, Wa -= (-1)^(d-l) v on the edge into level l
        if (lane >= 1 && lane <= (uint32_t)d) {
            const double r = ((d - (int)lane) & 1) ? -v : v;
            t.na[s] += 1;
            t.w[s] -= r;
        }
        wave_sync_mem();
    }
}

#ifndef ZC_CHESS_AGG_BACKUP
#define ZC_CHESS_AGG_BACKUP 1  // crude_backup_flush aggregates each flush's edges (A/B: 0)
#endif

// crude_chess_score's value.batch (mcts.cpp:116-118) and backprop (mcts.cpp:80-100) of one
// flush, the backup aggregated per edge.  The crude values are integers (material; +-1000 for
// a mate), so an edge's Na += its leaves and Wa -= the sum of their signed values equals the
// leaf-by-leaf updates exactly, whatever the order (every partial sum is an integer far below
// 2^53).  The flush's (leaf, level) edges are gathered in an LDS hash table (slot -> count,
// sum), eight leaves at a time (lane 8q + i: leaf j0 + q, level i + 1, + 8 per extra round),
// and every distinct edge is then updated once, all in one pass: one memory round trip per
// flush instead of a read-modify-write per leaf.  A flush of more than 64 leaves or with more
// (leaf, level) pairs than half the table takes the leaf-by-leaf chess_backup_flush.
constexpr int kBackupHash = 512;
struct BackupTable {
    uint32_t key[kBackupHash];  // slot + 1 (0: empty)
    int32_t cnt[kBackupHash];
    int32_t sum[kBackupHash];
};

__device__ __forceinline__ void backup_table_clear(BackupTable &T) {
    for (int e = (int)lane_id(); e < kBackupHash; e += 64) {
        T.key[e] = 0u;
        T.cnt[e] = 0;
        T.sum[e] = 0;
    }
    wave_sync_mem();
}

__device__ __forceinline__ void crude_values_backup(const ChessParams &p, const CTree &t, int g, const int32_t *ctl,
                                                    double *s_vals, int nb, BackupTable *T) {
    const uint32_t lane = lane_id();
    const uint32_t *meta = p.ca.meta + (size_t)g * p.max_batch;
    int dj = 0, vj = 0;  // lane j: leaf j's depth and crude value
    CSTAMP_T(cs4);
    for (int j = (int)lane; j < nb; j += 64) {
        const uint32_t mj = meta[j];
        const ChessNode *N = &t.nodes[mj & 0xFFFFu];
        const int nm = N->nmoves, chk = N->check, turn = N->st.turn, mat = N->material;
        vj = (nm == 0 && chk) ? 1000 : (turn * -2 + 1) * mat;
        dj = (int)(mj >> 16);
        s_vals[j] = (double)vj;
    }
    wave_sync_mem();
    CSTAMP_ADD(4, cs4);
    CSTAMP_T(cs5);
    int pairs = dj;
    for (int o = 32; o > 0; o >>= 1) pairs += __shfl_xor(pairs, o);
    if (!ZC_CHESS_AGG_BACKUP || !T || nb > 64 || pairs > kBackupHash / 2) {
        chess_backup_flush(p, t, g, ctl, s_vals, nb);
        CSTAMP_ADD(5, cs5);
        return;
    }
    const uint32_t *paths = p.ca.paths + (size_t)g * p.max_batch * kChessPath;
    const int qd = (int)(lane >> 3), i = (int)(lane & 7);
    for (int j0 = 0; j0 < nb; j0 += 8) {
        const int j = j0 + qd;
        const int d = __shfl(dj, j & 63), v = __shfl(vj, j & 63);
        const int dq = j < nb ? d : 0;
        int maxd = dq;
        for (int o = 32; o > 0; o >>= 1) maxd = max(maxd, __shfl_xor(maxd, o));
        for (int l0 = 1; l0 <= maxd; l0 += 8) {
            const int l = l0 + i;
            if (l <= dq) {
                const uint32_t sl = paths[(size_t)j * kChessPath + l];
                const int r = ((dq - l) & 1) ? -v : v;
                uint32_t h = (sl * 2654435761u) >> 23;  // 9 bits
                for (;;) {  // linear probing; the table is at most half full
                    const uint32_t prev = atomicCAS(&T->key[h], 0u, sl + 1u);
                    if (prev == 0u || prev == sl + 1u) break;
                    h = (h + 1u) & (uint32_t)(kBackupHash - 1);
                }
                atomicAdd(&T->cnt[h], 1);
                atomicAdd(&T->sum[h], r);
            }
        }
    }
    wave_sync_mem();
    // every distinct edge once: the eight entries of each lane read, updated and cleared together
    uint32_t key[kBackupHash / 64];
    int32_t cnt[kBackupHash / 64], sum[kBackupHash / 64];
#pragma unroll
    for (int k = 0; k < kBackupHash / 64; ++k) {
        const int e = k * 64 + (int)lane;
        key[k] = T->key[e];
        cnt[k] = T->cnt[e];
        sum[k] = T->sum[e];
    }
    int32_t na[kBackupHash / 64];
    double w[kBackupHash / 64];
#pragma unroll
    for (int k = 0; k < kBackupHash / 64; ++k) {
        na[k] = key[k] ? t.na[key[k] - 1u] : 0;
        w[k] = key[k] ? t.w[key[k] - 1u] : 0.0;
    }
#pragma unroll
    for (int k = 0; k < kBackupHash / 64; ++k) {
        if (key[k]) {
            t.na[key[k] - 1u] = na[k] + cnt[k];
            t.w[key[k] - 1u] = w[k] - (double)sum[k];
            const int e = k * 64 + (int)lane;
            T->key[e] = 0u;
            T->cnt[e] = 0;
            T->sum[e] = 0;
        }
    }
    wave_sync_mem();
    CSTAMP_ADD(5, cs5);
}

// ---------------------------------------------------------------- fused: crude_chess_score
// The whole search of one game from p.roots[gl] (root_init .. the last backup).
__device__ __forceinline__ void crude_search(const ChessParams &p, const CTree &t, CLds &L, double *s_vals, int gl, int g,
                             int32_t *ctl, Helper *h = nullptr, BackupTable *T = nullptr) {
    ConstDouble *logtab = (ConstDouble *)p.a.logtab;
    CSTAMP_T(cs7);
    root_init(p, t, L, gl, g, ctl);
    for (int done = 0; done < p.sims && !uni(ctl[cStatus]);) {
        CSTAMP_T(cs6);
        const int nb = chess_select_flush(p, t, L, logtab, g, ctl, done, min(p.bs, p.sims - done), h);
        CSTAMP_ADD(6, cs6);
        crude_values_backup(p, t, g, ctl, s_vals, nb, T);
        done += nb;
    }
    CSTAMP_ADD(7, cs7);
}

// Two waves per game: the leader runs the search, the helper generates the second child of
// each paired expansion (Helper).
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(2))) void chess_search_kernel(ChessParams p) {
    __shared__ CLds L;
    __shared__ double s_vals[256];
    __shared__ Helper H;
    __shared__ BackupTable T;
    const int gl = blockIdx.x;
    if (gl >= p.n_games) return;
    const int g = p.first_game + gl;
    const CTree t = ctree(p, g);
    if (__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) != 0) {
        helper_loop(H);
        return;
    }
    // the leader carries the serial chain (draws, commits, backups): it issues first when both
    // waves are ready (1.582 vs 1.691 ms per move, profiles/r05_ab_chess_variants.log)
    __builtin_amdgcn_s_setprio(1);
    int32_t *ctl = p.ca.ctl + (size_t)g * kCtlWords;
    CSTAMP_INIT();
    if (ZC_CHESS_AGG_BACKUP) backup_table_clear(T);
    crude_search(p, t, L, s_vals, gl, g, ctl, &H, &T);
    CSTAMP_FLUSH();
    finish(p, t, gl, g, ctl);
    helper_exit(&H);
}

// ---------------------------------------------------------------- chess self-play
// Engine.play_move + _evaluate (engine/engine.py:98-108, 148-153) of move m from q.roots[gl]:
// the position after the move (left in L.st), the mover's history push (play_move's deque,
// chess_backend.cpp:364-400), check_win / check_draw of the new position (:404-441:
// checkmate; stalemate, the fifty-move counter, both sides' histories repeating).  Returns
// the result (turn*2-1 with the new side to move, 0, or ZC_C4_ONGOING).
__device__ __attribute__((noinline)) int chess_play_judge(const ChessPlayParams &q, int gl, CLds &L, uint16_t *Lh, uint32_t m, int &err) {
    const uint32_t lane = lane_id();
    if (lane < 18) ((uint32_t *)&L.st)[lane] = ((const uint32_t *)&q.roots[gl])[lane];
    wave_sync_mem();
    const int mover = uni((int)L.st.turn);
    chessdev::apply_move_wave(L.st, m);
    wave_sync_mem();
    L.s.board[lane] = L.st.board[lane];
    wave_sync_mem();
    const int turn = uni((int)L.st.turn);
    bool check;
    const int k = chessdev::legal_moves_check(L.s.board, turn, L.s.legal, L.s.pseudo, L.s.region, check);
    uint16_t *h = q.hist + (size_t)gl * 2 * q.cap;
    int32_t *hl = q.hlen + 2 * (size_t)gl;
    const int len = uni(hl[mover]);
    if (len >= q.cap) err |= 1;  // a game longer than the history holds: flagged
    if (lane == 0) {
        h[(size_t)mover * q.cap + min(len, q.cap - 1)] = (uint16_t)m;
        hl[mover] = len + 1;
    }
    wave_sync_mem();
    const int rep = chessdev::repetitions(h, hl, q.cap, Lh);
    if (k < 0) {   // the legal-move list overflowed: the position cannot be judged.  The game
        err |= 8;  // ends here (refilled, recorded as a draw) instead of playing on from an
        return 0;  // unjudged position; err bit 8 makes check() / take() raise before any use
    }
    if (k == 0 && check) return turn * 2 - 1;
    if ((k == 0 && !check) || uni((int)L.st.fifty) >= 50 || rep == 3) return 0;
    return ZC_C4_ONGOING;
}

// After a step of game gl: its outputs at index o, its root to the post-move position or,
// when the game ended, to the initial position with empty histories (the refill of
// scripts/train.py:151-170).
__device__ void chess_play_commit(const ChessPlayParams &q, int gl, const CLds &L, size_t o, uint32_t m, int r) {
    const uint32_t lane = lane_id();
    if (lane < 18) {
        const uint32_t w = ((const uint32_t *)&L.st)[lane];
        ((uint32_t *)&q.out_states[o])[lane] = w;
        ((uint32_t *)&q.roots[gl])[lane] = r == ZC_C4_ONGOING ? w : ((const uint32_t *)q.init)[lane];
    }
    if (lane == 0) {
        if (q.out_moves) q.out_moves[o] = (uint16_t)m;
        q.out_results[o] = r;
        if (r != ZC_C4_ONGOING) {
            q.hlen[2 * (size_t)gl] = 0;
            q.hlen[2 * (size_t)gl + 1] = 0;
        }
    }
    wave_sync_mem();
}

__device__ __forceinline__ void chess_play_errors(const ChessPlayParams &q, int err) {
    if (lane_id() == 0 && err) {
        if (err & 1) atomicOr(q.err + 0, 1);
        if (err & 2) atomicOr(q.err + 1, 1);
        if (err & 4) atomicOr(q.err + 2, 1);
        if (err & 8) atomicOr(q.err + 1, 2);   // a position's legal-move list overflowed (bit 1)
    }
}

// Lockstep: one step of every game whose move some search (any mode) chose: q.in_moves[gl]
// (0xFFFF = the search found none: flagged, the game left as it is); q.search_stats flags a
// search that ran out of tree capacity.  Outputs at [gl].
__global__ __launch_bounds__(64) void chess_play_step_kernel(ChessPlayParams q, int n) {
    extern __shared__ uint16_t s_hist[];
    __shared__ CLds L;
    const int gl = blockIdx.x;
    if (gl >= n) return;
    int err = 0;
    if (q.search_stats && uni((int)q.search_stats[gl].status) == ZC_STATUS_CAPACITY) err |= 2;
    const uint32_t m = uni((uint32_t)q.in_moves[gl]);
    if (m == 0xFFFFu) {
        err |= 4;
        if (lane_id() < 18) ((uint32_t *)&L.st)[lane_id()] = ((const uint32_t *)&q.roots[gl])[lane_id()];
        wave_sync_mem();
        chess_play_commit(q, gl, L, (size_t)gl, m, ZC_C4_ONGOING);
    } else {
        const int r = chess_play_judge(q, gl, L, s_hist, m, err);
        chess_play_commit(q, gl, L, (size_t)gl, m, r);
    }
    chess_play_errors(q, err);
}

// Self-play with the crude score, `q.moves` moves per game in ONE launch (the chess form of
// c4_search.hip's c4_selfplay_kernel): per move the whole search from the game's root, the
// step above, the refill.  With q.ticket the games share q.budget moves (pooled); steps a
// game did not reach are ZC_SLOT_SKIP / move 0xFFFF.  Outputs [moves][n]; q.stats[gl] sums
// the moves' counters (reserved = games finished).
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(2))) void chess_selfplay_kernel(ChessParams p, ChessPlayParams q) {
    extern __shared__ uint16_t s_hist[];
    __shared__ CLds L;
    __shared__ double s_vals[256];
    __shared__ Helper H;
    __shared__ BackupTable T;
    const int gl = blockIdx.x;
    if (gl >= p.n_games) return;
    const int g = p.first_game + gl;
    const CTree t = ctree(p, g);
    if (__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) != 0) {  // the helper wave (Helper)
        helper_loop(H);
        return;
    }
    __builtin_amdgcn_s_setprio(1);  // the leader first (chess_search_kernel)
    if (ZC_CHESS_AGG_BACKUP) backup_table_clear(T);
    const uint32_t lane = lane_id();
    int32_t *ctl = p.ca.ctl + (size_t)g * kCtlWords;
    const uint64_t use_start = uni64(p.a.rngpos[2 * (size_t)g]);
    int64_t exp = 0, depth = 0;
    int finished = 0, status = 0, err = 0, mv = 0;
    for (; mv < q.moves; ++mv) {
        if (q.ticket) {
            int tk = 0;
            if (lane == 0) tk = atomicAdd(q.ticket, 1);
            if (uni(tk) >= q.budget) break;
        }
        crude_search(p, t, L, s_vals, gl, g, ctl, &H, &T);
        status = uni(ctl[cStatus]);
        exp += uni(ctl[cExp]);
        depth += uni(ctl[cDepth]);
        if (status) {  // a root without moves is never live here: flagged, the game stops
            err |= status == ZC_STATUS_CAPACITY ? 2 : 4;
            break;
        }
        const ChessNode *R = &t.nodes[0];
        const uint32_t base = uni(R->base);
        const int bi = best_root_slot(t, uni((int)R->nmoves), base);
        if (bi == 0x7FFFFFFF) {
            err |= 4;
            break;
        }
        const uint32_t m = uni((uint32_t)t.mv[base + bi]);
        const int r = chess_play_judge(q, gl, L, s_hist, m, err);
        chess_play_commit(q, gl, L, (size_t)mv * p.n_games + gl, m, r);
        finished += r != ZC_C4_ONGOING;
    }
    if (q.ticket && lane == 0) atomicMax(q.ticket + 1, mv);
    for (int k = mv + (int)lane; k < q.moves; k += 64) {
        const size_t o = (size_t)k * p.n_games + gl;
        q.out_moves[o] = 0xFFFF;
        q.out_results[o] = ZC_SLOT_SKIP;
    }
    chess_play_errors(q, err);
    if (lane == 0) {
        zc_game_stats st{};
        st.status = status;
        st.expansions = exp;
        st.depth_sum = depth;
        st.leaves = (int64_t)p.sims * mv;
        st.rng_words = (int64_t)(p.a.rngpos[2 * (size_t)g] - use_start);
        st.reserved = finished;
        q.stats[gl] = st;
    }
    helper_exit(&H);
}

// ---------------------------------------------------------------- stepwise (caller values)
__global__ __launch_bounds__(64) void chess_ext_begin_kernel(ChessParams p) {
    __shared__ CLds L;
    const int gl = blockIdx.x;
    if (gl >= p.n_games) return;
    const int g = p.first_game + gl;
    root_init(p, ctree(p, g), L, gl, g, p.ca.ctl + (size_t)g * kCtlWords);
}

__global__ __launch_bounds__(64) void chess_ext_select_kernel(ChessParams p) {
    __shared__ CLds L;
    const int gl = blockIdx.x;
    if (gl >= p.n_games) return;
    const int g = p.first_game + gl;
    const CTree t = ctree(p, g);
    int32_t *ctl = p.ca.ctl + (size_t)g * kCtlWords;
    const uint32_t lane = lane_id();
    int nb = 0;
    if (!uni(ctl[cStatus])) {
        const int done = p.flush * p.bs;
        nb = chess_select_flush(p, t, L, (ConstDouble *)p.a.logtab, g, ctl, done, min(p.bs, p.sims - done));
    } else if (lane == 0) {
        ctl[cNb] = 0;
    }
    if (lane == 0 && p.counts) p.counts[gl] = nb;
    const uint32_t *meta = p.ca.meta + (size_t)g * p.max_batch;
    const size_t obase = (size_t)gl * p.bs;
    for (int j = 0; j < nb; ++j) {
        const ChessNode *N = &t.nodes[uni(meta[j]) & 0xFFFFu];
        if (p.leaves && lane < 18) ((uint32_t *)&p.leaves[obase + j])[lane] = ((const uint32_t *)&N->st)[lane];
        if (p.planes) {
            // state_to_tensor (chess_backend.cpp:461-521): lane = square
            const uint32_t pc = N->st.board[lane];
            const char pieces[12] = {'P', 'N', 'B', 'R', 'Q', 'K', 'p', 'n', 'b', 'r', 'q', 'k'};
            int which = -1;
            for (int k = 0; k < 12; ++k)
                if (pc == (uint8_t)pieces[k]) {
                    which = k;
                    break;
                }
            const int turn = N->st.turn, castle = N->st.castle;
            for (int k = 0; k < 17; ++k) {
                float v;
                if (k < 12) v = k == which ? 1.0f : 0.0f;
                else if (k == 12) v = turn == 0 ? 1.0f : 0.0f;
                else v = (castle >> (k - 13)) & 1 ? 1.0f : 0.0f;
                const size_t o = ((obase + j) * 17 + k) * 64 + lane;
                if (p.planes_f16) ((__half *)p.planes)[o] = __float2half(v);
                else ((float *)p.planes)[o] = v;
            }
        }
    }
}

__global__ __launch_bounds__(64) void chess_ext_backup_kernel(ChessParams p) {
    const int gl = blockIdx.x;
    if (gl >= p.n_games) return;
    const int g = p.first_game + gl;
    const int32_t *ctl = p.ca.ctl + (size_t)g * kCtlWords;
    const int nb = uni(ctl[cNb]);
    if (uni(ctl[cStatus]) || nb == 0) return;
    chess_backup_flush(p, ctree(p, g), g, ctl, p.values + (size_t)gl * p.bs, nb);
}

__global__ __launch_bounds__(64) void chess_ext_end_kernel(ChessParams p) {
    const int gl = blockIdx.x;
    if (gl >= p.n_games) return;
    const int g = p.first_game + gl;
    finish(p, ctree(p, g), gl, g, p.ca.ctl + (size_t)g * kCtlWords);
}

// ---------------------------------------------------------------- host policy (§8(b))
// One game, one simulation per walk/expand pair, as c4_ext.hip's zc_c4_hp_*: the caller's
// policy picks among the untried moves between the two launches.
__global__ __launch_bounds__(64) void chess_hp_walk_kernel(ChessParams p) {
    const uint32_t lane = lane_id();
    const int g = p.first_game;
    const CTree t = ctree(p, g);
    int32_t *ctl = p.ca.ctl + (size_t)g * kCtlWords;
    int status = uni(ctl[cStatus]);
    zc_chess_hp_node *out = p.hp_node;
    if (status) {
        if (lane == 0) {
            out->node = -1;
            out->n_untried = 0;
            out->depth = 0;
        }
        return;
    }
    int node = 0, depth = 0, nN = p.flush * p.bs;
    uint32_t pathv = 0;
    chess_walk(p, t, (ConstDouble *)p.a.logtab, node, depth, nN, pathv, status);
    uint32_t *path = p.ca.paths + ((size_t)g * p.max_batch + p.hp_leaf) * kChessPath;
    if (lane < (uint32_t)kChessPath) path[lane] = pathv;
    const ChessNode *N = &t.nodes[node];
    const int nu = status ? 0 : uni((int)N->nu);
    const uint32_t base = uni(N->base);
    for (int i = (int)lane; i < nu; i += 64) out->untried[i] = t.mv[base + t.ut[base + i]];
    if (lane < 18) ((uint32_t *)&out->state)[lane] = ((const uint32_t *)&N->st)[lane];
    if (lane == 0) {
        out->node = node;
        out->n_untried = nu;
        out->depth = depth;
        ctl[cHpNode] = node;
        ctl[cHpNode + 1] = depth;
        ctl[cStatus] = status;
    }
}

__global__ __launch_bounds__(64) void chess_hp_expand_kernel(ChessParams p) {
    __shared__ CLds L;
    const uint32_t lane = lane_id();
    const int g = p.first_game;
    const CTree t = ctree(p, g);
    int32_t *ctl = p.ca.ctl + (size_t)g * kCtlWords;
    if (uni(ctl[cStatus])) return;
    const int node = uni(ctl[cHpNode]);
    int depth = uni(ctl[cHpNode + 1]);
    int nnodes = uni(ctl[cNodes]), slots = uni(ctl[cSlots]), status = 0;
    uint32_t *path = p.ca.paths + ((size_t)g * p.max_batch + p.hp_leaf) * kChessPath;
    ChessNode *N = &t.nodes[node];
    const int nu = uni((int)N->nu);
    int leaf = node;
    if (nu > 0) {
        const int local = p.hp_index;
        if (local < 0 || local >= nu) {
            if (lane == 0) ctl[cStatus] = ZC_STATUS_INTERNAL;
            return;
        }
        if (nnodes >= p.M) {  // out of tree capacity: reported before the node is changed
            if (lane == 0) ctl[cStatus] = ZC_STATUS_CAPACITY;
            return;
        }
        // expand (mcts.cpp:65-78) with the caller's pick: untried.erase(begin + local)
        const uint32_t base = uni(N->base);
        const int midx = uni((int)t.ut[base + local]);
        const uint32_t m = uni((uint32_t)t.mv[base + midx]);
        for (int b = local; b < nu - 1; b += 64) {
            const int i = b + (int)lane;
            uint8_t v = 0;
            if (i < nu - 1) v = t.ut[base + i + 1];
            wave_sync_mem();
            if (i < nu - 1) t.ut[base + i] = v;
        }
        if (lane == 0) N->nu = (uint16_t)(nu - 1);
        if (lane < 18) ((uint32_t *)&L.st)[lane] = ((const uint32_t *)&N->st)[lane];
        wave_sync_mem();
        chessdev::apply_move_wave(L.st, m);
        wave_sync_mem();
        const int child = nnodes++;
        create_node(t, L, child, node, midx, depth + 1, slots, status);
        ++depth;
        if (lane == 0) {
            t.ch[base + midx] = (uint16_t)child;
            path[depth] = base + (uint32_t)midx;
            ctl[cExp] += 1;
            ctl[cDepth] += depth;
        }
        leaf = child;
        wave_sync_mem();
    }
    if (p.leaves && lane < 18) ((uint32_t *)&p.leaves[0])[lane] = ((const uint32_t *)&t.nodes[leaf].st)[lane];
    if (lane == 0) {
        p.ca.meta[(size_t)g * p.max_batch + p.hp_leaf] = (uint32_t)leaf | ((uint32_t)depth << 16);
        ctl[cNodes] = nnodes;
        ctl[cSlots] = slots;
        ctl[cStatus] = status;
        ctl[cNb] = p.hp_leaf + 1;
    }
}

// ---------------------------------------------------------------- random_rollout on chess
// Value('random_rollout') (engine/value_functions.py:35-45) with the chess backend: while
// not check_win and not check_draw (chess_backend.cpp:404-441), play
// random.choice(list(get_legal_moves(state))) (:184-360; _randbelow on the game's stream);
// at the end -1 if the side to move (the loser of a checkmate) is the leaf's side to move,
// +1 for the other side's checkmate, 0 for a draw.
//
// check_draw's repetition half, has_repeated_prefix(hist, 2, 3) on both sides' histories
// (:148-180, KMP over the deque, most recent move first), is kept incrementally.  With the
// history a[0..n) in play order, KMP's test — some prefix of the deque whose smallest period
// p >= 2 divides its length at least 3 times — holds iff for some p >= 2 the last 3p moves
// have period p and are not all equal (<=: Fine and Wilf put the smallest period of the
// 3p-suffix below p, dividing it; =>: the 3p'-prefix of KMP's prefix is such a suffix).  So
// each side keeps c_p = the number of trailing i with a[i] == a[i-p], for every p <= n (one
// LDS counter per p, lanes over p): a push of x updates c_p = (x == a[n-p]) ? c_p + 1 : 0, and
// the test is c_p >= 2p and c_1 < 3p - 1 for some p >= 2.  O(n / 64) per ply.
struct RollSide {
    uint16_t *a;    // moves in play order
    uint16_t *cnt;  // cnt[p], p in [1, kRollCap]
    int n, c1;
    bool rep;
};

__device__ __forceinline__ void roll_side_init(RollSide &s) {
    const uint32_t lane = lane_id();
    bool hit = false;
    for (int b = 0; b < s.n; b += 64) {
        const int p = b + (int)lane + 1;
        if (p <= s.n) {
            int c = 0;
            for (int i = s.n - 1; i >= p && s.a[i] == s.a[i - p]; --i) ++c;
            s.cnt[p] = (uint16_t)c;
        }
    }
    if (lane == 0 && s.n + 1 <= kRollCap) s.cnt[s.n + 1] = 0;
    wave_sync_mem();
    s.c1 = s.n >= 1 ? uni((int)s.cnt[1]) : 0;
    for (int b = 0; b < s.n; b += 64) {
        const int p = b + (int)lane + 1;
        if (p >= 2 && p <= s.n && (int)s.cnt[p] >= 2 * p && s.c1 < 3 * p - 1) hit = true;
    }
    s.rep = __ballot(hit) != 0;
}

// play_move's history push (chess_backend.cpp:374) of move x, and the new repetition answer.
__device__ __forceinline__ void roll_side_push(RollSide &s, uint16_t x) {
    const uint32_t lane = lane_id();
    const int n = s.n;
    s.c1 = (n >= 1 && uni((int)s.a[n - 1]) == (int)x) ? s.c1 + 1 : 0;
    bool hit = false;
    for (int b = 0; b < n; b += 64) {
        const int p = b + (int)lane + 1;
        if (p <= n) {
            int c = s.cnt[p];
            c = s.a[n - p] == x ? c + 1 : 0;
            s.cnt[p] = (uint16_t)c;
            if (p >= 2 && c >= 2 * p && s.c1 < 3 * p - 1) hit = true;
        }
    }
    wave_sync_mem();
    if (lane == 0) {
        s.a[n] = x;
        if (n + 2 <= kRollCap) s.cnt[n + 2] = 0;   // c_p of a period the history reaches next push
    }
    wave_sync_mem();
    s.n = n + 1;
    s.rep = __ballot(hit) != 0;
}

// One rollout from the position in L.st with histories w (white's) / k (black's).  Returns
// the value; status ZC_STATUS_CAPACITY when a history outgrows kRollCap or a position its
// move list.
template <class R>
__device__ int chess_rollout(CLds &L, RollSide &w, RollSide &k, R &rng, int &status) {
    const uint32_t lane = lane_id();
    roll_side_init(w);
    roll_side_init(k);
    const int t0 = uni((int)L.st.turn);
    for (;;) {
        L.s.board[lane] = L.st.board[lane];
        wave_sync_mem();
        const int turn = uni((int)L.st.turn);
        bool check;
        const int nl = chessdev::legal_moves_check(L.s.board, turn, L.s.legal, L.s.pseudo, L.s.region, check);
        if (nl < 0) {
            status = ZC_STATUS_CAPACITY;
            return 0;
        }
        if (nl == 0 && check) return turn == t0 ? -1 : 1;                        // check_win
        if (nl == 0 || uni((int)L.st.fifty) >= 50 || (w.rep && k.rep)) return 0;   // check_draw
        const uint32_t r = rng_below(rng, (uint32_t)nl);
        const uint16_t m = (uint16_t)uni((int)L.s.legal[r]);
        if ((turn ? k.n : w.n) >= kRollCap) {
            status = ZC_STATUS_CAPACITY;
            return 0;
        }
        if (turn) roll_side_push(k, m);
        else roll_side_push(w, m);
        chessdev::apply_move_wave(L.st, m);
        wave_sync_mem();
    }
}

// Rollouts in order on game g's stream: the tree's pending leaves of p.flush (from_tree:
// histories = the root's + the path's moves, pushed by alternating movers from the root's
// side to move) or the p.n_states given states with their own histories.
__global__ __launch_bounds__(64) void chess_rollouts_kernel(ChessParams p, int from_tree) {
    extern __shared__ uint16_t s_roll[];   // a[2][kRollCap], cnt[2][kRollCap + 1]
    __shared__ CLds L;
    const uint32_t lane = lane_id();
    const int gl = blockIdx.x;
    if (gl >= p.n_games) return;
    const int g = p.first_game + gl;
    int32_t *ctl = p.ca.ctl + (size_t)g * kCtlWords;
    const CTree t = ctree(p, g);
    int status = 0;
    int nb;
    if (from_tree) {
        nb = uni(ctl[cStatus]) ? 0 : uni(ctl[cNb]);
    } else {
        nb = p.n_states;
    }
    Rng rng;
    const uint64_t use_now = uni64(p.a.rngpos[2 * (size_t)g]);
    rng_open(rng, p.a.ring + (size_t)g * kRingWords, use_now, uni64(p.a.rngpos[2 * (size_t)g + 1]));
    const uint32_t *paths = p.ca.paths + (size_t)g * p.max_batch * kChessPath;
    const uint32_t *meta = p.ca.meta + (size_t)g * p.max_batch;
    const int t0 = from_tree ? uni((int)t.nodes[0].st.turn) : 0;
    for (int j = 0; j < nb && !status; ++j) {
        const int hi = from_tree ? gl : j;   // whose histories
        const uint16_t *hs = p.rhist + (size_t)hi * 2 * p.rhcap;
        const int nw = uni(p.rhlen[2 * hi]), nk = uni(p.rhlen[2 * hi + 1]);
        if (nw > p.rhcap || nk > p.rhcap || nw < 0 || nk < 0) {
            // a history longer than its buffer: its most recent moves (what the repetition
            // draw reads) are missing, so refuse rather than roll out on a truncated history
            status = ZC_STATUS_CAPACITY;
            break;
        }
        RollSide w{s_roll, s_roll + 2 * kRollCap, nw, 0, false};
        RollSide k{s_roll + kRollCap, s_roll + 2 * kRollCap + kRollCap + 1, nk, 0, false};
        int d = 0;
        const uint32_t *pw = nullptr;
        if (from_tree) {
            const uint32_t m = uni(meta[j]);
            d = (int)(m >> 16);
            pw = paths + (size_t)j * kChessPath;
            const ChessNode *N = &t.nodes[m & 0xFFFFu];
            if (lane < 18) ((uint32_t *)&L.st)[lane] = ((const uint32_t *)&N->st)[lane];
        } else if (lane < 18) {
            ((uint32_t *)&L.st)[lane] = ((const uint32_t *)&p.rstates[j])[lane];
        }
        const int wt = (t0 == 0 ? (d + 1) / 2 : d / 2), bt = d - wt;   // path moves per side
        if (w.n + wt > kRollCap || k.n + bt > kRollCap) {
            status = ZC_STATUS_CAPACITY;
            break;
        }
        for (int i = (int)lane; i < w.n; i += 64) w.a[i] = hs[i];
        for (int i = (int)lane; i < k.n; i += 64) k.a[i] = hs[p.rhcap + i];
        wave_sync_mem();
        if (lane >= 1 && lane <= (uint32_t)d) {   // the move into level l was played by (t0 + l - 1) & 1
            const uint16_t mv = t.mv[pw[lane]];
            const int side = (t0 + (int)lane - 1) & 1;
            (side ? k.a + k.n : w.a + w.n)[(lane - 1) >> 1] = mv;
        }
        wave_sync_mem();
        w.n += wt;
        k.n += bt;
        const int v = chess_rollout(L, w, k, rng, status);
        if (lane == 0) p.rvalues[(size_t)gl * (from_tree ? p.bs : 0) + j] = (double)v;
    }
    wave_sync_mem();
    if (lane == 0) {
        rng_close(rng, use_now, p.a.rngpos + 2 * (size_t)g);
        if (p.rstatus) p.rstatus[gl] = status;
    }
}

// The moves from the root to each pending leaf of the flush (the host-value leaves' move
// histories): moves[leaf][l - 1] = the move into level l, depth[leaf].
__global__ __launch_bounds__(64) void chess_leaf_moves_kernel(ChessParams p) {
    const uint32_t lane = lane_id();
    const int gl = blockIdx.x;
    if (gl >= p.n_games) return;
    const int g = p.first_game + gl;
    const int32_t *ctl = p.ca.ctl + (size_t)g * kCtlWords;
    const CTree t = ctree(p, g);
    const int nb = uni(ctl[cStatus]) ? 0 : uni(ctl[cNb]);
    const uint32_t *paths = p.ca.paths + (size_t)g * p.max_batch * kChessPath;
    const uint32_t *meta = p.ca.meta + (size_t)g * p.max_batch;
    for (int j = 0; j < p.bs; ++j) {
        const size_t o = (size_t)gl * p.bs + j;
        const int d = j < nb ? (int)(uni(meta[j]) >> 16) : 0;
        if (lane == 0) p.path_depth[o] = d;
        if (lane >= 1 && lane <= (uint32_t)d) p.path_moves[o * kChessPath + lane - 1] = t.mv[paths[(size_t)j * kChessPath + lane]];
    }
}

}  // namespace

void launch_chess_hp_walk(const ChessParams &p, hipStream_t s) {
    hipLaunchKernelGGL(chess_hp_walk_kernel, dim3(1), dim3(64), 0, s, p);
}
void launch_chess_hp_expand(const ChessParams &p, hipStream_t s) {
    hipLaunchKernelGGL(chess_hp_expand_kernel, dim3(1), dim3(64), 0, s, p);
}

void launch_chess_search(const ChessParams &p, hipStream_t s) {
    hipLaunchKernelGGL(chess_search_kernel, dim3(p.n_games), dim3(128), 0, s, p);
}
void launch_chess_play_step(const ChessPlayParams &q, int n, hipStream_t s) {
    hipLaunchKernelGGL(chess_play_step_kernel, dim3(n), dim3(64), (size_t)q.cap * sizeof(uint16_t), s, q, n);
}
void launch_chess_selfplay(const ChessParams &p, const ChessPlayParams &q, hipStream_t s) {
    hipLaunchKernelGGL(chess_selfplay_kernel, dim3(p.n_games), dim3(128), (size_t)q.cap * sizeof(uint16_t), s, p, q);
}
int chess_selfplay_resident_games(int cap, int *out) {
    int blocks = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, (const void *)chess_selfplay_kernel, 128,
                                                     (size_t)cap * sizeof(uint16_t)) != hipSuccess)
        return -1;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return -1;
    *out = blocks * cus;
    return 0;
}
void launch_chess_ext_begin(const ChessParams &p, hipStream_t s) {
    hipLaunchKernelGGL(chess_ext_begin_kernel, dim3(p.n_games), dim3(64), 0, s, p);
}
void launch_chess_ext_select(const ChessParams &p, hipStream_t s) {
    hipLaunchKernelGGL(chess_ext_select_kernel, dim3(p.n_games), dim3(64), 0, s, p);
}
void launch_chess_ext_backup(const ChessParams &p, hipStream_t s) {
    hipLaunchKernelGGL(chess_ext_backup_kernel, dim3(p.n_games), dim3(64), 0, s, p);
}
void launch_chess_ext_end(const ChessParams &p, hipStream_t s) {
    hipLaunchKernelGGL(chess_ext_end_kernel, dim3(p.n_games), dim3(64), 0, s, p);
}
void launch_chess_rollouts(const ChessParams &p, bool from_tree, hipStream_t s) {
    const size_t lds = (size_t)(4 * kRollCap + 2) * sizeof(uint16_t);
    hipLaunchKernelGGL(chess_rollouts_kernel, dim3(p.n_games), dim3(64), lds, s, p, from_tree ? 1 : 0);
}
void launch_chess_leaf_moves(const ChessParams &p, hipStream_t s) {
    hipLaunchKernelGGL(chess_leaf_moves_kernel, dim3(p.n_games), dim3(64), 0, s, p);
}

}  // namespace zc

#if ZC_CHESS_STAMP
// diagnostic build only (not in include/zeroclone.h): copy / clear the phase stamps
extern "C" int zc_debug_chess_stamps(uint64_t *host, int n, int clear) {
    if (n > 4096 * zc::kCStamps) n = 4096 * zc::kCStamps;
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(zc::g_chess_stamp), (size_t)n * 8) != hipSuccess) return 1;
    if (clear) {
        static uint64_t zeros[4096 * zc::kCStamps];
        if (hipMemcpyToSymbol(HIP_SYMBOL(zc::g_chess_stamp), zeros, sizeof(zeros)) != hipSuccess) return 1;
    }
    return 0;
}
#endif
