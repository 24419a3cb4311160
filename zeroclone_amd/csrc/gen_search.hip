// gen_search.hip — the search tree of mcts.get_move for ANY game backend (SURVEY.md §8(b)'s
// fallback: "Unknown backend, value or policy objects must still work").
//
// The reference's search core (engine/mcts/src/mcts.cpp) is game-agnostic: it reaches the
// game only through backend.get_legal_moves / play_move (:65-78, :104-108), the policy
// callable (:67-70) and value.batch (:116).  Those are Python objects of the caller's; they
// stay on the host.  Everything else — the tree and its statistics (Node::N, Na, Wa, Qa,
// children, untried, :10-39), UCT selection (:41-63), the expansion bookkeeping (:65-78)
// and the pending-order backup (:80-100, :112-127) — lives here, on the device:
//
//   zc_gen_walk    select from the root: at each node with no untried move, the first
//                  child maximising UCT = Qa + c*sqrt(log N / Na) (+inf while Na = 0; a
//                  strict > scan from -1e100, null children skipped); stops at a node with
//                  untried moves, or one without children.  Returns the node and its
//                  untried move indices (list order), for the host's policy call.
//   zc_gen_expand  untried.erase(local), the child node with the host's move count, its
//                  edge; the leaf joins the pending flush (the walked node itself when it
//                  had nothing to expand).
//   zc_gen_backup  the flush's values, leaf by leaf in pending order (fp64, the reference's
//                  operation order): N += 1 up the path, Na += 1, Wa -= r, Qa = Wa / Na, r = -r.
//   zc_gen_end     the root child with the most visits (first maximum of child N).
//
// Layout: nodes [cap] (GenNode), per-slot SoA arrays [slot cap] — a node's moves occupy the
// slots [base, base + nmoves); untried[base + i], i < nu, are its untried move indices in
// list order.  One search at a time per engine, one wave per launch (each call is one step
// of a serial chain that waits on Python between steps).
#include "zc_internal.h"

namespace zc {
namespace {

__device__ __forceinline__ int uni_i(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ double uni_d(double x) {
    return __hiloint2double(uni_i(__double2hiint(x)), uni_i(__double2loint(x)));
}
__device__ __forceinline__ void wave_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

// UCT exactly as mcts.cpp:41-45 compiles (-ffast-math: vdivsd, vsqrtsd, vfmadd213sd), with
// log(N) from the engine's glibc table.
__device__ __forceinline__ double gen_uct(const GenParams &p, int n, int32_t na, double qa) {
    if (na == 0) return INFINITY;
    return fma(p.c, sqrt(p.logtab[n] / (double)na), qa);
}

__global__ __launch_bounds__(64) void gen_begin_kernel(GenParams p, int root_moves) {
    const int lane = (int)__lane_id();
    GenArena &a = p.a;
    if (lane == 0) {
        GenNode r{};
        r.base = 0;
        r.nmoves = root_moves;
        r.nu = root_moves;
        r.parent = -1;
        r.pact = -1;
        r.n = 0;
        r.depth = 0;
        a.nodes[0] = r;
        a.ctl[kGenNodes] = 1;
        a.ctl[kGenSlots] = root_moves;
        a.ctl[kGenPending] = 0;
        a.ctl[kGenWalked] = 0;
        a.ctl[kGenStatus] = 0;
        a.ctl[kGenExp] = 0;
        a.ctl[kGenDepth] = 0;
    }
    for (int i = lane; i < root_moves; i += 64) {
        a.na[i] = 0;
        a.wa[i] = 0.0;
        a.qa[i] = 0.0;
        a.child[i] = -1;
        a.untried[i] = i;
    }
}

__global__ __launch_bounds__(64) void gen_walk_kernel(GenParams p, int32_t *out, int out_cap) {
    const int lane = (int)__lane_id();
    GenArena &a = p.a;
    int node = 0, depth = 0;
    if (uni_i(a.ctl[kGenStatus]) == 0) {
        for (;;) {
            const GenNode N = a.nodes[node];
            const int nu = uni_i(N.nu), nm = uni_i(N.nmoves), base = uni_i(N.base), n = uni_i(N.n);
            if (nu > 0) break;  // select: a node with untried moves is returned
            // first i with v > best (best from -1e100), over the non-null children
            double best_v = -1e100;
            int best = -1;
            for (int c0 = 0; c0 < nm; c0 += 64) {
                const int i = c0 + lane;
                double v = -INFINITY;
                bool ok = false;
                if (i < nm && a.child[base + i] >= 0) {
                    v = gen_uct(p, n, a.na[base + i], a.qa[base + i]);
                    ok = v > -1e100;  // NaN and <= -1e100 never win
                }
                // the chunk's maximum, then its first lane
                double m = ok ? v : -INFINITY;
                for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o));
                const unsigned long long hit = __ballot(ok && v == m);
                if (hit) {
                    m = uni_d(m);
                    if (m > best_v) {
                        best_v = m;
                        best = c0 + __ffsll((long long)hit) - 1;
                    }
                }
            }
            if (best < 0) break;  // no children: the walk ends here (a terminal position)
            node = uni_i(a.child[base + best]);
            ++depth;
        }
    }
    const GenNode N = a.nodes[node];
    const int nu = uni_i(N.nu), base = uni_i(N.base);
    if (lane == 0) {
        a.ctl[kGenWalked] = node;
        out[0] = node;
        out[1] = nu;
        out[2] = N.nmoves;
        out[3] = depth;
        out[4] = a.ctl[kGenStatus];
    }
    for (int i = lane; i < nu && 5 + i < out_cap; i += 64) out[5 + i] = a.untried[base + i];
}

__global__ __launch_bounds__(64) void gen_expand_kernel(GenParams p, int local, int child_moves) {
    const int lane = (int)__lane_id();
    GenArena &a = p.a;
    if (uni_i(a.ctl[kGenStatus])) return;
    const int node = uni_i(a.ctl[kGenWalked]);
    GenNode *N = &a.nodes[node];
    const int nu = uni_i(N->nu), base = uni_i(N->base);
    int leaf = node, status = 0;
    const int pending = uni_i(a.ctl[kGenPending]);
    if (pending >= p.bs) status = ZC_STATUS_INTERNAL;  // the host flushes every bs leaves
    if (!status && local >= 0) {
        const int id = uni_i(a.ctl[kGenNodes]), slots = uni_i(a.ctl[kGenSlots]);
        if (local >= nu) status = ZC_STATUS_INTERNAL;
        else if (id >= p.a.node_cap || (int64_t)slots + child_moves > p.a.slot_cap) status = ZC_STATUS_CAPACITY;
        if (!status) {
            const int move_idx = uni_i(a.untried[base + local]);
            // untried.erase(begin + local): ascending chunks, each read before it is written
            for (int c0 = local; c0 < nu - 1; c0 += 64) {
                const int i = c0 + lane;
                int32_t v = 0;
                if (i < nu - 1) v = a.untried[base + i + 1];
                wave_fence();
                if (i < nu - 1) a.untried[base + i] = v;
                wave_fence();
            }
            const int depth = uni_i(N->depth) + 1;
            if (lane == 0) {
                N->nu = nu - 1;
                GenNode c{};
                c.base = slots;
                c.nmoves = child_moves;
                c.nu = child_moves;
                c.parent = node;
                c.pact = move_idx;
                c.n = 0;
                c.depth = depth;
                a.nodes[id] = c;
                a.child[base + move_idx] = id;
                a.ctl[kGenNodes] = id + 1;
                a.ctl[kGenSlots] = slots + child_moves;
                a.ctl[kGenExp] += 1;
                a.ctl[kGenDepth] += depth;
            }
            for (int i = lane; i < child_moves; i += 64) {
                a.na[slots + i] = 0;
                a.wa[slots + i] = 0.0;
                a.qa[slots + i] = 0.0;
                a.child[slots + i] = -1;
                a.untried[slots + i] = i;
            }
            leaf = id;
        }
    } else if (!status && nu > 0) {
        status = ZC_STATUS_INTERNAL;  // a node with untried moves is always expanded
    }
    if (lane == 0) {
        if (status) {
            a.ctl[kGenStatus] = status;
        } else {
            a.pending[pending] = leaf;
            a.ctl[kGenPending] = pending + 1;
        }
    }
}

// Backup is a serial chain over the pending leaves (pending order fixes the fp64 rounding of
// every Wa); lane 0 walks it.
__global__ __launch_bounds__(64) void gen_backup_kernel(GenParams p, int nb, const double *values) {
    GenArena &a = p.a;
    if (__lane_id() != 0 || a.ctl[kGenStatus]) return;
    if (a.ctl[kGenPending] != nb) {
        a.ctl[kGenStatus] = ZC_STATUS_INTERNAL;
        return;
    }
    for (int j = 0; j < nb; ++j) {
        int node = a.pending[j];
        double r = values[j];
        for (;;) {
            GenNode *N = &a.nodes[node];
            N->n += 1;
            const int par = N->parent;
            if (par < 0) break;
            const int s = a.nodes[par].base + N->pact;
            const int32_t na = a.na[s] + 1;
            const double wa = a.wa[s] - r;
            a.na[s] = na;
            a.wa[s] = wa;
            a.qa[s] = wa / (double)na;
            node = par;
            r = -r;
        }
    }
    a.ctl[kGenPending] = 0;
}

__global__ __launch_bounds__(64) void gen_end_kernel(GenParams p, int32_t *out, int32_t *root_na, int na_cap) {
    const int lane = (int)__lane_id();
    GenArena &a = p.a;
    const GenNode R = a.nodes[0];
    const int nm = uni_i(R.nmoves), base = uni_i(R.base);
    int best = -1, best_n = -1;
    for (int c0 = 0; c0 < nm; c0 += 64) {  // first i with child N > best N
        const int i = c0 + lane;
        const int ch = i < nm ? a.child[base + i] : -1;
        const int n = ch >= 0 ? a.nodes[ch].n : -1;
        int m = n;
        for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o));
        m = uni_i(m);
        if (m > best_n) {
            best_n = m;
            best = c0 + __ffsll((long long)__ballot(ch >= 0 && n == m)) - 1;
        }
        if (root_na && i < nm && i < na_cap) root_na[i] = a.na[base + i];
    }
    if (lane == 0) {
        out[0] = best;
        out[1] = a.ctl[kGenStatus];
        out[2] = a.ctl[kGenExp];
        out[3] = a.ctl[kGenDepth];
        out[4] = a.ctl[kGenNodes];
    }
}

}  // namespace

void launch_gen_begin(const GenParams &p, int root_moves, hipStream_t s) {
    hipLaunchKernelGGL(gen_begin_kernel, dim3(1), dim3(64), 0, s, p, root_moves);
}
void launch_gen_walk(const GenParams &p, int32_t *out, int out_cap, hipStream_t s) {
    hipLaunchKernelGGL(gen_walk_kernel, dim3(1), dim3(64), 0, s, p, out, out_cap);
}
void launch_gen_expand(const GenParams &p, int local, int child_moves, hipStream_t s) {
    hipLaunchKernelGGL(gen_expand_kernel, dim3(1), dim3(64), 0, s, p, local, child_moves);
}
void launch_gen_backup(const GenParams &p, int nb, const double *values, hipStream_t s) {
    hipLaunchKernelGGL(gen_backup_kernel, dim3(1), dim3(64), 0, s, p, nb, values);
}
void launch_gen_end(const GenParams &p, int32_t *out, int32_t *root_na, int na_cap, hipStream_t s) {
    hipLaunchKernelGGL(gen_end_kernel, dim3(1), dim3(64), 0, s, p, out, root_na, na_cap);
}

}  // namespace zc
