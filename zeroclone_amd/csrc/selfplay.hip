// selfplay.hip — device-resident self-play trajectories.
//
// Replaces the host side of the reference's self-play data path:
//   Engine.play_move's history append (engine/engine.py:98-108),
//   Engine.get_dataset (engine.py:60-89): each finished game's positions with side-to-move
//     labels — factor 0 (draw) or -1, alternating in sign, the game's list REVERSED, so
//     position i of an n-position game gets f * (-1)^(n-1-i),
//   scripts/train.py:simulate_games (:151-170): a finished game's slot starts a new game only
//     while fewer than the quota have started; every started game is played to its end.
//
// One thread per game slot.  Each slot keeps its current game's positions (opening first) in
// HBM; when the game ends the slot takes its place in the pool (prefix sums over the slots,
// so the layout is deterministic) and copies the game out — positions, labels, the move
// played from each position, and one game record — then restarts from the opening (or goes
// idle when the quota is spent).  Rows are
// opaque byte records (zc_c4_state: 24 B, zc_chess_state: 72 B), copied 8 bytes at a time.
#include "zc_internal.h"

namespace zc {
namespace {

constexpr int kRecThreads = 1024;

// Exclusive prefix sums over the workgroup of two counters at once (x: games, y: positions);
// returns the workgroup totals in tx / ty.
__device__ __forceinline__ void block_scan2(int &x, long long &y, int &tx, long long &ty) {
    __shared__ int s_x[kRecThreads / 64];
    __shared__ long long s_y[kRecThreads / 64];
    const int lane = (int)(threadIdx.x & 63), wv = (int)(threadIdx.x >> 6);
    int ix = x;
    long long iy = y;
    for (int o = 1; o < 64; o <<= 1) {
        const int ux = __shfl_up(ix, o);
        const long long uy = __shfl_up(iy, o);
        if (lane >= o) {
            ix += ux;
            iy += uy;
        }
    }
    if (lane == 63) {
        s_x[wv] = ix;
        s_y[wv] = iy;
    }
    __syncthreads();
    int bx = 0;
    long long by = 0;
    tx = 0;
    ty = 0;
    for (int w = 0; w < kRecThreads / 64; ++w) {
        if (w < wv) {
            bx += s_x[w];
            by += s_y[w];
        }
        tx += s_x[w];
        ty += s_y[w];
    }
    x = bx + ix - x;
    y = by + iy - y;
    __syncthreads();
}

// Pass 1 — one workgroup walks the slots 1024 at a time, so games that end in the same step
// get their game numbers and pool places in slot order (deterministic; the reference refills
// in the order its finished games are listed, train.py:160-167).  Per slot: the result, the
// append, and for a finished game its game record, its pool place (slot[2]) and length
// (slot[3], 0 = nothing to copy), the refill of the slot.  The copy is pass 2.
__global__ __launch_bounds__(kRecThreads) void traj_record_kernel(int n, zc_traj_buffers b, uint8_t *states,
                                                                  const int16_t *moves, int32_t *results,
                                                                  const int32_t *flags, const int32_t *rep) {
    const int W = b.row_bytes / 8;
    const uint64_t *init = (const uint64_t *)b.d_init;
    long long pos_base = b.d_ctl[kTrajPositions], game_base = b.d_ctl[kTrajGames], next = b.d_ctl[kTrajNext];
    long long finished = b.d_ctl[kTrajFinished];
    const long long quota = b.d_ctl[kTrajQuota];
    int overflow = 0;
    __syncthreads();
    for (int c0 = 0; c0 < n; c0 += kRecThreads) {
        const int g = c0 + (int)threadIdx.x;
        int fin = 0, len = 0, r = ZC_C4_ONGOING, game = -1;
        int32_t *slot = b.d_slot + 4 * (size_t)(g < n ? g : 0);
        uint64_t *row = (uint64_t *)(states + (size_t)(g < n ? g : 0) * b.row_bytes);
        if (g < n) {
            game = slot[1];
            if (game >= 0 && !flags && results[g] == ZC_SLOT_SKIP) {
                game = -2;  // pooled self-play: no move on this slot at this step, left as it is
                slot[3] = 0;
            } else if (game < 0) {  // idle slot (quota spent): held at the opening, nothing recorded
                for (int k = 0; k < W; ++k) row[k] = init[k];
                results[g] = ZC_SLOT_IDLE;
                slot[3] = 0;
            } else {
                if (flags) {
                    // chess: Engine._evaluate (engine.py:148-153) of the position after the
                    // move — check_win -> turn*2-1 (turn = side to move now), check_draw -> 0
                    // (stalemate, the fifty-move rule, or both sides' histories repeating)
                    const int turn = ((const uint8_t *)row)[64];
                    const int f = flags[g];
                    if (f & ZC_CHESS_WIN) r = turn * 2 - 1;
                    else if ((f & (ZC_CHESS_STALEMATE | ZC_CHESS_FIFTY)) || (rep && rep[g] == 3)) r = 0;
                    results[g] = r;
                } else {
                    r = results[g];
                }
                len = slot[0];
                if (len >= b.max_len) {  // longer than the slot holds: flagged
                    overflow |= 2;
                    len = b.max_len - 1;
                }
                uint64_t *hist = (uint64_t *)b.d_hist + ((size_t)g * b.max_len + len) * W;
                for (int k = 0; k < W; ++k) hist[k] = row[k];
                b.d_hmoves[(size_t)g * b.max_len + len - 1] = moves[g];
                ++len;
                fin = r != ZC_C4_ONGOING;
            }
        }
        int gi = fin;
        long long off = fin ? len : 0;
        int tg;
        long long tp;
        block_scan2(gi, off, tg, tp);
        if (g < n && game >= 0) {
            int copy = 0;
            if (fin) {
                const long long G = game_base + gi, P = pos_base + off;
                if (P + len > b.pool_cap || G >= b.games_cap) {  // dropped: no pass-2 copy
                    overflow |= 1;
                    uint64_t *h0 = (uint64_t *)b.d_hist + (size_t)g * b.max_len * W;
                    for (int k = 0; k < W; ++k) h0[k] = init[k];
                } else {
                    int64_t *rec = b.d_games + 4 * (size_t)G;
                    rec[0] = game;
                    rec[1] = ((int64_t)g << 32) | (uint32_t)(r + 1);  // slot | result + 1
                    rec[2] = P;
                    rec[3] = len;
                    slot[2] = (int32_t)P;
                    copy = len;
                }
                // the refill (train.py:165-167): a new game while fewer than `quota` started
                const long long nx = next + gi;
                slot[1] = nx < quota ? (int)nx : -1;
                for (int k = 0; k < W; ++k) row[k] = init[k];
                len = 1;
            }
            slot[0] = len;
            slot[3] = copy | (r == 0 ? 0 : (int)0x80000000);  // length to copy; bit 31: decisive
        }
        pos_base += tp;
        game_base += tg;
        next += tg;
        finished += tg;
    }
    const int ov = (__syncthreads_or(overflow & 1) ? 1 : 0) | (__syncthreads_or(overflow & 2) ? 2 : 0);
    if (threadIdx.x == 0) {
        b.d_ctl[kTrajPositions] = pos_base;
        b.d_ctl[kTrajGames] = game_base;
        b.d_ctl[kTrajNext] = next;
        b.d_ctl[kTrajFinished] = finished;
        b.d_ctl[kTrajOverflow] |= ov;
    }
}

// Pass 2 — one thread per (slot, position): a finished game's positions, labels and moves
// to its pool place (get_dataset: position i of n gets f * (-1)^(n-1-i), f = 0 for a draw,
// -1 otherwise); position 0's thread then restarts the slot's history at the opening.
__global__ void traj_copy_kernel(int n, zc_traj_buffers b) {
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const int g = (int)(t / b.max_len), i = (int)(t % b.max_len);
    if (g >= n) return;
    const int32_t *slot = b.d_slot + 4 * (size_t)g;
    const int s3 = slot[3];
    const int len = s3 & 0x7FFFFFFF;
    if (i >= len) return;
    const int W = b.row_bytes / 8;
    const long long P = slot[2] + (long long)i;
    uint64_t *hist = (uint64_t *)b.d_hist + ((size_t)g * b.max_len + i) * W;
    uint64_t *pool = (uint64_t *)b.d_pool + (size_t)P * W;
    for (int k = 0; k < W; ++k) pool[k] = hist[k];
    const int f0 = s3 < 0 ? -1 : 0;
    b.d_labels[P] = ((len - 1 - i) & 1) ? -f0 : f0;
    b.d_pool_moves[P] = i + 1 < len ? b.d_hmoves[(size_t)g * b.max_len + i] : (int16_t)-1;
    if (i == 0) {
        const uint64_t *init = (const uint64_t *)b.d_init;
        for (int k = 0; k < W; ++k) hist[k] = init[k];
    }
}

// ---------------------------------------------------------------- multi-step record
// The K steps of one self-play launch recorded at once.  Single steps number the games that
// finish in step k after every game of steps < k, in slot order inside a step, and give each
// its pool place in the same order; so a game's number and place are exclusive prefix sums
// over the [K][n] grid in step-major order — of 1 per finished game and of its length.
// Kernels: (A) one wave per slot, lane = step: the finished games' lengths fl[k][n] (and the
// slot's moves played); (B) one workgroup per step: the scan of its row; (C) one workgroup:
// the scan of the row totals, the counters' bases and their update; (D) one wave per slot:
// each finished game's record and positions, labels and moves to its pool place, then the
// unfinished game's new positions appended to the slot's history.
struct StepScratch {
    int32_t *fl, *exg, *exp, *played;   // [K][n], [K][n], [K][n], [n]
    int64_t *rowtot, *rowpre, *base;    // [K][2], [K][2], [4]
};

__host__ __device__ inline size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

__host__ __device__ inline size_t steps_scratch_layout(int n, int K, uint8_t *p, StepScratch *sc) {
    size_t o = 0;
    const size_t kn = (size_t)K * n * sizeof(int32_t);
    if (sc) sc->fl = (int32_t *)(p + o);
    o = align16(o + kn);
    if (sc) sc->exg = (int32_t *)(p + o);
    o = align16(o + kn);
    if (sc) sc->exp = (int32_t *)(p + o);
    o = align16(o + kn);
    if (sc) sc->played = (int32_t *)(p + o);
    o = align16(o + (size_t)n * sizeof(int32_t));
    if (sc) sc->rowtot = (int64_t *)(p + o);
    o = align16(o + (size_t)K * 2 * sizeof(int64_t));
    if (sc) sc->rowpre = (int64_t *)(p + o);
    o = align16(o + (size_t)K * 2 * sizeof(int64_t));
    if (sc) sc->base = (int64_t *)(p + o);
    return o + 4 * sizeof(int64_t);
}

__device__ __forceinline__ int steps_reached(int K, const int32_t *reached) {
    return reached ? min(K, max(*reached, 0)) : K;
}

constexpr int kSlotWaves = 4;

// (A) lane = step.  A slot's moves are the steps before its first ZC_SLOT_SKIP; a game that
// ends at step k has the positions since the previous finish (opening included) or, for the
// slot's game in progress at the launch's start, its history plus steps 0..k.
__global__ __launch_bounds__(kSlotWaves * 64) void traj_steps_lens_kernel(int n, int K, const int32_t *reached,
                                                                          const int32_t *slot,
                                                                          const int32_t *results, StepScratch sc) {
    const int lane = (int)(threadIdx.x & 63);
    const int g = (int)(blockIdx.x * kSlotWaves + (threadIdx.x >> 6));
    if (g >= n) return;
    const int Kr = steps_reached(K, reached);
    int lenc = slot[4 * (size_t)g];
    bool stopped = slot[4 * (size_t)g + 1] < 0;  // idle slot: nothing recorded
    int m = 0;
    for (int c0 = 0; c0 < Kr; c0 += 64) {
        const int k = c0 + lane;
        const bool valid = k < Kr;
        const int r = (valid && !stopped) ? results[(size_t)k * n + g] : ZC_SLOT_SKIP;
        const unsigned long long skip = __ballot(r == ZC_SLOT_SKIP);
        const int first_skip = skip ? __ffsll((long long)skip) - 1 : 64;
        const unsigned long long played = first_skip == 64 ? ~0ull : ((1ull << first_skip) - 1);
        const unsigned long long fin = __ballot(r != ZC_C4_ONGOING && r != ZC_SLOT_SKIP) & played;
        const unsigned long long prev = fin & ((1ull << lane) - 1);
        int L = 0;
        if ((fin >> lane) & 1) L = prev ? lane - (63 - __clzll((long long)prev)) + 1 : lenc + lane + 1;
        if (valid) sc.fl[(size_t)k * n + g] = L;
        const int np = __popcll(played);
        lenc = fin ? np - (63 - __clzll((long long)fin)) : lenc + np;
        m += np;
        stopped = stopped || first_skip < 64;
    }
    if (lane == 0) sc.played[g] = m;
}

// (B) one workgroup per step: exclusive prefixes of (finished, length) along the row.
__global__ __launch_bounds__(kRecThreads) void traj_steps_rows_kernel(int n, int K, const int32_t *reached,
                                                                      StepScratch sc) {
    const int k = (int)blockIdx.x;
    if (k >= steps_reached(K, reached)) return;
    const size_t row = (size_t)k * n;
    int gbase = 0;
    long long pbase = 0;
    for (int c0 = 0; c0 < n; c0 += kRecThreads) {
        const int g = c0 + (int)threadIdx.x;
        const int L = g < n ? sc.fl[row + g] : 0;
        int x = L > 0;
        long long y = L;
        int tx;
        long long ty;
        block_scan2(x, y, tx, ty);
        if (g < n) {
            sc.exg[row + g] = gbase + x;
            sc.exp[row + g] = (int32_t)(pbase + y);
        }
        gbase += tx;
        pbase += ty;
    }
    if (threadIdx.x == 0) {
        sc.rowtot[2 * k] = gbase;
        sc.rowtot[2 * k + 1] = pbase;
    }
}

// (C) one workgroup: the rows' exclusive prefixes, the counters' bases (for D) and their update.
__global__ __launch_bounds__(kRecThreads) void traj_steps_totals_kernel(int K, const int32_t *reached,
                                                                        zc_traj_buffers b, StepScratch sc) {
    const int Kr = steps_reached(K, reached);
    long long gb = 0, pb = 0;
    for (int c0 = 0; c0 < Kr; c0 += kRecThreads) {
        const int k = c0 + (int)threadIdx.x;
        int x = k < Kr ? (int)sc.rowtot[2 * k] : 0;
        long long y = k < Kr ? sc.rowtot[2 * k + 1] : 0;
        int tx;
        long long ty;
        block_scan2(x, y, tx, ty);
        if (k < Kr) {
            sc.rowpre[2 * k] = gb + x;
            sc.rowpre[2 * k + 1] = pb + y;
        }
        gb += tx;
        pb += ty;
    }
    if (threadIdx.x == 0) {
        sc.base[0] = b.d_ctl[kTrajPositions];
        sc.base[1] = b.d_ctl[kTrajGames];
        sc.base[2] = b.d_ctl[kTrajNext];
        sc.base[3] = b.d_ctl[kTrajQuota];
        b.d_ctl[kTrajPositions] += pb;
        b.d_ctl[kTrajGames] += gb;
        b.d_ctl[kTrajNext] += gb;
        b.d_ctl[kTrajFinished] += gb;
    }
}

// (D) one wave per slot.  Game `first` (in progress at the launch's start) has its first h =
// slot[0] positions in the slot's history; a later game starts at the opening (h = 1).
// Position i >= h of a game whose first step is bs came from step bs + i - h; the move from
// position i is the one that made position i + 1.
__global__ __launch_bounds__(kSlotWaves * 64) void traj_steps_copy_kernel(int n, int K, const int32_t *reached,
                                                                          zc_traj_buffers b, const uint8_t *states,
                                                                          const int16_t *moves,
                                                                          const int32_t *results, StepScratch sc) {
    const int lane = (int)(threadIdx.x & 63);
    const int g = (int)(blockIdx.x * kSlotWaves + (threadIdx.x >> 6));
    if (g >= n) return;
    int32_t *slot = b.d_slot + 4 * (size_t)g;
    int game = slot[1];
    if (game < 0) return;
    const int W = b.row_bytes / 8;
    const long long pos0 = sc.base[0], games0 = sc.base[1], next0 = sc.base[2], quota = sc.base[3];
    const uint64_t *init = (const uint64_t *)b.d_init;
    uint64_t *hist = (uint64_t *)b.d_hist + (size_t)g * b.max_len * W;
    int16_t *hmv = b.d_hmoves + (size_t)g * b.max_len;
    const int m = sc.played[g];
    int h = slot[0], bs = 0, ov = 0;
    bool first = true;
    for (int c0 = 0; c0 < m && game >= 0; c0 += 64) {
        const int k = c0 + lane;
        const int Lv = k < m ? sc.fl[(size_t)k * n + g] : 0;
        unsigned long long fin = __ballot(Lv > 0);
        while (fin && game >= 0) {
            const int j = __ffsll((long long)fin) - 1;
            fin &= fin - 1;
            const int kk = c0 + j;
            const size_t e = (size_t)kk * n + g;
            const int L = __shfl(Lv, j);
            const long long gi = sc.rowpre[2 * kk] + sc.exg[e];
            const long long G = games0 + gi, P = pos0 + sc.rowpre[2 * kk + 1] + sc.exp[e];
            const int r = results[e];
            if (L > b.max_len) ov |= 2;
            if (P + L > b.pool_cap || G >= b.games_cap) {
                ov |= 1;  // dropped
            } else {
                if (lane == 0) {
                    int64_t *rec = b.d_games + 4 * (size_t)G;
                    rec[0] = game;
                    rec[1] = ((int64_t)g << 32) | (uint32_t)(r + 1);
                    rec[2] = P;
                    rec[3] = L;
                }
                const int f0 = r == 0 ? 0 : -1;
                for (int i = lane; i < L; i += 64) {
                    const uint64_t *src = i < h ? (first ? hist + (size_t)i * W : init)
                                                : (const uint64_t *)(states + ((size_t)(bs + i - h) * n + g) * b.row_bytes);
                    uint64_t *dst = (uint64_t *)b.d_pool + (size_t)(P + i) * W;
                    for (int w = 0; w < W; ++w) dst[w] = src[w];
                    b.d_labels[P + i] = ((L - 1 - i) & 1) ? -f0 : f0;
                    b.d_pool_moves[P + i] = i + 1 >= L ? (int16_t)-1
                                            : (i + 1 < h ? hmv[i] : moves[(size_t)(bs + i + 1 - h) * n + g]);
                }
            }
            // the refill (train.py:165-167), numbered as single steps number it
            const long long nx = next0 + gi;
            if (nx < quota) {
                game = (int)nx;
            } else {
                game = -1;
                ov |= 4;
            }
            first = false;
            h = 1;
            bs = kk + 1;
        }
    }
    // the game in progress: its positions since bs appended to the history
    if (!first)
        for (int w = lane; w < W; w += 64) hist[w] = init[w];
    const int cnt = game >= 0 ? m - bs : 0;
    for (int t = lane; t < cnt; t += 64) {
        const int idx = h + t;
        if (idx >= b.max_len) {
            ov |= 2;
            continue;
        }
        const uint64_t *src = (const uint64_t *)(states + ((size_t)(bs + t) * n + g) * b.row_bytes);
        for (int w = 0; w < W; ++w) hist[(size_t)idx * W + w] = src[w];
        hmv[idx - 1] = moves[(size_t)(bs + t) * n + g];
    }
    ov = (__ballot(ov & 1) ? 1 : 0) | (__ballot(ov & 2) ? 2 : 0) | (__ballot(ov & 4) ? 4 : 0);
    if (lane == 0) {
        slot[0] = min(h + cnt, b.max_len);
        slot[1] = game;
        if (ov) atomicOr((unsigned long long *)(b.d_ctl + kTrajOverflow), (unsigned long long)ov);
    }
}

}  // namespace

size_t traj_steps_scratch_bytes(int n, int K) { return steps_scratch_layout(n, K, nullptr, nullptr); }

void launch_traj_record_steps(int n, int K, const zc_traj_buffers &b, const void *states, const int16_t *moves,
                              const int32_t *results, const int32_t *reached, void *scratch, hipStream_t s) {
    StepScratch sc;
    steps_scratch_layout(n, K, (uint8_t *)scratch, &sc);
    const dim3 slots((unsigned)((n + kSlotWaves - 1) / kSlotWaves)), wb(kSlotWaves * 64);
    hipLaunchKernelGGL(traj_steps_lens_kernel, slots, wb, 0, s, n, K, reached, (const int32_t *)b.d_slot, results, sc);
    hipLaunchKernelGGL(traj_steps_rows_kernel, dim3((unsigned)K), dim3(kRecThreads), 0, s, n, K, reached, sc);
    hipLaunchKernelGGL(traj_steps_totals_kernel, dim3(1), dim3(kRecThreads), 0, s, K, reached, b, sc);
    hipLaunchKernelGGL(traj_steps_copy_kernel, slots, wb, 0, s, n, K, reached, b, (const uint8_t *)states, moves,
                       results, sc);
}

void launch_traj_record(int n, const zc_traj_buffers &b, void *states, const int16_t *moves, int32_t *results,
                        const int32_t *flags, const int32_t *rep, hipStream_t s) {
    hipLaunchKernelGGL(traj_record_kernel, dim3(1), dim3(kRecThreads), 0, s, n, b, (uint8_t *)states, moves, results,
                       flags, rep);
    const long long threads = (long long)n * b.max_len;
    hipLaunchKernelGGL(traj_copy_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, n, b);
}

}  // namespace zc
