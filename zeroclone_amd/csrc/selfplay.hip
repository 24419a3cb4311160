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
                                                                  const int32_t *flags, const int32_t *rep,
                                                                  const int32_t *reached, int step) {
    if (reached && step >= *reached) return;  // a pooled run's step no game reached (whole block)
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
__global__ void traj_copy_kernel(int n, zc_traj_buffers b, const int32_t *reached, int step) {
    if (reached && step >= *reached) return;
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

}  // namespace

void launch_traj_record(int n, const zc_traj_buffers &b, void *states, const int16_t *moves, int32_t *results,
                        const int32_t *flags, const int32_t *rep, hipStream_t s, const int32_t *reached, int step) {
    hipLaunchKernelGGL(traj_record_kernel, dim3(1), dim3(kRecThreads), 0, s, n, b, (uint8_t *)states, moves, results,
                       flags, rep, reached, step);
    const long long threads = (long long)n * b.max_len;
    hipLaunchKernelGGL(traj_copy_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, n, b, reached,
                       step);
}

}  // namespace zc
