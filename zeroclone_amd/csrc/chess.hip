// chess.hip — batched chess rules on the GPU (engine/games/chess/src/chess_backend.cpp):
// get_legal_moves, play_move, check_win / the non-history part of check_draw, state_to_tensor
// and the fused "children" expansion used by perft and by tree expansion.  One wave per
// position for move generation (chess_device.h), one thread per position or square for the
// elementwise kernels.
#include <hip/hip_fp16.h>

#include "chess_device.h"
#include "zc_internal.h"

namespace zc {
namespace {

using namespace chessdev;

__device__ __forceinline__ void load_board(uint8_t *sb, const zc_chess_state &s) {
    sb[lane()] = s.board[lane()];
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

__global__ __launch_bounds__(64) void chess_legal_kernel(int n, const zc_chess_state *states, uint16_t *moves,
                                                        int32_t *counts) {
    __shared__ ChessScratch S;
    const int i = blockIdx.x;
    if (i >= n) return;
    load_board(S.board, states[i]);
    const int t = __builtin_amdgcn_readfirstlane(states[i].turn);
    const int k = legal_moves(S.board, t, S.legal, S.pseudo, S.region);
    for (int j = (int)lane(); j < k; j += 64) moves[(size_t)i * kMaxLegal + j] = S.legal[j];
    if (lane() == 0) counts[i] = k;
}

// Every legal move applied: children[i][j] = play_move(states[i], legal move j).
__global__ __launch_bounds__(64) void chess_children_kernel(int n, const zc_chess_state *states,
                                                           zc_chess_state *children, uint16_t *moves,
                                                           int32_t *counts) {
    __shared__ ChessScratch S;
    const int i = blockIdx.x;
    if (i >= n) return;
    const zc_chess_state st = states[i];
    load_board(S.board, st);
    const int t = __builtin_amdgcn_readfirstlane(st.turn);
    const int k = legal_moves(S.board, t, S.legal, S.pseudo, S.region);
    if (lane() == 0) counts[i] = k;
    for (int j = (int)lane(); j < k; j += 64) {
        zc_chess_state c = st;
        apply_move(c, S.legal[j]);
        children[(size_t)i * kMaxLegal + j] = c;
        if (moves) moves[(size_t)i * kMaxLegal + j] = S.legal[j];
    }
}

__global__ void chess_play_kernel(int n, const zc_chess_state *in, const uint16_t *moves, zc_chess_state *out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    zc_chess_state s = in[i];
    apply_move(s, moves[i]);
    out[i] = s;
}

// check_win (:404-412): no legal move and the side to move is in check; check_draw
// (:416-441) minus the history test: stalemate, or fifty counter >= 50.
__global__ __launch_bounds__(64) void chess_terminal_kernel(int n, const zc_chess_state *states, int32_t *flags) {
    __shared__ ChessScratch S;
    const int i = blockIdx.x;
    if (i >= n) return;
    const zc_chess_state st = states[i];
    load_board(S.board, st);
    const int t = __builtin_amdgcn_readfirstlane(st.turn);
    bool check;
    const int k = legal_moves_check(S.board, t, S.legal, S.pseudo, S.region, check);
    if (lane() == 0) {
        int f = 0;
        if (k == 0 && check) f |= ZC_CHESS_WIN;
        if (k == 0 && !check) f |= ZC_CHESS_STALEMATE;
        if (st.fifty >= 50) f |= ZC_CHESS_FIFTY;
        if (k < 0) f |= ZC_CHESS_OVERFLOW;
        flags[i] = f;
    }
}

// legal_moves_probe (the crude search's lazy nodes, chess_device.h): out[i] = -2 when the
// probe proved the position has a legal move without generating its list, else the length
// of the list it generated (-1: overflow).  Diagnostic / parity-test entry point.
__global__ __launch_bounds__(64) void chess_probe_kernel(int n, const zc_chess_state *states, int32_t *out) {
    __shared__ ChessScratch S;
    const int i = blockIdx.x;
    if (i >= n) return;
    load_board(S.board, states[i]);
    const int t = __builtin_amdgcn_readfirstlane(states[i].turn);
    bool check, lazy;
    const int k = legal_moves_probe(S.board, S.board[lane()], t, S.legal, S.pseudo, S.region, check, lazy);
    if (lane() == 0) out[i] = lazy ? -2 : k;
}

// has_repeated_prefix (:148-180) of both sides' move histories (chess_device.h::repetitions):
// hist[i][side][k] = that side's k-th move in play order (k < len[i][side] <= cap); out[i] =
// white's answer | black's << 1.  One wave per position, the history staged in LDS.
__global__ __launch_bounds__(64) void chess_repetition_kernel(int n, int cap, const uint16_t *hist, const int32_t *len,
                                                             int32_t *out) {
    __shared__ uint16_t Lh[kMaxHistory];
    const int i = blockIdx.x;
    if (i >= n) return;
    const int res = repetitions(hist + (size_t)i * 2 * cap, len + 2 * i, cap, Lh);
    if (lane() == 0) out[i] = res;
}

// state_to_tensor (:461-521): [17][8][8], planes 0-11 = PNBRQK pnbrqk, 12 = white to move,
// 13-16 = w_ck, w_cq, b_ck, b_cq.  One thread per (position, square).
__global__ void chess_planes_kernel(int n, const zc_chess_state *states, void *planes, int f16) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= (int64_t)n * 64) return;
    const int i = (int)(g >> 6), sq = (int)(g & 63);
    const zc_chess_state &s = states[i];
    const uint8_t pc = s.board[sq];
    const char pieces[12] = {'P', 'N', 'B', 'R', 'Q', 'K', 'p', 'n', 'b', 'r', 'q', 'k'};
    int which = -1;
    for (int k = 0; k < 12; ++k)
        if (pc == (uint8_t)pieces[k]) {
            which = k;
            break;
        }
    for (int k = 0; k < 17; ++k) {
        float v;
        if (k < 12) v = k == which ? 1.0f : 0.0f;
        else if (k == 12) v = s.turn == 0 ? 1.0f : 0.0f;
        else v = (s.castle >> (k - 13)) & 1 ? 1.0f : 0.0f;
        const size_t o = ((size_t)i * 17 + k) * 64 + sq;
        if (f16) ((__half *)planes)[o] = __float2half(v);
        else ((float *)planes)[o] = v;
    }
}

}  // namespace

void launch_chess_legal(int n, const zc_chess_state *s, uint16_t *moves, int32_t *counts, hipStream_t st) {
    hipLaunchKernelGGL(chess_legal_kernel, dim3(n), dim3(64), 0, st, n, s, moves, counts);
}
void launch_chess_probe(int n, const zc_chess_state *s, int32_t *out, hipStream_t st) {
    hipLaunchKernelGGL(chess_probe_kernel, dim3(n), dim3(64), 0, st, n, s, out);
}
void launch_chess_children(int n, const zc_chess_state *s, zc_chess_state *children, uint16_t *moves,
                           int32_t *counts, hipStream_t st) {
    hipLaunchKernelGGL(chess_children_kernel, dim3(n), dim3(64), 0, st, n, s, children, moves, counts);
}
void launch_chess_play(int n, const zc_chess_state *in, const uint16_t *moves, zc_chess_state *out, hipStream_t st) {
    hipLaunchKernelGGL(chess_play_kernel, dim3((n + 127) / 128), dim3(128), 0, st, n, in, moves, out);
}
void launch_chess_terminal(int n, const zc_chess_state *s, int32_t *flags, hipStream_t st) {
    hipLaunchKernelGGL(chess_terminal_kernel, dim3(n), dim3(64), 0, st, n, s, flags);
}
bool launch_chess_repetition(int n, int cap, const uint16_t *hist, const int32_t *len, int32_t *out, hipStream_t st) {
    if (cap < 1 || cap > kMaxHistory) return false;
    hipLaunchKernelGGL(chess_repetition_kernel, dim3(n), dim3(64), 0, st, n, cap, hist, len, out);
    return true;
}
void launch_chess_planes(int n, const zc_chess_state *s, void *planes, int f16, hipStream_t st) {
    const int64_t total = (int64_t)n * 64;
    hipLaunchKernelGGL(chess_planes_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, n, s, planes, f16);
}

}  // namespace zc
