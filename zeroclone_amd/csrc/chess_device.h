// chess_device.h — the reference's chess rules (engine/games/chess/src/chess_backend.cpp)
// as wave-level device functions for gfx950, shared by the chess kernels (chess.hip) and the
// chess tree search.
//
// Execution model: ONE POSITION PER WAVE, ONE SQUARE PER LANE.  The board stays in the
// reference's byte encoding (64 chars: ' ' empty, "PNBRQK" white, "pnbrqk" black, index 0 =
// a8) in LDS, so every quirk of the reference — unknown characters, missing kings — behaves
// identically.  get_legal_moves (:184-360) becomes:
//   1. lane s counts the pseudo-legal moves of the piece on square s (reference order:
//      pawn push / double push / captures dc=-1,+1; knight, bishop, rook, queen, king
//      direction tables :17-34), an exclusive prefix sum over lanes gives each square its
//      slot range — board-scan order is lane order — and lane s writes its moves there;
//   2. lanes take the pseudo-legal moves 64 at a time and test the mover's king on the
//      board after the move (:345-359) by reading LDS through a from/to override;
//   3. ballot + mbcnt compact the legal moves, preserving order.
// A move is packed in 16 bits: from square | to square << 6 | capture value << 12
// (fabs(piece_val) of the captured piece: 0, 1, 3, 5 or 9).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/zeroclone.h"

#ifndef CDEV_T  // diagnostic phase stamps (chess_tree.h under ZC_CHESS_STAMP); no-ops otherwise
#define CDEV_T(v)
#define CDEV_ADD(k, t0)
#endif

namespace zc {
namespace chessdev {
namespace {

constexpr int kMaxLegal = 256;   // the output capacity per position (real chess: <= 218)
constexpr int kMaxPseudo = 512;  // pseudo-legal scratch per position
constexpr int kMaxHistory = 4096;  // moves per side the repetition test takes
constexpr int kRegion = 28;     // per-lane generation region (a queen has <= 27 moves)

__device__ __forceinline__ uint32_t lane() { return __lane_id(); }

__device__ __forceinline__ bool empty_sq(uint32_t x) { return x == ' ' || x == 0; }
__device__ __forceinline__ bool is_white(uint32_t x) { return x >= 'A' && x <= 'Z'; }
__device__ __forceinline__ uint32_t upper(uint32_t x) { return (x >= 'a' && x <= 'z') ? x - 32u : x; }
__device__ __forceinline__ bool enemy(uint32_t x, int t) { return !empty_sq(x) && (t == 0 ? !is_white(x) : is_white(x)); }
__device__ __forceinline__ uint32_t piece_value(uint32_t x) {
    switch (upper(x)) {
        case 'P': return 1;
        case 'N': return 3;
        case 'B': return 3;
        case 'R': return 5;
        case 'Q': return 9;
        default: return 0;  // K (100) never appears as a capture
    }
}
__device__ __forceinline__ bool inb(int r, int c) { return (unsigned)r < 8u && (unsigned)c < 8u; }

// direction tables (chess_backend.cpp:17-34), compile-time constants: the loops over them
// are unrolled, so offsets become immediates instead of constant-memory loads
struct Dir {
    int dr, dc;
};
constexpr Dir kKnight[8] = {{-2, -1}, {-2, 1}, {-1, -2}, {-1, 2}, {1, -2}, {1, 2}, {2, -1}, {2, 1}};
constexpr Dir kAll8[8] = {{-1, -1}, {-1, 1}, {1, -1}, {1, 1}, {-1, 0}, {1, 0}, {0, -1}, {0, 1}};
// bishops use kAll8[0..4), rooks kAll8[4..8), queens and kings kAll8[0..8)

__device__ __forceinline__ uint32_t pack_move(int from, int to, uint32_t v) {
    return (uint32_t)from | ((uint32_t)to << 6) | (v << 12);
}

// Two views of the board answer the generator's and the legality test's questions:
//   ByteView: the reference's bytes in LDS, any character (unknown pieces, missing kings);
//   BitView:  uniform 64-bit masks built by ballots, used when every square holds one of
//             " PNBRQKpnbrqk" (or 0) and the mover has a king — every reachable position.
// Probes then become bit tests in registers instead of dependent LDS reads, and the check
// test is a handful of shifts and bit scans per ray instead of a walk square by square.
// probe(s): -2 empty; -1 not capturable (own piece, enemy king, unknown white/black char);
// otherwise the capture value fabs(piece_val) of the enemy piece on s.
struct ByteView {
    static constexpr bool kCheapProbe = false;  // probes are LDS reads
    const uint8_t *b;
    int t;
    __device__ __forceinline__ int probe(int s) const {
        const uint32_t x = b[s];
        if (empty_sq(x)) return -2;
        return (enemy(x, t) && upper(x) != 'K') ? (int)piece_value(x) : -1;
    }
    __device__ __forceinline__ uint32_t piece_at(int s) const { return b[s]; }
    __device__ __forceinline__ bool attacked(int k, int from, int to, uint32_t pc) const;
};

constexpr uint64_t kFileA = 0x0101010101010101ull;
constexpr uint64_t kNotA = ~kFileA, kNotH = ~(kFileA << 7);
constexpr uint64_t kNotAB = ~(kFileA | (kFileA << 1)), kNotGH = ~((kFileA << 6) | (kFileA << 7));
constexpr uint64_t kDiag = 0x8040201008040201ull;  // squares (i, i)
constexpr uint64_t kAnti = 0x0102040810204080ull;  // squares (i, 7 - i)
// A knight's / king's targets from square s as ONE signed shift of the pattern of a square
// whose targets do not wrap (knight: square 18 = (2, 2); king: square 9 = (1, 1)), the files
// a shift wraps into masked off (exhaustively equal to the eight masked shifts of kb).
constexpr uint64_t kKnight18 = 0xA1100110Aull, kKing9 = 0x70507ull;
__device__ __forceinline__ uint64_t shift_signed(uint64_t p, int d) { return d >= 0 ? p << d : p >> -d; }
__device__ __forceinline__ uint64_t knight_targets(int s) {
    const int c = s & 7;
    return shift_signed(kKnight18, s - 18) & (c < 2 ? kNotGH : c > 5 ? kNotAB : ~0ull);
}
__device__ __forceinline__ uint64_t king_targets(int s) {
    const int c = s & 7;
    return shift_signed(kKing9, s - 9) & (c == 0 ? kNotH : c == 7 ? kNotA : ~0ull);
}

struct BitView {
    static constexpr bool kCheapProbe = true;  // generation from masks (bit_piece_moves)
    uint64_t occ;              // non-empty squares
    uint64_t cap;              // capturable: the enemy's pieces other than kings
    uint64_t tP, tNB, tR;      // piece types (either colour), for capture values
    uint64_t eP, eN, eBQ, eRQ, eK;  // the enemy's attackers of the mover's king
    uint64_t kings;            // the mover's kings
    int t;
    __device__ __forceinline__ int probe(int s) const {
        if (!((occ >> s) & 1ull)) return -2;
        if (!((cap >> s) & 1ull)) return -1;
        return ((tP >> s) & 1ull) ? 1 : ((tNB >> s) & 1ull) ? 3 : ((tR >> s) & 1ull) ? 5 : 9;
    }
    __device__ __forceinline__ uint32_t piece_at(int s) const {  // only "is it the mover's king" is asked
        return ((kings >> s) & 1ull) ? (t == 0 ? 'K' : 'k') : 0u;
    }
    // the capture value of a move to `to` (0 when nothing capturable stands there)
    __device__ __forceinline__ uint32_t capval(int to) const {
        if (!((cap >> to) & 1ull)) return 0u;
        return ((tP >> to) & 1ull) ? 1u : ((tNB >> to) & 1ull) ? 3u : ((tR >> to) & 1ull) ? 5u : 9u;
    }
    // king_attacked (:85-144) for the mover's king on square k (0..63) after the piece on
    // `from` moved to `to` (-1, -1: the position as it stands): the moved piece is the
    // mover's, so it only blocks; the enemy piece it captured, if any, no longer attacks.
    __device__ __forceinline__ bool attacked(int k, int from, int to, uint32_t) const {
        const uint64_t fb = from >= 0 ? (1ull << from) : 0ull, tb = to >= 0 ? (1ull << to) : 0ull;
        const uint64_t keep = ~tb;
        const uint64_t o = (occ & ~fb) | tb;
        const uint64_t kb = 1ull << k;
        const uint64_t pawns = t == 0 ? (((kb >> 9) & kNotH) | ((kb >> 7) & kNotA))
                                      : (((kb << 7) & kNotH) | ((kb << 9) & kNotA));
        const uint64_t knights = knight_targets(k), king = king_targets(k);
        const bool leap = (((pawns & eP) | (knights & eN) | (king & eK)) & keep) != 0ull;
        // sliders: the nearest occupied square of each ray must not be an enemy slider of
        // the ray's kind (rook lines: rook or queen; diagonals: bishop or queen)
        const int r = k >> 3, c = k & 7;
        const uint64_t low = kb - 1ull, high = ~low & ~kb;
        const uint64_t file = kFileA << c, rank = 0xFFull << (8 * r);
        const int dd = r - c, da = r + c - 7;
        const uint64_t diag = dd >= 0 ? kDiag << (8 * dd) : kDiag >> (-8 * dd);
        const uint64_t anti = da >= 0 ? kAnti << (8 * da) : kAnti >> (-8 * da);
        const uint64_t ao = eRQ & keep, ad = eBQ & keep;
        auto lowest = [&](uint64_t ray, uint64_t a) {  // rays towards higher indices
            const uint64_t bl = ray & o;
            return (bl & (0ull - bl) & a) != 0ull;
        };
        auto highest = [&](uint64_t ray, uint64_t a) {  // rays towards lower indices
            const uint64_t bl = ray & o;
            return bl != 0ull && ((a >> (63 - __builtin_clzll(bl))) & 1ull);
        };
        // every test evaluated (no short-circuit branches: the lanes diverge on them)
        return ((int)leap | (int)lowest(file & high, ao) | (int)lowest(rank & high, ao) | (int)highest(file & low, ao) |
                (int)highest(rank & low, ao) | (int)lowest(diag & high, ad) | (int)lowest(anti & high, ad) |
                (int)highest(diag & low, ad) | (int)highest(anti & low, ad)) != 0;
    }
};

// Pseudo-legal moves of the piece `pc` on square s from the BitView's masks, in the
// reference's order (piece_moves below is the square-by-square statement of it), emitted
// WITHOUT their capture values (0): legal_moves_view adds BitView::capval in its lane-per-move
// legality pass, off the serial emission loops.  Target
// sets come from shifts and masked bit scans, then each set is emitted in its order — a
// knight's eight offsets (-17 ... +17) are in index order, a king's are tested one by one
// in kAll8 order, and a slider's rays run away from s (descending indices for the
// directions that lower the index, ascending for the others).
template <class F>
__device__ __forceinline__ void bit_piece_moves(const BitView &v, int s, uint32_t pc, F &&emit) {
    const int r = s >> 3, c = s & 7;
    const uint32_t up = upper(pc);
    const uint64_t empty = ~v.occ, ok = ~v.occ | v.cap;
    auto asc = [&](uint64_t T) {
        while (T) {
            const int to = __builtin_ctzll(T);
            T &= T - 1ull;
            emit(s, to, 0u);
        }
    };
    auto desc = [&](uint64_t T) {
        while (T) {
            const int to = 63 - __builtin_clzll(T);
            T &= ~(1ull << to);
            emit(s, to, 0u);
        }
    };
    const uint64_t kb = 1ull << s;
    if (up == 'P') {
        const bool white = pc == 'P';
        const int nr = r + (white ? -1 : 1);
        if ((unsigned)nr < 8u) {
            const int t1 = nr * 8 + c;
            if ((empty >> t1) & 1ull) {
                emit(s, t1, 0u);
                const int t2 = t1 + (white ? -8 : 8);
                if (r == (white ? 6 : 1) && ((empty >> t2) & 1ull)) emit(s, t2, 0u);
            }
            if (c > 0 && ((v.cap >> (t1 - 1)) & 1ull)) emit(s, t1 - 1, 0u);
            if (c < 7 && ((v.cap >> (t1 + 1)) & 1ull)) emit(s, t1 + 1, 0u);
        }
    } else if (up == 'N') {
        asc(ok & (((kb << 17) & kNotA) | ((kb << 15) & kNotH) | ((kb << 10) & kNotAB) | ((kb << 6) & kNotGH) |
                  ((kb >> 17) & kNotH) | ((kb >> 15) & kNotA) | ((kb >> 10) & kNotGH) | ((kb >> 6) & kNotAB)));
    } else if (up == 'K') {
        const uint64_t T = ok & (((kb << 1) & kNotA) | ((kb >> 1) & kNotH) | (kb << 8) | (kb >> 8) |
                                 ((kb << 9) & kNotA) | ((kb << 7) & kNotH) | ((kb >> 7) & kNotA) | ((kb >> 9) & kNotH));
        constexpr int off[8] = {-9, -7, 7, 9, -8, 8, -1, 1};  // kAll8 order
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int to = s + off[i];
            if ((unsigned)to < 64u && ((T >> to) & 1ull)) emit(s, to, 0u);
        }
    } else if (up == 'B' || up == 'R' || up == 'Q') {
        const uint64_t low = kb - 1ull, high = ~low & ~kb;
        const uint64_t file = kFileA << c, rank = 0xFFull << (8 * r);
        const int dd = r - c, da = r + c - 7;
        const uint64_t diag = dd >= 0 ? kDiag << (8 * dd) : kDiag >> (-8 * dd);
        const uint64_t anti = da >= 0 ? kAnti << (8 * da) : kAnti >> (-8 * da);
        auto up_ray = [&](uint64_t ray) {  // towards higher indices: through the nearest blocker
            const uint64_t bl = ray & v.occ, first = bl & (0ull - bl);
            asc(ok & (first ? ray & ((first << 1) - 1ull) : ray));
        };
        auto down_ray = [&](uint64_t ray) {  // towards lower indices
            const uint64_t bl = ray & v.occ;
            desc(ok & (bl ? ray & ~((1ull << (63 - __builtin_clzll(bl))) - 1ull) : ray));
        };
        if (up != 'R') {  // kAll8[0..4): (-1,-1) (-1,1) (1,-1) (1,1)
            down_ray(diag & low);
            down_ray(anti & low);
            up_ray(anti & high);
            up_ray(diag & high);
        }
        if (up != 'B') {  // kAll8[4..8): (-1,0) (1,0) (0,-1) (0,1)
            down_ray(file & low);
            up_ray(file & high);
            down_ray(rank & low);
            up_ray(rank & high);
        }
    }
}

__device__ __forceinline__ bool known_piece(uint32_t x) {  // 0, ' ', PNBRQK, pnbrqk
    constexpr uint64_t kLo = (1ull << 0) | (1ull << ' ');
    constexpr uint64_t kHi = (1ull << ('P' - 64)) | (1ull << ('N' - 64)) | (1ull << ('B' - 64)) |
                             (1ull << ('R' - 64)) | (1ull << ('Q' - 64)) | (1ull << ('K' - 64)) |
                             (1ull << ('p' - 64)) | (1ull << ('n' - 64)) | (1ull << ('b' - 64)) |
                             (1ull << ('r' - 64)) | (1ull << ('q' - 64)) | (1ull << ('k' - 64));
    return x < 64u ? ((kLo >> x) & 1ull) != 0ull : x < 128u ? ((kHi >> (x - 64u)) & 1ull) != 0ull : false;
}

// The BitView of the board for side t to move, built from x = this lane's square.  Returns
// false (view unusable) when some square holds another character or the mover has no king.
__device__ __forceinline__ bool make_bitview(uint32_t x, int t, BitView &v) {
    if (__ballot(!known_piece(x)) != 0ull) return false;
    const uint32_t up = upper(x);
    const bool filled = !empty_sq(x);
    const uint64_t white = __ballot(filled && is_white(x)), black = __ballot(filled && !is_white(x));
    const uint64_t en = t == 0 ? black : white, own = t == 0 ? white : black;
    const uint64_t P = __ballot(up == 'P'), N = __ballot(up == 'N'), B = __ballot(up == 'B');
    const uint64_t R = __ballot(up == 'R'), Q = __ballot(up == 'Q'), K = __ballot(up == 'K');
    v.occ = white | black;
    v.cap = en & ~K;
    v.tP = P;
    v.tNB = N | B;
    v.tR = R;
    v.eP = en & P;
    v.eN = en & N;
    v.eBQ = en & (B | Q);
    v.eRQ = en & (R | Q);
    v.eK = en & K;
    v.kings = own & K;
    v.t = t;
    return v.kings != 0ull;
}

// Pseudo-legal moves of the piece `pc` on square s (row r, col c); F(from, to, value) is
// called for each in the reference's order.  Returns nothing; the caller counts or stores.
template <class V, class F>
__device__ __forceinline__ void piece_moves(const V &b, int s, uint32_t pc, F &&emit) {
    const int r = s >> 3, c = s & 7;
    const uint32_t up = upper(pc);
    if (up == 'P') {
        const int dir = pc == 'P' ? -1 : 1;
        const int nr = r + dir;
        if (inb(nr, c) && b.probe(nr * 8 + c) == -2) {
            emit(s, nr * 8 + c, 0u);
            if (r == (pc == 'P' ? 6 : 1) && inb(nr + dir, c) && b.probe((nr + dir) * 8 + c) == -2)
                emit(s, (nr + dir) * 8 + c, 0u);
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int cc = c + (k ? 1 : -1);
            if (inb(nr, cc)) {
                const int x = b.probe(nr * 8 + cc);
                if (x >= 0) emit(s, nr * 8 + cc, (uint32_t)x);
            }
        }
    } else if (up == 'N' || up == 'K') {
        const bool kn = up == 'N';
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int rr = r + (kn ? kKnight[i].dr : kAll8[i].dr), cc = c + (kn ? kKnight[i].dc : kAll8[i].dc);
            if (!inb(rr, cc)) continue;
            const int x = b.probe(rr * 8 + cc);
            if (x == -2) emit(s, rr * 8 + cc, 0u);
            else if (x >= 0) emit(s, rr * 8 + cc, (uint32_t)x);
        }
    } else if (up == 'B' || up == 'R' || up == 'Q') {
        const int d0 = up == 'R' ? 4 : 0, d1 = up == 'B' ? 4 : 8;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (i < d0 || i >= d1) continue;
            const int dr = kAll8[i].dr, dc = kAll8[i].dc;
            int rr = r + dr, cc = c + dc;
            while (inb(rr, cc)) {
                const int x = b.probe(rr * 8 + cc);
                if (x == -2) {
                    emit(s, rr * 8 + cc, 0u);
                } else {
                    if (x >= 0) emit(s, rr * 8 + cc, (uint32_t)x);
                    break;
                }
                rr += dr;
                cc += dc;
            }
        }
    }
}

// king_attacked (:85-144) for the king of side t on (kr, kc) — (-1,-1) when absent, exactly
// as the reference probes then — on the board b with square `from` emptied and `pc` on `to`
// (the position after a non-castling move; promotion does not change the answer: the piece
// on `to` is the mover's either way and only blocks).
__device__ __forceinline__ bool attacked_after(const uint8_t *b, int t, int kr, int kc, int from, int to, uint32_t pc) {
    auto at = [&](int r, int c) -> uint32_t {
        const int s = r * 8 + c;
        return s == to ? pc : (s == from ? (uint32_t)' ' : (uint32_t)b[s]);
    };
    const int pr = t == 0 ? kr - 1 : kr + 1;
    const uint32_t pawn = t == 0 ? 'p' : 'P';
    if (inb(pr, kc - 1) && at(pr, kc - 1) == pawn) return true;
    if (inb(pr, kc + 1) && at(pr, kc + 1) == pawn) return true;
    const uint32_t kn = t ? 'N' : 'n';
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int rr = kr + kKnight[i].dr, cc = kc + kKnight[i].dc;
        if (inb(rr, cc) && at(rr, cc) == kn) return true;
    }
    const uint32_t q = t ? 'Q' : 'q';
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // rook lines (kAll8[4..8)) first, then bishop lines: same answer
        const int dr = kAll8[i].dr, dc = kAll8[i].dc;
        const uint32_t p1 = i < 4 ? (t ? 'B' : 'b') : (t ? 'R' : 'r');
        int rr = kr + dr, cc = kc + dc;
        while (inb(rr, cc)) {
            const uint32_t x = at(rr, cc);
            if (!empty_sq(x)) {
                if (x == p1 || x == q) return true;
                break;
            }
            rr += dr;
            cc += dc;
        }
    }
    const uint32_t kk = t ? 'K' : 'k';
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int rr = kr + kAll8[i].dr, cc = kc + kAll8[i].dc;
        if (inb(rr, cc) && at(rr, cc) == kk) return true;
    }
    return false;
}

__device__ __forceinline__ bool ByteView::attacked(int k, int from, int to, uint32_t pc) const {
    return attacked_after(b, t, k >= 0 ? (k >> 3) : -1, k >= 0 ? (k & 7) : -1, from, to, pc);
}

// Exclusive prefix sum over the wave (DPP row scan + row broadcasts).
__device__ __forceinline__ uint32_t wave_excl_sum(uint32_t x, uint32_t &total) {
    uint32_t v = x;
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);
    total = (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
    return v - x;
}

// Squares holding side's king (find_king :70-83 takes the first one; -1 when none).
__device__ __forceinline__ uint64_t king_mask(const uint8_t *b, int side) {
    return __ballot(b[lane()] == (side == 0 ? 'K' : 'k'));
}

// The BitView generator with one lane per (piece, direction) run instead of one lane per
// piece.  A piece's moves are up to eight runs in the reference's order — a slider's rays in
// kAll8 order (each away from s: descending indices for the directions that lower it), a
// knight's targets as one ascending run, a king's eight kAll8 targets as eight one-square
// runs, a pawn's push / double push / captures as four — so each square lane builds its
// runs' target masks, two exclusive scans over the squares place the runs (records in `rec`,
// 4 u32 each) and their moves (in `ps`), and then every lane emits ONE run: the serial loop
// is as long as the longest run (<= 8) instead of a piece's whole move list.  Capture values
// are added by the caller, as for bit_piece_moves.  Returns false, leaving nothing written,
// when the position has more than 128 runs (never in reachable chess: <= 16 pieces).
// The eight run masks of the piece on square s (bit_runs' first part; all zero for a square
// that is not the mover's), and desc: bit k set when run k is emitted from the highest index down.
__device__ __forceinline__ void run_masks(const BitView &v, int s, uint32_t pc, bool mine, uint64_t (&M)[8],
                                          uint32_t &desc) {
    // Every lane computes every piece kind's runs and keeps its own kind's by selects: the
    // kinds' branches diverge in every position, and their joins copied all eight masks.
    const int r = s >> 3, c = s & 7;
    const uint32_t up = upper(pc);
    const uint64_t empty = ~v.occ, ok = ~v.occ | v.cap;
    const uint64_t kb = 1ull << s;
    const bool isP = mine && up == 'P', isN = mine && up == 'N', isK = mine && up == 'K';
    const bool isS = mine && (up == 'B' || up == 'R' || up == 'Q');
    const bool diagS = isS && up != 'R', orthS = isS && up != 'B';
    const bool white = pc == 'P';
    const uint64_t fwd = white ? kb >> 8 : kb << 8;  // the pawn's push square (none from its last rank)
    const uint64_t p1 = fwd & empty;
    // slider lines through s
    const uint64_t low = kb - 1ull, high = ~low & ~kb;
    const uint64_t file = kFileA << c, rank = 0xFFull << (8 * r);
    const int dd = r - c, da = r + c - 7;
    const uint64_t diag = dd >= 0 ? kDiag << (8 * dd) : kDiag >> (-8 * dd);
    const uint64_t anti = da >= 0 ? kAnti << (8 * da) : kAnti >> (-8 * da);
    auto up_ray = [&](uint64_t ray) {  // towards higher indices: through the nearest blocker
        const uint64_t bl = ray & v.occ, first = bl & (0ull - bl);
        return ok & (first ? ray & ((first << 1) - 1ull) : ray);
    };
    auto down_ray = [&](uint64_t ray) {  // towards lower indices
        const uint64_t bl = ray & v.occ;
        return ok & (bl ? ray & ~((1ull << (63 - __builtin_clzll(bl))) - 1ull) : ray);
    };
#pragma unroll
    for (int k = 0; k < 8; ++k) {  // one run at a time, each mask consumed where it is made
        // run k of a slider: its ray in kAll8 order, away from s
        const uint64_t line = k == 0 || k == 3 ? diag : k == 1 || k == 2 ? anti : k < 6 ? file : rank;
        const bool dn = k == 0 || k == 1 || k == 4 || k == 6;
        uint64_t m = (k < 4 ? diagS : orthS) ? (dn ? down_ray(line & low) : up_ray(line & high)) : 0ull;
        // of a king: its neighbour in direction k (kAll8: -9, -7, 7, 9, -8, 8, -1, 1; no file wrap)
        const uint64_t nbk = k == 0 ? (kb >> 9) & kNotH : k == 1 ? (kb >> 7) & kNotA : k == 2 ? (kb << 7) & kNotH
                           : k == 3 ? (kb << 9) & kNotA : k == 4 ? kb >> 8 : k == 5 ? kb << 8
                           : k == 6 ? (kb >> 1) & kNotH : (kb << 1) & kNotA;
        m = isK ? ok & nbk : m;
        // of a pawn: push, double push, captures towards the lower / higher file
        if (k == 0) m = isP ? p1 : m;
        if (k == 1)
            m = isP ? ((p1 != 0ull && r == (white ? 6 : 1)) ? (white ? fwd >> 8 : fwd << 8) & empty : 0ull) : m;
        if (k == 2) m = isP ? (fwd >> 1) & kNotH & v.cap : m;
        if (k == 3) m = isP ? (fwd << 1) & kNotA & v.cap : m;
        // of a knight: every target, one ascending run
        if (k == 0)
            m = isN ? ok & knight_targets(s) : m;
        M[k] = m;
        __builtin_amdgcn_sched_barrier(0);
    }
    desc = isS ? 0x53u : 0u;  // runs 0, 1, 4, 6
}

__device__ __forceinline__ bool bit_runs(const BitView &v, int s, uint32_t pc, bool mine, uint16_t *ps, uint32_t *rec,
                                         uint32_t &total) {
    CDEV_T(cd12);
    uint64_t M[8];
    uint32_t desc;
    run_masks(v, s, pc, mine, M, desc);
    CDEV_ADD(12, cd12);
    uint32_t nruns = 0, nmoves = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        nruns += M[k] != 0ull ? 1u : 0u;
        nmoves += (uint32_t)__popcll(M[k]);
    }
    uint32_t runs_total;
    const uint32_t rbase = wave_excl_sum(nruns, runs_total);
    const uint32_t mbase = wave_excl_sum(nmoves, total);
    if (runs_total > 128u || total > (uint32_t)kMaxPseudo) return false;
    uint32_t ri = rbase, mo = mbase;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        if (M[k] != 0ull) {
            uint32_t *const q = rec + 4 * ri;
            q[0] = (uint32_t)M[k];
            q[1] = (uint32_t)(M[k] >> 32);
            q[2] = mo;
            q[3] = (uint32_t)s | (((desc >> k) & 1u) << 6);
            ++ri;
            mo += (uint32_t)__popcll(M[k]);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    CDEV_T(cd15);
    for (uint32_t base = 0; base < runs_total; base += 64) {
        const uint32_t j = base + lane();
        if (j < runs_total) {
            const uint32_t *const q = rec + 4 * j;
            uint64_t T = (uint64_t)q[0] | ((uint64_t)q[1] << 32);
            uint16_t *dst = ps + q[2];
            const uint32_t meta = q[3];
            const int from = (int)(meta & 63u);
            const bool down = (meta & 64u) != 0u;
            // a run has at most 8 targets (a knight's); ascending and descending runs share
            // one unrolled loop (their lanes would otherwise run two divergent loops in turn)
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if (T == 0ull) break;
                const int to = down ? 63 - __builtin_clzll(T) : __builtin_ctzll(T);
                T &= ~(1ull << to);
                dst[k] = (uint16_t)pack_move(from, to, 0u);
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    CDEV_ADD(15, cd15);
    return true;
}

template <class V>
__device__ __forceinline__ int legal_moves_view(const V &v, int t, uint32_t pc, uint64_t kings, uint16_t *out,
                                                uint16_t *ps, uint16_t *reg) {
    const uint32_t s = lane();
    const bool mine = !empty_sq(pc) && ((t == 0) == is_white(pc));
    uint32_t total = 0;
    CDEV_T(cd11);
    bool runs = false;  // the bit view's run-parallel generator (bit_runs) when it applies
    if constexpr (V::kCheapProbe) runs = bit_runs(v, (int)s, pc, mine, ps, (uint32_t *)reg, total);
    if (!runs) {
        // one generation pass into this lane's own region (a piece has at most 27
        // pseudo-legal moves), then each lane copies its run to its place in board-scan order
        uint16_t *const own = reg + s * kRegion;
        uint32_t cnt = 0;
        auto put = [&](int f, int to, uint32_t val) { own[cnt++] = (uint16_t)pack_move(f, to, val); };
        if (mine) {
            if constexpr (V::kCheapProbe) bit_piece_moves(v, (int)s, pc, put);
            else piece_moves(v, (int)s, pc, put);
        }
        const uint32_t off = wave_excl_sum(cnt, total);
        if (total > (uint32_t)kMaxPseudo) return -1;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        for (uint32_t k = 0; k < cnt; ++k) ps[off + k] = own[k];
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    CDEV_ADD(11, cd11);
    CDEV_T(cd13);
    const uint32_t kch = t == 0 ? 'K' : 'k';
    int n = 0;
    for (uint32_t base = 0; base < total; base += 64) {
        const uint32_t i = base + s;
        bool legal = false;
        uint32_t m = 0;
        if (i < total) {
            m = ps[i];
            const int from = (int)(m & 63u), to = (int)((m >> 6) & 63u);
            if constexpr (V::kCheapProbe) m |= v.capval(to) << 12;
            const uint32_t mp = v.piece_at(from);
            // find_king on the board after the move: first square holding the mover's king
            const uint64_t km = (kings & ~(1ull << from)) | (mp == kch ? (1ull << to) : 0ull);
            const int k = km ? __builtin_ctzll(km) : -1;
            legal = !v.attacked(k, from, to, mp);
        }
        const uint64_t L = __ballot(legal);
        const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(L >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)L, 0u));
        if (legal && n + rank < kMaxLegal) out[n + rank] = (uint16_t)m;
        n += __popcll(L);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    CDEV_ADD(13, cd13);
    return n > kMaxLegal ? -1 : n;
}

// get_legal_moves for the board in LDS `b` (64 bytes) with side to move t.  Writes the
// packed legal moves to out[0..n) (LDS or global); LDS scratch: pseudo-legal list `ps`
// (kMaxPseudo) and per-lane generation regions `reg` (64 x kRegion).
// Returns n (wave-uniform), or -1 when the position has more than kMaxPseudo pseudo-legal
// or kMaxLegal legal moves (never in reachable chess).
__device__ __forceinline__ int legal_moves(const uint8_t *b, int t, uint16_t *out, uint16_t *ps, uint16_t *reg) {
    const uint32_t pc = b[lane()];
    // insufficient material (:188-198): no P/R/Q of either colour and at most one minor
    const uint32_t up = upper(pc);
    const uint64_t heavy = __ballot(up == 'P' || up == 'R' || up == 'Q');
    const int minor = __popcll(__ballot(up == 'B' || up == 'N'));
    if (!heavy && minor <= 1) return 0;
    BitView bv;
    if (make_bitview(pc, t, bv)) return legal_moves_view(bv, t, pc, bv.kings, out, ps, reg);
    return legal_moves_view(ByteView{b, t}, t, pc, king_mask(b, t), out, ps, reg);
}

// get_legal_moves and, for a position without legal moves, king_attacked of the side to
// move (check_win, crude_chess_score's mate score) on one board view; `check` is false when
// the position has moves.
// (pc: this lane's square b[lane], when the caller has it in a register)
__device__ __forceinline__ int legal_moves_check(const uint8_t *b, uint32_t pc, int t, uint16_t *out, uint16_t *ps,
                                                 uint16_t *reg, bool &check) {
    CDEV_T(cd14);
    BitView bv;
    const bool fast = make_bitview(pc, t, bv);
    const uint64_t kings = fast ? bv.kings : king_mask(b, t);
    CDEV_ADD(14, cd14);
    const uint32_t up = upper(pc);
    const uint64_t heavy = __ballot(up == 'P' || up == 'R' || up == 'Q');
    const int minor = __popcll(__ballot(up == 'B' || up == 'N'));
    int n = 0;
    if (heavy || minor > 1)  // else insufficient material (:188-198): no moves
        n = fast ? legal_moves_view(bv, t, pc, kings, out, ps, reg)
                 : legal_moves_view(ByteView{b, t}, t, pc, kings, out, ps, reg);
    // every caller asks "in check?" only of a position without moves (checkmate against
    // stalemate): the king test runs only then, and `check` is false otherwise
    check = false;
    if (n == 0) {
        if (fast) {
            check = bv.attacked(__builtin_ctzll(kings), -1, -1, 0);
        } else {
            const int ks = kings ? __builtin_ctzll(kings) : -1;
            check = attacked_after(b, t, ks >= 0 ? ks >> 3 : -1, ks >= 0 ? ks & 7 : -1, -1, -1, 0);
        }
    }
    return n;
}

__device__ __forceinline__ int legal_moves_check(const uint8_t *b, int t, uint16_t *out, uint16_t *ps, uint16_t *reg,
                                                 bool &check) {
    return legal_moves_check(b, (uint32_t)b[lane()], t, out, ps, reg, check);
}

#ifndef ZC_CHESS_FREEPROBE
#define ZC_CHESS_FREEPROBE 1  // legal_moves_probe tries has_free_move first (A/B: 0)
#endif

// A sufficient test for "the mover has a legal move" (legal_moves_probe's common case): the
// mover's king (the first, as find_king) is not attacked, and some piece of the mover other than
// a king, standing on none of the king's eight lines, has a pseudo-legal move.  Such a move
// cannot unblock a line to the king (the piece is on none; its target only adds a blocker of
// the mover's) and cannot add a leaper attack (it removes at most the piece it captures), so
// BitView::attacked stays false after it and the move is legal.  The pseudo-legal moves are
// the generator's (a pawn's push or capture; a knight's target; a slider's or queen's first
// step along a line of its kind): a target that is empty or capturable.
__device__ __forceinline__ bool has_free_move(const BitView &v, int s, uint32_t pc, bool mine) {
    const int k = __builtin_ctzll(v.kings);  // the view has a king
    if (v.attacked(k, -1, -1, 0)) return false;
    const int r = s >> 3, c = s & 7, kr = k >> 3, kc = k & 7;
    const bool aligned = r == kr || c == kc || r - c == kr - kc || r + c == kr + kc;
    const uint32_t up = upper(pc);
    const uint64_t ok = ~v.occ | v.cap, kb = 1ull << s;
    const uint64_t near = king_targets(s) & ok;                              // one step, any line
    const uint64_t orth = near & ((kFileA << c) | (0xFFull << (8 * r)));    // ... along a rank or file
    const uint64_t fwd = pc == 'P' ? kb >> 8 : kb << 8;                     // a pawn's push square
    const uint64_t pawn = (fwd & ~v.occ) | ((((fwd >> 1) & kNotH) | ((fwd << 1) & kNotA)) & v.cap);
    const uint64_t T = up == 'P' ? pawn : up == 'N' ? knight_targets(s) & ok : up == 'B' ? near & ~orth
                     : up == 'R' ? orth : up == 'Q' ? near : 0ull;
    return __ballot(mine && !aligned && T != 0ull) != 0ull;
}

// Whether the position has a legal move, for a node that may never be expanded (the crude
// search's lazy nodes): has_free_move, else one pseudo-legal move per piece (its first run's
// first target) through the same legality test as legal_moves_view.  When one of them is
// legal, returns 1 with
// lazy = true and writes nothing (the list is generated if the node is ever expanded);
// otherwise — every tested move illegal (typically in check), a position the bit view does not
// cover, or insufficient material — the full legal_moves_check: the list in out, its length,
// and the check flag of a position without moves.
__device__ __forceinline__ int legal_moves_probe(const uint8_t *b, uint32_t pc, int t, uint16_t *out, uint16_t *ps,
                                                 uint16_t *reg, bool &check, bool &lazy) {
    lazy = false;
    BitView bv;
    const uint32_t up = upper(pc);
    const uint64_t heavy = __ballot(up == 'P' || up == 'R' || up == 'Q');
    const int minor = __popcll(__ballot(up == 'B' || up == 'N'));
    if ((heavy || minor > 1) && make_bitview(pc, t, bv)) {
        const int s = (int)lane();
        const bool mine = !empty_sq(pc) && ((t == 0) == is_white(pc));
        if (ZC_CHESS_FREEPROBE && has_free_move(bv, s, pc, mine)) {
            lazy = true;
            check = false;
            return 1;
        }
        uint64_t M[8];
        uint32_t desc;
        run_masks(bv, s, pc, mine, M, desc);
        uint64_t T = 0;
        bool down = false;
#pragma unroll
        for (int k = 7; k >= 0; --k) {  // the first non-empty run
            if (M[k] != 0ull) {
                T = M[k];
                down = ((desc >> k) & 1u) != 0u;
            }
        }
        bool legal = false;
        if (T != 0ull) {
            const int to = down ? 63 - __builtin_clzll(T) : __builtin_ctzll(T);
            const uint32_t kch = t == 0 ? 'K' : 'k';
            const uint32_t mp = bv.piece_at(s);
            const uint64_t km = (bv.kings & ~(1ull << s)) | (mp == kch ? (1ull << to) : 0ull);
            legal = !bv.attacked(__builtin_ctzll(km), s, to, mp);  // km != 0: the bit view has a king
        }
        if (__ballot(legal) != 0ull) {
            lazy = true;
            check = false;
            return 1;
        }
    }
    return legal_moves_check(b, pc, t, out, ps, reg, check);
}

// Sum of piece values, white positive (crude_chess_score's material), by ballots.
__device__ __forceinline__ int material(uint32_t x) {
    auto n = [&](uint32_t w, uint32_t bl) {
        return __popcll(__ballot(x == w)) - __popcll(__ballot(x == bl));
    };
    return n('P', 'p') + 3 * (n('N', 'n') + n('B', 'b')) + 5 * n('R', 'r') + 9 * n('Q', 'q');
}

// play_move (:364-400) without the history deques (those stay with the host State).
__device__ __forceinline__ void apply_move(zc_chess_state &o, uint32_t m) {
    const int from = (int)(m & 63u), to = (int)((m >> 6) & 63u);
    const int fc = from & 7, tc = to & 7, tr = to >> 3;
    uint8_t *b = o.board;
    const uint8_t pc = b[from], trg = b[to];
    const int turn = o.turn;
    o.turn = (uint8_t)(1 - turn);
    o.fifty = (uint8_t)(o.fifty + 1);
    if (pc == 'P' || pc == 'p' || !(trg == ' ' || trg == 0)) o.fifty = 0;
    if (pc == 'K' || (pc == 'R' && fc == 7)) o.castle &= (uint8_t)~1u;
    if (pc == 'K' || (pc == 'R' && fc == 0)) o.castle &= (uint8_t)~2u;
    if (pc == 'k' || (pc == 'r' && fc == 7)) o.castle &= (uint8_t)~4u;
    if (pc == 'k' || (pc == 'r' && fc == 0)) o.castle &= (uint8_t)~8u;
    if (pc == 'K' && tc - fc == 2) { b[61] = 'R'; b[63] = ' '; }
    if (pc == 'k' && tc - fc == 2) { b[5] = 'r'; b[7] = ' '; }
    if (pc == 'K' && tc - fc == -2) { b[59] = 'R'; b[56] = ' '; }
    if (pc == 'k' && tc - fc == -2) { b[3] = 'r'; b[0] = ' '; }
    b[to] = pc;
    b[from] = ' ';
    if (tr == 0 && pc == 'P') b[to] = 'Q';
    if (tr == 7 && pc == 'p') b[to] = 'q';
}

// apply_move with one square per lane (all lanes call it; the position in `o` is complete
// and visible to the wave): lane l computes square l of the position after the move from
// the writes apply_move makes, in their order — a castling rook's two squares, then
// b[to] = pc, b[from] = ' ', then the promotion on `to` — and lane 0 the counters.  The
// caller fences before the result is read.
__device__ __forceinline__ void apply_move_wave(zc_chess_state &o, uint32_t m) {
    const uint32_t l = lane();
    const int from = (int)(m & 63u), to = (int)((m >> 6) & 63u);
    const int fc = from & 7, tc = to & 7, tr = to >> 3;
    uint8_t *b = o.board;
    const uint32_t pc = b[from], trg = b[to], x0 = b[l];
    const int turn = o.turn;
    uint32_t x = x0;
    const int dcol = tc - fc;
    if (pc == 'K' && dcol == 2) x = l == 61 ? 'R' : l == 63 ? ' ' : x;
    if (pc == 'k' && dcol == 2) x = l == 5 ? 'r' : l == 7 ? ' ' : x;
    if (pc == 'K' && dcol == -2) x = l == 59 ? 'R' : l == 56 ? ' ' : x;
    if (pc == 'k' && dcol == -2) x = l == 3 ? 'r' : l == 0 ? ' ' : x;
    if ((int)l == to) x = pc;
    if ((int)l == from) x = ' ';
    if ((int)l == to && tr == 0 && pc == 'P') x = 'Q';
    if ((int)l == to && tr == 7 && pc == 'p') x = 'q';
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");  // every lane has read the old board
    if (x != x0) b[l] = (uint8_t)x;
    if (l == 0) {
        uint32_t fifty = (uint32_t)o.fifty + 1u, castle = o.castle;
        if (pc == 'P' || pc == 'p' || !(trg == ' ' || trg == 0)) fifty = 0;
        if (pc == 'K' || (pc == 'R' && fc == 7)) castle &= ~1u;
        if (pc == 'K' || (pc == 'R' && fc == 0)) castle &= ~2u;
        if (pc == 'k' || (pc == 'r' && fc == 7)) castle &= ~4u;
        if (pc == 'k' || (pc == 'r' && fc == 0)) castle &= ~8u;
        o.turn = (uint8_t)(1 - turn);
        o.fifty = (uint8_t)fifty;
        o.castle = (uint8_t)castle;
    }
}

// apply_move with the position in registers instead of LDS: lanes 0..17 of `stw` hold the
// zc_chess_state words of the position; returns this lane's square of the position after m
// (apply_move_wave's per-square rule) and, in w16, the new state word 16 (turn | fifty << 8 |
// castle << 16 | reserved[0] << 24).  Words 17.. are unchanged.
__device__ __forceinline__ uint32_t apply_move_regs(uint32_t stw, uint32_t m, uint32_t &w16) {
    const uint32_t l = lane();
    const int from = (int)(m & 63u), to = (int)((m >> 6) & 63u);
    const int fc = from & 7, tc = to & 7, tr = to >> 3;
    const uint32_t x0 = ((uint32_t)__shfl((int)stw, (int)(l >> 2)) >> (8u * (l & 3u))) & 0xFFu;
    const uint32_t pc = ((uint32_t)__builtin_amdgcn_readlane((int)stw, from >> 2) >> (8 * (from & 3))) & 0xFFu;
    const uint32_t trg = ((uint32_t)__builtin_amdgcn_readlane((int)stw, to >> 2) >> (8 * (to & 3))) & 0xFFu;
    const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)stw, 16);
    uint32_t x = x0;
    const int dcol = tc - fc;
    if (pc == 'K' && dcol == 2) x = l == 61 ? 'R' : l == 63 ? ' ' : x;
    if (pc == 'k' && dcol == 2) x = l == 5 ? 'r' : l == 7 ? ' ' : x;
    if (pc == 'K' && dcol == -2) x = l == 59 ? 'R' : l == 56 ? ' ' : x;
    if (pc == 'k' && dcol == -2) x = l == 3 ? 'r' : l == 0 ? ' ' : x;
    if ((int)l == to) x = pc;
    if ((int)l == from) x = ' ';
    if ((int)l == to && tr == 0 && pc == 'P') x = 'Q';
    if ((int)l == to && tr == 7 && pc == 'p') x = 'q';
    uint32_t fifty = ((w >> 8) & 0xFFu) + 1u, castle = (w >> 16) & 0xFFu;
    if (pc == 'P' || pc == 'p' || !(trg == ' ' || trg == 0)) fifty = 0;
    if (pc == 'K' || (pc == 'R' && fc == 7)) castle &= ~1u;
    if (pc == 'K' || (pc == 'R' && fc == 0)) castle &= ~2u;
    if (pc == 'k' || (pc == 'r' && fc == 7)) castle &= ~4u;
    if (pc == 'k' || (pc == 'r' && fc == 0)) castle &= ~8u;
    w16 = ((1u - (w & 0xFFu)) & 0xFFu) | ((fifty & 0xFFu) << 8) | (castle << 16) | (w & 0xFF000000u);
    return x;
}

// has_repeated_prefix (chess_backend.cpp:148-180; min_pattern_len 2, min_repeats 3) of the
// m moves h[0..m) in play order, most recent first (one wave; Lh: m u16 of LDS).  KMP's test
// — some prefix whose smallest period p >= 2 divides its length at least 3 times — is
// evaluated as: with M(q) = q + lcp(L, L shifted by q), the longest prefix of period q, some
// p >= 2 has R = p * floor(M(p) / p) >= 3p and R > M(1).  (Then the smallest period of the
// R-prefix is not 1, and by Fine and Wilf it divides p, so it repeats >= 3 times; conversely
// KMP's prefix is such an R or shorter.)  Lanes compare 64 shifted pairs per step.
__device__ __forceinline__ bool repeated_prefix(const uint16_t *h, int m, uint16_t *Lh) {
    const int l = (int)lane();
    for (int k = l; k < m; k += 64) Lh[k] = h[m - 1 - k];
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    bool rep = false;
    if (m >= 6) {
        int m1 = m;  // M(1): the opening run of one repeated move
        for (int base = 0; base < m; base += 64) {
            const int k = base + l;
            const uint64_t mm = __ballot(k < m && Lh[k] != Lh[0]);
            if (mm) {
                m1 = base + __builtin_ctzll(mm);
                break;
            }
        }
        for (int p = 2; 3 * p <= m && !rep; ++p) {
            int lcp = m - p;
            for (int base = 0; base < m - p; base += 64) {
                const int k = base + l;
                const uint64_t mm = __ballot(k < m - p && Lh[k] != Lh[k + p]);
                if (mm) {
                    lcp = base + __builtin_ctzll(mm);
                    break;
                }
            }
            const int R = (p + lcp) / p * p;
            rep = R >= 3 * p && R > m1;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    return rep;
}

// Both sides' repetition answers: white's | black's << 1 (check_draw's repetition draw is
// both, chess_backend.cpp:416-441).  hist[side][k] = that side's k-th move (k < len[side],
// at most cap read).
__device__ __forceinline__ int repetitions(const uint16_t *hist, const int32_t *len, int cap, uint16_t *Lh) {
    int res = 0;
    for (int side = 0; side < 2; ++side) {
        const int m = min(__builtin_amdgcn_readfirstlane(len[side]), cap);
        res |= (repeated_prefix(hist + (size_t)side * cap, m, Lh) ? 1 : 0) << side;
    }
    return res;
}

struct ChessScratch {
    uint8_t board[64];
    uint16_t legal[kMaxLegal];
    uint16_t pseudo[kMaxPseudo];
    alignas(16) uint16_t region[64 * kRegion];  // also bit_runs' 16-byte run records
};

}  // namespace
}  // namespace chessdev
}  // namespace zc
