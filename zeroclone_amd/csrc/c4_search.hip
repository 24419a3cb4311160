// c4_search.hip — batched Connect4 UCT search for gfx950 (MI355X).
//
// Replaces engine/mcts/src/mcts.cpp:102-160 (get_move) together with the callbacks it makes
// for c4_backend (engine/games/connect4/c4_backend.py), Policy('random')
// (engine/policy_functions.py:10-12) and Value('random_rollout')
// (engine/value_functions.py:35-45), for thousands of games per launch.
//
// Execution model: ONE GAME PER WAVE.  A game's search is a strictly serial chain (every
// random number comes from one CPython MT19937 stream, consumed in the reference's order),
// so the chip is filled with games, not with work from inside one game: 4096 games are
// 4096 waves, 16 per CU.  Inside a wave all control flow is wave-uniform, the game state
// (board, stream position, node counter) lives in SGPRs and runs on the scalar unit, and
// the 64 lanes take the parts that are parallel:
//   - selection: lane k scores child slot k (UCT in fp64, exactly mcts.cpp:41-45) and a
//     DPP reduction picks the first maximum;
//   - RNG: lane k holds word wbase+k of a 64-word window of the stream, so a
//     random.choice draw (with its rejection loop) is one ballot;
//   - rollouts: a block of plies is simulated at once, one ply per lane (c4_rollouts);
//   - backup: lane l updates tree level l of the leaf's path (all levels at once);
//   - stream refill: the MT recurrence is regenerated 192 words at a time.
// The whole move (every flush of `batch_size` leaves) runs in one launch; games never
// synchronise with each other.
#include "c4_device.h"
#include "counter_rng.h"

namespace zc {
namespace {


__device__ __forceinline__ uint64_t readlane64(uint64_t x, int l) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(x >> 32), l) << 32) |
           (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)x, l);
}

__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {  // set bits of m in lanes below this one
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Inclusive prefix SUM over the 64 lanes (DPP: row_shr 1,2,4,8, then row_bcast 15 / 31).
__device__ __forceinline__ uint32_t scan_add32(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);
    return x;
}

// Inclusive prefix OR within each 16-lane row (DPP row_shr 1, 2, 4, 8): four independent
// 16-lane scans per wave, of two values at once (the two halves of a bitboard), interleaved
// so that each DPP read finds its operand written two instructions earlier.
__device__ __forceinline__ void scan_or16x2(uint32_t &x, uint32_t &y) {
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);
    y |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)y, 0x111, 0xF, 0xF, false);
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);
    y |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)y, 0x112, 0xF, 0xF, false);
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);
    y |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)y, 0x114, 0xF, 0xF, false);
    x |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);
    y |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)y, 0x118, 0xF, 0xF, false);
}

// Values that are the same in every lane but should live in VGPRs (worked on by the VALU):
// the scalar unit is shared by the CU's four SIMDs and is the busier of the two here.
__device__ __forceinline__ uint64_t in_vgpr(uint64_t x) {
    __asm__("" : "+v"(x));
    return x;
}
// first set bit of a wave mask, 0xFFFFFFFF when empty (s_ff1_i32_b64)
__device__ __forceinline__ uint32_t ff1(uint64_t m) {
    uint32_t r;
    __asm__("s_ff1_i32_b64 %0, %1" : "=s"(r) : "s"(m));
    return r;
}

// Value.random_rollout (value_functions.py:35-45) for the nb pending leaves of one flush, in
// pending order (value.batch: mcts.cpp:118).  Per leaf, from the side to move `turn`:
//   while not check_win(s) and not check_draw(s): s = play(s, choice(list(legal(s))))
//   win -> -1 if the side to move at the end (the loser) is the leaf's side to move, else +1
// check_win looks at the LAST mover only (c4_backend.py:27, tokens[1 - turn]).
//
// Plies are simulated a BLOCK at a time over a 64-word view of the stream that starts at the
// next unconsumed word (rng_view).  While the legal set is unchanged, the draws are exactly
// the view words w with (w >> (32-k)) < n, in stream order — so one ballot yields the moves
// of every ply the view covers.  Lane k (an accepted word) is ply q_k = #accepted lanes below
// it; its column comes from the move order, its row from the column height plus #earlier
// accepted lanes in the same column (packed 4-bit per-column prefix sums).
//
// A column fill changes the legal set (n, k and the CPython order).  The block's FIRST fill
// is absorbed: the words after it are re-drawn under the new legal set (a second ballot and
// prefix sum over the same view; the order words after one or two fills come from a table
// of every column pair read at the block's start).  The block ends at its second fill, the
// board-full ply, its 31st ply or its last accepted word: ~1.29 blocks per rollout (2.12
// with 64-aligned windows and no absorption).  Absorbing every fill (~1.03 blocks) measured
// SLOWER (4,841 vs 3,554 rollout cycles per simulation), as did a second absorbed fill
// (+4.7 %) and an absorption computed branch-free in every block (+1 %).
//
// The win test runs on a COMPACTED copy of the block's plies: ply q goes (one forward lane
// permute) to lane (q & 1)*16 + q/2 and to that lane + 32, so rows 0 and 2 hold the first
// mover's plies in order, rows 1 and 3 the other side's.  One 16-lane prefix-OR scan per
// row then gives every ply its mover's new stones, and the copy lets rows 0/1 test the
// vertical and horizontal directions while rows 2/3 test the diagonals.  The first winning
// ply (if any) ends the rollout.
//
// Work is placed for the scalar unit's sake: the boards are uniform values kept in VGPRs,
// lane conditions are single compares whose ballots are used as v_cndmask masks, and the
// scalar unit only handles the masks, the block's end and the loop control.
#ifndef ZC_RV
#define ZC_RV 0  // experiment switches (tools/rv_libs.sh); 0 = the product kernel
#endif
#ifndef ZC_LAG_MODE
#define ZC_LAG_MODE 3  // free runs' pace balancing (A/B builds): 0 off, 1 per move, 2/3 per flush (2/3 levels)
#endif
// wave priority from a uniform level 0..3 (s_setprio takes an immediate)
__device__ __forceinline__ void set_prio(int lvl) {
    if (lvl >= 3) __builtin_amdgcn_s_setprio(3);
    else if (lvl == 2) __builtin_amdgcn_s_setprio(2);
    else if (lvl == 1) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
}
#ifndef ZC_RSTAMP
#define ZC_RSTAMP 0  // diagnostic build: 1..6 = accumulate one rollout region's cycles into *sub
#endif
// RMARK(k): region k ends here (s_memtime pinned by scheduling barriers; only when ZC_RSTAMP)
#define RMARK(k)                                                    \
    do {                                                            \
        if (ZC_RSTAMP && sub) {                                     \
            __builtin_amdgcn_sched_barrier(0);                      \
            const uint64_t now_ = __builtin_amdgcn_s_memtime();     \
            __builtin_amdgcn_sched_barrier(0);                      \
            if (ZC_RSTAMP == (k)) *sub += now_ - t_;                \
            t_ = now_;                                              \
        }                                                           \
    } while (0)
template <class R>
__device__ void c4_rollouts(Leaf *L, int nb, R &rng, const uint32_t *s_order, Counters &cn,
                            uint64_t *sub = nullptr) {
    uint64_t t_ = ZC_RSTAMP && sub ? __builtin_amdgcn_s_memtime() : 0;
    const uint32_t lane = lane_id();
    const uint32_t lrow = lane >> 4;
    const bool first_row = (lrow & 1u) == 0;                  // rows 0, 2: the block's first mover
    const uint32_t d1 = lrow < 2 ? 1u : 6u, d2 = lrow < 2 ? 7u : 8u;
    // lane 7a + b (< 49): the columns {a, b} (a == b: one column) whose fills a block may see
    const uint32_t pairbits = lane < 49u ? (1u << (lane / 7u)) | (1u << (lane % 7u)) : 0u;
    // per leaf, lane-parallel (lane = leaf of a group of 64): side to move / last mover stones,
    // 41 - stones (-2: has_four(last mover), the leaf is won), read out by readlane when the
    // leaf's turn comes
    for (int g = 0; g < nb; g += 64) {
      uint32_t lm_v = 0, ow_v = 0, hp_v = 0;
      int room_v = 0;
      {
        const int jj = g + (int)lane;
        if (jj < nb) {
            lm_v = L[jj].meta;
            ow_v = L[jj].ow;
            const uint64_t x0 = L[jj].p0, x1 = L[jj].p1;
            const uint64_t op_v = (lm_v >> 24) & 1u ? x0 : x1;
            room_v = has_four(op_v) ? -2 : 41 - __popcll(x0 | x1);
            const uint64_t oc = x0 | x1;  // column heights, 4 bits per column
            for (int c = 0; c < 7; ++c) hp_v |= (uint32_t)__popcll((oc >> (7 * c)) & 0x3Full) << (4 * c);
        }
      }
      const int jend = min(nb, g + 64);
      for (int j = g; j < jend; ++j) {
        RMARK(6);  // regions: 1 leaf setup, 2 view, 3 first segment, 4 absorbed fill, 5 win test, 6 block tail
        const int jl = j - g;
        const uint32_t lm = (uint32_t)__builtin_amdgcn_readlane((int)lm_v, jl);
        // the leaf's boards straight from LDS into VGPRs (one uniform address per read: a
        // broadcast), in flight while the first view is gathered
        const uint32_t tnv = (lm >> 24) & 1u;
        const uint64_t *const pp = &L[j].p0;
        uint64_t me = in_vgpr(pp[tnv]);       // side to move
        uint64_t op = in_vgpr(pp[tnv ^ 1u]);  // last mover
        uint32_t hp = (uint32_t)__builtin_amdgcn_readlane((int)hp_v, jl);  // column heights, carried across blocks
        const uint32_t low0 = (uint32_t)__builtin_amdgcn_readlane((int)ow_v, jl);
        const int room0 = __builtin_amdgcn_readlane(room_v, jl);
        const bool won = room0 == -2;
        int val = 0;
        int q = 0;  // plies played in this rollout (room0 - room when it ends)
        RMARK(1);
        if (won) {  // has_four(last mover)
            val = -1;
        } else if (room0 >= 0) {  // not check_draw
            int room = room0;
            int mask = (int)(lm >> 25);
            uint32_t ow = low0;
            uint32_t n = (ow >> 24) & 15u;
            uint32_t sh = (uint32_t)__builtin_clz(n);  // n >= 1 (room >= 0)
            // order words of the legal set minus the columns of `pairbits`, for the fills
            // (read as soon as the legal set is known, well before a fill needs it)
            uint32_t owp = s_order[(uint32_t)mask & ~pairbits];
            for (;;) {
                RMARK(6);
                uint32_t wv, v;
                uint64_t A;  // accepted words
                // a view without an accepted word (2^-64 at worst) is consumed whole, in a loop
                // of its own off the common path (no loop-carried copies of the stream position)
                if (rng.off >= (uint32_t)kWin) rng_advance(rng);
                wv = rng_view(rng);  // lane l: word off + l
                v = wv >> sh;
                A = __ballot(v < n);
                if (__builtin_expect(A == 0ull, 0)) {
                    do {
                        rng.off += (uint32_t)kWin;
                        rng_advance(rng);
                        wv = rng_view(rng);
                        v = wv >> sh;
                        A = __ballot(v < n);
                    } while (A == 0ull);
                }
#ifndef ZC_DIAG_WASTE
                cn.add(cn.blocks, 1);
#endif
                RMARK(2);
                const uint32_t cap_r = min((uint32_t)room, 30u);  // last ply index the board allows
                uint32_t qk = mbcnt(A);                            // this lane's ply in the block
                uint32_t col = (ow >> (3 * v)) & 7u;  // its column (if accepted; v < 8 as n < 8)
                // the ply's row: the column's height (hp, 4 bits per column, carried from block
                // to block) + earlier plies in the same column (4-bit per-column counters,
                // prefix-summed).  A nibble only overflows into the next column's after its own
                // column filled — beyond the block's end, in lanes never read.
                uint32_t one = mask_sel0(A, 1u << (4 * col));
                uint32_t sc = scan_add32(one);
                uint32_t row = ((sc - one + hp) >> (4 * col)) & 15u;  // the column's height + earlier plies in it
                uint32_t nacc = (uint32_t)__popcll(A);
                // the fills, kept as a wave mask (a per-lane bool merged across the absorption
                // would be materialised and compared again)
                uint64_t F = __ballot(row == 5u);
                // the block's end: its first fill, or the first ply past the cap / the view's last
                // accepted word (masks ANDed on the scalar unit, one lane compare)
                uint64_t E0 = A & (F | __ballot(qk >= min(cap_r, nacc - 1u)));
                uint32_t l0 = (uint32_t)__builtin_ctzll(E0);
                // the fills with room for more plies after them: the block's end is one of these
                // exactly when it is the first of them
                const uint64_t G = A & F & __ballot(qk < cap_r);
                // the first fill, with room for more plies: re-draw the words after it under
                // the new legal set
#if !(ZC_RV & 1)
                uint32_t lf = 64u;  // lane of the absorbed fill (64: none)
                uint32_t cf = 0;
                RMARK(3);
                if (ff1(G) == l0) {  // a fill with room for more plies
                    lf = l0;
                    cf = (uint32_t)__builtin_amdgcn_readlane((int)col, (int)lf);
                    const uint32_t ow2 = (uint32_t)__builtin_amdgcn_readlane((int)owp, (int)(8u * cf));
                    const uint32_t n2 = (ow2 >> 24) & 15u;
                    const uint32_t v2 = wv >> __clz(n2);
                    const uint64_t low = (2ull << lf) - 1ull;  // lanes 0..lf
                    A = (A & low) | (__ballot(v2 < n2) & ~low);
                    qk = mbcnt(A);
                    col = mask_sel(low, (ow2 >> (3 * v2)) & 7u, col);  // lanes after lf: the new order
                    one = mask_sel0(A, 1u << (4 * col));
                    sc = scan_add32(one);
                    row = ((sc - one + hp) >> (4 * col)) & 15u;
                    nacc = (uint32_t)__popcll(A);
                    F = __ballot(row == 5u) & ~low;  // the absorbed fill no longer ends the block
                    E0 = A & (F | __ballot(qk >= min(cap_r, nacc - 1u)));
                    l0 = (uint32_t)__builtin_ctzll(E0);
                }
                RMARK(4);
                // compact EVERY accepted word's ply by parity: ply q < 32 to lane (q & 1)*16 + q/2
                // (a forward lane permute; the other lanes, and plies >= 32, land in lanes 32..63),
                // then copy lanes 0..31 up over lanes 32..63.  No ply past the block's last one (at
                // lane l0) needs masking: each row's plies ascend along its lanes, so a later ply's
                // stones only reach its own prefix, and its win can only show up in a word lane
                // beyond l0 (the end is min(first win, l0) below)
                const uint32_t c = ((qk & 1u) << 4) | ((qk >> 1) & 15u) | (qk & 32u);
                const uint32_t b = __umul24(col, 7u) + row;  // the ply's cell (a 24-bit mad, not a 64-bit one)
                const uint32_t pl = (uint32_t)__builtin_amdgcn_ds_permute((int)(mask_sel(A, 63u, c) << 2), (int)b);
                const uint32_t pb = __builtin_amdgcn_permlane32_swap(pl, pl, false, false)[0];
                const uint64_t bit = 1ull << (pb & 63u);
                uint32_t blo = (uint32_t)bit, bhi = (uint32_t)(bit >> 32);
                scan_or16x2(blo, bhi);
                const uint64_t mine = ((uint64_t)bhi << 32) | blo;  // this row's stones so far
                const uint64_t bd = (first_row ? me : op) | mine;
                const uint64_t m1 = bd & (bd >> d1), m2 = bd & (bd >> d2);
                const uint64_t f4 = (m1 & (m1 >> (2 * d1))) | (m2 & (m2 >> (2 * d2)));
                const uint64_t W = __ballot(f4 != 0ull);
                // back to word order: the accepted lane of ply qk won if its compacted lane did
                const uint32_t W32 = (uint32_t)W | (uint32_t)(W >> 32);
                const uint64_t Ew = A & __ballot(((W32 >> (c & 31u)) & 1u) != 0u);
#else
                uint32_t lf = 64u;  // lane of the absorbed fill (64: none)
                uint32_t cf = 0;
                // compact EVERY accepted word's ply by parity: ply q < 32 to lane (q & 1)*16 + q/2
                // (a forward lane permute; the other lanes, and plies >= 32, land in lanes 32..63),
                // then copy lanes 0..31 up over lanes 32..63.  No ply past the block's last one (at
                // lane l0) needs masking: each row's plies ascend along its lanes, so a later ply's
                // stones only reach its own prefix, and its win can only show up in a word lane
                // beyond l0 (the end is min(first win, l0) below).  Returns the accepted word lanes
                // whose ply completed four; mine_ = each row's stones so far.
                auto win_test = [&](uint64_t A_, uint32_t qk_, uint32_t col_, uint32_t row_, uint64_t &mine_) {
                    const uint32_t c = ((qk_ & 1u) << 4) | ((qk_ >> 1) & 15u) | (qk_ & 32u);
                    const uint32_t b = __umul24(col_, 7u) + row_;  // the ply's cell (a 24-bit mad, not a 64-bit one)
                    const uint32_t pl = (uint32_t)__builtin_amdgcn_ds_permute((int)(mask_sel(A_, 63u, c) << 2), (int)b);
                    const uint32_t pb = __builtin_amdgcn_permlane32_swap(pl, pl, false, false)[0];
                    const uint64_t bit = 1ull << (pb & 63u);
                    uint32_t blo = (uint32_t)bit, bhi = (uint32_t)(bit >> 32);
                    scan_or16x2(blo, bhi);
                    mine_ = ((uint64_t)bhi << 32) | blo;  // this row's stones so far
                    const uint64_t bd = (first_row ? me : op) | mine_;
                    const uint64_t m1 = bd & (bd >> d1), m2 = bd & (bd >> d2);
                    const uint64_t f4 = (m1 & (m1 >> (2 * d1))) | (m2 & (m2 >> (2 * d2)));
                    const uint64_t W = __ballot(f4 != 0ull);
                    // back to word order: the accepted lane of ply qk won if its compacted lane did
                    const uint32_t W32 = (uint32_t)W | (uint32_t)(W >> 32);
                    return A_ & __ballot(((W32 >> (c & 31u)) & 1u) != 0u);
                };
                // ZC_RV & 1 (experiment): an absorbed fill's first segment (plies through the fill,
                // the same before and after the re-draw) is win-tested on the pre-re-draw plies,
                // independent of the re-draw, so the two chains can overlap; a win there ends the
                // block without the second test
                uint64_t Ew1 = 0, mine1 = 0;
                RMARK(3);
                if (ff1(G) == l0) {  // a fill with room for more plies
                    lf = l0;
                    cf = (uint32_t)__builtin_amdgcn_readlane((int)col, (int)lf);
                    const uint32_t ow2 = (uint32_t)__builtin_amdgcn_readlane((int)owp, (int)(8u * cf));
                    const uint32_t n2 = (ow2 >> 24) & 15u;
                    const uint32_t v2 = wv >> __clz(n2);
                    const uint64_t low = (2ull << lf) - 1ull;  // lanes 0..lf
                    if (ZC_RV & 1) Ew1 = win_test(A, qk, col, row, mine1) & low;
                    A = (A & low) | (__ballot(v2 < n2) & ~low);
                    qk = mbcnt(A);
                    col = mask_sel(low, (ow2 >> (3 * v2)) & 7u, col);  // lanes after lf: the new order
                    one = mask_sel0(A, 1u << (4 * col));
                    sc = scan_add32(one);
                    row = ((sc - one + hp) >> (4 * col)) & 15u;
                    nacc = (uint32_t)__popcll(A);
                    F = __ballot(row == 5u) & ~low;  // the absorbed fill no longer ends the block
                    E0 = A & (F | __ballot(qk >= min(cap_r, nacc - 1u)));
                    l0 = (uint32_t)__builtin_ctzll(E0);
                }
                RMARK(4);
                uint64_t mine, Ew;
                if ((ZC_RV & 1) && Ew1 != 0ull) {  // the win precedes the fill (l0 >= lf after the re-draw)
                    Ew = Ew1;
                    mine = mine1;
                } else {
                    Ew = win_test(A, qk, col, row, mine);
                }
#endif
                const uint32_t ew = ff1(Ew);
                const uint32_t endlane = min(ew, l0);
                const bool win = ew <= l0;  // (ff1 of an empty mask is 0xFFFFFFFF)
                const uint32_t endply = (uint32_t)__builtin_amdgcn_readlane((int)qk, (int)endlane);
                rng.off += endlane + 1u;  // words through the block's last ply are consumed
#ifdef ZC_DIAG_WASTE
                cn.add(cn.blocks, lf < 64u && endlane < lf ? 1 : 0);
                cn.add(cn.plies, lf < 64u ? 1 : 0);
#endif
                room -= (int)endply + 1;
                RMARK(5);
                if (win) {  // the ply's mover completed four
                    val = ((room0 - room) & 1) ? 1 : -1;  // an odd number of plies: the leaf's side won
                    break;
                }
                if (room < 0) {  // check_draw: board full
                    val = 0;
                    break;
                }
                // the rollout goes on (most end in their first block, so this is off the common
                // path): both sides' stones after ply endply — first mover through ply
                // 2*(endply/2) (row 0, inclusive), second mover through the odd plies <= endply
                // (row 1, inclusive scan at lane 15 + (endply+1)/2; none when endply = 0)
                {
                    const uint64_t s2 = readlane64(mine, (int)((endply + 31u) >> 1));
                    const uint64_t a2 = me | readlane64(mine, (int)(endply >> 1));
                    const uint64_t b2 = op | (endply ? s2 : 0ull);
                    const bool odd = endply & 1u;  // an even number of plies: the first mover is to move again
                    me = odd ? a2 : b2;
                    op = odd ? b2 : a2;
                }
                hp += (uint32_t)__builtin_amdgcn_readlane((int)sc, (int)endlane);  // plies per column through endlane
                // the legal set (and its CPython order) after the block's fills: the absorbed
                // one if it was played, and the one the block ended at
                const bool fa = endlane >= lf;
                const bool fe = (F >> endlane) & 1u;
                {  // unconditional (selects), so the block loop carries one copy of its state
                    const uint32_t ce = fe ? (uint32_t)__builtin_amdgcn_readlane((int)col, (int)endlane) : cf;
                    const uint32_t ca = fa ? cf : ce;
                    const bool ff = fa | fe;
                    mask = ff ? mask & ~((1 << ca) | (1 << ce)) : mask;
                    const uint32_t ownew = (uint32_t)__builtin_amdgcn_readlane((int)owp, (int)((7u * ca + ce) & 63u));
                    ow = ff ? ownew : ow;
                    owp = s_order[(uint32_t)mask & ~pairbits];
                }
                n = (ow >> 24) & 15u;
                sh = (uint32_t)__builtin_clz(n);
            }
            q = room0 - room;
        }
        L[j].val = val;  // uniform: every lane stores
#ifndef ZC_DIAG_WASTE
        cn.add(cn.plies, q);
#endif
      }
    }
}

// Philox rollout mode ("rollout fast mode", statistical parity only).
// Value.random_rollout's game (value_functions.py:35-45) — uniform random legal moves until
// check_win (last mover) or check_draw — with the random numbers taken from a per-leaf
// counter-based stream instead of the game's one MT19937 stream.  Leaves no longer depend on
// each other, so the flush's leaves roll out in parallel, one per lane.  Leaf j of the flush
// that starts at simulation `leaf0` seeds xoshiro128** with Philox4x32-10(counter = (leaf0 +
// j, tag, game, 0x0C4F0A57), key = seed), tag = the game's MT position at the search's start
// (a different stream every move); each ply takes one draw u and plays the k-th legal column
// in ascending order, k = (u * n) >> 32.  Specification: tests/c4_philox_ref.py.
__device__ void c4_rollouts_philox(Leaf *L, int nb, const uint8_t *s_sel, uint2 key, uint32_t leaf0, uint32_t tag,
                                   uint32_t game, Counters &cn) {
    const uint32_t lane = lane_id();
    for (int base = 0; base < nb; base += kBlock) {
        const int j = base + (int)lane;
        int val = 0, q = 0;
        if (j < nb) {
            const uint64_t x0 = L[j].p0, x1 = L[j].p1;
            const bool tn = (L[j].meta >> 24) & 1u;
            uint64_t me = tn ? x1 : x0;  // side to move
            uint64_t op = tn ? x0 : x1;  // last mover
            int stones = __popcll(me | op);
            if (has_four(op)) {
                val = -1;
            } else if (stones < 42) {
                uint32_t legal = (uint32_t)legal_mask(me | op);
                const uint4 sd = philox(make_uint4(leaf0 + (uint32_t)j, tag, game, 0x0C4F0A57u), key);
                Xoshiro128 x{sd.x | ((sd.x | sd.y | sd.z | sd.w) == 0u), sd.y, sd.z, sd.w};
                for (;;) {
                    const uint32_t n = (uint32_t)__popc(legal);
                    const uint32_t k = __umulhi(x.next(), n);
                    const uint32_t col = s_sel[legal * 8u + k];
                    const uint32_t h = (uint32_t)__popcll(((me | op) >> (7u * col)) & 0x3Full);
                    me |= 1ull << (7u * col + h);
                    ++q;
                    ++stones;
                    if (h == 5u) legal &= ~(1u << col);
                    if (has_four(me)) {  // the ply's mover completed four
                        val = (q & 1) ? 1 : -1;
                        break;
                    }
                    if (stones == 42) {  // check_draw
                        val = 0;
                        break;
                    }
                    const uint64_t t = me;
                    me = op;
                    op = t;
                }
            }
            L[j].val = val;
        }
        int tot = q;
        for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
        cn.add(cn.plies, tot);
    }
}

// ------------------------------------------------------------------ planned flush expansion
// select_flush (c4_device.h) walks the flush's fresh nodes one at a time: per node a view of
// draws, a Lehmer decode, the children built and stored, then a descent — ~2.9 k cycles per
// node at 16 waves per CU, 14 % of the search.  But below X0 the flush's shape does not depend
// on the draws: a node takes min(#untried, leaves left) draws, and once every untried move of
// it is drawn the next walk enters its LOWEST untried slot (its fresh children all score
// +inf; old children have Na >= 1), whatever the draws were — for X0 the lowest untried
// slot, for a fresh node slot 0.  So the chain of nodes X0 = C0, C1, ... (boards, move
// counts, draws per node) is known before any draw is decoded; only the node IDS on the chain
// (C_{i+1} = the child of the draw that took that slot) depend on the draws.
// select_flush_plan therefore (1) walks the chain on the scalar unit, running each node's
// draws (the same ballots + branch-free chain as select_flush) over a shared view and
// recording the node in an LDS table; (2) builds every fresh node and leaf in ONE
// lane-parallel pass, lane d = draw d = node f0 + d: its node's table entry, its r value, the
// Lehmer decode inside its node's draws, its parent id (the draw of the previous chain node
// that took position 0 of that node's untried list), its child's board, order word and
// records; (3) patches the chain nodes' child slots and untried words (LDS atomics) and
// X0's.  Same tree, same leaves, same stream consumption as select_flush (nb < 64: one lane
// per draw; the rollout search only — select_flush records leaf paths for the stepwise search).
struct ChainNode {
    uint64_t p0, p1;  // the node's stones
    uint32_t ow;      // its move-list order word
    uint32_t info;    // n (draws are over n, n-1, ...) | m << 4 | first draw << 8 | depth << 16 | turn << 24 | legal << 25
    uint32_t ul;      // its untried list (move indices in list order, 3 bits each)
    uint32_t pad;
};
static_assert(sizeof(ChainNode) == 32, "chain table entry");

__device__ __forceinline__ uint64_t lanes_in(int lo, int hi) {  // lanes lo .. hi-1 (0 <= lo <= hi <= 64)
    const uint64_t below_hi = hi >= 64 ? ~0ull : (1ull << hi) - 1ull;
    return below_hi & ~((1ull << lo) - 1ull);
}

// walk_hbm (c4_device.h) for the rollout search, with the next level's record fetched while
// the current level's UCT is computed: lane 8c + k loads slot k (child, Na, Wa) and header word
// k & 3 of child c's record as soon as the node's children are known, so the memory latency of
// a level hides under the previous level's fp64 arithmetic; the chosen child's slots then move
// to lanes k by three bpermutes.  Same walk, same path, same result.
__device__ __forceinline__ WalkEnd walk_hbm_prefetch(const Tree &t, ConstDouble *logtab, uint64_t rp0, uint64_t rp1,
                                                     int rturn, int done, double c, int &status) {
    const uint32_t lane = lane_id();
    const uint32_t k = lane & 7u, cs = lane >> 3;  // the slot this lane scores / the child it fetches
    int node = 0, depth = 0, turn = rturn, nN = done;  // nN = N(node) = Na of its in-edge
    uint64_t b0 = rp0, b1 = rp1;
    uint32_t pathv = (lane == 0) ? 0x00FF0000u : 0u;
    const uint8_t *R0 = t.rec(0);
    uint32_t u = uni(((const uint32_t *)R0)[1]), ow = uni(((const uint32_t *)R0)[3]);
    uint32_t ch = ((const uint16_t *)(R0 + 16))[k];
    int32_t na = ((const int32_t *)(R0 + 32))[k];
    int32_t wa = ((const int32_t *)(R0 + 64))[k];
    for (;;) {  // select (mcts.cpp:47-63) over HBM records
        if (untried_count(u)) break;  // untried moves left: expand here
        if (depth >= kMaxDepth - 2) {  // unreachable (a C4 tree is <= 42 deep); never spin
            status = ZC_STATUS_INTERNAL;
            u = 0;
            break;
        }
        const uint32_t nm = u >> 28;
        // the children's records, in flight during the selection below
        const uint32_t cid = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(cs << 2), (int)ch);
        uint32_t pch = 0xFFFFu, phd = 0u;
        int32_t pna = 0, pwa = 0;
        if (cs < nm && cid != 0xFFFFu) {
            const uint8_t *Rc = t.rec((int)cid);
            phd = ((const uint32_t *)Rc)[lane & 3u];
            pch = ((const uint16_t *)(Rc + 16))[k];
            pna = ((const int32_t *)(Rc + 32))[k];
            pwa = ((const int32_t *)(Rc + 64))[k];
        }
        const double lg = logtab[nN];  // log(N), glibc values tabulated on the host
        const bool valid = k < nm && ch != 0xFFFF;
        int best;
        const uint64_t unvisited = ((1ull << nm) - 1ull) & __ballot(ch != 0xFFFF) & __ballot(na == 0) & 0xFFull;
        if (unvisited) {  // +inf beats everything; first such slot
            best = __builtin_ctzll(unvisited);
        } else {
            // UCT (mcts.cpp:41-45) = fma(c, sqrt(log(N)/Na), Qa), first max in slot order
            const double q = valid ? (double)wa / (double)na : 0.0;
            const double v = valid ? fma(c, sqrt(lg / (double)na), q) : -INFINITY;
            int bi;
            if (ZC_MAX8) {
                const double mx = max8_first(v, &bi);
                if ((__ballot(mx == -INFINITY) & 1ull) != 0) break;  // no child: terminal leaf
            } else {
                double vv = v;
                bi = (int)k;
                argmax8(vv, bi);
                if ((__ballot(vv == -INFINITY) & 1ull) != 0) break;
                bi = uni(bi);
            }
            best = bi;
        }
        nN = __builtin_amdgcn_readlane(na, best);
        const uint64_t bit = drop_bit(b0 | b1, (int)((ow >> (3 * best)) & 7u));
        if (turn) b1 |= bit; else b0 |= bit;
        turn ^= 1;
        node = __builtin_amdgcn_readlane((int)ch, best);
        ++depth;
        if (lane == (uint32_t)depth) pathv = (uint32_t)node | ((uint32_t)best << 16);
        const int src = (int)((8u * (uint32_t)best + k) << 2);
        ch = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)pch);
        na = __builtin_amdgcn_ds_bpermute(src, pna);
        wa = __builtin_amdgcn_ds_bpermute(src, pwa);
        u = (uint32_t)__builtin_amdgcn_readlane((int)phd, 8 * best + 1);
        ow = (uint32_t)__builtin_amdgcn_readlane((int)phd, 8 * best + 3);
    }
    return WalkEnd{node, depth, turn, b0, b1, pathv, u, ow, ch};
}

template <bool STAMP, class RNG>
__device__ __forceinline__ void select_flush_plan(const Tree &t, Fresh *fresh, Leaf *leaves, ChainNode *chain,
                                                  const uint32_t *s_order, ConstDouble *logtab, RNG &rng,
                                                  Counters &cn, Stamp<STAMP> &stamp, int &nnodes, int &status,
                                                  uint64_t rp0, uint64_t rp1, int rturn, int done, int nb, double c,
                                                  FlushSel &fs) {
    const uint32_t lane = lane_id();
    const int f0 = nnodes;
    for (int i = (int)lane; i < nb; i += 64) {  // fresh slots: no children, zero in-edge counters
        fresh[i].na = 0;
        fresh[i].w = 0;
        *(uint4 *)fresh[i].ch = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
    }
#ifndef ZC_WALK_PREFETCH
#define ZC_WALK_PREFETCH 1
#endif
    const WalkEnd we = ZC_WALK_PREFETCH ? walk_hbm_prefetch(t, logtab, rp0, rp1, rturn, done, c, status)
                                        : walk_hbm<false>(t, logtab, rp0, rp1, rturn, done, c, status);
    fs.f0 = f0;
    fs.x0node = we.node;
    fs.d0 = we.depth;
    fs.ppath = we.pathv;
    fs.x_u = we.u;
    fs.x_ch = we.ch;
    fs.x0_dirty = false;
    stamp.mark(1);
    const uint32_t cnt0 = untried_count(we.u);
    if (cnt0 == 0) {  // X0 has no move (full board): every leaf of the flush is X0
        const uint32_t meta = (uint32_t)we.node | ((uint32_t)we.depth << 16) | ((uint32_t)we.turn << 24) |
                              ((uint32_t)legal_mask(we.b0 | we.b1) << 25);
        for (int i = (int)lane; i < nb; i += 64) leaves[i] = Leaf{we.b0, we.b1, meta, 0, we.ow, 0};
        wave_mem_order();
        stamp.mark(3);
        return;
    }

    // ---- (1) the chain, its draws and its table
    constexpr uint32_t kIdentList = 0x1AC688u;  // 0, 1, ..., 6
    uint64_t b0 = we.b0, b1 = we.b1;
    int turn = we.turn, depth = we.depth;
    uint32_t ow = we.ow, cm = (uint32_t)legal_mask(b0 | b1), n = cnt0, ul = 0;
    {
        uint32_t k = 0;
        for (uint32_t bb = 0; bb < 7; ++bb)
            if ((we.u >> bb) & 1u) ul |= bb << (3 * k++);
    }
    int d = 0, i = 0, T = -1;  // draws so far, chain node, the terminal chain node (full board)
    uint64_t Sm = 0;           // bit s: a chain node's first draw
    uint32_t raw = 0;          // lane d: the accepted word of draw d
    if (rng.off >= (uint32_t)kWin) rng_advance(rng);
    uint32_t w = rng_view(rng);  // lane l: word off + l
    uint32_t t3 = w >> 29;
    uint64_t gt = ~0ull, Fv = 0;  // the view: lanes after the last accepted word; accepted words
    int dv0 = 0;                  // first draw of the view
    for (;;) {
        const int m = min((int)n, nb - d);
        if (lane == 0)
            chain[i] = ChainNode{b0, b1, ow,
                                 n | ((uint32_t)m << 4) | ((uint32_t)d << 8) | ((uint32_t)depth << 16) |
                                     ((uint32_t)turn << 24) | (cm << 25),
                                 ul, 0u};
        if (m == 0) {  // a chain node without moves: the flush's remaining leaves are all it
            T = i;
            break;
        }
        Sm |= 1ull << d;
        int k = 0;
        for (;;) {  // this node's draws over n - k, n - k - 1, ... (a view at a time)
            const int rem = m - k, cnt = (int)n - k;  // rem: 1 .. 7
            // _randbelow(nn) accepts a word when (w >> (32 - bit_length(nn))) < nn, i.e. when its
            // top three bits t3 are below T(nn) = 4, 4, 6, 4, 5, 6, 7 for nn = 1 .. 7 (nn = 1, 2:
            // the top bit / two bits; nn = 3: the top two bits < 3).  Step s draws over cnt - s
            // moves: its threshold is nibble s of P (0 past rem: no word accepted).
            const uint32_t P = (0x04464567u >> (4u * (uint32_t)(7 - cnt))) & ((1u << (4u * (uint32_t)rem)) - 1u);
            uint64_t A[7];
#pragma unroll
            for (int s = 0; s < 7; ++s) A[s] = __ballot(t3 < ((P >> (4u * s)) & 15u));
            // the draws, a scalar chain: each takes the lowest accepted word after the last one
            // (s_ff1; none: -1, and gt = -2 << 63 = 0 stops the later steps), its bit = acc & ~gt
            uint64_t F = 0;
#pragma unroll
            for (int s = 0; s < 7; ++s) {
                const uint64_t acc = A[s] & gt;
                gt = (~1ull) << (ff1(acc) & 63u);
                F |= acc & ~gt;
            }
            Fv |= F;
            const int nd = __popcll(F);
            k += nd;
            d += nd;
            if (k < m) {  // the view ran out: all of it is consumed; its draws go to their lanes
                const uint32_t di = (uint32_t)dv0 + mbcnt64(Fv);
                const uint32_t got =
                    (uint32_t)__builtin_amdgcn_ds_permute((int)(mask_sel(Fv, 63u, di) << 2), (int)w);
                raw = mask_sel(lanes_in(dv0, d), raw, got);
                rng.off += (uint32_t)kWin;
                rng_advance(rng);
                w = rng_view(rng);
                t3 = w >> 29;
                gt = ~0ull;
                Fv = 0;
                dv0 = d;
                continue;
            }
            // the node's draws are done: the next node's start after its last word (the steps
            // past rem zeroed gt)
            gt = (~1ull) << (63 - __clzll(Fv));
            break;
        }
        if (d >= nb) break;
        // the next walk enters this node's lowest untried slot
        const int col = (int)((ow >> (3 * (ul & 7u))) & 7u);
        const uint64_t bit = drop_bit(b0 | b1, col);
        if (turn) b1 |= bit; else b0 |= bit;
        turn ^= 1;
        ++depth;
        if (bit & kTop) {
            cm &= ~(1u << col);
            ow = uni(s_order[cm]);
        }
        n = (ow >> 24) & 15u;
        ul = kIdentList;
        ++i;
    }
    {  // the last view's draws (it always has one: a view is only left once it ran out)
        const uint32_t di = (uint32_t)dv0 + mbcnt64(Fv);
        const uint32_t got = (uint32_t)__builtin_amdgcn_ds_permute((int)(mask_sel(Fv, 63u, di) << 2), (int)w);
        raw = mask_sel(lanes_in(dv0, d), raw, got);
        rng.off += (uint32_t)(63 - __clzll(Fv | 1ull)) + 1u;
    }
    const int D = d;  // fresh nodes f0 .. f0 + D - 1
    wave_mem_order();
    stamp.mark(2);

    // ---- (2) every fresh node and leaf, lane d = draw d
    const bool act = (int)lane < D;
    const uint32_t seg = act ? mbcnt64(Sm) + (uint32_t)((Sm >> lane) & 1ull) - 1u : 0u;
    const ChainNode e = chain[seg];
    const uint32_t s_i = (e.info >> 8) & 0xFFu;
    const uint32_t dd = lane - s_i;  // the draw's index inside its node
    const uint32_t r = raw >> __clz(act ? (e.info & 15u) - dd : 1u);
    // draw dd's position in the node's untried list as it was before the node's draws
    // (select_flush's Lehmer decode, each lane against its own node's earlier draws)
    uint32_t rp[6];
#pragma unroll
    for (int s = 0; s < 6; ++s) rp[s] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((s_i + (uint32_t)s) << 2), (int)r);
    uint32_t pl = r;
#pragma unroll
    for (int s = 5; s >= 0; --s) pl += (dd > (uint32_t)s && pl >= rp[s]) ? 1u : 0u;
    const uint32_t mi = (e.ul >> (3 * (pl & 7u))) & 7u;
    const uint64_t Z = __ballot(act && pl == 0);  // per chain node: the draw holding its lowest untried slot
    const uint64_t zl = Z & ((1ull << s_i) - 1ull);
    const int parent = seg == 0 ? we.node : f0 + 63 - __clzll(zl | 1ull);
    {
        const uint32_t col = (e.ow >> (3 * mi)) & 7u;
        const uint64_t bit = drop_bit(e.p0 | e.p1, (int)col);
        const uint32_t tn = (e.info >> 24) & 1u, ldepth = ((e.info >> 16) & 0xFFu) + 1u;
        const bool filled = (bit & kTop) != 0;
        const uint32_t c_lmask = (e.info >> 25) & ~(filled ? 1u << col : 0u);
        uint32_t c_low = e.ow;
        if (act && filled) c_low = s_order[c_lmask];
        if (act) {
            *(uint4 *)&fresh[lane] = make_uint4(untried_init((c_low >> 24) & 15u), c_low,
                                                (uint32_t)parent | (mi << 16) | (ldepth << 24), c_lmask);
            leaves[lane] = Leaf{tn ? e.p0 : (e.p0 | bit), tn ? (e.p1 | bit) : e.p1,
                                ((uint32_t)f0 + lane) | (ldepth << 16) | ((tn ^ 1u) << 24) | (c_lmask << 25), 0,
                                c_low, 0};
        }
    }
    if (T >= 0) {  // the terminal chain node (entered from the full node before it)
        const ChainNode et = chain[T];
        const uint32_t meta = (uint32_t)(f0 + 63 - __clzll(Z | 1ull)) | (((et.info >> 16) & 0xFFu) << 16) |
                              (((et.info >> 24) & 1u) << 24) | ((et.info >> 25) << 25);
        for (int jj = D + (int)lane; jj < nb; jj += 64) leaves[jj] = Leaf{et.p0, et.p1, meta, 0, et.ow, 0};
    }
    wave_mem_order();
    // ---- (3) the chain nodes' child slots and untried words; X0's
    if (act && seg != 0) {
        Fresh &P = fresh[parent - f0];
        P.ch[mi] = (uint16_t)(f0 + (int)lane);
        atomicAnd(&P.u, ~(1u << mi));
    }
    uint32_t slotbit = (act && seg == 0) ? 1u << mi : 0u;  // X0's draws are lanes 0 .. m0-1 (< 8)
    slotbit |= (uint32_t)dpp<0xB1>((int)slotbit);
    slotbit |= (uint32_t)dpp<0x4E>((int)slotbit);
    slotbit |= (uint32_t)dpp<0x141>((int)slotbit);
    const uint32_t ucl = uni(slotbit);
    const uint32_t sent =
        (uint32_t)__builtin_amdgcn_ds_permute((int)(((act && seg == 0) ? mi : 63u) << 2), (int)((uint32_t)f0 + lane));
    fs.x_ch = ((ucl >> (lane & 7u)) & 1u) ? sent : we.ch;
    fs.x_u = we.u & ~ucl;
    fs.x0_dirty = true;
    nnodes = f0 + D;
    wave_mem_order();
    {  // the flush's expansions and their depths (as select_flush)
        int dsum = 0;
        for (int base = 0; base < D; base += 64) {
            const int q = base + (int)lane;
            const uint32_t dep = q < D ? fresh[q].link >> 24 : 0u;
#pragma unroll
            for (int bit = 0; bit < 6; ++bit) dsum += __popcll(__ballot((dep >> bit) & 1u)) << bit;
        }
        cn.add(cn.expansions, D);
        cn.add(cn.depth_sum, dsum);
    }
    stamp.mark(3);
}

// ------------------------------------------------------------------ the planned flush, draws as a table chase
// select_flush_plan's step (1) spends ~110 scalar instructions per chain node (seven unrolled
// draw steps of five to seven SALU each, whatever the node's draw count, the view bookkeeping,
// the descent and the node's table entry written by lane 0) — about 26 SALU per simulation, the
// largest scalar cost of the walk.  But the chain's shape is known before any draw (see above),
// and with it the whole flush's sequence of draw counts: draw d of chain node i is over
// n_i - (d - d_i) moves.  _randbelow(cnt) accepts a word when its top three bits t3 are below
// T(cnt) (4, 4, 6, 4, 5, 6, 7 for cnt = 1..7): four acceptance classes c = T - 4.
// select_flush_plan2 therefore
//   (1a) walks the chain's shape on the scalar unit (boards, counts, first draws; each node's
//        fields go to VGPR lane i by v_writelane, no LDS table, no exec juggling);
//   (1b) builds, lane-parallel, a NEXT table over the 64-word view: lane l, byte c = 1 + the
//        first word >= l (of words 0..61) that a class-c draw accepts, or 63 (none; lanes 62
//        and 63 hold 63 in every byte, so the chase stays there);
//   (1c) chases it: draw d is q_{d+1} = byte c_d of readlane(table, q_d), one v_readlane and
//        one s_bfe_u32 per draw, and s_bitset1 records bit q of F; 63 -> bit 63 = the view ran
//        out (the failed draw rejected words q..61 and goes on at word 62 of a fresh view);
//   (2)  as select_flush_plan, the chain nodes' fields fetched by ds_bpermute.
// Same draws, same tree, same leaves, same stream consumption as select_flush_plan.
// s_bfe_u32 operand of a class-c draw: byte c of the table entry, 6 bits
__device__ __forceinline__ uint32_t draw_class_bfe(uint32_t cnt) {  // c = T(cnt) - 4
    return (6u << 16) | (((0xE480u >> (2u * cnt)) & 3u) << 3);
}

// The view's next-draw table (1b).
__device__ __forceinline__ uint32_t draw_table(uint32_t w) {
    const uint32_t lane = lane_id();
    const uint32_t t3 = lane < 62u ? (w >> 29) : 7u;
    uint32_t nx = 0;
#pragma unroll
    for (uint32_t c = 0; c < 4; ++c) {
        const uint64_t s = __ballot(t3 < 4u + c) >> lane;
        const uint32_t f = s ? lane + 1u + (uint32_t)__builtin_ctzll(s) : 63u;
        nx |= f << (8u * c);
    }
    return nx;
}

// lane i of v := the uniform value x (v_writelane_b32; no builtin in this toolchain; the lane
// select in M0, since one VALU instruction reads at most one SGPR here)
__device__ __forceinline__ void write_lane(int &v, uint32_t x, int i) {
    __asm__("v_writelane_b32 %0, %1, m0" : "+v"(v) : "s"(x), "{m0}"(i));
}

// one draw of the chase: the next position q = byte c of the table entry at q
__device__ __forceinline__ uint32_t draw_step(uint32_t nx, uint32_t q, uint32_t op) {
    const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)nx, (int)q);
    uint32_t r;
    __asm__("s_bfe_u32 %0, %1, %2" : "=s"(r) : "s"(x), "s"(op));
    return r;
}

// The first NDRAW draws of a view chased through its table: bit q of the result set for each
// draw's next position q (= its word + 1, 1..62), bit 63 = the view ran out.
template <int NDRAW>
__device__ __forceinline__ uint64_t draw_chase_fixed(uint32_t nx, uint32_t clsv) {
    uint64_t F = 0;
    uint32_t q = 0;
#pragma unroll
    for (int k = 0; k < NDRAW; ++k) {
        q = draw_step(nx, q, (uint32_t)__builtin_amdgcn_readlane((int)clsv, k));
        __asm__("s_bitset1_b64 %0, %1" : "+s"(F) : "s"(q));  // F |= 1 << q in one SALU
    }
    return F;
}

template <bool STAMP, class RNG>
__device__ __forceinline__ void select_flush_plan2(const Tree &t, Fresh *fresh, Leaf *leaves, const uint32_t *s_order,
                                                   ConstDouble *logtab, RNG &rng, Counters &cn, Stamp<STAMP> &stamp,
                                                   int &nnodes, int &status, uint64_t rp0, uint64_t rp1, int rturn,
                                                   int done, int nb, double c, FlushSel &fs) {
    const uint32_t lane = lane_id();
    const int f0 = nnodes;
#ifndef ZC_MERGED_BACKUP
#define ZC_MERGED_BACKUP 1  // 0: the fresh edges by LDS atomics up the parent links (A/B runs)
#endif
    for (int i = (int)lane; i < nb; i += 64) {  // fresh slots: no children (the in-edge counters: the backup)
        if (!ZC_MERGED_BACKUP) {
            fresh[i].na = 0;
            fresh[i].w = 0;
        }
        *(uint4 *)fresh[i].ch = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
    }
    const WalkEnd we = walk_hbm_prefetch(t, logtab, rp0, rp1, rturn, done, c, status);
    fs.f0 = f0;
    fs.x0node = we.node;
    fs.d0 = we.depth;
    fs.ppath = we.pathv;
    fs.x_u = we.u;
    fs.x_ch = we.ch;
    fs.x0_dirty = false;
    stamp.mark(1);
    const uint32_t cnt0 = untried_count(we.u);
    if (cnt0 == 0) {  // X0 has no move (full board): every leaf of the flush is X0
        const uint32_t meta = (uint32_t)we.node | ((uint32_t)we.depth << 16) | ((uint32_t)we.turn << 24) |
                              ((uint32_t)legal_mask(we.b0 | we.b1) << 25);
        for (int i = (int)lane; i < nb; i += 64) leaves[i] = Leaf{we.b0, we.b1, meta, 0, we.ow, 0};
        wave_mem_order();
        fs.planned = ZC_MERGED_BACKUP;  // D = 0: no fresh node
        stamp.mark(3);
        return;
    }

    // ---- (1a) the chain's shape: node i's fields in lane i of six VGPRs
    uint64_t b0 = we.b0, b1 = we.b1;
    int turn = we.turn;
    uint32_t ow = we.ow, cm = (uint32_t)legal_mask(b0 | b1), n = cnt0;
    uint32_t slot = (uint32_t)__builtin_ctz(we.u & 0x7Fu);  // X0: its lowest untried slot; fresh nodes: slot 0
    int d = 0, i = 0, T = -1;
    uint64_t Sm = 0;  // bit s: a chain node's first draw
    int v_b0l = 0, v_b0h = 0, v_b1l = 0, v_b1h = 0, v_ow = 0, v_cd = 0;  // v_cd: cm | first draw << 8 | n << 16
    for (;;) {
        const int m = min((int)n, nb - d);
        write_lane(v_b0l, (uint32_t)b0, i);
        write_lane(v_b0h, (uint32_t)(b0 >> 32), i);
        write_lane(v_b1l, (uint32_t)b1, i);
        write_lane(v_b1h, (uint32_t)(b1 >> 32), i);
        write_lane(v_ow, ow, i);
        write_lane(v_cd, cm | ((uint32_t)d << 8) | (n << 16), i);
        if (m == 0) {  // a chain node without moves: the flush's remaining leaves are all it
            T = i;
            break;
        }
        Sm |= 1ull << d;
        d += m;
        if (d >= nb) break;
        // the next walk enters this node's lowest untried slot
        const int col = (int)((ow >> (3 * slot)) & 7u);
        const uint64_t bit = drop_bit(b0 | b1, col);
        if (turn) b1 |= bit; else b0 |= bit;
        turn ^= 1;
        if (bit & kTop) {
            cm &= ~(1u << col);
            ow = uni(s_order[cm]);
        }
        n = (ow >> 24) & 15u;
        slot = 0;
        ++i;
    }
    const int D = d;  // fresh nodes f0 .. f0 + D - 1

    // lane d < D: its chain node's fields (ds_bpermute from lane seg), the draw's count and class
    const bool act = (int)lane < D;
    const uint32_t seg = act ? mbcnt64(Sm) + (uint32_t)((Sm >> lane) & 1ull) - 1u : 0u;
    const int sa = (int)(seg << 2);
    const uint32_t e_cd = (uint32_t)__builtin_amdgcn_ds_bpermute(sa, v_cd);
    const uint32_t s_i = (e_cd >> 8) & 0xFFu;  // the chain node's first draw
    const uint32_t dd = lane - s_i;            // the draw's index inside its node
    const uint32_t cnt = act ? (e_cd >> 16) - dd : 1u;
    const uint32_t clsv = draw_class_bfe(act ? cnt : 1u);

    // ---- (1b, 1c) the draws: raw (lane d: the accepted word of draw d)
    uint32_t raw = 0;
    {
        if (rng.off >= (uint32_t)kWin) rng_advance(rng);
        uint32_t w = rng_view(rng);
        uint32_t nx = draw_table(w);
        int V = 0;  // draws done
        uint64_t F = draw_chase_fixed<32>(nx, clsv);
        for (;;) {
            // this view's valid draws (bits 1..62 = the word after each), in draw order
            const uint64_t Fv = F & 0x7FFFFFFFFFFFFFFEull;
            const uint64_t G = Fv >> 1;  // lane p: word p is a draw
            const int nv = __popcll(G), need = D - V, take = min(nv, need);
            const uint32_t rank = mbcnt64(G);
            const bool send = ((G >> lane) & 1ull) && (int)rank < take;
            const uint32_t got = (uint32_t)__builtin_amdgcn_ds_permute(
                (int)((send ? (uint32_t)V + rank : 63u) << 2), (int)w);
            raw = mask_sel(lanes_in(V, V + take), raw, got);
            V += take;
            if (nv >= need) {  // done: the stream goes on after draw D-1's word
                const uint64_t lastw = __ballot(((G >> lane) & 1ull) && (int)rank == take - 1);
                rng.off += (uint32_t)__builtin_ctzll(lastw) + 1u;
                break;
            }
            uint32_t q;
            if (F >> 63) {  // ran out: the failed draw rejected words q..61 and goes on at word 62
                rng.off += 62u;
                if (rng.off >= (uint32_t)kWin) rng_advance(rng);
                w = rng_view(rng);
                nx = draw_table(w);
                q = 0;
            } else {  // (nb > 32) the fixed chase ended with the view left: go on in it
                q = nv ? 64u - (uint32_t)__clzll(G) : 0u;
                rng.off += q;
                if (rng.off >= (uint32_t)kWin) rng_advance(rng);
                w = rng_view(rng);
                nx = draw_table(w);
                q = 0;
            }
            // the rest of the draws from V, one at a time, in this view
            F = 0;
            for (int k = V; k < D; ++k) {
                q = draw_step(nx, q, (uint32_t)__builtin_amdgcn_readlane((int)clsv, k));
                F |= 1ull << q;
                if (q == 63u) break;
            }
        }
    }
    wave_mem_order();
    stamp.mark(2);

    // ---- (2) every fresh node and leaf, lane d = draw d
    const uint32_t e_ow = (uint32_t)__builtin_amdgcn_ds_bpermute(sa, v_ow);
    const uint64_t e_p0 = ((uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(sa, v_b0h) << 32) |
                          (uint32_t)__builtin_amdgcn_ds_bpermute(sa, v_b0l);
    const uint64_t e_p1 = ((uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(sa, v_b1h) << 32) |
                          (uint32_t)__builtin_amdgcn_ds_bpermute(sa, v_b1l);
    const uint32_t r = raw >> __clz(cnt);
    // draw dd's position in the node's untried list as it was before the node's draws
    // (select_flush's Lehmer decode, each lane against its own node's earlier draws)
    uint32_t rp[6];
#pragma unroll
    for (int s = 0; s < 6; ++s) rp[s] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((s_i + (uint32_t)s) << 2), (int)r);
    uint32_t pl = r;
#pragma unroll
    for (int s = 5; s >= 0; --s) pl += (dd > (uint32_t)s && pl >= rp[s]) ? 1u : 0u;
    // the move index: X0's untried list is the set bits of its untried mask in order (the
    // select table's row); a fresh node's is 0, 1, ..., n-1
    const uint32_t mi = seg == 0 ? (uint32_t)sel_table(s_order)[8u * (we.u & 0x7Fu) + (pl & 7u)] : pl;
    const uint64_t Z = __ballot(act && pl == 0);  // per chain node: the draw holding its lowest untried slot
    const uint64_t zl = Z & ((1ull << s_i) - 1ull);
    const int parent = seg == 0 ? we.node : f0 + 63 - __clzll(zl | 1ull);
    {
        const uint32_t col = (e_ow >> (3 * mi)) & 7u;
        const uint64_t bit = drop_bit(e_p0 | e_p1, (int)col);
        const uint32_t tn = (uint32_t)we.turn ^ (seg & 1u), ldepth = (uint32_t)we.depth + seg + 1u;
        const bool filled = (bit & kTop) != 0;
        const uint32_t c_lmask = (e_cd & 0x7Fu) & ~(filled ? 1u << col : 0u);
        uint32_t c_low = e_ow;
        if (act && filled) c_low = s_order[c_lmask];
        if (act) {
            *(uint4 *)&fresh[lane] = make_uint4(untried_init((c_low >> 24) & 15u), c_low,
                                                (uint32_t)parent | (mi << 16) | (ldepth << 24), c_lmask);
            leaves[lane] = Leaf{tn ? e_p0 : (e_p0 | bit), tn ? (e_p1 | bit) : e_p1,
                                ((uint32_t)f0 + lane) | (ldepth << 16) | ((tn ^ 1u) << 24) | (c_lmask << 25), 0,
                                c_low, 0};
        }
    }
    if (T >= 0) {  // the terminal chain node (entered from the full node before it)
        const uint64_t tp0 = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(v_b0h, T) << 32) |
                             (uint32_t)__builtin_amdgcn_readlane(v_b0l, T);
        const uint64_t tp1 = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(v_b1h, T) << 32) |
                             (uint32_t)__builtin_amdgcn_readlane(v_b1l, T);
        const uint32_t tcm = (uint32_t)__builtin_amdgcn_readlane(v_cd, T) & 0x7Fu;
        const uint32_t tow = (uint32_t)__builtin_amdgcn_readlane(v_ow, T);
        const uint32_t meta = (uint32_t)(f0 + 63 - __clzll(Z | 1ull)) | (((uint32_t)we.depth + (uint32_t)T) << 16) |
                              (((uint32_t)we.turn ^ ((uint32_t)T & 1u)) << 24) | (tcm << 25);
        for (int jj = D + (int)lane; jj < nb; jj += 64) leaves[jj] = Leaf{tp0, tp1, meta, 0, tow, 0};
    }
    wave_mem_order();
    // ---- (3) the chain nodes' child slots and untried words; X0's
    if (act && seg != 0) {
        Fresh &P = fresh[parent - f0];
        P.ch[mi] = (uint16_t)(f0 + (int)lane);
        atomicAnd(&P.u, ~(1u << mi));
    }
    uint32_t slotbit = (act && seg == 0) ? 1u << mi : 0u;  // X0's draws are lanes 0 .. m0-1 (< 8)
    slotbit |= (uint32_t)dpp<0xB1>((int)slotbit);
    slotbit |= (uint32_t)dpp<0x4E>((int)slotbit);
    slotbit |= (uint32_t)dpp<0x141>((int)slotbit);
    const uint32_t ucl = uni(slotbit);
    const uint32_t sent =
        (uint32_t)__builtin_amdgcn_ds_permute((int)(((act && seg == 0) ? mi : 63u) << 2), (int)((uint32_t)f0 + lane));
    fs.x_ch = ((ucl >> (lane & 7u)) & 1u) ? sent : we.ch;
    fs.x_u = we.u & ~ucl;
    fs.x0_dirty = true;
    fs.planned = ZC_MERGED_BACKUP;
    fs.D = D;
    fs.Sm = Sm;
    fs.Z = Z;
    nnodes = f0 + D;
    wave_mem_order();
    {  // the flush's expansions and their depths: depth_sum = sum over draws of (we.depth + seg + 1)
        const uint32_t dep = act ? (uint32_t)we.depth + seg + 1u : 0u;
        int dsum = 0;
#pragma unroll
        for (int bit = 0; bit < 6; ++bit) dsum += __popcll(__ballot((dep >> bit) & 1u)) << bit;
        cn.add(cn.expansions, D);
        cn.add(cn.depth_sum, dsum);
    }
    stamp.mark(3);
}

// ------------------------------------------------------------------ the search kernel
constexpr int kSearchWaves = 4;  // games (waves) per workgroup
__host__ __device__ constexpr size_t c4_search_wave_lds(int bs) {
    return ((size_t)kLRingBytes + (sizeof(Leaf) + sizeof(Fresh) + sizeof(uint16_t) * kMaxDepth) * (size_t)bs +
            kPathSpill + 15) & ~(size_t)15;
}

// Per-wave LDS of the search: the MT ring, fresh nodes, pending leaves, their paths.
struct SearchLds {
    uint32_t *s_order;  // the workgroup's tables: order[128] u32 + sel[128][8]
    uint32_t *ring;
    Fresh *fresh;
    Leaf *leaves;
    uint16_t *paths;
};

__device__ __forceinline__ SearchLds search_lds(uint8_t *s_dyn, int bs) {
    const uint32_t wave = threadIdx.x >> 6;
    uint8_t *const s_wave = s_dyn + kTabBytes + (size_t)wave * c4_search_wave_lds(bs);
    SearchLds L;
    L.s_order = (uint32_t *)s_dyn;
    L.ring = (uint32_t *)s_wave;
    L.fresh = (Fresh *)(s_wave + kLRingBytes);
    L.leaves = (Leaf *)(s_wave + kLRingBytes + sizeof(Fresh) * (size_t)bs);
    L.paths = (uint16_t *)(s_wave + kLRingBytes + (sizeof(Fresh) + sizeof(Leaf)) * (size_t)bs);
    return L;
}

// One whole search (mcts.get_move, mcts.cpp:102-160) of game g from p.roots[gl] (re-read
// every flush rather than held in registers); the tree ends in t, the stream in rng.
// STAMP = diagnostic build: lane 0 adds s_memtime deltas per phase into p.a.phase[g][0..7] =
// {-, first walk of a flush, resumed walks, expansion + leaf bookkeeping, rollouts, backup,
//  publish, rollout sub-region}.
// WALK (diagnostic, zc_debug_c4_walk_async): 1 = record every leaf's rollout value and every
// flush's rollout words (p.walk_vals / p.walk_words); 2 = replay them instead of running the
// rollouts — the tree walk, expansion, backup and publish alone on the identical tree.
// done / nnodes: the simulations already run and the tree's nodes (0 / 1: a new search from
// the root; else a carried move resumes, its tree as the last flush published it).  stop
// (carry launches): the pooled ticket counter — once it reaches `budget` the search returns
// at the next flush boundary with done < p.sims (the move is suspended, not abandoned).
template <bool STAMP, bool PHILOX, int WALK = 0>
__device__ __forceinline__ void search_move(const SearchParams &p, const SearchLds &L, int gl, int g, const Tree &t,
                                            LRng &rng, uint32_t tag, Counters &cn, int &status, int &done_io,
                                            int &nnodes_io, const int32_t *stop = nullptr, int32_t budget = 0,
                                            int *lagp = nullptr, const int32_t *progress = nullptr, int mv = 0) {
    int lag = lagp ? *lagp : 0;
    const uint32_t lane = lane_id();
    const uint32_t *const s_order = L.s_order;
    Fresh *const fresh = L.fresh;
    Leaf *const leaves = L.leaves;
    // log(N) table read through the constant address space: uniform index -> scalar loads,
    // which do not sit in the vector-memory counter the walk waits on.
    ConstDouble *logtab = (ConstDouble *)p.a.logtab;
    if (done_io == 0) {
        const zc_c4_state root = p.roots[gl];
        node_init(t, 0, 0xFFFF, 0xFF, 0, uni(s_order[legal_mask(uni64(root.stones[0]) | uni64(root.stones[1]))]));
    }
    int nnodes = done_io == 0 ? 1 : nnodes_io;
    wave_mem_order();

    Stamp<STAMP> stamp;
    int done = done_io;
    while (done < p.sims) {
        const int nb = min(p.bs, p.sims - done);
        stamp.mark(0);

        // ---- selection + expansion of nb leaves (mcts.cpp:129-147) -------------------------
        FlushSel fs;
        {
            const zc_c4_state root = p.roots[gl];
#ifndef ZC_NO_PLAN
#define ZC_NO_PLAN 0
#endif
            // one lane per draw and lane 63 free as the permutes' discard slot (bs < 64); the chain
            // table lives in the leaf-path area, which this search does not use
#ifndef ZC_PLAN2
#define ZC_PLAN2 1  // 0: the chain's draws node by node (select_flush_plan), for A/B runs
#endif
            if (!ZC_NO_PLAN && ZC_PLAN2 && p.bs < 64)
                select_flush_plan2<STAMP>(t, fresh, leaves, s_order, logtab, rng, cn, stamp, nnodes, status,
                                          uni64(root.stones[0]), uni64(root.stones[1]), uni(root.turn), done, nb,
                                          p.c, fs);
            else if (!ZC_NO_PLAN && p.bs < 64)
                select_flush_plan<STAMP>(t, fresh, leaves, (ChainNode *)L.paths, s_order, logtab, rng, cn, stamp,
                                         nnodes, status, uni64(root.stones[0]), uni64(root.stones[1]),
                                         uni(root.turn), done, nb, p.c, fs);
            else
                select_flush<false, STAMP>(t, fresh, leaves, nullptr, s_order, logtab, rng, cn, stamp, nnodes,
                                           status, uni64(root.stones[0]), uni64(root.stones[1]), uni(root.turn),
                                           done, nb, p.c, fs);
        }
        const int f0 = fs.f0, d0 = fs.d0;

        // ---- value.batch: random rollouts in pending order (mcts.cpp:112-124) ---------------
        const size_t wlog = (size_t)g * p.sims + done;
        const size_t wfl = (size_t)g * ((p.sims + p.bs - 1) / p.bs) + done / p.bs;
        if (WALK == 2) {   // replay: the recorded values, the stream moved past the recorded words
            for (int jj = (int)lane; jj < nb; jj += kBlock) leaves[jj].val = p.walk_vals[wlog + jj];
            lrng_skip(rng, uni(p.walk_words[wfl]));
        } else if (PHILOX) {
            c4_rollouts_philox(leaves, nb, sel_table(s_order),
                               make_uint2((uint32_t)p.philox_seed, (uint32_t)(p.philox_seed >> 32)), (uint32_t)done,
                               tag, (uint32_t)g, cn);
        } else {
            const int32_t u0 = rng.use();
            // The rollouts issue at a raised wave priority: a CU's 16 games are each in the walk,
            // the rollouts or the backup, and the arbiter then serves the compute-bound rollout
            // chains (scalar-unit bound) first while the walk's and the backup's memory round
            // trips are in flight.  Priority 1, 2 or 3: 1.62 ms against 1.73 per 4096 x 800
            // lockstep search; the memory phases raised instead: 1.70 (profiles/r05_ab_c4_wave_priority.log).
#ifndef ZC_ROLLOUT_PRIO
#define ZC_ROLLOUT_PRIO 1  // A/B builds: the rollouts' wave priority
#endif
            // `lag` (free runs): how far this game is behind the launch's average pace; its
            // phases run that many levels up, so the arbiter evens the games' paces out
            set_prio(lag + ZC_ROLLOUT_PRIO);
            c4_rollouts(leaves, nb, rng, s_order, cn, STAMP ? &stamp.ph[7] : nullptr);
            set_prio(lag);
            if (WALK == 1) {
                wave_mem_order();
                for (int jj = (int)lane; jj < nb; jj += kBlock) p.walk_vals[wlog + jj] = (int8_t)leaves[jj].val;
                if (lane == 0) p.walk_words[wfl] = (uint32_t)(rng.use() - u0);
            }
        }
        wave_mem_order();
        stamp.mark(4);

        // ---- backprop of the whole flush (mcts.cpp:80-100, :124-125) ------------------------
        // Leaf j adds Na += 1 and Wa -= v_j * (-1)^(d_j - l) on the edge into level l of its
        // path, l = 1..d_j.  Integer adds commute, so the flush is applied as a sum:
        //   levels 1..d0 (root -> X0, on every path): Na += nb, Wa -= (-1)^l * S with
        //     S = sum_j v_j (-1)^d_j — one read-modify-write per level, all levels at once;
        //   levels > d0 (fresh nodes): LDS atomics into the fresh node's in-edge counters,
        //     written to HBM with the fresh records below.
        // Node::N is not stored: it equals Na of the in-edge (root: leaves flushed so far).
        // the prefix edges' counters are read first, so their HBM latency overlaps the LDS work
        const bool pre = lane >= 1 && lane <= (uint32_t)d0;
        const int par = __shfl((int)(fs.ppath & 0xFFFFu), (int)lane - 1);
        const int act = (int)(fs.ppath >> 16);
        int32_t na0 = 0, w0 = 0, spent_v = 0;
        // carry launches: the budget's state, read beside the prefix counters (one round trip);
        // free runs: the launch's finished moves (pace balancing)
        if (stop) spent_v = __hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (ZC_LAG_MODE >= 2 && progress)
            spent_v = __hip_atomic_load(progress, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (pre) {
            na0 = t.na(par)[act];
            w0 = t.w(par)[act];
        }
        const int32_t spent = stop || (ZC_LAG_MODE >= 2 && progress) ? uni(spent_v) : 0;
        if (fs.planned) {
            // The planned flush's fresh nodes are the draws 0..D-1 (leaf j <-> node f0 + j for
            // j < D; the leaves D..nb-1 sit on the terminal chain node).  A fresh node's subtree is
            // itself, plus — for a chain node (a Z draw) — every leaf from the next chain node's
            // first draw on (the chain runs to the flush's end), so every fresh in-edge's counters
            // come from one prefix sum over the leaves (lane = leaf) of sv_j = v_j (-1)^d_j:
            //   Na = 1 + #leaves from there,  Wa = -(-1)^l (sv_self + suffix sum from there)
            // (Wa -= v_j (-1)^(d_j - l) summed; integers, so in any order) — no atomics, no
            // walk up the parent links.  They are written straight into the records below.
            const int jj = (int)lane;
            int v = 0, dl = 0;
            if (jj < nb) {
                v = leaves[jj].val;
                dl = (int)((leaves[jj].meta >> 16) & 0xFFu);
            }
            const int sv = (dl & 1) ? -v : v;
            const int P = (int)scan_add32((uint32_t)sv);
            const int S = __builtin_amdgcn_readlane(P, 63);  // sum over every leaf (the prefix levels' S)
            const int suf = S - P + sv;                      // sum over the leaves jj..nb-1
            const uint64_t above = jj < 63 ? fs.Sm >> (jj + 1) : 0ull;
            const int nxt = above ? jj + 1 + __builtin_ctzll(above) : fs.D;  // next chain node's first draw
            const int sufn = __builtin_amdgcn_ds_bpermute(nxt << 2, suf);
            const bool isz = (fs.Z >> jj) & 1ull;
            const int na_e = 1 + (isz ? nb - nxt : 0);
            const int ss = sv + (isz ? sufn : 0);
            const int w_e = (dl & 1) ? ss : -ss;
            if (pre) {
                const int dw = (lane & 1u) ? S : -S;  // Wa -= (-1)^l * S
                t.na(par)[act] = na0 + nb;
                t.w(par)[act] = w0 + dw;
            }
            stamp.mark(5);
            // ---- publish: each fresh node's header and child slots (its Na / Wa slots only hold
            // data where a child exists: the walk reads them for those slots alone), the fresh
            // in-edges' counters into their fresh parents, and X0's changes
            if (jj < fs.D) {
                const Fresh &F = fresh[jj];
                const uint4 ch = *(const uint4 *)F.ch;
                const uint32_t link = F.link;
                uint8_t *R = t.rec(f0 + jj);
                *(uint4 *)R = make_uint4(0u, F.u, link, F.ow);
                *(uint4 *)(R + 16) = ch;
                const int pn = (int)(link & 0xFFFFu);
                if (pn >= f0) {
                    const int pa = (int)((link >> 16) & 0xFFu);
                    t.na(pn)[pa] = na_e;
                    t.w(pn)[pa] = w_e;
                }
            }
            if (fs.x0_dirty) {
                const int x0node = fs.x0node;
                const uint32_t x_ch = fs.x_ch;
                const bool xf = x_ch != 0xFFFF && (int)x_ch >= f0;
                const int src = (xf ? (int)x_ch - f0 : 0) << 2;
                const int xna = __builtin_amdgcn_ds_bpermute(src, na_e);
                const int xw = __builtin_amdgcn_ds_bpermute(src, w_e);
                if (lane == 0) t.hdr(x0node)[1] = fs.x_u;
                if (lane < kSlots) {
                    t.child(x0node)[lane] = (uint16_t)x_ch;
                    if (xf) {  // edge into a fresh child
                        t.na(x0node)[lane] = xna;
                        t.w(x0node)[lane] = xw;
                    }
                }
            }
        } else {
            int S = 0;
            for (int base = 0; base < nb; base += 64) {
                // lane = leaf: S, and the fresh edges (levels d0+1..d of the leaf's path), one level
                // per step for all leaves at once
                const int jj = base + (int)lane;
                int v = 0, d = -1, sv = 0;
                if (jj < nb) {
                    const uint32_t meta = leaves[jj].meta;
                    v = leaves[jj].val;
                    d = (int)((meta >> 16) & 0xFFu);
                    sv = (d & 1) ? -v : v;
                }
                S += __popcll(__ballot(sv > 0)) - __popcll(__ballot(sv < 0));
                // the fresh edges: from the leaf up to X0's child along the fresh nodes' parent
                // links (every node below X0 is fresh, X0 and above are not)
                int nd = jj < nb ? (int)(leaves[jj].meta & 0xFFFFu) : -1, l = d;
                while (__ballot(nd >= f0)) {
                    if (nd >= f0) {
                        const int fi = nd - f0;
                        const int vl = ((d - l) & 1) ? -v : v;
                        atomicAdd(&fresh[fi].na, 1);
                        atomicAdd(&fresh[fi].w, -vl);
                        nd = (int)(fresh[fi].link & 0xFFFFu);
                        --l;
                    }
                }
            }
            if (pre) {
                const int dw = (lane & 1u) ? S : -S;  // Wa -= (-1)^l * S
                t.na(par)[act] = na0 + nb;
                t.w(par)[act] = w0 + dw;
            }
            wave_mem_order();
            stamp.mark(5);

            // ---- publish: X0's changes and every fresh node, in coalesced stores ------------------
            if (fs.x0_dirty) {
                const int x0node = fs.x0node;
                const uint32_t x_ch = fs.x_ch;
                if (lane == 0) t.hdr(x0node)[1] = fs.x_u;
                if (lane < kSlots) {
                    t.child(x0node)[lane] = (uint16_t)x_ch;
                    if (x_ch != 0xFFFF && (int)x_ch >= f0) {  // edge into a fresh child
                        t.na(x0node)[lane] = fresh[x_ch - f0].na;
                        t.w(x0node)[lane] = fresh[x_ch - f0].w;
                    }
                }
            }
            {
                const int nf = nnodes - f0;
                for (int base = 0; base < nf * 8; base += 64) {
                    const int idx = base + (int)lane;
                    if (idx < nf * 8) {
                        const int r = idx >> 3, slot = idx & 7;
                        const Fresh &F = fresh[r];
                        const uint16_t c = F.ch[slot];
                        int32_t na = 0, w = 0;
                        if (c != 0xFFFF) {
                            na = fresh[c - f0].na;
                            w = fresh[c - f0].w;
                        }
                        uint8_t *R = t.rec(f0 + r);
                        if (slot == 0) *(uint4 *)R = make_uint4(0u, F.u, F.link, F.ow);
                        ((uint16_t *)(R + 16))[slot] = c;
                        ((int32_t *)(R + 32))[slot] = na;
                        ((int32_t *)(R + 64))[slot] = w;
                    }
                }
            }
        }
        wave_mem_order();
        stamp.mark(6);
        done += nb;
        if (stop && done < p.sims && status == 0 && uni(spent) >= budget) break;  // suspend
        if (ZC_LAG_MODE >= 2 && progress) {  // behind the average (in simulations): 1; by a move or more: 2
            const int64_t own = ((int64_t)mv * p.sims + done) * p.n_games, avg = (int64_t)spent * p.sims;
            const int64_t mvn = (int64_t)p.sims * p.n_games;  // one move behind
            if (ZC_LAG_MODE == 4)  // behind by < 1/2 move: 1, < 1 move: 2, more: 3
                lag = own >= avg ? 0 : own + mvn / 2 > avg ? 1 : own + mvn > avg ? 2 : 3;
            else
                lag = own < avg ? (ZC_LAG_MODE == 3 && own + mvn <= avg ? 2 : ZC_LAG_MODE == 3 ? 1 : 2) : 0;
            set_prio(lag);
        }
    }
    done_io = done;
    nnodes_io = nnodes;
    if (lagp) *lagp = lag;
    if (STAMP && lane == 0)
        for (int k_ = 0; k_ < kPhases; ++k_) p.a.phase[kPhases * (size_t)g + k_] += (int64_t)stamp.ph[k_];
}

// The move (mcts.cpp:150-157): first max of child N over the root's move list -> its column;
// lanes 0..6 also get the visits of the child in their column (0 if illegal) in `na_col`.
__device__ __forceinline__ int best_column(const Tree &t, int &na_col) {
    const uint32_t lane = lane_id();
    const uint32_t k = lane & 7u;
    const uint32_t u = uni(t.hdr(0)[1]);
    const uint32_t ow = uni(t.hdr(0)[3]);
    const uint32_t nm = u >> 28;
    int bv = (k < nm) ? t.na(0)[k] : -1;
    int bi = (int)k;
    argmax8(bv, bi);
    const int best = uni(bi);
    int pos = -1;
    for (uint32_t s = 0; s < nm; ++s)
        if (((ow >> (3 * s)) & 7u) == lane) pos = (int)s;
    na_col = pos >= 0 ? t.na(0)[pos] : 0;
    return (int)((ow >> (3 * best)) & 7u);
}

template <bool STAMP, bool PHILOX, int WALK>
__device__ __forceinline__ void search_games(const SearchParams &p, uint8_t *s_dyn) {
    const SearchLds L = search_lds(s_dyn, p.bs);
    load_tables(L.s_order);
    __syncthreads();

    const uint32_t lane = lane_id();
    const int gl = (int)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));  // one wave per game
    if (gl >= p.n_games) return;
    const int g = p.game_ids ? uni(p.game_ids[gl]) : p.first_game + gl;
    {
        const zc_c4_state root = p.roots[gl];
        const uint64_t rp0 = uni64(root.stones[0]), rp1 = uni64(root.stones[1]);
        const int rturn = uni(root.turn);
        if (!valid_state(rp0, rp1, rturn) || legal_mask(rp0 | rp1) == 0) {
            if (lane == 0) {
                zc_game_stats st{};
                st.status = valid_state(rp0, rp1, rturn) ? ZC_STATUS_NO_MOVES : ZC_STATUS_BAD_STATE;
                p.out_stats[gl] = st;
                p.out_move[gl] = -1;
            }
            if (lane < 7) p.out_na[(size_t)gl * 7 + lane] = 0;
            return;
        }
    }
    const Arena &a = p.a;
    const Tree t{a.nodes + (size_t)g * p.M * kRecBytes};
    LRng rng;
    const uint64_t use0 = uni64(a.rngpos[2 * (size_t)g]);
    lrng_open(rng, L.ring, a.ring + (size_t)g * kRingWords, use0, uni64(a.rngpos[2 * (size_t)g + 1]));
    Counters cn;
    int status = 0, done = 0, nnodes = 1;
    search_move<STAMP, PHILOX, WALK>(p, L, gl, g, t, rng, uni((uint32_t)use0), cn, status, done, nnodes);
    int na_col;
    const int col = best_column(t, na_col);
    if (lane < 7) p.out_na[(size_t)gl * 7 + lane] = na_col;
    if (lane == 0) {
        p.out_move[gl] = col;
        zc_game_stats st{};
        st.status = status;
        st.expansions = cn.expansions;
        st.depth_sum = cn.depth_sum;
        st.leaves = p.sims;
        st.rollout_plies = cn.plies;
        st.rollout_blocks = cn.blocks;
        st.rng_words = rng.use();
        p.out_stats[gl] = st;
    }
    lrng_close(rng, a.ring + (size_t)g * kRingWords, use0, a.rngpos + 2 * (size_t)g);
}

template <bool STAMP, bool PHILOX>
__global__ __launch_bounds__(kSearchWaves * kBlock, 4) void c4_search_kernel(SearchParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t s_dyn[];
    search_games<STAMP, PHILOX, 0>(p, s_dyn);
}

// Diagnostic: the lockstep search with its rollouts recorded (WALK 1) or replayed (WALK 2):
// the tree-walk-only kernel whose time and HBM traffic measure the walk (tools/prof_walk.py).
template <int WALK>
__global__ __launch_bounds__(kSearchWaves * kBlock, 4) void c4_walk_kernel(SearchParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t s_dyn[];
    search_games<false, false, WALK>(p, s_dyn);
}

// Self-play without a global step: each wave plays `p.moves` consecutive moves of its game —
// search, Engine.play_move + _evaluate (engine.py:98-108, 148-153), and the refill of a
// finished game from the opening (train.py:151-170 with no game quota) — keeping its tree
// arena, its MT stream (in LDS) and its pace.  Games of different ages take different times
// per move (young games have the long rollouts); synchronising all games every move makes
// each launch wait for the slowest game, here the waves only meet at the end of the run.
// Step k's post-move position / move / result go to out_states[k*n + gl], out_moves[...],
// out_results[...] (the inputs of zc_traj_record_async for step k, replayed in step order
// after the launch); out_stats[gl] accumulates over the moves.
// Carried moves (zc_c4_selfplay_carry_async): a carry launch suspends each in-flight move at
// its next flush boundary once the pooled budget is spent, saving {simulations done, tree
// nodes, Philox tag} in a.carry[g] (the tree, the MT stream and the root stay in HBM).  EVERY
// self-play launch first resumes a carried move, without a ticket, so the game's moves are
// the moves an uninterrupted run plays; only carry launches suspend.
template <bool PHILOX>
__global__ __launch_bounds__(kSearchWaves * kBlock, 4) void c4_selfplay_kernel(SearchParams p) {
    extern __shared__ __attribute__((aligned(16))) uint8_t s_dyn[];
    const SearchLds L = search_lds(s_dyn, p.bs);
    load_tables(L.s_order);
    __syncthreads();

    const uint32_t lane = lane_id();
    const int gl = (int)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
    if (gl >= p.n_games) return;
    const int g = p.first_game + gl;
    const Arena &a = p.a;
    const Tree t{a.nodes + (size_t)g * p.M * kRecBytes};
    LRng rng;
    const uint64_t use0 = uni64(a.rngpos[2 * (size_t)g]);
    lrng_open(rng, L.ring, a.ring + (size_t)g * kRingWords, use0, uni64(a.rngpos[2 * (size_t)g + 1]));
    Counters cn;
    int status = 0;
    int finished = 0;
    int mv = 0;
    int64_t leaves = 0;
    uint64_t t_start = 0, t_last = 0;
    if (p.tstamps) t_start = t_last = __builtin_amdgcn_s_memrealtime();
    int lag = 0;             // pace level of free runs (search_move)
    uint4 cy = a.carry[g];   // a carried move: {done, nodes, tag, -} (done 0: none)
    cy = make_uint4(uni(cy.x), uni(cy.y), uni(cy.z), 0u);
    bool resume = cy.x != 0;
    for (; mv < p.moves; ++mv) {
        if (p.ticket && !resume) {  // pooled run: the next move only while the shared budget lasts
            int tk = 0;
            if (lane == 0) tk = atomicAdd(p.ticket, 1);
            if (uni(tk) >= p.budget) break;
        }
        if (p.tstamps) t_last = __builtin_amdgcn_s_memrealtime();
        zc_c4_state root = p.roots[gl];
        uint64_t s0 = uni64(root.stones[0]), s1 = uni64(root.stones[1]);
        int turn = uni(root.turn);
        if (!valid_state(s0, s1, turn) || legal_mask(s0 | s1) == 0) {  // never from play: flagged
            status = ZC_STATUS_BAD_STATE;
            break;
        }
        int done = resume ? (int)cy.x : 0, nnodes = resume ? (int)cy.y : 1;
        const uint32_t tag = resume ? cy.z : uni((uint32_t)(use0 + (uint64_t)(int64_t)rng.use()));
        const int done0 = done;
        // free runs (every game exactly p.moves moves, the launch waits for the slowest): a game
        // whose moves so far are below the launch's average raises its priority for this move
        if (ZC_LAG_MODE == 1 && p.progress) {
            const int32_t tot = __hip_atomic_load(p.progress, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            lag = (int64_t)mv * p.n_games < (int64_t)uni(tot) ? 2 : 0;
            set_prio(lag);
        }
        search_move<false, PHILOX>(p, L, gl, g, t, rng, tag, cn, status, done, nnodes, p.carry ? p.ticket : nullptr,
                                   p.budget, &lag, ZC_LAG_MODE ? p.progress : nullptr, mv);
        if (ZC_LAG_MODE && p.progress && lane == 0) atomicAdd(p.progress, 1);
        leaves += done - done0;
        if (done < p.sims) {  // suspended (carry launch, budget spent): the next launch resumes it
            if (lane == 0) a.carry[g] = make_uint4((uint32_t)done, (uint32_t)nnodes, tag, 0u);
            break;
        }
        if (resume && lane == 0) a.carry[g] = make_uint4(0u, 0u, 0u, 0u);
        resume = false;
        int na_col;
        const int col = best_column(t, na_col);
        // play_move + _evaluate (c4_play_kernel): check_win -> turn*2-1 with the new turn
        const uint64_t bit = drop_bit(s0 | s1, col);
        if (turn) s1 |= bit; else s0 |= bit;
        const bool won = has_four(turn ? s1 : s0);
        turn ^= 1;
        const int r = won ? turn * 2 - 1 : ((s0 | s1) == kFull ? 0 : ZC_C4_ONGOING);
        const size_t o = (size_t)mv * p.n_games + gl;
        if (lane == 0) {
            zc_c4_state post;
            post.stones[0] = s0;
            post.stones[1] = s1;
            post.turn = turn;
            post.reserved = 0;
            p.out_states[o] = post;
            p.out_moves16[o] = (int16_t)col;
            p.out_results[o] = r;
            p.io_roots[gl] = r == ZC_C4_ONGOING ? post : zc_c4_state{{0, 0}, 0, 0};
        }
        finished += r != ZC_C4_ONGOING;
        wave_mem_order();
    }
    if (p.ticket && lane == 0) atomicMax(p.ticket + 1, mv);
    if (p.tstamps && lane == 0) {
        uint64_t *ts = p.tstamps + 4 * (size_t)g;
        ts[0] = t_start;
        ts[1] = t_last;
        ts[2] = __builtin_amdgcn_s_memrealtime();
        // moves played | where the wave ran << 32: HW_ID bits 15:0 (wave slot, SIMD, CU, SH,
        // SE) and the XCC below them << 16
        const uint32_t hw = (uint32_t)__builtin_amdgcn_s_getreg(4 | (15 << 11)) |
                            ((uint32_t)__builtin_amdgcn_s_getreg(20 | (3 << 11)) << 16);
        ts[3] = (uint64_t)mv | ((uint64_t)hw << 32);
    }
    // steps this game did not reach (budget spent, or a bad root): skipped by the recording
    for (int k = mv + (int)lane; k < p.moves; k += kBlock) {
        const size_t o = (size_t)k * p.n_games + gl;
        p.out_moves16[o] = -1;
        p.out_results[o] = ZC_SLOT_SKIP;
    }
    if (lane == 0) {
        zc_game_stats st{};
        st.status = status;
        st.expansions = cn.expansions;
        st.depth_sum = cn.depth_sum;
        st.leaves = leaves;
        st.rollout_plies = cn.plies;
        st.rollout_blocks = cn.blocks;
        st.rng_words = rng.use();
        st.reserved = finished;
        p.out_stats[gl] = st;
    }
    lrng_close(rng, a.ring + (size_t)g * kRingWords, use0, a.rngpos + 2 * (size_t)g);
}

// ------------------------------------------------------------------ small kernels
__global__ __launch_bounds__(kBlock) void c4_rollout_debug_kernel(Arena a, int first_game, int n,
                                                                  const zc_c4_state *states, int32_t *out_value,
                                                                  int64_t *out_words) {
    __shared__ Leaf s_leaf[1];
    __shared__ uint32_t s_order[kTabBytes / 4];  // order + select tables
    load_tables(s_order);
    __syncthreads();
    const uint32_t lane = lane_id();
    const int gl = blockIdx.x;
    if (gl >= n) return;
    const int g = first_game + gl;
    Rng rng;
    const uint64_t use0 = uni64(a.rngpos[2 * (size_t)g]);
    rng_open(rng, a.ring + (size_t)g * kRingWords, use0, uni64(a.rngpos[2 * (size_t)g + 1]));
    const zc_c4_state s = states[gl];
    if (lane == 0) {
        s_leaf[0].p0 = s.stones[0];
        s_leaf[0].p1 = s.stones[1];
        s_leaf[0].meta = ((uint32_t)s.turn << 24) | ((uint32_t)legal_mask(s.stones[0] | s.stones[1]) << 25);
        s_leaf[0].ow = s_order[legal_mask(s.stones[0] | s.stones[1])];
    }
    wave_mem_order();
    Counters cn;
    c4_rollouts(s_leaf, 1, rng, s_order, cn);
    wave_mem_order();
    if (lane == 0) {
        out_value[gl] = s_leaf[0].val;
        out_words[gl] = rng.use();
        rng_close(rng, use0, a.rngpos + 2 * (size_t)g);
    }
}

// Value('random_rollout').batch: n states rolled out IN ORDER on one game's stream.
__global__ __launch_bounds__(kBlock) void c4_rollout_seq_kernel(Arena a, int g, int n, const zc_c4_state *states,
                                                                int32_t *out_value, int64_t *out_words) {
    __shared__ Leaf s_leaf[kBlock];
    __shared__ uint32_t s_order[kTabBytes / 4];  // order + select tables
    load_tables(s_order);
    __syncthreads();
    const uint32_t lane = lane_id();
    Rng rng;
    const uint64_t use0 = uni64(a.rngpos[2 * (size_t)g]);
    rng_open(rng, a.ring + (size_t)g * kRingWords, use0, uni64(a.rngpos[2 * (size_t)g + 1]));
    Counters cn;
    for (int base = 0; base < n; base += kBlock) {
        const int cnt = min(kBlock, n - base);
        if ((int)lane < cnt) {
            const zc_c4_state s = states[base + lane];
            s_leaf[lane].p0 = s.stones[0];
            s_leaf[lane].p1 = s.stones[1];
            s_leaf[lane].meta = ((uint32_t)s.turn << 24) | ((uint32_t)legal_mask(s.stones[0] | s.stones[1]) << 25);
            s_leaf[lane].ow = s_order[legal_mask(s.stones[0] | s.stones[1])];
        }
        wave_mem_order();
        rng_fill(rng, rng.use() + kLookahead);
        c4_rollouts(s_leaf, cnt, rng, s_order, cn);
        wave_mem_order();
        if ((int)lane < cnt) out_value[base + lane] = s_leaf[lane].val;
        wave_mem_order();
    }
    if (lane == 0) {
        out_words[0] = rng.use();
        rng_close(rng, use0, a.rngpos + 2 * (size_t)g);
    }
}

__global__ void c4_play_kernel(int n, zc_c4_state *states, const int32_t *moves, int32_t *results, int reset) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int col = moves[i];
    if (col < 0 || col > 6) {
        results[i] = ZC_C4_ONGOING;
        return;
    }
    zc_c4_state s = states[i];
    const int turn = s.turn & 1;
    s.stones[turn] |= drop_bit(s.stones[0] | s.stones[1], col);
    s.turn = turn ^ 1;
    int r = ZC_C4_ONGOING;
    if (has_four(s.stones[turn])) r = s.turn * 2 - 1;  // Engine._evaluate: check_win -> turn*2-1
    else if ((s.stones[0] | s.stones[1]) == kFull) r = 0;
    if (reset && r != ZC_C4_ONGOING) s = zc_c4_state{{0, 0}, 0, 0};
    states[i] = s;
    results[i] = r;
}

__global__ void uct_debug_kernel(int n, const double *logn, const int32_t *na, const double *q, double c,
                                 double *out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = na[i] == 0 ? INFINITY : fma(c, sqrt(logn[i] / (double)na[i]), q[i]);
}

}  // namespace

// Games per workgroup: up to kSearchWaves share the tables (4 x ~9.3 KB + 1.5 KB at bs 32, so
// four workgroups = 16 waves per CU fit the CU's 160 KB of LDS); fewer when a large batch
// would not fit one workgroup (sharing only lowers the LDS per game).
static int c4_search_wpg(int bs) {
    int w = kSearchWaves;
    while (w > 1 && kTabBytes + (size_t)w * c4_search_wave_lds(bs) > (size_t)(160 * 1024)) w >>= 1;
    return w;
}

size_t c4_search_lds_bytes(int bs) { return kTabBytes + (size_t)c4_search_wpg(bs) * c4_search_wave_lds(bs); }

void launch_c4_search(const SearchParams &p, hipStream_t s) {
    const int wpg = c4_search_wpg(p.bs);
    const size_t lds = c4_search_lds_bytes(p.bs);
    const dim3 grid((p.n_games + wpg - 1) / wpg), block(wpg * kBlock);
    if (p.philox) {
        if (p.stamp)
            hipLaunchKernelGGL((c4_search_kernel<true, true>), grid, block, lds, s, p);
        else
            hipLaunchKernelGGL((c4_search_kernel<false, true>), grid, block, lds, s, p);
    } else {
        if (p.stamp)
            hipLaunchKernelGGL((c4_search_kernel<true, false>), grid, block, lds, s, p);
        else
            hipLaunchKernelGGL((c4_search_kernel<false, false>), grid, block, lds, s, p);
    }
}

void launch_c4_walk(const SearchParams &p, int mode, hipStream_t s) {
    const int wpg = c4_search_wpg(p.bs);
    const size_t lds = c4_search_lds_bytes(p.bs);
    const dim3 grid((p.n_games + wpg - 1) / wpg), block(wpg * kBlock);
    if (mode == 1)
        hipLaunchKernelGGL((c4_walk_kernel<1>), grid, block, lds, s, p);
    else
        hipLaunchKernelGGL((c4_walk_kernel<2>), grid, block, lds, s, p);
}

void launch_c4_selfplay(const SearchParams &p, hipStream_t s) {
    const int wpg = c4_search_wpg(p.bs);
    const size_t lds = c4_search_lds_bytes(p.bs);
    const dim3 grid((p.n_games + wpg - 1) / wpg), block(wpg * kBlock);
    if (p.philox)
        hipLaunchKernelGGL((c4_selfplay_kernel<true>), grid, block, lds, s, p);
    else
        hipLaunchKernelGGL((c4_selfplay_kernel<false>), grid, block, lds, s, p);
}

int c4_selfplay_resident_games(int bs, int philox, int *out) {
    const int wpg = c4_search_wpg(bs);
    int blocks = 0, dev = 0, cus = 0;
    const void *fn = philox ? (const void *)c4_selfplay_kernel<true> : (const void *)c4_selfplay_kernel<false>;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, fn, wpg * kBlock, c4_search_lds_bytes(bs)) != hipSuccess)
        return -1;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return -1;
    *out = blocks * cus * wpg;
    return 0;
}

void launch_c4_rollout_debug(const Arena &a, int M, int first_game, int n, const zc_c4_state *states,
                             int32_t *out_value, int64_t *out_words, hipStream_t s) {
    (void)M;
    hipLaunchKernelGGL(c4_rollout_debug_kernel, dim3(n), dim3(kBlock), 0, s, a, first_game, n, states, out_value,
                       out_words);
}

void launch_c4_rollout_seq(const Arena &a, int game, int n, const zc_c4_state *states, int32_t *out_value,
                           int64_t *out_words, hipStream_t s) {
    hipLaunchKernelGGL(c4_rollout_seq_kernel, dim3(1), dim3(kBlock), 0, s, a, game, n, states, out_value, out_words);
}

void launch_c4_play(int n, zc_c4_state *states, const int32_t *moves, int32_t *results, int reset, hipStream_t s) {
    hipLaunchKernelGGL(c4_play_kernel, dim3((n + 255) / 256), dim3(256), 0, s, n, states, moves, results, reset);
}

void launch_uct_debug(int n, const double *logn, const int32_t *na, const double *q, double c, double *out,
                      hipStream_t s) {
    hipLaunchKernelGGL(uct_debug_kernel, dim3((n + 255) / 256), dim3(256), 0, s, n, logn, na, q, c, out);
}

}  // namespace zc
