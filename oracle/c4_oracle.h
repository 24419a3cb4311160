/* oracle/c4_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's Connect4 UCT search, used as the parity checker by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  The product
 * (zeroclone_amd/, libzeroclone_amd.so) never includes, links or calls this.
 *
 * Pinned against tests/golden/ JSON fixtures, which were produced by the reference itself
 * (tests/golden/gen_golden.py drives the unmodified engine/mcts C++ core + Python
 * backend/value/policy).
 */
#ifndef ZC_C4_ORACLE_H
#define ZC_C4_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* CPython 3.10 `random.Random` MT19937 state (Modules/_randommodule.c). */
typedef struct {
    uint32_t mt[624];
    int index;
    uint64_t drawn;   /* words consumed since seeding (oracle bookkeeping) */
} zco_mt;

void     zco_mt_seed(zco_mt *r, uint64_t seed);          /* random.seed(int >= 0)          */
uint32_t zco_mt_u32(zco_mt *r);                          /* getrandbits(32)                */
uint32_t zco_randbelow(zco_mt *r, uint32_t n);           /* Random._randbelow_with_getrandbits */

/* CPython set iteration order of {(i,0) for legal i}: out[0..n) = columns; returns n. */
int  zco_set_order(int mask, int *out);

/* Board: 42 chars row-major, row 0 = top, 'X' (turn 0), 'O' (turn 1), '.' empty. */
int  zco_check_win(const char *board, int turn);          /* c4_backend.py:25-44 */
int  zco_check_draw(const char *board);                   /* c4_backend.py:46-47 */
/* Value('random_rollout') from the side to move at `board` (value_functions.py:35-45). */
int  zco_rollout(const char *board, int turn, zco_mt *r);

/* One get_move call (mcts.cpp:102-160) with policy=random, value=random_rollout.
 * root_na[k] = visits of the k-th root move (root move list in set order), order[k] = its
 * column; returns the chosen column, or -1 (sims < 1 / no legal move).  *n_moves receives
 * the root's move count. */
int  zco_get_move(const char *board, int turn, zco_mt *r, int sims, double c, int bs,
                  int *root_na, int *order, int *n_moves);

/* The same search with Value.batch supplied by the caller: at every flush (mcts.cpp:112-127)
 * vfn(ctx, n, boards n*42 chars, turns, out_values) evaluates the n pending leaves in
 * pending order (value_functions.py:16-32).  Policy stays random.choice on r. */
typedef void (*zco_value_fn)(void *ctx, int n, const char *boards, const int *turns, double *out);
int  zco_get_move_valued(const char *board, int turn, zco_mt *r, int sims, double c, int bs,
                         int *root_na, int *order, int *n_moves, zco_value_fn vfn, void *ctx);

/* Convenience for the CPU baseline: n games, game g seeded with seeds[g], spread over
 * n_threads pthreads.  Boards are n*42 chars.  Returns 0. */
int  zco_get_move_batch(int n, const char *boards, const int *turns, const uint64_t *seeds,
                        int sims, double c, int bs, int n_threads,
                        int *out_move, int *out_root_na /* n*7 */, uint64_t *out_consumed);

/* Steady-state self-play (bench.py's CPU baseline on a burned-in pool's snapshot): game g
 * from boards[g] / turns[g] and MT state mts[g] (advanced in place) plays `moves` moves —
 * get_move, play, _evaluate, the refill of a finished game with the empty board — on
 * n_threads pthreads; out_expansions[g] = the nodes its searches created.  Returns 0. */
int  zco_selfplay_batch(int n, const char *boards, const int *turns, zco_mt *mts, int moves, int sims, double c,
                        int bs, int n_threads, uint64_t *out_expansions);

#ifdef __cplusplus
}
#endif
#endif
