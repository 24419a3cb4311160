/* chess_oracle.h — TEST INFRASTRUCTURE ONLY: C restatement of the reference chess rules
 * (engine/games/chess/src/chess_backend.cpp) for the parity tests.  See chess_oracle.c. */
#ifndef ZC_CHESS_ORACLE_H
#define ZC_CHESS_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZCC_MAX_MOVES 256
#define ZCC_HIST 512

typedef struct {
    uint8_t fr, fc, tr, tc;  /* (from_row, from_col, to_row, to_col); row 0 = rank 8 */
    double value;            /* capture value (Move's double)                        */
} zcc_move;

typedef struct {
    uint8_t board[64];  /* ' ' empty, "PNBRQK" white, "pnbrqk" black; index 0 = a8 */
    uint8_t turn;       /* 0 white to move                                           */
    uint8_t fifty;      /* fifty_move_rule_counter (uint8)                          */
    uint8_t castle;     /* bit 0 w_ck, 1 w_cq, 2 b_ck, 3 b_cq                        */
    uint8_t overflow;   /* history longer than ZCC_HIST was truncated                */
    int nhw, nhb;       /* history lengths (most recent move first)                  */
    zcc_move hw[ZCC_HIST], hb[ZCC_HIST];
} zcc_state;

/* The position without history (what a search tree node holds). */
typedef struct {
    uint8_t board[64];
    uint8_t turn, fifty, castle, pad;
} zcc_light;

void     zcc_init(zcc_state *s);                                       /* create_init_state */
int      zcc_from_fen(const char *fen, zcc_state *s);                  /* state_from_fen    */
int      zcc_legal_moves(const zcc_state *s, zcc_move *out);           /* get_legal_moves   */
void     zcc_play(const zcc_state *s, const zcc_move *m, zcc_state *o); /* play_move (o may be s) */
int      zcc_check_win(const zcc_state *s);
int      zcc_check_draw(const zcc_state *s);
int      zcc_repeated_prefix(const zcc_move *L, int n);               /* has_repeated_prefix(L,2,3) */
void     zcc_state_to_tensor(const zcc_state *s, float *out);          /* [17][8][8]        */
uint64_t zcc_perft(const zcc_state *s, int depth);

/* Value('crude_chess_score') (value_functions.py:48-55). */
double   zcc_crude_score(const zcc_light *l);
/* mcts.get_move (mcts.cpp:102-160) for chess: policy 0 = Policy('random'), 1 =
 * Policy('immediate_value', policy_freedom=freedom); vfn NULL = crude_chess_score, else
 * vfn(ctx, n, leaves, out) is Value.batch over the flush's pending leaves.  r is a
 * zco_mt* (c4_oracle.h).  Writes the root's moves and visits; returns the index of the
 * chosen root move (-1 if none). */
typedef void (*zcc_value_fn)(void *ctx, int n, const zcc_light *leaves, double *out);
int      zcc_get_move(const zcc_light *root, void *r, int sims, double c, int bs, int policy, double freedom,
                      zcc_value_fn vfn, void *ctx, int *root_na, zcc_move *root_moves, int *n_root);
/* crude-score self-play of n games from roots on their streams (bench.py's CPU baseline) */
int      zcc_selfplay_batch(int n, const zcc_light *roots, void *mts, int moves, int sims, double c, int bs, int policy,
                            double freedom, int n_threads, uint64_t *out_expansions);

/* Value('random_rollout') (value_functions.py:35-45) on the chess rules, stream r (zco_mt*):
 * -1 / +1 / 0 for the start's side to move, 2 if a history outgrew ZCC_HIST; *plies played. */
int      zcc_rollout(const zcc_state *s, void *r, int *plies);

#ifdef __cplusplus
}
#endif
#endif
