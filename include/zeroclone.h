/* zeroclone.h — C-ABI of libzeroclone_amd.so, the MI355X-native batched-MCTS engine.
 *
 * Drop-in boundary for the reference's search core.  The reference binds ONE function,
 *     mcts.get_move(state, value, policy, backend, simulations=1000, c=1.4, batch_size=32)
 *     (engine/mcts/src/bindings_mcts.cpp:9-11, implemented at engine/mcts/src/mcts.cpp:102-160)
 * and calls it once per game per move from Python threads (engine/engine.py:119-138).  Here
 * one call searches MANY games at once on the GPU; the Python layer in zeroclone_amd/
 * keeps the reference's get_move / Engine API on top of these entry points.
 *
 * Conventions: plain C types only; every function returns 0 (ZC_OK) or a negative
 * ZC_E* code and records a message retrievable with zc_last_error() (thread-local).
 * An engine is bound to one HIP device; calls on one engine are serialised internally.
 */
#ifndef ZEROCLONE_H
#define ZEROCLONE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZC_OK 0
#define ZC_EINVAL -1     /* bad argument (reference: ValueError / UB)               */
#define ZC_EHIP -2       /* HIP runtime error                                       */
#define ZC_ENOMEM -3     /* device allocation failed                                */
#define ZC_ECAPACITY -4  /* request exceeds the engine's configured capacity        */
#define ZC_EDEVICE -5    /* a kernel reported an internal error (status word)       */

/* Connect4 position.  Bit (7*col + r) of stones[p] is set when the cell in column `col`,
 * r-th row counted from the BOTTOM (r = 0..5), holds player p's token ('X' = player 0,
 * 'O' = player 1).  Bit 7*col+6 is a sentinel and must be 0.  In the reference's
 * c4_backend.State (engine/games/connect4/c4_backend.py:4-12) board[row][col] has row 0 at
 * the TOP, i.e. r = 5 - row.  `turn` is the side to move (State.turn). */
typedef struct zc_c4_state {
    uint64_t stones[2];
    int32_t turn;
    int32_t reserved;
} zc_c4_state;

/* Per-game counters of one search (all int64 so a device array of them is plain data). */
typedef struct zc_game_stats {
    int64_t expansions;      /* nodes created (= simulations that expanded)              */
    int64_t depth_sum;       /* sum over expansions of the new node's depth d (root = 0) */
    int64_t leaves;          /* leaves evaluated (= simulations)                          */
    int64_t rollout_plies;   /* plies played inside random rollouts                      */
    int64_t rng_words;       /* MT19937 words consumed                                   */
    int64_t status;          /* 0 = ok; nonzero = internal error code                    */
    int64_t rollout_blocks;  /* lane-parallel ply blocks the rollouts took                */
    int64_t reserved;
} zc_game_stats;

typedef struct zc_engine_config {
    int32_t device;          /* HIP device ordinal                                        */
    int32_t max_games;       /* games resident on this engine                             */
    int32_t max_sims;        /* simulations per move (tree capacity = max_sims + 1 nodes) */
    int32_t max_batch;       /* leaf batch size (reference batch_size)                    */
} zc_engine_config;

typedef struct zc_engine zc_engine;

const char *zc_version(void);
const char *zc_last_error(void);
int zc_device_count(int32_t *count);

/* An engine: its games' arena in ONE device allocation, a HIP stream and a pinned staging block
 * for the synchronous calls.  Streams and pinned blocks are taken from / returned to per-process
 * pools (creating a HIP stream costs milliseconds), so they outlive a destroyed engine until the
 * process exits.  Every game starts as random.seed(game index). */
int zc_engine_create(const zc_engine_config *cfg, zc_engine **out);
int zc_engine_destroy(zc_engine *eng);
/* Device bytes held by the engine. */
int zc_engine_footprint(const zc_engine *eng, int64_t *bytes);

/* ---- per-game random streams: CPython 3.10 `random.Random` (MT19937) -----------------
 * The reference draws every random number from Python's global `random` module
 * (engine/policy_functions.py:12, engine/value_functions.py:40).  Each engine game owns one
 * such stream; the search consumes it in exactly the reference's order. */
/* random.seed(seeds[i]) for games first..first+n-1 (seeds are non-negative ints < 2**64). */
int zc_rng_seed(zc_engine *eng, int32_t first_game, int32_t n_games, const uint64_t *seeds);
/* random.setstate((3, tuple(mt) + (index,), None)) / random.getstate() for one game. */
int zc_rng_set_state(zc_engine *eng, int32_t game, const uint32_t *mt624, int32_t index);
int zc_rng_get_state(zc_engine *eng, int32_t game, uint32_t *mt624, int32_t *index);

/* ---- Connect4 search: replaces mcts.get_move (mcts.cpp:102-160) for
 *      backend = c4_backend, policy = Policy('random'), value = Value('random_rollout').
 * Games first_game .. first_game+n_games-1 are searched from roots[i] with `sims`
 * simulations, exploration constant `c` and leaf batch `batch_size`.  Outputs:
 *   out_move[i]          chosen column (first max of child visit count, move-list order)
 *   out_root_na[7*i+col] visits of the root child that drops in column `col` (0 if illegal)
 *   out_stats[i]         counters (may be NULL)
 * A root with no legal move, sims < 1 or batch_size < 1 is ZC_EINVAL (the reference
 * indexes moves[-1] there: mcts.cpp:150-157).  Host pointers; blocks until done. */
int zc_c4_search(zc_engine *eng, int32_t first_game, int32_t n_games, const zc_c4_state *roots,
                 int32_t sims, double c, int32_t batch_size,
                 int32_t *out_move, int32_t *out_root_na, zc_game_stats *out_stats);

/* Same for an arbitrary set of engine games: entry i searches game games[i] (distinct). */
int zc_c4_search_games(zc_engine *eng, int32_t n_games, const int32_t *games, const zc_c4_state *roots,
                       int32_t sims, double c, int32_t batch_size,
                       int32_t *out_move, int32_t *out_root_na, zc_game_stats *out_stats);

/* Same, with DEVICE pointers, enqueued on `hip_stream` (a hipStream_t; NULL = the null
 * stream) without synchronising.  Argument validation that needs the roots happens on the
 * device: a bad root sets out_stats[i].status (ZC_STATUS_*). */
int zc_c4_search_async(zc_engine *eng, int32_t first_game, int32_t n_games, const zc_c4_state *d_roots,
                       int32_t sims, double c, int32_t batch_size,
                       int32_t *d_out_move, int32_t *d_out_root_na, zc_game_stats *d_out_stats,
                       void *hip_stream);

/* Self-play of games first..first+n-1 for `moves` consecutive moves in ONE launch, each game
 * at its own pace: per move the search above from d_roots[i], then Engine.play_move +
 * _evaluate (as zc_c4_play_async), and a finished game restarts from the opening (the refill
 * of scripts/train.py:151-170 without a game quota).  d_roots is updated in place.  Step k's
 * post-move position, column and result (ZC_C4_ONGOING / +-1 / 0) go to
 * d_out_states / d_out_moves / d_out_results[k*n + i] — exactly the inputs of
 * zc_traj_record_async for that step, which the caller replays in step order.
 * d_stats[i] sums the moves' counters (reserved = games finished).  Results equal `moves`
 * rounds of zc_c4_search_async + zc_c4_play_async; games never wait for each other, so a
 * launch no longer waits once per move for its slowest game. */
int zc_c4_selfplay_async(zc_engine *eng, int32_t first_game, int32_t n_games, zc_c4_state *d_roots, int32_t sims,
                         double c, int32_t batch_size, int32_t moves, zc_c4_state *d_out_states,
                         int16_t *d_out_moves, int32_t *d_out_results, zc_game_stats *d_stats, void *hip_stream);

/* Pooled self-play: the same launch, but the n games share a budget of `budget` moves drawn
 * one at a time from the device counter d_ticket[0] (d_ticket[0..1] zeroed by this call).  This
 * is a throughput schedule, not the reference's: scripts/train.py:151-170 is lockstep (every
 * unfinished game gets one move per play_mcts_parallel call).  A game that moves faster plays
 * more moves, so the launch ends when the budget is spent, not when its slowest game has
 * played `moves_cap` moves.  Each game plays at most moves_cap moves, and its k-th
 * move is exactly the k-th move of zc_c4_selfplay_async (same search, RNG stream, refill):
 * only how many moves each game gets differs (decided by the counter, not deterministic).
 * Steps a game did not reach get result ZC_SLOT_SKIP and move -1 in the [moves_cap][n]
 * outputs; zc_traj_record_async leaves such slots untouched.  d_stats[i].leaves = the
 * simulations game i ran in this launch.  A move carried over by zc_c4_selfplay_carry_async
 * is resumed first (no ticket) and finished.  budget <= moves_cap * n_games, < 2^31; n_games <=
 * zc_c4_pooled_max_games (ZC_EINVAL otherwise).  d_ticket: 2 int32 — the
 * counter, then the most moves any game played (the d_reached of zc_traj_record_steps_async). */
int zc_c4_selfplay_pooled_async(zc_engine *eng, int32_t first_game, int32_t n_games, zc_c4_state *d_roots,
                                int32_t sims, double c, int32_t batch_size, int32_t moves_cap, int64_t budget,
                                int32_t *d_ticket, zc_c4_state *d_out_states, int16_t *d_out_moves,
                                int32_t *d_out_results, zc_game_stats *d_stats, void *hip_stream);

/* zc_c4_selfplay_pooled_async whose in-flight moves CARRY OVER instead of finishing: once the
 * budget is spent (d_ticket[0] reached it), every game's search stops at its next flush boundary
 * (batch_size simulations), and its progress — simulations done, tree nodes, and the tree, the
 * MT19937 stream and the root, which stay in the engine's HBM arena — is kept for the game's
 * next self-play launch (this one, zc_c4_selfplay_pooled_async or zc_c4_selfplay_async), which
 * resumes that move first, without a ticket.  The launch's tail — games finishing moves
 * started just before the budget ran out, on an emptying device — moves into the next launch,
 * where it runs at full occupancy.  Each game's k-th finished move is still exactly the k-th
 * move of zc_c4_selfplay_async (the search is cut only between flushes, and resumed with the
 * same tree and stream).  Outputs as zc_c4_selfplay_pooled_async: the suspended move has no
 * row (ZC_SLOT_SKIP); d_stats counts the expansions and simulations this launch ran.  Until a
 * non-carry self-play launch over these games (or zc_c4_carry_discard), entry points that
 * would search or reseed them (zc_c4_search*, zc_c4_ext_begin, zc_c4_rollouts, zc_rng_seed,
 * zc_rng_set_state, the c4 debug searches) refuse with ZC_EINVAL. */
int zc_c4_selfplay_carry_async(zc_engine *eng, int32_t first_game, int32_t n_games, zc_c4_state *d_roots,
                               int32_t sims, double c, int32_t batch_size, int32_t moves_cap, int64_t budget,
                               int32_t *d_ticket, zc_c4_state *d_out_states, int16_t *d_out_moves,
                               int32_t *d_out_results, zc_game_stats *d_stats, void *hip_stream);

/* Drop the carried moves of games [first_game, first_game + n_games) (stream-ordered): their
 * next search starts afresh from whatever root they are given.  Their MT19937 streams stay
 * where the dropped searches left them, so those games' moves no longer follow an
 * uninterrupted run's — for restarting games (C4SelfPlay.start), not for pausing them. */
int zc_c4_carry_discard(zc_engine *eng, int32_t first_game, int32_t n_games, void *hip_stream);

/* The most games zc_c4_selfplay_pooled_async accepts at this batch size: the games the
 * self-play grid keeps resident on the device at once (occupancy x compute units).  A pooled
 * launch hands out its budget only to resident waves, so larger launches are refused.  The
 * count assumes the launch has the device to itself: beside other resident kernels (another
 * process on the GPU, concurrent streams) some workgroups may start only after the budget is
 * spent, and their games then play no move in that launch (each game's moves stay exact;
 * only the share of moves per game changes). */
int zc_c4_pooled_max_games(zc_engine *eng, int32_t batch_size, int32_t *out);

/* Random source of the Connect4 search's rollouts (all zc_c4_search* calls that follow):
 *   ZC_ROLLOUT_EXACT (default) — the game's CPython MT19937 stream in the reference's order;
 *     results are bit-identical to mcts.get_move.
 *   ZC_ROLLOUT_PHILOX — SURVEY §8(d) C2(ii) "rollout fast mode": the same random playout
 *     (uniform legal moves until a win or a full board, value_functions.py:35-45), but each
 *     leaf draws from its own xoshiro128** stream seeded by Philox4x32-10(counter = (leaf's
 *     simulation index, game's MT position at the search's start, game, 0x0C4F0A57), key =
 *     seed), so a flush's leaves roll out in parallel.  Expansion draws still come from the
 *     game's MT stream.  Statistical parity with the reference only (same distribution of
 *     playouts, different numbers); specification: tests/c4_philox_ref.py. */
#define ZC_ROLLOUT_EXACT 0
#define ZC_ROLLOUT_PHILOX 1
int zc_c4_set_rollout_mode(zc_engine *eng, int32_t mode, uint64_t seed);

/* Engine.play_move + Engine._evaluate on the device for n games (engine/engine.py:98-108,
 * 148-153): states[i] = c4_backend.play_move(states[i], (moves[i], 0)) and
 *   results[i] = turn*2-1 if check_win (i.e. +1 when 'X' just won), 0 if check_draw, else
 *   ZC_C4_ONGOING.
 * A negative move leaves the game untouched (result ZC_C4_ONGOING).  With reset != 0 a
 * finished game restarts from create_init_state() — the self-play refill of
 * scripts/train.py:151-170.  Device pointers, enqueued on hip_stream (NULL = null stream). */
int zc_c4_play_async(zc_engine *eng, int32_t n_games, zc_c4_state *d_states, const int32_t *d_moves,
                     int32_t *d_results, int32_t reset, void *hip_stream);
#define ZC_C4_ONGOING 2

#define ZC_STATUS_NO_MOVES 1     /* root has no legal move                                */
#define ZC_STATUS_BAD_STATE 2    /* sentinel bits set / overlapping stones / bad turn    */
#define ZC_STATUS_INTERNAL 3     /* search invariant violated (never expected)            */
#define ZC_STATUS_CAPACITY 4     /* chess: child-slot pool or leaf depth (63) exhausted   */

/* Value('random_rollout').batch(states, backend=c4_backend) (engine/value_functions.py:20-45)
 * on the device: the n states are rolled out IN ORDER on engine game `game`'s stream, as the
 * reference does with its one global `random` stream.  out_values[i] in {-1, 0, 1} is the
 * value for states[i]'s side to move; *out_words (may be NULL) = words consumed.  Host
 * pointers; blocks. */
int zc_c4_rollouts(zc_engine *eng, int32_t game, int32_t n_states, const zc_c4_state *states,
                   int32_t *out_values, int64_t *out_words);

/* ---- Connect4 stepwise search: the flush handed to the caller ------------------------
 * mcts.get_move (mcts.cpp:102-160) with ANY value function: the search pauses at every
 * flush (mcts.cpp:112-127) and the caller evaluates the pending leaves — with a neural
 * network on the same device (Value('network_*'), value_functions.py:61-99) or with any
 * Python Value.batch — then resumes the search with their values.  Policy stays
 * Policy('random') (random.choice on the game's stream).  Wa is fp64 here, summed in pending
 * order exactly as mcts.cpp:90-95 does.  Device pointers, enqueued on hip_stream (NULL =
 * null stream), never synchronising, so a whole move can be captured in a HIP graph:
 *
 *   zc_c4_ext_begin(...)
 *   for f in 0 .. ceil(sims / batch_size) - 1:
 *       zc_c4_ext_select(..., f, ...)   -> leaves / planes of flush f
 *       values = value.batch(leaves)    (caller: NN forward, host callback, ...)
 *       zc_c4_ext_backup(..., f, values)
 *   zc_c4_ext_end(...)                  -> move, root visit counts, stats
 *
 * The sims / c / batch_size given to begin hold until end; one stepwise search per engine
 * game range at a time.  Leaf j of game i (j < the flush's leaf count) is slot
 * i*batch_size + j of every per-leaf buffer. */
int zc_c4_ext_begin(zc_engine *eng, int32_t first_game, int32_t n_games, const zc_c4_state *d_roots,
                    int32_t sims, double c, int32_t batch_size, void *hip_stream);
/* Selection + expansion of flush `flush`.  Outputs (each may be NULL):
 *   d_leaves[i*bs + j]  leaf state (zc_c4_state)
 *   d_planes            c4_backend.state_to_tensor (c4_backend.py:52-61) of every leaf:
 *                       [n_games*bs][2][6][7], plane 0 = side to move, row 0 = top;
 *                       planes_dtype ZC_F32 or ZC_F16
 *   d_counts[i]         leaves in this flush (0 for a game whose root is bad/terminal) */
int zc_c4_ext_select(zc_engine *eng, int32_t first_game, int32_t n_games, int32_t flush,
                     zc_c4_state *d_leaves, void *d_planes, int32_t planes_dtype, int32_t *d_counts,
                     void *hip_stream);
#define ZC_F32 0
#define ZC_F16 1
/* planes only (zc_chess_puct_select): fp16 in the MFMA tower's input layout, NHWC
 * [n][64 squares][32 channels] (the 17 planes, then zeros) — no separate conversion launch */
#define ZC_F16_NHWC32 2
/* Backprop of flush `flush` (mcts.cpp:80-100 in pending order): d_values[i*bs + j] is the
 * value of leaf j for ITS side to move, as Value.batch returns it. */
int zc_c4_ext_backup(zc_engine *eng, int32_t first_game, int32_t n_games, int32_t flush, const double *d_values,
                     void *hip_stream);
/* Final move selection (mcts.cpp:150-157) and counters; outputs as zc_c4_search_async. */
int zc_c4_ext_end(zc_engine *eng, int32_t first_game, int32_t n_games, int32_t *d_out_move, int32_t *d_out_root_na,
                  zc_game_stats *d_out_stats, void *hip_stream);

/* ---- Connect4 stepwise search with a HOST policy (any Python callable) ---------------
 * The §8(b) fallback for a Policy that is neither Policy('random') nor
 * Policy('immediate_value'): mcts.cpp's expand (:65-78) calls policy(untried_moves) once
 * per expansion, so inside a zc_c4_ext_begin .. end search each simulation of flush f is
 *
 *   zc_c4_hp_walk(eng, game, f, j, d_node)      select (mcts.cpp:47-63) from the root over
 *                                                the device tree -> the node, its position and
 *                                                its untried moves (columns, list order)
 *   k = index of policy(untried) in untried      (caller, e.g. Python)
 *   zc_c4_hp_expand(eng, game, f, j, k, d_leaf) expand (mcts.cpp:65-78) with the k-th untried
 *                                                move (ignored when the node has none), leaf j
 *                                                of the pending flush -> d_leaf
 *
 * for j = 0 .. leaves of the flush - 1, then zc_c4_ext_backup(eng, game, 1, f, values) as
 * usual.  The engine's RNG stream is not used (the caller's policy and value own theirs).
 * One game per call; every call only enqueues on hip_stream. */
typedef struct zc_c4_hp_node {
    zc_c4_state state;   /* position of the node the walk stopped at */
    int32_t node;        /* its id in the game's tree */
    int32_t n_untried;   /* untried moves (0: no legal move, the node itself becomes the leaf) */
    int32_t depth;       /* plies below the root */
    int32_t untried[7];  /* columns of the untried moves, in the node's move-list order */
} zc_c4_hp_node;
int zc_c4_hp_walk(zc_engine *eng, int32_t game, int32_t flush, int32_t leaf, zc_c4_hp_node *d_node,
                  void *hip_stream);
int zc_c4_hp_expand(zc_engine *eng, int32_t game, int32_t flush, int32_t leaf, int32_t untried_index,
                    zc_c4_state *d_leaf, void *hip_stream);

/* ---- Connect4 rules on the host (engine/games/connect4/c4_backend.py) --------------- */
/* rows: 42 chars, row 0 = top, 'X', 'O', anything else = empty. */
int zc_c4_from_rows(const char *rows42, int32_t turn, zc_c4_state *out);
int zc_c4_to_rows(const zc_c4_state *s, char *rows42);
/* CPython iteration order of c4_backend.get_legal_moves' set for a legal-column mask
 * (bit c = column c playable); writes the columns to cols[0..n) and returns n (0..7). */
int zc_c4_legal_order(int32_t mask, int32_t *cols);

/* ---- Chess rules on the device (engine/games/chess/src/chess_backend.cpp) -----------
 * A position in the reference's own encoding (include/state.h State, minus the history
 * deques, which only check_draw's repetition test reads and which stay with the host State):
 *   board[64]  State.board: ' ' empty, "PNBRQK" white, "pnbrqk" black; index 0 = a8 (row 0 =
 *              rank 8), row-major
 *   turn       0 = white to move; fifty = fifty_move_rule_counter (uint8, wraps like it)
 *   castle     bit 0 w_ck, 1 w_cq, 2 b_ck, 3 b_cq
 * A move is a uint16: from | to << 6 | capture value << 12, squares = row*8 + col, capture
 * value = fabs(piece_val) of the captured piece (the Move tuple's double: 0,1,3,5,9).
 * Move lists hold ZC_CHESS_MAX_MOVES slots per position, in the reference's order. */
typedef struct zc_chess_state {
    uint8_t board[64];
    uint8_t turn;
    uint8_t fifty;
    uint8_t castle;
    uint8_t reserved[5];
} zc_chess_state;
#define ZC_CHESS_MAX_MOVES 256
#define ZC_CHESS_WIN 1        /* check_win: no legal move and in check                    */
#define ZC_CHESS_STALEMATE 2  /* no legal move, not in check (check_draw)                  */
#define ZC_CHESS_FIFTY 4      /* fifty_move_rule_counter >= 50 (check_draw)                */
#define ZC_CHESS_OVERFLOW 8   /* more than ZC_CHESS_MAX_MOVES legal moves (never in chess) */

/* get_legal_moves for n positions: d_moves[i*ZC_CHESS_MAX_MOVES + j], d_counts[i] (-1 =
 * overflow).  Device pointers, enqueued on hip_stream (NULL = null stream). */
int zc_chess_legal_moves_async(zc_engine *eng, int32_t n, const zc_chess_state *d_states, uint16_t *d_moves,
                               int32_t *d_counts, void *hip_stream);
/* play_move of every legal move: d_children[i*ZC_CHESS_MAX_MOVES + j] (and the moves, if
 * d_moves is not NULL). */
int zc_chess_children_async(zc_engine *eng, int32_t n, const zc_chess_state *d_states, zc_chess_state *d_children,
                            uint16_t *d_moves, int32_t *d_counts, void *hip_stream);
/* d_out[i] = play_move(d_in[i], d_moves[i]) (d_out may equal d_in). */
int zc_chess_play_async(zc_engine *eng, int32_t n, const zc_chess_state *d_in, const uint16_t *d_moves,
                        zc_chess_state *d_out, void *hip_stream);
/* ZC_CHESS_* flags per position (check_win; check_draw without the repetition test). */
int zc_chess_terminal_async(zc_engine *eng, int32_t n, const zc_chess_state *d_states, int32_t *d_flags,
                            void *hip_stream);
/* has_repeated_prefix (chess_backend.cpp:148-180, pattern >= 2 moves, >= 3 repeats) of both
 * sides' move histories: d_hist [n][2][cap] uint16 packed moves, each side's in play order
 * (oldest first; the test reads them most recent first, as the reference's deques),
 * d_len [n][2] moves per side (<= cap); d_out[n] = white's answer | black's << 1 — the
 * repetition draw of check_draw is both bits.  cap in [1, 4096]; no engine needed. */
int zc_chess_repetition_async(int32_t n, int32_t cap, const uint16_t *d_hist, const int32_t *d_len, int32_t *d_out,
                              void *hip_stream);
/* state_to_tensor: [n][17][8][8], planes_dtype ZC_F32 / ZC_F16. */
int zc_chess_planes_async(zc_engine *eng, int32_t n, const zc_chess_state *d_states, void *d_planes,
                          int32_t planes_dtype, void *hip_stream);
/* state_from_fen (:525-556) / create_init_state (:446-457) on the host. */
int zc_chess_from_fen(const char *fen, zc_chess_state *out);
int zc_chess_init(zc_chess_state *out);

/* ---- Chess tree search: mcts.get_move (mcts.cpp:102-160) with the chess backend ---------
 * Policy: ZC_POLICY_RANDOM = Policy('random'), ZC_POLICY_IMMEDIATE_VALUE =
 * Policy('immediate_value', policy_freedom=freedom) (engine/policy_functions.py:10-20), both
 * drawing from the game's CPython MT19937 stream.  Outputs (device):
 *   d_out_move[i]                       chosen move (packed uint16, 0xFFFF if none)
 *   d_out_root_na[i*ZC_CHESS_MAX_MOVES + j]  Na of root move j (the root's get_legal_moves order)
 *   d_out_stats[i]                      counters; status ZC_STATUS_CAPACITY when the game's
 *                                       child-slot pool (64 * (max_sims+1)) or the leaf depth
 *                                       limit (63) was exhausted
 * The engine allocates its chess tree arena on the first chess search.
 * zc_chess_search_async evaluates leaves with Value('crude_chess_score')
 * (value_functions.py:48-55, configs/crude_chess.yaml) inside the kernel; batch_size <= 256. */
#define ZC_POLICY_RANDOM 0
#define ZC_POLICY_IMMEDIATE_VALUE 1
/* Allocate the chess tree arena now (it is otherwise allocated by the first chess search —
 * which must then not be inside a HIP-graph capture). */
int zc_chess_reserve(zc_engine *eng);
int zc_chess_search_async(zc_engine *eng, int32_t first_game, int32_t n_games, const zc_chess_state *d_roots,
                          int32_t sims, double c, int32_t batch_size, int32_t policy, double freedom,
                          uint16_t *d_out_move, int32_t *d_out_root_na, zc_game_stats *d_out_stats,
                          void *hip_stream);
/* Stepwise chess search with caller-supplied values, as zc_c4_ext_*: the leaves of flush f
 * are exported as states (zc_chess_state) and state_to_tensor planes [n*bs][17][8][8]. */
int zc_chess_ext_begin(zc_engine *eng, int32_t first_game, int32_t n_games, const zc_chess_state *d_roots,
                       int32_t sims, double c, int32_t batch_size, int32_t policy, double freedom, void *hip_stream);
int zc_chess_ext_select(zc_engine *eng, int32_t first_game, int32_t n_games, int32_t flush,
                        zc_chess_state *d_leaves, void *d_planes, int32_t planes_dtype, int32_t *d_counts,
                        void *hip_stream);
int zc_chess_ext_backup(zc_engine *eng, int32_t first_game, int32_t n_games, int32_t flush, const double *d_values,
                        void *hip_stream);
int zc_chess_ext_end(zc_engine *eng, int32_t first_game, int32_t n_games, uint16_t *d_out_move,
                     int32_t *d_out_root_na, zc_game_stats *d_out_stats, void *hip_stream);

/* Host-policy chess search inside a zc_chess_ext_begin .. end search (as zc_c4_hp_*): the
 * walk returns the node's position and its untried moves (packed from | to << 6 |
 * capture value << 12, in the node's untried-list order, the list mcts.cpp:67-70 hands to
 * the policy); expand takes the index of the caller's pick in that list. */
typedef struct zc_chess_hp_node {
    zc_chess_state state;
    int32_t node;
    int32_t n_untried;
    int32_t depth;
    int32_t reserved;
    uint16_t untried[ZC_CHESS_MAX_MOVES];
} zc_chess_hp_node;
int zc_chess_hp_walk(zc_engine *eng, int32_t game, int32_t flush, int32_t leaf, zc_chess_hp_node *d_node,
                     void *hip_stream);
int zc_chess_hp_expand(zc_engine *eng, int32_t game, int32_t flush, int32_t leaf, int32_t untried_index,
                       zc_chess_state *d_leaf, void *hip_stream);

/* ---- Value('random_rollout') on the chess backend (engine/value_functions.py:35-45 with
 * engine/games/chess/src/chess_backend.cpp: check_win / check_draw incl. the repetition draw
 * over both move histories, random.choice(list(get_legal_moves)), play_move) --------------
 * Histories: d_hist [k][2][hist_cap] uint16 packed moves of white / black in play order
 * (oldest first: the reference's deques reversed), d_hist_len [k][2].  A rollout's history
 * may hold ZC_CHESS_ROLL_CAP moves per side; beyond that (or a move list overflow) the
 * rollout stops and d_status[i] = ZC_STATUS_CAPACITY.  Values: -1 / +1 / 0 for the side to
 * move at the rolled-out state.
 * zc_chess_rollouts_async replaces Value.batch (:20-22) called directly: the n_states states
 * (their own histories, k = n_states) rolled out in order on game `game`'s stream;
 * d_values[n_states], d_status[1] (may be NULL).
 * zc_chess_ext_rollouts, after zc_chess_ext_select(flush) (or the flush's zc_chess_hp_*
 * simulations): every game's pending leaves in pending order on its stream — the flush of
 * mcts.cpp:112-127 with this value — the leaf histories being the root's (k = n_games, game
 * first + i at i) plus the path's moves; d_values[n*bs] as zc_chess_ext_backup takes them,
 * d_status[n] (may be NULL).
 * zc_chess_ext_leaf_moves: the path of every pending leaf of the flush (what a host
 * Value.batch needs to rebuild the leaf's histories): d_moves[(i*bs + j)*64 + l - 1] = the
 * move into level l, d_depth[i*bs + j] = the leaf's depth (0 past the flush's leaves). */
#define ZC_CHESS_ROLL_CAP 2048
int zc_chess_rollouts_async(zc_engine *eng, int32_t game, int32_t n_states, const zc_chess_state *d_states,
                            const uint16_t *d_hist, const int32_t *d_hist_len, int32_t hist_cap, double *d_values,
                            int32_t *d_status, void *hip_stream);
int zc_chess_ext_rollouts(zc_engine *eng, int32_t first_game, int32_t n_games, int32_t flush, const uint16_t *d_hist,
                          const int32_t *d_hist_len, int32_t hist_cap, double *d_values, int32_t *d_status,
                          void *hip_stream);
int zc_chess_ext_leaf_moves(zc_engine *eng, int32_t first_game, int32_t n_games, int32_t flush, uint16_t *d_moves,
                            int32_t *d_depth, void *hip_stream);

/* ---- Chess self-play on the device (scripts/train.py:151-170) ------------
 * Engine.play_move + _evaluate (engine/engine.py:98-108, 148-153) for chess, with the move
 * histories the repetition draw needs (chess_backend.cpp:364-441) kept in HBM:
 *   d_roots    [n] the positions to move from (updated: the post-move position, or d_init
 *              once the game has ended — the refill of a finished game)
 *   d_hist     [n][2][hist_cap] uint16 each side's moves in play order (packed moves)
 *   d_hist_len [n][2] int32 (zeroed when a game ends; hist_cap <= 4096)
 *   d_err      [3] int32, OR-ed: a game longer than hist_cap moves per side | a search out
 *              of tree capacity | no move at a live root (the game stops moving)
 * Results are Engine._evaluate's: turn*2-1 (checkmate, turn = side to move after the move),
 * 0 (stalemate, fifty-move rule, both sides' histories repeating), ZC_C4_ONGOING. */
typedef struct zc_chess_play_buffers {
    zc_chess_state *d_roots;
    const zc_chess_state *d_init;
    uint16_t *d_hist;
    int32_t *d_hist_len;
    int32_t hist_cap, reserved;
    int32_t *d_err;
} zc_chess_play_buffers;
/* One step of n games whose moves a search chose (any mode; d_moves[i] = 0xFFFF: none,
 * flagged): d_out_states / d_out_results [n] are the post-move positions and results
 * (the inputs of zc_traj_record_async with d_flags = NULL); d_search_stats (may be NULL)
 * flags searches out of capacity.  No engine needed. */
int zc_chess_play_step_async(int32_t n, const zc_chess_play_buffers *b, const uint16_t *d_moves,
                             const zc_game_stats *d_search_stats, zc_chess_state *d_out_states,
                             int32_t *d_out_results, void *hip_stream);
/* Crude-score self-play (zc_chess_search_async's search) of games first..first+n-1 for
 * `moves` consecutive moves in ONE launch, each game at its own pace: search, step, refill.
 * Outputs [moves][n] (post-move positions, moves, results: zc_traj_record_steps_async's
 * inputs); d_stats[i] sums the moves' counters (reserved = games finished).  Equal to
 * `moves` rounds of zc_chess_search_async + zc_chess_play_step_async. */
int zc_chess_selfplay_async(zc_engine *eng, int32_t first_game, int32_t n_games, const zc_chess_play_buffers *b,
                            int32_t sims, double c, int32_t batch_size, int32_t policy, double freedom,
                            int32_t moves, zc_chess_state *d_out_states, uint16_t *d_out_moves,
                            int32_t *d_out_results, zc_game_stats *d_stats, void *hip_stream);
/* Pooled form (as zc_c4_selfplay_pooled_async): the games share `budget` moves drawn from
 * d_ticket[0], at most moves_cap each; unreached steps get ZC_SLOT_SKIP and move 0xFFFF;
 * d_ticket[1] = the most moves any game played.  n_games <= zc_chess_pooled_max_games. */
int zc_chess_selfplay_pooled_async(zc_engine *eng, int32_t first_game, int32_t n_games,
                                   const zc_chess_play_buffers *b, int32_t sims, double c, int32_t batch_size,
                                   int32_t policy, double freedom, int32_t moves_cap, int64_t budget,
                                   int32_t *d_ticket, zc_chess_state *d_out_states, uint16_t *d_out_moves,
                                   int32_t *d_out_results, zc_game_stats *d_stats, void *hip_stream);
int zc_chess_pooled_max_games(int32_t hist_cap, int32_t *out);

/* ---- Chess PUCT search (AlphaZero-style; no reference counterpart) -------
 * Selection by Q + c_puct * P * sqrt(sum N) / (1 + N) with priors P from a policy network,
 * virtual loss within a flush, Dirichlet(alpha) noise of weight eps on the root priors
 * (Philox stream keyed by seed, counter (game, search number)).  d_search_no (device int32
 * [n_games], may be NULL = 0 for every game): game i's search number — the noise and the
 * temperature sample of the search come from it, and end adds 1 to it, so consecutive
 * searches (or replays of a captured graph) of a game draw fresh noise.  Flush 0 evaluates the root alone; then
 * ceil((sims - 1) / batch_size) flushes of up to batch_size leaves: zc_chess_puct_flushes.
 * select exports leaves/planes as zc_chess_ext_select; backup takes per leaf slot the value
 * for the leaf's side to move and 4096 policy logits indexed from*64 + to (logits_dtype
 * ZC_F32 / ZC_F16, or ZC_F16_NHWC32: the tower's input layout straight away); end picks
 * the move with the most visits (temperature 0) or samples
 * proportionally to N^(1/temperature), and writes root visits (and, optionally, the root
 * priors after noise, float [n][ZC_CHESS_MAX_MOVES]). */
int zc_chess_puct_flushes(int32_t sims, int32_t batch_size);
int zc_chess_puct_begin(zc_engine *eng, int32_t first_game, int32_t n_games, const zc_chess_state *d_roots,
                        int32_t sims, double c_puct, int32_t batch_size, float dirichlet_alpha, float dirichlet_eps,
                        uint64_t seed, int32_t *d_search_no, void *hip_stream);
int zc_chess_puct_select(zc_engine *eng, int32_t first_game, int32_t n_games, int32_t flush,
                         zc_chess_state *d_leaves, void *d_planes, int32_t planes_dtype, int32_t *d_counts,
                         void *hip_stream);
int zc_chess_puct_backup(zc_engine *eng, int32_t first_game, int32_t n_games, int32_t flush, const double *d_values,
                         const void *d_logits, int32_t logits_dtype, void *hip_stream);
/* zc_chess_puct_backup with the values / logits of game i's leaf j at row i * rows_per_game +
 * j: 0 = batch_size (the layout select writes the planes in); for flush 0, the roots-only
 * flush (one leaf a game), any rows_per_game >= 1 — 1 lets the caller evaluate the n root
 * positions alone instead of n * batch_size slots.  EINVAL for rows_per_game > 0 on a later
 * flush. */
int zc_chess_puct_backup_ex(zc_engine *eng, int32_t first_game, int32_t n_games, int32_t flush,
                            const double *d_values, const void *d_logits, int32_t logits_dtype,
                            int32_t rows_per_game, void *hip_stream);
int zc_chess_puct_end(zc_engine *eng, int32_t first_game, int32_t n_games, float temperature, uint16_t *d_out_move,
                      int32_t *d_out_root_na, float *d_out_root_prior, zc_game_stats *d_out_stats, void *hip_stream);

/* ---- Connect4 PUCT search (AlphaZero-style; no reference counterpart) -----
 * The chess PUCT search's rules (above) on the Connect4 rules of c4_backend.py: moves in
 * CPython set order, a node is terminal when the last mover has four (value -1 for the side
 * to move) or the board is full (value 0).  Flush count as zc_chess_puct_flushes.  select
 * exports the leaves (zc_c4_state) and their state_to_tensor planes [2][6][7]; backup takes
 * per leaf slot the value for the side to move and 7 column logits (logits_dtype ZC_F32 /
 * ZC_F16); end writes the move (a column), root visits and, optionally, root priors after
 * noise, per column [n][7]. */
int zc_c4_puct_begin(zc_engine *eng, int32_t first_game, int32_t n_games, const zc_c4_state *d_roots, int32_t sims,
                     double c_puct, int32_t batch_size, float dirichlet_alpha, float dirichlet_eps, uint64_t seed,
                     int32_t *d_search_no, void *hip_stream);
int zc_c4_puct_select(zc_engine *eng, int32_t first_game, int32_t n_games, int32_t flush, zc_c4_state *d_leaves,
                      void *d_planes, int32_t planes_dtype, int32_t *d_counts, void *hip_stream);
int zc_c4_puct_backup(zc_engine *eng, int32_t first_game, int32_t n_games, int32_t flush, const double *d_values,
                      const void *d_logits, int32_t logits_dtype, void *hip_stream);
/* As zc_chess_puct_backup_ex, for the Connect4 PUCT search. */
int zc_c4_puct_backup_ex(zc_engine *eng, int32_t first_game, int32_t n_games, int32_t flush, const double *d_values,
                         const void *d_logits, int32_t logits_dtype, int32_t rows_per_game, void *hip_stream);
int zc_c4_puct_end(zc_engine *eng, int32_t first_game, int32_t n_games, float temperature, int32_t *d_out_move,
                   int32_t *d_out_root_na, float *d_out_root_prior, zc_game_stats *d_out_stats, void *hip_stream);
/* Test hook: game `game`'s Connect4 PUCT tree as raw 192-byte node records (stones X/O, move
 * order word, turn, #moves, evaluated, won, parent, parent slot, depth, children[8], N[8],
 * P[8] float, W[8] double); *out_count = nodes.  Synchronises the device. */
int zc_debug_c4_puct_tree(zc_engine *eng, int32_t game, int32_t max_nodes, void *out_nodes, int32_t *out_count);

/* ---- Value-network layers on the matrix cores (models/chess_value/network.py:24-45) -----
 * The residual tower of ValueNetwork with BatchNorm folded into the convolutions, NHWC fp16
 * activations ([n][h][w][c], a pixel's channels contiguous), 128 output channels.
 *   zc_net_conv3x3_async: out = act(conv3x3(in, weight) + bias (+ residual)), padding 1;
 *     weight [9][128][cin] fp16 (tap = ky*3+kx, then output channel, then input channel),
 *     bias [128] f32, residual NULL or [n][h][w][128] fp16, relu 0/1.  Shapes: (h, w) in
 *     {(8, 8), (6, 7)}, cin in {32, 128}; others are ZC_EINVAL.
 *   zc_net_conv3x3_pack_async: the same weights repacked for the streamed-weight kernel:
 *     packed[((tap*(cin/16) + kc)*4 + mb)*512 + lane*8 + e] =
 *     weight[tap][mb*32 + lane%32][kc*16 + 8*(lane/32) + e] (one contiguous 1-KB MFMA operand
 *     fragment per (tap, kc, mb)); same size as weight.  Pack once per weight set.
 *   zc_net_conv3x3_packed_async: zc_net_conv3x3_async on packed weights; bit-identical
 *     output, faster (every wave streams its own weight fragments from L2; no LDS staging).
 *   zc_net_tower_async: the whole residual tower in one launch (the stem and (nconv-1)/2
 *     residual blocks, network.py:33-36; every layer act = relu), activations kept on chip
 *     from input to output; bit-identical to the layer-by-layer packed launches.  d_in =
 *     [n][h*w][cin0] fp16 (zc_net_planes_to_nhwc_async), d_packed = the packed weights of the
 *     nconv layers back to back (stem 9*cin0*128 halfs, then 9*128*128 per layer), d_bias =
 *     [nconv][128] f32, d_out = [n][h*w][128] fp16 or NULL; all 16-byte aligned.  With
 *     d_values (fp64 [n]) the value head runs in the same launch on the on-chip activation
 *     (d_fc_w [128] f32, fc_b; bit-identical to zc_net_value_head_async), so a value-only
 *     network needs no d_out.  cin0 = 32, nconv odd, (h, w) in {(8, 8), (6, 7)}.  Runs the
 *     16x16x32 MFMA form (environment ZC_TOWER_MF=32: the 32x32x16 form; same outputs).
 *   zc_net_planes_to_nhwc_async: state_to_tensor planes [n][cin][h*w] fp16 -> [n][h*w][cpad],
 *     zero padded; cpad a multiple of 8 (16-byte rows), d_out 16-byte aligned.
 *   zc_net_value_head_async: mean over pixels -> dot(fc_w[128]) + fc_b -> tanh, as fp64
 *     values[n] (the input of zc_*_ext_backup).  d_act = [n][hw][128] fp16 (exactly 128
 *     channels), 16-byte aligned (ZC_EINVAL otherwise).
 * Device pointers, enqueued on hip_stream (NULL = null stream); no engine needed. */
int zc_net_conv3x3_async(int32_t n_boards, int32_t h, int32_t w, int32_t cin, const void *d_in, const void *d_weight,
                         const float *d_bias, const void *d_residual, void *d_out, int32_t relu, void *hip_stream);
int zc_net_conv3x3_pack_async(int32_t cin, const void *d_weight, void *d_packed, void *hip_stream);
int zc_net_conv3x3_packed_async(int32_t n_boards, int32_t h, int32_t w, int32_t cin, const void *d_in,
                                const void *d_packed_weight, const float *d_bias, const void *d_residual, void *d_out,
                                int32_t relu, void *hip_stream);
int zc_net_tower_async(int32_t n_boards, int32_t h, int32_t w, int32_t cin0, int32_t nconv, const void *d_in,
                       const void *d_packed_weights, const float *d_biases, void *d_out, const float *d_fc_w,
                       float fc_b, double *d_values, void *hip_stream);
/* zc_net_tower_policy_async: zc_net_tower_async with the policy head's 1x1 convolution (128 -> 32
 *   channels, BN folded, ReLU) folded into the same launch as an MFMA epilogue on the on-chip
 *   tower output (the PUCT network of SURVEY §8 a21 / config C5, which has no reference
 *   counterpart): d_pw = the 1x1 weights packed as MFMA A fragments
 *   [8][64][8] fp16 (nets.pack_policy_1x1), d_pb = [32] f32, d_pout = [n][h*w][32] fp16 (8-byte
 *   aligned) — the policy head's flatten + linear is then one GEMM over d_pout.  The value head
 *   (d_fc_w, fc_b, d_values) is required; no tower activation is written. */
int zc_net_tower_policy_async(int32_t n_boards, int32_t h, int32_t w, int32_t cin0, int32_t nconv, const void *d_in,
                              const void *d_packed_weights, const float *d_biases, const float *d_fc_w, float fc_b,
                              double *d_values, const void *d_pw, const float *d_pb, void *d_pout, void *hip_stream);
/* zc_net_tower_policy_ex_async: zc_net_tower_policy_async with policy_channels = 32 or 64 output
 *   channels (d_pw [policy_channels / 32][8][64][8], d_pb [policy_channels] f32, d_pout
 *   [n][h*w][policy_channels]) and the ReLU on (relu != 0) or off.  policy_channels 64, relu 0
 *   on an 8x8 board is the CONVOLUTIONAL policy head (nets.PolicyValueNetwork(head="conv"),
 *   AlphaZero's design): logit(from, to) = channel `to` at pixel `from`, so d_pout viewed as
 *   [n][4096] is the logits in the from*64 + to order zc_chess_puct_backup reads — no GEMM. */
int zc_net_tower_policy_ex_async(int32_t n_boards, int32_t h, int32_t w, int32_t cin0, int32_t nconv,
                                 const void *d_in, const void *d_packed_weights, const float *d_biases,
                                 const float *d_fc_w, float fc_b, double *d_values, const void *d_pw, const float *d_pb,
                                 int32_t policy_channels, int32_t relu, void *d_pout, void *hip_stream);
int zc_net_planes_to_nhwc_async(int32_t n, int32_t cin, int32_t hw, int32_t cpad, const void *d_planes, void *d_out,
                                void *hip_stream);
int zc_net_value_head_async(int32_t n, int32_t hw, const void *d_act, const float *d_fc_w, float fc_b, double *d_values,
                            void *hip_stream);

/* ---- self-play trajectories on the device ---------------------------
 * Replaces the host half of self-play data collection: Engine.play_move's history append
 * (engine/engine.py:98-108), Engine.get_dataset's labels (:60-89: factor 0 for a draw else
 * -1, alternating, the game's list reversed) and scripts/train.py:simulate_games's refill
 * and quota (:151-170: a slot starts a new game only while fewer than `quota` games have
 * started).  The caller owns every buffer (device memory):
 *   d_hist     [n][max_len] rows    the slot's current game, opening first
 *   d_hmoves   [n][max_len] int16   move played from each of those positions
 *   d_slot     [n][4] int32         {positions so far, game number (-1 = idle), scratch x2}
 *   d_pool     [pool_cap] rows      finished games' positions, game after game (pool_cap < 2^31)
 *   d_labels   [pool_cap] int32     get_dataset label of each pooled position
 *   d_pool_moves [pool_cap] int16   move played from it (-1 at the game's last position)
 *   d_games    [games_cap][4] int64 {game number, slot << 32 | (result + 1), first pooled
 *                                    position, positions}
 *   d_ctl      [8] int64            ZC_TRAJ_* counters below
 *   d_init     one row              the opening (create_init_state)
 * Rows are opaque records of row_bytes (a multiple of 8): a zc_c4_state is 24 bytes, a
 * zc_chess_state 72.  Games land in the pool in completion order (atomics); the game
 * records give each game's place. */
typedef struct zc_traj_buffers {
    int32_t row_bytes, max_len;
    int64_t pool_cap;
    int32_t games_cap, reserved;
    void *d_hist;
    int16_t *d_hmoves;
    int32_t *d_slot;
    void *d_pool;
    int32_t *d_labels;
    int16_t *d_pool_moves;
    int64_t *d_games;
    int64_t *d_ctl;
    const void *d_init;
} zc_traj_buffers;
#define ZC_TRAJ_POSITIONS 0  /* pool positions reserved                                */
#define ZC_TRAJ_GAMES 1      /* game records reserved                                  */
#define ZC_TRAJ_NEXT 2       /* game number the next refill takes                      */
#define ZC_TRAJ_QUOTA 3      /* games to start in total (simulate_games' total_games)  */
#define ZC_TRAJ_FINISHED 4   /* games finished                                         */
#define ZC_TRAJ_OVERFLOW 5   /* bit 0: pool full (games dropped); bit 1: a game longer than max_len;
                              * bit 2: the quota ran out inside a multi-step record */
#define ZC_SLOT_IDLE 3       /* result of an idle slot                                 */
#define ZC_SLOT_SKIP 4       /* Connect4 pooled self-play: no move at this step (slot untouched) */
/* After a move was played on every slot (d_states = positions after the move, d_moves =
 * the moves, int16: Connect4 column / packed chess move): append each position to its
 * slot's game; a finished game is copied to the pool and its slot restarts from d_init (the
 * position in d_states is reset too) or goes idle.  Results: Connect4 passes
 * d_results from zc_c4_play_async (reset = 0) and d_flags = d_rep = NULL; chess passes
 * d_flags from zc_chess_terminal_async and d_rep from zc_chess_repetition_async (NULL = no
 * repetition test) and d_results is written (Engine._evaluate).  Idle slots get
 * ZC_SLOT_IDLE; Connect4 slots whose result is ZC_SLOT_SKIP are left as they are.  No engine
 * needed; enqueued on hip_stream. */
int zc_traj_record_async(int32_t n, const zc_traj_buffers *buf, void *d_states, const int16_t *d_moves,
                         int32_t *d_results, const int32_t *d_flags, const int32_t *d_rep, void *hip_stream);
/* zc_traj_record_async for `steps` consecutive steps of a self-play launch (Connect4
 * zc_c4_selfplay*_async, chess zc_chess_selfplay*_async), with the same pool, game numbers,
 * labels and slot histories as `steps` single-step calls in step order — d_states / d_moves /
 * d_results are the launch's [steps][n] outputs (results already evaluated; ZC_SLOT_SKIP = no
 * move, only after a slot's last move).  Four launches whatever `steps` is: per slot the
 * finished games' lengths, a scan of (games, positions) over the [steps][n] grid in step-major
 * order (the order single steps number the games in), then one wave per slot copies its
 * finished games to their pool places and appends its unfinished game to its history.  With
 * d_reached (device int32, e.g. d_ticket + 1 of the pooled launches) only the steps
 * k < *d_reached are read.  Needs the unlimited quota (a refill that would pass the quota sets
 * ZC_TRAJ_OVERFLOW bit 2).  The launch's rows in d_states are not modified.  d_scratch: device
 * scratch of at least zc_traj_steps_scratch_bytes(n, steps) bytes, 16-byte aligned. */
int zc_traj_steps_scratch_bytes(int32_t n, int32_t steps, int64_t *bytes);
int zc_traj_record_steps_async(int32_t n, const zc_traj_buffers *buf, void *d_states, const int16_t *d_moves,
                               int32_t *d_results, int32_t steps, const int32_t *d_reached, void *d_scratch,
                               int64_t scratch_bytes, void *hip_stream);

/* ---- any game backend: SURVEY §8(b)'s fallback (gen_search.hip) ----------------------
 * mcts.get_move (mcts.cpp:102-160) for a backend the device knows nothing about: the caller
 * keeps the game states and move objects (backend.get_legal_moves / play_move, the policy
 * callable and value.batch are called on the host, where mcts.cpp calls them) and this
 * library keeps the tree — N, Na, Wa, Qa, children, untried lists — and does the selection,
 * the expansion bookkeeping and the backup on the device.  One search at a time per engine:
 *   zc_gen_begin(sims, c, batch_size, root_moves)      Node(root, moves) (:104-108)
 *   per simulation:
 *     zc_gen_walk(d_out, out_cap)    select (:47-63) -> d_out = {node, #untried, #moves,
 *                                    depth, status, untried move indices in list order...}
 *     zc_gen_expand(untried_index, child_moves)   expand (:65-78) with the policy's pick
 *                                    (list.index of its move among the untried ones) and
 *                                    len(get_legal_moves(play_move(state, move))); -1 when
 *                                    the walk ended at a node with nothing untried (the leaf
 *                                    is that node).  The new node's id is the count of nodes
 *                                    before it (root = 0), so the caller indexes its states.
 *     after every batch_size leaves, and at the end: zc_gen_backup(n, d_values) with
 *     value.batch's results in pending order (:112-127, backprop :80-100)
 *   zc_gen_end(d_out, d_root_na, na_cap)  d_out = {best root move index (first maximum of
 *     child N, -1 if none), status, expansions, depth sum, nodes}; root Na per move.
 * Child move slots come from a pool the caller grows with zc_gen_reserve before an expansion
 * would overflow it (zc_gen_capacity); zc_gen_begin reserves sims + 1 nodes.  d_values
 * fp64; all d_ pointers are device memory; calls are stream-ordered. */
int zc_gen_reserve(zc_engine *eng, int32_t nodes, int64_t slots);
int zc_gen_capacity(zc_engine *eng, int32_t *nodes, int64_t *slots);
int zc_gen_begin(zc_engine *eng, int32_t sims, double c, int32_t batch_size, int32_t root_moves, void *hip_stream);
int zc_gen_walk(zc_engine *eng, int32_t *d_out, int32_t out_cap, void *hip_stream);
int zc_gen_expand(zc_engine *eng, int32_t untried_index, int32_t child_moves, void *hip_stream);
int zc_gen_backup(zc_engine *eng, int32_t n_leaves, const double *d_values, void *hip_stream);
int zc_gen_end(zc_engine *eng, int32_t *d_out, int32_t *d_root_na, int32_t na_cap, void *hip_stream);

/* ---- self-test hooks (used by the parity tests) -------------------------------------
 * UCT score exactly as the search kernel computes it (mcts.cpp:41-45), evaluated ON THE
 * DEVICE for n inputs: out[i] = na[i]==0 ? +inf : fma(c, sqrt(logn[i]/na[i]), q[i]). */
int zc_debug_uct(zc_engine *eng, int32_t n, const double *logn, const int32_t *na, const double *q,
                 double c, double *out);
/* Value('random_rollout') on the device for n positions, game i using engine game
 * first_game+i's stream: out_value[i] in {-1,0,1}, out_words[i] = words consumed. */
int zc_debug_c4_rollout(zc_engine *eng, int32_t first_game, int32_t n, const zc_c4_state *states,
                        int32_t *out_value, int64_t *out_words);

/* The tree walk alone (the walk-roofline measurement, tools/prof_walk.py): the lockstep
 * Connect4 search of zc_c4_search_async with its rollouts recorded (mode 1: d_vals[g][sims]
 * int8 the value of every simulation's leaf, d_words[g][ceil(sims/bs)] the words each flush's
 * rollouts consumed; otherwise the normal search) or replayed (mode 2: the recorded values,
 * the stream moved past the recorded words, no rollout run) — from the same roots and streams
 * the replay builds the identical tree, so its time and HBM traffic are the walk's.
 * zc_debug_rng_copy copies games first..first+n-1's streams (ring + positions) to d_buf
 * (restore = 0) or back (restore = 1); d_buf holds n * (4096 * 4 + 16) bytes. */
int zc_debug_c4_walk_async(zc_engine *eng, int32_t first_game, int32_t n_games, const zc_c4_state *d_roots,
                           int32_t sims, double c, int32_t batch_size, int32_t mode, int8_t *d_vals, uint32_t *d_words,
                           int32_t *d_out_move, int32_t *d_out_root_na, zc_game_stats *d_out_stats, void *hip_stream);
int zc_debug_rng_copy(zc_engine *eng, int32_t first_game, int32_t n_games, void *d_buf, int32_t restore,
                      void *hip_stream);

/* A chess tree after a search (PUCT or UCT), copied to host buffers for the parity tests:
 * out_nodes = raw 96-byte node records (position, first slot, #moves, #untried, parent,
 * parent slot index, depth, material, mated flag, evaluated), then per child slot the packed
 * move, prior, Na, Wa and child node (0xFFFF = none); out_counts = {nodes, slots used}.
 * The in-check flag is computed only for a node WITH NO legal move (checkmate vs stalemate,
 * the one case every caller reads): it is 0 for every node that has moves, in check or not.
 * In a UCT tree (crude score, value network) a node never expanded is LAZY: #moves = 0xFFFF,
 * #untried = 1, no slots — its legal moves exist but are generated at its first expansion.
 * Synchronises the device. */
int zc_debug_chess_tree(zc_engine *eng, int32_t game, int32_t max_nodes, int32_t max_slots, void *out_nodes,
                        uint16_t *out_mv, float *out_prior, int32_t *out_na, double *out_w, uint16_t *out_child,
                        int32_t *out_counts);

/* The crude search's lazy-node probe (legal_moves_probe: a sufficient free-move test, then one
 * pseudo-legal move per piece through the legality test, then the full get_legal_moves) on n
 * positions: d_out[i] = -2 when it proved a legal move without generating the list, else the
 * generated list's length (-1 = overflow).  Device pointers, enqueued on hip_stream. */
int zc_debug_chess_probe_async(zc_engine *eng, int32_t n, const zc_chess_state *d_states, int32_t *d_out,
                               void *hip_stream);

/* Diagnostic phase stamps: returns (into out8, may be NULL) the shader-cycle sums since the
 * previous call, over all games, of {RNG generation, first walk of each flush, resumed
 * walks, expansion + leaf bookkeeping, rollouts, backup, publish, 0}, resets them, and switches
 * the stamped kernel build on (enable != 0) or off for later searches.  Synchronises the
 * device.  Stamped runs are for phase SHARES only, never for timing. */
int zc_debug_phase_cycles(zc_engine *eng, int32_t enable, int64_t *out8);
/* The same stamps per game (no reset): out[g * 8 + k] for games 0 .. n_games-1. */
int zc_debug_phase_cycles_games(zc_engine *eng, int32_t n_games, int64_t *out);

/* The network launches' A/B and test switches (process-wide; read from ZC_TOWER_MF,
 * ZC_TOWER_EPI, ZC_HEAD_RAW once when the library loads, never per launch): name "tower_mf"
 * (16 or 32: the fused tower's MFMA form; 0 = default), "tower_epi" (0 default, 1 the 16-byte
 * store epilogue, 2 the per-tile epilogue), "head_raw" (1: the value head returns its pre-tanh
 * sum — tests only).  Returns the previous value in *old (may be NULL); ZC_EINVAL for an
 * unknown name or value. */
int zc_debug_net_switch(const char *name, int32_t value, int32_t *old);
/* Launch-timeline stamps of the Connect4 self-play launches (the pooled launch's tail,
 * tools/launch_tail.py): with d_buf != NULL (device, 4 x uint64 per game of the engine),
 * every later Connect4 self-play launch (zc_c4_selfplay_async, its pooled form) writes per game {s_memrealtime at its wave's
 * start, at the start of its last move, at its end, moves played | placement << 32}
 * (placement: HW_ID bits 15:0 — wave slot, SIMD, CU, SH, SE — and the XCC << 16); NULL
 * switches them off. */
int zc_debug_c4_launch_stamps(zc_engine *eng, uint64_t *d_buf);

#ifdef __cplusplus
}
#endif
#endif
