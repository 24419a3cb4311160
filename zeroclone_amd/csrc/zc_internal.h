// zc_internal.h — engine state, HBM layout and launch declarations shared by the host
// API (engine.hip) and the kernels (c4_search.hip).  gfx950 only.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <mutex>
#include <string>

#include "../../include/zeroclone.h"

namespace zc {

// ---------------------------------------------------------------- HBM layout (Connect4)
// One game owns a contiguous arena of M = max_sims + 1 node records.  A record is one
// 128-byte line — everything selection reads for a node (mcts.cpp:10-39 Node, minus the
// Python objects) — so the per-level load of the tree walk is one L2 line per game:
//
//   +0   u32  (unused)     Node::N is not stored: it equals Na of the in-edge (root: the
//                          number of leaves flushed so far)
//   +4   u32  untried      bit i (i < 7) set while move i is untried    (Node::untried)
//                          bits 28..31: #moves                          (Node::moves.size())
//   +8   u32  link         parent (u16, 0xFFFF at the root) | pact << 16 | depth << 24
//                                                  (Node::parent, parent_action_idx)
//   +12  u32  order        packed 3-bit columns of the move list (CPython set order),
//                          bits 24..27: #moves
//   +16  u16  child[8]     0xFFFF = null                              (Node::children)
//   +32  i32  Na[8]                                                    (Node::Na)
//   +64  [8]  Wa           rollout search: i32 (rollout values are +-1 / 0, so Wa is an
//                          integer); stepwise search: f64.  Qa (Node::Qa) is formed as
//                          Wa / Na when the walk reads the edge — the IEEE quotient
//                          mcts.cpp:95 stores, so UCT's inputs are bit-identical
// Boards are not stored: the walk re-applies moves from the root.
constexpr int kRecBytes = 128;
constexpr int kSlots = 8;
constexpr int kMaxDepth = 44;          // levels 0..42 (a C4 game has at most 42 plies)
constexpr int kRingLog2 = 12;          // per-game MT19937 ring: 4096 raw words
constexpr int kRingWords = 1 << kRingLog2;
constexpr int kLookahead = 2048;       // words generated ahead at each flush start
constexpr int kChunk = 192;            // words per generation step (<= 227, multiple of 64)
constexpr int kBlock = 64;             // threads per workgroup: one wave = one game
constexpr int kPhases = 8;             // diagnostic phase-stamp slots per game

static_assert(kLookahead + kChunk + 624 + 192 < kRingWords, "ring must retain the current MT block");

struct Arena {
    uint8_t *nodes = nullptr;     // [G][M][128 B]
    uint32_t *ring = nullptr;     // [G][kRingWords]    raw (untempered) MT words
    uint64_t *rngpos = nullptr;   // [G][2]             {next word to use, words generated}
    double *logtab = nullptr;     // [M+2]              glibc log(n), n = 0..M+1
    uint4 *carry = nullptr;       // [G]                a carried self-play move {done, nodes, tag, 0}
    int32_t *progress = nullptr;  // [64]               free self-play runs: moves finished so far
    int64_t *phase = nullptr;     // [G][kPhases]       diagnostic phase cycles (stamp build)
    // staging for the synchronous host entry points
    zc_c4_state *roots = nullptr;
    int32_t *move = nullptr;
    int32_t *na = nullptr;
    int32_t *ids = nullptr;
    zc_game_stats *stats = nullptr;
    // stepwise (caller-valued) search: per-game control words and the pending flush
    int32_t *ext_ctl = nullptr;       // [G][kCtlWords]
    uint16_t *ext_paths = nullptr;    // [G][max_batch][kMaxDepth]  node ids of each leaf's path
    uint32_t *ext_meta = nullptr;     // [G][max_batch]             leaf node | depth << 16 | turn << 24
    zc_c4_state *ext_roots = nullptr; // [G]
};

// ext_ctl words of one game
enum : int {
    kCtlNodes = 0,   // nodes in the tree
    kCtlF0 = 1,      // first node of the pending flush
    kCtlD0 = 2,      // depth of the flush's X0
    kCtlNb = 3,      // leaves in the pending flush
    kCtlStatus = 5,  // ZC_STATUS_*
    kCtlExp = 6,     // expansions so far
    kCtlDepth = 7,   // sum of expansion depths
    kCtlUse0 = 8,    // (2 words) RNG position at begin
    kCtlHpNode = 10, // host-policy search, the last walk's end: node, depth | turn << 8 (word 11),
                     // position s0 lo/hi, s1 lo/hi (words 12..15)
    kCtlPath = 16,   // [kMaxDepth] root..X0: node | slot << 16
    kCtlWords = 64,
};

struct SearchParams {
    int first_game, n_games, sims, bs, M;
    double c;
    const int32_t *game_ids;  // optional: engine game of call entry i (else first_game + i)
    const zc_c4_state *roots;
    int32_t *out_move, *out_na;
    zc_game_stats *out_stats;
    Arena a;
    int max_batch;
    int stamp;
    int philox;            // rollouts: 0 = the game's MT19937 stream (exact), 1 = Philox mode
    uint64_t philox_seed;  // Philox key of the Philox rollout mode
    // self-play run (c4_selfplay_kernel): moves per game, per-step outputs [moves][n_games]
    int moves;
    zc_c4_state *io_roots;  // = roots, written after every move
    zc_c4_state *out_states;
    int16_t *out_moves16;
    int32_t *out_results;
    // pooled self-play: moves drawn from ticket[0] while < budget (null: `moves` per game);
    // ticket[1] = the most moves any game played
    int32_t *ticket;
    int32_t budget;
    int carry;   // 1: suspend in-flight moves once the budget is spent (zc_c4_selfplay_carry_async)
    int32_t *progress;  // free runs: the launch's finished moves (pace balancing; null: off)
    // walk diagnostic (c4_walk_kernel): per game the rollout value of every simulation
    // [G][sims] and the rollout words of every flush [G][ceil(sims / bs)]
    int8_t *walk_vals;
    uint32_t *walk_words;
    // launch-timeline diagnostic (zc_debug_c4_launch_stamps; null: off): per game of a
    // self-play launch {s_memrealtime at the wave's start, at its last move's start, at its end,
    // moves played}
    uint64_t *tstamps;
};

struct ExtParams {
    int first_game, n_games, sims, bs, M, max_batch, flush;
    double c;
    Arena a;
    const zc_c4_state *roots;  // begin
    zc_c4_state *leaves;       // select (optional)
    void *planes;              // select (optional)
    int planes_f16;
    int32_t *counts;           // select (optional)
    const double *values;      // backup
    int32_t *out_move, *out_na;
    zc_game_stats *out_stats;  // end
    // host-policy stepwise search (zc_c4_hp_*): leaf index in the flush, untried index, node out
    int hp_leaf, hp_index;
    zc_c4_hp_node *hp_node;
};

// ---------------------------------------------------------------- chess tree search
// Per game: M node records (ChessNode) and a pool of S child slots; node i's moves occupy
// slots [base, base + nmoves) in the reference's move order.  Slot arrays are SoA so the
// UCT scan over a node's children is a coalesced read per array.
constexpr int kChessPath = 64;      // deepest leaf a flush may hold (levels 0..63)
constexpr int kChessSlotsPerNode = 64;

struct ChessNode {
    zc_chess_state st;   // 72 B: the position (board bytes, turn, fifty, castling)
    uint32_t base;       // first child slot
    uint16_t nmoves;     // legal moves (Node::moves.size())
    uint16_t nu;         // untried moves left (Node::untried.size())
    uint16_t parent;     // 0xFFFF at the root
    uint16_t pact;       // slot index in the parent's move list (parent_action_idx)
    uint16_t depth;
    int16_t material;    // sum of piece values, white positive (crude_chess_score)
    uint8_t check;       // side to move in check, computed for a node without legal moves (0 otherwise)
    uint8_t evaluated;   // PUCT search: the network's priors are in the slots
    uint8_t pad[6];
};
static_assert(sizeof(ChessNode) == 96, "ChessNode is 96 bytes");

struct ChessArena {
    ChessNode *nodes = nullptr;  // [G][M]
    uint16_t *mv = nullptr;      // [G][S] packed move (from | to << 6 | value << 12)
    uint8_t *ut = nullptr;       // [G][S] untried list: indices into the node's moves, in order
    uint16_t *ch = nullptr;      // [G][S] child node, 0xFFFF = null
    int32_t *na = nullptr;       // [G][S] Na
    double *w = nullptr;         // [G][S] Wa (fp64, summed in pending order)
    float *prior = nullptr;      // [G][S] P (PUCT search: the policy network's prior)
    int32_t *ctl = nullptr;      // [G][kCtlWords]
    uint32_t *paths = nullptr;   // [G][max_batch][kChessPath] slot of the edge into each level
    uint32_t *meta = nullptr;    // [G][max_batch] leaf node | depth << 16
    zc_chess_state *roots = nullptr;  // [G]
    // the PUCT select's deferred expansions (chess_puct.hip): per leaf of the flush that created
    // its node, the node's generated moves [G][max_batch][256] and {#moves (-1: overflow),
    // material | check << 16} [G][max_batch][2], between the expand and commit kernels
    uint16_t *xmv = nullptr;
    int32_t *xinfo = nullptr;
    int64_t S = 0;
};

struct ChessParams {
    int first_game, n_games, sims, bs, M, max_batch, flush;
    double c;
    int policy;        // 0 = Policy('random'), 1 = Policy('immediate_value')
    double freedom;    // policy_freedom
    // immediate_value's candidate classes: bit 5 i + k set when capture value V[k] >= V[i] -
    // freedom (V = 0, 1, 3, 5, 9: the maximum V[i] among the untried moves), chess_params_cls_ok
    uint32_t cls_ok;
    Arena a;           // RNG ring / positions and the log table
    ChessArena ca;
    const zc_chess_state *roots;
    zc_chess_state *leaves;
    void *planes;
    int planes_f16;
    int32_t *counts;
    const double *values;
    uint16_t *out_move;
    int32_t *out_na;   // [n][ZC_CHESS_MAX_MOVES]
    zc_game_stats *out_stats;
    // PUCT search (chess_puct.hip)
    float dir_alpha, dir_eps;   // Dirichlet root noise
    uint64_t seed;              // counter-based RNG key (noise, temperature sampling)
    int32_t *search_no;         // [n] per-game search number (counter word; end adds 1), or null
    float temperature;          // end: 0 = most visits, > 0 = sample proportional to Na^(1/T)
    const void *logits;         // backup: [n*bs][4096] policy logits (from*64 + to)
    int logits_f16;
    int leaf_rows;              // backup: rows of values / logits per game (0: bs; 1: a roots-only flush)
    float *out_prior;           // end (optional): root priors after noise [n][ZC_CHESS_MAX_MOVES]
    // host-policy search (zc_chess_hp_*): leaf index in the flush, untried index, walk output
    int hp_leaf, hp_index;
    zc_chess_hp_node *hp_node;
    // random_rollout on chess (zc_chess_rollouts_async / zc_chess_ext_rollouts): the states'
    // (or the roots') move histories [n][2][rhcap] in play order, lengths [n][2]; values out
    const zc_chess_state *rstates;   // direct rollouts: the n_states states (else the tree's leaves)
    int n_states;
    const uint16_t *rhist;
    const int32_t *rhlen;
    int rhcap;
    double *rvalues;
    int32_t *rstatus;
    uint16_t *path_moves;            // zc_chess_ext_leaf_moves: [n*bs][kChessPath]
    int32_t *path_depth;             // [n*bs]
};

// ---------------------------------------------------------------- Connect4 PUCT search
// (c4_puct.hip; SURVEY §8 a21 on the target game).  One 192-byte record per node, slot k of
// the node's move list (CPython set order) at index k of every per-slot array.
struct C4PNode {
    uint64_t s0, s1;      // stones of 'X' / 'O'
    uint32_t order;       // packed 3-bit move-list columns | #moves << 24 (d_order of the legal mask)
    uint8_t turn;         // side to move
    uint8_t nmoves;       // moves searched from here: 0 at a terminal position
    uint8_t evaluated;    // the network's priors are in pr[]
    uint8_t won;          // the last mover has four (check_win)
    uint16_t parent;
    uint8_t pact, depth;
    uint32_t pad0;
    uint16_t child[8];    // 0xFFFF = none
    int32_t na[8];        // N (virtual losses included while a flush is pending)
    float pr[8];          // P
    double w[8];          // W (fp64)
    uint8_t pad1[16];
};

struct C4PuctParams {
    int first_game, n_games, sims, bs, M, max_batch, flush;
    double c;                 // c_puct
    C4PNode *nodes;           // [G][M]
    int32_t *ctl;             // [G][kCtlWords]
    uint32_t *paths;          // [G][max_batch][kMaxDepth] edge into level l: node | slot << 16
    uint32_t *meta;           // [G][max_batch] leaf node | depth << 16
    const zc_c4_state *roots;
    zc_c4_state *leaves;
    void *planes;
    int planes_f16;
    int32_t *counts;
    const double *values;
    const void *logits;       // backup: [n*bs][7] column logits
    int logits_f16;
    int leaf_rows;            // backup: rows of values / logits per game (0: bs; 1: a roots-only flush)
    float dir_alpha, dir_eps;
    uint64_t seed;
    int32_t *search_no;       // [n] per-game search number (counter word; end adds 1), or null
    float temperature;
    int32_t *out_move;        // column
    int32_t *out_na;          // [n][7] visits per column
    float *out_prior;         // [n][7] root priors per column (optional)
    zc_game_stats *out_stats;
};
void launch_c4_puct_begin(const C4PuctParams &p, hipStream_t s);
void launch_c4_puct_select(const C4PuctParams &p, hipStream_t s);
void launch_c4_puct_backup(const C4PuctParams &p, hipStream_t s);
void launch_c4_puct_end(const C4PuctParams &p, hipStream_t s);

// ---------------------------------------------------------------- any game backend
// (gen_search.hip; SURVEY §8(b)'s fallback).  The tree of one search; the game states and
// move objects stay with the caller (Python objects of an arbitrary backend).
struct GenNode {
    int32_t base;     // first slot of the node's moves
    int32_t nmoves;   // Node::moves.size()
    int32_t nu;       // Node::untried.size()
    int32_t parent;   // -1 at the root
    int32_t pact;     // parent_action_idx
    int32_t n;        // Node::N
    int32_t depth;
    int32_t pad;
};
enum : int { kGenNodes = 0, kGenSlots = 1, kGenPending = 2, kGenWalked = 3, kGenStatus = 4, kGenExp = 5,
             kGenDepth = 6, kGenCtlWords = 8 };
struct GenArena {
    GenNode *nodes = nullptr;    // [node_cap]
    int32_t *na = nullptr;       // [slot_cap] Na
    double *wa = nullptr;        // [slot_cap] Wa
    double *qa = nullptr;        // [slot_cap] Qa
    int32_t *child = nullptr;    // [slot_cap] child node, -1 = null
    int32_t *untried = nullptr;  // [slot_cap] untried move indices of the slot range's node
    int32_t *ctl = nullptr;      // [kGenCtlWords]
    int32_t *pending = nullptr;  // [max_batch] the pending flush's leaves
    int32_t node_cap = 0;
    int64_t slot_cap = 0;
};
struct GenParams {
    int sims, bs;
    double c;
    const double *logtab;
    GenArena a;
};
void launch_gen_begin(const GenParams &p, int root_moves, hipStream_t s);
void launch_gen_walk(const GenParams &p, int32_t *out, int out_cap, hipStream_t s);
void launch_gen_expand(const GenParams &p, int local, int child_moves, hipStream_t s);
void launch_gen_backup(const GenParams &p, int nb, const double *values, hipStream_t s);
void launch_gen_end(const GenParams &p, int32_t *out, int32_t *root_na, int na_cap, hipStream_t s);

// Chess self-play steps (chess_search.hip): Engine.play_move + _evaluate on the device, the
// move histories of the repetition draw in HBM, the refill of finished games.
struct ChessPlayParams {
    zc_chess_state *roots;        // [n] the positions to move from; updated (post-move or init)
    const zc_chess_state *init;   // the opening
    uint16_t *hist;               // [n][2][cap] each side's moves in play order
    int32_t *hlen;                // [n][2]
    int cap;
    int32_t *err;                 // [3] history overflow | search out of capacity | no move
    const uint16_t *in_moves;     // lockstep step: the searched moves [n]
    const zc_game_stats *search_stats;  // lockstep step (optional): the search's statuses [n]
    zc_chess_state *out_states;   // [moves][n] post-move positions
    uint16_t *out_moves;          // [moves][n]
    int32_t *out_results;         // [moves][n]
    int moves;
    int32_t *ticket;              // pooled: moves drawn while ticket[0] < budget; ticket[1] = most moves
    int32_t budget;
    zc_game_stats *stats;         // self-play launch: per-game sums
};
void launch_chess_play_step(const ChessPlayParams &q, int n, hipStream_t s);
void launch_chess_selfplay(const ChessParams &p, const ChessPlayParams &q, hipStream_t s);
int chess_selfplay_resident_games(int cap, int *out);

void launch_chess_search(const ChessParams &p, hipStream_t s);     // crude_chess_score, whole move
void launch_chess_ext_begin(const ChessParams &p, hipStream_t s);
void launch_chess_ext_select(const ChessParams &p, hipStream_t s);
void launch_chess_ext_backup(const ChessParams &p, hipStream_t s);
void launch_chess_ext_end(const ChessParams &p, hipStream_t s);
constexpr int kRollCap = ZC_CHESS_ROLL_CAP;   // random_rollout on chess: moves per side a rollout's history holds
void launch_chess_rollouts(const ChessParams &p, bool from_tree, hipStream_t s);
void launch_chess_leaf_moves(const ChessParams &p, hipStream_t s);
void launch_chess_hp_walk(const ChessParams &p, hipStream_t s);
void launch_chess_hp_expand(const ChessParams &p, hipStream_t s);

void launch_chess_puct_begin(const ChessParams &p, hipStream_t s);
void launch_chess_puct_select(const ChessParams &p, hipStream_t s);
void launch_chess_puct_backup(const ChessParams &p, hipStream_t s);
void launch_chess_puct_end(const ChessParams &p, hipStream_t s);

void launch_chess_legal(int n, const zc_chess_state *s, uint16_t *moves, int32_t *counts, hipStream_t st);
void launch_chess_probe(int n, const zc_chess_state *s, int32_t *out, hipStream_t st);
void launch_chess_children(int n, const zc_chess_state *s, zc_chess_state *children, uint16_t *moves,
                           int32_t *counts, hipStream_t st);
void launch_chess_play(int n, const zc_chess_state *in, const uint16_t *moves, zc_chess_state *out, hipStream_t st);
void launch_chess_terminal(int n, const zc_chess_state *s, int32_t *flags, hipStream_t st);
void launch_chess_planes(int n, const zc_chess_state *s, void *planes, int f16, hipStream_t st);
bool launch_chess_repetition(int n, int cap, const uint16_t *hist, const int32_t *len, int32_t *out, hipStream_t st);

bool launch_net_conv3x3(int n, int h, int w, int cin, const void *in, const void *wt, const float *bias,
                        const void *res, void *out, int relu, hipStream_t s);
bool launch_net_tower(int n, int h, int w, int cin0, int nconv, const void *in, const void *wall, const float *ball,
                      void *out, const float *fcw, float fcb, double *values, const void *pw, const float *pb,
                      void *pout, hipStream_t s, int pol_channels = 32, int pol_relu = 1);
bool launch_net_conv3x3_packed(int n, int h, int w, int cin, const void *in, const void *wp, const float *bias,
                               const void *res, void *out, int relu, hipStream_t s);
bool launch_net_pack_conv_weight(int cin, const void *w, void *packed, hipStream_t s);
void launch_net_planes_to_nhwc(int n, int cin, int hw, int cpad, const void *planes, void *out, hipStream_t s);
void launch_net_value_head(int n, int hw, const void *act, const float *fcw, float fcb, double *values, hipStream_t s);
bool net_switch(const char *name, int value, int *old);  // zc_debug_net_switch

size_t c4_search_lds_bytes(int bs);
void launch_c4_ext_begin(const ExtParams &p, hipStream_t s);
void launch_c4_ext_select(const ExtParams &p, hipStream_t s);
void launch_c4_ext_backup(const ExtParams &p, hipStream_t s);
void launch_c4_ext_end(const ExtParams &p, hipStream_t s);
void launch_c4_hp_walk(const ExtParams &p, hipStream_t s);
void launch_c4_hp_expand(const ExtParams &p, hipStream_t s);
void launch_c4_search(const SearchParams &p, hipStream_t s);
void launch_c4_walk(const SearchParams &p, int mode, hipStream_t s);   // diagnostic: 1 record, 2 replay
void launch_c4_selfplay(const SearchParams &p, hipStream_t s);
int c4_selfplay_resident_games(int bs, int philox, int *out);  // games the self-play grid keeps resident
void launch_c4_rollout_debug(const Arena &a, int M, int first_game, int n, const zc_c4_state *states,
                             int32_t *out_value, int64_t *out_words, hipStream_t s);
void launch_c4_rollout_seq(const Arena &a, int game, int n, const zc_c4_state *states, int32_t *out_value,
                           int64_t *out_words, hipStream_t s);
void launch_c4_play(int n, zc_c4_state *states, const int32_t *moves, int32_t *results, int reset, hipStream_t s);
enum : int { kTrajPositions = ZC_TRAJ_POSITIONS, kTrajGames = ZC_TRAJ_GAMES, kTrajNext = ZC_TRAJ_NEXT,
             kTrajQuota = ZC_TRAJ_QUOTA, kTrajFinished = ZC_TRAJ_FINISHED, kTrajOverflow = ZC_TRAJ_OVERFLOW };
void launch_traj_record(int n, const zc_traj_buffers &b, void *states, const int16_t *moves, int32_t *results,
                        const int32_t *flags, const int32_t *rep, hipStream_t s);
size_t traj_steps_scratch_bytes(int n, int K);
void launch_traj_record_steps(int n, int K, const zc_traj_buffers &b, const void *states, const int16_t *moves,
                              const int32_t *results, const int32_t *reached, void *scratch, hipStream_t s);
void launch_uct_debug(int n, const double *logn, const int32_t *na, const double *q, double c, double *out,
                      hipStream_t s);

}  // namespace zc

struct zc_engine {
    zc_engine_config cfg{};
    int M = 0;
    hipStream_t stream = nullptr;
    zc::Arena a;
    // zc_c4_search / zc_c4_search_games: the call's inputs and outputs packed in one device
    // block and staged through one pinned host block (one copy each way per call)
    uint8_t *io_d = nullptr, *io_h = nullptr;
    size_t io_h_bytes = 0;
    void *a_block = nullptr;  // the one device allocation `a` and io_d are carved from
    int64_t bytes = 0;
    int stamp = 0;
    uint64_t *tstamps = nullptr;  // zc_debug_c4_launch_stamps: device buffer, 4 words per game
    int rollout_mode = 0;        // ZC_ROLLOUT_EXACT / ZC_ROLLOUT_PHILOX
    uint64_t rollout_seed = 0;
    int carry_lo = 0, carry_hi = 0;  // games that may hold a carried self-play move (engine.hip check_carry)
    zc::ChessArena ca;  // allocated on the first chess search
    // the Connect4 PUCT tree (allocated on the first zc_c4_puct_begin) and its search in progress
    zc::C4PNode *c4p_nodes = nullptr;
    int32_t *c4p_ctl = nullptr;
    uint32_t *c4p_paths = nullptr, *c4p_meta = nullptr;
    int qx_first = 0, qx_n = 0, qx_sims = 0, qx_bs = 0;
    double qx_c = 0;
    float qx_alpha = 0, qx_eps = 0;
    uint64_t qx_seed = 0;
    int32_t *qx_search_no = nullptr;
    bool qx_active = false;
    // the chess PUCT search in progress
    int px_first = 0, px_n = 0, px_sims = 0, px_bs = 0;
    double px_c = 0;
    float px_alpha = 0, px_eps = 0;
    uint64_t px_seed = 0;
    int32_t *px_search_no = nullptr;
    bool px_active = false;
    // the chess stepwise search in progress
    int cx_first = 0, cx_n = 0, cx_sims = 0, cx_bs = 0, cx_policy = 0;
    double cx_c = 0, cx_freedom = 0;
    bool cx_active = false;
    // the any-backend search (zc_gen_*): its tree and the search in progress
    zc::GenArena ga;
    int gx_sims = 0, gx_bs = 0;
    double gx_c = 0;
    bool gx_active = false;
    // the stepwise search in progress (zc_c4_ext_begin .. end)
    int ext_first = 0, ext_n = 0, ext_sims = 0, ext_bs = 0, ext_flushes_done = 0;
    double ext_c = 0;
    bool ext_active = false;
    std::mutex mu;
};
