/* oracle/c4_oracle.c — TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline "port").
 *
 * A plain-C restatement of the reference's Connect4 search path, written for clarity and
 * independence from the GPU implementation (char boards, pointer-free node pool, no
 * bitboards).  Every function cites the reference line it restates.  Parity is pinned by
 * tests/test_oracle.py against tests/golden/ JSON fixtures, which the reference itself produced.
 *
 * Third-party arithmetic the reference relies on, restated here:
 *   - CPython 3.10 Modules/_randommodule.c: init_genrand / init_by_array / genrand_uint32,
 *     random.getrandbits(k<=32) = genrand_uint32() >> (32-k), Lib/random.py
 *     _randbelow_with_getrandbits and choice;
 *   - CPython 3.10 Objects/tupleobject.c tuplehash (xxHash-style) and Objects/setobject.c
 *     set_add_entry / set_table_resize / set_insert_clean, which fix the iteration order
 *     of the set returned by c4_backend.get_legal_moves;
 *   - glibc log(), IEEE div/sqrt, and the fma contraction GCC emits for mcts.cpp:44 under
 *     -O3 -march=native -ffast-math (objdump: vdivsd; vsqrtsd; vfmadd213sd).
 */
#define _GNU_SOURCE
#include "c4_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ CPython MT19937 */
#define MT_N 624
#define MT_M 397

static void mt_init_genrand(zco_mt *r, uint32_t s) {
    r->mt[0] = s;
    for (int i = 1; i < MT_N; i++)
        r->mt[i] = 1812433253u * (r->mt[i - 1] ^ (r->mt[i - 1] >> 30)) + (uint32_t)i;
    r->index = MT_N;
}

static void mt_init_by_array(zco_mt *r, const uint32_t *key, int len) {
    mt_init_genrand(r, 19650218u);
    int i = 1, j = 0;
    for (int k = (MT_N > len ? MT_N : len); k; k--) {
        r->mt[i] = (r->mt[i] ^ ((r->mt[i - 1] ^ (r->mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
        i++; j++;
        if (i >= MT_N) { r->mt[0] = r->mt[MT_N - 1]; i = 1; }
        if (j >= len) j = 0;
    }
    for (int k = MT_N - 1; k; k--) {
        r->mt[i] = (r->mt[i] ^ ((r->mt[i - 1] ^ (r->mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
        i++;
        if (i >= MT_N) { r->mt[0] = r->mt[MT_N - 1]; i = 1; }
    }
    r->mt[0] = 0x80000000u;
    r->index = MT_N;
    r->drawn = 0;
}

void zco_mt_seed(zco_mt *r, uint64_t seed) {
    /* random_seed(): key = abs(n) as little-endian 32-bit words, at least one word. */
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    mt_init_by_array(r, key, key[1] ? 2 : 1);
}

uint32_t zco_mt_u32(zco_mt *r) {
    static const uint32_t mag01[2] = {0u, 0x9908b0dfu};
    uint32_t y;
    if (r->index >= MT_N) {
        int kk;
        for (kk = 0; kk < MT_N - MT_M; kk++) {
            y = (r->mt[kk] & 0x80000000u) | (r->mt[kk + 1] & 0x7fffffffu);
            r->mt[kk] = r->mt[kk + MT_M] ^ (y >> 1) ^ mag01[y & 1u];
        }
        for (; kk < MT_N - 1; kk++) {
            y = (r->mt[kk] & 0x80000000u) | (r->mt[kk + 1] & 0x7fffffffu);
            r->mt[kk] = r->mt[kk + (MT_M - MT_N)] ^ (y >> 1) ^ mag01[y & 1u];
        }
        y = (r->mt[MT_N - 1] & 0x80000000u) | (r->mt[0] & 0x7fffffffu);
        r->mt[MT_N - 1] = r->mt[MT_M - 1] ^ (y >> 1) ^ mag01[y & 1u];
        r->index = 0;
    }
    y = r->mt[r->index++];
    r->drawn++;
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

uint32_t zco_randbelow(zco_mt *r, uint32_t n) {
    /* Lib/random.py _randbelow_with_getrandbits: k = n.bit_length(); reject r >= n. */
    if (n == 0) return 0;
    int k = 32 - __builtin_clz(n);
    uint32_t v = zco_mt_u32(r) >> (32 - k);
    while (v >= n) v = zco_mt_u32(r) >> (32 - k);
    return v;
}

/* -------------------------------------------------- CPython set order of {(i,0)} */
static uint64_t tuple2_hash(uint64_t a, uint64_t b) {
    const uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull,
                   P5 = 2870177450012600261ull;
    uint64_t acc = P5, lanes[2] = {a, b};
    for (int i = 0; i < 2; i++) {
        acc += lanes[i] * P2;
        acc = (acc << 31) | (acc >> 33);
        acc *= P1;
    }
    acc += 2 ^ (P5 ^ 3527539ull);
    if (acc == (uint64_t)-1) return 1546275796ull;
    return acc;
}

typedef struct { int key; uint64_t hash; int used; } sslot;

static void set_insert_clean(sslot *t, uint64_t mask, int key, uint64_t hash) {
    uint64_t perturb = hash, i = hash & mask;
    for (;;) {
        if (!t[i].used) goto put;
        if (i + 9 <= mask) {
            for (int j = 0; j < 9; j++) {
                i++;
                if (!t[i].used) goto put;
            }
        }
        perturb >>= 5;
        i = (i * 5 + 1 + perturb) & mask;
    }
put:
    t[i].used = 1; t[i].key = key; t[i].hash = hash;
}

int zco_set_order(int mask, int *out) {
    sslot tab[64];
    memset(tab, 0, sizeof tab);
    uint64_t tmask = 7;
    int fill = 0;
    for (int col = 0; col < 7; col++) {
        if (!((mask >> col) & 1)) continue;
        uint64_t h = tuple2_hash((uint64_t)col, 0);
        /* set_add_entry: elements are distinct, so this is a probe for the first free slot. */
        set_insert_clean(tab, tmask, col, h);
        fill++;
        if ((uint64_t)fill * 5 >= tmask * 3) {           /* set_table_resize(used*4) */
            uint64_t newsize = 8;
            while (newsize <= (uint64_t)fill * 4) newsize <<= 1;
            sslot old[64];
            memcpy(old, tab, sizeof tab);
            memset(tab, 0, sizeof tab);
            for (uint64_t s = 0; s <= tmask; s++)
                if (old[s].used) set_insert_clean(tab, newsize - 1, old[s].key, old[s].hash);
            tmask = newsize - 1;
        }
    }
    int n = 0;
    for (uint64_t s = 0; s <= tmask; s++)
        if (tab[s].used) out[n++] = tab[s].key;
    return n;
}

static int g_order[128][7], g_order_n[128];
static pthread_once_t g_order_once = PTHREAD_ONCE_INIT;
static void order_init(void) {
    for (int m = 0; m < 128; m++) g_order_n[m] = zco_set_order(m, g_order[m]);
}

/* ----------------------------------------------------------- c4_backend restatement */
#define AT(b, r, c) ((b)[(r) * 7 + (c)])
static const char TOK[2] = {'X', 'O'};

int zco_check_win(const char *b, int turn) {            /* c4_backend.py:25-44 */
    const char t = TOK[1 - turn];
    for (int r = 0; r < 6; r++)
        for (int c = 0; c < 4; c++)
            if (AT(b, r, c) == t && AT(b, r, c + 1) == t && AT(b, r, c + 2) == t && AT(b, r, c + 3) == t) return 1;
    for (int c = 0; c < 7; c++)
        for (int r = 0; r < 3; r++)
            if (AT(b, r, c) == t && AT(b, r + 1, c) == t && AT(b, r + 2, c) == t && AT(b, r + 3, c) == t) return 1;
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 4; c++)
            if (AT(b, r, c) == t && AT(b, r + 1, c + 1) == t && AT(b, r + 2, c + 2) == t && AT(b, r + 3, c + 3) == t) return 1;
    for (int r = 3; r < 6; r++)
        for (int c = 0; c < 4; c++)
            if (AT(b, r, c) == t && AT(b, r - 1, c + 1) == t && AT(b, r - 2, c + 2) == t && AT(b, r - 3, c + 3) == t) return 1;
    return 0;
}

int zco_check_draw(const char *b) {                      /* c4_backend.py:46-47 */
    for (int i = 0; i < 42; i++)
        if (b[i] == '.') return 0;
    return 1;
}

static int legal_mask(const char *b) {                  /* c4_backend.py:49-50 */
    int m = 0;
    for (int c = 0; c < 7; c++)
        if (AT(b, 0, c) == '.') m |= 1 << c;
    return m;
}

static void play(char *b, int *turn, int col) {         /* c4_backend.py:14-23 */
    for (int r = 5; r >= 0; r--)
        if (AT(b, r, col) == '.') { AT(b, r, col) = TOK[*turn]; break; }
    *turn = 1 - *turn;
}

int zco_rollout(const char *board, int turn, zco_mt *r) {   /* value_functions.py:35-45 */
    pthread_once(&g_order_once, order_init);
    char b[42];
    memcpy(b, board, 42);
    const int initial_turn = turn;
    while (!zco_check_win(b, turn) && !zco_check_draw(b)) {
        const int m = legal_mask(b);
        const int col = g_order[m][zco_randbelow(r, (uint32_t)g_order_n[m])];   /* random.choice(list(set)) */
        play(b, &turn, col);
    }
    if (zco_check_win(b, turn)) return turn == initial_turn ? -1 : 1;   /* loser = state.turn */
    return 0;
}

/* ------------------------------------------------------------ UCT search restatement */
typedef struct {
    char b[42];
    int turn;
    int n;                 /* number of moves                         mcts.cpp:27-28 */
    int mv[7];             /* columns, set order                      mcts.cpp:26    */
    int untried[7], nu;    /* indices into mv, in order               mcts.cpp:33    */
    int child[7];          /* node ids, -1 = null                     mcts.cpp:32    */
    int Na[7];
    double Wa[7], Qa[7];
    int parent, pact, N;
} onode;

static int new_node(onode *P, int *np, const char *b, int turn, int parent, int pact) {
    onode *x = &P[*np];
    memcpy(x->b, b, 42);
    x->turn = turn;
    const int m = legal_mask(b);
    x->n = g_order_n[m];
    for (int i = 0; i < x->n; i++) {
        x->mv[i] = g_order[m][i];
        x->untried[i] = i;
        x->child[i] = -1;
        x->Na[i] = 0;
        x->Wa[i] = 0.0;
        x->Qa[i] = 0.0;
    }
    x->nu = x->n;
    x->parent = parent;
    x->pact = pact;
    x->N = 0;
    return (*np)++;
}

static double uct(const onode *x, int a, double c) {   /* mcts.cpp:41-45 */
    if (x->Na[a] == 0) return INFINITY;
    return fma(c, sqrt(log((double)x->N) / (double)x->Na[a]), x->Qa[a]);
}

static int select_leaf(const onode *P, double c) {     /* mcts.cpp:47-63 */
    int node = 0;
    for (;;) {
        const onode *x = &P[node];
        if (x->nu > 0) return node;
        int best = -1;
        double bv = -1e100;
        for (int i = 0; i < x->n; i++) {
            if (x->child[i] < 0) continue;
            const double v = uct(x, i, c);
            if (v > bv) { bv = v; best = i; }
        }
        if (best == -1) return node;
        node = x->child[best];
    }
}

static int expand(onode *P, int *np, int node, zco_mt *r) {   /* mcts.cpp:65-78 */
    onode *x = &P[node];
    const int local = (int)zco_randbelow(r, (uint32_t)x->nu);  /* Policy.random: random.choice */
    const int move_idx = x->untried[local];
    for (int i = local; i + 1 < x->nu; i++) x->untried[i] = x->untried[i + 1];
    x->nu--;
    char b[42];
    memcpy(b, x->b, 42);
    int t = x->turn;
    play(b, &t, x->mv[move_idx]);
    const int child = new_node(P, np, b, t, node, move_idx);
    P[node].child[move_idx] = child;
    return child;
}

static void backprop(onode *P, int node, double v) {   /* mcts.cpp:80-100 */
    for (;;) {
        P[node].N += 1;
        const int p = P[node].parent;
        if (p < 0) break;
        const int a = P[node].pact;
        P[p].Na[a] += 1;
        P[p].Wa[a] -= v;
        P[p].Qa[a] = P[p].Wa[a] / (double)P[p].Na[a];
        node = p;
        v = -v;
    }
}

/* mcts.cpp:102-160.  vfn == NULL: Value('random_rollout') on the same stream; otherwise
 * vfn(ctx, n, boards, turns, out) is Value.batch over the flush's pending leaves. */
/* per thread: nodes of the last search (expansions = nodes - 1) */
static __thread int t_last_nodes;

static int get_move_impl(const char *board, int turn, zco_mt *r, int sims, double c, int bs,
                         int *root_na, int *order, int *n_moves, zco_value_fn vfn, void *ctx) {
    pthread_once(&g_order_once, order_init);
    if (bs < 1) bs = 1;
    onode *P = (onode *)malloc(sizeof(onode) * (size_t)(sims > 0 ? sims + 1 : 1));
    int np = 0;
    new_node(P, &np, board, turn, -1, -1);
    if (n_moves) *n_moves = P[0].n;
    int *pend = (int *)malloc(sizeof(int) * (size_t)bs);
    double *vals = (double *)malloc(sizeof(double) * (size_t)bs);
    char *lb = vfn ? (char *)malloc(42 * (size_t)bs) : NULL;
    int *lt = vfn ? (int *)malloc(sizeof(int) * (size_t)bs) : NULL;
    int npend = 0;
    for (int i = 0; i < sims; i++) {
        int node = select_leaf(P, c);
        int leaf = P[node].nu > 0 ? expand(P, &np, node, r) : node;
        pend[npend++] = leaf;
        if (npend >= bs || i == sims - 1) {            /* flush :112-127, final flush :149 */
            if (vfn) {
                for (int j = 0; j < npend; j++) {
                    memcpy(lb + 42 * (size_t)j, P[pend[j]].b, 42);
                    lt[j] = P[pend[j]].turn;
                }
                vfn(ctx, npend, lb, lt, vals);
            } else {
                for (int j = 0; j < npend; j++) vals[j] = zco_rollout(P[pend[j]].b, P[pend[j]].turn, r);
            }
            for (int j = 0; j < npend; j++) backprop(P, pend[j], vals[j]);
            npend = 0;
        }
    }
    int best = -1, bestN = -1;                         /* :150-155 first max of child N */
    for (int i = 0; i < P[0].n; i++) {
        const int ch = P[0].child[i];
        if (ch >= 0 && P[ch].N > bestN) { bestN = P[ch].N; best = i; }
    }
    for (int i = 0; i < P[0].n; i++) {
        if (root_na) root_na[i] = P[0].Na[i];
        if (order) order[i] = P[0].mv[i];
    }
    const int col = best >= 0 ? P[0].mv[best] : -1;
    t_last_nodes = np;
    free(lt);
    free(lb);
    free(vals);
    free(pend);
    free(P);
    return col;
}

int zco_get_move(const char *board, int turn, zco_mt *r, int sims, double c, int bs,
                 int *root_na, int *order, int *n_moves) {
    return get_move_impl(board, turn, r, sims, c, bs, root_na, order, n_moves, NULL, NULL);
}

int zco_get_move_valued(const char *board, int turn, zco_mt *r, int sims, double c, int bs,
                        int *root_na, int *order, int *n_moves, zco_value_fn vfn, void *ctx) {
    return get_move_impl(board, turn, r, sims, c, bs, root_na, order, n_moves, vfn, ctx);
}

/* ------------------------------------------------------------- threaded CPU baseline */
typedef struct {
    int lo, hi;
    const char *boards;
    const int *turns;
    const uint64_t *seeds;
    int sims, bs;
    double c;
    int *out_move, *out_na;
    uint64_t *out_consumed;
} job;

static void *worker(void *arg) {
    job *J = (job *)arg;
    for (int g = J->lo; g < J->hi; g++) {
        zco_mt r;
        zco_mt_seed(&r, J->seeds[g]);
        int na[7] = {0}, ord[7] = {0}, n = 0;
        J->out_move[g] = zco_get_move(J->boards + 42 * (size_t)g, J->turns[g], &r, J->sims, J->c, J->bs, na, ord, &n);
        if (J->out_na) {
            for (int k = 0; k < 7; k++) J->out_na[7 * (size_t)g + k] = 0;
            for (int k = 0; k < n; k++) J->out_na[7 * (size_t)g + ord[k]] = na[k];
        }
        if (J->out_consumed) J->out_consumed[g] = r.drawn;
    }
    return NULL;
}

int zco_get_move_batch(int n, const char *boards, const int *turns, const uint64_t *seeds,
                       int sims, double c, int bs, int n_threads,
                       int *out_move, int *out_root_na, uint64_t *out_consumed) {
    pthread_once(&g_order_once, order_init);
    if (n_threads < 1) n_threads = 1;
    if (n_threads > n) n_threads = n > 0 ? n : 1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)n_threads);
    job *J = (job *)malloc(sizeof(job) * (size_t)n_threads);
    for (int t = 0; t < n_threads; t++) {
        J[t] = (job){(int)((long)n * t / n_threads), (int)((long)n * (t + 1) / n_threads), boards, turns, seeds,
                     sims, bs, c, out_move, out_root_na, out_consumed};
        pthread_create(&th[t], NULL, worker, &J[t]);
    }
    for (int t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
    free(J);
    free(th);
    return 0;
}

/* ---------------------------------------------------- steady-state self-play baseline */
/* The CPU side of bench.py's like-for-like baseline: n games from given positions and
 * MT19937 states (a burned-in GPU pool's snapshot), each playing `moves` consecutive moves —
 * get_move (mcts.cpp:102-160), play_move + _evaluate (engine.py:98-108, 148-153) and the
 * refill of a finished game with the empty board (scripts/train.py:151-170) — spread over
 * n_threads pthreads.  out_expansions[g] = nodes created by game g's searches. */
typedef struct {
    int lo, hi, moves, sims, bs;
    double c;
    const char *boards;
    const int *turns;
    zco_mt *mts;
    uint64_t *out_exp;
} sp_job;

static void *sp_worker(void *arg) {
    sp_job *J = (sp_job *)arg;
    for (int g = J->lo; g < J->hi; g++) {
        char b[43];
        memcpy(b, J->boards + 42 * (size_t)g, 42);
        b[42] = 0;
        int t = J->turns[g];
        uint64_t exp = 0;
        for (int k = 0; k < J->moves; k++) {
            const int col = zco_get_move(b, t, &J->mts[g], J->sims, J->c, J->bs, NULL, NULL, NULL);
            exp += (uint64_t)(t_last_nodes - 1);
            if (col < 0) break;
            play(b, &t, col);
            if (zco_check_win(b, t) || zco_check_draw(b)) {
                memset(b, '.', 42);
                t = 0;
            }
        }
        J->out_exp[g] = exp;
    }
    return NULL;
}

int zco_selfplay_batch(int n, const char *boards, const int *turns, zco_mt *mts, int moves, int sims, double c,
                       int bs, int n_threads, uint64_t *out_expansions) {
    pthread_once(&g_order_once, order_init);
    if (n_threads < 1) n_threads = 1;
    if (n_threads > n) n_threads = n > 0 ? n : 1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)n_threads);
    sp_job *J = (sp_job *)malloc(sizeof(sp_job) * (size_t)n_threads);
    for (int q = 0; q < n_threads; q++) {
        J[q] = (sp_job){(int)((long)n * q / n_threads), (int)((long)n * (q + 1) / n_threads), moves, sims, bs, c,
                        boards, turns, mts, out_expansions};
        pthread_create(&th[q], NULL, sp_worker, &J[q]);
    }
    for (int q = 0; q < n_threads; q++) pthread_join(th[q], NULL);
    free(J);
    free(th);
    return 0;
}
