/* chess_oracle.c — TEST INFRASTRUCTURE ONLY: a plain-C restatement of the reference's chess
 * rules (engine/games/chess/src/chess_backend.cpp), used by tests/ and bench.py's
 * cpu_baseline to check the HIP move generator.  Never linked into the product.
 *
 * Every rule follows the reference, including its departures from standard chess:
 *   - get_legal_moves (:184-360): an insufficient-material early exit (no P/R/Q of either
 *     colour and at most one minor piece -> no moves); pseudo-legal moves in board-scan
 *     order (index 0 = a8, row-major) and, per piece, in the reference's direction order;
 *     the king can never be captured; no castling and no en passant are generated;
 *     each move carries fabs(piece value) of the captured piece (0 otherwise);
 *     legality = the mover's king is not attacked after play_move (:345-359), with the
 *     king searched on the board (-1,-1 when absent, as find_king :70-83).
 *   - play_move (:364-400): fifty counter (uint8, +1, reset on a pawn move or a capture),
 *     castling rights cleared by K moves / R moves FROM column 7 or 0 (any rank), rook hop
 *     for |dc| = 2 king moves, promotion to a queen on the last rank, move history pushed
 *     to the FRONT of the mover's list.
 *   - check_win (:404-412), check_draw (:416-441) with has_repeated_prefix (:148-180).
 *   - state_to_tensor (:461-521), state_from_fen (:525-556).
 * Pinned to the reference by tests/golden/chess_*.json (perft counts, ordered move lists
 * with capture values, terminal flags, tensors, play_move results).
 */
#include "chess_oracle.h"

#include <ctype.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

static const int KN[8][2] = {{-2, -1}, {-2, 1}, {-1, -2}, {-1, 2}, {1, -2}, {1, 2}, {2, -1}, {2, 1}};
static const int DIAG[4][2] = {{-1, -1}, {-1, 1}, {1, -1}, {1, 1}};
static const int ORTH[4][2] = {{-1, 0}, {1, 0}, {0, -1}, {0, 1}};
static const int ALL8[8][2] = {{-1, -1}, {-1, 1}, {1, -1}, {1, 1}, {-1, 0}, {1, 0}, {0, -1}, {0, 1}};

static int inb(int r, int c) { return (unsigned)r < 8 && (unsigned)c < 8; }
static int empty_sq(uint8_t x) { return x == ' ' || x == 0; }
static int is_white(uint8_t x) { return x >= 'A' && x <= 'Z'; }
static int enemy(uint8_t x, int turn) { return !empty_sq(x) && (turn == 0 ? !is_white(x) : is_white(x)); }
static int value_of(uint8_t x) {
    switch (toupper(x)) {
        case 'P': return 1;
        case 'N': return 3;
        case 'B': return 3;
        case 'R': return 5;
        case 'Q': return 9;
        case 'K': return 100;
        default: return 0;
    }
}

static void king_square(const zcc_state *s, int side, int *kr, int *kc) {
    const uint8_t k = side == 0 ? 'K' : 'k';
    for (int i = 0; i < 64; i++)
        if (s->board[i] == k) {
            *kr = i / 8;
            *kc = i % 8;
            return;
        }
    *kr = *kc = -1;
}

/* Is the king of side `t` (= s->turn in the reference) on (kr,kc) attacked? */
static int attacked(const zcc_state *s, int t, int kr, int kc) {
    const uint8_t *b = s->board;
    const int pr = t == 0 ? kr - 1 : kr + 1;
    const uint8_t pawn = t == 0 ? 'p' : 'P';
    for (int dc = -1; dc <= 1; dc += 2)
        if (inb(pr, kc + dc) && b[pr * 8 + kc + dc] == pawn) return 1;
    const uint8_t kn = t ? 'N' : 'n';
    for (int i = 0; i < 8; i++) {
        const int r = kr + KN[i][0], c = kc + KN[i][1];
        if (inb(r, c) && b[r * 8 + c] == kn) return 1;
    }
    const uint8_t q = t ? 'Q' : 'q', rk = t ? 'R' : 'r', bp = t ? 'B' : 'b';
    for (int pass = 0; pass < 2; pass++) {
        const int(*D)[2] = pass == 0 ? ORTH : DIAG;
        const uint8_t p1 = pass == 0 ? rk : bp;
        for (int i = 0; i < 4; i++) {
            int r = kr + D[i][0], c = kc + D[i][1];
            while (inb(r, c)) {
                const uint8_t x = b[r * 8 + c];
                if (!empty_sq(x)) {
                    if (x == p1 || x == q) return 1;
                    break;
                }
                r += D[i][0];
                c += D[i][1];
            }
        }
    }
    const uint8_t kk = t ? 'K' : 'k';
    for (int i = 0; i < 8; i++) {
        const int r = kr + ALL8[i][0], c = kc + ALL8[i][1];
        if (inb(r, c) && b[r * 8 + c] == kk) return 1;
    }
    return 0;
}

static void push(zcc_move *out, int *n, int fr, int fc, int tr, int tc, double v) {
    out[*n].fr = (uint8_t)fr;
    out[*n].fc = (uint8_t)fc;
    out[*n].tr = (uint8_t)tr;
    out[*n].tc = (uint8_t)tc;
    out[*n].value = v;
    (*n)++;
}

static int pseudo_moves(const zcc_state *s, zcc_move *out) {
    const int t = s->turn;
    int heavy = 0, minor = 0;
    for (int i = 0; i < 64; i++) {
        const int u = toupper(s->board[i]);
        if (u == 'P' || u == 'R' || u == 'Q') heavy++;
        if (u == 'B' || u == 'N') minor++;
    }
    if (heavy == 0 && minor <= 1) return 0;
    int n = 0;
    for (int idx = 0; idx < 64; idx++) {
        const uint8_t pc = s->board[idx];
        if (empty_sq(pc)) continue;
        if ((t == 0) != (is_white(pc) != 0)) continue;
        const int r = idx / 8, c = idx % 8, up = toupper(pc);
        if (up == 'P') {
            const int dir = pc == 'P' ? -1 : 1;
            const int nr = r + dir;
            if (inb(nr, c) && empty_sq(s->board[nr * 8 + c])) {
                push(out, &n, r, c, nr, c, 0.0);
                if (r == (pc == 'P' ? 6 : 1) && inb(nr + dir, c) && empty_sq(s->board[(nr + dir) * 8 + c]))
                    push(out, &n, r, c, nr + dir, c, 0.0);
            }
            for (int dc = -1; dc <= 1; dc += 2) {
                const int cc = c + dc;
                if (!inb(nr, cc)) continue;
                const uint8_t x = s->board[nr * 8 + cc];
                if (enemy(x, t) && toupper(x) != 'K') push(out, &n, r, c, nr, cc, fabs((double)value_of(x)));
            }
        } else if (up == 'N' || up == 'K') {
            const int(*D)[2] = up == 'N' ? KN : ALL8;
            for (int i = 0; i < 8; i++) {
                const int rr = r + D[i][0], cc = c + D[i][1];
                if (!inb(rr, cc)) continue;
                const uint8_t x = s->board[rr * 8 + cc];
                if (empty_sq(x)) push(out, &n, r, c, rr, cc, 0.0);
                else if (enemy(x, t) && toupper(x) != 'K') push(out, &n, r, c, rr, cc, fabs((double)value_of(x)));
            }
        } else if (up == 'B' || up == 'R' || up == 'Q') {
            const int(*D)[2] = up == 'B' ? DIAG : up == 'R' ? ORTH : ALL8;
            const int nd = up == 'Q' ? 8 : 4;
            for (int i = 0; i < nd; i++) {
                for (int k = 1;; k++) {
                    const int rr = r + D[i][0] * k, cc = c + D[i][1] * k;
                    if (!inb(rr, cc)) break;
                    const uint8_t x = s->board[rr * 8 + cc];
                    if (empty_sq(x)) {
                        push(out, &n, r, c, rr, cc, 0.0);
                        continue;
                    }
                    if (enemy(x, t) && toupper(x) != 'K') push(out, &n, r, c, rr, cc, fabs((double)value_of(x)));
                    break;
                }
            }
        }
    }
    return n;
}

void zcc_play(const zcc_state *s, const zcc_move *m, zcc_state *o) {
    const int turn = s->turn;
    if (o != s) memcpy(o, s, sizeof *o);
    uint8_t *b = o->board;
    o->turn = (uint8_t)(1 - turn);
    o->fifty = (uint8_t)(o->fifty + 1);
    if (turn == 0) {
        if (o->nhw < ZCC_HIST) {
            memmove(&o->hw[1], &o->hw[0], sizeof(zcc_move) * (size_t)o->nhw);
            o->hw[0] = *m;
            o->nhw++;
        } else {
            o->overflow = 1;
        }
    } else {
        if (o->nhb < ZCC_HIST) {
            memmove(&o->hb[1], &o->hb[0], sizeof(zcc_move) * (size_t)o->nhb);
            o->hb[0] = *m;
            o->nhb++;
        } else {
            o->overflow = 1;
        }
    }
    const int fr = m->fr, fc = m->fc, tr = m->tr, tc = m->tc;
    const uint8_t pc = b[fr * 8 + fc], trg = b[tr * 8 + tc];
    if (pc == 'P' || pc == 'p' || !empty_sq(trg)) o->fifty = 0;
    if (pc == 'K' || (pc == 'R' && fc == 7)) o->castle &= (uint8_t)~1u;
    if (pc == 'K' || (pc == 'R' && fc == 0)) o->castle &= (uint8_t)~2u;
    if (pc == 'k' || (pc == 'r' && fc == 7)) o->castle &= (uint8_t)~4u;
    if (pc == 'k' || (pc == 'r' && fc == 0)) o->castle &= (uint8_t)~8u;
    if (pc == 'K' && tc - fc == 2) { b[61] = 'R'; b[63] = ' '; }
    if (pc == 'k' && tc - fc == 2) { b[5] = 'r'; b[7] = ' '; }
    if (pc == 'K' && tc - fc == -2) { b[59] = 'R'; b[56] = ' '; }
    if (pc == 'k' && tc - fc == -2) { b[3] = 'r'; b[0] = ' '; }
    b[tr * 8 + tc] = pc;
    b[fr * 8 + fc] = ' ';
    if (tr == 0 && pc == 'P') b[tr * 8 + tc] = 'Q';
    if (tr == 7 && pc == 'p') b[tr * 8 + tc] = 'q';
}

int zcc_legal_moves(const zcc_state *s, zcc_move *out) {
    zcc_move ps[ZCC_MAX_MOVES];
    const int np = pseudo_moves(s, ps);
    int n = 0;
    zcc_state t;
    for (int i = 0; i < np; i++) {
        /* only the board matters for the test: skip the history copy */
        memcpy(t.board, s->board, 64);
        t.turn = s->turn;
        t.fifty = s->fifty;
        t.castle = s->castle;
        t.nhw = t.nhb = 0;
        t.overflow = 0;
        zcc_play(&t, &ps[i], &t);
        int kr, kc;
        king_square(&t, s->turn, &kr, &kc);
        if (!attacked(&t, s->turn, kr, kc)) out[n++] = ps[i];
    }
    return n;
}

static int in_check(const zcc_state *s) {
    int kr, kc;
    king_square(s, s->turn, &kr, &kc);
    return attacked(s, s->turn, kr, kc);
}

int zcc_check_win(const zcc_state *s) {
    zcc_move m[ZCC_MAX_MOVES];
    if (zcc_legal_moves(s, m)) return 0;
    return in_check(s);
}

static int move_eq(const zcc_move *a, const zcc_move *b) {
    return a->fr == b->fr && a->fc == b->fc && a->tr == b->tr && a->tc == b->tc && a->value == b->value;
}

/* has_repeated_prefix(L, 2, 3): some prefix of L (most recent move first) is a whole
 * number >= 3 of repeats of a block of >= 2 moves (KMP prefix function). */
int zcc_repeated_prefix(const zcc_move *L, int n) {
    if (n < 6) return 0;
    int *pi = (int *)calloc((size_t)n, sizeof(int));
    int j = 0;
    for (int i = 1; i < n; i++) {
        while (j > 0 && !move_eq(&L[i], &L[j])) j = pi[j - 1];
        if (move_eq(&L[i], &L[j])) ++j;
        pi[i] = j;
    }
    int found = 0;
    for (int i = 0; i < n && !found; i++) {
        const int len = i + 1, p = len - pi[i];
        if (p >= 2 && len % p == 0 && len / p >= 3) found = 1;
    }
    free(pi);
    return found;
}

int zcc_check_draw(const zcc_state *s) {
    zcc_move m[ZCC_MAX_MOVES];
    if (zcc_legal_moves(s, m) == 0 && !in_check(s)) return 1;
    if (s->fifty >= 50) return 1;
    return zcc_repeated_prefix(s->hw, s->nhw) && zcc_repeated_prefix(s->hb, s->nhb);
}

void zcc_init(zcc_state *s) {
    memset(s, 0, sizeof *s);
    const char *back = "rnbqkbnr";
    for (int i = 0; i < 8; i++) {
        s->board[i] = (uint8_t)back[i];
        s->board[8 + i] = 'p';
        s->board[48 + i] = 'P';
        s->board[56 + i] = (uint8_t)toupper(back[i]);
    }
    for (int i = 16; i < 48; i++) s->board[i] = ' ';
    s->castle = 15;
}

int zcc_from_fen(const char *fen, zcc_state *s) {
    memset(s, 0, sizeof *s);
    int idx = 0;
    const char *p = fen;
    while (*p && *p != ' ') {
        if (*p == '/') {
        } else if (isdigit((unsigned char)*p)) {
            for (int i = 0; i < *p - '0' && idx < 64; i++) s->board[idx++] = ' ';
        } else if (idx < 64) {
            s->board[idx++] = (uint8_t)*p;
        }
        p++;
    }
    if (idx != 64) return -1;
    while (*p == ' ') p++;
    s->turn = (p[0] == 'w' && (p[1] == ' ' || p[1] == 0)) ? 0 : 1;
    while (*p && *p != ' ') p++;
    while (*p == ' ') p++;
    while (*p && *p != ' ') {
        if (*p == 'K') s->castle |= 1;
        if (*p == 'Q') s->castle |= 2;
        if (*p == 'k') s->castle |= 4;
        if (*p == 'q') s->castle |= 8;
        p++;
    }
    while (*p == ' ') p++;
    while (*p && *p != ' ') p++; /* en passant: ignored */
    while (*p == ' ') p++;
    s->fifty = (uint8_t)atoi(p);
    return 0;
}

void zcc_state_to_tensor(const zcc_state *s, float *out) {
    static const char pieces[12] = {'P', 'N', 'B', 'R', 'Q', 'K', 'p', 'n', 'b', 'r', 'q', 'k'};
    memset(out, 0, sizeof(float) * 17 * 64);
    for (int i = 0; i < 64; i++)
        for (int k = 0; k < 12; k++)
            if (s->board[i] == (uint8_t)pieces[k]) {
                out[k * 64 + i] = 1.0f;
                break;
            }
    for (int i = 0; i < 64; i++) {
        out[12 * 64 + i] = s->turn == 0 ? 1.0f : 0.0f;
        for (int k = 0; k < 4; k++) out[(13 + k) * 64 + i] = (s->castle >> k) & 1 ? 1.0f : 0.0f;
    }
}

uint64_t zcc_perft(const zcc_state *s, int depth) {
    if (depth == 0) return 1;
    zcc_move m[ZCC_MAX_MOVES];
    const int n = zcc_legal_moves(s, m);
    if (depth == 1) return (uint64_t)n;
    uint64_t total = 0;
    zcc_state t;
    for (int i = 0; i < n; i++) {
        memcpy(t.board, s->board, 64);
        t.turn = s->turn;
        t.fifty = s->fifty;
        t.castle = s->castle;
        t.nhw = t.nhb = 0;
        t.overflow = 0;
        zcc_play(&t, &m[i], &t);
        total += zcc_perft(&t, depth - 1);
    }
    return total;
}

/* ------------------------------------------------------------- chess tree search (mcts.cpp) */
/* mcts.get_move (engine/mcts/src/mcts.cpp:102-160) over the chess rules above, with
 * Policy('random') or Policy('immediate_value') (engine/policy_functions.py:10-20) drawing
 * from the CPython MT19937 stream of c4_oracle.c, and Value('crude_chess_score')
 * (engine/value_functions.py:48-55) or a caller-supplied batch value function. */
#include "c4_oracle.h"

typedef struct {
    zcc_light s;
    int n, nu;
    zcc_move *mv;
    int *untried, *child, *Na;
    double *Wa, *Qa;
    int parent, pact, N;
} cnode;

static void light_to_state(const zcc_light *l, zcc_state *s) {
    memcpy(s->board, l->board, 64);
    s->turn = l->turn;
    s->fifty = l->fifty;
    s->castle = l->castle;
    s->nhw = s->nhb = 0;
    s->overflow = 0;
}

static int cnode_new(cnode *P, int *np, const zcc_light *l, int parent, int pact) {
    cnode *x = &P[*np];
    static __thread zcc_state tmp;
    zcc_move buf[ZCC_MAX_MOVES];
    light_to_state(l, &tmp);
    x->s = *l;
    x->n = zcc_legal_moves(&tmp, buf);
    x->nu = x->n;
    x->mv = (zcc_move *)malloc(sizeof(zcc_move) * (size_t)(x->n ? x->n : 1));
    memcpy(x->mv, buf, sizeof(zcc_move) * (size_t)x->n);
    x->untried = (int *)malloc(sizeof(int) * (size_t)(x->n ? x->n : 1));
    x->child = (int *)malloc(sizeof(int) * (size_t)(x->n ? x->n : 1));
    x->Na = (int *)calloc((size_t)(x->n ? x->n : 1), sizeof(int));
    x->Wa = (double *)calloc((size_t)(x->n ? x->n : 1), sizeof(double));
    x->Qa = (double *)calloc((size_t)(x->n ? x->n : 1), sizeof(double));
    for (int i = 0; i < x->n; i++) {
        x->untried[i] = i;
        x->child[i] = -1;
    }
    x->parent = parent;
    x->pact = pact;
    x->N = 0;
    return (*np)++;
}

double zcc_crude_score(const zcc_light *l) {   /* value_functions.py:48-55 */
    static __thread zcc_state tmp;
    light_to_state(l, &tmp);
    if (zcc_check_win(&tmp)) return 1000.0;
    int sum = 0;
    for (int i = 0; i < 64; i++) {
        switch (l->board[i]) {
            case 'P': sum += 1; break;
            case 'N': case 'B': sum += 3; break;
            case 'R': sum += 5; break;
            case 'Q': sum += 9; break;
            case 'p': sum -= 1; break;
            case 'n': case 'b': sum -= 3; break;
            case 'r': sum -= 5; break;
            case 'q': sum -= 9; break;
            default: break;
        }
    }
    const int factor = l->turn * -2 + 1;
    return (double)(factor * sum);
}

static int cselect(const cnode *P, double c) {   /* mcts.cpp:47-63 */
    int node = 0;
    for (;;) {
        const cnode *x = &P[node];
        if (x->nu > 0) return node;
        int best = -1;
        double bv = -1e100;
        for (int i = 0; i < x->n; i++) {
            if (x->child[i] < 0) continue;
            const double v = x->Na[i] == 0 ? INFINITY
                                           : fma(c, sqrt(log((double)x->N) / (double)x->Na[i]), x->Qa[i]);
            if (v > bv) { bv = v; best = i; }
        }
        if (best == -1) return node;
        node = x->child[best];
    }
}

static int cexpand(cnode *P, int *np, int node, zco_mt *r, int policy, double freedom) {   /* mcts.cpp:65-78 */
    cnode *x = &P[node];
    int local;
    if (policy == 1) {   /* immediate_value: choice among untried moves scoring >= best - freedom */
        double best = -INFINITY;
        for (int i = 0; i < x->nu; i++)
            if (x->mv[x->untried[i]].value > best) best = x->mv[x->untried[i]].value;
        int cand[ZCC_MAX_MOVES], k = 0;
        for (int i = 0; i < x->nu; i++)
            if (x->mv[x->untried[i]].value >= best - freedom) cand[k++] = i;
        local = cand[zco_randbelow(r, (uint32_t)k)];
    } else {
        local = (int)zco_randbelow(r, (uint32_t)x->nu);
    }
    const int move_idx = x->untried[local];
    for (int i = local; i + 1 < x->nu; i++) x->untried[i] = x->untried[i + 1];
    x->nu--;
    zcc_state tmp;
    light_to_state(&x->s, &tmp);
    zcc_play(&tmp, &x->mv[move_idx], &tmp);
    zcc_light l;
    memcpy(l.board, tmp.board, 64);
    l.turn = tmp.turn;
    l.fifty = tmp.fifty;
    l.castle = tmp.castle;
    const int ch = cnode_new(P, np, &l, node, move_idx);
    P[node].child[move_idx] = ch;
    return ch;
}

static void cbackprop(cnode *P, int node, double v) {   /* mcts.cpp:80-100 */
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

static __thread int t_chess_nodes;   /* nodes the calling thread's last zcc_get_move created */

int zcc_get_move(const zcc_light *root, void *rv, int sims, double c, int bs, int policy, double freedom,
                 zcc_value_fn vfn, void *ctx, int *root_na, zcc_move *root_moves, int *n_root) {
    zco_mt *r = (zco_mt *)rv;
    if (bs < 1) bs = 1;
    cnode *P = (cnode *)malloc(sizeof(cnode) * (size_t)(sims + 1));
    int np = 0;
    cnode_new(P, &np, root, -1, -1);
    int *pend = (int *)malloc(sizeof(int) * (size_t)bs);
    double *vals = (double *)malloc(sizeof(double) * (size_t)bs);
    zcc_light *lv = (zcc_light *)malloc(sizeof(zcc_light) * (size_t)bs);
    int npend = 0;
    for (int i = 0; i < sims; i++) {
        const int node = cselect(P, c);
        const int leaf = P[node].nu > 0 ? cexpand(P, &np, node, r, policy, freedom) : node;
        pend[npend++] = leaf;
        if (npend >= bs || i == sims - 1) {
            if (vfn) {
                for (int j = 0; j < npend; j++) lv[j] = P[pend[j]].s;
                vfn(ctx, npend, lv, vals);
            } else {
                for (int j = 0; j < npend; j++) vals[j] = zcc_crude_score(&P[pend[j]].s);
            }
            for (int j = 0; j < npend; j++) cbackprop(P, pend[j], vals[j]);
            npend = 0;
        }
    }
    int best = -1, bestN = -1;
    for (int i = 0; i < P[0].n; i++) {
        const int ch = P[0].child[i];
        if (ch >= 0 && P[ch].N > bestN) { bestN = P[ch].N; best = i; }
    }
    if (n_root) *n_root = P[0].n;
    for (int i = 0; i < P[0].n; i++) {
        if (root_na) root_na[i] = P[0].Na[i];
        if (root_moves) root_moves[i] = P[0].mv[i];
    }
    t_chess_nodes = np;
    for (int i = 0; i < np; i++) {
        free(P[i].mv);
        free(P[i].untried);
        free(P[i].child);
        free(P[i].Na);
        free(P[i].Wa);
        free(P[i].Qa);
    }
    free(lv);
    free(vals);
    free(pend);
    free(P);
    return best;
}

/* Value('random_rollout') (value_functions.py:35-45) with the chess backend, on the CPython
 * MT19937 stream r (a zco_mt*): while not check_win and not check_draw, play
 * random.choice(list(get_legal_moves(state))).  Returns -1 when the side to move at the end
 * (checkmated) is the start's side to move, +1 for the other side's checkmate, 0 for a draw;
 * 2 when a history outgrew ZCC_HIST (the restatement's limit).  *plies = moves played. */
int zcc_rollout(const zcc_state *start, void *rv, int *plies) {
    zco_mt *r = (zco_mt *)rv;
    zcc_state *s = (zcc_state *)malloc(sizeof(zcc_state));
    memcpy(s, start, sizeof *s);
    const int t0 = s->turn;
    zcc_move m[ZCC_MAX_MOVES];
    int q = 0, out;
    for (;;) {
        if (zcc_check_win(s)) {
            out = s->turn == t0 ? -1 : 1;
            break;
        }
        if (zcc_check_draw(s)) {
            out = 0;
            break;
        }
        const int n = zcc_legal_moves(s, m);
        const zcc_move mv = m[zco_randbelow(r, (uint32_t)n)];
        zcc_play(s, &mv, s);
        ++q;
        if (s->overflow) {
            out = 2;
            break;
        }
    }
    if (plies) *plies = q;
    free(s);
    return out;
}

/* Steady-state crude-score self-play from given positions and streams (bench.py's chess CPU
 * baseline on the GPU pool's snapshot; the caller of get_move is Engine.play_mcts +
 * scripts/train.py:151-170): per game, `moves` times: get_move (crude_chess_score, the
 * policy), play the best root move, and refill from the initial position when the game is
 * over (no legal move — check_win or stalemate — or check_draw: fifty moves, repetition over
 * the histories played since the snapshot).  out_expansions[g] = nodes created (the root
 * excluded), as the GPU counts them.  One pthread per slice of games. */
#include <pthread.h>

typedef struct {
    int lo, hi, moves, sims, bs, policy;
    double c, freedom;
    const zcc_light *roots;
    zco_mt *mts;
    uint64_t *out;
} csp_job;

static void *csp_worker(void *arg) {
    csp_job *J = (csp_job *)arg;
    zcc_state *s = (zcc_state *)malloc(sizeof(zcc_state));
    zcc_move mv[ZCC_MAX_MOVES];
    for (int g = J->lo; g < J->hi; g++) {
        light_to_state(&J->roots[g], s);
        uint64_t exp = 0;
        for (int k = 0; k < J->moves; k++) {
            zcc_light l;
            memcpy(l.board, s->board, 64);
            l.turn = s->turn;
            l.fifty = s->fifty;
            l.castle = s->castle;
            int n = 0;
            const int best = zcc_get_move(&l, &J->mts[g], J->sims, J->c, J->bs, J->policy, J->freedom, NULL, NULL,
                                          NULL, mv, &n);
            exp += (uint64_t)(t_chess_nodes - 1);
            if (best >= 0) zcc_play(s, &mv[best], s);
            if (best < 0 || s->overflow || zcc_legal_moves(s, mv) == 0 || zcc_check_draw(s)) zcc_init(s);
        }
        J->out[g] = exp;
    }
    free(s);
    return NULL;
}

int zcc_selfplay_batch(int n, const zcc_light *roots, void *mtv, int moves, int sims, double c, int bs, int policy,
                       double freedom, int n_threads, uint64_t *out_expansions) {
    zco_mt *mts = (zco_mt *)mtv;
    if (n_threads < 1) n_threads = 1;
    if (n_threads > n) n_threads = n > 0 ? n : 1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)n_threads);
    csp_job *J = (csp_job *)malloc(sizeof(csp_job) * (size_t)n_threads);
    for (int q = 0; q < n_threads; q++) {
        J[q] = (csp_job){(int)((long)n * q / n_threads), (int)((long)n * (q + 1) / n_threads), moves, sims, bs,
                         policy, c, freedom, roots, mts, out_expansions};
        pthread_create(&th[q], NULL, csp_worker, &J[q]);
    }
    for (int q = 0; q < n_threads; q++) pthread_join(th[q], NULL);
    free(J);
    free(th);
    return 0;
}
