// engine.hip — host side of the C-ABI (include/zeroclone.h): engine arena in HBM, per-game
// CPython-compatible random streams, argument checking, and the synchronous / stream-
// ordered search entry points.
#include <algorithm>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "c4_order_table.h"
#include "zc_internal.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define ZC_HIP(call)                                                                                   \
    do {                                                                                               \
        hipError_t e_ = (call);                                                                        \
        if (e_ != hipSuccess) return fail(ZC_EHIP, "%s failed: %s", #call, hipGetErrorString(e_));     \
    } while (0)

// CPython 3.10 Modules/_randommodule.c: random.seed(int) -> init_by_array(abs(n) as LE words).
void mt_init_by_array(uint32_t *mt, const uint32_t *key, int len) {
    mt[0] = 19650218u;
    for (int i = 1; i < 624; i++) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
    int i = 1, j = 0;
    for (int k = (624 > len ? 624 : len); k; k--) {
        mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
        i++;
        j++;
        if (i >= 624) { mt[0] = mt[623]; i = 1; }
        if (j >= len) j = 0;
    }
    for (int k = 623; k; k--) {
        mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
        i++;
        if (i >= 624) { mt[0] = mt[623]; i = 1; }
    }
    mt[0] = 0x80000000u;
}

template <class T>
int dalloc(zc_engine *e, T **p, size_t count) {
    const size_t bytes = count * sizeof(T);
    if (hipMalloc((void **)p, bytes ? bytes : 16) != hipSuccess)
        return fail(ZC_ENOMEM, "hipMalloc(%zu bytes) failed", bytes);
    e->bytes += (int64_t)bytes;
    return ZC_OK;
}

void free_chess(zc::ChessArena &c) {
    void *ptrs[] = {c.nodes, c.mv, c.ut, c.ch, c.na, c.w, c.prior, c.ctl, c.paths, c.meta, c.roots, c.xmv, c.xinfo};
    for (void *p : ptrs)
        if (p) (void)hipFree(p);
    c = zc::ChessArena{};
}

void free_gen(zc_engine *e) {
    zc::GenArena &g = e->ga;
    void *ptrs[] = {g.nodes, g.na, g.wa, g.qa, g.child, g.untried, g.ctl, g.pending};
    for (void *p : ptrs)
        if (p) (void)hipFree(p);
    g = zc::GenArena{};
}

// The Connect4 arena and the synchronous calls' IO block are carved from ONE device
// allocation (base == nullptr: the offsets only, for the size), at 256-byte offsets: an
// engine's creation and destruction cost one hipMalloc / hipFree, not sixteen (a hipFree of a
// megabyte-sized block takes ~0.1 ms on this stack).
// search_sync's packed call block per game: inputs (root, game id), outputs (move, the root's
// visits per column, stats)
constexpr size_t kIoIn = sizeof(zc_c4_state) + sizeof(int32_t);
constexpr size_t kIoOut = sizeof(int32_t) * 8 + sizeof(zc_game_stats);
constexpr size_t kIoBytes = kIoIn + kIoOut;

template <class T>
void carve(uint8_t *base, size_t &off, T **p, size_t count) {
    off = (off + 255) & ~(size_t)255;
    *p = base ? (T *)(base + off) : nullptr;
    off += (count ? count : 1) * sizeof(T);
}

size_t carve_arena(zc_engine *e, uint8_t *base) {
    zc::Arena &a = e->a;
    const size_t G = (size_t)e->cfg.max_games, M = (size_t)e->M, B = (size_t)e->cfg.max_batch;
    size_t off = 0;
    carve(base, off, &a.nodes, G * M * zc::kRecBytes);
    carve(base, off, &a.ring, G * zc::kRingWords);
    carve(base, off, &a.rngpos, G * 2);
    carve(base, off, &a.logtab, M + 2);
    carve(base, off, &a.carry, G);
    carve(base, off, &a.progress, 64);
    carve(base, off, &a.phase, G * zc::kPhases);
    carve(base, off, &a.roots, G);
    carve(base, off, &a.move, G);
    carve(base, off, &a.na, G * 7);
    carve(base, off, &a.ids, G);
    carve(base, off, &a.stats, G);
    carve(base, off, &a.ext_ctl, G * zc::kCtlWords);
    carve(base, off, &a.ext_paths, G * B * zc::kMaxDepth);
    carve(base, off, &a.ext_meta, G * B);
    carve(base, off, &a.ext_roots, G);
    carve(base, off, &e->io_d, G * kIoBytes + 16);
    return off;
}

// Streams and pinned host blocks outlive their engines in per-process pools: creating a HIP
// stream costs milliseconds on this stack (a hardware queue), and an engine per game (the
// reference's Engine per game) would pay it every game.
std::mutex g_pool_mu;
std::vector<std::pair<int, hipStream_t>> g_streams;      // (device, idle stream)
std::vector<std::pair<size_t, uint8_t *>> g_pinned;      // (bytes, idle pinned block)

hipStream_t take_stream(int dev) {
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        for (size_t i = 0; i < g_streams.size(); ++i)
            if (g_streams[i].first == dev) {
                hipStream_t s = g_streams[i].second;
                g_streams.erase(g_streams.begin() + (long)i);
                return s;
            }
    }
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return nullptr;
    return s;
}

void give_stream(int dev, hipStream_t s) {  // s is idle (synchronised)
    if (!s) return;
    std::lock_guard<std::mutex> lk(g_pool_mu);
    g_streams.emplace_back(dev, s);
}

// *bytes: the size wanted in, the block's real capacity out (the capacity is what the block
// returns to the pool under).  Best fit: the smallest idle block that is large enough.
uint8_t *take_pinned(size_t *bytes) {
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        long best = -1;
        for (size_t i = 0; i < g_pinned.size(); ++i)
            if (g_pinned[i].first >= *bytes && (best < 0 || g_pinned[i].first < g_pinned[(size_t)best].first))
                best = (long)i;
        if (best >= 0) {
            uint8_t *p = g_pinned[(size_t)best].second;
            *bytes = g_pinned[(size_t)best].first;
            g_pinned.erase(g_pinned.begin() + best);
            return p;
        }
    }
    void *p = nullptr;
    if (hipHostMalloc(&p, *bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
    return (uint8_t *)p;
}

void give_pinned(size_t bytes, uint8_t *p) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(g_pool_mu);
    g_pinned.emplace_back(bytes, p);
}

void free_arena(zc_engine *e) {
    if (e->a_block) (void)hipFree(e->a_block);
    e->a_block = nullptr;
    e->a = zc::Arena{};
    e->io_d = nullptr;
    give_pinned(e->io_h_bytes, e->io_h);
    e->io_h = nullptr;
}

int check_games(const zc_engine *e, int32_t first, int32_t n) {
    if (first < 0 || n < 0 || (int64_t)first + n > e->cfg.max_games)
        return fail(ZC_ECAPACITY, "games [%d, %d) outside engine capacity %d", first, first + n, e->cfg.max_games);
    return ZC_OK;
}

int check_search(const zc_engine *e, int32_t first, int32_t n, int32_t sims, double c, int32_t bs) {
    if (int r = check_games(e, first, n)) return r;
    if (sims < 1) return fail(ZC_EINVAL, "simulations must be >= 1 (got %d)", sims);
    if (bs < 1) return fail(ZC_EINVAL, "batch_size must be >= 1 (got %d)", bs);
    if (sims > e->cfg.max_sims) return fail(ZC_ECAPACITY, "simulations %d > engine max_sims %d", sims, e->cfg.max_sims);
    if (bs > e->cfg.max_batch) return fail(ZC_ECAPACITY, "batch_size %d > engine max_batch %d", bs, e->cfg.max_batch);
    if (!isfinite(c)) return fail(ZC_EINVAL, "c must be finite");
    return ZC_OK;
}

// Games with a self-play move carried over by zc_c4_selfplay_carry_async ([carry_lo, carry_hi),
// conservatively: every game a carry launch covered until a launch that resumes them all).
// Their trees and MT streams belong to the suspended searches: entry points that would search
// or reseed them refuse, so a game's moves stay the moves an uninterrupted run plays.
int check_carry(const zc_engine *e, int32_t first, int32_t n) {
    if (n > 0 && first < e->carry_hi && first + n > e->carry_lo)
        return fail(ZC_EINVAL, "games [%d, %d) overlap games [%d, %d) whose self-play moves are carried over "
                    "(zc_c4_selfplay_carry_async): finish them with zc_c4_selfplay_async / "
                    "zc_c4_selfplay_pooled_async over those games, or drop them with zc_c4_carry_discard",
                    first, first + n, e->carry_lo, e->carry_hi);
    return ZC_OK;
}

void carry_covered(zc_engine *e, int32_t first, int32_t n) {  // a launch that leaves none carried
    if (first <= e->carry_lo && first + n >= e->carry_hi) e->carry_lo = e->carry_hi = 0;
}

bool valid_c4(const zc_c4_state &s) {
    const uint64_t full = 0x0000040810204081ull * 0x3Full;
    if ((s.stones[0] & s.stones[1]) || ((s.stones[0] | s.stones[1]) & ~full) || (s.turn & ~1)) return false;
    const uint64_t occ = s.stones[0] | s.stones[1];
    for (int c = 0; c < 7; ++c) {
        const uint64_t col = (occ >> (7 * c)) & 0x3Full;
        if (col & (col + 1)) return false;
    }
    return true;
}

zc::SearchParams make_params(zc_engine *e, int32_t first, int32_t n, const zc_c4_state *roots, int32_t sims,
                             double c, int32_t bs, int32_t *mv, int32_t *na, zc_game_stats *st) {
    zc::SearchParams p{};
    p.first_game = first;
    p.n_games = n;
    p.sims = sims;
    p.bs = bs;
    p.M = e->M;
    p.c = c;
    p.roots = roots;
    p.out_move = mv;
    p.out_na = na;
    p.out_stats = st;
    p.a = e->a;
    p.max_batch = e->cfg.max_batch;
    p.stamp = e->stamp;
    p.tstamps = e->tstamps;
    p.philox = e->rollout_mode == ZC_ROLLOUT_PHILOX;
    p.philox_seed = e->rollout_seed;
    return p;
}

}  // namespace

// ---------------------------------------------------------------- stepwise search
namespace {
zc::ExtParams ext_params(zc_engine *e, int32_t first, int32_t n) {
    zc::ExtParams p{};
    p.first_game = first;
    p.n_games = n;
    p.sims = e->ext_sims;
    p.bs = e->ext_bs;
    p.M = e->M;
    p.max_batch = e->cfg.max_batch;
    p.c = e->ext_c;
    p.a = e->a;
    return p;
}

int check_ext_range(const zc_engine *e, int32_t first, int32_t n) {
    if (!e->ext_active) return fail(ZC_EINVAL, "no stepwise search in progress (call zc_c4_ext_begin first)");
    if (first < e->ext_first || n < 0 || (int64_t)first + n > (int64_t)e->ext_first + e->ext_n)
        return fail(ZC_EINVAL, "games [%d, %d) outside the stepwise search's range [%d, %d)", first, first + n,
                    e->ext_first, e->ext_first + e->ext_n);
    return ZC_OK;
}

int check_flush(const zc_engine *e, int32_t flush) {
    const int nflush = (e->ext_sims + e->ext_bs - 1) / e->ext_bs;
    if (flush < 0 || flush >= nflush) return fail(ZC_EINVAL, "flush %d outside [0, %d)", flush, nflush);
    return ZC_OK;
}
}  // namespace

extern "C" {

const char *zc_version(void) { return "zeroclone_amd 0.1.0 (gfx950)"; }

const char *zc_last_error(void) { return g_err.c_str(); }

int zc_device_count(int32_t *count) {
    int n = 0;
    ZC_HIP(hipGetDeviceCount(&n));
    *count = n;
    return ZC_OK;
}

int zc_engine_create(const zc_engine_config *cfg, zc_engine **out) {
    if (!cfg || !out) return fail(ZC_EINVAL, "null argument");
    *out = nullptr;
    if (cfg->max_games < 1) return fail(ZC_EINVAL, "max_games must be >= 1");
    if (cfg->max_sims < 1 || cfg->max_sims > 65533) return fail(ZC_EINVAL, "max_sims must be in [1, 65533]");
    if (cfg->max_batch < 1 || cfg->max_batch > 512) return fail(ZC_EINVAL, "max_batch must be in [1, 512]");
    int ndev = 0;
    ZC_HIP(hipGetDeviceCount(&ndev));
    if (cfg->device < 0 || cfg->device >= ndev) return fail(ZC_EINVAL, "device %d not present (%d devices)", cfg->device, ndev);
    ZC_HIP(hipSetDevice(cfg->device));

    zc_engine *e = new zc_engine();
    e->cfg = *cfg;
    e->M = cfg->max_sims + 1;
    const size_t G = (size_t)cfg->max_games, M = (size_t)e->M;
    zc::Arena &a = e->a;
    int rc = ZC_OK;
    const size_t block = carve_arena(e, nullptr);
    if (hipMalloc(&e->a_block, block) != hipSuccess) {
        e->a_block = nullptr;
        rc = fail(ZC_ENOMEM, "hipMalloc(%zu bytes) failed", block);
    } else {
        e->bytes += (int64_t)block;
        carve_arena(e, (uint8_t *)e->a_block);
    }
    if (!rc) {
        e->io_h_bytes = G * kIoBytes + 16;
        e->io_h = take_pinned(&e->io_h_bytes);
        if (!e->io_h) rc = fail(ZC_ENOMEM, "hipHostMalloc(%zu bytes) failed", e->io_h_bytes);
    }
    if (!rc && !(e->stream = take_stream(cfg->device))) rc = fail(ZC_EHIP, "hipStreamCreate failed");
    if (!rc && (hipMemsetAsync(a.phase, 0, G * zc::kPhases * sizeof(int64_t), e->stream) != hipSuccess ||
                hipMemsetAsync(a.ext_ctl, 0, G * zc::kCtlWords * sizeof(int32_t), e->stream) != hipSuccess ||
                hipMemsetAsync(a.carry, 0, G * sizeof(uint4), e->stream) != hipSuccess))
        rc = fail(ZC_EHIP, "memset failed");
    if (!rc) {
        // log(N) exactly as the reference gets it: glibc log on the host (mcts.cpp:44).
        std::vector<double> lg(M + 2);
        for (size_t n = 0; n < M + 2; ++n) lg[n] = log((double)n);
        if (hipMemcpyAsync(a.logtab, lg.data(), lg.size() * sizeof(double), hipMemcpyHostToDevice, e->stream) !=
                hipSuccess ||
            hipStreamSynchronize(e->stream) != hipSuccess)
            rc = fail(ZC_EHIP, "logtab upload failed");
    }
    if (rc) {
        (void)hipDeviceSynchronize();
        free_arena(e);
        give_stream(cfg->device, e->stream);
        delete e;
        return rc;
    }
    *out = e;
    // every game starts as random.seed(game index)
    std::vector<uint64_t> seeds(G);
    for (size_t g = 0; g < G; ++g) seeds[g] = g;
    return zc_rng_seed(e, 0, (int32_t)G, seeds.data());
}

int zc_engine_destroy(zc_engine *eng) {
    if (!eng) return ZC_OK;
    {
        std::lock_guard<std::mutex> lk(eng->mu);
        (void)hipSetDevice(eng->cfg.device);
        (void)hipStreamSynchronize(eng->stream);
        free_arena(eng);
        free_chess(eng->ca);
        free_gen(eng);
        void *c4p[] = {eng->c4p_nodes, eng->c4p_ctl, eng->c4p_paths, eng->c4p_meta};
        for (void *q : c4p)
            if (q) (void)hipFree(q);
        give_stream(eng->cfg.device, eng->stream);
    }
    delete eng;
    return ZC_OK;
}

int zc_engine_footprint(const zc_engine *eng, int64_t *bytes) {
    if (!eng || !bytes) return fail(ZC_EINVAL, "null argument");
    *bytes = eng->bytes;
    return ZC_OK;
}

int zc_rng_seed(zc_engine *eng, int32_t first, int32_t n, const uint64_t *seeds) {
    if (!eng || (!seeds && n)) return fail(ZC_EINVAL, "null argument");
    if (int r = check_games(eng, first, n)) return r;
    if (int r = check_carry(eng, first, n)) return r;
    std::lock_guard<std::mutex> lk(eng->mu);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    std::vector<uint32_t> words((size_t)n * 624);
    std::vector<uint64_t> pos((size_t)n * 2);
    for (int32_t i = 0; i < n; ++i) {
        const uint32_t key[2] = {(uint32_t)seeds[i], (uint32_t)(seeds[i] >> 32)};
        mt_init_by_array(&words[(size_t)i * 624], key, key[1] ? 2 : 1);
        pos[2 * (size_t)i] = 624;   // index 624: the next draw twists (random.seed leaves this)
        pos[2 * (size_t)i + 1] = 624;
    }
    if (n) {
        ZC_HIP(hipMemcpy2DAsync(eng->a.ring + (size_t)first * zc::kRingWords, zc::kRingWords * sizeof(uint32_t),
                                words.data(), 624 * sizeof(uint32_t), 624 * sizeof(uint32_t), (size_t)n,
                                hipMemcpyHostToDevice, eng->stream));
        ZC_HIP(hipMemcpyAsync(eng->a.rngpos + 2 * (size_t)first, pos.data(), pos.size() * sizeof(uint64_t),
                              hipMemcpyHostToDevice, eng->stream));
        ZC_HIP(hipStreamSynchronize(eng->stream));
    }
    return ZC_OK;
}

int zc_rng_set_state(zc_engine *eng, int32_t game, const uint32_t *mt624, int32_t index) {
    if (!eng || !mt624) return fail(ZC_EINVAL, "null argument");
    if (int r = check_games(eng, game, 1)) return r;
    if (int r = check_carry(eng, game, 1)) return r;
    if (index < 0 || index > 624) return fail(ZC_EINVAL, "MT index must be in [0, 624] (got %d)", index);
    std::lock_guard<std::mutex> lk(eng->mu);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    const uint64_t pos[2] = {(uint64_t)index, 624};
    ZC_HIP(hipMemcpyAsync(eng->a.ring + (size_t)game * zc::kRingWords, mt624, 624 * sizeof(uint32_t),
                          hipMemcpyHostToDevice, eng->stream));
    ZC_HIP(hipMemcpyAsync(eng->a.rngpos + 2 * (size_t)game, pos, sizeof pos, hipMemcpyHostToDevice, eng->stream));
    ZC_HIP(hipStreamSynchronize(eng->stream));
    return ZC_OK;
}

int zc_rng_get_state(zc_engine *eng, int32_t game, uint32_t *mt624, int32_t *index) {
    if (!eng || !mt624 || !index) return fail(ZC_EINVAL, "null argument");
    if (int r = check_games(eng, game, 1)) return r;
    std::lock_guard<std::mutex> lk(eng->mu);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    uint64_t pos[2];
    std::vector<uint32_t> ring(zc::kRingWords);
    ZC_HIP(hipMemcpyAsync(pos, eng->a.rngpos + 2 * (size_t)game, sizeof pos, hipMemcpyDeviceToHost, eng->stream));
    ZC_HIP(hipMemcpyAsync(ring.data(), eng->a.ring + (size_t)game * zc::kRingWords, zc::kRingWords * sizeof(uint32_t),
                          hipMemcpyDeviceToHost, eng->stream));
    ZC_HIP(hipStreamSynchronize(eng->stream));
    // Python's state after consuming word `use-1`: the 624-word block holding it, and the
    // offset of the next word inside that block (624 = block exhausted).  CPython twists a
    // whole block at once; the kernels generate words only as far as they read, so the
    // block's words beyond pos[1] (words generated) are completed here by the recurrence.
    const uint64_t use = pos[0];
    const uint64_t blk = use == 0 ? 0 : (use - 1) / 624;
    for (uint64_t p = std::max<uint64_t>(pos[1], 624); p < (blk + 1) * 624; ++p) {
        const uint32_t m = zc::kRingWords - 1;
        const uint32_t a = ring[(p - 624) & m], b = ring[(p - 623) & m], x = ring[(p - 227) & m];
        const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
        ring[p & m] = x ^ (y >> 1) ^ ((b & 1u) ? 0x9908b0dfu : 0u);
    }
    for (int i = 0; i < 624; ++i) mt624[i] = ring[(blk * 624 + (uint64_t)i) & (zc::kRingWords - 1)];
    *index = (int32_t)(use - blk * 624);
    return ZC_OK;
}

int zc_c4_selfplay_async(zc_engine *eng, int32_t first, int32_t n, zc_c4_state *d_roots, int32_t sims, double c,
                         int32_t bs, int32_t moves, zc_c4_state *d_out_states, int16_t *d_out_moves,
                         int32_t *d_out_results, zc_game_stats *d_stats, void *hip_stream) {
    if (!eng || (n && (!d_roots || !d_out_states || !d_out_moves || !d_out_results || !d_stats)))
        return fail(ZC_EINVAL, "null argument");
    if (int r = check_search(eng, first, n, sims, c, bs)) return r;
    if (moves < 1) return fail(ZC_EINVAL, "moves must be >= 1 (got %d)", moves);
    if (!n) return ZC_OK;
    std::lock_guard<std::mutex> lk(eng->mu);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    zc::SearchParams p = make_params(eng, first, n, d_roots, sims, c, bs, nullptr, nullptr, d_stats);
    p.moves = moves;
    p.io_roots = d_roots;
    p.out_states = d_out_states;
    p.out_moves16 = d_out_moves;
    p.out_results = d_out_results;
    // the pace-balancing counter (priorities only: two free runs of one engine in flight on
    // different streams would share it and balance less well, with the same outputs)
    ZC_HIP(hipMemsetAsync(eng->a.progress, 0, sizeof(int32_t), (hipStream_t)hip_stream));
    p.progress = eng->a.progress;
    zc::launch_c4_selfplay(p, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    carry_covered(eng, first, n);   // carried moves resume first and this launch suspends none
    return ZC_OK;
}

namespace {
int c4_pooled(zc_engine *eng, int32_t first, int32_t n, zc_c4_state *d_roots, int32_t sims, double c, int32_t bs,
              int32_t moves_cap, int64_t budget, int32_t *d_ticket, zc_c4_state *d_out_states, int16_t *d_out_moves,
              int32_t *d_out_results, zc_game_stats *d_stats, void *hip_stream, int carry) {
    if (!eng || (n && (!d_roots || !d_out_states || !d_out_moves || !d_out_results || !d_stats || !d_ticket)))
        return fail(ZC_EINVAL, "null argument");
    if (int r = check_search(eng, first, n, sims, c, bs)) return r;
    if (moves_cap < 1) return fail(ZC_EINVAL, "moves_cap must be >= 1 (got %d)", moves_cap);
    if (budget < 0 || budget > (int64_t)moves_cap * n || budget >= ((int64_t)1 << 31))
        return fail(ZC_EINVAL, "budget %lld outside [0, moves_cap x n_games] or >= 2^31", (long long)budget);
    if (!n) return ZC_OK;
    std::lock_guard<std::mutex> lk(eng->mu);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    // A wave takes its tickets only once resident: with more games than the chip holds at
    // once, the first waves could spend the whole budget and the rest never move.  Refused.
    // The check assumes the device runs nothing else: ranks sharing one GPU (bench.py
    // --share-device, a rehearsal mode) or concurrent kernels can still delay some
    // workgroups past the budget, and those games then make no move in that launch (their
    // rows report ZC_SLOT_IDLE; nothing is lost, only the moves' spread over games shifts).
    int resident = 0;
    if (zc::c4_selfplay_resident_games(bs, eng->rollout_mode == ZC_ROLLOUT_PHILOX, &resident))
        return fail(ZC_EHIP, "occupancy query failed");
    if (n > resident)
        return fail(ZC_EINVAL, "pooled self-play of %d games: at most %d (batch %d) are resident at once, and "
                    "the rest would never move; use zc_c4_selfplay_async or fewer games per launch", n, resident, bs);
    hipStream_t s = (hipStream_t)hip_stream;
    ZC_HIP(hipMemsetAsync(d_ticket, 0, 2 * sizeof(int32_t), s));
    zc::SearchParams p = make_params(eng, first, n, d_roots, sims, c, bs, nullptr, nullptr, d_stats);
    p.moves = moves_cap;
    p.io_roots = d_roots;
    p.out_states = d_out_states;
    p.out_moves16 = d_out_moves;
    p.out_results = d_out_results;
    p.ticket = d_ticket;
    p.budget = (int32_t)budget;
    p.carry = carry;
    zc::launch_c4_selfplay(p, s);
    ZC_HIP(hipGetLastError());
    if (!carry) {
        carry_covered(eng, first, n);
    } else if (eng->carry_hi <= eng->carry_lo) {
        eng->carry_lo = first;
        eng->carry_hi = first + n;
    } else {
        eng->carry_lo = std::min(eng->carry_lo, first);
        eng->carry_hi = std::max(eng->carry_hi, first + n);
    }
    return ZC_OK;
}
}  // namespace

int zc_c4_selfplay_pooled_async(zc_engine *eng, int32_t first, int32_t n, zc_c4_state *d_roots, int32_t sims,
                                double c, int32_t bs, int32_t moves_cap, int64_t budget, int32_t *d_ticket,
                                zc_c4_state *d_out_states, int16_t *d_out_moves, int32_t *d_out_results,
                                zc_game_stats *d_stats, void *hip_stream) {
    return c4_pooled(eng, first, n, d_roots, sims, c, bs, moves_cap, budget, d_ticket, d_out_states, d_out_moves,
                     d_out_results, d_stats, hip_stream, 0);
}

int zc_c4_selfplay_carry_async(zc_engine *eng, int32_t first, int32_t n, zc_c4_state *d_roots, int32_t sims,
                               double c, int32_t bs, int32_t moves_cap, int64_t budget, int32_t *d_ticket,
                               zc_c4_state *d_out_states, int16_t *d_out_moves, int32_t *d_out_results,
                               zc_game_stats *d_stats, void *hip_stream) {
    return c4_pooled(eng, first, n, d_roots, sims, c, bs, moves_cap, budget, d_ticket, d_out_states, d_out_moves,
                     d_out_results, d_stats, hip_stream, 1);
}

int zc_c4_carry_discard(zc_engine *eng, int32_t first, int32_t n, void *hip_stream) {
    if (!eng) return fail(ZC_EINVAL, "null argument");
    if (int r = check_games(eng, first, n)) return r;
    if (!n) return ZC_OK;
    std::lock_guard<std::mutex> lk(eng->mu);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    ZC_HIP(hipMemsetAsync(eng->a.carry + first, 0, (size_t)n * sizeof(uint4), (hipStream_t)hip_stream));
    carry_covered(eng, first, n);
    return ZC_OK;
}

int zc_c4_pooled_max_games(zc_engine *eng, int32_t batch_size, int32_t *out) {
    if (!eng || !out) return fail(ZC_EINVAL, "null argument");
    if (batch_size < 1 || batch_size > eng->cfg.max_batch) return fail(ZC_EINVAL, "bad batch_size %d", batch_size);
    std::lock_guard<std::mutex> lk(eng->mu);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    int r = 0;
    if (zc::c4_selfplay_resident_games(batch_size, eng->rollout_mode == ZC_ROLLOUT_PHILOX, &r))
        return fail(ZC_EHIP, "occupancy query failed");
    *out = r;
    return ZC_OK;
}

int zc_c4_search_async(zc_engine *eng, int32_t first, int32_t n, const zc_c4_state *d_roots, int32_t sims, double c,
                       int32_t bs, int32_t *d_move, int32_t *d_na, zc_game_stats *d_stats, void *hip_stream) {
    if (!eng || (n && (!d_roots || !d_move || !d_na || !d_stats))) return fail(ZC_EINVAL, "null argument");
    if (int r = check_search(eng, first, n, sims, c, bs)) return r;
    if (int r = check_carry(eng, first, n)) return r;
    if (!n) return ZC_OK;
    std::lock_guard<std::mutex> lk(eng->mu);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    hipStream_t s = (hipStream_t)hip_stream;
    zc::launch_c4_search(make_params(eng, first, n, d_roots, sims, c, bs, d_move, d_na, d_stats), s);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

namespace {
int search_sync(zc_engine *eng, int32_t first, int32_t n, const int32_t *ids, const zc_c4_state *roots, int32_t sims,
                double c, int32_t bs, int32_t *out_move, int32_t *out_na, zc_game_stats *out_stats) {
    std::lock_guard<std::mutex> lk(eng->mu);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    hipStream_t s = eng->stream;
    // inputs [roots | ids] and outputs [moves | visits (n x 7) | stats] at 16-byte offsets in
    // one block: one host-to-device and one device-to-host copy, both through pinned memory
    const size_t rb = (size_t)n * sizeof(zc_c4_state), ib = ids ? (size_t)n * sizeof(int32_t) : 0;
    const size_t ob = (rb + ib + 15) & ~(size_t)15;
    const size_t outb = (size_t)n * kIoOut;
    uint8_t *const hb = eng->io_h, *const db = eng->io_d;
    memcpy(hb, roots, rb);
    if (ids) memcpy(hb + rb, ids, ib);
    ZC_HIP(hipMemcpyAsync(db, hb, rb + ib, hipMemcpyHostToDevice, s));
    // from here on the pinned block may be in flight: every return drains the stream first, so
    // the next call's memcpy into the block cannot race this call's copies
    struct Drain {
        hipStream_t s;
        ~Drain() { (void)hipStreamSynchronize(s); }
    } drain{s};
    int32_t *const d_move = (int32_t *)(db + ob);
    zc::SearchParams p = make_params(eng, first, n, (const zc_c4_state *)db, sims, c, bs, d_move, d_move + n,
                                     (zc_game_stats *)(db + ob + (size_t)n * 32));
    p.game_ids = ids ? (const int32_t *)(db + rb) : nullptr;
    zc::launch_c4_search(p, s);
    ZC_HIP(hipGetLastError());
    ZC_HIP(hipMemcpyAsync(hb + ob, db + ob, outb, hipMemcpyDeviceToHost, s));
    ZC_HIP(hipStreamSynchronize(s));
    memcpy(out_move, hb + ob, (size_t)n * sizeof(int32_t));
    memcpy(out_na, hb + ob + (size_t)n * 4, (size_t)n * 7 * sizeof(int32_t));
    const zc_game_stats *const st = (const zc_game_stats *)(hb + ob + (size_t)n * 32);
    if (out_stats) memcpy(out_stats, st, (size_t)n * sizeof(zc_game_stats));
    for (int32_t i = 0; i < n; ++i) {
        const int g = ids ? ids[i] : first + i;
        if (st[i].status == ZC_STATUS_NO_MOVES)
            return fail(ZC_EINVAL, "game %d: root has no legal move (reference: undefined behaviour)", g);
        if (st[i].status == ZC_STATUS_INTERNAL)
            return fail(ZC_EDEVICE, "game %d: search invariant violated on the device", g);
        if (st[i].status)
            return fail(ZC_EINVAL, "game %d: invalid Connect4 state (status %lld)", g, (long long)st[i].status);
    }
    return ZC_OK;
}
}  // namespace

int zc_c4_set_rollout_mode(zc_engine *eng, int32_t mode, uint64_t seed) {
    if (!eng) return fail(ZC_EINVAL, "null argument");
    if (mode != ZC_ROLLOUT_EXACT && mode != ZC_ROLLOUT_PHILOX) return fail(ZC_EINVAL, "unknown rollout mode %d", mode);
    std::lock_guard<std::mutex> lk(eng->mu);
    eng->rollout_mode = mode;
    eng->rollout_seed = seed;
    return ZC_OK;
}

int zc_c4_search(zc_engine *eng, int32_t first, int32_t n, const zc_c4_state *roots, int32_t sims, double c,
                 int32_t bs, int32_t *out_move, int32_t *out_na, zc_game_stats *out_stats) {
    if (!eng || (n && (!roots || !out_move || !out_na))) return fail(ZC_EINVAL, "null argument");
    if (int r = check_search(eng, first, n, sims, c, bs)) return r;
    if (int r = check_carry(eng, first, n)) return r;
    if (!n) return ZC_OK;
    return search_sync(eng, first, n, nullptr, roots, sims, c, bs, out_move, out_na, out_stats);
}

int zc_c4_search_games(zc_engine *eng, int32_t n, const int32_t *games, const zc_c4_state *roots, int32_t sims,
                       double c, int32_t bs, int32_t *out_move, int32_t *out_na, zc_game_stats *out_stats) {
    if (!eng || (n && (!games || !roots || !out_move || !out_na))) return fail(ZC_EINVAL, "null argument");
    if (int r = check_search(eng, 0, 0, sims, c, bs)) return r;
    if (n > eng->cfg.max_games) return fail(ZC_ECAPACITY, "%d games > engine capacity %d", n, eng->cfg.max_games);
    std::vector<char> seen((size_t)eng->cfg.max_games, 0);
    for (int32_t i = 0; i < n; ++i) {
        if (games[i] < 0 || games[i] >= eng->cfg.max_games)
            return fail(ZC_ECAPACITY, "game %d outside engine capacity %d", games[i], eng->cfg.max_games);
        if (seen[(size_t)games[i]]++) return fail(ZC_EINVAL, "game %d listed twice", games[i]);
        if (int r = check_carry(eng, games[i], 1)) return r;
    }
    if (!n) return ZC_OK;
    return search_sync(eng, 0, n, games, roots, sims, c, bs, out_move, out_na, out_stats);
}

int zc_c4_play_async(zc_engine *eng, int32_t n, zc_c4_state *d_states, const int32_t *d_moves, int32_t *d_results,
                     int32_t reset, void *hip_stream) {
    if (!eng || n < 0 || (n && (!d_states || !d_moves || !d_results))) return fail(ZC_EINVAL, "bad argument");
    if (!n) return ZC_OK;
    std::lock_guard<std::mutex> lk(eng->mu);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    hipStream_t s = (hipStream_t)hip_stream;
    zc::launch_c4_play(n, d_states, d_moves, d_results, reset, s);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_c4_rollouts(zc_engine *eng, int32_t game, int32_t n, const zc_c4_state *states, int32_t *out_values,
                   int64_t *out_words) {
    if (!eng || n < 0 || (n && (!states || !out_values))) return fail(ZC_EINVAL, "bad argument");
    if (int r = check_games(eng, game, 1)) return r;
    if (int r = check_carry(eng, game, 1)) return r;
    for (int32_t i = 0; i < n; ++i)
        if (!valid_c4(states[i])) return fail(ZC_EINVAL, "state %d is not a valid Connect4 position", i);
    std::lock_guard<std::mutex> lk(eng->mu);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    hipStream_t s = eng->stream;
    zc_c4_state *ds = nullptr;
    int32_t *dv = nullptr;
    int64_t *dw = nullptr;
    ZC_HIP(hipMalloc(&ds, (n ? n : 1) * sizeof(zc_c4_state)));
    ZC_HIP(hipMalloc(&dv, (n ? n : 1) * sizeof(int32_t)));
    ZC_HIP(hipMalloc(&dw, sizeof(int64_t)));
    if (n) ZC_HIP(hipMemcpyAsync(ds, states, (size_t)n * sizeof(zc_c4_state), hipMemcpyHostToDevice, s));
    zc::launch_c4_rollout_seq(eng->a, game, n, ds, dv, dw, s);
    ZC_HIP(hipGetLastError());
    int64_t words = 0;
    if (n) ZC_HIP(hipMemcpyAsync(out_values, dv, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    ZC_HIP(hipMemcpyAsync(&words, dw, sizeof(int64_t), hipMemcpyDeviceToHost, s));
    ZC_HIP(hipStreamSynchronize(s));
    (void)hipFree(ds);
    (void)hipFree(dv);
    (void)hipFree(dw);
    if (out_words) *out_words = words;
    return ZC_OK;
}


int zc_c4_ext_begin(zc_engine *eng, int32_t first, int32_t n, const zc_c4_state *d_roots, int32_t sims, double c,
                    int32_t bs, void *hip_stream) {
    if (!eng || (n && !d_roots)) return fail(ZC_EINVAL, "null argument");
    if (int r = check_search(eng, first, n, sims, c, bs)) return r;
    if (int r = check_carry(eng, first, n)) return r;
    std::lock_guard<std::mutex> lk(eng->mu);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    eng->ext_first = first;
    eng->ext_n = n;
    eng->ext_sims = sims;
    eng->ext_bs = bs;
    eng->ext_c = c;
    eng->ext_active = true;
    if (!n) return ZC_OK;
    zc::ExtParams p = ext_params(eng, first, n);
    p.roots = d_roots;
    zc::launch_c4_ext_begin(p, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_c4_ext_select(zc_engine *eng, int32_t first, int32_t n, int32_t flush, zc_c4_state *d_leaves, void *d_planes,
                     int32_t planes_dtype, int32_t *d_counts, void *hip_stream) {
    if (!eng) return fail(ZC_EINVAL, "null argument");
    if (planes_dtype != ZC_F32 && planes_dtype != ZC_F16) return fail(ZC_EINVAL, "planes_dtype must be ZC_F32 or ZC_F16");
    std::lock_guard<std::mutex> lk(eng->mu);
    if (int r = check_ext_range(eng, first, n)) return r;
    if (int r = check_flush(eng, flush)) return r;
    if (!n) return ZC_OK;
    ZC_HIP(hipSetDevice(eng->cfg.device));
    zc::ExtParams p = ext_params(eng, first, n);
    p.flush = flush;
    p.leaves = d_leaves;
    p.planes = d_planes;
    p.planes_f16 = planes_dtype == ZC_F16;
    p.counts = d_counts;
    zc::launch_c4_ext_select(p, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_c4_ext_backup(zc_engine *eng, int32_t first, int32_t n, int32_t flush, const double *d_values,
                     void *hip_stream) {
    if (!eng || (n && !d_values)) return fail(ZC_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(eng->mu);
    if (int r = check_ext_range(eng, first, n)) return r;
    if (int r = check_flush(eng, flush)) return r;
    if (!n) return ZC_OK;
    ZC_HIP(hipSetDevice(eng->cfg.device));
    zc::ExtParams p = ext_params(eng, first, n);
    p.flush = flush;
    p.values = d_values;
    zc::launch_c4_ext_backup(p, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_c4_ext_end(zc_engine *eng, int32_t first, int32_t n, int32_t *d_move, int32_t *d_na, zc_game_stats *d_stats,
                  void *hip_stream) {
    if (!eng || (n && (!d_move || !d_na || !d_stats))) return fail(ZC_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(eng->mu);
    if (int r = check_ext_range(eng, first, n)) return r;
    if (!n) return ZC_OK;
    ZC_HIP(hipSetDevice(eng->cfg.device));
    zc::ExtParams p = ext_params(eng, first, n);
    p.out_move = d_move;
    p.out_na = d_na;
    p.out_stats = d_stats;
    zc::launch_c4_ext_end(p, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_c4_hp_walk(zc_engine *eng, int32_t game, int32_t flush, int32_t leaf, zc_c4_hp_node *d_node,
                  void *hip_stream) {
    if (!eng || !d_node) return fail(ZC_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(eng->mu);
    if (int r = check_ext_range(eng, game, 1)) return r;
    if (int r = check_flush(eng, flush)) return r;
    const int nb = std::min(eng->ext_bs, eng->ext_sims - flush * eng->ext_bs);
    if (leaf < 0 || leaf >= nb) return fail(ZC_EINVAL, "leaf %d outside flush %d's [0, %d)", leaf, flush, nb);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    zc::ExtParams p = ext_params(eng, game, 1);
    p.flush = flush;
    p.hp_leaf = leaf;
    p.hp_node = d_node;
    zc::launch_c4_hp_walk(p, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_c4_hp_expand(zc_engine *eng, int32_t game, int32_t flush, int32_t leaf, int32_t untried_index,
                    zc_c4_state *d_leaf, void *hip_stream) {
    if (!eng) return fail(ZC_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(eng->mu);
    if (int r = check_ext_range(eng, game, 1)) return r;
    if (int r = check_flush(eng, flush)) return r;
    const int nb = std::min(eng->ext_bs, eng->ext_sims - flush * eng->ext_bs);
    if (leaf < 0 || leaf >= nb) return fail(ZC_EINVAL, "leaf %d outside flush %d's [0, %d)", leaf, flush, nb);
    if (untried_index < -1 || untried_index > 6) return fail(ZC_EINVAL, "untried index %d outside [-1, 7)", untried_index);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    zc::ExtParams p = ext_params(eng, game, 1);
    p.flush = flush;
    p.hp_leaf = leaf;
    p.hp_index = untried_index;
    p.leaves = d_leaf;
    zc::launch_c4_hp_expand(p, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

// ---------------------------------------------------------------- chess rules
#define ZC_CHESS_ENTRY(cond)                                                   \
    if (!eng || n < 0 || (n && !(cond))) return fail(ZC_EINVAL, "bad argument"); \
    if (!n) return ZC_OK;                                                      \
    std::lock_guard<std::mutex> lk(eng->mu);                                   \
    ZC_HIP(hipSetDevice(eng->cfg.device));

int zc_chess_legal_moves_async(zc_engine *eng, int32_t n, const zc_chess_state *d_states, uint16_t *d_moves,
                               int32_t *d_counts, void *hip_stream) {
    ZC_CHESS_ENTRY(d_states && d_moves && d_counts)
    zc::launch_chess_legal(n, d_states, d_moves, d_counts, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_debug_chess_probe_async(zc_engine *eng, int32_t n, const zc_chess_state *d_states, int32_t *d_out,
                               void *hip_stream) {
    ZC_CHESS_ENTRY(d_states && d_out)
    zc::launch_chess_probe(n, d_states, d_out, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_chess_children_async(zc_engine *eng, int32_t n, const zc_chess_state *d_states, zc_chess_state *d_children,
                            uint16_t *d_moves, int32_t *d_counts, void *hip_stream) {
    ZC_CHESS_ENTRY(d_states && d_children && d_counts)
    zc::launch_chess_children(n, d_states, d_children, d_moves, d_counts, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_chess_play_async(zc_engine *eng, int32_t n, const zc_chess_state *d_in, const uint16_t *d_moves,
                        zc_chess_state *d_out, void *hip_stream) {
    ZC_CHESS_ENTRY(d_in && d_moves && d_out)
    zc::launch_chess_play(n, d_in, d_moves, d_out, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_chess_terminal_async(zc_engine *eng, int32_t n, const zc_chess_state *d_states, int32_t *d_flags,
                            void *hip_stream) {
    ZC_CHESS_ENTRY(d_states && d_flags)
    zc::launch_chess_terminal(n, d_states, d_flags, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_chess_repetition_async(int32_t n, int32_t cap, const uint16_t *d_hist, const int32_t *d_len, int32_t *d_out,
                              void *hip_stream) {
    if (n < 0 || (n && (!d_hist || !d_len || !d_out))) return fail(ZC_EINVAL, "bad argument");
    if (!n) return ZC_OK;
    if (!zc::launch_chess_repetition(n, cap, d_hist, d_len, d_out, (hipStream_t)hip_stream))
        return fail(ZC_EINVAL, "history capacity %d outside [1, 4096]", cap);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

namespace {
int check_traj(int32_t n, const zc_traj_buffers *buf, const void *d_states) {
    if (n < 0 || !buf) return fail(ZC_EINVAL, "bad argument");
    const zc_traj_buffers &b = *buf;
    if (b.row_bytes < 8 || (b.row_bytes & 7) || b.max_len < 2 || b.pool_cap < 0 || b.pool_cap > INT32_MAX ||
        b.games_cap < 0)
        return fail(ZC_EINVAL, "bad trajectory buffer shape (row_bytes %d, max_len %d)", b.row_bytes, b.max_len);
    if (!b.d_hist || !b.d_hmoves || !b.d_slot || !b.d_pool || !b.d_labels || !b.d_pool_moves || !b.d_games ||
        !b.d_ctl || !b.d_init)
        return fail(ZC_EINVAL, "null trajectory buffer");
    if (((uintptr_t)b.d_hist | (uintptr_t)b.d_pool | (uintptr_t)b.d_init | (uintptr_t)d_states) & 7)
        return fail(ZC_EINVAL, "rows must be 8-byte aligned");
    return ZC_OK;
}
}  // namespace

int zc_traj_steps_scratch_bytes(int32_t n, int32_t steps, int64_t *bytes) {
    if (n < 0 || steps < 0 || !bytes) return fail(ZC_EINVAL, "bad argument");
    *bytes = (int64_t)zc::traj_steps_scratch_bytes(n, steps);
    return ZC_OK;
}

int zc_traj_record_steps_async(int32_t n, const zc_traj_buffers *buf, void *d_states, const int16_t *d_moves,
                               int32_t *d_results, int32_t steps, const int32_t *d_reached, void *d_scratch,
                               int64_t scratch_bytes, void *hip_stream) {
    if (int r = check_traj(n, buf, d_states)) return r;
    if (steps < 0) return fail(ZC_EINVAL, "steps must be >= 0 (got %d)", steps);
    if ((int64_t)n * steps >= ((int64_t)1 << 31)) return fail(ZC_EINVAL, "n x steps must be < 2^31");
    if (n && steps && (!d_states || !d_moves || !d_results)) return fail(ZC_EINVAL, "bad argument");
    if (!n || !steps) return ZC_OK;
    if (!d_scratch || ((uintptr_t)d_scratch & 15) || scratch_bytes < (int64_t)zc::traj_steps_scratch_bytes(n, steps))
        return fail(ZC_EINVAL, "scratch: %lld bytes at %p, need %zu bytes 16-byte aligned", (long long)scratch_bytes,
                    d_scratch, zc::traj_steps_scratch_bytes(n, steps));
    zc::launch_traj_record_steps(n, steps, *buf, d_states, d_moves, d_results, d_reached, d_scratch,
                                 (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_traj_record_async(int32_t n, const zc_traj_buffers *buf, void *d_states, const int16_t *d_moves,
                         int32_t *d_results, const int32_t *d_flags, const int32_t *d_rep, void *hip_stream) {
    if (n < 0 || !buf) return fail(ZC_EINVAL, "bad argument");
    const zc_traj_buffers &b = *buf;
    if (b.row_bytes < 8 || (b.row_bytes & 7) || b.max_len < 2 || b.pool_cap < 0 || b.pool_cap > INT32_MAX ||
        b.games_cap < 0)
        return fail(ZC_EINVAL, "bad trajectory buffer shape (row_bytes %d, max_len %d)", b.row_bytes, b.max_len);
    if (!b.d_hist || !b.d_hmoves || !b.d_slot || !b.d_pool || !b.d_labels || !b.d_pool_moves || !b.d_games ||
        !b.d_ctl || !b.d_init)
        return fail(ZC_EINVAL, "null trajectory buffer");
    if (((uintptr_t)b.d_hist | (uintptr_t)b.d_pool | (uintptr_t)b.d_init | (uintptr_t)d_states) & 7)
        return fail(ZC_EINVAL, "rows must be 8-byte aligned");
    if (n && (!d_states || !d_moves || !d_results)) return fail(ZC_EINVAL, "bad argument");
    if (!n) return ZC_OK;
    zc::launch_traj_record(n, b, d_states, d_moves, d_results, d_flags, d_rep, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_chess_planes_async(zc_engine *eng, int32_t n, const zc_chess_state *d_states, void *d_planes,
                          int32_t planes_dtype, void *hip_stream) {
    if (planes_dtype != ZC_F32 && planes_dtype != ZC_F16) return fail(ZC_EINVAL, "planes_dtype must be ZC_F32 or ZC_F16");
    ZC_CHESS_ENTRY(d_states && d_planes)
    zc::launch_chess_planes(n, d_states, d_planes, planes_dtype == ZC_F16, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}
#undef ZC_CHESS_ENTRY

// ---------------------------------------------------------------- chess tree search
}  // extern "C"

namespace {
int ensure_chess(zc_engine *e) {
    zc::ChessArena &c = e->ca;
    if (c.nodes) return ZC_OK;
    const size_t G = (size_t)e->cfg.max_games, M = (size_t)e->M;
    const size_t S = M * zc::kChessSlotsPerNode;
    zc::ChessArena n{};
    n.S = (int64_t)S;
    int rc = ZC_OK;
    if (!rc) rc = dalloc(e, &n.nodes, G * M);
    if (!rc) rc = dalloc(e, &n.mv, G * S);
    if (!rc) rc = dalloc(e, &n.ut, G * S);
    if (!rc) rc = dalloc(e, &n.ch, G * S);
    if (!rc) rc = dalloc(e, &n.na, G * S);
    if (!rc) rc = dalloc(e, &n.w, G * S);
    if (!rc) rc = dalloc(e, &n.prior, G * S);
    if (!rc) rc = dalloc(e, &n.ctl, G * zc::kCtlWords);
    if (!rc) rc = dalloc(e, &n.paths, G * (size_t)e->cfg.max_batch * zc::kChessPath);
    if (!rc) rc = dalloc(e, &n.meta, G * (size_t)e->cfg.max_batch);
    if (!rc) rc = dalloc(e, &n.roots, G);
    if (!rc) rc = dalloc(e, &n.xmv, G * (size_t)e->cfg.max_batch * ZC_CHESS_MAX_MOVES);
    if (!rc) rc = dalloc(e, &n.xinfo, G * (size_t)e->cfg.max_batch * 2);
    if (!rc && hipMemset(n.ctl, 0, G * zc::kCtlWords * sizeof(int32_t)) != hipSuccess) rc = fail(ZC_EHIP, "memset failed");
    if (rc) {
        free_chess(n);
        return rc;
    }
    c = n;
    return ZC_OK;
}

zc::ChessParams chess_params(zc_engine *e, int32_t first, int32_t n, int32_t sims, double c, int32_t bs, int32_t policy,
                             double freedom) {
    zc::ChessParams p{};
    p.first_game = first;
    p.n_games = n;
    p.sims = sims;
    p.bs = bs;
    p.M = e->M;
    p.max_batch = e->cfg.max_batch;
    p.c = c;
    p.policy = policy;
    p.freedom = freedom;
    static const double kCapVal[5] = {0.0, 1.0, 3.0, 5.0, 9.0};
    for (int i = 0; i < 5; ++i)
        for (int k = 0; k < 5; ++k)
            if (kCapVal[k] >= kCapVal[i] - freedom) p.cls_ok |= 1u << (5 * i + k);
    p.a = e->a;
    p.ca = e->ca;
    return p;
}

int check_chess(zc_engine *e, int32_t first, int32_t n, int32_t sims, double c, int32_t bs, int32_t policy,
                double freedom) {
    if (int r = check_search(e, first, n, sims, c, bs)) return r;
    if (policy != ZC_POLICY_RANDOM && policy != ZC_POLICY_IMMEDIATE_VALUE)
        return fail(ZC_EINVAL, "policy must be ZC_POLICY_RANDOM or ZC_POLICY_IMMEDIATE_VALUE");
    if (!isfinite(freedom)) return fail(ZC_EINVAL, "policy_freedom must be finite");
    return ZC_OK;
}
}  // namespace

extern "C" {

int zc_chess_reserve(zc_engine *eng) {
    if (!eng) return fail(ZC_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(eng->mu);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    return ensure_chess(eng);
}

int zc_chess_search_async(zc_engine *eng, int32_t first, int32_t n, const zc_chess_state *d_roots, int32_t sims,
                          double c, int32_t bs, int32_t policy, double freedom, uint16_t *d_move, int32_t *d_na,
                          zc_game_stats *d_stats, void *hip_stream) {
    if (!eng || (n && (!d_roots || !d_move || !d_na || !d_stats))) return fail(ZC_EINVAL, "null argument");
    if (int r = check_chess(eng, first, n, sims, c, bs, policy, freedom)) return r;
    if (bs > 256) return fail(ZC_EINVAL, "batch_size %d > 256 (crude-score chess search)", bs);
    if (!n) return ZC_OK;
    std::lock_guard<std::mutex> lk(eng->mu);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    if (int r = ensure_chess(eng)) return r;
    zc::ChessParams p = chess_params(eng, first, n, sims, c, bs, policy, freedom);
    p.roots = d_roots;
    p.out_move = d_move;
    p.out_na = d_na;
    p.out_stats = d_stats;
    zc::launch_chess_search(p, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

}  // extern "C"

namespace {
int check_play_buffers(int32_t n, const zc_chess_play_buffers *b) {
    if (!b) return fail(ZC_EINVAL, "null play buffers");
    if (n && (!b->d_roots || !b->d_init || !b->d_hist || !b->d_hist_len || !b->d_err))
        return fail(ZC_EINVAL, "null play buffer");
    if (b->hist_cap < 1 || b->hist_cap > 4096) return fail(ZC_EINVAL, "hist_cap %d outside [1, 4096]", b->hist_cap);
    return ZC_OK;
}
zc::ChessPlayParams play_params(const zc_chess_play_buffers *b) {
    zc::ChessPlayParams q{};
    q.roots = b->d_roots;
    q.init = b->d_init;
    q.hist = b->d_hist;
    q.hlen = b->d_hist_len;
    q.cap = b->hist_cap;
    q.err = b->d_err;
    return q;
}
int chess_selfplay_common(zc_engine *eng, int32_t first, int32_t n, const zc_chess_play_buffers *b, int32_t sims,
                          double c, int32_t bs, int32_t policy, double freedom, int32_t moves, int64_t budget,
                          int32_t *d_ticket, zc_chess_state *d_out_states, uint16_t *d_out_moves,
                          int32_t *d_out_results, zc_game_stats *d_stats, void *hip_stream) {
    if (!eng || (n && (!d_out_states || !d_out_moves || !d_out_results || !d_stats))) return fail(ZC_EINVAL, "null argument");
    if (int r = check_play_buffers(n, b)) return r;
    if (int r = check_chess(eng, first, n, sims, c, bs, policy, freedom)) return r;
    if (bs > 256) return fail(ZC_EINVAL, "batch_size %d > 256 (crude-score chess search)", bs);
    if (moves < 1) return fail(ZC_EINVAL, "moves must be >= 1 (got %d)", moves);
    if (d_ticket && (budget < 0 || budget > (int64_t)moves * n || budget >= ((int64_t)1 << 31)))
        return fail(ZC_EINVAL, "budget %lld outside [0, moves_cap x n_games] or >= 2^31", (long long)budget);
    if (!n) return ZC_OK;
    std::lock_guard<std::mutex> lk(eng->mu);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    if (int r = ensure_chess(eng)) return r;
    hipStream_t s = (hipStream_t)hip_stream;
    if (d_ticket) {
        int resident = 0;
        if (zc::chess_selfplay_resident_games(b->hist_cap, &resident)) return fail(ZC_EHIP, "occupancy query failed");
        if (n > resident)
            return fail(ZC_EINVAL, "pooled chess self-play of %d games: at most %d are resident at once", n, resident);
        ZC_HIP(hipMemsetAsync(d_ticket, 0, 2 * sizeof(int32_t), s));
    }
    zc::ChessParams p = chess_params(eng, first, n, sims, c, bs, policy, freedom);
    p.roots = b->d_roots;
    zc::ChessPlayParams q = play_params(b);
    q.out_states = d_out_states;
    q.out_moves = d_out_moves;
    q.out_results = d_out_results;
    q.moves = moves;
    q.ticket = d_ticket;
    q.budget = (int32_t)budget;
    q.stats = d_stats;
    zc::launch_chess_selfplay(p, q, s);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}
}  // namespace

extern "C" {

int zc_chess_play_step_async(int32_t n, const zc_chess_play_buffers *b, const uint16_t *d_moves,
                             const zc_game_stats *d_search_stats, zc_chess_state *d_out_states,
                             int32_t *d_out_results, void *hip_stream) {
    if (n < 0 || (n && (!d_moves || !d_out_states || !d_out_results))) return fail(ZC_EINVAL, "bad argument");
    if (int r = check_play_buffers(n, b)) return r;
    if (!n) return ZC_OK;
    zc::ChessPlayParams q = play_params(b);
    q.in_moves = d_moves;
    q.search_stats = d_search_stats;
    q.out_states = d_out_states;
    q.out_results = d_out_results;
    zc::launch_chess_play_step(q, n, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_chess_selfplay_async(zc_engine *eng, int32_t first, int32_t n, const zc_chess_play_buffers *b, int32_t sims,
                            double c, int32_t bs, int32_t policy, double freedom, int32_t moves,
                            zc_chess_state *d_out_states, uint16_t *d_out_moves, int32_t *d_out_results,
                            zc_game_stats *d_stats, void *hip_stream) {
    return chess_selfplay_common(eng, first, n, b, sims, c, bs, policy, freedom, moves, 0, nullptr, d_out_states,
                                 d_out_moves, d_out_results, d_stats, hip_stream);
}

int zc_chess_selfplay_pooled_async(zc_engine *eng, int32_t first, int32_t n, const zc_chess_play_buffers *b,
                                   int32_t sims, double c, int32_t bs, int32_t policy, double freedom,
                                   int32_t moves_cap, int64_t budget, int32_t *d_ticket, zc_chess_state *d_out_states,
                                   uint16_t *d_out_moves, int32_t *d_out_results, zc_game_stats *d_stats,
                                   void *hip_stream) {
    if (n && !d_ticket) return fail(ZC_EINVAL, "null argument");
    return chess_selfplay_common(eng, first, n, b, sims, c, bs, policy, freedom, moves_cap, budget, d_ticket,
                                 d_out_states, d_out_moves, d_out_results, d_stats, hip_stream);
}

int zc_chess_pooled_max_games(int32_t hist_cap, int32_t *out) {
    if (!out || hist_cap < 1 || hist_cap > 4096) return fail(ZC_EINVAL, "bad argument");
    int r = 0;
    if (zc::chess_selfplay_resident_games(hist_cap, &r)) return fail(ZC_EHIP, "occupancy query failed");
    *out = r;
    return ZC_OK;
}

int zc_chess_ext_begin(zc_engine *eng, int32_t first, int32_t n, const zc_chess_state *d_roots, int32_t sims, double c,
                       int32_t bs, int32_t policy, double freedom, void *hip_stream) {
    if (!eng || (n && !d_roots)) return fail(ZC_EINVAL, "null argument");
    if (int r = check_chess(eng, first, n, sims, c, bs, policy, freedom)) return r;
    std::lock_guard<std::mutex> lk(eng->mu);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    if (int r = ensure_chess(eng)) return r;
    eng->cx_first = first;
    eng->cx_n = n;
    eng->cx_sims = sims;
    eng->cx_bs = bs;
    eng->cx_c = c;
    eng->cx_policy = policy;
    eng->cx_freedom = freedom;
    eng->cx_active = true;
    if (!n) return ZC_OK;
    zc::ChessParams p = chess_params(eng, first, n, sims, c, bs, policy, freedom);
    p.roots = d_roots;
    zc::launch_chess_ext_begin(p, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

}  // extern "C"

namespace {
int check_cx(zc_engine *e, int32_t first, int32_t n, int32_t flush, bool need_flush) {
    if (!e->cx_active) return fail(ZC_EINVAL, "no chess stepwise search in progress (call zc_chess_ext_begin first)");
    if (first < e->cx_first || n < 0 || (int64_t)first + n > (int64_t)e->cx_first + e->cx_n)
        return fail(ZC_EINVAL, "games [%d, %d) outside the stepwise search's range", first, first + n);
    const int nflush = (e->cx_sims + e->cx_bs - 1) / e->cx_bs;
    if (need_flush && (flush < 0 || flush >= nflush)) return fail(ZC_EINVAL, "flush %d outside [0, %d)", flush, nflush);
    return ZC_OK;
}
}  // namespace

extern "C" {

int zc_chess_ext_select(zc_engine *eng, int32_t first, int32_t n, int32_t flush, zc_chess_state *d_leaves,
                        void *d_planes, int32_t planes_dtype, int32_t *d_counts, void *hip_stream) {
    if (!eng) return fail(ZC_EINVAL, "null argument");
    if (planes_dtype != ZC_F32 && planes_dtype != ZC_F16) return fail(ZC_EINVAL, "planes_dtype must be ZC_F32 or ZC_F16");
    std::lock_guard<std::mutex> lk(eng->mu);
    if (int r = check_cx(eng, first, n, flush, true)) return r;
    if (!n) return ZC_OK;
    ZC_HIP(hipSetDevice(eng->cfg.device));
    zc::ChessParams p = chess_params(eng, first, n, eng->cx_sims, eng->cx_c, eng->cx_bs, eng->cx_policy, eng->cx_freedom);
    p.flush = flush;
    p.leaves = d_leaves;
    p.planes = d_planes;
    p.planes_f16 = planes_dtype == ZC_F16;
    p.counts = d_counts;
    zc::launch_chess_ext_select(p, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_chess_ext_backup(zc_engine *eng, int32_t first, int32_t n, int32_t flush, const double *d_values,
                        void *hip_stream) {
    if (!eng || (n && !d_values)) return fail(ZC_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(eng->mu);
    if (int r = check_cx(eng, first, n, flush, true)) return r;
    if (!n) return ZC_OK;
    ZC_HIP(hipSetDevice(eng->cfg.device));
    zc::ChessParams p = chess_params(eng, first, n, eng->cx_sims, eng->cx_c, eng->cx_bs, eng->cx_policy, eng->cx_freedom);
    p.flush = flush;
    p.values = d_values;
    zc::launch_chess_ext_backup(p, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_chess_ext_end(zc_engine *eng, int32_t first, int32_t n, uint16_t *d_move, int32_t *d_na, zc_game_stats *d_stats,
                     void *hip_stream) {
    if (!eng || (n && (!d_move || !d_na || !d_stats))) return fail(ZC_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(eng->mu);
    if (int r = check_cx(eng, first, n, 0, false)) return r;
    if (!n) return ZC_OK;
    ZC_HIP(hipSetDevice(eng->cfg.device));
    zc::ChessParams p = chess_params(eng, first, n, eng->cx_sims, eng->cx_c, eng->cx_bs, eng->cx_policy, eng->cx_freedom);
    p.out_move = d_move;
    p.out_na = d_na;
    p.out_stats = d_stats;
    zc::launch_chess_ext_end(p, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_chess_hp_walk(zc_engine *eng, int32_t game, int32_t flush, int32_t leaf, zc_chess_hp_node *d_node,
                     void *hip_stream) {
    if (!eng || !d_node) return fail(ZC_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(eng->mu);
    if (int r = check_cx(eng, game, 1, flush, true)) return r;
    const int nb = std::min(eng->cx_bs, eng->cx_sims - flush * eng->cx_bs);
    if (leaf < 0 || leaf >= nb) return fail(ZC_EINVAL, "leaf %d outside flush %d's [0, %d)", leaf, flush, nb);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    zc::ChessParams p = chess_params(eng, game, 1, eng->cx_sims, eng->cx_c, eng->cx_bs, eng->cx_policy, eng->cx_freedom);
    p.flush = flush;
    p.hp_leaf = leaf;
    p.hp_node = d_node;
    zc::launch_chess_hp_walk(p, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_chess_hp_expand(zc_engine *eng, int32_t game, int32_t flush, int32_t leaf, int32_t untried_index,
                       zc_chess_state *d_leaf, void *hip_stream) {
    if (!eng) return fail(ZC_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(eng->mu);
    if (int r = check_cx(eng, game, 1, flush, true)) return r;
    const int nb = std::min(eng->cx_bs, eng->cx_sims - flush * eng->cx_bs);
    if (leaf < 0 || leaf >= nb) return fail(ZC_EINVAL, "leaf %d outside flush %d's [0, %d)", leaf, flush, nb);
    if (untried_index < -1 || untried_index >= ZC_CHESS_MAX_MOVES)
        return fail(ZC_EINVAL, "untried index %d outside [-1, %d)", untried_index, ZC_CHESS_MAX_MOVES);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    zc::ChessParams p = chess_params(eng, game, 1, eng->cx_sims, eng->cx_c, eng->cx_bs, eng->cx_policy, eng->cx_freedom);
    p.flush = flush;
    p.hp_leaf = leaf;
    p.hp_index = untried_index;
    p.leaves = d_leaf;
    zc::launch_chess_hp_expand(p, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_chess_rollouts_async(zc_engine *eng, int32_t game, int32_t n_states, const zc_chess_state *d_states,
                            const uint16_t *d_hist, const int32_t *d_hist_len, int32_t hist_cap, double *d_values,
                            int32_t *d_status, void *hip_stream) {
    if (!eng || (n_states && (!d_states || !d_hist || !d_hist_len || !d_values))) return fail(ZC_EINVAL, "null argument");
    if (int r = check_games(eng, game, 1)) return r;
    if (n_states < 0 || hist_cap < 1) return fail(ZC_EINVAL, "n_states must be >= 0 and hist_cap >= 1");
    if (!n_states) return ZC_OK;
    std::lock_guard<std::mutex> lk(eng->mu);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    if (int r = ensure_chess(eng)) return r;
    zc::ChessParams p = chess_params(eng, game, 1, 1, 1.0, 1, 0, 0.0);
    p.rstates = d_states;
    p.n_states = n_states;
    p.rhist = d_hist;
    p.rhlen = d_hist_len;
    p.rhcap = hist_cap;
    p.rvalues = d_values;
    p.rstatus = d_status;
    zc::launch_chess_rollouts(p, false, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_chess_ext_rollouts(zc_engine *eng, int32_t first, int32_t n, int32_t flush, const uint16_t *d_hist,
                          const int32_t *d_hist_len, int32_t hist_cap, double *d_values, int32_t *d_status,
                          void *hip_stream) {
    if (!eng || (n && (!d_hist || !d_hist_len || !d_values))) return fail(ZC_EINVAL, "null argument");
    if (hist_cap < 1) return fail(ZC_EINVAL, "hist_cap must be >= 1");
    std::lock_guard<std::mutex> lk(eng->mu);
    if (int r = check_cx(eng, first, n, flush, true)) return r;
    if (!n) return ZC_OK;
    ZC_HIP(hipSetDevice(eng->cfg.device));
    zc::ChessParams p = chess_params(eng, first, n, eng->cx_sims, eng->cx_c, eng->cx_bs, eng->cx_policy, eng->cx_freedom);
    p.flush = flush;
    p.rhist = d_hist;
    p.rhlen = d_hist_len;
    p.rhcap = hist_cap;
    p.rvalues = d_values;
    p.rstatus = d_status;
    zc::launch_chess_rollouts(p, true, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_chess_ext_leaf_moves(zc_engine *eng, int32_t first, int32_t n, int32_t flush, uint16_t *d_moves,
                            int32_t *d_depth, void *hip_stream) {
    if (!eng || (n && (!d_moves || !d_depth))) return fail(ZC_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(eng->mu);
    if (int r = check_cx(eng, first, n, flush, true)) return r;
    if (!n) return ZC_OK;
    ZC_HIP(hipSetDevice(eng->cfg.device));
    zc::ChessParams p = chess_params(eng, first, n, eng->cx_sims, eng->cx_c, eng->cx_bs, eng->cx_policy, eng->cx_freedom);
    p.flush = flush;
    p.path_moves = d_moves;
    p.path_depth = d_depth;
    zc::launch_chess_leaf_moves(p, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

// ---------------------------------------------------------------- chess PUCT search
int zc_chess_puct_flushes(int32_t sims, int32_t bs) {
    if (sims < 2 || bs < 1) return fail(ZC_EINVAL, "PUCT search needs sims >= 2 and batch_size >= 1");
    return 1 + (sims - 1 + bs - 1) / bs;
}

}  // extern "C"

namespace {
zc::ChessParams puct_params(zc_engine *e, int32_t first, int32_t n) {
    zc::ChessParams p = chess_params(e, first, n, e->px_sims, e->px_c, e->px_bs, 0, 0.0);
    p.dir_alpha = e->px_alpha;
    p.dir_eps = e->px_eps;
    p.seed = e->px_seed;
    // d_search_no is indexed by game - first_game of the begin call; a launch over a
    // sub-range [first, first + n) indexes it from its own first game
    p.search_no = e->px_search_no ? e->px_search_no + (first - e->px_first) : nullptr;
    return p;
}
int check_px(zc_engine *e, int32_t first, int32_t n, int32_t flush, bool need_flush) {
    if (!e->px_active) return fail(ZC_EINVAL, "no PUCT search in progress (call zc_chess_puct_begin first)");
    if (first < e->px_first || n < 0 || (int64_t)first + n > (int64_t)e->px_first + e->px_n)
        return fail(ZC_EINVAL, "games [%d, %d) outside the PUCT search's range", first, first + n);
    const int nflush = 1 + (e->px_sims - 1 + e->px_bs - 1) / e->px_bs;
    if (need_flush && (flush < 0 || flush >= nflush)) return fail(ZC_EINVAL, "flush %d outside [0, %d)", flush, nflush);
    return ZC_OK;
}
}  // namespace

extern "C" {

int zc_chess_puct_begin(zc_engine *eng, int32_t first, int32_t n, const zc_chess_state *d_roots, int32_t sims,
                        double c_puct, int32_t bs, float alpha, float eps, uint64_t seed, int32_t *d_search_no,
                        void *hip_stream) {
    if (!eng || (n && !d_roots)) return fail(ZC_EINVAL, "null argument");
    if (int r = check_search(eng, first, n, sims, c_puct, bs)) return r;
    if (sims < 2) return fail(ZC_EINVAL, "PUCT search needs sims >= 2 (flush 0 evaluates the root)");
    if (!(alpha > 0.0f) || !(eps >= 0.0f && eps <= 1.0f)) return fail(ZC_EINVAL, "need alpha > 0 and 0 <= eps <= 1");
    std::lock_guard<std::mutex> lk(eng->mu);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    if (int r = ensure_chess(eng)) return r;
    eng->px_first = first;
    eng->px_n = n;
    eng->px_sims = sims;
    eng->px_bs = bs;
    eng->px_c = c_puct;
    eng->px_alpha = alpha;
    eng->px_eps = eps;
    eng->px_seed = seed;
    eng->px_search_no = d_search_no;
    eng->px_active = true;
    if (!n) return ZC_OK;
    zc::ChessParams p = puct_params(eng, first, n);
    p.roots = d_roots;
    zc::launch_chess_puct_begin(p, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_chess_puct_select(zc_engine *eng, int32_t first, int32_t n, int32_t flush, zc_chess_state *d_leaves,
                         void *d_planes, int32_t planes_dtype, int32_t *d_counts, void *hip_stream) {
    if (!eng) return fail(ZC_EINVAL, "null argument");
    if (planes_dtype != ZC_F32 && planes_dtype != ZC_F16 && planes_dtype != ZC_F16_NHWC32)
        return fail(ZC_EINVAL, "planes_dtype must be ZC_F32, ZC_F16 or ZC_F16_NHWC32");
    std::lock_guard<std::mutex> lk(eng->mu);
    if (int r = check_px(eng, first, n, flush, true)) return r;
    if (!n) return ZC_OK;
    ZC_HIP(hipSetDevice(eng->cfg.device));
    zc::ChessParams p = puct_params(eng, first, n);
    p.flush = flush;
    p.leaves = d_leaves;
    p.planes = d_planes;
    p.planes_f16 = planes_dtype == ZC_F16 ? 1 : planes_dtype == ZC_F16_NHWC32 ? 2 : 0;
    p.counts = d_counts;
    zc::launch_chess_puct_select(p, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_chess_puct_backup_ex(zc_engine *eng, int32_t first, int32_t n, int32_t flush, const double *d_values,
                            const void *d_logits, int32_t logits_dtype, int32_t rows_per_game, void *hip_stream) {
    if (!eng || (n && (!d_values || !d_logits))) return fail(ZC_EINVAL, "null argument");
    if (logits_dtype != ZC_F32 && logits_dtype != ZC_F16) return fail(ZC_EINVAL, "logits_dtype must be ZC_F32 or ZC_F16");
    if (rows_per_game < 0 || (rows_per_game > 0 && flush != 0))
        return fail(ZC_EINVAL, "rows_per_game must be 0 (batch_size rows), or >= 1 for flush 0 (the roots)");
    std::lock_guard<std::mutex> lk(eng->mu);
    if (int r = check_px(eng, first, n, flush, true)) return r;
    if (!n) return ZC_OK;
    ZC_HIP(hipSetDevice(eng->cfg.device));
    zc::ChessParams p = puct_params(eng, first, n);
    p.flush = flush;
    p.values = d_values;
    p.logits = d_logits;
    p.logits_f16 = logits_dtype == ZC_F16;
    p.leaf_rows = rows_per_game;
    zc::launch_chess_puct_backup(p, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_chess_puct_backup(zc_engine *eng, int32_t first, int32_t n, int32_t flush, const double *d_values,
                         const void *d_logits, int32_t logits_dtype, void *hip_stream) {
    return zc_chess_puct_backup_ex(eng, first, n, flush, d_values, d_logits, logits_dtype, 0, hip_stream);
}

int zc_chess_puct_end(zc_engine *eng, int32_t first, int32_t n, float temperature, uint16_t *d_move, int32_t *d_na,
                      float *d_prior, zc_game_stats *d_stats, void *hip_stream) {
    if (!eng || (n && (!d_move || !d_na || !d_stats))) return fail(ZC_EINVAL, "null argument");
    if (!(temperature >= 0.0f)) return fail(ZC_EINVAL, "temperature must be >= 0");
    std::lock_guard<std::mutex> lk(eng->mu);
    if (int r = check_px(eng, first, n, 0, false)) return r;
    if (!n) return ZC_OK;
    ZC_HIP(hipSetDevice(eng->cfg.device));
    zc::ChessParams p = puct_params(eng, first, n);
    p.temperature = temperature;
    p.out_move = d_move;
    p.out_na = d_na;
    p.out_prior = d_prior;
    p.out_stats = d_stats;
    zc::launch_chess_puct_end(p, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- Connect4 PUCT search
namespace {
int ensure_c4p(zc_engine *e) {
    if (e->c4p_nodes) return ZC_OK;
    const size_t G = (size_t)e->cfg.max_games, M = (size_t)e->M;
    int rc = dalloc(e, &e->c4p_nodes, G * M);
    if (!rc) rc = dalloc(e, &e->c4p_ctl, G * zc::kCtlWords);
    if (!rc) rc = dalloc(e, &e->c4p_paths, G * (size_t)e->cfg.max_batch * zc::kMaxDepth);
    if (!rc) rc = dalloc(e, &e->c4p_meta, G * (size_t)e->cfg.max_batch);
    if (!rc && hipMemset(e->c4p_ctl, 0, G * zc::kCtlWords * sizeof(int32_t)) != hipSuccess)
        rc = fail(ZC_EHIP, "memset failed");
    if (rc) {
        void *q[] = {e->c4p_nodes, e->c4p_ctl, e->c4p_paths, e->c4p_meta};
        for (void *x : q)
            if (x) (void)hipFree(x);
        e->c4p_nodes = nullptr;
        e->c4p_ctl = nullptr;
        e->c4p_paths = e->c4p_meta = nullptr;
    }
    return rc;
}
zc::C4PuctParams c4p_params(zc_engine *e, int32_t first, int32_t n) {
    zc::C4PuctParams p{};
    p.first_game = first;
    p.n_games = n;
    p.sims = e->qx_sims;
    p.bs = e->qx_bs;
    p.M = e->M;
    p.max_batch = e->cfg.max_batch;
    p.c = e->qx_c;
    p.nodes = e->c4p_nodes;
    p.ctl = e->c4p_ctl;
    p.paths = e->c4p_paths;
    p.meta = e->c4p_meta;
    p.dir_alpha = e->qx_alpha;
    p.dir_eps = e->qx_eps;
    p.seed = e->qx_seed;
    p.search_no = e->qx_search_no ? e->qx_search_no + (first - e->qx_first) : nullptr;
    return p;
}
int check_qx(zc_engine *e, int32_t first, int32_t n, int32_t flush, bool need_flush) {
    if (!e->qx_active) return fail(ZC_EINVAL, "no Connect4 PUCT search in progress (call zc_c4_puct_begin first)");
    if (first < e->qx_first || n < 0 || (int64_t)first + n > (int64_t)e->qx_first + e->qx_n)
        return fail(ZC_EINVAL, "games [%d, %d) outside the PUCT search's range", first, first + n);
    const int nflush = 1 + (e->qx_sims - 1 + e->qx_bs - 1) / e->qx_bs;
    if (need_flush && (flush < 0 || flush >= nflush)) return fail(ZC_EINVAL, "flush %d outside [0, %d)", flush, nflush);
    return ZC_OK;
}
}  // namespace

extern "C" {

int zc_c4_puct_begin(zc_engine *eng, int32_t first, int32_t n, const zc_c4_state *d_roots, int32_t sims,
                     double c_puct, int32_t bs, float alpha, float eps, uint64_t seed, int32_t *d_search_no,
                     void *hip_stream) {
    if (!eng || (n && !d_roots)) return fail(ZC_EINVAL, "null argument");
    if (int r = check_search(eng, first, n, sims, c_puct, bs)) return r;
    if (sims < 2) return fail(ZC_EINVAL, "PUCT search needs sims >= 2 (flush 0 evaluates the root)");
    if (!(alpha > 0.0f) || !(eps >= 0.0f && eps <= 1.0f)) return fail(ZC_EINVAL, "need alpha > 0 and 0 <= eps <= 1");
    std::lock_guard<std::mutex> lk(eng->mu);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    if (int r = ensure_c4p(eng)) return r;
    eng->qx_first = first;
    eng->qx_n = n;
    eng->qx_sims = sims;
    eng->qx_bs = bs;
    eng->qx_c = c_puct;
    eng->qx_alpha = alpha;
    eng->qx_eps = eps;
    eng->qx_seed = seed;
    eng->qx_search_no = d_search_no;
    eng->qx_active = true;
    if (!n) return ZC_OK;
    zc::C4PuctParams p = c4p_params(eng, first, n);
    p.roots = d_roots;
    zc::launch_c4_puct_begin(p, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_c4_puct_select(zc_engine *eng, int32_t first, int32_t n, int32_t flush, zc_c4_state *d_leaves, void *d_planes,
                      int32_t planes_dtype, int32_t *d_counts, void *hip_stream) {
    if (!eng) return fail(ZC_EINVAL, "null argument");
    if (planes_dtype != ZC_F32 && planes_dtype != ZC_F16) return fail(ZC_EINVAL, "planes_dtype must be ZC_F32 or ZC_F16");
    std::lock_guard<std::mutex> lk(eng->mu);
    if (int r = check_qx(eng, first, n, flush, true)) return r;
    if (!n) return ZC_OK;
    ZC_HIP(hipSetDevice(eng->cfg.device));
    zc::C4PuctParams p = c4p_params(eng, first, n);
    p.flush = flush;
    p.leaves = d_leaves;
    p.planes = d_planes;
    p.planes_f16 = planes_dtype == ZC_F16;
    p.counts = d_counts;
    zc::launch_c4_puct_select(p, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_c4_puct_backup_ex(zc_engine *eng, int32_t first, int32_t n, int32_t flush, const double *d_values,
                         const void *d_logits, int32_t logits_dtype, int32_t rows_per_game, void *hip_stream) {
    if (!eng || (n && (!d_values || !d_logits))) return fail(ZC_EINVAL, "null argument");
    if (logits_dtype != ZC_F32 && logits_dtype != ZC_F16) return fail(ZC_EINVAL, "logits_dtype must be ZC_F32 or ZC_F16");
    if (rows_per_game < 0 || (rows_per_game > 0 && flush != 0))
        return fail(ZC_EINVAL, "rows_per_game must be 0 (batch_size rows), or >= 1 for flush 0 (the roots)");
    std::lock_guard<std::mutex> lk(eng->mu);
    if (int r = check_qx(eng, first, n, flush, true)) return r;
    if (!n) return ZC_OK;
    ZC_HIP(hipSetDevice(eng->cfg.device));
    zc::C4PuctParams p = c4p_params(eng, first, n);
    p.flush = flush;
    p.values = d_values;
    p.logits = d_logits;
    p.logits_f16 = logits_dtype == ZC_F16;
    p.leaf_rows = rows_per_game;
    zc::launch_c4_puct_backup(p, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_c4_puct_backup(zc_engine *eng, int32_t first, int32_t n, int32_t flush, const double *d_values,
                      const void *d_logits, int32_t logits_dtype, void *hip_stream) {
    return zc_c4_puct_backup_ex(eng, first, n, flush, d_values, d_logits, logits_dtype, 0, hip_stream);
}

int zc_c4_puct_end(zc_engine *eng, int32_t first, int32_t n, float temperature, int32_t *d_move, int32_t *d_na,
                   float *d_prior, zc_game_stats *d_stats, void *hip_stream) {
    if (!eng || (n && (!d_move || !d_na || !d_stats))) return fail(ZC_EINVAL, "null argument");
    if (!(temperature >= 0.0f)) return fail(ZC_EINVAL, "temperature must be >= 0");
    std::lock_guard<std::mutex> lk(eng->mu);
    if (int r = check_qx(eng, first, n, 0, false)) return r;
    if (!n) return ZC_OK;
    ZC_HIP(hipSetDevice(eng->cfg.device));
    zc::C4PuctParams p = c4p_params(eng, first, n);
    p.temperature = temperature;
    p.out_move = d_move;
    p.out_na = d_na;
    p.out_prior = d_prior;
    p.out_stats = d_stats;
    zc::launch_c4_puct_end(p, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_debug_c4_puct_tree(zc_engine *eng, int32_t game, int32_t max_nodes, void *out_nodes, int32_t *out_count) {
    if (!eng || !out_nodes || !out_count) return fail(ZC_EINVAL, "null argument");
    if (int r = check_games(eng, game, 1)) return r;
    std::lock_guard<std::mutex> lk(eng->mu);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    if (!eng->c4p_nodes) return fail(ZC_EINVAL, "no Connect4 PUCT tree (no PUCT search has run)");
    ZC_HIP(hipDeviceSynchronize());
    int32_t nn = 0;
    ZC_HIP(hipMemcpy(&nn, eng->c4p_ctl + (size_t)game * zc::kCtlWords, sizeof nn, hipMemcpyDeviceToHost));
    if (nn > max_nodes) return fail(ZC_ECAPACITY, "tree has %d nodes (buffer: %d)", nn, max_nodes);
    ZC_HIP(hipMemcpy(out_nodes, eng->c4p_nodes + (size_t)game * eng->M, (size_t)nn * sizeof(zc::C4PNode),
                     hipMemcpyDeviceToHost));
    *out_count = nn;
    return ZC_OK;
}

int zc_debug_chess_tree(zc_engine *eng, int32_t game, int32_t max_nodes, int32_t max_slots, void *out_nodes,
                        uint16_t *out_mv, float *out_prior, int32_t *out_na, double *out_w, uint16_t *out_child,
                        int32_t *out_counts) {
    if (!eng || !out_nodes || !out_mv || !out_prior || !out_na || !out_w || !out_child || !out_counts)
        return fail(ZC_EINVAL, "null argument");
    if (int r = check_games(eng, game, 1)) return r;
    std::lock_guard<std::mutex> lk(eng->mu);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    const zc::ChessArena &c = eng->ca;
    if (!c.nodes) return fail(ZC_EINVAL, "no chess tree (no chess search has run)");
    ZC_HIP(hipStreamSynchronize(nullptr));
    ZC_HIP(hipDeviceSynchronize());
    int32_t ctl[2];  // per-game control words 0, 1: nodes, slots used
    ZC_HIP(hipMemcpy(ctl, c.ctl + (size_t)game * zc::kCtlWords, sizeof ctl, hipMemcpyDeviceToHost));
    if (ctl[0] > max_nodes || ctl[1] > max_slots)
        return fail(ZC_ECAPACITY, "tree has %d nodes / %d slots (buffers: %d / %d)", ctl[0], ctl[1], max_nodes, max_slots);
    const size_t no = (size_t)game * eng->M, so = (size_t)game * (size_t)c.S;
    ZC_HIP(hipMemcpy(out_nodes, c.nodes + no, (size_t)ctl[0] * sizeof(zc::ChessNode), hipMemcpyDeviceToHost));
    ZC_HIP(hipMemcpy(out_mv, c.mv + so, (size_t)ctl[1] * sizeof(uint16_t), hipMemcpyDeviceToHost));
    ZC_HIP(hipMemcpy(out_prior, c.prior + so, (size_t)ctl[1] * sizeof(float), hipMemcpyDeviceToHost));
    ZC_HIP(hipMemcpy(out_na, c.na + so, (size_t)ctl[1] * sizeof(int32_t), hipMemcpyDeviceToHost));
    ZC_HIP(hipMemcpy(out_w, c.w + so, (size_t)ctl[1] * sizeof(double), hipMemcpyDeviceToHost));
    ZC_HIP(hipMemcpy(out_child, c.ch + so, (size_t)ctl[1] * sizeof(uint16_t), hipMemcpyDeviceToHost));
    out_counts[0] = ctl[0];
    out_counts[1] = ctl[1];
    return ZC_OK;
}

// ---------------------------------------------------------------- value-network layers
int zc_net_conv3x3_async(int32_t n, int32_t h, int32_t w, int32_t cin, const void *d_in, const void *d_weight,
                         const float *d_bias, const void *d_residual, void *d_out, int32_t relu, void *hip_stream) {
    if (n < 0 || (n && (!d_in || !d_weight || !d_bias || !d_out))) return fail(ZC_EINVAL, "bad argument");
    if (!n) return ZC_OK;
    if (!zc::launch_net_conv3x3(n, h, w, cin, d_in, d_weight, d_bias, d_residual, d_out, relu ? 1 : 0,
                                (hipStream_t)hip_stream))
        return fail(ZC_EINVAL, "conv3x3 shape (h %d, w %d, cin %d) not supported", h, w, cin);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_net_conv3x3_pack_async(int32_t cin, const void *d_weight, void *d_packed, void *hip_stream) {
    if (!d_weight || !d_packed || ((uintptr_t)d_weight & 15) || ((uintptr_t)d_packed & 15))
        return fail(ZC_EINVAL, "bad argument");
    if (!zc::launch_net_pack_conv_weight(cin, d_weight, d_packed, (hipStream_t)hip_stream))
        return fail(ZC_EINVAL, "conv3x3 pack: cin %d not supported", cin);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_net_conv3x3_packed_async(int32_t n, int32_t h, int32_t w, int32_t cin, const void *d_in, const void *d_packed,
                                const float *d_bias, const void *d_residual, void *d_out, int32_t relu,
                                void *hip_stream) {
    if (n < 0 || (n && (!d_in || !d_packed || !d_bias || !d_out)) || ((uintptr_t)d_packed & 15))
        return fail(ZC_EINVAL, "bad argument");
    if (!n) return ZC_OK;
    if (!zc::launch_net_conv3x3_packed(n, h, w, cin, d_in, d_packed, d_bias, d_residual, d_out, relu ? 1 : 0,
                                       (hipStream_t)hip_stream))
        return fail(ZC_EINVAL, "conv3x3 shape (h %d, w %d, cin %d) not supported", h, w, cin);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_net_tower_async(int32_t n, int32_t h, int32_t w, int32_t cin0, int32_t nconv, const void *d_in,
                       const void *d_packed, const float *d_bias, void *d_out, const float *d_fc_w, float fc_b,
                       double *d_values, void *hip_stream) {
    if (n < 0 || (n && (!d_in || !d_packed || !d_bias || (!d_out && !d_values) || (d_values && !d_fc_w))) ||
        ((uintptr_t)d_packed & 15) || ((uintptr_t)d_in & 15) || ((uintptr_t)d_out & 15) || ((uintptr_t)d_bias & 15))
        return fail(ZC_EINVAL, "bad argument");
    if (!n) return ZC_OK;
    if (!zc::launch_net_tower(n, h, w, cin0, nconv, d_in, d_packed, d_bias, d_out, d_values ? d_fc_w : nullptr, fc_b,
                              d_values, nullptr, nullptr, nullptr, (hipStream_t)hip_stream))
        return fail(ZC_EINVAL, "tower shape (h %d, w %d, cin0 %d, %d convs) not supported", h, w, cin0, nconv);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_net_tower_policy_async(int32_t n, int32_t h, int32_t w, int32_t cin0, int32_t nconv, const void *d_in,
                              const void *d_packed, const float *d_bias, const float *d_fc_w, float fc_b,
                              double *d_values, const void *d_pw, const float *d_pb, void *d_pout, void *hip_stream) {
    if (n < 0 || (n && (!d_in || !d_packed || !d_bias || !d_fc_w || !d_values || !d_pw || !d_pb || !d_pout)) ||
        ((uintptr_t)d_packed & 15) || ((uintptr_t)d_in & 15) || ((uintptr_t)d_bias & 15) || ((uintptr_t)d_pw & 15) ||
        ((uintptr_t)d_pout & 7))
        return fail(ZC_EINVAL, "bad argument");
    if (!n) return ZC_OK;
    if (!zc::launch_net_tower(n, h, w, cin0, nconv, d_in, d_packed, d_bias, nullptr, d_fc_w, fc_b, d_values, d_pw,
                              d_pb, d_pout, (hipStream_t)hip_stream))
        return fail(ZC_EINVAL, "tower shape (h %d, w %d, cin0 %d, %d convs) not supported", h, w, cin0, nconv);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_net_tower_policy_ex_async(int32_t n, int32_t h, int32_t w, int32_t cin0, int32_t nconv, const void *d_in,
                                 const void *d_packed, const float *d_bias, const float *d_fc_w, float fc_b,
                                 double *d_values, const void *d_pw, const float *d_pb, int32_t policy_channels,
                                 int32_t relu, void *d_pout, void *hip_stream) {
    if (n < 0 || (n && (!d_in || !d_packed || !d_bias || !d_fc_w || !d_values || !d_pw || !d_pb || !d_pout)) ||
        ((uintptr_t)d_packed & 15) || ((uintptr_t)d_in & 15) || ((uintptr_t)d_bias & 15) || ((uintptr_t)d_pw & 15) ||
        ((uintptr_t)d_pb & 15) || ((uintptr_t)d_pout & 7) || (policy_channels != 32 && policy_channels != 64))
        return fail(ZC_EINVAL, "bad argument");
    if (!n) return ZC_OK;
    if (!zc::launch_net_tower(n, h, w, cin0, nconv, d_in, d_packed, d_bias, nullptr, d_fc_w, fc_b, d_values, d_pw,
                              d_pb, d_pout, (hipStream_t)hip_stream, policy_channels, relu))
        return fail(ZC_EINVAL, "tower shape (h %d, w %d, cin0 %d, %d convs) not supported", h, w, cin0, nconv);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_net_planes_to_nhwc_async(int32_t n, int32_t cin, int32_t hw, int32_t cpad, const void *d_planes, void *d_out,
                                void *hip_stream) {
    if (n < 0 || cin < 1 || hw < 1 || cpad < cin || (cpad & 7) || ((uintptr_t)d_out & 15) ||
        (n && (!d_planes || !d_out)))
        return fail(ZC_EINVAL, "bad argument");
    if (!n) return ZC_OK;
    zc::launch_net_planes_to_nhwc(n, cin, hw, cpad, d_planes, d_out, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_net_value_head_async(int32_t n, int32_t hw, const void *d_act, const float *d_fc_w, float fc_b,
                            double *d_values, void *hip_stream) {
    if (n < 0 || hw < 1 || (n && (!d_act || !d_fc_w || !d_values))) return fail(ZC_EINVAL, "bad argument");
    // the head reads whole 256-byte pixel rows (128 fp16 channels) in 16-byte pieces
    if ((uintptr_t)d_act & 15) return fail(ZC_EINVAL, "d_act must be 16-byte aligned (128-channel fp16 NHWC rows)");
    if (!n) return ZC_OK;
    zc::launch_net_value_head(n, hw, d_act, d_fc_w, fc_b, d_values, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_chess_from_fen(const char *fen, zc_chess_state *out) {
    // state_from_fen (chess_backend.cpp:525-556): placement, side, castling; en passant and
    // the full-move number are ignored; the half-move clock becomes the fifty counter.
    if (!fen || !out) return fail(ZC_EINVAL, "null argument");
    zc_chess_state s{};
    const char *p = fen;
    int idx = 0;
    for (; *p && *p != ' '; ++p) {
        if (*p == '/') continue;
        if (*p >= '0' && *p <= '9') {
            for (int i = 0; i < *p - '0'; ++i) {
                if (idx >= 64) return fail(ZC_EINVAL, "FEN placement longer than 64 squares");
                s.board[idx++] = ' ';
            }
        } else {
            if (idx >= 64) return fail(ZC_EINVAL, "FEN placement longer than 64 squares");
            s.board[idx++] = (uint8_t)*p;
        }
    }
    if (idx != 64) return fail(ZC_EINVAL, "FEN placement covers %d squares, not 64", idx);
    while (*p == ' ') ++p;
    s.turn = (p[0] == 'w' && (p[1] == ' ' || p[1] == 0)) ? 0 : 1;
    while (*p && *p != ' ') ++p;
    while (*p == ' ') ++p;
    for (; *p && *p != ' '; ++p) {
        if (*p == 'K') s.castle |= 1;
        if (*p == 'Q') s.castle |= 2;
        if (*p == 'k') s.castle |= 4;
        if (*p == 'q') s.castle |= 8;
    }
    while (*p == ' ') ++p;
    while (*p && *p != ' ') ++p;
    while (*p == ' ') ++p;
    s.fifty = (uint8_t)atoi(p);
    *out = s;
    return ZC_OK;
}

int zc_chess_init(zc_chess_state *out) {
    return zc_chess_from_fen("rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1", out);
}

int zc_c4_from_rows(const char *rows, int32_t turn, zc_c4_state *out) {
    if (!rows || !out) return fail(ZC_EINVAL, "null argument");
    if (turn != 0 && turn != 1) return fail(ZC_EINVAL, "turn must be 0 or 1");
    zc_c4_state s{};
    for (int r = 0; r < 6; ++r)
        for (int c = 0; c < 7; ++c) {
            const char ch = rows[r * 7 + c];
            const uint64_t bit = 1ull << (7 * c + (5 - r));
            if (ch == 'X') s.stones[0] |= bit;
            else if (ch == 'O') s.stones[1] |= bit;
        }
    s.turn = turn;
    *out = s;
    return ZC_OK;
}

int zc_c4_to_rows(const zc_c4_state *s, char *rows) {
    if (!s || !rows) return fail(ZC_EINVAL, "null argument");
    for (int r = 0; r < 6; ++r)
        for (int c = 0; c < 7; ++c) {
            const uint64_t bit = 1ull << (7 * c + (5 - r));
            rows[r * 7 + c] = (s->stones[0] & bit) ? 'X' : (s->stones[1] & bit) ? 'O' : ' ';
        }
    return ZC_OK;
}

int zc_c4_legal_order(int32_t mask, int32_t *cols) {
    if (mask < 0 || mask > 127 || !cols) return fail(ZC_EINVAL, "mask must be in [0, 127]");
    const uint32_t w = ZC_C4_ORDER_INIT[mask];
    const int n = (int)((w >> 24) & 15u);
    for (int k = 0; k < n; ++k) cols[k] = (int32_t)((w >> (3 * k)) & 7u);
    return n;
}

int zc_debug_uct(zc_engine *eng, int32_t n, const double *logn, const int32_t *na, const double *q, double c,
                 double *out) {
    if (!eng || n < 0) return fail(ZC_EINVAL, "bad argument");
    if (!n) return ZC_OK;
    std::lock_guard<std::mutex> lk(eng->mu);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    double *dl, *dq, *dout;
    int32_t *dn;
    ZC_HIP(hipMalloc(&dl, n * sizeof(double)));
    ZC_HIP(hipMalloc(&dq, n * sizeof(double)));
    ZC_HIP(hipMalloc(&dout, n * sizeof(double)));
    ZC_HIP(hipMalloc(&dn, n * sizeof(int32_t)));
    hipStream_t s = eng->stream;
    ZC_HIP(hipMemcpyAsync(dl, logn, n * sizeof(double), hipMemcpyHostToDevice, s));
    ZC_HIP(hipMemcpyAsync(dq, q, n * sizeof(double), hipMemcpyHostToDevice, s));
    ZC_HIP(hipMemcpyAsync(dn, na, n * sizeof(int32_t), hipMemcpyHostToDevice, s));
    zc::launch_uct_debug(n, dl, dn, dq, c, dout, s);
    ZC_HIP(hipGetLastError());
    ZC_HIP(hipMemcpyAsync(out, dout, n * sizeof(double), hipMemcpyDeviceToHost, s));
    ZC_HIP(hipStreamSynchronize(s));
    (void)hipFree(dl);
    (void)hipFree(dq);
    (void)hipFree(dout);
    (void)hipFree(dn);
    return ZC_OK;
}

int zc_debug_c4_rollout(zc_engine *eng, int32_t first, int32_t n, const zc_c4_state *states, int32_t *out_value,
                        int64_t *out_words) {
    if (!eng || (n && (!states || !out_value || !out_words))) return fail(ZC_EINVAL, "null argument");
    if (int r = check_games(eng, first, n)) return r;
    if (int r = check_carry(eng, first, n)) return r;
    for (int32_t i = 0; i < n; ++i)
        if (!valid_c4(states[i])) return fail(ZC_EINVAL, "state %d is not a valid Connect4 position", i);
    if (!n) return ZC_OK;
    std::lock_guard<std::mutex> lk(eng->mu);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    zc::Arena &a = eng->a;
    hipStream_t s = eng->stream;
    int64_t *dw;
    ZC_HIP(hipMalloc(&dw, n * sizeof(int64_t)));
    ZC_HIP(hipMemcpyAsync(a.roots, states, (size_t)n * sizeof(zc_c4_state), hipMemcpyHostToDevice, s));
    zc::launch_c4_rollout_debug(a, eng->M, first, n, a.roots, a.move, dw, s);
    ZC_HIP(hipGetLastError());
    ZC_HIP(hipMemcpyAsync(out_value, a.move, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    ZC_HIP(hipMemcpyAsync(out_words, dw, (size_t)n * sizeof(int64_t), hipMemcpyDeviceToHost, s));
    ZC_HIP(hipStreamSynchronize(s));
    (void)hipFree(dw);
    return ZC_OK;
}

int zc_debug_c4_walk_async(zc_engine *eng, int32_t first, int32_t n, const zc_c4_state *d_roots, int32_t sims,
                           double c, int32_t bs, int32_t mode, int8_t *d_vals, uint32_t *d_words, int32_t *d_move,
                           int32_t *d_na, zc_game_stats *d_stats, void *hip_stream) {
    if (!eng || (n && (!d_roots || !d_vals || !d_words || !d_move || !d_na || !d_stats)))
        return fail(ZC_EINVAL, "null argument");
    if (mode != 1 && mode != 2) return fail(ZC_EINVAL, "mode must be 1 (record) or 2 (replay)");
    if (int r = check_search(eng, first, n, sims, c, bs)) return r;
    if (int r = check_carry(eng, first, n)) return r;
    if (!n) return ZC_OK;
    std::lock_guard<std::mutex> lk(eng->mu);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    zc::SearchParams p = make_params(eng, first, n, d_roots, sims, c, bs, d_move, d_na, d_stats);
    if (p.philox || p.stamp) return fail(ZC_EINVAL, "the walk diagnostic runs the exact, unstamped search");
    // the logs are indexed by engine game (g * sims, g * flushes): shift so game `first` is row 0
    p.walk_vals = d_vals - (size_t)first * sims;
    p.walk_words = d_words - (size_t)first * ((sims + bs - 1) / bs);
    zc::launch_c4_walk(p, mode, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_debug_rng_copy(zc_engine *eng, int32_t first, int32_t n, void *d_buf, int32_t restore, void *hip_stream) {
    if (!eng || (n && !d_buf)) return fail(ZC_EINVAL, "null argument");
    if (int r = check_games(eng, first, n)) return r;
    if (!n) return ZC_OK;
    std::lock_guard<std::mutex> lk(eng->mu);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    hipStream_t s = (hipStream_t)hip_stream;
    uint8_t *ring = (uint8_t *)(eng->a.ring + (size_t)first * zc::kRingWords);
    uint8_t *pos = (uint8_t *)(eng->a.rngpos + 2 * (size_t)first);
    uint8_t *b = (uint8_t *)d_buf;
    const size_t rb = (size_t)n * zc::kRingWords * sizeof(uint32_t), pb = (size_t)n * 2 * sizeof(uint64_t);
    ZC_HIP(hipMemcpyAsync(restore ? ring : b, restore ? b : ring, rb, hipMemcpyDeviceToDevice, s));
    ZC_HIP(hipMemcpyAsync(restore ? pos : b + rb, restore ? b + rb : pos, pb, hipMemcpyDeviceToDevice, s));
    return ZC_OK;
}

int zc_debug_c4_launch_stamps(zc_engine *eng, uint64_t *d_buf) {
    if (!eng) return fail(ZC_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(eng->mu);
    eng->tstamps = d_buf;
    return ZC_OK;
}

int zc_debug_net_switch(const char *name, int32_t value, int32_t *old) {
    int prev = 0;
    if (!zc::net_switch(name, value, &prev))
        return fail(ZC_EINVAL, "zc_debug_net_switch: unknown switch or value (%s = %d)", name ? name : "(null)", value);
    if (old) *old = prev;
    return ZC_OK;
}

int zc_debug_phase_cycles_games(zc_engine *eng, int32_t n_games, int64_t *out) {
    if (!eng || !out) return fail(ZC_EINVAL, "null argument");
    if (n_games < 0 || n_games > eng->cfg.max_games) return fail(ZC_EINVAL, "n_games outside the engine");
    std::lock_guard<std::mutex> lk(eng->mu);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    ZC_HIP(hipDeviceSynchronize());
    ZC_HIP(hipMemcpy(out, eng->a.phase, (size_t)n_games * zc::kPhases * sizeof(int64_t), hipMemcpyDeviceToHost));
    return ZC_OK;
}

int zc_debug_phase_cycles(zc_engine *eng, int32_t enable, int64_t *out8) {
    if (!eng) return fail(ZC_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(eng->mu);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    ZC_HIP(hipDeviceSynchronize());
    const size_t G = (size_t)eng->cfg.max_games;
    constexpr int K = zc::kPhases;
    if (out8) {
        std::vector<int64_t> ph(G * K);
        ZC_HIP(hipMemcpy(ph.data(), eng->a.phase, ph.size() * sizeof(int64_t), hipMemcpyDeviceToHost));
        for (int k = 0; k < K; ++k) out8[k] = 0;
        for (size_t g = 0; g < G; ++g)
            for (int k = 0; k < K; ++k) out8[k] += ph[K * g + k];
    }
    ZC_HIP(hipMemset(eng->a.phase, 0, G * K * sizeof(int64_t)));
    eng->stamp = enable ? 1 : 0;
    return ZC_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- any game backend (gen_search.hip)
namespace {
size_t gen_slot_bytes() { return sizeof(int32_t) * 3 + sizeof(double) * 2; }  // na, child, untried, wa, qa

// Grow the any-backend tree to hold `nodes` nodes and `slots` move slots, keeping its
// content (the device is synchronised first: a search may be in flight).
int gen_reserve_locked(zc_engine *e, int64_t nodes, int64_t slots) {
    zc::GenArena &g = e->ga;
    if (!g.ctl) {
        if (hipMalloc((void **)&g.ctl, zc::kGenCtlWords * sizeof(int32_t)) != hipSuccess ||
            hipMalloc((void **)&g.pending, (size_t)e->cfg.max_batch * sizeof(int32_t)) != hipSuccess)
            return fail(ZC_ENOMEM, "hipMalloc failed (any-backend tree control)");
        if (hipMemset(g.ctl, 0, zc::kGenCtlWords * sizeof(int32_t)) != hipSuccess) return fail(ZC_EHIP, "memset failed");
        e->bytes += zc::kGenCtlWords * sizeof(int32_t) + (size_t)e->cfg.max_batch * sizeof(int32_t);
    }
    if (nodes <= g.node_cap && slots <= g.slot_cap) return ZC_OK;
    if (nodes > INT32_MAX || slots > INT32_MAX) return fail(ZC_ECAPACITY, "any-backend tree beyond 2^31 nodes or slots");
    const int64_t nn = std::max<int64_t>(nodes, g.node_cap), ns = std::max<int64_t>(slots, g.slot_cap);
    zc::GenArena n = g;
    bool ok = hipMalloc((void **)&n.nodes, (size_t)nn * sizeof(zc::GenNode)) == hipSuccess;
    ok = ok && hipMalloc((void **)&n.na, (size_t)ns * sizeof(int32_t)) == hipSuccess;
    ok = ok && hipMalloc((void **)&n.wa, (size_t)ns * sizeof(double)) == hipSuccess;
    ok = ok && hipMalloc((void **)&n.qa, (size_t)ns * sizeof(double)) == hipSuccess;
    ok = ok && hipMalloc((void **)&n.child, (size_t)ns * sizeof(int32_t)) == hipSuccess;
    ok = ok && hipMalloc((void **)&n.untried, (size_t)ns * sizeof(int32_t)) == hipSuccess;
    if (!ok) {
        void *ptrs[] = {n.nodes, n.na, n.wa, n.qa, n.child, n.untried};
        for (void *p : ptrs)
            if (p && p != g.nodes && p != g.na && p != g.wa && p != g.qa && p != g.child && p != g.untried)
                (void)hipFree(p);
        return fail(ZC_ENOMEM, "hipMalloc failed (any-backend tree of %lld nodes, %lld slots)", (long long)nn,
                    (long long)ns);
    }
    ZC_HIP(hipDeviceSynchronize());
    if (g.node_cap) {
        const size_t on = (size_t)g.node_cap, os = (size_t)g.slot_cap;
        ZC_HIP(hipMemcpy(n.nodes, g.nodes, on * sizeof(zc::GenNode), hipMemcpyDeviceToDevice));
        ZC_HIP(hipMemcpy(n.na, g.na, os * sizeof(int32_t), hipMemcpyDeviceToDevice));
        ZC_HIP(hipMemcpy(n.wa, g.wa, os * sizeof(double), hipMemcpyDeviceToDevice));
        ZC_HIP(hipMemcpy(n.qa, g.qa, os * sizeof(double), hipMemcpyDeviceToDevice));
        ZC_HIP(hipMemcpy(n.child, g.child, os * sizeof(int32_t), hipMemcpyDeviceToDevice));
        ZC_HIP(hipMemcpy(n.untried, g.untried, os * sizeof(int32_t), hipMemcpyDeviceToDevice));
        void *old[] = {g.nodes, g.na, g.wa, g.qa, g.child, g.untried};
        for (void *p : old) (void)hipFree(p);
    }
    e->bytes += (nn - g.node_cap) * (int64_t)sizeof(zc::GenNode) + (ns - g.slot_cap) * (int64_t)gen_slot_bytes();
    n.node_cap = (int32_t)nn;
    n.slot_cap = ns;
    g = n;
    return ZC_OK;
}

zc::GenParams gen_params(const zc_engine *e) {
    zc::GenParams p{};
    p.sims = e->gx_sims;
    p.bs = e->gx_bs;
    p.c = e->gx_c;
    p.logtab = e->a.logtab;
    p.a = e->ga;
    return p;
}

int check_gx(const zc_engine *e) {
    if (!e->gx_active) return fail(ZC_EINVAL, "no any-backend search in progress (call zc_gen_begin first)");
    return ZC_OK;
}
}  // namespace

extern "C" {

int zc_gen_reserve(zc_engine *eng, int32_t nodes, int64_t slots) {
    if (!eng) return fail(ZC_EINVAL, "null argument");
    if (nodes < 1 || slots < 0) return fail(ZC_EINVAL, "need nodes >= 1 and slots >= 0");
    std::lock_guard<std::mutex> lk(eng->mu);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    return gen_reserve_locked(eng, nodes, slots);
}

int zc_gen_capacity(zc_engine *eng, int32_t *nodes, int64_t *slots) {
    if (!eng || !nodes || !slots) return fail(ZC_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(eng->mu);
    *nodes = eng->ga.node_cap;
    *slots = eng->ga.slot_cap;
    return ZC_OK;
}

int zc_gen_begin(zc_engine *eng, int32_t sims, double c, int32_t bs, int32_t root_moves, void *hip_stream) {
    if (!eng) return fail(ZC_EINVAL, "null argument");
    if (int r = check_search(eng, 0, 0, sims, c, bs)) return r;
    if (root_moves < 0) return fail(ZC_EINVAL, "root_moves must be >= 0");
    std::lock_guard<std::mutex> lk(eng->mu);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    if (int r = gen_reserve_locked(eng, (int64_t)sims + 1, std::max<int64_t>(root_moves, eng->ga.slot_cap))) return r;
    eng->gx_sims = sims;
    eng->gx_bs = bs;
    eng->gx_c = c;
    eng->gx_active = true;
    zc::launch_gen_begin(gen_params(eng), root_moves, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_gen_walk(zc_engine *eng, int32_t *d_out, int32_t out_cap, void *hip_stream) {
    if (!eng || !d_out) return fail(ZC_EINVAL, "null argument");
    if (out_cap < 5) return fail(ZC_EINVAL, "out_cap must be >= 5");
    std::lock_guard<std::mutex> lk(eng->mu);
    if (int r = check_gx(eng)) return r;
    ZC_HIP(hipSetDevice(eng->cfg.device));
    zc::launch_gen_walk(gen_params(eng), d_out, out_cap, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_gen_expand(zc_engine *eng, int32_t untried_index, int32_t child_moves, void *hip_stream) {
    if (!eng) return fail(ZC_EINVAL, "null argument");
    if (untried_index < -1 || child_moves < 0) return fail(ZC_EINVAL, "bad untried_index / child_moves");
    std::lock_guard<std::mutex> lk(eng->mu);
    if (int r = check_gx(eng)) return r;
    ZC_HIP(hipSetDevice(eng->cfg.device));
    zc::launch_gen_expand(gen_params(eng), untried_index, child_moves, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_gen_backup(zc_engine *eng, int32_t n_leaves, const double *d_values, void *hip_stream) {
    if (!eng || (n_leaves && !d_values)) return fail(ZC_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(eng->mu);
    if (int r = check_gx(eng)) return r;
    if (n_leaves < 0 || n_leaves > eng->gx_bs) return fail(ZC_EINVAL, "n_leaves %d outside [0, batch_size]", n_leaves);
    ZC_HIP(hipSetDevice(eng->cfg.device));
    zc::launch_gen_backup(gen_params(eng), n_leaves, d_values, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    return ZC_OK;
}

int zc_gen_end(zc_engine *eng, int32_t *d_out, int32_t *d_root_na, int32_t na_cap, void *hip_stream) {
    if (!eng || !d_out) return fail(ZC_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(eng->mu);
    if (int r = check_gx(eng)) return r;
    ZC_HIP(hipSetDevice(eng->cfg.device));
    zc::launch_gen_end(gen_params(eng), d_out, d_root_na, d_root_na ? na_cap : 0, (hipStream_t)hip_stream);
    ZC_HIP(hipGetLastError());
    eng->gx_active = false;
    return ZC_OK;
}

}  // extern "C"
