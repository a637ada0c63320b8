// life_plan.cpp -- host-only partition, layout and halo plan (no HIP calls,
// callable without a GPU).
//
// Replaces the reference's MPI Cartesian set-up and exchange schedule:
//   MPI_Dims_create / MPI_Cart_create / MPI_Cart_coords  life_cart.c:117-121
//   decomposition()                                      life_cart.c:217-223
//   exchange_columns / exchange_rows / exchange_corners  life_cart.c:225-279
// The corner messages are dropped: columns go first, then rows of width+2
// carry the freshly received column apron (the corners) along.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "life_host.h"
#include "life_mi355x.h"

namespace {
constexpr int64_t kXoff = 128;  // owned x = 0 starts 128 B into a padded row
inline int64_t round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }
inline int cart_rank(int c0, int c1, int dims1) { return c0 * dims1 + c1; }
}  // namespace

extern "C" {

void life_decomposition(int64_t n, int p, int k, int64_t *start, int64_t *stop) {
    const int64_t l = n / p;  // life_cart.c:218
    *start = l * k;
    *stop = *start + l;
    if (k == p - 1) *stop = n;  // the last block takes the remainder (:221-222)
}

void life_dims_create(int n, int dims[2]) {
    // MPI_Dims_create(n, 2, {0,0}): most balanced factor pair, non-increasing.
    int d1 = 1;
    for (int f = 1; (int64_t)f * f <= n; f++)
        if (n % f == 0) d1 = f;
    dims[0] = n / d1;
    dims[1] = d1;
}

int life_dims_choose(int64_t nx, int64_t ny, int n, int policy, int dims[2]) {
    if (!dims || n < 1 || nx <= 0 || ny <= 0) return LIFE_EINVAL;
    switch (policy) {
    case LIFE_PARTITION_CART: life_dims_create(n, dims); break;
    case LIFE_PARTITION_ROWS: dims[0] = 1, dims[1] = n; break;
    case LIFE_PARTITION_COLS: dims[0] = n, dims[1] = 1; break;
    case LIFE_PARTITION_AUTO:
        // the shortest strip (the decomposition remainder goes to the last)
        if (ny / n >= LIFE_AUTO_MIN_STRIP_ROWS)
            dims[0] = 1, dims[1] = n;
        else
            life_dims_create(n, dims);
        break;
    default: return LIFE_EINVAL;
    }
    if (nx < dims[0] || ny < dims[1]) return LIFE_EINVAL;
    return LIFE_OK;
}

// Generations per halo exchange of the temporally blocked layout, per
// encoding: LIFE_TEMPORAL_DEPTH (bit) / LIFE_TEMPORAL_DEPTH_BYTE, or 8 / 12 /
// 16 / 24 / 32 from the environment variables of the same names (read once; every rank
// of a job must see the same values); 1 selects the one-generation layouts
// (a measurement knob: the HBM-bound kernels).  The byte encoding moves 8x
// the bytes per cell, so it amortises each HBM pass over more generations.
static int env_depth(const char *name, int dflt) {
    const char *e = getenv(name);
    const int v = e ? atoi(e) : 0;
    return v == 1 || v == 8 || v == 12 || v == 16 || v == 24 || v == 32 ? v : dflt;
}
static int temporal_depth(int kernel) {
    static const int kbit = env_depth("LIFE_TEMPORAL_DEPTH", LIFE_TEMPORAL_DEPTH);
    static const int kbyte = [] {  // the byte tiles are built for 16 or 32 ghost rows
        const int v = env_depth("LIFE_TEMPORAL_DEPTH_BYTE", LIFE_TEMPORAL_DEPTH_BYTE);
        return v == 1 || v == 16 ? v : 32;
    }();
    return kernel == LIFE_KERNEL_BIT ? kbit : kbyte;
}

// The temporally blocked stencil keeps one lane column of x-apron -- 64
// cells (one interleaved pair) for the bit encoding, 32 for the byte
// encoding -- and K-row y-aprons: every block must be at least that wide (a
// neighbour, or the shard itself when x wraps inside it, fills the apron
// columns) and, on a partitioned y axis, at least K rows tall.
static int64_t temporal_xapron(int kernel) { return kernel == LIFE_KERNEL_BIT ? 64 : 32; }
static bool temporal_ok(int64_t nx, int64_t ny, int dims0, int dims1, int K, int64_t xa) {
    for (int k = 0; k < dims0; k++) {
        int64_t s, e;
        life_decomposition(nx, dims0, k, &s, &e);
        if (e - s < xa) return false;
    }
    if (dims1 > 1)
        for (int k = 0; k < dims1; k++) {
            int64_t s, e;
            life_decomposition(ny, dims1, k, &s, &e);
            if (e - s < K) return false;
        }
    return true;
}

int life_layout_query(int64_t nx, int64_t ny, int dims0, int dims1, int rank, int kernel,
                      life_layout *out) {
    if (!out || nx <= 0 || ny <= 0 || dims0 <= 0 || dims1 <= 0 || rank < 0 ||
        rank >= dims0 * dims1 || (kernel != LIFE_KERNEL_BYTE && kernel != LIFE_KERNEL_BIT))
        return LIFE_EINVAL;
    if (nx < dims0 || ny < dims1) return LIFE_EINVAL;  // no empty blocks
    memset(out, 0, sizeof *out);
    const int c0 = rank / dims1, c1 = rank % dims1;  // MPI_Cart_coords, row-major
    int64_t xs, xe, ys, ye;
    life_decomposition(nx, dims0, c0, &xs, &xe);
    life_decomposition(ny, dims1, c1, &ys, &ye);
    out->w = xe - xs;
    out->h = ye - ys;
    out->x0 = xs;
    out->y0 = ys;
    out->kernel = kernel;
    out->coords[0] = c0;
    out->coords[1] = c1;
    const int K = temporal_depth(kernel);
    const int64_t xa = temporal_xapron(kernel);
    const bool temporal = K > 1 && temporal_ok(nx, ny, dims0, dims1, K, xa);
    out->xapron = temporal ? xa : 1;
    out->yapron = temporal ? K : 1;
    out->generations_per_exchange = temporal ? K : 1;
    const int64_t cells_per_unit = kernel == LIFE_KERNEL_BIT ? 128 : 16;
    out->units = (out->w + cells_per_unit - 1) / cells_per_unit;
    out->xoff = kXoff;
    // room for the last unit, the right apron (a cell, one 64-cell pair, or 32
    // byte cells) and the right extra dword; the temporal byte stencil reads
    // whole 32-byte words up to the one holding cell w+31
    out->pitch = round_up(kXoff + 16 * out->units + (temporal && kernel == LIFE_KERNEL_BYTE ? 64 : 16), 256);
    out->rows = out->h + 2 * out->yapron;
    return LIFE_OK;
}

}  // extern "C"

int64_t life::flow_chunk_passes(int64_t tiles, int64_t grid, int64_t cap) {
    if (tiles < 1 || grid < 0 || cap < 0) return 0;
    // items = passes * tiles; pulls = items + grid (each workgroup's last pull
    // finds the queue empty) must stay <= kFlowMaxHead
    int64_t n = (kFlowMaxHead - grid) / tiles;
    if (n < 0) n = 0;
    return cap > 0 && cap < n ? cap : n;
}

int64_t life::gather_frame_row_bytes(int64_t nx, int fmt) {
    return fmt == kGatherBits ? (nx + 7) / 8 : nx * (fmt == kGatherVtk ? 2 : 1);
}

int life::gather_plan(int64_t nx, int64_t ny, int dims0, int dims1, int kernel, int fmt, GatherPiece *pieces,
                      int max, int64_t *slot_bytes) {
    if (dims0 < 1 || dims1 < 1 || fmt < kGatherDense || fmt > kGatherBits || !pieces || !slot_bytes) return LIFE_EINVAL;
    const int world = dims0 * dims1;
    if (max < world) return LIFE_EINVAL;
    const int root = world - 1;  // life_collect: cart rank of (dims0-1, dims1-1)
    const int64_t frb = gather_frame_row_bytes(nx, fmt);
    int64_t big = 0;
    for (int k = 0; k < world; k++) {
        const int r = k == 0 ? root : k - 1;  // the root's own block, then the fan-in order
        life_layout L;
        if (life_layout_query(nx, ny, dims0, dims1, r, kernel, &L) != LIFE_OK) return LIFE_EINVAL;
        GatherPiece &p = pieces[k];
        p.rank = r;
        p.slot = k == 0 ? -1 : (k - 1) % 2;
        p.row_bytes = fmt == kGatherBits ? ((L.x0 & 7) + L.w + 7) / 8 : L.w * (fmt == kGatherVtk ? 2 : 1);
        p.rows = L.h;
        p.bytes = p.row_bytes * p.rows;
        p.dst = L.y0 * frb + (fmt == kGatherBits ? (L.x0 >> 3) : L.x0 * (fmt == kGatherVtk ? 2 : 1));
        p.shared_first = fmt == kGatherBits && (L.x0 & 7) != 0;
        p.shared_last = fmt == kGatherBits && ((L.x0 + L.w) & 7) != 0 && L.x0 + L.w < nx;
        if (p.bytes > big) big = p.bytes;
    }
    *slot_bytes = big;
    return world;
}

// The halo plan; `loop` (bit 0: x, bit 1: y) treats that axis, which the
// shard spans whole (dims == 1), as partitioned too, with the shard as its own
// left and right neighbour (LIFE_OPT_LOOPBACK: the transport's send/recv path
// exercised by one rank).
int life::halo_plan(int64_t nx, int64_t ny, int dims0, int dims1, int rank, int kernel, int loop,
                    life_halo_op *ops, int max_ops) {
    life_layout L;
    const int rc = life_layout_query(nx, ny, dims0, dims1, rank, kernel, &L);
    if (rc != LIFE_OK) return rc;
    const int c0 = L.coords[0], c1 = L.coords[1];
    const int64_t w = L.w, h = L.h, xa = L.xapron, ya = L.yapron;
    life_halo_op tmp[16];
    int n = 0;
    auto add = [&](int phase, int kind, int peer, int what, int64_t index, int64_t width, int64_t first,
                   int64_t count) {
        life_halo_op &o = tmp[n++];
        o.phase = phase;
        o.kind = kind;
        o.peer = peer;
        o.what = what;
        o.index = index;
        o.width = width;
        o.first = first;
        o.count = count;
    };
    const bool px = dims0 > 1 || (loop & 1), py = dims1 > 1 || (loop & 2);
    // Both axes exchanged by messages with K-deep temporal aprons: ONE phase
    // (one RCCL group per exchange instead of two back to back, round 5):
    // columns, whole padded rows (their x-apron bytes are stale and are
    // overwritten), and the four K x xapron corners explicitly, as
    // life_cart.c:257-273 exchanges them (there one cell each).  Sends go in
    // direction order E, W, S, N, SE, SW, NE, NW; each receive is listed in
    // the order of the direction its sender sends in, so the k-th message
    // between two ranks pairs up however many directions they share (dims 2,
    // the loopback's self).  Corners are received into staging and unpacked
    // after the group, over the stale row bytes.  Not for the loopback (the
    // shard its own peer in all eight directions): RCCL ran the sixteen
    // self-messages of one group in 39 us, longer than the two groups of the
    // column and row phases (19 + 14 us; 16384 x 32768, profiles/r05/g),
    // while distinct peers over xGMI are served by separate channels.
    const bool fused = px && py && L.generations_per_exchange > 1 && loop == 0;
    const int ph_rows = fused ? 0 : 1;
    // Phase 0: columns (dim 0 splits x), owned rows only.  MPI_Cart_shift(dim 0).
    if (!px) {
        add(0, LIFE_HALO_FILL, -1, LIFE_HALO_COLUMN, -xa, xa, ya, h);
    } else {
        const int right = cart_rank((c0 + 1) % dims0, c1, dims1);
        const int left = cart_rank((c0 - 1 + dims0) % dims0, c1, dims1);
        // life_cart.c:251-254 order: Send right, Recv left, Send left, Recv right.
        add(0, LIFE_HALO_SEND, right, LIFE_HALO_COLUMN, w - xa, xa, ya, h);
        add(0, LIFE_HALO_SEND, left, LIFE_HALO_COLUMN, 0, xa, ya, h);
        add(0, LIFE_HALO_RECV, left, LIFE_HALO_COLUMN, -xa, xa, ya, h);
        add(0, LIFE_HALO_RECV, right, LIFE_HALO_COLUMN, w, xa, ya, h);
    }
    // Phase 1 (phase 0 when fused): whole rows including the x-apron just
    // received (the corners), or with a stale x-apron the corners overwrite.
    if (!py) {
        add(1, LIFE_HALO_FILL, -1, LIFE_HALO_ROW, 0, ya, -xa, w + 2 * xa);
    } else {
        const int right = cart_rank(c0, (c1 + 1) % dims1, dims1);
        const int left = cart_rank(c0, (c1 - 1 + dims1) % dims1, dims1);
        // life_cart.c:235-238 order.  Padded row of owned row y is y + ya.
        add(ph_rows, LIFE_HALO_SEND, right, LIFE_HALO_ROW, h, ya, -xa, w + 2 * xa);
        add(ph_rows, LIFE_HALO_SEND, left, LIFE_HALO_ROW, ya, ya, -xa, w + 2 * xa);
        add(ph_rows, LIFE_HALO_RECV, left, LIFE_HALO_ROW, 0, ya, -xa, w + 2 * xa);
        add(ph_rows, LIFE_HALO_RECV, right, LIFE_HALO_ROW, h + ya, ya, -xa, w + 2 * xa);
    }
    if (fused) {
        // direction d = (dx, dy) in the order SE, SW, NE, NW; the shard at
        // (c0 + dx, c1 + dy) gets my corner next to it: x side by dx (my right
        // column w - xa, or cells [0, xa)), rows by dy (my bottom K rows,
        // padded h, or my top K, padded ya)
        static const int kDir[4][2] = {{1, 1}, {-1, 1}, {1, -1}, {-1, -1}};
        auto at = [&](int dx, int dy) {
            return cart_rank((c0 + dx + dims0) % dims0, (c1 + dy + dims1) % dims1, dims1);
        };
        for (const auto &d : kDir)
            add(0, LIFE_HALO_SEND, at(d[0], d[1]), LIFE_HALO_CORNER, d[0] > 0 ? w - xa : 0, xa, d[1] > 0 ? h : ya,
                ya);
        // the sender of direction d sits at -d: its corner lands in my apron
        // on the side facing it (left apron -xa when it is left of me)
        for (const auto &d : kDir)
            add(0, LIFE_HALO_RECV, at(-d[0], -d[1]), LIFE_HALO_CORNER, d[0] > 0 ? -xa : w, xa,
                d[1] > 0 ? 0 : h + ya, ya);
    }
    if (ops) {
        if (max_ops < n) return LIFE_EINVAL;
        memcpy(ops, tmp, sizeof(life_halo_op) * n);
    }
    return n;
}

extern "C" {

int life_halo_plan(int64_t nx, int64_t ny, int dims0, int dims1, int rank, int kernel,
                   life_halo_op *ops, int max_ops) {
    return life::halo_plan(nx, ny, dims0, dims1, rank, kernel, 0, ops, max_ops);
}

const char *life_strerror(int err) {
    switch (err) {
    case LIFE_OK: return "success";
    case LIFE_EINVAL: return "invalid argument";
    case LIFE_EHIP: return "HIP runtime error";
    case LIFE_ERCCL: return "RCCL error";
    case LIFE_ENOMEM: return "out of memory";
    case LIFE_ESTATE: return "invalid state";
    case LIFE_EIO: return "I/O or parse error";
    default: return "unknown error";
    }
}

// SURVEY 8(b)'s proposed name for the same function
const char *life_dev_strerror(int err) { return life_strerror(err); }

}  // extern "C"

namespace {
// Slots grouped by the time they fall free (a list schedule of a few item
// kinds keeps a handful of distinct free times).
struct SlotGroups {
    static constexpr int kMax = 32;
    double t[kMax];
    int64_t c[kMax];
    int n = 0;
    void add(double tt, int64_t cc) {
        for (int i = 0; i < n; i++)
            if (t[i] > tt - 1e-9 && t[i] < tt + 1e-9) {
                c[i] += cc;
                return;
            }
        if (n < kMax) {
            t[n] = tt;
            c[n++] = cc;
            return;
        }
        // (never reached at the shapes planned: merge into the latest group, which
        // only makes the estimate pessimistic)
        int j = 0;
        for (int i = 1; i < n; i++)
            if (t[i] > t[j]) j = i;
        if (tt > t[j]) t[j] = tt;
        c[j] += cc;
    }
    // deals `items` items of duration d, returns the latest end
    double deal(double d, int64_t items, double end) {
        while (items > 0 && n > 0) {
            int i = 0;
            for (int k = 1; k < n; k++)
                if (t[k] < t[i]) i = k;
            const int64_t k = c[i] < items ? c[i] : items;
            items -= k;
            const double nt = t[i] + d;
            if (k == c[i]) {
                t[i] = t[--n];
                c[i] = c[n];
            } else {
                c[i] -= k;
            }
            add(nt, k);
            if (nt > end) end = nt;
        }
        return end;
    }
};

struct TailKey {
    int64_t ntx, B, ty0, ty1, yend, T, T2, slots, pre;
    int mode;
    double c;
    bool operator==(const TailKey &o) const {
        return ntx == o.ntx && B == o.B && ty0 == o.ty0 && ty1 == o.ty1 && yend == o.yend && T == o.T && T2 == o.T2 &&
               slots == o.slots && pre == o.pre && mode == o.mode && c == o.c;
    }
};
}  // namespace

double life::tail_makespan2(int64_t ntx, int64_t B, int64_t F_rows, int64_t n2, int64_t slots, double c,
                            int64_t pre) {
    if (slots < 1) return 0.0;
    const int64_t nf = (pre > 0 ? pre : 0) + tail_row_items(ntx, B, F_rows);
    const int64_t r = nf / slots, rem = nf % slots;
    SlotGroups g;
    g.add((double)r, slots - rem);
    if (rem) g.add((double)(r + 1), rem);
    const double end = nf ? (double)(r + (rem ? 1 : 0)) : 0.0;
    return g.deal(c + (1.0 - c) * 0.5, tail_row_items(ntx, B, n2), end);
}

life::TailPlan life::tail_plan(int64_t ntx, int64_t B, int64_t ty0, int64_t ty1, int64_t yend, int64_t T,
                               int64_t T2, int64_t slots, int mode, double c, int64_t pre) {
    TailPlan none;
    none.F = ty1;
    if (ntx < 1 || ty1 <= ty0 || T < 1 || T2 < 1 || slots < 1 || mode < 1 || mode > 2 || pre < 0) return none;
    // the launch shares the slots with `pre` items dispatched before it
    const int64_t nall = pre + tail_row_items(ntx, B, ty1 - ty0);
    none.makespan = tail_makespan2(ntx, B, ty1 - ty0, 0, slots, c, pre);
    // Whole rounds: nothing to fill.  One round or less: the model's slots are
    // not independent there (a CU's three slots share its SIMDs, and a lone
    // tile runs faster), so it is not trusted to re-tile an underfilled launch.
    if (nall <= slots || nall % slots == 0) return none;
    static std::mutex mu;
    static std::vector<std::pair<TailKey, TailPlan>> cache;
    const TailKey key{ntx, B, ty0, ty1, yend, T, T2, slots, pre, mode, c};
    {
        std::lock_guard<std::mutex> lk(mu);
        for (const auto &e : cache)
            if (e.first == key) return e.second;
    }
    TailPlan best = none;
    auto halves = [&](int64_t F) -> int64_t {
        const int64_t left = yend - F * T;
        return left > 0 ? (left + T2 - 1) / T2 : 0;
    };
    if (mode == 1) {
        // round 4's rule: the fewest bottom rows whose half tiles fill one
        // round, when the last round is under half full
        if (nall % slots <= slots / 2) {
            int64_t q = 1;
            while (q < ty1 - ty0 && tail_row_items(ntx, B, (q * T + T2 - 1) / T2) < slots) ++q;
            if (q < ty1 - ty0) {
                best.F = ty1 - q;
                best.n2 = halves(best.F);
                best.makespan = tail_makespan2(ntx, B, best.F - ty0, best.n2, slots, c, pre);
            }
        }
    } else {
        // every split point (ties keep more full tiles)
        for (int64_t F = ty1 - 1; F >= ty0; --F) {
            const int64_t n2 = halves(F);
            const double t = tail_makespan2(ntx, B, F - ty0, n2, slots, c, pre);
            if (t < best.makespan - 1e-9) {
                best.F = F;
                best.n2 = n2;
                best.makespan = t;
            }
        }
    }
    std::lock_guard<std::mutex> lk(mu);
    if (cache.size() >= 512) cache.erase(cache.begin());
    cache.emplace_back(key, best);
    return best;
}
