// life_dev.hip -- C-ABI runtime of the MI355X Game-of-Life hot path.
//
// One life_dev owns the shards this process drives.  Each shard = one block of
// the dims[0] x dims[1] periodic Cartesian partition, double-buffered in HBM
// with a one-cell apron, one HIP stream, and (RCCL transport) one RCCL
// communicator rank.  Per generation (life_cart.c:73-74):
//   life_step     -> stencil kernel(s) cur -> nxt            (life_kernels.hip)
//   life_exchange -> phase x (columns), then phase y (rows of width+2),
//                    each either a periodic fill inside the shard
//                    (dims[d] == 1) or ncclSend/ncclRecv with the Cartesian
//                    neighbours (replaces life_cart.c:225-279).
// Overlap: the stencil is split into the boundary ring and the interior; the
// ring runs first, the halo exchange of the NEW state runs on the comm stream
// while the interior kernel runs on the compute stream.
#include <rccl/rccl.h>
#include <algorithm>
#include <stdarg.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include <chrono>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "life_kernels.h"
#include "life_mi355x.h"

namespace {

thread_local std::string g_err;

void set_err(const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
}

#define HIPCHK(expr)                                                                          \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess) {                                                               \
            set_err("%s:%d %s: %s", __FILE__, __LINE__, #expr, hipGetErrorString(e_));        \
            return e_ == hipErrorOutOfMemory ? LIFE_ENOMEM : LIFE_EHIP;                       \
        }                                                                                     \
    } while (0)

#define NCCLCHK(expr)                                                                         \
    do {                                                                                      \
        ncclResult_t r_ = (expr);                                                             \
        if (r_ != ncclSuccess) {                                                              \
            set_err("%s:%d %s: %s", __FILE__, __LINE__, #expr, ncclGetErrorString(r_));       \
            return LIFE_ERCCL;                                                                \
        }                                                                                     \
    } while (0)

#define CHK(expr)                     \
    do {                              \
        int rc_ = (expr);             \
        if (rc_ != LIFE_OK) return rc_; \
    } while (0)

struct TimedLaunch {
    hipEvent_t a = nullptr, b = nullptr;
    int launches = 1;  // kernel launches between a and b (back-to-back on one stream)
};

// Event set of one overlapped block (timing on): ring kernels, interior
// kernel, halo exchange, and the whole block on the compute stream.
struct PhaseEvents {
    hipEvent_t ring0 = nullptr, ring1 = nullptr, int0 = nullptr, int1 = nullptr, halo0 = nullptr,
               halo1 = nullptr, end = nullptr;
};

struct Shard {
    int rank = 0;    // global shard rank (Cartesian rank, row-major coords)
    int device = 0;
    life_layout lay{};
    uint8_t *buf[2] = {nullptr, nullptr};
    int cur = 0;
    hipStream_t stream = nullptr;   // compute: whole-block kernels, boundary ring
    hipStream_t stream2 = nullptr;  // compute: interior, concurrent with ring + halo
    hipStream_t comm_stream = nullptr;
    hipEvent_t ev_halo = nullptr, ev_sync = nullptr, ev_int = nullptr;
    hipEvent_t ev_entry = nullptr;  // life_dev_step entry fence (see there)
    // device span of the last step call (timing on): own_a / own_b recorded at
    // the call's two ends, or the kTimeCall pair borrowed (span_a / span_b)
    hipEvent_t own_a = nullptr, own_b = nullptr, span_a = nullptr, span_b = nullptr;
    ncclComm_t comm = nullptr;
    uint8_t *col_send = nullptr, *col_recv = nullptr;  // 2*h bytes each
    unsigned long long *d_count = nullptr;  // census: live count, checksum
    unsigned long long *h_count = nullptr;  // pinned, 2 entries
    uint8_t *sink = nullptr;  // stencil stores of lanes outside a region
    uint8_t *stage = nullptr;  // gather staging (grows on demand)
    size_t stage_bytes = 0;
    unsigned int *flow = nullptr;  // dataflow tiles: queue head, error word, per-tile pass counts (grows on demand)
    size_t flow_words = 0;
    bool flow_used = false;  // a dataflow launch since the last sync checked its error word
    std::vector<life_halo_op> plan;
    bool corners = false;  // the plan exchanges the four corner blocks itself (fused, one phase)
    std::vector<TimedLaunch> timers;
    size_t timers_used = 0;
    std::vector<PhaseEvents> phases;
    size_t phases_used = 0;
};

}  // namespace

// Tiles: generations per launch at most (the apron depth K allows up to K).
// Bit tiles hold m ghost rows per window end, so longer launches mean more
// ghost rows (2m of the 192-row pair window) but fewer window loads /
// stores: 12 measured best at 65536^2 (992 generations: 112.3-112.9 T; 10:
// 109.4-110.0, 14: 111.3-111.7, 16: 108.4; profiles/r03/r4g), and a
// 20-generation call then runs as two launches of 10 (97.1-97.5 T against
// 93.5-93.9 for one launch of 20; profiles/r03/r4d).  Byte tiles are HBM-bound below ~32 generations per
// pass: 32.  LIFE_BLOCK_GENS overrides both at load time; 0 = per encoding.
static const int kEnvBlockGens = [] {
    const char *e = getenv("LIFE_BLOCK_GENS");
    const int v = e ? atoi(e) : 0;
    return v >= 1 && v <= 32 ? v : 0;
}();
// LIFE_FLOW (0/1/2/3) sets LIFE_OPT_FLOW's default at load time; default 3,
// automatic (round 5): the dataflow form where a pass is only a few rounds
// of resident workgroups, so that a launch per pass would idle the chip in
// its tail (flow_auto below), the per-launch tiles elsewhere.
// With the natural-word tiles (384-row windows, 20 generations per pass) the
// dataflow form won (65536^2 95 -> 100 T, profiles/r02/flow_ab.txt); the
// pair tiles are half as tall, their items half as long, and the per-item
// queue / dependency / write-through cost now outweighs the launch tails it
// saves: 992 generations at 65536^2, per-launch tiles 109.4-112.9 T against
// 104.2-108.5 T for the dataflow form at every pass size 10-16
// (profiles/r03/r4g).
static const int kEnvFlow = [] {
    const char *e = getenv("LIFE_FLOW");
    const int v = e ? atoi(e) : 3;
    return v >= 0 && v <= 3 ? v : 3;
}();
// LIFE_FLOW_AUTO_ROUNDS (measurement knob, default 5): LIFE_OPT_FLOW 3 takes
// the dataflow form when a pass holds fewer rounds of resident workgroups.
static const double kFlowAutoRounds = [] {
    const char *e = getenv("LIFE_FLOW_AUTO_ROUNDS");
    const double v = e ? atof(e) : 0.0;
    return v > 0.0 ? v : 5.0;
}();
// LIFE_DEEP_HALO (0/1, default 1) sets LIFE_OPT_DEEP_HALO's default at load
// time (generation_block).
static const bool kEnvDeepHalo = [] {
    const char *e = getenv("LIFE_DEEP_HALO");
    return e ? atoi(e) != 0 : true;
}();
static int default_block_gens(int kernel) {
    return kEnvBlockGens ? kEnvBlockGens : (kernel == LIFE_KERNEL_BIT ? 12 : 32);
}
// LIFE_FLOW_MIN_PASSES (measurement knob, default 4): fewest passes a call
// runs in the dataflow form
static const int64_t kFlowMinPasses = [] {
    const char *e = getenv("LIFE_FLOW_MIN_PASSES");
    const int v = e ? atoi(e) : 0;
    return (int64_t)(v >= 2 ? v : 4);
}();
// How timed stencil launches are bracketed (LIFE_TIMING_MODE, measurement
// knob): 0 one event pair around a single-stream step call's launches (the
// default: one hipEventRecord before the first launch, none between
// launches), 1 per launch with hipEventRecord, 2 per launch stamped by the
// dispatch itself (hipExtLaunchKernel), 3 no events.
enum TimingMode { kTimeCall = 0, kTimeRecord = 1, kTimeExt = 2, kTimeOff = 3 };
// LIFE_STREAM_PRIORITY (0/1, default 0): ring + comm streams at the greatest
// HIP stream priority, the interior stream at the least (shard_alloc).
// Measured off (profiles/r04/a): the RCCL-loopback halo stays 0.23 ms beside
// the interior either way (86.5-91.2 T with, 90.0-90.8 T without), and the
// LOCAL 4-shard strong line drops 48.9 -> 34.4 T (its device copies on the
// high-priority stream slow the interior 0.148 -> 0.281 ms).
static bool stream_priorities() {
    static const bool v = [] {
        const char *e = getenv("LIFE_STREAM_PRIORITY");
        return e ? atoi(e) != 0 : false;
    }();
    return v;
}
static const int kEnvTimingMode = [] {
    const char *e = getenv("LIFE_TIMING_MODE");
    const int v = e ? atoi(e) : 0;
    return v >= 0 && v <= 3 ? v : 0;
}();

struct life_dev {
    int64_t nx = 0, ny = 0;
    int dims[2] = {1, 1};
    int world = 1;
    int kernel = LIFE_KERNEL_BYTE;
    int transport = LIFE_XPORT_LOCAL;
    bool rank_mode = false;
    bool timing = false;
    bool phase_events = true;  // timing on: also the overlapped schedule's phase events (life_dev_set_timing 1)
    bool launch_events = true;  // timing on: per-launch events of multi-stream calls (off: life_dev_set_timing 3)
    bool overlap = true;
    int block_gens = 0;  // tiles: generations per launch at most (LIFE_OPT_BLOCK_GENS; default_block_gens)
    int small_mode = 1;  // grids that fit one CU: 0 off, 1 VGPR kernel else LDS kernel, 2 LDS kernel,
                        // 3 windowed VGPR kernel over several CUs (else as 1), 4 as 1 never windowed
    int win_rows = 0, win_halo = 0;  // windowed kernel: strip height R, halo rows K (0: automatic)
    int loop = 0;  // LIFE_OPT_LOOPBACK: axes (bit 0 x, bit 1 y) whose halos the one shard exchanges with itself
    int last_path = LIFE_PATH_NONE;  // life_dev_last_path
    bool deep = kEnvDeepHalo;  // LIFE_OPT_DEEP_HALO: one K-deep exchange feeds several passes
    int since = 0;  // generations advanced since the aprons were last filled (deep halo)
    int flow = kEnvFlow;  // LIFE_OPT_FLOW: single-shard bit tiles as one persistent dataflow launch per
                          // step call (1: write-through hand-off, 2: plain stores + release; 0 off)
    int64_t flow_chunk = 0;  // LIFE_OPT_FLOW_CHUNK: passes per dataflow launch at most (0: automatic)
    TimedLaunch *call_timer = nullptr;  // kTimeCall: the pair bracketing the current step call
    std::vector<Shard> shards;
    double acc_ms = 0.0;
    int64_t acc_launches = 0;
    double acc_bytes = 0.0;    // algorithmic HBM bytes of the timed launches
    double acc_updates = 0.0;  // cell-updates they performed
    double acc_valu = 0.0;     // VALU lane-ops they issue (model; 0 where not modelled)
    // overlapped blocks of partitioned shards: summed ms per phase (timing on)
    double ph_ring = 0.0, ph_int = 0.0, ph_halo = 0.0, ph_block = 0.0;
    int64_t ph_blocks = 0;
    // the last step call (life_dev_call_stats): host time inside it, its
    // passes and the longest one's host time, whether span events exist
    double call_host_ms = 0.0, call_pass_max_ms = 0.0;
    int64_t call_passes = 0;
    bool call_spans = false;
};

namespace {

// Axis a's apron is filled by a halo exchange (dims[a] > 1, or the loopback
// test mode, where the single shard is its own neighbour on both axes).
bool part(const life_dev *d, int a) { return d->dims[a] > 1 || ((d->loop >> a) & 1); }
// The shard wraps x itself (the x-apron is filled by launch_wrap_columns).
bool self_wrap_x(const life_dev *d) { return !(d->loop & 1) && life::self_wrap_x(d->shards[0].lay, d->dims[0]); }
life::Wrap wrap_of(const life_dev *d) { return life::Wrap{!part(d, 0) && !self_wrap_x(d), !part(d, 1)}; }

// Allocation fill of every shard buffer (LIFE_POISON, read at each
// life_dev_create*): unset / 0 = zeros (a dead grid, what the reference's
// calloc gives); 1 = 0xA5 in both grid buffers (cells, aprons, pitch padding,
// slack rows), the column staging and the sink -- not a dead cell in either
// encoding, so a cell a kernel should have written but did not, or an apron
// read before its halo arrived, changes the result on every run instead of
// hiding behind a zeroed buffer that looks like a dead grid.
int alloc_fill_byte() {
    const char *e = getenv("LIFE_POISON");
    return e && atoi(e) != 0 ? 0xA5 : 0;
}

int shard_alloc(life_dev *d, Shard &s) {
    HIPCHK(hipSetDevice(s.device));
    // The streams first: every fill below is ordered on the stream that later
    // uses the buffer (the null stream does not order against non-blocking
    // streams), and finished before the shard is handed out.
    // Priorities (LIFE_STREAM_PRIORITY=1, off by default): the comm and ring
    // streams at the greatest priority, the interior at the least.
    int prio_lo = 0, prio_hi = 0;
    HIPCHK(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
    const bool prio = stream_priorities();
    HIPCHK(hipStreamCreateWithPriority(&s.stream, hipStreamNonBlocking, prio ? prio_hi : 0));
    HIPCHK(hipStreamCreateWithPriority(&s.stream2, hipStreamNonBlocking, prio ? prio_lo : 0));
    HIPCHK(hipStreamCreateWithPriority(&s.comm_stream, hipStreamNonBlocking, prio ? prio_hi : 0));
    const int fill = alloc_fill_byte();
    const int64_t slack = s.lay.generations_per_exchange > 1 ? life::kTemporalSlackRows : 0;
    const size_t bytes = (size_t)(s.lay.pitch * (s.lay.rows + slack));
    for (int i = 0; i < 2; i++) {
        HIPCHK(hipMalloc(&s.buf[i], bytes));
        HIPCHK(hipMemsetAsync(s.buf[i], fill, bytes, s.stream));
    }
    // (device-scope forms of these events, hipEventDisableSystemFence /
    // hipEventReleaseToDevice, measured flat: profiles/r06/h)
    HIPCHK(hipEventCreateWithFlags(&s.ev_int, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&s.ev_halo, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&s.ev_sync, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&s.ev_entry, hipEventDisableTiming));
    const size_t col_bytes = (size_t)life::column_stage_bytes(s.lay);
    HIPCHK(hipMalloc(&s.col_send, col_bytes));
    HIPCHK(hipMalloc(&s.col_recv, col_bytes));
    HIPCHK(hipMalloc(&s.d_count, 2 * sizeof(unsigned long long)));
    HIPCHK(hipMalloc(&s.sink, 1024));
    HIPCHK(hipMemsetAsync(s.col_send, fill, col_bytes, s.stream));
    HIPCHK(hipMemsetAsync(s.col_recv, fill, col_bytes, s.stream));
    HIPCHK(hipMemsetAsync(s.d_count, 0, 2 * sizeof(unsigned long long), s.stream));
    HIPCHK(hipMemsetAsync(s.sink, fill, 1024, s.stream));
    HIPCHK(hipStreamSynchronize(s.stream));
    HIPCHK(hipHostMalloc(&s.h_count, 2 * sizeof *s.h_count, hipHostMallocDefault));
    life_halo_op ops[16];
    const int n = life::halo_plan(d->nx, d->ny, d->dims[0], d->dims[1], s.rank, d->kernel, d->loop, ops, 16);
    if (n < 0) {
        set_err("halo plan failed for shard %d", s.rank);
        return LIFE_EINVAL;
    }
    s.plan.assign(ops, ops + n);
    s.corners = std::any_of(s.plan.begin(), s.plan.end(), [](const life_halo_op &o) { return o.what == LIFE_HALO_CORNER; });
    return LIFE_OK;
}

void shard_free(Shard &s) {
    (void)hipSetDevice(s.device);
    if (s.comm) (void)ncclCommDestroy(s.comm);
    for (auto &t : s.timers) {
        if (t.a) (void)hipEventDestroy(t.a);
        if (t.b) (void)hipEventDestroy(t.b);
    }
    for (auto &p : s.phases)
        for (hipEvent_t e : {p.ring0, p.ring1, p.int0, p.int1, p.halo0, p.halo1, p.end})
            if (e) (void)hipEventDestroy(e);
    for (uint8_t *p : {s.buf[0], s.buf[1], s.col_send, s.col_recv, s.sink, s.stage})
        if (p) (void)hipFree(p);
    if (s.flow) (void)hipFree(s.flow);
    if (s.d_count) (void)hipFree(s.d_count);
    if (s.h_count) (void)hipHostFree(s.h_count);
    for (hipEvent_t e : {s.ev_halo, s.ev_sync, s.ev_int, s.ev_entry, s.own_a, s.own_b})
        if (e) (void)hipEventDestroy(e);
    if (s.stream) (void)hipStreamDestroy(s.stream);
    if (s.stream2) (void)hipStreamDestroy(s.stream2);
    if (s.comm_stream) (void)hipStreamDestroy(s.comm_stream);
}

Shard *find_local(life_dev *d, int rank) {
    for (Shard &s : d->shards)
        if (s.rank == rank) return &s;
    return nullptr;
}

// LOCAL transport ordering around the copies of one halo phase, peers only
// (an all-to-all barrier cost 8 x 7 stream waits per step of an 8-shard
// pass: 1-2 ms of host time per pass, profiles/r04/b).  kind RECV (before the
// copies): each shard's stream waits for the shards it receives from -- their
// pack / previous phase is queued before their event.  kind SEND (after):
// each shard waits for the shards that copy from it, so nothing it enqueues
// next overwrites a message still being read.
int local_order(life_dev *d, bool comm, int phase, int kind) {
    auto st = [&](Shard &s) { return comm ? s.comm_stream : s.stream; };
    for (Shard &s : d->shards) {
        HIPCHK(hipSetDevice(s.device));
        HIPCHK(hipEventRecord(s.ev_sync, st(s)));
    }
    for (Shard &s : d->shards) {
        HIPCHK(hipSetDevice(s.device));
        int seen[16], ns = 0;
        for (const life_halo_op &o : s.plan) {
            if (o.phase != phase || o.kind != kind || o.peer == s.rank) continue;
            bool dup = false;
            for (int i = 0; i < ns; i++) dup |= seen[i] == o.peer;
            if (dup) continue;
            seen[ns++] = o.peer;
            Shard *t = find_local(d, o.peer);
            if (!t) {
                set_err("LOCAL transport: peer %d not in this process", o.peer);
                return LIFE_ESTATE;
            }
            HIPCHK(hipStreamWaitEvent(st(s), t->ev_sync, 0));
        }
    }
    return LIFE_OK;
}

// Pointer + size of the message of op `o` (the slot-th send or recv of its
// kind among its phase's ops of the same `what`): column ops go through the
// staging slots, corner ops (the fused plan) through the corner slots behind
// them, row ops are whole padded rows sent straight from / received straight
// into the buffer (every shard of one Cartesian column has the same pitch).
void op_buffer(const Shard &s, const life_halo_op &o, int slot, uint8_t *base, uint8_t **ptr, size_t *bytes) {
    const size_t cbr = (size_t)life::column_bytes_per_row(s.lay);
    uint8_t *st = o.kind == LIFE_HALO_SEND ? s.col_send : s.col_recv;
    if (o.what == LIFE_HALO_COLUMN) {
        const size_t per = (size_t)s.lay.h * cbr;
        *ptr = st + (size_t)slot * per;
        *bytes = per;
    } else if (o.what == LIFE_HALO_CORNER) {
        const size_t per = (size_t)s.lay.yapron * cbr;
        *ptr = st + 2 * (size_t)s.lay.h * cbr + (size_t)slot * per;
        *bytes = per;
    } else {
        *ptr = base + o.index * s.lay.pitch;
        *bytes = (size_t)(o.width * s.lay.pitch);
    }
}

// Staging slot of plan op i: earlier ops of its phase with the same kind and what.
int op_slot(const std::vector<life_halo_op> &plan, size_t i) {
    int n = 0;
    for (size_t k = 0; k < i; k++)
        n += plan[k].phase == plan[i].phase && plan[k].kind == plan[i].kind && plan[k].what == plan[i].what;
    return n;
}

// One halo phase on buffer `which` of every local shard, on stream sel.
int run_phase(life_dev *d, int phase, int which_rel, bool on_comm) {
    auto stream_of = [&](Shard &s) { return on_comm ? s.comm_stream : s.stream; };
    auto buf_of = [&](Shard &s) { return s.buf[s.cur ^ which_rel]; };
    // An axis that is not partitioned (dims[d] == 1, no loopback) has no halo: the stencil
    // wraps it itself (life_kernels.hip, row_ptr / WRAPX), or, for a temporal
    // layout whose width is not a multiple of 32, the shard copies its own
    // edge columns into its x-apron.
    if (!part(d, phase)) {
        if (phase == 0 && self_wrap_x(d))
            for (Shard &s : d->shards) {
                HIPCHK(hipSetDevice(s.device));
                HIPCHK(life::launch_wrap_columns(s.lay, buf_of(s), stream_of(s)));
            }
        return LIFE_OK;
    }
    bool any = false;  // a fused plan (both axes in phase 0) leaves phase 1 empty
    for (const life_halo_op &o : d->shards[0].plan) any |= o.phase == phase;
    if (!any) return LIFE_OK;
    if (phase == 0)
        for (Shard &s : d->shards) {
            HIPCHK(hipSetDevice(s.device));
            HIPCHK(life::launch_pack_columns(s.lay, buf_of(s), s.col_send, stream_of(s), s.corners));
        }
    if (d->transport == LIFE_XPORT_RCCL) {
        NCCLCHK(ncclGroupStart());
        for (Shard &s : d->shards) {
            for (size_t i = 0; i < s.plan.size(); i++) {
                const life_halo_op &o = s.plan[i];
                if (o.phase != phase) continue;
                uint8_t *p;
                size_t nb;
                op_buffer(s, o, op_slot(s.plan, i), buf_of(s), &p, &nb);
                if (o.kind == LIFE_HALO_SEND)
                    NCCLCHK(ncclSend(p, nb, ncclUint8, o.peer, s.comm, stream_of(s)));
                else
                    NCCLCHK(ncclRecv(p, nb, ncclUint8, o.peer, s.comm, stream_of(s)));
            }
        }
        NCCLCHK(ncclGroupEnd());
    } else {
        CHK(local_order(d, on_comm, phase, LIFE_HALO_RECV));
        for (Shard &s : d->shards) {
            HIPCHK(hipSetDevice(s.device));
            std::vector<int> seen_from;  // recvs from each peer so far
            for (size_t i = 0; i < s.plan.size(); i++) {
                const life_halo_op &o = s.plan[i];
                if (o.phase != phase || o.kind != LIFE_HALO_RECV) continue;
                const int slot = op_slot(s.plan, i);
                int kth = 0;  // this is the kth recv from o.peer
                for (int p : seen_from) kth += p == o.peer;
                seen_from.push_back(o.peer);
                Shard *src = find_local(d, o.peer);
                if (!src) {
                    set_err("LOCAL transport: peer %d not in this process", o.peer);
                    return LIFE_ESTATE;
                }
                // matching send: the kth send from src to s.rank
                int cnt = 0;
                const life_halo_op *match = nullptr;
                int match_slot = -1;
                for (size_t k = 0; k < src->plan.size(); k++) {
                    const life_halo_op &q = src->plan[k];
                    if (q.phase != phase || q.kind != LIFE_HALO_SEND) continue;
                    if (q.peer == s.rank && cnt++ == kth) {
                        match = &q;
                        match_slot = op_slot(src->plan, k);
                        break;
                    }
                }
                if (!match) {
                    set_err("LOCAL transport: no matching send %d->%d", o.peer, s.rank);
                    return LIFE_ESTATE;
                }
                uint8_t *dp, *sp;
                size_t dn, sn;
                op_buffer(s, o, slot, buf_of(s), &dp, &dn);
                op_buffer(*src, *match, match_slot, buf_of(*src), &sp, &sn);
                if (dn != sn) {
                    set_err("LOCAL transport: size mismatch %zu vs %zu", dn, sn);
                    return LIFE_ESTATE;
                }
                if (src->device == s.device)
                    HIPCHK(hipMemcpyAsync(dp, sp, dn, hipMemcpyDeviceToDevice, stream_of(s)));
                else
                    HIPCHK(hipMemcpyPeerAsync(dp, s.device, sp, src->device, dn, stream_of(s)));
            }
        }
        CHK(local_order(d, on_comm, phase, LIFE_HALO_SEND));
    }
    if (phase == 0)
        for (Shard &s : d->shards) {
            HIPCHK(hipSetDevice(s.device));
            HIPCHK(life::launch_unpack_columns(s.lay, buf_of(s), s.col_recv, stream_of(s), s.corners));
        }
    return LIFE_OK;
}

// Halo of buffer `which_rel` (0 = cur, 1 = nxt) on the compute streams.
// Every call fills the aprons K deep: the deep-halo count restarts.
int exchange(life_dev *d, int which_rel, bool on_comm) {
    CHK(run_phase(d, 0, which_rel, on_comm));
    CHK(run_phase(d, 1, which_rel, on_comm));
    d->since = 0;
    return LIFE_OK;
}

TimedLaunch *timer_slot(Shard &s, int *rc) {
    *rc = LIFE_OK;
    if (s.timers_used == s.timers.size()) {
        TimedLaunch t;
        if (hipEventCreate(&t.a) != hipSuccess || hipEventCreate(&t.b) != hipSuccess) {
            set_err("hipEventCreate failed");
            *rc = LIFE_EHIP;
            return nullptr;
        }
        s.timers.push_back(t);
    }
    s.timers[s.timers_used].launches = 1;
    return &s.timers[s.timers_used++];
}

// The timer of one timed launch: kTimeCall books it into the call's pair
// (*use_events false); the per-launch modes take a fresh pair.
int launch_timer(life_dev *d, Shard &s, int launches, TimedLaunch **t, bool *use_events) {
    *t = nullptr;
    *use_events = false;
    if (d->call_timer) {
        d->call_timer->launches += launches;
        *t = d->call_timer;
        return LIFE_OK;
    }
    if (kEnvTimingMode == kTimeOff || !d->launch_events) return LIFE_OK;
    int rc;
    *t = timer_slot(s, &rc);
    if (!*t) return rc;
    (*t)->launches = launches;
    *use_events = true;
    return LIFE_OK;
}

// Launches one stencil region on `st`; when timing is on and `timed`,
// brackets it with HIP events on that stream and books its algorithmic bytes
// (1 B read + 1 B written per BYTE cell, 2 bits per BIT cell).
int launch_region(life_dev *d, Shard &s, const life::Region &r, bool timed, hipStream_t st) {
    const uint8_t *in = s.buf[s.cur];
    uint8_t *out = s.buf[s.cur ^ 1];
    TimedLaunch *t = nullptr;
    bool ev = false;
    if (d->timing && timed) {
        CHK(launch_timer(d, s, 1, &t, &ev));
        if (ev) HIPCHK(hipEventRecord(t->a, st));
    }
    HIPCHK(life::launch_step(s.lay, in, out, s.sink, r, wrap_of(d), st));
    if (d->timing && timed && t) {  // (no timer counts it -- span-only timing, LIFE_TIMING_MODE=3: no booking)
        if (ev) HIPCHK(hipEventRecord(t->b, st));
        const bool bit = s.lay.kernel == LIFE_KERNEL_BIT;
        const int64_t cpu = bit ? 128 : 16;
        const int64_t xa = r.u0 * cpu, xb = r.u1 * cpu < s.lay.w ? r.u1 * cpu : s.lay.w;
        const double cells = (double)(xb - xa) * (double)(r.r1 - r.r0);
        d->acc_bytes += cells * (bit ? 0.25 : 2.0);
        d->acc_updates += cells;
    }
    return LIFE_OK;
}

int harvest_timers(life_dev *d) {
    for (Shard &s : d->shards) {
        HIPCHK(hipSetDevice(s.device));
        for (size_t i = 0; i < s.timers_used; i++) {
            HIPCHK(hipEventSynchronize(s.timers[i].b));
            float ms = 0.f;
            HIPCHK(hipEventElapsedTime(&ms, s.timers[i].a, s.timers[i].b));
            d->acc_ms += ms;
            d->acc_launches += s.timers[i].launches;
        }
        s.timers_used = 0;
    }
    return LIFE_OK;
}

PhaseEvents *phase_slot(Shard &s, int *rc) {
    *rc = LIFE_OK;
    if (s.phases_used == s.phases.size()) {
        PhaseEvents p;
        for (hipEvent_t *e : {&p.ring0, &p.ring1, &p.int0, &p.int1, &p.halo0, &p.halo1, &p.end})
            if (hipEventCreate(e) != hipSuccess) {
                set_err("hipEventCreate failed");
                *rc = LIFE_EHIP;
                return nullptr;
            }
        s.phases.push_back(p);
    }
    return &s.phases[s.phases_used++];
}

int harvest_phases(life_dev *d) {
    for (Shard &s : d->shards) {
        HIPCHK(hipSetDevice(s.device));
        for (size_t i = 0; i < s.phases_used; i++) {
            const PhaseEvents &p = s.phases[i];
            for (hipEvent_t e : {p.end, p.ring1, p.int1, p.halo1}) HIPCHK(hipEventSynchronize(e));
            float r = 0.f, n = 0.f, h = 0.f, b = 0.f;
            HIPCHK(hipEventElapsedTime(&r, p.ring0, p.ring1));
            HIPCHK(hipEventElapsedTime(&n, p.int0, p.int1));
            HIPCHK(hipEventElapsedTime(&h, p.halo0, p.halo1));
            HIPCHK(hipEventElapsedTime(&b, p.ring0, p.end));
            d->ph_ring += r;
            d->ph_int += n;
            d->ph_halo += h;
            d->ph_block += b;
            d->ph_blocks++;
        }
        s.phases_used = 0;
    }
    return LIFE_OK;
}

bool temporal(const life_dev *d) { return d->shards[0].lay.generations_per_exchange > 1; }

// Launches up to 4 tile regions of the temporal stencil as ONE kernel on
// `st` (m generations, cur -> nxt), optionally timed.
int launch_tiles(life_dev *d, Shard &s, const life::TileRegion *r, int nreg, int m, bool timed, hipStream_t st,
                 life::Extend ext_ = life::Extend{}, int64_t concurrent = 0) {
    const uint8_t *in = s.buf[s.cur];
    uint8_t *out = s.buf[s.cur ^ 1];
    TimedLaunch *t = nullptr;
    bool ev = false;
    if (d->timing && timed) CHK(launch_timer(d, s, 1, &t, &ev));
    double valu = 0.0;
    // events stamped by the dispatch itself: no event packets between the
    // launches of a multi-stream step (kTimeCall's one pair per call is for
    // single-stream calls)
    const life::Extend xt = ext_;
    const bool ext = ev && (kEnvTimingMode == kTimeExt || kEnvTimingMode == kTimeCall);
    if (ev && !ext) HIPCHK(hipEventRecord(t->a, st));
    HIPCHK(life::launch_tstep(s.lay, in, out, r, nreg, m, wrap_of(d), st, &valu, ext ? t->a : nullptr,
                              ext ? t->b : nullptr, xt, concurrent));
    if (ev && !ext) HIPCHK(hipEventRecord(t->b, st));
    if (d->timing && timed && t) {  // (no timer counts it -- span-only timing, LIFE_TIMING_MODE=3: no booking)
        const life::TileGeom g = life::tile_geom(life::extended_layout(s.lay, xt), m);
        for (int k = 0; k < nreg; k++) {
            // owned cells only (a deep-halo pass's apron rows are not counted)
            const int64_t xa = r[k].tx0 * g.lanes * g.cells, xb = std::min(r[k].tx1 * g.lanes * g.cells, s.lay.w);
            const int64_t ya = std::max(r[k].ty0 * g.rows - xt.y, (int64_t)0),
                          yb = std::min(r[k].ty1 * g.rows - xt.y, s.lay.h);
            if (xb > xa && yb > ya) {
                // compulsory HBM bytes of the launch: each owned cell's bit is
                // read once and written once per m-generation pass (0.25 B),
                // not once per generation -- that is the point of the blocking
                const double cells = (double)(xb - xa) * (double)(yb - ya);
                d->acc_bytes += cells * (s.lay.kernel == LIFE_KERNEL_BIT ? 0.25 : 2.0);
                d->acc_updates += cells * (double)m;
            }
        }
        d->acc_valu += valu;  // as tiled: tiles, banded items, half-height tail tiles
    }
    return LIFE_OK;
}

// LIFE_INTERIOR_TAIL (0/1, default 0, read once; A/B knob): 1 = the
// exchange pass's interior launch takes the banded half-height tail, planned
// with the ring's tiles counted as holding their slots; 0 = as in round 5,
// only a full-width interior (a row strip's) splits, planned alone.  Off by default: in
// r06f's ABAB loopback lines it shortened the interior by 4-9 % but the halo
// behind the ring was exposed longer by as much (the half tiles take the
// slots the RCCL kernels would get once the ring drains), so
// the block did not get shorter.
static bool interior_tail() {
    static const bool v = [] {
        const char *e = getenv("LIFE_INTERIOR_TAIL");
        return e ? atoi(e) != 0 : false;
    }();
    return v;
}

// The overlapped schedule of one exchange block (round 5, profiles/r05/c-d
// kernel traces): the ring tiles, then the halo of their new state (pack,
// RCCL / copies, unpack) on the compute stream `stream`, back to back in one
// hardware queue; the interior tiles concurrently on `stream2`.  The block
// ends with ONE cross-queue wait, placed on the stream whose work is
// predicted to end first: a queue that reaches a wait whose event has
// already fired passes it at once, while one that must sleep on it woke
// ~20 us after the event on MI355X (the halo's end to the next pass, r05d).
// So the work carries on in the queue predicted to finish last: the halo's
// (`stream`, which then waits for the interior) when the block is under
// three rounds of tiles -- small shards, where ring + halo outlast the
// interior (RCCL loopback, r05e: 16384x32768 1.1 rounds, 32768^2 2.2 rounds
// +8 % on the halo side; 32768x65536 4.3 rounds +1.7 % on the interior's) --
// else the interior's (`stream2` waits for the halo and the two handles are
// swapped, so `stream` always names the one that carries on).
// LIFE_JOIN (read once): 0 auto, 1 always the halo's stream, 2 always the
// interior's.
int join_mode() {
    static const int v = [] {
        const char *e = getenv("LIFE_JOIN");
        const int m = e ? atoi(e) : 0;
        return m >= 0 && m <= 2 ? m : 0;
    }();
    return v;
}

// Phase timing of one overlapped block (timing on): ring0 before the ring
// kernels on the compute stream, ring1 after them, halo0 / halo1 around the
// halo on the same stream; the interior kernel is bracketed on the second
// compute stream; `end` after the join on the stream that carries on.
int phase_begin(life_dev *d, Shard &s, PhaseEvents **pe) {
    *pe = nullptr;
    if (!d->timing || !d->phase_events) return LIFE_OK;
    int rc;
    *pe = phase_slot(s, &rc);
    if (!*pe) return rc;
    HIPCHK(hipEventRecord((*pe)->ring0, s.stream));
    return LIFE_OK;
}
int phase_ring(Shard &s, PhaseEvents *pe) {
    if (pe) {
        HIPCHK(hipEventRecord(pe->ring1, s.stream));
        HIPCHK(hipEventRecord(pe->halo0, s.stream));
    }
    return LIFE_OK;
}
// halo_side[si]: shard si carries on in its halo's stream (see join_mode).
int phase_end(life_dev *d, const std::vector<PhaseEvents *> &pe, const std::vector<char> &halo_side) {
    for (size_t si = 0; si < d->shards.size(); ++si) {
        Shard &s = d->shards[si];
        HIPCHK(hipSetDevice(s.device));
        if (pe[si]) HIPCHK(hipEventRecord(pe[si]->halo1, s.stream));
        // (priorities belong to the stream roles: no swap then)
        if (halo_side[si] || stream_priorities()) {
            HIPCHK(hipEventRecord(s.ev_int, s.stream2));
            HIPCHK(hipStreamWaitEvent(s.stream, s.ev_int, 0));
        } else {
            HIPCHK(hipEventRecord(s.ev_halo, s.stream));
            HIPCHK(hipStreamWaitEvent(s.stream2, s.ev_halo, 0));
            std::swap(s.stream, s.stream2);
        }
        if (pe[si]) HIPCHK(hipEventRecord(pe[si]->end, s.stream));
    }
    return LIFE_OK;
}
// The auto rule of join_mode: ring + interior tiles under three rounds of
// resident workgroups.
bool carry_on_halo_side(int64_t block_items, int slots) {
    const int m = join_mode();
    if (m != 0) return m == 1;
    return slots > 0 && block_items < 3 * (int64_t)slots;
}

// Generations the next temporal launch runs (remaining > 0): a step call
// is split into ceil(remaining / bmax) launches of nearly equal size (a
// 20-generation call runs 10 + 10, not 16 + 4); bmax = K capped by the block
// size.
int next_block(const life_dev *d, int64_t remaining) {
    const int K = d->shards[0].lay.generations_per_exchange;
    int bmax = std::min(K, 32);
    if (d->block_gens > 0) bmax = std::min(bmax, d->block_gens);
    const int64_t n = (remaining + bmax - 1) / bmax;
    return (int)((remaining + n - 1) / n);
}

// m <= K generations of the temporally blocked stencil on every shard, then
// one K-deep halo exchange.  Partitioned shards: the boundary ring (one
// multi-region launch) runs on the compute stream, the exchange of its new
// state on the comm stream, and the interior concurrently on the second
// compute stream.  The ring holds every tile that produces a cell the
// exchange sends: rows [0, K) and [h-K, h), columns [0, xa) and [w-xa, w)
// (xa = the x-apron, one lane column).  A self-wrapped x axis
// (life::self_wrap_x) counts as partitioned: its "exchange" is the column
// copy.
// Deep halo applies (generation_block): bit tiles, a partitioned axis, no
// self-wrapped x.
bool deep_halo(const life_dev *d) {
    return d->deep && d->kernel == LIFE_KERNEL_BIT && temporal(d) && (part(d, 0) || part(d, 1)) && !self_wrap_x(d);
}

int generation_block(life_dev *d, int m, bool last) {
    const bool rx = part(d, 0) || self_wrap_x(d), ry = part(d, 1);
    // Deep halo (bit tiles, partitioned axes, no self-wrapped x): the
    // exchange of a K-deep halo is skipped while the aprons still hold the
    // next pass's ghost cells -- this pass then also advances the apron cells
    // the next one reads (life::Extend) -- and runs after the pass whose
    // successor would outrun them.  A 20-generation call of two 10-generation
    // passes exchanges once instead of twice (life_cart.c:73-74 exchanges
    // every generation).
    // step_body cuts a call into passes that end on the K boundary, so the
    // exchange runs (overlapped with this pass) when the aprons are used up,
    // or at the call's end when the next call's first pass could not fit.
    const int K = d->shards[0].lay.generations_per_exchange;
    const bool deep = deep_halo(d);
    // aprons that no longer cover this pass (a longer pass than planned for,
    // or the deep halo switched off while they were part-used): refill first
    if (d->since + m > K) CHK(exchange(d, 0, false));
    const int bmax = std::min(std::min(K, 32), d->block_gens > 0 ? d->block_gens : 32);
    if (deep && d->since + m < K && !(last && d->since + m + bmax > K)) {
        life::Extend xt;
        xt.y = ry ? K - d->since - m : 0;
        xt.x = part(d, 0);
        for (Shard &s : d->shards) {
            HIPCHK(hipSetDevice(s.device));
            const life::TileGeom g = life::tile_geom(life::extended_layout(s.lay, xt), m);
            const life::TileRegion all{0, g.ntx, 0, g.nty};
            CHK(launch_tiles(d, s, &all, 1, m, true, s.stream, xt));
        }
        for (Shard &s : d->shards) s.cur ^= 1;
        d->since += m;
        return LIFE_OK;
    }
    std::vector<PhaseEvents *> pe(d->shards.size(), nullptr);
    std::vector<char> halo_side(d->shards.size(), 0);
    for (size_t si = 0; si < d->shards.size(); ++si) {
        Shard &s = d->shards[si];
        HIPCHK(hipSetDevice(s.device));
        const int64_t K = s.lay.generations_per_exchange;
        // grid of tiles: NX x NY, tile height uh; tile columns [0, ca) and
        // [cb, NX) hold the x-ring
        const life::TileGeom g = life::tile_geom(s.lay, m);
        const int64_t NX = g.ntx, NY = g.nty, uh = g.rows;
        int64_t ca = 0, cb = NX;
        if (rx) {  // the x-ring: tile columns holding cells [0, xa) and [w - xa, w)
            ca = 1;
            cb = std::max(std::min(((s.lay.w - s.lay.xapron) / g.cells) / g.lanes, NX), ca);
        }
        auto launch = [&](const life::TileRegion *r, int n, bool timed, hipStream_t st) -> int {
            return launch_tiles(d, s, r, n, m, timed, st);
        };
        if (!(rx || ry) || !d->overlap) {
            // one launch of every tile; a partitioned shard without overlap
            // (LIFE_OPT_OVERLAP 0) then exchanges its halo on the compute
            // stream, after the launch
            const life::TileRegion all{0, NX, 0, NY};
            CHK(launch(&all, 1, true, s.stream));
            continue;
        }
        // unit rows [0, ra) and [rb, NY), unit columns [0, ca) and [cb, NX)
        int64_t ra = 0, rb = NY;
        if (ry) {
            ra = std::min((K + uh - 1) / uh, NY);
            rb = std::max(std::min((s.lay.h - K) / uh, NY), ra);
        }
        life::TileRegion ring[4];
        int n = 0;
        if (ra > 0) ring[n++] = life::TileRegion{0, NX, 0, ra};
        if (rb < NY) ring[n++] = life::TileRegion{0, NX, rb, NY};
        if (rb > ra) {
            if (ca > 0) ring[n++] = life::TileRegion{0, ca, ra, rb};
            if (cb < NX) ring[n++] = life::TileRegion{cb, NX, ra, rb};
        }
        // the interior (second stream) starts after everything already on
        // the compute stream: a deep-halo pass before this one is not joined
        // into the other streams
        HIPCHK(hipEventRecord(s.ev_entry, s.stream));
        HIPCHK(hipStreamWaitEvent(s.stream2, s.ev_entry, 0));
        CHK(phase_begin(d, s, &pe[si]));
        CHK(launch(ring, n, false, s.stream));
        CHK(phase_ring(s, pe[si]));
        const life::TileRegion inner{ca, cb, ra, rb};
        int64_t ring_items = 0;
        for (int k = 0; k < n; k++) ring_items += life::region_items(g, ring[k]);
        const int64_t items = life::region_items(g, inner) + ring_items;
        halo_side[si] = carry_on_halo_side(items, life::tile_slots(s.lay)) ? 1 : 0;
        if (pe[si]) HIPCHK(hipEventRecord(pe[si]->int0, s.stream2));
        // LIFE_INTERIOR_TAIL=1: the interior's launch-tail plan counts the
        // ring's tiles, dispatched just before it, as holding their slots
        // (16384 x 32768's 584 interior tiles beside 249 ring tiles are one
        // round plus a tail); default: only a row strip's full-width interior
        // splits its tail, planned alone (round 5)
        const int64_t conc = interior_tail() ? ring_items : (ca == 0 && cb == NX ? 0 : -1);
        if (rb > ra && cb > ca) CHK(launch_tiles(d, s, &inner, 1, m, true, s.stream2, life::Extend{}, conc));
        if (pe[si]) HIPCHK(hipEventRecord(pe[si]->int1, s.stream2));
    }
    if (!(rx || ry)) {
        for (Shard &s : d->shards) s.cur ^= 1;
        return LIFE_OK;
    }
    if (!d->overlap) {
        for (Shard &s : d->shards) s.cur ^= 1;
        return exchange(d, 0, false);
    }
    CHK(exchange(d, 1, false));  // halo of nxt, behind the ring on the compute streams
    CHK(phase_end(d, pe, halo_side));
    for (Shard &s : d->shards) s.cur ^= 1;
    return LIFE_OK;
}

// One generation on every local shard (one-cell aprons).
int generation(life_dev *d) {
    const bool rx = part(d, 0), ry = part(d, 1);
    if (!d->overlap || !(rx || ry)) {
        for (Shard &s : d->shards) {
            HIPCHK(hipSetDevice(s.device));
            CHK(launch_region(d, s, life::Region{0, s.lay.units, 0, s.lay.h}, true, s.stream));
        }
        for (Shard &s : d->shards) s.cur ^= 1;
        return exchange(d, 0, false);
    }
    // Ring first (cells whose 3x3 neighbourhood reaches a partitioned axis'
    // apron) on the compute stream, then the halo of the new state on the
    // comm stream; the interior runs concurrently on the second compute stream.
    std::vector<PhaseEvents *> pe(d->shards.size(), nullptr);
    for (size_t si = 0; si < d->shards.size(); ++si) {
        Shard &s = d->shards[si];
        HIPCHK(hipSetDevice(s.device));
        // The interior (second stream) starts after everything on the compute
        // stream: phase_end joined the previous generation into ONE stream
        // only (and may have swapped the handles), so without this fence the
        // next interior could start beside the previous interior (still
        // reading cur) or beside the previous ring + halo.
        HIPCHK(hipEventRecord(s.ev_entry, s.stream));
        HIPCHK(hipStreamWaitEvent(s.stream2, s.ev_entry, 0));
        CHK(phase_begin(d, s, &pe[si]));
        const int64_t U = s.lay.units, H = s.lay.h;
        const int64_t ra = ry ? 1 : 0, rb = ry ? H - 1 : H;  // interior rows
        if (ry) {
            CHK(launch_region(d, s, life::Region{0, U, 0, 1}, false, s.stream));
            if (H > 1) CHK(launch_region(d, s, life::Region{0, U, H - 1, H}, false, s.stream));
        }
        if (rx && rb > ra) {
            CHK(launch_region(d, s, life::Region{0, 1, ra, rb}, false, s.stream));
            if (U > 1) CHK(launch_region(d, s, life::Region{U - 1, U, ra, rb}, false, s.stream));
        }
        CHK(phase_ring(s, pe[si]));
        const int64_t ua = rx ? 1 : 0, ub = rx ? U - 1 : U;
        if (pe[si]) HIPCHK(hipEventRecord(pe[si]->int0, s.stream2));
        if (rb > ra && ub > ua) CHK(launch_region(d, s, life::Region{ua, ub, ra, rb}, true, s.stream2));
        if (pe[si]) HIPCHK(hipEventRecord(pe[si]->int1, s.stream2));
    }
    CHK(exchange(d, 1, false));  // halo of nxt, behind the ring on the compute streams
    // one-generation launches are short: carry on in the interior's stream
    // unless LIFE_JOIN says otherwise
    CHK(phase_end(d, pe, std::vector<char>(d->shards.size(), join_mode() == 1 ? 1 : 0)));
    for (Shard &s : d->shards) s.cur ^= 1;
    return LIFE_OK;
}

// Seconds a rank-mode collective may take before it is declared dead
// (LIFE_COMM_TIMEOUT_S, default 600): a peer that died or never joined would
// otherwise leave this rank spinning in an RCCL kernel forever.
double comm_timeout_s() {
    static const double t = [] {
        const char *e = getenv("LIFE_COMM_TIMEOUT_S");
        const double v = e ? atof(e) : 0.0;
        return v > 0.0 ? v : 600.0;
    }();
    return t;
}

// hipStreamSynchronize with a deadline: polls the stream; on timeout aborts
// the shard's communicator (which ends RCCL kernels stuck on a missing peer)
// and fails with a message naming the operation.
int bounded_sync(Shard &s, const char *what, int peer, hipStream_t st = nullptr) {
    if (!st) st = s.stream;
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t e = hipStreamQuery(st);
        if (e == hipSuccess) return LIFE_OK;
        if (e != hipErrorNotReady) {
            set_err("%s (peer %d): %s", what, peer, hipGetErrorString(e));
            return LIFE_EHIP;
        }
        const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (dt > comm_timeout_s()) {
            if (s.comm) {
                (void)ncclCommAbort(s.comm);
                s.comm = nullptr;
            }
            set_err("%s: rank %d waited %.0f s for peer %d (LIFE_COMM_TIMEOUT_S); communicator aborted", what,
                    s.rank, dt, peer);
            return LIFE_ERCCL;
        }
        // busy-poll the first 20 ms (a step's end is seen within a few us,
        // as wait_stream), then back off to 1 ms naps
        if (dt > 0.02) std::this_thread::sleep_for(std::chrono::microseconds(1000));
    }
}

// Rank mode: a collective check that every rank passes the same `value`
// (an int64 max all-reduce of {value, -value}); bounded like the barrier.
int agree_all_ranks(life_dev *d, int value, const char *what) {
    for (Shard &s : d->shards) {
        if (!s.comm) continue;
        HIPCHK(hipSetDevice(s.device));
        int64_t *h = reinterpret_cast<int64_t *>(s.h_count);
        h[0] = value;
        h[1] = -(int64_t)value;
        HIPCHK(hipMemcpyAsync(s.d_count, h, 2 * sizeof(int64_t), hipMemcpyHostToDevice, s.stream));
        NCCLCHK(ncclAllReduce(s.d_count, s.d_count, 2, ncclInt64, ncclMax, s.comm, s.stream));
        HIPCHK(hipMemcpyAsync(h, s.d_count, 2 * sizeof(int64_t), hipMemcpyDeviceToHost, s.stream));
        CHK(bounded_sync(s, what, -1));
        const int64_t hi = h[0], lo = -h[1];
        if (hi != lo) {
            set_err("%s is collective in rank mode: ranks passed %lld .. %lld", what, (long long)lo, (long long)hi);
            return LIFE_EINVAL;
        }
    }
    return LIFE_OK;
}

int create_common(life_dev *d, const std::vector<int> &ranks, const std::vector<int> &devices) {
    for (size_t i = 0; i < ranks.size(); i++) {
        d->shards.emplace_back();
        Shard &s = d->shards.back();
        s.rank = ranks[i];
        s.device = devices[i];
        const int rc = life_layout_query(d->nx, d->ny, d->dims[0], d->dims[1], s.rank, d->kernel, &s.lay);
        if (rc != LIFE_OK) {
            set_err("layout: nx=%lld ny=%lld dims=%dx%d rank %d kernel %d", (long long)d->nx,
                    (long long)d->ny, d->dims[0], d->dims[1], s.rank, d->kernel);
            return rc;
        }
    }
    for (Shard &s : d->shards) CHK(shard_alloc(d, s));
    return LIFE_OK;
}

}  // namespace

static int flow_prewarm(life_dev *d);

// The launch-tail plans (life::tail_plan) of the passes this device's step
// calls will launch, computed up front: a plan's first search costs ~50 us of
// host time, which a timed call's first launch would otherwise wait for
// (deep-halo passes: every extension 0 .. K - m).
static void tail_prewarm(const life_dev *d) {
    const int mmax = d->block_gens > 0 ? d->block_gens : 12;
    for (size_t i = 0; i < d->shards.size(); ++i) {
        bool seen = false;  // identical blocks share their plans (cached by shape)
        for (size_t j = 0; j < i; ++j)
            seen |= d->shards[j].lay.w == d->shards[i].lay.w && d->shards[j].lay.h == d->shards[i].lay.h;
        if (!seen) life::prewarm_tail_plans(d->shards[i].lay, mmax, part(d, 1));
    }
}

extern "C" {

const char *life_last_error(void) { return g_err.c_str(); }

int life_dev_create_ex(int64_t nx, int64_t ny, int nshards, int dims0, int dims1, int kernel,
                       int transport, life_dev **out) {
    if (!out || nx <= 0 || ny <= 0 || nshards <= 0) return LIFE_EINVAL;
    *out = nullptr;
    int dims[2] = {dims0, dims1};
    if (dims0 <= 0 || dims1 <= 0) life_dims_create(nshards, dims);
    if (dims[0] * dims[1] != nshards) {
        set_err("dims %dx%d != %d shards", dims[0], dims[1], nshards);
        return LIFE_EINVAL;
    }
    int ndev = 0;
    {
        hipError_t e = hipGetDeviceCount(&ndev);
        if (e != hipSuccess || ndev <= 0) {
            set_err("no HIP device: %s", hipGetErrorString(e));
            return LIFE_EHIP;
        }
    }
    life_dev *d = new life_dev;
    d->nx = nx;
    d->ny = ny;
    d->dims[0] = dims[0];
    d->dims[1] = dims[1];
    d->world = nshards;
    d->kernel = kernel;
    d->block_gens = default_block_gens(kernel);
    std::vector<int> ranks, devices;
    for (int i = 0; i < nshards; i++) {
        ranks.push_back(i);
        devices.push_back(i % ndev);
    }
    const bool distinct = nshards <= ndev;
    if (transport == LIFE_XPORT_AUTO) transport = (distinct && nshards > 1) ? LIFE_XPORT_RCCL : LIFE_XPORT_LOCAL;
    if (transport == LIFE_XPORT_RCCL && !distinct) {
        set_err("RCCL transport needs one device per shard (%d shards, %d devices)", nshards, ndev);
        delete d;
        return LIFE_EINVAL;
    }
    d->transport = transport;
    int rc = create_common(d, ranks, devices);
    // RCCL: one communicator rank per shard, all driven by this process
    // (ncclCommInitAll; the halo phases group every shard's sends / recvs in
    // one ncclGroupStart/End).  A single shard gets a one-device communicator
    // too, so LIFE_OPT_LOOPBACK runs this exact path on a one-GPU box.
    if (rc == LIFE_OK && transport == LIFE_XPORT_RCCL) {
        std::vector<ncclComm_t> comms(nshards);
        ncclResult_t r = ncclCommInitAll(comms.data(), nshards, devices.data());
        if (r != ncclSuccess) {
            set_err("ncclCommInitAll: %s", ncclGetErrorString(r));
            rc = LIFE_ERCCL;
        } else {
            for (int i = 0; i < nshards; i++) d->shards[i].comm = comms[i];
        }
    }
    if (rc == LIFE_OK && transport == LIFE_XPORT_LOCAL && nshards > 1) {
        for (int a = 0; a < ndev && a < nshards; a++)
            for (int b = 0; b < ndev && b < nshards; b++)
                if (a != b) {
                    (void)hipSetDevice(a);
                    (void)hipDeviceEnablePeerAccess(b, 0);  // already-enabled is fine
                }
        (void)hipGetLastError();
    }
    if (rc != LIFE_OK) {
        life_dev_destroy(d);
        return rc;
    }
    // not fatal: the first dataflow call allocates and launches as it would
    if (flow_prewarm(d) != LIFE_OK) (void)hipGetLastError();
    tail_prewarm(d);
    *out = d;
    return LIFE_OK;
}

int life_dev_create(int64_t nx, int64_t ny, int nshards, int kernel, life_dev **out) {
    return life_dev_create_ex(nx, ny, nshards, 0, 0, kernel, LIFE_XPORT_AUTO, out);
}

int life_get_unique_id(uint8_t unique_id[128]) {
    ncclUniqueId id;
    NCCLCHK(ncclGetUniqueId(&id));
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    memcpy(unique_id, &id, sizeof id);
    return LIFE_OK;
}

int life_dev_create_rank(int64_t nx, int64_t ny, int kernel, int rank, int world, int dims0, int dims1,
                         const uint8_t unique_id[128], int device, life_dev **out) {
    if (!out || nx <= 0 || ny <= 0 || world <= 0 || rank < 0 || rank >= world) return LIFE_EINVAL;
    *out = nullptr;
    int dims[2] = {dims0, dims1};
    if (dims0 <= 0 || dims1 <= 0) life_dims_create(world, dims);
    if (dims[0] * dims[1] != world) return LIFE_EINVAL;
    life_dev *d = new life_dev;
    d->nx = nx;
    d->ny = ny;
    d->dims[0] = dims[0];
    d->dims[1] = dims[1];
    d->world = world;
    d->kernel = kernel;
    d->block_gens = default_block_gens(kernel);
    d->rank_mode = true;
    d->transport = LIFE_XPORT_RCCL;
    int rc = create_common(d, {rank}, {device});
    // A communicator whenever the caller hands a unique id, world 1 included
    // (then only the census all-reduce uses it; that is how a one-GPU box
    // exercises RCCL initialisation in the torchrun process set-up).
    if (rc == LIFE_OK && (world > 1 || unique_id)) {
        if (!unique_id) {
            rc = LIFE_EINVAL;
        } else {
            ncclUniqueId id;
            memcpy(&id, unique_id, sizeof id);
            (void)hipSetDevice(device);
            ncclResult_t r = ncclCommInitRank(&d->shards[0].comm, world, id, rank);
            if (r != ncclSuccess) {
                set_err("ncclCommInitRank(rank %d/%d): %s", rank, world, ncclGetErrorString(r));
                rc = LIFE_ERCCL;
            }
        }
    }
    if (rc != LIFE_OK) {
        life_dev_destroy(d);
        return rc;
    }
    // not fatal: the first dataflow call allocates and launches as it would
    if (flow_prewarm(d) != LIFE_OK) (void)hipGetLastError();
    tail_prewarm(d);
    *out = d;
    return LIFE_OK;
}

int life_dev_upload(life_dev *d, const uint8_t *grid) {
    if (!d || !grid) return LIFE_EINVAL;
    for (Shard &s : d->shards) {
        const life_layout &L = s.lay;
        HIPCHK(hipSetDevice(s.device));
        uint8_t *stage = nullptr;
        HIPCHK(hipMalloc(&stage, (size_t)(L.w * L.h)));
        // `grid` is the caller's pageable memory: the copy is ordered on the
        // shard's stream (not the null stream, which does not order against
        // the non-blocking shard streams) and waited for before this call
        // returns, so the caller may reuse `grid` at once.
        HIPCHK(hipMemcpy2DAsync(stage, (size_t)L.w, grid + L.y0 * d->nx + L.x0, (size_t)d->nx, (size_t)L.w,
                                (size_t)L.h, hipMemcpyHostToDevice, s.stream));
        HIPCHK(hipStreamSynchronize(s.stream));
        HIPCHK(life::launch_import_block(L, stage, s.buf[s.cur], s.stream));
        HIPCHK(hipStreamSynchronize(s.stream));
        HIPCHK(hipFree(stage));
    }
    CHK(exchange(d, 0, false));
    return life_dev_sync(d);
}

int life_dev_fill_random(life_dev *d, uint64_t seed, uint32_t thr32) {
    if (!d) return LIFE_EINVAL;
    uint64_t z = seed + 0x9E3779B97F4A7C15ull;  // key = splitmix64(seed)
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    const uint64_t key = z ^ (z >> 31);
    for (Shard &s : d->shards) {
        HIPCHK(hipSetDevice(s.device));
        HIPCHK(life::launch_fill_random(s.lay, d->nx, key, thr32, s.buf[s.cur], s.stream));
    }
    CHK(exchange(d, 0, false));
    return LIFE_OK;
}

// A single-shard grid small enough for one CU's LDS runs every generation of
// the call in one resident-workgroup launch (life_kernels.hip, small_kernel).
// Mode 1 (default) windows the VGPR kernel over several CUs when one
// workgroup would need strips of 4 rows or more (p46gun_big 500^2: 10 rows,
// 212 -> 632 Gcell/s windowed); mode 3 windows whenever the shape allows.
static life::RegWinPlan win_plan(const life_dev *d) {
    const life_layout &L = d->shards[0].lay;
    if (d->small_mode == 3 || (d->small_mode == 1 && life::reg_small_rows(L) >= 4))
        return life::reg_win_plan(L, d->win_rows, d->win_halo);
    return life::RegWinPlan{};
}

static bool small_grid(const life_dev *d) {
    if (d->world != 1 || d->shards.size() != 1 || d->small_mode == 0 || d->loop != 0) return false;
    const life_layout &L = d->shards[0].lay;
    if (win_plan(d).blocks > 0) return true;
    return (d->small_mode != 2 && life::reg_small_rows(L) > 0) ||
           life::small_lds_bytes(L) <= life::kSmallMaxLds;
}

static int step_small(life_dev *d, int64_t generations) {
    Shard &s = d->shards[0];
    HIPCHK(hipSetDevice(s.device));
    TimedLaunch *t = nullptr;
    if (d->timing) {
        // ONE event pair around the call's launches: events between the
        // windowed kernel's ~9 us launches measured 45 % slower (gaps)
        int rc;
        t = timer_slot(s, &rc);
        if (!t) return rc;
        HIPCHK(hipEventRecord(t->a, s.stream));
    }
    const life::RegWinPlan wp = win_plan(d);
    int launches = 1;
    if (wp.blocks > 0) {
        // K generations per launch, buffers swapped per launch; between the
        // launches of the call the grid stays in natural 32-cell words
        launches = 0;
        for (int64_t g = 0; g < generations; g += wp.K, ++launches) {
            const int m = (int)(generations - g < wp.K ? generations - g : wp.K);
            HIPCHK(life::launch_reg_win(s.lay, wp, s.buf[s.cur], s.buf[s.cur ^ 1], m, s.stream, g > 0,
                                        g + m < generations));
            s.cur ^= 1;
        }
    } else {
        if (d->small_mode != 2 && life::reg_small_rows(s.lay) > 0)
            HIPCHK(life::launch_reg_small(s.lay, s.buf[s.cur], s.buf[s.cur ^ 1], generations, s.stream));
        else
            HIPCHK(life::launch_small(s.lay, s.buf[s.cur], s.buf[s.cur ^ 1], generations, s.stream));
        s.cur ^= 1;
    }
    if (t) {
        HIPCHK(hipEventRecord(t->b, s.stream));
        t->launches = launches;  // stats: mean per launch
        // CU-resident: HBM sees one import and one export of the grid per launch
        const double cells = (double)s.lay.w * (double)s.lay.h;
        d->acc_bytes += (double)launches * cells * (s.lay.kernel == LIFE_KERNEL_BIT ? 0.25 : 2.0);
        d->acc_updates += cells * (double)generations;
    }
    return LIFE_OK;
}

// Whole passes of the dataflow tiles (life::launch_tflow) for a step call of
// `generations` on a single shard whose axes both wrap in the stencil;
// returns the generations it queued (a multiple of the pass size m), 0 when
// the call takes the per-launch path.
// The dataflow form a single-shard bit device runs its passes of m
// generations in (1 / 2, the hand-off forms), or 0 (per-launch tiles).
static int flow_form(const life_dev *d, int *m_out) {
    if (!d->flow || d->shards.size() != 1 || d->world != 1 || part(d, 0) || part(d, 1) || self_wrap_x(d) ||
        d->kernel != LIFE_KERNEL_BIT)
        return 0;
    const life_layout &L = d->shards[0].lay;
    int m = std::min(L.generations_per_exchange, 32);
    if (d->block_gens > 0) m = std::min(m, d->block_gens);
    *m_out = m;
    if (!life::flow_ok(L, m)) return 0;
    // automatic: the dataflow form (write-through hand-off) when a pass is
    // under kFlowAutoRounds rounds of resident workgroups -- 32768^2 (2.2
    // rounds of 768) +8 %, 32768 x 65536 (4.3) +1 %, 65536^2 (8.6) -3 %
    // (profiles/r05/a) -- except a pass of 1 to 1.5 rounds: it runs as one
    // full round plus the banded half-height tail (launch_tstep), its tiles
    // all finish together and the dataflow form has nothing to pipeline
    // (16384 x 32768, 833 tiles on 768 slots: per-launch tiles 83.2-83.8 T
    // against 73.7-75.2 T, profiles/r06/d; under one round the dataflow
    // form overlaps the passes in the idle slots)
    if (d->flow == 3) {
        const double rounds = (double)life::flow_items_per_pass(L, m) / (double)std::max(life::flow_slots(L), 1);
        return rounds < kFlowAutoRounds && !(rounds >= 1.0 && rounds < 1.5) ? 1 : 0;
    }
    return d->flow;
}

// Grows the shard's dataflow scratch (queue head, error word, per-tile pass
// counts) to the tile grid of m generations per pass.
static int flow_scratch(Shard &s, int m) {
    const life::TileGeom g = life::tile_geom(s.lay, m);
    const size_t words = (size_t)(2 + g.ntx * g.nty);
    if (words <= s.flow_words) return LIFE_OK;
    if (s.flow) (void)hipFree(s.flow);
    s.flow = nullptr;
    s.flow_words = 0;
    if (hipSetDevice(s.device) != hipSuccess || hipMalloc(&s.flow, words * sizeof(unsigned int)) != hipSuccess ||
        hipMemsetAsync(s.flow, 0, 2 * sizeof(unsigned int), s.stream) != hipSuccess) {
        set_err("dataflow scratch (%zu words)", words);
        return LIFE_ENOMEM;
    }
    s.flow_words = words;
    return LIFE_OK;
}

// At creation: the scratch and one empty launch of the dataflow instance the
// device's first dataflow call will run, so that call does not pay the
// kernel's first launch (~140 us before configs[2]'s dataflow launch inside
// its timed call, profiles/r05/l trace_32768).
static int flow_prewarm(life_dev *d) {
    int m = 0;
    const int form = flow_form(d, &m);
    if (form == 0) return LIFE_OK;
    Shard &s = d->shards[0];
    CHK(flow_scratch(s, m));
    HIPCHK(hipSetDevice(s.device));
    HIPCHK(life::prewarm_tflow(s.lay, m, form, s.flow, s.stream));
    HIPCHK(hipStreamSynchronize(s.stream));
    return LIFE_OK;
}

static int step_flow(life_dev *d, int64_t generations, int64_t *done) {
    *done = 0;
    int m = 0;
    const int form = flow_form(d, &m);
    if (form == 0) return LIFE_OK;
    Shard &s = d->shards[0];
    const life_layout &L = s.lay;
    const int64_t passes = generations / m;
    // a call of 2-3 passes ran 0.58 ms per 10-generation pass against 0.42 for
    // the per-launch tiles (profiles/r03/r4d); the dataflow form pays from
    // about 4 passes (0.474 ms per 12-generation pass in long runs)
    if (passes < kFlowMinPasses) return LIFE_OK;
    CHK(flow_scratch(s, m));
    HIPCHK(hipSetDevice(s.device));
    // The queue head is a 32-bit counter every resident workgroup bumps once
    // past the last item: split the passes so that items + grid stays below
    // 2^31 per launch (life::flow_chunk_passes), flipping the buffer parity
    // per chunk.
    const int64_t tiles = life::flow_items_per_pass(L, m);
    const int64_t per = life::flow_chunk_passes(tiles, life::flow_slots(L), d->flow_chunk);
    if (per < 1) return LIFE_OK;  // a grid too large for one pass per launch: per-launch tiles
    for (int64_t left = passes; left > 0;) {
        const int64_t n = std::min(left, per);
        TimedLaunch *t = nullptr;
        bool ev = false;
        if (d->timing) CHK(launch_timer(d, s, (int)n, &t, &ev));  // stats: mean per pass
        const bool ext = ev && kEnvTimingMode == kTimeExt;
        if (ev && !ext) HIPCHK(hipEventRecord(t->a, s.stream));
        HIPCHK(life::launch_tflow(L, s.buf[s.cur], s.buf[s.cur ^ 1], m, n, s.flow, s.flow + 2, wrap_of(d),
                                  form, s.stream, ext ? t->a : nullptr, ext ? t->b : nullptr));
        if (ev && !ext) HIPCHK(hipEventRecord(t->b, s.stream));
        // work is booked only beside a timer that counts the launch (as
        // launch_tiles / launch_region: LIFE_TIMING_MODE=3 and span-only
        // timing book nothing, so bytes / updates per launch stay consistent)
        if (d->timing && t) {
            const double cells = (double)L.w * (double)L.h;
            d->acc_bytes += (double)n * cells * 0.25;
            d->acc_updates += (double)n * cells * (double)m;
            d->acc_valu += (double)n * (double)life::flow_items_per_pass(L, m, true) * 64.0 *
                           life::tstep_valu_per_tile_lane(m, false);
        }
        if (n & 1) s.cur ^= 1;
        left -= n;
    }
    s.flow_used = true;
    *done = passes * m;
    return LIFE_OK;
}

static int step_body(life_dev *d, int64_t generations);
static int step_call(life_dev *d, int64_t generations);

static double ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}
static void note_pass(life_dev *d, std::chrono::steady_clock::time_point t0) {
    const double ms = ms_since(t0);
    d->call_passes++;
    if (ms > d->call_pass_max_ms) d->call_pass_max_ms = ms;
}

int life_dev_step(life_dev *d, int64_t generations) {
    if (!d || generations < 0) return LIFE_EINVAL;
    if (generations == 0) return LIFE_OK;
    const auto t0 = std::chrono::steady_clock::now();
    d->call_passes = 0;
    d->call_pass_max_ms = 0.0;
    d->call_spans = false;
    const int rc = step_call(d, generations);
    d->call_host_ms = ms_since(t0);
    return rc;
}

static int step_call(life_dev *d, int64_t generations) {
    // Entry fence: the second compute stream and the comm stream start after
    // everything already queued on the compute stream (an asynchronous
    // fill_random and its halo fill, a small-grid launch, a gather's export),
    // which the overlapped schedule would otherwise race.  A single shard
    // with no partitioned or self-wrapped axis steps on the compute stream
    // alone: no fence (4 runtime calls off a ~1 ms call's critical path).
    const bool one_stream = d->shards.size() == 1 && !part(d, 0) && !part(d, 1) && !self_wrap_x(d);
    for (Shard &s : d->shards) {
        if (one_stream) break;
        HIPCHK(hipSetDevice(s.device));
        HIPCHK(hipEventRecord(s.ev_entry, s.stream));
        HIPCHK(hipStreamWaitEvent(s.stream2, s.ev_entry, 0));
        HIPCHK(hipStreamWaitEvent(s.comm_stream, s.ev_entry, 0));
    }
    // kTimeCall: one event pair around all launches of a single-stream call
    if (d->timing && one_stream && kEnvTimingMode == kTimeCall && !small_grid(d) && temporal(d)) {
        Shard &s = d->shards[0];
        int rc;
        d->call_timer = timer_slot(s, &rc);
        if (!d->call_timer) return rc;
        d->call_timer->launches = 0;
        HIPCHK(hipEventRecord(d->call_timer->a, s.stream));
        rc = step_body(d, generations);
        TimedLaunch *t = d->call_timer;
        d->call_timer = nullptr;
        if (rc != LIFE_OK) {
            // drop the half-recorded pair (no event b): a later harvest
            // would fail on it and hide this call's error
            s.timers_used--;
            return rc;
        }
        HIPCHK(hipEventRecord(t->b, s.stream));
        s.span_a = t->a;  // the call's pair is its span
        s.span_b = t->b;
        d->call_spans = true;
        return LIFE_OK;
    }
    if (!d->timing) return step_body(d, generations);
    // timing on, any other call: one event at each end of the call on every
    // shard's compute stream (the entry fence above orders the other streams
    // after the first; every schedule joins them back into it at the end)
    for (Shard &s : d->shards) {
        HIPCHK(hipSetDevice(s.device));
        if (!s.own_a) HIPCHK(hipEventCreate(&s.own_a));
        if (!s.own_b) HIPCHK(hipEventCreate(&s.own_b));
        HIPCHK(hipEventRecord(s.own_a, s.stream));
    }
    CHK(step_body(d, generations));
    for (Shard &s : d->shards) {
        HIPCHK(hipSetDevice(s.device));
        HIPCHK(hipEventRecord(s.own_b, s.stream));
        s.span_a = s.own_a;
        s.span_b = s.own_b;
    }
    d->call_spans = true;
    return LIFE_OK;
}

// The launches of one step call (life_dev_step after its entry fence).
static int step_body(life_dev *d, int64_t generations) {
    if (small_grid(d)) {
        d->last_path = LIFE_PATH_SMALL;
        constexpr int64_t kChunk = 1 << 20;  // generations per resident launch
        for (int64_t g = 0; g < generations; g += kChunk)
            CHK(step_small(d, generations - g < kChunk ? generations - g : kChunk));
        // the LDS kernel wraps inside the CU and leaves the buffer's aprons
        // stale: refresh them (a self-wrapped x axis; no-op otherwise)
        return exchange(d, 0, false);
    }
    if (temporal(d)) {
        int64_t done = 0;
        CHK(step_flow(d, generations, &done));
        d->last_path = done > 0 ? LIFE_PATH_FLOW : LIFE_PATH_TILES;
        const int K = d->shards[0].lay.generations_per_exchange;
        for (int64_t g = done; g < generations;) {
            // deep halo: equal passes up to the next exchange boundary (32 =
            // 11 + 11 + 10 at 12 generations per pass at most)
            int64_t seg = generations - g;
            if (deep_halo(d) && d->since < K) seg = std::min(seg, (int64_t)(K - d->since));
            const int m = next_block(d, seg);
            const auto t0 = std::chrono::steady_clock::now();
            CHK(generation_block(d, m, g + m >= generations));
            note_pass(d, t0);
            g += m;
        }
        return LIFE_OK;
    }
    d->last_path = LIFE_PATH_ONEGEN;
    for (int64_t g = 0; g < generations; g++) {
        const auto t0 = std::chrono::steady_clock::now();
        CHK(generation(d));
        note_pass(d, t0);
    }
    return LIFE_OK;
}

int life_dev_last_path(life_dev *d) { return d ? d->last_path : LIFE_EINVAL; }

int life_device_count(void) {
    int n = 0;
    const hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        set_err("hipGetDeviceCount: %s", hipGetErrorString(e));
        return LIFE_EHIP;
    }
    return n;
}

int life_dev_barrier(life_dev *d) {
    if (!d) return LIFE_EINVAL;
    CHK(life_dev_sync(d));
    if (d->rank_mode)
        for (Shard &s : d->shards)
            if (s.comm) {
                // an all-reduce every rank must join: no rank leaves before all arrived
                HIPCHK(hipSetDevice(s.device));
                NCCLCHK(ncclAllReduce(s.d_count, s.d_count, 1, ncclUint64, ncclSum, s.comm, s.stream));
                CHK(bounded_sync(s, "barrier all-reduce", -1));
            }
    return LIFE_OK;
}

// hipStreamSynchronize, but polling the stream for the first milliseconds:
// the blocking wait woke ~10 us after the last kernel ended (profiles/r03/r4d
// trace), 1 % of a 20-generation 65536^2 call.
static hipError_t wait_stream(hipStream_t st) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        const hipError_t e = hipStreamQuery(st);
        if (e != hipErrorNotReady) return e;
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) return hipStreamSynchronize(st);
    }
}

int life_dev_sync(life_dev *d) {
    if (!d) return LIFE_EINVAL;
    for (Shard &s : d->shards) {
        HIPCHK(hipSetDevice(s.device));
        if (d->rank_mode && s.comm) {
            // a step's halo waits on RCCL peers: a peer that died must not
            // hang this rank (LIFE_COMM_TIMEOUT_S, then ncclCommAbort)
            CHK(bounded_sync(s, "sync: compute stream", -1, s.stream));
            CHK(bounded_sync(s, "sync: interior stream", -1, s.stream2));
            CHK(bounded_sync(s, "sync: halo stream", -1, s.comm_stream));
        } else {
            HIPCHK(wait_stream(s.stream));
            HIPCHK(wait_stream(s.stream2));
            HIPCHK(wait_stream(s.comm_stream));
        }
        if (s.flow_used) {
            // a dataflow launch whose dependency wait timed out (a broken
            // hand-off): its result cannot be trusted
            unsigned int err = 0;
            HIPCHK(hipMemcpyAsync(&err, s.flow + 1, sizeof err, hipMemcpyDeviceToHost, s.stream));
            HIPCHK(hipStreamSynchronize(s.stream));
            s.flow_used = false;
            if (err) {
                HIPCHK(hipMemsetAsync(s.flow + 1, 0, sizeof err, s.stream));
                HIPCHK(hipStreamSynchronize(s.stream));
                set_err("dataflow tiles: item %u waited too long for its neighbours (state is invalid)", err - 1);
                return LIFE_ESTATE;
            }
        }
    }
    return LIFE_OK;
}

}  // extern "C"

namespace {
// Device staging of one shard's export, kept between calls (a 65536^2 grid's
// frame is 4 GiB dense / 8 GiB as VTK text: no allocation per frame).
int stage_buffer(Shard &s, size_t bytes, uint8_t **out) {
    if (s.stage_bytes < bytes) {
        if (s.stage) HIPCHK(hipFree(s.stage));
        s.stage = nullptr;
        s.stage_bytes = 0;
        HIPCHK(hipMalloc(&s.stage, bytes));
        s.stage_bytes = bytes;
    }
    *out = s.stage;
    return LIFE_OK;
}

// life_collect in one of three frame formats: DENSE 0/1 cells (export
// kernel, 1 B per cell), VTK "%d\n" cell text (vtk kernel, 2 B per cell) or
// BITS packed rows (bits kernel, LIFEBITS: bit x & 7 of byte x >> 3).  Every
// shard exports its block on the device; in-process shards copy straight into
// place, rank mode sends the blocks to the root (world-1) over RCCL in the
// order of life::gather_plan.
enum class Frame { DENSE = life::kGatherDense, VTK = life::kGatherVtk, BITS = life::kGatherBits };

int gather_impl(life_dev *d, uint8_t *out, Frame fmt) {
    const int root = d->world - 1;  // life_collect: cart rank of (dims0-1, dims1-1)
    const bool have_root = find_local(d, root) != nullptr;
    if (have_root && !out) return LIFE_EINVAL;
    CHK(life_dev_sync(d));
    std::vector<life::GatherPiece> plan((size_t)d->world);
    int64_t slot = 0;
    if (life::gather_plan(d->nx, d->ny, d->dims[0], d->dims[1], d->kernel, (int)fmt, plan.data(), d->world,
                          &slot) != d->world) {
        set_err("gather plan failed");
        return LIFE_EINVAL;
    }
    auto piece_of = [&](int rank) -> const life::GatherPiece & {
        for (const life::GatherPiece &p : plan)
            if (p.rank == rank) return p;
        return plan[0];  // unreachable: every rank has a piece
    };
    const int64_t frb = life::gather_frame_row_bytes(d->nx, (int)fmt);
    auto export_block = [&](Shard &s, uint8_t **stage) -> int {
        const life_layout &L = s.lay;
        CHK(stage_buffer(s, (size_t)piece_of(s.rank).bytes, stage));
        if (fmt == Frame::DENSE)
            HIPCHK(life::launch_export_block(L, s.buf[s.cur], *stage, s.stream));
        else if (fmt == Frame::VTK)
            HIPCHK(life::launch_vtk_block(L, s.buf[s.cur], *stage, s.stream));
        else
            HIPCHK(life::launch_bits_block(L, s.buf[s.cur], *stage, s.stream));
        return LIFE_OK;
    };
    // BITS: a byte holding cells of two blocks (a block edge at x % 8 != 0)
    // is OR-ed together from both exports; those frame bytes start at 0
    std::vector<uint8_t> tmp;
    // `out` is the caller's pageable memory: each copy is ordered on the
    // stream that produced `src` (never the null stream) and waited for.
    auto place = [&](const life::GatherPiece &p, const uint8_t *src, hipStream_t st) -> int {
        const int64_t rb = p.row_bytes;
        uint8_t *dst = out + p.dst;
        if (!p.shared_first && !p.shared_last) {
            HIPCHK(hipMemcpy2DAsync(dst, (size_t)frb, src, (size_t)rb, (size_t)rb, (size_t)p.rows,
                                    hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            return LIFE_OK;
        }
        tmp.resize((size_t)p.bytes);
        HIPCHK(hipMemcpyAsync(tmp.data(), src, tmp.size(), hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        const bool f = p.shared_first, l = p.shared_last;
        for (int64_t y = 0; y < p.rows; y++) {
            uint8_t *o = dst + y * frb;
            const uint8_t *t = tmp.data() + y * rb;
            const int64_t a = f ? 1 : 0, b = l ? rb - 1 : rb;
            if (b > a) memcpy(o + a, t + a, (size_t)(b - a));
            if (f) o[0] |= t[0];
            if (l && (rb > 1 || !f)) o[rb - 1] |= t[rb - 1];
        }
        return LIFE_OK;
    };
    if (fmt == Frame::BITS && have_root) {
        // zero the shared bytes of every block boundary (all ranks' blocks)
        for (const life::GatherPiece &p : plan)
            if (p.shared_first)
                for (int64_t y = 0; y < p.rows; y++) out[p.dst + y * frb] = 0;
    }
    if (!d->rank_mode) {
        for (Shard &s : d->shards) {
            HIPCHK(hipSetDevice(s.device));
            uint8_t *stage;
            CHK(export_block(s, &stage));
        }
        for (Shard &s : d->shards) {  // every export is queued before the first copy waits
            HIPCHK(hipSetDevice(s.device));
            HIPCHK(hipStreamSynchronize(s.stream));
            CHK(place(piece_of(s.rank), s.stage, s.stream));
        }
        return LIFE_OK;
    }
    Shard &s = d->shards[0];
    HIPCHK(hipSetDevice(s.device));
    uint8_t *stage;
    CHK(export_block(s, &stage));
    if (s.rank != root) {
        if (!s.comm) {
            set_err("gather: rank %d has no communicator", s.rank);
            return LIFE_ESTATE;
        }
        NCCLCHK(ncclSend(stage, (size_t)piece_of(s.rank).bytes, ncclUint8, root, s.comm, s.stream));
        return bounded_sync(s, "gather: send to the root", root);
    }
    HIPCHK(hipStreamSynchronize(s.stream));
    // The root's own block sits in the front of the staging buffer; two
    // receive slots follow.  Block k+1 arrives over RCCL (non-blocking
    // stream) while the host copies block k out of the other slot (on the
    // idle second compute stream, into the caller's pageable memory), so the
    // fan-in of world-1 blocks is not serialised behind the D2H copies.
    CHK(place(plan[0], stage, s.stream));  // copied out first: the buffer may grow below
    CHK(stage_buffer(s, 2 * (size_t)slot, &stage));
    if (d->world > 1 && !s.comm) {
        set_err("gather: the root has no communicator");
        return LIFE_ESTATE;
    }
    for (size_t k = 1; k < plan.size(); k++) {
        const life::GatherPiece &p = plan[k];
        if (k == 1) NCCLCHK(ncclRecv(stage, (size_t)p.bytes, ncclUint8, p.rank, s.comm, s.stream));
        CHK(bounded_sync(s, "gather: receive at the root", p.rank));  // block k is in slot p.slot
        if (k + 1 < plan.size()) {
            const life::GatherPiece &q = plan[k + 1];
            NCCLCHK(ncclRecv(stage + (size_t)q.slot * (size_t)slot, (size_t)q.bytes, ncclUint8, q.rank, s.comm,
                             s.stream));
        }
        CHK(place(p, stage + (size_t)p.slot * (size_t)slot, s.stream2));
    }
    HIPCHK(hipStreamSynchronize(s.stream));
    return LIFE_OK;
}
}  // namespace

extern "C" {

int life_dev_gather(life_dev *d, uint8_t *grid) {
    if (!d) return LIFE_EINVAL;
    return gather_impl(d, grid, Frame::DENSE);
}

int life_dev_gather_vtk(life_dev *d, char *body) {
    if (!d) return LIFE_EINVAL;
    return gather_impl(d, reinterpret_cast<uint8_t *>(body), Frame::VTK);
}

int life_dev_gather_bits(life_dev *d, uint8_t *packed) {
    if (!d) return LIFE_EINVAL;
    return gather_impl(d, packed, Frame::BITS);
}

static int census(life_dev *d, unsigned long long out[2]) {
    out[0] = out[1] = 0;
    for (Shard &s : d->shards) {
        HIPCHK(hipSetDevice(s.device));
        HIPCHK(hipMemsetAsync(s.d_count, 0, 2 * sizeof(unsigned long long), s.stream));
        HIPCHK(life::launch_census(s.lay, d->nx, s.buf[s.cur], s.d_count, s.stream));
        if (d->rank_mode && s.comm)
            NCCLCHK(ncclAllReduce(s.d_count, s.d_count, 2, ncclUint64, ncclSum, s.comm, s.stream));
        HIPCHK(hipMemcpyAsync(s.h_count, s.d_count, 2 * sizeof *s.h_count, hipMemcpyDeviceToHost, s.stream));
        CHK(bounded_sync(s, "census all-reduce", -1));  // pinned destination
        out[0] += s.h_count[0];
        out[1] += s.h_count[1];
    }
    return LIFE_OK;
}

int64_t life_dev_live_count(life_dev *d) {
    if (!d) return LIFE_EINVAL;
    CHK(life_dev_sync(d));
    unsigned long long c[2];
    CHK(census(d, c));
    return (int64_t)c[0];
}

int life_dev_checksum(life_dev *d, uint64_t *sum) {
    if (!d || !sum) return LIFE_EINVAL;
    CHK(life_dev_sync(d));
    unsigned long long c[2];
    CHK(census(d, c));
    *sum = (uint64_t)c[1];
    return LIFE_OK;
}

int life_dev_layout(life_dev *d, int local_shard, life_layout *out) {
    if (!d || !out || local_shard < 0 || local_shard >= (int)d->shards.size()) return LIFE_EINVAL;
    *out = d->shards[local_shard].lay;
    return LIFE_OK;
}

int life_dev_world(life_dev *d, int *world, int *dims0, int *dims1, int *nlocal, int *transport) {
    if (!d) return LIFE_EINVAL;
    if (world) *world = d->world;
    if (dims0) *dims0 = d->dims[0];
    if (dims1) *dims1 = d->dims[1];
    if (nlocal) *nlocal = (int)d->shards.size();
    if (transport) *transport = d->transport;
    return LIFE_OK;
}

int life_dev_shard_info(life_dev *d, int local_shard, int *device, char pci_bus_id[64], int *rccl_nranks) {
    if (!d || local_shard < 0 || local_shard >= (int)d->shards.size()) return LIFE_EINVAL;
    const Shard &s = d->shards[local_shard];
    if (device) *device = s.device;
    if (pci_bus_id) HIPCHK(hipDeviceGetPCIBusId(pci_bus_id, 64, s.device));
    if (rccl_nranks) {
        int n = 0;
        if (s.comm) NCCLCHK(ncclCommCount(s.comm, &n));
        *rccl_nranks = n;
    }
    return LIFE_OK;
}

int life_dev_configure(life_dev *d, int option, int value) {
    if (!d) return LIFE_EINVAL;
    CHK(life_dev_sync(d));
    switch (option) {
    case LIFE_OPT_SMALL_GRID:
        if (value < 0 || value > 4) return LIFE_EINVAL;
        d->small_mode = value;
        return LIFE_OK;
    case LIFE_OPT_SMALL_WINDOW: {
        const int R = value >> 8, K = value & 255;  // R = 0 (value 0): automatic
        if (value != 0 && (K < 1 || R < 1 || R > 8 || R == 7)) return LIFE_EINVAL;
        // a window the shard cannot hold (own = strips*R - 2K rows < 1, or
        // >= h) would silently fall back to the unwindowed kernel: refuse it
        if (value != 0 && life::reg_win_plan(d->shards[0].lay, R, K).blocks == 0) {
            set_err("small-grid window R=%d K=%d does not fit this grid", R, K);
            return LIFE_EINVAL;
        }
        d->win_rows = R;
        d->win_halo = K;
        return LIFE_OK;
    }
    case LIFE_OPT_OVERLAP: d->overlap = value != 0; return LIFE_OK;
    case LIFE_OPT_BLOCK_GENS:
        if (value < 0 || value > 32) return LIFE_EINVAL;
        d->block_gens = value > 0 ? value : default_block_gens(d->kernel);
        tail_prewarm(d);
        return LIFE_OK;
    case LIFE_OPT_FLOW:
        if (value < 0 || value > 3) return LIFE_EINVAL;
        d->flow = value;
        return LIFE_OK;
    case LIFE_OPT_DEEP_HALO:
        if (value < 0 || value > 1) return LIFE_EINVAL;
        // Aprons valid only to the remaining depth K - since are refilled by
        // the next pass that needs more (generation_block).  But the option
        // decides which passes exchange, so in rank mode every rank must hold
        // the same value or their ncclSend / ncclRecv groups stop pairing up
        // (ADVICE r5): the call is collective there and checks agreement.
        if (d->rank_mode && d->world > 1) CHK(agree_all_ranks(d, value, "LIFE_OPT_DEEP_HALO"));
        d->deep = value != 0;
        return LIFE_OK;
    case LIFE_OPT_FLOW_CHUNK:
        if (value < 0) return LIFE_EINVAL;
        d->flow_chunk = value;
        return LIFE_OK;
    case LIFE_OPT_LOOPBACK: {
        // 1: both axes, 2: x only, 3: y only (the axes a real partition of
        // N GPUs cuts: N = 2's {2, 1} cuts x only)
        if (value < 0 || value > 3) return LIFE_EINVAL;
        if (d->world != 1 || d->shards.size() != 1) {
            set_err("loopback needs a single-shard world (world %d, %zu local shards)", d->world, d->shards.size());
            return LIFE_EINVAL;
        }
        Shard &s = d->shards[0];
        // the aprons a partitioned axis needs: at least K rows / one x-apron
        // of columns to send
        if (value && (s.lay.h < s.lay.yapron || s.lay.w < s.lay.xapron)) {
            set_err("loopback: %lld x %lld cells < the %lld-column / %lld-row halo", (long long)s.lay.w,
                    (long long)s.lay.h, (long long)s.lay.xapron, (long long)s.lay.yapron);
            return LIFE_EINVAL;
        }
        if (value && d->transport == LIFE_XPORT_RCCL && !s.comm) {
            set_err("loopback over RCCL needs a communicator (life_dev_create_rank with a unique id, or "
                    "life_dev_create_ex with LIFE_XPORT_RCCL)");
            return LIFE_EINVAL;
        }
        // the current state's aprons are refreshed on the next step's first
        // exchange only: fill them now from the shard itself
        d->loop = value == 0 ? 0 : value == 1 ? 3 : value == 2 ? 1 : 2;
        life_halo_op ops[16];
        const int n = life::halo_plan(d->nx, d->ny, d->dims[0], d->dims[1], s.rank, d->kernel, d->loop, ops, 16);
        if (n < 0) return LIFE_EINVAL;
        s.plan.assign(ops, ops + n);
        s.corners =
            std::any_of(s.plan.begin(), s.plan.end(), [](const life_halo_op &o) { return o.what == LIFE_HALO_CORNER; });
        CHK(exchange(d, 0, false));
        tail_prewarm(d);
        return life_dev_sync(d);
    }
    default: return LIFE_EINVAL;
    }
}

int life_dev_set_timing(life_dev *d, int on) {
    if (!d) return LIFE_EINVAL;
    CHK(harvest_timers(d));
    CHK(harvest_phases(d));
    if (on)  // a few event pairs up front: no hipEventCreate inside a timed step call
        for (Shard &s : d->shards) {
            HIPCHK(hipSetDevice(s.device));
            int rc = LIFE_OK;
            while (s.timers.size() < 8 && timer_slot(s, &rc)) {
            }
            if (rc != LIFE_OK) return rc;
            s.timers_used = 0;
        }
    d->ph_ring = d->ph_int = d->ph_halo = d->ph_block = 0.0;
    d->ph_blocks = 0;
    d->timing = on != 0;
    d->phase_events = on == 1;
    d->launch_events = on != 3;
    d->acc_ms = 0.0;
    d->acc_launches = 0;
    d->acc_bytes = 0.0;
    d->acc_updates = 0.0;
    d->acc_valu = 0.0;
    return LIFE_OK;
}

int life_dev_phase_stats(life_dev *d, double *ring_ms, double *interior_ms, double *halo_ms, double *block_ms,
                         int64_t *blocks) {
    if (!d) return LIFE_EINVAL;
    CHK(harvest_phases(d));
    const double n = d->ph_blocks ? (double)d->ph_blocks : 1.0;
    if (ring_ms) *ring_ms = d->ph_ring / n;
    if (interior_ms) *interior_ms = d->ph_int / n;
    if (halo_ms) *halo_ms = d->ph_halo / n;
    if (block_ms) *block_ms = d->ph_block / n;
    if (blocks) *blocks = d->ph_blocks;
    return LIFE_OK;
}

int life_dev_call_stats(life_dev *d, double *host_enqueue_ms, double *pass_enqueue_max_ms, int64_t *passes,
                        double *device_span_ms) {
    if (!d) return LIFE_EINVAL;
    double span = 0.0;
    if (d->call_spans)
        for (Shard &s : d->shards) {
            HIPCHK(hipSetDevice(s.device));
            HIPCHK(hipEventSynchronize(s.span_b));
            float ms = 0.f;
            HIPCHK(hipEventElapsedTime(&ms, s.span_a, s.span_b));
            span = std::max(span, (double)ms);
        }
    if (host_enqueue_ms) *host_enqueue_ms = d->call_host_ms;
    if (pass_enqueue_max_ms) *pass_enqueue_max_ms = d->call_pass_max_ms;
    if (passes) *passes = d->call_passes;
    if (device_span_ms) *device_span_ms = span;
    return LIFE_OK;
}

int life_dev_kernel_work(life_dev *d, double *cell_updates_per_launch, double *valu_ops_per_launch) {
    if (!d) return LIFE_EINVAL;
    CHK(harvest_timers(d));
    const double n = d->acc_launches ? (double)d->acc_launches : 1.0;
    if (cell_updates_per_launch) *cell_updates_per_launch = d->acc_updates / n;
    if (valu_ops_per_launch) *valu_ops_per_launch = d->acc_valu / n;
    return LIFE_OK;
}

int life_dev_kernel_stats(life_dev *d, double *avg_ms, int64_t *launches, double *bytes_per_launch) {
    if (!d) return LIFE_EINVAL;
    CHK(harvest_timers(d));
    const double n = d->acc_launches ? (double)d->acc_launches : 1.0;
    if (avg_ms) *avg_ms = d->acc_ms / n;
    if (launches) *launches = d->acc_launches;
    if (bytes_per_launch) *bytes_per_launch = d->acc_bytes / n;
    return LIFE_OK;
}

int life_tune(int kernel, int rows, int depth) {
    if ((rows && rows != 16 && rows != 32 && rows != 64) ||
        (depth && depth != 2 && depth != 4 && depth != 8 && depth != 18) ||
        kernel < -1 || kernel > LIFE_KERNEL_BIT)
        return LIFE_EINVAL;
    life::set_step_tuning(kernel, rows, depth);
    return LIFE_OK;
}

int life_tune_temporal(int kernel, int rows) {
    const bool bit_ok = rows == 16 || rows == 24;
    const bool byte_ok = rows == 32 || rows == 48;
    if (kernel < -1 || kernel > LIFE_KERNEL_BIT) return LIFE_EINVAL;
    if (rows && ((kernel == LIFE_KERNEL_BIT && !bit_ok) || (kernel == LIFE_KERNEL_BYTE && !byte_ok) ||
                 (kernel == -1 && !bit_ok && !byte_ok)))
        return LIFE_EINVAL;
    life::set_temporal_rows(kernel, rows);
    return LIFE_OK;
}

int life_measure_copy(int device, int64_t bytes, int reps, double *gbps) {
    if (!gbps || bytes < 16 || bytes % 16 || reps < 1) return LIFE_EINVAL;
    HIPCHK(hipSetDevice(device));
    void *a = nullptr, *b = nullptr;
    hipStream_t st = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int rc = LIFE_OK;
    float best = 0.f;
    auto run = [&]() -> int {
        HIPCHK(hipMalloc(&a, (size_t)bytes));
        HIPCHK(hipMalloc(&b, (size_t)bytes));
        HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        HIPCHK(hipEventCreate(&e0));
        HIPCHK(hipEventCreate(&e1));
        HIPCHK(hipMemsetAsync(a, 1, (size_t)bytes, st));
        HIPCHK(life::launch_copy(a, b, bytes, st));  // warm-up (page mapping, clocks)
        for (int r = 0; r < reps; r++) {
            HIPCHK(hipEventRecord(e0, st));
            HIPCHK(life::launch_copy(a, b, bytes, st));
            HIPCHK(hipEventRecord(e1, st));
            HIPCHK(hipEventSynchronize(e1));
            float ms = 0.f;
            HIPCHK(hipEventElapsedTime(&ms, e0, e1));
            if (best == 0.f || ms < best) best = ms;
        }
        return LIFE_OK;
    };
    rc = run();
    if (st) (void)hipStreamSynchronize(st);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (st) (void)hipStreamDestroy(st);
    if (a) (void)hipFree(a);
    if (b) (void)hipFree(b);
    if (rc == LIFE_OK) *gbps = 2.0 * (double)bytes / (best * 1e-3) / 1e9;
    return rc;
}

void life_dev_destroy(life_dev *d) {
    if (!d) return;
    for (Shard &s : d->shards) {
        (void)hipSetDevice(s.device);
        if (s.stream) (void)hipStreamSynchronize(s.stream);
        if (s.stream2) (void)hipStreamSynchronize(s.stream2);
        if (s.comm_stream) (void)hipStreamSynchronize(s.comm_stream);
    }
    for (Shard &s : d->shards) shard_free(s);
    delete d;
}

}  // extern "C"
