/*
 * life_mi355x.h -- C ABI of the MI355X-native Game-of-Life hot path.
 *
 * Drop-in boundary for the reference kekoveca/MPI-and-Open-MP.  The reference
 * has no library or FFI: its "operator interface" is the set of free functions
 * on `life_t` in 6-cartesian/life_cart.c:39-49, called only from main()
 * (life_cart.c:51-85).  Each entry point below names the reference function
 * it replaces.  Plain pointers and sizes only; no torch or HIP types.
 *
 * Grid convention (same as the reference's ind(), life_cart.c:11): cells are
 * 0/1, row-major, x fastest: cell (x, y) at grid[y*nx + x].  Indices are
 * 64-bit (the reference overflows int beyond ~46340^2, life_cart.c:101).
 *
 * Errors: every int-returning call returns LIFE_OK (0) or a negative
 * LIFE_E* code (the reference asserts or aborts via MPI_ERRORS_ARE_FATAL);
 * life_strerror() names it.  Not thread-safe: one host thread owns a handle.
 */
#ifndef LIFE_MI355X_H
#define LIFE_MI355X_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LIFE_OK 0
#define LIFE_EINVAL (-1)   /* bad argument (sizes, dims, empty block, ...) */
#define LIFE_EHIP (-2)     /* HIP runtime error (message: life_last_error()) */
#define LIFE_ERCCL (-3)    /* RCCL error */
#define LIFE_ENOMEM (-4)   /* host or device allocation failed */
#define LIFE_ESTATE (-5)   /* call not valid in this state */
#define LIFE_EIO (-6)      /* file I/O or parse error (driver helpers) */

/* Cell encoding / kernel family. */
#define LIFE_KERNEL_BYTE 0 /* 1 byte per cell, SWAR byte stencil */
#define LIFE_KERNEL_BIT 1  /* 1 bit per cell (32 cells/word), bit-sliced adder */

/* Halo transport between shards. */
#define LIFE_XPORT_AUTO 0  /* RCCL across processes/devices, LOCAL otherwise */
#define LIFE_XPORT_RCCL 1  /* ncclSend/ncclRecv (xGMI) */
#define LIFE_XPORT_LOCAL 2 /* device-to-device copies inside one process */

typedef struct life_dev life_dev; /* opaque: device memory, streams, RCCL comms */

/* ---------------------------------------------------------------- host only */

/* decomposition(): block k of n cells over p parts, the last block takes the
 * remainder.  Replaces life_cart.c:217-223 (and 5-gather/life_mpi.c:170-175). */
void life_decomposition(int64_t n, int p, int k, int64_t *start, int64_t *stop);

/* MPI_Dims_create(n, 2, {0,0}) as called in life_init (life_cart.c:117-118):
 * dims[0] >= dims[1], as balanced as possible. 2->{2,1}, 4->{2,2}, 8->{4,2}. */
void life_dims_create(int n, int dims[2]);

/* Partition shape for n shards of an nx x ny grid (the 1-D
 * row strips of 3-life/4-life/5-gather vs the 2-D blocks of 6-cartesian).
 * CART: life_dims_create (life_cart.c:117-118).  ROWS: {1, n}, horizontal
 * strips (5-gather/life_mpi.c:96-99 cuts y the same way): every halo message is
 * a run of whole padded rows, sent straight from the buffer with no pack
 * kernel.  COLS: {n, 1}.  AUTO: ROWS when every strip is at least
 * LIFE_AUTO_MIN_STRIP_ROWS tall, else CART -- measured
 * on MI355X with the LOCAL transport at 65536^2 per shard (DESIGN.md §6,
 * profiles/r01/partition_sweep.jsonl), row strips cost the owning GPU 0-6 %
 * less per generation than 2-D blocks with either encoding.  Returns
 * LIFE_EINVAL for n < 1, an unknown policy or a shape with empty blocks. */
#define LIFE_PARTITION_CART 0
#define LIFE_PARTITION_ROWS 1
#define LIFE_PARTITION_COLS 2
#define LIFE_PARTITION_AUTO 3
#define LIFE_AUTO_MIN_STRIP_ROWS 1024
int life_dims_choose(int64_t nx, int64_t ny, int n, int policy, int dims[2]);

/* One halo-exchange operation of a shard (replaces exchange_columns /
 * exchange_rows / exchange_corners, life_cart.c:225-279, and the 1-D ring
 * exchange of 5-gather/life_mpi.c:181-191).  Coordinates are the shard's
 * LOCAL frame: owned cells x in [0,w), y in [0,h); padded row of owned row y
 * is y + yapron; the apron is x in [-xapron, 0) u [w, w+xapron) and rows
 * y in [-yapron, 0) u [h, h+yapron) (see life_layout). */
#define LIFE_HALO_SEND 0
#define LIFE_HALO_RECV 1
#define LIFE_HALO_FILL 2   /* axis not partitioned (dims[d] == 1): wrapped inside the shard */
#define LIFE_HALO_COLUMN 0 /* cells x in [index, index+width) of padded rows [first, first+count) */
#define LIFE_HALO_ROW 1    /* padded rows [index, index+width), cells x in [first, first+count) */
#define LIFE_HALO_CORNER 2 /* as a column op: cells x in [index, index+width) of padded rows [first, first+count) */
typedef struct {
    int32_t phase; /* 0: x (columns) first, then 1: y (rows incl. corners); both axes
                      exchanged with temporal aprons: all in phase 0, corners explicit */
    int32_t kind;  /* LIFE_HALO_SEND / RECV / FILL */
    int32_t peer;  /* global shard rank, -1 for FILL */
    int32_t what;  /* LIFE_HALO_COLUMN / LIFE_HALO_ROW / LIFE_HALO_CORNER */
    int64_t index; /* first column x, or first padded row */
    int64_t first; /* first padded row (column op) or first cell x (row op) */
    int64_t count; /* rows (column op) or cells (row op) */
    int64_t width; /* columns (column op) or rows (row op) */
} life_halo_op;

/* Builds the per-exchange halo plan of shard `rank` of a dims[0] x dims[1]
 * periodic Cartesian partition (rank = c0*dims[1] + c1, dim 0 splits x, as
 * MPI_Cart_create(reorder=0) at life_cart.c:119-121) for cell encoding
 * `kernel` (apron widths from life_layout_query).  Writes up to max_ops ops
 * in execution order and returns their number (or LIFE_EINVAL).  Sends to
 * and receives from one peer are matched in issue order. */
int life_halo_plan(int64_t nx, int64_t ny, int dims0, int dims1, int rank, int kernel,
                   life_halo_op *ops, int max_ops);

/* Padded layout of a shard as allocated on the device: rows = h + 2*yapron
 * padded rows of `pitch` bytes; owned cell (x, y) lives in padded row
 * y + yapron at cell offset x from byte `xoff`.  Byte encoding: byte x.  Bit
 * encoding: 64-cell pairs of little-endian dwords, bit-interleaved -- cell x
 * is bit ((x & 63) >> 1) of dword 2*(x >> 6) + (x & 1) (floor division,
 * counted from xoff): the even cells of a pair in its first dword, the odd
 * cells in its second (the stencil's horizontal neighbours then need one
 * funnel shift per dword).  `generations_per_exchange` is how
 * many generations one halo exchange feeds: 1 for the one-cell apron; for
 * the temporally blocked stencil (x-apron of one lane column: 64 cells for
 * bits, 32 for bytes; K-row y-apron; blocks at least that wide) K =
 * LIFE_TEMPORAL_DEPTH (bit) or LIFE_TEMPORAL_DEPTH_BYTE (byte), or
 * 8/12/16/24/32 from the environment variables of the same names. */
#define LIFE_TEMPORAL_DEPTH 32
#define LIFE_TEMPORAL_DEPTH_BYTE 32
typedef struct {
    int64_t w, h;      /* owned block */
    int64_t x0, y0;    /* global origin of the block */
    int64_t pitch;     /* bytes per padded row */
    int64_t xoff;      /* byte offset of owned cell x = 0 in a padded row */
    int64_t rows;      /* h + 2*yapron */
    int64_t units;     /* 16-byte lanes per row the one-generation stencil walks */
    int64_t xapron;    /* apron width in cells (x) */
    int64_t yapron;    /* apron depth in rows (y) */
    int32_t kernel;    /* LIFE_KERNEL_* */
    int32_t coords[2]; /* Cartesian coordinates of the shard */
    int32_t generations_per_exchange;
    int32_t reserved;
} life_layout;

int life_layout_query(int64_t nx, int64_t ny, int dims0, int dims1, int rank, int kernel,
                      life_layout *out);

const char *life_strerror(int err);
const char *life_dev_strerror(int err); /* the same (SURVEY 8(b)'s name for it) */
const char *life_last_error(void); /* detail of the last LIFE_EHIP/ERCCL on this thread */

/* ---------------------------------------------------------------- device */

/* life_init (life_cart.c:92-144) minus the file parsing: sizes the global
 * nx x ny periodic grid, splits it over `nshards` shards driven by THIS
 * process (dims = life_dims_create(nshards)), one per visible device
 * (shard i on device i % device_count), and allocates double-buffered padded
 * blocks.  Transport AUTO: RCCL when every shard has its own device, LOCAL
 * device copies otherwise (e.g. several logical shards on one GPU). */
int life_dev_create(int64_t nx, int64_t ny, int nshards, int kernel, life_dev **out);

/* Same with every knob: dims (0,0 = dims_create), transport.  LIFE_XPORT_RCCL
 * needs one device per shard and builds one communicator rank per shard with
 * ncclCommInitAll -- a single shard included (a one-device communicator, so
 * LIFE_OPT_LOOPBACK exercises this single-process RCCL path on one GPU). */
int life_dev_create_ex(int64_t nx, int64_t ny, int nshards, int dims0, int dims1, int kernel,
                       int transport, life_dev **out);

/* One-process-per-GPU mode (torchrun / mpirun style): this process owns the
 * single shard `rank` of `world` on `device`; `unique_id` (128 bytes) comes
 * from life_get_unique_id() on rank 0, broadcast by the caller (required when
 * world > 1; with world == 1 it is optional and, if given, still builds a
 * one-rank RCCL communicator, used by the census all-reduce). */
int life_get_unique_id(uint8_t unique_id[128]);
int life_dev_create_rank(int64_t nx, int64_t ny, int kernel, int rank, int world, int dims0,
                         int dims1, const uint8_t unique_id[128], int device, life_dev **out);

/* The loaded cells of life_init (life_cart.c:104-109): `grid` is the full
 * nx*ny host grid (nonzero = alive); each local shard takes its block.  Then
 * fills the halos.  In rank mode every rank passes the full grid. */
int life_dev_upload(life_dev *d, const uint8_t *grid);

/* Device-side synthetic init (no host grid): cell(x,y) =
 * (splitmix64(splitmix64(seed) ^ (y*nx+x)) >> 32) < thr32,
 * splitmix64 the standard finaliser.  thr32 = density * 2^32. */
int life_dev_fill_random(life_dev *d, uint64_t seed, uint32_t thr32);

/* `generations` x (life_exchange + life_step): life_cart.c:73-74
 * (replaces life_exchange :275-279 and life_step :189-215). Asynchronous.
 * With a temporally blocked layout, up to generations_per_exchange
 * generations run per launch and the halo is exchanged once per launch. */
int life_dev_step(life_dev *d, int64_t generations);

/* life_collect (life_cart.c:281-305; MPI_Gather in 5-gather/life_mpi.c:177-179):
 * device-side gather of every block to the root shard (global rank
 * world-1, as the reference) and one copy into `grid` (nx*ny bytes, 0/1).
 * In rank mode only the root writes `grid` (others may pass NULL). Blocking. */
int life_dev_gather(life_dev *d, uint8_t *grid);

/* The same collect, formatted on the device as the cell-data body of
 * life_save_vtk (life_cart.c:181-185): "%d\n" per cell, y outer, x inner --
 * 2*nx*ny bytes of '0'/'1' and '\n' written to `body` (root only in rank
 * mode).  The caller writes the 10 header lines in front (driver/life.c). */
int life_dev_gather_vtk(life_dev *d, char *body);

/* The same collect as packed rows: ny rows of ceil(nx/8) bytes, cell x at
 * bit (x & 7) of byte (x >> 3) -- the body of the driver's LIFEBITS
 * checkpoint frame (driver/life.c save_bits), 1/16 of the VTK text and 1/8
 * of the dense grid over PCIe (root only in rank mode).  Blocking. */
int life_dev_gather_bits(life_dev *d, uint8_t *packed);

/* Live cells over the whole grid (all ranks). Blocking. */
int64_t life_dev_live_count(life_dev *d);

/* Position-weighted checksum of the whole grid (all ranks), independent of
 * the encoding and the partition: sum over live cells (x, y) of
 * mix64(y*nx + x + 1) mod 2^64, mix64(v) = t ^ (t >> 29), t = v *
 * 0x9E3779B97F4A7C15 mod 2^64.  Lets N-shard and 1-shard runs of one grid be
 * compared at sizes no host gather reaches.  Blocking. */
int life_dev_checksum(life_dev *d, uint64_t *sum);

int life_dev_sync(life_dev *d);
/* life_dev_sync, then (rank mode) an all-reduce every rank joins: the
 * synchronisation the reference gets from its blocking MPI calls; the driver
 * brackets its timer with it.  Blocking. */
int life_dev_barrier(life_dev *d);
/* Visible HIP devices (hipGetDeviceCount), or a negative LIFE_E* code. */
int life_device_count(void);
int life_dev_layout(life_dev *d, int local_shard, life_layout *out);
int life_dev_world(life_dev *d, int *world, int *dims0, int *dims1, int *nlocal, int *transport);
/* Where local shard `local_shard` runs (measurement support, so a multi-GPU
 * result can prove what it ran on): its HIP device ordinal, that device's PCI
 * bus id (hipDeviceGetPCIBusId; distinct per physical GPU, up to 63 chars +
 * NUL), and the rank count of its RCCL communicator (ncclCommCount; 0 when
 * the shard has none, e.g. LOCAL transport).  Any out pointer may be NULL. */
int life_dev_shard_info(life_dev *d, int local_shard, int *device, char pci_bus_id[64], int *rccl_nranks);

/* Kernel timing for roofline reporting: when on, every stencil launch is
 * bracketed by HIP events on the stream it runs on.  stats returns the mean
 * device time of one stencil launch (ms), the number of launches, and the
 * algorithmic HBM bytes one launch moves (1 B read + 1 B written per cell for
 * BYTE, 2 bits for BIT, over the cells that launch updates).  on = 1 also
 * records the overlapped schedule's phase events (life_dev_phase_stats: ring,
 * interior, halo, block); on = 2 times the launches only (their events are
 * stamped by the dispatches themselves), leaving no event packets between the
 * ring, halo and interior work of a partitioned step; on = 3 records only
 * the call's span (life_dev_call_stats) on a multi-stream call -- per-launch
 * events there put ~10 us between back-to-back launches (profiles/r05/c, d) --
 * while a single-stream call keeps its one event pair around all launches. */
int life_dev_set_timing(life_dev *d, int on);

/* Execution-path switches (defaults 1): LIFE_OPT_SMALL_GRID lets a
 * single-shard grid that fits one CU run all generations of a step call in
 * one resident-workgroup launch (1: the grid in VGPRs when its shape allows,
 * else in LDS; 2: LDS only; 0: off); LIFE_OPT_OVERLAP overlaps the halo
 * exchange with the interior kernel on partitioned grids.  Results are
 * identical either way (tests switch them to reach every kernel). */
#define LIFE_OPT_SMALL_GRID 1
#define LIFE_OPT_OVERLAP 2
/* (option 3, the sweep stencil, was removed: slower than the tiles in every
 * measured case, profiles/r02/sweep_ab.txt) */
/* LIFE_OPT_BLOCK_GENS: the tiled stencil's generations per launch at most
 * (1..32, capped by generations_per_exchange; 0: the default, 12 for bits
 * and 32 for bytes, or LIFE_BLOCK_GENS from the environment).  A step call of
 * g generations runs ceil(g / max) launches of nearly equal size; a bit
 * launch of m generations holds m ghost rows above and below each tile
 * (tile height 8R - 2m), a byte launch K. */
#define LIFE_OPT_BLOCK_GENS 5
/* LIFE_OPT_SMALL_GRID value 3: the register-resident small-grid kernel
 * WINDOWED over several CUs whenever the shape allows
 * (life_kernels.hip rsmall_kernel<.., WIN>): ceil(h / own) workgroups, each
 * holding its own rows plus K halo rows above and below for K generations
 * per launch; value 1 (default) windows only grids whose one-workgroup strips
 * would be 4 or more rows tall (p46gun_big).  LIFE_OPT_SMALL_WINDOW sets the
 * strip height R and K as value = R * 256 + K (R in 1..6 or 8, K <= 255;
 * default and value 0: automatic, R = 1, K = min(30, (strips - 4) / 2)).  Shapes it does
 * not fit run as value 1 without the window.  Value 4: as 1, never
 * windowed (the one-workgroup kernel; tests). */
#define LIFE_OPT_SMALL_WINDOW 4
/* LIFE_OPT_LOOPBACK (default 0; single-shard devices only): 1 runs the one
 * shard as a periodic Cartesian partition of itself -- both axes' halos are
 * exchanged through the transport with the shard as its own left and right
 * neighbour (two sends and two receives to one peer per phase, as at
 * dims = 2), the boundary ring and interior overlapped on their streams,
 * instead of the stencil wrapping the axes.  With a rank-mode device
 * (life_dev_create_rank, world 1, a unique id) the messages are RCCL
 * ncclSend/ncclRecv: how one GPU executes the multi-GPU data path.  Results
 * are identical either way.  The grid must be at least one halo deep
 * (generations_per_exchange rows).  Value 2 loops the x axis only, 3 the y
 * axis only (the other axis wraps in the stencil): the axes a real partition
 * cuts -- N = 2's {2, 1} blocks exchange columns only. */
#define LIFE_OPT_LOOPBACK 6
/* LIFE_OPT_FLOW (default 3, automatic, or LIFE_FLOW from the environment): a step call
 * on a single shard whose axes both wrap inside it (bit encoding, width a
 * multiple of 64) runs its whole passes of m generations (m = the block
 * size, LIFE_OPT_BLOCK_GENS; at least 4 passes) as ONE persistent launch: workgroups pull
 * (pass, tile) items in order and a tile starts when the tiles its window
 * reads have finished the previous pass, so no pass boundary drains the chip;
 * the remainder runs as an ordinary launch.  1: write-through hand-off
 * stores; 2: plain stores + a release fence per tile; 0: off; 3: form 1
 * when a pass is under 5 rounds of resident workgroups (its launch tail
 * would idle the chip: 32768^2), else off (65536^2, where the per-launch
 * tiles measured 3 % faster).  The byte encoding always runs
 * per-launch tiles.  Same results. */
#define LIFE_OPT_FLOW 7
/* LIFE_OPT_FLOW_CHUNK (default 0 = automatic): the dataflow launch's queue
 * head is a 32-bit counter, so a step call's passes are split over several
 * persistent launches, each with passes x tiles + resident workgroups below
 * 2^31 pulls; a positive value caps the passes per launch further (tests). */
#define LIFE_OPT_FLOW_CHUNK 8
/* LIFE_OPT_DEEP_HALO (default 1; LIFE_DEEP_HALO=0 at load time turns it
 * off): partitioned bit shards with K-deep aprons exchange their halo only
 * when the next pass would outrun it -- the passes in between also advance
 * the apron cells they will read (rows [-e, 0) and [h, h + e), the apron
 * pairs), so one exchange feeds up to K generations instead of one pass of
 * at most LIFE_OPT_BLOCK_GENS.  0: one exchange per pass.  Same results.
 * The value decides which passes exchange, so every rank must hold the same
 * one: in rank mode (world > 1) this option is COLLECTIVE -- every rank calls
 * it with the same value at the same step boundary; it checks agreement
 * with an RCCL all-reduce and fails with LIFE_EINVAL (all ranks keep the old
 * value) when ranks differ, or with LIFE_ERCCL after LIFE_COMM_TIMEOUT_S when
 * a rank never calls it.  Part-used aprons are refilled by the next step's
 * first pass that needs them.  Every life_dev_configure call waits for the
 * device (life_dev_sync). */
#define LIFE_OPT_DEEP_HALO 9
/* Option 10 (LIFE_OPT_SKEW, time-skewed ghost-free tiles) was retired in
 * round 5: 8 % slower per launch on MI355X; it now fails
 * with LIFE_EINVAL like any unknown option. */
int life_dev_configure(life_dev *d, int option, int value);
/* The kernel family that ran the bulk of the last life_dev_step call:
 * LIFE_PATH_ONEGEN (one generation per launch), _TILES (temporally blocked
 * tiles, one launch per pass), _FLOW (the dataflow tiles, LIFE_OPT_FLOW),
 * _SMALL (a small-grid resident kernel); _NONE before the first step. */
#define LIFE_PATH_NONE 0
#define LIFE_PATH_ONEGEN 1
#define LIFE_PATH_TILES 2
#define LIFE_PATH_FLOW 3
#define LIFE_PATH_SMALL 5
int life_dev_last_path(life_dev *d);
int life_dev_kernel_stats(life_dev *d, double *avg_ms, int64_t *launches, double *bytes_per_launch);
/* The same timed launches: mean cell-updates per launch (cells x generations
 * it advanced) and mean VALU lane-operations per launch (op-count model of
 * the temporal bit stencil; 0 for the HBM-bound one-generation kernels).
 * bytes_per_launch above is the COMPULSORY HBM traffic: one read + one write
 * of every updated cell's encoding per launch, so a temporally blocked launch
 * advancing K generations books its cells once, not K times. */
int life_dev_kernel_work(life_dev *d, double *cell_updates_per_launch, double *valu_ops_per_launch);
/* Partitioned shards, timing on: mean device time per overlapped block
 * (one exchange period: 1 generation, or up to K with temporal layouts) of
 * its phases, each shard's blocks averaged -- the boundary-ring kernels
 * (compute stream), the interior kernel (second compute stream, concurrent),
 * the halo exchange of the ring's new state (comm stream: pack, ncclSend /
 * ncclRecv or local copies, unpack; from the moment the ring is done), and
 * the whole block from the ring's start to the join of the three streams.
 * block - interior is what the halo and ring add to the critical path (0 when
 * fully hidden).  Zeros when no block was timed (unpartitioned grids). */
int life_dev_phase_stats(life_dev *d, double *ring_ms, double *interior_ms, double *halo_ms, double *block_ms,
                         int64_t *blocks);
/* Timing on: where the wall time of the LAST life_dev_step call went
 * (measurement support; no reference counterpart -- life_cart.c times whole
 * runs with MPI_Wtime).  host_enqueue_ms: CPU time spent inside the call
 * (every launch, event, RCCL group and copy it enqueues; the call returns
 * before the device finishes); pass_enqueue_max_ms: the longest single pass
 * (one generation_block / one generation) of it; passes: its passes;
 * device_span_ms: from the first piece of work of the call starting on the
 * device to the last one ending, max over the local shards (HIP events at
 * the call's two ends on the compute stream, where the call's streams are
 * joined).  A caller that brackets the call plus a sync with its own clock
 * sees elapsed - device_span = launch latency + host-side gaps + the sync's
 * wake-up.  Zeros before the first timed call. */
int life_dev_call_stats(life_dev *d, double *host_enqueue_ms, double *pass_enqueue_max_ms, int64_t *passes,
                        double *device_span_ms);

/* Stencil tuning for the whole process, per kernel family (-1: both): rows
 * each lane walks (16/32/64) and rows of loads kept in flight (2/4/8, or 18
 * = a 16-row strip's every row loaded before the first is computed; other
 * row counts then use 4); 0 keeps the current value.  Defaults come from measurement;
 * LIFE_STEP_ROWS / LIFE_STEP_DEPTH override them at load time. */
int life_tune(int kernel, int rows, int depth);

/* Temporal (generations_per_exchange = K > 1) tile height of encoding
 * `kernel` (-1: both, each taking the value if valid for it): register rows
 * per wave -- bit: 16/24 rows of 64-cell pairs (default 24), byte: 32/48
 * rows of 32-cell words (default 48); a tile is one workgroup of 8
 * vertically stacked waves, waves*rows - 2*ghost owned rows;
 * 0 keeps the current values; LIFE_TEMPORAL_ROWS / LIFE_TEMPORAL_ROWS_BYTE
 * override at load time. */
int life_tune_temporal(int kernel, int rows);

/* Measured HBM copy ceiling of `device` ("also report a
 * measured stream-copy ceiling"): a 16-B-per-lane grid-stride copy kernel over
 * two fresh `bytes`-sized buffers, best of `reps` runs timed with HIP events;
 * *gbps = 2 * bytes (read + write) / time.  Allocates and frees its buffers. */
int life_measure_copy(int device, int64_t bytes, int reps, double *gbps);

/* life_free (life_cart.c:146-157). */
void life_dev_destroy(life_dev *d);

#ifdef __cplusplus
}
#endif
#endif /* LIFE_MI355X_H */
