/*
 * life.c -- reference-compatible driver over the MI355X C ABI.
 *
 * Drop-in for the reference programs' main() (6-cartesian/life_cart.c:51-85,
 * 5-gather/life_mpi.c:36-63, 3-life/life_mpi.c:38-72):
 *
 *   life_mi355x file.cfg            same .cfg, same vtk/life_%06d.vtk bytes,
 *                                   same "%f\n" elapsed seconds on stdout
 *
 * Extensions (all optional; without them the program behaves as the
 * reference with one process and one GPU):
 *   --gpus N          shards driven by this process (one per GPU; with more
 *                     shards than GPUs they share devices, LOCAL transport)
 *   --kernel byte|bit cell encoding (default bit)
 *   --partition cart|rows|cols|auto   shard shape (life_dims_choose; default
 *                     cart = MPI_Dims_create as life_cart.c:117-118; rows =
 *                     the 1-D strips of 3-life/5-gather; the grid is the same)
 *   --nx N --ny N --steps N --save-steps N   override the .cfg header
 *   --random SEED[,DENSITY]                  device-side random init instead
 *                                            of the .cfg cells (no file needed)
 *   --no-vtk          skip frame output (timing runs)
 *   --format vtk|bits frame format: the reference's VTK text (default) or a
 *                     packed binary dump vtk/life_%06d.bits (checkpoint)
 *   --resume FILE     start from a .bits dump instead of the .cfg cells
 *   --live            print the live-cell count after the run to stderr
 *   --rank-mode       one-process-per-GPU mode even without a launcher (world 1)
 *
 * Under a launcher -- `torchrun --nproc-per-node P`, `mpirun -np P`
 * (MPICH: PMI_RANK/PMI_SIZE, Open MPI: OMPI_COMM_WORLD_*), as the reference
 * is run (3-life/job_life.sh:8) -- every process drives the one Cartesian
 * block of its rank on GPU LOCAL_RANK; the RCCL unique id goes from rank 0 to
 * the others over TCP (bootstrap.c); rank P-1 (the root of life_collect,
 * life_cart.c:283-286) writes the frames and prints the time.
 *
 * Frames: the VTK cell text is formatted on the device
 * (life_dev_gather_vtk) and written while the next generations run (the
 * step call is asynchronous), inside the reference's timed region.
 *
 * Differences from the reference, on purpose: malformed .cfg files and
 * save_steps <= 0 are errors (the reference loops forever / raises SIGFPE),
 * coordinates wrap with a true modulo (the reference's (i+nx)%nx is only
 * defined for i >= -nx), and sizes are 64-bit.
 */
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "bootstrap.h"
#include "life_mi355x.h"

static void die(const char *what, int rc) {
    fprintf(stderr, "life_mi355x: %s: %s%s%s\n", what, life_strerror(rc), *life_last_error() ? ": " : "",
            life_last_error());
    exit(1);
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static int64_t wrapi(int64_t i, int64_t n) { return ((i % n) + n) % n; }

typedef struct {
    int64_t steps, save_steps, nx, ny;
    uint8_t *grid; /* nx*ny 0/1 cells, row-major (NULL until loaded) */
} cfg_t;

/* .cfg loader: life_cart.c:92-111.  "steps\n save_steps\n nx ny\n" then one
 * "i j" live cell per line until EOF; cell (i, j) wraps periodically
 * (life_cart.c:106-109).  The file is mapped and the cell lines are parsed by
 * up to 16 threads, each on a line-aligned chunk writing straight into the
 * grid (a 32768^2 random pattern is a ~6 GB file).  A chunk whose token count
 * is odd (pairs not one per line) sends the whole body to the sequential
 * parser, which pairs tokens across lines like the reference's fscanf loop. */
typedef struct {
    const char *p, *end;
    int64_t nx, ny;
    uint8_t *grid;
    int status; /* 0 ok, 1 odd token count, 2 malformed */
} parse_job;

static int next_int(const char **pp, const char *end, long long *v) {
    const char *p = *pp;
    while (p < end && (*p == ' ' || *p == '\n' || *p == '\t' || *p == '\r')) p++;
    if (p == end) {
        *pp = p;
        return 0; /* EOF */
    }
    int neg = 0;
    if (*p == '-' || *p == '+') neg = *p++ == '-';
    if (p == end || *p < '0' || *p > '9') return -1;
    long long x = 0;
    while (p < end && *p >= '0' && *p <= '9') x = x * 10 + (*p++ - '0');
    if (p < end && !(*p == ' ' || *p == '\n' || *p == '\t' || *p == '\r')) return -1;
    *v = neg ? -x : x;
    *pp = p;
    return 1;
}

static void *parse_cells(void *arg) {
    parse_job *jb = (parse_job *)arg;
    const char *p = jb->p;
    long long i, j;
    for (;;) {
        int r = next_int(&p, jb->end, &i);
        if (r == 0) break;
        if (r < 0) {
            jb->status = 2;
            return NULL;
        }
        r = next_int(&p, jb->end, &j);
        if (r == 0) {
            jb->status = 1;
            return NULL;
        }
        if (r < 0) {
            jb->status = 2;
            return NULL;
        }
        /* u0[ind(i, j)] = 1; threads may store the same cell (duplicates,
         * wrapped coordinates): relaxed atomic stores, no data race */
        __atomic_store_n(&jb->grid[wrapi(j, jb->ny) * jb->nx + wrapi(i, jb->nx)], (uint8_t)1, __ATOMIC_RELAXED);
    }
    jb->status = 0;
    return NULL;
}

static int load_cfg(const char *path, cfg_t *c, int64_t o_nx, int64_t o_ny) {
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return LIFE_EIO;
    struct stat st;
    if (fstat(fd, &st) != 0) {
        close(fd);
        return LIFE_EIO;
    }
    const size_t len = (size_t)st.st_size;
    const char *base = len ? (const char *)mmap(NULL, len, PROT_READ, MAP_PRIVATE, fd, 0) : "";
    close(fd);
    if (base == MAP_FAILED) return LIFE_EIO;
    const char *p = base, *end = base + len;
    long long v[4];
    int rc = LIFE_OK;
    for (int k = 0; k < 4 && rc == LIFE_OK; k++)
        if (next_int(&p, end, &v[k]) != 1) rc = LIFE_EIO;
    if (rc == LIFE_OK && (v[2] <= 0 || v[3] <= 0)) rc = LIFE_EIO;
    if (rc == LIFE_OK) {
        c->steps = v[0];
        c->save_steps = v[1];
        c->nx = o_nx > 0 ? o_nx : v[2]; /* --nx/--ny override the header before the cells wrap */
        c->ny = o_ny > 0 ? o_ny : v[3];
        c->grid = (uint8_t *)calloc((size_t)(c->nx * c->ny), 1);
        if (!c->grid) rc = LIFE_ENOMEM;
    }
    if (rc == LIFE_OK) {
        enum { kMaxThreads = 16 };
        long np = sysconf(_SC_NPROCESSORS_ONLN);
        int nt = (int)((size_t)(end - p) / (1 << 22)); /* >= 4 MiB per thread */
        if (nt > kMaxThreads) nt = kMaxThreads;
        if (nt > np) nt = (int)np;
        if (nt < 1) nt = 1;
        parse_job jobs[kMaxThreads];
        pthread_t th[kMaxThreads];
        const char *q = p;
        for (int t = 0; t < nt; t++) { /* line-aligned chunks */
            const char *e = t == nt - 1 ? end : p + (size_t)(end - p) * (size_t)(t + 1) / (size_t)nt;
            while (e < end && *e != '\n') e++;
            jobs[t] = (parse_job){q, e, c->nx, c->ny, c->grid, 0};
            q = e;
        }
        int started = 0;
        for (int t = 1; t < nt; t++)
            if (pthread_create(&th[t], NULL, parse_cells, &jobs[t]) == 0) started = t;
            else break;
        parse_cells(&jobs[0]);
        for (int t = 1; t <= started; t++) pthread_join(th[t], NULL);
        for (int t = started + 1; t < nt; t++) parse_cells(&jobs[t]); /* threads that did not start */
        int odd = 0;
        for (int t = 0; t < nt; t++) {
            if (jobs[t].status == 2) rc = LIFE_EIO;
            odd |= jobs[t].status == 1;
        }
        if (rc == LIFE_OK && odd) { /* pairs split across lines: one sequential pass */
            parse_job all = {p, end, c->nx, c->ny, c->grid, 0};
            parse_cells(&all);
            if (all.status) rc = LIFE_EIO;
        }
    }
    if (len) munmap((void *)base, len);
    if (rc != LIFE_OK) {
        free(c->grid);
        c->grid = NULL;
    }
    return rc;
}

static FILE *open_frame(const char *path) {
    struct stat st;
    if (stat("vtk", &st) == -1) mkdir("vtk", 0700); /* life_cart.c:163-166 */
    return fopen(path, "w");
}

/* life_save_vtk: life_cart.c:159-187, byte-identical output; `body` is the
 * "%d\n"-per-cell text (y outer, x inner) formatted by life_dev_gather_vtk. */
static int save_vtk(const char *path, int64_t nx, int64_t ny, const char *body) {
    FILE *f = open_frame(path);
    if (!f) return LIFE_EIO;
    fprintf(f, "# vtk DataFile Version 3.0\n");
    fprintf(f, "Created by write_to_vtk2d\n");
    fprintf(f, "ASCII\n");
    fprintf(f, "DATASET STRUCTURED_POINTS\n");
    fprintf(f, "DIMENSIONS %lld %lld 1\n", (long long)nx + 1, (long long)ny + 1);
    fprintf(f, "SPACING %d %d 0.0\n", 1, 1);
    fprintf(f, "ORIGIN %d %d 0.0\n", 0, 0);
    fprintf(f, "CELL_DATA %lld\n", (long long)(nx * ny));
    fprintf(f, "SCALARS life int 1\n");
    fprintf(f, "LOOKUP_TABLE life_table\n");
    const size_t n = (size_t)(2 * nx * ny);
    const int ok = fwrite(body, 1, n, f) == n;
    return fclose(f) == 0 && ok ? LIFE_OK : LIFE_EIO;
}

/* Packed binary frame (extension, not in the reference): a text line
 * "LIFEBITS 1 <nx> <ny> <generation>\n", then ny rows of ceil(nx/8) bytes,
 * cell x of a row at bit (x & 7) of byte (x >> 3) -- packed on the device
 * (life_dev_gather_bits), written as one block. */
static int save_bits(const char *path, int64_t nx, int64_t ny, int64_t gen, const uint8_t *packed) {
    FILE *f = open_frame(path);
    if (!f) return LIFE_EIO;
    fprintf(f, "LIFEBITS 1 %lld %lld %lld\n", (long long)nx, (long long)ny, (long long)gen);
    const size_t n = (size_t)(ny * ((nx + 7) / 8));
    const int ok = fwrite(packed, 1, n, f) == n;
    return fclose(f) == 0 && ok ? LIFE_OK : LIFE_EIO;
}

static int load_bits(const char *path, int64_t *nx, int64_t *ny, int64_t *gen, uint8_t **grid) {
    FILE *f = fopen(path, "r");
    if (!f) return LIFE_EIO;
    long long v, a, b, g;
    if (fscanf(f, "LIFEBITS %lld %lld %lld %lld", &v, &a, &b, &g) != 4 || v != 1 || a <= 0 || b <= 0 || g < 0 ||
        fgetc(f) != '\n') {
        fclose(f);
        return LIFE_EIO;
    }
    const int64_t rb = (a + 7) / 8;
    uint8_t *row = (uint8_t *)malloc((size_t)rb);
    uint8_t *out = (uint8_t *)malloc((size_t)(a * b));
    int ok = row && out;
    for (int64_t y = 0; y < b && ok; y++) {
        ok = fread(row, 1, (size_t)rb, f) == (size_t)rb;
        for (int64_t x = 0; x < a && ok; x++) out[y * a + x] = (uint8_t)((row[x >> 3] >> (x & 7)) & 1u);
    }
    free(row);
    fclose(f);
    if (!ok) {
        free(out);
        return LIFE_EIO;
    }
    *nx = a;
    *ny = b;
    *gen = g;
    *grid = out;
    return LIFE_OK;
}

int main(int argc, char **argv) {
    const char *cfg_path = NULL, *resume = NULL;
    int gpus = 1, kernel = LIFE_KERNEL_BIT, vtk = 1, live = 0, have_random = 0, bits = 0, force_rank = 0;
    int partition = LIFE_PARTITION_CART;
    long long o_nx = -1, o_ny = -1, o_steps = -1, o_save = -1;
    unsigned long long seed = 0;
    double density = 0.5;
    for (int a = 1; a < argc; a++) {
        const char *s = argv[a];
        const int more = a + 1 < argc;
        if (!strcmp(s, "--gpus") && more) gpus = atoi(argv[++a]);
        else if (!strcmp(s, "--partition") && more) {
            const char *p = argv[++a];
            partition = !strcmp(p, "cart")   ? LIFE_PARTITION_CART
                        : !strcmp(p, "rows") ? LIFE_PARTITION_ROWS
                        : !strcmp(p, "cols") ? LIFE_PARTITION_COLS
                        : !strcmp(p, "auto") ? LIFE_PARTITION_AUTO
                                             : -1;
        }
        else if (!strcmp(s, "--kernel") && more) {
            const char *k = argv[++a];
            kernel = !strcmp(k, "byte") ? LIFE_KERNEL_BYTE : !strcmp(k, "bit") ? LIFE_KERNEL_BIT : -1;
        } else if (!strcmp(s, "--nx") && more) o_nx = atoll(argv[++a]);
        else if (!strcmp(s, "--ny") && more) o_ny = atoll(argv[++a]);
        else if (!strcmp(s, "--steps") && more) o_steps = atoll(argv[++a]);
        else if (!strcmp(s, "--save-steps") && more) o_save = atoll(argv[++a]);
        else if (!strcmp(s, "--random") && more) {
            have_random = 1;
            char *end;
            seed = strtoull(argv[++a], &end, 10);
            if (*end == ',') {
                char *dend;
                density = strtod(end + 1, &dend);
                if (*dend || !(density >= 0.0 && density <= 1.0)) {
                    fprintf(stderr, "life_mi355x: --random density must be in [0, 1]\n");
                    return 1;
                }
            }
        } else if (!strcmp(s, "--no-vtk")) vtk = 0;
        else if (!strcmp(s, "--format") && more) {
            const char *fm = argv[++a];
            bits = !strcmp(fm, "bits") ? 1 : !strcmp(fm, "vtk") ? 0 : -1;
        } else if (!strcmp(s, "--resume") && more) resume = argv[++a];
        else if (!strcmp(s, "--live")) live = 1;
        else if (!strcmp(s, "--rank-mode")) force_rank = 1;
        else if (s[0] != '-' && !cfg_path) cfg_path = s;
        else {
            cfg_path = NULL;
            have_random = 0;
            break;
        }
    }
    if (!cfg_path && !have_random && !resume) {
        printf("Usage: %s input file.\n", argv[0]); /* life_cart.c:53-56 */
        return 0;
    }
    if (kernel < 0 || gpus < 1 || bits < 0 || partition < 0) {
        fprintf(stderr, "life_mi355x: bad --kernel/--gpus/--format/--partition\n");
        return 1;
    }
    /* one process per GPU under a launcher (life_cart.c:114-115 takes rank and
     * size from MPI; here from the launcher's environment) */
    int rank = 0, world = 1, local_rank = 0;
    const int launched = life_launcher_ranks(&rank, &world, &local_rank);
    if (launched < 0) {
        fprintf(stderr, "life_mi355x: inconsistent launcher rank variables\n");
        return 1;
    }
    const int rank_mode = launched == 1 || force_rank;
    if (rank_mode && gpus != 1) {
        fprintf(stderr, "life_mi355x: --gpus drives several GPUs from one process; under a launcher every "
                        "rank drives its own GPU (drop --gpus)\n");
        return 1;
    }
    const int root = world - 1; /* life_collect's root: cart rank (dims0-1, dims1-1) = size-1 */

    cfg_t c = {0, 1, 0, 0, NULL};
    if (cfg_path && load_cfg(cfg_path, &c, resume ? -1 : o_nx, resume ? -1 : o_ny) != LIFE_OK) {
        fprintf(stderr, "life_mi355x: cannot read config '%s'\n", cfg_path);
        return 1;
    }
    uint8_t *resumed = NULL;
    int64_t gen0 = 0; /* generation the run starts from (a --resume dump's) */
    if (resume && load_bits(resume, &c.nx, &c.ny, &gen0, &resumed) != LIFE_OK) {
        fprintf(stderr, "life_mi355x: cannot read dump '%s'\n", resume);
        return 1;
    }
    if (o_nx > 0 && !resume) c.nx = o_nx;
    if (o_ny > 0 && !resume) c.ny = o_ny;
    if (o_steps >= 0) c.steps = o_steps;
    if (o_save >= 0) c.save_steps = o_save;
    if (c.nx <= 0 || c.ny <= 0 || c.steps < 0 || c.save_steps <= 0) {
        fprintf(stderr, "life_mi355x: bad sizes nx=%lld ny=%lld steps=%lld save_steps=%lld\n",
                (long long)c.nx, (long long)c.ny, (long long)c.steps, (long long)c.save_steps);
        return 1;
    }

    life_dev *d = NULL;
    int dims[2];
    int rc = life_dims_choose(c.nx, c.ny, rank_mode ? world : gpus, partition, dims);
    if (rc == LIFE_OK && rank_mode) {
        uint8_t uid[LIFE_UID_BYTES];
        memset(uid, 0, sizeof uid);
        if (rank == 0 && (rc = life_get_unique_id(uid)) != LIFE_OK) die("unique id", rc);
        if (life_bootstrap_id(rank, world, uid, 120.0) != 0) {
            fprintf(stderr, "life_mi355x: rank %d/%d: RCCL id bootstrap over TCP failed\n", rank, world);
            return 1;
        }
        const int ndev = life_device_count();
        if (ndev <= 0) die("no HIP device", LIFE_EHIP);
        /* RCCL prints its version banner to stdout when a communicator is
         * made; stdout carries only the elapsed time (as the reference's,
         * which run_life.sh appends to times.txt): send the banner to stderr */
        fflush(stdout);
        const int saved = dup(STDOUT_FILENO);
        if (saved >= 0) dup2(STDERR_FILENO, STDOUT_FILENO);
        rc = life_dev_create_rank(c.nx, c.ny, kernel, rank, world, dims[0], dims[1], uid, local_rank % ndev, &d);
        fflush(stdout);
        if (saved >= 0) {
            dup2(saved, STDOUT_FILENO);
            close(saved);
        }
    } else if (rc == LIFE_OK) {
        rc = life_dev_create_ex(c.nx, c.ny, gpus, dims[0], dims[1], kernel, LIFE_XPORT_AUTO, &d);
    }
    if (rc) die("create", rc);
    const int writer = !rank_mode || rank == root; /* the process that writes frames and prints */
    uint8_t *grid = NULL; /* packed rows: bits frames */
    char *body = NULL;    /* VTK cell text */
    if (vtk && bits && writer) {
        grid = (uint8_t *)calloc((size_t)(c.ny * ((c.nx + 7) / 8)), 1);
        if (!grid) die("host grid", LIFE_ENOMEM);
    }
    if (vtk && !bits && writer) {
        body = (char *)malloc((size_t)(2 * c.nx * c.ny));
        if (!body) die("host frame", LIFE_ENOMEM);
    }
    if (resume) {
        rc = life_dev_upload(d, resumed);
        free(resumed);
    } else if (have_random) {
        rc = life_dev_fill_random(d, seed, density >= 1.0 ? 0xFFFFFFFFu : (uint32_t)(density * 4294967296.0));
    } else {
        rc = life_dev_upload(d, c.grid);
    }
    if (rc) die("init", rc);
    free(c.grid);
    c.grid = NULL;

    /* life_cart.c:62-80: the timer starts after init and covers the frame
     * collects + VTK writes and every generation.  Generations and frame
     * numbers are absolute: a resumed run continues the dump's sequence and
     * --steps counts from generation 0. */
    if ((rc = life_dev_barrier(d))) die("barrier", rc);
    const double t0 = now_s();
    char path[64];
    for (int64_t i = gen0; i < c.steps;) {
        const int save = vtk && i % c.save_steps == 0;
        if (save) { /* collect (blocking, every rank), then write it while the GPU steps on */
            if ((rc = bits ? life_dev_gather_bits(d, grid) : life_dev_gather_vtk(d, body))) die("gather", rc);
            snprintf(path, sizeof path, bits ? "vtk/life_%06lld.bits" : "vtk/life_%06lld.vtk", (long long)i);
        }
        int64_t n = c.steps - i;
        if (vtk) {
            const int64_t to_save = c.save_steps - i % c.save_steps;
            if (to_save < n) n = to_save;
        }
        if ((rc = life_dev_step(d, n))) die("step", rc); /* asynchronous */
        if (save && writer && (rc = bits ? save_bits(path, c.nx, c.ny, i, grid) : save_vtk(path, c.nx, c.ny, body)))
            die(path, rc);
        i += n;
    }
    if ((rc = life_dev_sync(d))) die("sync", rc);
    if ((rc = life_dev_barrier(d))) die("barrier", rc);
    const double t1 = now_s();
    if (writer) printf("%f\n", t1 - t0);
    if (live) {
        const int64_t n = life_dev_live_count(d); /* collective in rank mode */
        if (writer) fprintf(stderr, "live %lld\n", (long long)n);
    }
    life_dev_destroy(d);
    free(grid);
    free(body);
    return 0;
}
