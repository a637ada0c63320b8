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
 *   --nx N --ny N --steps N --save-steps N   override the .cfg header
 *   --random SEED[,DENSITY]                  device-side random init instead
 *                                            of the .cfg cells (no file needed)
 *   --no-vtk          skip frame output (timing runs)
 *   --format vtk|bits frame format: the reference's VTK text (default) or a
 *                     packed binary dump vtk/life_%06d.bits (checkpoint)
 *   --resume FILE     start from a .bits dump instead of the .cfg cells
 *   --live            print the live-cell count after the run to stderr
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
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>

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
    int64_t ncells;   /* live-cell lines */
    int64_t *cells;   /* x0 y0 x1 y1 ... */
} cfg_t;

/* .cfg loader: life_cart.c:92-111.  "steps\n save_steps\n nx ny\n" then one
 * "i j" live cell per line until EOF. */
static int load_cfg(const char *path, cfg_t *c) {
    FILE *f = fopen(path, "r");
    if (!f) return LIFE_EIO;
    long long v[4];
    for (int k = 0; k < 4; k++)
        if (fscanf(f, "%lld", &v[k]) != 1) {
            fclose(f);
            return LIFE_EIO;
        }
    c->steps = v[0];
    c->save_steps = v[1];
    c->nx = v[2];
    c->ny = v[3];
    int64_t cap = 1024;
    c->cells = (int64_t *)malloc(sizeof(int64_t) * 2 * cap);
    c->ncells = 0;
    for (;;) {
        long long i, j;
        int r = fscanf(f, "%lld", &i);
        if (r == EOF) break;
        if (r != 1 || fscanf(f, "%lld", &j) != 1) {
            fclose(f);
            return LIFE_EIO;
        }
        if (c->ncells == cap) {
            cap *= 2;
            c->cells = (int64_t *)realloc(c->cells, sizeof(int64_t) * 2 * cap);
        }
        c->cells[2 * c->ncells] = i;
        c->cells[2 * c->ncells + 1] = j;
        c->ncells++;
    }
    fclose(f);
    return LIFE_OK;
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
 * cell x of a row at bit (x & 7) of byte (x >> 3). */
static int save_bits(const char *path, int64_t nx, int64_t ny, int64_t gen, const uint8_t *grid) {
    FILE *f = open_frame(path);
    if (!f) return LIFE_EIO;
    fprintf(f, "LIFEBITS 1 %lld %lld %lld\n", (long long)nx, (long long)ny, (long long)gen);
    const int64_t rb = (nx + 7) / 8;
    uint8_t *row = (uint8_t *)malloc((size_t)rb);
    int ok = 1;
    for (int64_t y = 0; y < ny && ok; y++) {
        memset(row, 0, (size_t)rb);
        for (int64_t x = 0; x < nx; x++) row[x >> 3] |= (uint8_t)((grid[y * nx + x] != 0) << (x & 7));
        ok = fwrite(row, 1, (size_t)rb, f) == (size_t)rb;
    }
    free(row);
    return fclose(f) == 0 && ok ? LIFE_OK : LIFE_EIO;
}

static int load_bits(const char *path, int64_t *nx, int64_t *ny, uint8_t **grid) {
    FILE *f = fopen(path, "r");
    if (!f) return LIFE_EIO;
    long long v, a, b, g;
    if (fscanf(f, "LIFEBITS %lld %lld %lld %lld", &v, &a, &b, &g) != 4 || v != 1 || a <= 0 || b <= 0 ||
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
    *grid = out;
    return LIFE_OK;
}

int main(int argc, char **argv) {
    const char *cfg_path = NULL, *resume = NULL;
    int gpus = 1, kernel = LIFE_KERNEL_BIT, vtk = 1, live = 0, have_random = 0, bits = 0;
    long long o_nx = -1, o_ny = -1, o_steps = -1, o_save = -1;
    unsigned long long seed = 0;
    double density = 0.5;
    for (int a = 1; a < argc; a++) {
        const char *s = argv[a];
        const int more = a + 1 < argc;
        if (!strcmp(s, "--gpus") && more) gpus = atoi(argv[++a]);
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
            if (*end == ',') density = atof(end + 1);
        } else if (!strcmp(s, "--no-vtk")) vtk = 0;
        else if (!strcmp(s, "--format") && more) {
            const char *fm = argv[++a];
            bits = !strcmp(fm, "bits") ? 1 : !strcmp(fm, "vtk") ? 0 : -1;
        } else if (!strcmp(s, "--resume") && more) resume = argv[++a];
        else if (!strcmp(s, "--live")) live = 1;
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
    if (kernel < 0 || gpus < 1 || bits < 0) {
        fprintf(stderr, "life_mi355x: bad --kernel/--gpus/--format\n");
        return 1;
    }

    cfg_t c = {0, 1, 0, 0, 0, NULL};
    if (cfg_path && load_cfg(cfg_path, &c) != LIFE_OK) {
        fprintf(stderr, "life_mi355x: cannot read config '%s'\n", cfg_path);
        return 1;
    }
    uint8_t *resumed = NULL;
    if (resume && load_bits(resume, &c.nx, &c.ny, &resumed) != LIFE_OK) {
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
    int rc = life_dev_create(c.nx, c.ny, gpus, kernel, &d);
    if (rc) die("create", rc);
    uint8_t *grid = NULL; /* dense cells: .cfg loading and bits frames */
    char *body = NULL;    /* VTK cell text */
    if ((vtk && bits) || (!have_random && !resume)) {
        grid = (uint8_t *)calloc((size_t)(c.nx * c.ny), 1);
        if (!grid) die("host grid", LIFE_ENOMEM);
    }
    if (vtk && !bits) {
        body = (char *)malloc((size_t)(2 * c.nx * c.ny));
        if (!body) die("host frame", LIFE_ENOMEM);
    }
    if (resume) {
        rc = life_dev_upload(d, resumed);
        free(resumed);
    } else if (have_random) {
        rc = life_dev_fill_random(d, seed, density >= 1.0 ? 0xFFFFFFFFu : (uint32_t)(density * 4294967296.0));
    } else {
        for (int64_t k = 0; k < c.ncells; k++) /* life_cart.c:106-109 */
            grid[wrapi(c.cells[2 * k + 1], c.ny) * c.nx + wrapi(c.cells[2 * k], c.nx)] = 1;
        rc = life_dev_upload(d, grid);
    }
    if (rc) die("init", rc);
    free(c.cells);

    /* life_cart.c:62-80: the timer starts after init and covers the frame
     * collects + VTK writes and every generation. */
    const double t0 = now_s();
    char path[64];
    for (int64_t i = 0; i < c.steps;) {
        const int save = vtk && i % c.save_steps == 0;
        if (save) { /* collect (blocking), then write it while the GPU steps on */
            if ((rc = bits ? life_dev_gather(d, grid) : life_dev_gather_vtk(d, body))) die("gather", rc);
            snprintf(path, sizeof path, bits ? "vtk/life_%06lld.bits" : "vtk/life_%06lld.vtk", (long long)i);
        }
        int64_t n = c.steps - i;
        if (vtk) {
            const int64_t to_save = c.save_steps - i % c.save_steps;
            if (to_save < n) n = to_save;
        }
        if ((rc = life_dev_step(d, n))) die("step", rc); /* asynchronous */
        if (save && (rc = bits ? save_bits(path, c.nx, c.ny, i, grid) : save_vtk(path, c.nx, c.ny, body)))
            die(path, rc);
        i += n;
    }
    if ((rc = life_dev_sync(d))) die("sync", rc);
    const double t1 = now_s();
    printf("%f\n", t1 - t0);
    if (live) fprintf(stderr, "live %lld\n", (long long)life_dev_live_count(d));
    life_dev_destroy(d);
    free(grid);
    free(body);
    return 0;
}
