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
 *   --live            print the live-cell count after the run to stderr
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

/* life_save_vtk: life_cart.c:159-187, byte-identical output. */
static int save_vtk(const char *path, int64_t nx, int64_t ny, const uint8_t *grid) {
    struct stat st;
    if (stat("vtk", &st) == -1) mkdir("vtk", 0700);
    FILE *f = fopen(path, "w");
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
    /* "%d\n" per cell, y outer, x inner: 2 bytes per 0/1 cell. */
    const size_t chunk = 1 << 20;
    char *buf = (char *)malloc(2 * chunk);
    const int64_t n = nx * ny;
    for (int64_t i = 0; i < n; i += chunk) {
        const int64_t m = n - i < (int64_t)chunk ? n - i : (int64_t)chunk;
        for (int64_t k = 0; k < m; k++) {
            buf[2 * k] = grid[i + k] ? '1' : '0';
            buf[2 * k + 1] = '\n';
        }
        fwrite(buf, 1, (size_t)(2 * m), f);
    }
    free(buf);
    return fclose(f) == 0 ? LIFE_OK : LIFE_EIO;
}

int main(int argc, char **argv) {
    const char *cfg_path = NULL;
    int gpus = 1, kernel = LIFE_KERNEL_BIT, vtk = 1, live = 0, have_random = 0;
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
        else if (!strcmp(s, "--live")) live = 1;
        else if (s[0] != '-' && !cfg_path) cfg_path = s;
        else {
            cfg_path = NULL;
            have_random = 0;
            break;
        }
    }
    if (!cfg_path && !have_random) {
        printf("Usage: %s input file.\n", argv[0]); /* life_cart.c:53-56 */
        return 0;
    }
    if (kernel < 0 || gpus < 1) {
        fprintf(stderr, "life_mi355x: bad --kernel/--gpus\n");
        return 1;
    }

    cfg_t c = {0, 1, 0, 0, 0, NULL};
    if (cfg_path && load_cfg(cfg_path, &c) != LIFE_OK) {
        fprintf(stderr, "life_mi355x: cannot read config '%s'\n", cfg_path);
        return 1;
    }
    if (o_nx > 0) c.nx = o_nx;
    if (o_ny > 0) c.ny = o_ny;
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
    uint8_t *grid = NULL;
    if (vtk || !have_random) {
        grid = (uint8_t *)calloc((size_t)(c.nx * c.ny), 1);
        if (!grid) die("host grid", LIFE_ENOMEM);
    }
    if (have_random) {
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
        if (vtk && i % c.save_steps == 0) {
            if ((rc = life_dev_gather(d, grid))) die("gather", rc);
            snprintf(path, sizeof path, "vtk/life_%06lld.vtk", (long long)i);
            if ((rc = save_vtk(path, c.nx, c.ny, grid))) die(path, rc);
        }
        int64_t n = c.steps - i;
        if (vtk) {
            const int64_t to_save = c.save_steps - i % c.save_steps;
            if (to_save < n) n = to_save;
        }
        if ((rc = life_dev_step(d, n))) die("step", rc);
        i += n;
    }
    if ((rc = life_dev_sync(d))) die("sync", rc);
    const double t1 = now_s();
    printf("%f\n", t1 - t0);
    if (live) fprintf(stderr, "live %lld\n", (long long)life_dev_live_count(d));
    life_dev_destroy(d);
    free(grid);
    return 0;
}
