/*
 * life_oracle.c -- CPU restatement of the reference's Game-of-Life hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see life_oracle.h).  Every function cites the
 * reference lines it restates; all paths are relative to the reference repo
 * kekoveca/MPI-and-Open-MP.
 */
#include "life_oracle.h"

#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ind(i,j) of 6-cartesian/life_cart.c:11 / 3-life/life2d.c:9, but valid for
 * every i >= -n (the reference's own precondition) and 64-bit. */
static inline int64_t wrap(int64_t i, int64_t n) { return (i + n) % n; }

/* The B3/S23 update of one cell, spelled exactly like
 * 3-life/life2d.c:108-123: n = sum of the 8 neighbours (same visiting order),
 * then u1 = 1 iff (n==3 && u0==0) || ((n==3||n==2) && u0==1). */
static inline uint8_t cell_rule(int n, uint8_t c) {
    uint8_t out = 0;
    if (n == 3 && c == 0) out = 1;
    if ((n == 3 || n == 2) && c == 1) out = 1;
    return out;
}

static void step_rows(int64_t nx, int64_t ny, const uint8_t *u0, uint8_t *u1,
                      int64_t x0, int64_t x1, int64_t y0, int64_t y1) {
    for (int64_t j = y0; j < y1; j++) {
        const uint8_t *rm = u0 + wrap(j - 1, ny) * nx;   /* row j-1 */
        const uint8_t *r0 = u0 + wrap(j, ny) * nx;       /* row j   */
        const uint8_t *rp = u0 + wrap(j + 1, ny) * nx;   /* row j+1 */
        uint8_t *o = u1 + wrap(j, ny) * nx;
        for (int64_t i = x0; i < x1; i++) {
            const int64_t im = wrap(i - 1, nx), ic = wrap(i, nx), ip = wrap(i + 1, nx);
            int n = 0;
            n += r0[ip];  /* ind(i+1, j)   life2d.c:109 */
            n += rp[ip];  /* ind(i+1, j+1) :110 */
            n += rp[ic];  /* ind(i,   j+1) :111 */
            n += r0[im];  /* ind(i-1, j)   :112 */
            n += rm[im];  /* ind(i-1, j-1) :113 */
            n += rm[ic];  /* ind(i,   j-1) :114 */
            n += rp[im];  /* ind(i-1, j+1) :115 */
            n += rm[ip];  /* ind(i+1, j-1) :116 */
            o[ic] = cell_rule(n, r0[ic]);  /* :117-123 */
        }
    }
}

void oracle_life_step(int64_t nx, int64_t ny, const uint8_t *u0, uint8_t *u1) {
    /* 3-life/life2d.c:104-130 (the pointer swap :126-129 is the caller's). */
    step_rows(nx, ny, u0, u1, 0, nx, 0, ny);
}

void oracle_life_step_block(int64_t nx, int64_t ny, const uint8_t *u0, uint8_t *u1,
                            int64_t x0, int64_t x1, int64_t y0, int64_t y1) {
    /* 6-cartesian/life_cart.c:189-210: loops j in [start1,stop1), i in [start0,stop0). */
    step_rows(nx, ny, u0, u1, x0, x1, y0, y1);
}

void oracle_step_padded(int64_t w, int64_t h, int64_t pitch, const uint8_t *in, uint8_t *out) {
    /* The same rule on a block whose 1-cell apron already holds the
     * neighbours' cells (what life_exchange leaves in u0 around the block,
     * 6-cartesian/life_cart.c:225-279). */
    for (int64_t y = 1; y <= h; y++) {
        const uint8_t *rm = in + (y - 1) * pitch, *r0 = in + y * pitch, *rp = in + (y + 1) * pitch;
        for (int64_t x = 1; x <= w; x++) {
            int n = r0[x + 1] + rp[x + 1] + rp[x] + r0[x - 1] + rm[x - 1] + rm[x] + rp[x - 1] + rm[x + 1];
            out[y * pitch + x] = cell_rule(n, r0[x]);
        }
    }
}

void oracle_life_run(int64_t nx, int64_t ny, uint8_t *grid, int64_t gens, int nthreads) {
    uint8_t *tmp = (uint8_t *)malloc((size_t)(nx * ny));
    uint8_t *a = grid, *b = tmp;
    if (nthreads < 1) nthreads = 1;
    for (int64_t g = 0; g < gens; g++) {
#ifdef _OPENMP
#pragma omp parallel num_threads(nthreads)
        {
            const int t = omp_get_thread_num(), nt = omp_get_num_threads();
            int64_t s, e;
            oracle_decomposition(ny, nt, t, &s, &e);  /* row strips, as 3-life/life_mpi.c */
            step_rows(nx, ny, a, b, 0, nx, s, e);
        }
#else
        step_rows(nx, ny, a, b, 0, nx, 0, ny);
#endif
        uint8_t *t = a; a = b; b = t;  /* life2d.c:126-129 */
    }
    if (a != grid) memcpy(grid, a, (size_t)(nx * ny));
    free(tmp);
}

uint64_t oracle_splitmix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void oracle_fill_random(int64_t nx, int64_t ny, uint64_t seed, uint32_t thr32, uint8_t *grid) {
    /* The reference has no generator; this is the build's own definition
     * (SURVEY.md §7 step 1), shared bit-for-bit with the device fill kernel. */
    const uint64_t key = oracle_splitmix64(seed);
    for (int64_t y = 0; y < ny; y++)
        for (int64_t x = 0; x < nx; x++) {
            const uint64_t idx = (uint64_t)(y * nx + x);
            grid[y * nx + x] = (uint32_t)(oracle_splitmix64(key ^ idx) >> 32) < thr32;
        }
}

void oracle_fill_random_window(int64_t nx, int64_t x0, int64_t y0, int64_t w, int64_t h, uint64_t seed,
                               uint32_t thr32, uint8_t *out) {
    const uint64_t key = oracle_splitmix64(seed);
    for (int64_t y = 0; y < h; y++)
        for (int64_t x = 0; x < w; x++) {
            const int64_t gx = ((x0 + x) % nx + nx) % nx;
            const uint64_t idx = (uint64_t)((y0 + y) * nx + gx);
            out[y * w + x] = (uint32_t)(oracle_splitmix64(key ^ idx) >> 32) < thr32;
        }
}

void oracle_decomposition(int64_t n, int p, int k, int64_t *start, int64_t *stop) {
    /* 6-cartesian/life_cart.c:217-223: equal blocks, the last takes the remainder. */
    const int64_t l = n / p;
    *start = l * k;
    *stop = *start + l;
    if (k == p - 1) *stop = n;
}

void oracle_dims_create(int n, int dims[2]) {
    /* MPI_Dims_create(n, 2, {0,0}) as called at life_cart.c:117-118: the most
     * balanced 2-factor split, dims[0] >= dims[1]. */
    int d1 = 1;
    for (int f = 1; (int64_t)f * f <= n; f++)
        if (n % f == 0) d1 = f;
    dims[0] = n / d1;
    dims[1] = d1;
}

int64_t oracle_live_count(int64_t n, const uint8_t *grid) {
    int64_t c = 0;
    for (int64_t i = 0; i < n; i++) c += grid[i] != 0;
    return c;
}
