/*
 * life_oracle.h -- CPU restatement of the reference's Game-of-Life hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker
 * (or the timed CPU baseline).  The product (liblife_mi355x.so) never links
 * or calls it.
 *
 * Parity pins (see tests/golden/ and oracle/make_golden.py):
 *   - every frame of the reference's own .cfg patterns (glider_10x10, conf1,
 *     p46gun, big_osc, test, p46gun_big gen 10000) as produced by the
 *     reference's serial program 3-life/life2d.c compiled from source;
 *   - random grids stepped by the reference's life_step itself
 *     (3-life/life2d.c:104-130, linked through oracle/_ref).
 *
 * Cells are uint8 0/1, row-major with x fastest: idx = x + y*nx, exactly the
 * reference's ind() (6-cartesian/life_cart.c:11) but in 64-bit arithmetic.
 */
#ifndef LIFE_ORACLE_H
#define LIFE_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One generation over the whole periodic grid: 3-life/life2d.c:104-130. */
void oracle_life_step(int64_t nx, int64_t ny, const uint8_t *u0, uint8_t *u1);

/* One generation over the block [x0,x1) x [y0,y1) of a full periodic grid,
 * the way every MPI rank runs it: 6-cartesian/life_cart.c:189-215.  Cells
 * outside the block are left untouched in u1. */
void oracle_life_step_block(int64_t nx, int64_t ny, const uint8_t *u0, uint8_t *u1,
                            int64_t x0, int64_t x1, int64_t y0, int64_t y1);

/* One generation of an apron-padded block: in/out are (h+2) rows of `pitch`
 * bytes, owned cell (x,y) at in[(y+1)*pitch + x+1].  Only owned cells of
 * `out` are written.  Used by the multi-rank (gloo) plan tests. */
void oracle_step_padded(int64_t w, int64_t h, int64_t pitch, const uint8_t *in, uint8_t *out);

/* `gens` generations in place, splitting rows over `nthreads` OpenMP threads
 * (nthreads <= 1: serial).  Used as the timed CPU baseline ("port"). */
void oracle_life_run(int64_t nx, int64_t ny, uint8_t *grid, int64_t gens, int nthreads);

/* Counter-based generator shared with the device fill kernel:
 * cell(x,y) = (splitmix64(splitmix64(seed) ^ (y*nx + x)) >> 32) < thr32. */
uint64_t oracle_splitmix64(uint64_t v);
void oracle_fill_random(int64_t nx, int64_t ny, uint64_t seed, uint32_t thr32, uint8_t *grid);
/* The same generator on a w x h window of a global nx-wide grid whose
 * top-left cell is (x0, y0); x wraps modulo nx (a band across the x = 0
 * seam), y does not. */
void oracle_fill_random_window(int64_t nx, int64_t x0, int64_t y0, int64_t w, int64_t h, uint64_t seed,
                               uint32_t thr32, uint8_t *out);

/* decomposition(): 6-cartesian/life_cart.c:217-223, 64-bit. */
void oracle_decomposition(int64_t n, int p, int k, int64_t *start, int64_t *stop);

/* MPI_Dims_create(n, 2, dims) with dims = {0,0}: balanced, non-increasing. */
void oracle_dims_create(int n, int dims[2]);

int64_t oracle_live_count(int64_t n, const uint8_t *grid);

#ifdef __cplusplus
}
#endif
#endif
