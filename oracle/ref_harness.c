/*
 * ref_harness.c -- links the REFERENCE's own serial Game of Life
 * (3-life/life2d.c, compiled from /root/reference by oracle/Makefile with
 * -Dmain=life2d_ref_main) into oracle/_ref/liblife2d_ref.so, so tests can
 * pin the restatement (life_oracle.c) against the reference's life_step,
 * life_init and life_save_vtk on inputs of any size.
 *
 * TEST INFRASTRUCTURE ONLY; never shipped in the product, never required on
 * the GPU box (tests skip what needs it when oracle/_ref is absent).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* Same layout as the reference's life_t (3-life/life2d.c:11-17). */
typedef struct {
    int nx, ny;
    int *u0;
    int *u1;
    int steps;
    int save_steps;
} life_t;

void life_init(const char *path, life_t *l);      /* 3-life/life2d.c:52-72 */
void life_free(life_t *l);                        /* :74-78 */
void life_step(life_t *l);                        /* :104-130 */
void life_save_vtk(const char *path, life_t *l);  /* :80-102 */

/* gens generations of the reference life_step on a uint8 grid (in place). */
int ref_life_run(int nx, int ny, uint8_t *grid, int gens) {
    life_t l;
    memset(&l, 0, sizeof l);
    l.nx = nx;
    l.ny = ny;
    l.u0 = (int *)calloc((size_t)nx * ny, sizeof(int));
    l.u1 = (int *)calloc((size_t)nx * ny, sizeof(int));
    if (!l.u0 || !l.u1) return -1;
    for (size_t i = 0; i < (size_t)nx * ny; i++) l.u0[i] = grid[i] ? 1 : 0;
    for (int g = 0; g < gens; g++) life_step(&l);
    for (size_t i = 0; i < (size_t)nx * ny; i++) grid[i] = (uint8_t)l.u0[i];
    life_free(&l);
    return 0;
}

/* Reference loader: fills steps/save_steps/nx/ny; if grid != NULL copies the
 * loaded cells (grid must hold nx*ny bytes: call once with NULL to size). */
int ref_load_cfg(const char *path, int *steps, int *save_steps, int *nx, int *ny, uint8_t *grid) {
    life_t l;
    memset(&l, 0, sizeof l);
    life_init(path, &l);
    *steps = l.steps;
    *save_steps = l.save_steps;
    *nx = l.nx;
    *ny = l.ny;
    if (grid)
        for (size_t i = 0; i < (size_t)l.nx * l.ny; i++) grid[i] = (uint8_t)l.u0[i];
    life_free(&l);
    return 0;
}

/* Reference VTK writer on a uint8 grid. */
int ref_save_vtk(const char *path, int nx, int ny, const uint8_t *grid) {
    life_t l;
    memset(&l, 0, sizeof l);
    l.nx = nx;
    l.ny = ny;
    l.u0 = (int *)calloc((size_t)nx * ny, sizeof(int));
    l.u1 = (int *)calloc((size_t)nx * ny, sizeof(int));
    for (size_t i = 0; i < (size_t)nx * ny; i++) l.u0[i] = grid[i];
    life_save_vtk(path, &l);
    life_free(&l);
    return 0;
}
