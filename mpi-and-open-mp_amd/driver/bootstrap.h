/* bootstrap.h -- launcher rank detection and RCCL unique-id exchange (driver only). */
#ifndef LIFE_BOOTSTRAP_H
#define LIFE_BOOTSTRAP_H

#include <stdint.h>

#define LIFE_UID_BYTES 128

/* Rank, world size and node-local rank from the launcher's environment:
 * RANK/WORLD_SIZE/LOCAL_RANK (torchrun), PMI_RANK/PMI_SIZE/MPI_LOCALRANKID
 * (MPICH hydra), OMPI_COMM_WORLD_RANK/_SIZE/_LOCAL_RANK (Open MPI).
 * Returns 1 when found, 0 when the process was not started by a launcher,
 * -1 for inconsistent values. */
int life_launcher_ranks(int *rank, int *world, int *local_rank);

/* Rank 0 sends `id` to every other rank over TCP (LIFE_BOOTSTRAP_ADDR or
 * MASTER_ADDR -- an IPv4 address or a host name, resolved by getaddrinfo --
 * default 127.0.0.1; port LIFE_BOOTSTRAP_PORT, MASTER_PORT + 1, or 29517);
 * the others receive it, retrying the connection.  Every rank gives up after
 * timeout_s seconds (rank 0 when a rank never connects).  Returns 0 on
 * success, -1 on failure or timeout. */
int life_bootstrap_id(int rank, int world, uint8_t id[LIFE_UID_BYTES], double timeout_s);

#endif
