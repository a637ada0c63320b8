/*
 * bootstrap.c -- launcher detection and RCCL unique-id exchange for the
 * driver's one-process-per-GPU mode.
 *
 * The reference is started as `mpirun -np P ./life_cart file.cfg`
 * (3-life/job_life.sh:8, 3-life/run_life.sh:5) and gets its rank and size
 * from MPI_Comm_rank / MPI_Comm_size (life_cart.c:114-115).  This driver has
 * no MPI: it reads the rank variables the common launchers export and passes
 * the 128-byte RCCL unique id from rank 0 to the others over one TCP
 * connection each (single node: 127.0.0.1 unless LIFE_BOOTSTRAP_ADDR /
 * MASTER_ADDR says otherwise).
 */
#include "bootstrap.h"

#include <arpa/inet.h>
#include <errno.h>
#include <netinet/in.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

static int env_int(const char *name, int *v) {
    const char *e = getenv(name);
    if (!e || !*e) return 0;
    char *end;
    const long x = strtol(e, &end, 10);
    if (*end || x < 0 || x > 1 << 20) return 0;
    *v = (int)x;
    return 1;
}

int life_launcher_ranks(int *rank, int *world, int *local_rank) {
    static const char *const names[][3] = {
        {"RANK", "WORLD_SIZE", "LOCAL_RANK"},                                             /* torchrun */
        {"PMI_RANK", "PMI_SIZE", "MPI_LOCALRANKID"},                                      /* MPICH hydra */
        {"OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_RANK"},  /* Open MPI */
    };
    for (size_t k = 0; k < sizeof names / sizeof names[0]; k++) {
        int r, w;
        if (env_int(names[k][0], &r) && env_int(names[k][1], &w)) {
            if (w < 1 || r >= w) return -1;
            int l = r;
            if (!env_int(names[k][2], &l)) l = r;
            *rank = r;
            *world = w;
            *local_rank = l;
            return 1;
        }
    }
    return 0;
}

static int bootstrap_port(void) {
    int p;
    if (env_int("LIFE_BOOTSTRAP_PORT", &p) && p > 0 && p < 65536) return p;
    if (env_int("MASTER_PORT", &p) && p > 0 && p < 65535) return p + 1;
    return 29517;
}

static const char *bootstrap_addr(void) {
    const char *a = getenv("LIFE_BOOTSTRAP_ADDR");
    if (a && *a) return a;
    a = getenv("MASTER_ADDR");
    return a && *a ? a : "127.0.0.1";
}

static int full_io(int fd, uint8_t *buf, size_t n, int send_) {
    size_t done = 0;
    while (done < n) {
        const ssize_t k = send_ ? send(fd, buf + done, n - done, MSG_NOSIGNAL) : recv(fd, buf + done, n - done, 0);
        if (k <= 0) {
            if (k < 0 && errno == EINTR) continue;
            return -1;
        }
        done += (size_t)k;
    }
    return 0;
}

/* Message: "LIFEUID1" + rank-0 world size (4 bytes, little endian) + id. */
enum { kMagic = 8, kMsg = 8 + 4 + LIFE_UID_BYTES };

int life_bootstrap_id(int rank, int world, uint8_t id[LIFE_UID_BYTES], double timeout_s) {
    if (world <= 1) return 0;
    struct sockaddr_in sa;
    memset(&sa, 0, sizeof sa);
    sa.sin_family = AF_INET;
    sa.sin_port = htons((uint16_t)bootstrap_port());
    if (inet_pton(AF_INET, bootstrap_addr(), &sa.sin_addr) != 1) return -1;
    uint8_t msg[kMsg];
    if (rank == 0) {
        const int ls = socket(AF_INET, SOCK_STREAM, 0);
        if (ls < 0) return -1;
        const int one = 1;
        setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
        if (bind(ls, (struct sockaddr *)&sa, sizeof sa) != 0 || listen(ls, world) != 0) {
            close(ls);
            return -1;
        }
        memcpy(msg, "LIFEUID1", kMagic);
        for (int b = 0; b < 4; b++) msg[kMagic + b] = (uint8_t)((unsigned)world >> (8 * b));
        memcpy(msg + kMagic + 4, id, LIFE_UID_BYTES);
        int rc = 0;
        for (int k = 1; k < world && rc == 0; k++) {
            const int fd = accept(ls, NULL, NULL);
            if (fd < 0) {
                if (errno == EINTR) {
                    k--;
                    continue;
                }
                rc = -1;
                break;
            }
            rc = full_io(fd, msg, sizeof msg, 1);
            close(fd);
        }
        close(ls);
        return rc;
    }
    struct timespec t0, t;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (;;) {  /* rank 0 may not be listening yet */
        const int fd = socket(AF_INET, SOCK_STREAM, 0);
        if (fd < 0) return -1;
        if (connect(fd, (struct sockaddr *)&sa, sizeof sa) == 0) {
            const int rc = full_io(fd, msg, sizeof msg, 0);
            close(fd);
            if (rc != 0 || memcmp(msg, "LIFEUID1", kMagic) != 0) return -1;
            unsigned w = 0;
            for (int b = 0; b < 4; b++) w |= (unsigned)msg[kMagic + b] << (8 * b);
            if ((int)w != world) return -1; /* another job on this port */
            memcpy(id, msg + kMagic + 4, LIFE_UID_BYTES);
            return 0;
        }
        close(fd);
        clock_gettime(CLOCK_MONOTONIC, &t);
        if ((double)(t.tv_sec - t0.tv_sec) + 1e-9 * (double)(t.tv_nsec - t0.tv_nsec) > timeout_s) return -1;
        usleep(20000);
    }
}
