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
 * MASTER_ADDR says otherwise; a host name such as torchrun's --standalone
 * MASTER_ADDR or "localhost" is resolved with getaddrinfo).  Every wait is
 * bounded by the caller's timeout: a rank that never connects, or a rank 0
 * that never answers, ends the bootstrap with an error instead of a hang.
 */
#include "bootstrap.h"

#include <arpa/inet.h>
#include <errno.h>
#include <netdb.h>
#include <netinet/in.h>
#include <poll.h>
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

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

/* IPv4 address of `host` (dotted quad or a name), port in network order. */
static int resolve(const char *host, int port, struct sockaddr_in *sa) {
    struct addrinfo hints, *res = NULL;
    memset(&hints, 0, sizeof hints);
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(host, NULL, &hints, &res) != 0 || !res) return -1;
    memcpy(sa, res->ai_addr, sizeof *sa);
    freeaddrinfo(res);
    sa->sin_port = htons((uint16_t)port);
    return 0;
}

/* Blocking send/recv of n bytes; the socket's SO_SNDTIMEO/SO_RCVTIMEO bound
 * each call. */
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

static void io_timeout(int fd, double seconds) {
    struct timeval tv;
    if (seconds < 0.001) seconds = 0.001;
    tv.tv_sec = (time_t)seconds;
    tv.tv_usec = (suseconds_t)((seconds - (double)tv.tv_sec) * 1e6);
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
    setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
}

/* Message: "LIFEUID1" + rank-0 world size (4 bytes, little endian) + id. */
enum { kMagic = 8, kMsg = 8 + 4 + LIFE_UID_BYTES };

int life_bootstrap_id(int rank, int world, uint8_t id[LIFE_UID_BYTES], double timeout_s) {
    if (world <= 1) return 0;
    struct sockaddr_in sa;
    memset(&sa, 0, sizeof sa);
    if (resolve(bootstrap_addr(), bootstrap_port(), &sa) != 0) return -1;
    const double deadline = now_s() + timeout_s;
    uint8_t msg[kMsg];
    if (rank == 0) {
        const int ls = socket(AF_INET, SOCK_STREAM, 0);
        if (ls < 0) return -1;
        const int one = 1;
        setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
        /* listen on every interface: the address the other ranks resolve
         * (MASTER_ADDR may name this host by any of its names) reaches it */
        struct sockaddr_in any = sa;
        any.sin_addr.s_addr = htonl(INADDR_ANY);
        if (bind(ls, (struct sockaddr *)&any, sizeof any) != 0 || listen(ls, world) != 0) {
            close(ls);
            return -1;
        }
        memcpy(msg, "LIFEUID1", kMagic);
        for (int b = 0; b < 4; b++) msg[kMagic + b] = (uint8_t)((unsigned)world >> (8 * b));
        memcpy(msg + kMagic + 4, id, LIFE_UID_BYTES);
        int rc = 0;
        for (int k = 1; k < world && rc == 0; k++) {
            /* a rank that died before connecting must not hang rank 0 */
            struct pollfd pf = {ls, POLLIN, 0};
            const double left = deadline - now_s();
            const int pr = left > 0 ? poll(&pf, 1, (int)(left * 1000.0) + 1) : 0;
            if (pr < 0 && errno == EINTR) {
                k--;
                continue;
            }
            if (pr <= 0) {
                rc = -1;
                break;
            }
            const int fd = accept(ls, NULL, NULL);
            if (fd < 0) {
                if (errno == EINTR) {
                    k--;
                    continue;
                }
                rc = -1;
                break;
            }
            io_timeout(fd, deadline - now_s());
            rc = full_io(fd, msg, sizeof msg, 1);
            close(fd);
        }
        close(ls);
        return rc;
    }
    for (;;) { /* rank 0 may not be listening yet */
        const int fd = socket(AF_INET, SOCK_STREAM, 0);
        if (fd < 0) return -1;
        if (connect(fd, (struct sockaddr *)&sa, sizeof sa) == 0) {
            io_timeout(fd, deadline - now_s());
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
        if (now_s() > deadline) return -1;
        usleep(20000);
    }
}
