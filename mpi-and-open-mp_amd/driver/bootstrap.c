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
 * MASTER_ADDR or "localhost" is resolved with getaddrinfo).  Rank 0 listens
 * on that address only, and answers a connection only after it presented the
 * job's token.  Every wait is bounded by the caller's timeout, connect()
 * included: a rank that never connects, or a rank 0 that never answers or
 * cannot be reached, ends the bootstrap with an error instead of a hang.
 */
#include "bootstrap.h"

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
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

/* 8-byte job token every rank of one job derives alike: FNV-1a over
 * LIFE_BOOTSTRAP_TOKEN (if set) or the launchers' job ids, the world size and
 * the port.  A rank must present it before rank 0 answers with the id, so a
 * stray connection (another job on the port, a scanner) neither receives the
 * id nor takes a real rank's slot. */
static uint64_t job_token(int world, int port) {
    static const char *const vars[] = {"LIFE_BOOTSTRAP_TOKEN", "TORCHELASTIC_RUN_ID", "PMI_KVSNAME",
                                       "PMIX_NAMESPACE", "OMPI_MCA_ess_base_jobid", "SLURM_JOB_ID"};
    uint64_t h = 1469598103934665603ull;
    char buf[64];
    snprintf(buf, sizeof buf, "life:%d:%d:", world, port);
    for (const char *c = buf; *c; c++) h = (h ^ (uint8_t)*c) * 1099511628211ull;
    for (size_t k = 0; k < sizeof vars / sizeof vars[0]; k++) {
        const char *v = getenv(vars[k]);
        if (!v) continue;
        for (const char *c = v; *c; c++) h = (h ^ (uint8_t)*c) * 1099511628211ull;
        h = (h ^ 0xFFu) * 1099511628211ull;
    }
    return h;
}

/* Hello (rank k -> 0): "LIFEHELO" + world (4 bytes LE) + token (8 bytes LE).
 * Answer (0 -> k): "LIFEUID1" + world (4 bytes LE) + id. */
enum { kMagic = 8, kHello = 8 + 4 + 8, kMsg = 8 + 4 + LIFE_UID_BYTES };

static void put_le(uint8_t *p, uint64_t v, int n) {
    for (int b = 0; b < n; b++) p[b] = (uint8_t)(v >> (8 * b));
}
static uint64_t get_le(const uint8_t *p, int n) {
    uint64_t v = 0;
    for (int b = 0; b < n; b++) v |= (uint64_t)p[b] << (8 * b);
    return v;
}

/* connect() bounded by the deadline (a blocking connect to an unreachable
 * host retries SYNs for minutes): non-blocking connect, poll for
 * writability, then SO_ERROR.  0 connected, -1 refused / failed (retry),
 * -2 deadline passed. */
static int connect_until(int fd, const struct sockaddr_in *sa, double deadline) {
    const int fl = fcntl(fd, F_GETFL, 0);
    if (fl < 0 || fcntl(fd, F_SETFL, fl | O_NONBLOCK) != 0) return -1;
    int rc = connect(fd, (const struct sockaddr *)sa, sizeof *sa);
    if (rc != 0 && errno == EINPROGRESS) {
        for (;;) {
            const double left = deadline - now_s();
            if (left <= 0) return -2;
            struct pollfd pf = {fd, POLLOUT, 0};
            const int pr = poll(&pf, 1, (int)(left * 1000.0) + 1);
            if (pr < 0 && errno == EINTR) continue;
            if (pr == 0) return -2;
            if (pr < 0) return -1;
            int err = 0;
            socklen_t len = sizeof err;
            if (getsockopt(fd, SOL_SOCKET, SO_ERROR, &err, &len) != 0 || err != 0) return -1;
            rc = 0;
            break;
        }
    }
    if (rc != 0) return -1;
    return fcntl(fd, F_SETFL, fl) == 0 ? 0 : -1;
}

int life_bootstrap_id(int rank, int world, uint8_t id[LIFE_UID_BYTES], double timeout_s) {
    if (world <= 1) return 0;
    struct sockaddr_in sa;
    memset(&sa, 0, sizeof sa);
    const int port = bootstrap_port();
    if (resolve(bootstrap_addr(), port, &sa) != 0) return -1;
    const uint64_t token = job_token(world, port);
    const double deadline = now_s() + timeout_s;
    uint8_t msg[kMsg], hello[kHello];
    if (rank == 0) {
        const int ls = socket(AF_INET, SOCK_STREAM, 0);
        if (ls < 0) return -1;
        const int one = 1;
        setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
        /* listen on the address the other ranks connect to (127.0.0.1 by
         * default: nothing off this host reaches it); every interface only
         * on request (LIFE_BOOTSTRAP_ANY=1, e.g. a NAT'd MASTER_ADDR that is
         * not an address of this host) */
        struct sockaddr_in at = sa;
        const char *any = getenv("LIFE_BOOTSTRAP_ANY");
        if (any && atoi(any) != 0) at.sin_addr.s_addr = htonl(INADDR_ANY);
        if (bind(ls, (struct sockaddr *)&at, sizeof at) != 0 || listen(ls, world) != 0) {
            fprintf(stderr, "life bootstrap: cannot listen on %s:%d (%s)%s\n", inet_ntoa(at.sin_addr), port,
                    strerror(errno),
                    errno == EADDRNOTAVAIL ? "; not an address of this host (LIFE_BOOTSTRAP_ANY=1 listens on all)"
                                           : "");
            close(ls);
            return -1;
        }
        memcpy(msg, "LIFEUID1", kMagic);
        put_le(msg + kMagic, (uint64_t)(unsigned)world, 4);
        memcpy(msg + kMagic + 4, id, LIFE_UID_BYTES);
        int rc = 0, served = 0;
        while (served < world - 1) {
            /* a rank that died before connecting must not hang rank 0 */
            struct pollfd pf = {ls, POLLIN, 0};
            const double left = deadline - now_s();
            const int pr = left > 0 ? poll(&pf, 1, (int)(left * 1000.0) + 1) : 0;
            if (pr < 0 && errno == EINTR) continue;
            if (pr <= 0) {
                rc = -1;
                break;
            }
            const int fd = accept(ls, NULL, NULL);
            if (fd < 0) {
                if (errno == EINTR || errno == ECONNABORTED) continue;
                rc = -1;
                break;
            }
            /* a peer that connects and says nothing gets 2 s, not the job's
             * whole timeout */
            const double hs = deadline - now_s() < 2.0 ? deadline - now_s() : 2.0;
            io_timeout(fd, hs);
            const int ok = full_io(fd, hello, sizeof hello, 0) == 0 && memcmp(hello, "LIFEHELO", kMagic) == 0 &&
                           get_le(hello + kMagic, 4) == (uint64_t)(unsigned)world &&
                           get_le(hello + kMagic + 4, 8) == token;
            if (ok) {
                io_timeout(fd, deadline - now_s());
                if (full_io(fd, msg, sizeof msg, 1) == 0) served++;
            }
            close(fd); /* a stranger is dropped without the id and without a slot */
        }
        close(ls);
        return rc;
    }
    memcpy(hello, "LIFEHELO", kMagic);
    put_le(hello + kMagic, (uint64_t)(unsigned)world, 4);
    put_le(hello + kMagic + 4, token, 8);
    for (;;) { /* rank 0 may not be listening yet */
        const int fd = socket(AF_INET, SOCK_STREAM, 0);
        if (fd < 0) return -1;
        const int c = connect_until(fd, &sa, deadline);
        if (c == 0) {
            io_timeout(fd, deadline - now_s());
            int rc = full_io(fd, hello, sizeof hello, 1);
            if (rc == 0) rc = full_io(fd, msg, sizeof msg, 0);
            close(fd);
            if (rc != 0 || memcmp(msg, "LIFEUID1", kMagic) != 0) return -1;
            if (get_le(msg + kMagic, 4) != (uint64_t)(unsigned)world) return -1; /* another job on this port */
            memcpy(id, msg + kMagic + 4, LIFE_UID_BYTES);
            return 0;
        }
        close(fd);
        if (c == -2 || now_s() > deadline) return -1;
        usleep(20000);
    }
}
