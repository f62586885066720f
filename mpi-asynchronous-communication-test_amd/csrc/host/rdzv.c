/*
 * rdzv.c -- RCCL unique-id hand-over between the GPU processes of one node,
 * through a file (no MPI, no torch): rank 0 writes it atomically, the others
 * poll.  Key: XG_RDZV_KEY, else MASTER_PORT + TORCHELASTIC_RUN_ID (torchrun),
 * else the parent pid (mpiexec / any launcher that forks all ranks).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "rdzv.h"
#include "xg.h"

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* RCCL unique-id hand-over through a file (single node). */
int xg_rendezvous(int rank, int nranks, unsigned char uid[XG_UNIQUE_ID_BYTES], char *path, size_t pathlen)
{
    const char *dir = getenv("XG_RDZV_DIR");
    const char *key = getenv("XG_RDZV_KEY");
    char kbuf[128];
    double t_start = now_s();
    if (!dir) dir = "/tmp";
    if (!key) {
        const char *port = getenv("MASTER_PORT"), *run = getenv("TORCHELASTIC_RUN_ID");
        /* the launcher (torchrun agent / mpiexec proxy) is every local rank's parent:
         * its pid keeps a stale file of an earlier launch on the same port from matching */
        if (port) snprintf(kbuf, sizeof kbuf, "p%s_%s_pp%ld", port, run ? run : "", (long)getppid());
        else snprintf(kbuf, sizeof kbuf, "pp%ld", (long)getppid());
        key = kbuf;
    }
    snprintf(path, pathlen, "%s/xg_rdzv_%s.bin", dir, key);
    if (rank == 0) {
        char tmp[4200];
        FILE *f;
        if (xg_get_unique_id(uid)) return -1;
        snprintf(tmp, sizeof tmp, "%s.%ld", path, (long)getpid());
        f = fopen(tmp, "wb");
        if (!f || fwrite(uid, 1, XG_UNIQUE_ID_BYTES, f) != XG_UNIQUE_ID_BYTES) { perror(tmp); return -1; }
        fclose(f);
        if (rename(tmp, path)) { perror(path); return -1; }
        return 0;
    }
    for (;;) {
        struct stat st;
        if (stat(path, &st) == 0 && st.st_mtime >= (time_t)t_start - 30) {
            FILE *f = fopen(path, "rb");
            if (f) {
                size_t n = fread(uid, 1, XG_UNIQUE_ID_BYTES, f);
                fclose(f);
                if (n == XG_UNIQUE_ID_BYTES) return 0;
            }
        }
        if (now_s() - t_start > 120) {
            fprintf(stderr, "rank %d/%d: no RCCL id at %s after 120 s\n", rank, nranks, path);
            return -1;
        }
        { struct timespec ts = {0, 2000000}; nanosleep(&ts, NULL); }
    }
}

int xg_env_int(const char *a, const char *b, int dflt)
{
    const char *v = getenv(a);
    if (!v && b) v = getenv(b);
    return v ? atoi(v) : dflt;
}
