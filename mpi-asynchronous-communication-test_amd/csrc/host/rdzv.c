/*
 * rdzv.c -- RCCL unique-id hand-over between the GPU processes of one node,
 * through a file (no MPI, no torch): rank 0 writes it atomically, the others
 * poll.  Key: XG_RDZV_KEY, else MASTER_PORT + TORCHELASTIC_RUN_ID (torchrun),
 * else the parent pid (mpiexec / any launcher that forks all ranks).
 */
#include <signal.h>
#include <spawn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

extern char **environ;

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

/* environment of child r: this process's, with the rank variables replaced (the last
 * CHILD_VARS entries are its own: free_child_env releases them) */
#define CHILD_VARS 5

/* the spawner has nothing to fall back on without host memory: say so and stop */
static void *xzalloc(size_t n, size_t size)
{
    void *p = calloc(n ? n : 1, size);
    if (!p) { fprintf(stderr, "xg_spawn_ranks: out of host memory\n"); exit(1); }
    return p;
}

static char **child_env(int r, int n, const char *key)
{
    size_t m = 0, i, k = 0;
    char **env;
    static const char *drop[] = {"RANK=", "LOCAL_RANK=", "WORLD_SIZE=", "LOCAL_WORLD_SIZE=", "XG_RDZV_KEY=", NULL};
    while (environ[m]) m++;
    env = (char **)xzalloc(m + 6, sizeof(char *));
    for (i = 0; i < m; ++i) {
        int j, skip = 0;
        for (j = 0; drop[j]; ++j)
            if (!strncmp(environ[i], drop[j], strlen(drop[j]))) skip = 1;
        if (!skip) env[k++] = environ[i];
    }
    env[k] = (char *)xzalloc(32, 1); snprintf(env[k++], 32, "RANK=%d", r);
    env[k] = (char *)xzalloc(32, 1); snprintf(env[k++], 32, "LOCAL_RANK=%d", r);
    env[k] = (char *)xzalloc(32, 1); snprintf(env[k++], 32, "WORLD_SIZE=%d", n);
    env[k] = (char *)xzalloc(32, 1); snprintf(env[k++], 32, "LOCAL_WORLD_SIZE=%d", n);
    env[k] = (char *)xzalloc(160, 1); snprintf(env[k++], 160, "XG_RDZV_KEY=%s", key);
    env[k] = NULL;
    return env;
}

static void free_child_env(char **env)
{
    size_t k = 0, i;
    while (env[k]) k++;
    for (i = k - CHILD_VARS; i < k; ++i) free(env[i]);
    free(env);
}

int xg_spawn_ranks(int ngpus, char **argv)
{
    pid_t *pid;
    int *st, r, left, worst = 0, failed = 0;
    char key[128];
    double t_fail = 0;
    if (ngpus <= 1 || getenv("RANK") || getenv("WORLD_SIZE") || getenv("PMI_RANK") || getenv("PMI_SIZE")) return -1;
    snprintf(key, sizeof key, "spawn%ld_%ld", (long)getpid(), (long)time(NULL));
    /* every rank on one device (XG_SHARE_GPU=1, runtime/ctx.hip): 1 hardware queue per process
     * whatever the environment says (the one-GPU boxes export HIP's default 4), or the command
     * processor time-slices the ranks' queues (profiles/r05/share_gpu_queues/) */
    if (getenv("XG_SHARE_GPU") && !strcmp(getenv("XG_SHARE_GPU"), "1")) setenv("GPU_MAX_HW_QUEUES", "1", 1);
    pid = (pid_t *)xzalloc(ngpus, sizeof(pid_t));
    st = (int *)xzalloc(ngpus, sizeof(int));
    for (r = 0; r < ngpus; ++r) {
        char **env = child_env(r, ngpus, key);
        if (posix_spawn(&pid[r], "/proc/self/exe", NULL, NULL, argv, env)) {
            perror("posix_spawn");
            pid[r] = 0;
            failed = 1;
            worst = 1;
        }
        free_child_env(env);
    }
    for (left = 0, r = 0; r < ngpus; ++r) left += pid[r] > 0;
    while (left > 0) {
        int status;
        pid_t w = waitpid(-1, &status, WNOHANG);
        if (w > 0) {
            for (r = 0; r < ngpus; ++r)
                if (pid[r] == w) {
                    int code = WIFEXITED(status) ? WEXITSTATUS(status) : 128 + WTERMSIG(status);
                    st[r] = code;
                    pid[r] = -1;
                    left--;
                    if (code > worst) worst = code;
                    if (code && !failed) {
                        fprintf(stderr, "rank %d failed (exit %d): stopping the job\n", r, code);
                        failed = 1;
                        t_fail = now_s();
                    }
                }
            continue;
        }
        if (failed && now_s() - t_fail > 10)      /* the survivors would wait for a dead peer */
            for (r = 0; r < ngpus; ++r)
                if (pid[r] > 0) kill(pid[r], now_s() - t_fail > 20 ? SIGKILL : SIGTERM);
        { struct timespec ts = {0, 50000000}; nanosleep(&ts, NULL); }
    }
    free(pid);
    free(st);
    return worst;
}
