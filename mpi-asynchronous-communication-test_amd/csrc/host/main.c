/*
 * main.c -- drop-in for the reference's ./test (mpi_test.c:2120-2347).
 *
 * Same getopt surface "hp:c:m:d:a:i:k:t:r:b:" (:2130), same defaults (:2121),
 * same header (:2171-2177), same per-method report and results.csv
 * (summarize_results, :2068-2118), same experiment loop (:2181-2343).
 *
 * Differences, by design:
 *  - One process per GPU; P logical ranks are block-mapped onto the GPUs.
 *    P defaults to the number of processes (as `mpiexec -n P`); host more
 *    logical ranks per GPU with --procs N or XG_PROCS=N.
 *  - Launch: single process, or any launcher that sets RANK/WORLD_SIZE
 *    (torchrun --no-python) or PMI_RANK/PMI_SIZE (mpiexec), or on its own
 *    with --gpus N (XG_GPUS=N): the process then starts the N GPU processes
 *    itself (xg_spawn_ranks) and exits with their highest exit code.  The RCCL
 *    unique id is handed over through a file in $XG_RDZV_DIR (default /tmp).
 *  - -m 0 runs methods 1..20 like the reference, TAM (15/16) included.
 *  - Extra, opt-in: --verify (or XG_VERIFY=1) checks every received byte on
 *    the GPU and prints one extra "| <label> verify ..." line per method;
 *    --fingerprint strong switches to the collision-free fingerprint.
 */
#include <errno.h>
#include <getopt.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "rdzv.h"
#include "xg.h"
#include "xg_sched.h"

static void usage(const char *argv0)   /* mpi_test.c:41-69 */
{
    const char *help =
        "Usage: %s [OPTION]... [FILE]...\n"
        "       [-h] Print help\n"
        "       [-a] number of aggregators (in the context of ROMIO)\n"
        "       [-p] number of processes per node (does not really matter)\n"
        "       [-d] data size\n"
        "       [-c] maximum communication size\n"
        "       [-i] number of experiments (MPI barrier between experiments)\n"
        "       [-k] number of iteration (run methods many times, there is no sync between individual runs)\n"
        "       [-m] method\n"
        "           0: All experiments\n"
        "           1: All to many without ordering (all-to-many)\n"
        "           2: Many to all without ordering (many-to-all)\n"
        "           3: All to many with ordering (all-to-many)\n"
        "           4: Many to all with ordering (many-to-all)\n"
        "           5: Many to all with alltoallw (many-to-all)\n"
        "           6: All to many sync (all-to-many sync)\n"
        "           7: All to many half sync (all-to-many half sync)\n"
        "           8: All to many with alltoallw (all-to-many benchmark)\n"
        "           9: All to many pairwise (all-to-many pairwise)\n"
        "           10: Many to all pairwise (many-to-all pairwise)\n"
        "           11: Many to all half sync (many-to-all half sync)\n"
        "           12: Many to all half sync2 (many-to-all half sync2)\n";
    fprintf(stderr, help, argv0);
}


#define DIE(...) do { fprintf(stderr, __VA_ARGS__); fputc('\n', stderr); exit(1); } while (0)
#define XGCALL(x) do { int rc_ = (x); if (rc_) DIE("xg call failed (%d): %s", rc_, #x); } while (0)

typedef struct {
    int P, A, d, c, ntimes, type, proc_node, barrier_type;
    int verify, fp_mode, pack_form;
    int64_t eager, pack_max, pack_min;
    int *rank_list;
    const char *prefix;
} opts_t;

static void run_method(xg_ctx *ctx, const opts_t *o, int method, int iter)
{
    const int g = xg_rank(ctx), G = xg_nranks(ctx);
    const char *label = xg_method_label(method);
    char err[512];
    int lo, hi, r, rc;
    int64_t bad = 0;
    xg_timer *timers, *reps = NULL, t0 = {0, 0, 0, 0, 0}, tmax = {0, 0, 0, 0, 0};
    xg_run_opts ro;
    double red[5], t_wall;

    xg_block_range(o->P, G, g, &lo, &hi);
    timers = (xg_timer *)calloc(hi - lo + 1, sizeof(xg_timer));
    xg_run_opts_default(&ro);
    ro.verify = o->verify; ro.fingerprint = o->fp_mode; ro.eager_limit = o->eager; ro.pack_max_seg = o->pack_max;
    ro.pack_min_bytes = o->pack_min;
    ro.pack_form = o->pack_form;
    ro.proc_node = o->proc_node; ro.barrier_type = o->barrier_type;
    if ((method == 15 || method == 16) && g == 0)   /* static_node_assignment, lustre_driver_test.c:361-363 */
        printf("static node assignment for %d node ( %d processes per node) of type %d\n", o->P, o->proc_node, 0);
    if (method == 13 && o->ntimes > 0)
        ro.rep_timers = reps = (xg_timer *)calloc((size_t)(hi - lo + 1) * o->ntimes, sizeof(xg_timer));
    t_wall = xg_now();
    rc = xg_run_method(ctx, method, o->P, o->A, o->d, o->rank_list, o->c, timers, iter, o->ntimes, &ro, &bad,
                       err, sizeof err);
    t_wall = xg_now() - t_wall;
    if (rc == XG_ESCHED) {          /* every process computes the same schedule */
        if (g == 0) fprintf(stderr, "| %s: %s\n", label, err);
        free(timers);
        free(reps);
        return;
    }
    if (rc) DIE("%s failed: %s", label, err);
    /* MPI_Reduce(&timer1, &max_timer1, 5, MPI_DOUBLE, MPI_MAX, 0, ...)  (:2184) */
    for (r = lo; r < hi; ++r) {
        const xg_timer *t = &timers[r - lo];
        if (r == 0) t0 = *t;
        if (t->post_request_time > tmax.post_request_time) tmax.post_request_time = t->post_request_time;
        if (t->send_wait_all_time > tmax.send_wait_all_time) tmax.send_wait_all_time = t->send_wait_all_time;
        if (t->recv_wait_all_time > tmax.recv_wait_all_time) tmax.recv_wait_all_time = t->recv_wait_all_time;
        if (t->total_time > tmax.total_time) tmax.total_time = t->total_time;
    }
    red[0] = tmax.post_request_time; red[1] = tmax.send_wait_all_time; red[2] = tmax.recv_wait_all_time;
    red[3] = (double)bad; red[4] = tmax.total_time;
    XGCALL(xg_allreduce_max(ctx, red, 5));
    tmax.post_request_time = red[0]; tmax.send_wait_all_time = red[1]; tmax.recv_wait_all_time = red[2];
    tmax.barrier_time = 0; tmax.total_time = red[4];
    if (reps) {   /* save_all_timing (:2279): gather every rank's timers[m] to rank 0, write the CSVs */
        size_t n = (size_t)o->P * o->ntimes * 5;
        double *all = (double *)calloc(n, sizeof(double));
        memcpy(all + (size_t)lo * o->ntimes * 5, reps, sizeof(xg_timer) * (size_t)(hi - lo) * o->ntimes);
        XGCALL(xg_allreduce_max(ctx, all, (int)n));       /* timers are >= 0: MAX = gather */
        if (g == 0) xg_save_all_timing(o->P, o->ntimes, o->c, (const xg_timer *)all, o->prefix);
        free(all);
        free(reps);
    }
    if (g == 0) {
        xg_summarize_results(o->P, o->A, o->d, o->c, o->ntimes, o->type, "results.csv", label, t0, tmax);
        if (o->verify) {
            const double bytes = (double)o->P * o->A * o->d * o->ntimes;
            printf("| %s verify = %s (bad receive slots, max over gpus = %.0f), aggregate = %.3f GB/s\n", label,
                   red[3] == 0 ? "OK" : "FAILED", red[3], tmax.total_time > 0 ? bytes / tmax.total_time / 1e9 : 0.0);
        }
    }
    (void)t_wall;
    free(timers);
}

int main(int argc, char **argv)
{
    /* defaults of mpi_test.c:2121 */
    int cb_nodes = 1, method = 0, data_size = 0, proc_node = 1, i, comm_size = 200000000, iter = 1, ntimes = 1;
    int aggregator_type = 1, barrier_type = 0, procs = 0, verify = 0, fp_mode = XG_FP_REFERENCE;
    int pack_form = XG_PACK_FORM_DEFAULT;
    int64_t eager = XG_MPICH_EAGER_LIMIT, pack_max = 4 << 20, pack_min = 64 << 10;
    char prefix[200];
    int rank, nranks, device, ngpu_dev;
    unsigned char uid[XG_UNIQUE_ID_BYTES];
    char rdzv_path[4096] = {0};
    xg_ctx *ctx;
    opts_t o;
    static struct option longopts[] = {
        {"procs", required_argument, 0, 1000},
        {"verify", no_argument, 0, 1001},
        {"fingerprint", required_argument, 0, 1002},
        {"eager-limit", required_argument, 0, 1003},
        {"pack-max-seg", required_argument, 0, 1004},
        {"gpus", required_argument, 0, 1005},
        {"pack-min", required_argument, 0, 1006},
        {"pack-form", required_argument, 0, 1007},
        {0, 0, 0, 0}};
    int ngpus = xg_env_int("XG_GPUS", NULL, 1);
    prefix[0] = '\0';

    rank = xg_env_int("RANK", "PMI_RANK", 0);
    nranks = xg_env_int("WORLD_SIZE", "PMI_SIZE", 1);
    device = xg_env_int("LOCAL_RANK", "MPI_LOCALRANKID", rank);
    procs = xg_env_int("XG_PROCS", NULL, 0);
    verify = xg_env_int("XG_VERIFY", NULL, 0);
    /* --fingerprint, --eager-limit, --pack-max-seg, --pack-min and --pack-form are options
     * only (their XG_* environment twins were folded in round 5) */

    while ((i = getopt_long(argc, argv, "hp:c:m:d:a:i:k:t:r:b:", longopts, NULL)) != EOF) {
        switch (i) {
        case 'm': method = atoi(optarg); break;
        case 'a': cb_nodes = atoi(optarg); break;
        case 'd': data_size = atoi(optarg); break;
        case 'c': comm_size = atoi(optarg); break;
        case 'i': iter = atoi(optarg); break;
        case 'p': proc_node = atoi(optarg); break;
        case 'k': ntimes = atoi(optarg); break;
        case 't': aggregator_type = atoi(optarg); break;
        case 'r': strncpy(prefix, optarg, sizeof prefix - 1); prefix[sizeof prefix - 1] = 0; break;
        case 'b': barrier_type = atoi(optarg); break;
        case 1000: procs = atoi(optarg); break;
        case 1001: verify = 1; break;
        case 1002: fp_mode = !strcmp(optarg, "strong") ? XG_FP_STRONG : XG_FP_REFERENCE; break;
        case 1003: eager = atoll(optarg); break;
        case 1004: pack_max = atoll(optarg); break;
        case 1005: ngpus = atoi(optarg); break;
        case 1006: pack_min = atoll(optarg); break;
        case 1007: pack_form = atoi(optarg); break;
        default:
            if (rank == 0) usage(argv[0]);
            return 0;
        }
    }

    /* no launcher + --gpus N (XG_GPUS=N): start the N GPU processes ourselves */
    if ((i = xg_spawn_ranks(ngpus, argv)) >= 0) return i;
    if (getenv("XG_SPAWN_STUB")) {    /* test hook: report the rank environment and stop */
        printf("spawn-stub RANK=%s LOCAL_RANK=%s WORLD_SIZE=%s XG_RDZV_KEY=%s\n", getenv("RANK"),
               getenv("LOCAL_RANK"), getenv("WORLD_SIZE"), getenv("XG_RDZV_KEY"));
        return 0;
    }
    if (procs <= 0) procs = nranks;
    if (nranks > procs) DIE("more GPU processes (%d) than logical ranks (%d)", nranks, procs);
    if (cb_nodes < 1 || cb_nodes > procs) DIE("-a %d: need 1 <= aggregators <= ranks (%d)", cb_nodes, procs);
    if (data_size < 0) DIE("-d must be >= 0");

    if (nranks > 1 && xg_rendezvous(rank, nranks, uid, rdzv_path, sizeof rdzv_path)) DIE("rendezvous failed");
    ngpu_dev = device;
    XGCALL(xg_init(&ctx, rank, nranks, ngpu_dev, uid));
    XGCALL(xg_barrier(ctx));
    if (nranks > 1) {
        /* every process plans every GPU's RCCL calls from its own command line: processes
         * started with different ones would post calls nobody pairs and hang -- compare a
         * digest (FNV-1a of argv and the planning settings, in 16-bit parts) first */
        static const char *keys[] = {"XG_PROCS", "XG_VERIFY", "XG_SELF_MAX", NULL};
        uint64_t h = 0xcbf29ce484222325ull;
        double red[8];
        int k;
        for (k = 1; k <= argc; ++k) {
            const char *str = k < argc ? argv[k] : "";
            size_t j, n = strlen(str) + 1;
            for (j = 0; j < n; ++j) h = (h ^ (unsigned char)str[j]) * 0x100000001b3ull;
        }
        for (k = 0; keys[k]; ++k) {
            const char *v = getenv(keys[k]);
            size_t j, n = v ? strlen(v) + 1 : 0;
            for (j = 0; j < n; ++j) h = (h ^ (unsigned char)v[j]) * 0x100000001b3ull;
            h = (h ^ (unsigned char)(k + 1)) * 0x100000001b3ull;
        }
        for (k = 0; k < 4; ++k) {
            red[k] = (double)((h >> (16 * k)) & 0xffff);
            red[4 + k] = -red[k];
        }
        XGCALL(xg_allreduce_max(ctx, red, 8));
        for (k = 0; k < 4; ++k)
            if (red[k] != -red[4 + k]) DIE("the GPU processes were started with different arguments or settings");
    }
    if (rank == 0 && rdzv_path[0]) unlink(rdzv_path);

    o.P = procs; o.A = cb_nodes; o.d = data_size; o.c = comm_size; o.ntimes = ntimes; o.type = aggregator_type;
    o.proc_node = proc_node; o.verify = verify; o.fp_mode = fp_mode; o.eager = eager; o.pack_max = pack_max; o.pack_min = pack_min;
    o.pack_form = pack_form;
    o.barrier_type = barrier_type; o.prefix = prefix;
    o.rank_list = (int *)malloc(sizeof(int) * cb_nodes);
    if (xg_aggregator_list(procs, cb_nodes, proc_node, aggregator_type, o.rank_list))
        DIE("-t %d: aggregator type not defined by the reference", aggregator_type);

    if (rank == 0) {   /* :2170-2179 */
        printf("total number of processes = %d, cb_nodes = %d, proc_node = %d, data size = %d, comm_size = %d, "
               "ntimes=%d\n", procs, cb_nodes, proc_node, data_size, comm_size, ntimes);
        printf("aggregators = ");
        for (i = 0; i < cb_nodes; ++i) printf("%d, ", o.rank_list[i]);
        printf("\n");
    }
    for (i = 0; i < iter; ++i) {   /* :2181-2343 */
        int m;
        for (m = 1; m <= 20; ++m)
            if ((method == 0 || method == m) && xg_method_direction(m) >= 0) run_method(ctx, &o, m, i);
        if (rank == 0) {
            printf("| --------------------------------------\n");
            fflush(stdout);
        }
    }
    free(o.rank_list);
    XGCALL(xg_finalize(ctx));
    return 0;
}
