/*
 * pt2pt.c -- drop-in for the reference's pt2pt_test (mpi_sendrecv_test.c).
 *
 * Two GPU processes; each of `-k` measurements times `-i` transfers of `-d`
 * bytes from rank 1 to rank 0 (the reference's Issend/Irecv/Wait pair,
 * :38-46) as RCCL send/recv over xGMI, with a barrier between measurements
 * (:48).  Rank 0 writes every measurement to sendrecv_results.csv and prints
 * the same summary line (:56-67).
 * Launch: torchrun --no-python --nproc-per-node 2 bin/pt2pt_test -d N -k K -i I, or
 * XG_GPUS=2 bin/pt2pt_test -d N -k K -i I (the process starts both ranks itself).
 */
#include <getopt.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>

#include "rdzv.h"
#include "xg.h"

#define DIE(...) do { fprintf(stderr, __VA_ARGS__); fputc('\n', stderr); exit(1); } while (0)

int main(int argc, char **argv)
{
    int rank, procs, i, ntimes = 0, data_size = 0, runs = 0, m;
    unsigned char uid[XG_UNIQUE_ID_BYTES];
    char path[4096] = {0};
    xg_ctx *ctx;
    rank = xg_env_int("RANK", "PMI_RANK", 0);
    procs = xg_env_int("WORLD_SIZE", "PMI_SIZE", 1);
    /* no launcher: XG_GPUS=2 starts the two GPU processes (xg_spawn_ranks) */
    if ((i = xg_spawn_ranks(xg_env_int("XG_GPUS", NULL, 1), argv)) >= 0) return i;
    while ((i = getopt(argc, argv, "hk:d:i:")) != EOF) {   /* :82-96 */
        switch (i) {
        case 'd': data_size = atoi(optarg); break;
        case 'k': ntimes = atoi(optarg); break;
        case 'i': runs = atoi(optarg); break;
        default: return 0;
        }
    }
    /* :97-99 -- MPICH's MPI_STATUS_IGNORE / MPI_STATUSES_IGNORE are both (void*)1 */
    printf("status = %lld, statuses = %lld\n", 1LL, 1LL);
    /* XG_PT2PT_SELF=1 (test hook, one process): rank 1's sends become self sends of rank 0 on a
     * 1-rank RCCL communicator, so the timing loop and report run on a one-GPU box */
    const int self = procs == 1 && getenv("XG_PT2PT_SELF") && atoi(getenv("XG_PT2PT_SELF"));
    if (procs != 2 && !self) return 0;                       /* pt2pt_statistics returns 1 (:25-27) */
    if (self) setenv("XG_SELF_COMM", "1", 1);
    else if (xg_rendezvous(rank, procs, uid, path, sizeof path)) DIE("rendezvous failed");
    if (xg_init(&ctx, rank, procs, xg_env_int("LOCAL_RANK", "MPI_LOCALRANKID", rank), self ? NULL : uid))
        DIE("xg_init failed");
    if (xg_barrier(ctx)) DIE("barrier failed");
    if (rank == 0 && path[0]) unlink(path);
    {
        double *tl = (double *)calloc(ntimes > 0 ? ntimes : 1, sizeof(double));
        double t0 = xg_now(), mean = 0, var = 0, total;
        for (m = 0; m < ntimes; ++m) {
            double gbps = 0, sec = 0;
            if (runs > 0 && data_size > 0 && xg_p2p_bench(ctx, data_size, 2, runs, &gbps, &sec)) DIE("p2p failed");
            tl[m] = sec * runs;
            if (xg_barrier(ctx)) DIE("barrier failed");
        }
        total = xg_now() - t0;
        if (rank == 0) {
            FILE *f = fopen("sendrecv_results.csv", "w");
            for (m = 0; m < ntimes; ++m) {
                if (f) fprintf(f, "%lf\n", tl[m]);
                mean += tl[m];
                var += tl[m] * tl[m];
            }
            if (f) fclose(f);
            mean = mean / m;
            printf("rank %d, mean = %lf, std = %lf, ntimes = %d, total_timing = %lf, mean*ntimes = %lf\n", rank, mean,
                   sqrt(var / m - mean * mean), ntimes, total, mean * m);
        }
        free(tl);
    }
    xg_finalize(ctx);
    return 0;
}
