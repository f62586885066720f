/*
 * report.c -- the reference's result report, byte-compatible.
 * summarize_results, mpi_test.c:2068-2118: eight "| <label> ..." lines and one
 * results.csv row (15-column header written when the file is created).
 */
#include "xg_sched.h"

#include <stdio.h>

int xg_summarize_results(int procs, int cb_nodes, int data_size, int comm_size, int ntimes,
                         int type, const char *filename, const char *prefix,
                         xg_timer t, xg_timer mx)
{
    FILE *f;
    printf("| --------------------------------------\n");
    printf("| %s rank 0 request post time = %lf\n", prefix, t.post_request_time);
    printf("| %s rank 0 send waitall time = %lf\n", prefix, t.send_wait_all_time);
    printf("| %s rank 0 recv waitall time = %lf\n", prefix, t.recv_wait_all_time);
    printf("| %s rank 0 total time = %lf\n", prefix, t.total_time);
    printf("| %s max request post time = %lf\n", prefix, mx.post_request_time);
    printf("| %s max send waitall time = %lf\n", prefix, mx.send_wait_all_time);
    printf("| %s max recv waitall time = %lf\n", prefix, mx.recv_wait_all_time);
    printf("| %s max total time = %lf\n", prefix, mx.total_time);
    f = fopen(filename, "r");
    if (f) {
        fclose(f);
        f = fopen(filename, "a");
    } else {
        f = fopen(filename, "w");
        if (f)
            fprintf(f, "Method,# of processes,# of aggregators,data size,max comm,ntimes,aggregator type,"
                       "rank 0 post_request_time,rank 0 send waitall time,rank 0 recv waitall time,"
                       "rank 0 total time,max post_request_time,max send waitall time,"
                       "max recv waitall time,max total time\n");
    }
    if (!f) return -1;
    fprintf(f, "%s,%d,%d,%d,%d,%d,%d,", prefix, procs, cb_nodes, data_size, comm_size, ntimes, type);
    fprintf(f, "%lf,%lf,%lf,%lf,", t.post_request_time, t.send_wait_all_time, t.recv_wait_all_time, t.total_time);
    fprintf(f, "%lf,%lf,%lf,%lf\n", mx.post_request_time, mx.send_wait_all_time, mx.recv_wait_all_time,
            mx.total_time);
    fclose(f);
    return 0;
}

/* save_all_timing, mpi_test.c:2008-2066 (rank 0 part, after the gather) */
int xg_save_all_timing(int procs, int ntimes, int comm_size, const xg_timer *timers, const char *prefix)
{
    static const char *names[4] = {"send_wait_all_times", "total_times", "post_request_time", "barrier_time"};
    static const int fields[4] = {1, 4, 0, 3};     /* xg_timer field index */
    char fn[512];
    int k, i, j;
    for (k = 0; k < 4; ++k) {
        FILE *f;
        snprintf(fn, sizeof fn, "%s%s_%d.csv", prefix ? prefix : "", names[k], comm_size);
        f = fopen(fn, "w");
        if (!f) return -1;
        for (i = 0; i < procs; ++i) {
            fprintf(f, "%d", i);
            for (j = 0; j < ntimes; ++j) fprintf(f, ",%lf", ((const double *)&timers[(size_t)i * ntimes + j])[fields[k]]);
            fprintf(f, "\n");
        }
        fclose(f);
    }
    return 0;
}
