/*
 * pieces.c -- how a copy launch is cut into workgroup pieces (host side of the copy kernel).
 *
 * One workgroup copies one piece.  A launch of w pieces puts ceil(w / CUs) of them on its
 * busiest CU, and the launch lasts about as long as that CU works: pieces x (piece bytes + a
 * fixed per-workgroup start).  xg_piece_size picks, among the launch's default piece size and
 * its halvings down to 4 KiB (a halving still divides power-of-two segment sizes, so no
 * segment gets a ragged tail piece), the one that least loads the busiest CU; ties keep the
 * larger piece.  Reference: the copies MPI does inside Irecv/Issend/Alltoallw for one step
 * (mpi_test.c:1776,1790, :627,912) -- here one launch per step and part.
 */
#include "xg_sched.h"

int64_t xg_piece_size(const int64_t *lens, int n, int64_t chunk, int cus, int64_t wg_cost)
{
    int64_t best_c = chunk, cand;
    double best = -1;
    int i;
    if (!lens || n <= 0 || chunk <= 0 || cus <= 0) return chunk;
    for (cand = chunk; cand >= 4096 && (cand & 15) == 0; cand /= 2) {
        int64_t w = 0;
        double cost;
        for (i = 0; i < n; ++i)
            if (lens[i] > 0) w += (lens[i] + cand - 1) / cand;
        if (!w) return chunk;
        cost = (double)((w + cus - 1) / cus) * (double)(cand + wg_cost);
        if (best < 0 || cost < best) {
            best = cost;
            best_c = cand;
        }
    }
    return best_c;
}
