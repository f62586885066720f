/*
 * pieces.c -- how copy launches are formed (host side of the copy kernel): how a launch is
 * cut into workgroup pieces, and whether a step's local copies may share a launch with the
 * previous step's unpacks.
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

#include <stdlib.h>

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

/* [off, end) of region buf */
typedef struct { int64_t lo, hi; } ival;

static int ival_cmp(const void *x, const void *y)
{
    const ival *a = (const ival *)x, *b = (const ival *)y;
    return a->lo < b->lo ? -1 : a->lo > b->lo;
}

/* Step s's local copies (after its stage copies, before its packs) against the bytes step
 * s-1's unpacks write: 1 if any of them reads or writes such a byte -- then they cannot share
 * one launch, whose workgroups run in any order (xg_runtime.hip fuses them otherwise).
 * Returns -1 for a bad step. */
int xg_step_local_meets_unpacks(const xg_devplan *dp, int s)
{
    const xg_stepplan *pv, *sp;
    ival *w[XG_NBUF] = {0};
    int64_t *reach[XG_NBUF] = {0};
    int nw[XG_NBUF] = {0}, i, k, hit = 0;
    if (!dp || s < 1 || s >= dp->nsteps) return -1;
    pv = &dp->steps[s - 1];
    sp = &dp->steps[s];
    for (k = 0; k < XG_NBUF; ++k) {
        w[k] = (ival *)malloc(sizeof(ival) * ((size_t)pv->post_count + 1));
        reach[k] = (int64_t *)malloc(sizeof(int64_t) * ((size_t)pv->post_count + 1));
        if (!w[k] || !reach[k]) { hit = 1; goto done; }   /* refuse the fusion when in doubt */
    }
    for (i = 0; i < pv->post_count; ++i) {
        const xg_copy *c = &dp->copies[pv->post_begin + i];
        if (c->len > 0 && c->dst_buf >= 0 && c->dst_buf < XG_NBUF) {
            w[c->dst_buf][nw[c->dst_buf]].lo = c->dst_off;
            w[c->dst_buf][nw[c->dst_buf]++].hi = c->dst_off + c->len;
        }
    }
    for (k = 0; k < XG_NBUF; ++k) {
        int64_t m = INT64_MIN;
        qsort(w[k], nw[k], sizeof(ival), ival_cmp);
        for (i = 0; i < nw[k]; ++i) reach[k][i] = m = w[k][i].hi > m ? w[k][i].hi : m;
    }
    for (i = sp->stage_count; i < sp->pre_count && !hit; ++i) {
        const xg_copy *c = &dp->copies[sp->pre_begin + i];
        int side;
        if (c->dst_buf == XG_BUF_STAGE_SEND) break;          /* the packs start */
        if (c->len <= 0) continue;
        for (side = 0; side < 2 && !hit; ++side) {
            const int buf = side ? c->dst_buf : c->src_buf;
            const int64_t a = side ? c->dst_off : c->src_off, b = a + c->len;
            int lo = 0, hi = nw[buf];                        /* intervals starting before b: [0, lo) */
            if (buf < 0 || buf >= XG_NBUF) continue;
            while (lo < hi) {
                const int mid = (lo + hi) / 2;
                if (w[buf][mid].lo < b) lo = mid + 1;
                else hi = mid;
            }
            hit = lo > 0 && reach[buf][lo - 1] > a;
        }
    }
done:
    for (k = 0; k < XG_NBUF; ++k) { free(w[k]); free(reach[k]); }
    return hit;
}
