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
 * one launch, whose workgroups run in any order (runtime/plan_load.hip fuses them otherwise).
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
            int lo = 0, hi;
            if (buf < 0 || buf >= XG_NBUF) continue;
            hi = nw[buf];                                    /* intervals starting before b: [0, lo) */
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

/* sorted intervals of one kind (reads or writes) of a set of copies, per region, with running
 * maxima of their ends: "does [a, b) of region buf meet any of them" in O(log n) */
typedef struct {
    ival *v[XG_NBUF];
    int64_t *reach[XG_NBUF];
    int n[XG_NBUF];
} ivset;

static int ivset_build(ivset *t, const xg_copy *c, int n, int dst_side)
{
    int i, k;
    for (k = 0; k < XG_NBUF; ++k) {
        t->n[k] = 0;
        t->v[k] = (ival *)malloc(sizeof(ival) * ((size_t)n + 1));
        t->reach[k] = (int64_t *)malloc(sizeof(int64_t) * ((size_t)n + 1));
        if (!t->v[k] || !t->reach[k]) return -1;
    }
    for (i = 0; i < n; ++i) {
        const int buf = dst_side ? c[i].dst_buf : c[i].src_buf;
        const int64_t off = dst_side ? c[i].dst_off : c[i].src_off;
        if (c[i].len <= 0 || buf < 0 || buf >= XG_NBUF) continue;
        t->v[buf][t->n[buf]].lo = off;
        t->v[buf][t->n[buf]++].hi = off + c[i].len;
    }
    for (k = 0; k < XG_NBUF; ++k) {
        int64_t m = INT64_MIN;
        qsort(t->v[k], t->n[k], sizeof(ival), ival_cmp);
        for (i = 0; i < t->n[k]; ++i) t->reach[k][i] = m = t->v[k][i].hi > m ? t->v[k][i].hi : m;
    }
    return 0;
}

static int ivset_meets(const ivset *t, int buf, int64_t a, int64_t b)
{
    int lo = 0, hi;
    if (buf < 0 || buf >= XG_NBUF) return 0;
    hi = t->n[buf];
    while (lo < hi) {                                  /* intervals starting before b: [0, lo) */
        const int mid = (lo + hi) / 2;
        if (t->v[buf][mid].lo < b) lo = mid + 1;
        else hi = mid;
    }
    return lo > 0 && t->reach[buf][lo - 1] > a;
}

static void ivset_free(ivset *t)
{
    int k;
    for (k = 0; k < XG_NBUF; ++k) { free(t->v[k]); free(t->reach[k]); }
}

/* Step s's stage copies (TAM rank-local memcpy's through SCRATCH) against its other pre copies
 * (local gather/scatter, packs): 1 if one of those reads or writes a byte a stage copy writes,
 * or writes a byte a stage copy reads -- then the stage copies need a launch of their own ahead
 * of the others (xg_devplan_build puts them first for that reason); 0 if all may share one
 * launch, whose workgroups run in any order; -1 for a bad step.  At the README configuration
 * m15 / m16's step 3 (14 stage copies into the aggregation buffers beside 434 local copies into
 * the receive slots) shares one launch. */
int xg_step_stage_meets_rest(const xg_devplan *dp, int s)
{
    const xg_stepplan *sp;
    ivset w = {{0}, {0}, {0}}, r = {{0}, {0}, {0}};
    int i, hit = 0;
    if (!dp || s < 0 || s >= dp->nsteps) return -1;
    sp = &dp->steps[s];
    if (sp->stage_count <= 0) return 0;
    if (ivset_build(&w, dp->copies + sp->pre_begin, sp->stage_count, 1) ||
        ivset_build(&r, dp->copies + sp->pre_begin, sp->stage_count, 0)) {
        hit = 1;                                       /* refuse the fusion when in doubt */
        goto done;
    }
    for (i = sp->stage_count; i < sp->pre_count && !hit; ++i) {
        const xg_copy *c = &dp->copies[sp->pre_begin + i];
        if (c->len <= 0) continue;
        hit = ivset_meets(&w, c->src_buf, c->src_off, c->src_off + c->len) ||
              ivset_meets(&w, c->dst_buf, c->dst_off, c->dst_off + c->len) ||
              ivset_meets(&r, c->dst_buf, c->dst_off, c->dst_off + c->len);
    }
done:
    ivset_free(&w);
    ivset_free(&r);
    return hit;
}
