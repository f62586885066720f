/*
 * hazard.c -- what the step engine's barrier after each step must order
 * (kernels.h step_engine_kernel, include/xg_sched.h xg_engine_hazards).
 *
 * Every engine step reads SEND (or earlier RECV bytes) and writes RECV.  The
 * engine lets a workgroup arrive at a barrier as soon as its stores are issued
 * and loads the next step's first unit while the barrier is pending; that is
 * only valid while the next step
 *   - reads no byte written since the last ordering point (read-after-write),
 *   - rewrites such bytes only with the SAME bytes: the same source bytes at
 *     the same source-destination offset (the -k repetitions of a method move
 *     the identical segments into the identical slots), and the sources are
 *     untouched since (a write into a source range is itself a read-after-write
 *     for the step that reads it).
 * Anything else is a hazard point: flag 2 (drain + release/acquire, no early
 * load).  The last step gets at least flag 1 (drained: its stamp anchors every
 * step time).  Pending writes are kept as disjoint intervals sorted by start,
 * each with its destination-minus-source delta.
 */
#include <stdlib.h>
#include <string.h>

#include "xg_sched.h"

typedef struct {
    uint64_t lo, hi;      /* destination byte range [lo, hi) */
    int64_t delta;        /* dst - src of the bytes written there */
} ivl;

static int cmp_ivl(const void *a, const void *b)
{
    const ivl *x = (const ivl *)a, *y = (const ivl *)b;
    if (x->lo != y->lo) return x->lo < y->lo ? -1 : 1;
    if (x->delta != y->delta) return x->delta < y->delta ? -1 : 1;
    return 0;
}

/* first interval with hi > a (his are increasing in a disjoint sorted list) */
static int first_after(const ivl *v, int n, uint64_t a)
{
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (v[mid].hi > a) hi = mid; else lo = mid + 1;
    }
    return lo;
}

/* 1 if [a, b) meets a pending write; with want_delta, 1 only if one it meets has another delta */
static int meets(const ivl *v, int n, uint64_t a, uint64_t b, int want, int64_t delta)
{
    int i;
    for (i = first_after(v, n, a); i < n && v[i].lo < b; ++i)
        if (!want || v[i].delta != delta) return 1;
    return 0;
}

/* Fast path, O(N log N) once: when no transfer reads bytes that any transfer writes (the
 * source and destination hulls are disjoint, as for every SEND -> RECV plan) and no two
 * writes of the same bytes carry different data (one sort of every write by address),
 * there is no hazard anywhere.  Returns 1 when that holds. */
static int hazard_free(const xg_span *xfer, int n)
{
    uint64_t slo = UINT64_MAX, shi = 0, dlo = UINT64_MAX, dhi = 0;
    int i, m = 0, ok = 1;
    for (i = 0; i < n; ++i)
        if (xfer[i].len) {
            if (xfer[i].src < slo) slo = xfer[i].src;
            if (xfer[i].src + xfer[i].len > shi) shi = xfer[i].src + xfer[i].len;
            if (xfer[i].dst < dlo) dlo = xfer[i].dst;
            if (xfer[i].dst + xfer[i].len > dhi) dhi = xfer[i].dst + xfer[i].len;
            m++;
        }
    if (!m) return 1;
    if (slo < dhi && dlo < shi) return 0;            /* a read may meet a write: full scan */
    ivl *w = (ivl *)malloc(sizeof(ivl) * (size_t)m);
    if (!w) return 0;
    for (i = 0, m = 0; i < n; ++i)
        if (xfer[i].len) {
            w[m].lo = xfer[i].dst;
            w[m].hi = xfer[i].dst + xfer[i].len;
            w[m].delta = (int64_t)(xfer[i].dst - xfer[i].src);
            m++;
        }
    qsort(w, (size_t)m, sizeof(ivl), cmp_ivl);
    uint64_t reach = 0;                               /* end of the writes seen so far ... */
    int64_t rdelta = 0;                               /* ... and the delta of the one reaching it */
    for (i = 0; i < m && ok; ++i) {
        if (i && w[i].lo < reach && w[i].delta != rdelta) ok = 0;   /* overlap, other bytes */
        if (w[i].hi > reach) {
            reach = w[i].hi;
            rdelta = w[i].delta;
        }
    }
    free(w);
    return ok;
}

int xg_engine_hazards(const xg_span *xfer, const int *step_begin, int nsteps, int force, int *flags)
{
    ivl *pend = NULL, *tmp = NULL;
    int npend = 0, cap = 0, s, k, nhaz = 0;
    if (nsteps <= 0) return 0;
    for (s = 0; s < nsteps; ++s) flags[s] = force ? 1 : 0;
    if (hazard_free(xfer, step_begin[nsteps])) {
        if (flags[nsteps - 1] < 1) flags[nsteps - 1] = 1;
        return 0;
    }
    cap = 64;
    pend = (ivl *)malloc(sizeof(ivl) * cap);
    tmp = (ivl *)malloc(sizeof(ivl) * cap);
    if (!pend || !tmp) abort();
    for (s = 0; s < nsteps; ++s) {
        const int b = step_begin[s], e = step_begin[s + 1];
        int hazard = 0, nnew = 0, n, m;
        /* does step s conflict with the writes pending since the last hazard point? */
        for (k = b; k < e && s > 0 && !hazard; ++k) {
            const xg_span *x = &xfer[k];
            if (!x->len) continue;
            if (meets(pend, npend, x->src, x->src + x->len, 0, 0) ||
                meets(pend, npend, x->dst, x->dst + x->len, 1, (int64_t)(x->dst - x->src)))
                hazard = 1;
        }
        if (hazard) {
            flags[s - 1] = 2;
            nhaz++;
            npend = 0;
        }
        /* add step s's writes, then re-sort and merge same-delta overlapping / touching runs */
        if (npend + (e - b) > cap) {
            cap = 2 * (npend + (e - b)) + 64;
            pend = (ivl *)realloc(pend, sizeof(ivl) * cap);
            tmp = (ivl *)realloc(tmp, sizeof(ivl) * cap);
            if (!pend || !tmp) abort();
        }
        for (k = b; k < e; ++k)
            if (xfer[k].len) {
                pend[npend + nnew].lo = xfer[k].dst;
                pend[npend + nnew].hi = xfer[k].dst + xfer[k].len;
                pend[npend + nnew].delta = (int64_t)(xfer[k].dst - xfer[k].src);
                nnew++;
            }
        n = npend + nnew;
        qsort(pend, n, sizeof(ivl), cmp_ivl);
        for (m = 0, k = 0; k < n; ++k) {
            if (m && tmp[m - 1].delta == pend[k].delta && pend[k].lo <= tmp[m - 1].hi) {
                if (pend[k].hi > tmp[m - 1].hi) tmp[m - 1].hi = pend[k].hi;
            } else if (m && pend[k].lo < tmp[m - 1].hi) {
                /* two writes of one step to the same bytes with different data: a race
                 * inside a step; order it before the next step at least */
                if (pend[k].hi > tmp[m - 1].hi) tmp[m - 1].hi = pend[k].hi;
                tmp[m - 1].delta = pend[k].delta;
                if (s + 1 < nsteps && flags[s] != 2) { flags[s] = 2; nhaz++; }
            } else {
                tmp[m++] = pend[k];
            }
        }
        memcpy(pend, tmp, sizeof(ivl) * m);
        npend = m;
        if (s + 1 < nsteps && flags[s] == 2) npend = 0;
    }
    if (flags[nsteps - 1] < 1) flags[nsteps - 1] = 1;
    free(pend);
    free(tmp);
    return nhaz;
}
