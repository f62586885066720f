/*
 * calls.c -- the RCCL calls of a device plan, and how RCCL pairs them across GPUs.
 *
 * xg_devplan_step_calls is THE definition of what GPU g posts in step s: one
 * ncclGroupStart/End around its send/recv calls (in this order; with self_max > 0
 * a cross-GPU step's small local part joins them as self send/recv pairs), then
 * one ncclAllReduce when the step ends in an in-loop MPI_Barrier.  The real
 * multi-GPU path of the runtime (runtime/exec.hip, enqueue_step) posts exactly
 * that list; the one-device virtual runner (xg_vplans_run / _rccl) moves exactly
 * the pairs xg_calls_match makes of every GPU's lists.
 *
 * xg_calls_match pairs calls the way RCCL does: per ordered GPU pair (g, h), the
 * k-th send of g to h with the k-th receive of h from g, in issue order over the
 * whole run -- RCCL's per-(peer, communicator) FIFO knows no steps.  A job is
 * accepted only if every such pair falls in ONE step and ONE group of it (a relay
 * step has two, separated by XG_CALL_FENCE) with ONE length and every
 * GPU ends the same steps with a barrier: then each step's groups pair among
 * themselves, every GPU posts its collectives in the same order, and no group
 * waits for one a peer posts later (the job cannot hang on a mismatch).
 *
 * Reference: the point-to-point calls the plans replace -- m1 MPI_Issend /
 * MPI_Irecv (mpi_test.c:1776,1790), m9 MPI_Sendrecv (:551,558), m5/m8
 * MPI_Alltoallw (:627,912) -- and the in-loop MPI_Barrier of m13/m17/m19.
 */
#include "xg_sched.h"

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* the step's local gather/scatter copies: pre copies after the stage copies, before the packs */
static void local_range(const xg_devplan *dp, const xg_stepplan *sp, int *b, int *e, int64_t *bytes)
{
    int i;
    *b = sp->pre_begin + sp->stage_count;
    *e = *b;
    *bytes = 0;
    for (i = sp->stage_count; i < sp->pre_count; ++i) {
        const xg_copy *c = &dp->copies[sp->pre_begin + i];
        if (c->dst_buf == XG_BUF_STAGE_SEND) break;
        *e = sp->pre_begin + i + 1;
        *bytes += c->len > 0 ? c->len : 0;
    }
}

int xg_devplan_step_self_calls(const xg_devplan *dp, int step, int64_t self_max)
{
    int b, e, i, n = 0;
    int64_t bytes;
    const xg_stepplan *sp;
    if (!dp || step < 0 || step >= dp->nsteps || self_max <= 0) return 0;
    sp = &dp->steps[step];
    if (!sp->p2p_count) return 0;
    local_range(dp, sp, &b, &e, &bytes);
    if (bytes > self_max) return 0;
    for (i = b; i < e; ++i) n += dp->copies[i].len > 0;
    return n;
}

static void put_p2p(xg_call *c, const xg_p2p *o)
{
    c->kind = o->is_send ? XG_CALL_SEND : XG_CALL_RECV;
    c->peer = o->peer;
    c->buf = o->buf;
    c->pad = 0;
    c->off = o->off;
    c->len = o->len;
}

int xg_devplan_step_calls(const xg_devplan *dp, int step, int64_t self_max, xg_call *out)
{
    const xg_stepplan *sp;
    int i, n = 0, g1;
    if (!dp || step < 0 || step >= dp->nsteps) return -1;
    sp = &dp->steps[step];
    /* group 0's send/recv calls (the plan lists a relay step's group 1 after them) */
    for (g1 = 0; g1 < sp->p2p_count && dp->p2p[sp->p2p_begin + g1].group == 0; ++g1, ++n)
        if (out) put_p2p(&out[n], &dp->p2p[sp->p2p_begin + g1]);
    if (xg_devplan_step_self_calls(dp, step, self_max)) {
        /* the step's local copies as self send + receive pairs inside its group: one RCCL
         * launch carries the whole step (RCCL pairs the k-th self send with the k-th self
         * receive, so each pair is one copy) */
        int b, e;
        int64_t bytes;
        local_range(dp, sp, &b, &e, &bytes);
        for (i = b; i < e; ++i) {
            const xg_copy *c = &dp->copies[i];
            if (c->len <= 0) continue;
            if (out) {
                out[n].kind = XG_CALL_SEND; out[n].peer = dp->gpu; out[n].buf = c->src_buf; out[n].pad = 0;
                out[n].off = c->src_off; out[n].len = c->len;
                out[n + 1].kind = XG_CALL_RECV; out[n + 1].peer = dp->gpu; out[n + 1].buf = c->dst_buf;
                out[n + 1].pad = 0; out[n + 1].off = c->dst_off; out[n + 1].len = c->len;
            }
            n += 2;
        }
    }
    if (g1 < sp->p2p_count) {
        /* a relay step's second group (the forwards and the direct second pieces) behind a fence:
         * the runtime closes group 0 (ncclGroupEnd) before it opens this one */
        if (out) {
            memset(&out[n], 0, sizeof out[n]);
            out[n].kind = XG_CALL_FENCE;
            out[n].peer = -1;
            out[n].buf = -1;
        }
        ++n;
        for (i = g1; i < sp->p2p_count; ++i, ++n)
            if (out) put_p2p(&out[n], &dp->p2p[sp->p2p_begin + i]);
    }
    if (sp->sync_after) {
        if (out) {
            memset(&out[n], 0, sizeof out[n]);
            out[n].kind = XG_CALL_BARRIER;
            out[n].peer = -1;
            out[n].buf = -1;
        }
        ++n;
    }
    return n;
}

static void fail(char *err, size_t errlen, const char *fmt, ...)
{
    va_list ap;
    if (!err || !errlen) return;
    va_start(ap, fmt);
    vsnprintf(err, errlen, fmt, ap);
    va_end(ap);
}

/* the step of call i of GPU g (step_begin is sorted) */
static int step_of(const int32_t *sb, int nsteps, int i)
{
    int lo = 0, hi = nsteps - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) / 2;
        if (sb[mid] <= i) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

int64_t xg_calls_match(int ngpus, int nsteps, const xg_call *const *calls, const int32_t *const *step_begin,
                       xg_call_pair *out, int64_t max_pairs, char *err, size_t errlen)
{
    const int G = ngpus;
    int g, h, s, ngrp = 1;
    int64_t k, nsend = 0, nrecv = 0, np = 0;
    int64_t *soff = NULL, *roff = NULL, *sfill = NULL, *rfill = NULL, *cnt = NULL;
    int32_t *sidx = NULL, *ridx = NULL;
    int32_t **grp = NULL;       /* per GPU and call: the group of its step the call is in */
    xg_call_pair *pairs = NULL;
    int64_t rc = -1;
    if (err && errlen) err[0] = 0;
    if (G < 1 || nsteps < 0 || !calls || !step_begin) {
        fail(err, errlen, "xg_calls_match: bad arguments");
        return -1;
    }
    /* shape of every list; the in-loop barriers: the same steps on every GPU, each the
     * step's last call (the collective follows the step's group on every GPU) */
    for (g = 0; g < G; ++g) {
        const int32_t *sb = step_begin[g];
        if (sb[0] != 0) {
            fail(err, errlen, "GPU %d: call list does not start at 0", g);
            return -1;
        }
        for (s = 0; s < nsteps; ++s) {
            int i, bar = 0, gi = 0;
            if (sb[s + 1] < sb[s]) {
                fail(err, errlen, "GPU %d: step %d has a negative call count", g, s);
                return -1;
            }
            for (i = sb[s]; i < sb[s + 1]; ++i) {
                const xg_call *c = &calls[g][i];
                if (c->kind == XG_CALL_BARRIER) {
                    bar = 1;
                    continue;
                }
                if (c->kind == XG_CALL_FENCE) {
                    if (bar) {
                        fail(err, errlen, "GPU %d step %d: a group fence after the step's barrier", g, s);
                        return -1;
                    }
                    if (++gi + 1 > ngrp) ngrp = gi + 1;
                    continue;
                }
                if (c->kind != XG_CALL_SEND && c->kind != XG_CALL_RECV) {
                    fail(err, errlen, "GPU %d step %d: call %d of unknown kind %d", g, s, i, c->kind);
                    return -1;
                }
                if (bar) {
                    fail(err, errlen, "GPU %d step %d: a send/recv after the step's barrier", g, s);
                    return -1;
                }
                if (c->peer < 0 || c->peer >= G || c->len < 0) {
                    fail(err, errlen, "GPU %d step %d: call %d to peer %d of %lld bytes", g, s, i, c->peer,
                         (long long)c->len);
                    return -1;
                }
                if (c->kind == XG_CALL_SEND) nsend++;
                else nrecv++;
            }
            if (g > 0) {
                int b0 = 0;
                for (i = step_begin[0][s]; i < step_begin[0][s + 1]; ++i) b0 |= calls[0][i].kind == XG_CALL_BARRIER;
                if (b0 != bar) {
                    fail(err, errlen, "step %d: GPU 0 %s a barrier, GPU %d %s", s, b0 ? "ends with" : "has no", g,
                         bar ? "ends with one" : "has none");
                    return -1;
                }
            }
        }
    }
    if (nsend != nrecv) {
        fail(err, errlen, "the job posts %lld sends and %lld receives", (long long)nsend, (long long)nrecv);
        return -1;
    }
    /* channel (g -> h): g's sends to h and h's receives from g, each in issue order */
    soff = (int64_t *)calloc((size_t)G * G + 1, sizeof(int64_t));
    roff = (int64_t *)calloc((size_t)G * G + 1, sizeof(int64_t));
    sfill = (int64_t *)calloc((size_t)G * G, sizeof(int64_t));
    rfill = (int64_t *)calloc((size_t)G * G, sizeof(int64_t));
    sidx = (int32_t *)malloc(sizeof(int32_t) * (size_t)(nsend + 1));
    ridx = (int32_t *)malloc(sizeof(int32_t) * (size_t)(nrecv + 1));
    if (!soff || !roff || !sfill || !rfill || !sidx || !ridx) {
        fail(err, errlen, "xg_calls_match: out of memory");
        goto done;
    }
    for (g = 0; g < G; ++g)
        for (k = 0; k < step_begin[g][nsteps]; ++k) {
            const xg_call *c = &calls[g][k];
            if (c->kind == XG_CALL_SEND) soff[(size_t)g * G + c->peer + 1]++;
            else if (c->kind == XG_CALL_RECV) roff[(size_t)c->peer * G + g + 1]++;
        }
    for (k = 0; k < (int64_t)G * G; ++k) {
        soff[k + 1] += soff[k];
        roff[k + 1] += roff[k];
    }
    for (g = 0; g < G; ++g)
        for (k = 0; k < step_begin[g][nsteps]; ++k) {
            const xg_call *c = &calls[g][k];
            if (c->kind == XG_CALL_SEND) {
                const size_t ch = (size_t)g * G + c->peer;
                sidx[soff[ch] + sfill[ch]++] = (int32_t)k;
            } else if (c->kind == XG_CALL_RECV) {
                const size_t ch = (size_t)c->peer * G + g;
                ridx[roff[ch] + rfill[ch]++] = (int32_t)k;
            }
        }
    pairs = (xg_call_pair *)malloc(sizeof(xg_call_pair) * (size_t)(nsend + 1));
    cnt = (int64_t *)calloc((size_t)nsteps * ngrp + 1, sizeof(int64_t));
    grp = (int32_t **)calloc((size_t)G, sizeof(int32_t *));
    if (!pairs || !cnt || !grp) {
        fail(err, errlen, "xg_calls_match: out of memory");
        goto done;
    }
    for (g = 0; g < G; ++g) {
        const int32_t *sb = step_begin[g];
        if (!(grp[g] = (int32_t *)malloc(sizeof(int32_t) * ((size_t)sb[nsteps] + 1)))) {
            fail(err, errlen, "xg_calls_match: out of memory");
            goto done;
        }
        for (s = 0; s < nsteps; ++s) {
            int i, gi = 0;
            for (i = sb[s]; i < sb[s + 1]; ++i) {
                gi += calls[g][i].kind == XG_CALL_FENCE;
                grp[g][i] = gi;
            }
        }
    }
    for (g = 0; g < G; ++g)
        for (h = 0; h < G; ++h) {
            const size_t ch = (size_t)g * G + h;
            const int64_t ns = soff[ch + 1] - soff[ch], nr = roff[ch + 1] - roff[ch];
            if (ns != nr) {
                fail(err, errlen, "GPU %d posts %lld sends to GPU %d, which posts %lld receives from it", g,
                     (long long)ns, h, (long long)nr);
                goto done;
            }
            for (k = 0; k < ns; ++k) {
                const int32_t si = sidx[soff[ch] + k], ri = ridx[roff[ch] + k];
                const int ss = step_of(step_begin[g], nsteps, si), rs = step_of(step_begin[h], nsteps, ri);
                const xg_call *sc = &calls[g][si], *rcv = &calls[h][ri];
                xg_call_pair *q = &pairs[np++];
                if (ss != rs) {
                    fail(err, errlen, "send %lld of GPU %d to GPU %d is posted in step %d, its receive in step %d",
                         (long long)k, g, h, ss, rs);
                    goto done;
                }
                if (grp[g][si] != grp[h][ri]) {
                    fail(err, errlen, "step %d: send %lld of GPU %d to GPU %d is in group %d, its receive in group %d",
                         ss, (long long)k, g, h, grp[g][si], grp[h][ri]);
                    goto done;
                }
                if (sc->len != rcv->len) {
                    fail(err, errlen, "step %d: send %lld of GPU %d to GPU %d carries %lld bytes, its receive %lld", ss,
                         (long long)k, g, h, (long long)sc->len, (long long)rcv->len);
                    goto done;
                }
                q->step = ss; q->src = g; q->dst = h; q->send_call = si; q->recv_call = ri; q->group = grp[g][si];
                q->len = sc->len;
                cnt[(size_t)ss * ngrp + q->group + 1]++;
            }
        }
    /* (step, group)-major, stable: inside a group by (src, dst, k) */
    for (k = 0; k < (int64_t)nsteps * ngrp; ++k) cnt[k + 1] += cnt[k];
    if (out && max_pairs >= np) {
        for (k = 0; k < np; ++k) out[cnt[(size_t)pairs[k].step * ngrp + pairs[k].group]++] = pairs[k];
    }
    rc = np;
done:
    free(soff); free(roff); free(sfill); free(rfill); free(sidx); free(ridx); free(pairs); free(cnt);
    for (g = 0; grp && g < G; ++g) free(grp[g]);
    free(grp);
    return rc;
}

int64_t xg_devplans_match(const xg_devplan *const *plans, int ngpus, int64_t self_max, xg_call_pair *out,
                          int64_t max_pairs, char *err, size_t errlen)
{
    const int G = ngpus;
    int g, s, nsteps;
    int64_t rc = -1;
    xg_call **calls = NULL;
    int32_t **sb = NULL;
    if (err && errlen) err[0] = 0;
    if (G < 1 || !plans || !plans[0]) {
        fail(err, errlen, "xg_devplans_match: bad arguments");
        return -1;
    }
    nsteps = plans[0]->nsteps;
    for (g = 0; g < G; ++g)
        if (!plans[g] || plans[g]->gpu != g || plans[g]->ngpus != G || plans[g]->nsteps != nsteps) {
            fail(err, errlen, "plan %d is not GPU %d of one %d-GPU job of %d steps", g, g, G, nsteps);
            return -1;
        }
    calls = (xg_call **)calloc(G, sizeof *calls);
    sb = (int32_t **)calloc(G, sizeof *sb);
    if (!calls || !sb) goto done;
    for (g = 0; g < G; ++g) {
        int n = 0;
        sb[g] = (int32_t *)malloc(sizeof(int32_t) * ((size_t)nsteps + 1));
        if (!sb[g]) goto done;
        for (s = 0; s < nsteps; ++s) {
            sb[g][s] = n;
            n += xg_devplan_step_calls(plans[g], s, self_max, NULL);
        }
        sb[g][nsteps] = n;
        calls[g] = (xg_call *)malloc(sizeof(xg_call) * ((size_t)n + 1));
        if (!calls[g]) goto done;
        for (s = 0; s < nsteps; ++s) xg_devplan_step_calls(plans[g], s, self_max, calls[g] + sb[g][s]);
    }
    rc = xg_calls_match(G, nsteps, (const xg_call *const *)calls, (const int32_t *const *)sb, out, max_pairs, err,
                        errlen);
done:
    if (rc < 0 && err && errlen && !err[0]) fail(err, errlen, "xg_devplans_match: out of memory");
    for (g = 0; calls && g < G; ++g) free(calls[g]);
    for (g = 0; sb && g < G; ++g) free(sb[g]);
    free(calls);
    free(sb);
    return rc;
}
