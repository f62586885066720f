/*
 * sched.c -- the host schedule: placement (create_aggregator_list), MPI matching of the per-rank
 * programs programs.c builds, the step compiler that turns the reference's per-process MPI
 * schedules into device-wide steps, per-rank traces and timers, and the block mapping of ranks
 * and regions onto GPUs.  Plain C99, no HIP.  See include/xg_sched.h.  The device-plan builder
 * over a compiled schedule is devplan.c.
 */
#include "sched_int.h"

#include <limits.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------ public: placement / labels */
int xg_aggregator_list(int procs, int cb_nodes, int proc_node, int type, int *rl)
{
    int i, remainder, ceiling, floor_;
    if (type == 1 || type == 2) {                 /* :1956-1990, quirk: remainder = procs / cb_nodes */
        remainder = procs / cb_nodes;
        ceiling = (procs + cb_nodes - 1) / cb_nodes;
        floor_ = procs / cb_nodes;
        for (i = 0; i < cb_nodes; ++i) {
            int v = i < remainder ? ceiling * i : ceiling * remainder + floor_ * (i - remainder);
            rl[i] = type == 1 ? v : (v - 16 + procs * 16) % procs;
        }
    } else if (type == 0) {                       /* :1970-1976 */
        for (i = 0; i < cb_nodes; ++i) rl[i] = i;
    } else if (type == 3) {                       /* :1991-2002 */
        remainder = 0;
        for (i = 0; i < cb_nodes; ++i) {
            rl[i] = remainder;
            remainder += proc_node;
            if (remainder >= procs) remainder = remainder % proc_node + 1;
        }
    } else {
        return -1;
    }
    return 0;
}

const char *xg_method_label(int method)   /* mpi_test.c:2186-2337 */
{
    static const char *labels[] = {
        NULL, "All to many", "Many to all", "All to many balanced", "Many to all balanced",
        "Many to all benchmark", "All to many sync", "All to many half sync", "All to many benchmark",
        "All to many pairwise", "Many to all pairwise", "Many to all half sync", "All to many half sync 2",
        "All to many scattered", "Many to all scattered", "All to many TAM", "Many to all TAM",
        "All to many node robin", "All to many balanced control", "All to many scattered isend",
        "All to many balanced presend",
    };
    return method >= 1 && method <= 20 ? labels[method] : NULL;
}

int xg_method_direction(int method)
{
    switch (method) {
    case 1: case 3: case 6: case 7: case 8: case 9: case 12: case 13: case 17: case 18: case 19: case 20:
        return XG_A2M;
    case 15: return XG_A2M;  /* all_to_many_tam: prepare_all_to_many_data layout (:380) */
    case 2: case 4: case 5: case 10: case 11: case 14: return XG_M2A;
    case 16: return XG_M2A;  /* many_to_all_tam: prepare_many_to_all_data layout (:329) */
    default: return -1;
    }
}

/* ------------------------------------------------------------------ matching */
typedef struct {
    int32_t coll, comm, a, b, tag, rank, post, idx;
    int64_t cnt;            /* bytes */
    int32_t lb, pad;        /* logical buffer of the data end (LB_*)  */
    int64_t off;            /* byte offset in it                      */
} pst_t;

/* channel = (collective, communicator, src, dst, tag); FIFO inside a channel */
static int pst_cmp(const void *x_, const void *y_)
{
    const pst_t *x = (const pst_t *)x_, *y = (const pst_t *)y_;
    if (x->coll != y->coll) return x->coll < y->coll ? -1 : 1;
    if (x->comm != y->comm) return x->comm < y->comm ? -1 : 1;
    if (x->a != y->a) return x->a < y->a ? -1 : 1;
    if (x->b != y->b) return x->b < y->b ? -1 : 1;
    if (x->tag != y->tag) return x->tag < y->tag ? -1 : 1;
    return x->post < y->post ? -1 : x->post > y->post;
}

static int same_channel(const pst_t *x, const pst_t *y)
{
    return x->coll == y->coll && x->comm == y->comm && x->a == y->a && x->b == y->b && x->tag == y->tag;
}

static xg_msg *new_msg(xg_sched *s)
{
    if (s->nmsg == s->msgcap) {
        s->msgcap = s->msgcap ? 2 * s->msgcap : 1024;
        s->msgs = (xg_msg *)realloc(s->msgs, sizeof(xg_msg) * s->msgcap);
        s->msg_spost = (int32_t *)realloc(s->msg_spost, sizeof(int32_t) * s->msgcap);
        s->msg_rpost = (int32_t *)realloc(s->msg_rpost, sizeof(int32_t) * s->msgcap);
        if (!s->msgs || !s->msg_spost || !s->msg_rpost) abort();
    }
    memset(&s->msgs[s->nmsg], 0, sizeof(xg_msg));
    s->msg_spost[s->nmsg] = s->msg_rpost[s->nmsg] = -1;
    return &s->msgs[s->nmsg++];
}

/* logical (buffer, offset) of rank r -> region + offset inside the rank's part of it */
static void phys_loc(const xg_sched *s, int r, int lb, int64_t off, int32_t *buf, int64_t *o)
{
    switch (lb) {
    case LB_SEND: *buf = XG_BUF_SEND; *o = off; break;
    case LB_RECV: *buf = XG_BUF_RECV; *o = off; break;
    case LB_CTRL: *buf = -1; *o = off; break;
    default: *buf = XG_BUF_SCRATCH; *o = s->scr_base[(size_t)r * NSCR + (lb - LB_AGG)] + off; break;
    }
}

/* TAM scratch of every rank: AGG | SBUF2 | RBUF, each 256-byte aligned */
static void scratch_layout(xg_sched *s)
{
    int r, k;
    s->scr_base = (int64_t *)xgi_xmalloc(sizeof(int64_t) * NSCR * s->P);
    s->scr_size = (int64_t *)xgi_xmalloc(sizeof(int64_t) * s->P);
    for (r = 0; r < s->P; ++r) {
        int64_t o = 0;
        for (k = 0; k < NSCR; ++k) {
            s->scr_base[(size_t)r * NSCR + k] = o;
            o += (s->progs[r].hi[LB_AGG + k] + 255) & ~(int64_t)255;
        }
        s->scr_size[r] = o;
    }
}

static int do_match(xg_sched *s, char *err, size_t errlen)
{
    int r, i, ns = 0, nr = 0, j;
    size_t tot_s = 0, tot_r = 0;
    pst_t *S, *R;
    for (r = 0; r < s->P; ++r)
        for (i = 0; i < s->progs[r].nops; ++i) {
            tot_s += s->progs[r].ops[i].kind == OP_SEND;
            tot_r += s->progs[r].ops[i].kind == OP_RECV;
        }
    S = (pst_t *)xgi_xmalloc(sizeof(pst_t) * tot_s);
    R = (pst_t *)xgi_xmalloc(sizeof(pst_t) * tot_r);
    for (r = 0; r < s->P; ++r) {
        const prog_t *p = &s->progs[r];
        for (i = 0; i < p->nops; ++i) {
            const op_t *o = &p->ops[i];
            if (o->kind == OP_SEND) {
                pst_t t = { o->coll, o->comm, r, o->peer, o->coll >= 0 ? 0 : o->tag, r, o->post, o->idx,
                            o->cnt * o->esz, o->sb, 0, o->idx >= 0 ? (int64_t)o->idx * s->d : o->off };
                S[ns++] = t;
            } else if (o->kind == OP_RECV) {
                pst_t t = { o->coll, o->comm, o->peer, r, o->coll >= 0 ? 0 : o->tag, r, o->post, o->idx,
                            o->cnt * o->esz, o->db, 0, o->idx >= 0 ? (int64_t)o->idx * s->d : o->off2 };
                R[nr++] = t;
            }
        }
    }
    qsort(S, ns, sizeof(pst_t), pst_cmp);
    qsort(R, nr, sizeof(pst_t), pst_cmp);
    for (i = 0, j = 0; i < ns || j < nr; ++i, ++j) {
        xg_msg *m;
        if (i >= ns || j >= nr || !same_channel(&S[i], &R[j])) {
            const pst_t *u = i < ns ? &S[i] : &R[j];
            snprintf(err, errlen, "unmatched point-to-point traffic %d -> %d (the reference would hang)", u->a, u->b);
            free(S); free(R);
            return -1;
        }
        if (S[i].cnt > R[j].cnt) {
            snprintf(err, errlen, "message truncated %d -> %d", S[i].a, S[i].b);
            free(S); free(R);
            return -1;
        }
        if ((S[i].lb == LB_CTRL) != (R[j].lb == LB_CTRL)) {
            snprintf(err, errlen, "size message matched with a data message %d -> %d", S[i].a, S[i].b);
            free(S); free(R);
            return -1;
        }
        m = new_msg(s);
        m->src = S[i].a; m->sseg = S[i].idx; m->dst = S[i].b; m->dslot = R[j].idx;
        m->len = S[i].cnt; m->step = -1;
        m->flags = (S[i].coll >= 0 ? XG_MSG_COLL : 0) | (S[i].lb == LB_CTRL ? XG_MSG_CTRL : 0);
        phys_loc(s, S[i].a, S[i].lb, S[i].off, &m->sbuf, &m->soff);
        phys_loc(s, R[j].b, R[j].lb, R[j].off, &m->dbuf, &m->doff);
        s->msg_spost[s->nmsg - 1] = S[i].post;
        s->msg_rpost[s->nmsg - 1] = R[j].post;
        s->post_msg[S[i].rank][S[i].post] = s->nmsg - 1;
        s->post_msg[R[j].rank][R[j].post] = s->nmsg - 1;
    }
    free(S); free(R);
    /* self copies become messages too (their step is set by the step compiler) */
    for (r = 0; r < s->P; ++r) {
        prog_t *p = &s->progs[r];
        for (i = 0; i < p->nops; ++i)
            if (p->ops[i].kind == OP_COPY) {
                const op_t *o = &p->ops[i];
                xg_msg *m = new_msg(s);
                m->src = m->dst = r; m->sseg = o->idx; m->dslot = o->idx2;
                m->len = o->cnt; m->step = -1; m->flags = XG_MSG_COPY;
                phys_loc(s, r, o->sb, o->idx >= 0 ? (int64_t)o->idx * s->d : o->off, &m->sbuf, &m->soff);
                phys_loc(s, r, o->db, o->idx2 >= 0 ? (int64_t)o->idx2 * s->d : o->off2, &m->dbuf, &m->doff);
                p->ops[i].post = s->nmsg - 1;
            }
    }
    return 0;
}

/* ------------------------------------------------------------------ step compiler */
static int compile_steps(xg_sched *s, char *err, size_t errlen)
{
    int P = s->P, r, progress = 1, maxstep = -1, b;
    int *pc = (int *)xgi_xmalloc(sizeof(int) * P), *epoch = (int *)xgi_xmalloc(sizeof(int) * P);
    int32_t **pe = (int32_t **)xgi_xmalloc(sizeof(int32_t *) * P);     /* post epoch */
    int nb = s->progs[0].nbarrier;
    int *arrived = (int *)xgi_xcalloc(nb + 1, sizeof(int)), *arr_epoch = (int *)xgi_xmalloc(sizeof(int) * (nb + 1));
    int *lw = (int *)xgi_xmalloc(sizeof(int) * NLB * P), *lrd = (int *)xgi_xmalloc(sizeof(int) * NLB * P);
    for (r = 0; r < NLB * P; ++r) lw[r] = lrd[r] = INT_MIN / 2;
    for (r = 1; r < P; ++r)
        if (s->progs[r].nbarrier != nb) {
            snprintf(err, errlen, "ranks disagree on the number of MPI_Barrier calls");
            free(arrived); free(arr_epoch); free(pc); free(epoch); free(pe); free(lw); free(lrd);
            return -1;
        }
    s->nbarrier = nb;
    s->barrier_epoch = (int32_t *)xgi_xmalloc(sizeof(int32_t) * (nb + 1));
    for (b = 0; b < nb; ++b) { arr_epoch[b] = -1; s->barrier_epoch[b] = INT_MIN; }
    for (r = 0; r < P; ++r) {
        int q;
        pc[r] = 0; epoch[r] = -1;
        pe[r] = (int32_t *)xgi_xmalloc(sizeof(int32_t) * (s->progs[r].nposts + 1));
        for (q = 0; q < s->progs[r].nposts; ++q) pe[r][q] = INT_MIN;
    }
    while (progress) {
        progress = 0;
        for (r = 0; r < P; ++r) {
            prog_t *p = &s->progs[r];
            while (pc[r] < p->nops) {
                op_t *o = &p->ops[pc[r]];
                if (o->kind == OP_BARRIER) {
                    /* collective: every rank arrives, all leave at the latest arrival epoch */
                    b = o->post;
                    if (o->eager_ok == 0) {                 /* first visit: register arrival */
                        o->eager_ok = 1;
                        arrived[b]++;
                        if (epoch[r] > arr_epoch[b]) arr_epoch[b] = epoch[r];
                    }
                    if (arrived[b] < P) break;
                    s->barrier_epoch[b] = arr_epoch[b];
                    if (arr_epoch[b] > epoch[r]) epoch[r] = arr_epoch[b];
                } else if (o->kind == OP_SEND || o->kind == OP_RECV) {
                    pe[r][o->post] = epoch[r];
                } else if (o->kind == OP_SYNC) {
                    if (o->idx > epoch[r]) epoch[r] = o->idx;
                    if (o->idx > maxstep) maxstep = o->idx;
                } else if (o->kind == OP_COPY) {
                    /* after everything the rank completed, after the last copy that wrote its
                     * source, after the last copy that read its destination; what the rank
                     * posts next moves no earlier than the copy (DESIGN.md "copy steps") */
                    int *w = lw + (size_t)r * NLB, *rd = lrd + (size_t)r * NLB;
                    int cs = epoch[r] + 1;
                    if (w[o->sb] + 1 > cs) cs = w[o->sb] + 1;
                    if (rd[o->db] + 1 > cs) cs = rd[o->db] + 1;
                    if (cs > w[o->db]) w[o->db] = cs;
                    if (cs > rd[o->sb]) rd[o->sb] = cs;
                    if (cs - 1 > epoch[r]) epoch[r] = cs - 1;
                    s->msgs[o->post].step = cs;
                    if (cs > maxstep) maxstep = cs;
                } else if (o->kind == OP_WAIT) {
                    int q, blocked = 0, e = epoch[r];
                    for (q = 0; q < o->wcnt; ++q) {
                        int post = p->pool[o->wbeg + q], mi;
                        xg_msg *m;
                        if (s->post_eager[r][post]) continue;       /* eager send: completes locally */
                        mi = s->post_msg[r][post];
                        m = &s->msgs[mi];
                        if (m->step < 0) {
                            int a = pe[m->src][s->msg_spost[mi]], b = pe[m->dst][s->msg_rpost[mi]];
                            if (a == INT_MIN || b == INT_MIN) { blocked = 1; break; }
                            m->step = (a > b ? a : b) + 1;
                            if (m->step > maxstep) maxstep = m->step;
                        }
                        if (m->step > e) e = m->step;
                    }
                    if (blocked) break;
                    epoch[r] = e;
                }
                pc[r]++;
                progress = 1;
            }
        }
    }
    for (r = 0; r < P; ++r)
        if (pc[r] < s->progs[r].nops) {
            snprintf(err, errlen,
                     "method %d deadlocks under MPI semantics at P=%d A=%d d=%lld c=%d (rank %d blocked; "
                     "the reference hangs here too)", s->method, s->P, s->A, (long long)s->d, s->c, r);
            break;
        }
    {
        int bad = r < P, i;
        for (i = 0; !bad && i < s->nmsg; ++i)
            if (s->msgs[i].step < 0) {      /* a message nobody waits for: runs after its posts */
                int a = pe[s->msgs[i].src][s->msg_spost[i]], b = pe[s->msgs[i].dst][s->msg_rpost[i]];
                s->msgs[i].step = (a > b ? a : b) + 1;
                if (s->msgs[i].step > maxstep) maxstep = s->msgs[i].step;
            }
        for (r = 0; r < P; ++r) free(pe[r]);
        free(pe); free(pc); free(epoch); free(arrived); free(arr_epoch); free(lw); free(lrd);
        s->nsteps = maxstep + 1;
        for (r = 0; r < P; ++r) {       /* reset the arrival marks used above */
            int i;
            for (i = 0; i < s->progs[r].nops; ++i)
                if (s->progs[r].ops[i].kind == OP_BARRIER) s->progs[r].ops[i].eager_ok = 0;
        }
        return bad ? -1 : 0;
    }
}

/* ------------------------------------------------------------------ build */
void xg_sched_free(xg_sched *s)
{
    int r;
    if (!s) return;
    if (s->progs)
        for (r = 0; r < s->P; ++r) { free(s->progs[r].ops); free(s->progs[r].pool); }
    if (s->post_msg)
        for (r = 0; r < s->P; ++r) { free(s->post_msg[r]); free(s->post_eager[r]); }
    free(s->post_msg); free(s->post_eager);
    free(s->progs); free(s->msgs); free(s->msg_spost); free(s->msg_rpost); free(s->post_count);
    free(s->barrier_epoch); free(s->scr_base); free(s->scr_size);
    free(s->rank_list); free(s->isagg); free(s->agg_prefix);
    free(s);
}

xg_sched *xg_sched_build(int method, int procs, int cb_nodes, int64_t data_size, int comm_size,
                         const int *rank_list, int ntimes, int proc_node, int barrier_type,
                         int64_t eager_limit, char *err, size_t errlen)
{
    return xg_sched_build_iter(method, procs, cb_nodes, data_size, comm_size, rank_list, ntimes, proc_node,
                               barrier_type, eager_limit, 0, err, errlen);
}

xg_sched *xg_sched_build_iter(int method, int procs, int cb_nodes, int64_t data_size, int comm_size,
                              const int *rank_list, int ntimes, int proc_node, int barrier_type,
                              int64_t eager_limit, int iter, char *err, size_t errlen)
{
    xg_sched *s;
    int r, i, *lastidx;
    char dummy[8];
    if (!err) { err = dummy; errlen = sizeof dummy; }
    err[0] = 0;
    if (xg_method_direction(method) < 0) {
        snprintf(err, errlen, "method %d is not a method of the reference (1..20)", method);
        return NULL;
    }
    if (proc_node < 1) proc_node = 1;
    if (procs < 1 || cb_nodes < 1 || cb_nodes > procs || data_size < 0 || ntimes < 0) {
        snprintf(err, errlen, "bad sizes P=%d A=%d d=%lld k=%d", procs, cb_nodes, (long long)data_size, ntimes);
        return NULL;
    }
    if (comm_size < 1) { snprintf(err, errlen, "comm_size must be >= 1 (the reference divides by it)"); return NULL; }
    for (i = 0; i < cb_nodes; ++i)
        if (rank_list[i] < 0 || rank_list[i] >= procs) { snprintf(err, errlen, "aggregator %d out of range", rank_list[i]); return NULL; }
    s = (xg_sched *)xgi_xcalloc(1, sizeof *s);
    s->method = method; s->P = procs; s->A = cb_nodes; s->d = data_size; s->c = comm_size;
    s->ntimes = ntimes; s->eager = eager_limit; s->dir = xg_method_direction(method);
    s->proc_node = proc_node; s->barrier_type = barrier_type; s->iter = iter;
    s->rank_list = (int *)xgi_xmalloc(sizeof(int) * cb_nodes);
    memcpy(s->rank_list, rank_list, sizeof(int) * cb_nodes);
    s->isagg = (int *)xgi_xcalloc(procs, sizeof(int));
    s->agg_prefix = (int *)xgi_xmalloc(sizeof(int) * (procs + 1));
    for (i = 0; i < cb_nodes; ++i) s->isagg[rank_list[i]] = 1;
    s->agg_prefix[0] = 0;
    for (r = 0; r < procs; ++r) s->agg_prefix[r + 1] = s->agg_prefix[r] + s->isagg[r];
    s->progs = (prog_t *)xgi_xcalloc(procs, sizeof(prog_t));
    lastidx = (int *)xgi_xmalloc(sizeof(int) * procs);
    for (r = 0; r < procs; ++r) lastidx[r] = -1;
    for (i = 0; i < cb_nodes; ++i) lastidx[rank_list[i]] = i;
    for (r = 0; r < procs; ++r) {
        ctx_t x;
        prog_t *p = &s->progs[r];
        x.p = p; x.rank = r; x.isagg = s->isagg[r]; x.myindex = 0;
        x.P = procs; x.A = cb_nodes; x.c = comm_size; x.ntimes = ntimes; x.d = data_size; x.rl = rank_list;
        x.proc_node = proc_node; x.barrier_type = barrier_type;
        x.method = method; x.iter = iter; x.isagg_all = s->isagg; x.lastidx = lastidx;
        p->rank = r;
        for (i = 0; i < cb_nodes; ++i)            /* last match, :111-115 / :183-187 */
            if (rank_list[i] == r) x.myindex = i;
        xgi_program(&x);
    }
    free(lastidx);
    scratch_layout(s);
    s->post_msg = (int32_t **)xgi_xcalloc(procs, sizeof(int32_t *));
    s->post_eager = (uint8_t **)xgi_xcalloc(procs, sizeof(uint8_t *));
    for (r = 0; r < procs; ++r) {
        prog_t *p = &s->progs[r];
        s->post_msg[r] = (int32_t *)xgi_xmalloc(sizeof(int32_t) * (p->nposts + 1));
        s->post_eager[r] = (uint8_t *)xgi_xcalloc(p->nposts + 1, 1);
        for (i = 0; i < p->nops; ++i)
            if (p->ops[i].kind == OP_SEND && p->ops[i].eager_ok && p->ops[i].cnt * p->ops[i].esz <= eager_limit)
                s->post_eager[r][p->ops[i].post] = 1;
    }
    if (do_match(s, err, errlen) || compile_steps(s, err, errlen)) {
        xg_sched_free(s);
        return NULL;
    }
    return s;
}

int xg_sched_nmsg(const xg_sched *s) { return s->nmsg; }
const xg_msg *xg_sched_msgs(const xg_sched *s) { return s->msgs; }
int xg_sched_nsteps(const xg_sched *s) { return s->nsteps; }
int xg_sched_direction(const xg_sched *s) { return s->dir; }
int xg_sched_procs(const xg_sched *s) { return s->P; }

/* ------------------------------------------------------------------ traces */
typedef struct { char *buf; size_t len, cap; } sbuf;
static void sb_put(sbuf *b, const char *str)
{
    size_t n = strlen(str);
    if (b->buf && b->len + n < b->cap) memcpy(b->buf + b->len, str, n + 1);
    else if (b->buf && b->len < b->cap) { memcpy(b->buf + b->len, str, b->cap - 1 - b->len); b->buf[b->cap - 1] = 0; }
    b->len += n;
}

static int icmp(const void *a, const void *b) { return *(const int *)a - *(const int *)b; }

size_t xg_sched_trace(const xg_sched *s, int rank, char *buf, size_t buflen)
{
    sbuf b = { buf, 0, buflen };
    const prog_t *p = &s->progs[rank];
    int i, first = 1;
    char tok[64];
    if (buf && buflen) buf[0] = 0;
    for (i = 0; i < p->nops; ++i) {
        const op_t *o = &p->ops[i];
        tok[0] = 0;
        if (o->kind == OP_BARRIER) strcpy(tok, "B");
        else if (o->kind == OP_A2AW) strcpy(tok, "A");
        else if (o->coll >= 0) continue;
        else if (o->kind == OP_SEND || o->kind == OP_RECV) {
            const char k = o->kind == OP_RECV ? 'r' : (o->isend ? 'i' : 's');
            if (o->comm == 0 && o->tag == rank + o->peer) snprintf(tok, sizeof tok, "%c%d:%lld", k, o->peer, (long long)o->cnt);
            else if (o->comm == 0) snprintf(tok, sizeof tok, "%c%d:%lld#%d", k, o->peer, (long long)o->cnt, o->tag);
            else snprintf(tok, sizeof tok, "%c%d:%lld@%d#%d", k, o->peer, (long long)o->cnt, o->comm, o->tag);
        }
        else if (o->kind == OP_WAIT) {
            int *v = (int *)xgi_xmalloc(sizeof(int) * (o->wcnt + 1)), a = 0;
            if (o->wcnt) memcpy(v, p->pool + o->wbeg, sizeof(int) * o->wcnt);
            qsort(v, o->wcnt, sizeof(int), icmp);
            if (!first) sb_put(&b, " ");
            first = 0;
            sb_put(&b, "w");
            while (a < o->wcnt) {
                int e = a;
                while (e + 1 < o->wcnt && v[e + 1] == v[e] + 1) ++e;
                if (a) sb_put(&b, ",");
                if (e == a) snprintf(tok, sizeof tok, "%d", v[a]);
                else snprintf(tok, sizeof tok, "%d-%d", v[a], v[e]);
                sb_put(&b, tok);
                a = e + 1;
            }
            free(v);
            continue;
        } else continue;
        if (!first) sb_put(&b, " ");
        first = 0;
        sb_put(&b, tok);
    }
    return b.len;
}

/* ------------------------------------------------------------------ timers */
static void count_posts(xg_sched *s, int ngpus)
{
    int r, i;
    if (s->post_count && s->pc_ngpus == ngpus) return;
    free(s->post_count);
    s->post_count = (int32_t *)xgi_xcalloc((size_t)ngpus * (s->nsteps + 1), sizeof(int32_t));
    s->pc_ngpus = ngpus;
    for (r = 0; r < s->P; ++r) {
        const prog_t *p = &s->progs[r];
        int g = xg_gpu_of(s->P, ngpus, r);
        for (i = 0; i < p->nops; ++i)
            if (p->ops[i].kind == OP_SEND || p->ops[i].kind == OP_RECV) {
                int st = s->msgs[s->post_msg[r][p->ops[i].post]].step;
                if (st >= 0) s->post_count[(size_t)g * (s->nsteps + 1) + st]++;
            }
    }
}

/* the request posts of GPU g's ranks per step (out[nsteps], zeroed here): what count_posts counts,
 * for one GPU, without touching the schedule's cache (the device-plan builder takes it const) */
void xgi_step_posts_of(const xg_sched *s, int ngpus, int g, int32_t *out, int nout)
{
    int r, i, lo, hi;
    memset(out, 0, sizeof(int32_t) * (size_t)nout);
    xg_block_range(s->P, ngpus, g, &lo, &hi);
    for (r = lo; r < hi; ++r) {
        const prog_t *p = &s->progs[r];
        for (i = 0; i < p->nops; ++i)
            if (p->ops[i].kind == OP_SEND || p->ops[i].kind == OP_RECV) {
                const int st = s->msgs[s->post_msg[r][p->ops[i].post]].step;
                if (st >= 0 && st < nout) out[st]++;
            }
    }
}

static void set_field(xg_timer *t, int f, double v)
{
    double *d = (double *)t;
    d[f] = v;
}

static double get_field(const xg_timer *t, int f) { return ((const double *)t)[f]; }

/* Replays rank `rank`'s program on the logical clock.  G: the method Timer;
 * R (may be NULL): timers[m] of every repetition m (m13). */
static int rank_timers(xg_sched *s, int ngpus, int rank, const double *step_done, const double *step_post,
                       xg_timer *G, xg_timer *R)
{
    const prog_t *p = &s->progs[rank];
    double clock = 0, postacc = 0, open_c[NF], open_p[NF], reg_c[NREG] = {0, 0}, reg_p[NREG] = {0, 0};
    int depth[NF] = {0, 0, 0, 0, 0}, i, rep = 0;
    const int32_t *pc = NULL;
    xg_timer dummy;
    if (ngpus < 1 || rank < 0 || rank >= s->P) return -1;
    if (step_post) {
        count_posts(s, ngpus);
        pc = s->post_count + (size_t)xg_gpu_of(s->P, ngpus, rank) * (s->nsteps + 1);
    }
    memset(G, 0, sizeof *G);
    if (R) memset(R, 0, sizeof(xg_timer) * (s->ntimes > 0 ? s->ntimes : 1));
    for (i = 0; i < p->nops; ++i) {
        const op_t *o = &p->ops[i];
        xg_timer *tg = o->tgt == TG_R ? (R ? &R[rep] : &dummy) : G;
        xg_timer *src = o->tgt2 == TG_R ? (R ? &R[rep] : &dummy) : G;
        switch (o->kind) {
        case OP_SEND:
        case OP_RECV: {
            int st = s->msgs[s->post_msg[rank][o->post]].step;
            if (pc && st >= 0 && pc[st] > 0) postacc += step_post[st] / pc[st];
            break;
        }
        case OP_WAIT: {
            int q;
            for (q = 0; q < o->wcnt; ++q) {
                int post = p->pool[o->wbeg + q], st;
                if (s->post_eager[rank][post]) continue;       /* eager send: completes locally */
                st = s->msgs[s->post_msg[rank][post]].step;
                if (st >= 0 && step_done[st] > clock) clock = step_done[st];
            }
            break;
        }
        case OP_BARRIER: {
            int e = s->barrier_epoch[o->post];
            if (e >= 0 && step_done[e] > clock) clock = step_done[e];
            break;
        }
        case OP_SYNC:
            if (o->idx >= 0 && o->idx < s->nsteps && step_done[o->idx] > clock) clock = step_done[o->idx];
            break;
        case OP_TMARK:
            if (o->sign > 0) {
                if (depth[o->field]++ == 0) { open_c[o->field] = clock; open_p[o->field] = postacc; }
            } else if (--depth[o->field] == 0) {
                double v = clock - open_c[o->field] + (o->field == F_POST ? postacc - open_p[o->field] : 0);
                set_field(G, o->field, get_field(G, o->field) + v);
            }
            break;
        case OP_REP: rep = o->idx < s->ntimes ? o->idx : 0; break;
        case OP_MARK: reg_c[o->idx] = clock; reg_p[o->idx] = postacc; break;
        case OP_ZERO: set_field(tg, o->field, 0); break;
        case OP_DELTA: {
            double v = clock - reg_c[o->idx] + (o->field == F_POST ? postacc - reg_p[o->idx] : 0);
            set_field(tg, o->field, (o->idx2 ? get_field(tg, o->field) : 0) + v);
            break;
        }
        case OP_ACC: set_field(tg, o->field, get_field(tg, o->field) + get_field(src, o->idx2)); break;
        case OP_COPYT: set_field(tg, o->field, get_field(src, o->idx2)); break;
        default: break;
        }
    }
    return 0;
}

int xg_sched_rank_timer(xg_sched *s, int ngpus, int rank, const double *step_done,
                        const double *step_post, xg_timer *out)
{
    return rank_timers(s, ngpus, rank, step_done, step_post, out, NULL);
}

int xg_sched_rank_rep_timers(xg_sched *s, int ngpus, int rank, const double *step_done,
                             const double *step_post, xg_timer *reps)
{
    xg_timer g;
    return rank_timers(s, ngpus, rank, step_done, step_post, &g, reps);
}

/* Which step completion times any rank's Timer reads (rank_timers): a rank's logical clock is the
 * completion time of the latest step among those it has awaited, and step times never decrease
 * in step order (one stream per GPU), so the clock is step_done[c] for c = the highest awaited
 * step so far; a bracket (TMARK, MARK, DELTA) reads it there.  need[c] = 1 for every such c, and
 * for the last step (a run's total); 0 elsewhere.  A step whose time nobody reads needs no mark
 * in the run: reporting it as the next read step's time changes no Timer field. */
int xg_sched_timed_steps(const xg_sched *s, uint8_t *need)
{
    int r, i, q, n = 0;
    if (!s || !need) return -1;
    memset(need, 0, (size_t)s->nsteps);
    for (r = 0; r < s->P; ++r) {
        const prog_t *p = &s->progs[r];
        int c = -1;
        for (i = 0; i < p->nops; ++i) {
            const op_t *o = &p->ops[i];
            int st = -1;
            switch (o->kind) {
            case OP_WAIT:
                for (q = 0; q < o->wcnt; ++q) {
                    const int post = p->pool[o->wbeg + q];
                    if (s->post_eager[r][post]) continue;
                    st = s->msgs[s->post_msg[r][post]].step;
                    if (st > c) c = st;
                }
                break;
            case OP_BARRIER:
                st = s->barrier_epoch[o->post];
                if (st > c) c = st;
                break;
            case OP_SYNC:
                if (o->idx >= 0 && o->idx < s->nsteps && o->idx > c) c = o->idx;
                break;
            case OP_TMARK:
            case OP_MARK:
            case OP_DELTA:
                if (c >= 0) need[c] = 1;
                break;
            default: break;
            }
        }
    }
    if (s->nsteps > 0) need[s->nsteps - 1] = 1;
    for (i = 0; i < s->nsteps; ++i) n += need[i];
    return n;
}

int xg_sched_ntimes(const xg_sched *s) { return s->ntimes; }

int xg_sched_barrier_epochs(const xg_sched *s, int32_t *out)
{
    if (out && s->nbarrier) memcpy(out, s->barrier_epoch, sizeof(int32_t) * s->nbarrier);
    return s->nbarrier;
}

/* ------------------------------------------------------------------ block mapping / layout */
void xg_block_range(int procs, int ngpus, int g, int *lo, int *hi)
{
    int rpg = (procs + ngpus - 1) / ngpus;
    *lo = g * rpg < procs ? g * rpg : procs;
    *hi = *lo + rpg < procs ? *lo + rpg : procs;
}

int xg_gpu_of(int procs, int ngpus, int rank)
{
    int rpg = (procs + ngpus - 1) / ngpus;
    return rank / rpg;
}

int xgi_nsend_segs(const xg_sched *s, int r)
{
    return s->dir == XG_A2M ? s->A : (s->isagg[r] ? s->P : 0);
}

int xgi_nrecv_slots(const xg_sched *s, int r)
{
    return s->dir == XG_A2M ? (s->isagg[r] ? s->P : 0) : s->A;
}

static int64_t rank_offset(const xg_sched *s, int ngpus, int rank, int recv)
{
    int lo, hi, g = xg_gpu_of(s->P, ngpus, rank);
    int per_rank = recv ? xgi_nrecv_slots(s, rank) : xgi_nsend_segs(s, rank);
    xg_block_range(s->P, ngpus, g, &lo, &hi);
    if (!per_rank) return -1;
    /* ranks with a buffer of this kind on the GPU are laid out rank-major */
    if ((s->dir == XG_A2M) == (recv != 0))
        return (int64_t)(s->agg_prefix[rank] - s->agg_prefix[lo]) * s->P * s->d;   /* aggregator buffers */
    return (int64_t)(rank - lo) * s->A * s->d;                                      /* every-rank buffers */
}

int64_t xg_send_offset(const xg_sched *s, int ngpus, int rank) { return rank_offset(s, ngpus, rank, 0); }
int64_t xg_recv_offset(const xg_sched *s, int ngpus, int rank) { return rank_offset(s, ngpus, rank, 1); }

int64_t xg_scratch_offset(const xg_sched *s, int ngpus, int rank)
{
    int lo, hi, r;
    int64_t o = 0;
    xg_block_range(s->P, ngpus, xg_gpu_of(s->P, ngpus, rank), &lo, &hi);
    if (!s->scr_size[rank]) return -1;
    for (r = lo; r < rank; ++r) o += s->scr_size[r];
    return o;
}

int64_t xg_region_bytes(const xg_sched *s, int ngpus, int g, int buf)
{
    int lo, hi, naggs;
    xg_block_range(s->P, ngpus, g, &lo, &hi);
    naggs = s->agg_prefix[hi] - s->agg_prefix[lo];
    if (buf == XG_BUF_SEND)
        return s->dir == XG_A2M ? (int64_t)(hi - lo) * s->A * s->d : (int64_t)naggs * s->P * s->d;
    if (buf == XG_BUF_RECV)
        return s->dir == XG_A2M ? (int64_t)naggs * s->P * s->d : (int64_t)(hi - lo) * s->A * s->d;
    if (buf == XG_BUF_SCRATCH) {
        int64_t t = 0;
        int r;
        for (r = lo; r < hi; ++r) t += s->scr_size[r];
        return t;
    }
    return 0;
}

