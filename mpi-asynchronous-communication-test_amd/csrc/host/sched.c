/*
 * sched.c -- per-rank program restatement of methods 1..20, MPI matching, and
 * the step compiler that turns the reference's per-process MPI schedules into
 * device-wide steps.  Plain C99, no HIP.  See include/xg_sched.h.
 *
 * Each method builder below follows the reference function line by line
 * (cited per function); the only translation is that an MPI call becomes an
 * op appended to the logical rank's program:
 *   Irecv/Issend  -> OP_RECV/OP_SEND post      Waitall -> OP_WAIT
 *   Send/Recv     -> post + OP_WAIT             Sendrecv -> 2 posts + OP_WAIT
 *   Alltoallw     -> OP_A2AW + collective posts + OP_WAIT
 *   memcpy (self) -> OP_COPY                    MPI_Wtime brackets -> OP_TMARK
 * Messages and copies name a logical buffer of their rank (LB_*): the method's
 * send segments / receive slots, or TAM's aggregation buffers, which live in
 * the SCRATCH region; TAM's MPI_INT size arrays are LB_CTRL (host data).
 */
#include "xg_sched.h"

#include <limits.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

enum { OP_BARRIER, OP_SEND, OP_RECV, OP_WAIT, OP_A2AW, OP_COPY, OP_TMARK,
       OP_REP, OP_MARK, OP_DELTA, OP_ACC, OP_COPYT, OP_ZERO, OP_SYNC };
/* timer fields in xg_timer order */
enum { F_POST = 0, F_SEND = 1, F_RECV = 2, F_BARRIER = 3, F_TOTAL = 4, NF = 5 };
/* logical buffers of a rank: send segments, receive slots, TAM's aggregate_buf /
 * send_buf2 / recv_buf (lustre_driver_test.c:1054-1068, :1116, :1150), size arrays */
enum { LB_SEND = 0, LB_RECV = 1, LB_AGG = 2, LB_SBUF2 = 3, LB_RBUF = 4, LB_CTRL = 5, NLB = 6 };
#define NSCR 3                  /* LB_AGG .. LB_RBUF live in SCRATCH */
/* per-repetition timer DSL (m13's timers[m], mpi_test.c:829-874): targets and registers */
enum { TG_G = 0, TG_R = 1 };
enum { REG_S = 0, REG_T2 = 1, NREG = 2 };

typedef struct {
    int8_t kind, eager_ok, field, sign;   /* eager_ok: Send / Sendrecv / Isend (not Issend)  */
    int8_t isend, comm, tgt, tgt2;        /* comm 0 = MPI_COMM_WORLD; tgt*: timer DSL        */
    int32_t coll;           /* -1: point-to-point; k: the rank's k-th Alltoallw */
    int32_t peer;
    int32_t tag;            /* matching tag (reference: rank + peer on WORLD)     */
    int32_t idx;            /* send: segment; recv: slot; copy: segment; DSL: rep / reg */
    int32_t idx2;           /* copy: slot; DSL: source field / mode               */
    int32_t post;           /* send/recv: post index; copy: message index; barrier: ordinal */
    int32_t wbeg, wcnt;     /* wait: range in the rank's pool                 */
    int64_t cnt;            /* elements (bytes unless esz > 1)                */
    int8_t sb, db, esz;     /* logical buffers (LB_*) of source / destination */
    int64_t off, off2;      /* byte offsets in sb / db when idx < 0 (TAM)     */
} op_t;

typedef struct {
    op_t *ops;
    int nops, cap;
    int32_t *pool;
    int npool, poolcap;
    int nposts, ncoll, nbarrier, rank;
    int64_t hi[NLB];        /* extent of every logical buffer the program touches */
} prog_t;

struct xg_sched {
    int method, P, A, ntimes, dir, c, proc_node, barrier_type;
    int nbarrier;                /* barriers per rank (same for every rank)          */
    int32_t *barrier_epoch;      /* step after which barrier k has completed (-1: none) */
    int64_t d, eager;
    int *rank_list;
    int *isagg, *agg_prefix;     /* agg_prefix[r] = number of aggregator ranks < r */
    prog_t *progs;
    xg_msg *msgs;
    int nmsg, msgcap;
    int32_t *msg_spost, *msg_rpost;
    int32_t **post_msg;          /* [rank][post] -> message */
    uint8_t **post_eager;        /* [rank][post] -> blocking send <= eager limit   */
    int nsteps;
    int pc_ngpus;                /* posts per (gpu, step), cached for one ngpus    */
    int32_t *post_count;
    int iter;                    /* TAM tags carry +100*iter                        */
    int64_t *scr_base;           /* [rank][NSCR] offset of AGG/SBUF2/RBUF in the rank's scratch */
    int64_t *scr_size;           /* [rank] scratch bytes                            */
};

/* ------------------------------------------------------------------ helpers */
static void *xmalloc(size_t n)
{
    void *p = malloc(n ? n : 1);
    if (!p) { fprintf(stderr, "xg_sched: out of host memory (%zu bytes)\n", n); abort(); }
    return p;
}

static op_t *push(prog_t *p)
{
    if (p->nops == p->cap) {
        p->cap = p->cap ? 2 * p->cap : 64;
        p->ops = (op_t *)realloc(p->ops, sizeof(op_t) * p->cap);
        if (!p->ops) abort();
    }
    op_t *o = &p->ops[p->nops++];
    memset(o, 0, sizeof *o);
    o->coll = -1;
    o->sb = LB_SEND; o->db = LB_RECV; o->esz = 1;
    return o;
}

/* send post; tag < 0 means the reference's rank + peer on MPI_COMM_WORLD */
static int post_send_ex(prog_t *p, int peer, int64_t cnt, int seg, int eager_ok, int isend, int comm, int tag)
{
    op_t *o = push(p);
    o->kind = OP_SEND; o->peer = peer; o->cnt = cnt; o->idx = seg;
    o->eager_ok = (int8_t)(eager_ok || isend); o->isend = (int8_t)isend; o->comm = (int8_t)comm;
    o->tag = tag >= 0 ? tag : p->rank + peer;
    o->post = p->nposts++;
    return o->post;
}

static int post_recv_ex(prog_t *p, int peer, int64_t cnt, int slot, int comm, int tag)
{
    op_t *o = push(p);
    o->kind = OP_RECV; o->peer = peer; o->cnt = cnt; o->idx = slot; o->comm = (int8_t)comm;
    o->tag = tag >= 0 ? tag : p->rank + peer;
    o->post = p->nposts++;
    return o->post;
}

static int post_send(prog_t *p, int peer, int64_t cnt, int seg, int blocking)
{
    return post_send_ex(p, peer, cnt, seg, blocking, 0, 0, -1);
}

static int post_recv(prog_t *p, int peer, int64_t cnt, int slot) { return post_recv_ex(p, peer, cnt, slot, 0, -1); }

static void barrier(prog_t *p)
{
    op_t *o = push(p);
    o->kind = OP_BARRIER;
    o->post = p->nbarrier++;
}

/* timer DSL (m13) */
static void t_rep(prog_t *p, int m) { op_t *o = push(p); o->kind = OP_REP; o->idx = m; }
static void t_mark(prog_t *p, int reg) { op_t *o = push(p); o->kind = OP_MARK; o->idx = reg; }
static void t_zero(prog_t *p, int tgt, int f) { op_t *o = push(p); o->kind = OP_ZERO; o->tgt = (int8_t)tgt; o->field = (int8_t)f; }
/* tgt.f (=|+=) clock - reg */
static void t_delta(prog_t *p, int tgt, int f, int reg, int add)
{
    op_t *o = push(p);
    o->kind = OP_DELTA; o->tgt = (int8_t)tgt; o->field = (int8_t)f; o->idx = reg; o->idx2 = add;
}
/* tgt.f += tgt2.f2  (kind OP_ACC) or  tgt.f = tgt2.f2 (OP_COPYT) */
static void t_acc(prog_t *p, int kind, int tgt, int f, int tgt2, int f2)
{
    op_t *o = push(p);
    o->kind = (int8_t)kind; o->tgt = (int8_t)tgt; o->field = (int8_t)f; o->tgt2 = (int8_t)tgt2; o->idx2 = f2;
}

static void wait_list(prog_t *p, const int *idx, int n)
{
    op_t *o;
    if (p->npool + n > p->poolcap) {
        while (p->npool + n > p->poolcap) p->poolcap = p->poolcap ? 2 * p->poolcap : 256;
        p->pool = (int32_t *)realloc(p->pool, sizeof(int32_t) * p->poolcap);
        if (!p->pool) abort();
    }
    o = push(p);
    o->kind = OP_WAIT; o->wbeg = p->npool; o->wcnt = n;
    if (n) memcpy(p->pool + p->npool, idx, sizeof(int) * n);
    p->npool += n;
}

static void wait1(prog_t *p, int a) { wait_list(p, &a, 1); }

static void send_blocking(prog_t *p, int peer, int64_t cnt, int seg) { wait1(p, post_send(p, peer, cnt, seg, 1)); }
static void recv_blocking(prog_t *p, int peer, int64_t cnt, int slot) { wait1(p, post_recv(p, peer, cnt, slot)); }

static void sendrecv(prog_t *p, int dst, int64_t scnt, int seg, int src, int64_t rcnt, int slot)
{
    int ab[2];
    ab[0] = post_send(p, dst, scnt, seg, 1);
    ab[1] = post_recv(p, src, rcnt, slot);
    wait_list(p, ab, 2);
}

static void tmark(prog_t *p, int field, int sign)
{
    op_t *o = push(p);
    o->kind = OP_TMARK; o->field = (int8_t)field; o->sign = (int8_t)sign;
}

static void tstart(prog_t *p, int f) { tmark(p, f, +1); }
static void tstop(prog_t *p, int f) { tmark(p, f, -1); }

static void copy_op(prog_t *p, int seg, int slot, int64_t cnt)
{
    op_t *o = push(p);
    o->kind = OP_COPY; o->idx = seg; o->idx2 = slot; o->cnt = cnt; o->post = -1;
}

static void extent(prog_t *p, int lb, int64_t end)
{
    if (end > p->hi[lb]) p->hi[lb] = end;
}

/* TAM point-to-point on (logical buffer, byte offset); cnt elements of esz bytes */
static int buf_send(prog_t *p, int peer, int64_t cnt, int esz, int lb, int64_t off, int tag, int isend)
{
    int q = post_send_ex(p, peer, cnt, -1, 0, isend, 0, tag);
    op_t *o = &p->ops[p->nops - 1];
    o->sb = (int8_t)lb; o->off = off; o->esz = (int8_t)esz;
    extent(p, lb, off + cnt * esz);
    return q;
}

static int buf_recv(prog_t *p, int peer, int64_t cnt, int esz, int lb, int64_t off, int tag)
{
    int q = post_recv_ex(p, peer, cnt, -1, 0, tag);
    op_t *o = &p->ops[p->nops - 1];
    o->db = (int8_t)lb; o->off2 = off; o->esz = (int8_t)esz;
    extent(p, lb, off + cnt * esz);
    return q;
}

/* memcpy inside one rank: n bytes from (sb, soff) to (db, doff) */
static void buf_copy(prog_t *p, int sb, int64_t soff, int db, int64_t doff, int64_t n)
{
    op_t *o = push(p);
    o->kind = OP_COPY; o->idx = o->idx2 = -1; o->cnt = n; o->post = -1;
    o->sb = (int8_t)sb; o->off = soff; o->db = (int8_t)db; o->off2 = doff;
    extent(p, sb, soff + n);
    extent(p, db, doff + n);
}

/* growable int list for request indices */
typedef struct { int *v; int n, cap; } ilist;
static void il_push(ilist *l, int x)
{
    if (l->n == l->cap) { l->cap = l->cap ? 2 * l->cap : 64; l->v = (int *)realloc(l->v, sizeof(int) * l->cap); if (!l->v) abort(); }
    l->v[l->n++] = x;
}

typedef struct {
    prog_t *p;
    int rank, isagg, myindex, P, A, c, ntimes, proc_node, barrier_type;
    int64_t d;
    const int *rl;
    int method, iter;
    const int *isagg_all;   /* [P] */
    const int *lastidx;     /* [P] last i with rl[i] == rank, -1 if none */
} ctx_t;

/* ------------------------------------------------------------------ methods */

/* all_to_many, mpi_test.c:1748-1824 */
static void m1_all_to_many(ctx_t *x)
{
    prog_t *p = x->p;
    int m, i, k, P = x->P, A = x->A;
    ilist l = {0};
    for (m = 0; m < x->ntimes; ++m) {
        if (x->c >= P) {                                    /* :1765-1784 */
            l.n = 0;
            tstart(p, F_POST);
            if (x->isagg)
                for (i = 0; i < P; ++i) il_push(&l, post_recv(p, i, x->d, i));
            for (i = 0; i < A; ++i) il_push(&l, post_send(p, x->rl[i], x->d, i, 0));
            tstop(p, F_POST);
            if (l.n) { tstart(p, F_RECV); wait_list(p, l.v, l.n); tstop(p, F_RECV); }
        } else {                                            /* :1785-1817 */
            int steps = (P + x->c - 1) / x->c;
            ilist sends = {0};
            tstart(p, F_POST);
            for (i = 0; i < A; ++i) il_push(&sends, post_send(p, x->rl[i], x->d, i, 0));
            tstop(p, F_POST);
            for (k = 0; k < steps; ++k) {
                l.n = 0;
                if (x->isagg) {
                    tstart(p, F_POST);
                    for (i = k; i < P; i += steps) il_push(&l, post_recv(p, i, x->d, i));
                    tstop(p, F_POST);
                }
                if (l.n) { tstart(p, F_RECV); wait_list(p, l.v, l.n); tstop(p, F_RECV); }
            }
            if (sends.n) { tstart(p, F_SEND); wait_list(p, sends.v, sends.n); tstop(p, F_SEND); }
            free(sends.v);
        }
    }
    free(l.v);
}

/* many_to_all, mpi_test.c:1871-1950 */
static void m2_many_to_all(ctx_t *x)
{
    prog_t *p = x->p;
    int m, i, k, P = x->P, A = x->A;
    ilist l = {0};
    for (m = 0; m < x->ntimes; ++m) {
        if (x->c >= P) {                                    /* :1889-1906 */
            l.n = 0;
            tstart(p, F_POST);
            for (i = 0; i < A; ++i) il_push(&l, post_recv(p, x->rl[i], x->d, i));
            if (x->isagg)
                for (i = 0; i < P; ++i) il_push(&l, post_send(p, i, x->d, i, 0));
            tstop(p, F_POST);
            if (l.n) { tstart(p, F_RECV); wait_list(p, l.v, l.n); tstop(p, F_RECV); }
        } else {                                            /* :1907-1943 */
            int steps = (P + x->c - 1) / x->c;
            ilist recvs = {0};
            tstart(p, F_POST);
            for (i = 0; i < A; ++i) il_push(&recvs, post_recv(p, x->rl[i], x->d, i));
            tstop(p, F_POST);
            for (k = 0; k < steps; ++k) {
                l.n = 0;
                if (x->isagg) {
                    tstart(p, F_POST);
                    for (i = k; i < P; i += steps) il_push(&l, post_send(p, i, x->d, i, 0));
                    tstop(p, F_POST);
                }
                if (l.n) { tstart(p, F_SEND); wait_list(p, l.v, l.n); tstop(p, F_SEND); }
            }
            if (recvs.n) { tstart(p, F_RECV); wait_list(p, recvs.v, recvs.n); tstop(p, F_RECV); }
            free(recvs.v);
        }
    }
    free(l.v);
}

/* window start of aggregator index idx in round k (mpi_test.c:1463-1467, :1478-1482) */
static long win_start(int idx, long k, int ceiling, int floor_, int remainder)
{
    return idx < remainder ? k + (long)idx * ceiling
                           : k + (long)remainder * ceiling + (long)(idx - remainder) * floor_;
}

/* window membership test, mpi_test.c:1483-1499 (= :1617-1633), edge cases included */
static int in_window(int rank, long temp, int cs, int P)
{
    if ((temp >= P && temp + cs >= P) || (temp < P && temp + cs < P))
        return rank >= temp % P && rank < (temp + cs) % P;
    return rank >= temp || rank < (temp + cs) % P;
}

static int send_start0(int rank, int ceiling, int floor_, int remainder)   /* :1449-1453 */
{
    if (rank >= remainder * ceiling) return remainder + (rank - remainder * ceiling) / floor_;
    return rank / ceiling;
}

/* all_to_many_balanced, mpi_test.c:1422-1517 */
static void m3_balanced(ctx_t *x)
{
    prog_t *p = x->p;
    int P = x->P, A = x->A, c = x->c, m, i, cs, k, xx;
    int ceiling = (P + A - 1) / A, floor_ = P / A, remainder = P % A;
    int bblock, send_start;
    ilist l = {0};
    if (c > P) c = P;
    bblock = c;
    send_start = send_start0(x->rank, ceiling, floor_, remainder);
    for (m = 0; m < x->ntimes; ++m) {
        cs = bblock;                                         /* :1455 reset */
        for (k = 0; k < P; k += cs) {
            if (P - k < cs) cs = P - k;
            l.n = 0;
            if (x->isagg) {
                for (i = 0; i < cs; ++i) {
                    int temp = (int)(win_start(x->myindex, (long)k + i, ceiling, floor_, remainder) % P);
                    if (temp != x->rank) {
                        tstart(p, F_POST);
                        il_push(&l, post_recv(p, temp, x->d, temp));
                        tstop(p, F_POST);
                    } else {
                        copy_op(p, x->myindex, temp, x->d);          /* :1473 */
                    }
                }
            }
            for (xx = 0; xx < A; ++xx) {
                long temp = win_start(send_start, k, ceiling, floor_, remainder);
                if (!in_window(x->rank, temp, cs, P)) break;
                if (x->rl[send_start] != x->rank)
                    il_push(&l, post_send(p, x->rl[send_start], x->d, send_start, 0));
                send_start = (send_start - 1 + A) % A;
            }
            if (l.n) {
                tstart(p, F_RECV);
                if (!x->isagg) tstart(p, F_SEND);
                wait_list(p, l.v, l.n);
                tstop(p, F_RECV);
                if (!x->isagg) tstop(p, F_SEND);
            }
        }
    }
    free(l.v);
}

/* many_to_all_balanced, mpi_test.c:1576-1663 (comm_size NOT reset between repetitions) */
static void m4_balanced(ctx_t *x)
{
    prog_t *p = x->p;
    int P = x->P, A = x->A, m, i, k, xx;
    int ceiling = (P + A - 1) / A, floor_ = P / A, remainder = P % A;
    int cs = x->c > P ? P : x->c;
    int send_start = send_start0(x->rank, ceiling, floor_, remainder);
    ilist l = {0};
    for (m = 0; m < x->ntimes; ++m) {
        for (k = 0; k < P; k += cs) {
            if (P - k < cs) cs = P - k;
            l.n = 0;
            tstart(p, F_POST);
            for (xx = 0; xx < A; ++xx) {
                long temp = win_start(send_start, k, ceiling, floor_, remainder);
                if (!in_window(x->rank, temp, cs, P)) break;
                if (x->rl[send_start] != x->rank)
                    il_push(&l, post_recv(p, x->rl[send_start], x->d, send_start));
                send_start = (send_start - 1 + A) % A;
            }
            if (x->isagg) {
                for (i = 0; i < cs; ++i) {
                    int temp = (int)(win_start(x->myindex, (long)k + i, ceiling, floor_, remainder) % P);
                    if (temp != x->rank)
                        il_push(&l, post_send(p, temp, x->d, temp, 0));
                    else
                        copy_op(p, temp, x->myindex, x->d);          /* :1646 */
                }
            }
            tstop(p, F_POST);
            if (l.n) { tstart(p, F_RECV); wait_list(p, l.v, l.n); tstop(p, F_RECV); }
        }
    }
    free(l.v);
}

/* *_alltoall_translate, mpi_test.c:233-262 (a2m) and :273-302 (m2a) */
static void translate(ctx_t *x, int dir, int64_t *sc, int64_t *sd, int64_t *rc, int64_t *rd)
{
    int i, P = x->P, A = x->A;
    int64_t d = x->d;
    memset(sc, 0, sizeof(int64_t) * P); memset(sd, 0, sizeof(int64_t) * P);
    memset(rc, 0, sizeof(int64_t) * P); memset(rd, 0, sizeof(int64_t) * P);
    if (dir == XG_A2M) {
        for (i = 0; i < A; ++i) { sd[x->rl[i]] = (int64_t)i * d; sc[x->rl[i]] = d; }
        if (x->isagg)
            for (i = 0; i < P; ++i) { rc[i] = d; rd[i] = (int64_t)i * d; }
    } else {
        rd[x->rl[0]] = 0; rc[x->rl[0]] = d;
        for (i = 1; i < A; ++i) { rd[x->rl[i]] = rd[x->rl[i - 1]] + d; rc[x->rl[i]] = d; }
        if (x->isagg)
            for (i = 0; i < P; ++i) { sc[i] = d; sd[i] = (int64_t)i * d; }
    }
}

/* many_to_all_benchmark :599-654 / all_to_many_benchmark :885-940 (MPI_Alltoallw) */
static void m_alltoallw(ctx_t *x, int dir)
{
    prog_t *p = x->p;
    int P = x->P, m, q;
    int64_t *sc = xmalloc(sizeof(int64_t) * 4 * P), *sd = sc + P, *rc = sc + 2 * P, *rd = sc + 3 * P;
    ilist l = {0};
    translate(x, dir, sc, sd, rc, rd);
    for (m = 0; m < x->ntimes; ++m) {
        op_t *a;
        int coll = p->ncoll++;
        a = push(p); a->kind = OP_A2AW; a->coll = coll;
        l.n = 0;
        for (q = 0; q < P; ++q)
            if (sc[q] > 0) { int id = post_send(p, q, sc[q], (int)(sd[q] / x->d), 0); p->ops[p->nops - 1].coll = coll; il_push(&l, id); }
        for (q = 0; q < P; ++q)
            if (rc[q] > 0) { int id = post_recv(p, q, rc[q], (int)(rd[q] / x->d)); p->ops[p->nops - 1].coll = coll; il_push(&l, id); }
        wait_list(p, l.v, l.n);
        p->ops[p->nops - 1].coll = coll;
    }
    free(l.v);
    free(sc);
}

/* all_to_many_sync, mpi_test.c:1665-1746 */
static void m6_sync(ctx_t *x)
{
    prog_t *p = x->p;
    int P = x->P, A = x->A, m, i, k, xx;
    int cs = x->c > A ? A : x->c;
    for (m = 0; m < x->ntimes; ++m) {
        for (k = 0; k < A; k += cs) {
            if (A - k < cs) cs = A - k;
            tstart(p, F_RECV);
            if (x->isagg) {
                for (i = 0; i < cs; ++i) {
                    int temp = (x->rank + k + i) % A;
                    int temp2 = (x->myindex - k - i + A) % A;
                    if (x->rl[temp] != x->rank && temp2 != x->rank) {
                        sendrecv(p, x->rl[temp], x->d, temp, temp2, x->d, temp2);
                    } else if (x->rl[temp] == x->rank) {
                        copy_op(p, temp, x->rank, x->d);             /* :1714 */
                        if (temp2 != x->rank) recv_blocking(p, temp2, x->d, temp2);
                    } else if (temp2 == x->rank) {
                        send_blocking(p, x->rl[temp], x->d, temp);
                    }
                    for (xx = temp2 + A; xx < P; xx += A)
                        if (x->rank != xx) recv_blocking(p, xx, x->d, xx);
                }
            } else {
                for (i = 0; i < cs; ++i) {
                    int temp = (x->rank + k + i) % A;
                    send_blocking(p, x->rl[temp], x->d, temp);
                }
            }
            tstop(p, F_RECV);
        }
    }
}

/* all_to_many_half_sync, mpi_test.c:1055-1114 */
static void m7_half_sync(ctx_t *x)
{
    prog_t *p = x->p;
    int P = x->P, A = x->A, m, i, k, xx;
    int cs = x->c > A ? A : x->c;
    ilist l = {0};
    for (m = 0; m < x->ntimes; ++m) {
        for (k = 0; k < A; k += cs) {
            if (A - k < cs) cs = A - k;
            l.n = 0;
            if (x->isagg)
                for (i = 0; i < cs; ++i)
                    for (xx = (x->myindex - k - i + A) % A; xx < P; xx += A)
                        il_push(&l, post_recv(p, xx, x->d, xx));
            for (i = 0; i < cs; ++i) {
                int temp = (x->rank + k + i) % A;
                send_blocking(p, x->rl[temp], x->d, temp);
            }
            tstart(p, F_RECV);
            if (l.n) wait_list(p, l.v, l.n);
            tstop(p, F_RECV);
        }
    }
    free(l.v);
}

/* many_to_all_half_sync, mpi_test.c:942-997 */
static void m11_half_sync(ctx_t *x)
{
    prog_t *p = x->p;
    int P = x->P, A = x->A, m, i, k, xx;
    int cs = x->c > P ? P : x->c;
    int stride = (P + A - 1) / A;
    ilist l = {0};
    for (m = 0; m < x->ntimes; ++m) {
        for (k = 0; k < P; k += cs) {
            if (P - k < cs) cs = P - k;
            l.n = 0;
            tstart(p, F_POST);
            if (x->isagg)
                for (i = 0; i < cs; ++i) {
                    int temp = (int)(((long)stride * x->myindex + k + i) % P);
                    il_push(&l, post_send(p, temp, x->d, temp, 0));
                }
            tstop(p, F_POST);
            tstart(p, F_RECV);
            for (xx = 0; xx < cs; ++xx)
                for (i = 0; i < A; ++i)
                    if (x->rank == (int)(((long)k + (long)i * stride + xx) % P))
                        recv_blocking(p, x->rl[i], x->d, i);
            if (l.n) wait_list(p, l.v, l.n);
            tstop(p, F_RECV);
        }
    }
    free(l.v);
}

/* all_to_many_half_sync2, mpi_test.c:999-1053 */
static void m12_half_sync2(ctx_t *x)
{
    prog_t *p = x->p;
    int P = x->P, A = x->A, m, i, k, xx;
    int cs = x->c > A ? A : x->c;
    ilist l = {0};
    for (m = 0; m < x->ntimes; ++m) {
        for (k = 0; k < A; k += cs) {
            if (A - k < cs) cs = A - k;
            l.n = 0;
            for (i = 0; i < cs; ++i) {
                int temp = (x->rank + k + i) % A;
                il_push(&l, post_send(p, x->rl[temp], x->d, temp, 0));
            }
            if (x->isagg)
                for (i = 0; i < cs; ++i)
                    for (xx = (x->myindex - k - i + A) % A; xx < P; xx += A)
                        recv_blocking(p, xx, x->d, xx);
            tstart(p, F_RECV);
            if (l.n) wait_list(p, l.v, l.n);
            tstop(p, F_RECV);
        }
    }
    free(l.v);
}

/* many_to_all_pairwise :421-508 / all_to_many_pairwise :510-597 */
/* "this rank has completed step k": its later posts move no earlier than k + 1, and its
 * clock reaches step k's completion (the pairwise fast form's stand-in for the 0-byte
 * MPI_Sendrecv rounds it leaves out) */
static void sync_step(prog_t *p, int k) { op_t *o = push(p); o->kind = OP_SYNC; o->idx = k; }

/* Large P: every rank makes P blocking MPI_Sendrecv calls per repetition, most of them
 * 0 bytes -- P^2 calls to materialise (268 M at P = 16384).  They keep every rank in
 * lockstep, so round i of repetition m is step m*P + i for every message; the fast form
 * posts only the directions that carry bytes, each behind a sync to the round before, and
 * ends with a sync to the last round (tests/test_host_sched.py checks it against the full
 * form: same messages, steps and rank timers).  XG_PAIRWISE_FAST=0/1 forces either form. */
static int pairwise_fast(int P)
{
    const char *e = getenv("XG_PAIRWISE_FAST");
    return e ? atoi(e) != 0 : P > 1024;
}

static void m_pairwise(ctx_t *x, int dir)
{
    prog_t *p = x->p;
    int P = x->P, m, i, pof2, src, dst;
    const int fast = pairwise_fast(P);
    int64_t *sc = xmalloc(sizeof(int64_t) * 4 * P), *sd = sc + P, *rc = sc + 2 * P, *rd = sc + 3 * P;
    translate(x, dir, sc, sd, rc, rd);
    i = 1;
    while (i < P) i *= 2;
    pof2 = i == P;
    for (m = 0; m < x->ntimes; ++m) {
        for (i = 0; i < P; ++i) {
            if (pof2) src = dst = x->rank ^ i;
            else { src = (x->rank - i + P) % P; dst = (x->rank + i) % P; }
            if (!fast) {
                sendrecv(p, dst, sc[dst], sc[dst] ? (int)(sd[dst] / x->d) : -1,
                         src, rc[src], rc[src] ? (int)(rd[src] / x->d) : -1);
                continue;
            }
            if (!sc[dst] && !rc[src]) continue;
            const int k = m * P + i;
            if (k > 0) sync_step(p, k - 1);
            if (sc[dst] && rc[src]) {
                sendrecv(p, dst, sc[dst], (int)(sd[dst] / x->d), src, rc[src], (int)(rd[src] / x->d));
            } else if (sc[dst]) {
                wait1(p, post_send(p, dst, sc[dst], (int)(sd[dst] / x->d), 1));
            } else {
                wait1(p, post_recv(p, src, rc[src], (int)(rd[src] / x->d)));
            }
        }
    }
    if (fast && x->ntimes > 0) sync_step(p, x->ntimes * P - 1);
    free(sc);
}

static int scattered_block(int P, int c)    /* :674-684, :740-750, :815-825 */
{
    if (c > P) c = P;
    return c != 0 ? c : P;
}

static void wait_bracket(prog_t *p, const ilist *l, int isagg)   /* recv (+send for non-aggregators) */
{
    tstart(p, F_RECV);
    if (!isagg) tstart(p, F_SEND);
    wait_list(p, l->v, l->n);
    tstop(p, F_RECV);
    if (!isagg) tstop(p, F_SEND);
}

/* all_to_many_scattered, mpi_test.c:797-882 (barrier type -b, per-repetition timers[m]) */
static void m13_scattered(ctx_t *x)
{
    prog_t *p = x->p;
    int P = x->P, m, i, ii, dst;
    int64_t *sc = xmalloc(sizeof(int64_t) * 4 * P), *sd = sc + P, *rc = sc + 2 * P, *rd = sc + 3 * P;
    int bblock = scattered_block(P, x->c);
    ilist l = {0};
    translate(x, XG_A2M, sc, sd, rc, rd);
    for (m = 0; m < x->ntimes; ++m) {
        t_rep(p, m);
        t_mark(p, REG_T2);
        t_zero(p, TG_R, F_BARRIER);
        for (ii = 0; ii < P; ii += bblock) {
            int ss = P - ii < bblock ? P - ii : bblock;
            l.n = 0;
            t_mark(p, REG_S);
            for (i = 0; i < ss; ++i) {
                dst = (x->rank + i + ii) % P;
                if (rc[dst]) il_push(&l, post_recv(p, dst, rc[dst], (int)(rd[dst] / x->d)));
            }
            for (i = 0; i < ss; ++i) {
                dst = (x->rank - i - ii + P) % P;
                if (sc[dst]) il_push(&l, post_send(p, dst, sc[dst], (int)(sd[dst] / x->d), 0));
            }
            t_delta(p, TG_R, F_POST, REG_S, 0);
            t_acc(p, OP_ACC, TG_G, F_POST, TG_R, F_POST);
            if (l.n) {
                t_mark(p, REG_S);
                wait_list(p, l.v, l.n);
                t_delta(p, TG_R, F_RECV, REG_S, 0);
                t_acc(p, OP_ACC, TG_G, F_RECV, TG_R, F_RECV);
                if (!x->isagg) {
                    t_acc(p, OP_ACC, TG_G, F_SEND, TG_R, F_RECV);
                    t_acc(p, OP_COPYT, TG_R, F_SEND, TG_R, F_RECV);
                }
            }
            if (x->barrier_type == 2) {
                t_mark(p, REG_S);
                barrier(p);
                t_delta(p, TG_R, F_BARRIER, REG_S, 1);
                t_acc(p, OP_ACC, TG_G, F_BARRIER, TG_R, F_BARRIER);
            }
        }
        t_delta(p, TG_R, F_TOTAL, REG_T2, 0);
        if (x->barrier_type == 1) {
            t_mark(p, REG_S);
            barrier(p);
            t_delta(p, TG_R, F_BARRIER, REG_S, 0);
            t_acc(p, OP_ACC, TG_G, F_BARRIER, TG_R, F_BARRIER);
        }
    }
    free(l.v);
    free(sc);
}

/* many_to_all_scattered, mpi_test.c:656-720 */
static void m14_scattered(ctx_t *x)
{
    prog_t *p = x->p;
    int P = x->P, m, i, ii, dst;
    int64_t *sc = xmalloc(sizeof(int64_t) * 4 * P), *sd = sc + P, *rc = sc + 2 * P, *rd = sc + 3 * P;
    int bblock = scattered_block(P, x->c);
    ilist l = {0};
    translate(x, XG_M2A, sc, sd, rc, rd);
    for (m = 0; m < x->ntimes; ++m)
        for (ii = 0; ii < P; ii += bblock) {
            int ss = P - ii < bblock ? P - ii : bblock;
            l.n = 0;
            tstart(p, F_POST);
            for (i = 0; i < ss; ++i) {
                dst = (x->rank + i + ii) % P;
                if (rc[dst]) il_push(&l, post_recv(p, dst, rc[dst], (int)(rd[dst] / x->d)));
            }
            for (i = 0; i < ss; ++i) {
                dst = (x->rank - i - ii + P) % P;
                if (sc[dst]) il_push(&l, post_send(p, dst, sc[dst], (int)(sd[dst] / x->d), 0));
            }
            tstop(p, F_POST);
            if (l.n) { tstart(p, F_RECV); wait_list(p, l.v, l.n); tstop(p, F_RECV); }
        }
    free(l.v);
    free(sc);
}

/* node_robin_map, mpi_test.c:1116-1133 */
static void node_robin(int rank, int proc_node, int P, int *map, int *rank_index)
{
    int i, j = 0, count = 0;
    *rank_index = 0;
    for (i = 0; i < P; ++i) {
        map[i] = count;
        if (count == rank) *rank_index = i;
        count += proc_node;
        if (count >= P) { j++; count = j; }
    }
}

/* all_to_many_node_robin, mpi_test.c:1135-1227 (a barrier inside every round) */
static void m17_node_robin(ctx_t *x)
{
    prog_t *p = x->p;
    int P = x->P, A = x->A, m, i, k, xx, cs, rank_index;
    int ceiling = (P + A - 1) / A, floor_ = P / A, remainder = P % A;
    int *map = (int *)xmalloc(sizeof(int) * P), bblock, send_start;
    ilist l = {0};
    node_robin(x->rank, x->proc_node, P, map, &rank_index);
    bblock = x->c > P ? P : x->c;
    send_start = send_start0(rank_index, ceiling, floor_, remainder);
    for (m = 0; m < x->ntimes; ++m) {
        cs = bblock;
        for (k = 0; k < P; k += cs) {
            if (P - k < cs) cs = P - k;
            l.n = 0;
            tstart(p, F_POST);
            if (x->isagg)
                for (i = 0; i < cs; ++i) {
                    int temp = map[win_start(x->myindex, (long)k + i, ceiling, floor_, remainder) % P];
                    il_push(&l, post_recv(p, temp, x->d, temp));
                }
            barrier(p);
            for (xx = 0; xx < A; ++xx) {
                long temp = win_start(send_start, k, ceiling, floor_, remainder);
                if (!in_window(rank_index, temp, cs, P)) break;
                il_push(&l, post_send(p, x->rl[send_start], x->d, send_start, 0));
                send_start = (send_start - 1 + A) % A;
            }
            tstop(p, F_POST);
            if (l.n) wait_bracket(p, &l, x->isagg);
        }
    }
    free(l.v);
    free(map);
}

/* all_to_many_balanced_control, mpi_test.c:1229-1336 (0-byte go-signals on a dup'd communicator) */
static void m18_balanced_control(ctx_t *x)
{
    prog_t *p = x->p;
    int P = x->P, A = x->A, m, i, k, xx, cs;
    int ceiling = (P + A - 1) / A, floor_ = P / A, remainder = P % A;
    int bblock = x->c > P ? P : x->c;
    int send_start = send_start0(x->rank, ceiling, floor_, remainder);
    ilist l = {0};
    for (m = 0; m < x->ntimes; ++m) {
        cs = bblock;
        for (k = 0; k < P; k += cs) {
            if (P - k < cs) cs = P - k;
            l.n = 0;
            tstart(p, F_POST);
            if (x->isagg)
                for (i = 0; i < cs; ++i) {
                    int temp = (int)(win_start(x->myindex, (long)k + i, ceiling, floor_, remainder) % P);
                    if (temp != x->rank) {
                        il_push(&l, post_recv(p, temp, x->d, temp));
                        il_push(&l, post_send_ex(p, temp, 0, -1, 1, 1, 1, x->rank + temp * 100));  /* :1283 */
                    } else {
                        copy_op(p, x->myindex, temp, x->d);                                       /* :1285 */
                    }
                }
            for (xx = 0; xx < A; ++xx) {
                long temp = win_start(send_start, k, ceiling, floor_, remainder);
                if (!in_window(x->rank, temp, cs, P)) break;
                if (x->rl[send_start] != x->rank) {
                    int peer = x->rl[send_start];
                    wait1(p, post_recv_ex(p, peer, 0, -1, 1, x->rank * 100 + peer));              /* :1299 */
                    il_push(&l, post_send(p, peer, x->d, send_start, 0));
                }
                send_start = (send_start - 1 + A) % A;
            }
            tstop(p, F_POST);
            if (l.n) wait_bracket(p, &l, x->isagg);
        }
    }
    free(l.v);
}

/* all_to_many_scattered_isend, mpi_test.c:722-795 (MPI_Isend; barrier before the total stop) */
static void m19_scattered_isend(ctx_t *x)
{
    prog_t *p = x->p;
    int P = x->P, m, i, ii, dst;
    int64_t *sc = xmalloc(sizeof(int64_t) * 4 * P), *sd = sc + P, *rc = sc + 2 * P, *rd = sc + 3 * P;
    int bblock = scattered_block(P, x->c);
    ilist l = {0};
    translate(x, XG_A2M, sc, sd, rc, rd);
    for (m = 0; m < x->ntimes; ++m)
        for (ii = 0; ii < P; ii += bblock) {
            int ss = P - ii < bblock ? P - ii : bblock;
            l.n = 0;
            for (i = 0; i < ss; ++i) {
                dst = (x->rank + i + ii) % P;
                if (rc[dst]) il_push(&l, post_recv(p, dst, rc[dst], (int)(rd[dst] / x->d)));
            }
            for (i = 0; i < ss; ++i) {
                dst = (x->rank - i - ii + P) % P;
                if (sc[dst]) {
                    if (!x->isagg) tstart(p, F_POST);
                    il_push(&l, post_send_ex(p, dst, sc[dst], (int)(sd[dst] / x->d), 1, 1, 0, -1));
                    if (!x->isagg) tstop(p, F_POST);
                }
            }
            if (l.n) wait_bracket(p, &l, x->isagg);
        }
    barrier(p);
    free(l.v);
    free(sc);
}

/* all_to_many_balanced_pre_send, mpi_test.c:1338-1419 */
static void m20_balanced_presend(ctx_t *x)
{
    prog_t *p = x->p;
    int P = x->P, A = x->A, m, i, k, cs;
    int ceiling = (P + A - 1) / A, floor_ = P / A, remainder = P % A;
    int bblock = x->c > P ? P : x->c;
    int send_start = send_start0(x->rank, ceiling, floor_, remainder);
    ilist l = {0}, sends = {0};
    for (m = 0; m < x->ntimes; ++m) {
        cs = bblock;
        sends.n = 0;
        for (k = 0; k < A; ++k) {
            i = (send_start - k + A) % A;
            if (x->rl[i] != x->rank) il_push(&sends, post_send(p, x->rl[i], x->d, i, 0));
        }
        for (k = 0; k < P; k += cs) {
            if (P - k < cs) cs = P - k;
            l.n = 0;
            if (x->isagg)
                for (i = 0; i < cs; ++i) {
                    int temp = (int)(win_start(x->myindex, (long)k + i, ceiling, floor_, remainder) % P);
                    if (temp != x->rank) {
                        tstart(p, F_POST);
                        il_push(&l, post_recv(p, temp, x->d, temp));
                        tstop(p, F_POST);
                    } else {
                        copy_op(p, x->myindex, temp, x->d);                                       /* :1398 */
                    }
                }
            if (l.n) { tstart(p, F_RECV); wait_list(p, l.v, l.n); tstop(p, F_RECV); }
        }
        if (sends.n) { tstart(p, F_SEND); wait_list(p, sends.v, sends.n); tstop(p, F_SEND); }
    }
    free(l.v);
    free(sends.v);
}

/* ------------------------------------------------------------------ TAM (m15 / m16) */
/* send_size[w] / recv_size[w] that all_to_many_tam / many_to_all_tam hand to
 * collective_write (mpi_test.c:393 / :343; counts of *_alltoall_translate) */
static int64_t tam_ss(const ctx_t *x, int r, int w)     /* bytes r sends to w */
{
    return x->method == 15 ? (x->isagg_all[w] ? x->d : 0) : (x->isagg_all[r] ? x->d : 0);
}

static int64_t tam_rs(const ctx_t *x, int r, int w)     /* bytes r receives from w */
{
    return x->method == 15 ? (x->isagg_all[r] ? x->d : 0) : (x->isagg_all[w] ? x->d : 0);
}

/* send_buf[w] / recv_buf[w] byte offsets: a2m send_buf2[rank_list[i]] = segment i
 * (:388-391), recv slot w; m2a send segment w, recv_buf2[rank_list[i]] = slot i (:335-339) */
static int64_t tam_sloc(const ctx_t *x, int w) { return (x->method == 15 ? x->lastidx[w] : w) * x->d; }
static int64_t tam_rloc(const ctx_t *x, int w) { return (x->method == 15 ? w : x->lastidx[w]) * x->d; }

/* collective_write, lustre_driver_test.c:944-1309, with static_node_assignment
 * type 0 (:404-427): nodes of proc_node consecutive ranks, proxy = first rank
 * of a node.  Tags are a + b + 100 * iter (:1006, :1012, :1094, ...). */
static void tam_collective_write(ctx_t *x)
{
    prog_t *p = x->p;
    const int P = x->P, pn = x->proc_node, rank = x->rank, it100 = 100 * x->iter;
    const int nrecvs = (P + pn - 1) / pn, lr0 = (rank / pn) * pn;
    const int npn = rank >= (nrecvs - 1) * pn ? P - pn * (nrecvs - 1) : pn;
    const int proxy = rank == lr0;
    int64_t total_send = 0, total_recv = 0, node_msg = 0, node_recv = 0, local = 0, off, ptr;
    int64_t *s_lens = NULL, *r_lens = NULL, *gsl = NULL, *grl = NULL, *ptrs = NULL;
    int i, w, v;
    ilist idx = {0};
    for (w = 0; w < P; ++w) { total_send += tam_ss(x, rank, w); total_recv += tam_rs(x, rank, w); }
    /* intra-node gather of the send/recv size arrays (:996-1018) */
    if (proxy)
        for (i = 1; i < npn; ++i)
            il_push(&idx, buf_recv(p, lr0 + i, 2 * P, 4, LB_CTRL, (int64_t)i * P * 8, lr0 + i + lr0 + it100));
    else
        il_push(&idx, buf_send(p, lr0, 2 * P, 4, LB_CTRL, 0, rank + lr0 + it100, 1));
    if (idx.n) { tstart(p, F_RECV); wait_list(p, idx.v, idx.n); tstop(p, F_RECV); }
    /* proxy: exclusive prefix sums over (local process i, target w) (:1027-1041) */
    if (proxy) {
        s_lens = (int64_t *)xmalloc(sizeof(int64_t) * npn * P);
        r_lens = (int64_t *)xmalloc(sizeof(int64_t) * npn * P);
        for (i = 0; i < npn; ++i)
            for (w = 0; w < P; ++w) {
                s_lens[i * P + w] = node_msg; node_msg += tam_ss(x, lr0 + i, w);
                r_lens[i * P + w] = node_recv; node_recv += tam_rs(x, lr0 + i, w);
            }
        local = node_msg > node_recv ? node_msg : node_recv;   /* local_buf = aggregate_buf + temp (:1054-1068) */
    }
    /* pack this process's messages into local_buf (:1069-1077) */
    off = 0;
    for (w = 0; w < P; ++w) {
        int64_t n = tam_ss(x, rank, w);
        if (n) { buf_copy(p, LB_SEND, tam_sloc(x, w), LB_AGG, local + off, n); off += n; }
    }
    /* messages to the local proxy (:1078-1107) */
    idx.n = 0;
    if (proxy) {
        if (total_send) buf_copy(p, LB_AGG, local, LB_AGG, 0, total_send);
        ptr = total_send;
        for (i = 1; i < npn; ++i) {
            int64_t t = i == npn - 1 ? node_msg - s_lens[i * P] : s_lens[(i + 1) * P] - s_lens[i * P];
            if (t) il_push(&idx, buf_recv(p, lr0 + i, t, 1, LB_AGG, ptr, lr0 + i + lr0 + it100));
            ptr += t;
        }
    } else if (total_send) {
        il_push(&idx, buf_send(p, lr0, total_send, 1, LB_AGG, local, rank + lr0 + it100, 0));
    }
    if (idx.n) { tstart(p, F_RECV); wait_list(p, idx.v, idx.n); tstop(p, F_RECV); }
    if (proxy) {
        /* inter-node exchange among the proxies (:1116-1197) */
        int64_t rb = 0, ptr2 = 0;
        gsl = (int64_t *)calloc(nrecvs, sizeof(int64_t));
        grl = (int64_t *)calloc(nrecvs, sizeof(int64_t));
        ptrs = (int64_t *)calloc(nrecvs, sizeof(int64_t));
        idx.n = 0;
        ptr = 0;
        for (i = 0; i < nrecvs; ++i) {
            int64_t temp2 = 0;
            int vhi = (i + 1) * pn < P ? (i + 1) * pn : P;
            for (v = i * pn; v < vhi; ++v)
                for (w = 0; w < npn; ++w) {
                    int t = w * P + v;
                    int64_t n = t < P * npn - 1 ? s_lens[t + 1] - s_lens[t] : node_msg - s_lens[t];
                    if (n) { buf_copy(p, LB_AGG, s_lens[t], LB_SBUF2, ptr + temp2, n); temp2 += n; }
                }
            ptr += temp2;
            gsl[i] = temp2;
            if (i * pn != rank) {
                il_push(&idx, buf_recv(p, i * pn, 1, 4, LB_CTRL, (int64_t)i * 4, i * pn + rank + it100));
                il_push(&idx, buf_send(p, i * pn, 1, 4, LB_CTRL, (int64_t)i * 4, i * pn + rank + it100, 0));
            }
        }
        /* what proxy i sends here: everything its node's ranks send to this node's ranks */
        for (i = 0; i < nrecvs; ++i) {
            if (i * pn == rank) { grl[i] = gsl[i]; continue; }
            {
                int whi = (i + 1) * pn < P ? (i + 1) * pn : P, mhi = lr0 + npn;
                for (w = i * pn; w < whi; ++w)
                    for (v = lr0; v < mhi; ++v) grl[i] += tam_ss(x, w, v);
            }
        }
        if (idx.n) { tstart(p, F_SEND); wait_list(p, idx.v, idx.n); tstop(p, F_SEND); }
        idx.n = 0;
        for (i = 0; i < nrecvs; ++i) {
            int peer = i * pn;
            if (i > 0) rb += grl[i - 1];
            if (rank != peer) {
                if (gsl[i]) il_push(&idx, buf_send(p, peer, gsl[i], 1, LB_SBUF2, ptr2, peer + rank + it100, 0));
                if (grl[i]) il_push(&idx, buf_recv(p, peer, grl[i], 1, LB_RBUF, rb, peer + rank + it100));
            } else if (grl[i]) {
                buf_copy(p, LB_SBUF2, ptr2, LB_RBUF, rb, grl[i]);
            }
            ptr2 += gsl[i];
            ptrs[i] = rb;
        }
        if (idx.n) { tstart(p, F_SEND); wait_list(p, idx.v, idx.n); tstop(p, F_SEND); }
    }
    /* local delivery (:1213-1285) */
    idx.n = 0;
    if (proxy) {
        if (total_recv)
            for (w = 0; w < P; ++w) {
                int64_t n = tam_rs(x, rank, w);
                if (n) buf_copy(p, LB_RBUF, ptrs[w / pn], LB_RECV, tam_rloc(x, w), n);
                ptrs[w / pn] += n;
            }
        ptr = 0;
        for (i = 1; i < npn; ++i) {
            int64_t t = i == npn - 1 ? node_recv - r_lens[i * P] : r_lens[(i + 1) * P] - r_lens[i * P];
            if (t) {
                int64_t ptr2 = ptr;
                for (w = 0; w < P; ++w) {
                    int64_t n = (i == npn - 1 && w == P - 1) ? node_recv - r_lens[i * P + w]
                                                             : r_lens[i * P + w + 1] - r_lens[i * P + w];
                    if (n) buf_copy(p, LB_RBUF, ptrs[w / pn], LB_AGG, ptr, n);
                    ptrs[w / pn] += n;
                    ptr += n;
                }
                il_push(&idx, buf_send(p, lr0 + i, t, 1, LB_AGG, ptr2, lr0 + i + lr0 + it100, 0));
            }
        }
    } else if (total_recv) {
        il_push(&idx, buf_recv(p, lr0, total_recv, 1, LB_AGG, local, rank + lr0 + it100));
    }
    if (idx.n) { tstart(p, F_RECV); wait_list(p, idx.v, idx.n); tstop(p, F_RECV); }
    if (!proxy && total_recv) {
        off = local;
        for (w = 0; w < P; ++w) {
            int64_t n = tam_rs(x, rank, w);
            if (n) { buf_copy(p, LB_AGG, off, LB_RECV, tam_rloc(x, w), n); off += n; }
        }
    }
    free(idx.v); free(s_lens); free(r_lens); free(gsl); free(grl); free(ptrs);
}

/* all_to_many_tam :366-419 / many_to_all_tam :313-364 */
static void m_tam(ctx_t *x)
{
    int m;
    for (m = 0; m < x->ntimes; ++m) tam_collective_write(x);
}

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
    s->scr_base = (int64_t *)xmalloc(sizeof(int64_t) * NSCR * s->P);
    s->scr_size = (int64_t *)xmalloc(sizeof(int64_t) * s->P);
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
    S = (pst_t *)xmalloc(sizeof(pst_t) * tot_s);
    R = (pst_t *)xmalloc(sizeof(pst_t) * tot_r);
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
    int *pc = (int *)xmalloc(sizeof(int) * P), *epoch = (int *)xmalloc(sizeof(int) * P);
    int32_t **pe = (int32_t **)xmalloc(sizeof(int32_t *) * P);     /* post epoch */
    int nb = s->progs[0].nbarrier;
    int *arrived = (int *)calloc(nb + 1, sizeof(int)), *arr_epoch = (int *)xmalloc(sizeof(int) * (nb + 1));
    int *lw = (int *)xmalloc(sizeof(int) * NLB * P), *lrd = (int *)xmalloc(sizeof(int) * NLB * P);
    for (r = 0; r < NLB * P; ++r) lw[r] = lrd[r] = INT_MIN / 2;
    for (r = 1; r < P; ++r)
        if (s->progs[r].nbarrier != nb) {
            snprintf(err, errlen, "ranks disagree on the number of MPI_Barrier calls");
            free(arrived); free(arr_epoch); free(pc); free(epoch); free(pe); free(lw); free(lrd);
            return -1;
        }
    s->nbarrier = nb;
    s->barrier_epoch = (int32_t *)xmalloc(sizeof(int32_t) * (nb + 1));
    for (b = 0; b < nb; ++b) { arr_epoch[b] = -1; s->barrier_epoch[b] = INT_MIN; }
    for (r = 0; r < P; ++r) {
        int q;
        pc[r] = 0; epoch[r] = -1;
        pe[r] = (int32_t *)xmalloc(sizeof(int32_t) * (s->progs[r].nposts + 1));
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
    s = (xg_sched *)calloc(1, sizeof *s);
    s->method = method; s->P = procs; s->A = cb_nodes; s->d = data_size; s->c = comm_size;
    s->ntimes = ntimes; s->eager = eager_limit; s->dir = xg_method_direction(method);
    s->proc_node = proc_node; s->barrier_type = barrier_type; s->iter = iter;
    s->rank_list = (int *)xmalloc(sizeof(int) * cb_nodes);
    memcpy(s->rank_list, rank_list, sizeof(int) * cb_nodes);
    s->isagg = (int *)calloc(procs, sizeof(int));
    s->agg_prefix = (int *)xmalloc(sizeof(int) * (procs + 1));
    for (i = 0; i < cb_nodes; ++i) s->isagg[rank_list[i]] = 1;
    s->agg_prefix[0] = 0;
    for (r = 0; r < procs; ++r) s->agg_prefix[r + 1] = s->agg_prefix[r] + s->isagg[r];
    s->progs = (prog_t *)calloc(procs, sizeof(prog_t));
    lastidx = (int *)xmalloc(sizeof(int) * procs);
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
        barrier(p);                                   /* MPI_Barrier before total_start */
        tstart(p, F_TOTAL);
        switch (method) {
        case 1: m1_all_to_many(&x); break;
        case 2: m2_many_to_all(&x); break;
        case 3: m3_balanced(&x); break;
        case 4: m4_balanced(&x); break;
        case 5: m_alltoallw(&x, XG_M2A); break;
        case 6: m6_sync(&x); break;
        case 7: m7_half_sync(&x); break;
        case 8: m_alltoallw(&x, XG_A2M); break;
        case 9: m_pairwise(&x, XG_A2M); break;
        case 10: m_pairwise(&x, XG_M2A); break;
        case 11: m11_half_sync(&x); break;
        case 12: m12_half_sync2(&x); break;
        case 13: m13_scattered(&x); break;
        case 14: m14_scattered(&x); break;
        case 15: case 16: m_tam(&x); break;
        case 17: m17_node_robin(&x); break;
        case 18: m18_balanced_control(&x); break;
        case 19: m19_scattered_isend(&x); break;
        case 20: m20_balanced_presend(&x); break;
        }
        tstop(p, F_TOTAL);
    }
    free(lastidx);
    scratch_layout(s);
    s->post_msg = (int32_t **)calloc(procs, sizeof(int32_t *));
    s->post_eager = (uint8_t **)calloc(procs, sizeof(uint8_t *));
    for (r = 0; r < procs; ++r) {
        prog_t *p = &s->progs[r];
        s->post_msg[r] = (int32_t *)xmalloc(sizeof(int32_t) * (p->nposts + 1));
        s->post_eager[r] = (uint8_t *)calloc(p->nposts + 1, 1);
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
            int *v = (int *)xmalloc(sizeof(int) * (o->wcnt + 1)), a = 0;
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
    s->post_count = (int32_t *)calloc((size_t)ngpus * (s->nsteps + 1), sizeof(int32_t));
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
static void step_posts_of(const xg_sched *s, int ngpus, int g, int32_t *out, int nout)
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

static int nsend_segs(const xg_sched *s, int r)
{
    return s->dir == XG_A2M ? s->A : (s->isagg[r] ? s->P : 0);
}

static int nrecv_slots(const xg_sched *s, int r)
{
    return s->dir == XG_A2M ? (s->isagg[r] ? s->P : 0) : s->A;
}

static int64_t rank_offset(const xg_sched *s, int ngpus, int rank, int recv)
{
    int lo, hi, g = xg_gpu_of(s->P, ngpus, rank);
    int per_rank = recv ? nrecv_slots(s, rank) : nsend_segs(s, rank);
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

/* ------------------------------------------------------------------ device plan */
/* Growable arrays of the device-plan builder.  The builder runs on every rank of a job and
 * must not stop one rank alone: when the host runs out of memory, a push lands in `sink` and
 * `fail` is set; xg_devplan_build_form then frees what it built and returns NULL, which the
 * caller turns into an error every rank agrees on (methods.c peers_agree). */
typedef struct { xg_copy *v; int n, cap, fail; xg_copy sink; } cvec;
typedef struct { xg_p2p *v; int n, cap, fail; xg_p2p sink; } pvec;
static xg_copy *cpush(cvec *c)
{
    if (c->n == c->cap) {
        const int cap = c->cap ? 2 * c->cap : 256;
        xg_copy *v = c->fail ? NULL : (xg_copy *)realloc(c->v, sizeof(xg_copy) * cap);
        if (!v) { c->fail = 1; memset(&c->sink, 0, sizeof c->sink); return &c->sink; }
        c->v = v; c->cap = cap;
    }
    memset(&c->v[c->n], 0, sizeof(xg_copy));
    return &c->v[c->n++];
}
static xg_p2p *ppush(pvec *c)
{
    if (c->n == c->cap) {
        const int cap = c->cap ? 2 * c->cap : 256;
        xg_p2p *v = c->fail ? NULL : (xg_p2p *)realloc(c->v, sizeof(xg_p2p) * cap);
        if (!v) { c->fail = 1; memset(&c->sink, 0, sizeof c->sink); return &c->sink; }
        c->v = v; c->cap = cap;
    }
    memset(&c->v[c->n], 0, sizeof(xg_p2p));
    return &c->v[c->n++];
}

void xg_devplan_free(xg_devplan *p)
{
    if (!p) return;
    free(p->copies); free(p->p2p); free(p->steps); free(p);
}

/* same decision on both ends of a (step, src gpu, dst gpu) transfer list: >= 2 segments, mean
 * below pack_max_seg, and at least pack_min bytes (below that one RCCL call per segment costs
 * less than the pack and unpack launches) */
static int use_pack(int n, int64_t total, int64_t pack_max_seg, int64_t pack_min)
{
    return pack_max_seg > 0 && n >= 2 && total / n < pack_max_seg && total >= pack_min;
}

/* region base of every rank hosted by the GPU the plan is for */
typedef struct { int64_t *base[XG_NBUF]; } plan_bases;

/* -> 0, or -1 when the host is out of memory (pb is then freeable) */
static int plan_bases_init(plan_bases *pb, const xg_sched *s, int G, int g)
{
    int lo, hi, r, k, fail = 0;
    int64_t scr = 0;
    (void)g;
    for (k = 0; k < XG_NBUF; ++k) fail |= !(pb->base[k] = (int64_t *)calloc(s->P + 1, sizeof(int64_t)));
    if (fail) return -1;
    for (r = 0; r < s->P; ++r) {
        pb->base[XG_BUF_SEND][r] = xg_send_offset(s, G, r);
        pb->base[XG_BUF_RECV][r] = xg_recv_offset(s, G, r);
    }
    for (k = 0; k < G; ++k) {
        xg_block_range(s->P, G, k, &lo, &hi);
        for (scr = 0, r = lo; r < hi; ++r) { pb->base[XG_BUF_SCRATCH][r] = scr; scr += s->scr_size[r]; }
    }
    return 0;
}

static void plan_bases_free(plan_bases *pb)
{
    int k;
    for (k = 0; k < XG_NBUF; ++k) free(pb->base[k]);
}

static int64_t src_off(const plan_bases *pb, const xg_msg *m) { return pb->base[m->sbuf][m->src] + m->soff; }
static int64_t dst_off(const plan_bases *pb, const xg_msg *m) { return pb->base[m->dbuf][m->dst] + m->doff; }

/* a message that moves device bytes (not a size message, not empty) */
static int moves(const xg_msg *m) { return m->len > 0 && !(m->flags & XG_MSG_CTRL); }

/* a rank-local memcpy through a TAM aggregation buffer */
static int is_stage(const xg_msg *m)
{
    return (m->flags & XG_MSG_COPY) && (m->sbuf == XG_BUF_SCRATCH || m->dbuf == XG_BUF_SCRATCH);
}

static void local_copy(xg_copy *c, const plan_bases *pb, const xg_msg *m)
{
    c->src_buf = m->sbuf; c->src_off = src_off(pb, m);
    c->dst_buf = m->dbuf; c->dst_off = dst_off(pb, m);
    c->len = m->len;
}

xg_devplan *xg_devplan_build(const xg_sched *s, int ngpus, int g, int64_t pack_max_seg)
{
    return xg_devplan_build_form(s, ngpus, g, pack_max_seg, 0, XG_PACK_FORM_DEFAULT);
}

xg_devplan *xg_devplan_build_ex(const xg_sched *s, int ngpus, int g, int64_t pack_max_seg, int64_t pack_min)
{
    return xg_devplan_build_form(s, ngpus, g, pack_max_seg, pack_min, XG_PACK_FORM_DEFAULT);
}

/* One-sided form of one packed (step, src GPU -> dst GPU) transfer list (XG_PACK_ONE_SIDED).
 * The messages are put in destination order (by_src = 0) or source order (by_src = 1) and
 * merged into RUNS, each contiguous on that side: one RCCL call per run.  A run that is
 * contiguous on the other side as well moves straight between the regions; any other one is
 * gathered into staging by the sender (destination order) or scattered out of it by the
 * receiver (source order) -- so every byte is copied on ONE side at most, where the two-sided
 * form packs and unpacks all of them.  This is the transpose the alltoallw datatypes of m5/m8
 * describe (mpi_test.c:233-302): e.g. all-to-many at P64 A16 on 8 GPUs, per peer the 16
 * segments of 8 senders for 2 aggregators -- 2 runs of 2 MiB, one per aggregator's receive
 * slots, gathered on the sending GPU; nothing is unpacked.  Of the two orders the one with
 * fewer copied bytes + XG_RUN_CALL_BYTES per call wins (ties: destination order).  Both GPUs
 * of the pair derive it from the same message list, so their calls pair one to one. */
typedef struct {
    int n, nrun, by_src, fail;   /* fail: out of host memory (the plan is discarded) */
    int *idx;                 /* message indices, run order */
    int *run_b;               /* run r = idx[run_b[r] .. run_b[r + 1]) */
    unsigned char *staged;    /* run r goes through staging */
} oneside;

static const xg_msg *os_msg(const xg_sched *s, const oneside *o, int i) { return &s->msgs[o->idx[i]]; }

typedef struct { int64_t off; int32_t buf, idx; } os_key;
static int os_cmp(const void *a, const void *b)
{
    const os_key *x = (const os_key *)a, *y = (const os_key *)b;
    if (x->buf != y->buf) return x->buf < y->buf ? -1 : 1;
    if (x->off != y->off) return x->off < y->off ? -1 : 1;
    return x->idx < y->idx ? -1 : x->idx > y->idx;      /* equal addresses: message order */
}

/* runs of `o` in the order by_src; returns the cost (copied bytes + calls) */
static int64_t os_layout(const xg_sched *s, const plan_bases *pb, oneside *o, int by_src)
{
    int i, r;
    int64_t cost = 0;
    os_key *key = (os_key *)malloc(sizeof(os_key) * ((size_t)o->n + 1));
    o->by_src = by_src;
    if (!key) {
        o->fail = 1;
        o->nrun = 0;
        return 0;
    }
    for (i = 0; i < o->n; ++i) {
        const xg_msg *m = os_msg(s, o, i);
        key[i].buf = by_src ? m->sbuf : m->dbuf;
        key[i].off = by_src ? src_off(pb, m) : dst_off(pb, m);
        key[i].idx = o->idx[i];
    }
    qsort(key, (size_t)o->n, sizeof(os_key), os_cmp);
    for (i = 0; i < o->n; ++i) o->idx[i] = key[i].idx;
    free(key);
    o->nrun = 0;
    for (i = 0; i < o->n; ++i) {
        const xg_msg *m = os_msg(s, o, i);
        if (i > 0) {
            const xg_msg *q = os_msg(s, o, i - 1);
            const int contiguous = by_src ? (m->sbuf == q->sbuf && src_off(pb, m) == src_off(pb, q) + q->len)
                                          : (m->dbuf == q->dbuf && dst_off(pb, m) == dst_off(pb, q) + q->len);
            if (contiguous) continue;
        }
        o->run_b[o->nrun++] = i;
    }
    o->run_b[o->nrun] = o->n;
    for (r = 0; r < o->nrun; ++r) {
        int64_t bytes = 0;
        int other = 1;      /* contiguous on the other side too */
        for (i = o->run_b[r]; i < o->run_b[r + 1]; ++i) {
            const xg_msg *m = os_msg(s, o, i);
            bytes += m->len;
            if (i > o->run_b[r]) {
                const xg_msg *q = os_msg(s, o, i - 1);
                other &= by_src ? (m->dbuf == q->dbuf && dst_off(pb, m) == dst_off(pb, q) + q->len)
                                : (m->sbuf == q->sbuf && src_off(pb, m) == src_off(pb, q) + q->len);
            }
        }
        o->staged[r] = !other;
        cost += (other ? 0 : bytes) + XG_RUN_CALL_BYTES;
    }
    return cost;
}

/* the one-sided form of the messages of step [b, e) from GPU gs to GPU gd */
static void os_build(const xg_sched *s, const plan_bases *pb, const int *order, int b, int e, int G, int gs,
                     int gd, oneside *o)
{
    int k;
    int64_t cost_d, cost_s;
    o->n = 0;
    for (k = b; k < e; ++k) {
        const xg_msg *m = &s->msgs[order[k]];
        if (moves(m) && xg_gpu_of(s->P, G, m->src) == gs && xg_gpu_of(s->P, G, m->dst) == gd) o->n++;
    }
    o->idx = (int *)malloc(sizeof(int) * ((size_t)o->n + 1));
    o->run_b = (int *)malloc(sizeof(int) * ((size_t)o->n + 2));
    o->staged = (unsigned char *)malloc((size_t)o->n + 1);
    if (!o->idx || !o->run_b || !o->staged) {
        free(o->idx); free(o->run_b); free(o->staged);
        o->idx = o->run_b = NULL;
        o->staged = NULL;
        o->n = o->nrun = 0;
        o->fail = 1;
        return;
    }
    o->n = 0;
    for (k = b; k < e; ++k) {
        const xg_msg *m = &s->msgs[order[k]];
        if (moves(m) && xg_gpu_of(s->P, G, m->src) == gs && xg_gpu_of(s->P, G, m->dst) == gd) o->idx[o->n++] = order[k];
    }
    cost_s = os_layout(s, pb, o, 1);
    cost_d = os_layout(s, pb, o, 0);
    if (cost_s < cost_d) os_layout(s, pb, o, 1);
}

/* frees the arrays; keeps `fail` for the caller to see */
static void os_free(oneside *o)
{
    const int fail = o->fail;
    free(o->idx); free(o->run_b); free(o->staged);
    memset(o, 0, sizeof *o);
    o->fail = fail;
}

/* ---- relay form (XG_RELAY, xg_sched.h): two-phase (Valiant) routing of one step.  Every
 * cross-GPU message is cut into G pieces: pieces 0 and 1 go straight to the destination (one per
 * RCCL group), piece 2 + i through relay GPU R[i].  Then EVERY link (a -> h) carries egress(a) / G
 * in the first group and every link (h -> b) ingress(b) / G in the second, whatever the step's
 * traffic matrix: the step costs (max egress + max ingress) / G of link time instead of its
 * busiest GPU pair's bytes.  A step is relayed when that is at most XG_RELAY_GAIN of the direct
 * cost and every cross-GPU message is >= XG_RELAY_MIN_BYTES (smaller pieces are latency, not
 * bandwidth).  Pairwise m9 / m10 (mpi_test.c:510-597, :421-508; partner rank ^ i, :531-545) at
 * configs[3] put every GPU's 16 MiB round on ONE of its 7 links: 16 -> 4 MiB of link time per
 * round.  Every GPU decides from the same message list, so all agree. */
static int relay_step(const xg_sched *s, const int *order, int b, int e, int G, int64_t *egress, int64_t *ingress,
                      int64_t *pair)
{
    int k, g, any = 0;
    int64_t direct = 0, emax = 0, imax = 0;
    if (G < 3) return 0;
    memset(egress, 0, sizeof(int64_t) * (size_t)G);
    memset(ingress, 0, sizeof(int64_t) * (size_t)G);
    memset(pair, 0, sizeof(int64_t) * (size_t)G * G);
    for (k = b; k < e; ++k) {
        const xg_msg *m = &s->msgs[order[k]];
        const int gs = xg_gpu_of(s->P, G, m->src), gd = xg_gpu_of(s->P, G, m->dst);
        if (!moves(m) || is_stage(m) || gs == gd) continue;
        if (m->len < XG_RELAY_MIN_BYTES) return 0;
        egress[gs] += m->len;
        ingress[gd] += m->len;
        pair[(size_t)gs * G + gd] += m->len;
        any = 1;
    }
    if (!any) return 0;
    for (g = 0; g < G * G; ++g) direct = pair[g] > direct ? pair[g] : direct;
    for (g = 0; g < G; ++g) {
        emax = egress[g] > emax ? egress[g] : emax;
        imax = ingress[g] > imax ? ingress[g] : imax;
    }
    return (double)(emax + imax) / G <= XG_RELAY_GAIN * (double)direct;
}

/* piece k of a relayed message of len bytes: [relay_cut(k), relay_cut(k + 1)), 16-B aligned cuts */
static int64_t relay_cut(int64_t len, int k, int G) { return k >= G ? len : ((len * k / G) & ~(int64_t)15); }

/* relay i (0 .. G-3) of a message from GPU gs to GPU gd: the GPUs other than gs, gd, ascending */
static int relay_gpu(int i, int gs, int gd)
{
    const int lo = gs < gd ? gs : gd, hi = gs < gd ? gd : gs;
    int h = i;
    if (h >= lo) ++h;
    if (h >= hi) ++h;
    return h;
}

static void relay_push(pvec *pp, int peer, int is_send, int buf, int64_t off, int64_t len, int group)
{
    xg_p2p *o;
    if (len <= 0) return;            /* a 0-byte piece (len < 16 G): no call on either side */
    o = ppush(pp);
    o->peer = peer; o->is_send = is_send; o->buf = buf; o->off = off; o->len = len; o->group = group;
}

/* GPU g's calls of one relayed step: group 0 = pieces 0 straight to the destination and pieces
 * 2 + i to relay R[i] (into its STAGE_RECV at *rbase on); group 1 = pieces 1 straight, and what g
 * holds as a relay forwarded to the destination.  Every list is in message order, so the k-th
 * send of any GPU to any other pairs with the k-th receive there, group by group. */
static void relay_calls(const xg_sched *s, const plan_bases *pb, const int *order, int b, int e, int G, int g,
                        pvec *pp, int64_t *rbase)
{
    int grp, k, i;
    int64_t roff = *rbase;
    for (grp = 0; grp < 2; ++grp) {
        roff = *rbase;
        for (k = b; k < e; ++k) {
            const xg_msg *m = &s->msgs[order[k]];
            const int gs = xg_gpu_of(s->P, G, m->src), gd = xg_gpu_of(s->P, G, m->dst);
            const int ri = g != gs && g != gd ? g - (g > gs) - (g > gd) : -1;   /* g's relay index */
            int64_t so, dof;
            if (!moves(m) || is_stage(m) || gs == gd) continue;
            so = src_off(pb, m);
            dof = dst_off(pb, m);
            if (g == gs) {
                relay_push(pp, gd, 1, m->sbuf, so + relay_cut(m->len, grp, G),
                           relay_cut(m->len, grp + 1, G) - relay_cut(m->len, grp, G), grp);
                for (i = 0; grp == 0 && i < G - 2; ++i)
                    relay_push(pp, relay_gpu(i, gs, gd), 1, m->sbuf, so + relay_cut(m->len, 2 + i, G),
                               relay_cut(m->len, 3 + i, G) - relay_cut(m->len, 2 + i, G), 0);
            }
            if (ri >= 0) {
                const int64_t len = relay_cut(m->len, 3 + ri, G) - relay_cut(m->len, 2 + ri, G);
                if (grp == 0) relay_push(pp, gs, 0, XG_BUF_STAGE_RECV, roff, len, 0);
                else relay_push(pp, gd, 1, XG_BUF_STAGE_RECV, roff, len, 1);
                roff += len > 0 ? len : 0;
            }
            if (g == gd) {
                relay_push(pp, gs, 0, m->dbuf, dof + relay_cut(m->len, grp, G),
                           relay_cut(m->len, grp + 1, G) - relay_cut(m->len, grp, G), grp);
                for (i = 0; grp == 1 && i < G - 2; ++i)
                    relay_push(pp, relay_gpu(i, gs, gd), 0, m->dbuf, dof + relay_cut(m->len, 2 + i, G),
                               relay_cut(m->len, 3 + i, G) - relay_cut(m->len, 2 + i, G), 1);
            }
        }
    }
    *rbase = roff;
}

xg_devplan *xg_devplan_build_form(const xg_sched *s, int ngpus, int g, int64_t pack_max_seg, int64_t pack_min,
                                  int form)
{
    xg_devplan *dp = (xg_devplan *)calloc(1, sizeof *dp);
    int nst = s->nsteps, i, st, G = ngpus, oom = 0;
    int *cnt = (int *)calloc(nst + 1, sizeof(int)), *order = (int *)malloc(sizeof(int) * (s->nmsg + 1));
    int *pos = (int *)malloc(sizeof(int) * (nst + 1));
    cvec pre, post;
    pvec pp;
    int64_t stage_s_max = 0, stage_r_max = 0;
    int *bucket_n = (int *)calloc((size_t)G * 2, sizeof(int));
    int64_t *bucket_b = (int64_t *)calloc((size_t)G * 2, sizeof(int64_t));
    oneside *os_out = (oneside *)calloc((size_t)G, sizeof(oneside)), *os_in = (oneside *)calloc((size_t)G, sizeof(oneside));
    int64_t *rl_e = (int64_t *)calloc((size_t)G, sizeof(int64_t)), *rl_i = (int64_t *)calloc((size_t)G, sizeof(int64_t));
    int64_t *rl_p = (int64_t *)calloc((size_t)G * G, sizeof(int64_t));
    plan_bases pb;
    memset(&pre, 0, sizeof pre); memset(&post, 0, sizeof post); memset(&pp, 0, sizeof pp);
    memset(&pb, 0, sizeof pb);
    if (form != XG_PACK_TWO_SIDED && form != XG_PACK_ONE_SIDED && form != XG_RELAY) form = XG_PACK_FORM_DEFAULT;
    if (form == XG_RELAY) pack_max_seg = 0;         /* relay form: every other step is direct */
    if (!dp || !cnt || !order || !pos || !bucket_n || !bucket_b || !os_out || !os_in || !rl_e || !rl_i || !rl_p ||
        plan_bases_init(&pb, s, G, g) ||
        !(dp->steps = (xg_stepplan *)calloc(nst + 1, sizeof(xg_stepplan)))) {
        oom = 1;
        goto done;
    }
    dp->gpu = g; dp->ngpus = G; dp->nsteps = nst;
    {   /* per step, the request posts of this GPU's ranks (graph replays share their launch time
         * out by them: xg_plan_run) */
        int32_t *posts = (int32_t *)calloc((size_t)nst + 1, sizeof(int32_t));
        if (!posts) { oom = 1; goto done; }
        step_posts_of(s, G, g, posts, nst);
        for (st = 0; st < nst; ++st) dp->steps[st].posts = posts[st];
        free(posts);
    }
    /* in-loop MPI_Barrier -> device-side barrier after the step it completes at (G > 1) */
    for (i = 0; i < s->nbarrier; ++i)
        if (G > 1 && s->barrier_epoch[i] >= 0 && s->barrier_epoch[i] < nst) dp->steps[s->barrier_epoch[i]].sync_after = 1;
    /* counting sort of messages by step, stable in message order */
    for (i = 0; i < s->nmsg; ++i) cnt[s->msgs[i].step + 1]++;
    for (st = 0; st < nst; ++st) cnt[st + 1] += cnt[st];
    memcpy(pos, cnt, sizeof(int) * (nst + 1));
    for (i = 0; i < s->nmsg; ++i) order[pos[s->msgs[i].step]++] = i;
    dp->region_bytes[XG_BUF_SEND] = xg_region_bytes(s, G, g, XG_BUF_SEND);
    dp->region_bytes[XG_BUF_RECV] = xg_region_bytes(s, G, g, XG_BUF_RECV);
    dp->region_bytes[XG_BUF_SCRATCH] = xg_region_bytes(s, G, g, XG_BUF_SCRATCH);
    for (st = 0; st < nst; ++st) {
        int b = cnt[st], e = cnt[st + 1], k, p;
        int64_t sbase = 0, rbase = 0;
        xg_stepplan *sp = &dp->steps[st];
        /* per-peer volume (out: [p], in: [G+p]) for the pack decision */
        memset(bucket_n, 0, sizeof(int) * 2 * G);
        memset(bucket_b, 0, sizeof(int64_t) * 2 * G);
        sp->pre_begin = pre.n;
        /* rank-local memcpy's through SCRATCH first, in a launch of their own: the
         * local messages and packs below may read what they write in this step */
        for (k = b; k < e; ++k) {
            const xg_msg *m = &s->msgs[order[k]];
            if (!moves(m) || !is_stage(m) || xg_gpu_of(s->P, G, m->src) != g) continue;
            local_copy(cpush(&pre), &pb, m);
            dp->local_bytes += m->len;
        }
        sp->stage_count = pre.n - sp->pre_begin;
        for (k = b; k < e; ++k) {
            const xg_msg *m = &s->msgs[order[k]];
            int gs = xg_gpu_of(s->P, G, m->src), gd = xg_gpu_of(s->P, G, m->dst);
            if (!moves(m) || is_stage(m)) continue;
            if (gs == g && gd == g) {
                local_copy(cpush(&pre), &pb, m);
                dp->local_bytes += m->len;
            } else if (gs == g) {
                bucket_n[gd]++; bucket_b[gd] += m->len;
            } else if (gd == g) {
                bucket_n[G + gs]++; bucket_b[G + gs] += m->len;
            }
        }
        /* the one-sided layout of every packed list of this GPU's, both directions */
        if (form == XG_PACK_ONE_SIDED)
            for (p = 0; p < G; ++p) {
                if (p == g) continue;
                if (bucket_n[p] && use_pack(bucket_n[p], bucket_b[p], pack_max_seg, pack_min))
                    os_build(s, &pb, order, b, e, G, g, p, &os_out[p]);
                if (bucket_n[G + p] && use_pack(bucket_n[G + p], bucket_b[G + p], pack_max_seg, pack_min))
                    os_build(s, &pb, order, b, e, G, p, g, &os_in[p]);
                oom |= os_out[p].fail | os_in[p].fail;
            }
        /* packs (into staging) join the pre-exchange copy launch */
        for (p = 0; p < G; ++p) {
            int64_t off = 0;
            if (p == g || !bucket_n[p] || !use_pack(bucket_n[p], bucket_b[p], pack_max_seg, pack_min)) continue;
            if (form == XG_PACK_ONE_SIDED) {
                const oneside *o = &os_out[p];
                int r;
                for (r = 0; r < o->nrun; ++r) {
                    if (o->by_src || !o->staged[r]) continue;     /* sent as it lies */
                    for (k = o->run_b[r]; k < o->run_b[r + 1]; ++k) {
                        const xg_msg *m = os_msg(s, o, k);
                        xg_copy *c = cpush(&pre);
                        c->src_buf = m->sbuf; c->src_off = src_off(&pb, m);
                        c->dst_buf = XG_BUF_STAGE_SEND; c->dst_off = sbase + off;
                        c->len = m->len;
                        off += m->len;
                    }
                }
                sbase += off;
                continue;
            }
            for (k = b; k < e; ++k) {
                const xg_msg *m = &s->msgs[order[k]];
                if (!moves(m) || xg_gpu_of(s->P, G, m->src) != g || xg_gpu_of(s->P, G, m->dst) != p) continue;
                {
                    xg_copy *c = cpush(&pre);
                    c->src_buf = m->sbuf; c->src_off = src_off(&pb, m);
                    c->dst_buf = XG_BUF_STAGE_SEND; c->dst_off = sbase + off;
                    c->len = m->len;
                    off += m->len;
                }
            }
            sbase += off;
        }
        sp->pre_count = pre.n - sp->pre_begin;
        /* the grouped exchange: per peer, sends then receives, message order */
        sp->p2p_begin = pp.n;
        sp->post_begin = post.n;
        if (form == XG_RELAY && relay_step(s, order, b, e, G, rl_e, rl_i, rl_p)) {
            /* every message over all G - 1 links of its source, then of its destination (two groups) */
            relay_calls(s, &pb, order, b, e, G, g, &pp, &rbase);
            for (p = 0; p < G; ++p)
                if (p != g) {
                    dp->remote_send_bytes += bucket_b[p];
                    dp->remote_recv_bytes += bucket_b[G + p];
                }
        } else {
            int64_t soff = 0;
            for (p = 0; p < G; ++p) {
                int pk;
                if (p == g) continue;
                if (bucket_n[p]) {
                    pk = use_pack(bucket_n[p], bucket_b[p], pack_max_seg, pack_min);
                    if (pk && form == XG_PACK_ONE_SIDED) {
                        const oneside *o = &os_out[p];
                        int r;
                        for (r = 0; r < o->nrun; ++r) {
                            xg_p2p *q = ppush(&pp);
                            int64_t len = 0;
                            for (k = o->run_b[r]; k < o->run_b[r + 1]; ++k) len += os_msg(s, o, k)->len;
                            q->peer = p; q->is_send = 1; q->len = len;
                            if (!o->by_src && o->staged[r]) {
                                q->buf = XG_BUF_STAGE_SEND; q->off = soff;
                                soff += len;
                            } else {
                                const xg_msg *m = os_msg(s, o, o->run_b[r]);
                                q->buf = m->sbuf; q->off = src_off(&pb, m);
                            }
                        }
                    } else if (pk) {
                        xg_p2p *o = ppush(&pp);
                        o->peer = p; o->is_send = 1; o->buf = XG_BUF_STAGE_SEND; o->off = soff; o->len = bucket_b[p];
                        soff += bucket_b[p];
                    } else {
                        for (k = b; k < e; ++k) {
                            const xg_msg *m = &s->msgs[order[k]];
                            if (!moves(m) || xg_gpu_of(s->P, G, m->src) != g || xg_gpu_of(s->P, G, m->dst) != p) continue;
                            {
                                xg_p2p *o = ppush(&pp);
                                o->peer = p; o->is_send = 1; o->buf = m->sbuf;
                                o->off = src_off(&pb, m); o->len = m->len;
                            }
                        }
                    }
                    dp->remote_send_bytes += bucket_b[p];
                }
                if (bucket_n[G + p]) {
                    pk = use_pack(bucket_n[G + p], bucket_b[G + p], pack_max_seg, pack_min);
                    if (pk && form == XG_PACK_ONE_SIDED) {
                        const oneside *o = &os_in[p];
                        int r;
                        for (r = 0; r < o->nrun; ++r) {
                            xg_p2p *q = ppush(&pp);
                            int64_t len = 0;
                            for (k = o->run_b[r]; k < o->run_b[r + 1]; ++k) len += os_msg(s, o, k)->len;
                            q->peer = p; q->is_send = 0; q->len = len;
                            if (o->by_src && o->staged[r]) {
                                int64_t off = 0;
                                q->buf = XG_BUF_STAGE_RECV; q->off = rbase;
                                for (k = o->run_b[r]; k < o->run_b[r + 1]; ++k) {
                                    const xg_msg *m = os_msg(s, o, k);
                                    xg_copy *c = cpush(&post);
                                    c->src_buf = XG_BUF_STAGE_RECV; c->src_off = rbase + off;
                                    c->dst_buf = m->dbuf; c->dst_off = dst_off(&pb, m);
                                    c->len = m->len;
                                    off += m->len;
                                }
                                rbase += len;
                            } else {
                                const xg_msg *m = os_msg(s, o, o->run_b[r]);
                                q->buf = m->dbuf; q->off = dst_off(&pb, m);
                            }
                        }
                    } else if (pk) {
                        xg_p2p *o = ppush(&pp);
                        int64_t off = 0;
                        o->peer = p; o->is_send = 0; o->buf = XG_BUF_STAGE_RECV; o->off = rbase; o->len = bucket_b[G + p];
                        for (k = b; k < e; ++k) {
                            const xg_msg *m = &s->msgs[order[k]];
                            if (!moves(m) || xg_gpu_of(s->P, G, m->src) != p || xg_gpu_of(s->P, G, m->dst) != g) continue;
                            {
                                xg_copy *c = cpush(&post);
                                c->src_buf = XG_BUF_STAGE_RECV; c->src_off = rbase + off;
                                c->dst_buf = m->dbuf; c->dst_off = dst_off(&pb, m);
                                c->len = m->len;
                                off += m->len;
                            }
                        }
                        rbase += bucket_b[G + p];
                    } else {
                        for (k = b; k < e; ++k) {
                            const xg_msg *m = &s->msgs[order[k]];
                            if (!moves(m) || xg_gpu_of(s->P, G, m->src) != p || xg_gpu_of(s->P, G, m->dst) != g) continue;
                            {
                                xg_p2p *o = ppush(&pp);
                                o->peer = p; o->is_send = 0; o->buf = m->dbuf;
                                o->off = dst_off(&pb, m); o->len = m->len;
                            }
                        }
                    }
                    dp->remote_recv_bytes += bucket_b[G + p];
                }
            }
            if (soff != sbase && !oom) { fprintf(stderr, "xg_devplan_build: staging mismatch\n"); abort(); }
        }
        sp->p2p_count = pp.n - sp->p2p_begin;
        sp->post_count = post.n - sp->post_begin;
        if (sbase > stage_s_max) stage_s_max = sbase;
        if (rbase > stage_r_max) stage_r_max = rbase;
        for (p = 0; p < G; ++p) {
            os_free(&os_out[p]);
            os_free(&os_in[p]);
        }
        if (oom) goto done;
    }
    /* post copies are stored after the pre copies in one array */
    oom |= pre.fail | post.fail | pp.fail;
    dp->ncopy = pre.n + post.n;
    if (!oom && (dp->copies = (xg_copy *)malloc(sizeof(xg_copy) * (dp->ncopy + 1)))) {
        if (pre.n) memcpy(dp->copies, pre.v, sizeof(xg_copy) * pre.n);
        if (post.n) memcpy(dp->copies + pre.n, post.v, sizeof(xg_copy) * post.n);
        for (st = 0; st < nst; ++st) dp->steps[st].post_begin += pre.n;
        dp->np2p = pp.n;
        dp->p2p = pp.v ? pp.v : (xg_p2p *)malloc(sizeof(xg_p2p));
        if (dp->p2p == pp.v) pp.v = NULL;           /* owned by the plan now */
        dp->region_bytes[XG_BUF_STAGE_SEND] = stage_s_max;
        dp->region_bytes[XG_BUF_STAGE_RECV] = stage_r_max;
    }
    oom |= !dp->copies || !dp->p2p;
done:
    free(pre.v); free(post.v); free(pp.v); free(cnt); free(order); free(pos); free(bucket_n); free(bucket_b);
    free(os_out); free(os_in); free(rl_e); free(rl_i); free(rl_p);
    plan_bases_free(&pb);
    if (oom) {
        xg_devplan_free(dp);
        return NULL;
    }
    return dp;
}

/* ------------------------------------------------------------------ fill / verify descriptors */
int xg_fill_runs(const xg_sched *s, int ngpus, int g, xg_segrun *out)
{
    int lo, hi, r, n = 0;
    xg_block_range(s->P, ngpus, g, &lo, &hi);
    for (r = lo; r < hi; ++r) {
        int ns = nsend_segs(s, r);
        if (!ns) continue;
        if (out) {   /* prepare_*_data: segment i of rank r carries seed i (:106-110, :195-199) */
            out[n].rank = r; out[n].seed0 = 0; out[n].nsegs = ns; out[n].pad = 0;
            out[n].off = xg_send_offset(s, ngpus, r);
        }
        n++;
    }
    return n;
}

int xg_verify_slots(const xg_sched *s, int ngpus, int g, xg_slot *out)
{
    int lo, hi, r, i, n = 0;
    xg_block_range(s->P, ngpus, g, &lo, &hi);
    for (r = lo; r < hi; ++r) {
        int nslots = nrecv_slots(s, r), myindex = 0;
        int64_t base;
        if (!nslots) continue;
        base = xg_recv_offset(s, ngpus, r);
        for (i = 0; i < s->A; ++i)
            if (s->rank_list[i] == r) myindex = i;
        for (i = 0; i < nslots; ++i, ++n) {
            if (!out) continue;
            /* check_buffer call sites: a2m (src=i, seed=myindex) :215; m2a (src=rank_list[i], seed=rank) :139 */
            out[n].src = s->dir == XG_A2M ? i : s->rank_list[i];
            out[n].seed = s->dir == XG_A2M ? myindex : r;
            out[n].dst = r; out[n].pad = 0;
            out[n].off = base + (int64_t)i * s->d;
        }
    }
    return n;
}
