/*
 * programs.c -- per-rank program restatement of methods 1..20 (and TAM m15 / m16).  Plain C99,
 * no HIP.  Each method builder below follows the reference function line by line (cited per
 * function); the only translation is that an MPI call becomes an op appended to the logical
 * rank's program:
 *   Irecv/Issend  -> OP_RECV/OP_SEND post      Waitall -> OP_WAIT
 *   Send/Recv     -> post + OP_WAIT             Sendrecv -> 2 posts + OP_WAIT
 *   Alltoallw     -> OP_A2AW + collective posts + OP_WAIT
 *   memcpy (self) -> OP_COPY                    MPI_Wtime brackets -> OP_TMARK
 * Messages and copies name a logical buffer of their rank (LB_*): the method's
 * send segments / receive slots, or TAM's aggregation buffers, which live in
 * the SCRATCH region; TAM's MPI_INT size arrays are LB_CTRL (host data).
 * sched.c matches the programs' posts into messages and compiles them into steps.
 */
#include "sched_int.h"

#include <limits.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
/* ------------------------------------------------------------------ helpers */
void *xgi_xmalloc(size_t n)
{
    void *p = malloc(n ? n : 1);
    if (!p) { fprintf(stderr, "xg_sched: out of host memory (%zu bytes)\n", n); abort(); }
    return p;
}

void *xgi_xcalloc(size_t n, size_t size)
{
    void *p = calloc(n ? n : 1, size ? size : 1);
    if (!p) { fprintf(stderr, "xg_sched: out of host memory (%zu x %zu bytes)\n", n, size); abort(); }
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
    int64_t *sc = xgi_xmalloc(sizeof(int64_t) * 4 * P), *sd = sc + P, *rc = sc + 2 * P, *rd = sc + 3 * P;
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
    int64_t *sc = xgi_xmalloc(sizeof(int64_t) * 4 * P), *sd = sc + P, *rc = sc + 2 * P, *rd = sc + 3 * P;
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
    int64_t *sc = xgi_xmalloc(sizeof(int64_t) * 4 * P), *sd = sc + P, *rc = sc + 2 * P, *rd = sc + 3 * P;
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
    int64_t *sc = xgi_xmalloc(sizeof(int64_t) * 4 * P), *sd = sc + P, *rc = sc + 2 * P, *rd = sc + 3 * P;
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
    int *map = (int *)xgi_xmalloc(sizeof(int) * P), bblock, send_start;
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
    int64_t *sc = xgi_xmalloc(sizeof(int64_t) * 4 * P), *sd = sc + P, *rc = sc + 2 * P, *rd = sc + 3 * P;
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
        s_lens = (int64_t *)xgi_xmalloc(sizeof(int64_t) * npn * P);
        r_lens = (int64_t *)xgi_xmalloc(sizeof(int64_t) * npn * P);
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


/* ------------------------------------------------------------------ dispatch */
void xgi_program(ctx_t *x)
{
    barrier(x->p);                      /* MPI_Barrier before total_start */
    tstart(x->p, F_TOTAL);
    switch (x->method) {
    case 1: m1_all_to_many(x); break;
    case 2: m2_many_to_all(x); break;
    case 3: m3_balanced(x); break;
    case 4: m4_balanced(x); break;
    case 5: m_alltoallw(x, XG_M2A); break;
    case 6: m6_sync(x); break;
    case 7: m7_half_sync(x); break;
    case 8: m_alltoallw(x, XG_A2M); break;
    case 9: m_pairwise(x, XG_A2M); break;
    case 10: m_pairwise(x, XG_M2A); break;
    case 11: m11_half_sync(x); break;
    case 12: m12_half_sync2(x); break;
    case 13: m13_scattered(x); break;
    case 14: m14_scattered(x); break;
    case 15: case 16: m_tam(x); break;
    case 17: m17_node_robin(x); break;
    case 18: m18_balanced_control(x); break;
    case 19: m19_scattered_isend(x); break;
    case 20: m20_balanced_presend(x); break;
    }
    tstop(x->p, F_TOTAL);
}
