/*
 * sched_int.h -- internals shared by the host schedule's translation units (libxghost, not
 * installed, not part of the C-ABI): the per-rank op programs the method restatements build
 * (programs.c), the schedule object matching and the step compiler fill (sched.c), and what the
 * device-plan builder (devplan.c) reads of it.  See include/xg_sched.h for the public side.
 */
#ifndef XG_SCHED_INT_H
#define XG_SCHED_INT_H

#include "xg_sched.h"

#include <stddef.h>
#include <stdint.h>

#define XGI __attribute__((visibility("hidden")))

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

/* one logical rank's method restatement in progress (programs.c) */
typedef struct {
    prog_t *p;
    int rank, isagg, myindex, P, A, c, ntimes, proc_node, barrier_type;
    int64_t d;
    const int *rl;
    int method, iter;
    const int *isagg_all;   /* [P] */
    const int *lastidx;     /* [P] last i with rl[i] == rank, -1 if none */
} ctx_t;

XGI void *xgi_xmalloc(size_t n);              /* abort on out of host memory */
XGI void *xgi_xcalloc(size_t n, size_t size);
/* the rank's whole program: MPI_Barrier, total_start, the method body, total_end */
XGI void xgi_program(ctx_t *x);
/* segments a rank sends / slots it receives (its share of SEND / RECV) */
XGI int xgi_nsend_segs(const xg_sched *s, int r);
XGI int xgi_nrecv_slots(const xg_sched *s, int r);
/* the request posts of GPU g's ranks per step (out[nout], zeroed here) */
XGI void xgi_step_posts_of(const xg_sched *s, int ngpus, int g, int32_t *out, int nout);

#endif
