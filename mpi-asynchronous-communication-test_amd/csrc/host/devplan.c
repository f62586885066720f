/*
 * devplan.c -- the per-GPU device plan of a compiled schedule (xg_devplan_build_form): per step,
 * the GPU's local copies, packs into per-peer staging, its RCCL calls in the direct, packed
 * one-sided / two-sided or relay form, and unpacks.  Plain C99, no HIP.  See include/xg_sched.h;
 * the calls each step posts and their pairing proof are calls.c.
 */
#include "sched_int.h"

#include <limits.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

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

/* ---- coalesced relay form (XG_RELAY_COALESCED, xg_sched.h): relay_step's steps, relay_cut's
 * pieces, relay_gpu's hops -- so every link carries what it carries in the relay form -- but one
 * RCCL call per (hop, kind) instead of one per piece.  RCCL serialises the calls of a group to
 * one peer at 2.7-4 us each (profiles/r06/relay_cost.log), and the relay form posts G calls per
 * message and direction: a pairwise round of 4 messages per GPU pair, 112 calls per GPU where
 * the direct form posts 8.  Here GPU g posts:
 *   group 0, per peer p: [pieces of g's messages to p that go straight (piece 0)],
 *                        [pieces of g's messages p relays, by destination];
 *            and receives the same two from p;
 *   group 1, per peer p: [g's own second pieces to p], then per source a (ascending): [the block
 *            of a's group-0 call that g relays to p] -- contiguous in g's STAGE_RECV, so it is
 *            forwarded as it lies; and receives the same from p.
 * A call of one piece moves in place (send from the segment, receive into the slot); a longer one
 * is packed into STAGE_SEND in the step's pre launch and unpacked out of STAGE_RECV after the
 * exchange (HBM copies, two orders of magnitude above a link's rate) -- unless its pieces average
 * >= XG_COALESCE_SPLIT: then it goes one call per piece, in place (rc_split).  STAGE_RECV holds the
 * unpacked receives from 0 on (the layout the device displacement scan rebuilds) and the relayed
 * blocks behind them.  A pairwise round: G - 1 sends + G - 1 receives per group. */
#define XG_WEIGHT_ONE 1024      /* a weighted step's shares: 1/1024ths of each GPU pair's bytes */

typedef struct {
    const xg_sched *s;
    const plan_bases *pb;
    int G, g, dry;          /* dry: only sum the unpacked bytes (the relay area starts behind them) */
    const int *bk, *bk_off; /* the step's cross messages by (source GPU, destination GPU), message order */
    const int *w;           /* weighted step: [(a * G + b) * G + h] = pair (a, b)'s share via h in
                               1/XG_WEIGHT_ONE (weighted_step); NULL: relay_cut's uniform pieces */
    const xg_msg **pm;      /* pieces of the call being built: message, offset in it, length */
    int64_t *po, *pl;
    int64_t *blk;           /* [a * G + b]: where the block of a's pieces for b that g relays lies */
    cvec *pre, *post;
    pvec *pp;
    int64_t sbase, ubase, rlbase, rl;   /* STAGE_SEND fill; STAGE_RECV unpack fill, relay area start / fill */
} rcx;

/* the piece of a message gs -> gd that travels via GPU h (relay_calls' assignment) */
static int rc_piece(int gs, int gd, int h) { return h == gd ? 0 : h == gs ? 1 : 2 + h - (h > gs) - (h > gd); }

/* cut at c / XG_WEIGHT_ONE of a message of len bytes, 16-B aligned (the last cut: len) */
static int64_t wcut(int64_t len, int c) { return c >= XG_WEIGHT_ONE ? len : ((len * c / XG_WEIGHT_ONE) & ~(int64_t)15); }

/* [lo, hi) of message m (a -> b) that travels via h: relay_cut's piece, or a weighted step's share,
 * the shares laid out in hop order (h = 0 .. G-1) */
static void rc_range(const rcx *x, const xg_msg *m, int a, int b, int h, int64_t *lo, int64_t *hi)
{
    if (x->w) {
        const int *w = &x->w[((size_t)a * x->G + b) * x->G];
        int c = 0, k;
        for (k = 0; k < h; ++k) c += w[k];
        *lo = wcut(m->len, c);
        *hi = w[h] ? wcut(m->len, c + w[h]) : *lo;
    } else {
        const int pi = rc_piece(a, b, h);
        *lo = relay_cut(m->len, pi, x->G);
        *hi = relay_cut(m->len, pi + 1, x->G);
    }
}

/* the pieces of the messages a -> b that travel via h (b < 0: every b other than a and h,
 * ascending), each message's in message order -> how many */
static int rc_collect(rcx *x, int a, int b, int h)
{
    const int G = x->G, b0 = b < 0 ? 0 : b, b1 = b < 0 ? G : b + 1;
    int n = 0, bb, k;
    for (bb = b0; bb < b1; ++bb) {
        if (bb == a || (b < 0 && bb == h)) continue;
        for (k = x->bk_off[a * G + bb]; k < x->bk_off[a * G + bb + 1]; ++k) {
            const xg_msg *m = &x->s->msgs[x->bk[k]];
            int64_t lo, hi;
            rc_range(x, m, a, bb, h, &lo, &hi);
            if (hi <= lo) continue;
            x->pm[n] = m; x->po[n] = lo; x->pl[n] = hi - lo; ++n;
        }
    }
    return n;
}

static int64_t rc_total(const rcx *x, int n)
{
    int64_t t = 0;
    int i;
    for (i = 0; i < n; ++i) t += x->pl[i];
    return t;
}

/* a call of n pieces goes one call per piece, in place, when its pieces are large: at >= 4 MiB a
 * piece an RCCL call (~3 us) costs less than packing and unpacking it (2 x its bytes of HBM traffic
 * at ~5 TB/s each way: >= 3 us) -- configs[4]'s 64 MiB segments, whose pieces are 8 MiB.  Both ends
 * of a call apply it to the same piece list, so the calls still pair one to one. */
#define XG_COALESCE_SPLIT ((int64_t)4 << 20)
static int rc_split(const rcx *x, int n) { return n > 1 && rc_total(x, n) >= XG_COALESCE_SPLIT * n; }

/* send the n collected pieces to peer in group grp: in place, or packed into STAGE_SEND */
static void rc_send(rcx *x, int n, int peer, int grp)
{
    int64_t t = 0;
    int i;
    if (!n || x->dry) return;
    if (n == 1 || rc_split(x, n)) {
        for (i = 0; i < n; ++i)
            relay_push(x->pp, peer, 1, x->pm[i]->sbuf, src_off(x->pb, x->pm[i]) + x->po[i], x->pl[i], grp);
        return;
    }
    for (i = 0; i < n; ++i) {
        xg_copy *c = cpush(x->pre);
        c->src_buf = x->pm[i]->sbuf; c->src_off = src_off(x->pb, x->pm[i]) + x->po[i];
        c->dst_buf = XG_BUF_STAGE_SEND; c->dst_off = x->sbase + t;
        c->len = x->pl[i];
        t += x->pl[i];
    }
    relay_push(x->pp, peer, 1, XG_BUF_STAGE_SEND, x->sbase, t, grp);
    x->sbase += t;
}

/* receive the n collected pieces (all ending at this GPU) from peer: in place, or into the unpack
 * area of STAGE_RECV with one unpack copy per piece */
static void rc_recv(rcx *x, int n, int peer, int grp)
{
    int64_t t = 0;
    int i;
    if (!n) return;
    if (n == 1 || rc_split(x, n)) {
        for (i = 0; i < n && !x->dry; ++i)
            relay_push(x->pp, peer, 0, x->pm[i]->dbuf, dst_off(x->pb, x->pm[i]) + x->po[i], x->pl[i], grp);
        return;
    }
    for (i = 0; i < n && !x->dry; ++i) {
        xg_copy *c = cpush(x->post);
        c->src_buf = XG_BUF_STAGE_RECV; c->src_off = x->ubase + t;
        c->dst_buf = x->pm[i]->dbuf; c->dst_off = dst_off(x->pb, x->pm[i]) + x->po[i];
        c->len = x->pl[i];
        t += x->pl[i];
    }
    if (x->dry) t = rc_total(x, n);
    else relay_push(x->pp, peer, 0, XG_BUF_STAGE_RECV, x->ubase, t, grp);
    x->ubase += t;
}

/* GPU g's calls of one relayed step (dry: only the unpack area's size, x->ubase) */
static void rc_step(rcx *x)
{
    const int G = x->G, g = x->g;
    int p, a, b, n;
    for (p = 0; p < G; ++p) {           /* group 0 */
        if (p == g) continue;
        rc_send(x, rc_collect(x, g, p, p), p, 0);
        rc_send(x, rc_collect(x, g, -1, p), p, 0);
        rc_recv(x, rc_collect(x, p, g, g), p, 0);
        n = rc_collect(x, p, -1, g);    /* what g relays for p: one receive into the relay area */
        if (n && !x->dry) {
            const int64_t at = x->rlbase + x->rl;
            int64_t t = 0;
            if (rc_split(x, n))         /* (or one per piece, as the sender splits them) */
                for (b = 0; b < n; ++b) {
                    relay_push(x->pp, p, 0, XG_BUF_STAGE_RECV, at + t, x->pl[b], 0);
                    t += x->pl[b];
                }
            else
                relay_push(x->pp, p, 0, XG_BUF_STAGE_RECV, at, rc_total(x, n), 0);
            for (t = 0, b = 0; b < G; ++b) {
                if (b == p || b == g) continue;
                x->blk[p * G + b] = at + t;
                t += rc_total(x, rc_collect(x, p, b, g));
            }
            x->rl += t;
        }
    }
    for (p = 0; p < G; ++p) {           /* group 1 */
        if (p == g) continue;
        rc_send(x, rc_collect(x, g, p, g), p, 1);
        for (a = 0; a < G && !x->dry; ++a)
            if (a != g && a != p && (n = rc_collect(x, a, p, g))) {
                /* the block of a's pieces for p, as it lies (one call, or one per piece) */
                int64_t at = x->blk[a * G + p];
                if (rc_split(x, n))
                    for (b = 0; b < n; at += x->pl[b], ++b) relay_push(x->pp, p, 1, XG_BUF_STAGE_RECV, at, x->pl[b], 1);
                else
                    relay_push(x->pp, p, 1, XG_BUF_STAGE_RECV, at, rc_total(x, n), 1);
            }
        rc_recv(x, rc_collect(x, p, g, p), p, 1);
        for (a = 0; a < G; ++a)
            if (a != g && a != p) rc_recv(x, rc_collect(x, a, g, p), p, 1);
    }
}

/* ---- weighted two-hop split (XG_RELAY_COALESCED on a step relay_step leaves direct).  A traffic
 * matrix that is not a permutation -- configs[4]'s m7 (mpi_test.c:942-997): every GPU sends 512 MiB
 * to each of 3-4 others per step, some GPUs receive from 4 -- gains nothing from the uniform cut
 * ((max egress + max ingress) / G is not below its busiest pair), yet a non-uniform one exists: the
 * best two-hop routing in two groups carries 0.78 of the direct form's busiest-link bytes
 * (profiles/r05/relay_lp.txt, an LP).  Per step, Frank-Wolfe on a soft-max of the busiest group-0
 * and group-1 links (profiles/relay_lp.py's fw_two_hop, here in C, 1000 iterations): every pair's bytes split over
 * its G paths -- straight in group 0 (h = b), straight in group 1 (h = a), via relay h -- starting
 * half straight in each group; each iteration moves 2 / (t + 3) of every pair onto its cheapest
 * path under the current gradient.  The best split seen is rounded to 1/1024ths (shares under
 * 16/1024 go to the pair's largest: each more hop is one more call), and the step is weighted
 * when its quantised link time is at
 * most XG_WEIGHTED_GAIN of the busiest pair's and every cross message is >= XG_RELAY_MIN_BYTES.
 * Deterministic: every GPU computes it from the same message list with the same code. */
#define XG_FW_ITERS 1000
#define XG_FW_SHARP 80.0
#define XG_WEIGHTED_GAIN 0.85

/* group-0 / group-1 link loads of split y (pairs pr[np][2], y[np][G] bytes) -> max l0 + max l1 */
static double fw_cost(int G, int np, const int *pr, const double *y, double *l0, double *l1)
{
    int i, h, k;
    double m0 = 0, m1 = 0;
    memset(l0, 0, sizeof(double) * (size_t)G * G);
    memset(l1, 0, sizeof(double) * (size_t)G * G);
    for (i = 0; i < np; ++i) {
        const int a = pr[2 * i], b = pr[2 * i + 1];
        for (h = 0; h < G; ++h) {
            if (h != a) l0[a * G + h] += y[i * G + h];
            if (h != b) l1[h * G + b] += y[i * G + h];
        }
    }
    for (k = 0; k < G * G; ++k) {
        m0 = l0[k] > m0 ? l0[k] : m0;
        m1 = l1[k] > m1 ? l1[k] : m1;
    }
    return m0 + m1;
}

/* The split is a pure function of the step's GPU-pair matrix, and every GPU's plan (each rank
 * builds all G of them for the pairing proof) asks for the same steps: a per-thread memo of the last
 * XG_FW_MEMO matrices (G <= 8), matched on the exact matrix, answers the repeats. */
#define XG_FW_MEMO 256
typedef struct { int G, rc; uint64_t key; double D[64]; int w[512]; } fw_memo;
static __thread fw_memo *fw_memo_tab;
static __thread unsigned fw_memo_next;

static uint64_t fw_key(const double *D, int n)
{
    uint64_t hsh = 1469598103934665603ull;
    int i;
    for (i = 0; i < n; ++i) {
        uint64_t v;
        memcpy(&v, &D[i], sizeof v);
        hsh = (hsh ^ v) * 1099511628211ull;
    }
    return hsh;
}

/* the memo entry of matrix D (G x G), or NULL */
static const fw_memo *fw_memo_find(const double *D, int G, uint64_t key)
{
    unsigned i;
    if (!fw_memo_tab || G > 8) return NULL;
    for (i = 0; i < XG_FW_MEMO; ++i)
        if (fw_memo_tab[i].G == G && fw_memo_tab[i].key == key &&
            !memcmp(fw_memo_tab[i].D, D, sizeof(double) * (size_t)G * G))
            return &fw_memo_tab[i];
    return NULL;
}

static void fw_memo_put(const double *D, int G, uint64_t key, const int *w, int rc)
{
    fw_memo *m;
    if (G > 8) return;
    if (!fw_memo_tab && !(fw_memo_tab = (fw_memo *)calloc(XG_FW_MEMO, sizeof(fw_memo)))) return;
    m = &fw_memo_tab[fw_memo_next++ % XG_FW_MEMO];
    m->G = G; m->rc = rc; m->key = key;
    memcpy(m->D, D, sizeof(double) * (size_t)G * G);
    memcpy(m->w, w, sizeof(int) * (size_t)G * G * G);
}

/* The weighted split of step [b, e) into w[(a * G + b) * G + h] (1/XG_WEIGHT_ONE) -> 1 when the
 * step is to be weighted, 0 when it stays direct, -1 out of host memory */
static int weighted_step(const xg_sched *s, const int *order, int b, int e, int G, int *w)
{
    uint64_t key = 0;
    const fw_memo *hit;
    int k, i, h, np = 0, t, rc = -1;
    double direct = 0, best = -1, cost;
    double *D = (double *)calloc((size_t)G * G, sizeof(double));
    int *pr = (int *)malloc(sizeof(int) * 2 * (size_t)G * G);
    double *y = (double *)calloc((size_t)G * G * G, sizeof(double)), *yb = (double *)calloc((size_t)G * G * G, sizeof(double));
    double *l0 = (double *)malloc(sizeof(double) * (size_t)G * G), *l1 = (double *)malloc(sizeof(double) * (size_t)G * G);
    double *g0 = (double *)malloc(sizeof(double) * (size_t)G * G), *g1 = (double *)malloc(sizeof(double) * (size_t)G * G);
    if (!D || !pr || !y || !yb || !l0 || !l1 || !g0 || !g1) goto done;
    rc = 0;
    if (G < 3) goto done;
    for (k = b; k < e; ++k) {
        const xg_msg *m = &s->msgs[order[k]];
        const int gs = xg_gpu_of(s->P, G, m->src), gd = xg_gpu_of(s->P, G, m->dst);
        if (!moves(m) || is_stage(m) || gs == gd) continue;
        if (m->len < XG_RELAY_MIN_BYTES) goto done;
        D[gs * G + gd] += (double)m->len;
    }
    for (i = 0; i < G * G; ++i) {
        direct = D[i] > direct ? D[i] : direct;
        if (D[i] > 0) {
            pr[2 * np] = i / G;
            pr[2 * np + 1] = i % G;
            y[(size_t)np * G + i / G] = y[(size_t)np * G + i % G] = D[i] / 2;   /* half straight in each group */
            ++np;
        }
    }
    if (!np) goto done;
    key = fw_key(D, G * G);
    if ((hit = fw_memo_find(D, G, key))) {
        memcpy(w, hit->w, sizeof(int) * (size_t)G * G * G);
        rc = hit->rc;
        goto done;
    }
    for (t = 0; t <= XG_FW_ITERS; ++t) {
        double m0 = 0, m1 = 0, z0 = 0, z1 = 0, beta;
        cost = fw_cost(G, np, pr, y, l0, l1);
        if (best < 0 || cost < best) {
            best = cost;
            memcpy(yb, y, sizeof(double) * (size_t)np * G);
        }
        if (t == XG_FW_ITERS) break;
        for (k = 0; k < G * G; ++k) {
            m0 = l0[k] > m0 ? l0[k] : m0;
            m1 = l1[k] > m1 ? l1[k] : m1;
        }
        beta = XG_FW_SHARP / cost;
        for (k = 0; k < G * G; ++k) {       /* links far below the busiest weigh nothing (< e^-30) */
            const double e0 = beta * (l0[k] - m0), e1 = beta * (l1[k] - m1);
            g0[k] = e0 > -30.0 ? exp(e0) : 0.0;
            g1[k] = e1 > -30.0 ? exp(e1) : 0.0;
            z0 += g0[k];
            z1 += g1[k];
        }
        for (k = 0, z0 = 1.0 / z0, z1 = 1.0 / z1; k < G * G; ++k) {     /* soft-max weights */
            g0[k] *= z0;
            g1[k] *= z1;
        }
        for (i = 0; i < np; ++i) {
            const int a = pr[2 * i], bb = pr[2 * i + 1];
            const double step = 2.0 / (t + 3), dem = D[a * G + bb];
            int arg = 0;
            double cmin = 0;
            for (h = 0; h < G; ++h) {
                const double c = (h != a ? g0[a * G + h] : 0.0) + (h != bb ? g1[h * G + bb] : 0.0);
                if (h == 0 || c < cmin) { cmin = c; arg = h; }
            }
            for (h = 0; h < G; ++h) y[(size_t)i * G + h] += step * ((h == arg ? dem : 0.0) - y[(size_t)i * G + h]);
        }
    }
    /* quantise the best split: 1/1024ths, small shares folded into the pair's largest */
    memset(w, 0, sizeof(int) * (size_t)G * G * G);
    for (i = 0; i < np; ++i) {
        const int a = pr[2 * i], bb = pr[2 * i + 1];
        int *wp = &w[((size_t)a * G + bb) * G], sum = 0, big = 0;
        for (h = 0; h < G; ++h) {
            const int q = (int)(yb[(size_t)i * G + h] / D[a * G + bb] * XG_WEIGHT_ONE + 0.5);
            wp[h] = q >= 16 ? q : 0;
            sum += wp[h];
            if (wp[h] > wp[big]) big = h;
        }
        wp[big] += XG_WEIGHT_ONE - sum;
        for (h = 0; h < G; ++h) yb[(size_t)i * G + h] = D[a * G + bb] * wp[h] / XG_WEIGHT_ONE;
    }
    rc = fw_cost(G, np, pr, yb, l0, l1) <= XG_WEIGHTED_GAIN * direct;
    fw_memo_put(D, G, key, w, rc);
done:
    free(D); free(pr); free(y); free(yb); free(l0); free(l1); free(g0); free(g1);
    return rc;
}

/* the coalesced relay calls of step [b, e) for GPU g: packs into pre, calls into pp, unpacks into
 * post; *sbase / *rbase: the step's STAGE_SEND / STAGE_RECV bytes.  -> 0, or -1 out of host memory */
static int relay_coalesced_calls(const xg_sched *s, const plan_bases *pb, const int *order, int b, int e, int G,
                                 int g, const int *w, cvec *pre, pvec *pp, cvec *post, int64_t *sbase, int64_t *rbase)
{
    int k, rc = -1;
    int *bk_off = (int *)calloc((size_t)G * G + 1, sizeof(int)), *fill = (int *)calloc((size_t)G * G, sizeof(int));
    int *bk = (int *)malloc(sizeof(int) * ((size_t)(e - b) + 1));
    const xg_msg **pm = (const xg_msg **)malloc(sizeof(xg_msg *) * ((size_t)(e - b) + 1));
    int64_t *po = (int64_t *)malloc(sizeof(int64_t) * ((size_t)(e - b) + 1));
    int64_t *pl = (int64_t *)malloc(sizeof(int64_t) * ((size_t)(e - b) + 1));
    int64_t *blk = (int64_t *)calloc((size_t)G * G, sizeof(int64_t));
    rcx x;
    if (!bk_off || !fill || !bk || !pm || !po || !pl || !blk) goto done;
    for (k = b; k < e; ++k) {
        const xg_msg *m = &s->msgs[order[k]];
        const int gs = xg_gpu_of(s->P, G, m->src), gd = xg_gpu_of(s->P, G, m->dst);
        if (moves(m) && !is_stage(m) && gs != gd) bk_off[gs * G + gd + 1]++;
    }
    for (k = 0; k < G * G; ++k) bk_off[k + 1] += bk_off[k];
    for (k = b; k < e; ++k) {
        const xg_msg *m = &s->msgs[order[k]];
        const int gs = xg_gpu_of(s->P, G, m->src), gd = xg_gpu_of(s->P, G, m->dst);
        if (moves(m) && !is_stage(m) && gs != gd) bk[bk_off[gs * G + gd] + fill[gs * G + gd]++] = order[k];
    }
    memset(&x, 0, sizeof x);
    x.s = s; x.pb = pb; x.G = G; x.g = g; x.bk = bk; x.bk_off = bk_off; x.pm = pm; x.po = po; x.pl = pl;
    x.blk = blk; x.pre = pre; x.post = post; x.pp = pp; x.w = w;
    x.dry = 1;
    rc_step(&x);                        /* the unpack area's size: the relay area goes behind it */
    x.rlbase = x.ubase;
    x.ubase = 0;
    x.dry = 0;
    rc_step(&x);
    *sbase = x.sbase;
    *rbase = x.rlbase + x.rl;
    rc = 0;
done:
    free(bk_off); free(fill); free(bk); free(pm); free(po); free(pl); free(blk);
    return rc;
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
    int *rl_w = (int *)calloc((size_t)G * G * G, sizeof(int));       /* a weighted step's shares */
    plan_bases pb;
    memset(&pre, 0, sizeof pre); memset(&post, 0, sizeof post); memset(&pp, 0, sizeof pp);
    memset(&pb, 0, sizeof pb);
    if (form != XG_PACK_TWO_SIDED && form != XG_PACK_ONE_SIDED && form != XG_RELAY && form != XG_RELAY_COALESCED)
        form = XG_PACK_FORM_DEFAULT;
    if (form == XG_RELAY || form == XG_RELAY_COALESCED) pack_max_seg = 0;   /* every other step is direct */
    if (!dp || !cnt || !order || !pos || !bucket_n || !bucket_b || !os_out || !os_in || !rl_e || !rl_i || !rl_p || !rl_w ||
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
        xgi_step_posts_of(s, G, g, posts, nst);
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
        int b = cnt[st], e = cnt[st + 1], k, p, relayed, weighted;
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
        sp->p2p_begin = pp.n;
        sp->post_begin = post.n;
        relayed = (form == XG_RELAY || form == XG_RELAY_COALESCED) && relay_step(s, order, b, e, G, rl_e, rl_i, rl_p);
        weighted = 0;
        if (!relayed && form == XG_RELAY_COALESCED) {
            /* a step the uniform cut does not help may still take a weighted two-hop split */
            const int ws = weighted_step(s, order, b, e, G, rl_w);
            oom |= ws < 0;
            weighted = ws > 0;
        }
        /* coalesced relay: its packs follow the local copies in the pre launch */
        if ((relayed || weighted) && form == XG_RELAY_COALESCED)
            oom |= relay_coalesced_calls(s, &pb, order, b, e, G, g, weighted ? rl_w : NULL, &pre, &pp, &post, &sbase,
                                         &rbase) != 0;
        relayed |= weighted;
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
        if (relayed) {
            /* every message over all G - 1 links of its source, then of its destination (two groups) */
            if (form == XG_RELAY) relay_calls(s, &pb, order, b, e, G, g, &pp, &rbase);
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
    free(os_out); free(os_in); free(rl_e); free(rl_i); free(rl_p); free(rl_w);
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
        int ns = xgi_nsend_segs(s, r);
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
        int nslots = xgi_nrecv_slots(s, r), myindex = 0;
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
