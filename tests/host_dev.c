/*
 * host_dev.c -- TEST INFRASTRUCTURE ONLY: a CPU stand-in for the device half of the
 * ABI (include/xg.h: context, regions, fill/verify, plans, barrier, allreduce), so
 * the CLI's multi-process path -- bin/test --gpus N: spawn, rendezvous, argument
 * digest, per-method schedule + pairing check, plan run, report -- runs on a machine
 * without GPUs (tests/test_cli_host_dev.py links it with main.c, rdzv.c, methods.c
 * and the host sources).  Never linked into the product (lib/libxg.so).
 *
 * It executes a device plan the way the runtime's enqueue_step orders it: stage
 * copies, the other pre copies (local gather/scatter and packs), the step's call
 * list exactly as xg_devplan_step_calls defines it (self send/recv pairs standing
 * in for the local copies when the step qualifies under XG_SELF_MAX), then the
 * unpacks, then the barrier.  Sends and receives travel through files in a
 * directory shared by the job's processes: message k from GPU g to GPU h is file
 * m_<g>_<h>_<k> -- RCCL's per-peer FIFO.  A receive whose message has a different
 * length fails the run (RCCL would corrupt or hang), as does a receive that waits
 * longer than XG_HOST_DEV_TIMEOUT seconds (default 60).
 *
 * XG_HOST_DEV_DIR (required for nranks > 1): parent of the job's message directory,
 * named by the unique id rank 0 hands over.  XG_HOST_DEV_CORRUPT=<g>: GPU g flips
 * one byte of every message it receives (the verify path must see it).
 * XG_HOST_DEV_FAIL_ALLOC=<g>: GPU g's region allocations fail (XG_ENOMEM), as hipMalloc
 * does when HBM is exhausted -- every rank must then stop alike.
 */
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "xg.h"
#include "xg_sched.h"

struct xg_ctx {
    int rank, nranks, corrupt, fail_alloc;
    int64_t self_max;          /* XG_SELF_MAX, as the runtime reads it at xg_init */
    char dir[3072];
    int64_t *sent, *recvd;     /* per peer: messages posted / taken */
    int64_t coll;              /* collectives so far */
    double timeout;
};

struct xg_regions {
    xg_ctx *ctx;
    unsigned char *p[XG_NBUF];
    int64_t n[XG_NBUF];
};

struct xg_plan {
    xg_ctx *ctx;
    xg_regions *r;
    const xg_devplan *dp;
    int64_t self_max;
    unsigned char *need;   /* xg_plan_set_step_marks: NULL = every step marked */
};

double xg_now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void nap(void)
{
    struct timespec ts = {0, 50000};
    nanosleep(&ts, NULL);
}

int xg_get_unique_id(void *uid)
{
    unsigned char *u = (unsigned char *)uid;
    uint64_t x = (uint64_t)getpid() * 0x9E3779B97F4A7C15ull ^ (uint64_t)(xg_now() * 1e9);
    int i;
    for (i = 0; i < XG_UNIQUE_ID_BYTES; ++i) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        u[i] = (unsigned char)x;
    }
    return XG_OK;
}

int xg_init(xg_ctx **out, int rank, int nranks, int device, const void *uid)
{
    xg_ctx *c;
    const char *env;
    (void)device;
    *out = NULL;
    if (nranks < 1 || rank < 0 || rank >= nranks) return XG_EARG;
    c = (xg_ctx *)calloc(1, sizeof *c);
    if (!c) return XG_ENOMEM;
    c->rank = rank;
    c->nranks = nranks;
    c->sent = (int64_t *)calloc(nranks, sizeof(int64_t));
    c->recvd = (int64_t *)calloc(nranks, sizeof(int64_t));
    env = getenv("XG_HOST_DEV_CORRUPT");
    c->corrupt = env ? atoi(env) : -1;
    env = getenv("XG_HOST_DEV_FAIL_ALLOC");
    c->fail_alloc = env ? atoi(env) == rank : 0;
    env = getenv("XG_SELF_MAX");
    c->self_max = env ? atoll(env) : (int64_t)256 << 10;
    env = getenv("XG_HOST_DEV_TIMEOUT");
    c->timeout = env ? atof(env) : 60.0;
    env = getenv("XG_HOST_DEV_DIR");
    if (nranks > 1) {
        const unsigned char *u = (const unsigned char *)uid;
        int i, n;
        if (!env || !uid) { fprintf(stderr, "host_dev: XG_HOST_DEV_DIR and a unique id needed\n"); return XG_EARG; }
        n = snprintf(c->dir, sizeof c->dir - 40, "%s/job_", env);
        for (i = 0; i < 8; ++i) n += snprintf(c->dir + n, 3, "%02x", u[i]);
        if (mkdir(c->dir, 0700) && errno != EEXIST) { perror(c->dir); return XG_EHIP; }
    }
    *out = c;
    return XG_OK;
}

int xg_finalize(xg_ctx *c)
{
    if (!c) return XG_OK;
    free(c->sent);
    free(c->recvd);
    free(c);
    return XG_OK;
}

int xg_rank(const xg_ctx *c) { return c->rank; }
int64_t xg_self_max(const xg_ctx *c) { return c->self_max; }
int xg_nranks(const xg_ctx *c) { return c->nranks; }

static int put_file(const char *dir, const char *name, const void *p, size_t n)
{
    char tmp[4096], path[4096];
    FILE *f;
    snprintf(tmp, sizeof tmp, "%s/.%s", dir, name);
    snprintf(path, sizeof path, "%s/%s", dir, name);
    f = fopen(tmp, "wb");
    if (!f) { perror(tmp); return XG_EHIP; }
    if (n && fwrite(p, 1, n, f) != n) { perror(tmp); fclose(f); return XG_EHIP; }
    fclose(f);
    if (rename(tmp, path)) { perror(path); return XG_EHIP; }
    return XG_OK;
}

/* wait for dir/name; its size in *n */
static int wait_file(const xg_ctx *c, const char *name, char *path, size_t pathlen, int64_t *n)
{
    struct stat st;
    double t0 = xg_now();
    snprintf(path, pathlen, "%s/%s", c->dir, name);
    while (stat(path, &st)) {
        if (xg_now() - t0 > c->timeout) {
            fprintf(stderr, "host_dev: GPU %d waited %.0f s for %s\n", c->rank, c->timeout, name);
            return XG_ERCCL;
        }
        nap();
    }
    *n = (int64_t)st.st_size;
    return XG_OK;
}

int xg_allreduce_max(xg_ctx *c, double *vals, int n)
{
    char name[64], path[4096];
    double *in;
    int64_t seq, sz;
    int r, i, rc;
    if (n < 0) return XG_EARG;
    if (c->nranks == 1) return XG_OK;
    seq = c->coll++;
    if (seq >= 2) {   /* every rank has read round seq-2: it entered round seq-1 */
        snprintf(path, sizeof path, "%s/a_%lld_%d", c->dir, (long long)(seq - 2), c->rank);
        unlink(path);
    }
    snprintf(name, sizeof name, "a_%lld_%d", (long long)seq, c->rank);
    if ((rc = put_file(c->dir, name, vals, sizeof(double) * (size_t)n))) return rc;
    in = (double *)malloc(sizeof(double) * (size_t)(n + 1));
    for (r = 0; r < c->nranks; ++r) {
        FILE *f;
        if (r == c->rank) continue;
        snprintf(name, sizeof name, "a_%lld_%d", (long long)seq, r);
        if ((rc = wait_file(c, name, path, sizeof path, &sz))) break;
        if (sz != (int64_t)sizeof(double) * n) {
            fprintf(stderr, "host_dev: allreduce %lld: GPU %d sent %lld values, GPU %d %d\n", (long long)seq, r,
                    (long long)(sz / 8), c->rank, n);
            rc = XG_ERCCL;
            break;
        }
        f = fopen(path, "rb");
        if (!f || (n && fread(in, sizeof(double), (size_t)n, f) != (size_t)n)) { rc = XG_EHIP; if (f) fclose(f); break; }
        fclose(f);
        for (i = 0; i < n; ++i)
            if (in[i] > vals[i]) vals[i] = in[i];
    }
    free(in);
    return rc;
}

int xg_barrier(xg_ctx *c)
{
    return xg_allreduce_max(c, NULL, 0);
}

/* ------------------------------------------------------------------ regions */
int xg_regions_alloc(xg_ctx *c, const int64_t region_bytes[XG_NBUF], xg_regions **out)
{
    xg_regions *r = (xg_regions *)calloc(1, sizeof *r);
    int b;
    *out = NULL;
    if (!r) return XG_ENOMEM;
    if (c->fail_alloc) {
        free(r);
        fprintf(stderr, "host_dev: GPU %d: region allocation fails (XG_HOST_DEV_FAIL_ALLOC)\n", c->rank);
        return XG_ENOMEM;
    }
    r->ctx = c;
    for (b = 0; b < XG_NBUF; ++b) {
        r->n[b] = region_bytes[b];
        r->p[b] = (unsigned char *)malloc(region_bytes[b] > 0 ? (size_t)region_bytes[b] : 1);
        if (!r->p[b]) { xg_regions_free(r); return XG_ENOMEM; }
        memset(r->p[b], 0xA5, region_bytes[b] > 0 ? (size_t)region_bytes[b] : 1);   /* not the fingerprint */
    }
    *out = r;
    return XG_OK;
}

int xg_regions_free(xg_regions *r)
{
    int b;
    if (!r) return XG_OK;
    for (b = 0; b < XG_NBUF; ++b) free(r->p[b]);
    free(r);
    return XG_OK;
}

/* fingerprints of oracle/xg_oracle.py (map_data, strong_data) */
static uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static unsigned char fp_byte(int mode, int rank, int seed, int it, int64_t o)
{
    if (mode == XG_FP_REFERENCE) return (unsigned char)((rank + seed + it + o) & 0xFF);
    {
        uint64_t key = ((uint64_t)rank << 42) ^ ((uint64_t)seed << 21) ^ (uint64_t)it;
        uint64_t w = mix64(key + (uint64_t)(o >> 3) * 0x9E3779B97F4A7C15ull);
        return (unsigned char)(w >> (8 * (o & 7)));
    }
}

static int inside(const xg_regions *r, int buf, int64_t off, int64_t len)
{
    return buf >= 0 && buf < XG_NBUF && off >= 0 && len >= 0 && off + len <= r->n[buf];
}

int xg_fill(xg_regions *r, const xg_segrun *runs, int nruns, int64_t d, int iter, int mode)
{
    int i, q;
    int64_t o;
    for (i = 0; i < nruns; ++i) {
        if (!inside(r, XG_BUF_SEND, runs[i].off, d * runs[i].nsegs)) return XG_EARG;
        for (q = 0; q < runs[i].nsegs; ++q) {
            unsigned char *p = r->p[XG_BUF_SEND] + runs[i].off + (int64_t)q * d;
            for (o = 0; o < d; ++o) p[o] = fp_byte(mode, runs[i].rank, runs[i].seed0 + q, iter, o);
        }
    }
    return XG_OK;
}

int xg_verify(xg_regions *r, const xg_slot *slots, int nslots, int64_t d, int iter, int mode, uint64_t *chk,
              int64_t *bad, int64_t *first_bad)
{
    int i;
    int64_t o;
    for (i = 0; i < nslots; ++i) {
        const unsigned char *p;
        int64_t nbad = 0, first = -1;
        uint64_t sum = 0;
        if (!inside(r, XG_BUF_RECV, slots[i].off, d)) return XG_EARG;
        p = r->p[XG_BUF_RECV] + slots[i].off;
        for (o = 0; o < d; ++o)
            if (p[o] != fp_byte(mode, slots[i].src, slots[i].seed, iter, o)) {
                if (first < 0) first = o;
                ++nbad;
            }
        for (o = 0; o < d; o += 8) {   /* xg_chk64 */
            uint64_t w = 0;
            int k;
            for (k = 0; k < 8 && o + k < d; ++k) w |= (uint64_t)p[o + k] << (8 * k);
            sum += mix64(w ^ (uint64_t)(o >> 3) * 0x9E3779B97F4A7C15ull);
        }
        sum += (uint64_t)d * 0xD6E8FEB86659FD93ull;
        if (chk) chk[i] = sum;
        if (bad) bad[i] = nbad;
        if (first_bad) first_bad[i] = first;
    }
    return XG_OK;
}

/* ------------------------------------------------------------------ plans */
int xg_plan_load(xg_ctx *c, xg_regions *r, const xg_devplan *dp, xg_plan **out)
{
    xg_plan *p;
    int i;
    *out = NULL;
    if (!dp || dp->gpu != c->rank || dp->ngpus != c->nranks) return XG_EARG;
    for (i = 0; i < dp->ncopy; ++i) {
        const xg_copy *k = &dp->copies[i];
        if (!inside(r, k->src_buf, k->src_off, k->len) || !inside(r, k->dst_buf, k->dst_off, k->len)) return XG_EARG;
    }
    for (i = 0; i < dp->np2p; ++i)
        if (!inside(r, dp->p2p[i].buf, dp->p2p[i].off, dp->p2p[i].len) || dp->p2p[i].peer < 0 ||
            dp->p2p[i].peer >= c->nranks)
            return XG_EARG;
    p = (xg_plan *)calloc(1, sizeof *p);
    if (!p) return XG_ENOMEM;
    p->ctx = c;
    p->r = r;
    p->dp = dp;
    p->self_max = c->nranks > 1 ? c->self_max : 0;
    *out = p;
    return XG_OK;
}

int xg_plan_free(xg_plan *p)
{
    if (p) free(p->need);
    free(p);
    return XG_OK;
}

static void copy(xg_regions *r, const xg_copy *k)
{
    if (k->len > 0) memmove(r->p[k->dst_buf] + k->dst_off, r->p[k->src_buf] + k->src_off, (size_t)k->len);
}

static int send_msg(xg_ctx *c, int peer, const unsigned char *src, int64_t len)
{
    char name[96];
    snprintf(name, sizeof name, "m_%d_%d_%lld", c->rank, peer, (long long)c->sent[peer]++);
    return put_file(c->dir, name, src, (size_t)len);
}

static int recv_msg(xg_ctx *c, int peer, unsigned char *dst, int64_t len)
{
    char name[96], path[4096];
    int64_t sz;
    FILE *f;
    int rc;
    snprintf(name, sizeof name, "m_%d_%d_%lld", peer, c->rank, (long long)c->recvd[peer]++);
    if ((rc = wait_file(c, name, path, sizeof path, &sz))) return rc;
    if (sz != len) {
        fprintf(stderr, "host_dev: GPU %d receive from %d: %lld bytes posted, %lld sent\n", c->rank, peer,
                (long long)len, (long long)sz);
        return XG_ERCCL;
    }
    f = fopen(path, "rb");
    if (!f || (sz && fread(dst, 1, (size_t)sz, f) != (size_t)sz)) { if (f) fclose(f); return XG_EHIP; }
    fclose(f);
    unlink(path);
    if (c->corrupt == c->rank && sz) dst[sz / 2] ^= 0x5A;
    return XG_OK;
}

int xg_plan_set_step_marks(xg_plan *p, const uint8_t *need)
{
    int s;
    if (!p) return XG_EARG;
    free(p->need);
    p->need = NULL;
    if (!need) return XG_OK;
    p->need = (unsigned char *)malloc((size_t)p->dp->nsteps + 1);
    if (!p->need) return XG_ENOMEM;
    for (s = 0; s < p->dp->nsteps; ++s) p->need[s] = need[s] || s == p->dp->nsteps - 1;
    return XG_OK;
}

int xg_plan_run(xg_plan *p, double *step_done, double *step_post, double *wall)
{
    xg_ctx *c = p->ctx;
    xg_regions *r = p->r;
    const xg_devplan *dp = p->dp;
    const double t0 = xg_now();
    xg_call *calls = NULL;
    int s, i, rc = XG_OK, cap = 0;
    for (s = 0; s < dp->nsteps && !rc; ++s) {
        const xg_stepplan *sp = &dp->steps[s];
        const int self = xg_devplan_step_self_calls(dp, s, p->self_max) > 0;
        int n = xg_devplan_step_calls(dp, s, p->self_max, NULL), local_end = sp->pre_begin + sp->stage_count;
        if (n > cap) {
            cap = n;
            calls = (xg_call *)realloc(calls, sizeof(xg_call) * (size_t)cap);
        }
        xg_devplan_step_calls(dp, s, p->self_max, calls);
        if (self)   /* the local copies (calls.c local_range) travel as the self pairs */
            while (local_end < sp->pre_begin + sp->pre_count && dp->copies[local_end].dst_buf != XG_BUF_STAGE_SEND)
                ++local_end;
        for (i = sp->pre_begin; i < sp->pre_begin + sp->pre_count; ++i)
            if (!self || i < sp->pre_begin + sp->stage_count || i >= local_end) copy(r, &dp->copies[i]);
        for (int g0 = 0; g0 < n && !rc;) {   /* per group (a relay step: two, split by a fence) */
            int g1 = g0;
            while (g1 < n && calls[g1].kind != XG_CALL_FENCE && calls[g1].kind != XG_CALL_BARRIER) ++g1;
            for (i = g0; i < g1 && !rc; ++i)     /* the group: every send posted, then every receive */
                if (calls[i].kind == XG_CALL_SEND)
                    rc = c->nranks == 1 ? XG_EARG   /* a one-GPU plan posts no calls */
                                        : send_msg(c, calls[i].peer, r->p[calls[i].buf] + calls[i].off, calls[i].len);
            for (i = g0; i < g1 && !rc; ++i)
                if (calls[i].kind == XG_CALL_RECV)
                    rc = recv_msg(c, calls[i].peer, r->p[calls[i].buf] + calls[i].off, calls[i].len);
            g0 = g1 + 1;
        }
        if (step_post) step_post[s] = xg_now() - t0;
        for (i = sp->post_begin; i < sp->post_begin + sp->post_count && !rc; ++i) copy(r, &dp->copies[i]);
        if (!rc && n && calls[n - 1].kind == XG_CALL_BARRIER) rc = xg_barrier(c);
        if (step_done) step_done[s] = xg_now() - t0;
    }
    free(calls);
    /* as the device runtime: an unmarked step is reported as done with the next marked one */
    if (step_done && p->need && !rc)
        for (s = dp->nsteps - 2; s >= 0; --s)
            if (!p->need[s]) step_done[s] = step_done[s + 1];
    if (wall) *wall = xg_now() - t0;
    return rc;
}

/* xg_p2p_bench's traffic (mode 0: all pairs, 1: ring, 2: rank 1 -> rank 0), reps times,
 * every received byte checked against the sender's pattern */
int xg_p2p_bench(xg_ctx *c, int64_t bytes, int mode, int reps, double *gbps, double *sec)
{
    const int G = c->nranks, g = c->rank;
    unsigned char *sbuf, *rbuf;
    int rep, h, rc = XG_OK;
    int64_t o, moved = 0;
    double t0;
    if (bytes < 0 || reps < 0 || mode < 0 || mode > 2 || G < 2) return XG_EARG;
    sbuf = (unsigned char *)malloc(bytes ? (size_t)bytes : 1);
    rbuf = (unsigned char *)malloc(bytes ? (size_t)bytes : 1);
    for (o = 0; o < bytes; ++o) sbuf[o] = (unsigned char)(g * 31 + o);
    if ((rc = xg_barrier(c))) goto out;
    t0 = xg_now();
    for (rep = 0; rep < reps && !rc; ++rep) {
        for (h = 0; h < G && !rc; ++h) {   /* sends first: a group never waits on its own receives */
            const int to = mode == 0 ? h != g : mode == 1 ? h == (g + 1) % G : g == 1 && h == 0;
            if (to) { rc = send_msg(c, h, sbuf, bytes); moved += bytes; }
        }
        for (h = 0; h < G && !rc; ++h) {
            const int from = mode == 0 ? h != g : mode == 1 ? h == (g + G - 1) % G : g == 0 && h == 1;
            if (!from) continue;
            if ((rc = recv_msg(c, h, rbuf, bytes))) break;
            for (o = 0; o < bytes; ++o)
                if (rbuf[o] != (unsigned char)(h * 31 + o)) {
                    fprintf(stderr, "host_dev: p2p byte %lld from GPU %d is wrong\n", (long long)o, h);
                    rc = XG_ERCCL;
                    break;
                }
        }
    }
    if (!rc) {
        const double t = xg_now() - t0;
        if (mode == 2) moved = bytes * (int64_t)reps;
        if (sec) *sec = reps ? t / reps : 0;
        if (gbps) *gbps = t > 0 ? moved / t / 1e9 : 0;
    }
out:
    free(sbuf);
    free(rbuf);
    return rc;
}
