/*
 * methods.c -- the reference's per-method operators on the MI355X runtime.
 * One call = prepare_*_data (regions + fingerprint, untimed) -> MPI_Barrier ->
 * the timed exchange -> Timer of every hosted logical rank -> clean_* ;
 * plus optional verification (the reference's commented-out check_buffer).
 * Compiled into libxg.so; links libxghost.so for schedules.
 */
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>

#include "xg.h"
#include "xg_sched.h"

void xg_run_opts_default(xg_run_opts *o)
{
    o->verify = 0;
    o->fingerprint = XG_FP_REFERENCE;
    o->eager_limit = XG_MPICH_EAGER_LIMIT;
    o->pack_max_seg = 4 << 20;
    o->proc_node = 1;
    o->barrier_type = 0;
    o->rep_timers = NULL;
    o->pack_min_bytes = 64 << 10;   /* latency-bound steps: one RCCL launch (profiles/r03/hybrid/) */
    o->pack_form = XG_PACK_FORM_DEFAULT;
}

#define TRY(x) do { rc = (x); if (rc) goto out; } while (0)

/* A G-GPU job's RCCL calls pair step by step as RCCL pairs them (xg_devplans_match over
 * every GPU's plan, calls.c), the calls listed with the self_max this process posts with
 * (xg_self_max: the exact lists enqueue_step hands RCCL).  -> XG_OK, XG_EARG (err says which
 * call would not pair) or XG_ENOMEM. */
static int pairing_ok(const xg_sched *s, int G, int64_t pack_max_seg, int64_t pack_min, int form, int64_t self_max,
                      char *err, size_t errlen)
{
    xg_devplan **plans = (xg_devplan **)calloc(G, sizeof *plans);
    int g, rc = XG_OK;
    char why[400];
    if (!plans) {
        snprintf(err, errlen, "pairing check: out of host memory");
        return XG_ENOMEM;
    }
    for (g = 0; g < G && rc == XG_OK; ++g)
        if (!(plans[g] = xg_devplan_build_form(s, G, g, pack_max_seg, pack_min, form))) {
            snprintf(err, errlen, "pairing check: out of host memory building GPU %d's plan", g);
            rc = XG_ENOMEM;
        }
    if (rc == XG_OK && xg_devplans_match((const xg_devplan *const *)plans, G, self_max, NULL, 0, why, sizeof why) < 0) {
        snprintf(err, errlen, "the GPUs' RCCL calls do not pair: %s", why);
        rc = XG_EARG;
    }
    for (g = 0; g < G; ++g) xg_devplan_free(plans[g]);
    free(plans);
    return rc;
}

/* One MAX reduction over the job: whether any GPU failed (and the highest code).  Each GPU plans,
 * allocates, fills and loads its part alone; one that failed must not return while its peers go
 * on to post RCCL calls it will never pair (they would wait forever), so every GPU learns the
 * outcome here and all return an error alike.  local_rc: this GPU's result so far. */
static int peers_agree(xg_ctx *ctx, int local_rc, char *err, size_t errlen)
{
    double red[2];
    int rc;
    red[0] = local_rc ? 1.0 : 0.0;
    red[1] = (double)local_rc;
    if ((rc = xg_allreduce_max(ctx, red, 2))) return local_rc ? local_rc : rc;
    if (red[0] == 0.0) return XG_OK;
    if (local_rc) return local_rc;
    snprintf(err, errlen, "another GPU of the job failed (code %d) setting up or running this method", (int)red[1]);
    return (int)red[1];
}

/* Every GPU of a job must plan from the same inputs: each derives every GPU's RCCL calls from
 * them, and a rank that planned from others would post calls nobody pairs -- the job would
 * hang in RCCL.  Before anything that could diverge (a schedule refused on one rank only), the
 * ranks compare a digest of the inputs (FNV-1a, in four 16-bit parts: exact as doubles) by one
 * MAX reduction of the parts and their negations; unequal inputs fail alike on every rank. */
static uint64_t fnv(uint64_t h, const void *p, size_t n)
{
    const unsigned char *b = (const unsigned char *)p;
    size_t i;
    for (i = 0; i < n; ++i) h = (h ^ b[i]) * 0x100000001b3ull;
    return h;
}

static int inputs_agree(xg_ctx *ctx, int method, int procs, int cb_nodes, int data_size, const int *rank_list,
                        int comm_size, int iter, int ntimes, const xg_run_opts *o, char *err, size_t errlen)
{
    int64_t v[14];
    double red[8];
    uint64_t h = 0xcbf29ce484222325ull;
    int i, rc;
    v[0] = method; v[1] = procs; v[2] = cb_nodes; v[3] = data_size; v[4] = comm_size; v[5] = iter;
    v[6] = ntimes; v[7] = o->eager_limit; v[8] = o->pack_max_seg; v[9] = o->pack_min_bytes;
    v[10] = o->proc_node; v[11] = o->barrier_type; v[12] = o->pack_form; v[13] = xg_self_max(ctx);
    h = fnv(h, v, sizeof v);
    h = fnv(h, rank_list, sizeof(int) * (size_t)cb_nodes);
    for (i = 0; i < 4; ++i) {
        red[i] = (double)((h >> (16 * i)) & 0xffff);
        red[4 + i] = -red[i];
    }
    if ((rc = xg_allreduce_max(ctx, red, 8))) return rc;
    for (i = 0; i < 4; ++i)
        if (red[i] != -red[4 + i]) {
            snprintf(err, errlen, "the GPU processes planned method %d from different inputs (arguments or "
                     "options differ between ranks)", method);
            return XG_EARG;
        }
    return XG_OK;
}

/* Set-up of one GPU's part (untimed, no collective call): schedule, pairing proof, device plan,
 * regions, fingerprint fill, plan upload and the host arrays.  -> XG_OK or the first error. */
static int setup(xg_ctx *ctx, int method, int procs, int cb_nodes, int data_size, const int *rank_list, int comm_size,
                 int iter, int ntimes, const xg_run_opts *o, xg_sched **s, xg_devplan **dp, xg_regions **reg,
                 xg_plan **plan, double **done, double **post, char *err, size_t errlen)
{
    const int g = xg_rank(ctx), G = xg_nranks(ctx);
    xg_segrun *runs;
    int rc, nruns;
    *s = xg_sched_build_iter(method, procs, cb_nodes, data_size, comm_size, rank_list, ntimes, o->proc_node,
                             o->barrier_type, o->eager_limit, iter, err, errlen);
    if (!*s) return XG_ESCHED;
    /* every GPU derives every GPU's calls from the same schedule, so every GPU refuses a job
     * that would not pair alike -- before any of them posts a call that could wait forever */
    if (G > 1 && (rc = pairing_ok(*s, G, o->pack_max_seg, o->pack_min_bytes, o->pack_form, xg_self_max(ctx), err,
                                  errlen)))
        return rc;
    if (!(*dp = xg_devplan_build_form(*s, G, g, o->pack_max_seg, o->pack_min_bytes, o->pack_form))) {
        snprintf(err, errlen, "device plan: out of host memory");
        return XG_ENOMEM;
    }
    if ((rc = xg_regions_alloc(ctx, (*dp)->region_bytes, reg))) {
        snprintf(err, errlen, "HBM regions of %lld + %lld + %lld + %lld + %lld bytes: allocation failed (%d)",
                 (long long)(*dp)->region_bytes[0], (long long)(*dp)->region_bytes[1],
                 (long long)(*dp)->region_bytes[2], (long long)(*dp)->region_bytes[3],
                 (long long)(*dp)->region_bytes[4], rc);
        return rc;
    }
    nruns = xg_fill_runs(*s, G, g, NULL);
    runs = (xg_segrun *)malloc(sizeof(xg_segrun) * (nruns + 1));
    *done = (double *)calloc(xg_sched_nsteps(*s) + 1, sizeof(double));
    *post = (double *)calloc(xg_sched_nsteps(*s) + 1, sizeof(double));
    if (!runs || !*done || !*post) {
        free(runs);
        snprintf(err, errlen, "out of host memory");
        return XG_ENOMEM;
    }
    xg_fill_runs(*s, G, g, runs);
    rc = xg_fill(*reg, runs, nruns, data_size, iter, o->fingerprint);
    free(runs);
    if (rc) return rc;
    if ((rc = xg_plan_load(ctx, *reg, *dp, plan))) return rc;
    {   /* a timed run marks only the steps whose completion time a Timer reads */
        uint8_t *need = (uint8_t *)malloc((size_t)xg_sched_nsteps(*s) + 1);
        if (!need) {
            snprintf(err, errlen, "out of host memory");
            return XG_ENOMEM;
        }
        xg_sched_timed_steps(*s, need);
        rc = xg_plan_set_step_marks(*plan, need);
        free(need);
    }
    return rc;
}

int xg_run_method(xg_ctx *ctx, int method, int procs, int cb_nodes, int data_size, const int *rank_list,
                  int comm_size, xg_timer *timers, int iter, int ntimes, const xg_run_opts *opts,
                  int64_t *bad_slots, char *err, size_t errlen)
{
    xg_run_opts dflt;
    const int g = xg_rank(ctx), G = xg_nranks(ctx);
    char ebuf[512];
    xg_sched *s = NULL;
    xg_devplan *dp = NULL;
    xg_regions *reg = NULL;
    xg_plan *plan = NULL;
    xg_slot *slots = NULL;
    int64_t *bad = NULL, nbad = 0;
    double *done = NULL, *post = NULL, wall = 0;
    int rc = 0, agreed = 0, lo, hi, r, i;
    if (!opts) { xg_run_opts_default(&dflt); opts = &dflt; }
    if (!err) { err = ebuf; errlen = sizeof ebuf; }
    err[0] = 0;
    if (bad_slots) *bad_slots = 0;
    if (G > 1 && (rc = inputs_agree(ctx, method, procs, cb_nodes, data_size, rank_list, comm_size, iter, ntimes, opts,
                                    err, errlen)))
        return rc;
    rc = setup(ctx, method, procs, cb_nodes, data_size, rank_list, comm_size, iter, ntimes, opts, &s, &dp, &reg, &plan,
               &done, &post, err, errlen);
    if (G > 1) rc = peers_agree(ctx, rc, err, errlen);      /* before the first call of the exchange */
    if (rc) goto out;
    agreed = 1;
    TRY(xg_barrier(ctx));                                   /* MPI_Barrier before total_start */
    TRY(xg_plan_run(plan, done, post, &wall));
    xg_block_range(procs, G, g, &lo, &hi);
    if (timers)
        for (r = lo; r < hi; ++r) xg_sched_rank_timer(s, G, r, done, post, &timers[r - lo]);
    if (opts->rep_timers && ntimes > 0)
        for (r = lo; r < hi; ++r)
            xg_sched_rank_rep_timers(s, G, r, done, post, opts->rep_timers + (size_t)(r - lo) * ntimes);
    if (opts->verify) {
        int ns = xg_verify_slots(s, G, g, NULL);
        slots = (xg_slot *)malloc(sizeof(xg_slot) * (ns + 1));
        bad = (int64_t *)calloc(ns + 1, sizeof(int64_t));
        if (!slots || !bad) {
            snprintf(err, errlen, "verify: out of host memory");
            rc = XG_ENOMEM;
            goto out;
        }
        xg_verify_slots(s, G, g, slots);
        TRY(xg_verify(reg, slots, ns, data_size, iter, opts->fingerprint, NULL, bad, NULL));
        for (i = 0; i < ns; ++i)
            if (bad[i]) {
                if (nbad == 0) fprintf(stderr, "rank %d, message is wrong from rank %d\n", slots[i].dst, slots[i].src);
                ++nbad;
            }
        if (bad_slots) *bad_slots = nbad;
    }
out:
    /* a GPU that failed after the set-up (the run, the verify) tells its peers too: the caller's
     * next collective (the timer reduction) must not wait for it.  A run that failed inside RCCL
     * may leave the communicator unusable -- then this reports that error as well. */
    if (G > 1 && agreed) rc = peers_agree(ctx, rc, err, errlen);
    if (rc && err[0] == 0) snprintf(err, errlen, "device error %d (see stderr)", rc);
    free(slots); free(bad); free(done); free(post);
    if (plan) xg_plan_free(plan);
    if (reg) xg_regions_free(reg);
    xg_devplan_free(dp);
    xg_sched_free(s);
    return rc;
}

#define XG_METHOD_DEF(name, m)                                                                    \
    XG_METHOD_DECL(name)                                                                          \
    {                                                                                             \
        char e[512];                                                                              \
        int rc = xg_run_method(ctx, m, procs, cb_nodes, data_size, rank_list, comm_size, timers,  \
                               iter, ntimes, NULL, NULL, e, sizeof e);                            \
        if (rc == XG_ESCHED) fprintf(stderr, "%s: %s\n", #name, e);                               \
        return rc;                                                                                \
    }
XG_METHOD_DEF(xg_all_to_many, 1)
XG_METHOD_DEF(xg_many_to_all, 2)
XG_METHOD_DEF(xg_all_to_many_balanced, 3)
XG_METHOD_DEF(xg_many_to_all_balanced, 4)
XG_METHOD_DEF(xg_many_to_all_benchmark, 5)
XG_METHOD_DEF(xg_all_to_many_sync, 6)
XG_METHOD_DEF(xg_all_to_many_half_sync, 7)
XG_METHOD_DEF(xg_all_to_many_benchmark, 8)
XG_METHOD_DEF(xg_all_to_many_pairwise, 9)
XG_METHOD_DEF(xg_many_to_all_pairwise, 10)
XG_METHOD_DEF(xg_many_to_all_half_sync, 11)
XG_METHOD_DEF(xg_all_to_many_half_sync2, 12)
XG_METHOD_DEF(xg_many_to_all_scattered, 14)
XG_METHOD_DEF(xg_all_to_many_balanced_control, 18)
XG_METHOD_DEF(xg_all_to_many_scattered_isend, 19)
XG_METHOD_DEF(xg_all_to_many_balanced_pre_send, 20)

int xg_all_to_many_scattered(xg_ctx *ctx, int procs, int cb_nodes, int data_size, int *rank_list, int comm_size,
                             int barrier_type, xg_timer *timers, xg_timer *rep_timers, int iter, int ntimes)
{
    xg_run_opts o;
    char e[512];
    int rc;
    xg_run_opts_default(&o);
    o.barrier_type = barrier_type;
    o.rep_timers = rep_timers;
    rc = xg_run_method(ctx, 13, procs, cb_nodes, data_size, rank_list, comm_size, timers, iter, ntimes, &o, NULL,
                       e, sizeof e);
    if (rc == XG_ESCHED) fprintf(stderr, "xg_all_to_many_scattered: %s\n", e);
    return rc;
}

static int run_with_proc_node(xg_ctx *ctx, int method, const char *name, int procs, int cb_nodes, int data_size,
                              int *rank_list, int comm_size, int proc_node, xg_timer *timers, int iter, int ntimes)
{
    xg_run_opts o;
    char e[512];
    int rc;
    xg_run_opts_default(&o);
    o.proc_node = proc_node;
    rc = xg_run_method(ctx, method, procs, cb_nodes, data_size, rank_list, comm_size, timers, iter, ntimes, &o, NULL,
                       e, sizeof e);
    if (rc == XG_ESCHED) fprintf(stderr, "%s: %s\n", name, e);
    return rc;
}

int xg_all_to_many_node_robin(xg_ctx *ctx, int procs, int cb_nodes, int data_size, int *rank_list, int comm_size,
                              int proc_node, xg_timer *timers, int iter, int ntimes)
{
    return run_with_proc_node(ctx, 17, "xg_all_to_many_node_robin", procs, cb_nodes, data_size, rank_list, comm_size,
                              proc_node, timers, iter, ntimes);
}

int xg_many_to_all_tam(xg_ctx *ctx, int procs, int cb_nodes, int data_size, int *rank_list, int comm_size,
                       int procs_node, xg_timer *timers, int iter, int ntimes)
{
    return run_with_proc_node(ctx, 16, "xg_many_to_all_tam", procs, cb_nodes, data_size, rank_list, comm_size,
                              procs_node, timers, iter, ntimes);
}

int xg_all_to_many_tam(xg_ctx *ctx, int procs, int cb_nodes, int data_size, int *rank_list, int comm_size,
                       int procs_node, xg_timer *timers, int iter, int ntimes)
{
    return run_with_proc_node(ctx, 15, "xg_all_to_many_tam", procs, cb_nodes, data_size, rank_list, comm_size,
                              procs_node, timers, iter, ntimes);
}
