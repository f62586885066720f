/*
 * xg.h -- device half of the MI355X aggregator-exchange framework (C-ABI).
 *
 * One process per GPU.  Everything the reference does with malloc'd host
 * buffers and MPI point-to-point calls happens here on HBM with hand-written
 * CDNA4 kernels (gfx950) and grouped RCCL send/recv over xGMI.  No torch
 * types, no HIP types in the signatures: plain pointers, sizes, int status
 * (0 = ok; otherwise an XG_E* code, with a file:line message on stderr --
 * the reference's unused ERR macro, mpi_test.c:15-22, made real).
 *
 * Interface replaced (reference file:line)               -> entry point
 *   MPI_Init / Comm_rank / Comm_size  mpi_test.c:2127-2129 -> xg_get_unique_id, xg_init
 *   MPI_Finalize                      mpi_test.c:2345      -> xg_finalize
 *   MPI_Barrier before each timed loop (e.g. :1762)        -> xg_barrier
 *   MPI_Reduce(5 doubles, MAX, root 0) (e.g. :2184)        -> xg_allreduce_max
 *   malloc in prepare_*_data  :94-133, :162-202            -> xg_regions_alloc
 *   fill_buffer / MAP_DATA    :71-77, :23                  -> xg_fill
 *   check_buffer              :83-92 (call sites :139,:215)-> xg_verify
 *   free in clean_*           :135-231                     -> xg_regions_free
 *   the timed Irecv/Issend/Send/Recv/Sendrecv/Waitall/
 *   Alltoallw loop of each method (:421-1950)              -> xg_plan_load + xg_plan_run
 *                                                            (xg_plan_enqueue for back-to-back runs)
 *   MPI_Wtime post / waitall brackets                      -> step_post / step_done of xg_plan_run
 */
#ifndef XG_H
#define XG_H

#include <stddef.h>
#include <stdint.h>

#include "xg_sched.h"

#ifdef __cplusplus
extern "C" {
#endif

#define XG_OK 0
#define XG_EHIP 1
#define XG_ERCCL 2
#define XG_EARG 3
#define XG_ENOMEM 4

#define XG_UNIQUE_ID_BYTES 128

typedef struct xg_ctx xg_ctx;
typedef struct xg_regions xg_regions;
typedef struct xg_plan xg_plan;

/* xg_segrun / xg_slot and their builders live in xg_sched.h (host layout). */
/* ------------------------------------------------------------------ context */
int xg_get_unique_id(void *uid /* XG_UNIQUE_ID_BYTES */);
/* rank/nranks: this process in the job (one per GPU).  device: HIP ordinal.
 * uid: from rank 0's xg_get_unique_id (ignored when nranks == 1). */
int xg_init(xg_ctx **out, int rank, int nranks, int device, const void *uid);
/* Test hook: GPU `rank` of an `nranks`-GPU job emulated on physical `device`
 * in this process (no communicator of its own).  Its plans run only via
 * xg_vplans_run / xg_vplans_run_rccl, which execute every GPU of the job on one
 * device and move each RCCL send/recv pair (xg_p2p) as a device-to-device copy
 * or through RCCL on a 1-rank communicator -- the multi-GPU device plans,
 * packing and unpacking exercised on one MI355X.  Barrier / MAX are local. */
int xg_init_virtual(xg_ctx **out, int rank, int nranks, int device);
int xg_finalize(xg_ctx *ctx);
int xg_rank(const xg_ctx *ctx);
int xg_nranks(const xg_ctx *ctx);
/* The self_max this context posts with (XG_SELF_MAX at xg_init, default 256 KiB): a cross-GPU
 * step whose local part moves <= this many bytes lists it as self send/recv pairs in its RCCL
 * group (xg_devplan_step_calls).  The pairing proof of a job must use the same value. */
int64_t xg_self_max(const xg_ctx *ctx);
int xg_barrier(xg_ctx *ctx);
int xg_allreduce_max(xg_ctx *ctx, double *vals, int n);       /* in place, MAX over all GPUs (any n) */
int xg_sync(xg_ctx *ctx);                                      /* this context's stream */
int xg_device_sync(xg_ctx *ctx);                               /* whole device (hipDeviceSynchronize) */
/* device name, CU count, HBM bytes (any pointer may be NULL) */
int xg_device_info(xg_ctx *ctx, char *name, size_t namelen, int *cus, size_t *hbm_bytes);
double xg_now(void);                                           /* host seconds (monotonic) */
/* Diagnostics: where this process's host thread last was in the library -- entry point, step,
 * posting or waiting for the device -- for a watchdog to print when a run does not return. */
const char *xg_debug_where(void);
/* ROCm runtime libraries (libamdhip64, librccl, libhsa-runtime64) mapped into this process from
 * outside the ROCm install libxg.so was built against (its library directory, recorded at build
 * time) and /opt/rocm*, $ROCM_PATH: e.g. torch's wheel bundles its own under the
 * same sonames, and a process that loaded them first binds libxg.so to another HIP runtime and
 * RCCL than it was built against (profiles/r04/torch_runtime/).  Returns how many; their paths,
 * comma-separated, in buf (may be NULL).  xg_get_unique_id and xg_init refuse (XG_EARG) when
 * this is > 0, so every entry point (bin/test, bin/pt2pt_test, bench.py, xg.py) does. */
int xg_foreign_runtime(char *buf, size_t len);
/* RCCL's version as ncclGetVersion reports it (e.g. 22703 for 2.27.3). */
int xg_rccl_version(int *version);

/* ------------------------------------------------------------------ HBM regions */
/* region_bytes: XG_BUF_SEND, XG_BUF_RECV, XG_BUF_STAGE_SEND, XG_BUF_STAGE_RECV,
 * XG_BUF_SCRATCH (xg_devplan.region_bytes).  The RECV region is poisoned (0xA5),
 * SCRATCH is zeroed. */
int xg_regions_alloc(xg_ctx *ctx, const int64_t region_bytes[XG_NBUF], xg_regions **out);
int xg_regions_free(xg_regions *r);
int xg_regions_poison(xg_regions *r);
/* Device pointer of a region (for tests that read buffers back). */
void *xg_regions_ptr(xg_regions *r, int buf);
int xg_regions_read(xg_regions *r, int buf, int64_t off, void *host, int64_t len);
/* Test hook: overwrite bytes of a region (e.g. corrupt one received byte to check
 * that xg_verify reports it). */
int xg_regions_write(xg_regions *r, int buf, int64_t off, const void *host, int64_t len);

int xg_fill(xg_regions *r, const xg_segrun *runs, int nruns, int64_t d, int iter, int mode);
/* Per slot: chk[i] = xg_chk64 of the slot bytes, bad[i] = number of bytes that
 * differ from the expected fingerprint, first_bad[i] = first differing offset
 * (or -1).  Any output pointer may be NULL. */
int xg_verify(xg_regions *r, const xg_slot *slots, int nslots, int64_t d, int iter, int mode,
              uint64_t *chk, int64_t *bad, int64_t *first_bad);

/* ------------------------------------------------------------------ plans */
int xg_plan_load(xg_ctx *ctx, xg_regions *r, const xg_devplan *dp, xg_plan **out);
int xg_plan_free(xg_plan *p);
int xg_plan_nsteps(const xg_plan *p);
/* Timed run (caller barriers first): enqueues every step, waits, and returns per
 * step the device completion time (seconds since the run started) and the host
 * enqueue time; *wall = host seconds from start to the final synchronisation.
 * What a step's completion time means: per-step launches -- the clock stamp of a
 * one-lane kernel that starts after its last launch, RCCL group or join (or, in a
 * chain of one-launch local steps, the start of the next launch), i.e. its bytes
 * stored; engine segments -- the wall-clock stamp at the
 * step's barrier, which for steps without a drain flag is when their stores were
 * ISSUED (not yet performed); only drained steps (hazard points and the last step
 * of every segment, which anchors the others) are delivery times.  A run's total
 * is therefore always a delivered time. */
int xg_plan_run(xg_plan *p, double *step_done, double *step_post, double *wall);
/* Enqueue all steps once without events or synchronisation (bench loops).  Check
 * the step engine's timeout word with xg_plan_check after synchronising. */
int xg_plan_enqueue(xg_plan *p);
/* XG_EHIP if a step-engine workgroup gave up at a grid barrier since the last
 * check (its launch then moved only part of the bytes); waits for the stream. */
int xg_plan_check(xg_plan *p);
/* Step engine: every maximal run of >= 2 GPU-local steps (no RCCL op, no in-loop
 * barrier, no unpack, each <= XG_ENGINE_MAX_STEP bytes; 0 = off) is ONE persistent
 * launch of up to one workgroup per CU (fewer if the device admits fewer), grid barrier +
 * wall-clock stamp per step; the other steps are their own launches.
 * Small hazard-free segments run on the solo engine instead: each step's pieces
 * dealt over up to XG_SOLO_RAILS independent rails (default 512 rails of one wave;
 * XG_SOLO_WAVES=16: 16-wave workgroups) that each keep their own step order and
 * never wait for one another.
 * xg_plan_engine: workgroups of the first such segment (0: none);
 * xg_plan_engine_rails: rails of the first solo segment (0: none);
 * xg_plan_engine_steps: steps inside segments (*nseg segments, *nhaz hazard
 * barriers, xg_engine_hazards); XG_ENGINE_DRAIN=1 drains every step's stores. */
int xg_plan_engine(const xg_plan *p);
int xg_plan_engine_rails(const xg_plan *p);
int xg_plan_engine_steps(const xg_plan *p, int *nseg, int *nhaz);
/* Kernel launches of one run (copy + engine launches; RCCL's own kernels aside). */
int xg_plan_launches(const xg_plan *p);
/* Staging displacements of the plan's packed segments as computed on the device
 * at load (one wavefront prefix scan per step and direction: the alltoallw
 * translate of mpi_test.c:233-302).  out == NULL: returns their number. */
int xg_plan_displs(const xg_plan *p, int64_t *out, int n);
/* plans[g] = GPU g's plan of one virtual job (xg_init_virtual, g = 0..n-1, same
 * schedule); step_done[nsteps]: device seconds from start to the end of each step. */
int xg_vplans_run(xg_plan *const *plans, int n, double *step_done);
/* Same, with every send/recv pair moved by RCCL: a 1-rank communicator on the
 * device, one ncclGroupStart/End of self ncclSend + ncclRecv per step (matched
 * in issue order) and ncclAllReduce for the in-loop barriers -- RCCL's calls on
 * the real plan buffers with one GPU. */
int xg_vplans_run_rccl(xg_plan *const *plans, int n, double *step_done);
/* Test hook: a virtual GPU's plan run ALONE by xg_plan_run / xg_plan_enqueue -- its copy
 * launches only, its RCCL calls and in-loop barriers left out (its received-from-peer slots
 * keep the poison) -- so one GPU's share of a job too large to emulate whole on one device
 * executes at full size.  XG_EARG for a non-virtual context or a plan with self calls. */
int xg_plan_set_local_only(xg_plan *p, int on);
/* Mark only the steps whose completion time a Timer reads (need: xg_sched_timed_steps of the
 * plan's schedule; NULL = every step, the default; the last step is always marked).  An unmarked
 * step costs no clock stamp in xg_plan_run and is reported as done when the next marked step is.
 * Engine segments and chains are marked at their last step regardless. */
int xg_plan_set_step_marks(xg_plan *p, const uint8_t *need);
/* Kernel timing session.  mode 1: every copy / engine launch of any plan on this
 * context is bracketed by HIP events on the stream it runs on (at most
 * max_launches); mode 2: one event pair on the main stream around the whole
 * session, launches and bytes counted.  xg_ktime_end waits for the stream and
 * returns the kernel time (mode 1: summed per launch; mode 2: the session),
 * the number of launches and their algorithmic HBM bytes (read + write). */
int xg_ktime_begin(xg_ctx *ctx, int max_launches, int mode);
int xg_ktime_end(xg_ctx *ctx, double *total_ms, int *launches, int64_t *bytes);
/* After a mode-1 session: launch k's time (ms) and algorithmic bytes (read + write). */
int xg_ktime_launch(xg_ctx *ctx, int k, double *ms, int64_t *bytes);

/* RCCL point-to-point ceiling (rccl-tests sendrecv analogue; GPU version of
 * pt2pt_test, mpi_sendrecv_test.c:15-74).  mode 0: all pairs, 1: ring,
 * 2: one direction rank 1 -> rank 0.  *gbps = bytes sent by this rank per
 * second (mode 2: bytes moved 1 -> 0), *sec = seconds per repetition. */
int xg_p2p_bench(xg_ctx *ctx, int64_t bytes, int mode, int reps, double *gbps, double *sec);
/* xg_p2p_bench mode 0 with every (rank, peer) transfer of `bytes` posted as `calls` (1..4096)
 * consecutive ncclSend / ncclRecv of 16-B aligned cuts of it, in one group: against calls = 1,
 * RCCL's cost per extra call to the same peer -- what the relay form (XG_RELAY, xg_sched.h),
 * which cuts every relayed message into G pieces, pays per step beside its link-time gain.
 * With XG_SELF_COMM on a one-rank context: rank 0 to itself. */
int xg_p2p_split_bench(xg_ctx *ctx, int64_t bytes, int calls, int reps, double *gbps, double *sec);
/* One link: `bytes` each way between this rank and `peer` (send + receive in one group), reps
 * times; peer < 0 or peer == this rank: idle (returns 0 rates).  Every rank agrees that all have
 * their buffers (a MAX all-reduce, idle ranks too) before any call is posted, so an allocation
 * that fails on one rank fails the round on all (XG_ENOMEM) instead of stranding its partner.  Every rank of a round calls it
 * with its partner of that round (a 1-factorisation of the ranks), so all links of the round run
 * at once and each is measured under the others' load (the per-peer sweep of the N > 1 bench
 * line: link asymmetry shows as the spread).  *gbps = bytes this rank sent per second. */
int xg_p2p_pair_bench(xg_ctx *ctx, int64_t bytes, int peer, int reps, double *gbps, double *sec);

/* Tuning: bytes per copy workgroup (default 32768; chunk_bytes 0 keeps it) and copy kernel
 * variant: 0 (default) = copy_kernel_g<4> with non-temporal loads/stores for launches moving
 * >= 128 MiB (source + destination past the 256 MiB Infinity Cache) and plain ones below;
 * 1 = always plain, 6 = always non-temporal (XG_EARG for any other).  variant < 0 keeps the
 * current one; XG_COPY_VARIANT at xg_init.  Applies to plans loaded afterwards. */
int xg_set_copy_params(xg_ctx *ctx, int64_t chunk_bytes, int variant);

/* ------------------------------------------------------------------ method operators
 * The reference's per-method operator API (e.g. all_to_many, mpi_test.c:1748):
 *   int fn(int rank, int isagg, int procs, int cb_nodes, int data_size,
 *          int *rank_list, int comm_size, Timer *timer, int iter, int ntimes)
 * Here one call runs the method for EVERY logical rank this GPU hosts
 * (xg_block_range), so `timers` holds one Timer per hosted rank (in rank
 * order) -- the generalisation of "the calling rank's Timer"; rank and isagg
 * are implied.  Like the reference, the callee owns its buffers (allocated,
 * fingerprinted with `iter`, timed -k `ntimes` times, freed).  Returns 0, or
 * an XG_E* code; XG_ESCHED when the schedule cannot complete under MPI
 * semantics (the reference hangs there) -- err gets the reason. */
#define XG_ESCHED 5

typedef struct {
    int verify;              /* 1: check every received byte afterwards (check_buffer, :83-92) */
    int fingerprint;         /* XG_FP_REFERENCE (MAP_DATA) or XG_FP_STRONG                    */
    int64_t eager_limit;     /* blocking sends <= this complete locally (XG_MPICH_EAGER_LIMIT)  */
    int64_t pack_max_seg;    /* p2p staging threshold (xg_devplan_build)                       */
    int proc_node;           /* -p (m17's node_robin_map)                                       */
    int barrier_type;        /* -b (m13)                                                        */
    xg_timer *rep_timers;    /* out, optional: hosted ranks x ntimes timers[m] (m13)            */
    int64_t pack_min_bytes;  /* ... and pack only (step, peer) lists of >= this many bytes        */
    int pack_form;           /* XG_PACK_ONE_SIDED / XG_PACK_TWO_SIDED (xg_devplan_build_form)   */
} xg_run_opts;

void xg_run_opts_default(xg_run_opts *o);

/* bad_slots (may be NULL): receive slots of this GPU that failed verification. */
int xg_run_method(xg_ctx *ctx, int method, int procs, int cb_nodes, int data_size, const int *rank_list,
                  int comm_size, xg_timer *timers, int iter, int ntimes, const xg_run_opts *opts,
                  int64_t *bad_slots, char *err, size_t errlen);

/* The operators under the reference's names (mpi_test.c line of the original). */
#define XG_METHOD_DECL(name)                                                                     \
    int name(xg_ctx *ctx, int procs, int cb_nodes, int data_size, int *rank_list, int comm_size, \
             xg_timer *timers, int iter, int ntimes)
XG_METHOD_DECL(xg_all_to_many);                 /* m1  :1748 */
XG_METHOD_DECL(xg_many_to_all);                 /* m2  :1871 */
XG_METHOD_DECL(xg_all_to_many_balanced);        /* m3  :1422 */
XG_METHOD_DECL(xg_many_to_all_balanced);        /* m4  :1576 */
XG_METHOD_DECL(xg_many_to_all_benchmark);       /* m5  :599  */
XG_METHOD_DECL(xg_all_to_many_sync);            /* m6  :1665 */
XG_METHOD_DECL(xg_all_to_many_half_sync);       /* m7  :1055 */
XG_METHOD_DECL(xg_all_to_many_benchmark);       /* m8  :885  */
XG_METHOD_DECL(xg_all_to_many_pairwise);        /* m9  :510  */
XG_METHOD_DECL(xg_many_to_all_pairwise);        /* m10 :421  */
XG_METHOD_DECL(xg_many_to_all_half_sync);       /* m11 :942  */
XG_METHOD_DECL(xg_all_to_many_half_sync2);      /* m12 :999  */
XG_METHOD_DECL(xg_many_to_all_scattered);       /* m14 :656  */
XG_METHOD_DECL(xg_all_to_many_balanced_control);/* m18 :1229 */
XG_METHOD_DECL(xg_all_to_many_scattered_isend); /* m19 :722  */
XG_METHOD_DECL(xg_all_to_many_balanced_pre_send);/* m20 :1338 */
/* m13 / m17 / m15 / m16 take the reference's extra arguments (:797, :1135, :366, :313) */
int xg_all_to_many_scattered(xg_ctx *ctx, int procs, int cb_nodes, int data_size, int *rank_list, int comm_size,
                             int barrier_type, xg_timer *timers, xg_timer *rep_timers, int iter, int ntimes);
int xg_all_to_many_node_robin(xg_ctx *ctx, int procs, int cb_nodes, int data_size, int *rank_list, int comm_size,
                              int proc_node, xg_timer *timers, int iter, int ntimes);
/* TAM: collective_write over static_node_assignment type 0 nodes of procs_node ranks
 * (lustre_driver_test.c:944-1309, :359-429) */
int xg_all_to_many_tam(xg_ctx *ctx, int procs, int cb_nodes, int data_size, int *rank_list, int comm_size,
                       int procs_node, xg_timer *timers, int iter, int ntimes);       /* m15 :366 */
int xg_many_to_all_tam(xg_ctx *ctx, int procs, int cb_nodes, int data_size, int *rank_list, int comm_size,
                       int procs_node, xg_timer *timers, int iter, int ntimes);       /* m16 :313 */

#ifdef __cplusplus
}
#endif
#endif
