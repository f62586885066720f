/*
 * xg_sched.h -- host-side (plain C, no HIP headers) half of the MI355X
 * aggregator-exchange framework.
 *
 * The reference (QiaoK/MPI-Asynchronous-Communication-Test, mpi_test.c) runs
 * one MPI process per rank; each method issues Irecv/Issend/Send/Recv/
 * Sendrecv/Waitall/Alltoallw calls.  Here every logical rank's program is
 * restated literally (same loops, same quirks), matched with MPI semantics,
 * and compiled into a list of device-wide STEPS: step s holds every segment
 * that can move once everything of steps < s is delivered (earliest-step
 * schedule; MPI eager protocol for small blocking sends).  Each GPU then
 * executes its share of each step as one gather/scatter kernel + one grouped
 * RCCL exchange (xg.h).
 *
 * Interfaces replaced (reference file:line):
 *   xg_aggregator_list  <- create_aggregator_list        mpi_test.c:1952-2006
 *   xg_sched_build      <- the body of each method       mpi_test.c:421-1950
 *                          (+ *_alltoall_translate :233-302; TAM m15/m16
 *                          :313-419 -> collective_write +
 *                          static_node_assignment, lustre_driver_test.c:359-429, :944-1309)
 *   xg_sched_rank_timer <- the MPI_Wtime brackets filling Timer   :25-31
 *   xg_summarize_results<- summarize_results             mpi_test.c:2068-2118
 */
#ifndef XG_SCHED_H
#define XG_SCHED_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Timer of the reference, field order preserved (mpi_test.c:25-31): MPI_Reduce
 * reduces it as 5 doubles. */
typedef struct {
    double post_request_time;
    double send_wait_all_time;
    double recv_wait_all_time;
    double barrier_time;
    double total_time;
} xg_timer;

enum { XG_A2M = 0, XG_M2A = 1 };

/* One matched message (one d-byte segment; zero-length for the pairwise
 * methods' non-participating pairs).  sseg: index of the segment in the
 * sender's send buffer; dslot: index of the slot in the receiver's receive
 * buffer (-1 when the message lives elsewhere: TAM aggregation buffers).
 * sbuf/soff and dbuf/doff: where its bytes are read and written, as a region
 * (XG_BUF_SEND / RECV / SCRATCH) and a byte offset inside that rank's part of
 * it.  step: the device-wide step it moves in.  Self memcpy's of m3/m4/m6
 * (mpi_test.c:1473, :1646, :1714) and of TAM (lustre_driver_test.c:1069-1285)
 * are messages with src == dst and XG_MSG_COPY. */
typedef struct {
    int32_t src, sseg, dst, dslot;
    int64_t len;
    int32_t step;
    int32_t flags;
    int32_t sbuf, dbuf;       /* -1: host-side control data (XG_MSG_CTRL) */
    int64_t soff, doff;
} xg_msg;

#define XG_MSG_COPY 1
#define XG_MSG_COLL 2   /* part of an MPI_Alltoallw */
#define XG_MSG_CTRL 4   /* TAM size exchange (MPI_INT arrays): orders steps, moves no device bytes */

#define XG_MPICH_EAGER_LIMIT 65424   /* see DESIGN.md "blocking-send semantics" */

typedef struct xg_sched xg_sched;

/* create_aggregator_list (mpi_test.c:1952-2006).  Returns 0, or -1 for an
 * aggregator type the reference does not define. */
int xg_aggregator_list(int procs, int cb_nodes, int proc_node, int type, int *rank_list);

/* Label printed by summarize_results for a method (mpi_test.c:2186-2337), NULL if not 1..20. */
const char *xg_method_label(int method);
/* XG_A2M or XG_M2A (the buffer layout of the method); -1 if not 1..20. */
int xg_method_direction(int method);

/* Build the schedule of one method run (all `ntimes` repetitions), methods
 * 1..20.  proc_node (-p) matters to m17 (node_robin_map, :1116-1133) and to
 * m15/m16 (processes per node of static_node_assignment type 0); barrier_type
 * (-b) to m13.  The schedule of m15/m16 depends on the iteration (its tags
 * carry +100*iter): build it with xg_sched_build_iter.
 * eager_limit: blocking sends and Isends of <= eager_limit bytes complete
 * locally (XG_MPICH_EAGER_LIMIT reproduces the reference on the image's MPICH).
 * Returns NULL and writes a message into err on failure, e.g. when the
 * programs deadlock under MPI semantics (the reference hangs there too). */
xg_sched *xg_sched_build(int method, int procs, int cb_nodes, int64_t data_size, int comm_size,
                         const int *rank_list, int ntimes, int proc_node, int barrier_type,
                         int64_t eager_limit, char *err, size_t errlen);
xg_sched *xg_sched_build_iter(int method, int procs, int cb_nodes, int64_t data_size, int comm_size,
                              const int *rank_list, int ntimes, int proc_node, int barrier_type,
                              int64_t eager_limit, int iter, char *err, size_t errlen);
void xg_sched_free(xg_sched *s);

int xg_sched_nmsg(const xg_sched *s);
const xg_msg *xg_sched_msgs(const xg_sched *s);
int xg_sched_nsteps(const xg_sched *s);
int xg_sched_direction(const xg_sched *s);
int xg_sched_procs(const xg_sched *s);

/* Canonical MPI call trace of one logical rank (same token format as the
 * PMPI capture in tests/golden/); returns the length written (truncated to
 * buflen-1) or the needed length if buf is NULL.  Pairwise m9/m10 above P = 1024
 * (or with XG_PAIRWISE_FAST=1) are planned in a fast form that leaves out the
 * 0-byte MPI_Sendrecv rounds: their trace is then NOT the reference's call trace
 * (same byte-carrying posts, other completions; tests/test_host_sched.py). */
size_t xg_sched_trace(const xg_sched *s, int rank, char *buf, size_t buflen);

/* Per-rank timer from device step timestamps (ranks block-mapped on ngpus):
 *   step_done[s]  seconds from the timed-region start until step s completed
 *                 on the GPU that hosts `rank`;
 *   step_post[s]  host seconds spent enqueuing step s on that GPU (may be NULL);
 *                 it is shared out over the requests that GPU's ranks post in s.
 * Each reference timer bracket (MPI_Wtime pairs) becomes an interval of the
 * rank's logical clock, which advances at completion points to the step
 * completion time of the awaited messages; a post bracket adds the share of
 * enqueue time of the requests it posts. */
int xg_sched_rank_timer(xg_sched *s, int ngpus, int rank, const double *step_done,
                        const double *step_post, xg_timer *out);
/* timers[m] of every repetition (m13, mpi_test.c:829-874; zero for other methods):
 * reps has xg_sched_ntimes(s) entries. */
int xg_sched_rank_rep_timers(xg_sched *s, int ngpus, int rank, const double *step_done,
                             const double *step_post, xg_timer *reps);
int xg_sched_ntimes(const xg_sched *s);
/* The steps whose completion time some rank's Timer reads (need[nsteps]: 1 = read; the last
 * step always is).  Every other step may be timed as the next read step without changing any
 * Timer field (a run then marks only these: xg_plan_set_step_marks).  -> how many. */
int xg_sched_timed_steps(const xg_sched *s, uint8_t *need);
/* step after which the k-th MPI_Barrier of the method completes (-1: before step 0);
 * returns the number of barriers (out may be NULL). */
int xg_sched_barrier_epochs(const xg_sched *s, int32_t *out);

/* ---------------------------------------------------------------- device plan
 * Block mapping of logical ranks onto G GPUs: gpu(r) = r / ceil(P/G).
 * Buffers of GPU g (byte offsets inside four regions):
 *   XG_BUF_SEND  send segments of its ranks (a2m: each local rank A segs;
 *                m2a: each local aggregator rank P segs), rank-major
 *   XG_BUF_RECV  receive slots (a2m: each local aggregator rank P slots;
 *                m2a: each local rank A slots), rank-major
 *   XG_BUF_STAGE_SEND / XG_BUF_STAGE_RECV  packed per-peer staging
 *   XG_BUF_SCRATCH  TAM aggregation buffers of its ranks (aggregate_buf,
 *                send_buf2, recv_buf of collective_write), rank-major
 */
enum { XG_BUF_SEND = 0, XG_BUF_RECV = 1, XG_BUF_STAGE_SEND = 2, XG_BUF_STAGE_RECV = 3, XG_BUF_SCRATCH = 4,
       XG_NBUF = 5 };

typedef struct {
    int64_t src_off, dst_off, len;
    int32_t src_buf, dst_buf;
} xg_copy;

typedef struct {
    int64_t off, len;
    int32_t peer, buf;
    int32_t is_send;
    int32_t group;                    /* RCCL group of the step: 0, or 1 (relay form: the forwards) */
} xg_p2p;

typedef struct {
    int32_t pre_begin, pre_count;     /* local copies + packs   (before the exchange) */
    int32_t p2p_begin, p2p_count;     /* grouped RCCL send/recv                       */
    int32_t post_begin, post_count;   /* unpacks                (after the exchange)  */
    int32_t sync_after;               /* 1: device-side barrier of all GPUs after it  */
    int32_t stage_count;              /* the first stage_count pre copies (rank-local
                                         memcpy's through SCRATCH) run in a launch of
                                         their own, ahead of the other pre copies     */
    int32_t posts;                    /* request posts (Isend/Irecv/... ) the GPU's ranks
                                         make in this step: a graph replay shares its
                                         launch time out in proportion (xg_plan_run)  */
} xg_stepplan;

typedef struct {
    int32_t gpu, ngpus, nsteps, pad;
    int64_t region_bytes[XG_NBUF];    /* send, recv, stage_send, stage_recv, scratch  */
    int32_t ncopy, np2p;
    xg_copy *copies;
    xg_p2p *p2p;
    xg_stepplan *steps;
    int64_t local_bytes, remote_send_bytes, remote_recv_bytes;   /* per whole plan  */
} xg_devplan;

/* Ranks hosted by GPU g: [*lo, *hi). */
void xg_block_range(int procs, int ngpus, int g, int *lo, int *hi);
int xg_gpu_of(int procs, int ngpus, int rank);

/* Region sizes and per-rank region offsets (-1 if the rank has no such buffer
 * on that GPU). */
int64_t xg_send_offset(const xg_sched *s, int ngpus, int rank);
int64_t xg_recv_offset(const xg_sched *s, int ngpus, int rank);
int64_t xg_scratch_offset(const xg_sched *s, int ngpus, int rank);
int64_t xg_region_bytes(const xg_sched *s, int ngpus, int g, int buf);

/* Build GPU g's share of every step.  pack_max_seg: per (step, peer), pack the
 * segments into one staging buffer when there are >= 2 and their mean length
 * is < pack_max_seg (0 = never pack); otherwise one RCCL op per segment. */
xg_devplan *xg_devplan_build(const xg_sched *s, int ngpus, int g, int64_t pack_max_seg);
/* The same, packing a (step, peer) transfer list only when it also moves >= pack_min bytes
 * (smaller lists go one RCCL call per segment: cheaper than a pack and an unpack launch). */
xg_devplan *xg_devplan_build_ex(const xg_sched *s, int ngpus, int g, int64_t pack_max_seg, int64_t pack_min);
/* The same with the form of a packed list chosen (the two above use XG_PACK_FORM_DEFAULT):
 *   XG_PACK_TWO_SIDED  one staging buffer per peer per direction: the sender packs every
 *                      segment, one RCCL call, the receiver unpacks every segment;
 *   XG_PACK_ONE_SIDED  the list in destination (or source) order, merged into runs that are
 *                      contiguous there: one RCCL call per run, straight into (out of) the
 *                      slots; only the runs not contiguous on the other side are staged, by
 *                      the sender (or the receiver) -- each byte copied on one side at most.
 *                      Of the two orders the one with fewer copied bytes + XG_RUN_CALL_BYTES
 *                      per call; ties: destination order (devplan.c, oneside).
 * One-sided halves the copied bytes but posts more calls (configs[2] on 8 GPUs: 2 per peer and
 * direction instead of 1).  On one MI355X, where a virtual 8-GPU job moves every pair as an
 * RCCL self send/recv and those serialize at ~3 us per call, two-sided is the faster form
 * (profiles/r03/pack_forms/), so it is the default; bench.py times direct, one-sided and
 * two-sided per method at N > 1 and keeps the fastest.  Any other form value means
 * XG_PACK_FORM_DEFAULT.  The alltoallw translate this replaces: mpi_test.c:233-302. */
/*   XG_RELAY           no packing; two-phase (Valiant) routing of the steps it pays for: each
 *                      cross-GPU message of such a step is cut into G 16-B aligned pieces; pieces
 *                      0 and 1 go straight to the destination (piece 0 in the step's first RCCL
 *                      group, piece 1 in its second), piece 2 + i through relay GPU R[i] (the G - 2
 *                      GPUs other than source and destination, ascending): received into the
 *                      relay's STAGE_RECV in the first group, forwarded in the second.  Every link
 *                      (a -> h) then carries egress(a) / G in group 0 and every link (h -> b)
 *                      ingress(b) / G in group 1, whatever the traffic matrix.  A step is relayed
 *                      when (max egress + max ingress) / G <= XG_RELAY_GAIN x its busiest GPU pair's
 *                      bytes and every cross-GPU message is >= XG_RELAY_MIN_BYTES: pairwise m9 / m10
 *                      (one XOR partner per round, 16 -> 4 MiB of link time per round at configs[3]),
 *                      configs[4]'s half-sync m11.  Other steps: direct.  No copy kernel touches a
 *                      relayed byte (link-load table).
 *   XG_RELAY_COALESCED the relay form's steps, pieces and hops (the same link load), with each
 *                      hop's pieces gathered into one call: group 0, per peer h, one call for the
 *                      pieces that end at h and one for those h relays (by destination); group 1,
 *                      per peer b, one call for this GPU's own second pieces and one per source
 *                      whose pieces it forwards to b.  A call of one piece moves in place; a longer
 *                      one is packed into STAGE_SEND / unpacked out of STAGE_RECV.  Pairwise rounds:
 *                      G - 1 sends + G - 1 receives per group, where XG_RELAY posts a call per
 *                      piece (RCCL's per-call cost: profiles/r06/relay_cost.log).  A step the
 *                      uniform cut does not help may take a weighted two-hop split instead
 *                      (Frank-Wolfe per step, shares in 1/1024ths of each GPU pair) when that
 *                      carries <= 0.85 of its busiest pair's bytes: configs[4]'s m7. */
enum { XG_PACK_TWO_SIDED = 0, XG_PACK_ONE_SIDED = 1, XG_RELAY = 2, XG_RELAY_COALESCED = 3 };
#define XG_PACK_FORM_DEFAULT XG_PACK_TWO_SIDED
#define XG_RUN_CALL_BYTES (1 << 20)
#define XG_RELAY_MIN_BYTES (1 << 20)
#define XG_RELAY_GAIN 0.8
xg_devplan *xg_devplan_build_form(const xg_sched *s, int ngpus, int g, int64_t pack_max_seg, int64_t pack_min,
                                  int form);
/* All three return NULL (nothing leaked) when the host runs out of memory while building: every
 * rank of a job builds plans, and xg_run_method turns a NULL on any rank into an error all ranks
 * agree on before any of them posts a call.  xg_devplan_free(NULL) is a no-op. */
void xg_devplan_free(xg_devplan *p);

/* ---------------------------------------------------------------- RCCL calls (calls.c)
 * The calls GPU dp->gpu posts in step `step`, in issue order: its send/recv calls
 * (one ncclGroupStart/End around them; a relay step's second group follows an
 * XG_CALL_FENCE), then XG_CALL_BARRIER (one ncclAllReduce)
 * when the step ends in an in-loop MPI_Barrier.  self_max > 0: a step that posts
 * cross-GPU calls and whose local gather/scatter copies move <= self_max bytes
 * posts those copies inside the same group as self send/recv pairs (peer = dp->gpu,
 * send then receive per copy; xg_devplan_step_self_calls counts them, 0 = the copies
 * stay copy-kernel launches) -- one RCCL launch then carries the whole step.  The
 * runtime posts exactly this list (replaces the Issend/Irecv/Sendrecv/Alltoallw
 * posts, mpi_test.c:1776,1790, :551,558, :627,912).  Returns the count (out may be
 * NULL), -1 for a bad step. */
enum { XG_CALL_SEND = 1, XG_CALL_RECV = 2, XG_CALL_BARRIER = 3, XG_CALL_FENCE = 4 };
typedef struct {
    int32_t kind, peer, buf, pad;     /* peer: GPU; buf: region (XG_BUF_*) */
    int64_t off, len;
} xg_call;
int xg_devplan_step_calls(const xg_devplan *dp, int step, int64_t self_max, xg_call *out);
int xg_devplan_step_self_calls(const xg_devplan *dp, int step, int64_t self_max);

/* RCCL's pairing of the calls of a G-GPU job: per ordered GPU pair (src, dst), the
 * k-th send of src to dst with the k-th receive of dst from src, in issue order
 * over the WHOLE run (RCCL's per-peer FIFO knows no steps).  calls[g] / step_begin[g]
 * (nsteps + 1 entries): GPU g's calls and where each step's start.  Accepted only if
 * every pair falls in one step and one group of it (groups: separated by XG_CALL_FENCE)
 * with one length and every GPU ends the same steps with a barrier (each its step's
 * last call) -- then no group can wait for one a peer posts later.  Returns the number
 * of pairs, written in (step, group) order (inside a group by src, dst, k) to out when
 * max_pairs suffices; -1 and a reason in err otherwise. */
typedef struct {
    int32_t step, src, dst;
    int32_t send_call, recv_call;     /* indices into calls[src] / calls[dst] */
    int32_t group;                    /* the step's RCCL group both calls are in */
    int64_t len;
} xg_call_pair;
int64_t xg_calls_match(int ngpus, int nsteps, const xg_call *const *calls, const int32_t *const *step_begin,
                       xg_call_pair *out, int64_t max_pairs, char *err, size_t errlen);
/* The same over the G device plans of one job (plans[g]: GPU g's, same schedule), their
 * calls listed with self_max as xg_devplan_step_calls lists them. */
int64_t xg_devplans_match(const xg_devplan *const *plans, int ngpus, int64_t self_max, xg_call_pair *out,
                          int64_t max_pairs, char *err, size_t errlen);

/* Step engine ordering (xg.h xg_plan_engine; kernels.h step_engine_kernel).  The
 * transfers of step s are xfer[step_begin[s] .. step_begin[s+1]) (device addresses
 * as integers).  flags[s] says what the barrier after step s orders:
 *   2  step s+1 reads bytes written since the last hazard point, or rewrites them
 *      with other bytes (another source at another dst-src offset): stores drained
 *      + agent release/acquire, and no early load of step s+1;
 *   1  stores drained before arriving (the last step; every step with force);
 *   0  nothing (identical rewrites of the -k repetitions are not hazards).
 * Returns the number of hazard points (flag 2). */
typedef struct { uint64_t src, dst, len; } xg_span;
int xg_engine_hazards(const xg_span *xfer, const int *step_begin, int nsteps, int force, int *flags);

/* Solo engine tables of one hazard-free run of steps (xg.h XG_SOLO_RAILS; kernels.h
 * solo_engine_kernel, whose constants must equal these).  Pieces of <= XG_SOLO_PIECE
 * bytes, every transfer 16-B aligned and within XG_SOLO_OFF_MAX 16-B units of
 * src_base / dst_base; dealt round-robin over rails = min(rails_max, pieces / waves, >= 1).
 * Per rail r, npieces descriptors at descs[r * npieces]: bits 0-23 source offset,
 * 24-47 destination offset (16-B units from the bases), 48-54 length (16-B units;
 * 0 = empty padding), 55-59 `before` = how many of its row's step barriers precede
 * it.  meta: [rails][nrows + 1] barriers per row (rows of `waves` pieces), then
 * [rails][nsteps] the step each barrier closes, in order, -1 past the last (a rail
 * places a barrier only after a step it had pieces in, in front of its next piece),
 * then [rails] the rows that hold real pieces (the rest is padding, never executed).
 * descs / meta NULL: fill *shape only.  Returns 0, or XG_EARG (xg.h) for bad input or
 * npieces > XG_SOLO_MAX_PIECES (*shape still filled), XG_ENOMEM. */
#define XG_SOLO_WAVES 16         /* waves of a workgroup rail; `waves` = 1: every rail one wave */
#define XG_SOLO_MAX_RAILS 512
#define XG_SOLO_PIECE 1024
#define XG_SOLO_K 8
#define XG_SOLO_MAX_STEPS 2048
#define XG_SOLO_MAX_PIECES 4608
#define XG_SOLO_OFF_MAX (1ull << 24)
/* waves = 1 (one-wave rails): the WIDE form -- descriptor = src | dst << 32 (granules, so
 * windows of XG_SOLO_WIDE_OFF_MAX granules), and each row's meta word = barrier count (bits
 * 0-7, all preceding the row's one piece) | the piece's length in granules << 8. */
#define XG_SOLO_WIDE_OFF_MAX (1ull << 32)
typedef struct { int32_t rails, npieces, nrows, nmeta; } xg_solo_shape;
int xg_solo_tables(const xg_span *xfer, const int *step_begin, int nsteps, int rails_max, int waves,
                   uint64_t src_base, uint64_t dst_base, xg_solo_shape *shape, uint64_t *descs, int *meta);
/* The same with offsets and lengths in units of `granule` bytes (16, 4 or 1; 4 and 1 only
 * for one-wave rails): every transfer granule-aligned, offsets within XG_SOLO_OFF_MAX
 * granules of the bases; bits 0-23 source, 24-47 destination offset, then the length
 * (7, 9 or 11 bits: up to XG_SOLO_PIECE bytes), then `before` at XG_SOLO_BEFORE_SHIFT.
 * Segment sizes that are not multiples of 16 (any -d) run on 4-B or 1-B accesses. */
#define XG_SOLO_BEFORE_SHIFT(g) ((g) == 16 ? 55 : (g) == 4 ? 57 : 59)
int xg_solo_tables_g(const xg_span *xfer, const int *step_begin, int nsteps, int rails_max, int waves, int granule,
                     uint64_t src_base, uint64_t dst_base, xg_solo_shape *shape, uint64_t *descs, int *meta);
/* Step times of a solo segment [s0, s1) from its rails' stamps (stamps[r * stride + t], 0 =
 * the rail closed nothing there): out[t] = max over rails of the rail's latest stamp <= t. */
void xg_solo_reduce_stamps(const uint64_t *stamps, int rails, int64_t stride, int s0, int s1, uint64_t *out);

/* Piece (= workgroup) size of one copy launch over copies of lengths lens[n]: among chunk,
 * chunk/2, ... >= 4 KiB (16-B multiples), the one whose busiest CU -- ceil(pieces / cus)
 * pieces of (size + wg_cost) bytes -- has the least work; ties keep the larger (pieces.c). */
int64_t xg_piece_size(const int64_t *lens, int n, int64_t chunk, int cus, int64_t wg_cost);
/* 1 if a local gather/scatter copy of step s (after its stage copies, before its packs)
 * reads or writes bytes that step s-1's unpacks write -- then the two may not share one copy
 * launch; 0 if they may; -1 for a bad step (pieces.c). */
int xg_step_local_meets_unpacks(const xg_devplan *dp, int s);
/* 1 if a pre copy of step s after its stage copies (local gather/scatter, packs) reads or writes
 * bytes a stage copy writes, or writes bytes one reads -- then the stage copies keep a launch of
 * their own; 0 if all may share one launch; -1 for a bad step (pieces.c). */
int xg_step_stage_meets_rest(const xg_devplan *dp, int s);

/* fill: `nsegs` consecutive d-byte segments at `off` in the SEND region,
 * segment i = fingerprint(rank, seed0 + i, iter) (prepare_*_data loops). */
typedef struct { int32_t rank, seed0; int64_t off; int32_t nsegs, pad; } xg_segrun;
/* verify: one d-byte receive slot at `off` in the RECV region that must hold
 * fingerprint(src, seed, iter); dst is the receiving logical rank. */
typedef struct { int32_t src, seed, dst, pad; int64_t off; } xg_slot;

enum { XG_FP_REFERENCE = 0, XG_FP_STRONG = 1 };   /* fingerprint modes */

/* Fill/verify descriptors of GPU g (host side, from the schedule's layout).
 * Return the count; out may be NULL to query it. */
int xg_fill_runs(const xg_sched *s, int ngpus, int g, xg_segrun *out);
int xg_verify_slots(const xg_sched *s, int ngpus, int g, xg_slot *out);

/* save_all_timing (mpi_test.c:2008-2066): the four per-repetition CSVs of m13,
 * <prefix>send_wait_all_times_<c>.csv, total_times, post_request_time,
 * barrier_time; timers = procs x ntimes, rank-major. */
int xg_save_all_timing(int procs, int ntimes, int comm_size, const xg_timer *timers, const char *prefix);

/* ---------------------------------------------------------------- report
 * summarize_results (mpi_test.c:2068-2118): 8 "| ..." lines on stdout and one
 * appended row (header on first write) in `filename`. */
int xg_summarize_results(int procs, int cb_nodes, int data_size, int comm_size, int ntimes,
                         int type, const char *filename, const char *prefix,
                         xg_timer timer1, xg_timer max_timer1);

#ifdef __cplusplus
}
#endif
#endif
