/*
 * oracle/pmpi_capture.c -- TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * PMPI interposition layer used to pin the oracle against the REAL reference.
 * It is linked (by oracle/Makefile) together with the unmodified reference
 * objects compiled from /root/reference/mpi_test.c + lustre_driver_test.c, and
 * records, per MPI rank, every point-to-point call the reference makes on the
 * hot path (methods 1-12) plus a checksum of every received segment:
 *
 *   B                         MPI_Barrier            (e.g. mpi_test.c:1762, :863, :1188)
 *   S <idx> <peer> <cnt> <tag> <comm> <mode>  send post; mode n = Issend (:1776),
 *                             i = Isend (:771, :1283), b = Send (:1099), r = Sendrecv (:1706)
 *   R <idx> <peer> <cnt> <tag> <comm> <addr>  recv post (Irecv :1772, Recv :982, Sendrecv :1706)
 *                             comm: 0 = MPI_COMM_WORLD, k = k-th other communicator seen
 *   W <idx> <idx> ...         one completion point   (Waitall :1781, blocking calls)
 *   D <src> <cnt> <addr> <chk>  bytes received       (checked when the wait returns)
 *   A <recvcounts...>         MPI_Alltoallw           (:627, :637, :912, :922)
 *   E                         MPI_Reduce = end of one method run (:2184 ...)
 *
 * The checksum is xg_chk64 (see DESIGN.md "checksum"): position-keyed
 * splitmix64 words summed mod 2^64, plus a length term.  The same function is
 * implemented by the numpy oracle and the HIP verify kernel.
 *
 * Output: $XG_CAPTURE_DIR/cap_<rank>.txt (one file per rank).
 */
#include <mpi.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static FILE *cap_fp;
static MPI_Comm comms[16];
static int ncomms;

static int comm_id(MPI_Comm c)
{
    int i;
    if (c == MPI_COMM_WORLD) return 0;
    for (i = 0; i < ncomms; ++i)
        if (comms[i] == c) return i + 1;
    if (ncomms < 16) comms[ncomms++] = c;
    return ncomms;
}
static int cap_rank = -1;
static long post_idx;

typedef struct {
    MPI_Request req;
    long idx;
    int is_recv, peer, count;
    const void *buf;
} live_req;

#define MAX_LIVE 65536
static live_req live[MAX_LIVE];
static int nlive;

static uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static uint64_t chk64(const unsigned char *p, long n)
{
    uint64_t s = (uint64_t)n * 0xD6E8FEB86659FD93ULL;
    long q, nw = (n + 7) / 8;
    for (q = 0; q < nw; ++q) {
        uint64_t w = 0;
        int b;
        for (b = 0; b < 8 && q * 8 + b < n; ++b)
            w |= (uint64_t)p[q * 8 + b] << (8 * b);
        s += mix64(w ^ ((uint64_t)q * 0x9E3779B97F4A7C15ULL));
    }
    return s;
}

static void cap_open(void)
{
    char path[4096];
    const char *dir;
    if (cap_fp) return;
    PMPI_Comm_rank(MPI_COMM_WORLD, &cap_rank);
    dir = getenv("XG_CAPTURE_DIR");
    snprintf(path, sizeof path, "%s/cap_%d.txt", dir ? dir : ".", cap_rank);
    cap_fp = fopen(path, "w");
    if (!cap_fp) { perror(path); PMPI_Abort(MPI_COMM_WORLD, 3); }
}

static void add_live(MPI_Request r, long idx, int is_recv, int peer, int count, const void *buf)
{
    if (nlive >= MAX_LIVE) { fprintf(stderr, "capture: too many live requests\n"); PMPI_Abort(MPI_COMM_WORLD, 4); }
    live[nlive].req = r; live[nlive].idx = idx; live[nlive].is_recv = is_recv;
    live[nlive].peer = peer; live[nlive].count = count; live[nlive].buf = buf;
    nlive++;
}

static int find_live(MPI_Request r)
{
    int i;
    for (i = 0; i < nlive; ++i)
        if (live[i].req == r) return i;
    return -1;
}

static void drop_live(int i) { live[i] = live[--nlive]; }

static void emit_data(int src, int count, const void *buf)
{
    if (count <= 0) return;   /* zero-byte messages carry no data (pairwise m9/m10, m18 signals) */
    fprintf(cap_fp, "D %d %d %p %016llx\n", src, count, buf,
            (unsigned long long)chk64((const unsigned char *)buf, count));
}

int MPI_Barrier(MPI_Comm comm)
{
    cap_open();
    fprintf(cap_fp, "B\n");
    return PMPI_Barrier(comm);
}

int MPI_Reduce(const void *sb, void *rb, int count, MPI_Datatype dt, MPI_Op op, int root, MPI_Comm comm)
{
    cap_open();
    fprintf(cap_fp, "E\n");
    fflush(cap_fp);
    post_idx = 0;
    nlive = 0;
    return PMPI_Reduce(sb, rb, count, dt, op, root, comm);
}

static int isend_common(int sync, const void *buf, int count, MPI_Datatype dt, int dest, int tag,
                        MPI_Comm comm, MPI_Request *req)
{
    int rc;
    cap_open();
    rc = sync ? PMPI_Issend(buf, count, dt, dest, tag, comm, req)
              : PMPI_Isend(buf, count, dt, dest, tag, comm, req);
    fprintf(cap_fp, "S %ld %d %d %d %d %c\n", post_idx, dest, count, tag, comm_id(comm), sync ? 'n' : 'i');
    add_live(*req, post_idx, 0, dest, count, buf);
    post_idx++;
    return rc;
}

int MPI_Issend(const void *buf, int count, MPI_Datatype dt, int dest, int tag, MPI_Comm comm, MPI_Request *req)
{ return isend_common(1, buf, count, dt, dest, tag, comm, req); }

int MPI_Isend(const void *buf, int count, MPI_Datatype dt, int dest, int tag, MPI_Comm comm, MPI_Request *req)
{ return isend_common(0, buf, count, dt, dest, tag, comm, req); }

int MPI_Irecv(void *buf, int count, MPI_Datatype dt, int src, int tag, MPI_Comm comm, MPI_Request *req)
{
    int rc;
    cap_open();
    rc = PMPI_Irecv(buf, count, dt, src, tag, comm, req);
    fprintf(cap_fp, "R %ld %d %d %d %d %p\n", post_idx, src, count, tag, comm_id(comm), buf);
    add_live(*req, post_idx, 1, src, count, buf);
    post_idx++;
    return rc;
}

int MPI_Waitall(int n, MPI_Request reqs[], MPI_Status st[])
{
    int i, rc, *slot = (int *)malloc(sizeof(int) * (n > 0 ? n : 1));
    cap_open();
    fprintf(cap_fp, "W");
    for (i = 0; i < n; ++i) {
        slot[i] = reqs[i] == MPI_REQUEST_NULL ? -1 : find_live(reqs[i]);
        if (slot[i] >= 0) fprintf(cap_fp, " %ld", live[slot[i]].idx);
    }
    fprintf(cap_fp, "\n");
    rc = PMPI_Waitall(n, reqs, st);
    /* emit data for completed receives, then drop them (highest slot first keeps indices valid) */
    for (i = 0; i < n; ++i)
        if (slot[i] >= 0 && live[slot[i]].is_recv)
            emit_data(live[slot[i]].peer, live[slot[i]].count, live[slot[i]].buf);
    {
        /* collect & drop */
        int k, j;
        for (k = 0; k < n; ++k) {
            int best = -1;
            for (j = 0; j < n; ++j)
                if (slot[j] >= 0 && (best < 0 || slot[j] > slot[best])) best = j;
            if (best < 0) break;
            drop_live(slot[best]);
            slot[best] = -1;
        }
    }
    free(slot);
    return rc;
}

int MPI_Wait(MPI_Request *req, MPI_Status *st)
{
    return MPI_Waitall(1, req, st == MPI_STATUS_IGNORE ? MPI_STATUSES_IGNORE : st);
}

int MPI_Send(const void *buf, int count, MPI_Datatype dt, int dest, int tag, MPI_Comm comm)
{
    int rc;
    cap_open();
    fprintf(cap_fp, "S %ld %d %d %d %d b\nW %ld\n", post_idx, dest, count, tag, comm_id(comm), post_idx);
    post_idx++;
    rc = PMPI_Send(buf, count, dt, dest, tag, comm);
    return rc;
}

int MPI_Recv(void *buf, int count, MPI_Datatype dt, int src, int tag, MPI_Comm comm, MPI_Status *st)
{
    int rc;
    cap_open();
    fprintf(cap_fp, "R %ld %d %d %d %d %p\nW %ld\n", post_idx, src, count, tag, comm_id(comm), buf, post_idx);
    post_idx++;
    rc = PMPI_Recv(buf, count, dt, src, tag, comm, st);
    emit_data(src, count, buf);
    return rc;
}

int MPI_Sendrecv(const void *sbuf, int scount, MPI_Datatype sdt, int dest, int stag,
                 void *rbuf, int rcount, MPI_Datatype rdt, int src, int rtag,
                 MPI_Comm comm, MPI_Status *st)
{
    int rc;
    cap_open();
    fprintf(cap_fp, "S %ld %d %d %d %d r\nR %ld %d %d %d %d %p\nW %ld %ld\n", post_idx, dest, scount, stag,
            comm_id(comm), post_idx + 1, src, rcount, rtag, comm_id(comm), rbuf, post_idx, post_idx + 1);
    post_idx += 2;
    rc = PMPI_Sendrecv(sbuf, scount, sdt, dest, stag, rbuf, rcount, rdt, src, rtag, comm, st);
    if (rbuf && rcount > 0) emit_data(src, rcount, rbuf);
    return rc;
}

int MPI_Alltoallw(const void *sbuf, const int scounts[], const int sdispls[], const MPI_Datatype stypes[],
                  void *rbuf, const int rcounts[], const int rdispls[], const MPI_Datatype rtypes[],
                  MPI_Comm comm)
{
    int rc, i, n;
    cap_open();
    PMPI_Comm_size(comm, &n);
    fprintf(cap_fp, "A");
    for (i = 0; i < n; ++i) fprintf(cap_fp, " %d", scounts[i]);
    fprintf(cap_fp, " |");
    for (i = 0; i < n; ++i) fprintf(cap_fp, " %d", rcounts[i]);
    fprintf(cap_fp, "\n");
    rc = PMPI_Alltoallw(sbuf, scounts, sdispls, stypes, rbuf, rcounts, rdispls, rtypes, comm);
    for (i = 0; i < n; ++i)
        if (rcounts[i] > 0) emit_data(i, rcounts[i], (const char *)rbuf + rdispls[i]);
    return rc;
}

int MPI_Finalize(void)
{
    if (cap_fp) { fclose(cap_fp); cap_fp = NULL; }
    return PMPI_Finalize();
}
