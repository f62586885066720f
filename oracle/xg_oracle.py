"""xg_oracle -- CPU restatement of the reference hot path.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker.  The product (libxghost / libxg) never
calls it.

What it restates (every function cites the reference line it follows):
  * aggregator placement            create_aggregator_list   mpi_test.c:1952-2006
  * segment fingerprint             MAP_DATA / fill_buffer   mpi_test.c:23, :71-77
  * buffer layouts                  prepare_*_data           mpi_test.c:94-133, :162-202
  * alltoallw counts/displacements  *_alltoall_translate     mpi_test.c:233-302
  * the per-rank MPI programs of methods 1..14, 17..20         mpi_test.c:421-1950
  * TAM (m15/m16): static_node_assignment + collective_write   lustre_driver_test.c:359-429, :944-1309
  * MPI point-to-point matching (non-overtaking per (src,dst,tag)) and
    collective matching for MPI_Alltoallw, executed with byte copies.

It is pinned against the real reference: tests/golden/ holds per-rank MPI
call traces and received-segment checksums captured with oracle/pmpi_capture.c
from the reference binary (tests/golden/make_golden.py); tests/test_oracle.py
checks this module against every one of them.

Program ops (one list per rank, in program order):
  ('B',)                               MPI_Barrier (collective; before or inside the timed region)
  ('s', peer, cnt, seg, eager_ok, comm, tag, isend)
                                       send post.  Issend: eager_ok False; Send / Sendrecv half /
                                       Isend: eager_ok True (complete locally when cnt <= eager
                                       limit).  comm 0 = MPI_COMM_WORLD; tag None = rank + peer.
  ('r', peer, cnt, slot, comm, tag)    recv post (Irecv / Recv / Sendrecv half)
  ('w', [post indices])                one completion point (Waitall / blocking call)
  ('A', [(peer,cnt,seg)], [(peer,cnt,slot)])   MPI_Alltoallw (posts + completion)
  ('c', seg, slot, cnt)                self memcpy (mpi_test.c:1473, :1646, :1714, :1285, :1398)
  ('t', field, +1|-1)                  timer bracket: field in post|send|recv|barrier|total
  ('rep', m) ('mark', reg) ('delta', tgt, field, reg, mode) ('acc', dst, dfield, src, sfield)
  ('copyt', dst, dfield, src, sfield) ('zero', tgt, field)
                                       per-repetition timers of m13 (timers[m], :829-874):
                                       tgt 'G' = the method Timer, 'R' = timers[m]
Post indices count 's' and 'r' ops (and the posts of an 'A') in program order.
"""
import numpy as np

A2M_METHODS = (1, 3, 6, 7, 8, 9, 12, 13, 15, 17, 18, 19, 20)
M2A_METHODS = (2, 4, 5, 10, 11, 14, 16)
METHODS = tuple(range(1, 21))
TAM_METHODS = (15, 16)
LABELS = {  # mpi_test.c:2186 ... :2337
    1: "All to many", 2: "Many to all", 3: "All to many balanced", 4: "Many to all balanced",
    5: "Many to all benchmark", 6: "All to many sync", 7: "All to many half sync",
    8: "All to many benchmark", 9: "All to many pairwise", 10: "Many to all pairwise",
    11: "Many to all half sync", 12: "All to many half sync 2", 13: "All to many scattered",
    14: "Many to all scattered", 15: "All to many TAM", 16: "Many to all TAM",
    17: "All to many node robin", 18: "All to many balanced control",
    19: "All to many scattered isend", 20: "All to many balanced presend",
}


def direction(method):
    return "a2m" if method in A2M_METHODS else "m2a"


# --------------------------------------------------------------------------- placement
def aggregator_list(P, A, proc_node=1, agg_type=1):
    """create_aggregator_list, mpi_test.c:1952-2006 (incl. the type-1 quirk remainder = P / A, :1957)."""
    out = []
    if agg_type == 1:
        remainder, ceiling, floor = P // A, (P + A - 1) // A, P // A
        for i in range(A):
            out.append(ceiling * i if i < remainder else ceiling * remainder + floor * (i - remainder))
    elif agg_type == 0:
        out = list(range(A))
    elif agg_type == 2:
        remainder, ceiling, floor = P // A, (P + A - 1) // A, P // A
        for i in range(A):
            v = ceiling * i if i < remainder else ceiling * remainder + floor * (i - remainder)
            out.append((v - 16 + P * 16) % P)
    elif agg_type == 3:
        remainder = 0
        for i in range(A):
            out.append(remainder)
            remainder += proc_node
            if remainder >= P:
                remainder = remainder % proc_node + 1
    else:  # the reference leaves rank_list uninitialised for other types
        raise ValueError("aggregator type %d" % agg_type)
    return out


# --------------------------------------------------------------------------- bytes
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)
GOLD = np.uint64(0x9E3779B97F4A7C15)
LENK = 0xD6E8FEB86659FD93


def _mix64(z):
    z = (z ^ (z >> np.uint64(30))) * M1
    z = (z ^ (z >> np.uint64(27))) * M2
    return z ^ (z >> np.uint64(31))


def map_data(rank, seed, it, n):
    """fill_buffer, mpi_test.c:71-77: byte o = (char)(rank + o + seed + iter)."""
    return ((np.arange(n, dtype=np.int64) + (rank + seed + it)) & 0xFF).astype(np.uint8)


def strong_data(rank, seed, it, n):
    """Strong fingerprint (build extension, mode 1): byte o = byte (o&7) of
    mix64(key + (o>>3) * GOLD), key = rank<<42 ^ seed<<21 ^ iter.  Makes every
    (rank, seed, iter, offset) distinct, so a misroute the reference's weak
    MAP_DATA cannot see (equal rank+seed) is caught."""
    with np.errstate(over="ignore"):
        key = np.uint64((rank << 42) ^ (seed << 21) ^ it)
        nw = (n + 7) // 8
        words = _mix64(key + np.arange(nw, dtype=np.uint64) * GOLD)
    return words.view(np.uint8)[:n].copy()


def fingerprint(mode, rank, seed, it, n):
    return map_data(rank, seed, it, n) if mode == 0 else strong_data(rank, seed, it, n)


def chk64(buf):
    """xg_chk64: sum_q mix64(w_q ^ q*GOLD) + n*LENK (mod 2^64), w_q = LE u64 word q (zero padded)."""
    buf = np.asarray(buf, dtype=np.uint8)
    n = buf.size
    nw = (n + 7) // 8
    pad = np.zeros(nw * 8, dtype=np.uint8)
    pad[:n] = buf
    with np.errstate(over="ignore"):
        w = pad.view("<u8")
        h = _mix64(w ^ (np.arange(nw, dtype=np.uint64) * GOLD))
        s = int(h.sum(dtype=np.uint64)) + n * LENK
    return s & 0xFFFFFFFFFFFFFFFF


# --------------------------------------------------------------------------- layouts
def layout(method, P, A, rank_list):
    """Per-rank (n_send_segs, n_recv_slots); prepare_all_to_many_data :162-202 /
    prepare_many_to_all_data :94-133 (span = 1, so every segment is d bytes)."""
    aggs = set(rank_list)
    if direction(method) == "a2m":
        return {r: (A, P if r in aggs else 0) for r in range(P)}
    return {r: (P if r in aggs else 0, A) for r in range(P)}


def seg_seed(method, rank, seg):
    """Seed of send segment `seg` of `rank`: a2m seg index = aggregator index (:195-199);
    m2a seg index = destination rank (:106-110)."""
    return seg


def expected_recv(method, P, A, d, rank_list, it, mode=0):
    """Closed form of every receive slot: a2m aggregator index a, slot s <- MAP(s, seed=a);
    m2a rank r, slot i <- MAP(rank_list[i], seed=r) (check_buffer call sites :139, :215)."""
    out = {}
    if direction(method) == "a2m":
        for a, g in enumerate(rank_list):
            out[g] = np.concatenate([fingerprint(mode, s, a, it, d) for s in range(P)]) if P else None
    else:
        for r in range(P):
            out[r] = np.concatenate([fingerprint(mode, g, r, it, d) for g in rank_list])
    return out


# --------------------------------------------------------------------------- programs
class _Prog:
    def __init__(self):
        self.ops = []
        self.nposts = 0

    def s(self, peer, cnt, seg, eager_ok=False, comm=0, tag=None, isend=False, buf=None, off=0, esz=1):
        """buf None: segment `seg` of the SEND buffer; otherwise bytes [off, off+cnt*esz) of the
        rank's buffer `buf` ('AGG', 'SBUF2', 'RBUF', 'CTRL...')."""
        self.ops.append(("s", peer, cnt, seg, eager_ok or isend, comm, tag, isend, buf, off, esz))
        self.nposts += 1
        return self.nposts - 1

    def r(self, peer, cnt, slot, comm=0, tag=None, buf=None, off=0, esz=1):
        self.ops.append(("r", peer, cnt, slot, comm, tag, buf, off, esz))
        self.nposts += 1
        return self.nposts - 1

    def cp(self, sbuf, soff, dbuf, doff, n):
        """memcpy between (buffer, offset) locations of this rank; SEND/RECV offsets in bytes."""
        self.ops.append(("C", sbuf, soff, dbuf, doff, n))

    def w(self, idxs):
        self.ops.append(("w", list(idxs)))

    def send(self, peer, cnt, seg):          # blocking MPI_Send
        self.w([self.s(peer, cnt, seg, True)])

    def recv(self, peer, cnt, slot, comm=0, tag=None):   # blocking MPI_Recv
        self.w([self.r(peer, cnt, slot, comm, tag)])

    def ctrl(self, name, data):
        """host-side int array whose bytes a size message carries (TAM)."""
        self.ops.append(("K", name, np.asarray(data, dtype="<i4").view(np.uint8).copy()))

    def sendrecv(self, dst, scnt, seg, src, rcnt, slot):   # MPI_Sendrecv
        a = self.s(dst, scnt, seg, True)
        b = self.r(src, rcnt, slot)
        self.w([a, b])

    def t(self, field, sign):
        self.ops.append(("t", field, sign))

    def op(self, *args):
        self.ops.append(tuple(args))

    def alltoallw(self, sends, recvs):
        self.ops.append(("A", list(sends), list(recvs)))
        self.nposts += len(sends) + len(recvs)


def _window_start(idx, k, ceiling, floor, remainder):
    # mpi_test.c:1463-1467 / :1478-1482 (even block split by aggregator index)
    return k + idx * ceiling if idx < remainder else k + remainder * ceiling + (idx - remainder) * floor


def _in_window(rank, temp, cs, P):
    # the window test of mpi_test.c:1483-1499 (identical at :1617-1633), including its edge cases
    if (temp >= P and temp + cs >= P) or (temp < P and temp + cs < P):
        return temp % P <= rank < (temp + cs) % P
    return rank >= temp or rank < (temp + cs) % P


def programs(method, P, A, d, c, rank_list, ntimes, proc_node=1, barrier_type=0, it=0):
    """Per-rank op lists of method `method` exactly as the reference issues them."""
    aggidx = {g: i for i, g in enumerate(rank_list)}
    progs = []
    for rank in range(P):
        isagg = rank in aggidx
        # prepare_*: myindex is the LAST matching index (:111-115, :183-187)
        myindex = max(i for i, g in enumerate(rank_list) if g == rank) if isagg else 0
        p = _Prog()
        p.ops.append(("B",))
        p.t("total", +1)
        fn = _METHODS[method]
        if method in (13, 17):
            fn(p, rank, isagg, myindex, P, A, d, c, rank_list, ntimes, proc_node, barrier_type)
        elif method in (15, 16):
            fn(p, rank, isagg, myindex, P, A, d, c, rank_list, ntimes, proc_node, it)
        else:
            fn(p, rank, isagg, myindex, P, A, d, c, rank_list, ntimes)
        p.t("total", -1)
        progs.append(p.ops)
    return progs


def _m1(p, rank, isagg, myindex, P, A, d, c, rl, ntimes):          # all_to_many :1748-1824
    for _ in range(ntimes):
        if c >= P:
            p.t("post", +1)
            idx = []
            if isagg:
                idx += [p.r(i, d, i) for i in range(P)]
            idx += [p.s(rl[i], d, i) for i in range(A)]
            p.t("post", -1)
            if idx:
                p.t("recv", +1); p.w(idx); p.t("recv", -1)
        else:
            p.t("post", +1)
            sends = [p.s(rl[i], d, i) for i in range(A)]
            p.t("post", -1)
            steps = (P + c - 1) // c
            for k in range(steps):
                idx = []
                if isagg:
                    p.t("post", +1)
                    idx = [p.r(i, d, i) for i in range(k, P, steps)]
                    p.t("post", -1)
                if idx:
                    p.t("recv", +1); p.w(idx); p.t("recv", -1)
            if sends:
                p.t("send", +1); p.w(sends); p.t("send", -1)


def _m2(p, rank, isagg, myindex, P, A, d, c, rl, ntimes):          # many_to_all :1871-1950
    for _ in range(ntimes):
        if c >= P:
            p.t("post", +1)
            idx = [p.r(rl[i], d, i) for i in range(A)]
            if isagg:
                idx += [p.s(i, d, i) for i in range(P)]
            p.t("post", -1)
            if idx:
                p.t("recv", +1); p.w(idx); p.t("recv", -1)
        else:
            p.t("post", +1)
            recvs = [p.r(rl[i], d, i) for i in range(A)]
            p.t("post", -1)
            steps = (P + c - 1) // c
            for k in range(steps):
                idx = []
                if isagg:
                    p.t("post", +1)
                    idx = [p.s(i, d, i) for i in range(k, P, steps)]
                    p.t("post", -1)
                if idx:
                    p.t("send", +1); p.w(idx); p.t("send", -1)
            if recvs:
                p.t("recv", +1); p.w(recvs); p.t("recv", -1)


def _split(P, A):
    return (P + A - 1) // A, P // A, P % A


def _send_start(rank, ceiling, floor, remainder):                    # :1449-1453 / :1599-1603
    if rank >= remainder * ceiling:
        return remainder + (rank - remainder * ceiling) // floor
    return rank // ceiling


def _m3(p, rank, isagg, myindex, P, A, d, c, rl, ntimes):          # all_to_many_balanced :1422-1517
    if c > P:
        c = P
    bblock = c
    ceiling, floor, remainder = _split(P, A)
    send_start = _send_start(rank, ceiling, floor, remainder)
    for _ in range(ntimes):
        cs = bblock
        k = 0
        while k < P:
            if P - k < cs:
                cs = P - k
            idx = []
            if isagg:
                for i in range(cs):
                    temp = _window_start(myindex, k + i, ceiling, floor, remainder) % P
                    if temp != rank:
                        p.t("post", +1); idx.append(p.r(temp, d, temp)); p.t("post", -1)
                    else:
                        p.ops.append(("c", myindex, temp, d))
            for _x in range(A):
                temp = _window_start(send_start, k, ceiling, floor, remainder)
                if _in_window(rank, temp, cs, P):
                    if rl[send_start] != rank:
                        idx.append(p.s(rl[send_start], d, send_start))
                else:
                    break
                send_start = (send_start - 1 + A) % A
            if idx:
                fields = ("recv",) if isagg else ("recv", "send")
                for f in fields:
                    p.t(f, +1)
                p.w(idx)
                for f in fields:
                    p.t(f, -1)
            k += cs


def _m4(p, rank, isagg, myindex, P, A, d, c, rl, ntimes):          # many_to_all_balanced :1576-1663
    cs = P if c > P else c          # NOT reset between repetitions (:1604-1608)
    ceiling, floor, remainder = _split(P, A)
    send_start = _send_start(rank, ceiling, floor, remainder)
    for _ in range(ntimes):
        k = 0
        while k < P:
            if P - k < cs:
                cs = P - k
            idx = []
            p.t("post", +1)
            for _x in range(A):
                temp = _window_start(send_start, k, ceiling, floor, remainder)
                if _in_window(rank, temp, cs, P):
                    if rl[send_start] != rank:
                        idx.append(p.r(rl[send_start], d, send_start))
                else:
                    break
                send_start = (send_start - 1 + A) % A
            if isagg:
                for i in range(cs):
                    temp = _window_start(myindex, k + i, ceiling, floor, remainder) % P
                    if temp != rank:
                        idx.append(p.s(temp, d, temp))
                    else:
                        p.ops.append(("c", temp, myindex, d))
            p.t("post", -1)
            if idx:
                p.t("recv", +1); p.w(idx); p.t("recv", -1)
            k += cs


def _a2m_translate(rank, isagg, P, A, d, rl):                       # :233-262
    sc, sd = [0] * P, [0] * P
    for i in range(A):
        sd[rl[i]] = i * d
        sc[rl[i]] = d
    rc, rd = ([d] * P, [i * d for i in range(P)]) if isagg else ([0] * P, [0] * P)
    return sc, sd, rc, rd


def _m2a_translate(rank, isagg, P, A, d, rl):                       # :273-302
    rc, rd = [0] * P, [0] * P
    rd[rl[0]] = 0
    rc[rl[0]] = d
    for i in range(1, A):
        rd[rl[i]] = rd[rl[i - 1]] + d
        rc[rl[i]] = d
    sc, sd = ([d] * P, [i * d for i in range(P)]) if isagg else ([0] * P, [0] * P)
    return sc, sd, rc, rd


def _alltoallw(translate):
    def run(p, rank, isagg, myindex, P, A, d, c, rl, ntimes):       # :599-654 / :885-940
        sc, sd, rc, rd = translate(rank, isagg, P, A, d, rl)
        sends = [(q, sc[q], sd[q] // d if d else 0) for q in range(P) if sc[q] > 0]
        recvs = [(q, rc[q], rd[q] // d if d else 0) for q in range(P) if rc[q] > 0]
        for _ in range(ntimes):
            p.alltoallw(sends, recvs)
    return run


def _m6(p, rank, isagg, myindex, P, A, d, c, rl, ntimes):          # all_to_many_sync :1665-1746
    cs = A if c > A else c
    for _ in range(ntimes):
        k = 0
        while k < A:
            if A - k < cs:
                cs = A - k
            p.t("recv", +1)
            if isagg:
                for i in range(cs):
                    temp = (rank + k + i) % A
                    temp2 = (myindex - k - i + A) % A
                    if rl[temp] != rank and temp2 != rank:
                        p.sendrecv(rl[temp], d, temp, temp2, d, temp2)
                    elif rl[temp] == rank:
                        p.ops.append(("c", temp, rank, d))
                        if temp2 != rank:
                            p.recv(temp2, d, temp2)
                    elif temp2 == rank:
                        p.send(rl[temp], d, temp)
                    x = temp2 + A
                    while x < P:
                        if rank != x:
                            p.recv(x, d, x)
                        x += A
            else:
                for i in range(cs):
                    temp = (rank + k + i) % A
                    p.send(rl[temp], d, temp)
            p.t("recv", -1)
            k += cs


def _m7(p, rank, isagg, myindex, P, A, d, c, rl, ntimes):          # all_to_many_half_sync :1055-1114
    cs = A if c > A else c
    for _ in range(ntimes):
        k = 0
        while k < A:
            if A - k < cs:
                cs = A - k
            idx = []
            if isagg:
                for i in range(cs):
                    x = (myindex - k - i + A) % A
                    while x < P:
                        idx.append(p.r(x, d, x))
                        x += A
            for i in range(cs):
                temp = (rank + k + i) % A
                p.send(rl[temp], d, temp)
            p.t("recv", +1)
            if idx:
                p.w(idx)
            p.t("recv", -1)
            k += cs


def _m11(p, rank, isagg, myindex, P, A, d, c, rl, ntimes):         # many_to_all_half_sync :942-997
    cs = P if c > P else c
    stride = (P + A - 1) // A
    for _ in range(ntimes):
        k = 0
        while k < P:
            if P - k < cs:
                cs = P - k
            idx = []
            p.t("post", +1)
            if isagg:
                for i in range(cs):
                    temp = (stride * myindex + k + i) % P
                    idx.append(p.s(temp, d, temp))
            p.t("post", -1)
            p.t("recv", +1)
            for x in range(cs):
                for i in range(A):
                    if rank == (k + i * stride + x) % P:
                        p.recv(rl[i], d, i)
            if idx:
                p.w(idx)
            p.t("recv", -1)
            k += cs


def _m12(p, rank, isagg, myindex, P, A, d, c, rl, ntimes):         # all_to_many_half_sync2 :999-1053
    cs = A if c > A else c
    for _ in range(ntimes):
        k = 0
        while k < A:
            if A - k < cs:
                cs = A - k
            idx = []
            for i in range(cs):
                temp = (rank + k + i) % A
                idx.append(p.s(rl[temp], d, temp))
            if isagg:
                for i in range(cs):
                    x = (myindex - k - i + A) % A
                    while x < P:
                        p.recv(x, d, x)
                        x += A
            p.t("recv", +1)
            if idx:
                p.w(idx)
            p.t("recv", -1)
            k += cs


def _pairwise(translate):
    def run(p, rank, isagg, myindex, P, A, d, c, rl, ntimes):       # :421-508 / :510-597
        sc, sd, rc, rd = translate(rank, isagg, P, A, d, rl)
        i = 1
        while i < P:
            i *= 2
        pof2 = i == P
        for _ in range(ntimes):
            for i in range(P):
                if pof2:
                    src = dst = rank ^ i
                else:
                    src, dst = (rank - i + P) % P, (rank + i) % P
                p.sendrecv(dst, sc[dst], sd[dst] // d if sc[dst] else -1,
                           src, rc[src], rd[src] // d if rc[src] else -1)
    return run


def _scattered_block(P, c):
    # :740-750 / :815-825 / :674-684
    if c > P:
        c = P
    return c if c != 0 else P


def _m13(p, rank, isagg, myindex, P, A, d, c, rl, ntimes, proc_node=1, barrier_type=0):
    """all_to_many_scattered, mpi_test.c:797-882 (barrier type -b, per-repetition timers[m])."""
    sc, sd, rc, rd = _a2m_translate(rank, isagg, P, A, d, rl)
    bblock = _scattered_block(P, c)
    for m in range(ntimes):
        p.op("rep", m)
        p.op("mark", "T2")
        p.op("zero", "R", "barrier")
        for ii in range(0, P, bblock):
            ss = min(P - ii, bblock)
            idx = []
            p.op("mark", "S")
            for i in range(ss):
                dst = (rank + i + ii) % P
                if rc[dst]:
                    idx.append(p.r(dst, rc[dst], rd[dst] // d if d else 0))
            for i in range(ss):
                dst = (rank - i - ii + P) % P
                if sc[dst]:
                    idx.append(p.s(dst, sc[dst], sd[dst] // d if d else 0))
            p.op("delta", "R", "post", "S", "set")
            p.op("acc", "G", "post", "R", "post")
            if idx:
                p.op("mark", "S")
                p.w(idx)
                p.op("delta", "R", "recv", "S", "set")
                p.op("acc", "G", "recv", "R", "recv")
                if not isagg:
                    p.op("acc", "G", "send", "R", "recv")
                    p.op("copyt", "R", "send", "R", "recv")
            if barrier_type == 2:
                p.op("mark", "S")
                p.ops.append(("B",))
                p.op("delta", "R", "barrier", "S", "add")
                p.op("acc", "G", "barrier", "R", "barrier")
        p.op("delta", "R", "total", "T2", "set")
        if barrier_type == 1:
            p.op("mark", "S")
            p.ops.append(("B",))
            p.op("delta", "R", "barrier", "S", "set")
            p.op("acc", "G", "barrier", "R", "barrier")


def _m14(p, rank, isagg, myindex, P, A, d, c, rl, ntimes):
    """many_to_all_scattered, mpi_test.c:656-720."""
    sc, sd, rc, rd = _m2a_translate(rank, isagg, P, A, d, rl)
    bblock = _scattered_block(P, c)
    for _ in range(ntimes):
        for ii in range(0, P, bblock):
            ss = min(P - ii, bblock)
            idx = []
            p.t("post", +1)
            for i in range(ss):
                dst = (rank + i + ii) % P
                if rc[dst]:
                    idx.append(p.r(dst, rc[dst], rd[dst] // d if d else 0))
            for i in range(ss):
                dst = (rank - i - ii + P) % P
                if sc[dst]:
                    idx.append(p.s(dst, sc[dst], sd[dst] // d if d else 0))
            p.t("post", -1)
            if idx:
                p.t("recv", +1); p.w(idx); p.t("recv", -1)


def node_robin_map(rank, proc_node, P):
    """node_robin_map, mpi_test.c:1116-1133 -> (map, rank_index)."""
    mp, count, j, rank_index = [0] * P, 0, 0, 0
    for i in range(P):
        mp[i] = count
        if count == rank:
            rank_index = i
        count += proc_node
        if count >= P:
            j += 1
            count = j
    return mp, rank_index


def _m17(p, rank, isagg, myindex, P, A, d, c, rl, ntimes, proc_node=1, barrier_type=0):
    """all_to_many_node_robin, mpi_test.c:1135-1227 (barrier inside every round)."""
    mp, rank_index = node_robin_map(rank, proc_node, P)
    if c > P:
        c = P
    bblock = c
    ceiling, floor, remainder = _split(P, A)
    send_start = _send_start(rank_index, ceiling, floor, remainder)
    for _ in range(ntimes):
        cs = bblock
        k = 0
        while k < P:
            if P - k < cs:
                cs = P - k
            idx = []
            p.t("post", +1)
            if isagg:
                for i in range(cs):
                    temp = mp[_window_start(myindex, k + i, ceiling, floor, remainder) % P]
                    idx.append(p.r(temp, d, temp))
            p.ops.append(("B",))
            for _x in range(A):
                temp = _window_start(send_start, k, ceiling, floor, remainder)
                if not _in_window(rank_index, temp, cs, P):
                    break
                idx.append(p.s(rl[send_start], d, send_start))
                send_start = (send_start - 1 + A) % A
            p.t("post", -1)
            if idx:
                fields = ("recv",) if isagg else ("recv", "send")
                for f in fields:
                    p.t(f, +1)
                p.w(idx)
                for f in fields:
                    p.t(f, -1)
            k += cs


def _m18(p, rank, isagg, myindex, P, A, d, c, rl, ntimes):
    """all_to_many_balanced_control, mpi_test.c:1229-1336 (0-byte go-signals on a dup'd comm)."""
    if c > P:
        c = P
    bblock = c
    ceiling, floor, remainder = _split(P, A)
    send_start = _send_start(rank, ceiling, floor, remainder)
    for _ in range(ntimes):
        cs = bblock
        k = 0
        while k < P:
            if P - k < cs:
                cs = P - k
            idx = []
            p.t("post", +1)
            if isagg:
                for i in range(cs):
                    temp = _window_start(myindex, k + i, ceiling, floor, remainder) % P
                    if temp != rank:
                        idx.append(p.r(temp, d, temp))
                        idx.append(p.s(temp, 0, -1, comm=1, tag=rank + temp * 100, isend=True))
                    else:
                        p.ops.append(("c", myindex, temp, d))
            for _x in range(A):
                temp = _window_start(send_start, k, ceiling, floor, remainder)
                if not _in_window(rank, temp, cs, P):
                    break
                if rl[send_start] != rank:
                    p.recv(rl[send_start], 0, -1, comm=1, tag=rank * 100 + rl[send_start])
                    idx.append(p.s(rl[send_start], d, send_start))
                send_start = (send_start - 1 + A) % A
            p.t("post", -1)
            if idx:
                fields = ("recv",) if isagg else ("recv", "send")
                for f in fields:
                    p.t(f, +1)
                p.w(idx)
                for f in fields:
                    p.t(f, -1)
            k += cs


def _m19(p, rank, isagg, myindex, P, A, d, c, rl, ntimes):
    """all_to_many_scattered_isend, mpi_test.c:722-795 (MPI_Isend; barrier before the total stop)."""
    sc, sd, rc, rd = _a2m_translate(rank, isagg, P, A, d, rl)
    bblock = _scattered_block(P, c)
    for _ in range(ntimes):
        for ii in range(0, P, bblock):
            ss = min(P - ii, bblock)
            idx = []
            for i in range(ss):
                dst = (rank + i + ii) % P
                if rc[dst]:
                    idx.append(p.r(dst, rc[dst], rd[dst] // d if d else 0))
            for i in range(ss):
                dst = (rank - i - ii + P) % P
                if sc[dst]:
                    if not isagg:
                        p.t("post", +1)
                    idx.append(p.s(dst, sc[dst], sd[dst] // d if d else 0, isend=True))
                    if not isagg:
                        p.t("post", -1)
            if idx:
                fields = ("recv",) if isagg else ("recv", "send")
                for f in fields:
                    p.t(f, +1)
                p.w(idx)
                for f in fields:
                    p.t(f, -1)
    p.ops.append(("B",))


def _m20(p, rank, isagg, myindex, P, A, d, c, rl, ntimes):
    """all_to_many_balanced_pre_send, mpi_test.c:1338-1419."""
    if c > P:
        c = P
    bblock = c
    ceiling, floor, remainder = _split(P, A)
    send_start = _send_start(rank, ceiling, floor, remainder)
    for _ in range(ntimes):
        cs = bblock
        sends = []
        for k in range(A):
            i = (send_start - k + A) % A
            if rl[i] != rank:
                sends.append(p.s(rl[i], d, i))
        k = 0
        while k < P:
            if P - k < cs:
                cs = P - k
            idx = []
            if isagg:
                for i in range(cs):
                    temp = _window_start(myindex, k + i, ceiling, floor, remainder) % P
                    if temp != rank:
                        p.t("post", +1); idx.append(p.r(temp, d, temp)); p.t("post", -1)
                    else:
                        p.ops.append(("c", myindex, temp, d))
            if idx:
                p.t("recv", +1); p.w(idx); p.t("recv", -1)
            k += cs
        if sends:
            p.t("send", +1); p.w(sends); p.t("send", -1)


def static_node_assignment(rank, P, proc_node):
    """static_node_assignment type 0 (lustre_driver_test.c:404-427) as called by the TAM methods
    (mpi_test.c:341, :395): nodes of proc_node consecutive ranks; proxy = first rank of a node.
    -> (nprocs_node of this rank, nrecvs, local_ranks, global_receivers, process_node_list)"""
    nrecvs = (P + proc_node - 1) // proc_node
    local_ranks = [(rank // proc_node) * proc_node + i for i in range(proc_node)]
    receivers = [i * proc_node for i in range(nrecvs)]
    node_of = [i // proc_node for i in range(P)]
    npn = proc_node
    if rank >= (nrecvs - 1) * proc_node:
        npn = P - proc_node * (nrecvs - 1)
    return npn, nrecvs, local_ranks, receivers, node_of


def _tam_sizes(method, P, A, d, rl):
    """send_size / recv_size per rank as handed to collective_write (mpi_test.c:343, :393)."""
    ss, rs = {}, {}
    for r in range(P):
        isagg = r in rl
        if method == 15:
            sc, sd, rc, rd = _a2m_translate(r, isagg, P, A, d, rl)
        else:
            sc, sd, rc, rd = _m2a_translate(r, isagg, P, A, d, rl)
        ss[r], rs[r] = sc, rc
    return ss, rs


def _tam_locs(method, rank, P, rl, d):
    """send_buf[w] / recv_buf[w] locations (byte offsets in SEND / RECV): a2m send_buf2[rank_list[i]] =
    segment i (:388-391), recv slot w; m2a send segment w, recv_buf2[rank_list[i]] = slot i (:335-339)."""
    if method == 15:
        sloc = {g: i * d for i, g in enumerate(rl)}
        rloc = {w: w * d for w in range(P)}
    else:
        sloc = {w: w * d for w in range(P)}
        rloc = {g: i * d for i, g in enumerate(rl)}
    return sloc, rloc


def _tam(method):
    def run(p, rank, isagg, myindex, P, A, d, c, rl, ntimes, proc_node=1, it=0):
        """all_to_many_tam :366-419 / many_to_all_tam :313-364 -> collective_write, lustre_driver_test.c:944-1309."""
        ss_all, rs_all = _tam_sizes(method, P, A, d, rl)
        sloc, rloc = _tam_locs(method, rank, P, rl, d)
        for _ in range(ntimes):
            _collective_write(p, rank, P, proc_node, ss_all, rs_all, sloc, rloc, it)
    return run


def _collective_write(p, rank, P, proc_node, ss_all, rs_all, sloc, rloc, it):
    npn, nrecvs, lr, gr, node_of = static_node_assignment(rank, P, proc_node)
    proxy = rank == lr[0]
    ssz, rsz = ss_all[rank], rs_all[rank]
    total_send, total_recv = sum(ssz), sum(rsz)
    # tags of :1006, :1012, :1094, ...: a + b + 100*iter (None = the default rank + peer, iter 0)
    tg = lambda a, b: None if it == 0 else a + b + 100 * it   # noqa: E731
    # ---- intra-node gather of the send/recv sizes (:996-1018)
    idx = []
    if proxy:
        for i in range(1, npn):
            idx.append(p.r(lr[i], 2 * P, -1, tag=tg(lr[i], lr[0]), buf="CTRL_LL", off=i * P * 8, esz=4))
    else:
        p.ctrl("CTRL_MY", list(ssz) + list(rsz))
        idx.append(p.s(lr[0], 2 * P, -1, isend=True, tag=tg(rank, lr[0]), buf="CTRL_MY", off=0, esz=4))
    if idx:
        p.t("recv", +1); p.w(idx); p.t("recv", -1)
    # proxy: exclusive prefix sums over (local process i, target w) (:1027-1041)
    if proxy:
        s_lens, r_lens, node_msg, node_recv = [], [], 0, 0
        for i in range(npn):
            for w in range(P):
                s_lens.append(node_msg); node_msg += ss_all[lr[i]][w]
                r_lens.append(node_recv); node_recv += rs_all[lr[i]][w]
        temp = max(node_msg, node_recv)
    else:
        temp = 0
    local = temp                                     # local_buf = aggregate_buf + temp (:1054-1068)
    # ---- pack this process's messages into local_buf (:1069-1077)
    off = 0
    for w in range(P):
        if ssz[w]:
            p.cp("SEND", sloc[w], "AGG", local + off, ssz[w])
            off += ssz[w]
    # ---- messages to the local proxy (:1078-1107)
    idx = []
    if proxy:
        if total_send:
            p.cp("AGG", local, "AGG", 0, total_send)
        ptr = total_send
        for i in range(1, npn):
            t = (node_msg - s_lens[i * P]) if i == npn - 1 else (s_lens[(i + 1) * P] - s_lens[i * P])
            if t:
                idx.append(p.r(lr[i], t, -1, tag=tg(lr[i], lr[0]), buf="AGG", off=ptr))
            ptr += t
    elif total_send:
        idx.append(p.s(lr[0], total_send, -1, tag=tg(rank, lr[0]), buf="AGG", off=local))
    if idx:
        p.t("recv", +1); p.w(idx); p.t("recv", -1)
    if proxy:
        # ---- inter-node exchange among proxies (:1116-1197)
        idx, ptr, gsl, grl = [], 0, [0] * nrecvs, [0] * nrecvs
        for i in range(nrecvs):
            temp2 = 0
            for v in range(P):
                if node_of[v] != i:
                    continue
                for w in range(npn):
                    t = w * P + v
                    n = (s_lens[t + 1] - s_lens[t]) if t < P * npn - 1 else (node_msg - s_lens[t])
                    if n:
                        p.cp("AGG", s_lens[t], "SBUF2", ptr + temp2, n)
                        temp2 += n
            ptr += temp2
            gsl[i] = temp2
            r_rank = gr[i]
            if r_rank != rank:
                p.ctrl("CTRL_GS%d" % i, [temp2])
                idx.append(p.r(r_rank, 1, -1, tag=tg(r_rank, rank), buf="CTRL_GR%d" % i, off=0, esz=4))
                idx.append(p.s(r_rank, 1, -1, tag=tg(r_rank, rank), buf="CTRL_GS%d" % i, off=0, esz=4))
        # what proxy i sends here: everything its node's ranks send to this node's ranks
        for i in range(nrecvs):
            if gr[i] == rank:
                grl[i] = gsl[i]
            else:
                grl[i] = sum(ss_all[w][v] for w in range(P) if node_of[w] == i for v in range(P)
                             if node_of[v] == node_of[rank])
        if idx:
            p.t("send", +1); p.w(idx); p.t("send", -1)
        idx, ptr2, rb, ptrs = [], 0, 0, []
        for i in range(nrecvs):
            r_rank = gr[i]
            if i > 0:
                rb += grl[i - 1]
            if rank != r_rank:
                if gsl[i]:
                    idx.append(p.s(r_rank, gsl[i], -1, tag=tg(r_rank, rank), buf="SBUF2", off=ptr2))
                if grl[i]:
                    idx.append(p.r(r_rank, grl[i], -1, tag=tg(r_rank, rank), buf="RBUF", off=rb))
            elif grl[i]:
                p.cp("SBUF2", ptr2, "RBUF", rb, grl[i])
            ptr2 += gsl[i]
            ptrs.append(rb)
        if idx:
            p.t("send", +1); p.w(idx); p.t("send", -1)
    # ---- local delivery (:1213-1285)
    idx = []
    if proxy:
        if total_recv:
            for w in range(P):
                if rsz[w]:
                    p.cp("RBUF", ptrs[node_of[w]], "RECV", rloc[w], rsz[w])
                ptrs[node_of[w]] += rsz[w]
        ptr = 0
        for i in range(1, npn):
            t = (node_recv - r_lens[i * P]) if i == npn - 1 else (r_lens[(i + 1) * P] - r_lens[i * P])
            if t:
                ptr2 = ptr
                for w in range(P):
                    if i == npn - 1 and w == P - 1:
                        n = node_recv - r_lens[i * P + w]
                    else:
                        n = r_lens[i * P + w + 1] - r_lens[i * P + w]
                    if n:
                        p.cp("RBUF", ptrs[node_of[w]], "AGG", ptr, n)
                    ptrs[node_of[w]] += n
                    ptr += n
                idx.append(p.s(lr[i], t, -1, tag=tg(lr[i], lr[0]), buf="AGG", off=ptr2))
    elif total_recv:
        idx.append(p.r(lr[0], total_recv, -1, tag=tg(rank, lr[0]), buf="AGG", off=local))
    if idx:
        p.t("recv", +1); p.w(idx); p.t("recv", -1)
    if not proxy and total_recv:
        off = local
        for i in range(P):
            if rsz[i]:
                p.cp("AGG", off, "RECV", rloc[i], rsz[i])
                off += rsz[i]


_METHODS = {
    1: _m1, 2: _m2, 3: _m3, 4: _m4, 5: _alltoallw(_m2a_translate), 6: _m6, 7: _m7,
    8: _alltoallw(_a2m_translate), 9: _pairwise(_a2m_translate), 10: _pairwise(_m2a_translate),
    11: _m11, 12: _m12, 13: _m13, 14: _m14, 15: _tam(15), 16: _tam(16), 17: _m17, 18: _m18, 19: _m19,
    20: _m20,
}


# --------------------------------------------------------------------------- traces
def _idx_list(idxs):
    idxs = sorted(idxs)
    out, i = [], 0
    while i < len(idxs):
        j = i
        while j + 1 < len(idxs) and idxs[j + 1] == idxs[j] + 1:
            j += 1
        out.append(str(idxs[i]) if i == j else "%d-%d" % (idxs[i], idxs[j]))
        i = j + 1
    return ",".join(out)


def _tok(kind, peer, cnt, comm, tag):
    if comm == 0:
        return "%s%d:%d" % (kind, peer, cnt) if tag is None else "%s%d:%d#%d" % (kind, peer, cnt, tag)
    return "%s%d:%d@%d#%d" % (kind, peer, cnt, comm, tag)


def trace_tokens(ops, ntimes_split=False):
    """Canonical token string, identical to the PMPI capture format (tests/golden/make_golden.py)."""
    toks = []
    for op in ops:
        k = op[0]
        if k == "B":
            toks.append("B")
        elif k == "s":
            kind = "i" if op[7] else "s"
            toks.append(_tok(kind, op[1], op[2], op[5], op[6]))
        elif k == "r":
            toks.append(_tok("r", op[1], op[2], op[4], op[5]))
        elif k == "w":
            toks.append("w" + _idx_list(op[1]))
        elif k == "A":
            toks.append("A")
    return " ".join(toks)


# --------------------------------------------------------------------------- execution
def match(progs):
    """MPI matching.  Returns the message list [(src, seg, dst, slot, bytes, s_post, r_post)]
    where s_post / r_post are the post indices at the sender / receiver.
    Point-to-point: FIFO per (communicator, src, dst, tag) (MPI non-overtaking); the
    reference's tag is src+dst on MPI_COMM_WORLD.  Alltoallw: the k-th call of every
    rank forms one collective."""
    from collections import defaultdict, deque
    sends = defaultdict(deque)
    recvs = defaultdict(deque)
    coll_s = defaultdict(dict)   # k -> {(src,dst): (cnt, seg, post)}
    coll_r = defaultdict(dict)
    for r, ops in enumerate(progs):
        post, ncoll = 0, 0
        for op in ops:
            if op[0] == "s":
                tag = r + op[1] if op[6] is None else op[6]
                sends[(op[5], r, op[1], tag)].append((op[3], op[2] * op[10], post)); post += 1
            elif op[0] == "r":
                tag = r + op[1] if op[5] is None else op[5]
                recvs[(op[4], op[1], r, tag)].append((op[3], op[2] * op[8], post)); post += 1
            elif op[0] == "A":
                for q, cnt, seg in op[1]:
                    coll_s[ncoll][(r, q)] = (cnt, seg, post); post += 1
                for q, cnt, slot in op[2]:
                    coll_r[ncoll][(q, r)] = (cnt, slot, post); post += 1
                ncoll += 1
    msgs = []
    for key in sorted(set(sends) | set(recvs)):
        s, rq = sends[key], recvs[key]
        if len(s) != len(rq):
            raise RuntimeError("unmatched point-to-point traffic on %s: %d sends, %d recvs" % (key, len(s), len(rq)))
        for (seg, scnt, sp), (slot, rcnt, rp) in zip(s, rq):
            if scnt > rcnt:
                raise RuntimeError("message truncated on %s" % (key,))
            msgs.append((key[1], seg, key[2], slot, scnt, sp, rp))
    for k in coll_s:
        if set(coll_s[k]) != set(coll_r[k]):
            raise RuntimeError("alltoallw count mismatch")
        for (src, dst), (cnt, seg, sp) in coll_s[k].items():
            rcnt, slot, rp = coll_r[k][(src, dst)]
            msgs.append((src, seg, dst, slot, cnt, sp, rp))
    return msgs


def execute(method, P, A, d, rank_list, progs, it, mode=0, record=None, eager_limit=None, buffers=None):
    """Run the matched programs with MPI semantics on bytes; returns {rank: RECV buffer}.

    Sends snapshot their bytes when posted (MPI forbids touching a send buffer before it
    completes), receives land at the completion point that waits for them, copies and
    size arrays run in program order, barriers are collective.  record (dict, optional)
    gets, per rank, every received message as (src, count, chk64 of its first `count`
    bytes) in completion order -- what oracle/pmpi_capture.c logs as D lines.  buffers (dict,
    optional) gets every rank's final {buffer name: bytes}."""
    if eager_limit is None:
        eager_limit = MPICH_EAGER_LIMIT
    lay = layout(method, P, A, rank_list)
    bufs = []
    for r in range(P):
        n_send, n_recv = lay[r]
        bufs.append({
            "SEND": np.concatenate([fingerprint(mode, r, seg_seed(method, r, q), it, d) for q in range(n_send)])
            if n_send else np.zeros(0, np.uint8),
            "RECV": np.full(n_recv * d, 0xA5, np.uint8)})

    def region(r, name, lo, n):
        b = bufs[r].get(name)
        if b is None or b.size < lo + n:
            nb = np.zeros(max(lo + n, 0), np.uint8)
            if b is not None:
                nb[:b.size] = b
            bufs[r][name] = b = nb
        return b[lo:lo + n]

    def send_loc(r, op):       # ('s', peer, cnt, seg, eager_ok, comm, tag, isend, buf, off, esz)
        n = op[2] * (op[10] if len(op) > 10 else 1)
        if len(op) > 8 and op[8] is not None:
            return op[8], op[9], n
        return "SEND", max(op[3], 0) * d, n

    def recv_loc(r, op):       # ('r', peer, cnt, slot, comm, tag, buf, off, esz)
        n = op[2] * (op[8] if len(op) > 8 else 1)
        if len(op) > 6 and op[6] is not None:
            return op[6], op[7], n
        return "RECV", max(op[3], 0) * d, n

    msgs = match(progs)
    by_post = {}
    for mi, (src, _seg, dst, _slot, _cnt, sp, rp) in enumerate(msgs):
        by_post[(src, sp)] = mi
        by_post[(dst, rp)] = mi
    post_op = {}
    for r, ops in enumerate(progs):
        q = 0
        for op in ops:
            if op[0] in ("s", "r"):
                post_op[(r, q)] = op
                q += 1
            elif op[0] == "A":
                for peer, cnt, seg in op[1]:
                    post_op[(r, q)] = ("s", peer, cnt, seg, False, 0, None, False)
                    q += 1
                for peer, cnt, slot in op[2]:
                    post_op[(r, q)] = ("r", peer, cnt, slot, 0, None)
                    q += 1
    snap, posted = {}, set()
    pc, npost, nbar = [0] * P, [0] * P, [0] * P
    arrivals = {}
    if record is not None:
        for r in range(P):
            record.setdefault(r, [])

    def post(r, q):
        op = post_op[(r, q)]
        posted.add((r, q))
        if op[0] == "s":
            name, lo, n = send_loc(r, op)
            snap[by_post[(r, q)]] = region(r, name, lo, n).copy()

    def can_complete(r, q):
        mi = by_post[(r, q)]
        src, _s, dst, _sl, cnt, sp, rp = msgs[mi]
        op = post_op[(r, q)]
        if op[0] == "r":
            return (src, sp) in posted
        if op[4] and cnt <= eager_limit:               # eager send (bytes): completes locally
            return True
        return (dst, rp) in posted

    def complete(r, qs):
        for q in qs:
            op = post_op[(r, q)]
            if op[0] != "r":
                continue
            mi = by_post[(r, q)]
            name, lo, n = recv_loc(r, op)
            data = snap[mi]
            region(r, name, lo, n)[:data.size] = data
            if record is not None and op[2] > 0:
                b = bufs[r][name]
                record[r].append((msgs[mi][0], op[2], chk64(b[lo:lo + op[2]])))

    progress = True
    while progress:
        progress = False
        for r in range(P):
            ops = progs[r]
            while pc[r] < len(ops):
                op = ops[pc[r]]
                k = op[0]
                if k == "B":
                    arr = arrivals.setdefault(nbar[r], set())
                    arr.add(r)
                    if len(arr) < P:
                        break
                    nbar[r] += 1
                elif k in ("s", "r"):
                    post(r, npost[r])
                    npost[r] += 1
                elif k == "A":
                    first = npost[r]
                    n = len(op[1]) + len(op[2])
                    if (r, first) not in posted:
                        for q in range(first, first + n):
                            post(r, q)
                    qs = list(range(first, first + n))
                    if not all(can_complete(r, q) for q in qs):
                        break
                    complete(r, qs)
                    npost[r] += n
                elif k == "w":
                    if not all(can_complete(r, q) for q in op[1]):
                        break
                    complete(r, op[1])
                elif k == "c":
                    _, seg, slot, cnt = op
                    region(r, "RECV", slot * d, cnt)[:] = region(r, "SEND", seg * d, cnt)
                elif k == "C":
                    _, sb, so, db, do, n = op
                    src = region(r, sb, so, n).copy()
                    region(r, db, do, n)[:] = src
                elif k == "K":
                    region(r, op[1], 0, op[2].size)[:] = op[2]
                pc[r] += 1
                progress = True
    if any(pc[r] < len(progs[r]) for r in range(P)):
        raise RuntimeError("deadlock while executing")
    if buffers is not None:
        buffers.update({r: bufs[r] for r in range(P)})
    return {r: bufs[r]["RECV"][:lay[r][1] * d] for r in range(P)}


MPICH_EAGER_LIMIT = 65424   # measured on the image's MPICH 3.3.2 ch3:nemesis


def asap_steps(progs, msgs=None, eager_limit=MPICH_EAGER_LIMIT, info=None):
    """Earliest-step schedule of the matched messages: a message moves in step
    1 + max(step of every message completed by an earlier completion point of
    EITHER endpoint before it was posted).  Issend is synchronous; a blocking
    MPI_Send / MPI_Sendrecv send of <= eager_limit bytes completes locally (MPI
    eager protocol), so it does not hold its sender's completion point.
    Returns (step per message, n_steps).  Raises on a cycle (the reference
    deadlocks there as well, e.g. m6 at P32 A14 d64KiB c3)."""
    if msgs is None:
        msgs = match(progs)
    P = len(progs)
    eager = set()
    for r, ops in enumerate(progs):
        post = 0
        for op in ops:
            if op[0] == "s":
                if op[4] and op[2] * op[10] <= eager_limit:   # blocking send / Isend of <= eager limit
                    eager.add((r, post))
                post += 1
            elif op[0] == "r":
                post += 1
            elif op[0] == "A":
                post += len(op[1]) + len(op[2])
    by_post = {}
    for mi, (src, _seg, dst, _slot, _cnt, sp, rp) in enumerate(msgs):
        by_post[(src, sp)] = mi
        by_post[(dst, rp)] = mi
    post_epoch = {}            # (rank, post) -> epoch of that rank when posted
    step = [None] * len(msgs)
    pc = [0] * P
    epoch = [-1] * P
    npost = [0] * P
    done = [False] * P
    nbar = [0] * P                  # barriers passed per rank
    arrivals = {}                   # barrier k -> {rank: epoch at arrival}
    barrier_epochs = []             # epoch at which barrier k completes (global)
    NEG = -(1 << 40)
    last_w = [dict() for _ in range(P)]     # rank -> buffer -> last step a copy wrote it
    last_r = [dict() for _ in range(P)]     # rank -> buffer -> last step a copy read it
    copy_steps = []
    progress = True
    while progress:
        progress = False
        for r in range(P):
            ops = progs[r]
            while pc[r] < len(ops):
                op = ops[pc[r]]
                k = op[0]
                if k == "B":        # collective: completes when every rank has arrived
                    b = nbar[r]
                    arr = arrivals.setdefault(b, {})
                    arr[r] = epoch[r]
                    if len(arr) < P:
                        break
                    e = max(arr.values())
                    if len(barrier_epochs) <= b:
                        barrier_epochs.append(e)
                    epoch[r] = max(epoch[r], e)
                    nbar[r] += 1
                elif k in ("s", "r"):
                    post_epoch[(r, npost[r])] = epoch[r]
                    npost[r] += 1
                elif k == "A":
                    n = len(op[1]) + len(op[2])
                    if (r, "A", pc[r]) not in post_epoch:      # post once, then wait
                        post_epoch[(r, "A", pc[r])] = npost[r]
                        for _ in range(n):
                            post_epoch[(r, npost[r])] = epoch[r]
                            npost[r] += 1
                    first = post_epoch[(r, "A", pc[r])]
                    # the collective completes all of its own posts
                    if not _try_wait(r, range(first, first + n), by_post, msgs, post_epoch, step, epoch):
                        break
                elif k == "w":
                    if not _try_wait(r, [q for q in op[1] if (r, q) not in eager],
                                     by_post, msgs, post_epoch, step, epoch):
                        break
                elif k in ("c", "C"):
                    # memcpy: after everything the rank completed (epoch), after the last copy
                    # that wrote its source, after the last copy that read its destination; what
                    # the rank posts next moves no earlier than the copy (DESIGN.md "copy steps")
                    sb, db = ("SEND", "RECV") if k == "c" else (op[1], op[3])
                    cs = max(epoch[r] + 1, last_w[r].get(sb, NEG) + 1, last_r[r].get(db, NEG) + 1)
                    last_w[r][db] = max(last_w[r].get(db, NEG), cs)
                    last_r[r][sb] = max(last_r[r].get(sb, NEG), cs)
                    epoch[r] = max(epoch[r], cs - 1)
                    copy_steps.append((r, cs))
                pc[r] += 1
                progress = True
            if pc[r] == len(ops):
                done[r] = True
    if not all(done):
        raise RuntimeError("deadlock: ranks %s blocked" % [r for r in range(P) if not done[r]])
    nsteps = max([s for s in step if s is not None] + [c for _, c in copy_steps] + [-1]) + 1
    if info is not None:
        info["barrier_epochs"] = barrier_epochs
        info["copy_steps"] = copy_steps
    return step, nsteps


def _try_wait(r, posts, by_post, msgs, post_epoch, step, epoch):
    mids = [by_post[(r, q)] for q in posts]
    for mi in mids:
        if step[mi] is None:
            src, _seg, dst, _slot, _cnt, sp, rp = msgs[mi]
            if (src, sp) not in post_epoch or (dst, rp) not in post_epoch:
                return False
            step[mi] = max(post_epoch[(src, sp)], post_epoch[(dst, rp)]) + 1
    if mids:
        epoch[r] = max(epoch[r], max(step[mi] for mi in mids))
    return True
