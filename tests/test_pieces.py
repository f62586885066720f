"""xg_piece_size (csrc/host/pieces.c): the workgroup piece size of a copy launch -- the one
whose busiest CU has the least work, ties to the larger piece."""


def test_known_launch_classes(xg):
    K = 1024
    assert xg.piece_size([256 * K] * 112) == 16 * K          # 28 MiB pack: 896 x 32K (3.5 / CU) -> 1792 x 16K (7 / CU)
    assert xg.piece_size([256 * K] * 16) == 16 * K           # 4 MiB gather: 128 x 32K (half the CUs idle) -> 256 x 16K
    assert xg.piece_size([1 << 20] * 448) == 32 * K          # the bench's 448 MiB launches: 56 per CU, unchanged
    assert xg.piece_size([32 * K] * 448) == 32 * K           # 14 MiB of 32 KiB segments: a tie stays 32 KiB
    assert xg.piece_size([1 << 20] * 448, chunk=32 * K, cus=256, wg_cost=0) == 32 * K


def test_rule_against_brute_force(xg):
    import random
    rng = random.Random(5)
    for _ in range(300):
        n = rng.randint(1, 3000)
        lens = [rng.choice([0, 16, 1000, 2048, 4096, 8192, 65536, 256 << 10, 1 << 20, 48 << 10]) for _ in range(n)]
        cus, cost, chunk = rng.choice([64, 256]), rng.choice([0, 2048, 8192]), 32768
        best, bc, c = None, chunk, chunk
        while c >= 4096:
            w = sum((x + c - 1) // c for x in lens if x > 0)
            if w == 0:
                break
            v = ((w + cus - 1) // cus) * (c + cost)
            if best is None or v < best:
                best, bc = v, c
            c //= 2
        assert xg.piece_size(lens, chunk, cus, cost) == bc


def _plan(xg, steps):
    """a hand-made xg_devplan: steps = [(stage, local, packs, unpacks)], each a list of
    (src_buf, src_off, dst_buf, dst_off, len)"""
    import ctypes as C
    copies, sp, posts = [], [], []
    for stage, local, packs, _unp in steps:
        b = len(copies)
        copies += stage + local + packs
        sp.append([b, len(stage) + len(local) + len(packs), 0, 0, 0, 0, 0, len(stage)])
    for i, (_s, _l, _p, unp) in enumerate(steps):
        sp[i][4], sp[i][5] = len(copies), len(unp)
        copies += unp
    arr = (xg.Copy * max(1, len(copies)))(*[xg.Copy(so, do, n, sb, db) for sb, so, db, do, n in copies])
    st = (xg.StepPlan * len(sp))(*[xg.StepPlan(*x) for x in sp])
    dp = xg.DevPlan()
    dp.gpu, dp.ngpus, dp.nsteps = 0, 2, len(sp)
    dp.ncopy, dp.np2p = len(copies), 0
    dp.copies = C.cast(arr, C.POINTER(xg.Copy))
    dp.steps = C.cast(st, C.POINTER(xg.StepPlan))
    dp._keep = (arr, st)
    return dp


def test_local_meets_unpacks(xg):
    import ctypes as C
    S, R, SS, SR = xg.BUF_SEND, xg.BUF_RECV, xg.BUF_STAGE_SEND, xg.BUF_STAGE_RECV
    unp = [(SR, 0, R, 1000, 100), (SR, 100, R, 5000, 50)]           # step 0 writes RECV [1000,1100), [5000,5050)
    cases = [
        ([(S, 0, R, 2000, 64)], 0),              # disjoint
        ([(S, 0, R, 1099, 1)], 1),               # writes the last byte an unpack writes
        ([(S, 0, R, 900, 100)], 0),              # ends exactly where the unpack starts
        ([(R, 5049, S, 0, 8)], 1),               # reads a byte an unpack writes
        ([(S, 0, R, 4000, 1001)], 1),            # covers a whole unpack
        ([(S, 0, R, 0, 16), (S, 16, R, 1050, 4)], 1),
    ]
    for local, want in cases:
        dp = _plan(xg, [([], [], [(S, 0, SS, 0, 150)], unp), ([], local, [(S, 0, SS, 0, 8)], [])])
        assert xg.host().xg_step_local_meets_unpacks(C.byref(dp), 1) == want, (local, want)
    dp = _plan(xg, [([], [], [], unp)])
    assert xg.host().xg_step_local_meets_unpacks(C.byref(dp), 0) == -1


def test_real_plans_never_meet_their_unpacks(xg):
    """every golden-shape plan on 2 and 8 GPUs, packed: no local copy touches the previous
    step's unpacked bytes (so the fused launch may take a small local part)"""
    from conftest import golden_configs, load_golden
    for cfg in golden_configs():
        meta, _, _ = load_golden(cfg)
        for m in meta["method_list"]:
            s = xg.Schedule(m, meta["P"], meta["A"], meta["d"], meta["c"], meta["aggregators"], ntimes=meta["ntimes"],
                            proc_node=meta["proc_node"], barrier_type=meta["barrier"])
            for G in (2, 8):
                if G > meta["P"]:
                    continue
                for g in range(G):
                    v = s.devplan(G, g, 1 << 30)
                    for st in range(1, v.nsteps):
                        assert v.local_meets_unpacks(st) == 0, (cfg, m, G, g, st)


def test_stage_meets_rest(xg):
    """xg_step_stage_meets_rest: a stage copy's written bytes read or written by another pre copy
    of the step, or its read bytes written by one, keep the stage copies in a launch of their own"""
    import ctypes as C
    S, R, SC, SS = xg.BUF_SEND, xg.BUF_RECV, xg.BUF_SCRATCH, xg.BUF_STAGE_SEND
    stage = [(S, 0, SC, 1000, 100), (SC, 4000, SC, 6000, 50)]     # writes SCRATCH [1000,1100), [6000,6050); reads S [0,100), SC [4000,4050)
    cases = [
        ([(S, 200, R, 0, 64)], [], 0),                # disjoint
        ([(SC, 1099, R, 0, 1)], [], 1),               # reads the last byte a stage copy writes
        ([(SC, 900, R, 0, 100)], [], 0),              # ends where a stage write starts
        ([(S, 200, SC, 6049, 1)], [], 1),             # writes a byte a stage copy writes
        ([(S, 200, SC, 4010, 8)], [], 1),             # writes a byte a stage copy reads
        ([(S, 0, R, 0, 100)], [], 0),                 # reads what a stage copy reads: fine
        ([], [(SC, 1050, SS, 0, 10)], 1),             # a pack reads a stage copy's output
        ([(S, 200, R, 0, 8)], [(S, 300, SS, 0, 8)], 0),
    ]
    for local, packs, want in cases:
        dp = _plan(xg, [(stage, local, packs, [])])
        assert xg.host().xg_step_stage_meets_rest(C.byref(dp), 0) == want, (local, packs, want)
    dp = _plan(xg, [([], [(S, 0, R, 0, 8)], [], [])])
    assert xg.host().xg_step_stage_meets_rest(C.byref(dp), 0) == 0           # no stage copies
    assert xg.host().xg_step_stage_meets_rest(C.byref(dp), 1) == -1


def _brute_stage_meets_rest(v, st):
    pb, pc, _qb, _qc, _ob, _oc = v.steps[st]
    sc = v.stage_count[st]
    stage, rest = v.copies[pb:pb + sc], v.copies[pb + sc:pb + pc]
    def ov(b1, o1, n1, b2, o2, n2):
        return n1 > 0 and n2 > 0 and b1 == b2 and o1 < o2 + n2 and o2 < o1 + n1
    for sb, so, db, do, n in stage:
        for rsb, rso, rdb, rdo, rn in rest:
            if ov(rsb, rso, rn, db, do, n) or ov(rdb, rdo, rn, db, do, n) or ov(rdb, rdo, rn, sb, so, n):
                return 1
    return 0


def test_stage_meets_rest_on_real_plans(xg):
    """every golden-shape TAM plan (m15 / m16) on 1, 2 and 8 GPUs: the C test equals a brute-force
    overlap check step by step, and the README configuration's step 3 may share one launch"""
    from conftest import golden_configs, load_golden
    fusable = 0
    for cfg in golden_configs():
        meta, _, _ = load_golden(cfg)
        for m in (15, 16):
            if m not in meta["method_list"]:
                continue
            s = xg.Schedule(m, meta["P"], meta["A"], meta["d"], meta["c"], meta["aggregators"], ntimes=meta["ntimes"],
                            proc_node=meta["proc_node"], barrier_type=meta["barrier"])
            for G in (1, 2, 8):
                if G > meta["P"]:
                    continue
                for g in range(G):
                    v = s.devplan(G, g, 1 << 30)
                    for st in range(v.nsteps):
                        if not v.stage_count[st]:
                            continue
                        got = v.stage_meets_rest(st)
                        assert got == _brute_stage_meets_rest(v, st), (cfg, m, G, g, st)
                        fusable += got == 0 and v.steps[st][1] > v.stage_count[st]
    assert fusable > 0
    rl = xg.aggregator_list(32, 14)
    for m in (15, 16):
        v = xg.Schedule(m, 32, 14, 2048, 3, rl, ntimes=1).devplan(1, 0)
        assert v.stage_count[3] and v.steps[3][1] > v.stage_count[3] and v.stage_meets_rest(3) == 0
