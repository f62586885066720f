"""Per-GPU HBM footprint of the 8-GPU BASELINE configurations (CPU, from the device plans).

configs[4] (P256 A64 -d 64 MiB, -c 1..8, m7/m11/m12) is the largest: on 8 GPUs each
GPU holds 32 ranks' send segments (128 GiB) and 8 aggregators' receive slots
(128 GiB); the per-peer staging buffers -- the relay form's forwarding staging (<= 1.5 GiB
at m11 -c 8), the coalesced relay form's packed pieces and forwarded blocks (<= 5.5 GiB, m11 -c 8) --
must not push that past one MI355X's 288 GB.
"""
import pytest

HBM = 288 * 10 ** 9           # MI355X HBM3E, spec (decimal GB: the conservative reading)


@pytest.mark.parametrize("case", [
    (256, 64, 64 << 20, (7, 11, 12), range(1, 9)),        # configs[4]
    (256, 32, 4 << 20, (1, 2, 9, 10), (200000000,)),      # configs[3]
    (64, 16, 256 << 10, (5, 8), (200000000,)),            # configs[2]
], ids=["configs4", "configs3", "configs2"])
def test_per_gpu_regions_fit_288gb(xg, case):
    P, A, d, methods, cs = case
    rl = xg.aggregator_list(P, A)
    for m in methods:
        for c in cs:
            s = xg.Schedule(m, P, A, d, c, rl, ntimes=1)
            # direct, packed, relay, coalesced (the coalesced form at the sweep's ends: suite time)
            for pack, form in ((0, -1), (4 << 20, -1), (0, 2)) + (((0, 3),) if c in (1, 8, 200000000) else ()):
                tot = 0
                for g in range(8):
                    v = s.devplan(8, g, pack, 0, form)
                    need = sum(v.region_bytes)
                    # plan tables: <= 24 B per 32 KiB piece, 32 B per RCCL op
                    need += 24 * (sum(x[4] for x in v.copies) // 32768 + len(v.copies)) + 32 * len(v.p2p)
                    assert need < HBM, (m, c, pack, form, g, need)
                    if form == 3:
                        assert v.region_bytes[2] + v.region_bytes[3] <= 5632 << 20, (m, c, g, v.region_bytes)
                    tot += v.region_bytes[0] + v.region_bytes[1]
                assert tot == 2 * P * A * d          # every segment and slot lives on exactly one GPU
