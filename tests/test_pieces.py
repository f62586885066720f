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
