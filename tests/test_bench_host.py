"""Host-side pieces of bench.py (no GPU): eval-batch splitting and the persistent decode
roofline's algorithmic byte count."""
import bench


def test_split_batches_reference_and_balanced():
    assert bench.split_batches(1045, 64)[-1] == (1024, 1045)
    assert len(bench.split_batches(1045, 64)) == 17
    assert bench.split_batches(131, 64) == [(0, 64), (64, 128), (128, 131)]
    bal = bench.split_batches(131, 64, parts=5)
    assert [b - a for a, b in bal] == [27, 26, 26, 26, 26]
    assert bal[0][0] == 0 and bal[-1][1] == 131
    # more parts than batches of 64 never exceeds B rows; fewer parts than needed keeps <= B
    assert all(b - a <= 64 for a, b in bench.split_batches(1045, 64, parts=5))
    assert bench.split_batches(3, 64, parts=5) == [(0, 1), (1, 2), (2, 3)]


def test_persist_launch_bytes():
    row = 12 * 2 * 768 * 2
    # 2 rows, prompt 10 and 12, 3 steps (steps 1, 2 in the launch): step t at position
    # plen - 1 + t reads that many cached keys: 10 + 11 and 12 + 13
    got = bench.persist_launch_bytes(1000, [10, 12], 3)
    assert got == 2 * 1000 + row * ((10 + 11) + (12 + 13) + 2 * 2)
    assert bench.persist_launch_bytes(1000, [10], 1) == 0


def test_choose_row_split_keeps_grids_coresident():
    """ConcurrentRunner's row_split choice (zsaac.pipeline.choose_row_split): simulated begins and
    finishes in random order, 5 pipelines, G = 48 on 256 CUs -- the workgroups in flight never
    exceed the CUs, and a shard of two or three batches runs its first ones at row_split 2."""
    import random
    from zsaac.pipeline import choose_row_split
    G, CUS, P = 48, 256, 5
    rng = random.Random(0)
    for n in list(range(1, 24)) * 20:
        active, nxt, chosen = {}, 0, []
        while nxt < n or active:
            free = [i for i in range(P) if i not in active]
            if nxt < n and free and rng.random() < 0.7:
                rs = choose_row_split(sum(active.values()), n - nxt, G, CUS)
                active[free[0]] = rs * G
                chosen.append(rs)
                nxt += 1
                assert sum(active.values()) <= CUS, (n, chosen)
            elif active:
                del active[rng.choice(list(active))]
    assert choose_row_split(0, 2, G, CUS) == 2 and choose_row_split(0, 3, G, CUS) == 2
    assert choose_row_split(96, 2, G, CUS) == 2 and choose_row_split(0, 5, G, CUS) == 1
