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


def test_choose_persist_shape_keeps_grids_coresident():
    """ConcurrentRunner's persistent grid shape choice (zsaac.pipeline.choose_persist_shape):
    simulated begins and finishes in random order, shapes (col_split, row_split) of 96 / 48 / 24
    workgroups on 256 CUs with CUs // 24 pipelines -- the workgroups in flight never exceed the
    CUs, a shard of two or three batches runs its first ones on the largest grid, and a long run
    of batches takes the smallest."""
    import random
    from zsaac import ops
    from zsaac.pipeline import choose_persist_shape, persist_shapes
    CUS = 256
    for spec in ("12,11,21", "12,11", "21", "11,21"):
        shapes = persist_shapes(spec)
        grids = [ops.decode_persist_grid(rs, cs) for cs, rs in shapes]
        assert grids == sorted(grids, reverse=True)
        P = CUS // grids[-1]
        rng = random.Random(0)
        for n in list(range(1, 24)) * 10:
            active, nxt, chosen = {}, 0, []
            while nxt < n or active:
                free = [i for i in range(P) if i not in active]
                if nxt < n and free and rng.random() < 0.7:
                    cs, rs = choose_persist_shape(sum(active.values()), n - nxt, shapes, CUS)
                    active[free[0]] = ops.decode_persist_grid(rs, cs)
                    chosen.append((cs, rs))
                    nxt += 1
                    assert sum(active.values()) <= CUS, (spec, n, chosen)
                elif active:
                    del active[rng.choice(list(active))]
        assert choose_persist_shape(0, 2, shapes, CUS) == shapes[0]
        assert choose_persist_shape(0, 17, shapes, CUS) == shapes[-1]
    sh = persist_shapes("12,11,21")
    assert sh == [(1, 2), (1, 1), (2, 1)]
    assert choose_persist_shape(96, 2, sh, CUS) == (1, 2)
    assert choose_persist_shape(0, 5, sh, CUS) == (1, 2)
    assert choose_persist_shape(0, 8, sh, CUS) == (1, 1)
