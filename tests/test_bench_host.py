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


def test_choose_persist_grid_keeps_grids_coresident():
    """ConcurrentRunner's persistent grid choice (zsaac.pipeline.choose_persist_grid), pure host
    logic: simulated begins and finishes in random order, grids of 192 / 96 / 48 half-CU
    workgroups within a budget of workgroup slots, budget // 48 pipelines -- the workgroups in
    flight never exceed the budget, a shard of two or three batches runs its first ones on the
    largest grid, and a long run of batches takes the smallest."""
    import random
    from zsaac.pipeline import choose_persist_grid, persist_grids
    for budget in (256, 384, 512):
        for spec in ("192,96,48", "96,48", "48", "192,48"):
            grids = persist_grids(spec)
            assert grids == sorted(grids, reverse=True)
            P = budget // grids[-1]
            rng = random.Random(0)
            for n in list(range(1, 24)) * 10:
                active, nxt, chosen = {}, 0, []
                while nxt < n or active:
                    free = [i for i in range(P) if i not in active]
                    if nxt < n and free and rng.random() < 0.7:
                        g = choose_persist_grid(sum(active.values()), n - nxt, grids, budget)
                        active[free[0]] = g
                        chosen.append(g)
                        nxt += 1
                        assert sum(active.values()) <= budget, (spec, n, chosen)
                    elif active:
                        del active[rng.choice(list(active))]
            assert choose_persist_grid(0, 17, grids, budget) == grids[-1]
    g = persist_grids("192,96,48")
    assert g == [192, 96, 48]
    assert choose_persist_grid(0, 2, g, 256) == 192         # 192 + one 48 beside it
    assert choose_persist_grid(0, 3, g, 256) == 96          # 96 + two 48s
    assert choose_persist_grid(96, 2, g, 256) == 96
    assert choose_persist_grid(0, 6, g, 512) == 192
    assert choose_persist_grid(0, 5, g, 256) == 48


def test_persist_grids_env(monkeypatch):
    """An explicit spec is never overridden by the environment (ZSAAC_PERSIST_GRID applies only
    when no spec is given)."""
    from zsaac.pipeline import persist_grids
    monkeypatch.setenv("ZSAAC_PERSIST_GRID", "96")
    assert persist_grids("192,48") == [192, 48]
    assert persist_grids() == [96]
    monkeypatch.delenv("ZSAAC_PERSIST_GRID")
    monkeypatch.setenv("ZSAAC_PERSIST_GRIDS", "48,96")
    assert persist_grids() == [96, 48]
