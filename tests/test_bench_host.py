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
