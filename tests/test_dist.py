"""CPU, world_size 2 with gloo: clip sharding + the token-id all-gather reassemble the batch in
clip order (the N>1 path of bench.py / predict driver)."""
import os
import socket

import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, T, q):
    import torch.distributed as dist
    from zsaac.dist import gather_token_ids, shard_range
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_range(n, rank, world)
    # "decode" of the local shard: clip c emits ids c*100 + t for t < (c % 5) + 1
    ids = torch.zeros(hi - lo, T, dtype=torch.int32)
    lens = torch.zeros(hi - lo, dtype=torch.int32)
    for i, c in enumerate(range(lo, hi)):
        L = c % 5 + 1
        ids[i, :L] = torch.arange(L, dtype=torch.int32) + c * 100
        lens[i] = L
    counts = [shard_range(n, r, world)[1] - shard_range(n, r, world)[0] for r in range(world)]
    all_ids, all_len = gather_token_ids(ids, lens, counts)
    if rank == 0:
        q.put((all_ids.tolist(), all_len.tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_gather_token_ids_gloo_world2():
    n, T, world = 7, 6, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, n, T, q)) for r in range(world)]
    for p in ps:
        p.start()
    ids, lens = q.get(timeout=120)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    for c in range(n):
        L = c % 5 + 1
        assert lens[c] == L
        assert ids[c][:L] == [c * 100 + t for t in range(L)]


def _bench_worker(rank, world, port, n, B, q):
    """The bench's N>1 path: shard_range over a fixed clip set, per-batch CaptionBatch-like
    results (greedy and beam), zsaac.dist.collect_captions; and the C4 embedding gather."""
    import torch.distributed as dist
    from types import SimpleNamespace
    from zsaac import dist as zd
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = zd.shard_range(n, rank, world)
    counts = zd.shard_counts(n, world)
    T = 9
    greedy, beam = [], []
    for b0 in range(lo, hi, B):                  # the rank's eval batches, last one ragged
        clips = list(range(b0, min(hi, b0 + B)))
        ids = torch.zeros(len(clips), T, dtype=torch.int32)
        ln = torch.zeros(len(clips), dtype=torch.int32)
        bids = torch.zeros(len(clips), 3, T, dtype=torch.int32)
        bl = torch.ones(len(clips), 3)
        sc = torch.zeros(len(clips), 3)
        for i, c in enumerate(clips):
            L = c % 7 + 1
            ids[i, :L] = torch.arange(L, dtype=torch.int32) + 1000 * c
            ln[i] = L
            best = c % 3                           # beam `best` has the best score / length
            for k in range(3):
                bids[i, k, :L] = torch.arange(L, dtype=torch.int32) + 1000 * c + 100 * k
                bl[i, k] = L
                sc[i, k] = -10.0 + (5.0 if k == best else 0.0)
        greedy.append(SimpleNamespace(ids=ids, lengths=ln, scores=None))
        beam.append(SimpleNamespace(ids=bids, lengths=bl, scores=sc))
    gi, gl = zd.collect_captions(greedy, counts)
    bi, bl = zd.collect_captions(beam, counts)
    emb = torch.arange(lo, hi, dtype=torch.float32).view(-1, 1).repeat(1, 4)
    ge = zd.gather_rows(emb, counts)
    if rank == 0:
        q.put((gi.tolist(), gl.tolist(), bi.tolist(), bl.tolist(), ge.tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_bench_gather_path_gloo_world2():
    n, B, world = 45, 8, 2                        # 23 + 22 clips: ragged last batches
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_bench_worker, args=(r, world, port, n, B, q)) for r in range(world)]
    for p in ps:
        p.start()
    gi, gl, bi, bl, ge = q.get(timeout=120)
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert len(gi) == n and len(bi) == n and len(ge) == n
    for c in range(n):
        L = c % 7 + 1
        assert gl[c] == L and gi[c][:L] == [1000 * c + t for t in range(L)]
        assert bl[c] == L and bi[c][:L] == [1000 * c + 100 * (c % 3) + t for t in range(L)]
        assert ge[c] == [float(c)] * 4


class _CpuRunner:
    """A CPU stand-in for zsaac.pipeline.ConcurrentRunner: one 'caption' per clip derived from its
    waveform (so the test can recompute it from bench.synthetic_clips), after a rank-dependent
    sleep (so the job time must be the slower rank's)."""
    delay = 0.0

    def __init__(self, pipe, n_inflight=2, streams=None, grids=None, budget=None, **kw):
        self.pipes, self.n_inflight, self.gave_up = [pipe], n_inflight, 0
        self.grid, self.decode_steps = [], []

    def warmup(self, wav):
        pass

    def decoders(self):
        return [p.decoder for p in self.pipes]

    def run(self, batches, keep=None, inputs="wav"):
        import time
        from types import SimpleNamespace
        time.sleep(self.delay)
        self.grid = [0] * len(batches)
        self.decode_steps = [1] * len(batches)
        return [SimpleNamespace(ids=_fake_ids(b), lengths=_fake_len(b), scores=None)
                for b in batches]


def _fake_ids(wav):
    return (wav[:, :6] * 1e4).round().to(torch.int32)


def _fake_len(wav):
    return (wav[:, 0].abs() * 1e4).round().to(torch.int32) % 6 + 1


def _run_captions_worker(rank, world, port, n, B, reps, q):
    """bench.run_captions' world > 1 branch on CPU (gloo): collect_captions inside the timed
    region, the barrier, the all_reduce(MAX) of each repetition's time, the median."""
    import sys
    import torch.distributed as dist
    from types import SimpleNamespace
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    import zsaac.pipeline as zp
    from zsaac import dist as zd
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.synchronize = lambda *a, **k: None       # no GPU here: nothing to wait for
    bench.run_streams = lambda device, k: [None] * k
    zp.ConcurrentRunner = _CpuRunner
    _CpuRunner.delay = 0.05 * rank                      # rank 1 is the slow one
    lo, hi = zd.shard_range(n, rank, world)
    counts = zd.shard_counts(n, world)
    pipe = SimpleNamespace(cfg=SimpleNamespace(batch=B, beam=0),
                           decoder=SimpleNamespace(n_captures=0, rows_stepped=0, persist=False))
    args = SimpleNamespace(persist_budget=0)
    dt, outs, runner, info = bench.run_captions(args, world, rank, torch.device("cpu"), pipe,
                                                hi - lo, lo, counts, 2, 1, reps=reps)
    ids, lens = zd.collect_captions(outs, counts)
    q.put((rank, dt, info["timed_reps_s"], info["persist_gave_up"],
           ids.tolist() if rank == 0 else None, lens.tolist() if rank == 0 else None))
    dist.barrier()
    dist.destroy_process_group()


def test_run_captions_world2_gloo():
    """bench.run_captions at world 2 (its world > 1 branch, bench.py): both ranks report the
    slower rank's time for every repetition (all_reduce MAX), the median of `reps`, and the
    gathered captions are every clip's in clip order (ragged shards: 13 + 12 clips, batches of 4)."""
    n, B, world, reps = 25, 4, 2, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_run_captions_worker, args=(r, world, port, n, B, reps, q))
          for r in range(world)]
    for p in ps:
        p.start()
    got = dict((r[0], r[1:]) for r in (q.get(timeout=180) for _ in range(world)))
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    (dt0, reps0, gu0, ids, lens), (dt1, reps1, gu1, _, _) = got[0], got[1]
    assert len(reps0) == reps and reps0 == reps1          # the same (max-over-ranks) times
    assert dt0 == dt1 and min(reps0) >= 0.05               # rank 1's 50 ms sleep bounds them
    assert abs(dt0 - sorted(reps0)[reps // 2]) < 1e-4       # the median (times rounded to 10 us)
    assert gu0 == gu1 == 0
    wav = bench.synthetic_clips(n, 0, torch.device("cpu"))
    assert lens == _fake_len(wav).tolist()
    assert all(ids[c][:lens[c]] == _fake_ids(wav)[c, :lens[c]].tolist() for c in range(n))
