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
