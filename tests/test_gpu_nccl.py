"""GPU, world size 1 over RCCL (torch.distributed backend "nccl"): the bench's N > 1 collectives
on device tensors -- zsaac/dist.py gather_rows (the C4 embedding all-gather) and
collect_captions (the caption path's one all-gather of token ids + lengths) -- in a fresh process
whose FIRST GPU call is the process-group bring-up, as a bench rank's is.  The gathered rows must
equal the local ones (world 1), for ragged counts, greedy and beam batches, and a real bs-64
caption batch of the bench's pipeline; and C4 end to end: bench.main_embeddings (batched HTSAT
encode_audio + gather_rows) against the oracle's f32 embedding chain."""
import os
import socket

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      LOCAL_RANK="0")
    import torch
    import torch.distributed as dist
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        import bench
        from zsaac import dist as zd
        from zsaac.pipeline import CaptionBatch
        dev = torch.device("cuda", 0)
        out = {"backend": dist.get_backend()}
        # C4: [n, 1024] f32 embeddings
        emb = torch.randn(37, 1024, device=dev)
        g = zd.gather_rows(emb, [37])
        out["gather_rows"] = bool(torch.equal(g, emb))
        # greedy + beam CaptionBatch results (ragged lengths)
        ids = torch.randint(0, 50000, (5, 67), device=dev, dtype=torch.int32)
        ln = torch.tensor([1, 67, 3, 20, 9], device=dev, dtype=torch.int32)
        z = torch.zeros(5, device=dev)
        gr = CaptionBatch(ids, ln, None, z, z, z, None, z)
        bids = torch.randint(0, 50000, (3, 5, 67), device=dev, dtype=torch.int32)
        bl = torch.randint(1, 67, (3, 5), device=dev).float()
        bs = -torch.rand(3, 5, device=dev) * bl
        z3 = torch.zeros(3, device=dev)
        bm = CaptionBatch(bids, bl, bs, z3, z3, z3, None, z3)
        gi, gl = zd.collect_captions([gr], [5])
        out["collect_greedy"] = bool(torch.equal(gi, ids) and torch.equal(gl, ln))
        bi, bL = zd.collect_captions([bm], [3])
        best = (bs / bl).argmax(1)
        ar = torch.arange(3, device=dev)
        out["collect_beam"] = bool(torch.equal(bi, bids[ar, best]) and
                                   torch.equal(bL, bl[ar, best].int()))
        # a real caption batch of the bench pipeline (HTSAT + MLP + greedy, 64 clips)

        class A:
            batch, group, dtype, encoder, mapper, beam, entry_length, compact = \
                64, 1, "bf16", "htsat", "mlp", 0, 67, 1
            encoder_batch = 64
        pipe, _, _ = bench.build(A, dev)
        r = pipe.caption_wav(bench.synthetic_clips(64, 0, dev))
        ci, cl = zd.collect_captions([r], [64])
        out["collect_pipeline"] = bool(torch.equal(ci, r.ids) and torch.equal(cl, r.lengths.int()))
        # C4: bench.main_embeddings (batched HTSAT encode_audio, then the RCCL gather_rows of the
        # [N, 1024] embeddings) on 10 clips in passes of 4, against the f32 oracle chain
        # (wav -> log-mel -> HTSAT -> audio_proj) on clips 1 and 9 (= pool row 1: the bench
        # re-encodes a 2-pass window of waveforms)
        import numpy as np
        from types import SimpleNamespace
        from oracle import audio as OA, frontend as OF
        from zsaac import synthetic as S

        class E:
            batch, group, dtype, encoder, mapper, beam, entry_length, compact = \
                4, 1, "bf16", "htsat", "mlp", 0, 67, 1
            encoder_batch = 4
        epipe, _, asd = bench.build(E, dev)
        eargs = SimpleNamespace(steps=None, clips=10, warmup=1, encoder="htsat", dtype="bf16")
        res, embs = bench.main_embeddings(eargs, 1, 0, dev, epipe)
        out["c4_value"] = res["value"]
        out["c4_rows"] = int(embs.shape[0])
        wav = bench.synthetic_clips(2, 0, torch.device("cpu"))[1:2]
        with torch.no_grad():
            ref = OA.audio_project(OA.htsat_embedding(OF.logmel(wav), asd), asd)[0].numpy()
        got = embs.cpu().numpy()
        cos = [float((got[c] * ref).sum() / np.linalg.norm(got[c]) / np.linalg.norm(ref))
               for c in (1, 9)]
        out["c4_cos"] = cos
        out["c4_same_clip"] = bool(np.array_equal(got[1], got[9]))
        torch.cuda.synchronize()
        dist.barrier()
        dist.destroy_process_group()
        q.put(out)
    except Exception as e:        # reported to the parent (the test fails with the message)
        q.put({"error": repr(e)})


def test_nccl_world1_collectives(cuda):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    res = q.get(timeout=420)
    p.join(timeout=60)
    assert "error" not in res, res
    assert p.exitcode == 0
    assert res["backend"] == "nccl"
    for k in ("gather_rows", "collect_greedy", "collect_beam", "collect_pipeline"):
        assert res[k], (k, res)
    # C4 (BASELINE.json configs[3]): bench.main_embeddings' batched encode + RCCL gather_rows
    assert res["c4_rows"] == 10 and res["c4_value"] > 0
    assert res["c4_same_clip"], "the same waveform must give the same embedding in any pass"
    assert min(res["c4_cos"]) > 0.995, res["c4_cos"]      # bf16 encoder vs the f32 oracle
