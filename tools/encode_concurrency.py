#!/usr/bin/env python3
"""k bs-64 HTSAT encodes (+ mapper + prefill) on k dedicated streams at once vs one alone: does
the begin phase of ConcurrentRunner scale with CU-seconds, or do concurrent begins slow each
other beyond that?

    python tools/encode_concurrency.py [reps=5]
"""
import os
import sys
import time
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))

import torch  # noqa: E402

import bench  # noqa: E402
from zsaac import ops  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    dev = torch.device("cuda", 0)
    args = SimpleNamespace(dtype="bf16", group=1, encoder="htsat", mapper="mlp", batch=64,
                           encoder_batch=0, beam=0, entry_length=67, compact=1)
    pipe, _, _ = bench.build(args, dev)
    pipes = [pipe] + [pipe.twin() for _ in range(4)]
    streams = ops.dedicated_streams(5, dev)
    wav = bench.synthetic_clips(64, 0, dev)

    def enc(p):
        p.encode(wav)

    def begin(p):
        emb = p.encode(wav)
        # prompt + mapper + prefill, no decode launch (begin_emb up to step 0 of greedy)
        from zsaac import ops as o
        B, Pmax = 64, p.Pmax
        o.prompt_assemble(emb, p.labels, p.cfg.sound_effect_num, p.label_tok, p.label_len,
                          p.hard_ids[:B], p.hard_len[:B])
        o.l2norm(emb, out=p.prefix[:B])
        soft = p.mapper(p.prefix[:B])
        d = p.decoder
        o.prefill_embed(p.hard_ids[:B], p.hard_len[:B], soft, p.mapper.soft_ld, p.cfg.prefix_length,
                        p.gpt.wte, p.gpt.wpe, B, Pmax, p.embed[:B * Pmax], d.x, d.plen, d.last_row)
        d.prefill(B, Pmax)

    for name, fn in (("encode", enc), ("begin", begin)):
        for k in (1, 2, 3, 5):
            ts = []
            for r in range(reps + 1):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for p, s in zip(pipes[:k], streams[:k]):
                    s.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(s):
                        fn(p)
                for s in streams[:k]:
                    torch.cuda.current_stream().wait_stream(s)
                torch.cuda.synchronize()
                if r:
                    ts.append((time.perf_counter() - t0) * 1e3)
            ts.sort()
            print(f"{name:6s} x{k}: {ts[len(ts) // 2]:7.2f} ms ({ts[len(ts) // 2] / k:6.2f} ms per batch)",
                  flush=True)


if __name__ == "__main__":
    main()
