#!/usr/bin/env python3
"""Are the headline schedule's ids those of a single-stream run?  1045 embeddings (the
c2_gpt2init golden's, perturbed per clip as tests/test_gpu_persist.py does) in 17 batches of
<= 64 on the golden's weights, decoded several ways; per variant the batches whose ids differ from
the first single-stream run, and for each such batch the first differing (row, step).

    python tools/conc_check.py            (ZSAAC_LIB selects another in-tree build)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))
import torch  # noqa: E402


def main():
    from tools import idparity
    from zsaac import synthetic as S
    from zsaac.pipeline import CaptionConfig, CaptionPipeline, ConcurrentRunner
    dev = torch.device("cuda", 0)
    g = idparity.load("c2_gpt2init")
    csd = S.gpt2_state_dict(**idparity.golden_gpt2_kw(g))
    csd.update(S.mlp_mapper_state_dict(1))
    cfg = CaptionConfig(dtype=torch.bfloat16, batch=64, entry_length=int(g["entry_length"]),
                        persist_decode=True)
    p = CaptionPipeline(csd, None, S.label_table(), S.label_token_table(), cfg, device=dev)
    base = torch.from_numpy(g["clap_emb"]).to(dev)
    n = 1045
    i = torch.arange(n, device=dev, dtype=torch.float32)[:, None]
    emb = base[torch.arange(n, device=dev) % base.shape[0]] * (1.0 + 0.05 * torch.sin(0.37 * i))
    batches = [emb[a:a + 64] for a in range(0, n, 64)]

    def seq(order, grid=48):
        p.decoder.persist_grid = grid
        out = [None] * len(batches)
        for k in order:
            out[k] = p.caption_emb(batches[k]).captions()
        return out

    ref = seq(range(len(batches)))

    def report(name, caps, extra=None):
        bad = []
        for k, c in enumerate(caps):
            if c != ref[k]:
                first = None
                for r, (x, y) in enumerate(zip(c, ref[k])):
                    if x != y:
                        s = next((t for t, (a, b) in enumerate(zip(x, y)) if a != b), min(len(x), len(y)))
                        first = (r, s)
                        break
                bad.append({"batch": k, "first_row_step": first})
        r = {"variant": name, "batches_differing": bad}
        if extra:
            r.update(extra)
        print(json.dumps(r), flush=True)

    report("single_again", seq(range(len(batches))))
    report("single_reverse", seq(reversed(range(len(batches)))))
    report("single_g96", seq(range(len(batches)), 96))
    p.decoder.persist = False
    report("single_phases", seq(range(len(batches))))
    p.decoder.persist = True
    runner = ConcurrentRunner(p, 10)
    runner.warmup_emb(batches[0])
    for rep in range(3):
        outs = runner.run(batches, inputs="emb")
        report(f"concurrent_{rep}", [o.captions() for o in outs],
               {"grids": runner.grid, "gave_up": runner.gave_up,
                "assign": runner.assign})
    runner1 = ConcurrentRunner(p, 1)
    outs = runner1.run(batches, inputs="emb")
    report("runner_1_inflight", [o.captions() for o in outs])


if __name__ == "__main__":
    main()
