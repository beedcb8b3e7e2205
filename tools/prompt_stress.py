#!/usr/bin/env python3
"""Is prompt_assemble (sound-effect choice + hard-prompt template, gpt2.hip prompt_kernel)
deterministic when it runs beside decode grids on other streams?  The c2_gpt2init-derived 1045
embeddings (tools/conc_stress.py), their hard prompts computed alone, then `reps` rounds of: ten
pipelines decoding (persistent grids, their own streams) while the prompts of all 17 batches are
recomputed on ten other streams; prints every (round, batch, row) whose prompt differs, and the
similarity gap between the chosen and the reference label there.

    python tools/prompt_stress.py [reps=40] [mode=decode|lmhead|grid|gemm|none]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))
import torch  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    # what runs beside the prompts: "decode" (step 0's LM head + the persistent grid), "lmhead"
    # (step 0's device work only: LM head / greedy init + step), "grid" (the persistent grid only,
    # from a saved post-step-0 state), "gemm" (lean GEMM launches), "none"
    mode = sys.argv[2] if len(sys.argv) > 2 else "decode"
    from tools import idparity
    from zsaac import ops, synthetic as S
    from zsaac.pipeline import CaptionConfig, CaptionPipeline
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
    k = cfg.sound_effect_num
    nb = len(batches)

    def prompts(bufs):
        for j, b in enumerate(batches):
            hid, hl, ch = bufs[j]
            ops.prompt_assemble(b, p.labels, k, p.label_tok, p.label_len, hid[:b.shape[0]],
                                hl[:b.shape[0]], ch[:b.shape[0]])

    def mk():
        return [(torch.zeros(64, p.h_cap, device=dev, dtype=torch.int32),
                 torch.zeros(64, device=dev, dtype=torch.int32),
                 torch.zeros(64, max(k, 1), device=dev, dtype=torch.int32)) for _ in batches]
    ref = mk()
    prompts(ref)
    torch.cuda.synchronize()
    sim = (emb.double() @ p.labels.double().t()).float()           # for the report (f64)
    pipes = [p] + [p.twin() for _ in range(9)]
    dstreams = ops.dedicated_streams(10, dev, priority=-1)
    pstreams = ops.dedicated_streams(10, dev, priority=-1)
    for q, s in zip(pipes, dstreams):
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            q.caption_emb(batches[0])
        q.decoder.persist_grid = 48
    torch.cuda.synchronize()
    saved = []
    for q, s in zip(pipes, dstreams):
        with torch.cuda.stream(s):
            q.decoder.greedy_begin_device(64)
        saved.append([t.clone() for t in q.decoder._state()])
    torch.cuda.synchronize()
    ga = torch.randn(4096, 768, device=dev, dtype=torch.bfloat16)
    gw = torch.randn(3072, 768, device=dev, dtype=torch.bfloat16)
    go = [torch.empty(4096, 3072, device=dev, dtype=torch.bfloat16) for _ in dstreams]
    go2 = [torch.empty(1728, 2304, device=dev, dtype=torch.bfloat16) for _ in dstreams]

    def beside(qi, q, s):
        with torch.cuda.stream(s):
            if mode == "decode":
                q.decoder.greedy_begin(64)
            elif mode == "lmhead":
                for _ in range(20):
                    q.decoder.greedy_begin_device(64)
            elif mode == "grid":
                for t, v in zip(q.decoder._state(), saved[qi]):
                    t.copy_(v)
                q.decoder._persist_pending = 64
                q.decoder.launch_pending()
            elif mode == "gemm":
                for _ in range(10):
                    ops.gemm(ga, gw, go[qi])                              # 128x128 2-stage
                    ops.gemm(ga[:1728], gw[:2304], go2[qi])                # 8-wave 3-stage
    got = [mk() for _ in range(len(pstreams))]
    bad = []
    for r in range(reps):
        for qi, (q, s) in enumerate(zip(pipes, dstreams)):
            beside(qi, q, s)
        for j, s in enumerate(pstreams):
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                prompts(got[j])
        torch.cuda.synchronize()
        for j in range(len(pstreams)):
            for bi in range(nb):
                h0, h1 = ref[bi][2], got[j][bi][2]
                rows = (h0 != h1).any(dim=1).nonzero().flatten().tolist()
                for row in rows:
                    c = bi * 64 + row
                    a, b = int(h0[row, 0]), int(h1[row, 0])
                    bad.append({"round": r, "stream": j, "batch": bi, "row": row,
                                "ref_labels": h0[row].tolist(), "got_labels": h1[row].tolist(),
                                "sims_ref": [round(float(sim[c, x]), 8) for x in h0[row].tolist()],
                                "sims_got": [round(float(sim[c, x]), 8) for x in h1[row].tolist()]})
    print(json.dumps({"reps": reps, "mode": mode, "lib": os.environ.get("ZSAAC_LIB", ""), "differences": len(bad),
                      "first": bad[:10]}), flush=True)


if __name__ == "__main__":
    main()
