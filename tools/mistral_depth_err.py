#!/usr/bin/env python3
"""Diagnostic: first-step logit error of the fp8 and bf16 Mistral engines against the f32 engine
on shared-value random weights, by depth (is a 7B-geometry deviation numerical growth through the
layers, or a path error?).  python tools/mistral_depth_err.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))
import torch  # noqa: E402


RESID = os.environ.get("RESID", "0") == "1"


def main():
    from zsaac import synthetic as S
    from zsaac.mistral import MistralDecoder, MistralWeights
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(5)
    B, D = 8, 4096
    hard = torch.randint(3, 32000, (B, 9), device=dev, generator=g).to(torch.int32)
    soft = torch.randn(B, 10, D, device=dev, generator=g) * 0.5
    for L in (1, 2, 4, 8, 16, 32):
        cfg = dict(S.MISTRAL_7B, layers=L)
        ws = {m: MistralWeights.synthetic(dev, cfg, seed=11, mode=m, shared_values=True,
                                          resid_init=RESID) for m in ("f32", "bf16", "fp8")}
        emb = torch.cat([ws["f32"].emb.float()[hard.long()], soft], 1)
        lg, hn = {}, {}
        for m, w in ws.items():
            d = MistralDecoder(w, max_batch=B, max_prompt=32, max_new=8)
            h = d.hidden_states(emb)[:, -1]
            hn[m] = h
            lg[m] = h @ w.lm.float().t()
            del d
        std = float(lg["f32"].std())
        out = {"layers": L, "logit_std": round(std, 3)}
        for m in ("bf16", "fp8"):
            out[m + "_err_over_std"] = round(float((lg[m] - lg["f32"]).abs().max()) / std, 4)
            out[m + "_hidden_rel"] = round(float((hn[m] - hn["f32"]).norm() / hn["f32"].norm()), 5)
        print(json.dumps(out), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
