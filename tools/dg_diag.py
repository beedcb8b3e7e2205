#!/usr/bin/env python3
"""Diagnostic for the grid decode's canonical arithmetic: runs ONE decode step (entry_length 2) of
a golden batch as the persistent launch at grids 48 / 96 / 192 and as the phase launches, and
compares the hand-off buffers the step leaves (layer 11's q, att, hid and the final x in bf16),
the new K/V rows of every layer and the ids, byte for byte, against grid 48's persistent launch.

    python tools/dg_diag.py [golden=c1_greedy] [steps=2]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))
import torch  # noqa: E402

WS = {"q": (4096, 64 * 768 * 2), "att": (4096 + 98304, 98304), "xb": (4096 + 2 * 98304, 98304),
      "hid": (4096 + 3 * 98304, 64 * 3072 * 2)}


def main():
    from tools import idparity
    from tests.test_gpu_persist import _pipe
    name = sys.argv[1] if len(sys.argv) > 1 else "c1_greedy"
    entry = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    g = idparity.load(name)
    dev = torch.device("cuda", 0)
    emb = torch.from_numpy(g["clap_emb"]).to(dev)
    B = emb.shape[0]
    snaps = {}
    for mode in ("persist", "phases"):
        p = _pipe(g, dev, mode == "persist", entry_length=entry)
        d = p.decoder
        for grid in (48, 96, 192, 192, 48):
            if mode == "persist":
                d.persist_grid = grid
            else:
                d.phase_grid = grid
                d.graphs.clear()
            out = p.caption_emb(emb)
            torch.cuda.synchronize()
            base = d.persist_ws.data_ptr()
            off = (-base) % 256
            ws = d.persist_ws[off:]
            s = {k: ws[o:o + n].clone() for k, (o, n) in WS.items()}
            pos = d.pos[:B].long() - 1           # the row the last step appended
            for l in range(12):
                kc = d.kc[l][:B]
                s[f"k{l}"] = kc[torch.arange(B), :, pos].clone()
                s[f"v{l}"] = d.vc[l][:B][torch.arange(B), :, pos].clone()
            s["ids"] = d.out_ids[:B].clone()
            snaps[mode, grid, len(snaps)] = s
    ref = snaps["persist", 48, 0]
    rep = {}
    for key, s in snaps.items():
        diff = {}
        for k, t in s.items():
            if not torch.equal(t, ref[k]):
                n = int((t != ref[k]).sum())
                diff[k] = n
        rep[f"{key[0]}{key[1]}#{key[2]}"] = diff
    print(json.dumps(rep), flush=True)


if __name__ == "__main__":
    main()
