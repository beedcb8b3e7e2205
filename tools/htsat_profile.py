#!/usr/bin/env python3
"""Per-stage / per-op timing of the HTSAT encoder at one 64-clip eval batch (single stream).

Replays AudioEncoder._htsat's op sequence with a HIP event around every op (one stream, so the
events bracket exactly that op's kernels) and prints: stage, op, ms per batch, and the op's
algorithmic HBM bytes / time.  Then times encode() back to back.

    python tools/htsat_profile.py [reps=5] [clips per pass=64]
"""
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))

import torch  # noqa: E402

from zsaac import ops, synthetic as S  # noqa: E402
from zsaac.encoder import AudioEncoder, DEPTHS, HEADS, WIN  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    dev = torch.device("cuda", 0)
    sd = S.htsat_state_dict(3)
    sd.update(S.audio_proj_state_dict(5))
    enc = AudioEncoder(sd, "htsat", torch.bfloat16, B, dev)
    wav = (torch.randn(B, 320000, device=dev) * 0.1).clamp_(-1, 1)
    enc.encode(wav)
    torch.cuda.synchronize()
    tot = defaultdict(float)
    byts = {}
    w = enc.w

    def timed(key, nbytes, fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        tot[key] += e0.elapsed_time(e1)
        byts[key] = nbytes

    for _ in range(reps):
        timed(("fe", "logmel"), B * 320000 * 4 + B * 1001 * 64 * 4,
              lambda: ops.logmel(wav, enc.tables, bn=w.bn0, out=enc.logmel[:B]))
        timed(("fe", "wav2img"), B * 1001 * 64 * 4 + B * 65536 * 4,
              lambda: ops.wav2img(enc.logmel[:B], out=enc.img[:B]))
        M, C, res = B * 4096, 96, 64
        x = enc.x[:M * C].view(M, C)
        timed(("fe", "patch_embed"), B * 65536 * 4 + M * C * 4,
              lambda: ops.patch_embed(enc.img[:B], w.pe_w, w.pe_b, *w.pe_ln, out=x))
        for i, (depth, heads) in enumerate(zip(DEPTHS, HEADS)):
            st = f"s{i + 1}"
            for j in range(depth):
                blk = w.blocks[i][j]
                shift = 0 if (j % 2 == 0 or res <= WIN) else WIN // 2
                if "qkv_p" in blk:
                    timed((st, "swin_block"), M * C * 8,
                          lambda: ops.swin_block(x, B, res, res, C, heads, shift, blk))
                    continue
                h = enc.h[:M * C].view(M, C)
                qkv = enc.qkv[:M * 3 * C].view(M, 3 * C)
                att = enc.att[:M * C].view(M, C)
                hid = enc.hid[:M * 4 * C].view(M, 4 * C)
                timed((st, "ln1"), M * C * 6, lambda: ops.layernorm(x, *blk["n1"], out=h))
                timed((st, "qkv"), M * C * 2 + M * 3 * C * 2,
                      lambda: ops.gemm(h, blk["qkv_w"], qkv, bias=blk["qkv_b"]))
                timed((st, "wattn"), M * 4 * C * 2,
                      lambda: ops.window_attention(qkv, B, res, res, C, heads, shift, blk["rel"], att))
                timed((st, "proj"), M * C * 2 + M * C * 8,
                      lambda: ops.gemm(att, blk["proj_w"], x, bias=blk["proj_b"], residual=x))
                timed((st, "ln2"), M * C * 6, lambda: ops.layernorm(x, *blk["n2"], out=h))
                timed((st, "fc1"), M * C * 2 + M * 4 * C * 2,
                      lambda: ops.gemm(h, blk["fc1_w"], hid, bias=blk["fc1_b"], act=ops.ACT_GELU_ERF))
                timed((st, "fc2"), M * 4 * C * 2 + M * C * 8,
                      lambda: ops.gemm(hid, blk["fc2_w"], x, bias=blk["fc2_b"], residual=x))
            if i < len(DEPTHS) - 1:
                mg = w.merges[i]
                Mo = M // 4
                y = enc.mrg[:Mo * 4 * C].view(Mo, 4 * C)
                timed((st, "merge_ln"), M * C * 4 + M * C * 2,
                      lambda: ops.patch_merge_ln(x, B, res, res, C, *mg["n"], out=y))
                nxt = (enc.x2 if x.data_ptr() == enc.x.data_ptr() else enc.x)[:Mo * 2 * C].view(Mo, 2 * C)
                timed((st, "merge_gemm"), M * C * 2 + Mo * 2 * C * 4,
                      lambda: ops.gemm(y, mg["red_w"], nxt))
                x, M, C, res = nxt, Mo, 2 * C, res // 2
        timed(("s4", "ln_meanpool"), M * C * 4,
              lambda: ops.ln_meanpool(x, B, res * res, C, *w.norm, out=enc.feat[:B]))
    total = sum(tot.values()) / reps
    print(f"{'stage':6s} {'op':12s} {'ms/batch':>9s} {'%':>6s} {'GB/s(algo)':>11s}")
    per_stage = defaultdict(float)
    for (st, op), t in tot.items():
        ms = t / reps
        per_stage[st] += ms
        print(f"{st:6s} {op:12s} {ms:9.4f} {100 * ms / total:6.1f} {byts[(st, op)] / ms / 1e6:11.0f}")
    for st, ms in per_stage.items():
        print(f"{st:6s} {'TOTAL':12s} {ms:9.4f} {100 * ms / total:6.1f}")
    print(f"total {total:.3f} ms per {B} clips (single stream, events around every op)")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        enc.encode(wav)
    e1.record()
    e1.synchronize()
    print(f"encode() back to back: {e0.elapsed_time(e1) / reps:.3f} ms per {B} clips")


if __name__ == "__main__":
    main()
