#!/usr/bin/env python3
"""Micro-benchmarks of individual zsaac kernels on the GPU (graph-replayed back-to-back launches,
HIP events on the launching stream).  Used to choose kernel variants; not part of the product.

    python tools/mbench.py gemm      # decode-shaped GEMMs, skinny modes vs tiled vs torch
    python tools/mbench.py attn      # decode attention
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))

import torch  # noqa: E402


def timeit(fn, reps=100, rounds=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
        g.replay()
        ts = []
        for _ in range(rounds):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            g.replay()
            e1.record(s)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3 / reps)
    torch.cuda.current_stream().wait_stream(s)
    ts.sort()
    return ts[len(ts) // 2]


def bench_gemm():
    from zsaac import ops
    from zsaac._lib import call
    dev = torch.device("cuda", 0)
    shapes = [(64, 2304, 768, "qkv"), (64, 768, 768, "proj"), (64, 3072, 768, "fc"),
              (64, 768, 3072, "mproj"), (64, 7680, 3840, "mlp2"), (64, 50304, 768, "lm-ish")]
    for M, N, K, name in shapes:
        ops.reserve_skinny_workspace(dev, M, N, K)
        a = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) * 0.02).bfloat16()
        b = torch.randn(N, device=dev)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        wbytes = N * K * 2
        res = {}
        for mode in (0, 1):
            call("zs_tune_set", b"skinny_mode", mode)
            res[f"skinny{mode}"] = timeit(lambda: ops.gemm(a, w, out, bias=b))
        call("zs_tune_set", b"skinny_mode", 1)
        res["tiled"] = timeit(lambda: ops.gemm(a, w, out, bias=b, split_k=1))
        res["torch"] = timeit(lambda: torch.nn.functional.linear(a, w, b.bfloat16()))
        print(f"{name:6s} M{M} N{N} K{K} W={wbytes / 1e6:.1f}MB  " +
              "  ".join(f"{k}={v:7.2f}us ({wbytes / v / 1e3:6.0f} GB/s)" for k, v in res.items()),
              flush=True)


def bench_gemm_m():
    """Decode GEMM shapes at M = 64..1280 (continuous batching / beam rows): ours vs hipBLASLt."""
    from zsaac import ops
    dev = torch.device("cuda", 0)
    for M in (64, 256, 1280, 1856, 16384, 65536):
        for N, K, name in ((2304, 768, "qkv"), (768, 768, "proj"), (3072, 768, "fc"), (768, 3072, "mproj")):
            ws = ops.skinny_workspace(dev, [(M, N, K)])
            a = torch.randn(M, K, device=dev).bfloat16()
            w = (torch.randn(N, K, device=dev) * 0.02).bfloat16()
            b = torch.randn(N, device=dev)
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            from zsaac._lib import call
            res = {}
            if ws is not None:
                res["skinny"] = timeit(lambda: ops.gemm(a, w, out, bias=b, workspace=ws))
            res["fast"] = timeit(lambda: ops.gemm(a, w, out, bias=b, split_k=1))
            call("zs_tune_set", b"gemm_fast", 0)
            res["old"] = timeit(lambda: ops.gemm(a, w, out, bias=b, split_k=1))
            call("zs_tune_set", b"gemm_fast", 1)
            res["torch"] = timeit(lambda: torch.nn.functional.linear(a, w, b.bfloat16()))
            print(f"M{M:5d} {name:6s} N{N} K{K}  " + "  ".join(f"{k}={v:7.2f}us" for k, v in res.items()),
                  flush=True)


def bench_gemm_c3():
    """The C3 beam decode's GEMMs (M = 1280 rows) under each lean tile the dispatch can force
    (fast_tile 100 + lt) against the default pick, TF/s."""
    from zsaac import ops
    from zsaac._lib import call
    dev = torch.device("cuda", 0)
    M = int(os.environ.get("ZS_M", 1280))
    for N, K, name in ((2304, 768, "qkv"), (768, 768, "proj"), (3072, 768, "fc"), (768, 3072, "mproj")):
        a = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) * 0.02).bfloat16()
        b = torch.randn(N, device=dev)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        res = {"default": timeit(lambda: ops.gemm(a, w, out, bias=b, split_k=1))}
        ws = torch.zeros(8 * M * N, device=dev)
        for sk in (2, 3, 4, 6):               # split-K on the fast tiles + the reduce launch
            if K % (32 * sk) == 0:
                res[f"sk{sk}"] = timeit(lambda: ops.gemm(a, w, out, bias=b, split_k=sk, workspace=ws))
        for lt in (1, 2, 3, 5, 6, 8, 9, 10, 11, 12, 13):
            call("zs_tune_set", b"fast_tile", 100 + lt)
            try:
                res[f"lt{lt}"] = timeit(lambda: ops.gemm(a, w, out, bias=b, split_k=1))
            except Exception:
                pass
            call("zs_tune_set", b"fast_tile", 0)
        fl = 2 * M * N * K
        print(f"M{M} {name:6s} N{N} K{K}  " + "  ".join(f"{k}={v:6.2f}us/{fl / v / 1e6:4.0f}"
                                                   for k, v in res.items()), flush=True)


def bench_gemm_htsat():
    """HTSAT encoder GEMM shapes for one 64-clip batch: tokens 4096/1024/256/64 per clip."""
    from zsaac import ops
    from zsaac._lib import call
    dev = torch.device("cuda", 0)
    clips = int(os.environ.get("ZS_CLIPS", 64))
    for C, T in ((96, 4096), (192, 1024), (384, 256), (768, 64)):
        M = clips * T
        shapes = [(3 * C, C, "qkv"), (C, C, "proj"), (4 * C, C, "fc1"), (C, 4 * C, "fc2")]
        if C < 768:
            shapes.append((2 * C, 4 * C, "merge"))
            Mm = M // 4
        for N, K, name in shapes:
            Mr = Mm if name == "merge" else M
            a = torch.randn(Mr, K, device=dev).bfloat16()
            w = (torch.randn(N, K, device=dev) * 0.02).bfloat16()
            b = torch.randn(N, device=dev)
            out = torch.empty(Mr, N, device=dev, dtype=torch.bfloat16)
            res = {}
            for t, nm in ((0, "auto"), (4, "128x128"), (15, "256x128w8"), (16, "128x256w8")):
                call("zs_tune_set", b"fast_tile", t)
                res[nm] = timeit(lambda: ops.gemm(a, w, out, bias=b, split_k=1), reps=20)
            call("zs_tune_set", b"fast_tile", 0)
            call("zs_tune_set", b"gemm_fast", 0)
            res["old"] = timeit(lambda: ops.gemm(a, w, out, bias=b, split_k=1), reps=20)
            call("zs_tune_set", b"gemm_fast", 1)
            res["torch"] = timeit(lambda: torch.nn.functional.linear(a, w, b.bfloat16()), reps=20)
            gbs = (Mr * K + Mr * N + N * K) * 2 / res["auto"] / 1e3
            tf = 2 * Mr * N * K / 1e6
            print(f"C{C:4d} M{Mr:7d} {name:6s} N{N:5d} K{K:5d} auto {gbs:5.0f} GB/s " +
                  "  ".join(f"{k}={v:8.2f}us/{tf / v:5.0f}TF" for k, v in res.items()), flush=True)


def bench_gemm_f32():
    """The f32 parity mode's tiled GEMMs (HTSAT unfused at 64 clips + GPT-2 prefill at 64 x 27
    rows): zs_gemm f32 vs torch.nn.functional.linear (hipBLASLt, exact f32), us and TF/s."""
    from zsaac import ops
    dev = torch.device("cuda", 0)
    shapes = []
    clips = int(os.environ.get("ZS_CLIPS", 64))
    for C, T in ((96, 4096), (192, 1024), (384, 256), (768, 64)):
        M = clips * T
        shapes += [(M, 3 * C, C, f"C{C} qkv"), (M, C, C, f"C{C} proj"), (M, 4 * C, C, f"C{C} fc1"),
                   (M, C, 4 * C, f"C{C} fc2")]
        if C < 768:
            shapes.append((M // 4, 2 * C, 4 * C, f"C{C} merge"))
    P = 64 * 27
    shapes += [(P, 2304, 768, "pre qkv"), (P, 768, 768, "pre proj"), (P, 3072, 768, "pre fc"),
               (P, 768, 3072, "pre mproj")]
    tot = {"zs": 0.0, "torch": 0.0}
    for M, N, K, name in shapes:
        a = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev) * 0.02
        b = torch.randn(N, device=dev)
        out = torch.empty(M, N, device=dev)
        from zsaac._lib import call
        r = {"zs": timeit(lambda: ops.gemm(a, w, out, bias=b, split_k=1), reps=10)}
        ref = torch.nn.functional.linear(a.double(), w.double(), b.double())
        err_new = float(((out.double() - ref).abs().max() / ref.abs().max()))
        call("zs_tune_set", b"f32_fast", 0)
        r["old"] = timeit(lambda: ops.gemm(a, w, out, bias=b, split_k=1), reps=10)
        err_old = float(((out.double() - ref).abs().max() / ref.abs().max()))
        call("zs_tune_set", b"f32_fast", 1)
        r["torch"] = timeit(lambda: torch.nn.functional.linear(a, w, b), reps=10)
        tot.setdefault("old", 0.0)
        for k in tot:
            tot[k] += r[k] * (2 if not name.endswith("merge") and not name.startswith("pre") and
                              not name.startswith("C768") else 1)
        fl = 2 * M * N * K
        gbs = (M * K + M * N + N * K) * 4 / r["zs"] / 1e3
        print(f"{name:10s} M{M:7d} N{N:5d} K{K:5d}  " +
              "  ".join(f"{k}={v:8.1f}us/{fl / v / 1e6:4.0f}TF" for k, v in r.items()) +
              f"  zs {gbs:5.0f} GB/s  err new {err_new:.1e} old {err_old:.1e}", flush=True)
    print(f"sum (HTSAT blocks x2 per stage except C768 x1... see shapes): {tot}", flush=True)


def bench_gemm_f32_tiles():
    """The f32 parity mode's big tiled GEMM shapes under each zs_tune_set("f32_tile", t) variant
    (gemm.hip dispatch_fast_f32), us per shape and the HTSAT + prefill total; outputs must be
    bit-identical to variant 0 (the same k order)."""
    from zsaac import ops
    from zsaac._lib import call
    dev = torch.device("cuda", 0)
    shapes = []
    clips = int(os.environ.get("ZS_CLIPS", 64))
    for C, T in ((96, 4096), (192, 1024), (384, 256), (768, 64)):
        M = clips * T
        shapes += [(M, 3 * C, C, f"C{C} qkv", 2), (M, C, C, f"C{C} proj", 2),
                   (M, 4 * C, C, f"C{C} fc1", 2), (M, C, 4 * C, f"C{C} fc2", 2)]
        if C < 768:
            shapes.append((M // 4, 2 * C, 4 * C, f"C{C} merge", 1))
    P = 64 * 27
    shapes += [(P, 2304, 768, "pre qkv", 12), (P, 768, 768, "pre proj", 12), (P, 3072, 768, "pre fc", 12),
               (P, 768, 3072, "pre mproj", 12)]
    tot = {}
    for M, N, K, name, mult in shapes:
        a = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev) * 0.02
        b = torch.randn(N, device=dev)
        out = torch.empty(M, N, device=dev)
        row = []
        ref = None
        for t in (8, 0, 10, 11):
            call("zs_tune_set", b"f32_tile", t)
            us = timeit(lambda: ops.gemm(a, w, out, bias=b, split_k=1), reps=10)
            same = True if ref is None else bool(torch.equal(out, ref))
            if ref is None:
                ref = out.clone()
            tot[t] = tot.get(t, 0.0) + us * mult
            row.append(f"t{t}={us:7.1f}{'' if same else '!'}")
        call("zs_tune_set", b"f32_tile", 8)       # the default
        print(f"{name:10s} M{M:7d} N{N:5d} K{K:5d}  " + " ".join(row), flush=True)
    print("weighted total us (HTSAT x2 per block, prefill x12 layers):",
          {t: round(v, 1) for t, v in tot.items()}, flush=True)


def bench_gemm_dbg():
    """Where the fast GEMM's time goes: full / no-MFMA / no-DMA at a few encoder shapes."""
    from zsaac import ops
    from zsaac._lib import call
    dev = torch.device("cuda", 0)
    shapes = [(4096, 2304, 768), (16384, 1152, 384), (65536, 768, 192), (262144, 288, 96),
              (65536, 2304, 768)]
    if os.environ.get("ZS_DBG_SHAPES"):
        shapes = [tuple(int(x) for x in t.split("x")) for t in os.environ["ZS_DBG_SHAPES"].split(",")]
    for M, N, K in shapes:
        a = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) * 0.02).bfloat16()
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        res = {}
        tiles = [(int(t), f"t{t}", 1) for t in os.environ.get("ZS_TILES", "").split(",") if t]
        dbgs = [(int(d), f"d{d}") for d in os.environ.get("ZS_DBGS", "").split(",") if d]
        for t, nm, pers in (tiles or ((4, "128x128P", 1), (15, "256x128w8", 1), (16, "128x256w8", 1))):
            call("zs_tune_set", b"fast_tile", t)
            call("zs_tune_set", b"fast_persist", pers)
            for d, dn in (dbgs or ((0, "full"), (3, "noLoop"), (4, "noEpi"))):
                call("zs_tune_set", b"gemm_dbg", d)
                res[f"{nm}/{dn}"] = timeit(lambda: ops.gemm(a, w, out, split_k=1), reps=20)
        call("zs_tune_set", b"gemm_dbg", 0)
        call("zs_tune_set", b"fast_tile", 0)
        call("zs_tune_set", b"fast_persist", 1)
        res["torch"] = timeit(lambda: torch.nn.functional.linear(a, w), reps=20)
        print(f"M{M:6d} N{N:5d} K{K:4d} " + "  ".join(f"{k}={v:7.1f}" for k, v in res.items()),
              flush=True)


def bench_rows():
    """Row-group GEMM (M <= 64) and its LN-fused form at decode shapes vs rows / columns / K,
    hot weights (graph-replayed back-to-back launches); launch floor for comparison."""
    from zsaac import ops
    dev = torch.device("cuda", 0)
    t_empty = timeit(lambda: torch.cuda._sleep(0), reps=100) if False else None
    x = torch.randn(64, 768, device=dev)
    lw, lb = torch.ones(768, device=dev), torch.zeros(768, device=dev)
    for N, K in ((768, 768), (2304, 768), (3072, 768), (768, 3072), (256, 768), (64, 768)):
        w = (torch.randn(N, K, device=dev) * 0.02).bfloat16()
        bias = torch.randn(N, device=dev)
        r = {}
        for M in (1, 16, 64):
            a = torch.randn(M, K, device=dev).bfloat16()
            o = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            of = torch.empty(M, N, device=dev)
            r[f"M{M}"] = timeit(lambda: ops.gemm(a, w, o))
            r[f"M{M}+b+r"] = timeit(lambda: ops.gemm(a, w, of, bias=bias, residual=of))
            if K == 768:
                r[f"M{M}ln"] = timeit(lambda: ops.gemm_ln(x[:M], lw, lb, w, o, bias=bias))
        print(f"rows N{N} K{K} " + "  ".join(f"{k}={v:6.2f}" for k, v in r.items()), flush=True)


def bench_overhead():
    """Per-launch cost of tiny kernels in a graph-replayed chain (the floor every decode-step
    kernel pays): cast of 64 floats, LayerNorm at 64 / 2048 rows, a 128x128x64 GEMM."""
    from zsaac import ops
    dev = torch.device("cuda", 0)
    x = torch.randn(2048, 768, device=dev)
    y = torch.empty(2048, 768, device=dev, dtype=torch.bfloat16)
    w = torch.ones(768, device=dev)
    b = torch.zeros(768, device=dev)
    t = torch.empty(64, device=dev, dtype=torch.bfloat16)
    a = torch.randn(128, 64, device=dev).bfloat16()
    wt = torch.randn(128, 64, device=dev).bfloat16()
    o = torch.empty(128, 128, device=dev, dtype=torch.bfloat16)
    r = {
        "cast64": timeit(lambda: ops.cast(x.view(-1)[:64], t), reps=200),
        "ln64": timeit(lambda: ops.layernorm(x[:64], w, b, out=y[:64]), reps=200),
        "ln2048": timeit(lambda: ops.layernorm(x, w, b, out=y), reps=200),
        "gemm128": timeit(lambda: ops.gemm(a, wt, o, split_k=1), reps=200),
    }
    print("  ".join(f"{k}={v:6.2f}us" for k, v in r.items()), flush=True)


def bench_lmhead():
    """LM head GEMM + fused row reductions at decode row counts (topk 1 greedy, 8 beam)."""
    from zsaac import ops
    dev = torch.device("cuda", 0)
    V, K = 50257, 768
    w = (torch.randn(V, K, device=dev) * 0.05).bfloat16()
    nblk = ops.lmhead_nblk(V)
    for M in (64, 256, 1280, 2048, 8192):
        a = torch.randn(M, K, device=dev).bfloat16()
        ps = torch.empty(M, nblk, 2, device=dev)
        res = {}
        for k in (1, 5):
            pv = torch.empty(M, nblk, k, device=dev)
            pi = torch.empty(M, nblk, k, device=dev, dtype=torch.int32)
            res[f"topk{k}"] = timeit(lambda: ops.lmhead_topk(a, w, k, ps, pv, pi), reps=20)
            res[f"topk{k}_nostat"] = timeit(lambda: ops.lmhead_topk(a, w, k, None, pv, pi), reps=20)
        lo = torch.empty(M, V, device=dev, dtype=torch.bfloat16)
        res["zs_gemm_bf16out"] = timeit(lambda: ops.gemm(a, w, lo), reps=20)
        pv = torch.empty(M, nblk, 1, device=dev)
        pi = torch.empty(M, nblk, 1, device=dev, dtype=torch.int32)
        res["rownorm"] = timeit(lambda: ops.lmhead_topk(a, w, 1, ps, pv, pi, row_norm=True), reps=20)
        res["torch_gemm"] = timeit(lambda: a @ w.t(), reps=20)
        fl = 2 * M * V * K
        print(f"lmhead M{M:5d} " + "  ".join(f"{k}={v:8.2f}us ({fl / v / 1e6:6.0f} TF/s)" for k, v in res.items()),
              flush=True)


def bench_front():
    """Front end + HTSAT edge kernels for one 64-clip batch."""
    from zsaac import ops
    from zsaac.frontend import make_tables
    dev = torch.device("cuda", 0)
    B = 64
    wav = (torch.randn(B, 320000, device=dev) * 0.1).clamp_(-1, 1)
    tabs = make_tables(dev)
    lm = torch.empty(B, 1001, 64, device=dev)
    from zsaac._lib import call
    for wv in (1, 0):
        call("zs_tune_set", b"logmel_wave", wv)
        print(f"logmel B64 wave={wv}: {timeit(lambda: ops.logmel(wav, tabs, out=lm), reps=10):8.1f}us", flush=True)
    call("zs_tune_set", b"logmel_wave", 1)
    img = torch.empty(B, 256, 256, device=dev)
    print(f"wav2img B64:     {timeit(lambda: ops.wav2img(lm, out=img), reps=10):8.1f}us", flush=True)
    w, b = torch.randn(96, 16, device=dev), torch.randn(96, device=dev)
    lw, lb = torch.randn(96, device=dev), torch.randn(96, device=dev)
    x = torch.empty(B * 4096, 96, device=dev)
    print(f"patch_embed B64: {timeit(lambda: ops.patch_embed(img, w, b, lw, lb, out=x), reps=10):8.1f}us", flush=True)
    for H, C in ((64, 96), (32, 192), (16, 384)):
        xm = torch.randn(B * H * H, C, device=dev)
        yw, yb = torch.randn(4 * C, device=dev), torch.randn(4 * C, device=dev)
        ym = torch.empty(B * H * H // 4, 4 * C, device=dev, dtype=torch.bfloat16)
        t = timeit(lambda: ops.patch_merge_ln(xm, B, H, H, C, yw, yb, ym), reps=10)
        byts = xm.numel() * 4 + ym.numel() * 2
        print(f"patch_merge_ln H{H} C{C}: {t:8.1f}us ({byts / t / 1e3:5.0f} GB/s)", flush=True)
    for C in (96, 192, 384, 768):
        M = B * 4096 * 96 // C
        xl = torch.randn(M, C, device=dev)
        ylo = torch.empty(M, C, device=dev, dtype=torch.bfloat16)
        wl, bl = torch.randn(C, device=dev), torch.randn(C, device=dev)
        t = timeit(lambda: ops.layernorm(xl, wl, bl, out=ylo), reps=10)
        print(f"layernorm M{M} C{C}: {t:8.1f}us ({M * C * 6 / t / 1e3:5.0f} GB/s)", flush=True)
    xs = torch.randn(B * 64, 768, device=dev)
    lw2, lb2 = torch.randn(768, device=dev), torch.randn(768, device=dev)
    feat = torch.empty(B, 768, device=dev)
    print(f"ln_meanpool B64: {timeit(lambda: ops.ln_meanpool(xs, B, 64, 768, lw2, lb2, feat), reps=10):8.1f}us", flush=True)


def bench_window():
    """HTSAT window attention per stage for one 64-clip batch: MFMA vs VALU kernel."""
    from zsaac import ops
    from zsaac._lib import call
    dev = torch.device("cuda", 0)
    B = 64
    for res, heads, shift in ((64, 4, 4), (32, 8, 4), (16, 16, 4), (8, 32, 0)):
        C = 24 * heads
        qkv = torch.randn(B * res * res, 3 * C, device=dev).bfloat16()
        table = torch.randn(225, heads, device=dev)
        out = torch.empty(B * res * res, C, device=dev, dtype=torch.bfloat16)
        res_t = {}
        for v in (1, 0):
            call("zs_tune_set", b"window_mfma", v)
            res_t["mfma" if v else "valu"] = timeit(
                lambda: ops.window_attention(qkv, B, res, res, C, heads, shift, table, out), reps=10)
        call("zs_tune_set", b"window_mfma", 1)
        byts = qkv.numel() * 2 + out.numel() * 2
        print(f"window res{res:3d} heads{heads:3d} " + "  ".join(f"{k}={v:8.1f}us" for k, v in res_t.items())
              + f"  ({byts / res_t['mfma'] / 1e3:6.0f} GB/s mfma)", flush=True)


def bench_decode_gemm():
    """Decode-step GEMMs at 2048 rows with cold weights (rotating > 256 MiB of W copies), per tile,
    with the decoder's epilogues (proj/mproj: f32 out + residual; fc: GELU), and split-K."""
    from zsaac import ops
    from zsaac._lib import call
    dev = torch.device("cuda", 0)
    M = int(os.environ.get("ZS_M", "2048"))
    ws = torch.empty(8 * M * 3072, device=dev)
    for N, K, name in ((2304, 768, "qkv"), (768, 768, "proj"), (3072, 768, "fc"), (768, 3072, "mproj")):
        a = torch.randn(M, K, device=dev).bfloat16()
        w0 = (torch.randn(N, K, device=dev) * 0.02).bfloat16()
        wsl = [w0] + [w0.clone() for _ in range(max(1, (640 << 20) // w0.nbytes))]
        b = torch.randn(N, device=dev)
        f32 = name in ("proj", "mproj")
        out = torch.empty(M, N, device=dev, dtype=torch.float32 if f32 else torch.bfloat16)
        res = torch.randn(M, N, device=dev) if f32 else None
        act = ops.ACT_GELU_TANH if name == "fc" else ops.ACT_NONE
        it = [0]

        def run(sk=1):
            ops.gemm(a, wsl[it[0] % len(wsl)], out, bias=b, residual=res, act=act, split_k=sk,
                     workspace=ws if sk > 1 else None)
            it[0] += 1
        r = {}
        tiles = os.environ.get("ZS_TILES")
        tl = ([(int(t), f"t{t}") for t in tiles.split(",")] if tiles else
              [(0, "auto"), (4, "128x128"), (15, "256x128w8"), (16, "128x256w8"), (8, "128x64"),
               (9, "64x128")])
        for t, nm in tl:
            call("zs_tune_set", b"fast_tile", t)
            lean = os.environ.get("ZS_LEAN")
            if lean is not None:
                call("zs_tune_set", b"gemm_lean", int(lean))
            r[nm] = timeit(run, reps=len(wsl))
        for sk in ((2, 3, 4) if not tiles else ()):
            call("zs_tune_set", b"fast_tile", 4)
            r[f"128sk{sk}"] = timeit(lambda: run(sk), reps=len(wsl))
        call("zs_tune_set", b"fast_tile", 0)
        fl = 2 * M * N * K
        print(f"M{M} {name:6s} " + "  ".join(f"{k}={v:5.1f}({fl / v / 1e6:4.0f})" for k, v in r.items()), flush=True)


def bench_attn():
    """Decode attention at the bench's decode shape (2048 rows x 12 heads, Lmax 102): attn6 /
    attn5 / LDS-staged, HBM GB/s of the K/V bytes read."""
    from zsaac import ops
    from zsaac._lib import call
    dev = torch.device("cuda", 0)
    R, D, H, Lmax = int(os.environ.get("ZS_M", 2048)), 768, 12, 102
    kc = torch.randn(R, H, Lmax, 64, device=dev).bfloat16()
    vc = torch.randn_like(kc)
    qkv = torch.randn(R, 3 * D, device=dev).bfloat16()
    out = torch.empty(R, D, device=dev, dtype=torch.bfloat16)
    for L in (32, 64, 96):
        pos = torch.full((R,), L - 1, device=dev, dtype=torch.int32)
        byts = R * H * L * 64 * 2 * 2
        r = {}
        for v in [int(x) for x in os.environ.get("ZS_VARIANTS", "3,2,1").split(",")]:
            call("zs_tune_set", b"decode_attn5", v)
            r[v] = timeit(lambda: ops.decode_attention(qkv, R, D, H, kc, vc, Lmax, pos, out), reps=20)
        call("zs_tune_set", b"decode_attn5", 2)
        print(f"decode_attn R={R} L={L}: " + "  ".join(
            f"v{v}={t:7.2f}us ({byts / t / 1e3:5.0f} GB/s)" for v, t in r.items()), flush=True)
    x = torch.randn(R, 768, device=dev)
    w, bb = torch.randn(768, device=dev), torch.randn(768, device=dev)
    y = torch.empty(R, 768, device=dev, dtype=torch.bfloat16)
    t = timeit(lambda: ops.layernorm(x, w, bb, out=y))
    print(f"layernorm {R}x768: {t:7.2f}us ({R * 768 * 6 / t / 1e3:5.0f} GB/s)")


def bench_gemm_big():
    """bf16 GEMMs of >= 1k rows: the 256 x 256 multi-phase tile (gemm_big) against the lean
    128 x 128 / 8-wave tiles (gemm_big=0) and torch (hipBLASLt); TFLOP/s."""
    from zsaac import ops
    from zsaac._lib import call
    dev = torch.device("cuda", 0)
    shapes = [(1600, 2304, 768, "prefill qkv"), (1600, 3072, 768, "prefill fc"),
              (1280, 3072, 768, "c3 fc"), (1280, 768, 3072, "c3 mproj"),
              (8192, 3072, 768, "tput fc"), (8192, 768, 3072, "tput mproj"),
              (8192, 2304, 768, "tput qkv"), (4096, 4096, 4096, "4k"), (8192, 8192, 8192, "8k"),
              (2048, 3072, 768, "bert fc-ish")]
    for M, N, K, name in shapes:
        a = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) * 0.02).bfloat16()
        b = torch.randn(N, device=dev)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        res = {}
        for arm, knobs in (("big", {"fast_tile": 18}), ("auto", {}), ("lean", {"gemm_big": 0})):
            for k, v in knobs.items():
                call("zs_tune_set", k.encode(), v)
            res[arm] = timeit(lambda: ops.gemm(a, w, out, bias=b, split_k=1), reps=10)
            call("zs_tune_set", b"fast_tile", 0)
            call("zs_tune_set", b"gemm_big", 1)
        res["torch"] = timeit(lambda: torch.nn.functional.linear(a, w, b.bfloat16()), reps=10)
        print(f"{name:12s} {M}x{N}x{K}: " + "  ".join(
            f"{k}={v:8.1f}us ({fl / v / 1e6:6.0f} TF)" for k, v in res.items()), flush=True)


def bench_attn_beam():
    """Beam decode attention (C3: 256 clips x beam 5 = 1280 rows, kvrow indirection as
    generate_beam's reordered caches): the R > 128 variants (decode_attn5 knob) and the small-R
    kernels with their row cap lifted (small_rmax), GB/s of the K/V bytes read."""
    from zsaac import ops
    from zsaac._lib import call
    dev = torch.device("cuda", 0)
    R, D, H, Lmax, beam = int(os.environ.get("ZS_M", 1280)), 768, 12, 102, 5
    kc = torch.randn(R, H, Lmax, 64, device=dev).bfloat16()
    vc = torch.randn_like(kc)
    qkv = torch.randn(R, 3 * D, device=dev).bfloat16()
    out = torch.empty(R, D, device=dev, dtype=torch.bfloat16)
    # kvrow: each row's keys come from the rows of its own clip (a clip's 5 beams)
    clip = torch.arange(R, device=dev) // beam
    kvrow = (clip[:, None] * beam + torch.randint(0, beam, (R, Lmax), device=dev)).int().contiguous()
    arms = [("v4", {"decode_attn5": 4}), ("v4_noxcd", {"decode_attn5": 4, "beam_xcd": 1}),
            ("v3", {"decode_attn5": 3}), ("v2", {"decode_attn5": 2}),
            ("v5", {"decode_attn5": 5}), ("v6", {"decode_attn5": 6}),
            ("small128", {"small_rmax": 4096, "attn_split": 0}),
            ("small_s1", {"small_rmax": 4096, "attn_split": 1}),
            ("small_s3", {"small_rmax": 4096, "attn_split": 3})]
    for L in (30, 60, 90):
        pos = torch.full((R,), L - 1, device=dev, dtype=torch.int32)
        byts = R * H * L * 64 * 2 * 2
        r = {}
        for name, knobs in arms:
            for k, v in knobs.items():
                call("zs_tune_set", k.encode(), v)
            r[name] = timeit(lambda: ops.decode_attention(qkv, R, D, H, kc, vc, Lmax, pos, out,
                                                          kvrow=kvrow), reps=20)
            call("zs_tune_set", b"decode_attn5", 6)
            call("zs_tune_set", b"small_rmax", 128)
            call("zs_tune_set", b"attn_split", 3)
            call("zs_tune_set", b"beam_xcd", 5)
        print(f"beam attn R={R} L={L}: " + "  ".join(
            f"{n}={t:7.2f}us ({byts / t / 1e3:5.0f} GB/s)" for n, t in r.items()), flush=True)


def bench_inflight():
    """End-to-end clips/s vs the number of concurrently decoded bs=64 batches."""
    sys.path.insert(0, ROOT)
    import bench
    from zsaac.pipeline import ConcurrentRunner

    class A:
        batch, dtype, encoder, mapper, beam, entry_length = 64, "bf16", "htsat", "mlp", 0, 67
    pipe, _, _ = bench.build(A, torch.device("cuda", 0))
    g = torch.Generator(device="cuda").manual_seed(1)
    wavs = [(torch.randn(64, 320000, device="cuda", generator=g) * 0.1).clamp_(-1, 1) for _ in range(8)]
    for k in (1, 2, 4, 6, 8):
        runner = ConcurrentRunner(pipe, k)
        runner.warmup(wavs[0])
        torch.cuda.synchronize()
        nb = max(8, 3 * k)
        t = time.perf_counter()
        runner.run([wavs[i % len(wavs)] for i in range(nb)])
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        print(f"inflight={k}: {nb * 64 / dt:8.1f} clips/s  ({dt / nb * 1e3:.1f} ms/batch)  "
              f"decode steps {runner.decode_steps}", flush=True)


def bench_buckets():
    """Greedy decode chunk time per compaction bucket (G32 = 2048 rows, one stream) vs the
    uncompacted chunk: is a step's time proportional to its rows?"""
    sys.path.insert(0, ROOT)
    import bench

    class A:
        batch, dtype, encoder, mapper, beam, entry_length, group = 64, "bf16", "htsat", "mlp", 0, 67, 32
    pipe, _, _ = bench.build(A, torch.device("cuda", 0))
    g = torch.Generator(device="cuda").manual_seed(1)
    wav = (torch.randn(2048, 320000, device="cuda", generator=g) * 0.1).clamp_(-1, 1)
    pipe.caption_wav(wav)
    dec = pipe.decoder
    R = dec._cgreedy
    print(f"rows {R}, chunk {dec.chunk}, done {int(dec.done.sum())}", flush=True)
    plans = [("full", dec._active[0], dec._active[1], None)]
    for Rb in range(dec.min_bucket, R + 1, dec.bucket):
        plans.append((f"Rb={Rb}",) + dec._chunk_plan(Rb))
    for name, key, body, pre in plans:
        gr = dec._graph(key, body, pre)
        gr.replay()
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(4):
                gr.replay()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) / 4 / dec.chunk)
        ts.sort()
        print(f"{name:10s} {ts[2] * 1e3:8.1f} us/step", flush=True)


def bench_compact_ab():
    """End-to-end clips/s (G32 batches of 2048) with/without compaction, fixed vs adaptive
    buckets, 1 and 2 batches in flight."""
    sys.path.insert(0, ROOT)
    import bench
    from zsaac.pipeline import ConcurrentRunner
    g = torch.Generator(device="cuda").manual_seed(1)
    wavs = [(torch.randn(2048, 320000, device="cuda", generator=g) * 0.1).clamp_(-1, 1) for _ in range(2)]
    for compact in (0, 1):
        class A:
            batch, dtype, encoder, mapper, beam, entry_length, group = 64, "bf16", "htsat", "mlp", 0, 67, 32
        A.compact = compact
        pipe, _, _ = bench.build(A, torch.device("cuda", 0))
        for k in (1, 2):
            runner = ConcurrentRunner(pipe, k)
            runner.warmup(wavs[0])
            for fixed in ((0, 1) if compact else (0,)):
                for p in runner.pipes:
                    if fixed:
                        p.decoder._bucket_rows = lambda R, alive: R
                    else:
                        p.decoder.__dict__.pop("_bucket_rows", None)
                runner.run(wavs[:k])
                torch.cuda.synchronize()
                nb = 4
                t = time.perf_counter()
                runner.run([wavs[i % 2] for i in range(nb)])
                torch.cuda.synchronize()
                dt = time.perf_counter() - t
                print(f"compact={compact} fixed={fixed} inflight={k}: {nb * 2048 / dt:8.1f} clips/s",
                      flush=True)
            del runner
        del pipe
        torch.cuda.empty_cache()


def bench_host():
    """Host (Python + ctypes) enqueue time vs GPU time of one group's begin_wav (encode 32 x 64
    clips + mapper + prefill + step 0), and of one decode chunk."""
    sys.path.insert(0, ROOT)
    import bench

    class A:
        batch, dtype, encoder, mapper, beam, entry_length, group, compact = \
            64, "bf16", "htsat", "mlp", 0, 67, 32, 1
    pipe, _, _ = bench.build(A, torch.device("cuda", 0))
    g = torch.Generator(device="cuda").manual_seed(1)
    wav = (torch.randn(2048, 320000, device="cuda", generator=g) * 0.1).clamp_(-1, 1)
    pipe.caption_wav(wav)
    torch.cuda.synchronize()
    for what, fn in (("encode 2048", lambda: pipe.encode(wav)), ("begin_wav 2048", lambda: pipe.begin_wav(wav)),
                     ("encode 64", lambda: pipe.encoder.encode(wav[:64]))):
        for _ in range(2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            t = time.perf_counter()
            fn()
            th = time.perf_counter() - t
            e1.record()
            e1.synchronize()
            print(f"{what:16s} host {th * 1e3:8.2f} ms   gpu {e0.elapsed_time(e1):8.2f} ms", flush=True)


if __name__ == "__main__":
    if os.environ.get("ZS_TUNE"):          # e.g. ZS_TUNE=fast_xcd=0,fast_tile=4
        from zsaac._lib import call
        for kv in os.environ["ZS_TUNE"].split(","):
            k, v = kv.split("=")
            call("zs_tune_set", k.encode(), int(v))
    which = sys.argv[1:] or ["gemm", "attn"]
    for wname in which:
        {"gemm": bench_gemm, "rows": bench_rows, "gemm_m": bench_gemm_m, "gemm_c3": bench_gemm_c3, "gemm_htsat": bench_gemm_htsat, "gemm_f32": bench_gemm_f32, "gemm_f32_tiles": bench_gemm_f32_tiles, "gemm_dbg": bench_gemm_dbg, "lmhead": bench_lmhead, "overhead": bench_overhead, "front": bench_front, "window": bench_window, "decode_gemm": bench_decode_gemm, "attn": bench_attn, "attn_beam": bench_attn_beam, "gemm_big": bench_gemm_big, "inflight": bench_inflight, "buckets": bench_buckets, "compact_ab": bench_compact_ab, "host": bench_host}[wname]()
