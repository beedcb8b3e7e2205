"""oracle/mistral.py pinned to the reference's C5 Mistral caption path goldens
(tests/golden/mistral.npz: ClapCaption_Mistralai_prompt.clap_to_gpt + MistralForCausalLM.generate
as predict_mistralai_multilingual.py:97-111 run them)."""
import numpy as np
import torch

from oracle import mistral as OM
from zsaac import synthetic as S


def _strip(row, eos=2):
    row = [int(t) for t in row]
    if eos in row:
        row = row[:row.index(eos) + 1]
    return row


def test_mistral_generate_vs_reference(golden):
    g = golden("mistral.npz")
    sd = S.mistral_state_dict()
    mlp = S.mlp_mapper_state_dict(31, prefix_length=10, d=1024)
    emb = torch.from_numpy(g["clap_emb"])[:, None]
    hard = torch.from_numpy(g["hard_ids"])
    for tag in ("en", "fr"):
        pe, _ = OM.clap_to_gpt(emb, hard, torch.from_numpy(g[f"tag_{tag}"]), sd, mlp)
        got = OM.generate(pe, sd, 8, 2, 1e-5)
        ref = g[f"ids_{tag}"]
        for b in range(ref.shape[0]):
            assert got[b] == _strip(ref[b]), (tag, b)


def test_fp8_pack_tiles_layout():
    """zs_fp8_gemm_rows' weight layout (include/zsaac.h): block (split s, tile t, group w, k block j),
    lane l = W[128 t + 16 w + (l & 15)][1024 s + 64 j + 16 (l >> 4) .. +16], rows past N zero."""
    import torch
    from zsaac.mistral import fp8_pack_tiles
    N, K = 200, 2048
    q = torch.randint(0, 255, (N, K), dtype=torch.uint8, generator=torch.Generator().manual_seed(0))
    p = fp8_pack_tiles(q)
    NT = 2
    assert p.numel() == NT * 128 * K
    blk = p.view(K // 1024, NT, 8, 16, 64, 16)
    for n, k in [(0, 0), (17, 1000), (127, 1023), (128, 1024), (199, 2047), (250, 77)]:
        s, kk = divmod(k, 1024)
        j, r = divmod(kk, 64)
        g, b = divmod(r, 16)
        t, nn = divmod(n, 128)
        w, fr = divmod(nn, 16)
        assert int(blk[s, t, w, j, 16 * g + fr, b]) == (int(q[n, k]) if n < N else 0)


# The NF4 code (QLoRA, Dettmers et al. 2023, Appendix E; bitsandbytes functional.py's
# get_4bit_type("nf4")), as a bitsandbytes checkpoint stores it in ``weight.quant_map``.
NF4 = [-1.0, -0.6961928009986877, -0.5250730514526367, -0.39491748809814453,
       -0.28444138169288635, -0.18477343022823334, -0.09105003625154495, 0.0,
       0.07958029955625534, 0.16093020141124725, 0.24611230194568634, 0.33791524171829224,
       0.44070982933044434, 0.5626170039176941, 0.7229568362236023, 1.0]


def _bnb_nf4(w, blocksize=64, nested=True, nbs=256):
    """Hand-built bitsandbytes NF4 (+ double quant) entries for weight w: nearest NF4 code per
    element of each absmax-scaled block, packed two per byte (first element high nibble); absmax
    re-quantized to uint8 over a 256-entry code after subtracting its mean (nested_offset)."""
    import json
    flat = w.float().flatten()
    n = flat.numel()
    nb = (n + blocksize - 1) // blocksize
    pad = torch.zeros(nb * blocksize)
    pad[:n] = flat
    absmax = pad.view(nb, blocksize).abs().amax(1)
    scaled = pad.view(nb, blocksize) / absmax[:, None]
    code = torch.tensor(NF4)
    q = (scaled.flatten()[:n, None] - code[None]).abs().argmin(1)
    if n % 2:
        q = torch.cat([q, torch.zeros(1, dtype=torch.long)])
    packed = ((q[0::2] << 4) | q[1::2]).to(torch.uint8)[:, None]
    st = {"quant_type": "nf4", "blocksize": blocksize, "dtype": "bfloat16",
          "shape": list(w.shape)}
    sd = {"weight": packed, "weight.quant_map": code.clone()}
    if nested:
        off = float(absmax.mean())
        a = absmax - off
        nn_ = (a.numel() + nbs - 1) // nbs
        ap = torch.zeros(nn_ * nbs)
        ap[:a.numel()] = a
        namax = ap.view(nn_, nbs).abs().amax(1).clamp(min=1e-12)
        ncode = torch.linspace(-1, 1, 256)
        aq = ((ap.view(nn_, nbs) / namax[:, None]).flatten()[:a.numel(), None]
              - ncode[None]).abs().argmin(1).to(torch.uint8)
        sd.update({"weight.absmax": aq, "weight.nested_absmax": namax,
                   "weight.nested_quant_map": ncode})
        st.update({"nested_blocksize": nbs, "nested_offset": off, "nested_dtype": "float32"})
    else:
        sd["weight.absmax"] = absmax
    sd["weight.quant_state.bitsandbytes__nf4"] = torch.tensor(
        list(json.dumps(st).encode()), dtype=torch.uint8)
    return sd, q[:n], absmax


def test_bnb_nf4_nibble_order_and_blocks():
    """First element in the high nibble; one absmax per 64-element block."""
    from zsaac.mistral import dequantize_bnb_4bit
    import json
    st = {"quant_type": "nf4", "blocksize": 64, "dtype": "float16", "shape": [2, 64]}
    sd = {"w": torch.tensor([0x0F] * 32 + [0xF0] * 32, dtype=torch.uint8),
          "w.quant_map": torch.tensor(NF4), "w.absmax": torch.tensor([2.0, 0.5]),
          "w.quant_state.bitsandbytes__nf4": torch.tensor(list(json.dumps(st).encode()),
                                                          dtype=torch.uint8)}
    w = dequantize_bnb_4bit(sd, "w")
    assert w.shape == (2, 64)
    assert torch.equal(w[0, 0::2], torch.full((32,), -2.0))
    assert torch.equal(w[0, 1::2], torch.full((32,), 2.0))
    assert torch.equal(w[1, 0::2], torch.full((32,), 0.5))
    assert torch.equal(w[1, 1::2], torch.full((32,), -0.5))


def test_bnb_nf4_double_quant_dequant():
    from zsaac.mistral import dequantize_bnb_4bit
    g = torch.Generator().manual_seed(3)
    w = torch.randn(96, 200, generator=g) * 0.02
    for nested in (False, True):
        sd, q, absmax = _bnb_nf4(w, nested=nested)
        got = dequantize_bnb_4bit(sd, "weight")
        assert got.shape == w.shape
        exact = (torch.tensor(NF4)[q] * absmax.repeat_interleave(64)[:w.numel()]).view(w.shape)
        if nested:
            # absmax round-trips through the 256-entry code: relative error <= half a step
            assert torch.allclose(got, exact, rtol=2e-2, atol=1e-6)
        else:
            assert torch.equal(got, exact)
        # NF4 error bound: half the widest code gap times the block absmax
        assert (got - w).abs().max() <= 0.17 * float(absmax.max()) + 1e-6


def test_merge_peft_dequantizes_nf4_base():
    """merge_peft_state_dict on a 4-bit peft checkpoint: base dequantized, LoRA merged."""
    from zsaac.mistral import merge_peft_state_dict
    g = torch.Generator().manual_seed(4)
    W = torch.randn(64, 128, generator=g) * 0.05
    A = torch.randn(8, 128, generator=g) * 0.01
    B = torch.randn(64, 8, generator=g) * 0.01
    base = "LMmodel.base_model.model.model.layers.0.self_attn.q_proj"
    qsd, q, absmax = _bnb_nf4(W, nested=True)
    sd = {base + ".base_layer." + k: v for k, v in qsd.items()}
    sd[base + ".lora_A.default.weight"] = A
    sd[base + ".lora_B.default.weight"] = B
    sd["LMmodel.base_model.model.model.norm.weight"] = torch.ones(128)
    out = merge_peft_state_dict(sd, prefix="LMmodel.")
    assert set(out) == {"model.layers.0.self_attn.q_proj.weight", "model.norm.weight"}
    from zsaac.mistral import dequantize_bnb_4bit
    deq = dequantize_bnb_4bit(qsd, "weight")
    assert torch.allclose(out["model.layers.0.self_attn.q_proj.weight"], deq + 2.0 * (B @ A),
                          atol=1e-7)
