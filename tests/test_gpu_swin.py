"""Fused Swin block (zs_swin_block, csrc/swin.hip) against the oracle's SwinTransformerBlock
(oracle/audio.py swin_block, restating htsat.py:427-474) and against the unfused HIP op sequence
(LayerNorm -> qkv GEMM -> window attention -> proj GEMM -> LayerNorm -> fc1 -> fc2).

Tolerances (bf16 operands, f32 accumulation and residual stream): vs the fp32 oracle with the same
bf16-valued weights, max |err| <= 2e-2 * max|ref| on the block's update (x_out - x_in); vs the
unfused HIP path (same rounding points, different summation order) 1e-2."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _block_sd(C, heads, seed, dev):
    g = torch.Generator().manual_seed(seed)

    def r(*s, scale=1.0):
        # bf16-representable values: the fused kernel and the oracle see identical weights
        return (torch.randn(*s, generator=g) * scale).to(torch.bfloat16).float()

    n = "blk."
    sd = {
        n + "norm1.weight": 1 + 0.1 * torch.randn(C, generator=g), n + "norm1.bias": 0.1 * torch.randn(C, generator=g),
        n + "attn.qkv.weight": r(3 * C, C, scale=C ** -0.5), n + "attn.qkv.bias": 0.1 * torch.randn(3 * C, generator=g),
        n + "attn.relative_position_bias_table": torch.randn(225, heads, generator=g),
        n + "attn.proj.weight": r(C, C, scale=C ** -0.5), n + "attn.proj.bias": 0.1 * torch.randn(C, generator=g),
        n + "norm2.weight": 1 + 0.1 * torch.randn(C, generator=g), n + "norm2.bias": 0.1 * torch.randn(C, generator=g),
        n + "mlp.fc1.weight": r(4 * C, C, scale=C ** -0.5), n + "mlp.fc1.bias": 0.1 * torch.randn(4 * C, generator=g),
        n + "mlp.fc2.weight": r(C, 4 * C, scale=(4 * C) ** -0.5), n + "mlp.fc2.bias": 0.1 * torch.randn(C, generator=g),
    }
    return sd


def _kernel_blk(sd, C, dev):
    from zsaac.encoder import pack_frags, pack_qkv
    n = "blk."
    f = lambda k: sd[n + k].to(dev).float().contiguous()
    bf = lambda k: sd[n + k].to(dev).to(torch.bfloat16).contiguous()
    blk = {"n1": (f("norm1.weight"), f("norm1.bias")), "qkv_w": bf("attn.qkv.weight"),
           "qkv_b": f("attn.qkv.bias"), "rel": f("attn.relative_position_bias_table"),
           "proj_w": bf("attn.proj.weight"), "proj_b": f("attn.proj.bias"),
           "n2": (f("norm2.weight"), f("norm2.bias")), "fc1_w": bf("mlp.fc1.weight"),
           "fc1_b": f("mlp.fc1.bias"), "fc2_w": bf("mlp.fc2.weight"), "fc2_b": f("mlp.fc2.bias")}
    blk["qkv_p"], blk["qkv_bp"] = pack_qkv(blk["qkv_w"], blk["qkv_b"], C)
    blk["proj_p"] = pack_frags(blk["proj_w"])
    blk["fc1_p"] = pack_frags(blk["fc1_w"])
    blk["fc2_p"] = pack_frags(blk["fc2_w"])
    return blk


def _unfused(x, B, res, C, heads, shift, blk):
    from zsaac import ops
    M = x.shape[0]
    dev = x.device
    h = torch.empty(M, C, device=dev, dtype=torch.bfloat16)
    qkv = torch.empty(M, 3 * C, device=dev, dtype=torch.bfloat16)
    att = torch.empty(M, C, device=dev, dtype=torch.bfloat16)
    hid = torch.empty(M, 4 * C, device=dev, dtype=torch.bfloat16)
    ops.layernorm(x, *blk["n1"], out=h)
    ops.gemm(h, blk["qkv_w"], qkv, bias=blk["qkv_b"])
    ops.window_attention(qkv, B, res, res, C, heads, shift, blk["rel"], att)
    ops.gemm(att, blk["proj_w"], x, bias=blk["proj_b"], residual=x)
    ops.layernorm(x, *blk["n2"], out=h)
    ops.gemm(h, blk["fc1_w"], hid, bias=blk["fc1_b"], act=ops.ACT_GELU_ERF)
    ops.gemm(hid, blk["fc2_w"], x, bias=blk["fc2_b"], residual=x)
    return x


@pytest.mark.parametrize("C,res,B", [(96, 64, 2), (192, 32, 3), (384, 16, 2), (96, 16, 1)])
@pytest.mark.parametrize("shift", [0, 4])
def test_swin_block_fused(cuda, C, res, B, shift):
    from oracle import audio as A
    from zsaac import ops
    heads = C // 24
    sd = _block_sd(C, heads, seed=C + shift, dev=cuda)
    blk = _kernel_blk(sd, C, cuda)
    g = torch.Generator().manual_seed(7 + C)
    x0 = torch.randn(B, res * res, C, generator=g)
    ref = A.swin_block(x0, sd, "blk.", res, res, heads, shift)
    x = x0.reshape(-1, C).to(cuda).contiguous()
    ops.swin_block(x, B, res, res, C, heads, shift, blk)
    xu = _unfused(x0.reshape(-1, C).to(cuda).contiguous(), B, res, C, heads, shift, blk)
    torch.cuda.synchronize()
    upd_ref = (ref - x0).reshape(-1, C)
    upd = x.cpu() - x0.reshape(-1, C)
    upd_u = xu.cpu() - x0.reshape(-1, C)
    scale = float(upd_ref.abs().max())
    err = float((upd - upd_ref).abs().max()) / scale
    err_u = float((upd_u - upd_ref).abs().max()) / scale
    err_fu = float((upd - upd_u).abs().max()) / scale
    assert err < 2e-2, (err, err_u)
    assert err_fu < 1e-2, (err_fu, err, err_u)
    assert torch.isfinite(x).all()


def test_htsat_fused_matches_unfused(cuda, monkeypatch):
    """Whole HTSAT encoder, fused Swin blocks vs the unfused op sequence (same packed weights)."""
    from zsaac import synthetic as S
    from zsaac import encoder as E
    sd = S.htsat_state_dict(3)
    sd.update(S.audio_proj_state_dict(5))
    wav = S.synthetic_waveforms(3).to(cuda)
    monkeypatch.setattr(E, "FUSED_SWIN_C", (96, 192, 384))
    ef = E.AudioEncoder(sd, "htsat", torch.bfloat16, 4, cuda)
    monkeypatch.setattr(E, "FUSED_SWIN_C", ())
    eu = E.AudioEncoder(sd, "htsat", torch.bfloat16, 4, cuda)
    assert "qkv_p" in ef.w.blocks[0][0] and "qkv_p" not in eu.w.blocks[0][0]
    a = ef.encode(wav).clone()
    b = eu.encode(wav).clone()
    cos = torch.nn.functional.cosine_similarity(a, b, dim=-1)
    assert float(cos.min()) > 0.999, cos


def test_htsat_encode_graphed_bit_identical(cuda):
    """Encoder.encode_graphed (the concurrent runner's up-front passes: everything after the
    log-mel front end replayed from a per-size hipGraph captured on a side stream) gives exactly
    encode()'s embeddings, at two batch sizes and on a second replay."""
    from zsaac import synthetic as S
    from zsaac import encoder as E
    sd = S.htsat_state_dict(3)
    sd.update(S.audio_proj_state_dict(5))
    wav = S.synthetic_waveforms(4).to(cuda)
    enc = E.AudioEncoder(sd, "htsat", torch.bfloat16, 4, cuda)
    ref = {B: enc.encode(wav[:B]).clone() for B in (4, 3)}
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        got = [(B, enc.encode_graphed(wav[:B]).clone()) for B in (4, 3, 4, 3)]
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    for B, e in got:
        assert torch.equal(e, ref[B]), B
