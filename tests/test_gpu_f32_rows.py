"""GPU: the f32 row-group decode GEMMs (csrc/gemm_rows.hip gemm_rows_f32_kernel) against a
torch fp32 reference of the same op -- zs_gemm_ln_f32 (LayerNorm with its affine in f32, then
the product, bias, gelu_new / residual) and its no-LayerNorm form (the projections) -- at the GPT-2 decode
shapes and ragged row counts.  Tolerance: exact f32 products with a different summation order
than torch's, |err| <= 2e-5 * max|ref| + 1e-5."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _tol(ref):
    return 2e-5 * float(ref.abs().max()) + 1e-5


@pytest.mark.parametrize("M,N,K,act", [(64, 2304, 768, 0), (64, 3072, 768, "gelu"), (7, 3072, 768, "gelu"),
                                       (33, 1000, 1024, 0), (1, 2304, 768, 0)])
def test_gemm_ln_f32(cuda, M, N, K, act):
    from zsaac import ops
    g = torch.Generator().manual_seed(M * 7 + N)
    x = (torch.randn(M, K, generator=g) * 3 + 0.5).to(cuda)
    lw = (1 + 0.1 * torch.randn(K, generator=g)).to(cuda)
    lb = (0.1 * torch.randn(K, generator=g)).to(cuda)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(cuda)
    b = (0.1 * torch.randn(N, generator=g)).to(cuda)
    out = torch.empty(M, N, device=cuda)
    a = ops.ACT_GELU_TANH if act == "gelu" else ops.ACT_NONE
    ops.gemm_ln_f32(x, lw, lb, w, out, bias=b, act=a)
    ref = torch.nn.functional.layer_norm(x.double(), (K,), lw.double(), lb.double(), 1e-5) @ w.double().t() + b.double()
    if act == "gelu":
        ref = torch.nn.functional.gelu(ref, approximate="tanh")
    assert float((out.double() - ref).abs().max()) <= _tol(ref)


@pytest.mark.parametrize("M,N,K", [(64, 768, 768), (64, 768, 3072), (21, 768, 3072), (5, 640, 1024)])
def test_gemm_rows_f32_residual(cuda, M, N, K):
    from zsaac import ops
    g = torch.Generator().manual_seed(M + N + K)
    a = torch.randn(M, K, generator=g).to(cuda)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(cuda)
    b = torch.randn(N, generator=g).to(cuda)
    x = torch.randn(M, N, generator=g).to(cuda)
    ref = a.double() @ w.double().t() + b.double() + x.double()
    ops.gemm_ln_f32(a, None, None, w, x, bias=b, residual=x)
    assert float((x.double() - ref).abs().max()) <= _tol(ref)
