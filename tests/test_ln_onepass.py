"""CPU bound on the bf16 grid decode's ONE-pass LayerNorm statistics (decode_grid.hip ln_stats /
ln_row: sum x and sum x^2 of the bf16 row in f32, var = E[x^2] - mean^2) against the two-pass
form (mean, then the squared deviations), on rows with a large per-row mean offset -- the case
where the one-pass variance cancels.

The kernel sums each wave's K quarter (192 values) per lane group in f32 (v_dot2: bf16 pairs,
exact products, f32 accumulate), then adds the 4 lanes of a row and the 4 waves' partials; the
restatement below follows that order.  The bound: rstd's relative error stays below half a bf16
ulp (2^-9) -- the precision the normalised row is consumed at -- for |mean| / std up to 64
(measured: 2e-7 at 1, 2e-5 at 16, 3e-4 at 64, 1.3e-3 at 128); GPT-2's residual rows have
|mean| / std of order 0.1-1 (their large dims are a few outliers, which raise E[x^2] with the
variance).
"""
import numpy as np
import pytest


def _bf16(x):
    u = np.asarray(x, np.float32).view(np.uint32)
    u = ((u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000).astype(np.uint32)
    return u.view(np.float32)


def _one_pass_rstd(x):
    """x: bf16-valued f32 [768] -> rstd as the kernel computes it (f32 throughout)."""
    f = np.float32
    xq = x.reshape(4, 4, 6, 8)          # wave, lane group (l / 16), k-step, 8 elements
    s = np.zeros((4, 4), f)
    q = np.zeros((4, 4), f)
    for w in range(4):
        for g in range(4):
            for i in range(6):
                for e in range(0, 8, 2):      # v_dot2: two exact products, one f32 add
                    a, b = xq[w, g, i, e], xq[w, g, i, e + 1]
                    s[w, g] = f(s[w, g] + f(np.float64(a) + np.float64(b)))
                    q[w, g] = f(q[w, g] + f(np.float64(a) * a + np.float64(b) * b))
    sw = [f(f(s[w, 0] + s[w, 1]) + f(s[w, 2] + s[w, 3])) for w in range(4)]
    qw = [f(f(q[w, 0] + q[w, 1]) + f(q[w, 2] + q[w, 3])) for w in range(4)]
    mean = f(f(f(sw[0] + sw[1]) + f(sw[2] + sw[3])) * f(1.0 / 768))
    ex2 = f(f(f(qw[0] + qw[1]) + f(qw[2] + qw[3])) * f(1.0 / 768))
    var = max(f(ex2 - f(mean * mean)), f(0.0))
    return f(1.0) / np.sqrt(f(var + f(1e-5)))


@pytest.mark.parametrize("ratio", [0.0, 0.5, 2.0, 8.0, 16.0, 64.0])
def test_one_pass_rstd_within_half_bf16_ulp(ratio):
    rng = np.random.default_rng(int(ratio * 10) + 1)
    worst = 0.0
    for scale in (0.05, 1.0, 20.0):
        for _ in range(20):
            x = _bf16(rng.standard_normal(768).astype(np.float32) * scale
                      + np.float32(ratio * scale) * rng.choice([-1.0, 1.0]))
            xd = x.astype(np.float64)
            ref = 1.0 / np.sqrt(((xd - xd.mean()) ** 2).mean() + 1e-5)     # two-pass, f64
            worst = max(worst, abs(float(_one_pass_rstd(x)) / ref - 1.0))
    assert worst < 2.0 ** -9, f"|mean|/std = {ratio}: rstd relative error {worst:.2e}"
