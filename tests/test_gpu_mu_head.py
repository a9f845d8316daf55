"""phc_mu_head_fwd / _dgrad / _wgrad (phc_head.hip): the actor's fp32 mu head on the fp32-input
MFMA vs float64 torch (needs an MI355X).  Reference: policies/phc_policy.py:40-61 (nn.Linear(512,
num_actions) in fp32) and its autograd (clean_pufferl/core.py:298-354).

Forward and input gradient run on the bf16-x3 kernels (k_head_fwd_x3 / k_head_dgrad_x3: each fp32
operand split exactly into three bf16 parts, the six products above 2^-16 of hi*hi accumulated in
fp32, the dropped ones below 2^-23 of |x||w|); H = 256 / 512 / 1024 take that path.  The weight
gradient is on the fp32-input MFMA (exact products).  Both are fp32-class (the reference's own
mu head runs TF32, 2^-11, under set_float32_matmul_precision("high")), so one bound serves both:
the error against float64 is a few ulps of the row's absolute sum, |err| <= 2e-6 * sum |terms|."""

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _check(out, ref, scale):
    err = (out.double() - ref).abs()
    assert (err <= 2e-6 * scale + 1e-30).all(), f"max err {err.max().item():.3g}, max scale {scale.max().item():.3g}"


@pytest.mark.parametrize("M,H,A", [(32768, 512, 69), (1000, 512, 69), (77, 256, 1), (300, 512, 80), (129, 1024, 17)])
def test_mu_head_fwd_dgrad(M, H, A):
    from puffer_phc_amd import _native as N

    g = torch.Generator(device=DEV).manual_seed(M + A)
    h = torch.randn((M, H), device=DEV, generator=g)
    w = torch.randn((A, H), device=DEV, generator=g) / H ** 0.5
    b = torch.randn(A, device=DEV, generator=g)
    mu = N.mu_head_fwd(h, w, b)
    ref = h.double() @ w.double().t() + b.double()
    _check(mu, ref, h.double().abs() @ w.double().abs().t() + b.double().abs())
    dmu = torch.randn((M, A), device=DEV, generator=g)
    dh = N.mu_head_dgrad(dmu, w)
    _check(dh, dmu.double() @ w.double(), dmu.double().abs() @ w.double().abs())


@pytest.mark.parametrize("splits", [1, 7, 128])
@pytest.mark.parametrize("M,H,A", [(32768, 512, 69), (1001, 512, 69), (64, 256, 3)])
def test_mu_head_wgrad(M, H, A, splits):
    from puffer_phc_amd import _native as N

    g = torch.Generator(device=DEV).manual_seed(splits + M)
    h = torch.randn((M, H), device=DEV, generator=g)
    dmu = torch.randn((M, A), device=DEV, generator=g)
    part = N.mu_head_wgrad_parts(dmu, h, splits)
    assert part.shape == (min(splits, M), A, H)
    ref = dmu.double().t() @ h.double()
    _check(part.double().sum(0), ref, dmu.double().abs().t() @ h.double().abs())


def test_mu_head_rejects_bad_shapes():
    from puffer_phc_amd import _native as N

    h = torch.randn((16, 512), device=DEV)
    with pytest.raises(RuntimeError):
        N.mu_head_fwd(h, torch.randn((81, 512), device=DEV), torch.zeros(81, device=DEV))
