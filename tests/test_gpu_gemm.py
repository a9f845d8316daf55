"""phc_twin_gemm (phc_gemm.hip): the half-precision MFMA GEMM with fused twin-trunk epilogues vs
plain PyTorch fp32 (needs an MI355X).

Tolerances: the STORE epilogue on small-integer operands is bit-exact (every product and partial
sum is an integer below 2^24, so fp32 accumulation in any order gives the same value; asymmetric
operands catch a transposed output).  The fused epilogues on random data are compared with the
fp32 product of the same half-precision operands followed by the torch ops: GEMM sums differ only
in fp32 summation order (rel. 2e-5), a half-precision output by one rounding (rel. 2^-10 f16).
"""

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _ints(shape, g, dtype, lo=-4, hi=5):
    return torch.randint(lo, hi, shape, device=DEV, generator=g).to(dtype)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("m,n,k,batch", [(300, 200, 192, 2), (256, 128, 64, 1), (1000, 69, 960, 1)])
def test_store_exact_integer_operands(dtype, m, n, k, batch):
    from puffer_phc_amd import _native as N

    g = torch.Generator(device=DEV).manual_seed(0)
    a = _ints((batch, m, k), g, dtype)
    b = _ints((batch, n, k), g, dtype, lo=-3, hi=7)  # asymmetric range
    out = torch.empty((batch, m, n), device=DEV)
    N.twin_gemm(a, b, N.EPI_STORE, out, (batch, n))
    ref = torch.bmm(a.float(), b.float().transpose(1, 2))
    assert torch.equal(out, ref)


def test_strided_operand_and_shared_a():
    """A row-strided view (lda > k, the zero-padded first layer) and an A shared by both batches."""
    from puffer_phc_amd import _native as N

    g = torch.Generator(device=DEV).manual_seed(1)
    base = _ints((200, 256), g, torch.float16)
    a = base[:, :192]
    b = _ints((2, 96, 192), g, torch.float16)
    out = torch.empty((2, 200, 96), device=DEV)
    N.twin_gemm(a, b, N.EPI_STORE, out, (2, 96))
    ref = torch.einsum("mk,bnk->bmn", a.float(), b.float())
    assert torch.equal(out, ref)


@pytest.mark.parametrize("pre_dtype", [torch.float32, torch.float16])
def test_bias_silu_split_to_grouped(pre_dtype):
    """Layer 1: one [m, k] x [2n, k]^T GEMM, pre kept SPLIT [m, 2n] (fp32, or f16 as autocast keeps
    it), silu written GROUPED [2, m, n] in f16 — the twin layout conversion of phc_bias_act_fwd,
    fused."""
    from puffer_phc_amd import _native as N

    g = torch.Generator(device=DEV).manual_seed(2)
    m, n, k = 333, 256, 128
    a = torch.randn((m, k), device=DEV, generator=g).half()
    w = (torch.randn((2 * n, k), device=DEV, generator=g) / k ** 0.5).half()
    bias = torch.randn(2 * n, device=DEV, generator=g)
    pre = torch.empty((m, 2 * n), device=DEV, dtype=pre_dtype)
    z = torch.empty((2, m, n), dtype=torch.float16, device=DEV)
    N.twin_gemm(a, w, N.EPI_BIAS_SILU, z, (2, n), bias=bias, aux=pre, aux_layout=N.SPLIT, out_layout=N.GROUPED)
    ref_pre = a.float() @ w.float().t() + bias
    if pre_dtype == torch.float32:
        torch.testing.assert_close(pre, ref_pre, rtol=2e-5, atol=2e-5)
    else:
        torch.testing.assert_close(pre.float(), ref_pre, rtol=2.0 ** -10, atol=2e-5)
    ref_z = torch.nn.functional.silu(ref_pre).view(m, 2, n).permute(1, 0, 2)
    torch.testing.assert_close(z.float(), ref_z, rtol=2.0 ** -10, atol=2e-5)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_bias_fp32_out_batched(dtype):
    from puffer_phc_amd import _native as N

    g = torch.Generator(device=DEV).manual_seed(3)
    m, n, k = 500, 192, 256
    a = torch.randn((2, m, k), device=DEV, generator=g).to(dtype)
    w = (torch.randn((2, n, k), device=DEV, generator=g) / k ** 0.5).to(dtype)
    bias = torch.randn(2 * n, device=DEV, generator=g)
    y = torch.empty((2, m, n), device=DEV)
    N.twin_gemm(a, w, N.EPI_BIAS, y, (2, n), bias=bias)
    ref = torch.bmm(a.float(), w.float().transpose(1, 2)) + bias.view(2, 1, n)
    torch.testing.assert_close(y, ref, rtol=2e-5, atol=2e-5)


@pytest.mark.parametrize("pre_dtype", [torch.float32, torch.float16])
@pytest.mark.parametrize("out_layout", [0, 1])
def test_silu_grad_and_bias_grad(out_layout, pre_dtype):
    """Input gradient of a SiLU layer: dz = g @ W (W pre-transposed to [k_in, n_out]), then
    dz * silu'(pre + b) rounded to f16, and the bias gradient from the fp32 products."""
    from puffer_phc_amd import _native as N

    g = torch.Generator(device=DEV).manual_seed(4)
    m, n_out, k_in = 777, 192, 256
    gr = torch.randn((2, m, n_out), device=DEV, generator=g).half()
    w = (torch.randn((2, n_out, k_in), device=DEV, generator=g) / n_out ** 0.5).half()
    wt = w.transpose(1, 2).contiguous()  # [2, k_in, n_out]
    pre_shape = (m, 2 * k_in) if out_layout == N.SPLIT else (2, m, k_in)
    pre = (torch.randn(pre_shape, device=DEV, generator=g) * 2).to(pre_dtype)
    pb = torch.randn(2 * k_in, device=DEV, generator=g)
    gout = torch.empty(pre_shape, dtype=torch.float16, device=DEV)
    db = torch.empty(2 * k_in, device=DEV)
    N.twin_gemm(gr, wt, N.EPI_SILU_GRAD, gout, (2, k_in), bias=pb, aux=pre, aux_layout=out_layout,
                out_layout=out_layout, bias_grad=db)

    def grouped(t):
        return t.view(m, 2, k_in).permute(1, 0, 2) if out_layout == N.SPLIT else t

    dz = torch.bmm(gr.float(), w.float())  # [2, m, k_in]
    p = (grouped(pre).float() + pb.view(2, 1, k_in)).clone().requires_grad_(True)
    torch.nn.functional.silu(p).backward(dz)
    torch.testing.assert_close(grouped(gout).float(), p.grad, rtol=2.0 ** -10, atol=1e-4)
    torch.testing.assert_close(db, p.grad.sum(1).reshape(-1), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("m", [777, 8192])  # 128 x 128 tiles; 256 x 256 tiles (>= 256 tiles)
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_relu_epilogues(dtype, m):
    """BIAS_RELU (the discriminator's Linear + ReLU) and RELU_GRAD (its backward from the ReLU
    output, bias-gradient column sums from the fp32 products) vs torch in fp32."""
    from puffer_phc_amd import _native as N

    g = torch.Generator(device=DEV).manual_seed(6)
    k, n = 512, 1024
    x = torch.randn((m, k), device=DEV, generator=g).to(dtype)
    w = (torch.randn((n, k), device=DEV, generator=g) / k ** 0.5).to(dtype)
    b = torch.randn(n, device=DEV, generator=g) * 0.3
    h = torch.empty((m, n), dtype=dtype, device=DEV)
    N.twin_gemm(x, w, N.EPI_BIAS_RELU, h, (1, n), bias=b)
    ref = torch.relu(x.float() @ w.float().t() + b)
    eps = 2.0 ** -8 if dtype == torch.float16 else 2.0 ** -5
    torch.testing.assert_close(h.float(), ref.to(dtype).float(), rtol=eps, atol=1e-3)
    assert 0.2 < float((h > 0).float().mean()) < 0.8
    # backward: gin = (gr @ W^T-layout) * [h > 0]; W given as [n_in=n, n_out] for gr [m, n_out]
    n_out = 256
    gr = torch.randn((m, n_out), device=DEV, generator=g).to(dtype)
    w2 = (torch.randn((n_out, n), device=DEV, generator=g) / n_out ** 0.5).to(dtype)
    w2t = w2.t().contiguous()  # [n, n_out]
    gin = torch.empty((m, n), dtype=dtype, device=DEV)
    db = torch.empty(n, device=DEV)
    N.twin_gemm(gr, w2t, N.EPI_RELU_GRAD, gin, (1, n), aux=h, bias_grad=db)
    full = (gr.float() @ w2.float()) * (h.float() > 0)
    torch.testing.assert_close(gin.float(), full.to(dtype).float(), rtol=eps, atol=1e-3)
    torch.testing.assert_close(db, full.sum(0), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("epi", ["bias_silu", "bias_f32", "silu_grad"])
def test_large_ragged_256_tiles(epi):
    """Shapes large enough for the 256 x 256 tile configuration (>= 512 tiles), with ragged rows
    (16500 = 64.45 tiles) and ragged columns (1000 = 3.9 tiles): masked rows / columns of the
    register epilogue, twin offsets across the batch."""
    from puffer_phc_amd import _native as N

    g = torch.Generator(device=DEV).manual_seed(7)
    m, n, k = 16500, 1000, 192
    a = torch.randn((2, m, k), device=DEV, generator=g).half()
    w = (torch.randn((2, n, k), device=DEV, generator=g) / k ** 0.5).half()
    b = torch.randn(2 * n, device=DEV, generator=g)
    y = torch.bmm(a.float(), w.float().transpose(1, 2))  # [2, m, n]
    if epi == "bias_f32":
        out = torch.empty((2, m, n), device=DEV)
        N.twin_gemm(a, w, N.EPI_BIAS, out, (2, n), bias=b)
        torch.testing.assert_close(out, y + b.view(2, 1, n), rtol=2e-5, atol=2e-5)
    elif epi == "bias_silu":
        out = torch.empty((2, m, n), dtype=torch.float16, device=DEV)
        pre = torch.empty((2, m, n), dtype=torch.float16, device=DEV)
        N.twin_gemm(a, w, N.EPI_BIAS_SILU, out, (2, n), bias=b, aux=pre)
        ref = y + b.view(2, 1, n)
        torch.testing.assert_close(pre.float(), ref, rtol=2.0 ** -10, atol=1e-4)
        torch.testing.assert_close(out.float(), torch.nn.functional.silu(ref), rtol=2.0 ** -10, atol=1e-4)
    else:
        pre = (torch.randn((2, m, n), device=DEV, generator=g) * 2).half()
        gout = torch.empty((2, m, n), dtype=torch.float16, device=DEV)
        db = torch.empty(2 * n, device=DEV)
        N.twin_gemm(a, w, N.EPI_SILU_GRAD, gout, (2, n), aux=pre, bias_grad=db)
        p = pre.float().clone().requires_grad_(True)
        torch.nn.functional.silu(p).backward(y)
        torch.testing.assert_close(gout.float(), p.grad, rtol=2.0 ** -10, atol=1e-4)
        torch.testing.assert_close(db, p.grad.sum(1).reshape(-1), rtol=1e-4, atol=2e-2)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("m,n,rows,batch,splits,shared_z", [
    (512, 256, 1024, 2, 4, False),    # whole 256 tiles, split-K
    (4096, 960, 2048, 1, 2, False),   # layer 1 as the trunk backward runs it: ragged 960 columns
    (200, 136, 640, 2, 5, True),      # ragged rows and columns of one tile, shared z, odd split
])
def test_weight_grad_exact_integer_operands(dtype, m, n, rows, batch, splits, shared_z):
    """phc_weight_grad: out[s][b] = g[b][rows_s]^T z[b][rows_s] on small-integer operands, bit-exact
    against fp32 torch (every partial sum is an integer below 2^24); asymmetric ranges catch a
    transposed fragment, the shared / ragged cases the column clamp of the transposed staging."""
    from puffer_phc_amd import _native as N

    gen = torch.Generator(device=DEV).manual_seed(11)
    g = _ints((batch, rows, m), gen, dtype)
    z = _ints((rows, n) if shared_z else (batch, rows, n), gen, dtype, lo=-3, hi=7)
    part = N.weight_grad(g, z, splits)
    zz = z.expand(batch, rows, n) if shared_z else z
    gs = g.float().view(batch, splits, rows // splits, m)
    zs = zz.float().reshape(batch, splits, rows // splits, n)
    ref = torch.einsum("bsrm,bsrn->sbmn", gs, zs)
    assert torch.equal(part, ref)


def test_weight_grad_random_strided():
    """A row-strided g (the SPLIT [rows, 2k] first-layer input gradient viewed per trunk) on
    random data: rel. 1e-5 of the fp32 product (summation order only)."""
    from puffer_phc_amd import _native as N

    gen = torch.Generator(device=DEV).manual_seed(12)
    rows = 4096
    gp = torch.randn((rows, 1024), device=DEV, generator=gen).half()
    x = torch.randn((rows, 320), device=DEV, generator=gen).half()
    part = N.weight_grad(gp[:, 512:], x, 4)
    ref = gp[:, 512:].float().t() @ x.float()
    torch.testing.assert_close(part.sum(0)[0], ref, rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_weight_grad_group_exact_integer_operands(dtype):
    """phc_weight_grad_group: three problems in one launch — a twin layer (batch 2), the first
    layer's SPLIT input gradient against a shared padded input (batch 1, rows split over two
    destinations, padded columns dropped) and a ragged single one — accumulated into existing
    destinations; bit-exact on small integers."""
    from puffer_phc_amd import _native as N

    gen = torch.Generator(device=DEV).manual_seed(13)
    rows = 1024
    g1, z1 = _ints((2, rows, 256), gen, dtype), _ints((2, rows, 512), gen, dtype, lo=-3, hi=7)
    gp, xc = _ints((rows, 2 * 128), gen, dtype), _ints((rows, 192), gen, dtype, lo=-3, hi=7)
    xc[:, 180:] = 0  # padding columns
    g3, z3 = _ints((1, rows, 72), gen, dtype), _ints((1, rows, 40), gen, dtype, lo=-3, hi=7)
    d1 = [torch.randint(-50, 50, (256, 512), device=DEV, generator=gen).float() for _ in range(2)]
    d2 = [torch.randint(-50, 50, (128, 180), device=DEV, generator=gen).float() for _ in range(2)]
    d3 = [torch.zeros((72, 40), device=DEV)]
    e1 = [d + (g1[b].float().t() @ z1[b].float()) for b, d in enumerate(d1)]
    full2 = gp.float().t() @ xc.float()[:, :180]
    e2 = [d2[0] + full2[:128], d2[1] + full2[128:]]
    e3 = [g3[0].float().t() @ z3[0].float()]
    N.weight_grad_group([(g1, z1, d1, 256, 512), (gp, xc, d2, 128, 180), (g3, z3, d3, 72, 40)], accumulate=True)
    for got, exp in zip(d1 + d2 + d3, e1 + e2 + e3):
        assert torch.equal(got, exp)


def test_rejects_unpadded_k():
    from puffer_phc_amd import _native as N

    a = torch.zeros((64, 934), dtype=torch.float16, device=DEV)
    b = torch.zeros((64, 934), dtype=torch.float16, device=DEV)
    out = torch.empty((64, 64), device=DEV)
    with pytest.raises(RuntimeError, match="multiple of 64"):
        N.twin_gemm(a, b, N.EPI_STORE, out, (1, 64))


@pytest.mark.parametrize("epi", ["bias_silu", "silu_grad"])
@pytest.mark.parametrize("max_wg", [7, 100, 256])
def test_persistent_grid_matches_one_tile_per_workgroup(epi, max_wg):
    """max_workgroups: a persistent grid looping over the tiles gives the one-tile-per-workgroup
    result bit for bit (256 x 256 tiles, several tiles per workgroup, a ragged last step).  This
    is the case that exposed LDS-DMA reads racing other waves' DMA when the K-step barrier relied
    on __syncthreads (phc_gemm.hip dma_barrier)."""
    from puffer_phc_amd import _native as N

    g = torch.Generator(device=DEV).manual_seed(9)
    m, n, k = 8192 + 77, 512, 1024
    a = torch.randn((2, m, k), device=DEV, generator=g).half()
    w = (torch.randn((2, n, k), device=DEV, generator=g) / k ** 0.5).half()
    bias = torch.randn(2 * n, device=DEV, generator=g)
    outs = []
    for mwg in (0, max_wg):
        out = torch.empty((2, m, n), dtype=torch.float16, device=DEV)
        if epi == "bias_silu":
            aux = torch.empty((2, m, n), dtype=torch.float16, device=DEV)
            N.twin_gemm(a, w, N.EPI_BIAS_SILU, out, (2, n), bias=bias, aux=aux, max_workgroups=mwg)
            outs.append((out, aux))
        else:
            aux = (torch.randn((2, m, n), device=DEV, generator=torch.Generator(device=DEV).manual_seed(5)) * 2).half()
            db = torch.empty(2 * n, device=DEV)
            N.twin_gemm(a, w, N.EPI_SILU_GRAD, out, (2, n), bias=bias, aux=aux, bias_grad=db, max_workgroups=mwg)
            outs.append((out, db))
    torch.testing.assert_close(outs[1][0], outs[0][0], rtol=0, atol=0)
    torch.testing.assert_close(outs[1][1], outs[0][1], rtol=0, atol=0)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("epi", ["store", "bias_f32", "bias_silu", "bias_silu_noaux", "bias_relu", "bias_silu_d"])
@pytest.mark.parametrize("shape", [(4160, 700), (4352, 768)])
def test_wave_specialised_persistent_matches_one_tile(dtype, epi, shape):
    """The forward epilogues run wave-specialised in a persistent grid (kWsTile: waves 0-3 issue the
    operand DMA and stage the bias row, waves 4-7 store; the default for the training GEMMs, which
    have more 256 x 256 tiles than CUs) and must equal the one-tile-per-workgroup kernel bit for bit:
    every epilogue, both operand types, whole and ragged tiles (rows 4160 = 16.25 tiles, columns 700),
    fp32 and half outputs, with and without the pre-activation (or its derivative, BIAS_SILU_D); whole
    tiles only (4352 x 768) as well."""
    from puffer_phc_amd import _native as N

    g = torch.Generator(device=DEV).manual_seed(11)
    (m, n), k = shape, 448
    a = torch.randn((2, m, k), device=DEV, generator=g).to(dtype)
    w = (torch.randn((2, n, k), device=DEV, generator=g) / k ** 0.5).to(dtype)
    bias = torch.randn(2 * n, device=DEV, generator=g)
    ep = {"store": N.EPI_STORE, "bias_f32": N.EPI_BIAS, "bias_silu": N.EPI_BIAS_SILU,
          "bias_silu_noaux": N.EPI_BIAS_SILU, "bias_relu": N.EPI_BIAS_RELU, "bias_silu_d": N.EPI_BIAS_SILU_D}[epi]
    odt = torch.float32 if epi == "bias_f32" else dtype
    outs = []
    for mwg in (0, 37):  # 37 workgroups: 48 tiles each loop over several (and a ragged last step)
        out = torch.full((2, m, n), 7.0, dtype=odt, device=DEV)
        aux = torch.full((2, m, n), 7.0, dtype=dtype, device=DEV) if epi in ("bias_silu", "bias_silu_d") else None
        N.twin_gemm(a, w, ep, out, (2, n), bias=None if epi == "store" else bias, aux=aux, max_workgroups=mwg)
        outs.append((out, aux))
    assert torch.equal(outs[1][0], outs[0][0])
    if outs[0][1] is not None:
        assert torch.equal(outs[1][1], outs[0][1])
    ref = torch.bmm(a.float(), w.float().transpose(1, 2)) + (0 if epi == "store" else bias.view(2, 1, n))
    if epi == "bias_silu_d":
        s = torch.sigmoid(ref)
        torch.testing.assert_close(outs[0][1].float(), s * (1 + ref * (1 - s)), rtol=2.0 ** -7, atol=2e-3)
    elif epi == "bias_silu":
        torch.testing.assert_close(outs[0][1].float(), ref, rtol=2.0 ** -7, atol=2e-3)
    if epi in ("bias_silu", "bias_silu_noaux", "bias_silu_d"):
        ref = torch.nn.functional.silu(ref)
    elif epi == "bias_relu":
        ref = torch.relu(ref)
    eps = 2.0 ** -8 if dtype == torch.float16 else 2.0 ** -5
    torch.testing.assert_close(outs[0][0].float(), ref, rtol=eps if odt != torch.float32 else 2e-5, atol=2e-3)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("m", [777, 16500])  # 128 x 128 tiles; 256 x 256 tiles (wave-specialised forward grid)
def test_silu_deriv_aux_pair(dtype, m):
    """PHC_EPI_BIAS_SILU_D stores silu'(pre) (s (1 + z (1 - s))) as the aux and the same activation as
    BIAS_SILU (bit for bit); PHC_EPI_DSILU_GRAD multiplies the input gradient by that aux and gives
    SILU_GRAD's result (from the pre-activation) within the aux's rounding, bias-gradient sums too."""
    from puffer_phc_amd import _native as N

    g = torch.Generator(device=DEV).manual_seed(12)
    k, n, nout = 192, 1000, 256
    a = torch.randn((2, m, k), device=DEV, generator=g).to(dtype)
    w = (torch.randn((2, n, k), device=DEV, generator=g) / k ** 0.5).to(dtype)
    b = torch.randn(2 * n, device=DEV, generator=g)
    y0, pre = torch.empty((2, m, n), dtype=dtype, device=DEV), torch.empty((2, m, n), dtype=dtype, device=DEV)
    y1, dsl = torch.empty((2, m, n), dtype=dtype, device=DEV), torch.empty((2, m, n), dtype=dtype, device=DEV)
    N.twin_gemm(a, w, N.EPI_BIAS_SILU, y0, (2, n), bias=b, aux=pre)
    N.twin_gemm(a, w, N.EPI_BIAS_SILU_D, y1, (2, n), bias=b, aux=dsl)
    assert torch.equal(y0, y1)
    z = torch.bmm(a.float(), w.float().transpose(1, 2)) + b.view(2, 1, n)
    s = torch.sigmoid(z)
    eps = 2.0 ** -10 if dtype == torch.float16 else 2.0 ** -7
    torch.testing.assert_close(dsl.float(), s * (1 + z * (1 - s)), rtol=eps, atol=2e-3)
    # backward: gp = (gout @ W) * silu'(z); W given as [n_in = n, n_out] for gout [2, m, n_out]
    gout = (torch.randn((2, m, nout), device=DEV, generator=g) * 0.5).to(dtype)
    wt = (torch.randn((2, n, nout), device=DEV, generator=g) / nout ** 0.5).to(dtype)
    gp0, gp1 = torch.empty((2, m, n), dtype=dtype, device=DEV), torch.empty((2, m, n), dtype=dtype, device=DEV)
    db0, db1 = torch.empty(2 * n, device=DEV), torch.empty(2 * n, device=DEV)
    N.twin_gemm(gout, wt, N.EPI_SILU_GRAD, gp0, (2, n), aux=pre, bias_grad=db0)
    N.twin_gemm(gout, wt, N.EPI_DSILU_GRAD, gp1, (2, n), aux=dsl, bias_grad=db1)
    full = torch.bmm(gout.float(), wt.float().transpose(1, 2)) * (s * (1 + z * (1 - s)))
    tol = 2.0 ** -8 if dtype == torch.float16 else 2.0 ** -5
    torch.testing.assert_close(gp1.float(), full, rtol=tol, atol=5e-3)
    torch.testing.assert_close(gp1.float(), gp0.float(), rtol=tol, atol=5e-3)
    torch.testing.assert_close(db1, full.sum(1).reshape(-1), rtol=2e-2, atol=0.5)
    with pytest.raises(RuntimeError):  # the derivative aux already holds the bias
        N.twin_gemm(gout, wt, N.EPI_DSILU_GRAD, gp1, (2, n), bias=b, aux=dsl)
