"""MX-FP8 path (BASELINE config 5, GPU only): the block-scaled MFMA's operand/scale layout, the quantiser (bit-exact
against the host reference `tests/mx_ref.py`), the fp8 GEMM epilogues and the AdaLN -> MX producer."""
import pytest
import torch
import torch.nn.functional as F

from tests import mx_ref as R

pytestmark = pytest.mark.gpu
dev = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from videopainter_amd import _native
    _native.lib()


def rel(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


def e4m3(x):
    return x.to(torch.float8_e4m3fn).view(torch.uint8)


def test_mx_mfma_probe_layout():
    """Exact small-multiple operands and random per-lane E8M0 scales: lane l supplies the scale of row l % 16 and
    K-block l // 16, for both operands; C = A_deq @ B_deq^T exactly (all products and sums exact in fp32)."""
    from videopainter_amd import _native as NV
    if not NV.has_diag():  # a hardware layout self-test: the diagnostic library only (include/vp_hip_diag.h)
        pytest.skip("diagnostic entry point: run with VP_HIP_LIB=videopainter_amd/_lib/libvp_hip_diag.so")
    from videopainter_amd import kernels as K
    g = torch.Generator().manual_seed(0)
    A = torch.randint(-8, 9, (16, 128), generator=g).float() / 4
    B = torch.randint(-8, 9, (16, 128), generator=g).float() / 4
    B[:, 0] += torch.arange(16).float() / 4  # asymmetric
    sa = torch.randint(124, 131, (64,), generator=g).to(torch.uint8)
    sb = torch.randint(124, 131, (64,), generator=g).to(torch.uint8)
    C = K.mx_mfma_probe(e4m3(A).to(dev), e4m3(B).to(dev), sa.to(dev), sb.to(dev)).cpu().double()
    scA = 2.0 ** (sa.double().view(4, 16).T - 127)  # [row, block]
    scB = 2.0 ** (sb.double().view(4, 16).T - 127)
    Ad = (A.double().view(16, 4, 32) * scA[:, :, None]).view(16, 128)
    Bd = (B.double().view(16, 4, 32) * scB[:, :, None]).view(16, 128)
    assert torch.equal(C, Ad @ Bd.T)


def _mixed(rows, Kk, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(rows, Kk, generator=g)
    mag = 10.0 ** torch.empty(rows, Kk // 32).uniform_(-3, 3, generator=g)
    x = x * mag.repeat_interleave(32, dim=1)
    x[0, :32] = 0.0                      # all-zero block
    x[1, :32] = 0.0
    x[1, 5] = 448.0                      # amax exactly 448 * 2^0
    x[2, 32:64] = 1e-38                  # subnormal-ratio block
    return x.to(torch.bfloat16)


def test_mx_quantize_bit_exact():
    from videopainter_amd import kernels as K
    x = _mixed(300, 384, 1)
    m = K.mx_quantize(x.to(dev))
    q_ref, s_ref = R.quantize(x)
    assert torch.equal(m.q[:300].cpu(), q_ref)
    assert torch.equal(m.scales.cpu(), s_ref)
    # dequantised error is bounded by half an e4m3 ulp of the block scale
    err = (R.dequantize(m.q, m.scales, 300, 384) - x.float()).abs()
    assert float(err.max()) <= float(x.float().abs().max()) * 2 ** -4


@pytest.fixture(params=["5", "13"], ids=["gemm8_v5", "gemm8_v13"])
def gemm8_variant(request, knobs):
    """fp8 GEMM main loop: 13 (default: the bf16 default's staggered read-first pipeline) or 5 (VP_GEMM8_VARIANT)."""
    knobs.setenv("VP_GEMM8_VARIANT", request.param)
    return request.param


@pytest.mark.parametrize("M,Nn,Kk", [(300, 512, 256), (700, 768, 384), (513, 256, 3072), (256, 512, 1536)])
def test_gemm_mx_bias(M, Nn, Kk, gemm8_variant):
    """fp8 GEMM against the fp64 product of the dequantised operands (the only error left is fp32 accumulation and
    the bf16 output rounding); short K runs the pipeline's tail only, K >= 640 its steady state."""
    from videopainter_amd import kernels as K
    g = torch.Generator().manual_seed(M + Kk)
    a = (torch.randn(M, Kk, generator=g)).to(torch.bfloat16)
    w = (torch.randn(Nn, Kk, generator=g) * Kk ** -0.5).to(torch.bfloat16)
    b = (torch.randn(Nn, generator=g) * 0.1).to(torch.bfloat16)
    A, W = K.mx_quantize(a.to(dev)), K.mx_quantize(w.to(dev))
    out = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
    K.gemm_mx(A, [W], [b.to(dev)], out)
    ref = R.dequantize(A.q, A.scales, M, Kk).double() @ R.dequantize(W.q, W.scales, Nn, Kk).double().T + b.double()
    assert rel(out, ref) < 4e-3
    # and against the un-quantised bf16 product: the fp8 error band (e4m3 has a 3-bit mantissa)
    assert rel(out, a.double() @ w.double().T + b.double()) < 6e-2


def test_gemm_mx_main_loops_bit_identical(knobs):
    """The two fp8 main loops run the same MFMAs in the same order per accumulator: bit-identical outputs."""
    from videopainter_amd import kernels as K
    g = torch.Generator().manual_seed(5)
    M, Nn, Kk = 1000, 768, 2048
    a = torch.randn(M, Kk, generator=g).to(torch.bfloat16)
    w = (torch.randn(Nn, Kk, generator=g) * Kk ** -0.5).to(torch.bfloat16)
    A, W = K.mx_quantize(a.to(dev)), K.mx_quantize(w.to(dev))
    outs = []
    for v in ("5", "13"):
        knobs.setenv("VP_GEMM8_VARIANT", v)
        out = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
        K.gemm_mx(A, [W], [None], out)
        outs.append(out)
    assert torch.equal(outs[0], outs[1])


def test_gemm_mx_gelu_to_mx_and_gated(gemm8_variant):
    """FF1 (bias + GELU-tanh, output re-quantised to MX in the epilogue) feeding FF2 (gated residual + masked branch
    injection), the fp8 FeedForward of the block."""
    from videopainter_amd import kernels as K
    from videopainter_amd import _native as N
    Bt, T, Nv, D, FF = 2, 10, 246, 256, 1024
    Ntok = T + Nv
    M = Bt * Ntok
    g = torch.Generator().manual_seed(7)
    x = torch.randn(M, D, generator=g).to(torch.bfloat16)
    w1 = (torch.randn(FF, D, generator=g) * D ** -0.5).to(torch.bfloat16)
    b1 = (torch.randn(FF, generator=g) * 0.1).to(torch.bfloat16)
    w2 = (torch.randn(D, FF, generator=g) * FF ** -0.5).to(torch.bfloat16)
    b2 = (torch.randn(D, generator=g) * 0.1).to(torch.bfloat16)
    X, W1, W2 = (K.mx_quantize(t.to(dev)) for t in (x, w1, w2))
    H = K.MXTensor(M, FF, dev)
    K.gemm_mx(X, [W1], [b1.to(dev)], H, epilogue=N.EPI_BIAS_GELU_MXFP8)
    h_ref = F.gelu(R.dequantize(X.q, X.scales, M, D).double() @ R.dequantize(W1.q, W1.scales, FF, D).double().T
                   + b1.double(), approximate="tanh")
    h = R.dequantize(H.q, H.scales, M, FF)
    assert rel(h, h_ref) < 4e-2
    resid = torch.randn(Bt, Ntok, D, generator=g).to(torch.bfloat16)
    mod = (torch.randn(Bt, 6 * D, generator=g) * 0.5).to(torch.bfloat16)
    inj = torch.randn(Bt, Nv, D, generator=g).to(torch.bfloat16)
    tm = (torch.rand(Bt, Nv, generator=g) > 0.5).to(torch.uint8)
    out = torch.empty(Bt, Ntok, D, device=dev, dtype=torch.bfloat16)
    injd = inj.to(dev)
    K.gemm_mx(H, [W2], [b2.to(dev)], out.view(M, D), epilogue=N.EPI_GATED, resid=resid.to(dev).view(M, D),
              mod=mod.to(dev), tokens_per_batch=Ntok, text_len=T, inject=injd, inject_mask=tm.to(dev))
    y = (h.double() @ R.dequantize(W2.q, W2.scales, D, FF).double().T + b2.double()).view(Bt, Ntok, D)
    ref = resid.double().clone()
    ref[:, :T] += mod.double()[:, None, 5 * D:6 * D] * y[:, :T]
    ref[:, T:] += mod.double()[:, None, 2 * D:3 * D] * y[:, T:]
    ref[:, T:] += inj.double() * (tm[..., None] == 0)
    assert rel(out, ref) < 6e-3


def test_adaln_modulate_mx_matches_quantised_bf16_path():
    """The MX producer quantises exactly the values the bf16 AdaLN kernel writes (byte-identical to quantising them
    on the host)."""
    from videopainter_amd import kernels as K
    Bt, T, Nv, D = 2, 7, 121, 3072
    g = torch.Generator().manual_seed(9)
    x = (torch.randn(Bt, T + Nv, D, generator=g) * 3 + 1).to(torch.bfloat16).to(dev)
    lw = (1 + 0.1 * torch.randn(D, generator=g)).to(torch.bfloat16).to(dev)
    lb = (0.1 * torch.randn(D, generator=g)).to(torch.bfloat16).to(dev)
    mod = (torch.randn(Bt, 6 * D, generator=g) * 0.5).to(torch.bfloat16).to(dev)
    y16 = K.adaln_modulate(x, lw, lb, mod, T, 1e-5)
    yq = K.adaln_modulate_mx(x, lw, lb, mod, T, 1e-5)
    q_ref, s_ref = R.quantize(y16.view(-1, D))
    assert torch.equal(yq.q[:Bt * (T + Nv)].cpu(), q_ref)
    assert torch.equal(yq.scales.cpu(), s_ref)
