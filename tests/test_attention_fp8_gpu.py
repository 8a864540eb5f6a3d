"""fp8 attention (BASELINE config 5, GPU only): the 32x32x64 block-scaled MFMA layout, the e4m3 producers (qk-norm +
RoPE, V^T pack; bit-exact against host restatements) and the attention kernel against fp64 attention of the same
quantised operands (tolerance: P is rounded to e4m3 inside the kernel) and against the bf16 path."""

import numpy as np
import pytest
import torch

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

def f8(u):
    return u.cpu().contiguous().view(torch.float8_e4m3fn).double()

def tile_key(k):
    hh, g, e = k >> 5, (k >> 4) & 1, k & 15
    return 32 * hh + 8 * (e >> 2) + 4 * g + (e & 3)

def test_mx_mfma_probe32_layout():
    """Lane l supplies row l % 32, K-chunks l/32 and l/32 + 2, and the scale of (row l % 32, K-block l/32)."""
    from videopainter_amd import _native as NV
    if not NV.has_diag():  # a hardware layout self-test: the diagnostic library only (include/vp_hip_diag.h)
        pytest.skip("diagnostic entry point: run with VP_HIP_LIB=videopainter_amd/_lib/libvp_hip_diag.so")
    from videopainter_amd import kernels as K
    g = torch.Generator().manual_seed(0)
    A = torch.randint(-8, 9, (32, 64), generator=g).float() / 4
    B = torch.randint(-8, 9, (32, 64), generator=g).float() / 4
    B[:, 0] += torch.arange(32).float() / 4
    sa = torch.randint(124, 131, (64,), generator=g).to(torch.uint8)
    sb = torch.randint(124, 131, (64,), generator=g).to(torch.uint8)
    C = K.mx_mfma_probe32(e4m3(A).to(dev), e4m3(B).to(dev), sa.to(dev), sb.to(dev)).cpu().double()
    scA = 2.0 ** (sa.double().view(2, 32).T - 127)  # [row, K-block]
    scB = 2.0 ** (sb.double().view(2, 32).T - 127)
    Ad = (f8(e4m3(A)).view(32, 2, 32) * scA[:, :, None]).view(32, 64)   # e4m3 values (B's ramp rounds)
    Bd = (f8(e4m3(B)).view(32, 2, 32) * scB[:, :, None]).view(32, 64)
    assert torch.equal(C, Ad @ Bd.T)

def v_pack_ref(v: torch.Tensor, heads: int):
    """Host restatement of vp_v_pack_fp8: V [B, N, H*64] -> V^T e4m3 [B, H, 64, npad] (tile K-slot order) + scales."""
    B, Nk, _ = v.shape
    nt = (Nk + 63) // 64
    npad = nt * 64
    vv = torch.zeros(B, npad, heads, 64)
    vv[:, :Nk] = v.float().cpu().view(B, Nk, heads, 64)
    perm = torch.tensor([tile_key(k) for k in range(64)])
    keys = (torch.arange(nt)[:, None] * 64 + perm[None, :]).reshape(-1)       # slot -> key
    vt = vv[:, keys].permute(0, 2, 3, 1).contiguous()                          # [B, H, 64 d, npad slots]
    blocks = vt.view(B, heads, 64, nt * 2, 32).numpy()
    ex = R.block_exponent(np.abs(blocks).max(axis=4))                          # [B, H, 64, nt*2]
    scaled = np.clip(blocks * R.pow2(-ex)[..., None], -448, 448).astype(np.float32)
    q = torch.from_numpy(scaled).view(B, heads, 64, npad).to(torch.float8_e4m3fn).view(torch.uint8)
    sc = np.zeros((B, heads, nt, 64, 2), dtype=np.uint8)                       # [.., tile, lane, d-half]
    exr = ex.reshape(B, heads, 2, 32, nt, 2)                                   # d = 32 dh + r, block = 2 t + kb
    for dh in range(2):
        for kb in range(2):
            sc[:, :, :, 32 * kb:32 * kb + 32, dh] = (exr[:, :, dh, :, :, kb] + 127).transpose(0, 1, 3, 2)
    return q, torch.from_numpy(sc.reshape(-1)), npad

@pytest.mark.parametrize("Nk", [300, 64, 1])
def test_v_pack_bit_exact(Nk):
    from videopainter_amd import kernels as K
    g = torch.Generator().manual_seed(Nk)
    B, H = 2, 3
    v = torch.randn(B, Nk, H * 64, generator=g) * 10.0 ** torch.empty(B, Nk, 1).uniform_(-2, 2, generator=g)
    v = v.to(torch.bfloat16)
    vp = K.v_pack_fp8(v.to(dev), H)
    q_ref, s_ref, npad = v_pack_ref(v, H)
    assert vp.npad == npad
    assert torch.equal(vp.vt.cpu().view(B, H, 64, npad), q_ref)
    assert torch.equal(vp.vs.cpu(), s_ref)

def _rope(n, seed):
    g = torch.Generator().manual_seed(seed)
    ang = torch.rand(n, 32, generator=g) * 6.28
    cos = ang.cos().repeat_interleave(2, dim=1).contiguous()
    sin = ang.sin().repeat_interleave(2, dim=1).contiguous()
    return cos.to(dev), sin.to(dev)

def test_head_norm_rope_fp8_matches_bf16_kernel():
    """The e4m3 producer quantises exactly the bf16 values the bf16 kernel writes, times the factor."""
    from videopainter_amd import kernels as K
    B, T, Nv, H = 2, 5, 70, 3
    g = torch.Generator().manual_seed(3)
    x = (torch.randn(B, T + Nv, 3 * H * 64, generator=g) * 2 + 0.5).to(torch.bfloat16).to(dev)
    lw = (1 + 0.2 * torch.randn(64, generator=g)).to(torch.bfloat16).to(dev)
    lb = (0.2 * torch.randn(64, generator=g)).to(torch.bfloat16).to(dev)
    rope = _rope(Nv, 1)
    q = x[..., :H * 64]
    ref = torch.empty(B, T + Nv, H * 64, device=dev, dtype=torch.bfloat16)
    K.head_norm_rope(q, ref, H, T, lw, lb, 1e-6, rope)
    a = K.qk_fp8_exponent(lw, lb, 0.125 * K.LOG2E)
    mul = 0.125 * K.LOG2E * 2.0 ** a
    q8 = K.head_norm_rope_fp8(q, H, T, lw, lb, 1e-6, rope, mul)
    assert float(ref.float().abs().max()) * mul <= 448
    assert torch.equal(q8.cpu(), e4m3(ref.float().cpu() * mul))

def _attn_case(B, H, Nq, seed, late_spike=False):
    g = torch.Generator().manual_seed(seed)
    q = torch.randn(B, Nq, H * 64, generator=g)
    k = torch.randn(B, Nq, H * 64, generator=g)
    v = torch.randn(B, Nq, H * 64, generator=g) * 2
    if late_spike:
        # a key late in the sequence aligned with every query: the running max jumps long after the first tile
        k[:, Nq - 3] = q.mean(dim=1) * 6
    return q.to(torch.bfloat16), k.to(torch.bfloat16), v.to(torch.bfloat16)

def _ref_fp64(q8, k8, vt, vs, npad, Nk, H, q_exp, k_exp):
    """fp64 attention of the dequantised operands (log2-domain scores as the kernel computes them)."""
    B, Nq, _ = q8.shape
    qd = f8(q8).view(B, Nq, H, 64) * 2.0 ** -q_exp          # = q * scale * log2 e
    kd = f8(k8).view(B, Nk, H, 64) * 2.0 ** -k_exp
    nt = npad // 64
    vtd = f8(vt).view(B, H, 64, nt * 2, 32)
    sc = vs.cpu().view(B, H, nt, 2, 32, 2).double()          # [.., tile, kb, r, dh]
    e = sc.permute(0, 1, 5, 4, 2, 3).reshape(B, H, 64, nt * 2) - 127   # [.., d = 32 dh + r, block]
    vtd = (vtd * 2.0 ** e[..., None]).view(B, H, 64, npad)
    perm = torch.tensor([tile_key(k) for k in range(64)])
    keys = (torch.arange(nt)[:, None] * 64 + perm[None, :]).reshape(-1)
    vd = torch.zeros(B, H, npad, 64, dtype=torch.float64)
    vd[:, :, keys] = vtd.transpose(2, 3)
    vd = vd[:, :, :Nk]
    s = torch.einsum("bqhd,bkhd->bhqk", qd, kd)
    p = torch.exp2(s - s.amax(dim=-1, keepdim=True))
    o = torch.einsum("bhqk,bhkd->bqhd", p / p.sum(dim=-1, keepdim=True), vd)
    return o.reshape(B, Nq, H * 64)

@pytest.fixture(params=["2", "3", "5"], ids=["lin", "lin2", "skew"])
def attn8_variant(request, knobs):
    """VP_ATTN8_VARIANT: 2 = P by linear mantissa interpolation, 3 = the same codes packed by v_cvt_pknorm_u16_f32 +
    a byte gather, 5 = the lin2 kernel with its tile loop skewed by one tile (default).  (1 = exp2 + RNE pack and
    4 = the software-pipelined f8p were rejected A/B forms, pruned in round 6.)"""
    from videopainter_amd import kernels as K
    if not K.attention_variant_built("fp8:" + request.param):
        pytest.skip(f"fp8 attention variant {request.param} is not in this build")
    knobs.setenv("VP_ATTN8_VARIANT", request.param)
    return request.param


# tile counts 5 / 32 / 2 / 1 / 3: both tail paths of the pipelined kernel (an odd and an even number of tiles after
# the first), a single partial tile, a one-key last tile
@pytest.mark.parametrize("B,H,N,late", [(2, 3, 300, False), (1, 2, 2000, True), (1, 1, 65, False), (1, 2, 40, False),
                                        (2, 1, 130, False)])
def test_attention_fp8(B, H, N, late, attn8_variant):
    from videopainter_amd import kernels as K
    q, k, v = _attn_case(B, H, N, N, late)
    qd, kd, vd = q.to(dev), k.to(dev), v.to(dev)
    q_exp, k_exp = 5, 4
    q8 = e4m3(q.float() * 0.125 * K.LOG2E * 2.0 ** q_exp).to(dev)
    k8 = e4m3(k.float() * 2.0 ** k_exp).to(dev)
    vp = K.v_pack_fp8(vd, H)
    out = torch.empty(B, N, H * 64, device=dev, dtype=torch.bfloat16)
    K.attention_fp8(q8, k8, vp, out, H, q_exp, k_exp)
    ref = _ref_fp64(q8, k8, vp.vt, vp.vs, vp.npad, N, H, q_exp, k_exp)
    # the kernel's own error on top of the operand quantisation: P rounded to e4m3 (2^-4 relative; the linear
    # codes 3.2 % rms against 2.7 %) — on random data ~2-3 % of the (cancelling) output; a wrong key/slot
    # permutation would give ~100 %
    print(f"fp8 attention variant {attn8_variant} B={B} H={H} N={N}: rel vs fp64 {rel(out, ref):.3e}")
    assert rel(out, ref) < 4e-2
    # against the bf16 kernel on the un-quantised operands: the fp8 error band
    o16 = torch.empty_like(out)
    K.attention(qd, kd, vd, o16, H, scale=0.125)
    assert rel(out, o16) < 8e-2
    # blend epilogue (prev-clip path): out = 0.7 * A + 0.3 * A
    o2 = torch.empty_like(out)
    K.attention_fp8(q8, k8, vp, o2, H, q_exp, k_exp, out_scale=0.7)
    K.attention_fp8(q8, k8, vp, o2, H, q_exp, k_exp, out_scale=0.3, accumulate=True)
    assert rel(o2, out) < 1e-2


# partial last tiles of every size class (1, 3, 4, 5, 33, 63 keys) and one- to three-tile sequences
@pytest.mark.parametrize("N", [65, 67, 68, 69, 97, 127, 128, 129, 1000])
@pytest.mark.parametrize("var", ["5"])
def test_attention_fp8_skewed_bit_identical(N, var, knobs):
    """The skewed loop (variant 5, the default) computes the same P codes, rescale decisions and accumulation order as
    variant 3; its last-tile mask zeroes the P codes of the keys past Nk (duplicates of key Nk - 1) where variant 3
    sets their scores to -inf: the outputs are equal bit for bit, also through the blend epilogue."""
    from videopainter_amd import kernels as K
    B, H = 2, 3
    q, k, v = _attn_case(B, H, N, 1000 + N, late_spike=N >= 1000)
    q_exp, k_exp = 5, 4
    q8 = e4m3(q.float() * 0.125 * K.LOG2E * 2.0 ** q_exp).to(dev)
    k8 = e4m3(k.float() * 2.0 ** k_exp).to(dev)
    vp = K.v_pack_fp8(v.to(dev), H)
    outs = {}
    for vv in ("3", var):
        knobs.setenv("VP_ATTN8_VARIANT", vv)
        o = torch.empty(B, N, H * 64, device=dev, dtype=torch.bfloat16)
        K.attention_fp8(q8, k8, vp, o, H, q_exp, k_exp, out_scale=0.7)
        K.attention_fp8(q8, k8, vp, o, H, q_exp, k_exp, out_scale=0.3, accumulate=True)
        outs[vv] = o
    torch.cuda.synchronize()
    assert torch.isfinite(outs[var].float()).all()
    assert torch.equal(outs["3"].view(torch.int16), outs[var].view(torch.int16))


@pytest.mark.parametrize("B,H,N", [(1, 24, 12000), (2, 9, 15000)])
def test_attention_fp8_persistent_bit_identical(B, H, N, knobs):
    """The persistent default fp8 kernel (query blocks by per-XCD ticket, ABI 20 workspace) against one workgroup per
    block (VP_ATTN_PERSIST=0): every block's arithmetic is the same whoever runs it — equal bit for bit."""
    from videopainter_amd import kernels as K
    from videopainter_amd import _native as N_
    import ctypes as C
    q, k, v = _attn_case(B, H, N, 4000 + N, late_spike=True)
    q_exp, k_exp = 5, 4
    q8 = e4m3(q.float() * 0.125 * K.LOG2E * 2.0 ** q_exp).to(dev)
    k8 = e4m3(k.float() * 2.0 ** k_exp).to(dev)
    vp = K.v_pack_fp8(v.to(dev), H)
    dd = N_.AttnFp8Desc()
    dd.base.B, dd.base.H, dd.base.Nq = B, H, N
    assert N_.lib().vp_attention_fp8_workspace_bytes(C.byref(dd)) > 0  # the persistent path is taken
    outs = []
    for persist in ("1", "0"):
        knobs.setenv("VP_ATTN_PERSIST", persist)
        o = torch.empty(B, N, H * 64, device=dev, dtype=torch.bfloat16)
        K.attention_fp8(q8, k8, vp, o, H, q_exp, k_exp)
        outs.append(o)
    torch.cuda.synchronize()
    assert torch.isfinite(outs[0].float()).all()
    assert torch.equal(outs[0].view(torch.int16), outs[1].view(torch.int16))


def _ln_rows(x, H):
    """Per-head LayerNorm(64) without affine: the |x| = 8 rows CogVideoX's qk-norm produces."""
    B, N, _ = x.shape
    xh = x.view(B, N, H, 64)
    xh = (xh - xh.mean(-1, keepdim=True)) / xh.std(-1, unbiased=False, keepdim=True)
    return xh.reshape(B, N, H * 64)


def _sdpa_fp32_chunked(q, k, v, H, scale=0.125, chunk=4096):
    B, N, D = q.shape
    out = torch.empty(B, N, D, device=q.device, dtype=torch.float32)
    for h in range(H):
        sl = slice(h * 64, (h + 1) * 64)
        kh, vh = k[..., sl].float(), v[..., sl].float()
        for c0 in range(0, N, chunk):
            s = torch.einsum("bqd,bkd->bqk", q[:, c0:c0 + chunk, sl].float(), kh) * scale
            out[:, c0:c0 + chunk, sl] = torch.softmax(s, dim=-1) @ vh
            del s
    return out


def test_attention_fp8_and_bf16_at_config5_length(attn8_variant):
    """BASELINE config 5's sequence length (N = 226 + 46 800 = 47 026) on two heads, LayerNorm-shaped q / k (what
    the qk-norm feeds the kernel): the fp8 kernel against fp32 attention on the same bf16 operands (re-stated fp8
    band: 6e-2 — P in e4m3 keeps 3 mantissa bits), and both bf16 kernels (running max / bounded scores) within
    1e-2."""
    from videopainter_amd import kernels as K
    B, H, N = 1, 2, 47026
    g = torch.Generator().manual_seed(47)
    q = _ln_rows(torch.randn(B, N, H * 64, generator=g), H).to(torch.bfloat16).to(dev)
    k = _ln_rows(torch.randn(B, N, H * 64, generator=g) + 0.3 * torch.randn(B, 1, H * 64, generator=g),
                 H).to(torch.bfloat16).to(dev)
    v = (torch.randn(B, N, H * 64, generator=g) * 2).to(torch.bfloat16).to(dev)
    ref = _sdpa_fp32_chunked(q, k, v, H)
    o16 = torch.empty(B, N, H * 64, device=dev, dtype=torch.bfloat16)
    for bounded in (False, True):  # |s| <= 8 * 8 * 0.125 * log2 e = 11.5 here: inside the bounded-score contract
        K.attention(q, k, v, o16, H, scale=0.125, bounded_scores=bounded)
        r16 = rel(o16, ref)
        print(f"bf16 attention (bounded={bounded}) at N={N}: rel {r16:.3e}")
        assert r16 < 1e-2
    ones = torch.ones(64, device=dev, dtype=torch.bfloat16)
    zeros = torch.zeros(64, device=dev, dtype=torch.bfloat16)
    q_exp = K.qk_fp8_exponent(ones, zeros, 0.125 * K.LOG2E)
    k_exp = K.qk_fp8_exponent(ones, zeros)
    q8 = e4m3(q.float().cpu() * 0.125 * K.LOG2E * 2.0 ** q_exp).to(dev)
    k8 = e4m3(k.float().cpu() * 2.0 ** k_exp).to(dev)
    vp = K.v_pack_fp8(v, H)
    o8 = torch.empty(B, N, H * 64, device=dev, dtype=torch.bfloat16)
    K.attention_fp8(q8, k8, vp, o8, H, q_exp, k_exp)
    r8 = rel(o8, ref)
    print(f"fp8 attention (variant {attn8_variant}) at N={N}: rel vs fp32 {r8:.3e}")
    assert r8 < 6e-2
