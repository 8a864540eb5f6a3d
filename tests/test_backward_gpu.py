"""Backward kernels — GPU tests against torch autograd in fp32 on the same bf16 inputs."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.mark.parametrize("B,H,N,Nk", [(1, 2, 300, 300), (2, 3, 1378, 1378), (1, 1, 65, 200), (1, 2, 4500, 4500)])
def test_attention_backward_matches_autograd(B, H, N, Nk):
    from videopainter_amd import kernels as K
    torch.manual_seed(N + H)
    dev = "cuda"
    # qk-LayerNorm-like magnitudes (|q|, |k| ~ 8): scores of a few units after the 1/8 scale
    q = torch.randn(B, N, H * 64, device=dev).bfloat16()
    k = torch.randn(B, Nk, H * 64, device=dev).bfloat16()
    v = torch.randn(B, Nk, H * 64, device=dev).bfloat16()
    o = torch.empty(B, N, H * 64, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B, H, N, device=dev, dtype=torch.float32)
    K.attention(q, k, v, o, H, lse=lse)
    do = torch.randn(B, N, H * 64, device=dev).bfloat16()
    dq, dk, dv = K.attention_bwd(q, k, v, o, do, lse, H)
    qf, kf, vf = (t.float().view(t.shape[0], t.shape[1], H, 64).transpose(1, 2).requires_grad_() for t in (q, k, v))
    p = torch.softmax((qf @ kf.transpose(-1, -2)) * 0.125, -1)
    of = p @ vf
    # lse: log2-sum-exp2 of the log2-unit scores
    ref_lse = torch.logsumexp((qf @ kf.transpose(-1, -2)) * 0.125, -1) / torch.log(torch.tensor(2.0))
    assert rel(lse, ref_lse.detach() * 1.0) < 1e-3
    of.backward(do.float().view(B, N, H, 64).transpose(1, 2))
    for name, got, want in (("dq", dq, qf.grad), ("dk", dk, kf.grad), ("dv", dv, vf.grad)):
        w = want.transpose(1, 2).reshape(got.shape)
        r = rel(got.float(), w)
        print(f"attention bwd B={B} H={H} N={N} Nk={Nk} {name}: rel {r:.3e}")
        assert r < 2e-2, name


@pytest.mark.parametrize("B,H,N,Nk", [(1, 2, 300, 300), (1, 1, 65, 200), (2, 2, 1378, 1410), (1, 2, 4500, 4500),
                                      (1, 1, 128, 96), (1, 1, 200, 64)])
def test_attention_backward_variants_bit_identical(knobs, B, H, N, Nk):
    """VP_ATTN_BWD_VARIANT 1 (default: conflict-free swizzle, peeled last key tile, no in-loop waits on the next
    tile's DMA) against 0 (round 2's kernels): the same products in the same order, so the same bits — full tiles,
    partial last tiles of 8 / 32 / 44 / 62 / 36 keys or queries, a key count below one tile."""
    from videopainter_amd import kernels as K
    torch.manual_seed(N * 7 + Nk)
    dev = "cuda"
    q = torch.randn(B, N, H * 64, device=dev).bfloat16()
    k = torch.randn(B, Nk, H * 64, device=dev).bfloat16()
    v = torch.randn(B, Nk, H * 64, device=dev).bfloat16()
    o = torch.empty(B, N, H * 64, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B, H, N, device=dev, dtype=torch.float32)
    K.attention(q, k, v, o, H, lse=lse)
    do = torch.randn(B, N, H * 64, device=dev).bfloat16()
    got = {}
    for var in ("0", "1"):
        knobs.setenv("VP_ATTN_BWD_VARIANT", var)
        got[var] = K.attention_bwd(q, k, v, o, do, lse, H)
        torch.cuda.synchronize()
    for var in ("1",):
        for name, a, b in zip(("dq", "dk", "dv"), got["0"], got[var]):
            assert torch.equal(a, b), (var, name)


@pytest.mark.parametrize("B,H,N,Nk", [(1, 48, 17776, 17776), (2, 17, 8010, 7003)])
def test_attention_backward_tail_split_matches_unsplit(knobs, B, H, N, Nk):
    """The grid-tail split of the backward (the last partial round's blocks as key- / query-range pieces at the end of
    each grid, their fp32 sums merged): the training shape (6 672 blocks of each kernel: 16 dQ / 528 dK-dV remainder
    blocks) and a ragged one, against the unsplit launch — the same sums in another order, so bf16-rounding level."""
    import ctypes as C
    from videopainter_amd import _native as N_
    from videopainter_amd import kernels as K
    torch.manual_seed(N + Nk)
    dev = "cuda"
    q = torch.randn(B, N, H * 64, device=dev).bfloat16()
    k = torch.randn(B, Nk, H * 64, device=dev).bfloat16()
    v = torch.randn(B, Nk, H * 64, device=dev).bfloat16()
    o = torch.empty(B, N, H * 64, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B, H, N, device=dev, dtype=torch.float32)
    K.attention(q, k, v, o, H, lse=lse)
    do = torch.randn(B, N, H * 64, device=dev).bfloat16()
    d = N_.AttnBwdDesc()
    d.B, d.H, d.Nq, d.Nk, d.head_dim = B, H, N, Nk, 64
    for nm, t in (("Q", q), ("K", k), ("V", v), ("O", o), ("dO", do), ("dQ", q), ("dK", k), ("dV", v)):
        setattr(d, nm, t.data_ptr())
    for nm, t in (("q", q), ("k", k), ("v", v), ("o", o), ("do", do), ("dq", q), ("dk", k), ("dv", v)):
        setattr(d, f"{nm}_sb", t.stride(0))
        setattr(d, f"{nm}_sn", t.stride(1))
    d.lse, d.delta = lse.data_ptr(), lse.data_ptr()
    assert N_.lib().vp_attention_bwd_workspace_bytes(C.byref(d)) > 0  # the split is active for this shape
    split = K.attention_bwd(q, k, v, o, do, lse, H)
    knobs.setenv("VP_ATTN_NO_SPLIT", "1")
    whole = K.attention_bwd(q, k, v, o, do, lse, H)
    for name, a, b in zip(("dq", "dk", "dv"), split, whole):
        r = rel(a.float(), b.float())
        print(f"bwd tail split B={B} H={H} N={N} Nk={Nk} {name}: rel {r:.3e}")
        assert r < 2e-3, name
