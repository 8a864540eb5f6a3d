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
