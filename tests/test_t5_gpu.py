"""T5 v1.1 encoder on the HIP kernels (videopainter_amd/t5.py, csrc/t5.hip) — GPU tests.

Kernel level against plain torch fp32 on the same bf16 inputs.  Model level against transformers' T5EncoderModel fp32
outputs (tests/golden/t5.safetensors, made with the installed transformers 5.15; the reference pins 4.42.2), gate =
1.25 x the drift of a bf16 run of the 4.42.2 eager algorithm (the pinned oracle in bf16, recorded by make_golden) +
1e-3.  (transformers 5.x's own bf16 run is recorded too; it drifts less because its sdpa path keeps q.k in fp32.)
"""
import os

import pytest
import torch
import torch.nn.functional as F
from safetensors.torch import load_file

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def rel(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.fixture(scope="module")
def K():
    from videopainter_amd import kernels
    return kernels


def test_rms_norm_mul_gather(K):
    torch.manual_seed(0)
    x = torch.randn(452, 4096, device="cuda").bfloat16() * 3
    w = (1 + 0.1 * torch.randn(4096, device="cuda")).bfloat16()
    y = K.rms_norm(x, w, 1e-6)
    xf = x.float()
    ref = w.float() * (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-6)).bfloat16().float()
    assert rel(y.float(), ref) < 4e-3
    a, b = torch.randn(64, 256, device="cuda").bfloat16(), torch.randn(64, 256, device="cuda").bfloat16()
    assert torch.equal(K.mul(a, b), (a.float() * b.float()).bfloat16())
    table = torch.randn(100, 128, device="cuda").bfloat16()
    ids = torch.randint(0, 100, (2, 9), device="cuda")
    assert torch.equal(K.embedding_gather(table, ids), table[ids.flatten()])


@pytest.mark.parametrize("L,H,masked", [(226, 64, False), (226, 2, True), (77, 4, False)])
def test_t5_attention_matches_torch(K, L, H, masked):
    from videopainter_amd.t5 import relative_position_buckets
    torch.manual_seed(L + H)
    B = 2
    qkv = (0.25 * torch.randn(B * L, 3 * H * 64, device="cuda")).bfloat16()  # scores ~ N(0, 4): not one-hot
    table = (0.5 * torch.randn(32, H, device="cuda")).bfloat16()
    buckets = relative_position_buckets(L, 32, 128).cuda()
    mask = None
    if masked:
        mask = torch.ones(B, L, dtype=torch.int64, device="cuda")
        mask[0, 40:] = 0
        mask[1, 200:] = 0
    out = K.t5_attention(qkv, B, L, H, table, buckets, mask)
    q, k, v = qkv.float().view(B, L, 3, H, 64).unbind(2)
    q, k, v = (t.transpose(1, 2) for t in (q, k, v))
    bias = table.float()[buckets.long()].permute(2, 0, 1)[None]
    s = (q @ k.transpose(-1, -2)).bfloat16().float() + bias
    if mask is not None:
        s = s + (1 - mask[:, None, None, :].float()) * torch.finfo(torch.bfloat16).min
    p = torch.softmax(s, -1).bfloat16().float()
    ref = (p @ v).transpose(1, 2).reshape(B * L, H * 64)
    r = rel(out.float(), ref)
    print(f"t5 attention L={L} H={H} masked={masked}: rel {r:.2e}")
    assert r < 1e-2


@pytest.mark.parametrize("L,H,masked", [(226, 64, False), (226, 2, True), (77, 4, False), (33, 3, True),
                                         (384, 2, False)])
def test_t5_attention_mfma_matches_scalar_kernel(K, L, H, masked, knobs):
    """The MFMA T5 attention (default) against the scalar-FMA kernel (VP_T5_ATTN=scalar) on the same operands: the
    same roundings (bf16 scores + bias, fp32 softmax, bf16 weights), only the fp32 summation orders differ, so the
    outputs agree to a few bf16 ulps; key padding (L not a multiple of 32) and masked keys included."""
    from videopainter_amd.t5 import relative_position_buckets
    torch.manual_seed(7 * L + H)
    B = 2
    qkv = (0.25 * torch.randn(B * L, 3 * H * 64, device="cuda")).bfloat16()
    table = (0.5 * torch.randn(32, H, device="cuda")).bfloat16()
    buckets = relative_position_buckets(L, 32, 128).cuda()
    mask = None
    if masked:
        mask = torch.ones(B, L, dtype=torch.int64, device="cuda")
        mask[0, L // 3:] = 0
        mask[1, L - 5:] = 0
    out = K.t5_attention(qkv, B, L, H, table, buckets, mask)
    knobs.setenv("VP_T5_ATTN", "scalar")
    ref = K.t5_attention(qkv, B, L, H, table, buckets, mask)
    r = rel(out.float(), ref.float())
    print(f"t5 attention mfma vs scalar L={L} H={H} masked={masked}: rel {r:.2e}, "
          f"max |d| {(out.float() - ref.float()).abs().max().item():.2e}")
    assert torch.isfinite(out.float()).all()
    assert r < 3e-3


def _model(cfg, seed):
    from videopainter_amd.t5 import T5EncoderModel
    from tests.golden.cases import t5_weights
    m = T5EncoderModel.from_config(cfg, device="cuda")
    m.load_state_dict({k: torch.from_numpy(v) for k, v in t5_weights(cfg, seed).items()})
    return m


@pytest.mark.parametrize("tag", ["tiny", "xxl2"])
def test_t5_encoder_matches_transformers(tag):
    from tests.golden.cases import T5_TINY_CFG, T5_XXL2_CFG, T5_SEEDS, t5_inputs
    from videopainter_amd.config import full_t5_config
    cfg, seed = (T5_TINY_CFG, T5_SEEDS[0]) if tag == "tiny" else (T5_XXL2_CFG, T5_SEEDS[1])
    g = load_file(os.path.join(GOLD, "t5.safetensors"))
    m = _model(cfg, seed)
    ids, mask = t5_inputs(full_t5_config(cfg)["vocab_size"], key=f"t5{tag}")
    with torch.no_grad():
        y = m(ids.cuda())[0]
    stride = 1 if tag == "tiny" else 8
    drift = float(g[f"{tag}.oracle_bf16_rel"][0])
    r = rel(y[..., ::stride].float(), g[f"{tag}.out"])
    print(f"t5 {tag}: HIP {r:.3e}, 4.42 eager algorithm in bf16 {drift:.3e} (transformers 5.15 sdpa bf16 "
          f"{float(g[f'{tag}.ref_bf16_rel'][0]):.3e})")
    assert y.shape == (2, 226, full_t5_config(cfg)["d_model"]) and y.dtype == torch.bfloat16
    assert r <= 1.25 * drift + 1e-3
    if tag == "tiny":
        with torch.no_grad():
            ym = m(ids.cuda(), attention_mask=mask.cuda())[0]
        rm = rel(ym.float(), g["tiny.masked.out"])
        print(f"t5 tiny masked: HIP {rm:.3e}")
        assert rm <= 1.25 * drift + 1e-3
        # the pipeline's call form: text_encoder(ids)[0], hidden states on request
        with torch.no_grad():
            o = m(input_ids=ids.cuda(), output_hidden_states=True)
        assert len(o.hidden_states) == full_t5_config(cfg)["num_layers"] + 1
        assert torch.equal(o.hidden_states[-1], o.last_hidden_state)


def test_t5_hip_graph_replay_matches_eager():
    """enable_hip_graphs(): the captured 24-layer stack replays bit-identically to the eager forward, for a second
    input of the same shape too (static input buffers refreshed per call), with and without an attention mask."""
    from tests.golden.cases import T5_TINY_CFG
    from videopainter_amd import kernels as K
    from videopainter_amd.t5 import T5EncoderModel
    m = T5EncoderModel.from_config(dict(T5_TINY_CFG), device="cuda")
    for i, (name, p) in enumerate(m.named_parameters()):
        if p.dim() == 1:
            p.data.fill_(1.0)
        else:
            K.fill_normal_(p.data, 77 + i, 0.0, p.shape[1] ** -0.5)
    g = torch.Generator().manual_seed(5)
    for use_mask in (False, True):
        runs = []
        for _ in range(2):
            ids = torch.randint(0, T5_TINY_CFG.get("vocab_size", 32128), (2, 40), generator=g).cuda()
            mask = torch.ones(2, 40, dtype=torch.int64, device="cuda")
            mask[1, 30:] = 0
            kw = dict(attention_mask=mask) if use_mask else {}
            with torch.no_grad():
                m.enable_hip_graphs(False)
                e = m(input_ids=ids, **kw)[0].clone()
                m.enable_hip_graphs(True)
                r = m(input_ids=ids, **kw)[0]
            runs.append((e, r))
        for e, r in runs:
            assert torch.equal(e, r)
        assert not torch.equal(runs[0][0], runs[1][0])
        # a round trip through the host (model CPU offload) moves every parameter: the captured graphs must not be
        # replayed on the freed storage
        m.cpu()
        m.cuda()
        with torch.no_grad():
            r2 = m(input_ids=ids, **kw)[0]
        assert torch.equal(runs[-1][0], r2)
