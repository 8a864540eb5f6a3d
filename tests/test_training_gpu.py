"""Training backward (videopainter_amd/autograd.py, csrc/backward.hip) — GPU tests.

Kernel level: each backward kernel against torch autograd in fp32 on the same bf16 inputs.
Block / model level: gradients of the HIP path against autograd of the CPU oracle (oracle/cogvideox_oracle.py, the
reference's algorithm restated) in fp32 with the same bf16-rounded weights and inputs.  The band per gradient
tensor is the oracle's own bf16 drift (the same autograd graph run in bf16 on the CPU, i.e. what the reference's
bf16 training computes):  rel(HIP, fp32) <= GATE_MUL * rel(oracle_bf16, fp32) + GATE_ADD.
"""

import pytest
import torch
import torch.nn.functional as F

from tests.golden.cases import TINY_CFG, TINY_BRANCH_CFG, tiny_inputs, tiny_weights

pytestmark = pytest.mark.gpu
dev = "cuda"
GATE_MUL, GATE_ADD = 1.25, 1e-3  # the model tests' rule (tests/test_model_gpu.py)


def rel(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.fixture(scope="module")
def K():
    from videopainter_amd import kernels
    return kernels


# ------------------------------------------------------------------------------------------------------------------
# kernels
# ------------------------------------------------------------------------------------------------------------------

def test_transpose_colsum_wgrad(K):
    torch.manual_seed(1)
    x = torch.randn(3, 77, 136, device=dev).bfloat16()
    t = K.transpose(x, pad_to=64)
    assert t.shape == (136, 256)
    assert torch.equal(t[:, :231], x.reshape(231, 136).t())
    assert torch.count_nonzero(t[:, 231:]) == 0
    a = torch.randn(2 * 300, 96, device=dev).bfloat16()
    b = torch.randn(2 * 300, 96, device=dev).bfloat16()
    s = K.colsum(a, b, tokens_per_batch=300, text_len=8)
    p = (a.float() * b.float()).view(2, 300, 96)
    want = torch.stack((p[:, 8:].sum(1), p[:, :8].sum(1)), 1)
    assert rel(s, want) < 1e-5
    dy = torch.randn(1000, 192, device=dev).bfloat16()
    xx = torch.randn(1000, 136, device=dev).bfloat16()
    assert rel(K.wgrad(dy, xx).float(), dy.float().t() @ xx.float()) < 4e-3


def test_adaln_backward_matches_autograd(K):
    torch.manual_seed(2)
    B, N, T, D = 2, 300, 8, 384
    x = torch.randn(B, N, D, device=dev).bfloat16()
    w = (1 + 0.1 * torch.randn(D, device=dev)).bfloat16()
    bb = (0.1 * torch.randn(D, device=dev)).bfloat16()
    mod = (0.3 * torch.randn(B, 6 * D, device=dev)).bfloat16()
    dy = torch.randn(B, N, D, device=dev).bfloat16()
    dx = torch.zeros_like(x)
    n_out, dn_out, xh_out = (torch.empty_like(x) for _ in range(3))
    K.adaln_bwd(x, dy, dx, T, w, bb, 1e-5, mod, n_out=n_out, dn_out=dn_out, xhat_out=xh_out)
    xf = x.float().requires_grad_()
    wf, bf = w.float().requires_grad_(), bb.float().requires_grad_()
    m = mod.float().view(B, 6, D).requires_grad_()
    n = F.layer_norm(xf, (D,), wf, bf, 1e-5)
    sc = torch.cat([m[:, 4:5].expand(B, T, D), m[:, 1:2].expand(B, N - T, D)], 1)
    sh = torch.cat([m[:, 3:4].expand(B, T, D), m[:, 0:1].expand(B, N - T, D)], 1)
    (n * (1 + sc) + sh).backward(dy.float())
    assert rel(dx.float(), xf.grad) < 1e-2
    M = B * N
    assert rel(K.colsum(dn_out.view(M, D), xh_out.view(M, D))[0, 0], wf.grad) < 1e-2
    assert rel(K.colsum(dn_out.view(M, D))[0, 0], bf.grad) < 1e-2
    dsc = K.colsum(dy.view(M, D), n_out.view(M, D), tokens_per_batch=N, text_len=T)
    assert rel(dsc[:, 0], m.grad[:, 1]) < 1e-2 and rel(dsc[:, 1], m.grad[:, 4]) < 1e-2


def test_head_norm_rope_backward_matches_autograd(K):
    from oracle.cogvideox_oracle import apply_rotary_emb, prepare_rotary_positional_embeddings
    from videopainter_amd.modules import LayerNorm
    torch.manual_seed(3)
    B, H, T = 2, 3, 8
    cos, sin = prepare_rotary_positional_embeddings(16 * 8, 24 * 8, 3, 64)
    N = T + cos.shape[0]
    x = torch.randn(B, N, H * 64, device=dev).bfloat16()
    dy = torch.randn(B, N, H * 64, device=dev).bfloat16()
    ln = LayerNorm(64, 1e-6, True).to(dev)
    with torch.no_grad():
        ln.weight.copy_(1 + 0.2 * torch.randn(64))
        ln.bias.copy_(0.1 * torch.randn(64))
    dw, db = torch.zeros(64, device=dev), torch.zeros(64, device=dev)
    dx = K.head_norm_rope_bwd(x, dy, torch.empty_like(x), H, T, ln, (cos.to(dev), sin.to(dev)), (dw, db))
    xf = x.float().view(B, N, H, 64).transpose(1, 2).requires_grad_()
    wf, bf = ln.weight.float().detach().requires_grad_(), ln.bias.float().detach().requires_grad_()
    y = F.layer_norm(xf, (64,), wf, bf, 1e-6)
    y = torch.cat([y[:, :, :T], apply_rotary_emb(y[:, :, T:], cos.to(dev), sin.to(dev))], 2)
    y.backward(dy.float().view(B, N, H, 64).transpose(1, 2))
    assert rel(dx.float(), xf.grad.transpose(1, 2).reshape(B, N, H * 64)) < 1e-2
    assert rel(dw, wf.grad) < 1e-2 and rel(db, bf.grad) < 1e-2


# ------------------------------------------------------------------------------------------------------------------
# block and model against the oracle's autograd
# ------------------------------------------------------------------------------------------------------------------

def _models(train_branch=True, wo_text=False):
    from videopainter_amd import CogVideoXTransformer3DModel, CogvideoXBranchModel, device_scope
    tsd, bsd = tiny_weights()
    with device_scope(dev):
        tr = CogVideoXTransformer3DModel(**TINY_CFG)
        br = CogvideoXBranchModel(**dict(TINY_BRANCH_CFG, wo_text=wo_text))
    tr.load_diffusers_state_dict({k: torch.from_numpy(v) for k, v in tsd.items()})
    br.load_diffusers_state_dict({k: torch.from_numpy(v) for k, v in bsd.items()})
    br.requires_grad_(train_branch)
    return tr, br, tsd, bsd


def _check(name, got, want, ref16):
    r = rel(got.float(), want)
    r16 = rel(ref16.float(), want)
    print(f"{name:48s} HIP {r:.3e}  oracle-bf16 {r16:.3e}")
    assert r <= GATE_MUL * r16 + GATE_ADD, (name, r, r16)


def test_block_backward_matches_oracle():
    """One trainable branch block: d x, d temb and every parameter gradient."""
    from oracle import cogvideox_oracle as O
    from videopainter_amd.autograd import block_apply
    from videopainter_amd.config import full_config
    _, br, _, bsd = _models()
    cfg = full_config(TINY_BRANCH_CFG, True)
    i = tiny_inputs()
    T = i["enc"].shape[1]
    D = 128
    torch.manual_seed(4)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, T + 288, D, generator=g).bfloat16()
    temb = torch.randn(2, 32, generator=g).bfloat16()
    dout = torch.randn(2, T + 288, D, generator=g).bfloat16()
    blk = br.transformer_blocks[0]
    xd = x.to(dev).requires_grad_()
    td = temb.to(dev).requires_grad_()
    out = block_apply(blk, xd, T, td, (i["rope"][0].to(dev), i["rope"][1].to(dev)))
    out.backward(dout.to(dev))
    names = [n for n, _ in blk.named_parameters()]
    ours = {n: p.grad for n, p in blk.named_parameters()}

    def oracle(dtype):
        sd = {k[len("transformer_blocks.0."):]: torch.from_numpy(v).to(dtype).requires_grad_()
              for k, v in bsd.items() if k.startswith("transformer_blocks.0.")}
        xo = x.to(dtype).requires_grad_()
        to = temb.to(dtype).requires_grad_()
        h, e = O.block_forward({f"b.{k}": v for k, v in sd.items()}, "b", cfg, xo[:, T:], xo[:, :T], to,
                               i["rope"])
        torch.cat([e, h], 1).backward(dout.to(dtype))
        return xo.grad, to.grad, {k: sd[k].grad for k in names}

    gx32, gt32, gp32 = oracle(torch.float32)
    gx16, gt16, gp16 = oracle(torch.bfloat16)
    _check("dx", xd.grad, gx32, gx16)
    _check("dtemb", td.grad, gt32, gt16)
    for n in names:
        _check(n, ours[n], gp32[n], gp16[n])


@pytest.mark.parametrize("lora", [False, True], ids=["plain", "lora"])
def test_saved_attention_backward_is_bit_identical(monkeypatch, lora):
    """autograd.SAVE_ACTIVATIONS (the training forward keeps every intermediate the backward reads) and
    SAVE_ATTENTION (the attention output + lse only) against the full recompute: the same forward output bits (the
    saving forward's fused QKV / GELU epilogues with their aux outputs = forward_joint's launches) and the same
    gradient bits
    (also with an unfused trainable adapter on the projections), up to the atomic-order noise of the qk-norm affine
    sums."""
    from videopainter_amd import autograd as AG
    from videopainter_amd.autograd import block_apply
    tr, br, _, _ = _models()
    blk = br.transformer_blocks[0]
    if lora:  # the VideoPainterID path: adapters on the frozen transformer's projections
        tr.add_adapter({"r": 8, "lora_alpha": 8, "target_modules": ["to_q", "to_k", "to_v", "to_out.0"]})
        blk = tr.transformer_blocks[0]
        g0 = torch.Generator().manual_seed(9)
        with torch.no_grad():
            for l in (blk.attn1.to_q, blk.attn1.to_k, blk.attn1.to_v, blk.attn1.to_out[0]):
                l.lora_B.weight.copy_(torch.randn(l.lora_B.weight.shape, generator=g0).to(dev) * 0.05)
    i = tiny_inputs()
    T = i["enc"].shape[1]
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, T + 288, 128, generator=g).bfloat16()
    temb = torch.randn(2, 32, generator=g).bfloat16()
    dout = torch.randn(2, T + 288, 128, generator=g).bfloat16()
    res = []
    # all intermediates kept (the training forward runs the backward's front) / the attention only / recompute all
    for acts, attn in ((True, True), (False, True), (False, False)):
        monkeypatch.setattr(AG, "SAVE_ACTIVATIONS", acts)
        monkeypatch.setattr(AG, "SAVE_ATTENTION", attn)
        for p in blk.parameters():
            p.grad = None
        xd = x.to(dev).requires_grad_()
        td = temb.to(dev).requires_grad_()
        out = block_apply(blk, xd, T, td, (i["rope"][0].to(dev), i["rope"][1].to(dev)))
        out.backward(dout.to(dev))
        res.append((out.detach(), xd.grad, td.grad,
                    {n: p.grad.clone() for n, p in blk.named_parameters() if p.grad is not None}))
    o0, gx0, gt0, gp0 = res[-1]
    for o1, gx1, gt1, gp1 in res[:-1]:
        assert torch.equal(o1, o0) and torch.equal(gx1, gx0) and torch.equal(gt1, gt0)
        assert gp1.keys() == gp0.keys() and len(gp1) > 0
        for n in gp1:
            if ".norm_q." in n or ".norm_k." in n:
                # (the qk-norm affine gradients are summed with fp32 atomics across workgroups: run-to-run noise)
                assert rel(gp1[n].float(), gp0[n].float()) < 1e-5, n
            else:
                assert torch.equal(gp1[n], gp0[n]), n


def test_frozen_block_with_loaded_adapter_input_gradient(monkeypatch):
    """a frozen transformer block carrying a LOADED (unfused) adapter, trained through for its
    input only (the branch's injection path), with SAVE_ACTIVATIONS on: the saving forward keeps no xn / xq for a
    frozen block, and the backward's unfused-adapter dgrad must not read them.  The input gradient equals the
    full-recompute one bit for bit."""
    from videopainter_amd import autograd as AG
    from videopainter_amd.autograd import block_apply
    from videopainter_amd.lora import attach_lora_
    tr, _, _, _ = _models()
    blk = tr.transformer_blocks[0]
    g0 = torch.Generator().manual_seed(11)
    sd = {}
    for n, lin in (("to_q", blk.attn1.to_q), ("to_k", blk.attn1.to_k), ("to_v", blk.attn1.to_v),
                   ("to_out.0", blk.attn1.to_out[0])):
        o, k = lin.weight.shape
        sd[f"transformer_blocks.0.attn1.{n}.lora_A.weight"] = torch.randn(8, k, generator=g0) * 0.1
        sd[f"transformer_blocks.0.attn1.{n}.lora_B.weight"] = torch.randn(o, 8, generator=g0) * 0.05
    attach_lora_(tr, sd)
    for p in blk.parameters():
        p.requires_grad_(False)
    i = tiny_inputs()
    T = i["enc"].shape[1]
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, T + 288, 128, generator=g).bfloat16()
    temb = torch.randn(2, 32, generator=g).bfloat16()
    dout = torch.randn(2, T + 288, 128, generator=g).bfloat16()
    res = []
    for acts, attn in ((True, True), (False, True), (False, False)):
        monkeypatch.setattr(AG, "SAVE_ACTIVATIONS", acts)
        monkeypatch.setattr(AG, "SAVE_ATTENTION", attn)
        xd = x.to(dev).requires_grad_()
        out = block_apply(blk, xd, T, temb.to(dev), (i["rope"][0].to(dev), i["rope"][1].to(dev)))
        out.backward(dout.to(dev))
        res.append((out.detach(), xd.grad))
    for o1, gx1 in res[:-1]:
        assert torch.equal(o1, res[-1][0]) and torch.equal(gx1, res[-1][1])
    assert float(res[0][1].float().abs().max()) > 0


@pytest.mark.parametrize("wo_text", [False, True], ids=["text", "wo_text"])
def test_branch_gradients_through_frozen_transformer(wo_text):
    """The training step (train_cogvideox_inpainting_i2v_video.py:1856-1892): branch (trainable) -> samples injected
    into the frozen transformer under the mask -> output -> backward.  Every branch parameter gradient.  wo_text:
    the script's --wo_text (:556-558, passed at :1403 and :1864), the branch's blocks on the video tokens alone."""
    from oracle import cogvideox_oracle as O
    from videopainter_amd.config import full_config
    tr, br, tsd, bsd = _models(wo_text=wo_text)
    i = tiny_inputs()
    g = torch.Generator().manual_seed(6)
    R = torch.randn(i["video"].shape, generator=g).bfloat16()
    samples = br(hidden_states=i["video"].to(dev).bfloat16(), encoder_hidden_states=i["enc"].to(dev).bfloat16(),
                 branch_cond=i["branch_cond"].to(dev).bfloat16(), timestep=i["timestep"].to(dev),
                 image_rotary_emb=i["rope"], wo_text=wo_text, return_dict=False)[0]
    out = tr(hidden_states=i["hidden"].to(dev).bfloat16(), encoder_hidden_states=i["enc"].to(dev).bfloat16(),
             timestep=i["timestep"].to(dev), image_rotary_emb=i["rope"], branch_block_samples=samples,
             branch_block_masks=i["mask"].to(dev), return_dict=False)[0]
    assert out.requires_grad
    out.backward(R.to(dev))
    trainable = [n for n, _ in br.named_parameters()]
    ours = {n: p.grad for n, p in br.named_parameters()}
    assert all(p.grad is None for p in tr.parameters())

    def oracle(dtype):
        tp = {k: torch.from_numpy(v).to(dtype) for k, v in tsd.items()}
        bp = {k: torch.from_numpy(v).to(dtype).requires_grad_(k in trainable) for k, v in bsd.items()}
        s = O.branch_forward(bp, full_config(TINY_BRANCH_CFG, True), i["video"].to(dtype), i["enc"].to(dtype),
                             i["branch_cond"].to(dtype), i["timestep"], i["rope"], wo_text=wo_text)
        o = O.transformer_forward(tp, full_config(TINY_CFG), i["hidden"].to(dtype), i["enc"].to(dtype),
                                  i["timestep"], i["rope"], branch_block_samples=s,
                                  branch_block_masks=i["mask"].to(dtype))[0]
        o.backward(R.to(dtype))
        return o.detach(), {k: bp[k].grad for k in trainable}

    o32, gp32 = oracle(torch.float32)
    o16, gp16 = oracle(torch.bfloat16)
    _check("output", out.detach(), o32, o16)
    used = [n for n in trainable if gp32[n] is not None]
    # the branch's norm_final / norm_out / proj_out / branch_x_embedder exist but are not on its forward path
    assert sorted(n for n in trainable if ours[n] is None) == sorted(n for n in trainable if gp32[n] is None)
    assert any(n.startswith("time_embedding") for n in used) and any(n.startswith("patch_embed") for n in used)
    for n in used:
        _check(n, ours[n], gp32[n], gp16[n])


def _resample_mask(T, tok_mask):
    m = torch.zeros(tok_mask.shape[0], T + tok_mask.shape[1], dtype=torch.bool)
    m[:, T:] = tok_mask.bool()
    return m


def test_resample_block_backward_matches_oracle():
    """One block with the ID-resample processor (window 0: attention over [K; LN(mask . k) + RoPE], [V; mask . v],
    attention_processor.py:2223-2304), every parameter trainable: d x, d temb and every parameter gradient (the
    norm_k affine gets the null keys' share) against the oracle's autograd (attn_resample)."""
    from oracle import cogvideox_oracle as O
    from videopainter_amd import CogVideoXTransformer3DModel, device_scope
    from videopainter_amd.autograd import block_apply
    from videopainter_amd.config import full_config
    tsd, _ = tiny_weights()
    with device_scope(dev):
        tr = CogVideoXTransformer3DModel(**dict(TINY_CFG, id_pool_resample_learnable=True))
    tr.load_diffusers_state_dict({k: torch.from_numpy(v) for k, v in tsd.items()})
    cfg = dict(full_config(TINY_CFG), id_pool_resample_learnable=True)
    i = tiny_inputs()
    T = i["enc"].shape[1]
    D = 128
    Nv = i["rope"][0].shape[0]
    g = torch.Generator().manual_seed(15)
    x = torch.randn(2, T + Nv, D, generator=g).bfloat16()
    temb = torch.randn(2, TINY_CFG["time_embed_dim"], generator=g).bfloat16()
    dout = torch.randn(2, T + Nv, D, generator=g).bfloat16()
    tm = (torch.rand(2, Nv, generator=g) < 0.4)
    rm = _resample_mask(T, tm)
    blk = tr.transformer_blocks[0]
    blk.requires_grad_(True)
    xd = x.to(dev).requires_grad_()
    td = temb.to(dev).requires_grad_()
    out = block_apply(blk, xd, T, td, (i["rope"][0].to(dev), i["rope"][1].to(dev)),
                      resample_mask=rm.to(dev).to(torch.uint8))
    out.backward(dout.to(dev))
    names = [n for n, _ in blk.named_parameters()]
    ours = {n: p.grad for n, p in blk.named_parameters()}

    def oracle(dtype):
        sd = {k[len("transformer_blocks.0."):]: torch.from_numpy(v).to(dtype).requires_grad_()
              for k, v in tsd.items() if k.startswith("transformer_blocks.0.")}
        xo = x.to(dtype).requires_grad_()
        to = temb.to(dtype).requires_grad_()
        h, e = O.block_forward({f"b.{k}": v for k, v in sd.items()}, "b", cfg, xo[:, T:], xo[:, :T], to,
                               i["rope"], resample_mask=rm.to(dtype), resample=True)
        torch.cat([e, h], 1).backward(dout.to(dtype))
        return xo.grad, to.grad, {k: sd[k].grad for k in names}

    gx32, gt32, gp32 = oracle(torch.float32)
    gx16, gt16, gp16 = oracle(torch.bfloat16)
    _check("dx", xd.grad, gx32, gx16)
    _check("dtemb", td.grad, gt32, gt16)
    for n in names:
        _check(n, ours[n], gp32[n], gp16[n])


def test_resample_lora_training_step_matches_oracle():
    """VideoPainterID's training step (train/train_cogvideox_inpainting_i2v_video_resample.py:1520-1526, 1940-1961):
    LoRA (r 4, alpha 8) added on to_q / to_k / to_v / to_out.0 of the frozen transformer, resample processor
    (id_pool_resample_learnable, window 0), frozen branch samples injected under the mask, backward of a random
    cotangent: the output and every LoRA factor's gradient against the oracle's autograd of
    W = W0 + (alpha / r) B A (our adapters run unfused: the projections on K-augmented operands).  Then an in-place
    update of the factors (what the optimizer step does) reaches the next forward through the rebuilt operands."""
    from oracle import cogvideox_oracle as O
    from videopainter_amd.config import full_config
    from videopainter_amd import CogVideoXTransformer3DModel, device_scope
    _, br, tsd, bsd = _models(train_branch=False)
    with device_scope(dev):
        tr = CogVideoXTransformer3DModel(**dict(TINY_CFG, id_pool_resample_learnable=True))
    tr.load_diffusers_state_dict({k: torch.from_numpy(v) for k, v in tsd.items()})
    tr.add_adapter({"r": 4, "lora_alpha": 8, "init_lora_weights": True,
                    "target_modules": ["to_q", "to_k", "to_v", "to_out.0"]})
    trainable = [n for n, p in tr.named_parameters() if p.requires_grad]
    assert trainable and all(".lora_A.weight" in n or ".lora_B.weight" in n for n in trainable)
    assert len(trainable) == 2 * 4 * TINY_CFG["num_layers"]
    g = torch.Generator().manual_seed(7)
    facs = {}
    with torch.no_grad():  # PEFT starts B at 0 (dA = 0): a trained-looking pair instead
        for n, p in tr.named_parameters():
            if p.requires_grad:
                p.copy_(torch.randn(p.shape, generator=g) * 0.05)
                facs[n] = p.detach().float().cpu()
    i = tiny_inputs()
    R = torch.randn(i["video"].shape, generator=g).bfloat16()
    samples = br(hidden_states=i["video"].to(dev).bfloat16(), encoder_hidden_states=i["enc"].to(dev).bfloat16(),
                 branch_cond=i["branch_cond"].to(dev).bfloat16(), timestep=i["timestep"].to(dev),
                 image_rotary_emb=i["rope"], return_dict=False)[0]
    out = tr(hidden_states=i["hidden"].to(dev).bfloat16(), encoder_hidden_states=i["enc"].to(dev).bfloat16(),
             timestep=i["timestep"].to(dev), image_rotary_emb=i["rope"], branch_block_samples=samples,
             branch_block_masks=i["mask"].to(dev), id_pool_resample_learnable=True, return_dict=False)[0]
    assert out.requires_grad
    out.backward(R.to(dev))
    ours = {n: p.grad for n, p in tr.named_parameters() if p.requires_grad}

    def oracle(dtype, factors, grad=True):
        tp = {k: torch.from_numpy(v).to(dtype) for k, v in tsd.items()}
        leaves = {n: v.detach().clone().to(dtype).requires_grad_(grad) for n, v in factors.items()}
        for n in leaves:
            if n.endswith(".lora_A.weight"):
                mod = n[:-len(".lora_A.weight")]
                tp[mod + ".weight"] = tp[mod + ".weight"] + 2.0 * (leaves[mod + ".lora_B.weight"] @ leaves[n])
        bp = {k: torch.from_numpy(v).to(dtype) for k, v in bsd.items()}
        s = O.branch_forward(bp, full_config(TINY_BRANCH_CFG, True), i["video"].to(dtype), i["enc"].to(dtype),
                             i["branch_cond"].to(dtype), i["timestep"], i["rope"])
        o = O.transformer_forward(tp, dict(full_config(TINY_CFG), id_pool_resample_learnable=True),
                                  i["hidden"].to(dtype), i["enc"].to(dtype), i["timestep"], i["rope"],
                                  branch_block_samples=s, branch_block_masks=i["mask"].to(dtype),
                                  id_pool_resample_learnable=True)[0]
        if grad:
            o.backward(R.to(dtype))
        return o.detach(), {n: leaves[n].grad for n in leaves}

    missing = [n for n in trainable if ours[n] is None]
    assert not missing, (missing, [n for n in trainable if ours[n] is not None][:4])
    o32, gp32 = oracle(torch.float32, facs)
    o16, gp16 = oracle(torch.bfloat16, facs)
    _check("output", out.detach(), o32, o16)
    for n in trainable:
        _check(n, ours[n], gp32[n], gp16[n])

    # the optimizer step updates the factors in place: the next forward runs on the re-folded weights
    with torch.no_grad():
        for n, p in tr.named_parameters():
            if p.requires_grad:
                p.add_(-0.5 * p.grad)
                facs[n] = p.detach().float().cpu()
    with torch.no_grad():
        out2 = tr(hidden_states=i["hidden"].to(dev).bfloat16(), encoder_hidden_states=i["enc"].to(dev).bfloat16(),
                  timestep=i["timestep"].to(dev), image_rotary_emb=i["rope"], branch_block_samples=samples,
                  branch_block_masks=i["mask"].to(dev), id_pool_resample_learnable=True, return_dict=False)[0]
    o2_32 = oracle(torch.float32, facs, grad=False)[0]
    o2_16 = oracle(torch.bfloat16, facs, grad=False)[0]
    _check("output after the factor update", out2, o2_32, o2_16)


def test_unfused_lora_keeps_a_sub_ulp_factor_update():
    """PEFT applies a trainable adapter unfused (y = x W0^T + s (x A^T) B^T), so a factor update far below a bf16
    ulp of W0 still moves the projection.  Weights of magnitude 1 (ulp 2^-7) with s B A = 2e-3 per element: folding
    would leave W0 bit-identical (the update is < half an ulp), while the augmented GEMM adds the delta
    s (x A^T) B^T (~0.25, several output ulps) in fp32.  q / k / v of the fused QKV and to_out.0 against fp32."""
    from videopainter_amd import CogVideoXTransformer3DModel, device_scope
    from videopainter_amd.attention_processor import _qkv, project_out
    with device_scope(dev):
        tr = CogVideoXTransformer3DModel(**TINY_CFG)
    tr.init_synthetic_weights_(5)
    tr.add_adapter({"r": 4, "lora_alpha": 8, "target_modules": ["to_q", "to_k", "to_v", "to_out.0"]})
    a = tr.transformer_blocks[0].attn1
    g = torch.Generator().manual_seed(11)
    lins = (a.to_q, a.to_k, a.to_v, a.to_out[0])
    D = a.to_q.weight.shape[1]
    sgn = torch.where(torch.rand(D, generator=g) < 0.5, -1.0, 1.0)
    with torch.no_grad():
        for l in lins:
            l.weight.copy_(torch.where(torch.rand(l.weight.shape, generator=g) < 0.5, -1.0, 1.0))
            l.bias.zero_()
            A = torch.zeros_like(l.lora_A.weight, device="cpu")
            A[0] = sgn
            l.lora_A.weight.copy_(A)
            l.lora_B.weight.fill_(1e-3)   # s B A = 2 * 1e-3 * (+-1): a quarter of W0's ulp
    x = (sgn[None, :] * (0.5 + torch.rand(64, D, generator=g))).to(torch.bfloat16)

    def want(l):
        xf = x.float()
        return xf @ l.weight.float().cpu().t() + 2.0 * (xf @ l.lora_A.weight.float().cpu().t()) @ \
            l.lora_B.weight.float().cpu().t()

    q = _qkv(a, x.view(1, 64, D).to(dev)).view(64, 3, -1)
    o = torch.empty(64, a.to_out[0].weight.shape[0], device=dev, dtype=torch.bfloat16)
    project_out(a.to_out[0], x.to(dev), o)
    torch.cuda.synchronize()
    for got, l in ((q[:, 0], a.to_q), (q[:, 1], a.to_k), (q[:, 2], a.to_v), (o, a.to_out[0])):
        w = want(l)
        base = x.float() @ l.weight.float().cpu().t()
        delta = (w - base).abs().mean().item()
        assert delta > 0.2, delta
        err = (got.float().cpu() - w).abs()
        # bf16 output rounding (relative 2^-9) plus the bf16 T = x A^T and s B: far below the delta a fold loses
        assert bool((err <= w.abs() * 2.0 ** -8 + 0.01).all()), err.max().item()
        assert err.mean().item() < 0.25 * delta, (err.mean().item(), delta)
        assert ((got.float().cpu() - base).abs().mean().item()) > 0.5 * delta
