"""LoRA adapters (videopainter_amd/lora.py), CPU only.

The reference applies the VideoPainterID adapter unfused through PEFT (not installed here, so its forward cannot be
run: parity against PEFT itself is unpinned).  What is checked: loaded and trainable adapters run unfused on the
K-augmented operands (W0 untouched, the tail bf16(s B), s = lora_scale — the CogVideoX loader's alpha = r — or
alpha / r * lora_scale for kohya files); the explicit fold (fuse_lora / the stateless fold_lora_) equals the LoRA
forward it replaces, W x + s B (A x); keys in the pipeline-level format ("transformer." prefix, PEFT
"lora_A"/"lora_B"); unknown modules are rejected; fold + unfold restores the weights up to bf16 rounding."""
import os

import pytest
import torch
from safetensors.torch import save_file

from tests.golden.cases import TINY_CFG


def _model():
    from videopainter_amd import CogVideoXTransformer3DModel
    m = CogVideoXTransformer3DModel(**TINY_CFG)
    g = torch.Generator().manual_seed(0)
    with torch.no_grad():
        for p in m.parameters():
            p.copy_((torch.randn(p.shape, generator=g) * 0.05).to(p.dtype))
    return m


def _bf(sd):
    """The factors as the loader keeps them (the model dtype, as PEFT's injected LoRA layers hold them)."""
    return {k: (v if k.endswith(".alpha") else v.to(torch.bfloat16)) for k, v in sd.items()}


def _adapter(m, r=8, kohya_alpha=None, seed=1):
    g = torch.Generator().manual_seed(seed)
    sd = {}
    for i in range(len(m.transformer_blocks)):
        for t in ("to_q", "to_k", "to_v", "to_out.0"):
            lin = dict(m.named_modules())[f"transformer_blocks.{i}.attn1.{t}"]
            out_f, in_f = lin.weight.shape
            A = torch.randn(r, in_f, generator=g) * 0.1
            B = torch.randn(out_f, r, generator=g) * 0.1
            base = f"transformer.transformer_blocks.{i}.attn1.{t}"
            if kohya_alpha is None:
                sd[f"{base}.lora_A.weight"], sd[f"{base}.lora_B.weight"] = A, B
            else:
                sd[f"{base}.lora_down.weight"], sd[f"{base}.lora_up.weight"] = A, B
                sd[f"{base}.alpha"] = torch.tensor(float(kohya_alpha))
    return sd


@pytest.mark.parametrize("fmt", ["peft", "kohya"])
def test_fold_matches_lora_forward(tmp_path, fmt):
    from videopainter_amd.lora import load_lora_into_transformer
    m = _model()
    r, alpha, scale = 8, (4.0 if fmt == "kohya" else None), 0.7
    sd = _adapter(m, r, alpha)
    save_file(sd, os.path.join(tmp_path, "pytorch_lora_weights.safetensors"))
    lin = dict(m.named_modules())["transformer_blocks.1.attn1.to_k"]
    W0 = lin.weight.detach().float().clone()
    x = torch.randn(5, W0.shape[1])
    base = "transformer.transformer_blocks.1.attn1.to_k"
    A = sd[f"{base}.lora_A.weight" if fmt == "peft" else f"{base}.lora_down.weight"]
    B = sd[f"{base}.lora_B.weight" if fmt == "peft" else f"{base}.lora_up.weight"]
    s = scale * (alpha / r if alpha is not None else 1.0)
    want = x @ W0.T + s * (x @ A.T) @ B.T      # the unfused LoRA forward (PEFT: base + scaling * B(A x))
    n = load_lora_into_transformer(m, str(tmp_path), lora_scale=scale)
    assert n == 4 * len(m.transformer_blocks)
    got = x @ lin.weight.float().T
    assert torch.allclose(got, want, rtol=0, atol=2e-2 * float(want.abs().max()))  # bf16 weight rounding
    # every other parameter is untouched
    m2 = _model()
    for (k, a), (_, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        if not any(t in k for t in ("to_q", "to_k", "to_v", "to_out")) or k.endswith("bias"):
            assert torch.equal(a, b), k


def test_fold_unfold_roundtrip_and_rejects_unknown_modules():
    from videopainter_amd.lora import fold_lora_, unfold_lora_
    m = _model()
    W0 = {k: v.float().clone() for k, v in m.state_dict().items()}
    sd = _adapter(m)
    fold_lora_(m, sd)
    unfold_lora_(m, sd)
    for k, v in m.state_dict().items():
        assert torch.allclose(v.float(), W0[k], atol=2e-3), k
    bad = {"transformer.nope.lora_A.weight": torch.zeros(2, 4), "transformer.nope.lora_B.weight": torch.zeros(4, 2)}
    with pytest.raises(KeyError):
        fold_lora_(m, bad)
    assert fold_lora_(m, bad, strict=False) == 0
    half = {"transformer.transformer_blocks.0.attn1.to_q.lora_A.weight": torch.zeros(2, 128)}
    with pytest.raises(ValueError):
        fold_lora_(m, half)


@pytest.mark.parametrize("fmt", ["peft", "kohya"])
def test_loaded_adapter_runs_unfused_and_fuse_is_exact(tmp_path, fmt):
    """load_lora_weights keeps W0 (the adapter is applied unfused, as the reference's PEFT does,
    infer/inpaint.py:310-316): at every per-call scale (cogvideox_transformer_3d.py:490-499) the augmented weight
    tail is bf16(s B) with s = scale (x alpha / r for kohya files) while the state dict stays W0 bit for bit;
    fuse_lora(scale) equals a fresh fold at that scale bit for bit, and unfuse_lora restores W0 exactly."""
    from videopainter_amd.lora import AugmentedProjection, fold_lora_
    r, alpha = 8, (4.0 if fmt == "kohya" else None)
    sd = _adapter(_model(), r, alpha)
    save_file(sd, os.path.join(tmp_path, "pytorch_lora_weights.safetensors"))
    m = _model()
    w0 = {k: v.clone() for k, v in m.state_dict().items()}
    m.load_lora_weights(str(tmp_path), adapter_name="test_1")
    assert m.get_list_adapters() == ["test_1"]
    a = m.transformer_blocks[1].attn1
    for scale in (0.5, 1.0, 0.25, 1.0):
        m._call_lora_scale({"scale": scale})
        assert all(torch.equal(v, w0[k]) for k, v in m.state_dict().items()), scale
        aug = AugmentedProjection.of((a.to_q, a.to_k, a.to_v))
        s = scale * (alpha / r if alpha is not None else 1.0)
        for i, (lin, w) in enumerate(zip((a.to_q, a.to_k, a.to_v), aug.weights())):
            t = ("to_q", "to_k", "to_v")[i]
            base = f"transformer.transformer_blocks.1.attn1.{t}"
            B = sd[f"{base}.lora_B.weight" if alpha is None else f"{base}.lora_up.weight"]
            c0 = aug.block_col(i)
            assert torch.equal(w[:, :aug.K], lin.weight)
            assert torch.equal(w[:, c0:c0 + r], (B.to(torch.bfloat16).float() * s).to(torch.bfloat16))
            assert not w[:, aug.K:c0].any() and not w[:, c0 + r:].any()
    with pytest.raises(ValueError, match="already loaded"):
        m.load_lora_weights(str(tmp_path), adapter_name="test_1")
    m.fuse_lora(lora_scale=0.5)
    want = _model()
    fold_lora_(want, _bf(sd), 0.5)
    assert all(torch.equal(v, want.state_dict()[k]) for k, v in m.state_dict().items())
    assert AugmentedProjection.of((a.to_q,)) is None  # fused: nothing left to apply unfused
    m._call_lora_scale({"scale": 1.0})  # a fused adapter no longer follows the per-call scale
    assert all(torch.equal(v, want.state_dict()[k]) for k, v in m.state_dict().items())
    m.unfuse_lora()
    assert all(torch.equal(v, w0[k]) for k, v in m.state_dict().items())
    assert AugmentedProjection.of((a.to_q,)) is not None


def test_set_adapters_weights_and_fuse(tmp_path):
    """set_adapters(names, weights) weights each unfused adapter (the others off); fuse_lora pins the folded scale."""
    from videopainter_amd.lora import AugmentedProjection, fold_lora_, module_pairs
    g = torch.Generator().manual_seed(3)
    sd1, sd2 = _adapter(_model(), 8), _adapter(_model(), 4)
    for sd in (sd2,):
        for k in sd:
            sd[k] = torch.randn(sd[k].shape, generator=g) * 0.05
    save_file(sd1, os.path.join(tmp_path, "a1.safetensors"))
    save_file(sd2, os.path.join(tmp_path, "a2.safetensors"))
    m = _model()
    m.load_lora_weights(str(tmp_path), weight_name="a1.safetensors", adapter_name="one")
    m.load_lora_weights(str(tmp_path), weight_name="a2.safetensors", adapter_name="two")
    lin = m.transformer_blocks[0].attn1.to_v
    assert [A.shape[0] for A, _, _ in module_pairs(lin)] == [8, 4]
    aug = AugmentedProjection.of((lin,))
    assert aug.r == 64 and aug.weights()[0].shape == (lin.weight.shape[0], aug.K + 64)
    m.set_adapters(["two"], [0.5])
    ps = module_pairs(lin)
    assert len(ps) == 1 and ps[0][0].shape[0] == 4 and ps[0][2] == 0.5
    m.fuse_lora(lora_scale=2.0)   # pinned: 2.0 * 0.5 on adapter two
    m._call_lora_scale({"scale": 1.0})
    want = _model()
    fold_lora_(want, _bf(sd2), 1.0)
    assert all(torch.equal(a, b) for a, b in zip(m.state_dict().values(), want.state_dict().values()))


def test_uncovered_adapter_module_is_folded_and_follows_the_scale(tmp_path):
    """An adapter on a Linear the augmented GEMMs do not cover (here proj_out) is folded at load time from a kept
    base, exactly re-folded at each per-call scale; the attention projections of the same file stay unfused."""
    from videopainter_amd.lora import fold_lora_, module_pairs
    m = _model()
    g = torch.Generator().manual_seed(5)
    W = m.proj_out.weight
    sd = {"transformer.proj_out.lora_A.weight": torch.randn(4, W.shape[1], generator=g) * 0.1,
          "transformer.proj_out.lora_B.weight": torch.randn(W.shape[0], 4, generator=g) * 0.1,
          "transformer.transformer_blocks.0.attn1.to_q.lora_A.weight": torch.randn(4, 128, generator=g) * 0.1,
          "transformer.transformer_blocks.0.attn1.to_q.lora_B.weight": torch.randn(128, 4, generator=g) * 0.1}
    save_file(sd, os.path.join(tmp_path, "pytorch_lora_weights.safetensors"))
    w0 = m.transformer_blocks[0].attn1.to_q.weight.clone()
    m.load_lora_weights(str(tmp_path))
    assert torch.equal(m.transformer_blocks[0].attn1.to_q.weight, w0) and module_pairs(m.transformer_blocks[0].attn1.to_q)
    for scale in (1.0, 0.3):
        m._call_lora_scale({"scale": scale})
        want = _model()
        fold_lora_(want, _bf({k: v for k, v in sd.items() if "proj_out" in k}), scale)
        assert torch.equal(m.proj_out.weight, want.proj_out.weight), scale


def test_trainable_adapter_rejects_uncovered_targets_before_mutating():
    """a trainable factor on a Linear the augmented GEMMs do not cover would get no forward
    delta and no gradient, so add_adapter raises — before any factor, freeze or state is attached."""
    from videopainter_amd.lora import lora_state
    m = _model()
    before = {n: p.requires_grad for n, p in m.named_parameters()}
    with pytest.raises(ValueError, match="attention projections"):
        m.add_adapter({"r": 4, "lora_alpha": 4, "target_modules": ["to_q", "proj_out"]})
    assert {n: p.requires_grad for n, p in m.named_parameters()} == before
    assert not any(hasattr(l, "lora_A") for l in m.modules())
    st = lora_state(m)
    assert st is None or not st.adapters


def test_fp8_qkv_conflict_raises_before_mutating():
    """with the MX-FP8 QKV projection enabled, adding an unfused adapter on q / k / v raises up
    front (the fp8 GEMM has no augmented form), leaving the model as it was."""
    m = _model()
    blk = m.transformer_blocks[0]
    blk.qkv_mx = ("stub",)  # what enable_fp8_qkv(True) sets (its quantisation needs the GPU)
    with pytest.raises(NotImplementedError, match="fp8 QKV"):
        m.add_adapter({"r": 4, "lora_alpha": 4})
    assert not any(hasattr(l, "lora_A") for l in m.modules())


def test_trainable_adapter_runs_unfused_on_augmented_operands():
    """add_adapter (PEFT's LoraConfig on to_q/k/v/out.0): factors under PEFT's saved names, base frozen, B = 0; the
    adapter is never folded (W stays W0 after a factor update: the delta is added in output space, as PEFT's
    unfused forward does); segment i's K-augmented operands [x | x A_i^T] x [W0_i | s B_i]^T equal
    x W0_i^T + s (x A_i^T) B_i^T, each projection's factors in its own 64-padded rank block."""
    import torch
    from videopainter_amd import CogVideoXTransformer3DModel
    from videopainter_amd.lora import AugmentedProjection, trainable_pair
    from tests.golden.cases import TINY_CFG
    tr = CogVideoXTransformer3DModel(**TINY_CFG)
    tr.init_synthetic_weights_(3)
    w0 = {n: p.detach().clone() for n, p in tr.named_parameters()}
    tr.add_adapter({"r": 4, "lora_alpha": 8, "target_modules": ["to_q", "to_k", "to_v", "to_out.0"]})
    train = {n: p for n, p in tr.named_parameters() if p.requires_grad}
    L = TINY_CFG["num_layers"]
    assert len(train) == 8 * L
    assert set(tr.get_lora_state_dict()) == set(train)
    assert "transformer_blocks.0.attn1.to_out.0.lora_B.weight" in train
    a = tr.transformer_blocks[0].attn1
    lin = a.to_q
    assert lin.lora_A.weight.shape == (4, lin.weight.shape[1]) and lin.lora_B.weight.shape == (lin.weight.shape[0], 4)
    assert torch.count_nonzero(lin.lora_B.weight) == 0 and torch.count_nonzero(lin.lora_A.weight) > 0
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for l in (a.to_q, a.to_k, a.to_v):
            l.lora_B.weight.copy_(torch.randn(l.lora_B.weight.shape, generator=g) * 0.1)
    for n, p in tr.named_parameters():
        if n in w0:
            assert torch.equal(p, w0[n]), n   # never folded
    A, B, s = trainable_pair(lin)
    assert A is lin.lora_A.weight and B is lin.lora_B.weight and s == 2.0
    tr._call_lora_scale({"scale": 0.5})
    assert trainable_pair(lin)[2] == 1.0
    tr._call_lora_scale({"scale": 1.0})
    aug = AugmentedProjection.of((a.to_q, a.to_k, a.to_v))
    # 128-wide projections: narrower than a GEMM tile, so the block-diagonal form over the whole T
    assert aug.r == 64 and aug.R == 192 and aug.full and aug.tail is None
    x = torch.randn(16, aug.K, generator=g)
    T = x @ aug.a_cat().float().t()
    for i, (l, w) in enumerate(zip((a.to_q, a.to_k, a.to_v), aug.weights())):
        assert w.shape == (l.weight.shape[0], aug.K + aug.R)
        xa = torch.cat([x, T], 1)
        want = x @ l.weight.float().t() + 2.0 * (x @ l.lora_A.weight.float().t()) @ l.lora_B.weight.float().t()
        got = xa @ w.float().t()
        assert torch.allclose(got, want, rtol=2e-2, atol=2e-2), (got - want).abs().max()
    # an in-place factor update (the optimizer step) rebuilds the cached operands
    w_before = aug.weights()[0]
    with torch.no_grad():
        lin.lora_B.weight.add_(1.0)
    w_after = AugmentedProjection.of((a.to_q, a.to_k, a.to_v)).weights()[0]
    assert w_after is not w_before and not torch.equal(w_after, w_before)
    assert AugmentedProjection.of((tr.transformer_blocks[0].ff.net[0].proj,)) is None


def test_augmented_operands_with_the_per_segment_tail():
    """512-wide projections (8 heads): the per-segment A tail layout — W_aug_i = [W0_i | s B_i] (K + r columns),
    segment i reading rank block i of T (a_tail_off[i] = i r) — equals the unmerged LoRA of each projection; the
    prev-clip K/V group shares the fused QKV group's per-Linear weight cache."""
    from videopainter_amd import CogVideoXTransformer3DModel
    from videopainter_amd.lora import AugmentedProjection
    cfg = dict(TINY_CFG, num_attention_heads=8)  # 512-wide: K + r >= 8 K-tiles
    tr = CogVideoXTransformer3DModel(**cfg)
    tr.init_synthetic_weights_(4)
    tr.add_adapter({"r": 8, "lora_alpha": 4})
    a = tr.transformer_blocks[1].attn1
    g = torch.Generator().manual_seed(2)
    with torch.no_grad():
        for l in (a.to_q, a.to_k, a.to_v):
            l.lora_B.weight.copy_(torch.randn(l.lora_B.weight.shape, generator=g) * 0.1)
    aug = AugmentedProjection.of((a.to_q, a.to_k, a.to_v))
    assert not aug.full and aug.r == 64 and aug.tail == (aug.K, [0, 64, 128])
    assert AugmentedProjection.of((a.to_out[0],)).tail is None  # one projection: a plain GEMM on [x | T]
    x = torch.randn(8, aug.K, generator=g)
    T = x @ aug.a_cat().float().t()
    for i, (l, w) in enumerate(zip((a.to_q, a.to_k, a.to_v), aug.weights())):
        assert w.shape == (l.weight.shape[0], aug.K + aug.r)
        xa = torch.cat([x, T[:, i * 64:(i + 1) * 64]], 1)  # what segment i reads
        want = x @ l.weight.float().t() + 0.5 * (x @ l.lora_A.weight.float().t()) @ l.lora_B.weight.float().t()
        assert torch.allclose(xa @ w.float().t(), want, rtol=2e-2, atol=2e-2)
    assert AugmentedProjection.of((a.to_k, a.to_v)).weights()[0] is aug.weights()[1]


def test_augmented_rows_are_written_in_place():
    """lora.augmented_rows: with unfused adapters the producer's [B, N, K] output is the first K columns of the
    x_aug buffer, and AugmentedProjection.input finds that buffer (no copy of x); any other tensor — a plain one, a
    foreign [M, K + R] buffer, a buffer that was freed — takes the copying path."""
    import gc
    from videopainter_amd import CogVideoXTransformer3DModel
    from videopainter_amd.lora import AugmentedProjection, _AUG_BUFFERS, _augmented_base, augmented_rows
    tr = CogVideoXTransformer3DModel(**TINY_CFG)
    tr.init_synthetic_weights_(4)
    a = tr.transformer_blocks[0].attn1
    lins = (a.to_q, a.to_k, a.to_v)
    D = a.to_q.weight.shape[1]
    plain = augmented_rows(lins, 2, 3, D, "cpu")
    assert plain._base is None and plain.shape == (2, 3, D)  # no adapters: a plain tensor
    tr.add_adapter({"r": 8, "lora_alpha": 8})
    aug = AugmentedProjection.of(lins)
    xv = augmented_rows(lins, 2, 3, D, "cpu")
    assert xv.shape == (2, 3, D) and xv.stride() == (3 * (D + aug.R), D + aug.R, 1)
    base = _augmented_base(xv.view(6, D), 6, D + aug.R)
    assert base is not None and base.shape == (6, D + aug.R) and base.data_ptr() == xv.data_ptr()
    foreign = torch.empty(6, D + aug.R)
    assert _augmented_base(foreign[:, :D], 6, D + aug.R) is None
    assert _augmented_base(xv.view(6, D), 6, D + aug.R + 64) is None  # another projection group's width
    n = len(_AUG_BUFFERS)
    del xv, base
    gc.collect()
    assert len(_AUG_BUFFERS) == n - 1  # the registry forgets freed buffers
