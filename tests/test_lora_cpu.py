"""Load-time LoRA folding (videopainter_amd/lora.py), CPU only.

The reference applies the VideoPainterID adapter unfused through PEFT (not installed here, so its forward cannot be
run: parity against PEFT itself is unpinned).  What is checked: the fold equals the LoRA forward it replaces,
W x + s B (A x) with s = lora_scale (the CogVideoX loader's alpha = r) or alpha / r * lora_scale for kohya files;
keys in the pipeline-level format ("transformer." prefix, PEFT "lora_A"/"lora_B"); unknown modules are rejected;
fold + unfold restores the weights up to bf16 rounding."""
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
def test_runtime_scale_refold_is_exact(tmp_path, fmt):
    """attention_kwargs["scale"] per call (reference cogvideox_transformer_3d.py:490-499): the model keeps the base
    weights of the adapted layers, so folding at another scale equals folding that scale from scratch, bit for bit,
    in any order of scales."""
    from videopainter_amd.lora import fold_lora_
    sd = _adapter(_model(), 8, 4.0 if fmt == "kohya" else None)
    save_file(sd, os.path.join(tmp_path, "pytorch_lora_weights.safetensors"))

    def fresh(scale):
        m = _model()
        fold_lora_(m, sd, scale)
        return m.state_dict()

    m = _model()
    m.load_lora_weights(str(tmp_path), lora_scale=0.5, adapter_name="test_1")
    assert m.get_list_adapters() == ["test_1"]
    for scale in (0.5, 1.0, 0.25, 1.0, 0.5):
        m.set_lora_scale(scale)
        want = fresh(scale)
        assert all(torch.equal(v, want[k]) for k, v in m.state_dict().items()), scale
    with pytest.raises(ValueError, match="already loaded"):
        m.load_lora_weights(str(tmp_path), adapter_name="test_1")


def test_set_adapters_weights_and_fuse(tmp_path):
    """set_adapters(names, weights) scales each folded adapter (others off); fuse_lora pins the folded scale."""
    from videopainter_amd.lora import fold_lora_
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
    m.set_adapters(["two"], [0.5])
    want = _model()
    fold_lora_(want, sd2, 0.5)
    assert all(torch.equal(a, b) for a, b in zip(m.state_dict().values(), want.state_dict().values()))
    m.fuse_lora(lora_scale=2.0)   # pinned: 2.0 * 0.5 on adapter two
    m._call_lora_scale({"scale": 1.0})
    want = _model()
    fold_lora_(want, sd2, 1.0)
    assert all(torch.equal(a, b) for a, b in zip(m.state_dict().values(), want.state_dict().values()))


def test_trainable_adapter_runs_unfused_on_augmented_operands():
    """add_adapter (PEFT's LoraConfig on to_q/k/v/out.0): factors under PEFT's saved names, base frozen, B = 0; the
    adapter is never folded (W stays W0 after a factor update: the delta is added in output space, as PEFT's
    unfused forward does); the projection's K-augmented operands [x | x A^T] x [W0 | s B]^T equal
    x W0^T + s (x A^T) B^T, with the factors of q / k / v in their own rank blocks."""
    import torch
    from videopainter_amd import CogVideoXTransformer3DModel
    from videopainter_amd.lora import AUG_ALIGN, AugmentedProjection, trainable_pair
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
    assert aug.R == 12 and aug.Rp == AUG_ALIGN and aug.offs == [0, 4, 8]
    x = torch.randn(16, aug.K, generator=g)
    xa = torch.cat([x, x @ aug.a_cat().float().t()], 1)
    for l, w in zip((a.to_q, a.to_k, a.to_v), aug.weights()):
        assert w.shape == (l.weight.shape[0], aug.K + aug.Rp)
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
