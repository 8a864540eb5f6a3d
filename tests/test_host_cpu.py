"""Host-side logic on CPU (no GPU): configs/state-dict layout, checkpoint round trip, position tables and the
scheduler's host scalars against the oracle."""
import math
import os

import numpy as np
import pytest
import torch

from oracle import cogvideox_oracle as O
from tests.golden.cases import TINY_CFG, TINY_BRANCH_CFG, tiny_weights


def test_5b_i2v_state_dict_layout_on_meta():
    from videopainter_amd import CogVideoXTransformer3DModel, CogvideoXBranchModel, COGVIDEOX_5B_I2V, device_scope
    from videopainter_amd.config import full_config, state_dict_shapes
    with device_scope("meta"):
        tr = CogVideoXTransformer3DModel(**COGVIDEOX_5B_I2V)
        br = CogvideoXBranchModel(**dict(COGVIDEOX_5B_I2V, num_layers=2))
    for m, branch in ((tr, False), (br, True)):
        sd = m.state_dict()
        ref = state_dict_shapes(full_config(dict(m.config), branch), branch)
        assert list(sd) == list(ref)
        assert all(tuple(sd[k].shape) == ref[k] for k in ref)
    n = sum(p.numel() for p in tr.state_dict().values())
    assert abs(n - (5.570e9 + 54.6e6)) / 5.6e9 < 0.01  # SURVEY.md Appendix A (+ learned pos-emb buffer)


def test_checkpoint_round_trip_and_config_overrides(tmp_path):
    from videopainter_amd import CogVideoXTransformer3DModel, CogvideoXBranchModel
    tsd, bsd = tiny_weights()
    tr = CogVideoXTransformer3DModel(**TINY_CFG)
    tr.load_diffusers_state_dict({k: torch.from_numpy(v) for k, v in tsd.items()})
    tr.save_pretrained(str(tmp_path / "transformer"))
    tr2 = CogVideoXTransformer3DModel.from_pretrained(str(tmp_path), subfolder="transformer",
                                                      id_pool_resample_learnable=True)
    assert tr2.config.id_pool_resample_learnable is True
    assert all(torch.equal(a, b) for a, b in zip(tr.state_dict().values(), tr2.state_dict().values()))
    from videopainter_amd.attention_processor import CogVideoXAttnProcessor2_0_resample
    assert isinstance(tr2.transformer_blocks[0].attn1.processor, CogVideoXAttnProcessor2_0_resample)
    br = CogvideoXBranchModel.from_transformer(tr, num_layers=2, attention_head_dim=64, num_attention_heads=2)
    w = br.patch_embed.proj.weight
    assert w.shape[1] == 33
    assert torch.equal(w[:, :16], tr.patch_embed.proj.weight[:, :16]) and torch.equal(w[:, 16:32], w[:, :16])
    assert float(w[:, 32:].abs().max()) == 0.0
    assert float(br.branch_blocks[0].weight.abs().max()) == 0.0  # zero_module
    with pytest.raises(ValueError):
        CogVideoXTransformer3DModel(**dict(TINY_CFG, use_rotary_positional_embeddings=False))


def test_from_transformer_initialises_uncopied_parameters_and_rejects_shape_mismatch():
    """branch_cogvideox.py:255-293: parameters the reference never copies (text_proj, norms, head) keep PyTorch's
    default init (finite, Linear U(+-1/sqrt(fan_in)), LayerNorm 1/0), and load_state_dict(strict=False) raises on a
    size mismatch (the default attention_head_dim=128 against a 64-dim transformer)."""
    from videopainter_amd import CogVideoXTransformer3DModel, CogvideoXBranchModel
    tsd, _ = tiny_weights()
    tr = CogVideoXTransformer3DModel(**TINY_CFG)
    tr.load_diffusers_state_dict({k: torch.from_numpy(v) for k, v in tsd.items()})
    br = CogvideoXBranchModel.from_transformer(tr, num_layers=2, attention_head_dim=64, num_attention_heads=2)
    for k, v in br.state_dict().items():
        assert torch.isfinite(v.float()).all(), k
    tp = br.patch_embed.text_proj.weight.float()
    bound = 1.0 / tp.shape[1] ** 0.5
    assert 0.0 < float(tp.abs().max()) <= bound * 1.01
    assert float(tp.std()) > 0.3 * bound
    assert torch.equal(br.norm_final.weight.float(), torch.ones_like(br.norm_final.weight.float()))
    assert float(br.branch_x_embedder.weight.abs().max()) == 0.0
    assert torch.equal(br.transformer_blocks[1].attn1.to_q.weight, tr.transformer_blocks[1].attn1.to_q.weight)
    with pytest.raises(RuntimeError, match="size mismatch"):
        CogvideoXBranchModel.from_transformer(tr, num_layers=2, attention_head_dim=128, num_attention_heads=1)


def test_rope_and_sincos_tables_match_oracle():
    from videopainter_amd.embeddings import prepare_rotary_positional_embeddings, joint_sincos_pos_embedding
    for (h, w, f) in ((480, 720, 13), (256, 384, 3), (720, 1280, 13)):
        c1, s1 = prepare_rotary_positional_embeddings(h, w, f, 64)
        c2, s2 = O.prepare_rotary_positional_embeddings(h, w, f, 64)
        assert torch.equal(c1, c2) and torch.equal(s1, s2)
    cfg = dict(num_attention_heads=2, attention_head_dim=64, patch_size=2, max_text_seq_length=8,
               temporal_compression_ratio=4, spatial_interpolation_scale=1.875, temporal_interpolation_scale=1.0)
    a = joint_sincos_pos_embedding(128, 2, 8, 16, 24, 9)
    b = O.sincos_joint_pos_embedding(cfg, 16, 24, 9)
    assert torch.equal(a, b)


def test_scheduler_host_scalars_match_oracle():
    from videopainter_amd.scheduler import CogVideoXDPMScheduler
    s = CogVideoXDPMScheduler(snr_shift_scale=1.0, prediction_type="v_prediction", rescale_betas_zero_snr=True,
                              clip_sample=False, set_alpha_to_one=True, timestep_spacing="trailing")
    s.set_timesteps(50)
    o = O.DPMSchedulerOracle()
    o.set_timesteps(50)
    assert torch.equal(s.timesteps, o.timesteps)
    ts = [int(t) for t in s.timesteps]
    for i, t in enumerate(ts):
        c = s.coefficients(t, ts[i - 1] if i else None)
        r = o.coefficients(t, ts[i - 1] if i else None)
        for k in ("m1", "m2", "mn"):
            assert c[k] == float(r["mult" + k[1:]] if k != "mn" else r["mult_noise"])
    assert ts[0] == 999 and ts[-1] == 19


def test_dynamic_cfg_matches_reference_formula():
    g = O.dynamic_cfg_scale(6.0, 50, 999)
    assert math.isclose(g, 1 + 6.0 * ((1 - math.cos(math.pi * ((50 - 999) / 50) ** 5.0)) / 2))


def test_fuse_qkv_projections_is_a_documented_no_op():
    """cogvideox_transformer_3d.py:432-470: the drop-in's Q, K, V always run as one GEMM, so fuse / unfuse keep the
    weights and state-dict keys and restore the processors like the reference."""
    import torch
    from videopainter_amd import CogVideoXTransformer3DModel, CogvideoXBranchModel
    from tests.golden.cases import TINY_CFG, TINY_BRANCH_CFG
    for cls, cfg in ((CogVideoXTransformer3DModel, TINY_CFG), (CogvideoXBranchModel, TINY_BRANCH_CFG)):
        m = cls(**cfg)
        m.init_synthetic_weights_(3, host_exact=True)
        before = {k: v.clone() for k, v in m.state_dict().items()}
        procs = m.attn_processors
        m.fuse_qkv_projections()
        assert m.original_attn_processors == procs
        after = m.state_dict()
        assert list(after) == list(before) and all(torch.equal(after[k], before[k]) for k in before)
        m.unfuse_qkv_projections()
        assert m.attn_processors == procs


def test_branch_wo_text_construction():
    """wo_text (branch_cogvideox.py:74,123,263-269): the flag reaches the config and every block's processor, and
    from_transformer carries it; the forward's mode check runs before any device work."""
    import pytest
    import torch
    from videopainter_amd import CogVideoXTransformer3DModel, CogvideoXBranchModel
    from videopainter_amd.attention_processor import CogVideoXAttnProcessor2_0_wo_text
    from tests.golden.cases import TINY_CFG, TINY_BRANCH_CFG
    br = CogvideoXBranchModel(**dict(TINY_BRANCH_CFG, wo_text=True))
    assert br.config.wo_text is True and br.wo_text
    assert all(isinstance(b.attn1.processor, CogVideoXAttnProcessor2_0_wo_text) and b.wo_text
               for b in br.transformer_blocks)
    tr = CogVideoXTransformer3DModel(**TINY_CFG)
    tr.init_synthetic_weights_(2)
    b2 = CogvideoXBranchModel.from_transformer(tr, num_layers=2, attention_head_dim=64, num_attention_heads=2,
                                               wo_text=True)
    assert b2.config.wo_text is True and all(b.wo_text for b in b2.transformer_blocks)
    assert not any(b.wo_text for b in CogvideoXBranchModel(**TINY_BRANCH_CFG).transformer_blocks)
    x = torch.zeros(1, 3, 16, 16, 24)
    with pytest.raises(ValueError):
        b2(hidden_states=x, encoder_hidden_states=torch.zeros(1, 8, 32), branch_cond=torch.zeros(1, 3, 17, 16, 24),
           timestep=torch.tensor([10]), image_rotary_emb=None, wo_text=True)
