"""Model configs and state-dict layouts of the two model classes on the hot path.

Constructor kwargs mirror `@register_to_config` of the reference classes:
  `CogVideoXTransformer3DModel.__init__`  DF/models/transformers/cogvideox_transformer_3d.py:274-303
  `CogvideoXBranchModel.__init__`         DF/models/branch_cogvideox.py:46-76
State-dict keys/shapes follow SURVEY.md Appendix B (dumped from the reference).
"""
from __future__ import annotations

import inspect
from typing import Dict, Tuple

TRANSFORMER_DEFAULTS = dict(
    num_attention_heads=30, attention_head_dim=64, in_channels=16, out_channels=16, flip_sin_to_cos=True,
    freq_shift=0, time_embed_dim=512, text_embed_dim=4096, num_layers=30, dropout=0.0, attention_bias=True,
    sample_width=90, sample_height=60, sample_frames=49, patch_size=2, temporal_compression_ratio=4,
    max_text_seq_length=226, activation_fn="gelu-approximate", timestep_activation_fn="silu",
    norm_elementwise_affine=True, norm_eps=1e-5, spatial_interpolation_scale=1.875, temporal_interpolation_scale=1.0,
    use_rotary_positional_embeddings=False, use_learned_positional_embeddings=False, id_pool_resample_learnable=False,
)

BRANCH_DEFAULTS = dict(TRANSFORMER_DEFAULTS)
BRANCH_DEFAULTS["wo_text"] = False

# CogVideoX-5b-I2V (diffusers/scripts/convert_cogvideox_to_diffusers.py:147-153,205-209)
COGVIDEOX_5B_I2V = dict(
    num_attention_heads=48, attention_head_dim=64, in_channels=32, out_channels=16, time_embed_dim=512,
    text_embed_dim=4096, num_layers=42, use_rotary_positional_embeddings=True, use_learned_positional_embeddings=True,
    sample_height=60, sample_width=90, sample_frames=49, patch_size=2, max_text_seq_length=226,
)


def full_config(kwargs: dict, branch: bool = False) -> dict:
    base = dict(BRANCH_DEFAULTS if branch else TRANSFORMER_DEFAULTS)
    unknown = set(kwargs) - set(base) - {"_class_name", "_diffusers_version", "_name_or_path"}
    if unknown:
        raise TypeError(f"unexpected config keys: {sorted(unknown)}")
    base.update({k: v for k, v in kwargs.items() if not k.startswith("_")})
    return base


def patch_in_channels(cfg: dict, branch: bool) -> int:
    """Branch patch embed sees noisy latents + masked latents + mask (branch_cogvideox.py:90)."""
    c = cfg["in_channels"]
    if not branch:
        return c
    return c * 2 + 1 if c == 16 else c + 1


def num_patches(cfg: dict) -> int:
    p = cfg["patch_size"]
    f = (cfg["sample_frames"] - 1) // cfg["temporal_compression_ratio"] + 1
    return (cfg["sample_height"] // p) * (cfg["sample_width"] // p) * f


def block_shapes(dim: int, temb: int, ff_mult: int = 4, prefix: str = "") -> Dict[str, Tuple[int, ...]]:
    s = {}
    s[prefix + "norm1.linear.weight"] = (6 * dim, temb)
    s[prefix + "norm1.linear.bias"] = (6 * dim,)
    s[prefix + "norm1.norm.weight"] = (dim,)
    s[prefix + "norm1.norm.bias"] = (dim,)
    for n in ("to_q", "to_k", "to_v", "to_out.0"):
        s[prefix + f"attn1.{n}.weight"] = (dim, dim)
        s[prefix + f"attn1.{n}.bias"] = (dim,)
    s[prefix + "norm2.linear.weight"] = (6 * dim, temb)
    s[prefix + "norm2.linear.bias"] = (6 * dim,)
    s[prefix + "norm2.norm.weight"] = (dim,)
    s[prefix + "norm2.norm.bias"] = (dim,)
    s[prefix + "ff.net.0.proj.weight"] = (ff_mult * dim, dim)
    s[prefix + "ff.net.0.proj.bias"] = (ff_mult * dim,)
    s[prefix + "ff.net.2.weight"] = (dim, ff_mult * dim)
    s[prefix + "ff.net.2.bias"] = (dim,)
    return s


def state_dict_shapes(cfg: dict, branch: bool = False) -> Dict[str, Tuple[int, ...]]:
    """Ordered like the reference's `state_dict()` (module registration order)."""
    d = cfg["num_attention_heads"] * cfg["attention_head_dim"]
    hd = cfg["attention_head_dim"]
    p = cfg["patch_size"]
    temb = cfg["time_embed_dim"]
    s: Dict[str, Tuple[int, ...]] = {}
    if cfg["use_learned_positional_embeddings"]:
        s["patch_embed.pos_embedding"] = (1, cfg["max_text_seq_length"] + num_patches(cfg), d)
    s["patch_embed.proj.weight"] = (d, patch_in_channels(cfg, branch), p, p)
    s["patch_embed.proj.bias"] = (d,)
    s["patch_embed.text_proj.weight"] = (d, cfg["text_embed_dim"])
    s["patch_embed.text_proj.bias"] = (d,)
    s["time_embedding.linear_1.weight"] = (temb, d)
    s["time_embedding.linear_1.bias"] = (temb,)
    s["time_embedding.linear_2.weight"] = (temb, temb)
    s["time_embedding.linear_2.bias"] = (temb,)
    for i in range(cfg["num_layers"]):
        bs = block_shapes(d, temb, prefix=f"transformer_blocks.{i}.")
        # insert qk-norm params in reference order (after norm1, before to_q)
        out = {}
        for k, v in bs.items():
            if k.endswith("attn1.to_q.weight"):
                out[f"transformer_blocks.{i}.attn1.norm_q.weight"] = (hd,)
                out[f"transformer_blocks.{i}.attn1.norm_q.bias"] = (hd,)
                out[f"transformer_blocks.{i}.attn1.norm_k.weight"] = (hd,)
                out[f"transformer_blocks.{i}.attn1.norm_k.bias"] = (hd,)
            out[k] = v
        s.update(out)
    s["norm_final.weight"] = (d,)
    s["norm_final.bias"] = (d,)
    s["norm_out.linear.weight"] = (2 * d, temb)
    s["norm_out.linear.bias"] = (2 * d,)
    s["norm_out.norm.weight"] = (d,)
    s["norm_out.norm.bias"] = (d,)
    s["proj_out.weight"] = (p * p * cfg["out_channels"], d)
    s["proj_out.bias"] = (p * p * cfg["out_channels"],)
    if branch:
        for j in range(cfg["num_layers"]):
            s[f"branch_blocks.{j}.weight"] = (d, d)
            s[f"branch_blocks.{j}.bias"] = (d,)
        s["branch_x_embedder.weight"] = (d, cfg["in_channels"])
        s["branch_x_embedder.bias"] = (d,)
    return s


def config_signature_check(cls, cfg: dict) -> None:
    sig = inspect.signature(cls.__init__)
    for k in cfg:
        if k not in sig.parameters:
            raise TypeError(f"{cls.__name__} got unexpected config key {k}")
