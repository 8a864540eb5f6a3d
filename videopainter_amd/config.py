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


# `AutoencoderKLCogVideoX.__init__` DF/models/autoencoders/autoencoder_kl_cogvideox.py:921-954 (CogVideoX-5b's
# checkpoint overrides scaling_factor = 0.7)
VAE_DEFAULTS = dict(
    in_channels=3, out_channels=3,
    down_block_types=("CogVideoXDownBlock3D",) * 4, up_block_types=("CogVideoXUpBlock3D",) * 4,
    block_out_channels=(128, 256, 256, 512), latent_channels=16, layers_per_block=3, act_fn="silu", norm_eps=1e-6,
    norm_num_groups=32, temporal_compression_ratio=4, sample_height=480, sample_width=720, scaling_factor=1.15258426,
    shift_factor=None, latents_mean=None, latents_std=None, force_upcast=True, use_quant_conv=False,
    use_post_quant_conv=False,
)


def full_vae_config(kwargs: dict) -> dict:
    base = dict(VAE_DEFAULTS)
    unknown = set(kwargs) - set(base) - {"_class_name", "_diffusers_version", "_name_or_path"}
    if unknown:
        raise TypeError(f"unexpected VAE config keys: {sorted(unknown)}")
    base.update({k: v for k, v in kwargs.items() if not k.startswith("_")})
    base["block_out_channels"] = tuple(base["block_out_channels"])
    return base


def _vae_resnet_shapes(s: dict, p: str, cin: int, cout: int, zq: int = 0) -> None:
    """`CogVideoXResnetBlock3D` :218-275 with temb_channels = 0 (no temb_proj) and the 1x1x1 SafeConv3d shortcut."""
    def norm(n, c):
        if zq:  # CogVideoXSpatialNorm3D :164-173
            s[f"{p}.{n}.norm_layer.weight"] = (c,)
            s[f"{p}.{n}.norm_layer.bias"] = (c,)
            for cv in ("conv_y", "conv_b"):
                s[f"{p}.{n}.{cv}.conv.weight"] = (c, zq, 1, 1, 1)
                s[f"{p}.{n}.{cv}.conv.bias"] = (c,)
        else:
            s[f"{p}.{n}.weight"] = (c,)
            s[f"{p}.{n}.bias"] = (c,)
    norm("norm1", cin)
    norm("norm2", cout)
    s[f"{p}.conv1.conv.weight"] = (cout, cin, 3, 3, 3)
    s[f"{p}.conv1.conv.bias"] = (cout,)
    s[f"{p}.conv2.conv.weight"] = (cout, cout, 3, 3, 3)
    s[f"{p}.conv2.conv.bias"] = (cout,)
    if cin != cout:
        s[f"{p}.conv_shortcut.weight"] = (cout, cin, 1, 1, 1)
        s[f"{p}.conv_shortcut.bias"] = (cout,)


def vae_state_dict_shapes(cfg: dict) -> Dict[str, Tuple[int, ...]]:
    """State-dict keys / shapes of `AutoencoderKLCogVideoX` (encoder :635-704, decoder :769-845), registration order."""
    ch = list(cfg["block_out_channels"])
    nb, L, lpb = len(ch), cfg["latent_channels"], cfg["layers_per_block"]
    s: Dict[str, Tuple[int, ...]] = {}
    s["encoder.conv_in.conv.weight"] = (ch[0], cfg["in_channels"], 3, 3, 3)
    s["encoder.conv_in.conv.bias"] = (ch[0],)
    cout = ch[0]
    for i in range(nb):
        cin, cout = cout, ch[i]
        for j in range(lpb):
            _vae_resnet_shapes(s, f"encoder.down_blocks.{i}.resnets.{j}", cin if j == 0 else cout, cout)
        if i < nb - 1:
            s[f"encoder.down_blocks.{i}.downsamplers.0.conv.weight"] = (cout, cout, 3, 3)
            s[f"encoder.down_blocks.{i}.downsamplers.0.conv.bias"] = (cout,)
    for j in range(2):
        _vae_resnet_shapes(s, f"encoder.mid_block.resnets.{j}", ch[-1], ch[-1])
    s["encoder.norm_out.weight"] = (ch[-1],)
    s["encoder.norm_out.bias"] = (ch[-1],)
    s["encoder.conv_out.conv.weight"] = (2 * L, ch[-1], 3, 3, 3)
    s["encoder.conv_out.conv.bias"] = (2 * L,)
    rch = ch[::-1]
    s["decoder.conv_in.conv.weight"] = (rch[0], L, 3, 3, 3)
    s["decoder.conv_in.conv.bias"] = (rch[0],)
    for j in range(2):
        _vae_resnet_shapes(s, f"decoder.mid_block.resnets.{j}", rch[0], rch[0], zq=L)
    cout = rch[0]
    for i in range(nb):
        cin, cout = cout, rch[i]
        for j in range(lpb + 1):
            _vae_resnet_shapes(s, f"decoder.up_blocks.{i}.resnets.{j}", cin if j == 0 else cout, cout, zq=L)
        if i < nb - 1:
            s[f"decoder.up_blocks.{i}.upsamplers.0.conv.weight"] = (cout, cout, 3, 3)
            s[f"decoder.up_blocks.{i}.upsamplers.0.conv.bias"] = (cout,)
    s["decoder.norm_out.norm_layer.weight"] = (rch[-1],)
    s["decoder.norm_out.norm_layer.bias"] = (rch[-1],)
    for cv in ("conv_y", "conv_b"):
        s[f"decoder.norm_out.{cv}.conv.weight"] = (rch[-1], L, 1, 1, 1)
        s[f"decoder.norm_out.{cv}.conv.bias"] = (rch[-1],)
    s["decoder.conv_out.conv.weight"] = (cfg["out_channels"], rch[-1], 3, 3, 3)
    s["decoder.conv_out.conv.bias"] = (cfg["out_channels"],)
    # (:979-980: 1x1x1 SafeConv3d with out_channels-based widths, registered after the decoder)
    oc = cfg["out_channels"]
    if cfg.get("use_quant_conv"):
        s["quant_conv.weight"] = (2 * oc, 2 * oc, 1, 1, 1)
        s["quant_conv.bias"] = (2 * oc,)
    if cfg.get("use_post_quant_conv"):
        s["post_quant_conv.weight"] = (oc, oc, 1, 1, 1)
        s["post_quant_conv.bias"] = (oc,)
    return s


def config_signature_check(cls, cfg: dict) -> None:
    sig = inspect.signature(cls.__init__)
    for k in cfg:
        if k not in sig.parameters:
            raise TypeError(f"{cls.__name__} got unexpected config key {k}")


# T5 v1.1 encoder config fields (transformers T5Config) — defaults = CogVideoX's text encoder, google t5-v1_1-xxl
T5_DEFAULTS = dict(
    vocab_size=32128, d_model=4096, d_kv=64, d_ff=10240, num_layers=24, num_decoder_layers=24, num_heads=64,
    relative_attention_num_buckets=32, relative_attention_max_distance=128, dropout_rate=0.1,
    layer_norm_epsilon=1e-6, initializer_factor=1.0, feed_forward_proj="gated-gelu", is_encoder_decoder=True,
    use_cache=True, pad_token_id=0, eos_token_id=1, decoder_start_token_id=0, tie_word_embeddings=False,
    classifier_dropout=0.0, dense_act_fn="gelu_new", is_gated_act=True,
)


def full_t5_config(kwargs: dict) -> dict:
    base = dict(T5_DEFAULTS)
    base.update({k: v for k, v in kwargs.items() if not k.startswith("_")})
    ff = base["feed_forward_proj"].split("-")
    base["is_gated_act"] = ff[0] == "gated"
    base["dense_act_fn"] = "gelu_new" if ff[-1] == "gelu" else ff[-1]
    return base


def t5_state_dict_shapes(cfg: dict) -> Dict[str, Tuple[int, ...]]:
    """`T5EncoderModel.state_dict()` keys / shapes (gated FF: wi_0 / wi_1; the relative bias lives in block 0)."""
    D, inner, F = cfg["d_model"], cfg["num_heads"] * cfg["d_kv"], cfg["d_ff"]
    s: Dict[str, Tuple[int, ...]] = {"shared.weight": (cfg["vocab_size"], D),
                                     "encoder.embed_tokens.weight": (cfg["vocab_size"], D)}
    for i in range(cfg["num_layers"]):
        p = f"encoder.block.{i}.layer"
        for n in ("q", "k", "v"):
            s[f"{p}.0.SelfAttention.{n}.weight"] = (inner, D)
        s[f"{p}.0.SelfAttention.o.weight"] = (D, inner)
        if i == 0:
            s[f"{p}.0.SelfAttention.relative_attention_bias.weight"] = (cfg["relative_attention_num_buckets"],
                                                                         cfg["num_heads"])
        s[f"{p}.0.layer_norm.weight"] = (D,)
        if cfg["is_gated_act"]:
            s[f"{p}.1.DenseReluDense.wi_0.weight"] = (F, D)
            s[f"{p}.1.DenseReluDense.wi_1.weight"] = (F, D)
        else:
            s[f"{p}.1.DenseReluDense.wi.weight"] = (F, D)
        s[f"{p}.1.DenseReluDense.wo.weight"] = (D, F)
        s[f"{p}.1.layer_norm.weight"] = (D,)
    s["encoder.final_layer_norm.weight"] = (D,)
    return s
