"""CPU ORACLE for the T5 v1.1 encoder — TEST INFRASTRUCTURE ONLY (same rules as cogvideox_oracle.py: only tests/ and
the bench's CPU baseline may import it; the product path `videopainter_amd.t5` never does).

A functional plain-PyTorch restatement of transformers' `T5EncoderModel` (modeling_t5.py; the reference pins
transformers==4.42.2 in requirements.txt, this container has 5.15.0 — the encoder math is the same in both) as the
CogVideoX pipeline calls it (`_get_t5_prompt_embeds`, …_anyl.py:216-256: input ids only, no attention mask):
T5LayerNorm (RMS, fp32 statistics), T5Attention with the bucketed relative-position bias of layer 0 shared by every
layer and no 1/sqrt(d) scaling, T5DenseGatedActDense with gelu_new (tanh form), residual adds, final layer norm.
Pinned to transformers' own outputs by tests/golden/t5.safetensors (tests/test_oracle_golden.py).
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch

SD = Dict[str, torch.Tensor]


def relative_position_bucket(relative_position: torch.Tensor, num_buckets: int = 32, max_distance: int = 128):
    """`T5Attention._relative_position_bucket`, bidirectional (the encoder)."""
    num_buckets //= 2
    buckets = (relative_position > 0).to(torch.long) * num_buckets
    rp = torch.abs(relative_position)
    max_exact = num_buckets // 2
    is_small = rp < max_exact
    large = max_exact + (torch.log(rp.float() / max_exact) / math.log(max_distance / max_exact)
                         * (num_buckets - max_exact)).to(torch.long)
    large = torch.minimum(large, torch.full_like(large, num_buckets - 1))
    return buckets + torch.where(is_small, rp, large)


def bucket_matrix(L: int, num_buckets: int, max_distance: int) -> torch.Tensor:
    """[L, L] bucket of (query i, key j): relative position j - i (`compute_bias`)."""
    ctx = torch.arange(L, dtype=torch.long)[:, None]
    mem = torch.arange(L, dtype=torch.long)[None, :]
    return relative_position_bucket(mem - ctx, num_buckets, max_distance)


def rms_norm(x, w, eps):
    """`T5LayerNorm.forward`: fp32 variance, x * rsqrt, cast to the weight dtype when it is half precision."""
    var = x.to(torch.float32).pow(2).mean(-1, keepdim=True)
    x = x * torch.rsqrt(var + eps)
    if w.dtype in (torch.float16, torch.bfloat16):
        x = x.to(w.dtype)
    return w * x


def gelu_new(x):
    return 0.5 * x * (1.0 + torch.tanh(math.sqrt(2.0 / math.pi) * (x + 0.044715 * torch.pow(x, 3.0))))


def encoder_forward(sd: SD, cfg: dict, input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor] = None):
    """`T5EncoderModel.forward(input_ids)[0]` (the last hidden state)."""
    H, dkv, eps = cfg["num_heads"], cfg["d_kv"], cfg["layer_norm_epsilon"]
    B, L = input_ids.shape
    h = sd["shared.weight"][input_ids]
    bucket = bucket_matrix(L, cfg["relative_attention_num_buckets"], cfg["relative_attention_max_distance"])
    rab = sd["encoder.block.0.layer.0.SelfAttention.relative_attention_bias.weight"]
    bias = rab[bucket].permute(2, 0, 1).unsqueeze(0)  # [1, H, L, L]
    if attention_mask is not None:
        ext = (1.0 - attention_mask[:, None, None, :].to(bias.dtype)) * torch.finfo(bias.dtype).min
        bias = bias + ext
    for i in range(cfg["num_layers"]):
        p = f"encoder.block.{i}.layer"
        n = rms_norm(h, sd[f"{p}.0.layer_norm.weight"], eps)

        def proj(x, name):
            w = sd[f"{p}.0.SelfAttention.{name}.weight"]
            return (x.to(w.dtype) @ w.t()).view(B, L, H, dkv).transpose(1, 2)
        q, k, v = proj(n, "q"), proj(n, "k"), proj(n, "v")
        scores = q @ k.transpose(3, 2) + bias
        w_att = torch.softmax(scores.float(), dim=-1).type_as(scores)
        o = (w_att @ v).transpose(1, 2).reshape(B, L, H * dkv)
        wo = sd[f"{p}.0.SelfAttention.o.weight"]
        h = h + o.to(wo.dtype) @ wo.t()
        n = rms_norm(h, sd[f"{p}.1.layer_norm.weight"], eps)
        w0, w1, w2 = (sd[f"{p}.1.DenseReluDense.{k_}.weight"] for k_ in ("wi_0", "wi_1", "wo"))
        f = gelu_new(n.to(w0.dtype) @ w0.t()) * (n.to(w1.dtype) @ w1.t())
        h = h + f.to(w2.dtype) @ w2.t()
    return rms_norm(h, sd["encoder.final_layer_norm.weight"], eps)
