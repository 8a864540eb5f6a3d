"""`T5EncoderModel` on the HIP kernels: CogVideoX's text encoder (T5 v1.1 XXL), called once per
prompt by the pipeline's `_get_t5_prompt_embeds` (…_anyl.py:216-256) as `text_encoder(input_ids)[0]`.

Reference algorithm: transformers `modeling_t5.py` (the reference pins transformers==4.42.2): token embedding,
per layer T5LayerNorm -> fused q|k|v projection -> self-attention with the bucketed relative-position bias (computed
by layer 0, shared by all layers; no 1/sqrt(d) scaling) -> o projection + residual -> T5LayerNorm -> gated-GELU
FeedForward (gelu_new(x wi_0) * (x wi_1)) wo + residual; final T5LayerNorm.

HIP: vp_embedding_gather_bf16, vp_rms_norm_bf16, vp_gemm_bf16 (q|k|v as 3 weight segments; the residual adds are the
VP_EPI_BIAS_ADDROWS epilogue writing the stream in place; wi_0 with the GELU-tanh epilogue), vp_mul_bf16,
vp_t5_attention_bf16.  The relative-position bucket matrix is host integer/log arithmetic, computed once per length.
The residual stream is bf16 (the reference keeps `wo` in fp32 under from_pretrained(torch_dtype=bf16), which makes
its stream fp32 after the first FeedForward; the parity tests gate on the reference's own bf16 drift).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import torch
import torch.nn as nn

from . import _native as N
from . import kernels as K
from . import weights as W
from .config import full_t5_config, t5_state_dict_shapes
from .modules import FrozenConfig
from . import modules as _M


def relative_position_buckets(L: int, num_buckets: int, max_distance: int) -> torch.Tensor:
    """`T5Attention._relative_position_bucket` (bidirectional) of relative position j - i, as int32 [L, L]."""
    rel = torch.arange(L)[None, :] - torch.arange(L)[:, None]
    nb = num_buckets // 2
    out = (rel > 0).to(torch.long) * nb
    rp = rel.abs()
    max_exact = nb // 2
    large = max_exact + (torch.log(rp.float() / max_exact) / math.log(max_distance / max_exact)
                         * (nb - max_exact)).to(torch.long)
    large = torch.minimum(large, torch.full_like(large, nb - 1))
    return (out + torch.where(rp < max_exact, rp, large)).to(torch.int32)


@dataclass
class BaseModelOutput:
    last_hidden_state: torch.Tensor
    hidden_states: Optional[Tuple[torch.Tensor, ...]] = None
    attentions: Optional[Tuple[torch.Tensor, ...]] = None

    def __getitem__(self, i):
        return self.to_tuple()[i]

    def to_tuple(self):
        return tuple(v for v in (self.last_hidden_state, self.hidden_states, self.attentions) if v is not None)


class _Node(nn.Module):
    """A level of the reference's module tree (parameters only)."""


class T5EncoderModel(nn.Module):
    """Drop-in for transformers' `T5EncoderModel` (encoder-only T5 v1.1, gated GELU), inference only."""

    _keep_in_fp32_modules = ["wo"]  # reference behaviour recorded for callers; the HIP path computes in bf16

    def __init__(self, config=None, **kwargs):
        nn.Module.__init__(self)  # never a re-based library base's __init__ (integration.install)
        cfg = dict(config.to_dict() if hasattr(config, "to_dict") else (config or {}))
        cfg.update(kwargs)
        cfg = full_t5_config(cfg)
        if not cfg["is_gated_act"] or cfg["dense_act_fn"] != "gelu_new":
            raise NotImplementedError("only the T5 v1.1 gated-gelu FeedForward (CogVideoX's text encoder)")
        if cfg["d_kv"] != 64:
            raise NotImplementedError("the attention kernel is written for d_kv = 64")
        object.__setattr__(self, "_internal_config", FrozenConfig(cfg))
        for key, shape in t5_state_dict_shapes(cfg).items():
            parts = key.split(".")
            mod = self
            for p in parts[:-1]:
                if p not in mod._modules:
                    mod.add_module(p, _Node())
                mod = mod._modules[p]
            # encoder.embed_tokens is tied to shared (T5EncoderModel.__init__): the same parameter
            mod.register_parameter(parts[-1], self.shared.weight if key == "encoder.embed_tokens.weight"
                                   else _M._empty(*shape))
        self._buckets: Dict[Tuple[int, str], torch.Tensor] = {}
        self._graphs_on = False
        self._graph_cache: Dict[tuple, tuple] = {}
        self._qkv: Dict[int, Tuple[torch.Tensor, ...]] = {}

    @property
    def config(self) -> FrozenConfig:
        return self._internal_config

    @property
    def dtype(self):
        return self.shared.weight.dtype

    @property
    def device(self):
        return self.shared.weight.device

    @classmethod
    def from_config(cls, config: dict, device=None, dtype=torch.bfloat16, **overrides):
        cfg = {k: v for k, v in dict(config).items() if not k.startswith("_")}
        cfg.update(overrides)
        with _M.device_scope(device or _M._DEFAULT_DEVICE, dtype):
            return cls(cfg)

    @classmethod
    def from_pretrained(cls, pretrained_model_name_or_path: str, subfolder: Optional[str] = None,
                        torch_dtype=torch.bfloat16, device=None, **kwargs):
        """config.json + model*.safetensors of a transformers T5 encoder folder (e.g. subfolder="text_encoder")."""
        import glob
        import json
        from safetensors.torch import load_file
        d = os.path.join(pretrained_model_name_or_path, subfolder) if subfolder else pretrained_model_name_or_path
        if not os.path.isdir(d):
            raise FileNotFoundError(f"{d} is not a local directory (no hub access)")
        with open(os.path.join(d, "config.json")) as f:
            cfg = json.load(f)
        cfg = {k: v for k, v in cfg.items() if k in full_t5_config({})}
        cfg.update(kwargs)
        model = cls.from_config(cfg, device=device or "cpu", dtype=torch_dtype or torch.bfloat16)
        sd = {}
        for f in sorted(glob.glob(os.path.join(d, "*.safetensors"))):
            sd.update(load_file(f, device=str(device or "cpu")))
        model.load_state_dict(sd, strict=False)
        return model

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        sd = dict(state_dict)
        if "shared.weight" not in sd and "encoder.embed_tokens.weight" in sd:
            sd["shared.weight"] = sd["encoder.embed_tokens.weight"]
        sd.pop("encoder.embed_tokens.weight", None)
        own = {k: v for k, v in self.state_dict().items() if k != "encoder.embed_tokens.weight"}
        missing = [k for k in own if k not in sd]
        unexpected = [k for k in sd if k not in own]
        if missing or (strict and unexpected):
            raise RuntimeError(f"T5 state dict mismatch: missing={missing[:8]} unexpected={unexpected[:8]}")
        with torch.no_grad():
            for k, t in own.items():
                if tuple(sd[k].shape) != tuple(t.shape):
                    raise RuntimeError(f"{k}: shape {tuple(sd[k].shape)} != {tuple(t.shape)}")
                t.copy_(sd[k].to(device=t.device, dtype=t.dtype))
        self._qkv.clear()
        self._graph_cache.clear()
        return self

    def _apply(self, fn, *args, **kwargs):
        # .to() / .cpu() / .cuda() may move every parameter: captured graphs hold the old addresses
        self._qkv = {}
        self._buckets = {}
        if hasattr(self, "_graph_cache"):
            self._graph_cache.clear()
        return super()._apply(fn, *args, **kwargs)

    def get_input_embeddings(self):
        return self.shared

    def _layer(self, i: int):
        return self.encoder.block._modules[str(i)].layer

    def _bucket_matrix(self, L: int, device) -> torch.Tensor:
        key = (L, str(device))
        b = self._buckets.get(key)
        if b is None:
            b = relative_position_buckets(L, self.config.relative_attention_num_buckets,
                                          self.config.relative_attention_max_distance).to(device)
            self._buckets[key] = b
        return b

    def enable_hip_graphs(self, on: bool = True):
        """Replay the 24-layer stack as one captured HIP graph per (batch, length, masked) shape: the encoder runs
        once per prompt at M = B x 226 rows, where the ~220 kernel launches of an eager forward (and their host-side
        descriptor building) take longer than the kernels themselves.  Same kernels, same results."""
        self._graphs_on = bool(on)
        if not on:
            self._graph_cache.clear()
        return self

    def _layers(self, h, mask, B: int, L: int, output_hidden_states: bool = False):
        """The encoder stack on the HIP kernels: h [B*L, d_model] bf16 (consumed in place) -> final-norm output."""
        cfg = self.config
        dev = h.device
        buckets = self._bucket_matrix(L, dev)
        rab = self._layer(0)._modules["0"].SelfAttention.relative_attention_bias.weight
        H, eps = cfg.num_heads, cfg.layer_norm_epsilon
        hidden = [h.view(B, L, -1)] if output_hidden_states else None
        if hidden is not None:
            hidden[0] = hidden[0].clone()
        for i in range(cfg.num_layers):
            ly = self._layer(i)
            sa, ff = ly._modules["0"], ly._modules["1"]
            n = K.rms_norm(h, sa.layer_norm.weight, eps)
            att = sa.SelfAttention
            qkv = torch.empty(B * L, 3 * H * 64, device=dev, dtype=torch.bfloat16)
            K.gemm(n, [att.q.weight, att.k.weight, att.v.weight], [None, None, None], qkv)
            o = K.t5_attention(qkv, B, L, H, rab, buckets, mask)
            K.gemm(o, [att.o.weight], [None], h, epilogue=N.EPI_BIAS_ADDROWS, addrows=h)
            n = K.rms_norm(h, ff.layer_norm.weight, eps)
            dd = ff.DenseReluDense
            g = torch.empty(B * L, cfg.d_ff, device=dev, dtype=torch.bfloat16)
            u = torch.empty_like(g)
            K.gemm(n, [dd.wi_0.weight], [None], g, epilogue=N.EPI_BIAS_GELU)
            K.gemm(n, [dd.wi_1.weight], [None], u)
            K.mul(g, u, out=g)
            K.gemm(g, [dd.wo.weight], [None], h, epilogue=N.EPI_BIAS_ADDROWS, addrows=h)
            if hidden is not None:
                hidden.append(h.view(B, L, -1).clone())
        y = K.rms_norm(h, self.encoder.final_layer_norm.weight, eps).view(B, L, -1)
        if hidden is not None:
            hidden[-1] = y
        return y, hidden

    def _replay(self, h, mask, B: int, L: int):
        key = (B, L, mask is not None, str(h.device))
        ent = self._graph_cache.get(key)
        if ent is None:
            s_h = h.clone()
            s_m = None if mask is None else mask.clone()
            # warm-up on a side stream (allocator, kernel attributes), then capture
            side = torch.cuda.Stream(device=h.device)
            side.wait_stream(torch.cuda.current_stream(h.device))
            with torch.cuda.stream(side):
                self._layers(s_h.clone(), s_m, B, L)
            torch.cuda.current_stream(h.device).wait_stream(side)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                s_y, _ = self._layers(s_h, s_m, B, L)
            ent = (graph, s_h, s_m, s_y)
            self._graph_cache[key] = ent
        graph, s_h, s_m, s_y = ent
        s_h.copy_(h)
        if s_m is not None:
            s_m.copy_(mask)
        graph.replay()
        return s_y.clone()

    def forward(self, input_ids: Optional[torch.Tensor] = None, attention_mask: Optional[torch.Tensor] = None,
                head_mask=None, inputs_embeds: Optional[torch.Tensor] = None, output_attentions: Optional[bool] = None,
                output_hidden_states: Optional[bool] = None, return_dict: Optional[bool] = None):
        if output_attentions:
            raise NotImplementedError("output_attentions: the fused attention kernel does not materialise weights")
        if head_mask is not None:
            raise NotImplementedError("head_mask")
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            raise NotImplementedError("the HIP T5 encoder is inference only; call under torch.no_grad()")
        cfg = self.config
        dev = self.device
        if not dev.type == "cuda":
            raise ValueError("the T5 encoder runs on the HIP kernels: move it to the GPU first")
        with torch.cuda.device(dev):
            if inputs_embeds is not None:
                B, L = inputs_embeds.shape[:2]
                h = inputs_embeds.to(device=dev, dtype=torch.bfloat16).reshape(B * L, -1).contiguous()
            else:
                ids = input_ids.to(dev, torch.int64)
                B, L = ids.shape
                if int(ids.min()) < 0 or int(ids.max()) >= cfg.vocab_size:
                    raise IndexError("input_ids out of the vocabulary range")
                h = K.embedding_gather(self.shared.weight, ids)
            mask = None if attention_mask is None else attention_mask.to(dev, torch.int64)
            if self._graphs_on and not output_hidden_states:
                y, hidden = self._replay(h, mask, B, L), None
            else:
                y, hidden = self._layers(h, mask, B, L, output_hidden_states)
        out = BaseModelOutput(last_hidden_state=y, hidden_states=tuple(hidden) if hidden is not None else None)
        if return_dict is False:
            return out.to_tuple()
        return out
