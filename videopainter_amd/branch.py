"""VideoPainter context encoder on the HIP kernels — drop-in for the reference `CogvideoXBranchModel`
(DF/models/branch_cogvideox.py:43-434): same constructor kwargs, state-dict keys (incl. the unused head and
`branch_x_embedder`), `from_transformer`, and `forward` signature / return forms.

The branch's patch embedding sees cat(noisy latents 16ch, masked-video latents 16ch, mask 1ch) = 33 channels; the
channel concat is folded into the im2col kernel (two sources), and K = 132 is zero-padded to 192 for the MFMA GEMM.
The per-block zero-init linears run over the block outputs' video rows; `conditioning_scale` is fused into the GEMM
epilogue.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Tuple, Union

import torch
import torch.nn as nn

from . import kernels as K
from . import _native as NAT
from .attention_processor import CogVideoXAttnProcessor2_0_wo_text, _rope_dev
from .config import patch_in_channels
from .modules import Linear
from .transformer import BF16, CogVideoXTransformer3DModel, _bf


@dataclass
class CogvideoxBranchOutput:
    branch_block_samples: Tuple[torch.Tensor]


class CogvideoXBranchModel(CogVideoXTransformer3DModel):
    _is_branch = True

    def __init__(self, num_attention_heads: int = 30, attention_head_dim: int = 64, in_channels: int = 16,
                 out_channels: Optional[int] = 16, flip_sin_to_cos: bool = True, freq_shift: int = 0,
                 time_embed_dim: int = 512, text_embed_dim: int = 4096, num_layers: int = 30, dropout: float = 0.0,
                 attention_bias: bool = True, sample_width: int = 90, sample_height: int = 60,
                 sample_frames: int = 49, patch_size: int = 2, temporal_compression_ratio: int = 4,
                 max_text_seq_length: int = 226, activation_fn: str = "gelu-approximate",
                 timestep_activation_fn: str = "silu", norm_elementwise_affine: bool = True, norm_eps: float = 1e-5,
                 spatial_interpolation_scale: float = 1.875, temporal_interpolation_scale: float = 1.0,
                 use_rotary_positional_embeddings: bool = False, use_learned_positional_embeddings: bool = False,
                 wo_text: bool = False, id_pool_resample_learnable: bool = False):
        kw = {k: v for k, v in locals().items() if k not in ("self", "__class__")}
        self._pending_cfg = kw
        super().__init__(**{k: v for k, v in kw.items() if k != "wo_text"})
        self.wo_text = bool(wo_text)
        if wo_text:  # the blocks' text-free processor (branch_cogvideox.py:123, cogvideox_transformer_3d.py:96-97)
            for blk in self.transformer_blocks:
                blk.wo_text = True
                blk.processor = CogVideoXAttnProcessor2_0_wo_text()
                blk.attn1.set_processor(blk.processor)
        inner = num_attention_heads * attention_head_dim
        self.branch_blocks = nn.ModuleList([Linear(inner, inner) for _ in range(num_layers)])
        self.branch_x_embedder = Linear(in_channels, inner)

    def _init_config(self, kwargs: dict):
        super()._init_config(self._pending_cfg)

    def _patch_channels(self):
        return patch_in_channels(dict(self.config), True)

    def _block_resample(self):
        return False  # branch blocks always use the standard processor (branch_cogvideox.py:124)

    @classmethod
    def from_transformer(cls, transformer, num_layers: int = 4, attention_head_dim: int = 128,
                         num_attention_heads: int = 24, load_weights_from_transformer=True, wo_text: bool = False):
        """branch_cogvideox.py:255-293.  Parameters the reference does not copy keep its constructor's
        initialisation (PyTorch defaults; `branch_blocks` / `branch_x_embedder` zero, :143-145); the block copy is
        `load_state_dict(strict=False)`, which skips missing keys but raises on a shape mismatch (e.g. the default
        attention_head_dim=128 against a 64-dim transformer)."""
        cfg = {k: v for k, v in dict(transformer.config).items() if not k.startswith("_")}
        cfg.update(num_layers=num_layers, attention_head_dim=attention_head_dim,
                   num_attention_heads=num_attention_heads, wo_text=wo_text)
        dev = transformer.proj_out.weight.device
        branch = cls.from_config(cfg, device=dev, dtype=transformer.proj_out.weight.dtype)
        branch.reset_parameters_()
        with torch.no_grad():
            for lin in list(branch.branch_blocks) + [branch.branch_x_embedder]:  # zero_module (:143-145)
                lin.weight.zero_()
                lin.bias.zero_()
        if load_weights_from_transformer:
            with torch.no_grad():
                w = torch.zeros_like(branch.patch_embed.proj.weight)
                tw = transformer.patch_embed.proj.weight
                c = cfg["in_channels"]
                if c == 16:
                    w[:, :c] = tw
                    w[:, c:2 * c] = tw
                elif c == 32:
                    w[:, :c // 2] = tw[:, :c // 2]
                    w[:, c // 2:c] = tw[:, :c // 2]
                else:
                    raise ValueError(f"in_channels {c} is not supported")
                branch.patch_embed.proj.weight.copy_(w)
                branch.patch_embed.proj.bias.copy_(transformer.patch_embed.proj.bias)
                te, bte = transformer.time_embedding, branch.time_embedding
                for a, b in ((bte.linear_1, te.linear_1), (bte.linear_2, te.linear_2)):
                    a.weight.copy_(b.weight)
                    a.bias.copy_(b.bias)
                tsd = transformer.transformer_blocks.state_dict()
                bsd = branch.transformer_blocks.state_dict()
                bad = [f"{k}: {tuple(tsd[k].shape)} vs {tuple(v.shape)}" for k, v in bsd.items()
                       if k in tsd and tsd[k].shape != v.shape]
                if bad:
                    raise RuntimeError("Error(s) in loading state_dict for ModuleList: size mismatch for "
                                       + "; ".join(bad[:4]))
                for k, v in bsd.items():  # strict=False: the first `num_layers` blocks
                    if k in tsd:
                        v.copy_(tsd[k])
        return branch

    def forward(self, hidden_states: torch.Tensor, encoder_hidden_states: torch.Tensor = None,
                branch_cond: torch.Tensor = None, branch_mode: torch.Tensor = None, conditioning_scale=1.0,
                timestep: Union[int, float, torch.LongTensor] = None, timestep_cond: Optional[torch.Tensor] = None,
                image_rotary_emb: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
                attention_kwargs: Optional[Dict[str, Any]] = None, mask_add: Optional[bool] = False,
                wo_text: Optional[bool] = False, return_dict: bool = True):
        """branch_cogvideox.py:295-434.  Returns a list of [B, Nv, D] bf16 injection tensors (views of one
        [B, T + Nv, D] buffer per block; the text rows of that buffer are scratch).  wo_text (:382-412, the training
        scripts' --wo_text): the blocks run on the video tokens alone (`forward_joint` with no text rows = the
        reference's `forward_wo_text`: the video AdaLN chunks, attention over the video tokens with RoPE on all of
        them, the video gates); the text embedding is computed and left unused, as the reference does.  The mode
        needs a branch built with wo_text=True and the reverse (the reference's blocks fail on either mismatch)."""
        from . import autograd as AG
        train = AG.needs_grad(self, hidden_states, encoder_hidden_states, branch_cond)
        if bool(wo_text) != self.wo_text:
            raise ValueError(f"forward(wo_text={bool(wo_text)}) on a branch built with wo_text={self.wo_text} (the "
                             "reference's blocks take the matching processor at construction, "
                             "cogvideox_transformer_3d.py:96-97)")
        if wo_text and image_rotary_emb is None and train:
            raise NotImplementedError("wo_text without image_rotary_emb (the reference's attention-free quirk, "
                                      "attention_processor.py:2349-2358) is inference-only")
        if timestep_cond is not None:
            raise ValueError("timestep_cond requires a cond_proj, which CogVideoX's TimestepEmbedding does not have")
        dev = self.proj_out.weight.device
        B, F, C, H, W = hidden_states.shape
        cfg = self.config
        hs = _bf(hidden_states.to(dev))
        bc = _bf(branch_cond.to(dev))
        enc = _bf(encoder_hidden_states.to(dev))
        T = enc.shape[1]
        D = cfg.num_attention_heads * cfg.attention_head_dim
        emb = self._time_embed(timestep, B, dev)
        rope = _rope_dev(image_rotary_emb, dev, grid=(F, H // cfg.patch_size, W // cfg.patch_size))
        scale = float(conditioning_scale)
        if train:
            # the training step's branch call (train_cogvideox_inpainting_i2v_video.py:1856-1865): differentiable
            x = AG.patch_embed_apply(self.patch_embed, enc, hs, bc)
            if wo_text:
                x, T = x[:, T:].contiguous(), 0
            outs = []
            for block, lin in zip(self.transformer_blocks, self.branch_blocks):
                x = AG.block_apply(block, x, T, emb, rope)
                outs.append(AG.row_linear_apply(x, lin, scale)[:, T:])
            outs = None if len(outs) == 0 else outs
            return (outs,) if not return_dict else CogvideoxBranchOutput(branch_block_samples=outs)
        x = self.patch_embed.embed(enc, hs, bc)
        if wo_text:  # the video rows alone (one copy per forward); the blocks see no text
            x, T = x[:, T:].contiguous(), 0
        Ntok = x.shape[1]
        samples = []
        for i, block in enumerate(self.transformer_blocks):
            x = block.forward_joint(x, T, emb, rope)
            samples.append(x)
        outs = []
        for s, lin in zip(samples, self.branch_blocks):
            o = torch.empty(B, Ntok, D, device=dev, dtype=BF16)
            epi = NAT.EPI_BIAS if scale == 1.0 else NAT.EPI_BIAS_SCALE
            K.gemm(s.view(B * Ntok, D), [lin.weight], [lin.bias], o.view(B * Ntok, D), epilogue=epi, alpha=scale)
            outs.append(o[:, T:])
        outs = None if len(outs) == 0 else outs
        if not return_dict:
            return (outs,)
        return CogvideoxBranchOutput(branch_block_samples=outs)
