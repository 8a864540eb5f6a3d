"""Reference-side binding: let the reference's own pipelines take the drop-in models unchanged.

The reference builds its pipelines with `DiffusionPipeline.from_pretrained(path, transformer=..., branch=..., vae=...,
text_encoder=...)` (infer/inpaint.py:286-316, train/train_cogvideox_inpainting_i2v_video.py:1949-1958).  For every
passed component the loader runs `maybe_raise_or_warn` (diffusers/pipelines/pipeline_loading_utils.py:242-265,
called from pipeline_utils.py:861-866), which requires the object's class to be a subclass of the library's base
class for that slot: `diffusers.ModelMixin` for the transformer, the branch and the VAE, transformers'
`PreTrainedModel` for the text encoder.  The drop-ins are plain `nn.Module`s (this package imports neither library),
so the check raises `ValueError: ... should be diffusers.models.modeling_utils.ModelMixin`.

`install()` is called once, in the caller's process, after diffusers (and transformers) are importable:

    import videopainter_amd as vp
    from videopainter_amd.integration import install
    install()                          # or install(diffusers_module, transformers_module)
    pipe = CogVideoXI2VDualInpaintAnyLPipeline.from_pretrained(model_path, transformer=vp_tr, branch=vp_br, ...)

It does two things, nothing else:
  * re-bases the drop-ins' root classes onto the libraries' base classes (`vp.modules.ModelMixin` and
    `vp.vae.AutoencoderKLCogVideoX` onto `diffusers.ModelMixin`, `vp.t5.T5EncoderModel` onto `PreTrainedModel`), so
    `issubclass(vp.CogVideoXTransformer3DModel, diffusers.ModelMixin)` holds for existing and future instances.  The
    drop-ins' own methods and properties stay first in the MRO (their forward, config, dtype, device,
    from_pretrained, save_pretrained are unchanged) and their constructors never run the bases' `__init__`;
  * routes the pipelines' LoRA entry points (`CogVideoXLoraLoaderMixin.load_lora_weights`, `get_list_adapters`,
    `set_adapters`, `fuse_lora`; loaders/lora_pipeline.py:2447-2705) to the drop-in transformer's folded adapters
    when the pipeline holds one (videopainter_amd/lora.py: the reference's `attention_kwargs["scale"]` is honoured
    per call), and to the original methods otherwise.
`uninstall()` restores both.
"""
from __future__ import annotations

import importlib
from typing import Optional

import torch.nn as nn

_STATE: dict = {}


def _root_classes():
    from . import modules, t5, vae
    return {"model": modules.ModelMixin, "vae": vae.AutoencoderKLCogVideoX, "t5": t5.T5EncoderModel}


def _is_vp(obj) -> bool:
    return type(obj).__module__.split(".")[0] == __name__.split(".")[0]


def install(diffusers_module=None, transformers_module=None) -> dict:
    """Make the drop-ins pass the reference loader's class check and bridge the pipelines' LoRA calls.
    Idempotent.  Returns {class name: new base} of what was re-based."""
    if _STATE:
        return dict(_STATE["rebased"])
    diffusers = diffusers_module or importlib.import_module("diffusers")
    try:
        transformers = transformers_module or importlib.import_module("transformers")
    except ImportError:  # no text encoder slot to satisfy
        transformers = None
    roots = _root_classes()
    bases = {"model": diffusers.ModelMixin, "vae": diffusers.ModelMixin}
    if transformers is not None:
        bases["t5"] = transformers.PreTrainedModel
    saved, rebased = {}, {}
    for key, base in bases.items():
        cls = roots[key]
        if cls.__bases__ != (nn.Module,):
            raise RuntimeError(f"{cls.__qualname__} has bases {cls.__bases__}; expected (torch.nn.Module,)")
        saved[key] = cls.__bases__
        cls.__bases__ = (base,)
        rebased[cls.__qualname__] = f"{base.__module__}.{base.__qualname__}"
    lora_saved = _bridge_lora(diffusers)
    _STATE.update(saved=saved, rebased=rebased, lora=lora_saved)
    return dict(rebased)


def uninstall() -> None:
    if not _STATE:
        return
    roots = _root_classes()
    for key, b in _STATE["saved"].items():
        roots[key].__bases__ = b
    for (cls, name), fn in _STATE["lora"].items():
        setattr(cls, name, fn)
    _STATE.clear()


def _bridge_lora(diffusers) -> dict:
    """CogVideoXLoraLoaderMixin's entry points -> the drop-in transformer's folded adapters (lora.py)."""
    try:
        mixin = importlib.import_module(diffusers.__name__ + ".loaders").CogVideoXLoraLoaderMixin
    except (ImportError, AttributeError):
        return {}
    saved = {}

    def tr_of(pipe):
        tr = getattr(pipe, getattr(pipe, "transformer_name", "transformer"), None)
        return tr if tr is not None and _is_vp(tr) else None

    orig = {n: getattr(mixin, n) for n in ("load_lora_weights", "get_list_adapters", "set_adapters", "fuse_lora")
            if hasattr(mixin, n)}

    def load_lora_weights(self, pretrained_model_name_or_path_or_dict, adapter_name: Optional[str] = None, **kw):
        tr = tr_of(self)
        if tr is None:
            return orig["load_lora_weights"](self, pretrained_model_name_or_path_or_dict, adapter_name=adapter_name,
                                             **kw)
        if isinstance(pretrained_model_name_or_path_or_dict, dict):
            from .lora import attach_lora_
            sd = pretrained_model_name_or_path_or_dict
            if any(k.startswith("transformer.") for k in sd):
                sd = {k: v for k, v in sd.items() if k.startswith("transformer.")}
            attach_lora_(tr, sd, 1.0, adapter_name)
        else:
            tr.load_lora_weights(pretrained_model_name_or_path_or_dict,
                                 weight_name=kw.get("weight_name", "pytorch_lora_weights.safetensors"),
                                 adapter_name=adapter_name)

    def get_list_adapters(self):
        tr = tr_of(self)
        if tr is None:
            return orig["get_list_adapters"](self)
        names = tr.get_list_adapters()
        return {"transformer": names} if names else {}

    def set_adapters(self, adapter_names, adapter_weights=None):
        tr = tr_of(self)
        if tr is None:
            return orig["set_adapters"](self, adapter_names, adapter_weights)
        tr.set_adapters(adapter_names, adapter_weights)

    def fuse_lora(self, components=("transformer",), lora_scale: float = 1.0, **kw):
        tr = tr_of(self)
        if tr is None:
            return orig["fuse_lora"](self, components=components, lora_scale=lora_scale, **kw)
        tr.fuse_lora(lora_scale)

    for name, fn in (("load_lora_weights", load_lora_weights), ("get_list_adapters", get_list_adapters),
                     ("set_adapters", set_adapters), ("fuse_lora", fuse_lora)):
        if name in orig:
            saved[(mixin, name)] = orig[name]
            fn.__doc__ = (orig[name].__doc__ or "") + "\n[videopainter_amd] routed to the drop-in transformer."
            setattr(mixin, name, fn)
    return saved
