"""videopainter_amd — MI355X-native (gfx950) VideoPainter denoising hot path.

Drop-in model classes for the reference's vendored diffusers (same constructor kwargs, state-dict keys and forward
signatures), running every arithmetic op of the per-step forward in hand-written HIP kernels (libvp_hip.so).
"""
from .config import COGVIDEOX_5B_I2V  # noqa: F401
from .modules import device_scope  # noqa: F401


def __getattr__(name):
    # lazy: importing the package must not require the native library (CPU-side tooling, build checks)
    if name in ("CogVideoXTransformer3DModel", "CogVideoXBlock", "Transformer2DModelOutput"):
        from . import transformer
        return getattr(transformer, name)
    if name in ("CogvideoXBranchModel", "CogvideoxBranchOutput"):
        from . import branch
        return getattr(branch, name)
    if name in ("CogVideoXAttnProcessor2_0", "CogVideoXAttnProcessor2_0_resample", "CogVideoXAttnProcessor2_0_wo_text",
                "Attention"):
        from . import attention_processor
        return getattr(attention_processor, name)
    if name in ("CogVideoXDPMScheduler",):
        from . import scheduler
        return getattr(scheduler, name)
    if name in ("AutoencoderKLCogVideoX",):
        from . import vae
        return getattr(vae, name)
    if name in ("T5EncoderModel",):
        from . import t5
        return getattr(t5, name)
    if name in ("CogVideoXI2VDualInpaintAnyLHarness",):
        from . import pipeline
        return getattr(pipeline, name)
    raise AttributeError(name)
