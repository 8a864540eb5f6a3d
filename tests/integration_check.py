"""The reference's own pipelines built around the drop-in models (VERDICT r02 "what's missing" 1).

Run in a subprocess by tests/test_integration_cpu.py (integration.install() re-bases classes process-wide, so it
stays out of the pytest process).  Needs the reference's vendored diffusers (/root/reference/diffusers/src) and
transformers; CPU only (the drop-ins are constructed and loaded, never run).

Steps, each an assertion:
  1. a tiny reference CogVideoXI2VDualInpaintAnyLPipeline (tiny transformer / branch / VAE / T5, no tokenizer) is
     saved with `save_pretrained`, as a checkpoint directory;
  2. the drop-ins load that directory with their own `from_pretrained` (state dicts equal to the reference's);
  3. without install(), `from_pretrained(dir, transformer=drop_in)` raises the loader's ValueError
     (pipeline_loading_utils.py:242-265);
  4. after install(), both reference pipelines the scripts build (infer/inpaint.py:286-316 and
     train/train_cogvideox_inpainting_i2v_video.py:1949-1958) construct with every drop-in passed, and hold them;
  5. `pipe.load_lora_weights(dir, weight_name=..., adapter_name="test_1", target_modules=["transformer"])`
     (infer/inpaint.py:310-315) attaches the adapter to the drop-in unfused, `get_list_adapters()` reports it,
     `fuse_lora` folds it.
Prints one JSON line with what it checked.
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SRC = "/root/reference/diffusers/src"


def main(tmp: str) -> None:
    sys.path.insert(0, REPO)
    sys.path.insert(0, REF_SRC)
    import torch
    import transformers.utils as _tu
    # the reference pins transformers 4.42.2; 5.x dropped this constant, which the reference's pipeline loader
    # imports (pipeline_loading_utils.py:49) — the same one-line environment fix tests/golden/make_golden.py makes
    _tu.FLAX_WEIGHTS_NAME = getattr(_tu, "FLAX_WEIGHTS_NAME", "flax_model.msgpack")
    from safetensors.torch import save_file
    from diffusers import AutoencoderKLCogVideoX as RefVAE, CogVideoXDPMScheduler
    from diffusers.models.transformers.cogvideox_transformer_3d import CogVideoXTransformer3DModel as RefTr
    from diffusers.models.branch_cogvideox import CogvideoXBranchModel as RefBr
    from diffusers.pipelines.cogvideo.pipeline_cogvideox_inpainting_i2v_branch_anyl import (
        CogVideoXI2VDualInpaintAnyLPipeline)
    from diffusers.pipelines.cogvideo.pipeline_cogvideox_inpainting_i2v_branch import (
        CogVideoXI2VDualInpaintPipeline)
    from transformers import T5Config, T5EncoderModel as RefT5
    from tests.golden.cases import TINY_CFG, TINY_BRANCH_CFG, VAE_TINY_CFG, T5_TINY_CFG
    from videopainter_amd.config import full_t5_config

    torch.manual_seed(0)
    ref = dict(transformer=RefTr(**TINY_CFG).eval(), branch=RefBr(**TINY_BRANCH_CFG).eval(),
               vae=RefVAE(**VAE_TINY_CFG).eval(),
               text_encoder=RefT5(T5Config(**{k: v for k, v in full_t5_config(T5_TINY_CFG).items()
                                              if k not in ("dense_act_fn", "is_gated_act")})).eval())
    sch = CogVideoXDPMScheduler(snr_shift_scale=1.0, prediction_type="v_prediction", rescale_betas_zero_snr=True,
                                timestep_spacing="trailing")
    CogVideoXI2VDualInpaintAnyLPipeline(tokenizer=None, scheduler=sch, **ref).save_pretrained(tmp)

    import videopainter_amd as vp
    dt = torch.bfloat16
    drop = dict(transformer=vp.CogVideoXTransformer3DModel.from_pretrained(tmp, subfolder="transformer",
                                                                           torch_dtype=dt),
                branch=vp.CogvideoXBranchModel.from_pretrained(os.path.join(tmp, "branch"), torch_dtype=dt),
                vae=vp.AutoencoderKLCogVideoX.from_pretrained(tmp, subfolder="vae"),
                text_encoder=vp.T5EncoderModel.from_pretrained(tmp, subfolder="text_encoder"))
    for name, m in drop.items():
        want = ref[name].state_dict()
        got = m.state_dict()
        assert set(got) == set(want) or name == "text_encoder", (name, set(got) ^ set(want))
        for k, v in got.items():
            if k in want:
                assert torch.equal(v.float(), want[k].to(v.dtype).float()), (name, k)

    rejected = None
    try:
        CogVideoXI2VDualInpaintAnyLPipeline.from_pretrained(tmp, transformer=drop["transformer"], tokenizer=None,
                                                            torch_dtype=dt)
    except ValueError as e:
        rejected = str(e).split(" is of type")[-1][:160]
    assert rejected is not None, "the reference loader accepted a plain nn.Module: the check under test is gone"

    from videopainter_amd.integration import install
    rebased = install()
    import diffusers
    import transformers
    assert issubclass(vp.CogVideoXTransformer3DModel, diffusers.ModelMixin)
    assert issubclass(vp.CogvideoXBranchModel, diffusers.ModelMixin)
    assert issubclass(vp.AutoencoderKLCogVideoX, diffusers.ModelMixin)
    assert issubclass(vp.T5EncoderModel, transformers.PreTrainedModel)

    # infer/inpaint.py:303-307 (+ the VAE / text encoder swapped in the same call)
    # (tokenizer=None: the tiny checkpoint has none; the tokenizer is host string processing, not a drop-in)
    pipe = CogVideoXI2VDualInpaintAnyLPipeline.from_pretrained(tmp, tokenizer=None, torch_dtype=dt, **drop)
    for name, m in drop.items():
        assert getattr(pipe, name) is m, name
    assert type(pipe.scheduler).__name__ == "CogVideoXDPMScheduler"
    assert pipe.vae_scale_factor_spatial == 2 ** (len(VAE_TINY_CFG["block_out_channels"]) - 1)
    assert pipe.vae_scale_factor_temporal == VAE_TINY_CFG["temporal_compression_ratio"]
    assert pipe.transformer.config.patch_size == ref["transformer"].config.patch_size
    assert pipe.text_encoder.dtype == dt and pipe.transformer.dtype == dt
    assert str(pipe.device) == "cpu"  # _execution_device walks the components' .device
    # train/train_cogvideox_inpainting_i2v_video.py:1949-1958 (validation pipeline)
    pipe2 = CogVideoXI2VDualInpaintPipeline.from_pretrained(tmp, transformer=drop["transformer"],
                                                            text_encoder=drop["text_encoder"], vae=drop["vae"],
                                                            branch=drop["branch"], scheduler=sch, tokenizer=None,
                                                            torch_dtype=dt)
    assert pipe2.transformer is drop["transformer"] and pipe2.branch is drop["branch"]

    # infer/inpaint.py:310-318: the ID-resample adapter through the pipeline's LoRA entry points
    tr = drop["transformer"]
    g = torch.Generator().manual_seed(1)
    sd = {}
    for b in range(TINY_CFG["num_layers"]):
        for t in ("to_q", "to_k", "to_v", "to_out.0"):
            w = dict(tr.named_modules())[f"transformer_blocks.{b}.attn1.{t}"].weight
            sd[f"transformer.transformer_blocks.{b}.attn1.{t}.lora_A.weight"] = torch.randn(4, w.shape[1],
                                                                                           generator=g) * 0.1
            sd[f"transformer.transformer_blocks.{b}.attn1.{t}.lora_B.weight"] = torch.randn(w.shape[0], 4,
                                                                                           generator=g) * 0.1
    lora_dir = os.path.join(tmp, "lora")
    os.makedirs(lora_dir)
    save_file(sd, os.path.join(lora_dir, "pytorch_lora_weights.safetensors"))
    w0 = tr.transformer_blocks[0].attn1.to_q.weight.detach().float().clone()
    pipe.load_lora_weights(lora_dir, weight_name="pytorch_lora_weights.safetensors", adapter_name="test_1",
                           target_modules=["transformer"])
    adapters = pipe.get_list_adapters()
    assert adapters == {"transformer": ["test_1"]}, adapters
    A = sd["transformer.transformer_blocks.0.attn1.to_q.lora_A.weight"]
    B = sd["transformer.transformer_blocks.0.attn1.to_q.lora_B.weight"]
    # applied unfused, as the reference's PEFT does: W0 untouched, the augmented weight tail = s B (s = 1)
    from videopainter_amd.lora import AugmentedProjection
    q = tr.transformer_blocks[0].attn1.to_q
    assert torch.equal(q.weight.float(), w0)
    wa = AugmentedProjection.of((q,)).weights()[0]
    assert torch.equal(wa[:, :w0.shape[1]].float(), w0) and torch.equal(wa[:, w0.shape[1]:w0.shape[1] + 4],
                                                                       B.to(dt).float().to(dt))
    pipe.fuse_lora(lora_scale=1.0)  # the explicit fold (infer/inpaint.py:316, commented out there)
    assert torch.equal(q.weight, (w0 + B.to(dt).float() @ A.to(dt).float()).to(dt))
    print(json.dumps({"rejected_before_install": rejected, "rebased": rebased,
                      "pipelines": ["CogVideoXI2VDualInpaintAnyLPipeline", "CogVideoXI2VDualInpaintPipeline"],
                      "lora_adapters": adapters}))


if __name__ == "__main__":
    main(sys.argv[1])
