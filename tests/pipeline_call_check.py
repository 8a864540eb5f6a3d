"""The reference pipeline's `__call__` around the drop-ins (VERDICT r03 "what's missing" 1).

`infer/inpaint.py:435-453` calls `CogVideoXI2VDualInpaintAnyLPipeline.__call__` (…_anyl.py:633-1083) unchanged; that
loop reads the components' configs, dtype and device, calls the branch / transformer forwards with its own keyword
sets and return forms, and calls `vae.encode(x).latent_dist.sample(generator)` and `vae.decode(z).sample`.  The
drop-ins run on the GPU only and the reference never travels to the GPU box, so the contract is pinned in three parts:

  record   the reference pipeline runs once on its own tiny models (2 windows of 9 frames at stride 8, ID-resample +
           prev-clip, CFG, mask_add, replace_gt, 2 steps, output_type="np", bf16 as infer/inpaint.py runs it) with
           every attribute read the PIPELINE'S
           OWN CODE makes on a component (caller-frame filtered), every method call it makes (argument / keyword
           descriptors) and the return forms (recursively, with the attribute reads on returned objects) recorded
           -> tests/golden/pipeline_contract.json (`python tests/pipeline_call_check.py record`).
  check    (CPU, here) the recording is reproduced exactly; every recorded attribute resolves on the install()-ed
           drop-ins with the reference's value; every recorded call binds to the drop-in method's signature; and the
           reference `__call__` runs end to end on the drop-in transformer and branch objects — their forwards
           swapped, in this process only, for the oracle behind a shim that first binds the pipeline's arguments to
           the drop-in forward's signature — with the final frames equal to the reference pipeline's.
  (GPU)    tests/test_pipeline_contract_gpu.py replays every recorded call on the drop-ins on the GPU with tensors of
           the recorded shapes and compares the return forms with the recorded ones (no reference needed).
Prints one JSON line.
"""
import inspect
import json
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SRC = "/root/reference/diffusers/src"
FIXTURE = os.path.join(REPO, "tests", "golden", "pipeline_contract.json")
COMPONENTS = ("transformer", "branch", "vae")

# the call of infer/inpaint.py:435-453 at a tiny size (prompt embeddings instead of prompt: no tokenizer offline)
NUM_FRAMES, STRIDE, TOTAL_FRAMES, STEPS = 9, 8, 17, 2


def _setup():
    sys.path.insert(0, REPO)
    sys.path.insert(0, REF_SRC)
    import transformers.utils as _tu
    # the reference pins transformers 4.42.2; 5.x dropped this constant, which its pipeline loader imports
    _tu.FLAX_WEIGHTS_NAME = getattr(_tu, "FLAX_WEIGHTS_NAME", "flax_model.msgpack")


def describe(x, depth=0):
    """Structure descriptor of a value: tensors by shape / dtype, sequences / dicts recursively, scalars by value,
    other objects by class name."""
    import torch
    if isinstance(x, torch.Tensor):
        return {"tensor": list(x.shape), "dtype": str(x.dtype).replace("torch.", "")}
    if isinstance(x, torch.Generator):
        return {"generator": True}
    if isinstance(x, (list, tuple)):
        return {"seq": type(x).__name__, "items": [describe(v, depth + 1) for v in x]}
    if isinstance(x, dict) and type(x) is dict:
        return {"dict": {str(k): describe(v, depth + 1) for k, v in x.items()}}
    if x is None or isinstance(x, (bool, int, str)):
        return {"value": x}
    if isinstance(x, float):
        return {"value": x if math.isfinite(x) else str(x)}
    return {"object": type(x).__name__}


class _Rec:
    """Proxy of a value a component returned: records the attributes the pipeline reads on it (and calls)."""

    def __init__(self, obj, log):
        object.__setattr__(self, "_o", obj)
        object.__setattr__(self, "_log", log)

    def __getattr__(self, name):
        v = getattr(self._o, name)
        entry = {"attr": name}
        self._log.append(entry)
        if callable(v) and not hasattr(v, "shape"):
            def call(*a, **kw):
                r = v(*a, **kw)
                entry["call"] = {"args": [describe(x) for x in a], "kwargs": {k: describe(x) for k, x in kw.items()},
                                 "ret": describe(r)}
                return r
            return call
        entry["value"] = describe(v)
        sub = []
        entry["uses"] = sub
        return _Rec(v, sub) if not hasattr(v, "shape") else v

    def __getitem__(self, i):
        v = self._o[i]
        self._log.append({"item": i if isinstance(i, int) else str(i), "value": describe(v)})
        return v

    def __iter__(self):
        return iter(self._o)

    def __len__(self):
        return len(self._o)


def _pipeline_frame(depth=2):
    f = sys._getframe(depth)
    return f.f_code.co_filename.endswith("pipeline_cogvideox_inpainting_i2v_branch_anyl.py")


def instrument(name, module, log):
    """Record the pipeline code's attribute reads on `module` (and on its config) and its calls of forward / encode /
    decode, with the return forms and the reads made on returned objects."""
    import torch
    cls = type(module)

    class Recorded(cls):
        def __getattribute__(self, attr):
            v = super().__getattribute__(attr)
            if not attr.startswith("__") and _pipeline_frame():
                if attr in ("config",):
                    log["attrs"].setdefault(f"{name}.config", {})
                    return _ConfigRec(v, log["attrs"][f"{name}.config"])
                if not callable(v) or isinstance(v, (torch.dtype, torch.device)):
                    log["attrs"].setdefault(name, {})[attr] = describe(v) if not isinstance(
                        v, (torch.dtype, torch.device)) else {"value": str(v)}
                else:
                    log["methods_read"].setdefault(name, set()).add(attr)
            return v

    Recorded.__name__ = cls.__name__
    Recorded.__qualname__ = cls.__qualname__
    module.__class__ = Recorded

    def wrap(meth_name):
        orig = getattr(module, meth_name)

        def rec(*a, **kw):
            r = orig(*a, **kw)
            uses = []
            log["calls"].append({"obj": name, "method": meth_name, "args": [describe(x) for x in a],
                                 "kwargs": {k: describe(x) for k, x in kw.items()}, "ret": describe(r),
                                 "ret_uses": uses})
            return r if isinstance(r, (tuple, list)) or hasattr(r, "shape") else _Rec(r, uses)
        object.__setattr__(module, meth_name, rec)  # instance attribute: nn.Module.__call__ runs self.forward
    for m in (("forward",) if name != "vae" else ("encode", "decode")):
        wrap(m)


class _ConfigRec:
    def __init__(self, cfg, log):
        object.__setattr__(self, "_c", cfg)
        object.__setattr__(self, "_log", log)

    def __getattr__(self, k):
        v = getattr(self._c, k)
        self._log[k] = describe(tuple(v) if isinstance(v, list) else v)
        return v

    def __getitem__(self, k):
        return self.__getattr__(k)


def tiny_reference(dtype):
    """Tiny reference components (transformer with the ID-resample processor, 2-layer branch, 4-level VAE), weights
    from the shared counter-based RNG (tests/golden/cases.py), scheduler as infer/inpaint.py builds it."""
    import torch
    from diffusers import AutoencoderKLCogVideoX as RefVAE, CogVideoXDPMScheduler
    from diffusers.models.transformers.cogvideox_transformer_3d import CogVideoXTransformer3DModel as RefTr
    from diffusers.models.branch_cogvideox import CogvideoXBranchModel as RefBr
    from tests.golden.cases import TINY_CFG, TINY_BRANCH_CFG, VAE_TINY_CFG, tiny_weights
    tsd, bsd = tiny_weights()
    tr = RefTr(**dict(TINY_CFG, id_pool_resample_learnable=True)).eval()
    tr.load_state_dict({k: torch.from_numpy(v) for k, v in tsd.items()})
    br = RefBr(**TINY_BRANCH_CFG).eval()
    br.load_state_dict({k: torch.from_numpy(v) for k, v in bsd.items()})
    torch.manual_seed(5)
    vae = RefVAE(**VAE_TINY_CFG).eval()
    sch = CogVideoXDPMScheduler(snr_shift_scale=1.0, prediction_type="v_prediction", rescale_betas_zero_snr=True,
                                clip_sample=False, set_alpha_to_one=True, timestep_spacing="trailing")
    return dict(transformer=tr.to(dtype), branch=br.to(dtype), vae=vae.to(dtype), scheduler=sch)


def call_inputs():
    """PIL frames / masks / first image and prompt embeddings for the infer/inpaint.py call, deterministic."""
    import numpy as np
    import torch
    from PIL import Image
    from tests.golden.cases import TINY_H, TINY_W, TINY_T
    g = np.random.default_rng(7)
    H, W = TINY_H * 8, TINY_W * 8
    frames = [Image.fromarray(g.integers(0, 256, (H, W, 3), dtype=np.uint8)) for _ in range(TOTAL_FRAMES)]
    masks = []
    for i in range(TOTAL_FRAMES):
        m = np.zeros((H, W, 3), dtype=np.uint8)
        if i > 0:  # first_frame_gt: frame 0 unmasked (infer/inpaint.py:425-430)
            m[H // 4 + (i % 3):H // 4 + H // 2, W // 4:W // 4 + W // 2 + (i % 5)] = 255
        masks.append(Image.fromarray(m))
    pe = torch.from_numpy(g.standard_normal((1, TINY_T, 32)).astype(np.float32))
    npe = torch.from_numpy(g.standard_normal((1, TINY_T, 32)).astype(np.float32))
    return dict(image=frames[0], video=frames, masks=masks, prompt_embeds=pe, negative_prompt_embeds=npe,
                height=H, width=W)


def run_pipeline(pipe, dtype):
    import torch
    inp = call_inputs()
    return pipe(image=inp["image"], prompt_embeds=inp["prompt_embeds"].to(dtype),
                negative_prompt_embeds=inp["negative_prompt_embeds"].to(dtype), num_videos_per_prompt=1,
                num_inference_steps=STEPS, num_frames=NUM_FRAMES, use_dynamic_cfg=True, guidance_scale=6.0,
                generator=torch.Generator().manual_seed(42), video=inp["video"], masks=inp["masks"], strength=1.0,
                replace_gt=True, mask_add=True, stride=STRIDE, prev_clip_weight=0.5, id_pool_resample_learnable=True,
                height=inp["height"], width=inp["width"], max_sequence_length=inp["prompt_embeds"].shape[1],
                output_type="np").frames[0]


def record(dtype_name="bfloat16"):
    """Run the reference pipeline on its own tiny models with the recorder, in the dtype infer/inpaint.py runs it in
    (bf16; fp32 for the end-to-end comparison); returns (log, frames)."""
    import torch
    from diffusers.pipelines.cogvideo.pipeline_cogvideox_inpainting_i2v_branch_anyl import (
        CogVideoXI2VDualInpaintAnyLPipeline)
    dtype = getattr(torch, dtype_name)
    comps = tiny_reference(dtype)
    log = {"attrs": {}, "methods_read": {}, "calls": []}
    for n in COMPONENTS:
        instrument(n, comps[n], log)
    pipe = CogVideoXI2VDualInpaintAnyLPipeline(tokenizer=None, text_encoder=None, **comps)
    frames = run_pipeline(pipe, dtype)
    log["methods_read"] = {k: sorted(v) for k, v in log["methods_read"].items()}
    log["call"] = {"num_frames": NUM_FRAMES, "stride": STRIDE, "total_frames": TOTAL_FRAMES, "steps": STEPS,
                   "windows": (TOTAL_FRAMES - NUM_FRAMES) // STRIDE + 1, "dtype": dtype_name}
    return log, frames


def _oracle_forward(module, cfg, kind):
    """The module's forward as the oracle computes it, behind a shim that first binds the pipeline's arguments to the
    DROP-IN forward's signature (a keyword the drop-in does not declare raises TypeError) and then returns the
    drop-in's return form for those arguments (transformer.py / branch.py `forward`, return_dict=False)."""
    import torch
    from oracle import cogvideox_oracle as O
    sig = inspect.signature(type(module).forward)
    sd = {k: v.float() for k, v in module.state_dict().items()}

    def fwd(*a, **kw):
        b = sig.bind(module, *a, **kw)
        b.apply_defaults()
        p = b.arguments
        rope = p["image_rotary_emb"]
        if kind == "branch":
            out = O.branch_forward(sd, cfg, p["hidden_states"].float(), p["encoder_hidden_states"].float(),
                                   p["branch_cond"].float(), p["timestep"], rope, p["conditioning_scale"])
            out = [o.to(p["hidden_states"].dtype) for o in out]
            return (out,) if not p["return_dict"] else {"block_samples": out}
        akw = p["attention_kwargs"]
        if akw and "prev_hidden_states" in akw:
            akw = dict(akw, prev_hidden_states={i: h.float() for i, h in akw["prev_hidden_states"].items()})
        res = O.transformer_forward(sd, cfg, p["hidden_states"].float(), p["encoder_hidden_states"].float(),
                                    p["timestep"], rope, akw, [s.float() for s in p["branch_block_samples"]]
                                    if p["branch_block_samples"] is not None else None,
                                    p["branch_block_masks"].float() if p["branch_block_masks"] is not None else None,
                                    p["add_first"], p["return_hidden_states"], p["return_resample_mask"],
                                    p["id_pool_resample_learnable"])
        dt = p["hidden_states"].dtype
        res = (res[0].to(dt),) + tuple(([h.to(dt) for h in r] if isinstance(r, list) else r) for r in res[1:])
        return res if not p["return_dict"] else {"sample": res[0]}
    return fwd


def check():
    import numpy as np
    import torch
    from diffusers.pipelines.cogvideo.pipeline_cogvideox_inpainting_i2v_branch_anyl import (
        CogVideoXI2VDualInpaintAnyLPipeline)
    from tests.golden.cases import TINY_CFG, TINY_BRANCH_CFG
    from videopainter_amd.config import full_config
    out = {}
    # 1. the recording (bf16, as infer/inpaint.py runs the pipeline) is what the committed fixture says
    log, _ = record("bfloat16")
    want = json.load(open(FIXTURE))
    got = json.loads(json.dumps(log))
    assert got == want, "the reference pipeline's recorded contract differs from tests/golden/pipeline_contract.json"
    _, ref_frames = record("float32")
    out["recorded_calls"] = len(log["calls"])
    out["recorded_attrs"] = sum(len(v) for v in log["attrs"].values())

    # 2. the drop-ins, loaded from the saved reference pipeline, after install()
    import tempfile
    tmp = tempfile.mkdtemp(prefix="vp_pipe_")
    comps = tiny_reference(torch.float32)
    CogVideoXI2VDualInpaintAnyLPipeline(tokenizer=None, text_encoder=None, **comps).save_pretrained(tmp)
    import videopainter_amd as vp
    from videopainter_amd.integration import install
    install()
    f32 = torch.float32
    drop = dict(transformer=vp.CogVideoXTransformer3DModel.from_pretrained(tmp, subfolder="transformer",
                                                                           torch_dtype=f32),
                branch=vp.CogvideoXBranchModel.from_pretrained(os.path.join(tmp, "branch"), torch_dtype=f32),
                vae=vp.AutoencoderKLCogVideoX.from_pretrained(tmp, subfolder="vae"))
    n_attr = 0
    for key, attrs in want["attrs"].items():
        name, _, sub = key.partition(".")
        obj = drop[name].config if sub == "config" else drop[name]
        for a, d in attrs.items():
            v = getattr(obj, a)
            if isinstance(v, (torch.dtype, torch.device)):
                continue  # dtype / device: the drop-ins' own (bf16 on the GPU); resolving is the contract
            assert json.loads(json.dumps(describe(tuple(v) if isinstance(v, list) else v))) == d, (key, a, v, d)
            n_attr += 1
    for name, meths in want["methods_read"].items():
        for m in meths:
            assert callable(getattr(drop[name], m)), (name, m)
    n_bind = 0
    for c in want["calls"]:
        meth = getattr(type(drop[c["obj"]]), c["method"])
        inspect.signature(meth).bind(drop[c["obj"]], *([None] * len(c["args"])), **{k: None for k in c["kwargs"]})
        n_bind += 1
    out["attrs_resolved"] = n_attr
    out["calls_bound"] = n_bind

    # 3. the reference __call__ end to end on the drop-in transformer / branch objects (oracle compute behind the
    #    drop-in signatures), the reference VAE (its contract: the GPU replay test)
    drop["transformer"].forward = _oracle_forward(drop["transformer"],
                                                  full_config(dict(TINY_CFG, id_pool_resample_learnable=True)),
                                                  "transformer")
    drop["branch"].forward = _oracle_forward(drop["branch"], full_config(TINY_BRANCH_CFG, True), "branch")
    pipe = CogVideoXI2VDualInpaintAnyLPipeline(tokenizer=None, text_encoder=None, transformer=drop["transformer"],
                                               branch=drop["branch"], vae=comps["vae"], scheduler=comps["scheduler"])
    frames = run_pipeline(pipe, torch.float32)
    ref = np.asarray(ref_frames, dtype=np.float64)
    got_f = np.asarray(frames, dtype=np.float64)
    assert got_f.shape == ref.shape, (got_f.shape, ref.shape)
    err = float(np.abs(got_f - ref).max())
    out["frames"] = list(ref.shape)
    out["frames_max_abs_diff"] = err
    assert err < 1e-3, err
    print(json.dumps(out))


if __name__ == "__main__":
    _setup()
    if sys.argv[1] == "record":
        lg, _ = record()
        with open(FIXTURE, "w") as f:
            json.dump(lg, f, indent=1, sort_keys=True)
        print(json.dumps({"written": FIXTURE, "calls": len(lg["calls"])}))
    else:
        check()
