"""Replay of the reference pipeline's recorded calls on the drop-ins, on the GPU (tests/pipeline_call_check.py).

tests/golden/pipeline_contract.json holds what `CogVideoXI2VDualInpaintAnyLPipeline.__call__` (…_anyl.py:633-1083)
did to its components in the infer/inpaint.py call (2 windows, ID-resample + prev-clip, CFG, mask_add, replace_gt):
every branch / transformer forward and VAE encode / decode with its argument and keyword structure, the return forms,
and the attributes it read on the returned objects (`.latent_dist.sample(generator)`, `.sample`).  Each recorded call
is replayed here on the tiny drop-ins with random tensors of the recorded shapes and dtypes (the recording runs the
pipeline in bf16, as infer/inpaint.py does), and the drop-in's return form is compared with the reference's: the
same nesting, lengths, shapes and dtypes.  The CPU side (tests/test_integration_cpu.py) checks that the recording
is current and runs the whole `__call__` on the drop-in objects."""
import json
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
dev = "cuda"


@pytest.fixture(scope="module")
def contract():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    with open(os.path.join(HERE, "golden", "pipeline_contract.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def drop_ins():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tests.golden.cases import TINY_CFG, TINY_BRANCH_CFG, VAE_TINY_CFG, tiny_weights
    from videopainter_amd import AutoencoderKLCogVideoX, CogVideoXTransformer3DModel, CogvideoXBranchModel
    from videopainter_amd import device_scope
    tsd, bsd = tiny_weights()
    with device_scope(dev):
        tr = CogVideoXTransformer3DModel(**dict(TINY_CFG, id_pool_resample_learnable=True))
        br = CogvideoXBranchModel(**TINY_BRANCH_CFG)
    tr.load_diffusers_state_dict({k: torch.from_numpy(v) for k, v in tsd.items()})
    br.load_diffusers_state_dict({k: torch.from_numpy(v) for k, v in bsd.items()})
    vae = AutoencoderKLCogVideoX(**VAE_TINY_CFG)
    vae.init_synthetic_weights_(7)
    vae = vae.to(dev)
    return {"transformer": tr, "branch": br, "vae": vae}


def build(d, g):
    """A value of the recorded structure d (random tensors of the recorded dtype)."""
    if "tensor" in d:
        shape, dt = d["tensor"], getattr(torch, d["dtype"])
        if dt == torch.bool:
            return torch.rand(shape, generator=g) < 0.5
        if dt in (torch.int64, torch.int32):
            return torch.full(shape, 500, dtype=dt)
        return (torch.rand(shape, generator=g) * 2 - 1).to(dt)
    if "generator" in d:
        return torch.Generator().manual_seed(3)
    if "seq" in d:
        items = [build(x, g) for x in d["items"]]
        return tuple(items) if d["seq"] == "tuple" else items
    if "dict" in d:
        return {int(k) if k.isdigit() else k: build(v, g) for k, v in d["dict"].items()}
    if "value" in d:
        return d["value"]
    raise AssertionError(f"cannot build {d}")


def to_dev(x):
    if isinstance(x, torch.Tensor):
        return x.to(dev)
    if isinstance(x, (list, tuple)):
        return type(x)(to_dev(v) for v in x)
    if isinstance(x, dict):
        return {k: to_dev(v) for k, v in x.items()}
    return x


def same_form(got, want, where):
    """got (a value) has the recorded form want (a descriptor)."""
    if "tensor" in want:
        assert isinstance(got, torch.Tensor), (where, type(got))
        assert list(got.shape) == want["tensor"], (where, tuple(got.shape), want["tensor"])
        assert got.dtype == getattr(torch, want["dtype"]), (where, got.dtype, want["dtype"])
        return
    if "seq" in want:
        assert isinstance(got, (list, tuple)), (where, type(got))
        assert type(got).__name__ == want["seq"], (where, type(got).__name__, want["seq"])
        assert len(got) == len(want["items"]), (where, len(got), len(want["items"]))
        for i, (a, b) in enumerate(zip(got, want["items"])):
            same_form(a, b, f"{where}[{i}]")
        return
    if "object" in want:
        assert type(got).__name__ == want["object"], (where, type(got).__name__, want["object"])
        return
    raise AssertionError(f"{where}: unexpected descriptor {want}")


def replay_uses(obj, uses, where, g):
    for u in uses:
        if "attr" not in u:
            continue
        v = getattr(obj, u["attr"])
        if "call" in u:
            c = u["call"]
            r = v(*[build(a, g) for a in c["args"]], **{k: build(a, g) for k, a in c["kwargs"].items()})
            same_form(r, c["ret"], f"{where}.{u['attr']}()")
        else:
            same_form(v, u["value"], f"{where}.{u['attr']}")
            replay_uses(v, u.get("uses", []), f"{where}.{u['attr']}", g)


def test_recorded_attributes_resolve(contract, drop_ins):
    for key, attrs in contract["attrs"].items():
        name, _, sub = key.partition(".")
        obj = drop_ins[name].config if sub == "config" else drop_ins[name]
        for a, d in attrs.items():
            v = getattr(obj, a)
            v = tuple(v) if isinstance(v, list) else v
            if "value" in d:
                assert v == d["value"], (key, a, v, d)
            elif "seq" in d:
                assert [x["value"] for x in d["items"]] == list(v), (key, a, v, d)


def test_recorded_calls_replay_with_the_reference_return_forms(contract, drop_ins):
    g = torch.Generator().manual_seed(0)
    n = 0
    with torch.no_grad():
        for i, c in enumerate(contract["calls"]):
            m = getattr(drop_ins[c["obj"]], c["method"])
            args = to_dev([build(a, g) for a in c["args"]])
            kw = to_dev({k: build(v, g) for k, v in c["kwargs"].items()})
            r = m(*args, **kw)
            where = f"call {i} {c['obj']}.{c['method']}"
            same_form(r, c["ret"], where)
            replay_uses(r, c["ret_uses"], where, g)
            n += 1
    torch.cuda.synchronize()
    assert n == len(contract["calls"]) > 0
