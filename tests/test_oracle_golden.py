"""Pin the CPU oracle (oracle/cogvideox_oracle.py) against golden vectors recorded from the reference.

CPU-only (no `gpu` marker).  Tolerance: fp32 vs fp32, rel-L2 <= 1e-5 (same torch ops, same order of operations; the
only differences are in how tensors are sliced/concatenated).
"""
import os

import numpy as np
import pytest
import torch
from safetensors.torch import load_file

from oracle import cogvideox_oracle as O
from tests.golden.cases import (TINY_CFG, TINY_BRANCH_CFG, tiny_inputs, tiny_weights, full_block_case, PIPE_CASE)
from videopainter_amd.config import full_config

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def rel(a, b):
    a = a.double()
    b = b.double()
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.fixture(scope="module")
def tiny():
    tsd, bsd = tiny_weights()
    tsd = {k: torch.from_numpy(v) for k, v in tsd.items()}
    bsd = {k: torch.from_numpy(v) for k, v in bsd.items()}
    return dict(tsd=tsd, bsd=bsd, inp=tiny_inputs(), gold=load_file(os.path.join(GOLD, "tiny.safetensors")),
                tcfg=full_config(TINY_CFG), bcfg=full_config(TINY_BRANCH_CFG, True))


def _branch(t):
    i = t["inp"]
    return O.branch_forward(t["bsd"], t["bcfg"], i["video"], i["enc"], i["branch_cond"], i["timestep"], i["rope"])


def test_branch(tiny):
    bs = _branch(tiny)
    for j, s in enumerate(bs):
        assert rel(s, tiny["gold"][f"branch.{j}"]) < 1e-5


def test_branch_wo_text(tiny):
    """wo_text (branch_cogvideox.py:400-412): the blocks' forward_wo_text on the video tokens alone."""
    i = tiny["inp"]
    gold = load_file(os.path.join(GOLD, "wo_text.safetensors"))
    outs = O.branch_forward(tiny["bsd"], tiny["bcfg"], i["video"], i["enc"], i["branch_cond"], i["timestep"],
                            i["rope"], wo_text=True)
    assert len(outs) == TINY_BRANCH_CFG["num_layers"]
    for j, o in enumerate(outs):
        assert rel(o, gold[f"wo_text.f32.{j}"]) <= 1e-5, j
        # a different function of the inputs than the text-conditioned branch
        assert rel(o, tiny["gold"][f"branch.{j}"]) > 1e-4
    # no RoPE: the reference's processor never attends and scrambles its input (attention_processor.py:2349-2358)
    outs = O.branch_forward(tiny["bsd"], tiny["bcfg"], i["video"], i["enc"], i["branch_cond"], i["timestep"], None,
                            wo_text=True)
    for j, o in enumerate(outs):
        assert rel(o, gold[f"wo_text_norope.f32.{j}"]) <= 1e-5, j


def test_transformer_std_with_hidden_states(tiny):
    i = tiny["inp"]
    bs = [tiny["gold"]["branch.0"], tiny["gold"]["branch.1"]]
    out, hs, rm = O.transformer_forward(tiny["tsd"], tiny["tcfg"], i["hidden"], i["enc"], i["timestep"], i["rope"],
                                        branch_block_samples=bs, branch_block_masks=i["mask"],
                                        return_hidden_states=True, return_resample_mask=True)
    g = tiny["gold"]
    assert rel(out, g["std.out"]) < 1e-5
    for k, h in enumerate(hs):
        assert rel(h, g[f"std.hs.{k}"]) < 1e-5
    assert torch.equal(rm.float(), g["std.resample_mask"])


@pytest.mark.parametrize("mode", ["nomask", "addfirst", "prevclip"])
def test_transformer_modes(tiny, mode):
    i = tiny["inp"]
    g = tiny["gold"]
    bs = [g["branch.0"], g["branch.1"]]
    kw = dict(branch_block_samples=bs, branch_block_masks=i["mask"])
    if mode == "nomask":
        kw["branch_block_masks"] = None
    if mode == "addfirst":
        kw["add_first"] = True
    if mode == "prevclip":
        prev = {k: g[f"std.hs.{k}"] for k in range(4)}
        kw["attention_kwargs"] = {"prev_hidden_states": prev, "prev_clip_weight": 0.5,
                                  "prev_resample_mask": g["std.resample_mask"].bool()}
    out = O.transformer_forward(tiny["tsd"], tiny["tcfg"], i["hidden"], i["enc"], i["timestep"], i["rope"], **kw)[0]
    assert rel(out, g[f"{mode}.out"]) < 1e-5


@pytest.mark.parametrize("mode", ["sg_masks", "sg_branchmask", "sg_nobranchmask"])
def test_transformer_self_guidance(tiny, mode):
    """Self-guidance (cogvideox_transformer_3d.py:483-484, 518-523, 593-608) against the reference's own run
    (tests/golden/selfguide.safetensors): the guidance states take the unmasked video rows before the injection;
    self_guidance_masks, when given, are the token mask of the injection too."""
    from tests.golden.cases import selfguide_inputs
    i = tiny["inp"]
    g = tiny["gold"]
    sg = selfguide_inputs()
    gold = load_file(os.path.join(GOLD, "selfguide.safetensors"))
    kw = dict(branch_block_samples=[g["branch.0"], g["branch.1"]], self_guidance_hidden_states=sg["states"],
              branch_block_masks=None if mode == "sg_nobranchmask" else i["mask"],
              self_guidance_masks=None if mode == "sg_branchmask" else sg["mask"])
    out = O.transformer_forward(tiny["tsd"], tiny["tcfg"], i["hidden"], i["enc"], i["timestep"], i["rope"], **kw)[0]
    assert rel(out, gold[f"{mode}.out"]) < 1e-5
    # the guidance changes the output (a different function than the plain masked run)
    assert rel(out, g["std.out"]) > 1e-3


def test_transformer_resample(tiny):
    i = tiny["inp"]
    g = tiny["gold"]
    cfg = dict(tiny["tcfg"], id_pool_resample_learnable=True)
    bs = [g["branch.0"], g["branch.1"]]
    out, hs, rm = O.transformer_forward(tiny["tsd"], cfg, i["hidden"], i["enc"], i["timestep"], i["rope"],
                                        branch_block_samples=bs, branch_block_masks=i["mask"],
                                        return_hidden_states=True, return_resample_mask=True,
                                        id_pool_resample_learnable=True)
    assert rel(out, g["resample0.out"]) < 1e-5
    assert rel(hs[3], g["resample0.hs.3"]) < 1e-5
    prev = {k: h for k, h in enumerate(hs)}
    out1 = O.transformer_forward(tiny["tsd"], cfg, i["hidden2"], i["enc"], i["timestep"], i["rope"],
                                 attention_kwargs={"prev_hidden_states": prev, "prev_clip_weight": 0.5,
                                                   "prev_resample_mask": rm},
                                 branch_block_samples=bs, branch_block_masks=i["mask"], return_hidden_states=True,
                                 return_resample_mask=True, id_pool_resample_learnable=True)[0]
    assert rel(out1, g["resample1.out"]) < 1e-5


def test_scheduler():
    g = load_file(os.path.join(GOLD, "sched.safetensors"))
    from videopainter_amd.weights import synth_tensor
    s = O.DPMSchedulerOracle()
    ts = s.set_timesteps(50)
    assert torch.equal(ts.float(), g["timesteps"])
    assert torch.allclose(s.alphas_cumprod.float(), g["alphas_cumprod"])
    shape = (1, 3, 4, 8, 12)
    sample = torch.from_numpy(synth_tensor("sched.sample", shape)).to(torch.bfloat16)
    gen = torch.Generator().manual_seed(11)
    old = None
    for i in range(3):
        mo = torch.from_numpy(synth_tensor(f"sched.model_output.{i}", shape, bf16=False))
        n1 = torch.randn(shape, generator=gen, dtype=torch.bfloat16)
        n2 = torch.randn(shape, generator=gen, dtype=torch.bfloat16) if (old is not None) else None
        sample, old = s.step(mo, old, int(ts[i]), int(ts[i - 1]) if i > 0 else None, sample, n1, n2)
        sample = sample.to(torch.bfloat16)
        assert torch.equal(sample.float(), g[f"step{i}.prev_sample"])
        assert torch.equal(old.float(), g[f"step{i}.pred_original"])
    gt = torch.from_numpy(synth_tensor("sched.gt", shape)).to(torch.bfloat16)
    nz = torch.from_numpy(synth_tensor("sched.noise", shape)).to(torch.bfloat16)
    assert torch.equal(s.add_noise(gt, nz, torch.tensor([int(ts[5])])).float(), g["add_noise"])


def test_rope_tables_match_pipeline_convention():
    cos, sin = O.prepare_rotary_positional_embeddings(480, 720, 13, 64)
    assert cos.shape == (13 * 30 * 45, 64)
    # t block = 16 dims, h/w = 24 dims each; pairs are interleaved (repeat_interleave)
    assert torch.equal(cos[:, 0::2], cos[:, 1::2])
    assert torch.allclose(cos[0], torch.ones(64))


def test_full_width_block():
    g = load_file(os.path.join(GOLD, "block_full.safetensors"))
    c = full_block_case()
    sd = {"b." + k: torch.from_numpy(v) for k, v in c["weights"].items()}
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    h, e = O.block_forward(sd, "b", dict(num_attention_heads=48, norm_eps=1e-5), c["h"], c["e"], c["temb"], c["rope"])
    flat = torch.cat([e, h], dim=1).reshape(-1)
    assert rel(flat[::97], g["slice"]) < 1e-5
    d = g["digest"]
    # digest was reduced in fp32 by the generator; compare like with like
    assert abs(float(flat.norm()) - float(d[2])) / float(d[2]) < 1e-5


@pytest.mark.parametrize("tag", ["tiny", "5b"])
def test_vae_oracle_matches_reference(tag):
    """oracle/vae_oracle.py against the reference AutoencoderKLCogVideoX run (tests/golden/vae.safetensors): encode
    (two frame batches 9 + 8 with the causal caches carried across, and one batch of 9) and decode (latent batches
    3 + 2, and 3), fp32."""
    from oracle import vae_oracle as V
    from tests.golden.cases import VAE_TINY_CFG, VAE_5B_CFG, VAE_SEEDS, vae_inputs, vae_weights
    from videopainter_amd.config import full_vae_config
    cfg, seed = (VAE_TINY_CFG, VAE_SEEDS[0]) if tag == "tiny" else (VAE_5B_CFG, VAE_SEEDS[1])
    sd = {k: torch.from_numpy(v) for k, v in vae_weights(cfg, seed).items()}
    cfg = full_vae_config(cfg)
    g = load_file(os.path.join(GOLD, "vae.safetensors"))
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    for frames, lf in ((17, 5), (9, 3)):
        x, z = vae_inputs(frames, 64, 96, lf, key=f"vae{frames}")
        with torch.no_grad():
            mean, logvar, _ = V.latent_dist(V.encode(sd, cfg, x))
            dec = V.decode(sd, cfg, z)
        assert rel(mean, g[f"{tag}.f{frames}.mean"]) < 1e-5
        assert rel(logvar, g[f"{tag}.f{frames}.logvar"]) < 1e-5
        assert rel(dec, g[f"{tag}.f{frames}.decode"]) < 1e-5


def test_vae_quant_conv_oracle_matches_reference():
    """use_quant_conv / use_post_quant_conv (autoencoder_kl_cogvideox.py:979-980, 1101-1102, 1152-1153) against the
    reference's own run (tests/golden/vae_quant.safetensors: tiny VAE, out = latent channels = 16)."""
    from oracle import vae_oracle as V
    from tests.golden.cases import VAE_QUANT_CFG, VAE_SEEDS, vae_inputs, vae_weights
    from videopainter_amd.config import full_vae_config
    sd = {k: torch.from_numpy(v) for k, v in vae_weights(VAE_QUANT_CFG, VAE_SEEDS[0]).items()}
    assert "quant_conv.weight" in sd and "post_quant_conv.weight" in sd
    cfg = full_vae_config(VAE_QUANT_CFG)
    g = load_file(os.path.join(GOLD, "vae_quant.safetensors"))
    x, z = vae_inputs(9, 64, 96, 3, key="vaeq")
    with torch.no_grad():
        mean, logvar, _ = V.latent_dist(V.encode(sd, cfg, x))
        dec = V.decode(sd, cfg, z)
    assert rel(mean, g["mean"]) < 1e-5 and rel(logvar, g["logvar"]) < 1e-5
    assert rel(dec[..., ::2, ::2], g["decode_s2"]) < 1e-5


def test_vae_tiled_oracle_matches_reference():
    """Tiled + sliced encode / decode (tests/golden/vae_tiled.safetensors: tiny VAE, sample 128x192, B = 2)."""
    from oracle import vae_oracle as V
    from tests.golden.cases import VAE_TINY_CFG, VAE_SEEDS, vae_inputs, vae_weights
    from videopainter_amd.config import full_vae_config
    cfg = full_vae_config(dict(VAE_TINY_CFG, sample_height=128, sample_width=192))
    sd = {k: torch.from_numpy(v) for k, v in vae_weights(VAE_TINY_CFG, VAE_SEEDS[0]).items()}
    g = load_file(os.path.join(GOLD, "vae_tiled.safetensors"))
    x0, z0 = vae_inputs(9, 128, 192, 3, key="vaet0")
    x1, z1 = vae_inputs(9, 128, 192, 3, key="vaet1")
    with torch.no_grad():
        p = torch.cat([V.tiled(sd, cfg, x, True) for x in (x0, x1)])
        mean, logvar, _ = V.latent_dist(p)
        dec = torch.cat([V.tiled(sd, cfg, z, False) for z in (z0, z1)])
    assert rel(mean, g["mean"]) < 1e-5 and rel(logvar, g["logvar"]) < 1e-5
    assert tuple(dec.shape) == tuple(int(v) for v in g["decode_shape"])
    assert rel(dec[..., ::2, ::2], g["decode_s2"]) < 1e-5


@pytest.mark.parametrize("tag", ["tiny", "xxl2"])
def test_t5_oracle_matches_transformers(tag):
    """oracle/t5_oracle.py against transformers' T5EncoderModel (tests/golden/t5.safetensors), fp32."""
    from oracle import t5_oracle as T
    from tests.golden.cases import T5_TINY_CFG, T5_XXL2_CFG, T5_SEEDS, t5_inputs, t5_weights
    from videopainter_amd.config import full_t5_config
    cfg, seed = (T5_TINY_CFG, T5_SEEDS[0]) if tag == "tiny" else (T5_XXL2_CFG, T5_SEEDS[1])
    fc = full_t5_config(cfg)
    sd = {k: torch.from_numpy(v) for k, v in t5_weights(cfg, seed).items()}
    g = load_file(os.path.join(GOLD, "t5.safetensors"))
    ids, mask = t5_inputs(fc["vocab_size"], key=f"t5{tag}")
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    with torch.no_grad():
        y = T.encoder_forward(sd, fc, ids)
        stride = 1 if tag == "tiny" else 8
        assert rel(y[..., ::stride], g[f"{tag}.out"]) < 1e-5
        if tag == "tiny":
            assert rel(T.encoder_forward(sd, fc, ids, mask), g["tiny.masked.out"]) < 1e-5


def test_pipe_pixel_inputs_are_the_reference_processor_outputs():
    """tests/golden/cases.pipe_pixel_inputs rebuilds the video / mask / first-frame processors' outputs the reference
    pipeline produced (pipe_pixels.safetensors holds their fp64 digests, not the tensors)."""
    from tests.golden.cases import pipe_pixel_inputs
    g = load_file(os.path.join(GOLD, "pipe_pixels.safetensors"))
    inp = pipe_pixel_inputs()
    for k, t in (("video", inp["video"]), ("masks", inp["masks"]), ("image", inp["image"])):
        d = torch.tensor([t.double().sum(), t.double().abs().sum(), t.double().norm()], dtype=torch.float64)
        assert torch.allclose(d, g[f"{k}_digest"], rtol=1e-12, atol=1e-9), k


@pytest.mark.parametrize("steps", [1, 2])
def test_config4_chain_fixture_pins_the_draws_and_masks(steps):
    """tests/golden/config4_chain.safetensors (the full-size chained any-length run of the reference pipeline): the
    generator draws tests/golden/cases.chain4_draws regenerates are the reference run's (fp64 digests), and each
    window's recorded latent mask is the nearest-frame / nearest-pixel pick of cases.chain4_pixel_masks (the
    reference's F.interpolate of the window's pixel masks, default mode 'nearest') with frame 0 of window 0 clear."""
    from tests.golden.cases import CHAIN4_FIXTURES, chain4_case, chain4_draws, chain4_pixel_masks
    path = os.path.join(GOLD, CHAIN4_FIXTURES[steps])
    if not os.path.exists(path):
        pytest.skip(f"{CHAIN4_FIXTURES[steps]} not generated")
    g = load_file(path)
    c = chain4_case(steps)
    draws = chain4_draws(steps)
    assert len(draws) == (c["total_frames"] // c["stride"]) * (1 + c["steps"])
    for i, dr in enumerate(draws):
        d = torch.tensor([dr.double().sum(), dr.double().abs().sum(), dr.double().norm()], dtype=torch.float64)
        assert torch.allclose(d, g[f"draw.{i}.digest"], rtol=1e-12, atol=1e-9), i
    pm = torch.from_numpy(np.ascontiguousarray(chain4_pixel_masks())).float()  # [98, 480, 720]
    for w in range(c["total_frames"] // c["stride"]):
        win = pm[w * c["stride"]:w * c["stride"] + c["num_frames"]][None, None]
        want = torch.nn.functional.interpolate(win, size=(13, 60, 90))  # anyl.py:438-440
        assert torch.equal(g[f"w{w}.mask"].float(), want), w
    assert tuple(int(v) for v in g["final_shape"]) == (1, 25, 16, 60, 90)
    assert float(g["ref_bf16_rel"][0]) < 2e-2
