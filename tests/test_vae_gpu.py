"""CogVideoX VAE on the HIP kernels (videopainter_amd/vae.py, csrc/vae.hip) — GPU tests.

Kernel level: each kernel against plain torch fp32 of the same op on the same bf16-valued inputs (conv3d: every
gather mode the VAE uses — causal frame cache, 1x1x1, stride 2 with right/bottom padding, nearest x2 in space and
time, padded input channels, narrow / wide outputs, residual epilogue; GroupNorm with the spatial-norm modulation).
Model level: encode / decode against the reference's own fp32 outputs (tests/golden/vae*.safetensors, made by
importing the reference AutoencoderKLCogVideoX), gate = 1.25 x the drift of a bf16 run of the same model + 1e-3 (the
5b-shaped model's bf16 drift is the reference's own, recorded by make_golden; the tiny model's is the pinned oracle
run in bf16 here).
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F
from safetensors.torch import load_file

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def rel(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.fixture(scope="module")
def K():
    from videopainter_amd import kernels
    return kernels


def _bf(t):
    return t.to(torch.bfloat16).float()


def _cl(x_ncdhw, cpad):
    """NCDHW -> channels-last with zero channel padding (test-side layout, torch)."""
    x = x_ncdhw.permute(0, 2, 3, 4, 1)
    if cpad > x.shape[-1]:
        x = F.pad(x, (0, cpad - x.shape[-1]))
    return x.contiguous()


def _wl(w, cpad):
    w = w.permute(0, 2, 3, 4, 1)
    if cpad > w.shape[-1]:
        w = F.pad(w, (0, cpad - w.shape[-1]))
    return w.contiguous()


@pytest.mark.parametrize("cin,cout,k,T,H,W,cached", [
    (8, 128, 3, 5, 12, 20, False),     # conv_in-like (3 channels padded to 8)
    (16, 512, 3, 3, 8, 12, True),      # decoder conv_in with a frame cache
    (128, 128, 3, 9, 16, 24, True),    # resnet conv, cache from a previous frame batch
    (256, 512, 1, 4, 10, 14, False),   # conv_shortcut 1x1x1
    (128, 3, 3, 4, 16, 24, False),     # decoder conv_out (3 outputs, BN = 32 path)
    (512, 32, 3, 2, 6, 10, True),      # encoder conv_out (2L)
    (32, 64, 3, 3, 9, 11, False),      # odd spatial sizes, BN = 64 path
])
def test_causal_conv3d_matches_torch(K, cin, cout, k, T, H, W, cached):
    torch.manual_seed(cin * 7 + cout)
    dev = "cuda"
    cl = max(8, cin)
    creal = 3 if cin == 8 else cin
    x = _bf(torch.randn(2, creal, T, H, W))
    hist = _bf(torch.randn(2, creal, 2, H, W)) if cached else None
    w = _bf(torch.randn(cout, creal, k, k, k) / (creal * k ** 3) ** 0.5)
    b = _bf(torch.randn(cout) * 0.1)
    resid = _bf(torch.randn(2, cout, T, H, W)) if cout % 8 == 0 else None
    # reference: CogVideoXCausalConv3d semantics in fp32
    if k == 3:
        head = hist if cached else x[:, :, :1].repeat(1, 1, 2, 1, 1)
        xp = F.pad(torch.cat([head, x], 2), (1, 1, 1, 1))
    else:
        xp = x
    ref = F.conv3d(xp, w, b)
    if resid is not None:
        ref = _bf(ref) + resid
    tmap = list(range(T))
    if k == 3:
        tmap = ([-1, -2] if cached else [0, 0]) + tmap
    y = K.conv3d(_cl(x, cl).to(dev, torch.bfloat16), _wl(w, cl).to(dev, torch.bfloat16), b.to(dev, torch.bfloat16),
                 Tout=T, Hout=H, Wout=W, tmap=tmap,
                 hist=_cl(hist, cl).to(dev, torch.bfloat16) if cached else None, pad=k // 2,
                 resid=_cl(resid, cout).to(dev, torch.bfloat16) if resid is not None else None)
    ldy = y.shape[-1]
    assert ldy == (cout + 7) // 8 * 8
    got = y[..., :cout].float().permute(0, 4, 1, 2, 3).cpu()
    assert torch.all(y[..., cout:] == 0)
    r = rel(got, ref)
    print(f"conv cin={cin} cout={cout} k={k}: rel {r:.2e}")
    assert r < 4e-3


@pytest.mark.parametrize("C,T,H,W", [(128, 3, 16, 24), (256, 2, 9, 13)])
def test_downsample_conv_stride2(K, C, T, H, W):
    """CogVideoXDownsample3D's conv: pad (0, 1, 0, 1) then 3x3 stride 2 per frame."""
    torch.manual_seed(C)
    x = _bf(torch.randn(1, C, T, H, W))
    w = _bf(torch.randn(C, C, 3, 3) / (9 * C) ** 0.5)
    b = _bf(torch.randn(C) * 0.1)
    xf = F.pad(x, (0, 1, 0, 1)).permute(0, 2, 1, 3, 4).reshape(T, C, H + 1, W + 1)
    ref = F.conv2d(xf, w, b, stride=2)
    Ho, Wo = ref.shape[-2:]
    ref = ref.reshape(1, T, C, Ho, Wo).permute(0, 2, 1, 3, 4)
    y = K.conv3d(_cl(x, C).cuda().bfloat16(), _wl(w.unsqueeze(2), C).cuda().bfloat16(), b.cuda().bfloat16(), Tout=T,
                 Hout=(H - 2) // 2 + 1, Wout=(W - 2) // 2 + 1, tmap=list(range(T)), stride=2)
    assert (Ho, Wo) == y.shape[2:4]
    assert rel(y.float().permute(0, 4, 1, 2, 3).cpu(), ref) < 4e-3


@pytest.mark.parametrize("T,compress", [(3, True), (2, True), (1, True), (4, False)])
def test_upsample_conv_nearest_x2(K, T, compress):
    """CogVideoXUpsample3D: nearest x2 (time too when compress_time; first frame single when odd) + 3x3 conv pad 1."""
    torch.manual_seed(T)
    C, H, W = 128, 6, 10
    x = _bf(torch.randn(1, C, T, H, W))
    w = _bf(torch.randn(C, C, 3, 3) / (9 * C) ** 0.5)
    b = _bf(torch.randn(C) * 0.1)
    if compress and T > 1 and T % 2 == 1:
        up = torch.cat([F.interpolate(x[:, :, 0], scale_factor=2.0)[:, :, None],
                        F.interpolate(x[:, :, 1:], scale_factor=2.0)], 2)
        tmap = [0] + [1 + k // 2 for k in range(2 * (T - 1))]
    elif compress and T > 1:
        up = F.interpolate(x, scale_factor=2.0)
        tmap = [k // 2 for k in range(2 * T)]
    else:
        up = torch.stack([F.interpolate(x[:, :, t], scale_factor=2.0) for t in range(T)], 2)
        tmap = list(range(T))
    To = up.shape[2]
    ref = F.conv2d(up.permute(0, 2, 1, 3, 4).reshape(To, C, 2 * H, 2 * W), w, b, padding=1)
    ref = ref.reshape(1, To, C, 2 * H, 2 * W).permute(0, 2, 1, 3, 4)
    y = K.conv3d(_cl(x, C).cuda().bfloat16(), _wl(w.unsqueeze(2), C).cuda().bfloat16(), b.cuda().bfloat16(), Tout=To,
                 Hout=2 * H, Wout=2 * W, tmap=tmap, pad=1, up=2)
    assert rel(y.float().permute(0, 4, 1, 2, 3).cpu(), ref) < 4e-3


def test_conv3d_rejects_bad_descriptors(K):
    x = torch.zeros(1, 2, 4, 4, 24, device="cuda", dtype=torch.bfloat16)  # 24 channels: not a power of two
    w = torch.zeros(8, 3, 3, 3, 24, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="VP_ERR_UNSUPPORTED"):
        K.conv3d(x, w, None, Tout=2, Hout=4, Wout=4, tmap=[0, 0, 0, 1], pad=1)
    x = torch.zeros(1, 2, 4, 4, 16, device="cuda", dtype=torch.bfloat16)
    w = torch.zeros(8, 3, 3, 3, 16, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="VP_ERR_ARG"):  # tmap names a frame x does not have
        K.conv3d(x, w, None, Tout=2, Hout=4, Wout=4, tmap=[0, 0, 0, 2], pad=1)
    with pytest.raises(RuntimeError, match="VP_ERR_ARG"):  # a cache frame without a cache
        K.conv3d(x, w, None, Tout=2, Hout=4, Wout=4, tmap=[-1, -2, 0, 1], pad=1)


@pytest.mark.parametrize("C,G,mod", [(128, 32, False), (512, 32, True), (32, 32, False), (256, 32, True)])
def test_group_norm_silu_and_spatial_norm(K, C, G, mod):
    torch.manual_seed(C + mod)
    B, T, H, W = 2, 5, 16, 24
    x = _bf(torch.randn(B, C, T, H, W) * 2 + 3)  # |mean| > std: exercises the shifted sums
    g = _bf(1 + 0.1 * torch.randn(C))
    bt = _bf(0.1 * torch.randn(C))
    ref = F.group_norm(x, G, g, bt, 1e-6)
    tz = None
    m = None
    if mod:
        Tz, Hz, Wz = 2, 2, 3
        zy = _bf(torch.randn(B, C, Tz, Hz, Wz))
        zb = _bf(torch.randn(B, C, Tz, Hz, Wz))
        first = lambda z: F.interpolate(z[:, :, :1], size=(1, H, W))  # noqa: E731
        rest = lambda z: F.interpolate(z[:, :, 1:], size=(T - 1, H, W))  # noqa: E731
        ref = ref * torch.cat([first(zy), rest(zy)], 2) + torch.cat([first(zb), rest(zb)], 2)
        from videopainter_amd.vae import _spatial_norm_tmap
        tz = _spatial_norm_tmap(T, Tz)
        m = torch.cat([_cl(zy, C), _cl(zb, C)], -1).cuda().bfloat16()
    ref = F.silu(ref)
    y = K.group_norm(_cl(x, C).cuda().bfloat16(), g.cuda().bfloat16(), bt.cuda().bfloat16(), G, 1e-6, silu=True,
                     mod=m, tzmap=tz)
    r = rel(y.float().permute(0, 4, 1, 2, 3).cpu(), ref)
    print(f"group norm C={C} mod={mod}: rel {r:.2e}")
    assert r < 4e-3


def test_time_pool_layout_latent_dist_blend(K):
    torch.manual_seed(3)
    x = _bf(torch.randn(2, 7, 5, 6, 16)).cuda().bfloat16()
    y = K.time_pool2(x).float()
    ref = torch.cat([x[:, :1].float(), (x[:, 1::2].float() + x[:, 2::2].float()) / 2], 1)
    assert torch.equal(y, _bf(ref.cpu()).cuda())
    xe = x[:, :6].contiguous()
    assert torch.equal(K.time_pool2(xe).float(), _bf(((xe[:, 0::2].float() + xe[:, 1::2].float()) / 2).cpu()).cuda())
    v = torch.randn(2, 3, 4, 5, 6, device="cuda")
    cl = K.ncdhw_to_ndhwc(v, 8)
    assert torch.equal(cl[..., :3].float(), _bf(v.permute(0, 2, 3, 4, 1).cpu()).cuda()) and torch.all(cl[..., 3:] == 0)
    assert torch.equal(K.ndhwc_to_ncdhw(cl, 3).float(), _bf(v.cpu()).cuda())
    p = (torch.randn(1, 3, 4, 5, 32, device="cuda") * 20).bfloat16()
    noise = torch.randn(1, 16, 3, 4, 5, device="cuda").bfloat16()
    mean, logvar, smp = K.latent_dist(p, 16, noise)
    pm = p.float().permute(0, 4, 1, 2, 3)
    assert torch.equal(mean.float(), pm[:, :16])
    lv = pm[:, 16:].clamp(-30, 20)
    assert torch.equal(logvar.float(), _bf(lv.cpu()).cuda())
    assert rel(smp.float(), pm[:, :16] + torch.exp(0.5 * _bf(lv.cpu()).cuda()) * noise.float()) < 4e-3
    a = torch.randn(1, 2, 10, 12, 8, device="cuda").bfloat16()
    b0 = torch.randn(1, 2, 7, 12, 8, device="cuda").bfloat16()
    b = b0.clone()
    K.tile_blend_(a, b, 0, 4)
    ref = b0.float().clone()
    for yy in range(4):
        ref[:, :, yy] = a.float()[:, :, -4 + yy] * (1 - yy / 4) + b0.float()[:, :, yy] * (yy / 4)
    assert rel(b.float(), ref) < 4e-3 and torch.equal(b[:, :, 4:], b0[:, :, 4:])


def _vae(cfg, seed, **over):
    from videopainter_amd.vae import AutoencoderKLCogVideoX
    from tests.golden.cases import vae_weights
    m = AutoencoderKLCogVideoX.from_config(dict(cfg, **over), device="cuda")
    m.load_diffusers_state_dict({k: torch.from_numpy(v) for k, v in vae_weights(cfg, seed).items()})
    return m


@pytest.mark.parametrize("tag", ["tiny", "5b"])
def test_vae_encode_decode_matches_reference(tag):
    from tests.golden.cases import VAE_TINY_CFG, VAE_5B_CFG, VAE_SEEDS, vae_inputs, vae_weights
    from videopainter_amd.config import full_vae_config
    cfg, seed = (VAE_TINY_CFG, VAE_SEEDS[0]) if tag == "tiny" else (VAE_5B_CFG, VAE_SEEDS[1])
    g = load_file(os.path.join(GOLD, "vae.safetensors"))
    m = _vae(cfg, seed)
    for frames, lf in ((17, 5), (9, 3)):
        x, z = vae_inputs(frames, 64, 96, lf, key=f"vae{frames}")
        with torch.no_grad():
            post = m.encode(x.cuda()).latent_dist
            dec = m.decode(z.cuda()).sample
        if tag == "5b":
            drift_mean, drift_dec = [float(v) for v in g[f"5b.f{frames}.ref_bf16_rel"]]
        else:
            from oracle import vae_oracle as V
            sd16 = {k: torch.from_numpy(v).bfloat16() for k, v in vae_weights(cfg, seed).items()}
            fc = full_vae_config(cfg)
            with torch.no_grad():
                drift_mean = rel(V.latent_dist(V.encode(sd16, fc, x.bfloat16()))[0].float(), g[f"tiny.f{frames}.mean"])
                drift_dec = rel(V.decode(sd16, fc, z.bfloat16()).float(), g[f"tiny.f{frames}.decode"])
        rm = rel(post.mean.float(), g[f"{tag}.f{frames}.mean"])
        rl = rel(post.logvar.float(), g[f"{tag}.f{frames}.logvar"])
        rd = rel(dec.float(), g[f"{tag}.f{frames}.decode"])
        print(f"vae {tag} f{frames}: mean {rm:.3e} (bf16 ref {drift_mean:.3e}) logvar {rl:.3e} decode {rd:.3e} "
              f"(bf16 ref {drift_dec:.3e})")
        assert tuple(dec.shape) == tuple(g[f"{tag}.f{frames}.decode"].shape)
        assert rm <= 1.25 * drift_mean + 1e-3
        assert rd <= 1.25 * drift_dec + 1e-3
        assert rl <= 2.5 * drift_mean + 2e-3  # logvar ~ N(0, 0.5^2) around 0: relative error of a near-zero field


def test_vae_quant_conv_matches_reference():
    """use_quant_conv / use_post_quant_conv (1x1x1 convs after the encoder / before the decoder, the decoder's spatial
    norms conditioned on the post-quant latent; reference :979-980, 1101-1102, 1152-1153) against the reference's fp32
    run, gated on the oracle's own bf16 run; a config the reference cannot run (out != latent channels) raises."""
    from oracle import vae_oracle as V
    from tests.golden.cases import VAE_QUANT_CFG, VAE_SEEDS, VAE_TINY_CFG, vae_inputs, vae_weights
    from videopainter_amd.config import full_vae_config
    from videopainter_amd.vae import AutoencoderKLCogVideoX
    g = load_file(os.path.join(GOLD, "vae_quant.safetensors"))
    m = _vae(VAE_QUANT_CFG, VAE_SEEDS[0])
    x, z = vae_inputs(9, 64, 96, 3, key="vaeq")
    with torch.no_grad():
        post = m.encode(x.cuda()).latent_dist
        dec = m.decode(z.cuda()).sample
    sd16 = {k: torch.from_numpy(v).bfloat16() for k, v in vae_weights(VAE_QUANT_CFG, VAE_SEEDS[0]).items()}
    fc = full_vae_config(VAE_QUANT_CFG)
    with torch.no_grad():
        drift_mean = rel(V.latent_dist(V.encode(sd16, fc, x.bfloat16()))[0].float(), g["mean"])
        drift_dec = rel(V.decode(sd16, fc, z.bfloat16()).float()[..., ::2, ::2], g["decode_s2"])
    rm, rd = rel(post.mean.float(), g["mean"]), rel(dec[..., ::2, ::2].float(), g["decode_s2"])
    print(f"vae quant: mean {rm:.3e} (bf16 ref {drift_mean:.3e}) decode {rd:.3e} (bf16 ref {drift_dec:.3e})")
    assert tuple(dec.shape) == (1, 16, 9, 64, 96)
    assert rm <= 1.25 * drift_mean + 1e-3
    assert rd <= 1.25 * drift_dec + 1e-3
    with pytest.raises(ValueError):
        AutoencoderKLCogVideoX.from_config(dict(VAE_TINY_CFG, use_quant_conv=True), device="cuda")


def test_vae_tiled_sliced_matches_reference():
    """enable_tiling + enable_slicing on B = 2 (the any-length inference setting, infer/inpaint.py:413-415): the
    blend order and the reference's crop arithmetic (decode comes out 140 x 202 at this size)."""
    from tests.golden.cases import VAE_TINY_CFG, VAE_SEEDS, vae_inputs
    g = load_file(os.path.join(GOLD, "vae_tiled.safetensors"))
    m = _vae(VAE_TINY_CFG, VAE_SEEDS[0], sample_height=128, sample_width=192)
    m.enable_tiling()
    m.enable_slicing()
    x0, z0 = vae_inputs(9, 128, 192, 3, key="vaet0")
    x1, z1 = vae_inputs(9, 128, 192, 3, key="vaet1")
    with torch.no_grad():
        post = m.encode(torch.cat([x0, x1]).cuda()).latent_dist
        dec = m.decode(torch.cat([z0, z1]).cuda()).sample
    assert tuple(dec.shape) == tuple(int(v) for v in g["decode_shape"])
    rm, rd = rel(post.mean.float(), g["mean"]), rel(dec[..., ::2, ::2].float(), g["decode_s2"])
    print(f"vae tiled: mean {rm:.3e} decode {rd:.3e}")
    assert rm < 2e-2 and rd < 2e-2


def test_vae_posterior_sample_uses_generator_noise():
    """latent_dist.sample(generator) = mean + exp(logvar / 2) * randn(generator) (vae.py:780-789)."""
    from tests.golden.cases import VAE_TINY_CFG, VAE_SEEDS, vae_inputs
    m = _vae(VAE_TINY_CFG, VAE_SEEDS[0])
    x, _ = vae_inputs(9, 64, 96, 3, key="vae9")
    with torch.no_grad():
        post = m.encode(x.cuda()).latent_dist
        s = post.sample(torch.Generator().manual_seed(5))
    n = torch.randn(post.mean.shape, generator=torch.Generator().manual_seed(5), dtype=torch.bfloat16)
    ref = post.mean.float().cpu() + torch.exp(0.5 * post.logvar.float().cpu()) * n.float()
    assert rel(s.float(), ref) < 4e-3
    assert torch.equal(post.mode(), post.mean)
