"""Numerics of each HIP kernel against a plain-PyTorch fp32 reference of the same op (GPU only)."""

import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

dev = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from videopainter_amd import _native
    _native.lib()


@pytest.fixture(params=["5", "11", "13", "1"],
                ids=["gemm_v5", "gemm_v11", "gemm_v13", "gemm_v1"])
def gemm_variant(request, knobs):
    from videopainter_amd import kernels as K
    if not K.gemm_variant_built(request.param):
        pytest.skip(f"GEMM variant {request.param} is not in this build")
    knobs.setenv("VP_GEMM_VARIANT", request.param)
    return request.param


UNBOUNDED_VARIANTS = ("p2a", "p2w", "p2w2", "p2s", "a16")


def need_variant(name, knobs=None):
    """Skip unless the attention variant is in this library build (every variant the tests name is built since the
    round-6 pruning); with knobs, select it through its environment switch."""
    from videopainter_amd import kernels as K
    if not K.attention_variant_built(name):
        pytest.skip(f"attention variant {name} is not in this build")
    if knobs is not None:
        knobs.delenv("VP_ATTN_UNBOUNDED_MODE", raising=False)
        knobs.delenv("VP_ATTN_BOUNDED_MODE", raising=False)
        knobs.setenv("VP_ATTN_UNBOUNDED_MODE" if name in UNBOUNDED_VARIANTS else "VP_ATTN_BOUNDED_MODE", name)


@pytest.fixture(params=["p2a", "p2w", "p2w2", "p2s", "a16", "p2", "s16"],
                ids=lambda v: f"attn_{v}")
def attn_variant(request, knobs):
    """Unbounded-score launches (no VP_ATTN_BOUNDED_SCORES): p2a (the library default: the p2 pipeline with an
    anchored reference point and the a16 re-run of flagged blocks), p2w / p2w2 (p2a in 8-wave workgroups), p2s (p2a's
    pipeline on the 16x16x32 MFMA), a16 (the
    anchored-softmax 16x16x32 kernel).  Bounded-score launches (include/vp_hip.h VP_ATTN_BOUNDED_SCORES, the host
    proved the bound; the library default is p2a there too): p2, s16.  (The rejected variants of rounds 1-5 were
    pruned in round 6.)"""
    need_variant(request.param, knobs)
    return request.param


def attn_kw(variant, q, k, scale=0.125, k2=None):
    """bounded_scores for the variant, after checking on the host that the inputs satisfy the bound (the contract
    the processors establish from the qk-norm weights)."""
    if variant in UNBOUNDED_VARIANTS:
        return {}
    kk = k if k2 is None else torch.cat([k, k2], 1)
    B, Nq, D = q.shape
    H = D // 64
    qh = q.float().cpu().view(B, Nq, H, 64).transpose(1, 2)
    kh = kk.float().cpu().view(B, -1, H, 64).transpose(1, 2)
    smax = float((qh @ kh.transpose(-1, -2)).abs().max()) * scale * 1.4426950408889634
    assert smax <= 60.0, f"test inputs exceed the bounded-score contract ({smax:.1f})"
    return dict(bounded_scores=True)


def rel(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


def bf(x):
    return x.to(torch.bfloat16)


def rnd(*shape, std=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * std)


def test_gemm_layout_exact(gemm_variant):
    """Small-integer operands: every product and sum is exact in fp32 -> bit-exact check of the fragment maps."""
    from videopainter_amd import kernels as K
    g = torch.Generator().manual_seed(1)
    M, Nn, Kk = 300, 512, 128
    a = torch.randint(-3, 4, (M, Kk), generator=g).float()
    w = torch.randint(-3, 4, (Nn, Kk), generator=g).float()
    w[:, 0] += torch.arange(Nn).float() % 7  # asymmetric
    b = torch.randint(-4, 5, (Nn,), generator=g).float()
    out = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
    K.gemm(bf(a).to(dev), [bf(w).to(dev)], [bf(b).to(dev)], out)
    ref = a @ w.T + b
    assert torch.equal(out.float().cpu(), bf(ref).float())


@pytest.mark.parametrize("M,Nn,Kk", [(1000, 768, 512), (35, 64, 3072), (513, 256, 192), (300, 128, 32),
                                     (77, 384, 136), (200, 320, 64), (129, 256, 320), (64, 512, 448)])
def test_gemm_bias_random(M, Nn, Kk, gemm_variant):
    from videopainter_amd import kernels as K
    a, w, b = bf(rnd(M, Kk, seed=2)), bf(rnd(Nn, Kk, std=Kk ** -0.5, seed=3)), bf(rnd(Nn, std=0.1, seed=4))
    out = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
    K.gemm(a.to(dev), [w.to(dev)], [b.to(dev)], out)
    ref = a.float() @ w.float().T + b.float()
    assert rel(out, ref) < 4e-3


def test_gemm_large_row_stride():
    """A whose rows span more than 2^31 bytes (M * lda * 2: FF2's input at config 5 is 94052 x 12288): the default
    pipeline addresses A from a 64-bit tile base, so it must stay correct (and not fall back)."""
    from videopainter_amd import kernels as K
    M, Kk, Nn, lda = 33000, 128, 256, 33024
    big = torch.empty(M, lda, device=dev, dtype=torch.bfloat16)
    a = bf(rnd(M, Kk, seed=11))
    big[:, :Kk] = a.to(dev)
    w, b = bf(rnd(Nn, Kk, std=Kk ** -0.5, seed=12)), bf(rnd(Nn, std=0.1, seed=13))
    out = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
    K.gemm(big[:, :Kk], [w.to(dev)], [b.to(dev)], out, lda=lda)
    del big
    ref = a.float() @ w.float().T + b.float()
    assert rel(out, ref) < 4e-3
    assert rel(out[-300:], ref[-300:]) < 4e-3  # the rows past 2^31 bytes


@pytest.mark.parametrize("D,Kk", [(256, 256), (128, 96)])
def test_gemm_segments_gelu_scale(D, Kk, gemm_variant):
    from videopainter_amd import kernels as K
    from videopainter_amd import _native as N
    M = 700
    a = bf(rnd(M, Kk, seed=5))
    ws = [bf(rnd(D, Kk, std=Kk ** -0.5, seed=6 + i)) for i in range(3)]
    bs = [bf(rnd(D, std=0.1, seed=16 + i)) for i in range(3)]
    out = torch.empty(M, 3 * D, device=dev, dtype=torch.bfloat16)
    K.gemm(a.to(dev), [w.to(dev) for w in ws], [b.to(dev) for b in bs], out)
    ref = a.float() @ torch.cat(ws).float().T + torch.cat(bs).float()
    assert rel(out, ref) < 4e-3
    out2 = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    K.gemm(a.to(dev), [ws[0].to(dev)], [bs[0].to(dev)], out2, epilogue=N.EPI_BIAS_GELU)
    ref2 = F.gelu(a.float() @ ws[0].float().T + bs[0].float(), approximate="tanh")
    assert rel(out2, ref2) < 6e-3
    K.gemm(a.to(dev), [ws[0].to(dev)], [bs[0].to(dev)], out2, epilogue=N.EPI_BIAS_SCALE, alpha=0.37)
    assert rel(out2, (a.float() @ ws[0].float().T + bs[0].float()) * 0.37) < 6e-3


def test_gemm_gated_inject_and_remap(gemm_variant):
    from videopainter_amd import kernels as K
    from videopainter_amd import _native as N
    B, T, Nv, D, Kk = 2, 10, 250, 256, 512
    Ntok = T + Nv
    a = bf(rnd(B * Ntok, Kk, seed=30))
    w = bf(rnd(D, Kk, std=Kk ** -0.5, seed=31))
    b = bf(rnd(D, std=0.1, seed=32))
    resid = bf(rnd(B, Ntok, D, seed=33))
    mod = bf(rnd(B, 6 * D, seed=34))
    inj = bf(rnd(B, Nv, D, seed=35))
    tm = (torch.rand(B, Nv, generator=torch.Generator().manual_seed(3)) > 0.5).to(torch.uint8)
    out = torch.empty(B, Ntok, D, device=dev, dtype=torch.bfloat16)
    K.gemm(a.to(dev), [w.to(dev)], [b.to(dev)], out.view(-1, D), epilogue=N.EPI_GATED, resid=resid.to(dev),
           mod=mod.to(dev), tokens_per_batch=Ntok, text_len=T, inject=inj.to(dev), inject_ld=D,
           inject_bstride=Nv * D, inject_mask=tm.to(dev))
    y = (a.float() @ w.float().T + b.float()).view(B, Ntok, D)
    gate = mod.float()[:, 2 * D:3 * D][:, None]
    egate = mod.float()[:, 5 * D:6 * D][:, None]
    ref = resid.float().clone()
    ref[:, :T] += egate * y[:, :T]
    ref[:, T:] += gate * y[:, T:]
    ref[:, T:] += inj.float() * (tm[..., None] == 0)
    assert rel(out, ref) < 5e-3
    # row remap + addrows (patch-embed video rows placed after the text rows of each batch)
    out2 = torch.zeros(B, Ntok, D, device=dev, dtype=torch.bfloat16)
    pos = bf(rnd(Ntok, D, seed=36))
    a2 = bf(rnd(B * Nv, 128, seed=37))
    w2 = bf(rnd(D, 128, std=128 ** -0.5, seed=38))
    K.gemm(a2.to(dev), [w2.to(dev)], [b.to(dev)], out2.view(-1, D), epilogue=N.EPI_BIAS_ADDROWS, rows_per_group=Nv,
           group_stride=Ntok, row_offset=T, addrows=pos.to(dev), addrows_offset=T)
    ref2 = (a2.float() @ w2.float().T + b.float()).view(B, Nv, D) + pos.float()[T:]
    assert rel(out2[:, T:], ref2) < 5e-3
    assert float(out2[:, :T].abs().max()) == 0.0


@pytest.mark.parametrize("inject", [True, False], ids=["inject", "noinject"])
def test_gemm_gated_row_pass_forms_bit_identical(inject):
    """The gated epilogue's branch-free row pass (tokens_per_batch, rows_per_group >= 256: preloaded residual rows,
    the tile's gate vectors, injection flags staged in LDS) against its per-row form (taken here by cutting the output
    into groups of 128 rows at the same places: rows_per_group = group_stride = 128), bit for bit: same arithmetic per
    element.  Rows of both batches and the text / video split land in one tile (Ntok = 320)."""
    from videopainter_amd import kernels as K
    from videopainter_amd import _native as N
    B, T, Nv, D, Kk = 2, 64, 256, 512, 512
    Ntok = T + Nv
    M = B * Ntok
    a = bf(rnd(M, Kk, seed=40)).to(dev)
    w = bf(rnd(D, Kk, std=Kk ** -0.5, seed=41)).to(dev)
    b = bf(rnd(D, std=0.1, seed=42)).to(dev)
    resid = bf(rnd(B, Ntok, D, seed=43)).to(dev)
    mod = bf(rnd(B, 6 * D, seed=44)).to(dev)
    kw = dict(epilogue=N.EPI_GATED, resid=resid, mod=mod, tokens_per_batch=Ntok, text_len=T)
    if inject:
        inj = bf(rnd(B, Nv, D, seed=45)).to(dev)
        tm = (torch.rand(B, Nv, generator=torch.Generator().manual_seed(4)) > 0.5).to(torch.uint8).to(dev)
        kw.update(inject=inj, inject_ld=D, inject_bstride=Nv * D, inject_mask=tm)
    assert M % 128 == 0
    outs = []
    for rpg in (M, 128):
        out = torch.empty(B, Ntok, D, device=dev, dtype=torch.bfloat16)
        K.gemm(a, [w], [b], out.view(-1, D), rows_per_group=rpg, group_stride=rpg, **kw)
        outs.append(out)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("epi", ["bias", "gelu"])
def test_gemm_plain_row_pass_forms_bit_identical(epi):
    """Output row placement of the epilogues without row-wise inputs: one row group (rows_per_group = M) and groups of
    128 rows at group_stride 128 (the same output rows) give the same bits."""
    from videopainter_amd import kernels as K
    from videopainter_amd import _native as N
    M, D, Kk = 640, 768, 512
    a = bf(rnd(M, Kk, seed=50)).to(dev)
    w = bf(rnd(D, Kk, std=Kk ** -0.5, seed=51)).to(dev)
    b = bf(rnd(D, std=0.1, seed=52)).to(dev)
    e = N.EPI_BIAS if epi == "bias" else N.EPI_BIAS_GELU
    outs = []
    for rpg in (M, 128):
        out = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
        K.gemm(a, [w], [b], out, epilogue=e, rows_per_group=rpg, group_stride=rpg)
        outs.append(out)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("epi", ["bias", "gelu"])
def test_gemm_tail_split_round(epi, knobs):
    """Tail mode (gemm.hip tail_plan): 17 x 16 = 272 tiles on the 256-CU chip leave a last round of 16 tiles, which
    runs as split-K workgroups (2 x 512-K chunks, compact fp32 partials) + a reduce that applies the epilogue; the
    ragged last M-tile is among them.  Against torch fp32 and against the same GEMM without the tail split
    (VP_GEMM_NO_TAIL): the two differ only by the fp32 summation order of two K halves."""
    from videopainter_amd import kernels as K
    from videopainter_amd import _native as N
    M, D, Kk = 17 * 256 - 100, 4096, 1024
    a = bf(rnd(M, Kk, seed=60)).to(dev)
    w = bf(rnd(D, Kk, std=Kk ** -0.5, seed=61)).to(dev)
    b = bf(rnd(D, std=0.1, seed=62)).to(dev)
    e = N.EPI_BIAS if epi == "bias" else N.EPI_BIAS_GELU
    out = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    K.gemm(a, [w], [b], out, epilogue=e)
    knobs.setenv("VP_GEMM_NO_TAIL", "1")
    ref_k = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    K.gemm(a, [w], [b], ref_k, epilogue=e)
    y = a.float() @ w.float().T + b.float()
    if epi == "gelu":
        y = F.gelu(y, approximate="tanh")
    assert rel(out, y) < 4e-3
    diff = (out.float() - ref_k.float()).abs()
    assert float(diff.max()) <= float(ref_k.float().abs().max()) * 2 ** -7
    assert rel(out, ref_k) < 1e-3


@pytest.mark.parametrize("inject", [True, False], ids=["inject", "noinject"])
def test_gemm_tail_split_gated_training_shape(inject, knobs):
    """Tail mode at the training shape's N = 3072 GEMMs (M = 17 776: 70 x 12 = 840 tiles = 3 rounds + 72, a round
    28 % full — split since round 6, 3 x 1024-K chunks) with the gated residual epilogue (text / video gates of two
    batches, masked branch injection) applied by the reduce: against the unsplit launch (VP_GEMM_NO_TAIL) and torch
    fp32, and the old quarter-round rule (VP_GEMM_NO_TAIL=q) leaves this shape unsplit."""
    from videopainter_amd import kernels as K
    from videopainter_amd import _native as N
    import ctypes as C
    B, T, Nv, D, Kk = 2, 226, 8662, 3072, 3072
    Ntok = T + Nv
    M = B * Ntok
    a = bf(rnd(M, Kk, seed=63)).to(dev)
    w = bf(rnd(D, Kk, std=Kk ** -0.5, seed=64)).to(dev)
    b = bf(rnd(D, std=0.1, seed=65)).to(dev)
    resid = bf(rnd(B, Ntok, D, seed=66)).to(dev)
    mod = bf(rnd(B, 6 * D, seed=67)).to(dev)
    kw = dict(epilogue=N.EPI_GATED, resid=resid, mod=mod, tokens_per_batch=Ntok, text_len=T)
    if inject:
        inj = bf(rnd(B, Nv, D, seed=68)).to(dev)
        tm = (torch.rand(B, Nv, generator=torch.Generator().manual_seed(6)) > 0.5).to(torch.uint8).to(dev)
        kw.update(inject=inj, inject_ld=D, inject_bstride=Nv * D, inject_mask=tm)
    d = N.GemmDesc()
    d.M, d.N, d.K, d.epilogue, d.n_seg = M, D, Kk, N.EPI_GATED, D
    part = 72 * 3 * 256 * 256 * 4
    # the tail split is active (+ the persistent launch's ticket counters, if any)
    assert part <= N.lib().vp_gemm_bf16_workspace_bytes(C.byref(d)) <= part + 64
    out = torch.empty(B, Ntok, D, device=dev, dtype=torch.bfloat16)
    K.gemm(a, [w], [b], out.view(-1, D), **kw)
    knobs.setenv("VP_GEMM_NO_TAIL", "q")
    assert N.lib().vp_gemm_bf16_workspace_bytes(C.byref(d)) <= 64
    knobs.setenv("VP_GEMM_NO_TAIL", "1")
    ref_k = torch.empty_like(out)
    K.gemm(a, [w], [b], ref_k.view(-1, D), **kw)
    y = (a.float() @ w.float().T + b.float()).view(B, Ntok, D)
    gate = mod.float()[:, 2 * D:3 * D][:, None]
    egate = mod.float()[:, 5 * D:6 * D][:, None]
    ref = resid.float().clone()
    ref[:, :T] += egate * y[:, :T]
    ref[:, T:] += gate * y[:, T:]
    if inject:
        ref[:, T:] += inj.float() * (tm[..., None] == 0)
    assert rel(out, ref) < 5e-3
    assert rel(out, ref_k) < 1e-3
    # the main grid's tiles are untouched by the split: every row of the first 3 rounds' tiles is bit-identical
    assert torch.equal(out.view(-1, D)[:256], ref_k.view(-1, D)[:256])


def _sdpa(q, k, v):
    return F.scaled_dot_product_attention(q.float(), k.float(), v.float())


@pytest.mark.parametrize("Nq,Nk", [(300, 300), (64, 1000), (517, 77)])
def test_attention_random(Nq, Nk, attn_variant):
    from videopainter_amd import kernels as K
    B, H = 2, 3
    q, k, v = (bf(rnd(B, n, H * 64, seed=s)) for s, n in ((40, Nq), (41, Nk), (42, Nk)))
    out = torch.empty(B, Nq, H * 64, device=dev, dtype=torch.bfloat16)
    K.attention(q.to(dev), k.to(dev), v.to(dev), out, H, **attn_kw(attn_variant, q, k))
    hd = lambda x: x.view(B, -1, H, 64).transpose(1, 2)  # noqa: E731
    ref = _sdpa(hd(q), hd(k), hd(v)).transpose(1, 2).reshape(B, Nq, H * 64)
    assert rel(out, ref) < 1e-2


def test_attention_strided_qkv_and_segments_and_blend(attn_variant):
    """Q/K/V read straight out of a fused [B, N, 3D] projection buffer; a second K/V segment (resample) and the
    prev-clip blend (out = (1-w) A1 + w A2)."""
    from videopainter_amd import kernels as K
    B, H, Nn, N2 = 2, 2, 333, 200
    D = H * 64
    qkv = bf(rnd(B, Nn, 3 * D, seed=50)).to(dev)
    k2, v2 = bf(rnd(B, N2, D, seed=51)).to(dev), bf(rnd(B, N2, D, seed=52)).to(dev)
    q, k, v = qkv[..., :D], qkv[..., D:2 * D], qkv[..., 2 * D:]
    out = torch.empty(B, Nn, D, device=dev, dtype=torch.bfloat16)
    kw = attn_kw(attn_variant, q, k, k2=k2)
    K.attention(q, k, v, out, H, k2=k2, v2=v2, **kw)
    hd = lambda x: x.float().cpu().reshape(B, -1, H, 64).transpose(1, 2)  # noqa: E731
    ref = _sdpa(hd(q), torch.cat([hd(k), hd(k2)], 2), torch.cat([hd(v), hd(v2)], 2))
    ref = ref.transpose(1, 2).reshape(B, Nn, D)
    assert rel(out, ref) < 1e-2
    w = 0.3
    K.attention(q, k, v, out, H, out_scale=1 - w, **kw)
    K.attention(q, k2, v2, out, H, out_scale=w, accumulate=True, **kw)
    r1 = _sdpa(hd(q), hd(k), hd(v)).transpose(1, 2).reshape(B, Nn, D)
    r2 = _sdpa(hd(q), hd(k2), hd(v2)).transpose(1, 2).reshape(B, Nn, D)
    assert rel(out, (1 - w) * r1 + w * r2) < 1e-2


def test_attention_forced_rescale(attn_variant):
    """Spike one key so the running max jumps in a late tile (cdna_hip_programming.md §5.4 rule 26)."""
    from videopainter_amd import kernels as K
    B, H, Nn = 1, 1, 640
    q = rnd(B, Nn, 64, seed=60)
    k = rnd(B, Nn, 64, seed=61)
    v = rnd(B, Nn, 64, seed=62)
    k[0, 600] = q[0, :].mean(0) * 12  # large logit late in the sequence for many queries
    k[0, 70] = -k[0, 600]
    q, k, v = bf(q), bf(k), bf(v)
    out = torch.empty(B, Nn, 64, device=dev, dtype=torch.bfloat16)
    K.attention(q.to(dev), k.to(dev), v.to(dev), out, H, **attn_kw(attn_variant, q, k))
    ref = _sdpa(q[:, None], k[:, None], v[:, None])[:, 0]
    assert rel(out, ref) < 1e-2


def _ref64(q, k, v, H, scale=0.125):
    """fp64 attention on the CPU (exact reference for score ranges far beyond fp32 exp)."""
    B, Nq = q.shape[:2]
    hd = lambda x: x.double().cpu().reshape(B, -1, H, 64).transpose(1, 2)  # noqa: E731
    s = hd(q) @ hd(k).transpose(-1, -2) * scale
    return (torch.softmax(s, -1) @ hd(v)).transpose(1, 2).reshape(B, Nq, H * 64)


@pytest.mark.parametrize("mode", ["p2a", "p2w", "p2w2", "p2s", "a16"])
@pytest.mark.parametrize("gamma", [1.0, 6.0])
def test_attention_large_gamma_scores(gamma, mode, knobs):
    """qk-LayerNorm outputs with |gamma| up to 6 (scores over hundreds of log2 units, far outside the bounded-score
    contract): the anchored kernel (no running max) against fp64 attention, at a config-2-like length for 2 heads."""
    from videopainter_amd import kernels as K
    need_variant(mode, knobs)
    B, H, Nn = 1, 2, 4500
    g = torch.Generator().manual_seed(int(gamma * 10))
    gam = torch.rand(H * 64, generator=g) * gamma  # per-channel gains in [0, gamma]
    ln = lambda x: (x - x.mean(-1, keepdim=True)) / x.std(-1, keepdim=True, unbiased=False)  # noqa: E731
    q = bf(ln(torch.randn(B, Nn, H, 64, generator=g)).reshape(B, Nn, H * 64) * gam)
    k = bf(ln(torch.randn(B, Nn, H, 64, generator=g)).reshape(B, Nn, H * 64) * gam)
    v = bf(torch.randn(B, Nn, H * 64, generator=g))
    out = torch.empty(B, Nn, H * 64, device=dev, dtype=torch.bfloat16)
    K.attention(q.to(dev), k.to(dev), v.to(dev), out, H)
    r = rel(out, _ref64(q, k, v, H))
    hd = lambda x: x.double().reshape(B, -1, H, 64).transpose(1, 2)  # noqa: E731
    span = float((hd(q) @ hd(k).transpose(-1, -2)).abs().max()) * 0.125 * 1.4426950408889634
    print(f"gamma {gamma} {mode}: max |score| {span:.0f} log2 units, rel vs fp64 {r:.3e}")
    assert torch.isfinite(out.float()).all() and r < 1e-2


@pytest.mark.parametrize("mode", ["p2a", "p2w", "p2w2", "p2s", "a16"])
@pytest.mark.parametrize("jump", [40.0, 90.0, 200.0])
def test_attention_anchored_late_jump(jump, mode, knobs):
    """The anchored kernels' guarded paths: a late key whose score exceeds every earlier one by `jump` log2 units for
    half the queries — 40: within the first reference's range; 90: row sums pass 2^64 (a16) / 2^62 (p2a): the
    rescale branch; 200: exp2 overflows inside a tile (a16: the exact two-pass re-run of the workgroup; p2a: the block
    is flagged and re-run by a16).  Against fp64 attention."""
    from videopainter_amd import kernels as K
    need_variant(mode, knobs)
    B, H, Nn = 1, 1, 1500
    g = torch.Generator().manual_seed(int(jump))
    q = torch.randn(B, Nn, 64, generator=g) * 0.3
    k = torch.randn(B, Nn, 64, generator=g) * 0.3
    v = torch.randn(B, Nn, 64, generator=g)
    u = torch.randn(64, generator=g)
    u = u / u.norm()
    q[:, ::2] += 4.0 * u                       # even queries align with u
    # key 1300 (tile 10): score vs even queries ~ 4 * a * 0.125 * log2 e  = jump  ->  a = jump / (0.5 * log2 e)
    k[0, 1300] = u * (jump / (0.5 * 1.4426950408889634))
    q, k, v = bf(q), bf(k), bf(v)
    out = torch.empty(B, Nn, 64, device=dev, dtype=torch.bfloat16)
    K.attention(q.to(dev), k.to(dev), v.to(dev), out, H)
    r = rel(out, _ref64(q, k, v, H))
    print(f"late jump {jump}: rel vs fp64 {r:.3e}")
    assert torch.isfinite(out.float()).all() and r < 1e-2


def test_attention_persistent_flagged_blocks_and_streams(knobs):
    """The persistent p2a launch (1 152 blocks: tickets, then the tail pieces) with blocks whose late scores overflow
    exp2 in a tile (flagged, stored nothing, re-run by a16): bit-identical to one workgroup per block, finite, the
    spiked heads against fp64 attention; and two launches on two streams at once, each with its own workspace,
    match the serial result."""
    from videopainter_amd import kernels as K
    B, H, Nn = 1, 48, 6000
    g = torch.Generator().manual_seed(7)
    q = torch.randn(B, Nn, H, 64, generator=g) * 0.3
    k = torch.randn(B, Nn, H, 64, generator=g) * 0.3
    v = torch.randn(B, Nn, H, 64, generator=g)
    u = torch.randn(64, generator=g)
    u = u / u.norm()
    for hh in (3, 40):  # two heads get a late key 200 log2 units above every earlier score for the even queries
        q[0, ::2, hh] += 4.0 * u
        k[0, 5000, hh] = u * (200.0 / (0.5 * 1.4426950408889634))
    q, k, v = (bf(x.reshape(B, Nn, H * 64)).to(dev) for x in (q, k, v))
    outs = []
    for persist in ("1", "0"):
        knobs.setenv("VP_ATTN_PERSIST", persist)
        o = torch.empty(B, Nn, H * 64, device=dev, dtype=torch.bfloat16)
        K.attention(q, k, v, o, H)
        outs.append(o)
    assert torch.isfinite(outs[0].float()).all()
    assert torch.equal(outs[0], outs[1])
    for hh in (3, 40):
        sl = slice(hh * 64, (hh + 1) * 64)
        qh, kh, vh = (x[0, :, sl].double() for x in (q, k, v))
        ref = torch.softmax((qh @ kh.T) * 0.125, -1) @ vh
        assert rel(outs[0][0, :, sl], ref) < 1e-2
    knobs.setenv("VP_ATTN_PERSIST", "1")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    o1, o2 = torch.empty_like(outs[0]), torch.empty_like(outs[0])
    torch.cuda.synchronize()
    with torch.cuda.stream(s1):
        K.attention(q, k, v, o1, H)
    with torch.cuda.stream(s2):
        K.attention(q, k, v, o2, H)
    torch.cuda.synchronize()
    assert torch.equal(o1, outs[0]) and torch.equal(o2, outs[0])


@pytest.mark.parametrize("mode", ["p2a", "p2w", "p2w2", "p2s", "a16"])
@pytest.mark.parametrize("Nn,pos", [(1500, 1300), (3000, 2900), (6000, 5000)])
def test_attention_anchored_late_jump_whole_blocks(Nn, pos, mode, knobs):
    """test_attention_anchored_late_jump's overflow case (a late key 200 log2 units above every earlier score for the
    even queries) on WHOLE blocks (VP_ATTN_NO_SPLIT: no tail pieces): the anchored kernels must flag the block (its
    O turns NaN: inf P against V of both signs) so a16 re-runs it — this file's -fno-honor-nans had folded the NaN
    half of the test away and p2a stored NaN rows.  Against fp64 attention."""
    from videopainter_amd import kernels as K
    need_variant(mode, knobs)
    knobs.setenv("VP_ATTN_NO_SPLIT", "1")
    g = torch.Generator().manual_seed(200)
    q = torch.randn(1, Nn, 64, generator=g) * 0.3
    k = torch.randn(1, Nn, 64, generator=g) * 0.3
    v = torch.randn(1, Nn, 64, generator=g)
    u = torch.randn(64, generator=g)
    u = u / u.norm()
    q[:, ::2] += 4.0 * u
    k[0, pos] = u * (200.0 / (0.5 * 1.4426950408889634))
    q, k, v = bf(q), bf(k), bf(v)
    out = torch.full((1, Nn, 64), 7.0, device=dev, dtype=torch.bfloat16)
    K.attention(q.to(dev), k.to(dev), v.to(dev), out, 1)
    assert torch.isfinite(out.float()).all()
    assert rel(out, _ref64(q, k, v, 1)) < 1e-2


@pytest.mark.parametrize("mode", ["p2a", "p2w", "p2w2", "p2s", "a16"])
def test_attention_stepwise_max_growth(mode, knobs):
    """Running max grows by 0 / 0.5 / 3 / 8 nats at tile seams, so the deferred-max test (tile sum > 2^8) takes both
    branches many times within one query block (cdna_hip_programming.md §5.4 rule 26); for the anchored kernel the
    row sums pass 2^64 repeatedly (its rescale branch).  (Scores up to ~300 in log2 units: outside the bounded-score
    contract.)"""
    from videopainter_amd import kernels as K
    need_variant(mode, knobs)
    B, H, Nn = 1, 2, 1100
    g = torch.Generator().manual_seed(80)
    u = torch.randn(64, generator=g)
    u = u / u.norm()
    q = rnd(B, Nn, 2 * 64, seed=81) + 2.0 * torch.cat([u, -u])
    k = rnd(B, Nn, 2 * 64, seed=82)
    steps = torch.tensor([0.0, 0.5, 3.0, 8.0])[torch.randint(0, 4, (Nn // 64 + 1,), generator=g)]
    coef = 4.0 * torch.cumsum(steps, 0)[torch.arange(Nn) // 64]  # logit += 2 * coef / 8 per key
    k = k + coef[None, :, None] * torch.cat([u, -u])
    v = rnd(B, Nn, 2 * 64, seed=83)
    q, k, v = bf(q), bf(k), bf(v)
    out = torch.empty(B, Nn, 2 * 64, device=dev, dtype=torch.bfloat16)
    K.attention(q.to(dev), k.to(dev), v.to(dev), out, H)
    hd = lambda t: t.view(B, Nn, H, 64).transpose(1, 2)
    ref = _sdpa(hd(q), hd(k), hd(v)).transpose(1, 2).reshape(B, Nn, 2 * 64)
    assert rel(out, ref) < 1e-2


def test_adaln_and_final_norm():
    from videopainter_amd import kernels as K
    B, T, Nv, D = 2, 7, 100, 3072
    x = bf(rnd(B, T + Nv, D, seed=70) * 3 + 1)
    lw, lb = bf(1 + 0.1 * rnd(D, seed=71)), bf(0.1 * rnd(D, seed=72))
    mod = bf(rnd(B, 6 * D, seed=73) * 0.5)
    y = K.adaln_modulate(x.to(dev), lw.to(dev), lb.to(dev), mod.to(dev), T, 1e-5)
    n = F.layer_norm(x.float(), (D,), lw.float(), lb.float(), 1e-5)
    m = mod.float()
    ref = torch.empty_like(n)
    ref[:, T:] = n[:, T:] * (1 + m[:, None, D:2 * D]) + m[:, None, 0:D]
    ref[:, :T] = n[:, :T] * (1 + m[:, None, 4 * D:5 * D]) + m[:, None, 3 * D:4 * D]
    assert rel(y, ref) < 8e-3
    # rows at a wider stride (the first D columns of an unfused-LoRA x_aug buffer): the same bits, the rest untouched
    buf = torch.full((B * (T + Nv), D + 192), 7.0, device=dev, dtype=torch.bfloat16)
    ys = K.adaln_modulate(x.to(dev), lw.to(dev), lb.to(dev), mod.to(dev), T, 1e-5,
                          out=buf[:, :D].view(B, T + Nv, D))
    assert torch.equal(ys, y) and bool((buf[:, D:] == 7.0).all())
    mod2 = bf(rnd(B, 2 * D, seed=74) * 0.5)
    lw2, lb2 = bf(1 + 0.1 * rnd(D, seed=75)), bf(0.1 * rnd(D, seed=76))
    z = K.final_norm(x.to(dev), T, lw.to(dev), lb.to(dev), lw2.to(dev), lb2.to(dev), 1e-5, mod2.to(dev))
    n1 = F.layer_norm(x.float()[:, T:], (D,), lw.float(), lb.float(), 1e-5)
    n2 = F.layer_norm(n1, (D,), lw2.float(), lb2.float(), 1e-5)
    ref2 = n2 * (1 + mod2.float()[:, None, D:]) + mod2.float()[:, None, :D]
    assert rel(z, ref2) < 8e-3


def test_head_norm_rope_and_masked_null_key():
    from videopainter_amd import kernels as K
    from oracle.cogvideox_oracle import apply_rotary_emb, prepare_rotary_positional_embeddings
    B, T, H = 2, 8, 2
    cos, sin = prepare_rotary_positional_embeddings(128, 192, 3, 64)
    Nv = cos.shape[0]
    Ntok = T + Nv
    x = bf(rnd(B, Ntok, 3 * H * 64, seed=80))
    lw, lb = bf(1 + 0.1 * rnd(64, seed=81)), bf(0.1 * rnd(64, seed=82))
    xd = x.to(dev)
    k_in = xd[..., H * 64:2 * H * 64]
    mask = (torch.rand(B, Ntok, generator=torch.Generator().manual_seed(4)) > 0.4).to(torch.uint8)
    mask[:, :T] = 0
    k2 = torch.empty(B, Ntok, H * 64, device=dev, dtype=torch.bfloat16)
    K.head_norm_rope(k_in, k2, H, T, lw.to(dev), lb.to(dev), 1e-6, (cos.to(dev), sin.to(dev)), tok_mask=mask.to(dev),
                     pre_scale=0.5)
    K.head_norm_rope(k_in, k_in, H, T, lw.to(dev), lb.to(dev), 1e-6, (cos.to(dev), sin.to(dev)))
    kr = x.float()[..., H * 64:2 * H * 64].view(B, Ntok, H, 64).transpose(1, 2)
    n = F.layer_norm(kr, (64,), lw.float(), lb.float(), 1e-6)
    n[:, :, T:] = apply_rotary_emb(n[:, :, T:], cos, sin)
    ref = n.transpose(1, 2).reshape(B, Ntok, H * 64)
    assert rel(xd[..., H * 64:2 * H * 64], ref) < 8e-3
    km = kr * mask[:, None, :, None].float() * 0.5
    n2 = F.layer_norm(km, (64,), lw.float(), lb.float(), 1e-6)
    n2[:, :, T:] = apply_rotary_emb(n2[:, :, T:], cos, sin)
    ref2 = n2.transpose(1, 2).reshape(B, Ntok, H * 64)
    assert rel(k2, ref2) < 8e-3
    # masked rows are the (rotated) LN bias exactly in the first text rows
    assert torch.equal(k2[0, 0, :64].cpu(), lb)


@pytest.mark.parametrize("H,T,rope", [(2, 8, True), (4, 5, True), (2, 0, False)])
def test_gemm_qknorm_rope_epilogue_matches_separate_kernels(H, T, rope, gemm_variant):
    """EPI_BIAS_QKNORM_ROPE (the fused QKV projection) == GEMM + vp_head_norm_rope_bf16 on q and k, bit for bit
    (one shared device routine); v untouched; ragged M (not a multiple of the 256-row tile)."""
    from types import SimpleNamespace

    from videopainter_amd import _native as NAT
    from videopainter_amd import kernels as K
    from oracle.cogvideox_oracle import apply_rotary_emb, prepare_rotary_positional_embeddings
    B, D = 2, H * 64
    cos, sin = prepare_rotary_positional_embeddings(128, 192, 3, 64)
    Nv = cos.shape[0]
    Ntok = T + Nv
    x = bf(rnd(B * Ntok, 128, seed=101)).to(dev)
    ws = [bf(rnd(D, 128, std=0.1, seed=102 + i)).to(dev) for i in range(3)]
    bs = [bf(rnd(D, std=0.1, seed=105 + i)).to(dev) for i in range(3)]
    lns = [SimpleNamespace(weight=bf(1 + 0.1 * rnd(64, seed=108 + i)).to(dev),
                           bias=bf(0.1 * rnd(64, seed=110 + i)).to(dev), eps=(1e-6, 1e-5)[i]) for i in range(2)]
    rp = (cos.to(dev), sin.to(dev)) if rope else None
    want = torch.empty(B * Ntok, 3 * D, device=dev, dtype=torch.bfloat16)
    K.gemm(x, ws, bs, want)
    w3 = want.view(B, Ntok, 3 * D)
    for s in range(2):
        K.head_norm_rope(w3[..., s * D:(s + 1) * D], w3[..., s * D:(s + 1) * D], H, T, lns[s].weight, lns[s].bias,
                         lns[s].eps, rp)
    got = torch.full((B * Ntok, 3 * D), float("nan"), device=dev, dtype=torch.bfloat16)
    K.gemm(x, ws, bs, got, epilogue=NAT.EPI_BIAS_QKNORM_ROPE, qk_norm=tuple(lns), rope=rp, tokens_per_batch=Ntok,
           text_len=T)
    assert torch.equal(got, want)
    if rope:
        # the separable form (the transformer's RopeTables carry their grid): the epilogue reads per-axis rows, with
        # the same values, so the same bits
        from videopainter_amd.attention_processor import RopeTables
        assert Nv == 3 * 8 * 12
        rt = RopeTables(rp)
        rt.grid = (3, 8, 12)
        assert K.rope_axis_tables(rt, rt.grid) is not None
        got_sep = torch.full_like(got, float("nan"))
        K.gemm(x, ws, bs, got_sep, epilogue=NAT.EPI_BIAS_QKNORM_ROPE, qk_norm=tuple(lns), rope=rt,
               tokens_per_batch=Ntok, text_len=T)
        assert torch.equal(got_sep, want)
    # and against plain torch fp32 (LN over each head, rotary on video tokens)
    y = bf(x.float().cpu() @ torch.cat(ws).float().cpu().T + torch.cat(bs).float().cpu()).view(B, Ntok, 3 * D)
    for s in range(2):
        h = y[..., s * D:(s + 1) * D].view(B, Ntok, H, 64).transpose(1, 2)
        n = F.layer_norm(h, (64,), lns[s].weight.float().cpu(), lns[s].bias.float().cpu(), lns[s].eps)
        if rope:
            n[:, :, T:] = apply_rotary_emb(n[:, :, T:], cos, sin)
        assert rel(got.view(B, Ntok, 3 * D)[..., s * D:(s + 1) * D], n.transpose(1, 2).reshape(B, Ntok, D)) < 8e-3


@pytest.mark.parametrize("M,N,K", [(600, 512, 128), (4352, 4096, 1024), (1000, 768, 512)],
                         ids=["v5_runtime_epi", "tail_split", "v13"])
def test_gemm_gelu_aux_and_gelu_bwd_epilogues_match_separate_launches(M, N, K):
    """ABI 17, the training forward / backward: EPI_BIAS_GELU with an aux output writes GELU(z) to C and z to aux —
    bit for bit the FF1 GEMM's plain output and vp_gelu_bf16 of it; EPI_GELU_BWD == the dgrad GEMM then
    vp_gelu_bwd_bf16, bit for bit.  Shapes: K < 512 (the runtime-epilogue main loop), a tail-split grid (4352 x 4096:
    272 tiles, the last 16 as split-K workgroups + reduce), the default loop with ragged M."""
    from videopainter_amd import _native as NAT
    from videopainter_amd import kernels as K_
    x = bf(rnd(M, K, seed=201)).to(dev)
    w = bf(rnd(N, K, std=K ** -0.5, seed=202)).to(dev)
    b = bf(rnd(N, std=0.3, seed=203)).to(dev)
    z_want = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    K_.gemm(x, [w], [b], z_want)
    h_want = K_.gelu(z_want)
    h_fused = torch.empty_like(h_want)
    K_.gemm(x, [w], [b], h_fused, epilogue=NAT.EPI_BIAS_GELU)
    assert torch.equal(h_fused, h_want)  # (the existing fused GELU: the same bits as the separate pass)
    h, z = torch.full_like(h_want, float("nan")), torch.full_like(z_want, float("nan"))
    K_.gemm(x, [w], [b], h, epilogue=NAT.EPI_BIAS_GELU, aux=z)
    assert torch.equal(z, z_want)
    assert torch.equal(h, h_want)
    # the backward: dz = (dh W) * GELU'(z) with dh [M, K'] against W^T — here the same GEMM shape (a = x, W = w)
    dz_plain = torch.empty_like(z_want)
    K_.gemm(x, [w], [None], dz_plain)
    g_want = K_.gelu_bwd(dz_plain, z_want)
    g = torch.full_like(g_want, float("nan"))
    K_.gemm(x, [w], [None], g, epilogue=NAT.EPI_GELU_BWD, z=z_want)
    assert torch.equal(g, g_want)
    # against torch fp32: gelu_backward(approximate="tanh")
    zf = z_want.float().requires_grad_(True)
    F.gelu(zf, approximate="tanh").backward(dz_plain.float())
    assert rel(g, zf.grad) < 8e-3


def test_gemm_qknorm_aux_keeps_prenorm_qk():
    """ABI 17: the fused QKV epilogue with an aux output stores the pre-norm q | k (the LayerNorm backward's input)
    and leaves C bit-identical to the epilogue without it; at K = 128 (runtime-epilogue loop) and K = 512 (the
    default loop's aux instance); the LoRA tail form's aux instance runs in tests/test_training_gpu.py."""
    from types import SimpleNamespace

    from videopainter_amd import _native as NAT
    from videopainter_amd import kernels as K_
    from oracle.cogvideox_oracle import prepare_rotary_positional_embeddings
    H, T, B = 4, 17, 2
    D = H * 64
    cos, sin = prepare_rotary_positional_embeddings(128, 192, 3, 64)
    Ntok = T + cos.shape[0]
    rp = (cos.to(dev), sin.to(dev))
    lns = [SimpleNamespace(weight=bf(1 + 0.1 * rnd(64, seed=308 + i)).to(dev),
                           bias=bf(0.1 * rnd(64, seed=310 + i)).to(dev), eps=1e-6) for i in range(2)]
    for Kd in (128, 512):
        x = bf(rnd(B * Ntok, Kd, seed=301)).to(dev)
        ws = [bf(rnd(D, Kd, std=Kd ** -0.5, seed=302 + i)).to(dev) for i in range(3)]
        bs = [bf(rnd(D, std=0.1, seed=305 + i)).to(dev) for i in range(3)]
        plain = torch.empty(B * Ntok, 3 * D, device=dev, dtype=torch.bfloat16)
        K_.gemm(x, ws, bs, plain)
        kw = dict(epilogue=NAT.EPI_BIAS_QKNORM_ROPE, qk_norm=tuple(lns), rope=rp, tokens_per_batch=Ntok, text_len=T)
        want = torch.empty_like(plain)
        K_.gemm(x, ws, bs, want, **kw)
        got = torch.full_like(plain, float("nan"))
        aux = torch.full((B * Ntok, 2 * D), float("nan"), device=dev, dtype=torch.bfloat16)
        K_.gemm(x, ws, bs, got, aux=aux, **kw)
        assert torch.equal(got, want), Kd
        assert torch.equal(aux, plain[:, :2 * D]), Kd
        with pytest.raises(ValueError):
            K_.gemm(x, ws, bs, got, aux=aux)  # aux only with the GELU / fused-QKV epilogues


@pytest.mark.parametrize("r", [64, 256])
def test_gemm_a_tail_matches_materialized_operands(r):
    """The per-segment A tail (vp_gemm_desc.a_tail_k / a_tail_off; unfused LoRA, lora.AugmentedProjection): segment s
    of one launch reading x_aug = [x | T_0 | T_1 | T_2] with its K-tiles past K0 shifted to T_s gives, bit for bit,
    the GEMM of that segment alone on the materialised operand [x | T_s] — for the fused QKV with its qk-norm + RoPE
    epilogue, the plain bias epilogue and the gated residual of to_out (one segment) — and ragged M."""
    from types import SimpleNamespace

    from videopainter_amd import _native as N
    from videopainter_amd import kernels as K
    B, T, Nv, H = 2, 37, 1263, 4
    Ntok, D = T + Nv, H * 64
    K0 = 512
    xa = bf(rnd(B * Ntok, K0 + 3 * r, seed=140)).to(dev)
    ws = [bf(rnd(D, K0 + r, std=(K0 + r) ** -0.5, seed=141 + i)).to(dev) for i in range(3)]
    bs = [bf(rnd(D, std=0.1, seed=144 + i)).to(dev) for i in range(3)]
    lns = tuple(SimpleNamespace(weight=bf(1 + 0.1 * rnd(64, seed=147 + i)).to(dev),
                                bias=bf(0.1 * rnd(64, seed=149 + i)).to(dev), eps=1e-6) for i in range(2))
    cos, sin = rnd(Nv, 64, seed=151).to(dev), rnd(Nv, 64, seed=152).to(dev)
    resid = bf(rnd(B, Ntok, D, seed=153)).to(dev)
    mod = bf(rnd(B, 6 * D, seed=154)).to(dev)
    tail = (K0, [0, r, 2 * r])
    mat = [torch.cat([xa[:, :K0], xa[:, K0 + s * r:K0 + (s + 1) * r]], 1).contiguous() for s in range(3)]
    # bias, 3 segments
    o = torch.empty(B * Ntok, 3 * D, device=dev, dtype=torch.bfloat16)
    K.gemm(xa, ws, bs, o, a_tail=tail)
    for s in range(3):
        ref = torch.empty(B * Ntok, D, device=dev, dtype=torch.bfloat16)
        K.gemm(mat[s], [ws[s]], [bs[s]], ref)
        assert torch.equal(o[:, s * D:(s + 1) * D], ref), ("bias", s)
    # the fused QKV epilogue: q / k through LayerNorm(64) + RoPE, v plain (materialised: one 3-segment launch on a
    # stacked operand is impossible, so compare each segment's pre-norm GEMM through the unfused epilogue kernels)
    o = torch.empty(B, Ntok, 3 * D, device=dev, dtype=torch.bfloat16)
    K.gemm(xa, ws, bs, o.view(-1, 3 * D), epilogue=N.EPI_BIAS_QKNORM_ROPE, qk_norm=lns, rope=(cos, sin),
           tokens_per_batch=Ntok, text_len=T, a_tail=tail)
    pres = []
    for s in range(3):
        pre = torch.empty(B, Ntok, D, device=dev, dtype=torch.bfloat16)
        K.gemm(mat[s], [ws[s]], [bs[s]], pre.view(-1, D))
        if s < 2:
            ref = torch.empty_like(pre)
            K.head_norm_rope(pre, ref, H, T, lns[s].weight, lns[s].bias, lns[s].eps, (cos, sin))
        else:
            ref = pre
        assert torch.equal(o[..., s * D:(s + 1) * D], ref), ("qknorm", s)
        if s < 2:
            pres.append(pre)
    # the same with the aux output (ABI 17, the training forward: the pre-norm q | k) — the aux instance of the
    # tail form: C unchanged, aux = the pre-norm segments
    o2 = torch.empty_like(o)
    aux = torch.empty(B * Ntok, 2 * D, device=dev, dtype=torch.bfloat16)
    K.gemm(xa, ws, bs, o2.view(-1, 3 * D), epilogue=N.EPI_BIAS_QKNORM_ROPE, qk_norm=lns, rope=(cos, sin),
           tokens_per_batch=Ntok, text_len=T, a_tail=tail, aux=aux)
    assert torch.equal(o2, o)
    for s in range(2):
        assert torch.equal(aux[:, s * D:(s + 1) * D], pres[s].view(-1, D)), ("aux", s)
    # the gated residual (to_out: one segment reading T_0)
    o = torch.empty(B * Ntok, D, device=dev, dtype=torch.bfloat16)
    K.gemm(xa, ws[:1], bs[:1], o, epilogue=N.EPI_GATED, resid=resid, mod=mod, tokens_per_batch=Ntok, text_len=T,
           a_tail=(K0, [0]))
    ref = torch.empty_like(o)
    K.gemm(mat[0], ws[:1], bs[:1], ref, epilogue=N.EPI_GATED, resid=resid, mod=mod, tokens_per_batch=Ntok,
           text_len=T)
    assert torch.equal(o, ref)


@pytest.mark.parametrize("Kk", [512, 640, 3072])
def test_gemm_staggered_matches_quadrant_pipeline(Kk, knobs):
    """Variant 11 (the quadrant pipeline with the two wave groups staggered by one barrier), variant 13 (the default:
    11 with each slot's fragment reads before its DMA), variant 12 (two
    32-MFMA phases and one barrier per K-tile) and variant 30 (two workgroups per CU, 256 x 128 tiles, 32-K steps)
    give variant 5's result bit for bit for every epilogue kind — same MFMA order per accumulator — with ragged M, nk = 8 / 10 / 48 K-tiles
    (the steady loop, the 4-tile tail and the shortest staggered prologue), the row remap and the injection."""
    from types import SimpleNamespace

    from videopainter_amd import _native as N
    from videopainter_amd import kernels as K
    B, T, Nv, H = 2, 37, 1263, 4
    Ntok, D = T + Nv, H * 64  # M = 2600: 11 row tiles (ragged); 3 segments of 256 -> 33 tiles, nwg 32
    a = bf(rnd(B * Ntok, Kk, seed=120)).to(dev)
    ws = [bf(rnd(D, Kk, std=Kk ** -0.5, seed=121 + i)).to(dev) for i in range(3)]
    bs = [bf(rnd(D, std=0.1, seed=124 + i)).to(dev) for i in range(3)]
    resid = bf(rnd(B, Ntok, D, seed=127)).to(dev)
    mod = bf(rnd(B, 6 * D, seed=128)).to(dev)
    inj = bf(rnd(B, Nv, D, seed=129)).to(dev)
    tm = (torch.rand(B, Nv, generator=torch.Generator().manual_seed(5)) > 0.5).to(torch.uint8).to(dev)
    pos = bf(rnd(Ntok, D, seed=130)).to(dev)
    lns = tuple(SimpleNamespace(weight=bf(1 + 0.1 * rnd(64, seed=131 + i)).to(dev),
                                bias=bf(0.1 * rnd(64, seed=133 + i)).to(dev), eps=1e-6) for i in range(2))
    cos, sin = rnd(Nv, 64, seed=135).to(dev), rnd(Nv, 64, seed=136).to(dev)
    cases = {
        "bias3": lambda out: K.gemm(a, ws, bs, out.view(-1, 3 * D)),
        "qknorm": lambda out: K.gemm(a, ws, bs, out.view(-1, 3 * D), epilogue=N.EPI_BIAS_QKNORM_ROPE, qk_norm=lns,
                                     rope=(cos, sin), tokens_per_batch=Ntok, text_len=T),
        "gelu": lambda out: K.gemm(a, ws[:1], bs[:1], out.view(-1, D), epilogue=N.EPI_BIAS_GELU),
        "scale": lambda out: K.gemm(a, ws[:1], bs[:1], out.view(-1, D), epilogue=N.EPI_BIAS_SCALE, alpha=0.37),
        "gated": lambda out: K.gemm(a, ws[:1], bs[:1], out.view(-1, D), epilogue=N.EPI_GATED, resid=resid, mod=mod,
                                    tokens_per_batch=Ntok, text_len=T, inject=inj, inject_ld=D,
                                    inject_bstride=Nv * D, inject_mask=tm),
        "addrows": lambda out: K.gemm(a[:B * Nv], ws[:1], bs[:1], out.view(-1, D), epilogue=N.EPI_BIAS_ADDROWS,
                                      rows_per_group=Nv, group_stride=Ntok, row_offset=T, addrows=pos,
                                      addrows_offset=T),
    }
    for name, fn in cases.items():
        width = 3 * D if name in ("bias3", "qknorm") else D
        outs = []
        for v in [x for x in ("5", "11", "13") if K.gemm_variant_built(x)]:
            knobs.setenv("VP_GEMM_VARIANT", v)
            o = torch.full((B, Ntok, width), float("nan"), device=dev, dtype=torch.bfloat16)
            if name == "addrows":
                o.zero_()
            fn(o)
            outs.append(o)
        assert all(torch.equal(outs[0], o) for o in outs[1:]), name
        assert not torch.isnan(outs[1].float()).any(), name


def test_linear_small_timestep_patchify_unpatchify_mask():
    from videopainter_amd import kernels as K
    from oracle.cogvideox_oracle import timestep_embedding
    ts = torch.tensor([999, 377, 3, 0])
    e = K.timestep_embedding(ts.to(dev), 3072)
    assert rel(e, timestep_embedding(ts, 3072)) < 4e-3
    x = bf(rnd(4, 512, seed=90))
    w, b = bf(rnd(18432, 512, std=512 ** -0.5, seed=91)), bf(rnd(18432, std=0.1, seed=92))
    y = K.linear_small(x.to(dev), w.to(dev), b.to(dev), act_in=K.ACT_SILU)
    ref = F.linear(bf(F.silu(x.float())).float(), w.float(), b.float())
    assert rel(y, ref) < 4e-3
    y2 = K.linear_small(x.to(dev), w[:512].contiguous().to(dev), b[:512].contiguous().to(dev), act_out=K.ACT_SILU)
    assert rel(y2, F.silu(F.linear(x.float(), w[:512].float(), b[:512].float()))) < 6e-3
    B, Fr, H, W = 2, 3, 16, 24
    s1, s2 = bf(rnd(B, Fr, 16, H, W, seed=93)), bf(rnd(B, Fr, 17, H, W, seed=94))
    cols = K.patchify(s1.to(dev), s2.to(dev), 2, 192)
    wconv = rnd(64, 33, 2, 2, seed=95)
    got = cols.float().cpu()[:, :132] @ wconv.reshape(64, -1).T
    ref = F.conv2d(torch.cat([s1, s2], 2).float().reshape(-1, 33, H, W), wconv, stride=2)
    ref = ref.view(B, Fr, 64, -1).transpose(2, 3).reshape(-1, 64)
    assert rel(got, ref) < 1e-5
    assert float(cols[:, 132:].float().abs().max()) == 0.0
    proj = bf(rnd(B * Fr * (H // 2) * (W // 2), 64, seed=96))
    up = K.unpatchify(proj.to(dev), B, Fr, 16, H, W, 2)
    ref = proj.reshape(B, Fr, H // 2, W // 2, -1, 2, 2).permute(0, 1, 4, 2, 5, 3, 6).flatten(5, 6).flatten(3, 4)
    assert torch.equal(up.cpu(), ref)
    m = (torch.rand(B, Fr, 1, H, W, generator=torch.Generator().manual_seed(5)) > 0.8).float()
    tm = K.patch_mask(m.to(dev), 2)
    ref = (F.avg_pool2d(m.reshape(-1, 1, H, W), 2) > 0).view(B, Fr, -1).reshape(B, -1)
    assert torch.equal(tm.cpu().bool(), ref)


@pytest.mark.parametrize("Nq,Nk2", [(333, 0), (1500, 700), (17776, 0)])
def test_attention_tail_split_matches_unsplit(Nq, Nk2, knobs):
    """The grid-tail split (last partial round of workgroups run as key-range workgroups + a merge pass) against the
    unsplit launch of the default kernel: the same attention up to the merge's rounding; at config-2 length the
    split is exactly what the step runs (6720 blocks on 512 slots)."""
    from videopainter_amd import kernels as K
    from videopainter_amd import _native as N
    import ctypes as C
    B, H = 2, 2 if Nq < 17776 else 48
    D = H * 64
    q, k, v = (bf(rnd(B, Nq, D, seed=s)).to(dev) for s in (70, 71, 72))
    kw = {}
    if Nk2:
        kw = dict(k2=bf(rnd(B, Nk2, D, seed=73)).to(dev), v2=bf(rnd(B, Nk2, D, seed=74)).to(dev))
    d = N.AttnDesc()
    d.B, d.H, d.Nq, d.head_dim, d.Nk, d.Nk2 = B, H, Nq, 64, Nq, Nk2
    d.Q = d.K = d.V = d.O = q.data_ptr()
    d.q_sn = d.k_sn = d.v_sn = d.o_sn = D
    d.q_sb = d.k_sb = d.v_sb = d.o_sb = Nq * D
    if Nk2:
        d.K2 = d.V2 = q.data_ptr()
        d.k2_sn = d.v2_sn = D
        d.k2_sb = d.v2_sb = Nk2 * D
    assert N.lib().vp_attention_workspace_bytes(C.byref(d)) > 0  # the split is active for this shape
    out_s = torch.empty(B, Nq, D, device=dev, dtype=torch.bfloat16)
    K.attention(q, k, v, out_s, H, **kw)
    knobs.setenv("VP_ATTN_NO_SPLIT", "1")
    out_u = torch.empty_like(out_s)
    K.attention(q, k, v, out_u, H, **kw)
    # bf16 P is rounded against each range's own running max, so the two differ at bf16 noise level
    assert rel(out_s, out_u) < 5e-3
    if Nq < 17776:
        hd = lambda x: x.float().cpu().reshape(B, -1, H, 64).transpose(1, 2)  # noqa: E731
        kk, vv = hd(k), hd(v)
        if Nk2:
            kk, vv = torch.cat([kk, hd(kw["k2"])], 2), torch.cat([vv, hd(kw["v2"])], 2)
        ref = _sdpa(hd(q), kk, vv).transpose(1, 2).reshape(B, Nq, D)
        assert rel(out_s, ref) < 1e-2 and rel(out_u, ref) < 1e-2


@pytest.mark.parametrize("persist", ["1", "0"], ids=["persistent", "grid"])
@pytest.mark.parametrize("mode", ["p2a", "p2"])
@pytest.mark.parametrize("Nq,Nk2,H,tail", [(8000, 700, 17, "default"), (8000, 700, 17, "0:8"), (8000, 700, 17, "1:4"),
                                           (17776, 0, 48, "default"), (17776, 0, 48, "1:4"), (17776, 0, 48, "2:2")])
def test_attention_one_launch_tail_matches_unsplit(Nq, Nk2, H, tail, mode, persist, knobs):
    """VP_ATTN_TAIL = "R:S": the remainder blocks plus R whole rounds run as S key-range pieces each at the END of the
    main grid (one launch, then the merge pass) — against the unsplit launch; the l_extra / k2_len path through the
    pieces as well (the merge adds the null-key mass once).  persistent: the default p2 / p2a instance that takes the
    blocks and then the pieces by ticket (VP_ATTN_PERSIST); grid: one workgroup per block or piece."""
    knobs.setenv("VP_ATTN_PERSIST", persist)
    from videopainter_amd import kernels as K
    from videopainter_amd import _native as N
    import ctypes as C
    need_variant(mode, knobs)
    B, D = 2, H * 64
    sc = 0.5 if mode == "p2" else 1.0
    q, k, v = (bf(rnd(B, Nq, D, seed=s) * sc).to(dev) for s in (90, 91, 92))
    kw = dict(bounded_scores=mode == "p2")
    if Nk2:
        kw.update(k2=bf(rnd(B, Nk2, D, seed=93) * sc).to(dev), v2=bf(rnd(B, Nk2, D, seed=94)).to(dev),
                  k2_len=torch.tensor([Nk2 - 100, Nk2], dtype=torch.int32, device=dev),
                  l_extra=(torch.randn(B, H, Nq, generator=torch.Generator().manual_seed(95)) * 2).to(dev))
    knobs.setenv("VP_ATTN_BOUNDED_MODE" if mode == "p2" else "VP_ATTN_UNBOUNDED_MODE", mode)
    if tail != "default":
        knobs.setenv("VP_ATTN_TAIL", tail)
    d = N.AttnDesc()
    d.B, d.H, d.Nq, d.head_dim, d.Nk, d.Nk2 = B, H, Nq, 64, Nq, 0
    d.Q = d.K = d.V = d.O = q.data_ptr()
    d.q_sn = d.k_sn = d.v_sn = d.o_sn = D
    d.q_sb = d.k_sb = d.v_sb = d.o_sb = Nq * D
    d.flags = K.ATTN_BOUNDED_SCORES if mode == "p2" else 0
    nblk = B * H * ((Nq + 255) // 256)
    # default: R = 0, S = min(8, ceil(2 slots / remainder))
    R, S = (0, min(8, -(-1024 // (nblk % 512)))) if tail == "default" else (int(x) for x in tail.split(":"))
    assert nblk % 512 + (R + 1) * 512 <= nblk  # (the plan keeps at least one whole round unsplit)
    ws = N.lib().vp_attention_workspace_bytes(C.byref(d))
    assert ws >= (nblk % 512 + R * 512) * S * 256 * 66 * 4  # the one-launch split is active for this shape
    out_s = torch.empty(B, Nq, D, device=dev, dtype=torch.bfloat16)
    K.attention(q, k, v, out_s, H, **kw)
    knobs.setenv("VP_ATTN_NO_SPLIT", "1")
    knobs.setenv("VP_ATTN_PERSIST", "0")
    out_u = torch.empty_like(out_s)
    K.attention(q, k, v, out_u, H, **kw)
    assert rel(out_s, out_u) < 5e-3


@pytest.mark.parametrize("mode", ["p2a", "p2"])
@pytest.mark.parametrize("B,Nq,H", [(2, 17776, 48), (1, 17776, 48), (2, 4100, 33)])
def test_attention_persistent_bit_identical_without_tail(B, Nq, H, mode, knobs):
    """The persistent p2 / p2a instance (blocks by per-XCD tickets, then stolen across XCDs) computes every block
    exactly as its own workgroup would: without the tail split the outputs and the softmax statistics are
    bit-identical to one workgroup per block, whatever order the tickets came in."""
    from videopainter_amd import kernels as K
    need_variant(mode, knobs)
    D = H * 64
    sc = 0.5 if mode == "p2" else 1.0
    q, k, v = (bf(rnd(B, Nq, D, seed=s) * sc).to(dev) for s in (96, 97, 98))
    knobs.setenv("VP_ATTN_BOUNDED_MODE" if mode == "p2" else "VP_ATTN_UNBOUNDED_MODE", mode)
    knobs.setenv("VP_ATTN_NO_SPLIT", "1")
    outs, lses = [], []
    for persist in ("1", "0"):
        knobs.setenv("VP_ATTN_PERSIST", persist)
        o = torch.empty(B, Nq, D, device=dev, dtype=torch.bfloat16)
        lse = torch.empty(B, H, Nq, device=dev, dtype=torch.float32)
        K.attention(q, k, v, o, H, bounded_scores=mode == "p2", lse=lse)
        outs.append(o)
        lses.append(lse)
    assert torch.equal(outs[0], outs[1])
    assert torch.equal(lses[0], lses[1])


@pytest.mark.parametrize("mode", ["p2", "s16"])
@pytest.mark.parametrize("Nq,Nk2", [(1500, 700), (17776, 0)])
def test_attention_bounded_tail_split_matches_unsplit(Nq, Nk2, mode, knobs):
    """The bounded-score kernels' grid-tail split instances (partials + merge) against their unsplit launch and, at
    small size, against fp32 attention."""
    from videopainter_amd import kernels as K
    need_variant(mode, knobs)
    B, H = 2, 2 if Nq < 17776 else 48
    D = H * 64
    q, k, v = (bf(rnd(B, Nq, D, seed=s) * 0.5).to(dev) for s in (80, 81, 82))
    kw = dict(bounded_scores=True)
    if Nk2:
        kw.update(k2=bf(rnd(B, Nk2, D, seed=83) * 0.5).to(dev), v2=bf(rnd(B, Nk2, D, seed=84)).to(dev))
    out_s = torch.empty(B, Nq, D, device=dev, dtype=torch.bfloat16)
    K.attention(q, k, v, out_s, H, **kw)
    knobs.setenv("VP_ATTN_NO_SPLIT", "1")
    out_u = torch.empty_like(out_s)
    K.attention(q, k, v, out_u, H, **kw)
    assert rel(out_s, out_u) < 5e-3
    if Nq < 17776:
        hd = lambda x: x.float().cpu().reshape(B, -1, H, 64).transpose(1, 2)  # noqa: E731
        kk, vv = hd(k), hd(v)
        if Nk2:
            kk, vv = torch.cat([kk, hd(kw["k2"])], 2), torch.cat([vv, hd(kw["v2"])], 2)
        ref = _sdpa(hd(q), kk, vv).transpose(1, 2).reshape(B, Nq, D)
        assert rel(out_s, ref) < 1e-2 and rel(out_u, ref) < 1e-2


@pytest.mark.parametrize("epi", ["bias", "gelu", "scale", "addrows"])
@pytest.mark.parametrize("M,Nn,Kk,segs", [(452, 1536, 4096, 3), (200, 2048, 2560, 1), (37, 512, 1024, 1)])
def test_gemm_splitk_small_m(M, Nn, Kk, segs, epi):
    """Split-K path (vp_gemm_bf16_ws) for GEMMs with too few output tiles (the T5 encoder's projections): every
    epilogue it serves against torch fp32, the reduce's fixed chunk order makes it deterministic, and the plan really
    splits.  Tolerance: bf16 output rounding (the chunked fp32 sum differs from the unsplit one only in fp32 order)."""
    from videopainter_amd import _native as N
    from videopainter_amd import kernels as K
    torch.manual_seed(M + Nn)
    a = torch.randn(M, Kk, device=dev).bfloat16()
    ws = [(torch.randn(Nn // segs, Kk, device=dev) * Kk ** -0.5).bfloat16() for _ in range(segs)]
    bs = [(torch.randn(Nn // segs, device=dev) * 0.1).bfloat16() for _ in range(segs)]
    w = torch.cat(ws)
    b = torch.cat(bs)
    y = (a.float() @ w.float().t() + b.float()).bfloat16().float()
    kw = {}
    out = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
    if epi == "gelu":
        kw["epilogue"] = N.EPI_BIAS_GELU
        ref = F.gelu(y, approximate="tanh")
    elif epi == "scale":
        kw.update(epilogue=N.EPI_BIAS_SCALE, alpha=0.7)
        ref = y * 0.7
    elif epi == "addrows":
        out = torch.randn(M, Nn, device=dev).bfloat16()  # in place, like the T5 residual adds
        kw.update(epilogue=N.EPI_BIAS_ADDROWS, addrows=out)
        ref = y + out.float()
    else:
        ref = y
    d = N.GemmDesc()
    d.M, d.N, d.K, d.epilogue, d.n_seg = M, Nn, Kk, kw.get("epilogue", N.EPI_BIAS), Nn // segs
    assert N.lib().vp_gemm_bf16_workspace_bytes(d) > 0, "expected the split-K plan for this shape"
    K.gemm(a, ws, bs, out, **kw)
    got = out.float()
    err = (got - ref).abs().max().item()
    assert err <= 0.02 * ref.abs().max().item() + 1e-2, err
    if epi != "addrows":
        again = torch.empty_like(out)
        K.gemm(a, ws, bs, again, **kw)
        assert torch.equal(again, out)


@pytest.mark.parametrize("B,N", [(2, 1378), (1, 17776), (3, 65)])
def test_partition_rows_index_and_permuted_writes(B, N):
    """vp_partition_rows_index (stable: set rows first, then the clear rows, each in order; device-side counts) and
    the permuted writes of vp_head_norm_rope_bf16 / vp_mask_scale_rows_bf16 (row n -> dst_rows[b, n]), bit-equal to
    the unpermuted kernels followed by the permutation."""
    from videopainter_amd import kernels as K
    g = torch.Generator().manual_seed(N)
    m = (torch.rand(B, N, generator=g) < 0.37).to(torch.uint8)
    m[0, :min(N, 10)] = 0
    dst, cnt = K.partition_rows_index(m.to(dev))
    for b in range(B):
        want = torch.empty(N, dtype=torch.int64)
        idx1 = torch.nonzero(m[b]).flatten()
        idx0 = torch.nonzero(m[b] == 0).flatten()
        want[idx1] = torch.arange(len(idx1))
        want[idx0] = len(idx1) + torch.arange(len(idx0))
        assert int(cnt[b]) == len(idx1)
        assert torch.equal(dst[b].cpu().long(), want)
    H, T = 2, min(8, N // 2)
    D = H * 64
    x = bf(rnd(B, N, D, seed=5)).to(dev)
    lw, lb = bf(rnd(64, seed=6)).to(dev), bf(rnd(64, seed=7) * 0.1).to(dev)
    cos, sin = (torch.rand(N - T, 64, generator=g) * 2 - 1).to(dev), (torch.rand(N - T, 64, generator=g) * 2 - 1).to(dev)
    ref = torch.empty_like(x)
    K.head_norm_rope(x, ref, H, T, lw, lb, 1e-6, (cos, sin), tok_mask=m.to(dev), pre_scale=0.5)
    got = torch.empty_like(x)
    K.head_norm_rope(x, got, H, T, lw, lb, 1e-6, (cos, sin), tok_mask=m.to(dev), pre_scale=0.5, dst_rows=dst)
    vref = torch.empty_like(x)
    K.mask_scale_rows(x, vref, m.to(dev), 0.5)
    vgot = torch.empty_like(x)
    K.mask_scale_rows(x, vgot, m.to(dev), 0.5, dst_rows=dst)
    for b in range(B):
        perm = dst[b].long()
        assert torch.equal(got[b][perm], ref[b]) and torch.equal(vgot[b][perm], vref[b])
        assert not vgot[b, int(cnt[b]):].any()  # the null keys' values are zero (the k2_full contract)


@pytest.mark.parametrize("mode", ["s16", "a16", "p2a", "p2w", "p2w2", "p2s", "p2"])
def test_attention_k2_full_hint(mode, knobs):
    """The k2_full hint (segment-2 keys past k2_full[b] have zero values: row sums only) gives the attention of the
    same segments without the hint; per-batch split points, one straddling a tile, one past every tile."""
    from videopainter_amd import kernels as K
    need_variant(mode, knobs)
    kw = {} if mode in UNBOUNDED_VARIANTS else dict(bounded_scores=True)
    B, H, Nn, N2 = 3, 2, 700, 900
    D = H * 64
    q, k, v = (bf(rnd(B, Nn, D, seed=s) * 0.5).to(dev) for s in (90, 91, 92))
    k2, v2 = bf(rnd(B, N2, D, seed=93) * 0.5).to(dev), bf(rnd(B, N2, D, seed=94)).to(dev)
    full = torch.tensor([300, 0, 900], dtype=torch.int32)
    for b in range(B):
        v2[b, int(full[b]):] = 0
    o_ref = torch.empty(B, Nn, D, device=dev, dtype=torch.bfloat16)
    K.attention(q, k, v, o_ref, H, k2=k2, v2=v2, **kw)
    o = torch.empty_like(o_ref)
    K.attention(q, k, v, o, H, k2=k2, v2=v2, k2_full=full.to(dev), **kw)
    hd = lambda x: x.float().cpu().reshape(B, -1, H, 64).transpose(1, 2)  # noqa: E731
    ref = _sdpa(hd(q), torch.cat([hd(k), hd(k2)], 2), torch.cat([hd(v), hd(v2)], 2)).transpose(1, 2).reshape(B, Nn, D)
    # (p2a does not take the hint: the hinted launch runs a16, whose bf16 P is rounded against other anchors)
    assert rel(o, ref) < 1e-2 and rel(o, o_ref) < (5e-3 if mode in ("p2a", "p2w", "p2w2", "p2s") else 2e-3)


def _grid_rope(F_, Hh, Ww):
    from oracle.cogvideox_oracle import prepare_rotary_positional_embeddings
    cos, sin = prepare_rotary_positional_embeddings(Hh * 16, Ww * 16, F_, 64)
    return cos.float(), sin.float()


def _null_mass_ref(q, H, T, cos, sin, beta, m, scale):
    """fp64: log2 sum over the mask-0 rows j of 2^(scale log2 e q.k_j), k_j = beta (text) / RoPE(beta) rounded to
    bf16 (video: the key the reference's bf16 apply_rotary_emb writes)."""
    B, Ntok, _ = q.shape
    bt = beta.double().cpu()
    rot = torch.stack([-bt[1::2], bt[0::2]], -1).reshape(64)  # apply_rotary_emb's interleaved pairs
    kv = (bt[None] * cos.double() + rot[None] * sin.double()).to(torch.bfloat16).double()
    keys = torch.cat([bt[None].expand(T, 64), kv], 0)
    qh = q.double().cpu().view(B, Ntok, H, 64)
    s = torch.einsum("bnhd,kd->bhnk", qh, keys) * (scale * 1.4426950408889634)
    s = s.masked_fill(m.cpu().bool()[:, None, None, :], float("-inf"))
    return torch.logsumexp(s * 0.6931471805599453, -1) / 0.6931471805599453


def test_null_key_mass_matches_explicit_null_keys():
    """The resample processor's null keys in closed form (resample.hip, DESIGN_LOG.md §3.0) against the explicit sum over
    every mask-0 row in fp64: text rows all / partly null, a video row with 8 runs (the per-column fallback), an
    all-null and a no-null row, a batch row without any null key (-inf)."""
    from videopainter_amd import kernels as K
    B, H, T, F_, Hh, Ww = 3, 3, 7, 3, 5, 16
    grid = (F_, Hh, Ww)
    cos, sin = _grid_rope(*grid)
    Ntok = T + F_ * Hh * Ww
    g = torch.Generator().manual_seed(5)
    m = torch.rand(B, Ntok, generator=g) < 0.5
    m[0, :T] = False
    vid = m[:, T:].view(B, F_, Hh, Ww)
    vid[0, 1, 2] = torch.arange(Ww) % 2 == 1
    vid[1, 0, 0] = False
    vid[1, 2, 4] = True
    m[2] = True
    m8 = m.to(torch.uint8).to(dev)
    q = bf(rnd(B, Ntok, H * 64, seed=60) * 1.5).to(dev)
    beta = bf(rnd(64, seed=61) * 0.8).to(dev)
    axes = K.rope_axis_tables((cos.to(dev), sin.to(dev)), grid)
    assert axes is not None
    segs, meta = K.mask_null_segments(m8, T, grid)
    # the segment records against a host scan: runs of equal consecutive rows with null keys
    mc = m.cpu()
    for b in range(B):
        for t in range(F_):
            rows = []
            for y in range(Hh):
                row = mc[b, T + (t * Hh + y) * Ww:T + (t * Hh + y + 1) * Ww]
                runs, x = [], 0
                while x < Ww:
                    if row[x]:
                        x += 1
                        continue
                    x0 = x
                    while x < Ww and not row[x]:
                        x += 1
                    runs.append((x0, x))
                rows.append(runs)
            want = []
            for y, runs in enumerate(rows):
                if y > 0 and runs == rows[y - 1] and len(runs) <= 6 and want and want[-1][1] == y:
                    want[-1][1] = y + 1
                elif runs:
                    want.append([y, y + 1, runs])
            got = segs[(b * F_ + t) * Hh:(b * F_ + t) * Hh + int(meta[b * F_ + t])].cpu()
            assert len(got) == len(want), (b, t)
            for r, (y0, y1, runs) in zip(got.tolist(), want):
                n = len(runs) if len(runs) <= 6 else 255
                assert (r[0], r[1], r[2]) == (y0, y1, n), (b, t, r, y0, y1, runs)
                if n != 255:
                    assert [(r[4 + 2 * k], r[5 + 2 * k]) for k in range(n)] == runs
        assert int(meta[B * F_ + b]) == int((~mc[b, :T]).sum())
    assert int(segs[(0 * F_ + 1) * Hh:(0 * F_ + 1) * Hh + int(meta[1]), 2].eq(255).sum()) == 1  # the 8-run row
    lx = K.null_key_mass(q, H, T, grid, beta, axes, m8, (segs, meta), 0.125).double().cpu()
    ref = _null_mass_ref(q, H, T, cos, sin, beta, m, 0.125)
    assert torch.isinf(lx[2]).all() and (lx[2] < 0).all()
    assert torch.isfinite(lx[:2]).all()
    err = float((lx[:2] - ref[:2]).abs().max())
    assert err < 2e-4, err


@pytest.mark.parametrize("split", [True, False], ids=["tailsplit", "nosplit"])
@pytest.mark.parametrize("mode", ["s16", "a16", "p2a", "p2w", "p2w2", "p2s", "p2"])
def test_attention_k2_len_and_l_extra(mode, split, knobs):
    """k2_len (only the first k2_len[b] keys of segment 2) and l_extra (extra row-sum mass per query, log2 score
    units) against fp64 attention over the truncated segments with 2^l_extra added to each denominator.  At this size
    every block is in the grid tail: the split launch (with empty key ranges where k2_len = 0 leaves fewer tiles than
    splits) and the combine kernel carry l_extra; a16 / p2a also get masses far above their anchors (a16: the exact
    re-run; p2a: a non-finite row sum, so the block is flagged and re-run by a16)."""
    from videopainter_amd import kernels as K
    need_variant(mode, knobs)
    kw = {} if mode in UNBOUNDED_VARIANTS else dict(bounded_scores=True)
    if not split:
        knobs.setenv("VP_ATTN_NO_SPLIT", "1")
    B, H, Nn, N2 = 3, 2, 700, 900
    D = H * 64
    q, k, v = (bf(rnd(B, Nn, D, seed=s) * 0.5).to(dev) for s in (95, 96, 97))
    k2, v2 = bf(rnd(B, N2, D, seed=98) * 0.5).to(dev), bf(rnd(B, N2, D, seed=99)).to(dev)
    klen = torch.tensor([300, 0, 900], dtype=torch.int32)
    lx = rnd(B, H, Nn, seed=100) * 4.0 + 3.0
    lx[:, :, ::7] = float("-inf")
    if mode in UNBOUNDED_VARIANTS:
        lx[0, 0, 5::50] = 150.0
        lx[1, 1, 9::60] = 90.0
    o = torch.empty(B, Nn, D, device=dev, dtype=torch.bfloat16)
    K.attention(q, k, v, o, H, k2=k2, v2=v2, k2_len=klen.to(dev), l_extra=lx.to(dev), **kw)
    hd = lambda x: x.double().cpu().reshape(x.shape[0], -1, H, 64).transpose(1, 2)  # noqa: E731
    ref = torch.empty(B, H, Nn, 64, dtype=torch.float64)
    for b in range(B):
        n2 = int(klen[b])
        kk = torch.cat([hd(k[b:b + 1]), hd(k2[b:b + 1, :n2])], 2)[0]
        vv = torch.cat([hd(v[b:b + 1]), hd(v2[b:b + 1, :n2])], 2)[0]
        s = (hd(q[b:b + 1])[0] @ kk.transpose(-1, -2)) * (0.125 * 1.4426950408889634)
        ex = lx[b].double()
        mx = torch.maximum(s.amax(-1), ex)
        p = torch.exp2(s - mx[..., None])
        ref[b] = (p @ vv) / (p.sum(-1) + torch.exp2(ex - mx))[..., None]
    ref = ref.transpose(1, 2).reshape(B, Nn, D)
    assert torch.isfinite(o.float()).all()
    assert rel(o, ref) < 1e-2, rel(o, ref)


@pytest.mark.parametrize("split", [True, False], ids=["tailsplit", "nosplit"])
@pytest.mark.parametrize("mode", ["p2a", "p2w", "p2w2", "p2s", "p2"])
def test_attention_segment2_fast_path_bit_identical(mode, split, knobs):
    """Segment 2 with segment 1's row strides (the resample processor's layout: K2 / V2 as slices of a [B, N, 3D]
    buffer) streams its full 128-key tiles on segment 1's precomputed lane offsets; the same keys as contiguous
    tensors take the general DMA path.  Only the addressing differs, so the outputs are equal bit for bit — with
    k2_len leaving partial and whole-tile segment ends (0, 128, 300, 1024 keys) and l_extra."""
    from videopainter_amd import kernels as K
    need_variant(mode, knobs)
    kw = {} if mode in UNBOUNDED_VARIANTS else dict(bounded_scores=True)
    if not split:
        knobs.setenv("VP_ATTN_NO_SPLIT", "1")
    B, H, Nn = 4, 2, 700
    D = H * 64
    qkv = bf(rnd(B, Nn, 3 * D, seed=61) * 0.5).to(dev)
    q, k, v = qkv[..., :D], qkv[..., D:2 * D], qkv[..., 2 * D:]
    kv2 = bf(rnd(B, 1024, 3 * D, seed=62) * 0.5).to(dev)
    k2s, v2s = kv2[..., :D], kv2[..., D:2 * D]
    assert k2s.stride(1) == k.stride(1) and v2s.stride(1) == v.stride(1)
    klen = torch.tensor([300, 0, 1024, 128], dtype=torch.int32, device=dev)
    lx = (rnd(B, H, Nn, seed=63) * 4.0 + 3.0).to(dev)
    outs = []
    for k2, v2 in ((k2s, v2s), (k2s.contiguous(), v2s.contiguous())):
        o = torch.empty(B, Nn, D, device=dev, dtype=torch.bfloat16)
        K.attention(q, k, v, o, H, k2=k2, v2=v2, k2_len=klen, l_extra=lx, **kw)
        outs.append(o)
    torch.cuda.synchronize()
    assert torch.isfinite(outs[0].float()).all()
    assert torch.equal(outs[0].view(torch.int16), outs[1].view(torch.int16))


@pytest.mark.parametrize("split", [True, False], ids=["tailsplit", "nosplit"])
@pytest.mark.parametrize("spread", [False, True], ids=["even", "spread"])
@pytest.mark.parametrize("mode", ["p2a", "p2w", "p2w2", "p2s", "a16", "p2", "s16"])
def test_attention_lse_matches_reference(mode, spread, split, knobs):
    """The softmax statistics the backward reads (lse = log2 sum_k 2^(scale log2e q.k), fp32 [B, H, Nq]) and the
    output against fp64, per variant.  spread: queries of very different norms in one wave (x0.02 .. x2.5), so an
    anchored kernel's shared reference point sits far above some queries' scores."""
    from videopainter_amd import kernels as K
    need_variant(mode, knobs)
    if not split:
        knobs.setenv("VP_ATTN_NO_SPLIT", "1")
    B, H, Nn = 2, 2, 700
    D = H * 64
    q, k, v = (rnd(B, Nn, D, seed=s) * 0.5 for s in (195, 196, 197))
    if spread:
        q = q * torch.where(torch.arange(Nn) % 3 == 0, 0.02, 2.5)[None, :, None]
    q, k, v = (bf(x).to(dev) for x in (q, k, v))
    kw = attn_kw(mode, q, k)
    o = torch.empty(B, Nn, D, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B, H, Nn, device=dev, dtype=torch.float32)
    K.attention(q, k, v, o, H, lse=lse, **kw)
    hd = lambda x: x.double().cpu().reshape(B, -1, H, 64).transpose(1, 2)  # noqa: E731
    s = (hd(q) @ hd(k).transpose(-1, -2)) * (0.125 * 1.4426950408889634)
    ref_lse = torch.logsumexp(s * math.log(2.0), -1) / math.log(2.0)
    ref = (torch.softmax(s * math.log(2.0), -1) @ hd(v)).transpose(1, 2).reshape(B, Nn, D)
    err = float((lse.double().cpu() - ref_lse).abs().max())
    bias = float((lse.double().cpu() - ref_lse).mean())
    print(f"lse {mode} spread={spread} split={split}: max err {err:.2e} mean {bias:.2e} out rel {rel(o, ref):.2e}")
    assert err < 4e-3, err
    assert rel(o, ref) < 1e-2, rel(o, ref)


@pytest.mark.parametrize("M,K_,act_in,act_out", [(2, 512, 1, 0), (1, 512, 0, 1), (2, 256, 0, 0), (2, 3072, 1, 0)])
def test_linear_small_fast_path_bit_identical(M, K_, act_in, act_out):
    """vp_linear_small_bf16's weight-streaming kernel (M <= 2, K <= 512, 16-byte aligned rows) against its general
    kernel (taken here through an x row stride that is not a multiple of 8): the same per-lane products and wave sums,
    so bit-identical; both against torch fp32."""
    from videopainter_amd import kernels as K
    x = bf(rnd(M, K_, seed=300))
    w, b = bf(rnd(4100, K_, std=K_ ** -0.5, seed=301)), bf(rnd(4100, std=0.1, seed=302))
    xd = x.to(dev)
    xs = torch.zeros(M, K_ + 4, device=dev, dtype=torch.bfloat16)
    xs[:, :K_] = xd
    y_fast = K.linear_small(xd, w.to(dev), b.to(dev), act_in=act_in, act_out=act_out)
    y_gen = K.linear_small(xs[:, :K_], w.to(dev), b.to(dev), act_in=act_in, act_out=act_out)
    assert torch.equal(y_fast, y_gen)
    xin = bf(F.silu(x.float())).float() if act_in else x.float()
    ref = F.linear(xin, w.float(), b.float())
    if act_out:
        ref = F.silu(ref)
    assert rel(y_fast, ref) < 6e-3
