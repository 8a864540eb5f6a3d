"""Ulysses head-parallel split (videopainter_amd/ulysses.py) on the GPU: P ranks emulated by P threads on one
device (ThreadComm: the same per-rank launches, exchanges as local copies) against the unsplit forward of the same
models.  Row-local kernels give identical rows and attention runs per (batch, head) workgroup, so the split is
bit-identical to the unsplit forward at this size (measured: rel 0; at sizes where the attention grid's tail split
engages, a head-group launch may partition a few query blocks' keys differently — the full-size rehearsal is
`bench.py --mode ulysses`).  Both processors of the any-length pipeline are covered, with the window hand-off."""
import pytest
import torch

pytestmark = pytest.mark.gpu
dev = "cuda"


def rel(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


@pytest.fixture(scope="module")
def env():
    from videopainter_amd import CogVideoXTransformer3DModel, CogvideoXBranchModel, device_scope
    from videopainter_amd.embeddings import prepare_rotary_positional_embeddings
    from tests.golden.cases import TINY_CFG
    cfg = dict(TINY_CFG, num_attention_heads=4, max_text_seq_length=10, num_layers=3)
    with device_scope(dev):
        tr = CogVideoXTransformer3DModel(**cfg)
        br = CogvideoXBranchModel(**dict(cfg, num_layers=2))
    tr.init_synthetic_weights_(11)
    br.init_synthetic_weights_(12)
    g = torch.Generator().manual_seed(13)
    B, F, H, W = 2, 3, 16, 24
    video = torch.randn(B, F, 16, H, W, generator=g)
    mask = torch.zeros(B, F, 1, H, W)
    mask[:, 1:, :, 4:12, 6:18] = 1.0
    inp = dict(video=video.to(dev).bfloat16(),
               hidden=torch.cat([video, torch.randn(B, F, 16, H, W, generator=g)], 2).to(dev).bfloat16(),
               cond=torch.cat([video * (1 - mask), mask], 2).to(dev).bfloat16(),
               enc=torch.randn(B, 10, 32, generator=g).to(dev).bfloat16(), mask=mask.to(dev).bfloat16(),
               ts=torch.tensor([500, 500], device=dev),
               rope=tuple(t.to(dev) for t in prepare_rotary_positional_embeddings(H * 8, W * 8, F, 64)))
    with torch.no_grad():
        bs = br(hidden_states=inp["video"], encoder_hidden_states=inp["enc"], branch_cond=inp["cond"],
                timestep=inp["ts"], image_rotary_emb=inp["rope"], return_dict=False)[0]
        ref, hs = tr(hidden_states=inp["hidden"], encoder_hidden_states=inp["enc"], timestep=inp["ts"],
                     image_rotary_emb=inp["rope"], branch_block_samples=bs, branch_block_masks=inp["mask"],
                     return_hidden_states=True, return_dict=False)[:2]
    return dict(tr=tr, br=br, inp=inp, ref=ref, hs=[h.clone() for h in hs], bs=[b.clone() for b in bs])


@pytest.mark.parametrize("P", [2, 4])
def test_ulysses_split_matches_unsplit(env, P):
    from videopainter_amd import ulysses as U
    i = env["inp"]
    comm = U.ThreadComm(P)

    def rank_fn(r):
        samples = U.branch_forward(env["br"], comm, r, i["video"], i["enc"], i["cond"], i["ts"], i["rope"])
        out, hsl = U.transformer_forward(env["tr"], comm, r, i["hidden"], i["enc"], i["ts"], i["rope"], samples,
                                         i["mask"], return_hidden_states=True)
        return out, hsl, samples

    res = comm.run(rank_fn)
    T = 10
    N = env["hs"][0].shape[1]
    for r, (out, hsl, samples) in enumerate(res):
        ro = rel(out, env["ref"])
        print(f"P={P} rank {r}: noise prediction rel {ro:.2e}")
        assert out.shape == env["ref"].shape and torch.equal(out, env["ref"])
        sh = U.Shard(N, T, P, r)
        for k, h in enumerate(hsl):
            assert rel(h[:, :sh.valid], env["hs"][k][:, sh.r0:sh.r0 + sh.valid]) < 1e-3, (r, k)
        for j, s in enumerate(samples):  # the branch samples: this shard's video rows
            k = max(0, min(sh.nv, N - T - sh.v0))
            assert rel(s[:, :k], env["bs"][j][:, sh.v0:sh.v0 + k]) < 1e-3
    assert all(torch.equal(res[0][0], o[0]) for o in res)  # every rank holds the same prediction


def test_ulysses_harness_call_forms(env):
    """UlyssesModels exposes the harness's call forms (branch(...)[0]; transformer(...) -> (pred, hs, mask))."""
    from videopainter_amd import ulysses as U
    i = env["inp"]
    comm = U.ThreadComm(2)

    def rank_fn(r):
        m = U.UlyssesModels(env["tr"], env["br"], comm, rank=r)
        bs = m.branch(hidden_states=i["video"], encoder_hidden_states=i["enc"], branch_cond=i["cond"],
                      timestep=i["ts"], image_rotary_emb=i["rope"], return_dict=False)[0]
        return m.transformer(hidden_states=i["hidden"], encoder_hidden_states=i["enc"], timestep=i["ts"],
                             image_rotary_emb=i["rope"], branch_block_samples=bs, branch_block_masks=i["mask"],
                             return_hidden_states=True, return_resample_mask=True, return_dict=False)

    for pred, hsl, rm in comm.run(rank_fn):
        assert rel(pred, env["ref"]) < 1e-3 and len(hsl) == 3 and rm.shape == (2, env["hs"][0].shape[1])


@pytest.mark.parametrize("P", [2, 4])
@pytest.mark.parametrize("resample", [True, False], ids=["resample", "standard"])
def test_ulysses_any_length_window_handoff(env, P, resample):
    """The any-length pipeline's processors under the split (anyl.py:962-988): window 0 and a later window that
    gets window 0's hidden states (the split's own shard states), prev_clip_weight 0.5 and the previous resample
    mask — the ID-resample processor (masked second K / V segment, null keys in closed form) and the standard one
    (the previous-clip blend) — against the unsplit forward of the same model."""
    from videopainter_amd import CogVideoXTransformer3DModel, device_scope
    from videopainter_amd import ulysses as U
    from tests.golden.cases import TINY_CFG
    i = env["inp"]
    g = torch.Generator().manual_seed(21)
    hidden2 = (i["hidden"].float().cpu() + 0.5 * torch.randn(i["hidden"].shape, generator=g)).to(dev).bfloat16()
    if resample:
        cfg = dict(TINY_CFG, num_attention_heads=4, max_text_seq_length=10, num_layers=3,
                   id_pool_resample_learnable=True)
        with device_scope(dev):
            tr = CogVideoXTransformer3DModel(**cfg)
        tr.init_synthetic_weights_(11)
    else:
        tr = env["tr"]
    bs = env["bs"]
    kw = dict(encoder_hidden_states=i["enc"], timestep=i["ts"], image_rotary_emb=i["rope"], branch_block_samples=bs,
              branch_block_masks=i["mask"], id_pool_resample_learnable=resample, return_dict=False)
    with torch.no_grad():
        ref0, hs0, rm0 = tr(hidden_states=i["hidden"], return_hidden_states=True, return_resample_mask=True, **kw)
        ref1 = tr(hidden_states=hidden2, attention_kwargs={"prev_hidden_states": dict(enumerate(hs0)),
                                                           "prev_clip_weight": 0.5, "prev_resample_mask": rm0},
                  **kw)[0]
    comm = U.ThreadComm(P)

    def rank_fn(r):
        samples = U.branch_forward(env["br"], comm, r, i["video"], i["enc"], i["cond"], i["ts"], i["rope"])
        out0, hsl = U.transformer_forward(tr, comm, r, i["hidden"], i["enc"], i["ts"], i["rope"], samples, i["mask"],
                                          return_hidden_states=True, id_pool_resample_learnable=resample)
        out1 = U.transformer_forward(tr, comm, r, hidden2, i["enc"], i["ts"], i["rope"], samples, i["mask"],
                                     id_pool_resample_learnable=resample, prev_hidden_states=dict(enumerate(hsl)),
                                     prev_clip_weight=0.5, prev_resample_mask=rm0)[0]
        return out0, out1

    for r, (out0, out1) in enumerate(comm.run(rank_fn)):
        r0, r1 = rel(out0, ref0), rel(out1, ref1)
        print(f"P={P} {'resample' if resample else 'standard'} rank {r}: window 0 rel {r0:.2e}, window 1 rel {r1:.2e}")
        assert out0.shape == ref0.shape and out1.shape == ref1.shape
        assert r0 < 1e-3 and r1 < 1e-3, (r, r0, r1)
    if resample:
        del tr
