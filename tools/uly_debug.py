"""Debug helper: Ulysses split vs unsplit at P=1/2, intermediate tensors (branch samples, block-0 output)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


def main():
    from videopainter_amd import CogVideoXTransformer3DModel, CogvideoXBranchModel, device_scope
    from videopainter_amd import ulysses as U
    from videopainter_amd.embeddings import prepare_rotary_positional_embeddings
    from tests.golden.cases import TINY_CFG
    dev = "cuda"
    cfg = dict(TINY_CFG, num_attention_heads=4, max_text_seq_length=10, num_layers=3)
    with device_scope(dev):
        tr = CogVideoXTransformer3DModel(**cfg)
        br = CogvideoXBranchModel(**dict(cfg, num_layers=2))
    tr.init_synthetic_weights_(11)
    br.init_synthetic_weights_(12)
    g = torch.Generator().manual_seed(13)
    B, F, H, W = 2, 3, 16, 24
    video = torch.randn(B, F, 16, H, W, generator=g)
    cond = torch.cat([video, torch.zeros(B, F, 1, H, W)], 2).to(dev).bfloat16()
    enc = torch.randn(B, 10, 32, generator=g).to(dev).bfloat16()
    ts = torch.tensor([500, 500], device=dev)
    rope = tuple(t.to(dev) for t in prepare_rotary_positional_embeddings(H * 8, W * 8, F, 64))
    vid = video.to(dev).bfloat16()
    with torch.no_grad():
        bs = br(hidden_states=vid, encoder_hidden_states=enc, branch_cond=cond, timestep=ts, image_rotary_emb=rope,
                return_dict=False)[0]
    hidden = torch.cat([vid, vid * 0.5], 2)
    mask = torch.zeros(B, F, 1, H, W, device=dev, dtype=torch.bfloat16)
    mask[:, 1:, :, 4:12, 6:18] = 1
    with torch.no_grad():
        ref, hs = tr(hidden_states=hidden, encoder_hidden_states=enc, timestep=ts, image_rotary_emb=rope,
                     branch_block_samples=bs, branch_block_masks=mask, return_hidden_states=True, return_dict=False)[:2]
        ref = ref.clone()
        hs = [h.clone() for h in hs]
    for P in (1, 2):
        comm = U.ThreadComm(P)

        def fn(r):
            s = U.branch_forward(br, comm, r, vid, enc, cond, ts, rope)
            return U.transformer_forward(tr, comm, r, hidden, enc, ts, rope, s, mask, return_hidden_states=True)
        res = comm.run(fn)
        N = hs[0].shape[1]
        for r, (out, hsl) in enumerate(res):
            sh = U.Shard(N, 10, P, r)
            print("tr", P, r, f"out {rel(out, ref):.2e}", [f"{rel(h[:, :sh.valid], g[:, sh.r0:sh.r0 + sh.valid]):.2e}"
                                                           for h, g in zip(hsl, hs)], flush=True)
        comm = U.ThreadComm(P)
        res = comm.run(lambda r: U.branch_forward(br, comm, r, vid, enc, cond, ts, rope))
        for r, samples in enumerate(res):
            sh = U.Shard(bs[0].shape[1] + 10, 10, P, r)
            k = min(sh.nv, bs[0].shape[1] - sh.v0)
            print(P, r, [f"{rel(s[:, :k], b[:, sh.v0:sh.v0 + k]):.2e}" for s, b in zip(samples, bs)], flush=True)


if __name__ == "__main__":
    main()
