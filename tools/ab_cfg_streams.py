"""A/B of the CFG-half stream split (CogVideoXTransformer3DModel.enable_cfg_streams) on the config-2 bench step,
interleaved in one process: rounds x (off, on) of `--steps` timed steps each, then the noise prediction of one
forward in both modes compared (max |diff|, rel-L2).

    python tools/ab_cfg_streams.py --rounds 3 --steps 3
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--branch", action="store_true", help="also split the branch")
    args = ap.parse_args()
    bench.set_config(2)
    from videopainter_amd.pipeline import CogVideoXI2VDualInpaintAnyLHarness
    from videopainter_amd.scheduler import CogVideoXDPMScheduler
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tr, br, _ = bench.build_models(dev, 1234, 0, 1)
    sch = CogVideoXDPMScheduler(snr_shift_scale=1.0, prediction_type="v_prediction", rescale_betas_zero_snr=True,
                                clip_sample=False, set_alpha_to_one=True, timestep_spacing="trailing")
    sch.set_timesteps(50)
    ts = sch.timesteps.cpu()
    h = CogVideoXI2VDualInpaintAnyLHarness(tr, br, sch)
    st, pe = bench.make_state(h, dev, 42)
    rope = h.rope_for(bench.F, bench.HL, bench.WL)
    gen = torch.Generator().manual_seed(42)

    def set_mode(on):
        tr.enable_cfg_streams(on)
        if args.branch and hasattr(br, "enable_cfg_streams"):
            br.enable_cfg_streams(on)

    def steps(n, k0):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n):
            h.step(st, (k0 + i) % len(ts), ts, pe, rope, guidance_scale=6.0, use_dynamic_cfg=True, replace_gt=True,
                   mask_add=True, generator=gen)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    res = {False: [], True: []}
    with torch.no_grad():
        for on in (False, True):  # warm both (allocator pools, cached bounds)
            set_mode(on)
            steps(1, 1)
        for r in range(args.rounds):
            for on in (False, True):
                set_mode(on)
                ms = steps(args.steps, 2 + r)
                res[on].append(ms)
                print(f"round {r} cfg_streams={on}: {ms:.1f} ms/step", flush=True)
        # numerics: one transformer forward in both modes on the same inputs
        lmi = torch.cat([torch.cat([st.latents] * 2), st.image_in], dim=2)
        t2 = torch.full((2,), 501, device=dev, dtype=torch.int64)
        outs = {}
        for on in (False, True):
            set_mode(on)
            bs = br(hidden_states=torch.cat([st.latents] * 2), encoder_hidden_states=pe, branch_cond=st.branch_in,
                    timestep=t2, image_rotary_emb=rope, return_dict=False)[0]
            outs[on] = tr(hidden_states=lmi, encoder_hidden_states=pe, branch_block_samples=bs, timestep=t2,
                          image_rotary_emb=rope, branch_block_masks=st.mask1, return_dict=False)[0].float()
        d = outs[True] - outs[False]
        print(f"numerics: max|diff| {d.abs().max().item():.3e}, rel-L2 {(d.norm() / outs[False].norm()).item():.3e}, "
              f"bit-identical {bool((d == 0).all())}")
    for on in (False, True):
        v = sorted(res[on])
        print(f"cfg_streams={on}: median {v[len(v) // 2]:.1f} ms/step, min {v[0]:.1f}")


if __name__ == "__main__":
    main()
