"""World-size-2 gloo tests of the multi-GPU plumbing (CPU): weight broadcast from rank 0 in flat buckets and the
bench's max-over-ranks timing rule."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from videopainter_amd.distributed import init, broadcast_module, max_over_ranks
    from videopainter_amd import CogVideoXTransformer3DModel
    from tests.golden.cases import TINY_CFG
    init("gloo")
    torch.manual_seed(100 + rank)
    m = CogVideoXTransformer3DModel(**TINY_CFG)
    with torch.no_grad():
        for p in m.state_dict().values():
            p.copy_(torch.randn(p.shape) * (rank + 1))
    broadcast_module(m, src=0, bucket_bytes=1 << 16)  # small buckets: exercises the multi-tensor flatten path
    digest = float(sum(p.double().sum() for p in m.state_dict().values()))
    t = max_over_ranks(1.0 + rank)
    q.put((rank, digest, t))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_broadcast_and_max_over_ranks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in ps]
    for p in ps:
        p.join(60)
    res.sort()
    assert res[0][1] == res[1][1], "ranks disagree after broadcast"
    assert res[0][2] == res[1][2] == 2.0


# ------------------------------------------------------------------------------------------------------------------
# any-length window chain on a stage pipeline + CFG split, exercised with a toy window function that
# has the real data dependencies: each step needs both CFG halves (all-gathered across a pair), window w needs
# window w-1's final latents (conditioning), last-step states and mask, and the scheduler noise continues ONE
# generator stream across windows.
# ------------------------------------------------------------------------------------------------------------------

SHAPE = (1, 3, 2, 4, 4)   # [1, F, C, h, w]
NTOK, DD = 5, 6


def _toy_clips(n_clips, n_windows):
    clips = []
    for j in range(n_clips):
        g = torch.Generator().manual_seed(1000 + j)
        wins = []
        for w in range(n_windows):
            gg = torch.Generator().manual_seed(77 * j + w)
            wins.append({"latents": torch.randn(SHAPE, generator=gg),
                         "image_latents": torch.randn(SHAPE, generator=gg) if w == 0 else None})
        clips.append({"windows": wins, "generator": g})
    return clips


def _toy_window(pair, clips):
    def run_window(j, w, win, img, prev_states, prev_mask, capture):
        g = clips[j]["generator"]
        halves = [0, 1] if pair is None else [pair.cfg_index]
        x = win["latents"].clone()
        for step in range(3):
            preds = []
            for c in halves:
                r = 0 if pair is not None else c
                extra = 0.0
                if prev_states is not None:
                    extra = float(prev_states[0][r].mean()) + 0.5 * float(prev_mask[r].float().mean())
                preds.append(torch.tanh(x * (1.0 + 0.1 * c) + img.mean() + extra + step))
            pred = torch.cat(preds) if pair is None else pair.allgather(preds[0])
            x = x + 0.1 * (pred[0:1] + 6.0 * (pred[1:2] - pred[0:1])) + 0.01 * torch.randn(SHAPE, generator=g)
        rows = len(halves)
        states = None
        if capture:
            states = {k: torch.full((rows, NTOK, DD), float(x.mean()) * (k + 1)) + torch.tensor(halves).view(-1, 1, 1)
                      for k in range(2)}
        mask = (torch.arange(NTOK)[None, :].repeat(rows, 1) + int(x.sum() > 0)) % 2 == 0
        return x, states, mask
    return run_window


def _image_for(w, win, prev):
    if w == 0:
        return win["image_latents"]
    img = torch.zeros(SHAPE)
    img[:, 0] = prev[:, -1]
    return img


def _assemble(lats):
    return torch.cat([lats[0]] + [t[:, 1:] for t in lats[1:]], dim=1)  # stride == num_frames style overlap


def _serial(n_clips, n_windows):
    clips = _toy_clips(n_clips, n_windows)
    rw = _toy_window(None, clips)
    out = []
    for j, clip in enumerate(clips):
        lat, st, m = None, None, None
        lats = []
        for w, win in enumerate(clip["windows"]):
            lat, st, m = rw(j, w, win, _image_for(w, win, lat), st, m, w < n_windows - 1)
            lats.append(lat)
        out.append(_assemble(lats))
    return out


def _chain_worker(rank, world, port, cfg_split, n_clips, n_windows, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from videopainter_amd.distributed import init, WindowStages, run_window_chain
    init("gloo")
    stages = WindowStages(cfg_split=cfg_split)
    clips = _toy_clips(n_clips, n_windows)
    rows = 1 if cfg_split else 2
    vids = run_window_chain(stages, clips, _toy_window(stages.pair, clips), _image_for, _assemble,
                            torch.empty(SHAPE), (rows, NTOK, DD), (rows, NTOK))
    q.put((rank, [v.clone() for v in vids]))
    dist.destroy_process_group()


def _run(world, cfg_split, n_clips, n_windows):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_chain_worker, args=(r, world, port, cfg_split, n_clips, n_windows, q))
          for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in ps]
    for p in ps:
        p.join(60)
    return res


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,cfg_split,n_windows", [(2, False, 4), (2, True, 3), (4, True, 3)],
                         ids=["2stages", "cfg_pair", "2stages_x_cfg_wraparound"])
def test_window_chain_pipeline_matches_serial_gloo(world, cfg_split, n_windows):
    ref = _serial(2, n_windows)
    for rank, vids in _run(world, cfg_split, 2, n_windows):
        assert len(vids) == 2
        for v, r in zip(vids, ref):
            assert torch.equal(v, r), f"rank {rank}: pipelined window chain differs from the serial loop"


def _concurrent_worker(rank, world, port, n_windows, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from videopainter_amd.distributed import init, run_windows_concurrent
    init("gloo")
    wins = [dict(x=torch.full(SHAPE, float(w + 1))) for w in range(n_windows)]
    ran = []

    def rw(w, win):
        ran.append(w)
        return win["x"] * 2 + w

    out = run_windows_concurrent(wins, rw, _assemble, torch.empty(SHAPE))
    q.put((rank, out.clone(), ran))
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_concurrent_windows_allgather_gloo():
    """The labelled non-parity mode: windows round-robin over the ranks, one all-gather, every rank assembles the
    same clip as a single process running all windows."""
    n_windows, world = 5, 2
    ref = _assemble([torch.full(SHAPE, float(w + 1)) * 2 + w for w in range(n_windows)])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_concurrent_worker, args=(r, world, port, n_windows, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=100) for _ in ps]
    for p in ps:
        p.join(60)
    for rank, out, ran in res:
        assert ran == list(range(rank, n_windows, world))
        assert torch.equal(out, ref)
