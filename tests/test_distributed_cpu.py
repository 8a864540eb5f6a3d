"""World-size-2 gloo tests of the multi-GPU plumbing (CPU): weight broadcast from rank 0 in flat buckets and the
bench's max-over-ranks timing rule."""
import os
import socket

import pytest
import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp



def _portable(x):
    """Tensors crossing the result queue as numpy copies: a queued torch tensor is shared by file descriptor through
    the sending process, which may already have exited when the parent reads it (FileNotFoundError under load)."""
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy().copy()
    if isinstance(x, (list, tuple)):
        return type(x)(_portable(v) for v in x)
    return x


def _restore(x):
    if isinstance(x, np.ndarray):
        return torch.from_numpy(x)
    if isinstance(x, (list, tuple)):
        return type(x)(_restore(v) for v in x)
    return x

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, method="scatter_allgather"):
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
    if rank == 0:
        want = [p.clone() for p in m.state_dict().values()]
    broadcast_module(m, src=0, bucket_bytes=1 << 16, method=method)  # small buckets: the multi-tensor path
    digest = float(sum(p.double().sum() for p in m.state_dict().values()))
    if rank == 0:
        assert all(torch.equal(a, b) for a, b in zip(want, m.state_dict().values()))
    t = max_over_ranks(1.0 + rank)
    q.put(_portable((rank, digest, t)))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,method", [(2, "scatter_allgather"), (3, "scatter_allgather"), (4, "scatter_allgather"),
                                          (2, "broadcast")])
def test_broadcast_and_max_over_ranks_gloo(world, method):
    """Weight replication (both methods; world 3 exercises the padded shards) is an exact copy of rank 0's
    weights on every rank, and the bench's timing rule takes the max over ranks."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, method)) for r in range(world)]
    for p in ps:
        p.start()
    res = [_restore(q.get(timeout=240)) for _ in ps]
    for p in ps:
        p.join(60)
    res.sort()
    assert all(r[1] == res[0][1] for r in res), "ranks disagree after replication"
    assert all(r[2] == float(world) for r in res)


def _digest_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from videopainter_amd.distributed import init, broadcast_module, verify_replicas
    from videopainter_amd import CogVideoXTransformer3DModel
    from tests.golden.cases import TINY_CFG
    init("gloo")
    torch.manual_seed(200 + rank)
    m = CogVideoXTransformer3DModel(**TINY_CFG)
    with torch.no_grad():
        for p in m.state_dict().values():
            p.copy_(torch.randn(p.shape))
    before = verify_replicas(m, bucket_bytes=1 << 16)
    broadcast_module(m, src=0, bucket_bytes=1 << 16)
    after = verify_replicas(m, bucket_bytes=1 << 16)
    with torch.no_grad():  # one flipped bit of one weight on the last rank
        if rank == world - 1:
            w = m.transformer_blocks[1].attn1.to_k.weight
            w.view(torch.int16)[3, 5] ^= 1
    corrupted = verify_replicas(m, bucket_bytes=1 << 16)
    q.put(_portable((rank, before, after, corrupted)))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_replica_digests_detect_divergence_gloo():
    """bench.py's self-check of the weight replication (distributed.verify_replicas, per-bucket digests compared by
    a MIN and a MAX all-reduce): different weights before the broadcast are caught, identical weights after it
    pass, and a single flipped bit on one rank afterwards is caught on every rank."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_digest_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(_restore(q.get(timeout=240)) for _ in ps)
    for p in ps:
        p.join(60)
    for _, before, after, corrupted in res:
        assert before[0] is False and after[0] is True and corrupted[0] is False
        assert after[1] > 1  # several buckets (the multi-bucket path)


def _bench_worker(rank, world, port, mode, q):
    """bench.py's rank logic (clip assignment, warm-up + barrier-bracketed timed steps, max over ranks, whole-job
    value) with the toy window step instead of the HIP model (GPU-free)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import bench
    from videopainter_amd.distributed import init, barrier, max_over_ranks, CFGPair
    init("gloo")
    pair = CFGPair() if mode == "cfgpair" else None
    clip = bench.clip_of(rank, mode)
    clips = _toy_clips(max(1, world), 1)
    g = torch.Generator().manual_seed(5 + clip)
    x = clips[clip]["windows"][0]["latents"].clone()
    halves = [0, 1] if pair is None else [pair.cfg_index]
    state = {"x": x}

    def one(i):
        preds = torch.cat([torch.tanh(state["x"] * (1.0 + 0.1 * c) + i) for c in halves])
        if pair is not None:
            preds = pair.allgather(preds)
        state["x"] = state["x"] + 0.1 * (preds[0:1] + 6.0 * (preds[1:2] - preds[0:1])) + 0.01 * torch.randn(
            SHAPE, generator=g)

    elapsed = bench.timed_steps(one, lambda: barrier(), warmup=2, steps=3)
    emax = max_over_ranks(elapsed)
    n_clips, value = bench.job_value(emax, 3, world, mode)
    q.put(_portable((rank, clip, state["x"].clone(), elapsed, emax, n_clips, value)))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("mode", ["dp", "cfgpair"])
def test_bench_rank_logic_gloo(mode):
    """World size 2: dp gives each rank its own clip (2 clips), cfgpair puts both CFG halves of ONE clip on the pair
    (latents bit-identical on both ranks, equal to the single-process B=2 run); value = clips x steps / max time."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_bench_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([_restore(q.get(timeout=240)) for _ in ps], key=lambda r: r[0])
    for p in ps:
        p.join(60)
    emax = max(r[3] for r in res)
    for rank, clip, x, el, em, n_clips, value in res:
        assert em == emax
        assert n_clips == (1 if mode == "cfgpair" else 2)
        assert abs(value - n_clips * 3 / emax) < 1e-12
    if mode == "cfgpair":
        assert res[0][1] == res[1][1] == 0 and torch.equal(res[0][2], res[1][2])
        # the same clip stepped by one process at B=2
        g = torch.Generator().manual_seed(5)
        x = _toy_clips(world, 1)[0]["windows"][0]["latents"].clone()
        for i in range(5):
            preds = torch.cat([torch.tanh(x * (1.0 + 0.1 * c) + i) for c in (0, 1)])
            x = x + 0.1 * (preds[0:1] + 6.0 * (preds[1:2] - preds[0:1])) + 0.01 * torch.randn(SHAPE, generator=g)
        assert torch.equal(res[0][2], x)
    else:
        assert [r[1] for r in res] == [0, 1]


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
    q.put(_portable((rank, [v.clone() for v in vids])))
    dist.destroy_process_group()


def _run(world, cfg_split, n_clips, n_windows):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_chain_worker, args=(r, world, port, cfg_split, n_clips, n_windows, q))
          for r in range(world)]
    for p in ps:
        p.start()
    res = [_restore(q.get(timeout=240)) for _ in ps]
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
    q.put(_portable((rank, out.clone(), ran)))
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
    res = [_restore(q.get(timeout=100)) for _ in ps]
    for p in ps:
        p.join(60)
    for rank, out, ran in res:
        assert ran == list(range(rank, n_windows, world))
        assert torch.equal(out, ref)
