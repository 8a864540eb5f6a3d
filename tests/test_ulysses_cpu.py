"""Ulysses head-parallel split (videopainter_amd/ulysses.py): shard geometry, the all-to-all layouts, and the RCCL
communicator's semantics against the thread-emulated one — on the CPU (gloo, world size 2)."""
import socket

import pytest
import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from videopainter_amd.ulysses import Shard, ThreadComm, DistComm, qkv_to_heads, heads_to_rows


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


@pytest.mark.parametrize("N,T,P", [(17776, 226, 8), (1378, 226, 4), (298, 10, 4), (600, 226, 2), (80, 30, 2)])
def test_shard_geometry(N, T, P):
    shards = [Shard(N, T, P, r) for r in range(P)]
    assert sum(s.valid for s in shards) == N and all(s.n * P == s.Npad >= N for s in shards)
    # text rows: a prefix of each shard, T of them in total
    assert sum(s.tl for s in shards) == T
    # the shards' video rows, in rank order, are the video indices 0 .. Npad - T - 1
    vid = []
    for s in shards:
        assert s.r0 + s.tl >= T or s.tl == s.n
        vid += list(range(s.v0, s.v0 + s.nv))
    assert vid == list(range(shards[0].Npad - T))


@pytest.mark.parametrize("N,T,P", [(300, 226, 8), (50, 30, 3)])
def test_shard_of_text_rows_only_raises(N, T, P):
    """T >= ceil(N / P): the first shard would hold no video row (empty proj_out / row-local launches)."""
    with pytest.raises(ValueError, match="only text rows"):
        Shard(N, T, P, 0)


def _global_qkv(B, Npad, H, P):
    D = H * 64
    r = torch.arange(Npad, dtype=torch.float32).view(1, Npad, 1)
    c = torch.arange(3 * D, dtype=torch.float32).view(1, 1, 3 * D)
    b = torch.arange(B, dtype=torch.float32).view(B, 1, 1)
    return b * 1e7 + r * 1e4 + c


@pytest.mark.parametrize("P", [2, 4])
def test_all_to_all_layouts_thread_comm(P):
    B, n, H = 2, 5, 4
    Npad, D, Dp = n * P, H * 64, H * 64 // P
    g = _global_qkv(B, Npad, H, P)
    comm = ThreadComm(P)

    def rank_fn(rank):
        full = qkv_to_heads(comm, rank, g[:, rank * n:(rank + 1) * n].contiguous())
        o_full = full[..., :Dp] * 1.0  # stand-in output of head group `rank` for every row: its q columns
        return full, heads_to_rows(comm, rank, o_full.contiguous())

    res = comm.run(rank_fn)
    for rank, (full, back) in enumerate(res):
        for part in range(3):  # q | k | v of head group `rank`, every row in global order
            want = g[..., part * D + rank * Dp: part * D + (rank + 1) * Dp]
            assert torch.equal(full[..., part * Dp:(part + 1) * Dp], want)
        # back to rows: this shard's rows, all heads (the q columns)
        assert torch.equal(back, g[:, rank * n:(rank + 1) * n, :D])


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    comm = DistComm()
    B, n, H = 2, 3, 4
    g = _global_qkv(B, n * world, H, world)
    full = qkv_to_heads(comm, rank, g[:, rank * n:(rank + 1) * n].contiguous())
    back = heads_to_rows(comm, rank, full[..., :H * 64 // world].contiguous())
    gat = comm.all_gather(rank, torch.full((2, 3), float(rank)))
    q.put(_portable((rank, full, back, gat)))
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_dist_comm_matches_thread_comm_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([_restore(q.get(timeout=240)) for _ in ps], key=lambda t: t[0])
    for p in ps:
        p.join(60)
    B, n, H = 2, 3, 4
    g = _global_qkv(B, n * world, H, world)
    comm = ThreadComm(world)
    want = comm.run(lambda r: (qkv_to_heads(comm, r, g[:, r * n:(r + 1) * n].contiguous())))
    for rank, full, back, gat in res:
        assert torch.equal(full, want[rank])
        assert torch.equal(back, g[:, rank * n:(rank + 1) * n, :H * 64])
        assert torch.equal(gat, torch.stack([torch.full((2, 3), 0.0), torch.full((2, 3), 1.0)]))


def test_transformer_view_applies_the_per_call_lora_scale(monkeypatch):
    """The head-parallel view re-folds attached LoRA adapters to the call's attention_kwargs["scale"] (default 1.0)
    before its forward, as the single-GPU forward does."""
    import types
    import torch
    from videopainter_amd import ulysses as U
    seen = []
    model = types.SimpleNamespace(config=types.SimpleNamespace(patch_size=2), proj_out=None,
                                  _call_lora_scale=lambda kw: seen.append(dict(kw) if kw else kw))
    monkeypatch.setattr(U, "transformer_forward", lambda *a, **k: (torch.zeros(1), []))
    view = U._TransformerView(model, types.SimpleNamespace(comm=None, rank=0))
    view(torch.zeros(1), torch.zeros(1, 3, 4), 0, attention_kwargs={"scale": 0.5}, return_dict=False)
    view(torch.zeros(1), torch.zeros(1, 3, 4), 0, return_dict=False)
    assert seen == [{"scale": 0.5}, None]
