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
