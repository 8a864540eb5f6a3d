"""The RCCL code path on one GPU: torch.distributed over backend "nccl" (= RCCL on ROCm) at world size 1, device
tensors, no host staging.  At world size 1 the collectives are identities, so the checks are exact: the weight
replication (broadcast_module, both methods), the replica check (verify_replicas' MIN/MAX all-reduce), the CFG
all-gather (CFGPair.allgather), the bench's max-over-ranks timing rule and the barrier all run through RCCL and
leave every byte as it was.  The multi-rank behaviour of the same functions is covered on gloo
(tests/test_distributed_cpu.py); a multi-GPU node is the driver's."""
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture
def rccl_world1(monkeypatch):
    import torch.distributed as dist
    from videopainter_amd import distributed as VD
    for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", str(_free_port())), ("RANK", "0"),
                 ("WORLD_SIZE", "1"), ("LOCAL_RANK", "0")):
        monkeypatch.setenv(k, v)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    VD.init("nccl", dev)  # the bench's init, with device_id (distributed.py init)
    try:
        assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
        yield dev
    finally:
        dist.destroy_process_group()


def _model(dev):
    from videopainter_amd import CogVideoXTransformer3DModel, device_scope
    from tests.golden.cases import TINY_CFG
    with device_scope(dev):
        m = CogVideoXTransformer3DModel(**TINY_CFG)
    m.init_synthetic_weights_(5)
    return m


def test_weight_replication_and_replica_check_on_rccl(rccl_world1):
    from videopainter_amd import distributed as VD
    dev = rccl_world1
    m = _model(dev)
    sd = m.state_dict()
    assert all(t.is_cuda for t in sd.values())
    before = {k: t.clone() for k, t in sd.items()}
    for t in sd.values():  # device tensors go to RCCL as they are (no host hop)
        assert VD._staged(t).host is False
    small = 1 << 16  # many buckets: every dtype boundary and the bucket split run
    for method in ("scatter_allgather", "broadcast"):
        VD.broadcast_module(m, src=0, bucket_bytes=small, method=method, always=True)
        torch.cuda.synchronize()
        for k, t in m.state_dict().items():
            assert torch.equal(t, before[k]), f"{method} changed {k}"
        ok, n = VD.verify_replicas(m, bucket_bytes=small, always=True)
        assert ok and n == VD.bucket_digests(list(sd.values()), small).shape[0] and n > 4
    # the replica check would see a difference in any bucket: the digests are position-weighted byte sums
    d0 = VD.bucket_digests(list(sd.values()), small)
    p = next(iter(m.parameters()))
    with torch.no_grad():
        p.view(-1)[3] += 1.0
    assert not torch.equal(d0, VD.bucket_digests(list(m.state_dict().values()), small))


def test_cfg_allgather_max_over_ranks_and_barrier_on_rccl(rccl_world1):
    import torch.distributed as dist
    from videopainter_amd import distributed as VD
    dev = rccl_world1
    pair = VD.CFGPair(group=dist.group.WORLD, cfg_index=0)
    assert pair.backend == "nccl"
    g = torch.Generator(device=dev).manual_seed(3)
    for dt in (torch.float32, torch.bfloat16):
        half = torch.randn(1, 13, 16, 60, 90, device=dev, generator=g).to(dt)  # one CFG half's noise prediction
        got = pair.allgather(half)
        assert got.shape == half.shape and got.dtype == dt and torch.equal(got, half)
    assert VD.max_over_ranks(1.25, dev) == 1.25
    VD.barrier(dev)
    t = torch.tensor([2.5], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)  # the timing rule's collective itself (max_over_ranks skips it at N=1)
    assert float(t.item()) == 2.5
    # the window-stage placement at one stage: every window on this rank, no hand-off
    st = VD.WindowStages()
    assert st.stages == 1 and st.stage_of(5) == 0 and st.peer(0) == 0
    like = torch.zeros(1, 13, 16, 60, 90, device=dev)
    local = {w: torch.full_like(like, float(w)) for w in range(3)}
    assert [float(t[0, 0, 0, 0, 0]) for t in st.gather_windows(local, 3, like)] == [0.0, 1.0, 2.0]
    allg = VD.allgather_windows(local, 3, like)
    assert all(torch.equal(a, local[w]) for w, a in enumerate(allg))
