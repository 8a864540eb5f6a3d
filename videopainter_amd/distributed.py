"""Multi-GPU plumbing for the hot path (one process per GPU, torch.distributed; backend "nccl" = RCCL on ROCm).

What shards:
  * independent clips (configs 2/3 scaled to N GPUs): data-parallel replicas — weights broadcast once from rank 0,
    no per-step collective ("weak" scaling);
  * the any-length window chain (config 4) does NOT shard a single clip: window k needs window k-1's final latents
    and last-step hidden states (anyl.py:866-872, 962-988), so it stays serial on one rank.
Collectives here are issued in large flat buckets (few, big messages suit point-to-point xGMI rings).
"""
from __future__ import annotations

import os
from typing import Iterable, List

import torch
import torch.distributed as dist

BUCKET_BYTES = 512 << 20  # 512 MiB broadcast buckets


def env_rank_world():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), \
        int(os.environ.get("LOCAL_RANK", "0"))


def init(backend: str = "nccl", device=None):
    if dist.is_initialized():
        return
    kw = {}
    if backend == "nccl" and device is not None:
        kw["device_id"] = device
    dist.init_process_group(backend, **kw)


def _buckets(tensors: List[torch.Tensor], limit: int):
    cur, size = [], 0
    for t in tensors:
        nb = t.numel() * t.element_size()
        if cur and (size + nb > limit or t.dtype != cur[0].dtype or t.device != cur[0].device):
            yield cur
            cur, size = [], 0
        cur.append(t)
        size += nb
    if cur:
        yield cur


@torch.no_grad()
def broadcast_tensors(tensors: Iterable[torch.Tensor], src: int = 0, bucket_bytes: int = BUCKET_BYTES) -> None:
    """Broadcast tensors from `src` in flat buckets (one collective per <= bucket_bytes of same-dtype tensors)."""
    ts = [t for t in tensors if t.numel() > 0]
    for b in _buckets(ts, bucket_bytes):
        if len(b) == 1:
            dist.broadcast(b[0], src=src)
            continue
        flat = torch.cat([t.reshape(-1) for t in b])
        dist.broadcast(flat, src=src)
        off = 0
        for t in b:
            n = t.numel()
            t.copy_(flat[off:off + n].view_as(t))
            off += n


def broadcast_module(module: torch.nn.Module, src: int = 0, bucket_bytes: int = BUCKET_BYTES) -> None:
    """Replicate a model's parameters and buffers from rank `src` (config 3: weights over RCCL/xGMI)."""
    broadcast_tensors(list(module.state_dict().values()), src=src, bucket_bytes=bucket_bytes)


def max_over_ranks(value: float, device=None) -> float:
    """The bench's timing rule: the slowest rank's elapsed time."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier(device=None):
    if dist.is_initialized() and dist.get_world_size() > 1:
        if device is not None and dist.get_backend() == "nccl":
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()
