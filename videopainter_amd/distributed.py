"""Multi-GPU plumbing for the hot path (one process per GPU, torch.distributed; backend "nccl" = RCCL on ROCm).

What shards:
  * independent clips (configs 2/3 scaled to N GPUs): data-parallel replicas — weights broadcast once from rank 0,
    no per-step collective ("weak" scaling);
  * the two CFG halves of one clip (latency mode, `CFGPair`): each rank of a pair runs B=1; one all-gather of the
    fp32/bf16 noise prediction [1,13,16,60,90] per step; both ranks then run the identical CFG + DPM step;
  * the any-length window chain (config 4, `WindowStages`): window k needs window k-1's final latents and, with
    prev_clip_weight > 0, its last-step 42-layer hidden states (anyl.py:866-872, 962-988), so a single clip is a
    serial chain.  It is placed as a pipeline — window w on stage w % S, S = world / (2 if CFG-split else 1) — with a
    point-to-point hand-off (latents + hidden states + resample mask, ncclSend/Recv over xGMI) between consecutive
    stages, so several clips stream through the stages concurrently; at the end every rank all-gathers the
    windows' latents and averages the overlaps exactly as the serial loop does (anyl.py:1052-1069).
Collectives here are issued in large flat buckets (few, big messages suit point-to-point xGMI rings).
"""
from __future__ import annotations

import os
from typing import Callable, Dict, Iterable, List, Optional

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


class _staged:
    """The tensor a collective should run on: itself on RCCL, a host copy when the backend cannot take device
    tensors (gloo: the single-GPU rehearsal, VP_BENCH_DIST_BACKEND=gloo).  Copies back on exit, so the caller's
    code path (and the collective calls) are the same on every backend."""

    def __init__(self, t: torch.Tensor, group=None, writeback: bool = True):
        self.t = t
        self.host = t.is_cuda and dist.get_backend(group) != "nccl"
        self.writeback = writeback
        self.work = t.detach().cpu() if self.host else t

    def __enter__(self) -> torch.Tensor:
        return self.work

    def __exit__(self, *exc):
        if self.host and self.writeback and exc[0] is None:
            self.t.copy_(self.work)
        return False


def _all_gather_rows(out: torch.Tensor, inp: torch.Tensor, group=None) -> None:
    """all_gather_into_tensor on any backend (gloo takes host tensors only: staged)."""
    if not out.is_contiguous():
        raise ValueError("all-gather output must be contiguous")
    with _staged(out, group) as o, _staged(inp.contiguous(), group, writeback=False) as i:
        dist.all_gather_into_tensor(o.view(-1), i.view(-1), group=group)  # flat: one layout rule for every backend


def _send(t: torch.Tensor, dst: int) -> None:
    with _staged(t.contiguous(), writeback=False) as w:
        dist.send(w, dst)


def _recv(t: torch.Tensor, src: int) -> None:
    with _staged(t) as w:
        dist.recv(w, src)


@torch.no_grad()
def broadcast_tensors(tensors: Iterable[torch.Tensor], src: int = 0, bucket_bytes: int = BUCKET_BYTES,
                      method: str = "scatter_allgather", always: bool = False) -> None:
    """Replicate tensors from `src` in flat buckets (one exchange per <= bucket_bytes of same-dtype tensors).

    method "broadcast": one RCCL broadcast per bucket (a pipelined ring: every byte crosses every hop, so a bucket
    costs ~bytes / one link's bandwidth).  method "scatter_allgather" (default): the bucket is split into world
    shards; the source sends shard r straight to rank r (point-to-point, all of the source's xGMI links at once) and
    an all-gather then circulates the shards (each rank forwards (world-1)/world of the bucket) — on a fully
    connected 8-GPU node the source no longer serialises the whole payload through one link.  Both are exact copies.
    always: run the collectives at world size 1 too (they are identities there; the RCCL path on one GPU, tests/
    test_distributed_gpu.py and bench.py --rccl-world1)."""
    ts = [t for t in tensors if t.numel() > 0]
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    for b in _buckets(ts, bucket_bytes):
        if world == 1 and not always:
            continue
        if method == "broadcast" and len(b) == 1:
            with _staged(b[0]) as t:
                dist.broadcast(t, src=src)
            continue
        n = sum(t.numel() for t in b)
        per = (n + world - 1) // world
        flat = torch.empty(per * world, dtype=b[0].dtype, device=b[0].device)
        if rank == src:
            off = 0
            for t in b:
                flat[off:off + t.numel()].copy_(t.reshape(-1))
                off += t.numel()
        with _staged(flat) as work:
            if method == "broadcast":
                dist.broadcast(work, src=src)
            elif method == "scatter_allgather":
                # point-to-point scatter (RCCL has no native scatter): batched sends from the source, then one
                # all-gather of the shards.  The same calls run on every backend (gloo in the CPU tests).
                shard = torch.empty(per, dtype=work.dtype, device=work.device)
                ops = []
                if rank == src:
                    for r in range(world):
                        if r != src:
                            ops.append(dist.P2POp(dist.isend, work[r * per:(r + 1) * per], r))
                    shard.copy_(work[src * per:(src + 1) * per])
                else:
                    ops.append(dist.P2POp(dist.irecv, shard, src))
                for req in (dist.batch_isend_irecv(ops) if ops else []):
                    req.wait()
                dist.all_gather_into_tensor(work, shard)
            else:
                raise ValueError(f"unknown replication method {method!r}")
        if rank != src:
            off = 0
            for t in b:
                t.copy_(flat[off:off + t.numel()].view_as(t))
                off += t.numel()


def broadcast_module(module: torch.nn.Module, src: int = 0, bucket_bytes: int = BUCKET_BYTES,
                     method: str = "scatter_allgather", always: bool = False) -> None:
    """Replicate a model's parameters and buffers from rank `src` (config 3: weights over RCCL/xGMI)."""
    broadcast_tensors(list(module.state_dict().values()), src=src, bucket_bytes=bucket_bytes, method=method,
                      always=always)


@torch.no_grad()
def bucket_digests(tensors: Iterable[torch.Tensor], bucket_bytes: int = BUCKET_BYTES) -> torch.Tensor:
    """Per replication bucket (the buckets broadcast_tensors sends): the sum of the raw bit patterns and their sum
    weighted by (position mod 997) + 1, in int64 on the tensors' device — one row [sum, weighted] per bucket.  Two
    ranks agree on a row only if the bucket's bytes agree (up to a collision of both sums)."""
    rows = []
    for b in _buckets([t for t in tensors if t.numel() > 0], bucket_bytes):
        s0 = torch.zeros((), dtype=torch.int64, device=b[0].device)
        s1 = torch.zeros((), dtype=torch.int64, device=b[0].device)
        off = 0
        for t in b:
            flat = t.detach().reshape(-1)
            isz = flat.element_size()
            bits = flat.view({1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}[isz]).to(torch.int64)
            if isz == 2:
                bits = bits & 0xFFFF
            elif isz == 4:
                bits = bits & 0xFFFFFFFF
            w = (torch.arange(off, off + flat.numel(), device=flat.device, dtype=torch.int64) % 997) + 1
            s0 += bits.sum()
            s1 += (bits * w).sum()
            off += flat.numel()
        rows.append(torch.stack([s0, s1]))
    return torch.stack(rows) if rows else torch.zeros(0, 2, dtype=torch.int64)


@torch.no_grad()
def verify_replicas(module: torch.nn.Module, bucket_bytes: int = BUCKET_BYTES, group=None, always: bool = False):
    """After broadcast_module: does every rank hold rank 0's bytes?  Each rank digests its buckets
    (bucket_digests, on the device), one all-reduce of MIN and one of MAX compare them across ranks (the same calls
    on RCCL and gloo).  Returns (identical on every rank, number of buckets); collective: every rank must call it.
    always: all-reduce at world size 1 too (as broadcast_tensors)."""
    d = bucket_digests(list(module.state_dict().values()), bucket_bytes)
    if not dist.is_initialized() or (dist.get_world_size(group) == 1 and not always):
        return True, int(d.shape[0])
    lo, hi = d.clone(), d.clone()
    with _staged(lo, group) as a:
        dist.all_reduce(a, op=dist.ReduceOp.MIN, group=group)
    with _staged(hi, group) as a:
        dist.all_reduce(a, op=dist.ReduceOp.MAX, group=group)
    return bool(torch.equal(lo, hi)), int(d.shape[0])


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


# ----------------------------------------------------------------------------------------------------------------
# CFG split: one clip on a pair of ranks
# ----------------------------------------------------------------------------------------------------------------

def _pair_groups(world: int, size: int):
    """Every rank must create every group (torch.distributed.new_group contract)."""
    groups = []
    for p in range(world // size):
        groups.append(dist.new_group(list(range(p * size, (p + 1) * size))))
    return groups


class CFGPair:
    """Ranks (2p, 2p+1) share one clip: cfg_index 0 runs the unconditional half of the CFG batch, 1 the text half
    (the order of `torch.cat([negative_prompt_embeds, prompt_embeds])`, anyl.py:805-806).  An explicit `group` may
    have any size (a one-rank group: the all-gather on one GPU, tests/test_distributed_gpu.py)."""

    def __init__(self, group=None, cfg_index: Optional[int] = None):
        rank, world = dist.get_rank(), dist.get_world_size()
        if group is None:
            if world % 2:
                raise ValueError(f"CFG split needs an even world size, got {world}")
            group = _pair_groups(world, 2)[rank // 2]
        self.group = group
        self.cfg_index = rank % 2 if cfg_index is None else cfg_index
        self.backend = dist.get_backend(group)

    def allgather(self, half: torch.Tensor) -> torch.Tensor:
        """[1, ...] on each rank of the pair -> [2, ...] = (uncond, text) on both ([group size, ...] in general)."""
        if half.shape[0] != 1:
            raise ValueError("each CFG rank holds a batch of 1")
        half = half.contiguous()
        out = torch.empty((dist.get_world_size(self.group),) + tuple(half.shape[1:]), dtype=half.dtype,
                          device=half.device)
        _all_gather_rows(out, half, self.group)
        return out


# ----------------------------------------------------------------------------------------------------------------
# any-length window chain as a pipeline over stages
# ----------------------------------------------------------------------------------------------------------------

class WindowStages:
    """Stage placement of the window chain: S = world / cfg stages; rank = stage * cfg + cfg_index."""

    def __init__(self, cfg_split: bool = False):
        self.rank, self.world = dist.get_rank(), dist.get_world_size()
        self.cfg = 2 if cfg_split else 1
        if self.world % self.cfg:
            raise ValueError(f"world size {self.world} is not a multiple of the CFG group size {self.cfg}")
        self.stages = self.world // self.cfg
        self.stage = self.rank // self.cfg
        self.cfg_index = self.rank % self.cfg
        self.pair = CFGPair() if cfg_split else None

    def stage_of(self, window: int) -> int:
        return window % self.stages

    def peer(self, stage: int) -> int:
        """The rank of `stage` that holds this rank's CFG half."""
        return stage * self.cfg + self.cfg_index

    # hand-off payload: latents [1,F,C,h,w]; last-step hidden states {layer: [b,N,D]}; resample mask [b,N] bool;
    # the CPU generator's state (the reference draws every window's scheduler noise from ONE generator, so the
    # next window continues the stream exactly where this one stopped)
    def send_handoff(self, dst_stage: int, latents: torch.Tensor, states: Optional[dict],
                     mask: Optional[torch.Tensor], generator: Optional[torch.Generator] = None) -> None:
        dst = self.peer(dst_stage)
        dev = latents.device
        _send(latents.contiguous(), dst)
        gs = generator.get_state() if generator is not None else None
        flags = torch.tensor([0 if states is None else len(states), 0 if mask is None else 1,
                              0 if gs is None else gs.numel()], dtype=torch.int64, device=dev)
        _send(flags, dst)
        if states is not None:
            for k in sorted(states):
                _send(states[k].contiguous(), dst)
        if mask is not None:
            _send(mask.to(torch.uint8).contiguous(), dst)
        if gs is not None:
            _send(gs.to(dev), dst)

    def recv_handoff(self, src_stage: int, lat_like: torch.Tensor, state_shape, mask_shape,
                     generator: Optional[torch.Generator] = None):
        src = self.peer(src_stage)
        dev = lat_like.device
        lat = torch.empty_like(lat_like)
        _recv(lat, src)
        flags = torch.empty(3, dtype=torch.int64, device=dev)
        _recv(flags, src)
        n_states, has_mask, gs_n = (int(x) for x in flags.tolist())
        states = None
        if n_states:
            states = {}
            for k in range(n_states):
                t = torch.empty(state_shape, dtype=lat_like.dtype, device=dev)
                _recv(t, src)
                states[k] = t
        mask = None
        if has_mask:
            m = torch.empty(mask_shape, dtype=torch.uint8, device=dev)
            _recv(m, src)
            mask = m.bool()
        if gs_n:
            g = torch.empty(gs_n, dtype=torch.uint8, device=dev)
            _recv(g, src)
            if generator is None:
                raise ValueError("the previous stage handed off a generator state but this rank has no generator")
            generator.set_state(g.cpu())
        return lat, states, mask

    def gather_windows(self, local: Dict[int, torch.Tensor], n_windows: int, like: torch.Tensor) -> List[torch.Tensor]:
        """All-gather every window's final latents (each stage holds the windows placed on it)."""
        if self.world == 1:
            return [local[w] for w in range(n_windows)]
        per = (n_windows + self.stages - 1) // self.stages
        buf = torch.zeros((per,) + tuple(like.shape), dtype=like.dtype, device=like.device)
        for w, t in local.items():
            buf[w // self.stages] = t
        allb = torch.empty((self.world,) + tuple(buf.shape), dtype=buf.dtype, device=buf.device)
        _all_gather_rows(allb, buf)
        return [allb[self.peer(self.stage_of(w))][w // self.stages] for w in range(n_windows)]


def run_window_chain(stages: WindowStages, clips: List[dict], run_window: Callable, image_latents_for: Callable,
                     assemble: Callable, lat_like: torch.Tensor, state_shape, mask_shape) -> List[torch.Tensor]:
    """Pipeline-parallel any-length loop over several clips.

    clips[j] = {"windows": [...], "generator": torch.Generator or None};
    run_window(j, w, win, image_latents, prev_states, prev_mask, capture) -> (latents, states, mask);
    image_latents_for(w, win, prev_latents) -> conditioning latents; assemble(list of window latents) -> video.
    lat_like: a device tensor shaped/typed like one window's latents.  Each stage walks the clips in order and,
    within a clip, its own windows in order, so every receive waits only on an earlier window of the same clip (no
    cycle, hence no deadlock, for any window count).  Returns the assembled video of every clip on every rank."""
    videos = []
    for j, clip in enumerate(clips):
        wins = clip["windows"]
        gen = clip.get("generator")
        n = len(wins)
        local = {}
        carry = (None, None, None)  # hand-off between two windows placed on the same stage stays in place
        for w in range(n):
            if stages.stage_of(w) != stages.stage:
                continue
            prev_lat, prev_states, prev_mask = None, None, None
            if w > 0:
                if stages.stage_of(w - 1) == stages.stage:
                    prev_lat, prev_states, prev_mask = carry
                else:
                    prev_lat, prev_states, prev_mask = stages.recv_handoff(stages.stage_of(w - 1), lat_like,
                                                                           state_shape, mask_shape, gen)
            img = image_latents_for(w, wins[w], prev_lat)
            lat, states, mask = run_window(j, w, wins[w], img, prev_states, prev_mask, w < n - 1)
            if w < n - 1:
                if stages.stage_of(w + 1) == stages.stage:
                    carry = (lat, states, mask)
                else:
                    stages.send_handoff(stages.stage_of(w + 1), lat, states, mask, gen)
            local[w] = lat
        videos.append(assemble(stages.gather_windows(local, n, lat_like)))
    return videos


# ----------------------------------------------------------------------------------------------------------------
# concurrent windows: the north-star's literal "segments sharded across GPUs + all-gather of the overlap latents".
# NOT the reference's semantics: the reference chains windows (window k conditions on window k-1's
# final latents and, with prev_clip_weight > 0, its last-step hidden states, anyl.py:862-872, 962-988).  Here every
# window conditions on its own first frame and no previous-window states, so all windows run at once; only the
# overlap averaging of the assembled clip couples them.  Opt-in, labelled, and never used by the parity tests.
# ----------------------------------------------------------------------------------------------------------------

def allgather_windows(local: Dict[int, torch.Tensor], n_windows: int, like: torch.Tensor) -> List[torch.Tensor]:
    """Window w lives on rank w % world; returns every window's latents on every rank (one all-gather over xGMI)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return [local[w] for w in range(n_windows)]
    world, rank = dist.get_world_size(), dist.get_rank()
    per = (n_windows + world - 1) // world
    buf = torch.zeros((per,) + tuple(like.shape), dtype=like.dtype, device=like.device)
    for w, t in local.items():
        if w % world != rank:
            raise ValueError(f"window {w} is not placed on rank {rank}")
        buf[w // world] = t
    allb = torch.empty((world,) + tuple(buf.shape), dtype=buf.dtype, device=buf.device)
    _all_gather_rows(allb, buf)
    return [allb[w % world][w // world] for w in range(n_windows)]


def run_windows_concurrent(windows: List[dict], run_window: Callable, assemble: Callable,
                           lat_like: torch.Tensor) -> torch.Tensor:
    """NON-PARITY any-length mode: rank r runs windows r, r + world, ... independently (each window's own
    `image_latents`, no previous-window hand-off), then one all-gather of the window latents and the reference's
    overlap averaging.  run_window(w, win) -> latents.  Returns the assembled clip on every rank."""
    rank = dist.get_rank() if dist.is_initialized() else 0
    world = dist.get_world_size() if dist.is_initialized() else 1
    local = {w: run_window(w, windows[w]) for w in range(rank, len(windows), world)}
    return assemble(allgather_windows(local, len(windows), lat_like))
