"""Host reference of the MX-FP8 format (include/vp_hip.h): e4m3 elements, one E8M0 scale per 32 K-elements,
scales in 256-row x 128-column tiles of 1 KiB.  Test infrastructure only (numpy + torch's float8_e4m3fn)."""
from __future__ import annotations

import numpy as np
import torch


def scale_offset(r, kb, K):
    r = np.asarray(r, dtype=np.int64)
    kb = np.asarray(kb, dtype=np.int64)
    return ((r >> 8) * (K >> 7) + (kb >> 2)) * 1024 + (kb & 3) * 256 + (r & 15) * 16 + ((r >> 4) & 15)


def scale_bytes(rows, K):
    return ((rows + 255) // 256) * (K // 128) * 1024


def block_exponent(amax: np.ndarray) -> np.ndarray:
    """s = ceil(log2(amax / 448)) with the kernel's float32 arithmetic; -127 for an all-zero block."""
    amax = amax.astype(np.float32)
    ratio = (amax * np.float32(1.0 / 448.0)).astype(np.float32)
    u = ratio.view(np.uint32)
    ex = ((u >> 23) & 0xFF).astype(np.int64)
    e = ex - 127 + ((u & 0x7FFFFF) != 0)
    e = np.where(ex == 0, -126, e)
    e = np.where(amax > 0, e, -127)
    return np.clip(e, -127, 127)


def pow2(e: np.ndarray) -> np.ndarray:
    return np.ldexp(np.float32(1.0), e.astype(np.int32)).astype(np.float32)


def quantize(x: torch.Tensor):
    """bf16/fp32 [rows, K] -> (q uint8 [rows, K], scales uint8 [scale_bytes])."""
    xf = x.float().cpu().numpy().astype(np.float32)
    rows, K = xf.shape
    blocks = xf.reshape(rows, K // 32, 32)
    e = block_exponent(np.abs(blocks).max(axis=2))
    scaled = (blocks * pow2(-e)[..., None]).astype(np.float32)
    scaled = np.clip(scaled, -448.0, 448.0).reshape(rows, K)
    q = torch.from_numpy(scaled).to(torch.float8_e4m3fn).view(torch.uint8)
    sc = np.zeros(scale_bytes(rows, K), dtype=np.uint8)
    rr, kk = np.meshgrid(np.arange(rows), np.arange(K // 32), indexing="ij")
    sc[scale_offset(rr, kk, K)] = (e + 127).astype(np.uint8)
    return q, torch.from_numpy(sc)


def dequantize(q: torch.Tensor, scales: torch.Tensor, rows: int, K: int) -> torch.Tensor:
    qf = q[:rows, :K].cpu().contiguous().view(torch.float8_e4m3fn).float().numpy()
    sc = scales.cpu().numpy()
    rr, kk = np.meshgrid(np.arange(rows), np.arange(K // 32), indexing="ij")
    e = sc[scale_offset(rr, kk, K)].astype(np.int64) - 127
    out = qf.reshape(rows, K // 32, 32) * pow2(e)[..., None]
    return torch.from_numpy(out.reshape(rows, K).astype(np.float32))
