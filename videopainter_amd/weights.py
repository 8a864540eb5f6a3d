"""Deterministic synthetic weights/inputs and diffusers-format checkpoint I/O.

There are no real CogVideoX-5b-I2V / VideoPainter checkpoints offline, so every parity fixture and
every benchmark runs on random-init weights of the reference architecture.  Parity fixtures need weights that are
reproducible on any host without torch's RNG, so they come from a counter-based generator: splitmix64 over
(hash(name), element index) -> two uniforms -> Box-Muller normal.  The same bits come out of numpy here, on the GPU
box, and in the golden-vector generator (`tests/golden/make_golden.py`).

Checkpoint format is the reference's: `config.json` + `diffusion_pytorch_model.safetensors` with the state-dict keys
of `CogVideoXTransformer3DModel` / `CogvideoXBranchModel` (reference
`diffusers/src/diffusers/models/modeling_utils.py:266,412`).
"""
from __future__ import annotations

import json
import math
import os
from typing import Dict, Iterable, Optional, Tuple

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _fnv1a64(text: str) -> int:
    h = 0xCBF29CE484222325
    for ch in text.encode("utf-8"):
        h ^= ch
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def counter_seed(key: str, seed: int = 0) -> int:
    """64-bit stream base for (key, seed); the device generator (`vp_fill_normal_bf16`) uses the same base."""
    return (_fnv1a64(key) ^ ((seed * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF)) & 0xFFFFFFFFFFFFFFFF


def counter_normal(key: str, n: int, seed: int = 0) -> np.ndarray:
    """n standard normals (float32), a pure function of (key, seed, index)."""
    base = np.uint64(counter_seed(key, seed))
    out = np.empty(n, dtype=np.float32)
    chunk = 1 << 22
    for s in range(0, n, chunk):
        idx = np.arange(s, min(n, s + chunk), dtype=np.uint64)
        with np.errstate(over="ignore"):
            r1 = _splitmix64(base + np.uint64(2) * idx)
            r2 = _splitmix64(base + np.uint64(2) * idx + np.uint64(1))
        u1 = ((r1 >> np.uint64(11)).astype(np.float64) + 1.0) * (1.0 / 9007199254740992.0)
        u2 = (r2 >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
        out[s:s + len(idx)] = (np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * math.pi * u2)).astype(np.float32)
    return out


def counter_uniform(key: str, n: int, seed: int = 0) -> np.ndarray:
    base = np.uint64((_fnv1a64(key) ^ ((seed * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF)) & 0xFFFFFFFFFFFFFFFF)
    idx = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        r = _splitmix64(base + idx)
    return ((r >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)).astype(np.float32)


def round_bf16(a: np.ndarray) -> np.ndarray:
    """Round float32 -> bfloat16 (round-to-nearest-even) and back, in numpy."""
    a = np.ascontiguousarray(a, dtype=np.float32)
    u = a.view(np.uint32).astype(np.uint64)
    r = ((u + np.uint64(0x7FFF) + ((u >> np.uint64(16)) & np.uint64(1))) >> np.uint64(16)) << np.uint64(16)
    return r.astype(np.uint32).view(np.float32).reshape(a.shape)


def param_std(name: str, shape: Tuple[int, ...]) -> Tuple[float, float]:
    """(mean, std) used for a synthetic parameter, by its diffusers state-dict name.

    Linear / conv weights: N(0, 1/fan_in).  AdaLN linears (norm*.linear) are scaled by 0.5 so 42-layer residual
    streams stay O(1..10).  LayerNorm gammas ~ 1 + N(0, 0.05^2), betas / biases ~ N(0, 0.02^2).  The branch's
    zero-initialised linears (`branch_blocks.*`, `branch_x_embedder`, reference `branch_cogvideox.py:143-147`) are
    randomised like any linear so the injection path is exercised.
    """
    leaf = name.rsplit(".", 1)[-1]
    if name.endswith("pos_embedding"):
        return 0.0, 0.5
    is_norm = ".norm" in name or name.startswith("norm") or "norm_q" in name or "norm_k" in name
    if len(shape) == 1:
        if is_norm and leaf == "weight":
            return 1.0, 0.05
        return 0.0, 0.02
    fan_in = int(np.prod(shape[1:]))
    std = 1.0 / math.sqrt(fan_in)
    if is_norm:
        std *= 0.5
    return 0.0, std


def synth_param(name: str, shape: Tuple[int, ...], seed: int = 0, bf16: bool = True) -> np.ndarray:
    mean, std = param_std(name, shape)
    n = int(np.prod(shape))
    a = (counter_normal(name, n, seed) * np.float32(std) + np.float32(mean)).reshape(shape)
    if name.endswith("pos_embedding"):
        # joint embedding: text rows are zero in the reference (embeddings.py:384-389)
        pass
    return round_bf16(a) if bf16 else a


def synth_state_dict(shapes: Dict[str, Tuple[int, ...]], seed: int = 0, bf16: bool = True) -> Dict[str, np.ndarray]:
    return {k: synth_param(k, tuple(s), seed, bf16) for k, s in shapes.items()}


def synth_tensor(key: str, shape: Tuple[int, ...], seed: int = 0, std: float = 1.0, bf16: bool = True) -> np.ndarray:
    a = (counter_normal(key, int(np.prod(shape)), seed) * np.float32(std)).reshape(shape)
    return round_bf16(a) if bf16 else a


# ----------------------------------------------------------------------------------------------------------------
# diffusers checkpoint format
# ----------------------------------------------------------------------------------------------------------------

WEIGHTS_NAME = "diffusion_pytorch_model.safetensors"
CONFIG_NAME = "config.json"


def load_config(path: str, subfolder: Optional[str] = None) -> dict:
    d = os.path.join(path, subfolder) if subfolder else path
    with open(os.path.join(d, CONFIG_NAME)) as f:
        return json.load(f)


def save_config(path: str, config: dict, class_name: str) -> None:
    os.makedirs(path, exist_ok=True)
    cfg = dict(config)
    cfg["_class_name"] = class_name
    with open(os.path.join(path, CONFIG_NAME), "w") as f:
        json.dump(cfg, f, indent=2, sort_keys=True)


def weight_files(path: str, subfolder: Optional[str] = None) -> Iterable[str]:
    d = os.path.join(path, subfolder) if subfolder else path
    single = os.path.join(d, WEIGHTS_NAME)
    if os.path.exists(single):
        return [single]
    index = os.path.join(d, WEIGHTS_NAME.replace(".safetensors", ".safetensors.index.json"))
    if os.path.exists(index):
        with open(index) as f:
            files = sorted(set(json.load(f)["weight_map"].values()))
        return [os.path.join(d, x) for x in files]
    raise FileNotFoundError(f"no {WEIGHTS_NAME} (or sharded index) under {d}")
