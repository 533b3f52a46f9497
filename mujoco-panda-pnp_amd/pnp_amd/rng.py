"""Philox4x32-10 counter RNG for the synthetic benchmark inputs (BASELINE.md "Baseline plan").

key = seed (20250808 by default), counter = (global env index, draw index, 0, 0): every env's
inputs depend only on its global index, so a batch sharded over N GPUs (rank r owns envs
[r*B, (r+1)*B)) sees bit-identical inputs at any GPU count.
"""
from __future__ import annotations

import numpy as np

SEED = 20250808
_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)


def philox4x32(counter: np.ndarray, key: tuple[int, int]) -> np.ndarray:
    """counter [N,4] uint32 -> [N,4] uint32 (10 rounds)."""
    c = np.array(counter, dtype=np.uint32, copy=True)
    k0, k1 = np.uint32(key[0] & 0xFFFFFFFF), np.uint32(key[1] & 0xFFFFFFFF)
    for _ in range(10):
        p0 = c[:, 0].astype(np.uint64) * _M0
        p1 = c[:, 2].astype(np.uint64) * _M1
        hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), (p0 & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), (p1 & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        c = np.stack([hi1 ^ c[:, 1] ^ k0, lo1, hi0 ^ c[:, 3] ^ k1, lo0], axis=1)
        k0 = np.uint32((int(k0) + int(_W0)) & 0xFFFFFFFF)
        k1 = np.uint32((int(k1) + int(_W1)) & 0xFFFFFFFF)
    return c


def uniform(env_index: np.ndarray, ndraw: int, seed: int = SEED, stream: int = 0) -> np.ndarray:
    """[N, ndraw] float64 uniforms in [0, 1) for the given global env indices."""
    env_index = np.asarray(env_index, np.uint64)
    n = env_index.size
    blocks = (ndraw + 3) // 4
    ctr = np.zeros((n * blocks, 4), np.uint32)
    ctr[:, 0] = np.repeat(env_index & np.uint64(0xFFFFFFFF), blocks).astype(np.uint32)
    ctr[:, 1] = np.tile(np.arange(blocks, dtype=np.uint32), n)
    ctr[:, 2] = np.uint32(stream)
    ctr[:, 3] = np.repeat(env_index >> np.uint64(32), blocks).astype(np.uint32)
    bits = philox4x32(ctr, (seed, seed >> 32)).reshape(n, blocks * 4)[:, :ndraw]
    return bits.astype(np.float64) * (1.0 / 4294967296.0)
