"""Seeded synthetic workloads for the batched CCEH path.

Keys are produced by splitmix64 over a counter, a bijection on u64, so a key
stream is duplicate-free by construction.  0, INVALID (2^64-1) and SENTINEL
(2^64-2) are never emitted (they are remapped; the chance of hitting one is
~2^-62 per key).  The same generator exists on the device
(``pmdfc_gen_keys`` in include/pmdfc_cceh.h) and tests pin the two together.

Key shapes mirror the reference harnesses:
  * uniform u64 keys, value = key          (server/test_KV.cpp:204-221)
  * replay shape key = (inode<<32) + 4096*page  (server/replay_KV.cpp:218-242)
"""
from __future__ import annotations

import numpy as np

INVALID = np.uint64(0xFFFFFFFFFFFFFFFF)
SENTINEL = np.uint64(0xFFFFFFFFFFFFFFFE)

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(x: np.ndarray) -> np.ndarray:
    """splitmix64 finalizer of (x + golden); x is a uint64 array."""
    with np.errstate(over="ignore"):
        z = x.astype(np.uint64) + _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return z


def uniform_keys(seed: int, start: int, n: int) -> np.ndarray:
    """Keys number start..start+n-1 of stream `seed` (unique within a stream)."""
    with np.errstate(over="ignore"):
        ctr = np.arange(start, start + n, dtype=np.uint64) + (np.uint64(seed) << np.uint64(40))
    k = splitmix64(ctr)
    bad = (k == 0) | (k == INVALID) | (k == SENTINEL)
    if bad.any():
        k[bad] = np.uint64(0x5555555555555555) + ctr[bad]
    return k


def replay_keys(inode: np.ndarray, page: np.ndarray) -> np.ndarray:
    """server/replay_KV.cpp:218-242: key = (inode << 32) + offset + 4096*b."""
    return (inode.astype(np.uint64) << np.uint64(32)) + np.uint64(4096) * page.astype(np.uint64)


def zipf_ranks(rng: np.random.Generator, n_items: int, theta: float, size: int) -> np.ndarray:
    """YCSB-style Zipf(theta) ranks in [0, n_items) (Gray et al. generator)."""
    zetan = _zeta(n_items, theta)
    zeta2 = _zeta(2, theta)
    alpha = 1.0 / (1.0 - theta)
    eta = (1 - (2.0 / n_items) ** (1 - theta)) / (1 - zeta2 / zetan)
    u = rng.random(size)
    uz = u * zetan
    r = (n_items * (eta * u - eta + 1) ** alpha).astype(np.int64)
    r = np.where(uz < 1.0, 0, np.where(uz < 1.0 + 0.5 ** theta, 1, r))
    return np.clip(r, 0, n_items - 1)


def _zeta(n: int, theta: float) -> float:
    # exact for small n, Euler-Maclaurin tail for large n
    m = min(n, 1 << 20)
    s = float(np.sum(1.0 / np.arange(1, m + 1, dtype=np.float64) ** theta))
    if n > m:
        a, b = float(m), float(n)
        s += (b ** (1 - theta) - a ** (1 - theta)) / (1 - theta)
        s += 0.5 * (b ** -theta - a ** -theta)
    return s


def scramble(ranks: np.ndarray, n_items: int, seed: int) -> np.ndarray:
    """Fixed seeded permutation of [0, n_items) applied to Zipf ranks so hot
    keys spread over segments."""
    # affine bijection mod n_items with an odd multiplier coprime to n_items
    rng = np.random.default_rng(seed)
    while True:
        a = int(rng.integers(1, n_items)) | 1
        if np.gcd(a, n_items) == 1:
            break
    b = int(rng.integers(0, n_items))
    return ((ranks.astype(np.int64) * a + b) % n_items).astype(np.int64)


def synth_trace(seed: int, n_lines: int, n_inodes: int = 1 << 20) -> bytes:
    """A large replay_KV-format trace (server/replay_KV.cpp:24-31) built with
    numpy: 40% W / 50% R / 10% O lines, page-aligned offsets, sizes of 1-16
    pages; reads revisit earlier writes' (inode, offset).  Duplicate-page
    writes stay far below the 33-copy limit at these sizes."""
    rng = np.random.default_rng(seed)
    u = rng.random(n_lines)
    op = np.where(u < 0.4, "W", np.where(u < 0.9, "R", "O"))
    ino = rng.integers(1, n_inodes + 1, n_lines)
    off = 4096 * rng.integers(0, 256, n_lines)
    wi = np.nonzero(op == "W")[0]
    ri = np.nonzero(op == "R")[0]
    src = wi[np.clip(np.searchsorted(wi, ri) - 1 - rng.integers(0, 64, ri.size), 0, None)] if wi.size else ri
    ino[ri], off[ri] = ino[src], off[src]
    size = 4096 * rng.integers(1, 17, n_lines) - rng.integers(0, 2, n_lines) * 100
    lines = [f"{i} {i * 7}.{i % 1000:03d} {o} {a} 1048576 {b} {c}" for i, o, a, b, c in
             zip(range(n_lines), op.tolist(), ino.tolist(), off.tolist(), size.tolist())]
    return ("\n".join(lines) + "\n").encode()
