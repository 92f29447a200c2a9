"""K1 proof-of-work search: Python front end of ``csrc/pow_search.hip``.

The GPU kernel filters nonces on digest word H0 (exact for difficulty < 8); every candidate is
re-checked here against the full reference predicate (upow/manager.py:130-151) before it is
reported, so a result is always a header the reference node would accept.
"""
from __future__ import annotations

import hashlib
import os
import time
from dataclasses import dataclass
from typing import List, Optional

from ..models.block import PowTarget
from ..utils import metrics
from .native import gpu_available, lib

NONCE_SPACE = 1 << 32


@dataclass
class PowJob:
    header: bytes          # full header with the nonce bytes zeroed (108 B v2 / 138 B v1)
    target: PowTarget
    tmask: int
    tword: int
    frac_shift: int
    frac_limit: int

    @staticmethod
    def create(prefix: bytes, target: PowTarget) -> 'PowJob':
        if len(prefix) not in (104, 134):
            raise ValueError(f'header prefix must be 104 (v2) or 134 (v1) bytes, got {len(prefix)}')
        if target.frac_nibble >= 0 and target.frac_nibble < 8:
            fs, fl = 28 - 4 * target.frac_nibble, target.frac_limit
        else:
            fs, fl = 0, 16
        return PowJob(bytes(prefix) + b'\0\0\0\0', target, target.masks[0], target.words[0], fs, fl)

    @property
    def v2(self) -> bool:
        return len(self.header) == 108

    def word_to_nonce(self, w: int) -> int:
        return int.from_bytes(w.to_bytes(4, 'big'), 'little') if self.v2 else w

    def nonce_to_word(self, n: int) -> int:
        return int.from_bytes(n.to_bytes(4, 'little'), 'big') if self.v2 else n

    def header_with_nonce(self, nonce: int) -> bytes:
        return self.header[:-4] + nonce.to_bytes(4, 'little')

    def exact_check(self, nonce: int) -> bool:
        return self.target.check_hex(hashlib.sha256(self.header_with_nonce(nonce)).hexdigest())

    def native_args(self):
        return (self.header, self.tmask, self.tword, self.frac_shift, self.frac_limit)


@dataclass
class PowSearchResult:
    searched: int
    candidates: int
    nonces: List[int]  # exact-checked valid nonces, in nonce-word order


def search(job: PowJob, start: int = 0, count: int = NONCE_SPACE, device: Optional[str] = None,
           threads: Optional[int] = None, grid_blocks: int = 0, chunk_iters: int = 0,
           cap: int = 1 << 16, variant: int = 0) -> PowSearchResult:
    """Search nonce *words* [start, start+count). ``device`` = 'gpu' | 'cpu' | None (auto)."""
    L = lib()
    if device is None:
        device = 'gpu' if gpu_available() else 'cpu'
    t0 = time.perf_counter()
    if device == 'gpu':
        searched, hits, words = L.pow_search_gpu(*job.native_args(), start, count, grid_blocks, chunk_iters,
                                                 cap, variant)
    else:
        searched, hits, words = L.pow_search_host(*job.native_args(), start, count,
                                                  threads or max(1, os.cpu_count() or 1))
    dt = time.perf_counter() - t0
    metrics.inc('upow_pow_hashes_total', searched, labels={'device': device}, help='nonces hashed by PoW search')
    if dt > 0:
        metrics.set_gauge('upow_pow_hashrate', searched / dt, labels={'device': device},
                          help='H/s of the last PoW search call')
    nonces = []
    for w in sorted(words):
        n = job.word_to_nonce(w)
        if job.exact_check(n):
            nonces.append(n)
    return PowSearchResult(searched, hits, nonces)
