"""Batched SHA-256 front end (K3/K4): txids and merkle leaves.

``batch`` hashes many messages in one call: the gfx950 one-message-per-lane kernel
(csrc/sha256_batch.hip) for large batches on a GPU box, the threaded host C++ core otherwise.
The merkle root keeps the reference definition (upow/manager.py:365-378): leaves are the txids of
the transactions sorted by raw bytes; the final chained hash over 32*N bytes is sequential and
runs on the host.
"""
from __future__ import annotations

import hashlib
import os
from typing import Iterable, List, Optional, Sequence

import numpy as np

from .native import gpu_available, lib

GPU_MIN_BATCH = int(os.environ.get('UPOW_SHA_GPU_MIN_BATCH', '4096'))


def batch(messages: Sequence[bytes], device: Optional[str] = None) -> List[bytes]:
    n = len(messages)
    if n == 0:
        return []
    if device is None:
        device = 'gpu' if (gpu_available() and n >= GPU_MIN_BATCH) else 'cpu'
    data = np.frombuffer(b''.join(messages), dtype=np.uint8)
    offs = np.zeros(n + 1, dtype=np.int64)
    np.cumsum([len(m) for m in messages], out=offs[1:])
    L = lib()
    if device == 'gpu':
        out = L.sha256_batch_gpu(data, offs)
    else:
        out = L.sha256_batch_host(data, offs, max(1, min(os.cpu_count() or 1, 16)))
    return [out[32 * i:32 * i + 32] for i in range(n)]


def merkle_root(tx_bytes: Iterable[bytes], device: Optional[str] = None) -> str:
    ordered = sorted(tx_bytes)
    h = hashlib.sha256()
    for d in batch(ordered, device=device):
        h.update(d)
    return h.hexdigest()
