"""P-256 front end: single sign/verify (host C++) and batched verify/decompress (gfx950 kernels).

Batch record layout (160 B, little-endian like the wire format): ``qx | qy | r | s | e`` where ``e``
is the SHA-256 digest of the signed message (big-endian, as hashed). Status codes: 1 valid,
0 invalid, 2 public key not on the curve, 3 r or s outside [1, n] — fastecdsa raises for 2 and 3
(reference transaction_input.py:100-109), which :func:`verify` reproduces with ``EcdsaError``.
"""
from __future__ import annotations

import hashlib
import os
from typing import Iterable, List, Optional, Sequence, Tuple, Union

import numpy as np

from ..utils import coalesce
from ..utils.cpus import cpu_budget
from ..utils import p256 as oracle
from ..utils.p256 import EcdsaError, Point
from .native import gpu_available, lib

VALID, INVALID, BAD_KEY, BAD_RANGE = 1, 0, 2, 3
# below this many signatures (or keys) a batch runs on host threads. The quad kernel's latency floor is
# ~1.3 ms whatever the batch (one signature's double-scalar chain on four lanes); 16 host threads pass it
# near 100 signatures on an MI355X box (a 200-tx sync block: 2.5 ms host vs 1.4 ms GPU, docs/PERF.md)
GPU_MIN_BATCH = int(os.environ.get('UPOW_P256_GPU_MIN_BATCH', '64'))


def _msg(m: Union[str, bytes]) -> bytes:
    return m.encode() if isinstance(m, str) else bytes(m)


def public_key(d: int) -> Point:
    out = lib().p256_pubkey(int(d).to_bytes(32, 'big'))
    if out is None:
        raise ValueError('private key out of range')
    return Point(int.from_bytes(out[:32], 'little'), int.from_bytes(out[32:], 'little'), check=False)


def sign(msg: Union[str, bytes], d: int) -> Tuple[int, int]:
    res = lib().p256_sign(int(d).to_bytes(32, 'big'), hashlib.sha256(_msg(msg)).digest())
    if res is None:
        raise ValueError('signing failed')
    return int.from_bytes(res[0], 'little'), int.from_bytes(res[1], 'little')


def record(q: Point, sig: Tuple[int, int], digest: bytes) -> bytes:
    r, s = sig
    if not (0 <= r < 1 << 256 and 0 <= s < 1 << 256):
        raise EcdsaError('signature component out of range')
    return (q.x.to_bytes(32, 'little') + q.y.to_bytes(32, 'little') + r.to_bytes(32, 'little')
            + s.to_bytes(32, 'little') + digest)


def verify_records(records: Union[bytes, bytearray, np.ndarray], device: Optional[str] = None,
                   threads: int = 0) -> np.ndarray:
    """Batched verify of packed 160-byte records -> uint8 status array."""
    buf = records if isinstance(records, np.ndarray) else np.frombuffer(bytes(records), dtype=np.uint8)
    n = buf.size // 160
    if device is None:
        device = 'gpu' if (gpu_available() and n >= GPU_MIN_BATCH) else 'cpu'
    st = lib().p256_verify(buf, device == 'gpu', threads or max(1, min(cpu_budget(), 16)))
    return np.frombuffer(st, dtype=np.uint8)


def verify(sig: Tuple[int, int], msg: Union[str, bytes], q: Point) -> bool:
    """fastecdsa.ecdsa.verify(sig, msg, Q, P256) contract, on the host C++ core."""
    r, s = sig
    if r >= 1 << 256 or s >= 1 << 256 or r < 0 or s < 0:
        raise EcdsaError('Invalid Signature: r/s out of range')
    st = verify_records(record(q, sig, hashlib.sha256(_msg(msg)).digest()), device='cpu', threads=1)[0]
    if st == BAD_KEY:
        raise EcdsaError('Invalid public key, point is not on curve P256')
    if st == BAD_RANGE:
        raise EcdsaError('Invalid Signature: r or s is not a positive integer smaller than the curve order')
    return bool(st == VALID)


# ---------------------------------------------------------------------------------------------- admission
# reference: every /push_tx verifies its signatures one at a time on the node's event loop
# (transaction_input.py:100-109 via fastecdsa). Inside an admission context (utils/coalesce.py) the
# checks of concurrent requests are verified together on an executor thread: on the GPU when the batch is
# large enough to beat a round trip, else on host threads. The event loop never runs an ECDSA verify.
ADMISSION_GPU_MIN = int(os.environ.get('UPOW_ADMISSION_GPU_MIN', '32'))


def _verify_batch(recs: List[bytes]) -> bytes:
    n = len(recs)
    gpu = gpu_available() and n >= ADMISSION_GPU_MIN
    return lib().p256_verify(np.frombuffer(b''.join(recs), dtype=np.uint8), gpu, max(1, min(n, 8)))


async def verify_async(sig: Tuple[int, int], msg: Union[str, bytes], q: Point) -> bool:
    """:func:`verify` (same result, same exceptions); inside an admission context it goes through the
    event loop's signature coalescer instead of running on the loop."""
    if not coalesce.ADMISSION.get():
        return verify(sig, msg, q)
    r, s = sig
    if r >= 1 << 256 or s >= 1 << 256 or r < 0 or s < 0:
        raise EcdsaError('Invalid Signature: r/s out of range')
    st = await coalesce.coalescer('p256-admit', _verify_batch).submit(record(q, sig, hashlib.sha256(_msg(msg)).digest()))
    if st == BAD_KEY:
        raise EcdsaError('Invalid public key, point is not on curve P256')
    if st == BAD_RANGE:
        raise EcdsaError('Invalid Signature: r or s is not a positive integer smaller than the curve order')
    return st == VALID


def decompress(addresses33: Sequence[bytes], device: Optional[str] = None):
    """Batch decompression of 33-byte addresses -> (list of (x, y) or None)."""
    n = len(addresses33)
    if n == 0:
        return []
    buf = b''.join(bytes(a) for a in addresses33)
    if device is None:
        device = 'gpu' if (gpu_available() and n >= GPU_MIN_BATCH) else 'cpu'
    out, ok = lib().p256_decompress(buf, device == 'gpu')
    res = []
    for i in range(n):
        if ok[i]:
            res.append((int.from_bytes(out[64 * i:64 * i + 32], 'little'),
                        int.from_bytes(out[64 * i + 32:64 * i + 64], 'little')))
        else:
            res.append(None)
    return res


__all__ = ['public_key', 'sign', 'verify', 'verify_async', 'verify_records', 'decompress', 'record', 'EcdsaError', 'oracle']
