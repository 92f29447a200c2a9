"""Cross-GPU transaction-verify parallelism.

The reference verifies a block's signatures one after another in one process
(``manager.py:628-632`` → ``transaction_input.py:100-120``). Transactions of a block are independent
(an output created inside the block cannot be spent inside it: the pre-block UTXO lookup of
``manager.py:531,545-564`` rejects that), so on a G-GPU node the signature batch is split into G
contiguous shards:

  * every rank holds the same block (the cluster leader broadcast it once over xGMI as a 'block' op,
    parallel/cluster.py) and builds the same job list deterministically;
  * rank r verifies shard r with the batched P-256 kernel on its own GPU;
  * the per-signature status bytes are all-gathered (1 B per signature: ~8 KB for a 2 MB block —
    one small RCCL all-gather), so every replica reaches the same verdict and reports the same
    first failing tx; :func:`first_failure` is the 8-byte all-reduce(MIN) variant for callers that
    only need the block verdict.

Mempool and ledger replication are the cluster's op stream (parallel/cluster.py: batched 'txs' ops,
'block' ops applied by every replica), not functions of this module.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np

from ..ops import p256 as op
from .dist import DistContext

RECORD = 160


def shard_bounds(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous, balanced [lo, hi) of ``n`` items for ``rank``; shards differ by at most one item."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def verify_records_dp(ctx: DistContext, records, device: Optional[str] = None) -> np.ndarray:
    """Sharded batched verify: returns the FULL status vector on every rank.

    ``records`` is the same packed 160-byte record buffer on every rank (deterministic job build)."""
    buf = records if isinstance(records, np.ndarray) else np.frombuffer(bytes(records), dtype=np.uint8)
    n = buf.size // RECORD
    if not ctx.is_distributed:
        return op.verify_records(buf, device=device)
    lo, hi = shard_bounds(n, ctx.world, ctx.rank)
    local = op.verify_records(buf[lo * RECORD:hi * RECORD], device=device) if hi > lo else np.zeros(0, np.uint8)
    parts = ctx.all_gather_bytes(local.tobytes())
    out = np.frombuffer(b''.join(parts), dtype=np.uint8)
    assert out.size == n, (out.size, n)
    return out


def verify_shard_dp(ctx: DistContext, local_records, n_total: int, device: Optional[str] = None) -> np.ndarray:
    """Like :func:`verify_records_dp` for a rank that holds the records of its own shard only
    (``shard_bounds(n_total, world, rank)``, ledger/pagesync.py builds no others): verify them, all-gather
    the status bytes, return the FULL status vector on every rank."""
    buf = local_records if isinstance(local_records, np.ndarray) else np.frombuffer(bytes(local_records), np.uint8)
    lo, hi = shard_bounds(n_total, ctx.world, ctx.rank)
    assert buf.size == (hi - lo) * RECORD, (buf.size, lo, hi)
    local = op.verify_records(buf, device=device) if hi > lo else np.zeros(0, np.uint8)
    out = np.frombuffer(b''.join(ctx.all_gather_bytes(local.tobytes())), dtype=np.uint8)
    assert out.size == n_total, (out.size, n_total)
    return out


def first_failure(ctx: DistContext, local_status: np.ndarray, lo: int, n_total: int) -> int:
    """All-reduce(MIN) of the first non-valid global index; ``-1`` when every signature is valid."""
    bad = np.nonzero(local_status != op.VALID)[0]
    mine = int(lo + bad[0]) if len(bad) else n_total
    g = ctx.allreduce_min(mine)
    return -1 if g >= n_total else g


def verify_shard_first_failure(ctx: DistContext, records, device: Optional[str] = None) -> int:
    """Verdict-only path: each rank verifies its shard, one 8-byte all-reduce decides the block."""
    buf = records if isinstance(records, np.ndarray) else np.frombuffer(bytes(records), dtype=np.uint8)
    n = buf.size // RECORD
    lo, hi = shard_bounds(n, ctx.world, ctx.rank) if ctx.is_distributed else (0, n)
    local = op.verify_records(buf[lo * RECORD:hi * RECORD], device=device) if hi > lo else np.zeros(0, np.uint8)
    return first_failure(ctx, local, lo, n)


__all__ = ['shard_bounds', 'verify_records_dp', 'verify_shard_dp', 'first_failure', 'verify_shard_first_failure']
