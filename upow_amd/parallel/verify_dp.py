"""Cross-GPU transaction-verify parallelism and ledger replication.

The reference verifies a block's signatures one after another in one process
(``manager.py:628-632`` → ``transaction_input.py:100-120``). Transactions of a block are independent
(an output created inside the block cannot be spent inside it: the pre-block UTXO lookup of
``manager.py:531,545-564`` rejects that), so on a G-GPU node the signature batch is split into G
contiguous shards:

  * every rank holds the same block (it was broadcast once over xGMI, :func:`broadcast_block`) and
    builds the same job list deterministically;
  * rank r verifies shard r with the batched P-256 kernel on its own GPU;
  * the per-signature status bytes are all-gathered (1 B per signature: ~8 KB for a 2 MB block —
    one small RCCL all-gather), so every replica reaches the same verdict and reports the same
    first failing tx; :func:`first_failure` is the 8-byte all-reduce(MIN) variant for callers that
    only need the block verdict.

Mempool: new pending txs seen by any rank are exchanged with one variable-length all-gather
(:func:`gather_mempool`) instead of the reference's per-tx HTTP re-propagation between processes.

Replication: :func:`replicate_block` broadcasts an accepted block (header + tx hex) from the rank that
received it; every rank applies it to its own ledger + HBM UTXO index, which stay bit-identical
because block application is deterministic (checked by comparing UTXO-set hashes in the tests).
"""
from __future__ import annotations

import json
from typing import List, Optional, Sequence, Tuple

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


# ------------------------------------------------------------------------------------------ mempool
def gather_mempool(ctx: DistContext, new_tx_hexes: Sequence[str]) -> List[str]:
    """Union of every rank's new pending txs (first-seen order by rank, duplicates dropped)."""
    payload = '\n'.join(new_tx_hexes).encode()
    seen, out = set(), []
    for part in ctx.all_gather_bytes(payload):
        for h in part.decode().split('\n') if part else ():
            if h and h not in seen:
                seen.add(h)
                out.append(h)
    return out


# ------------------------------------------------------------------------------------------ blocks
def broadcast_block(ctx: DistContext, block_content: Optional[str], txs: Optional[Sequence[str]], src: int = 0
                    ) -> Tuple[str, List[str]]:
    """Ship one block (header hex + tx hex list, <= ~4 MB) from ``src`` to every rank."""
    data = None
    if ctx.rank == src:
        data = json.dumps({'b': block_content, 't': list(txs or [])}, separators=(',', ':')).encode()
    raw = ctx.broadcast_bytes(data, src=src, max_len=0)
    obj = json.loads(raw.decode())
    return obj['b'], obj['t']


async def replicate_block(ctx: DistContext, block_content: Optional[str], txs: Optional[Sequence[str]],
                          src: int = 0) -> bool:
    """Broadcast a block from ``src`` and apply it on this rank's ledger replica.

    Returns the global verdict (all ranks must agree; a disagreement means the replicas diverged and
    raises)."""
    from ..ledger import manager
    from ..models.transaction import Transaction
    block_content, txs = broadcast_block(ctx, block_content, txs, src=src)
    transactions = [await Transaction.from_hex(h) for h in txs]
    ok = await manager.create_block(block_content, transactions)
    agree = ctx.allreduce_sum(1 if ok else 0)
    if agree not in (0, ctx.world):
        raise RuntimeError(f'ledger replicas diverged on block apply ({agree}/{ctx.world} accepted)')
    return bool(ok)


__all__ = ['shard_bounds', 'verify_records_dp', 'first_failure', 'verify_shard_first_failure', 'gather_mempool',
           'broadcast_block', 'replicate_block']
