"""Local devnet helpers: mine blocks straight into a ledger (tests, benches, examples).

Mining uses the same PoW search as the miner CLI (gfx950 kernel when a GPU is visible, the
threaded host C++ search otherwise) and the same node entry point (``manager.create_block``).
"""
from __future__ import annotations

import hashlib
from decimal import Decimal
from typing import List, Optional

from .constants import GENESIS_PREV_HASH
from .models.block import PowTarget, get_transactions_merkle_tree, header_prefix
from .ops.pow import PowJob, search
from .utils.codec import timestamp


async def mine_header(address: str, transactions: List, ts: Optional[int] = None, device: Optional[str] = None,
                      chunk: int = 1 << 22) -> str:
    """Find a header for the next block on top of ``Database.instance``'s tip."""
    from .ledger import manager
    manager.Manager.difficulty = None
    difficulty, last_block = await manager.get_difficulty()
    prev = last_block['hash'] if 'hash' in last_block else GENESIS_PREV_HASH
    if ts is None:
        ts = max(timestamp(), last_block.get('timestamp', 0) + 1)
    merkle = get_transactions_merkle_tree([t.hex() if hasattr(t, 'hex') and not isinstance(t, (str, bytes)) else t
                                           for t in transactions])
    target = PowTarget.from_difficulty(prev, difficulty)
    job = PowJob.create(header_prefix(prev, address, merkle, ts, difficulty), target)
    if 'hash' not in last_block:
        return job.header_with_nonce(0).hex()  # first block: no PoW check (manager.py:137-138)
    start, step = 0, 1 << 12
    while start < 1 << 32:
        n = min(step, (1 << 32) - start)
        r = search(job, start, n, device=device)
        if r.nonces:
            return job.header_with_nonce(r.nonces[0]).hex()
        start += n
        step = min(step * 8, chunk)
    raise RuntimeError('nonce space exhausted')


def mine_header_raw(prev: str, address: str, merkle: str, ts: int, difficulty, device: Optional[str] = None,
                    chunk: int = 1 << 24) -> str:
    """Mine a header on an explicit previous hash (no ledger access)."""
    job = PowJob.create(header_prefix(prev, address, merkle, ts, difficulty), PowTarget.from_difficulty(prev, difficulty))
    start, step = 0, 1 << 12
    while start < 1 << 32:
        n = min(step, (1 << 32) - start)
        r = search(job, start, n, device=device)
        if r.nonces:
            return job.header_with_nonce(r.nonces[0]).hex()
        start += n
        step = min(step * 8, chunk)
    raise RuntimeError('nonce space exhausted')


async def mine_block(address: str, transactions: List = (), ts: Optional[int] = None,
                     device: Optional[str] = None) -> str:
    """Mine and apply one block; returns its hash. Raises with the node's error on rejection."""
    from .ledger import manager
    txs = list(transactions)
    content = await mine_header(address, txs, ts=ts, device=device)
    errors = []
    if not await manager.create_block(content, txs, error_list=errors):
        raise RuntimeError(errors[0] if errors else 'block rejected')
    return hashlib.sha256(bytes.fromhex(content)).hexdigest()
