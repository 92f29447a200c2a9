"""Host-memory index of the mempool tables, so ``/push_tx`` admission never waits for SQL.

reference: ``add_pending_transaction`` (upow/database.py:93-115) INSERTs into ``pending_transactions``
and ``pending_spent_outputs``, and ``verify_pending`` asks ``get_pending_spent_outputs``
(database.py:832-838) whether an input is already spent by a mempool tx; ``create_block`` deletes the
confirmed txs and their inputs from both tables (manager.py:717-730). Here block writes reach SQLite
through the journal's background materialiser (csrc/ledger_writer.cpp), so a SQL read of a mempool table
right after a block has to wait for that block's rows to land (tens of ms for a full block). This index
holds what admission needs — the pending tx hashes (with their propagation time) and the outpoints they
spend — and follows every writer of the two tables:

* admission adds the tx here and journals its two INSERTs as one small batch (no FK wait: the inputs were
  just found unspent, so their txs are confirmed);
* a block removes its txs and inputs here when it commits (native and object paths);
* any other Python-side write to a mempool table drops the index; the next use re-reads it from SQL.

Keys are raw bytes: 32-byte tx hashes, 36-byte outpoints (txid || index u32 LE), the layout of the
block codec's input records, so a block's removal is a slice of its arrays, not a hex round trip.

Each pending tx also keeps its block-template sort key — ``ORDER BY fees / LENGTH(tx_hex) DESC,
LENGTH(tx_hex), tx_hex`` (reference database.py:173-174) — so ``/get_mining_info`` orders the mempool
with one C-level sort of precomputed tuples instead of re-reading and re-keying every row from SQL.
"""
from __future__ import annotations

import threading
from decimal import Decimal
from typing import Dict, Iterable, List, Optional, Set, Tuple

import numpy as np


def outpoint_key(tx_hash: str, index: int) -> bytes:
    return bytes.fromhex(tx_hash) + int(index).to_bytes(4, 'little')


def _fee_text(fees) -> str:
    """The fee as plain decimal text (``numeric()`` strings pass through; a Decimal in exponent form is
    expanded) for the native index's exact 1e-8-unit parse."""
    return fees if isinstance(fees, str) else format(Decimal(fees), 'f')


class MempoolIndex:
    """The index in C++ (csrc/mempool_index.cpp ``MempoolIndexCore``): admissions are hash-map probes, and a
    committed block's raw txid / outpoint arrays leave it in one call without the GIL. ``lock`` serialises
    an admission's reserve + journal + sequence record against a block's confirm (ledger/database.py)."""

    def __init__(self, tx_rows: Iterable[Tuple[str, int, str, str]], spent_rows: Iterable[Tuple[str, int]]):
        """``tx_rows``: (tx_hash, propagation_time, tx_hex, fees) of pending_transactions."""
        from ..ops.native import lib
        self.lock = threading.Lock()
        self.core = lib().MempoolIndexCore()
        self.core.load([(h, int(t), hx, _fee_text(f)) for h, t, hx, f in tx_rows],
                       [(h, int(i)) for h, i in spent_rows])

    def __len__(self) -> int:
        return len(self.core)

    def empty(self) -> bool:
        return self.core.empty()

    def has_tx(self, tx_hash: str) -> bool:
        try:
            return self.core.has_tx(tx_hash)
        except ValueError:
            return False

    def spent_of(self, outputs: Iterable[Tuple[str, int]]) -> List[Tuple[str, int]]:
        """The outpoints among ``outputs`` that a mempool tx already spends (unique, first seen)."""
        return self.core.spent_of([(h, int(i)) for h, i in outputs])

    def ordered(self, limit: int) -> List[Tuple[str, bytes]]:
        """(tx hex, raw tx hash) of the pending txs in block-template order, up to ``limit`` hex
        characters in total."""
        with self.lock:
            return self.core.ordered(int(limit))

    def hex_in_order(self, tx_hashes: Iterable[str]) -> List[str]:
        """tx hex of the pending txs among ``tx_hashes``, in admission (table row) order."""
        with self.lock:
            return self.core.hex_in_order(list(tx_hashes))

    def mining_template(self, limit: int, head: int):
        """(first ``head`` hexes, tx hashes, the hashes as a JSON array body) of the txs ``ordered``
        selects, re-sorted by hex string as ``/get_mining_info`` publishes them."""
        with self.lock:
            first, hashes, frag, _ = self.core.mining_template(int(limit), int(head))
        return first, hashes, frag

    def ordered_hex(self, limit: int) -> List[str]:
        return [hx for hx, _ in self.ordered(limit)]

    def try_add(self, tx_hash: str, ptime: int, inputs: List[Tuple[str, int]], tx_hex: str, fees) -> Optional[str]:
        """Reserve a tx and its inputs (caller holds ``lock``); returns why it cannot be added, or None."""
        return self.core.try_add(tx_hash, int(ptime), [(h, int(i)) for h, i in inputs], tx_hex, _fee_text(fees))

    def set_seq(self, tx_hash: str, inputs: List[Tuple[str, int]], seq: int):
        """Record the journal sequence of an admission's batch (caller holds ``lock``)."""
        self.core.set_seq(tx_hash, [(h, int(i)) for h, i in inputs], int(seq))

    def confirm_raw(self, txids: np.ndarray, in_keys: np.ndarray, after: Optional[int] = None, on_hits=None):
        """A committed block's txs (n x 32) and spent outpoints (n x >=36 records) leave the mempool;
        returns the raw tx hashes and outpoints that were in it (and those admitted after ``after``).
        ``on_hits(index, hit_tx, hit_in)`` runs under ``lock`` right after the removal (cluster replication)."""
        t = np.ascontiguousarray(np.asarray(txids, dtype=np.uint8).reshape(-1, 32))
        k = np.asarray(in_keys, dtype=np.uint8)
        k = np.ascontiguousarray(k.reshape(-1, k.shape[-1] if k.ndim == 2 and k.shape[0] else 40))
        with self.lock:
            res = self.core.confirm_raw(t, k, after)
            if on_hits is not None and (res[0] or res[1]):
                on_hits(self, res[0], res[1])
            return res

    def confirm(self, tx_hashes: List[str], inputs: List[Tuple[str, int]], after: Optional[int] = None, on_hits=None):
        t = np.frombuffer(b''.join(bytes.fromhex(h) for h in tx_hashes), dtype=np.uint8).reshape(-1, 32)
        k = np.frombuffer(b''.join(outpoint_key(h, i) for h, i in inputs), dtype=np.uint8).reshape(-1, 36)
        return self.confirm_raw(t, k, after, on_hits)

    def maybe_stale(self, now: int, delta: int) -> bool:
        """Could a pending tx be older than ``delta`` seconds? The minimum propagation time only moves down
        between recomputes, so False is exact and True is re-checked against the current entries."""
        with self.lock:
            return self.core.maybe_stale(int(now), int(delta))


__all__ = ['MempoolIndex', 'outpoint_key']
