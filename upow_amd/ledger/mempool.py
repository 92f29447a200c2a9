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
from operator import itemgetter
from typing import Dict, Iterable, List, Optional, Set, Tuple

import numpy as np


def outpoint_key(tx_hash: str, index: int) -> bytes:
    return bytes.fromhex(tx_hash) + int(index).to_bytes(4, 'little')


def _rows_raw(arr: np.ndarray, width: int) -> List[bytes]:
    """The leading ``width`` bytes of each row of an n x k uint8 array, as bytes objects."""
    a = np.ascontiguousarray(np.asarray(arr, dtype=np.uint8)[:, :width])
    return a.view(f'V{width}').ravel().tolist()  # void scalars -> bytes, built in C


_second = itemgetter(1)


def order_key(tx_hex: str, fees) -> tuple:
    return (-(Decimal(fees) / len(tx_hex)), len(tx_hex), tx_hex)


class MempoolIndex:
    def __init__(self, tx_rows: Iterable[Tuple[str, int, str, str]], spent_rows: Iterable[Tuple[str, int]]):
        """``tx_rows``: (tx_hash, propagation_time, tx_hex, fees) of pending_transactions."""
        self.lock = threading.Lock()
        self.txs: Dict[bytes, int] = {}  # tx hash -> propagation time
        self.keys: Dict[bytes, tuple] = {}  # tx hash -> order_key
        for h, t, hx, fees in tx_rows:
            k = bytes.fromhex(h)
            self.txs[k] = int(t)
            self.keys[k] = order_key(hx, fees)
        self.spent: Set[bytes] = {outpoint_key(h, i) for h, i in spent_rows}
        # journal sequence of each admission's INSERT batch (rows loaded from SQL: 0, already materialised).
        # A block confirming a tx whose admission was journaled AFTER the block's own batch cannot rely on
        # that batch's DELETEs (they ran before the INSERTs): it needs a follow-up delete.
        self.seq: Dict[bytes, int] = {}
        self.spent_seq: Dict[bytes, int] = {}
        self.min_ptime: Optional[int] = min(self.txs.values()) if self.txs else None

    def empty(self) -> bool:
        return not self.txs and not self.spent

    def has_tx(self, tx_hash: str) -> bool:
        return bytes.fromhex(tx_hash) in self.txs

    def spent_of(self, outputs: Iterable[Tuple[str, int]]) -> List[Tuple[str, int]]:
        """The outpoints among ``outputs`` that a mempool tx already spends (unique, first seen)."""
        seen = dict.fromkeys((h, int(i)) for h, i in outputs)
        return [o for o in seen if outpoint_key(*o) in self.spent]

    def ordered(self, limit: int) -> List[Tuple[str, bytes]]:
        """(tx hex, raw tx hash) of the pending txs in block-template order, up to ``limit`` hex
        characters in total."""
        with self.lock:
            items = sorted(self.keys.items(), key=_second)
        out, size = [], 0
        for h, k in items:
            if size + k[1] > limit:
                break
            out.append((k[2], h))
            size += k[1]
        return out

    def hex_in_order(self, tx_hashes: Iterable[str]) -> List[str]:
        """tx hex of the pending txs among ``tx_hashes``, in admission (table row) order."""
        want = set()
        for h in tx_hashes:
            try:
                want.add(bytes.fromhex(h))
            except ValueError:
                continue
        with self.lock:
            if len(want) == 1:
                k = self.keys.get(next(iter(want)))
                return [k[2]] if k is not None else []
            return [k[2] for h, k in self.keys.items() if h in want]

    def ordered_hex(self, limit: int) -> List[str]:
        return [hx for hx, _ in self.ordered(limit)]

    def try_add(self, tx_hash: str, ptime: int, inputs: List[Tuple[str, int]], tx_hex: str, fees) -> Optional[str]:
        """Reserve a tx and its inputs (caller holds ``lock``); returns why it cannot be added, or None."""
        h = bytes.fromhex(tx_hash)
        if h in self.txs:
            return 'duplicate'
        keys = [outpoint_key(a, i) for a, i in inputs]
        if any(k in self.spent for k in keys):
            return 'double spend'
        self.txs[h] = int(ptime)
        self.keys[h] = order_key(tx_hex, fees)
        self.spent.update(keys)
        if self.min_ptime is None or ptime < self.min_ptime:
            self.min_ptime = int(ptime)
        return None

    def set_seq(self, tx_hash: str, inputs: List[Tuple[str, int]], seq: int):
        """Record the journal sequence of an admission's batch (caller holds ``lock``)."""
        self.seq[bytes.fromhex(tx_hash)] = int(seq)
        for a, i in inputs:
            self.spent_seq[outpoint_key(a, i)] = int(seq)

    def _confirm(self, tx_keys: List[bytes], in_keys: List[bytes], after: Optional[int] = None):
        """Remove confirmed txs and outpoints; returns (hit_tx, hit_in, late_tx, late_in) where the late
        lists hold the hits whose admission was journaled after sequence ``after``."""
        with self.lock:
            hit_tx = []
            if self.txs:
                pop = self.txs.pop
                hit_tx = [k for k in tx_keys if pop(k, None) is not None]
                for k in hit_tx:
                    del self.keys[k]
            hit_in = []
            if self.spent and in_keys:
                hit_in = list(self.spent.intersection(in_keys))
                self.spent.difference_update(hit_in)
            late_tx, late_in = [], []
            if hit_tx:
                sq = self.seq.pop
                late_tx = [k for k in hit_tx if sq(k, 0) > (after or 0)] if after is not None else []
            if hit_in:
                sq = self.spent_seq.pop
                late_in = [k for k in hit_in if sq(k, 0) > (after or 0)] if after is not None else []
            if not self.txs:
                self.min_ptime = None
            return hit_tx, hit_in, late_tx, late_in

    def confirm_raw(self, txids: np.ndarray, in_keys: np.ndarray, after: Optional[int] = None):
        """A committed block's txs (n x 32) and spent outpoints (n x >=36 records) leave the mempool;
        returns the raw tx hashes and outpoints that were in it (and those admitted after ``after``)."""
        return self._confirm(_rows_raw(txids, 32) if len(txids) else [],
                             _rows_raw(in_keys, 36) if len(in_keys) else [], after)

    def confirm(self, tx_hashes: List[str], inputs: List[Tuple[str, int]], after: Optional[int] = None):
        return self._confirm([bytes.fromhex(h) for h in tx_hashes], [outpoint_key(h, i) for h, i in inputs], after)

    def maybe_stale(self, now: int, delta: int) -> bool:
        """Could a pending tx be older than ``delta`` seconds? ``min_ptime`` only moves down between
        recomputes, so False is exact and True is re-checked against the current entries."""
        with self.lock:
            if self.min_ptime is None or now - self.min_ptime <= delta:
                return False
            self.min_ptime = min(self.txs.values()) if self.txs else None
            return self.min_ptime is not None and now - self.min_ptime > delta


__all__ = ['MempoolIndex', 'outpoint_key']
