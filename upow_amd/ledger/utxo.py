"""UTXO index: outpoint (txid, index) -> which of the seven output tables holds it.

reference: the reference answers every "is this outpoint unspent, and in which table" question with
``SELECT ... WHERE (tx_hash, index) = ANY($1::tx_output[])`` against PostgreSQL
(upow/database.py:788-825). Here the ledger keeps that relation in an index with two backends:

* ``gpu``  — the HBM open-addressing table of ``csrc/utxo_table.hip`` (probe/insert/erase kernels,
  one lane per outpoint; a whole block's inputs are one launch);
* ``host`` — a Python dict (CPU-only containers and small test ledgers).

Both expose the same batch API; the SQLite tables stay authoritative for address queries and the
index is rebuilt from them after a rollback.
"""
from __future__ import annotations

import os
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

TAG_BY_TABLE = {
    'unspent_outputs': 0,
    'inode_registration_output': 1,
    'validator_registration_output': 2,
    'validators_voting_power': 3,
    'delegates_voting_power': 4,
    'validators_ballot': 5,
    'inodes_ballot': 6,
}
TABLE_BY_TAG = {v: k for k, v in TAG_BY_TABLE.items()}
MISSING = 0xFF

Outpoint = Tuple[str, int]


def pack_records(keys: Sequence[Outpoint], tags=None) -> np.ndarray:
    """40-byte records {txid raw 32 B, u32 index, u32 tag} for the native table."""
    n = len(keys)
    rec = np.zeros((n, 40), dtype=np.uint8)
    if n == 0:
        return rec
    raw = b''.join(bytes.fromhex(h) for h, _ in keys)
    rec[:, :32] = np.frombuffer(raw, dtype=np.uint8).reshape(n, 32)
    idx = np.fromiter((int(i) for _, i in keys), dtype=np.uint32, count=n)
    rec[:, 32:36] = idx.view(np.uint8).reshape(n, 4)
    if tags is None:
        t = np.full(n, MISSING, dtype=np.uint32)
    elif isinstance(tags, int):
        t = np.full(n, tags, dtype=np.uint32)
    else:
        t = np.asarray(tags, dtype=np.uint32)
    rec[:, 36:40] = t.view(np.uint8).reshape(n, 4)
    return rec


class _HostBackend:
    def __init__(self):
        self.d: Dict[Outpoint, int] = {}

    def reset(self, keys, tags):
        self.d = {(h, int(i)): int(t) for (h, i), t in zip(keys, tags)}

    def insert(self, keys, tags):
        for (h, i), t in zip(keys, tags):
            self.d[(h, int(i))] = int(t)

    def probe(self, keys) -> np.ndarray:
        return np.array([self.d.get((h, int(i)), MISSING) for h, i in keys], dtype=np.uint8)

    def erase(self, keys, tag=None) -> np.ndarray:
        out = np.zeros(len(keys), dtype=np.uint8)
        for n, (h, i) in enumerate(keys):
            k = (h, int(i))
            t = self.d.get(k)
            if t is not None and (tag is None or t == tag):
                del self.d[k]
                out[n] = 1
        return out

    def records(self) -> np.ndarray:
        return pack_records(list(self.d.keys()), list(self.d.values()))

    def __len__(self):
        return len(self.d)


class _GpuBackend:
    """HBM table; grows (rehash via dump + re-insert) past 50 % load."""

    def __init__(self, log2_cap: int = 20):
        from ..ops.native import require_gpu
        self.L = require_gpu()
        self.log2 = log2_cap
        self.h = self.L.utxo_create(log2_cap)
        self.count = 0
        self.tombs = 0

    def __del__(self):
        try:
            self.L.utxo_destroy(self.h)
        except Exception:
            pass

    def _ensure(self, extra: int):
        need = self.count + self.tombs + extra
        if need * 2 <= (1 << self.log2):
            return
        recs = np.frombuffer(self.L.utxo_dump(self.h), dtype=np.uint8).reshape(-1, 40)
        while (len(recs) + extra) * 2 > (1 << self.log2):
            self.log2 += 1
        self.L.utxo_destroy(self.h)
        self.h = self.L.utxo_create(self.log2)
        if len(recs):
            assert self.L.utxo_insert(self.h, np.ascontiguousarray(recs)) == 0
        self.count, self.tombs = len(recs), 0

    def reset(self, keys, tags):
        self.L.utxo_destroy(self.h)
        self.log2 = int(np.ceil(np.log2(max(2 * len(keys), 1 << 20))))
        self.h = self.L.utxo_create(self.log2)
        self.count = self.tombs = 0
        self.insert(keys, tags)

    def insert(self, keys, tags):
        if not len(keys):
            return
        self._ensure(len(keys))
        failed = self.L.utxo_insert(self.h, pack_records(keys, list(tags)))
        if failed:
            raise RuntimeError(f'UTXO table insert failed for {failed} entries')
        self.count += len(keys)

    def insert_records(self, recs: np.ndarray):
        self._ensure(len(recs))
        if self.L.utxo_insert(self.h, recs):
            raise RuntimeError('UTXO table insert failed')
        self.count += len(recs)

    def probe(self, keys) -> np.ndarray:
        if not len(keys):
            return np.zeros(0, dtype=np.uint8)
        return np.frombuffer(self.L.utxo_probe(self.h, pack_records(keys)), dtype=np.uint8)

    def probe_records(self, recs: np.ndarray) -> np.ndarray:
        return np.frombuffer(self.L.utxo_probe(self.h, recs), dtype=np.uint8)

    def erase(self, keys, tag=None) -> np.ndarray:
        if not len(keys):
            return np.zeros(0, dtype=np.uint8)
        out = np.frombuffer(self.L.utxo_erase(self.h, pack_records(keys, MISSING if tag is None else tag)),
                            dtype=np.uint8)
        k = int(out.sum())
        self.count -= k
        self.tombs += k
        return out

    def records(self) -> np.ndarray:
        return np.frombuffer(self.L.utxo_dump(self.h), dtype=np.uint8).reshape(-1, 40)

    def __len__(self):
        return self.count


def default_backend() -> str:
    env = os.environ.get('UPOW_UTXO_BACKEND')
    if env:
        return env
    from ..ops.native import gpu_available
    try:
        return 'gpu' if gpu_available() else 'host'
    except Exception:
        return 'host'


class UtxoIndex:
    def __init__(self, backend: Optional[str] = None):
        self.backend_name = backend or default_backend()
        self.be = _GpuBackend() if self.backend_name == 'gpu' else _HostBackend()

    def reset(self, keys: Sequence[Outpoint], tags: Sequence[int]):
        self.be.reset(list(keys), list(tags))

    def insert(self, keys: Sequence[Outpoint], tag):
        keys = list(keys)
        tags = [tag] * len(keys) if isinstance(tag, int) else list(tag)
        self.be.insert(keys, tags)

    def probe(self, keys: Sequence[Outpoint]) -> np.ndarray:
        return self.be.probe(list(keys))

    def erase(self, keys: Sequence[Outpoint], tag: Optional[int] = None) -> np.ndarray:
        return self.be.erase(list(keys), tag)

    def filter(self, outputs: Iterable[Outpoint], tag: int) -> List[Outpoint]:
        """Outpoints of ``outputs`` present in table ``tag`` (unique, in first-seen order)."""
        uniq = list(dict.fromkeys((h, int(i)) for h, i in outputs))
        if not uniq:
            return []
        t = self.probe(uniq)
        return [k for k, v in zip(uniq, t) if v == tag]

    def records(self) -> np.ndarray:
        """All live entries as 40-byte records, in canonical (txid, index) order."""
        return sort_records(np.ascontiguousarray(self.be.records()))

    def reset_records(self, recs: np.ndarray):
        """Replace the whole index with packed records (snapshot restore: one H2D copy + insert launch)."""
        recs = np.ascontiguousarray(recs, dtype=np.uint8).reshape(-1, 40)
        if isinstance(self.be, _GpuBackend):
            self.be.reset([], [])
            if len(recs):
                self.be.insert_records(recs)
        else:
            idx = recs[:, 32:36].copy().view(np.uint32).ravel()
            tags = recs[:, 36:40].copy().view(np.uint32).ravel()
            self.be.d = {(bytes(recs[n, :32]).hex(), int(idx[n])): int(tags[n]) for n in range(len(recs))}

    def set_hash(self, tag: int = 0) -> str:
        """K12 from the index: SHA-256 over (txid || index byte) of table ``tag`` sorted by (txid, index)
        — byte-identical to ``Database.get_unspent_outputs_hash`` (reference database.py:827-830)."""
        import hashlib
        recs = self.records()
        recs = recs[recs[:, 36:40].copy().view(np.uint32).ravel() == tag]
        payload = np.concatenate([recs[:, :32], recs[:, 32:33]], axis=1)  # index byte (the reference's bytes([i]))
        return hashlib.sha256(payload.tobytes()).hexdigest()

    def __len__(self):
        return len(self.be)


def sort_records(recs: np.ndarray) -> np.ndarray:
    """Sort packed records by (txid bytes, index): the SQL ``ORDER BY tx_hash, index`` order."""
    if len(recs) < 2:
        return recs
    be = recs[:, :32].copy().view('>u8')  # 4 big-endian words compare like the hex strings
    idx = recs[:, 32:36].copy().view(np.uint32).ravel()
    order = np.lexsort((idx, be[:, 3], be[:, 2], be[:, 1], be[:, 0]))
    return recs[order]
