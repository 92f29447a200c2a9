"""UTXO index: outpoint (txid, index) -> which of the seven output tables holds it.

reference: the reference answers every "is this outpoint unspent, and in which table" question with
``SELECT ... WHERE (tx_hash, index) = ANY($1::tx_output[])`` against PostgreSQL
(upow/database.py:788-825). Here the ledger keeps that relation in an index with two backends:

* ``gpu``  — the HBM open-addressing table of ``csrc/utxo_table.hip`` (probe/insert/erase kernels,
  one lane per outpoint; a whole block's inputs are one launch);
* ``host`` — the same table in C++ on the host (``csrc/utxo_host.cpp``; CPU-only nodes and the test
  suite), or a Python dict (``host-py``, and when the extension is not built).

Both expose the same batch API; the SQLite tables stay authoritative for address queries and the
index is rebuilt from them after a rollback.
"""
from __future__ import annotations

import functools
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

# per-outpoint payload carried by the index (csrc/utxo_table.hip UtxoPayload): the spent output's
# amount in smallest units, flags (bit 0: unspent_outputs.is_stake = 1) and its raw address bytes
# (33 compressed / 64 uncompressed)
PAYLOAD_DTYPE = np.dtype([('amount', '<u8'), ('len', '<u4'), ('flags', '<u4'), ('addr', 'u1', (64,))])
FLAG_STAKE = 1
STAKE_ANY, STAKE_EXCLUDE, STAKE_ONLY = 0, 1, 2  # address-scan selectors
assert PAYLOAD_DTYPE.itemsize == 80


def make_payload(amounts: Sequence[Optional[int]], addrs: Sequence[Optional[bytes]],
                 stake: Optional[Sequence] = None) -> np.ndarray:
    """Payload records; an unknown amount/address gives len 0 (consumers then fall back to SQL).
    ``stake``: per-output is_stake values (truthy -> FLAG_STAKE)."""
    n = len(amounts)
    p = np.zeros(n, dtype=PAYLOAD_DTYPE)
    if n == 0:
        return p
    if stake is not None:
        p['flags'] = np.fromiter((FLAG_STAKE if s else 0 for s in stake), dtype=np.uint32, count=n)
    raw = np.zeros((n, 64), dtype=np.uint8)
    lens = np.zeros(n, dtype=np.uint32)
    amt = np.zeros(n, dtype=np.uint64)
    for k, (a, b) in enumerate(zip(amounts, addrs)):
        if a is None or b is None or len(b) not in (33, 64) or a < 0 or a >= 1 << 64:
            continue
        raw[k, :len(b)] = np.frombuffer(bytes(b), dtype=np.uint8)
        lens[k] = len(b)
        amt[k] = a
    p['amount'] = amt
    p['len'] = lens
    p['addr'] = raw
    return p

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
        self.p: Dict[Outpoint, bytes] = {}  # raw 80-byte payloads
        self.by_addr: Dict[bytes, Dict[Outpoint, None]] = {}  # owner address bytes -> outpoints (K14 on the host)

    def reset(self, keys, tags, payload=None):
        self.d, self.p, self.by_addr = {}, {}, {}
        self.insert(keys, tags, payload)

    def insert(self, keys, tags, payload=None) -> int:
        """Returns the number of outpoints already present (left untouched, like the HBM table)."""
        raw = payload.tobytes() if payload is not None else None
        dups = 0
        for n, ((h, i), t) in enumerate(zip(keys, tags)):
            k = (h, int(i))
            if k in self.d:
                dups += 1
                continue
            self.d[k] = int(t)
            p = self.p[k] = raw[80 * n:80 * n + 80] if raw is not None else bytes(80)
            a = self._addr(p)
            if a:
                self.by_addr.setdefault(a, {})[k] = None
        return dups

    def probe(self, keys) -> np.ndarray:
        return np.array([self.d.get((h, int(i)), MISSING) for h, i in keys], dtype=np.uint8)

    def lookup(self, keys):
        zero = bytes(80)
        tags = np.array([self.d.get((h, int(i)), MISSING) for h, i in keys], dtype=np.uint8)
        pay = np.frombuffer(b''.join(self.p.get((h, int(i)), zero) for h, i in keys), dtype=PAYLOAD_DTYPE)
        return tags, pay

    def erase(self, keys, tag=None) -> np.ndarray:
        out = np.zeros(len(keys), dtype=np.uint8)
        for n, (h, i) in enumerate(keys):
            k = (h, int(i))
            t = self.d.get(k)
            if t is not None and (tag is None or t == tag):
                del self.d[k]
                a = self._addr(self.p.pop(k, None))
                owned = self.by_addr.get(a)
                if owned is not None:
                    owned.pop(k, None)
                    if not owned:
                        del self.by_addr[a]
                out[n] = 1
        return out

    def records(self) -> np.ndarray:
        return pack_records(list(self.d.keys()), list(self.d.values()))

    def address_scan(self, addr: bytes, tag_mask: int, stake_sel: int = STAKE_ANY):
        def stake_ok(k, t):
            if stake_sel == STAKE_ANY:
                return True
            st = t == 0 and bool(int.from_bytes(self.p.get(k, bytes(80))[12:16], 'little') & FLAG_STAKE)
            return st == (stake_sel == STAKE_ONLY)
        hits = [k for k in self.by_addr.get(bytes(addr), ()) if (tag_mask >> self.d[k]) & 1 and stake_ok(k, self.d[k])]
        pay = np.frombuffer(b''.join(self.p[k] for k in hits), dtype=PAYLOAD_DTYPE)
        return pack_records(hits, [self.d[k] for k in hits]), pay

    @staticmethod
    def _addr(raw: Optional[bytes]) -> bytes:
        if not raw:
            return b''
        n = int.from_bytes(raw[8:12], 'little')
        return raw[16:16 + n]

    def records_payload(self):
        keys = list(self.d.keys())
        pay = np.frombuffer(b''.join(self.p.get(k, bytes(80)) for k in keys), dtype=PAYLOAD_DTYPE)
        return pack_records(keys, [self.d[k] for k in keys]), pay

    def __len__(self):
        return len(self.d)


class _NativeHostBackend:
    """The host table in C++ (csrc/utxo_host.cpp ``HostUtxo``): the HBM table's record contract — keys
    (txid, index & 0xff), tag-filtered erase, zero payload when absent, an owner-address index for K14 — as
    one call per batch of packed records, so the CPU block path never walks its outpoints in Python."""

    def __init__(self):
        from ..ops.native import lib
        self.L = lib()
        self.t = self.L.HostUtxo()

    def reset(self, keys, tags, payload=None):
        self.t.clear()
        return self.insert(keys, tags, payload)

    def insert(self, keys, tags, payload=None) -> int:
        if not len(keys):
            return 0
        return self.insert_records(pack_records(keys, list(tags)), payload)

    def insert_records(self, recs: np.ndarray, payload=None) -> int:
        if not len(recs):
            return 0
        pay = None if payload is None else np.ascontiguousarray(payload).view(np.uint8)
        return int(self.t.insert(np.ascontiguousarray(recs), pay))

    def lookup_records(self, recs: np.ndarray):
        tags, pay = self.t.lookup(np.ascontiguousarray(recs))
        return tags, pay.view(PAYLOAD_DTYPE)

    def lookup(self, keys):
        if not len(keys):
            return np.zeros(0, dtype=np.uint8), np.zeros(0, dtype=PAYLOAD_DTYPE)
        return self.lookup_records(pack_records(keys))

    def probe_records(self, recs: np.ndarray) -> np.ndarray:
        return self.t.probe(np.ascontiguousarray(recs))

    def probe(self, keys) -> np.ndarray:
        if not len(keys):
            return np.zeros(0, dtype=np.uint8)
        return self.probe_records(pack_records(keys))

    def erase_records(self, recs: np.ndarray) -> np.ndarray:
        if not len(recs):
            return np.zeros(0, dtype=np.uint8)
        return self.t.erase(np.ascontiguousarray(recs))

    def erase(self, keys, tag=None) -> np.ndarray:
        if not len(keys):
            return np.zeros(0, dtype=np.uint8)
        return self.erase_records(pack_records(keys, MISSING if tag is None else tag))

    def records(self) -> np.ndarray:
        return self.t.dump(False)[0].reshape(-1, 40)

    def records_payload(self):
        raw, pay = self.t.dump(True)
        return raw.reshape(-1, 40), pay.view(PAYLOAD_DTYPE)

    def address_scan(self, addr: bytes, tag_mask: int, stake_sel: int = STAKE_ANY):
        raw, pay = self.t.address_scan(bytes(addr), tag_mask, stake_sel)
        return raw.reshape(-1, 40), pay.view(PAYLOAD_DTYPE)

    def __len__(self):
        return len(self.t)


class _GpuBackend:
    """HBM table; grows (rehash via dump + re-insert) past 50 % load."""

    def __init__(self, log2_cap: int = 20):
        from ..ops.native import require_gpu
        self.L = require_gpu()
        self.log2 = log2_cap
        self.h = self.L.utxo_create(log2_cap)
        self.count = 0
        self.tombs = 0
        self.pending = None  # (inserts, erases) of an async block apply not yet booked

    def __del__(self):
        try:
            self.L.utxo_destroy(self.h)
        except Exception:
            pass

    def apply_async(self, ins: Sequence[Tuple[np.ndarray, Optional[np.ndarray]]], dels: np.ndarray) -> int:
        """One committed block's inserts (groups of records + payloads) then erases, queued on the node
        stream without waiting (csrc/utxo_table.hip utxo_apply_async); every later pass on the table runs
        behind them. The counters are booked by :meth:`complete` (the caller's next access). Returns the
        previous apply's duplicates."""
        dups = self.complete()
        n_ins = sum(len(r) for r, _ in ins)
        self._ensure(n_ins)
        groups = [(np.ascontiguousarray(r), None if p is None else np.ascontiguousarray(p).view(np.uint8))
                  for r, p in ins]
        self.L.utxo_apply_async(self.h, groups, np.ascontiguousarray(dels))
        self.pending = (n_ins, len(dels))
        return dups

    def complete(self) -> int:
        """Book the pending async apply's counters (waits for it): returns its duplicates."""
        if self.pending is None:
            return 0
        n_ins, _ = self.pending
        self.pending = None
        _, failed, dups, erased = self.L.utxo_apply_wait(self.h)
        if failed:
            raise RuntimeError(f'UTXO table insert failed for {failed} entries')
        self.count += n_ins - dups - erased
        self.tombs += erased
        return dups

    def _ensure(self, extra: int):
        """Past 50 % load (live entries + tombstones + the coming inserts) the table is rebuilt on the device
        (``utxo_rehash``): at the same size when dropping the tombstones is enough, else grown. The set never
        leaves HBM (the dump + host re-insert this replaced moved it over PCIe twice, a ~50 ms stall per
        rebuild on a 5 M-outpoint set, every ~30 blocks of 2 MB)."""
        need = self.count + self.tombs + extra
        if need * 2 <= (1 << self.log2):
            return
        log2 = self.log2
        # headroom: after the rebuild the live set and the coming inserts fill at most a third of the table,
        # so tombstones have room to accumulate before the next one
        while (self.count + extra) * 3 > (1 << log2):
            log2 += 1
        moved, failed = self.L.utxo_rehash(self.h, log2)
        if failed or moved != self.count:
            raise RuntimeError(f'UTXO table rehash moved {moved} of {self.count} entries ({failed} found no slot)')
        self.log2, self.tombs = log2, 0

    def reset(self, keys, tags, payload=None):
        self.L.utxo_destroy(self.h)
        self.log2 = int(np.ceil(np.log2(max(2 * len(keys), 1 << 20))))
        self.h = self.L.utxo_create(self.log2)
        self.count = self.tombs = 0
        self.insert(keys, tags, payload)

    def insert(self, keys, tags, payload=None):
        if not len(keys):
            return 0
        return self.insert_records(pack_records(keys, list(tags)), payload)

    def insert_records(self, recs: np.ndarray, payload=None):
        if not len(recs):
            return
        self._ensure(len(recs))
        pay = None if payload is None else np.ascontiguousarray(payload).view(np.uint8)
        failed, dups = self.L.utxo_insert(self.h, np.ascontiguousarray(recs), pay)
        if failed:
            raise RuntimeError(f'UTXO table insert failed for {failed} entries')
        self.count += len(recs) - dups
        return dups

    def lookup_records(self, recs: np.ndarray):
        tags, pay = self.L.utxo_lookup(self.h, np.ascontiguousarray(recs))
        return np.frombuffer(tags, dtype=np.uint8), np.frombuffer(pay, dtype=PAYLOAD_DTYPE)

    def lookup(self, keys):
        if not len(keys):
            return np.zeros(0, dtype=np.uint8), np.zeros(0, dtype=PAYLOAD_DTYPE)
        return self.lookup_records(pack_records(keys))

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

    def address_scan(self, addr: bytes, tag_mask: int, stake_sel: int = STAKE_ANY):
        raw, pay, _total = self.L.utxo_address_scan(self.h, addr, tag_mask, stake_sel)
        return np.frombuffer(raw, dtype=np.uint8).reshape(-1, 40), np.frombuffer(pay, dtype=PAYLOAD_DTYPE)

    def records_payload(self):
        raw, pay = self.L.utxo_dump_payload(self.h)
        return np.frombuffer(raw, dtype=np.uint8).reshape(-1, 40), np.frombuffer(pay, dtype=PAYLOAD_DTYPE)

    def __len__(self):
        return self.count


def _host_backend(name: str):
    """``host``: the C++ table when the extension is built, else the dict; ``host-py``: the dict."""
    if name != 'host-py':
        try:
            from ..ops.native import lib
            if hasattr(lib(), 'HostUtxo'):
                return _NativeHostBackend()
        except Exception:
            pass
    return _HostBackend()


def default_backend() -> str:
    env = os.environ.get('UPOW_UTXO_BACKEND')
    if env:
        return env
    from ..ops.native import gpu_available
    try:
        return 'gpu' if gpu_available() else 'host'
    except Exception:
        return 'host'


# UPOW_UTXO_ASYNC=0: the block path's index update as synchronous insert + erase calls (A/B)
ASYNC_APPLY = os.environ.get('UPOW_UTXO_ASYNC', '1') != '0'


def _locked(fn):
    """Run under the index lock, after any deferred writes (:meth:`UtxoIndex.defer_block`) reached the
    backend: every read and every direct write sees the index as the committed blocks left it."""
    @functools.wraps(fn)
    def wrapper(self, *args, **kwargs):
        with self.lock:
            if self._pend_ins or self._pend_del:
                self._apply_pending()
            if self._gpu and self.be.pending is not None:
                self._dups(self.be.complete())
            return fn(self, *args, **kwargs)
    return wrapper


class UtxoIndex:
    def __init__(self, backend: Optional[str] = None):
        import threading
        self.lock = threading.RLock()
        self.backend_name = backend or default_backend()
        self.be = _GpuBackend() if self.backend_name == 'gpu' else _host_backend(self.backend_name)
        self._gpu = isinstance(self.be, _GpuBackend)
        self._rec = self._gpu or isinstance(self.be, _NativeHostBackend)  # packed records in, no Python walk
        self.duplicates = 0  # inserts of an outpoint that was already live (skipped; a ledger bug if ever > 0)
        # deferred writes of committed blocks (a sync page's blocks, ledger/pagesync.py): applied as ONE insert
        # launch and ONE erase launch before anything else touches the index
        self._pend_ins: List[Tuple[np.ndarray, Optional[np.ndarray]]] = []
        self._pend_del: List[np.ndarray] = []
        self.deferred_flushes = 0

    def defer_block(self, ins: Sequence[Tuple[np.ndarray, Optional[np.ndarray]]], spent: np.ndarray):
        """Record one committed block's index writes (created-output records + payloads, spent records)
        without touching the backend. Applying every deferred insert, then every deferred erase, equals
        applying the blocks in order: an outpoint is created at most once, spent at most once, and only
        after its creation (the page plan checks both before a block takes this path)."""
        with self.lock:
            for recs, pay in ins:
                if len(recs):
                    self._pend_ins.append((recs, pay))
            if len(spent):
                self._pend_del.append(spent)

    def settle(self):
        """Apply the deferred writes now and book any async apply (no-op when there is neither)."""
        with self.lock:
            if self._pend_ins or self._pend_del:
                self._apply_pending()
            if self._gpu and self.be.pending is not None:
                self._dups(self.be.complete())

    def apply_block(self, ins: Sequence[Tuple[np.ndarray, Optional[np.ndarray]]], spent: np.ndarray):
        """The block path's index update after the commit point: the block's created outputs (records +
        payloads, one or more groups) in, then its spent records out. GPU backend: one H2D copy, one insert
        and one erase launch queued on the node stream, no wait (``_GpuBackend.apply_async``): the next
        block's lookup is queued behind them, and its counters are booked at the next access."""
        with self.lock:
            if self._pend_ins or self._pend_del:
                self._apply_pending()
            self._apply(list(ins), [spent] if len(spent) else [])

    def _apply(self, ins, dels):
        ins = [(r, p) for r, p in ins if len(r)]
        if ins and any(p is None for _, p in ins):  # payloads for every group or for none
            ins = [(r, None) for r, _ in ins]
        spent = np.ascontiguousarray(np.concatenate(dels)) if len(dels) > 1 else \
            (np.ascontiguousarray(dels[0]) if dels else np.zeros((0, 40), np.uint8))
        if self._gpu and ASYNC_APPLY:
            if ins or len(spent):
                self._dups(self.be.apply_async(ins, spent))
            return
        recs = np.ascontiguousarray(np.concatenate([r for r, _ in ins])) if ins else np.zeros((0, 40), np.uint8)
        pay = None if (not ins or ins[0][1] is None) else np.ascontiguousarray(np.concatenate([p for _, p in ins]))
        if len(recs):
            self._insert_records(recs, pay)
        if len(spent):
            self._erase_records(spent)

    def _apply_pending(self):
        ins, dels = self._pend_ins, self._pend_del
        self._pend_ins, self._pend_del = [], []
        self.deferred_flushes += 1
        self._apply(ins, dels)

    def _dups(self, n: int):
        if n:
            self.duplicates += int(n)
            import logging
            logging.getLogger('upow').error(f'UTXO index: {n} insert(s) of an already live outpoint skipped')

    @_locked
    def reset(self, keys: Sequence[Outpoint], tags: Sequence[int], payload: Optional[np.ndarray] = None):
        self.be.reset(list(keys), list(tags), payload)

    @_locked
    def insert(self, keys: Sequence[Outpoint], tag, payload: Optional[np.ndarray] = None):
        keys = list(keys)
        tags = [tag] * len(keys) if isinstance(tag, int) else list(tag)
        self._dups(self.be.insert(keys, tags, payload))

    @_locked
    def insert_records(self, recs: np.ndarray, payload: Optional[np.ndarray] = None):
        """Insert packed 40-byte key records (tags inside) — the block fast path's form."""
        self._insert_records(recs, payload)

    def _insert_records(self, recs: np.ndarray, payload: Optional[np.ndarray] = None):
        if self._rec:
            self._dups(self.be.insert_records(recs, payload))
            return
        idx = recs[:, 32:36].copy().view(np.uint32).ravel()
        tags = recs[:, 36:40].copy().view(np.uint32).ravel()
        keys = [(bytes(recs[n, :32]).hex(), int(idx[n])) for n in range(len(recs))]
        self._dups(self.be.insert(keys, [int(t) for t in tags], payload))

    @_locked
    def lookup(self, keys: Sequence[Outpoint]):
        """(tags uint8[n], payload PAYLOAD_DTYPE[n]) for each outpoint (tag 0xff / len 0 when absent)."""
        return self.be.lookup(list(keys))

    @_locked
    def lookup_records(self, recs: np.ndarray):
        if self._rec:
            return self.be.lookup_records(recs)
        idx = recs[:, 32:36].copy().view(np.uint32).ravel()
        return self.be.lookup([(bytes(recs[n, :32]).hex(), int(idx[n])) for n in range(len(recs))])

    @_locked
    def erase_records(self, recs: np.ndarray) -> np.ndarray:
        return self._erase_records(recs)

    def _erase_records(self, recs: np.ndarray) -> np.ndarray:
        if isinstance(self.be, _GpuBackend):
            if not len(recs):
                return np.zeros(0, dtype=np.uint8)
            out = np.frombuffer(self.be.L.utxo_erase(self.be.h, np.ascontiguousarray(recs)), dtype=np.uint8)
            k = int(out.sum())
            self.be.count -= k
            self.be.tombs += k
            return out
        if self._rec:
            return self.be.erase_records(recs)
        if not len(recs):
            return np.zeros(0, dtype=np.uint8)
        idx = recs[:, 32:36].copy().view(np.uint32).ravel()
        tags = recs[:, 36:40].copy().view(np.uint32).ravel()
        keys = [(bytes(recs[n, :32]).hex(), int(idx[n])) for n in range(len(recs))]
        out = np.zeros(len(recs), dtype=np.uint8)
        for tag in np.unique(tags).tolist():  # per-record tag filter, like the HBM erase kernel
            sel = np.nonzero(tags == tag)[0]
            out[sel] = self.be.erase([keys[k] for k in sel.tolist()], None if tag == MISSING else int(tag))
        return out

    @_locked
    def probe(self, keys: Sequence[Outpoint]) -> np.ndarray:
        return self.be.probe(list(keys))

    @_locked
    def erase(self, keys: Sequence[Outpoint], tag: Optional[int] = None) -> np.ndarray:
        return self.be.erase(list(keys), tag)

    @_locked
    def filter(self, outputs: Iterable[Outpoint], tag: int) -> List[Outpoint]:
        """Outpoints of ``outputs`` present in table ``tag`` (unique, in first-seen order)."""
        uniq = list(dict.fromkeys((h, int(i)) for h, i in outputs))
        if not uniq:
            return []
        t = self.probe(uniq)
        return [k for k, v in zip(uniq, t) if v == tag]

    @_locked
    def records(self) -> np.ndarray:
        """All live entries as 40-byte records, in canonical (txid, index) order."""
        return sort_records(np.ascontiguousarray(self.be.records()))

    @_locked
    def address_outputs(self, addr: bytes, tags: Iterable[int] = (0,), stake_sel: int = STAKE_ANY):
        """K14 (reference ``database.py:909-937,1138-1205``): the live outpoints whose payload address is
        ``addr`` (raw 33/64 bytes, prefix normalised as stored) in the given tables, as (records, payloads)
        in canonical (txid, index) order, plus their amount sum in smallest units. GPU backend: one
        ``utxo_address_scan`` launch over the HBM table instead of an index walk."""
        mask = 0
        for t in tags:
            mask |= 1 << int(t)
        recs, pay = self.be.address_scan(bytes(addr), mask, stake_sel)
        order = sort_order(np.ascontiguousarray(recs))
        recs, pay = np.ascontiguousarray(recs[order]), np.ascontiguousarray(pay[order])
        return recs, pay, int(pay['amount'].sum()) if len(pay) else 0

    @_locked
    def records_payload(self, sort: bool = True):
        """(records, payloads) of every live entry, in canonical (txid, index) order (``sort=False``: in the
        backend's own order, for a caller that sorts later off the ledger's critical path)."""
        recs, pay = self.be.records_payload()
        if not sort:
            return recs, pay
        order = sort_order(np.ascontiguousarray(recs))
        return np.ascontiguousarray(recs[order]), np.ascontiguousarray(pay[order])

    @_locked
    def reset_records(self, recs: np.ndarray, payload: Optional[np.ndarray] = None):
        """Replace the whole index with packed records (snapshot restore: one H2D copy + insert launch)."""
        recs = np.ascontiguousarray(recs, dtype=np.uint8).reshape(-1, 40)
        if self._rec:
            self.be.reset([], [])
            if len(recs):
                self.be.insert_records(recs, payload)
        else:
            idx = recs[:, 32:36].copy().view(np.uint32).ravel()
            tags = recs[:, 36:40].copy().view(np.uint32).ravel()
            keys = [(bytes(recs[n, :32]).hex(), int(idx[n])) for n in range(len(recs))]
            self.be.reset(keys, [int(t) for t in tags], payload)

    @_locked
    def block_inputs(self, in_keys: np.ndarray, in_start: np.ndarray, out_amount: np.ndarray,
                     out_start: np.ndarray, want_tag: int = 0):
        """One pass over a block's inputs: K7 lookup (tag + payload), K10 duplicate detection and K11
        per-tx fees. GPU backend: one H2D/D2H round trip and three kernels (csrc/utxo_table.hip).

        Returns (tags u8[n_in], payload[n_in], dup_of u32[n_in] (1 + earlier duplicate, else 0),
        fee i64[n_tx], missing u32[n_tx], n_dup)."""
        in_start = np.ascontiguousarray(in_start, dtype=np.int32)
        out_start = np.ascontiguousarray(out_start, dtype=np.int32)
        out_amount = np.ascontiguousarray(out_amount, dtype=np.uint64)
        if isinstance(self.be, _GpuBackend):
            # the segment arrays are read in place; the outputs are arrays the pass filled from its pinned staging
            t, p, d, f, m, nd = self.be.L.utxo_block_inputs(self.be.h, np.ascontiguousarray(in_keys), in_start,
                                                            out_amount, out_start, want_tag)
            return t, p.view(PAYLOAD_DTYPE), d, f, m, int(nd)
        tags, pay = self.lookup_records(in_keys)
        n_in = len(in_keys)
        dup_of = np.zeros(n_in, dtype=np.uint32)
        if n_in > 1:  # K10: (txid, index byte) seen earlier in the block -> 1 + the first occurrence
            k = np.ascontiguousarray(in_keys[:, :33]).view(np.dtype((np.void, 33))).ravel()
            _, first, inv = np.unique(k, return_index=True, return_inverse=True)
            first = first[inv.ravel()]
            later = first != np.arange(n_in)
            dup_of[later] = first[later] + 1
        bad = ((tags != want_tag) | (pay['len'] == 0)).astype(np.int64)
        amt = pay['amount'].astype(np.int64)

        def seg_sum(x, starts):  # per-tx sums over contiguous segments (empty segments -> 0)
            cs = np.concatenate([[0], np.cumsum(x, dtype=np.int64)])
            return cs[starts[1:]] - cs[starts[:-1]]
        ins = seg_sum(amt, in_start)
        outs = seg_sum(out_amount.astype(np.int64), out_start)
        miss = seg_sum(bad, in_start).astype(np.uint32)
        return tags, pay, dup_of, ins - outs, miss, int((dup_of > 0).sum())

    @_locked
    def set_message(self, tag: int = 0) -> np.ndarray:
        """K12's message: (txid || index byte) of every outpoint of table ``tag`` sorted by (txid, index).
        GPU backend: compaction + stable LSD radix sort + message gather on the device."""
        if isinstance(self.be, _GpuBackend):
            return self.be.L.utxo_set_message(self.be.h, tag)
        recs = self.records()
        recs = recs[recs[:, 36:40].copy().view(np.uint32).ravel() == tag]
        # records() is in canonical (txid, index) order; index byte = the reference's bytes([i])
        return np.ascontiguousarray(np.concatenate([recs[:, :32], recs[:, 32:33]], axis=1)).ravel()

    def k12_snapshot(self, tag: int = 0):
        """K12 at this block, computed later: returns a callable giving the hex digest (the same value
        :meth:`set_hash` gives now). GPU backend: the snapshot is one compaction launch on the node stream;
        the callable (meant for a worker thread) sorts, gathers and hashes on the aux stream."""
        with self.lock:
            if self._pend_ins or self._pend_del:
                self._apply_pending()
            if isinstance(self.be, _GpuBackend):  # queued behind any async apply on the node stream
                L, sid = self.be.L, self.be.L.utxo_k12_snapshot(self.be.h, tag)
                return lambda: L.utxo_k12_digest(sid)[0].hex()
        msg = self.set_message(tag)
        import hashlib
        return lambda: hashlib.sha256(msg).hexdigest()

    def set_hash(self, tag: int = 0) -> str:
        """K12 from the index: SHA-256 over :meth:`set_message` — byte-identical to
        ``Database.get_unspent_outputs_hash`` (reference database.py:827-830). The sequential hash tail
        runs outside the index lock (hashlib releases the GIL), so block application is not held up by it."""
        import hashlib
        return hashlib.sha256(self.set_message(tag)).hexdigest()

    def __len__(self):
        self.settle()
        return len(self.be)


def sort_order(recs: np.ndarray) -> np.ndarray:
    """Permutation sorting packed records by (txid bytes, index): SQL ``ORDER BY tx_hash, index``."""
    if len(recs) < 2:
        return np.arange(len(recs))
    be = recs[:, :32].copy().view('>u8')  # 4 big-endian words compare like the hex strings
    idx = recs[:, 32:36].copy().view(np.uint32).ravel()
    return np.lexsort((idx, be[:, 3], be[:, 2], be[:, 1], be[:, 0]))


def sort_records(recs: np.ndarray) -> np.ndarray:
    return recs[sort_order(recs)] if len(recs) >= 2 else recs
