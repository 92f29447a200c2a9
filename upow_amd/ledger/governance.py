"""Indexed governance state: stakes, registrations, voting power and ballots held in memory.

reference: every governance aggregate is recomputed from PostgreSQL on each call —
``get_active_inodes`` (upow/database.py:1377-1388) walks every registered inode →
``get_inode_vote_ratio_by_address`` (1390-1418) → per ballot ``get_validators_stake`` (1127-1136) →
per delegate ballot ``get_address_stake`` (1189-1205), and each ``check_pending_txs`` variant re-reads and
re-parses the mempool (1189-1290). ``create_block`` runs that cascade for every block (manager.py:650-757).

Here the rows of the six governance tables and the staked outputs of ``unspent_outputs`` live in a native
store (csrc/gov_index.cpp ``GovStore``) that follows every write to those tables (both block paths,
rollback): each row keeps what the reference's joins read — its address column, the amount
(``transactions.outputs_amounts[index]``), the voter (``transactions.inputs_addresses[index]``) and the
block timestamp — in insertion (= rowid) order, indexed by address string, by voter string and by the
point an address denotes. The emission cascade (delegate stake → validator stake → inode power) is kept
there as exact decimal running sums updated along the dependency edges of each row change, bit-identical
to the reference's sequential ``Decimal`` sums (value and exponent); a sum that cannot be kept exactly is
recomputed here the reference's way. The block path's governance rules run in the store too
(ledger/govcheck.py). This class is the Python face: the reference's query shapes over the store, and the
mempool overlay of the ``check_pending_txs`` variants (pending-spent outpoints, pending stake outputs per
address), rebuilt once per mempool version with each pending tx parsed once.
"""
from __future__ import annotations

import functools
import threading
from decimal import Decimal
from typing import Dict, Iterable, List, Optional, Set, Tuple

from ..constants import SMALLEST
from ..utils.codec import round_up_decimal

GOV_TABLES = ('inode_registration_output', 'validator_registration_output', 'validators_voting_power',
              'delegates_voting_power', 'validators_ballot', 'inodes_ballot')
STAKE = 'stake'  # staked rows of unspent_outputs (is_stake = 1)
Key = Tuple[str, int]


_FORMS: Dict[str, List[str]] = {}


def _forms(address: str) -> List[str]:
    """Both string forms of an address (codec.address_forms: a point decompression + two encodings),
    memoised: an aggregate recomputation asks for every voter's forms."""
    hit = _FORMS.get(address)
    if hit is None:
        from ..utils.codec import address_forms
        if len(_FORMS) > (1 << 20):
            _FORMS.clear()
        hit = _FORMS[address] = address_forms(address)
    return hit


def _at(arr, i):
    return arr[i] if arr is not None and 0 <= i < len(arr) else None


def point_key(raw: bytes) -> Optional[bytes]:
    """The point an address denotes, as its normalised 33-byte compressed encoding — without a square
    root: a 33-byte address keeps x with prefix 43 (odd y) or 42, a 64-byte one (x LE || y LE) takes the
    parity of y. Two address strings are in each other's ``address_forms`` exactly when their keys match."""
    if len(raw) == 33:
        return bytes([43 if raw[0] == 43 else 42]) + bytes(raw[1:])
    if len(raw) == 64:
        return bytes([43 if raw[32] & 1 else 42]) + bytes(raw[:32])
    return None


_PT: Dict[str, Optional[bytes]] = {}


def point_key_of(address: Optional[str]) -> Optional[bytes]:
    """point_key of an address string (string_to_bytes semantics: hex first, then base58), memoised."""
    if address is None:
        return None
    hit = _PT.get(address, b'')
    if hit != b'':
        return hit
    from ..utils.codec import string_to_bytes
    try:
        hit = point_key(string_to_bytes(address))
    except Exception:
        hit = None
    if len(_PT) > (1 << 20):
        _PT.clear()
    _PT[address] = hit
    return hit


TID = {t: k for k, t in enumerate(GOV_TABLES)}
TID[STAKE] = len(GOV_TABLES)


def _k36(key: Key) -> bytes:
    return bytes.fromhex(key[0]) + int(key[1]).to_bytes(4, 'little')


def _kpy(raw: bytes) -> Key:
    return raw[:32].hex(), int.from_bytes(raw[32:36], 'little')


def _row_args(key: Key, address, amount, voter, ts) -> tuple:
    return _k36(key), address, amount, voter, ts, point_key_of(address), point_key_of(voter)


def _dec(t) -> Optional[Decimal]:
    return None if t is None else Decimal(t)


class _TableView:
    """One table of the native store, with the dict-shaped accessors tests and tools use."""

    def __init__(self, gov: 'GovernanceIndex', name: str):
        self.gov, self.name, self.tid = gov, name, TID[name]

    @property
    def rows(self) -> Dict[Key, tuple]:
        """key -> (address, amount, voter, ts), in insertion (rowid) order."""
        return {_kpy(r[0]): (r[1], r[2], r[3], r[4]) for r in self.gov.store.rows(self.tid)}

    def __len__(self):
        return self.gov.store.count(self.tid)

    def add(self, key: Key, address, amount, voter, ts):
        self.gov.store.add_rows(self.tid, [_row_args(key, address, amount, voter, ts)])

    def remove(self, key: Key) -> bool:
        return self.gov.store.remove_keys(self.tid, _k36(key)) > 0


class _GovLock:
    """The index lock, aware of a deferred block apply (:meth:`GovernanceIndex.defer`): every acquirer
    outside the apply thread first waits for the last block's apply to finish (re-raising its error), so
    no reader ever sees the index between a block's commit and its governance update."""

    def __init__(self):
        self._lock = threading.RLock()
        self.job = None  # Future of the last deferred apply
        self.worker_ident = None

    def settle(self):
        job = self.job
        if job is not None and threading.get_ident() != self.worker_ident:
            job.result()

    def acquire(self, blocking: bool = True, timeout: float = -1) -> bool:
        self.settle()
        return self._lock.acquire(blocking, timeout)

    def release(self):
        self._lock.release()

    def __enter__(self):
        self.acquire()
        return self

    def __exit__(self, *exc):
        self._lock.release()
        return False


_APPLY_POOL = None


def _locked(fn):
    """Serialise index access: block application (ledger thread) and API queries (HTTP loop) share it."""
    @functools.wraps(fn)
    def wrapper(self, *args, **kwargs):
        with self.lock:
            return fn(self, *args, **kwargs)
    return wrapper


class GovernanceIndex:
    def __init__(self, db):
        from ..ops.native import lib
        self.db = db
        self.lock = _GovLock()
        self.store = lib().GovStore()
        self.tables: Dict[str, _TableView] = {t: _TableView(self, t) for t in (*GOV_TABLES, STAKE)}
        self.version = 0
        self._memo: dict = {}
        self._memo_version = -1
        self._pending = None  # (mempool version, pending-spent set, pending stake per address, pending votes)
        self._parsed: Dict[str, tuple] = {}  # pending tx hash -> (stake outputs, is a delegate vote)
        self._blob = None  # (overlay, pending-spent keys as 36-byte records)

    def defer(self, fn):
        """Run ``fn`` (a block's index update) on the governance apply thread, under the index lock. The
        block path moves on at once (the next block's decode, UTXO pass and signatures do not read the
        index); every later acquirer of the lock waits for it first."""
        global _APPLY_POOL
        from concurrent.futures import ThreadPoolExecutor
        if _APPLY_POOL is None:
            _APPLY_POOL = ThreadPoolExecutor(max_workers=1, thread_name_prefix='upow-gov-apply')
        self.lock.settle()  # one deferred apply at a time, in block order

        def run():
            self.lock.worker_ident = threading.get_ident()
            with self.lock._lock:
                fn()
        self.lock.job = _APPLY_POOL.submit(run)

    # ------------------------------------------------------------------ maintenance
    def _rows_sql(self, table: str, where: str = '', args: tuple = ()):
        src = 'unspent_outputs' if table == STAKE else table
        cond = ['u.is_stake = 1'] if table == STAKE else []
        if where:
            cond.append(where)
        w = ('WHERE ' + ' AND '.join(cond)) if cond else ''
        txq = self.db._txq  # correlated lookups: pushed into each file of a split transactions table
        rows = self.db._q(f'SELECT u.tx_hash, u."index", u.address, {txq("outputs_amounts", "u.tx_hash")}, '
                          f'{txq("inputs_addresses", "u.tx_hash")}, (SELECT b.timestamp FROM blocks b WHERE b.hash = '
                          f'{txq("block_hash", "u.tx_hash")}), {txq("rowid", "u.tx_hash")} FROM {src} u {w} ORDER BY u.rowid',
                          args)
        return [r[:6] for r in rows if r[6] is not None]  # (INNER JOIN transactions)

    def _add_sql_rows(self, table: str, rows, only: Optional[Set[Key]] = None):
        import json
        batch = []
        for h, i, address, am, ia, ts in rows:
            key = (h, int(i))
            if only is not None and key not in only:
                continue
            amount = _at(json.loads(am) if am else [], int(i))
            voter = _at(json.loads(ia) if ia else [], int(i))
            batch.append(_row_args(key, address, amount, voter, ts))
        if batch:
            self.store.add_rows(TID[table], batch)

    @_locked
    def rebuild(self):
        self.store.clear()
        for t in self.tables:
            self._add_sql_rows(t, self._rows_sql(t))
        self.store.build()
        self.version += 1

    @_locked
    def added(self, table: str, keys: List[Key]):
        """Rows just inserted into ``table`` (or staked outputs into unspent_outputs): mirror them
        with the same joins the reference's queries use."""
        if not keys:
            return
        want = {(h, int(i)) for h, i in keys}
        hashes = sorted({h for h, _ in want})
        for k in range(0, len(hashes), 500):
            chunk = hashes[k:k + 500]
            self._add_sql_rows(table, self._rows_sql(table, f'u.tx_hash IN ({",".join("?" * len(chunk))})',
                                                     tuple(chunk)), want)
        self.version += 1

    @_locked
    def removed(self, table: str, keys: Iterable[Key]):
        if self.store.remove_keys(TID[table], b''.join(_k36(k) for k in keys)):
            self.version += 1

    @_locked
    def stake_keys(self) -> Dict[Key, tuple]:
        return self.tables[STAKE].rows

    # ------------------------------------------------------------------ mempool overlay
    @_locked
    def _overlay(self):
        ver = self.db._mempool_ver
        if self._pending is not None and self._pending[0] == ver:
            return self._pending
        from ..models.transaction import Transaction
        from ..utils.codec import TransactionType
        spent = {(r[0], r[1]) for r in self.db._q('SELECT tx_hash, "index" FROM pending_spent_outputs')}
        stake: Dict[str, Decimal] = {}
        live = {}
        votes = 0  # pending VOTE_AS_DELEGATE txs (the unstake rule consults them, transaction.py:474-477)
        for h, tx_hex in self.db._q('SELECT tx_hash, tx_hex FROM pending_transactions ORDER BY rowid'):
            hit = self._parsed.get(h)
            if hit is None:
                tx = Transaction.parse(tx_hex)[0]
                hit = ([(o.address, o.amount) for o in tx.outputs if o.is_stake is True],
                       getattr(tx, 'transaction_type', None) == TransactionType.VOTE_AS_DELEGATE)
            live[h] = hit
            votes += hit[1]
            for address, amount in hit[0]:
                stake[address] = stake.get(address, Decimal(0)) + amount
        self._parsed = live
        self._pending = (ver, spent, stake, votes)
        return self._pending

    @_locked
    def pending_vote_as_delegate(self) -> int:
        return self._overlay()[3]

    @_locked
    def pending_blob(self) -> bytes:
        """The pending-spent outpoints as concatenated 36-byte keys (the native rule check's form)."""
        ov = self._overlay()
        if self._blob is None or self._blob[0] is not ov:
            self._blob = (ov, b''.join(_k36(k) for k in ov[1]))
        return self._blob[1]

    @_locked
    def has_point(self, table: str, pt: Optional[bytes], check_pending: bool, voter: bool = False) -> bool:
        """Is there a live row of ``table`` whose address (``voter``: voter) denotes point ``pt``?"""
        keys = self.store.keys_by_point(TID[table], pt, voter)
        if not keys:
            return False
        if not check_pending:
            return True
        pend = self.pending_spent(True)
        return any(_kpy(keys[o:o + 36]) not in pend for o in range(0, len(keys), 36))

    @_locked
    def pending_spent(self, check_pending: bool) -> Set[Key]:
        return self._overlay()[1] if check_pending else set()

    # ------------------------------------------------------------------ queries (reference semantics)
    @_locked
    def amount_rows(self, table: str, forms: List[str], check_pending: bool) -> List[Tuple[str, int, object]]:
        """``_amount_rows``: (tx_hash, index, amount) of rows whose address is in ``forms``, rowid order."""
        pend = self.pending_spent(check_pending)
        out = []
        for r in self.store.rows_by(TID[table], list(forms), False):
            k = _kpy(r[0])
            if k not in pend:
                out.append((k[0], k[1], r[2]))
        return out

    @_locked
    def address_rows(self, table: str, forms: List[str], check_pending: bool) -> List[tuple]:
        """(tx_hash, index, amount, address) of rows whose address is in ``forms``, rowid order."""
        pend = self.pending_spent(check_pending)
        out = []
        for r in self.store.rows_by(TID[table], list(forms), False):
            k = _kpy(r[0])
            if k not in pend:
                out.append((k[0], k[1], r[2], r[1]))
        return out

    @_locked
    def ballot_rows(self, table: str, receiver_forms: Optional[List[str]], check_pending: bool,
                    voter_forms: Optional[Set[str]] = None, order: bool = True):
        """``_ballot_rows``: (tx_hash, receiver, vote, voter, index), ordered by (tx_hash, rowid) or rowid."""
        tid = TID[table]
        rows = self.store.rows(tid) if receiver_forms is None else self.store.rows_by(tid, list(receiver_forms), False)
        if order:
            rows.sort(key=lambda r: r[0][:32])  # stable: rowid order within a tx hash
        pend = self.pending_spent(check_pending)
        out = []
        for raw, address, amount, voter, _ in rows:
            k = _kpy(raw)
            if k in pend:
                continue
            if voter_forms is not None and voter not in voter_forms:
                continue
            out.append((k[0], address, Decimal(amount) / SMALLEST if amount is not None else None, voter, k[1]))
        return out

    @_locked
    def spent_votes(self, table: str, voter_forms: Set[str], check_pending: bool):
        pend = self.pending_spent(check_pending)
        out = []
        for r in self.store.rows_by(TID[table], list(voter_forms), True):
            k = _kpy(r[0])
            if k not in pend:
                out.append((k, r[2]))
        return out

    @_locked
    def registered_inodes(self, check_pending: bool):
        pend = self.pending_spent(check_pending)
        return [(r[1], r[4]) for r in self.store.rows(TID['inode_registration_output'])
                if r[4] is not None and _kpy(r[0]) not in pend]

    @_locked
    def inode_count(self, check_pending: bool) -> int:
        if not check_pending:
            return self.store.count(TID['inode_registration_output'])
        pend = self.pending_spent(True)
        return sum(1 for r in self.store.rows(TID['inode_registration_output']) if _kpy(r[0]) not in pend)

    @_locked
    def address_stake(self, forms: List[str], check_pending: bool) -> Decimal:
        pt = point_key_of(forms[0]) if forms else None
        if not check_pending and pt is not None:
            hit = _dec(self.store.stake(pt))
            if hit is not None:
                return hit
        stake = sum((Decimal(a) / SMALLEST for _, _, a in self.amount_rows(STAKE, forms, check_pending)), Decimal(0))
        if check_pending:
            pstake = self._overlay()[2]
            for f in forms:
                stake += pstake.get(f, Decimal(0))
        return stake

    def _memo_get(self, key, fn):
        if self._memo_version != self.version:
            self._memo = {}
            self._memo_version = self.version
        hit = self._memo.get(key)
        if hit is None:
            hit = self._memo[key] = fn()
        return hit

    @_locked
    def validators_stake(self, forms: List[str], check_pending: bool) -> Decimal:
        """get_validators_stake (database.py:1127-1136): sum of vote x delegate stake / 10 over the
        validator's delegate ballots."""
        def compute():
            ballot = self.ballot_rows('validators_ballot', forms, check_pending)
            ratio = [(vote * self.address_stake(_forms(delegate), False)) / 10
                     for _, _, vote, delegate, _ in ballot]
            return round_up_decimal(sum(ratio, Decimal(0)))
        if check_pending:
            return compute()
        pt = point_key_of(forms[0]) if forms else None
        hit = _dec(self.store.validator_stake(pt)) if pt is not None else None
        return hit if hit is not None else compute()

    @_locked
    def inode_power(self, forms: List[str], check_pending: bool) -> Decimal:
        """get_inode_vote_ratio_by_address (database.py:1390-1418)."""
        def compute():
            rows = self.ballot_rows('inodes_ballot', forms, check_pending, order=False)
            ratio = [(vote * self.validators_stake(_forms(validator), False)) / 10
                     for _, _, vote, validator, _ in rows]
            return round_up_decimal(sum(ratio, Decimal(0)))
        if check_pending:
            return compute()
        pt = point_key_of(forms[0]) if forms else None
        hit = _dec(self.store.inode_power(pt)) if pt is not None else None
        return hit if hit is not None else compute()

    @_locked
    def inodes_with_power(self, check_pending: bool):
        """get_all_registered_inode_with_vote: [(wallet, power, registration timestamp)]."""
        def compute():
            return [(address, self.inode_power(list(reversed(_forms(address))), check_pending), ts)
                    for address, ts in self.registered_inodes(check_pending)]
        if check_pending:
            return compute()
        return self._memo_get('inodes', compute)


__all__ = ['GovernanceIndex', 'GOV_TABLES', 'STAKE']
