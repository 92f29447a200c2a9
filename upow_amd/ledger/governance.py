"""Indexed governance state: stakes, registrations, voting power and ballots held in memory.

reference: every governance aggregate is recomputed from PostgreSQL on each call —
``get_active_inodes`` (upow/database.py:1377-1388) walks every registered inode →
``get_inode_vote_ratio_by_address`` (1390-1418) → per ballot ``get_validators_stake`` (1127-1136) →
per delegate ballot ``get_address_stake`` (1189-1205), and each ``check_pending_txs`` variant re-reads and
re-parses the mempool (1189-1290). ``create_block`` runs that cascade for every block (manager.py:650-757).

Here the rows of the six governance tables and the staked outputs of ``unspent_outputs`` live in an
index that follows every write to those tables (block apply through either block path, rollback by
rebuild). Each row keeps what the reference's joins read: its address column, the amount
(``transactions.outputs_amounts[index]``), the voter (``transactions.inputs_addresses[index]``) and, for
inode registrations, the block timestamp. Rows keep table (rowid) order: SQLite assigns a new row
``max(rowid) + 1``, so insertion order among live rows is rowid order.

Aggregates are memoised per index version (any governance write bumps it), so a block without
governance transactions costs O(1) here. The mempool overlay of the ``check_pending_txs`` variants
(pending-spent outpoints, pending stake outputs per address) is rebuilt once per mempool version, each
pending tx parsed once.
"""
from __future__ import annotations

import functools
import threading
from decimal import Context, Decimal, DivisionByZero, Inexact, InvalidOperation, Overflow, Rounded
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


class _Table:
    __slots__ = ('rows', 'seq', 'by_addr', 'by_voter', 'by_pt', 'by_voter_pt', 'next_seq', 'name', 'changed')

    def __init__(self, name: str = '', changed=None):
        self.name = name
        self.changed = changed  # callback(table, address point, voter point) on every add/remove
        self.rows: Dict[Key, tuple] = {}  # key -> (address, amount, voter, ts); insertion (rowid) order
        self.seq: Dict[Key, int] = {}  # key -> insertion sequence (sort key for rowid order)
        self.by_addr: Dict[Optional[str], Dict[Key, None]] = {}
        self.by_voter: Dict[Optional[str], Dict[Key, None]] = {}
        # by the point the address denotes (both string forms at once): the native block path's
        # governance checks ask "is this key registered / staked / voting" with raw address bytes
        self.by_pt: Dict[Optional[bytes], Dict[Key, None]] = {}
        self.by_voter_pt: Dict[Optional[bytes], Dict[Key, None]] = {}
        self.next_seq = 0

    def add(self, key: Key, address, amount, voter, ts):
        if key in self.rows:
            self.remove(key)
        self.rows[key] = (address, amount, voter, ts)
        self.seq[key] = self.next_seq
        self.next_seq += 1
        self.by_addr.setdefault(address, {})[key] = None
        self.by_voter.setdefault(voter, {})[key] = None
        pa, pv = point_key_of(address), point_key_of(voter)
        self.by_pt.setdefault(pa, {})[key] = None
        self.by_voter_pt.setdefault(pv, {})[key] = None
        if self.changed is not None:
            self.changed(self.name, key, self.rows[key], 1)

    def remove(self, key: Key) -> bool:
        row = self.rows.pop(key, None)
        if row is None:
            return False
        del self.seq[key]
        if self.changed is not None:
            self.changed(self.name, key, row, -1)
        for idx, k in ((self.by_addr, row[0]), (self.by_voter, row[2]), (self.by_pt, point_key_of(row[0])),
                       (self.by_voter_pt, point_key_of(row[2]))):
            d = idx.get(k)
            if d is not None:
                d.pop(key, None)
                if not d:
                    del idx[k]
        return True

    def keys_for(self, index, values: Iterable) -> List[Key]:
        """Keys of rows whose column is in ``values``, in table (rowid) order."""
        found: Dict[Key, None] = {}
        for v in values:
            for k in index.get(v, ()):
                found[k] = None
        if len(found) < 2:
            return list(found)
        return sorted(found, key=self.seq.__getitem__)


def _locked(fn):
    """Serialise index access: block application (ledger thread) and API queries (HTTP loop) share it."""
    @functools.wraps(fn)
    def wrapper(self, *args, **kwargs):
        with self.lock:
            return fn(self, *args, **kwargs)
    return wrapper


_EXACT = Context(prec=28, traps=[Inexact, Rounded, InvalidOperation, DivisionByZero, Overflow])


class _ExactSum:
    """``sum(terms, Decimal(0))`` maintained under additions and removals of terms. Exact decimal arithmetic
    (any rounding trips the trap and marks the sum unusable, so the caller recomputes sequentially); the
    result carries the exponent a sequential sum from ``Decimal(0)`` would have — min(0, term exponents) —
    so value AND representation match the reference's left-to-right sum."""
    __slots__ = ('value', 'exps', 'ok', 'cached')

    def __init__(self):
        self.value = Decimal(0)
        self.exps: Dict[int, int] = {}
        self.ok = True
        self.cached = None

    def update(self, term, sign: int):
        self.cached = None
        if not self.ok:
            return
        try:
            self.value = _EXACT.add(self.value, term) if sign > 0 else _EXACT.subtract(self.value, term)
            e = term.as_tuple().exponent
        except Exception:
            self.ok = False
            return
        n = self.exps.get(e, 0) + sign
        if n:
            self.exps[e] = n
        else:
            del self.exps[e]

    def result(self) -> Optional[Decimal]:
        if not self.ok:
            return None
        if self.cached is not None:
            return self.cached
        if not self.exps:
            return Decimal(0)
        try:
            self.cached = _EXACT.quantize(self.value, Decimal(1).scaleb(min(0, min(self.exps))))
        except Exception:
            return None
        return self.cached


class _Cascade:
    """The emission aggregates of get_active_inodes (database.py:1377-1426) as running sums:

      stake(D)       = sum over D's staked outputs of amount / SMALLEST                 (1189-1205)
      vstake(V)      = round_up(sum over ballots to V of vote * stake(voter) / 10)     (1127-1136)
      ipower(I)      = round_up(sum over ballots to I of vote * vstake(voter) / 10)    (1390-1418)

    keyed by the point an address denotes. A row change updates its own term and propagates only along
    its dependents (a stake change re-terms that delegate's ballots; a changed validator stake re-terms
    that validator's inode ballots). Each term is computed with the reference's expression, so values are
    bit-identical to the sequential recomputation; an entity whose sum cannot be kept exactly (or whose
    rows lack a vote or voter) answers None and the caller recomputes it the reference's way."""

    def __init__(self, gov: 'GovernanceIndex'):
        self.gov = gov
        self.build()

    def build(self):
        self.astake: Dict[Optional[bytes], _ExactSum] = {}
        self.vsum: Dict[Optional[bytes], _ExactSum] = {}
        self.isum: Dict[Optional[bytes], _ExactSum] = {}
        self.vterm: Dict[Key, tuple] = {}   # validators_ballot key -> (receiver pt, term)
        self.iterm: Dict[Key, tuple] = {}   # inodes_ballot key -> (receiver pt, term)
        self.vval: Dict[Optional[bytes], Decimal] = {}
        self.bad_v, self.bad_i = set(), set()
        self.pending_v: Set[Optional[bytes]] = set()  # validators whose stake may have changed (propagated lazily)
        t = self.gov.tables
        for k, row in t[STAKE].rows.items():
            self._stake_row(row, 1, propagate=False)
        for k, row in t['validators_ballot'].rows.items():
            self._vballot(k, row, 1, propagate=False)
        self.vval = {}
        for k, row in t['inodes_ballot'].rows.items():
            self._iballot(k, row, 1)

    # ---- results
    def stake(self, pt) -> Optional[Decimal]:
        s = self.astake.get(pt)
        return Decimal(0) if s is None else s.result()

    def validator_stake(self, pt) -> Optional[Decimal]:
        if self.pending_v:
            self._flush()
        return self._vstake(pt)

    def _vstake(self, pt) -> Optional[Decimal]:
        if pt in self.bad_v:
            return None
        hit = self.vval.get(pt)
        if hit is None:
            s = self.vsum.get(pt)
            r = Decimal(0) if s is None else s.result()
            if r is None:
                return None
            hit = self.vval[pt] = round_up_decimal(r)
        return hit

    def inode_power(self, pt) -> Optional[Decimal]:
        if self.pending_v:
            self._flush()
        if pt in self.bad_i:
            return None
        s = self.isum.get(pt)
        r = Decimal(0) if s is None else s.result()
        return None if r is None else round_up_decimal(r)

    # ---- terms
    @staticmethod
    def _vote(row):
        return Decimal(row[1]) / SMALLEST if row[1] is not None else None

    def _vballot(self, key, row, sign, propagate=True):
        recv = point_key_of(row[0])
        if sign > 0:
            vote, voter = self._vote(row), point_key_of(row[2])
            st = self.stake(voter) if voter is not None else None
            if vote is None or st is None:
                self.bad_v.add(recv)
                term = None
            else:
                term = (vote * st) / 10
                self.vsum.setdefault(recv, _ExactSum()).update(term, 1)
            self.vterm[key] = (recv, term)
        else:
            recv, term = self.vterm.pop(key, (recv, None))
            if term is not None:
                self.vsum.setdefault(recv, _ExactSum()).update(term, -1)
        if propagate:
            self._validator_changed(recv)

    def _iballot(self, key, row, sign):
        recv = point_key_of(row[0])
        if sign > 0:
            vote, voter = self._vote(row), point_key_of(row[2])
            vs = self._vstake(voter) if voter is not None else None
            if vote is None or vs is None:
                self.bad_i.add(recv)
                term = None
            else:
                term = (vote * vs) / 10
                self.isum.setdefault(recv, _ExactSum()).update(term, 1)
            self.iterm[key] = (recv, term)
        else:
            recv, term = self.iterm.pop(key, (recv, None))
            if term is not None:
                self.isum.setdefault(recv, _ExactSum()).update(term, -1)

    def _stake_row(self, row, sign, propagate=True):
        pt = point_key_of(row[0])
        if row[1] is None:
            self.astake.setdefault(pt, _ExactSum()).ok = False
        else:
            self.astake.setdefault(pt, _ExactSum()).update(Decimal(row[1]) / SMALLEST, sign)
        if propagate:  # re-term every ballot this delegate cast
            vb = self.gov.tables['validators_ballot']
            for k in list(vb.by_voter_pt.get(pt, ())):
                row_k = vb.rows[k]
                self._vballot(k, row_k, -1, propagate=False)
                self._vballot(k, row_k, 1, propagate=True)

    def _validator_changed(self, pt):
        self.pending_v.add(pt)
        self.vval.pop(pt, None)

    def _flush(self):
        """Re-term the inode ballots of every validator whose stake may have changed since the last query
        (once per validator however many of its ballots or delegates changed in between)."""
        ib = self.gov.tables['inodes_ballot']
        while self.pending_v:
            pt = self.pending_v.pop()
            for k in list(ib.by_voter_pt.get(pt, ())):
                row_k = ib.rows[k]
                self._iballot(k, row_k, -1)
                self._iballot(k, row_k, 1)

    def row_changed(self, table: str, key: Key, row: tuple, sign: int):
        if table == STAKE:
            self._stake_row(row, sign)
        elif table == 'validators_ballot':
            self._vballot(key, row, sign)
        elif table == 'inodes_ballot':
            self._iballot(key, row, sign)


class GovernanceIndex:
    def __init__(self, db):
        self.db = db
        self.lock = threading.RLock()
        self.tables: Dict[str, _Table] = {t: _Table(t, self._changed) for t in (*GOV_TABLES, STAKE)}
        self.version = 0
        # the emission cascade (get_active_inodes -> inode power -> validator stake -> delegate stake) kept
        # as exact running sums that follow every row change (_Cascade), so a block costs O(its changes)
        self.cascade = _Cascade(self)
        self._memo: dict = {}
        self._memo_version = -1
        self._pending = None  # (mempool version, pending-spent set, pending stake per address)
        self._parsed: Dict[str, list] = {}  # pending tx hash -> [(address, amount, is_stake)] of its outputs

    # ------------------------------------------------------------------ maintenance
    def _rows_sql(self, table: str, where: str = '', args: tuple = ()):
        src = 'unspent_outputs' if table == STAKE else table
        cond = ['u.is_stake = 1'] if table == STAKE else []
        if where:
            cond.append(where)
        w = ('WHERE ' + ' AND '.join(cond)) if cond else ''
        return self.db._q(f'SELECT u.tx_hash, u."index", u.address, t.outputs_amounts, t.inputs_addresses, b.timestamp '
                          f'FROM {src} u INNER JOIN transactions t ON t.tx_hash = u.tx_hash '
                          f'LEFT JOIN blocks b ON b.hash = t.block_hash {w} ORDER BY u.rowid', args)

    def _add_sql_rows(self, table: str, rows, only: Optional[Set[Key]] = None):
        import json
        tab = self.tables[table]
        for h, i, address, am, ia, ts in rows:
            key = (h, int(i))
            if only is not None and key not in only:
                continue
            amount = _at(json.loads(am) if am else [], int(i))
            voter = _at(json.loads(ia) if ia else [], int(i))
            tab.add(key, address, amount, voter, ts)

    def _changed(self, table: str, key: Key, row: tuple, sign: int):
        self.cascade.row_changed(table, key, row, sign)

    @_locked
    def rebuild(self):
        for t in self.tables:
            self.tables[t] = _Table(t, None)
            self._add_sql_rows(t, self._rows_sql(t))
            self.tables[t].changed = self._changed
        self.cascade.build()
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
        tab = self.tables[table]
        hit = False
        for h, i in keys:
            hit |= tab.remove((h, int(i)))
        if hit:
            self.version += 1

    @_locked
    def stake_keys(self) -> Dict[Key, tuple]:
        return dict(self.tables[STAKE].rows)

    @_locked
    def stake_raw(self):
        """(keys, n x 36 raw (txid || u32 index) array) of the staked outputs, memoised per version: the
        native block path tests a block's spent outpoints against it with one vectorised isin."""
        def build():
            import numpy as np
            keys = list(self.tables[STAKE].rows)
            raw = np.zeros((len(keys), 36), dtype=np.uint8)
            for k, (h, i) in enumerate(keys):
                raw[k, :32] = np.frombuffer(bytes.fromhex(h), dtype=np.uint8)
                raw[k, 32:36] = np.frombuffer(int(i).to_bytes(4, 'little'), dtype=np.uint8)
            return keys, np.ascontiguousarray(raw).view('V36').ravel()
        return self._memo_get('stake_raw', build)

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
    def has_point(self, table: str, pt: Optional[bytes], check_pending: bool, voter: bool = False) -> bool:
        """Is there a live row of ``table`` whose address (``voter``: voter) denotes point ``pt``?"""
        tab = self.tables[table]
        keys = (tab.by_voter_pt if voter else tab.by_pt).get(pt)
        if not keys:
            return False
        if not check_pending:
            return True
        pend = self.pending_spent(True)
        return any(k not in pend for k in keys)

    @_locked
    def pending_spent(self, check_pending: bool) -> Set[Key]:
        return self._overlay()[1] if check_pending else set()

    # ------------------------------------------------------------------ queries (reference semantics)
    @_locked
    def amount_rows(self, table: str, forms: List[str], check_pending: bool) -> List[Tuple[str, int, object]]:
        """``_amount_rows``: (tx_hash, index, amount) of rows whose address is in ``forms``, rowid order."""
        tab = self.tables[table]
        pend = self.pending_spent(check_pending)
        return [(h, i, tab.rows[(h, i)][1]) for h, i in tab.keys_for(tab.by_addr, forms) if (h, i) not in pend]

    @_locked
    def ballot_rows(self, table: str, receiver_forms: Optional[List[str]], check_pending: bool,
                    voter_forms: Optional[Set[str]] = None, order: bool = True):
        """``_ballot_rows``: (tx_hash, receiver, vote, voter, index), ordered by (tx_hash, rowid) or rowid."""
        tab = self.tables[table]
        keys = list(tab.rows) if receiver_forms is None else tab.keys_for(tab.by_addr, receiver_forms)
        if order:
            keys.sort(key=lambda k: k[0])  # stable: rowid order within a tx hash
        pend = self.pending_spent(check_pending)
        out = []
        for k in keys:
            if k in pend:
                continue
            address, amount, voter, _ = tab.rows[k]
            if voter_forms is not None and voter not in voter_forms:
                continue
            out.append((k[0], address, Decimal(amount) / SMALLEST if amount is not None else None, voter, k[1]))
        return out

    @_locked
    def spent_votes(self, table: str, voter_forms: Set[str], check_pending: bool):
        tab = self.tables[table]
        pend = self.pending_spent(check_pending)
        return [(k, tab.rows[k][1]) for k in tab.keys_for(tab.by_voter, voter_forms) if k not in pend]

    @_locked
    def registered_inodes(self, check_pending: bool):
        tab = self.tables['inode_registration_output']
        pend = self.pending_spent(check_pending)
        return [(row[0], row[3]) for k, row in tab.rows.items() if k not in pend and row[3] is not None]

    @_locked
    def address_stake(self, forms: List[str], check_pending: bool) -> Decimal:
        if not check_pending:
            hit = self.cascade.stake(point_key_of(forms[0]) if forms else None)
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
        hit = self.cascade.validator_stake(point_key_of(forms[0]) if forms else None)
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
        hit = self.cascade.inode_power(point_key_of(forms[0]) if forms else None)
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
