"""Governance rules of a block's transactions, checked in batch on the native block path.

reference: ``Transaction.verify`` → the nine rule checks of upow/upow_transactions/transaction.py:240-479
(stake, unstake, validator registration, revokes, inode (de-)registration, votes), each run per tx with
several SQL round trips (upow/database.py:939-1436) against the ledger as it stood BEFORE the block —
txs of one block never see each other — plus, for the ``check_pending_txs`` variants, the mempool.

Here the same predicates read the in-memory :class:`GovernanceIndex` (ledger/governance.py) keyed by the
point an address denotes (``point_key``: both string forms of an address at once, no square root), the
output-type columns of the decoded block and the spent outputs' payloads from the HBM UTXO pass:

* per-tx sums (vote ranges, registration amounts, voting power) are segment reductions over the output
  columns, computed once for the whole block;
* the per-tx predicates are dictionary probes; ``get_active_inodes`` is evaluated at most once per
  block and variant.

The checker only ever answers "every governance tx passes". A failing rule — or a case whose exact
answer depends on reference quirks that are not worth reproducing here (a pending stake tx of the same
address, a pending vote when an unstake is checked, a ballot that is not its tx's output 0) — hands the
block to the object path, which reproduces the reference's verdict and error message."""
from __future__ import annotations

from datetime import timedelta
from typing import Optional

import numpy as np

from ..constants import MAX_INODES, SMALLEST
from ..utils import codec
from ..utils.codec import OutputType, TransactionType
from .governance import STAKE, point_key, point_key_of

T = TransactionType
O = OutputType
INODE_T, VALIDATOR_T = 'inode_registration_output', 'validator_registration_output'
VVP_T, DVP_T = 'validators_voting_power', 'delegates_voting_power'
IBALLOT_T, VBALLOT_T = 'inodes_ballot', 'validators_ballot'

# the table each tx type spends from (database.py:589-621 remove_outputs; transaction.py:99-124)
SPEND_TABLE = {int(T.INODE_DE_REGISTRATION): INODE_T, int(T.VOTE_AS_VALIDATOR): VVP_T,
               int(T.VOTE_AS_DELEGATE): DVP_T, int(T.REVOKE_AS_VALIDATOR): IBALLOT_T,
               int(T.REVOKE_AS_DELEGATE): VBALLOT_T}
# the table each output type lands in (database.py:524-580 add_transaction_outputs)
OUTPUT_TABLE = {int(O.REGULAR): 'unspent_outputs', int(O.STAKE): 'unspent_outputs', int(O.UN_STAKE): 'unspent_outputs',
                int(O.INODE_REGISTRATION): INODE_T, int(O.VALIDATOR_REGISTRATION): VALIDATOR_T,
                int(O.VALIDATOR_VOTING_POWER): VVP_T, int(O.DELEGATE_VOTING_POWER): DVP_T,
                int(O.VOTE_AS_VALIDATOR): IBALLOT_T, int(O.VOTE_AS_DELEGATE): VBALLOT_T}
UNSTAKE_EXCEPTION = '8befeb253bc6eddd8501f5b27a02b195f5c06a51ccf788213cbedafe7cc49c53'  # transaction.py:472
_REVOKES = (int(T.REVOKE_AS_VALIDATOR), int(T.REVOKE_AS_DELEGATE))


def _seg(values: np.ndarray, starts: np.ndarray) -> np.ndarray:
    """Per-tx sums of an int64 output column (every tx of a fast block has at least one output)."""
    return np.add.reduceat(values, starts[:-1]) if len(values) else np.zeros(len(starts) - 1, np.int64)


class BlockGovernance:
    """One block's governance view: which txs are governance-relevant, what each input spends, and
    (after :meth:`check`) the signer keys of revoke txs."""

    def __init__(self, tx_type: np.ndarray, out_type: np.ndarray, out_tx: np.ndarray, out_start: np.ndarray,
                 in_tx: np.ndarray):
        self.n = len(tx_type)
        self.tx_type = tx_type
        self.out_type = out_type
        self.out_tx = out_tx
        self.out_start = out_start
        self.in_tx = in_tx
        gov_out = out_type != 0
        has_gov_out = np.zeros(self.n, dtype=bool)
        if gov_out.any():
            has_gov_out[np.unique(out_tx[gov_out])] = True
        self.gov = (tx_type != 0) | has_gov_out
        self.any = bool(self.gov.any())

    def spend_tags(self, tag_by_table: dict) -> np.ndarray:
        """Expected UTXO-index tag of every input (the table its tx type spends from)."""
        lut = np.full(256, tag_by_table['unspent_outputs'], dtype=np.uint8)
        for t, table in SPEND_TABLE.items():
            lut[t] = tag_by_table[table]
        return lut[self.tx_type][self.in_tx]

    def output_tags(self, tag_by_table: dict) -> np.ndarray:
        lut = np.zeros(256, dtype=np.uint32)
        for t, table in OUTPUT_TABLE.items():
            lut[t] = tag_by_table[table]
        return lut[self.out_type]

    def fee_adjust(self, fee: np.ndarray, out_amount: np.ndarray) -> np.ndarray:
        """get_fees (transaction.py:499-518): only REGULAR-type txs carry fees, and voting-power outputs do
        not count against their inputs; every other tx type has fee 0 (the device pass subtracted every
        output from every tx's inputs)."""
        vp = (self.out_type == O.VALIDATOR_VOTING_POWER) | (self.out_type == O.DELEGATE_VOTING_POWER)
        f = fee + _seg(np.where(vp, out_amount.astype(np.int64), 0), self.out_start)
        return np.where(self.tx_type == 0, f, 0)

    async def check(self, db, in_start: np.ndarray, out_amount: np.ndarray, out_addr: np.ndarray,
                    out_len: np.ndarray, in_keys: np.ndarray, pay, txid: np.ndarray) -> Optional[dict]:
        """Every governance tx's rules (transaction.py:196-221 order). Returns the signer overrides of
        revoke inputs {input index: address bytes} when all pass, None for the object path."""
        g = db.gov
        if g is None:
            return None
        try:
            return await self._check(db, g, in_start, out_amount, out_addr, out_len, in_keys, pay, txid)
        except Exception:  # anything unexpected: the object path decides (and raises what the reference raises)
            return None

    async def _check(self, db, g, in_start, out_amount, out_addr, out_len, in_keys, pay, txid):
        S = SMALLEST
        ot, amt = self.out_type, out_amount.astype(np.int64)
        starts = self.out_start

        def ssum(t):
            return _seg(np.where(ot == t, amt, 0), starts)

        def last_of(t):  # index of the last output of type t per tx (the reference's ``receiver``), -1 if none
            return np.maximum.reduceat(np.where(ot == t, np.arange(len(ot)), -1), starts[:-1])
        gov_idx = np.nonzero(self.gov)[0]
        gov_k = gov_idx.tolist()
        tt = self.tx_type.tolist()
        cnt = {t: _seg((ot == t).astype(np.int64), starts) for t in (O.STAKE, O.UN_STAKE, O.INODE_REGISTRATION,
                                                                    O.VALIDATOR_VOTING_POWER)}
        has = {t: (cnt[t] > 0).tolist() for t in (O.STAKE, O.UN_STAKE, O.INODE_REGISTRATION)}
        sums = {t: ssum(t).tolist() for t in (O.DELEGATE_VOTING_POWER, O.VALIDATOR_REGISTRATION, O.INODE_REGISTRATION,
                                              O.VOTE_AS_VALIDATOR, O.VOTE_AS_DELEGATE)}
        n_vvp = cnt[O.VALIDATOR_VOTING_POWER].tolist()
        last_vvp = last_of(O.VALIDATOR_VOTING_POWER).tolist()
        recv = {O.VOTE_AS_VALIDATOR: last_of(O.VOTE_AS_VALIDATOR).tolist(),
                O.VOTE_AS_DELEGATE: last_of(O.VOTE_AS_DELEGATE).tolist()}
        ins = in_start.tolist()
        # point keys of every governance tx's input-0 owner, vectorised: [43 if odd y else 42] || x
        j0 = in_start[gov_idx]
        pa, pl = pay['addr'][j0], pay['len'][j0]
        pts = np.empty((len(j0), 33), dtype=np.uint8)
        pts[:, 1:] = np.where((pl == 33)[:, None], pa[:, 1:33], pa[:, :32])
        odd = np.where(pl == 33, pa[:, 0] == 43, (pa[:, 32] & 1) == 1)
        pts[:, 0] = np.where(odd, 43, 42)
        if np.any((pl != 33) & (pl != 64)):
            return None
        pt_of = dict(zip(gov_k, pts.view('V33').ravel().tolist()))
        p_addr, p_len = pay['addr'], pay['len']

        def out_pt(o):
            return point_key(bytes(out_addr[o, :out_len[o]]))

        memo = {}

        async def active(cp: bool):
            if cp not in memo:
                memo[cp] = await db.get_active_inodes(cp)
            return memo[cp]

        with g.lock:
            pend = g.pending_spent(True)
            T_ = g.tables
            stake_pt, inode_pt, valid_pt = T_[STAKE].by_pt, T_[INODE_T].by_pt, T_[VALIDATOR_T].by_pt
            dvp_pt, vb_voter = T_[DVP_T].by_pt, T_[VBALLOT_T].by_voter_pt

            def live(index, pt, cp):
                keys = index.get(pt)
                if not keys:
                    return False
                return not cp or not pend or any(k not in pend for k in keys)

            def delegate_power(pt):  # get_delegates_all_power: voting power outputs + cast delegate ballots
                return live(dvp_pt, pt, False) or live(vb_voter, pt, False)
            signers = {}
            now = None
            for k in gov_k:
                t = tt[k]
                pt0 = pt_of[k]
                # stake (transaction.py:434-465)
                if has[O.STAKE][k]:
                    if live(stake_pt, pt0, False) and not codec.is_blockchain_syncing:
                        return None
                    j0k = ins[k]
                    if codec.bytes_to_string(bytes(p_addr[j0k, :p_len[j0k]])) in g._overlay()[2]:
                        return None  # a pending stake tx of this address: the reference's tx_hash quirk decides
                    power = sums[O.DELEGATE_VOTING_POWER][k]
                    if power > 0:
                        if power != 10 * S or delegate_power(pt0):
                            return None
                    elif not delegate_power(pt0):
                        return None
                # unstake (transaction.py:467-479)
                if has[O.UN_STAKE][k]:
                    if live(vb_voter, pt0, False) and bytes(txid[k]).hex() != UNSTAKE_EXCEPTION:
                        return None
                    if g.pending_vote_as_delegate():
                        return None
                if t == 0:
                    if has[O.INODE_REGISTRATION][k]:
                        pass  # checked below
                    else:
                        continue
                if t == T.VOTE_AS_DELEGATE:  # transaction.py:292-316 (block validation: stake without mempool)
                    v = sums[O.VOTE_AS_DELEGATE][k]
                    if v > 10 * S or v <= 0 or live(inode_pt, pt0, True) or not live(stake_pt, pt0, False):
                        return None
                    if not live(valid_pt, out_pt(recv[O.VOTE_AS_DELEGATE][k]), True):
                        return None
                    continue
                if t == T.VOTE_AS_VALIDATOR:  # transaction.py:258-290
                    v = sums[O.VOTE_AS_VALIDATOR][k]
                    if v > 10 * S or v <= 0 or live(inode_pt, pt0, True) or not live(valid_pt, pt0, True):
                        return None
                    if not live(inode_pt, out_pt(recv[O.VOTE_AS_VALIDATOR][k]), True):
                        return None
                    continue
                if t == T.VALIDATOR_REGISTRATION:  # transaction.py:371-398
                    if not live(stake_pt, pt0, False) or live(valid_pt, pt0, True) or live(inode_pt, pt0, True):
                        return None
                    if sums[O.VALIDATOR_REGISTRATION][k] != 100 * S or n_vvp[k] != 1 or amt[last_vvp[k]] != 10 * S:
                        return None
                if t in _REVOKES:  # transaction.py:400-432: signed by the voter of each ballot input
                    table = IBALLOT_T if t == T.REVOKE_AS_VALIDATOR else VBALLOT_T
                    rows = T_[table].rows
                    valid = False
                    for j in range(ins[k], ins[k + 1]):
                        key = (bytes(in_keys[j, :32]).hex(), int.from_bytes(bytes(in_keys[j, 32:36]), 'little'))
                        row = rows.get(key)
                        if row is None or key[1] != 0 or row[2] is None or row[3] is None:
                            return None  # voter = inputs_addresses[0] of the ballot tx = the row's voter iff index 0
                        vraw = codec.string_to_bytes(row[2])
                        if len(vraw) not in (33, 64):
                            return None
                        signers[j] = vraw
                        if now is None:
                            from .database import _dt, _utcnow
                            now = _utcnow()
                        valid = valid or now - _dt(row[3]) >= timedelta(hours=48)
                    voter_pt = point_key(signers[ins[k]])
                    if t == T.REVOKE_AS_VALIDATOR and not live(valid_pt, voter_pt, True):
                        return None
                    if not live(stake_pt, voter_pt, False) or not valid:
                        return None
                if t == T.INODE_DE_REGISTRATION:  # transaction.py:240-256
                    j0k = ins[k]
                    address = codec.bytes_to_string(bytes(p_addr[j0k, :p_len[j0k]]))
                    if not live(inode_pt, pt0, False):
                        return None
                    if any(e.get('wallet') == address for e in await active(False)):
                        return None
                if has[O.INODE_REGISTRATION][k]:  # transaction.py:318-352
                    j0k = ins[k]
                    address = codec.bytes_to_string(bytes(p_addr[j0k, :p_len[j0k]]))
                    if sums[O.INODE_REGISTRATION][k] != 1000 * S or not live(stake_pt, pt0, False) or \
                            live(inode_pt, pt0, True) or live(valid_pt, pt0, True):
                        return None
                    if len(await active(True)) >= MAX_INODES:
                        return None
                    if any(e.get('wallet') == address for e in await active(False)):
                        return None
        return {'signers': signers}


__all__ = ['BlockGovernance', 'SPEND_TABLE', 'OUTPUT_TABLE', 'UNSTAKE_EXCEPTION']
