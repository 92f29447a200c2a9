"""Governance rules of a block's transactions, checked in batch on the native block path.

reference: ``Transaction.verify`` → the nine rule checks of upow/upow_transactions/transaction.py:240-479
(stake, unstake, validator registration, revokes, inode (de-)registration, votes), each run per tx with
several SQL round trips (upow/database.py:939-1436) against the ledger as it stood BEFORE the block —
txs of one block never see each other — plus, for the ``check_pending_txs`` variants, the mempool.

Here the same predicates run natively over the whole block in one call (csrc/gov_index.cpp
``GovStore.check_block``), against the governance store that :class:`GovernanceIndex`
(ledger/governance.py) keeps, keyed by the point an address denotes (both string forms of an address at
once, no square root), with the output-type columns of the decoded block and the spent outputs' payloads
from the HBM UTXO pass: per-tx sums and last-receiver lookups are one pass over the output columns, each
predicate a hash probe; ``get_active_inodes`` is evaluated only when an inode (de-)registration needs it.

The checker only ever answers "every governance tx passes". A failing rule — or a case whose exact
answer depends on reference quirks that are not worth reproducing here (a pending stake tx of the same
address, a pending vote when an unstake is checked, a ballot that is not its tx's output 0) — hands the
block to the object path, which reproduces the reference's verdict and error message."""
from __future__ import annotations

import time
from typing import Optional

import numpy as np

from ..constants import MAX_INODES
from ..utils import codec
from ..utils.codec import OutputType, TransactionType

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


def _seg(values: np.ndarray, starts: np.ndarray) -> np.ndarray:
    """Per-tx sums of an int64 output column (every tx of a fast block has at least one output)."""
    return np.add.reduceat(values, starts[:-1]) if len(values) else np.zeros(len(starts) - 1, np.int64)


class BlockGovernance:
    """One block's governance view: which txs are governance-relevant, what each input spends, and
    (after :meth:`check`) the signer keys of revoke txs."""

    def __init__(self, tx_type: np.ndarray, out_type: np.ndarray, out_tx: np.ndarray, out_start: np.ndarray,
                 in_tx: np.ndarray):
        from ..ops.native import lib
        self.n = len(tx_type)
        self.tx_type = np.ascontiguousarray(tx_type, dtype=np.uint8)
        self.out_type = np.ascontiguousarray(out_type, dtype=np.uint8)
        self.out_tx = np.ascontiguousarray(out_tx, dtype=np.int32)
        self.out_start = np.ascontiguousarray(out_start, dtype=np.int32)
        self.in_tx = np.ascontiguousarray(in_tx, dtype=np.int32)
        # one native pass (csrc/gov_index.cpp gov_block_mask): a non-REGULAR tx type or any non-REGULAR output
        gov, self.any = lib().gov_block_mask(self.tx_type, self.out_type, self.out_tx, self.n, len(self.out_type))
        self.gov = np.frombuffer(gov, dtype=np.uint8).astype(bool)

    def inputs(self, tag_by_table: dict, tags: np.ndarray, pay: np.ndarray, fee: np.ndarray, out_amount: np.ndarray):
        """After the UTXO pass, in one native pass (gov_block_inputs): every input's expected tag
        (:meth:`spend_tags`), whether any input is not live in its table or has no payload, and the fees of
        :meth:`fee_adjust`. Returns (in_tag u8[n_in], bad, fee i64[n])."""
        from ..ops.native import lib
        lut = np.full(256, tag_by_table['unspent_outputs'], dtype=np.uint8)
        for t, table in SPEND_TABLE.items():
            lut[t] = tag_by_table[table]
        tags = np.ascontiguousarray(tags, dtype=np.uint8)
        in_tag, bad, f = lib().gov_block_inputs(self.tx_type, self.in_tx, tags, np.ascontiguousarray(pay).view(np.uint8), lut,
                                               self.out_type, self.out_start,
                                               np.ascontiguousarray(out_amount, dtype=np.uint64),
                                               np.ascontiguousarray(fee, dtype=np.int64), self.n, len(tags),
                                               len(self.out_type))
        return np.frombuffer(in_tag, dtype=np.uint8), bool(bad), np.frombuffer(f, dtype=np.int64)

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
        """One native call over the whole block (csrc/gov_index.cpp GovStore.check_block); ``get_active_inodes``
        is evaluated only when an inode (de-)registration needs it, then the call is repeated with it."""
        args = [np.ascontiguousarray(self.tx_type, dtype=np.uint8), np.ascontiguousarray(self.out_type, dtype=np.uint8),
                np.ascontiguousarray(out_amount, dtype=np.uint64), np.ascontiguousarray(out_addr, dtype=np.uint8),
                np.ascontiguousarray(out_len, dtype=np.uint8), np.ascontiguousarray(self.out_start, dtype=np.int32),
                np.ascontiguousarray(in_start, dtype=np.int32), np.ascontiguousarray(in_keys, dtype=np.uint8),
                np.ascontiguousarray(pay).view(np.uint8), np.ascontiguousarray(txid, dtype=np.uint8),
                self.gov.astype(np.uint8), self.n, time.time(), bool(codec.is_blockchain_syncing)]
        active_false = active_true = None
        for _ in range(2):
            with g.lock:
                pend, pstake, votes = g.pending_blob(), set(g._overlay()[2]), g.pending_vote_as_delegate()
                status, signers = g.store.check_block(*args, pend, pstake, votes, active_false, active_true,
                                                      MAX_INODES)
            if status != 2:
                break
            active_false = [e.get('wallet') for e in await db.get_active_inodes(False)]
            active_true = len(await db.get_active_inodes(True))
        return {'signers': signers} if status == 0 else None


__all__ = ['BlockGovernance', 'SPEND_TABLE', 'OUTPUT_TABLE', 'UNSTAKE_EXCEPTION']
