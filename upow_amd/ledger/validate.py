"""Batched block-transaction validation (the MI355X replacement of manager.py:628-632).

reference: ``for tx in transactions: await tx.verify(check_double_spend=False)`` — one fastecdsa
verify (or two, with the ASCII-hex fallback of transaction_input.py:107-109) per distinct
(public key, signature) of each input, one Python square root per address.

Here, for a whole block:
 1. every address that will be turned into a point (outputs, input owners, revoke voters) is
    decompressed in ONE batch (``p256_decompress`` kernel);
 2. every signature job of every tx is collected with the reference's de-duplication rule
    (``(input.public_key, input.signed)``, transaction.py:148-163) and verified in ONE batched
    P-256 launch over the raw-bytes digests; only the failures are re-run over the ASCII-hex digests;
 3. the per-tx rule checks (governance, outputs, fees) then run in block order, and the first
    failing tx is reported exactly like the reference loop would.
"""
from __future__ import annotations

import hashlib
import os
from time import perf_counter
from typing import List, Optional

import numpy as np

from ..models.transaction import Transaction
from ..ops import p256 as op
from ..utils import codec, metrics
from ..utils.codec import TransactionType
from ..utils.logger import get_logger

logger = get_logger(__name__)
timings: dict = {}
_dist_ctx = None  # set on multi-GPU nodes: the signature batch is sharded across ranks (parallel/verify_dp.py)
# sharding threshold: below this many signatures every replica verifies the whole batch itself. One GPU
# verifies a 2 MB block's ~8,300 signatures in ~1.2 ms (the quad kernel's latency floor); splitting them
# saves under a millisecond and costs an all-gather plus the host syncs around it, so the cluster path only
# shards batches that fill more than a chip (initial-sync batches, mempool bursts). Every replica sees the
# same batch size, so all of them take the same branch.
SHARD_MIN = int(os.environ.get('UPOW_CLUSTER_SHARD_MIN', '32768'))


def set_dist_context(ctx) -> None:
    """Shard block signature verification over the ranks of ``ctx`` (every rank must call
    :func:`verify_block_transactions` on the same block)."""
    global _dist_ctx
    _dist_ctx = ctx if (ctx is not None and ctx.is_distributed) else None


def overlappable(n_sigs: int) -> bool:
    """True when :func:`_verify` of ``n_sigs`` signatures issues no collective (any thread may run it)."""
    return _dist_ctx is None or n_sigs < SHARD_MIN


def _verify(recs: bytes, device):
    if _dist_ctx is not None and len(recs) // 160 >= SHARD_MIN:
        from ..parallel.verify_dp import verify_records_dp
        return verify_records_dp(_dist_ctx, recs, device=device)
    return op.verify_records(recs, device=device)

_REVOKE = (TransactionType.REVOKE_AS_VALIDATOR, TransactionType.REVOKE_AS_DELEGATE)


def _related_address_bytes(tx: Transaction):
    out = []
    for i in tx.inputs:
        info = i.transaction_info
        if info is None:
            continue
        try:
            if tx.transaction_type in _REVOKE:
                out.append(codec.string_to_bytes(info['inputs_addresses'][0]))
            else:
                out.append(codec.string_to_bytes(info['outputs_addresses'][i.index]))
        except (IndexError, KeyError, ValueError, TypeError):
            pass
    return out


async def verify_block_transactions(transactions: List[Transaction], device: Optional[str] = None
                                    ) -> Optional[Transaction]:
    """Return the first transaction (in block order) that fails verification, or None."""
    if not transactions:
        return None
    t0 = perf_counter()
    # 1) batch point decompression
    addr = []
    for tx in transactions:
        addr.extend(o.address_bytes for o in tx.outputs)
        addr.extend(_related_address_bytes(tx))
    codec.prefetch_points(addr)
    t1 = perf_counter()

    # 2) signature jobs
    jobs_q, jobs_sig, jobs_msg, jobs_tx = [], [], [], []
    tx_state = []  # per tx: None (ok so far) | 'unsigned' | Exception
    for k, tx in enumerate(transactions):
        state = None
        voter = tx.transaction_type in _REVOKE
        msg = tx.hex(False)
        checked = []
        try:
            for i in tx.inputs:
                if i.signed is None:
                    state = 'unsigned'
                    break
                pk = await (i.get_voter_public_key() if voter else i.get_public_key())
                key = (i.public_key, i.signed)
                if key in checked:
                    continue
                checked.append(key)
                jobs_q.append(pk)
                jobs_sig.append(i.signed)
                jobs_msg.append(msg)
                jobs_tx.append(k)
        except Exception as e:  # surfaced when the reference loop would reach this tx
            state = e
        tx_state.append(state)
    t2 = perf_counter()

    n = len(jobs_q)
    status = np.zeros(n, dtype=np.uint8)
    if n:
        recs = bytearray(160 * n)
        bad_range = np.zeros(n, dtype=bool)
        for j in range(n):
            q, (r, s) = jobs_q[j], jobs_sig[j]
            if not (0 <= r < 1 << 256 and 0 <= s < 1 << 256):
                bad_range[j] = True
                continue
            recs[160 * j:160 * j + 160] = op.record(q, (r, s), hashlib.sha256(bytes.fromhex(jobs_msg[j])).digest())
        status = _verify(bytes(recs), device).copy()
        status[bad_range] = op.BAD_RANGE
        retry = np.nonzero(status == op.INVALID)[0]
        if len(retry):
            recs2 = bytearray(160 * len(retry))
            for m, j in enumerate(retry):
                recs2[160 * m:160 * m + 160] = op.record(jobs_q[j], jobs_sig[j],
                                                         hashlib.sha256(jobs_msg[j].encode()).digest())
            st2 = _verify(bytes(recs2), device)
            status[retry] = np.where(st2 == op.VALID, op.VALID, status[retry])
    t3 = perf_counter()

    # 3) per-tx rules in block order
    job_pos = 0
    bad = None
    for k, tx in enumerate(transactions):
        my_jobs = []
        while job_pos < n and jobs_tx[job_pos] == k:
            my_jobs.append(job_pos)
            job_pos += 1
        await tx._fill_transaction_inputs()
        if not await tx.verify_rules():
            bad = tx
            break
        st = tx_state[k]
        if isinstance(st, Exception):
            raise st
        if st == 'unsigned':
            logger.error('not signed')
            bad = tx
            break
        sig_ok = True
        for j in my_jobs:
            if status[j] == op.BAD_KEY:
                raise op.EcdsaError('Invalid public key, point is not on curve P256')
            if status[j] == op.BAD_RANGE:
                raise op.EcdsaError('Invalid Signature: r or s is not a positive integer smaller than the curve order')
            if status[j] != op.VALID:
                logger.error('signature not valid')
                sig_ok = False
                break
        if not sig_ok:
            bad = tx
            break
        if not tx._verify_outputs():
            logger.error('invalid outputs')
            bad = tx
            break
        if await tx.get_fees() < 0:
            logger.error('We are not the Federal Reserve')
            bad = tx
            break
    t4 = perf_counter()
    timings.update({'decompress_s': t1 - t0, 'collect_s': t2 - t1, 'ecdsa_s': t3 - t2, 'rules_s': t4 - t3,
                    'signatures': n, 'txs': len(transactions)})
    metrics.inc('upow_signatures_verified_total', n, help='P-256 signatures verified in block validation')
    for stage in ('decompress', 'collect', 'ecdsa', 'rules'):
        metrics.set_gauge('upow_block_stage_seconds', timings[stage + '_s'], labels={'stage': stage},
                          help='stage wall time of the last validated block')
    return bad
