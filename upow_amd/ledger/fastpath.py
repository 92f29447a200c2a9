"""Native block path: validate and apply a block given as tx hex strings, without Transaction objects.

reference: ``POST /push_block`` → ``manager.create_block`` (upow/manager.py:422-757), which builds one
Python object graph per tx, checks it input by input and writes it row by row. This module runs the
same checks over whole-block arrays:

  1. ``_native.decode_block_txs`` (csrc/txcodec.cpp): decode + canonical re-serialisation + txids +
     signed-message digests + address strings + JSON columns + merkle root, threaded in C++;
  2. one HBM UTXO ``lookup`` launch for every input: existence in ``unspent_outputs`` AND the spent
     output's amount and address (the payload the table carries), so no SQL read is needed;
  3. one batched point decompression for every key involved (signers and outputs), one batched
     P-256 verify (sharded over ranks on a multi-GPU node; otherwise on a helper thread while this thread
     renders the apply columns' address strings) + the ASCII-hex retry pass;
  4. fees, output validity and the merkle root as array arithmetic;
  5. the ledger writes of ``_apply_block`` as ONE journal batch of column-major bulk statements
     (csrc/ledger_writer.cpp: the journal append is the commit point, a background thread on its own
     SQLite connection materialises the tables) + one index insert launch + one erase launch.

Scope: every tx type. Governance transactions (stake/unstake outputs, inode and validator registration,
votes, revokes) ride the same arrays: each input is looked up in the table its tx type spends from, their
rules run in batch against the governance index (ledger/govcheck.py), revokes are verified against the
voter's key, and their outputs and spends are journaled into the governance tables in the same batch.
Txs with 1 < k < n signatures take the native path too: their inputs are grouped by the owner keys the UTXO
pass returns, in order of first appearance, and signature g verifies against group g's key
(``_resolve_groups``). ANY failed check hands the block to the object path (``manager._create_block``),
which then reproduces the reference's exact verdict, error message or exception — with one exception: when
every other rule of every tx held and the only failures are plainly invalid signatures (under both message
forms), the verdict and message are already known (the object path stops at the first such tx in block
order with "transaction <hash> has been not verified"), so the block is rejected here, and a hostile block of
bad signatures costs one batched verify instead of a per-tx Python re-validation.
``tests/test_fastpath.py`` runs both paths over the same blocks and compares the whole ledger and the errors.
"""
from __future__ import annotations

import os
from decimal import Decimal
from time import perf_counter
from typing import List, Optional

import numpy as np

from ..constants import MAX_BLOCK_SIZE_HEX, SMALLEST
from ..models.transaction import Transaction
from ..ops import p256 as op
from ..ops.native import gpu_available, lib
from ..utils import metrics, roctx
from ..utils.codec import TransactionType, get_transaction_type_from_message, sha256
from ..utils.hexspans import HexSpans
from ..utils.logger import get_logger
from .govcheck import BlockGovernance
from ..utils.cpus import cpu_budget  # noqa: F401 (re-exported: node/__main__.py)
from .utxo import TAG_BY_TABLE

logger = get_logger(__name__)


def _codec_threads() -> int:
    """Host threads for the block codec: the usable CPUs (cpu_budget), capped at 16, minus two for the
    ledger's materialiser threads that run concurrently."""
    return max(1, min(16, cpu_budget()) - 2)


THREADS = int(os.environ.get('UPOW_CODEC_THREADS', '0')) or _codec_threads()
ENABLED = os.environ.get('UPOW_FASTPATH', '1') != '0'
timings: dict = {}
last_path = None  # 'native' | 'object' for the last block (tests, metrics)
AMOUNT_LIMIT = 1 << 52  # > max supply in smallest units; keeps per-tx int64 sums exact


_VERIFY_POOL = None


def _verify_pool():
    """One helper thread for the block's signature verify (overlapped with the apply strings)."""
    global _VERIFY_POOL
    if _VERIFY_POOL is None:
        from concurrent.futures import ThreadPoolExecutor
        _VERIFY_POOL = ThreadPoolExecutor(max_workers=1, thread_name_prefix='upow-block-verify')
    return _VERIFY_POOL


def _i32(d, k):
    return np.frombuffer(d[k], dtype=np.int32)


# signer keys decompressed, curve checks and the signature verify in one GPU stream order for a block whose
# addresses are all 33-byte keys (UPOW_FUSED_VERIFY=0: the host key stage + separate verify, the A/B form)
FUSED_VERIFY = os.environ.get('UPOW_FUSED_VERIFY', '1') != '0'
_FUSED_HOST = os.environ.get('UPOW_FUSED_VERIFY') == 'host'  # the same stages on the host (CPU tests of this path)


def decode_raw(tx_hexes, threads: int) -> dict:
    """The codec's dict for a list of str or a :class:`~upow_amd.utils.hexspans.HexSpans` (read in place
    from its body: csrc/txcodec.cpp ``decode_block_spans``)."""
    if isinstance(tx_hexes, HexSpans):
        return lib().decode_block_spans(tx_hexes.buf, np.ascontiguousarray(tx_hexes.spans).tobytes(),
                                        list(tx_hexes.extra), threads)
    return lib().decode_block_txs(tx_hexes if isinstance(tx_hexes, list) else list(tx_hexes), threads)


def decode(tx_hexes: List[str], threads: int = 0) -> Optional[dict]:
    """Native decode; None when the block needs the object path."""
    if not ENABLED:
        return None
    d = decode_raw(tx_hexes, threads or THREADS)
    if not d['all_fast']:
        return None
    if isinstance(tx_hexes, HexSpans):  # the txs' text is the body's; str objects only for the rare fixes
        fix = d.pop('hex_fix')
        if fix:
            tx_hexes = tx_hexes.tolist()
            for k, h in fix:
                tx_hexes[k] = h
        d['hex'] = tx_hexes
    # tx types from the messages: decided natively except for encodings only Python's int() can judge
    tx_type = np.frombuffer(d['tx_type'], dtype=np.uint8).copy()
    ask = np.nonzero(tx_type == 255)[0]
    if len(ask):
        msg_off, msg_len = _i32(d, 'msg_off'), _i32(d, 'msg_len')
        for k in ask.tolist():
            h = d['hex'][k]
            msg = bytes.fromhex(h[2 * msg_off[k]:2 * (msg_off[k] + msg_len[k])])
            tx_type[k] = int(get_transaction_type_from_message(msg))
    d['_tx_type'] = tx_type
    return d


def _signer_records_general(pay, out_addr, out_len, job_input, sigs, sig_ids, digest, job_tx, gpu_min):
    """Verify records when the block has 64-byte (version-1) addresses: 33-byte keys decompressed in one
    batch, 64-byte ones checked on the curve in one batch (csrc/p256.hip ``p256_on_curve``); None when any
    key is invalid."""
    all_addr = np.concatenate([pay['addr'], out_addr]) if len(out_addr) else np.ascontiguousarray(pay['addr'])
    all_len = np.concatenate([pay['len'].astype(np.uint8), out_len])
    xy = np.zeros((len(all_addr), 64), dtype=np.uint8)
    ok = np.ones(len(all_addr), dtype=bool)
    c33 = np.nonzero(all_len == 33)[0]
    if len(c33):
        comp = np.ascontiguousarray(all_addr[c33, :33])
        ubytes, inv_b = lib().unique_rows(comp, 33)
        inv = np.frombuffer(inv_b, dtype=np.int32)
        ubuf = np.frombuffer(ubytes, dtype=np.uint8)
        out, okb = lib().p256_decompress(ubuf, len(ubuf) // 33 >= gpu_min)
        xy[c33] = np.frombuffer(out, dtype=np.uint8).reshape(-1, 64)[inv]
        ok[c33] = np.frombuffer(okb, dtype=np.uint8).astype(bool)[inv]
    c64 = np.nonzero(all_len == 64)[0]
    if len(c64):  # 64-byte keys: one native on-curve batch (transaction_output.py:25-26 per output)
        full = np.ascontiguousarray(all_addr[c64, :64])
        xy[c64] = full
        okb = lib().p256_on_curve(full, len(c64) >= gpu_min, THREADS)
        ok[c64] = np.frombuffer(okb, dtype=np.uint8).astype(bool)
    if not ok.all():
        return None
    return np.ascontiguousarray(np.concatenate([xy[job_input], sigs[sig_ids], digest[job_tx]], axis=1)).tobytes()


def _owner_key(addr: np.ndarray, n: int) -> bytes:
    """The public key an input's owner address stands for, as the parser's grouping sees it
    (``point_to_string(get_public_key())``): x plus the parity of y. A 33-byte address carries the parity
    in its prefix (43 odd, anything else even), a 64-byte one in y's low byte."""
    if n == 33:
        return bytes(addr[1:33]) + (b'\x01' if addr[0] == 43 else b'\x00')
    return bytes(addr[:32]) + bytes([addr[32] & 1])


def _resolve_groups(grouped, job_input, pay, in_start, sig_start, tx_type):
    """Signature -> input assignment of txs with 1 < k < n signatures (reference transaction.py:578-590):
    the inputs grouped by owner key in order of first appearance, signature g for group g. The verify job of
    signature g is group g's first input (the reference checks each (key, signature) pair once). None when
    the group count is not the signature count (the parser raises, or leaves inputs unsigned) or the tx
    type verifies against other keys (revokes are signed by voters): the object path decides those."""
    out = lib().resolve_groups(np.ascontiguousarray(grouped, dtype=np.int64), np.ascontiguousarray(in_start, np.int32),
                               np.ascontiguousarray(sig_start, np.int32), np.ascontiguousarray(tx_type, np.uint8),
                               np.ascontiguousarray(pay['addr']), np.ascontiguousarray(pay['len'], dtype=np.uint8),
                               np.ascontiguousarray(job_input, dtype=np.int64))  # csrc/txcodec.cpp
    return None if out is None else np.frombuffer(out, dtype=np.int64)


def _resolve_groups_py(grouped, job_input, pay, in_start, sig_start, tx_type):
    """The same assignment in Python (the reference form the native one is tested against)."""
    job_input = job_input.copy()
    for t in np.asarray(grouped).tolist():
        if int(tx_type[t]) != 0:
            return None
        first = {}
        for j in range(int(in_start[t]), int(in_start[t + 1])):
            first.setdefault(_owner_key(pay['addr'][j], int(pay['len'][j])), j)
        s0, s1 = int(sig_start[t]), int(sig_start[t + 1])
        if len(first) != s1 - s0:
            return None
        job_input[s0:s1] = list(first.values())  # dicts keep insertion order: group g = g-th new key
    return job_input


def _with_signers(pay: np.ndarray, signers: dict) -> np.ndarray:
    """``pay`` with the address of each input in ``signers`` ({input index: address bytes}) replaced:
    one scatter per address length instead of three numpy calls per input."""
    out = pay.copy()
    js = np.fromiter(signers.keys(), dtype=np.int64, count=len(signers))
    raws = list(signers.values())
    lens = np.fromiter(map(len, raws), dtype=np.int64, count=len(raws))
    out['addr'][js] = 0
    for n in np.unique(lens).tolist():
        sel = np.nonzero(lens == n)[0]
        out['addr'][js[sel], :n] = np.frombuffer(b''.join(raws[k] for k in sel.tolist()), dtype=np.uint8).reshape(-1, n)
        out['len'][js[sel]] = n
    return out


async def create_block_from_hex(block_content: str, tx_hexes: List[str], error_list: list = None,
                                last_block: dict = None, coinbase=None, mirror: bool = True,
                                decoded: Optional[dict] = None, page=None) -> bool:
    """``create_block(block_content, [Transaction.from_hex(h) for h in tx_hexes])``, natively when possible.

    ``decoded``: ``decode(tx_hexes)`` computed ahead of time (the sync pipeline decodes block k+1 on a
    host thread while block k is applied); None means decode here. ``page``: this block's share of a sync
    page's plan (ledger/pagesync.py ``PageBlock``: UTXO pass and signature verdicts already resolved).

    With ``coinbase`` (a CoinbaseTransaction) this is the sync variant ``create_block_in_syncing_old``
    (manager.py:760-835), which trusts the supplied coinbase instead of rebuilding it.

    On a multi-GPU cluster node (parallel/cluster.py) the leader first broadcasts the block to the
    follower replicas (``mirror``); every rank validates it, and the replicas agree in one all-reduce
    right BEFORE any of them commits it (``cluster.commit_point``)."""
    from ..parallel import cluster
    c = cluster.get()
    if c is not None and c.leader and mirror and not c.replaying:
        from ..parallel.cluster import flush_txs, pack_txs
        flush_txs()  # the followers' mempools first: block rules consult pending txs
        c.send('block', pack_txs(tx_hexes), content=block_content, cb=coinbase.hex() if coinbase is not None else None)
    err = None
    # agree before commit: every replica votes right before its journal write (cluster.commit_point) and
    # writes only if all voted yes; a replica that rejects (or fails before that point) votes no at the end
    gate, token = cluster.open_gate('block')
    try:
        ok = await _create_block_from_hex(block_content, tx_hexes, error_list, last_block, coinbase, decoded, page)
    except Exception as e:  # every replica must still take part in the agreement
        ok, err = False, e
    ok = cluster.close_gate(gate, token, ok)
    if err is not None and (c is None or c.leader):
        raise err
    return ok


async def _create_block_from_hex(block_content: str, tx_hexes: List[str], error_list: list = None,
                                 last_block: dict = None, coinbase=None, decoded: Optional[dict] = None,
                                 page=None) -> bool:
    global last_path
    from . import manager
    if error_list is None:
        error_list = []
    t0 = perf_counter()

    async def object_path(locked: bool):
        txs = [await Transaction.from_hex(h) for h in tx_hexes]
        if coinbase is not None:
            fn = manager._create_block_in_syncing_old if locked else manager.create_block_in_syncing_old
            return await fn(block_content, txs, coinbase, last_block, error_list)
        fn = manager._create_block if locked else manager.create_block
        return await fn(block_content, txs, last_block, error_list)

    roctx.push('block:decode')
    dec = decoded if decoded is not None else (decode(tx_hexes) if tx_hexes else None)
    roctx.pop()
    timings['decode_s'] = perf_counter() - t0
    from .database import Database
    if dec is None:
        last_path = 'object'
        if not Database.instance.lean:
            return await object_path(False)
        async with manager.ledger_lock():
            await _leave_lean(Database.instance)
            return await object_path(True)
    async with manager.ledger_lock():
        d0 = roctx.depth()
        try:
            ok = await _create_block_fast(block_content, dec, error_list, last_block, t0, coinbase, page)
        finally:
            roctx.unwind(d0)
            # the block record's fdatasync overlapped the index updates; it is durable before the block is
            # answered or gossiped
            from .database import Database
            with roctx.stage('block:durable'):
                Database.instance.wait_durable()
        last_path = 'native'
        if ok is None:
            last_path = 'object'
            await _leave_lean(Database.instance)
            ok = await object_path(True)
        label = ('sync' if coinbase is not None else 'push') if last_path == 'object' else 'native'
        manager._record_block_metrics(ok, perf_counter() - t0, len(tx_hexes), label)
        return ok


async def _leave_lean(db):
    """The object path reads the SQL tables (inputs resolved from ``transactions``): a lean cluster follower
    (ledger/lean.py) first brings them to its tip, and this block continues in full mode."""
    if db.lean:
        from . import lean
        await lean.materialise(db, online=True)


async def _create_block_fast(block_content: str, d: dict, error_list: list, last_block: Optional[dict],
                             t0: float, coinbase=None, page=None) -> Optional[bool]:
    """True/False for a decided block; None = hand over to the object path."""
    from . import manager, validate
    from .database import Database
    database: Database = Database.instance
    manager.Manager.difficulty = None
    if last_block is None or last_block['id'] % manager.BLOCKS_COUNT == 0:
        difficulty, last_block = await manager.calculate_difficulty()
    else:
        difficulty, last_block = await manager.get_difficulty()
    hdr = await manager.check_block_header(block_content, (difficulty, last_block), error_list)
    if hdr is None:
        return False
    block_no, merkle_tree = hdr
    if page is None:
        logger.info(f'{"Syncing" if coinbase is not None else "Creating"} block no. {block_no} (native path, {d["n"]} txs)')
    elif logger.isEnabledFor(10):  # a sync page logs per chunk (ledger/pagesync.py); per block only at DEBUG
        logger.debug(f'Syncing block no. {block_no} (page plan, {d["n"]} txs)')
    if block_no in manager.double_spend_dict:
        return None
    n = int(d['n'])
    if int(_i32(d, 'hex_len').sum()) > MAX_BLOCK_SIZE_HEX:
        return None
    t1 = perf_counter()
    roctx.push('block:utxo_pass')

    # ---- inputs: one device pass = lookup (existence in unspent_outputs + amount + address),
    #      duplicate detection and per-tx fees (csrc/utxo_table.hip utxo_block_inputs)
    in_keys = np.frombuffer(d['in_keys'], dtype=np.uint8).reshape(-1, 40)
    n_in = len(in_keys)
    in_start, out_start = _i32(d, 'in_start'), _i32(d, 'out_start')
    out_amount = np.frombuffer(d['out_amount'], dtype=np.uint64)
    in_tx, out_tx = _i32(d, 'in_tx'), _i32(d, 'out_tx')
    out_type = np.frombuffer(d['out_type'], dtype=np.uint8)
    bg = BlockGovernance(d['_tx_type'], out_type, out_tx, out_start, in_tx)
    if page is not None:
        # a sync page's plan (ledger/pagesync.py) already resolved this block's inputs against the pre-page
        # index plus the outputs of the page's earlier blocks, and found them live, unique and plain
        if bg.any:
            return None
        tags, pay, fee, missing, n_dup = page.tags, page.pay, page.fee.copy(), None, 0
    else:
        tags, pay, dup_of, fee, missing, n_dup = database.utxo.block_inputs(
            in_keys, in_start, out_amount, out_start, TAG_BY_TABLE['unspent_outputs'])
    if n_dup:
        return None
    in_tag = None
    if bg.any:
        # each input must be live in the table its tx type spends from (manager.py:531-543); fees per get_fees
        in_tag, bad, fee = bg.inputs(TAG_BY_TABLE, tags, pay, fee, out_amount)
        if bad:
            return None
    elif missing is not None and np.any(missing):
        return None
    in_amount = pay['amount']
    if (n_in and in_amount.max() >= AMOUNT_LIMIT) or (len(out_amount) and out_amount.max() >= AMOUNT_LIMIT):
        return None
    t2 = perf_counter()
    roctx.pop()
    roctx.push('block:gov_rules')

    txid = np.frombuffer(d['txid'], dtype=np.uint8).reshape(-1, 32)
    out_len = np.frombuffer(d['out_len'], dtype=np.uint8)
    out_addr = np.frombuffer(d['out_addr'], dtype=np.uint8).reshape(-1, 64)
    signers = None
    if bg.any:
        # governance rules against the pre-block state (ledger/govcheck.py); revokes are signed by voters
        gres = await bg.check(database, in_start, out_amount, out_addr, out_len, in_keys, pay, txid)
        if gres is None:
            return None
        signers = gres['signers'] or None
    t_gov = perf_counter()
    roctx.pop()
    roctx.push('block:signer_records')

    # ---- keys + verify records: every distinct 33-byte key (signers + outputs) decompressed in one
    #      batch, then the 160-byte records of the signature jobs, in one native call
    #      (csrc/txcodec.cpp block_signer_records); blocks with 64-byte addresses take the numpy path
    # one job per distinct signature, checked with its first input's key (the codec numbers signatures in
    # order of first use, so the first input of each is a column of its own)
    job_input = _i32(d, 'sig_first_in').astype(np.int64)
    grouped = np.nonzero(np.frombuffer(d['grouped'], dtype=np.uint8))[0] if 'grouped' in d else ()
    if len(grouped):
        job_input = _resolve_groups(grouped, job_input, pay, in_start, _i32(d, 'sig_start'), d['_tx_type'])
        if job_input is None:
            return None
    sig_ids = np.arange(len(job_input), dtype=np.int64)
    sigs = np.frombuffer(d['sigs'], dtype=np.uint8).reshape(-1, 64)
    digest = np.frombuffer(d['digest'], dtype=np.uint8).reshape(-1, 32)
    job_tx = in_tx[job_input]
    n_jobs = len(job_input)
    gpu_min = op.GPU_MIN_BATCH if gpu_available() else 1 << 62
    over = {}
    if signers:  # the voters' keys replace the owners' for revoke inputs, passed as a short override list
        raws = list(signers.values())
        ov_addr = np.zeros((len(raws), 64), np.uint8)
        for k, r in enumerate(raws):
            ov_addr[k, :len(r)] = np.frombuffer(r, np.uint8)
        over = {'over_idx': np.fromiter(signers.keys(), dtype=np.int64, count=len(signers)), 'over_addr': ov_addr,
                'over_len': np.fromiter(map(len, raws), dtype=np.uint8, count=len(raws))}
    pre_status = None
    fused = False
    if page is not None and not signers and page.n_jobs == n_jobs:
        # the page verified this block's signatures in its one batch, with these very keys (and checked every
        # output address of the page on the curve)
        kst, rec_bytes, pre_status = 1, page.recs, page.status
    elif (FUSED_VERIFY and not signers and n_jobs and (n_jobs >= gpu_min or _FUSED_HOST) and validate.overlappable(n_jobs)
          and bool(np.all(pay['len'] == 33)) and bool(np.all(out_len == 33))):
        # keys, records and verify in one GPU stream order (csrc/txcodec.cpp block_verify_fused), issued below
        # on the verify thread: the key stage leaves the host path
        fused, kst, rec_bytes = True, 1, None
    else:
        kst, rec_bytes = lib().block_signer_records(
            np.ascontiguousarray(pay['addr']), pay['len'].astype(np.uint8), out_addr, out_len,
            job_input.astype(np.int64), sigs, sig_ids.astype(np.int64), digest, job_tx.astype(np.int64), gpu_min,
            **over)
    if kst == 0:  # a signer key or an output address is off-curve: the object path decides
        return None
    if kst < 0:
        sig_pay = _with_signers(pay, signers) if signers else pay
        rec_bytes = _signer_records_general(sig_pay, out_addr, out_len, job_input, sigs, sig_ids, digest, job_tx,
                                            gpu_min)
        if rec_bytes is None:
            return None
    recs = np.frombuffer(rec_bytes, dtype=np.uint8).reshape(-1, 160) if rec_bytes is not None else None
    if np.any(out_amount == 0):
        return None
    t3 = perf_counter()
    roctx.pop()
    roctx.push('block:ecdsa')

    # ---- signatures: one batched verify (+ the reference's ASCII-hex retry for the failures). The verify
    #      runs on a helper thread (the native call releases the GIL) while this thread renders the apply
    #      columns' strings on the host pool below: the kernel's ~1.2 ms and the strings' ~1 ms overlap. A
    #      verify sharded over a cluster's ranks issues collectives and stays on this, the owner, thread.
    # fees first (REGULAR txs; voting-power outputs excluded, governance txs carry none): a negative fee hands
    # the block to the object path before anything is rendered
    if np.any(fee < 0):
        return None
    if fused:
        vfut = _verify_pool().submit(lib().block_verify_fused, np.ascontiguousarray(pay['addr']),
                                     np.ascontiguousarray(pay['len'], dtype=np.uint8), out_addr, out_len,
                                     job_input.astype(np.int64), sigs, sig_ids, digest, job_tx.astype(np.int64),
                                     # the packing runs on this verify thread alone: the host pool takes one
                                     # parallel region at a time, and the apply strings below hold it
                                     1, not _FUSED_HOST)
    else:
        vfut = _verify_pool().submit(validate._verify, rec_bytes, None) \
            if n_jobs and pre_status is None and validate.overlappable(n_jobs) else None
    out_index = np.arange(len(out_tx), dtype=np.int64) - out_start[out_tx]
    out_cols = (out_index, ('arena', *d['out_addr_str']), txid[out_tx], out_amount, out_addr, out_len)
    lean = database.lean  # a lean cluster follower (ledger/lean.py): no SQL rows, so no apply strings
    try:
        # ---- columns for the ledger writes: views of the codec's buffers, encoded natively into one journal
        #      batch by csrc/ledger_writer.cpp (tx hashes rendered from the raw digests, text arenas for strings)
        roctx.push('apply:strings')
        ts0 = perf_counter()
        L = lib()
        in_str = addr_pairs = tx_cols = None
        if not lean or bg.any:  # a lean replica's governance index still takes the input owners' strings
            in_str = L.input_address_strings(np.ascontiguousarray(pay['addr']),
                                             np.ascontiguousarray(pay['len'], dtype=np.uint8), d['in_start'], THREADS,
                                             True)
        if not lean:
            in_json = in_str[:2]
            # the block's address_transactions rows (each tx's distinct input owners and output addresses)
            addr_pairs = L.address_pairs(in_str[2], in_str[3], d['in_start'], *d['out_addr_str'], d['out_start'],
                                         THREADS)
            fee_str = ('arena', *L.fee_strings(np.ascontiguousarray(fee, dtype=np.int64).tobytes()))
            tx_cols = [('hex32', txid, 32, 0), ('hexarena', *d['canon']), ('arena', *in_json),
                       ('arena', *d['out_addr_json']), ('arena', *d['out_amount_json']), fee_str]
        gov_cols = None
        if bg.any:
            gov_cols = {'out_tag': bg.output_tags(TAG_BY_TABLE), 'out_type': out_type, 'in_tag': in_tag,
                        'gov_tx': bg.gov, 'out_tx': out_tx, 'out_start': out_start, 'in_start': in_start,
                        'in_str': in_str[2:]}
        strings_s = perf_counter() - ts0
        roctx.pop()
    except BaseException:
        # no launch outlives this block, but the first error is the one that propagates: a failure of the
        # overlapped verify must not replace the apply-columns error being raised here
        if vfut is not None:
            from concurrent.futures import wait
            wait([vfut])
        raise
    # the verify's verdict
    if fused:
        _, st_b, keys_ok, items = vfut.result()
        if not keys_ok:  # an address off the curve: the object path decides
            return None
        status = np.frombuffer(st_b, dtype=np.uint8).copy()
        if items is not None:  # some signature failed: its record, for the ASCII-hex retry
            recs = np.frombuffer(items, dtype=np.uint8).reshape(-1, 160)
    else:
        status = (pre_status if pre_status is not None else vfut.result() if vfut is not None else
                  validate._verify(rec_bytes, None) if n_jobs else np.zeros(0, np.uint8)).copy()
    retry = np.nonzero(status == op.INVALID)[0]
    if len(retry):
        signed_len = _i32(d, 'signed_len')
        rr = recs[retry].copy()
        txs_retry = job_tx[retry].astype(np.int64)
        # one native batch (host pool) of SHA-256 over the signed prefix of each failing tx's hex text:
        # a hostile block full of bad signatures costs one pass, not a Python loop per signature
        hx, at = d['hex'], txs_retry
        if not isinstance(hx, list):  # a HexSpans: str objects for the failing txs only
            hx, at = [hx[k] for k in txs_retry.tolist()], np.arange(len(txs_retry), dtype=np.int64)
        rr[:, 128:] = np.frombuffer(lib().sha256_hex_prefixes(hx, at, 2 * signed_len[txs_retry].astype(np.int64),
                                                              THREADS), np.uint8).reshape(-1, 32)
        st2 = validate._verify(np.ascontiguousarray(rr).tobytes(), None)
        status[retry] = np.where(st2 == op.VALID, op.VALID, status[retry])
    if np.any(status != op.VALID):
        bad = np.nonzero(status != op.VALID)[0]
        if np.all(status[bad] == op.INVALID):
            # plainly invalid signatures (under both message forms) with every other rule of every tx held:
            # the object path stops at the first such tx in block order (manager.py create_block →
            # verify_block_transactions) with this message. Deciding it here spares a hostile block full of
            # bad signatures the per-tx Python re-validation.
            k = int(job_tx[bad].min())
            error_list.append(error := f'transaction {txid[k].tobytes().hex()} has been not verified')
            logger.error(error)
            return False
        return None  # malformed keys or out-of-range scalars: the object path raises what the reference raises
    # the merkle root was computed on the codec's thread while the stages above ran
    if d['merkle_job'].result() != merkle_tree:
        return None
    t4 = perf_counter()
    roctx.pop()
    roctx.push('block:apply')

    fees_total = Decimal(int(fee.sum())) / SMALLEST
    validate.timings.update({'decompress_s': t3 - t_gov, 'collect_s': 0.0, 'ecdsa_s': t4 - t3,
                             'rules_s': t_gov - t2, 'strings_s': strings_s, 'signatures': n_jobs, 'txs': n})
    metrics.inc('upow_signatures_verified_total', n_jobs, help='P-256 signatures verified in block validation')
    manager.last_block_timings.update({'utxo_s': t2 - t1, 'verify_s': t4 - t2, 'merkle_s': 0.0,
                                       'total_s': t4 - t0, 'txs': n})

    async def apply(block_hash, address, random, block_reward, content_time, coinbase_transaction):
        ta = perf_counter()
        roctx.push('apply:coinbase')
        from .database import numeric
        block_row = {'id': block_no, 'hash': block_hash, 'content': block_content, 'address': address,
                     'random': int(random), 'difficulty': numeric(difficulty, 1),
                     'reward': numeric(block_reward + fees_total, 6), 'timestamp': int(content_time)}
        # a sync page's plan already split the trusted coinbase and built its index records (pagesync)
        pre_cb = coinbase_transaction.__dict__.get('_upow_cb_index')
        cb_outputs = pre_cb[0] if pre_cb else Database.split_outputs([coinbase_transaction])['unspent_outputs']
        submitted = database._submitted
        roctx.pop()
        try:
            if lean:
                seq = database.apply_lean_block(block_row, cb_outputs, n, out_cols, in_keys, pay, txid, gov=gov_cols,
                                                cb_index=pre_cb[1:] if pre_cb else None)
            else:
                cb_row = await database._tx_row(coinbase_transaction, block_hash)
                seq = database.apply_native_block(block_row, cb_row, cb_outputs, n, tx_cols, out_cols, in_keys, pay,
                                                  gov=gov_cols, addr_pairs=addr_pairs,
                                                  cb_index=pre_cb[1:] if pre_cb else None)
        except Exception as e:
            if database._submitted != submitted:
                raise  # committed to the journal: a failure after the commit point is not a rejection
            logger.error(f'Transaction of {block_no} has not been added in block {e}')
            manager.Manager.difficulty = None
            return False
        timings.update(getattr(database, 'last_apply_stages', {}))
        timings.update({'apply_commit_s': perf_counter() - ta, 'journal_seq': seq,
                        'gov_index_s': getattr(database, 'last_gov_index_s', 0.0) if gov_cols is not None else 0.0})
        return True

    if coinbase is not None:
        res = await manager._finalize_sync_block(block_no, block_content, fees_total, n, apply, coinbase, t0)
    else:
        res = await manager._finalize_block(block_no, block_content, fees_total, n, apply, error_list, t0)
    timings.update({'decode_to_checks_s': t1 - t0, 'apply_s': perf_counter() - t4})
    return res


__all__ = ['create_block_from_hex', 'decode']
