"""Page-batched chain sync: a ``/get_blocks`` page validated as one batch, applied block by block.

reference: ``create_blocks`` (upow/node/main.py:97-150) applies a page of up to 1,000 blocks one after
another, each through ``create_block_in_syncing_old`` → ``check_block`` (upow/manager.py:422-647,
760-835): every block pays its own UTXO round trips and verifies its signatures one at a time
(manager.py:628-632). Mainnet blocks are small (1-200 txs), so on the GPU path of ``ledger/fastpath.py``
each block would pay the verify kernel's ~1.2 ms latency floor for a handful of signatures, plus a device
round trip per UTXO pass and per index update.

Here a page is cut into chunks of ``CHUNK`` blocks (default 128). For each chunk:

  1. decode (csrc/txcodec.cpp) — on a helper thread, while the previous chunk is being applied;
  2. a *plan* over the whole chunk (:func:`build_plan`): ONE HBM lookup of every input of the chunk, then
     each input is resolved either from that pre-chunk index or from the outputs of an earlier block of the
     chunk (its payload computed exactly as the apply will insert it), checked unique across the chunk, and
     every signature of every eligible block is verified in ONE batched launch (on a multi-GPU cluster node
     each rank verifies a contiguous shard, then one all-gather of status bytes: ``parallel/verify_dp.py``).
     Signature validity depends on the state only through the signer key, the address of the spent output,
     which is immutable once created; the plan resolves it before any block of the chunk is applied;
  3. the blocks are applied in order through the ordinary native path with the plan's UTXO pass and
     verdicts (``fastpath.create_block_from_hex(page=...)``): header, difficulty, fees, merkle, coinbase and
     the ledger writes are per block as before. The HBM index writes of the page are deferred
     (``UtxoIndex.defer_block``) and reach the device as one insert and one erase launch;
  4. durability is one journal fdatasync for the whole page (``Database.group_commit``): a crash loses at
     most the unsynced tail of the page, and the node fetches it again after the restart (it resumes at its
     last durable block, like any sync).

A block the plan cannot vouch for — governance txs, an input it cannot resolve, a double spend, an
off-curve key, an undecodable tx — takes the ordinary per-block path (``page=None``), which settles the
deferred index writes first and reproduces the reference's verdict exactly. After a block whose effects the
plan did not model (the object path), the rest of the chunk is planned again against the settled index.
"""
from __future__ import annotations

import asyncio
import os
from dataclasses import dataclass
from time import perf_counter, process_time
from typing import List, Optional

import numpy as np

from ..ops import p256 as op
from ..ops.native import gpu_available, lib
from ..utils.codec import OutputType, TransactionType
from ..utils.hexspans import HexSpans
from ..utils.logger import get_logger
from .utxo import MISSING, PAYLOAD_DTYPE, TAG_BY_TABLE, make_payload, pack_records

logger = get_logger(__name__)

ENABLED = os.environ.get('UPOW_PAGE_SYNC', '1') != '0'
CHUNK = max(1, int(os.environ.get('UPOW_SYNC_CHUNK', '128')))
# UPOW_SHARD_KEYS=0: every cluster rank decompresses and checks ALL of a chunk's keys (the A/B of the shard)
SHARD_KEYS = os.environ.get('UPOW_SHARD_KEYS', '1') != '0'
TAG_U = TAG_BY_TABLE['unspent_outputs']
_REVOKE = (int(TransactionType.REVOKE_AS_VALIDATOR), int(TransactionType.REVOKE_AS_DELEGATE))
_HASH_MUL = np.uint64(0x9E3779B97F4A7C15)
stats: dict = {}  # last page: blocks by path, plans, signatures (bench, /metrics)


@dataclass
class PageBlock:
    """One block's share of a chunk plan: its inputs' table tags and payloads (as the HBM UTXO pass would
    return them at this block), per-tx fees, and its verify records with their precomputed statuses."""
    tags: np.ndarray
    pay: np.ndarray
    fee: np.ndarray
    n_jobs: int
    recs: Optional[bytes]  # None on a cluster rank that built the records of its own verify shard only
    status: np.ndarray


@dataclass
class Item:
    block: dict  # the /get_blocks entry's block row (id, hash, content, ...)
    all_hexes: list  # every tx of the entry, coinbase included
    hexes: list  # the txs without the trusted coinbase
    cb_hex: Optional[str]  # the coinbase candidate's hex (flag 3), parsed on the ledger thread
    dec: Optional[dict]  # fastpath.decode(hexes), None when the block needs the object path


def _i32(d, k):
    return np.frombuffer(d[k], dtype=np.int32)


def _coinbase_index(hexes: List[str]) -> Optional[int]:
    """The first tx the codec flags as a coinbase (specifier 36, whatever bytes follow it: the reference's
    parser, transaction.py:548-555, and txdecode.h TX_COINBASE). A well-formed coinbase ends in its specifier,
    so the txs whose hex ends in 24 are asked first; the txs before the first such coinbase (all of them when
    there is none) are then decoded for their flags, so a coinbase with trailing bytes ahead of it is still
    the one split off, as the reference and ``node/main.py _scan_sync_block`` split it."""
    from .fastpath import THREADS, decode_raw
    L = lib()
    if isinstance(hexes, HexSpans):  # the tails read from the body: a str only for the candidates
        tails = hexes.tail2() + [h[-2:].encode() for h in hexes.extra]
        cand = [k for k, t in enumerate(tails) if t == b'24']
    else:
        cand = [k for k, h in enumerate(hexes) if h.endswith('24')]
    first = None
    for k in cand:
        if L.decode_block_txs([hexes[k]], 1)['flags'][0] == 3:
            first = k
            break
    upto = len(hexes) if first is None else first
    if upto:
        flags = decode_raw(hexes[:upto], 1 if upto < 512 else THREADS)['flags']
        k = next((i for i, f in enumerate(flags) if f == 3), None)
        if k is not None:
            return k
    return first


def prepare(info: dict) -> Item:
    """Host-thread half of a block (no ledger state): split off the coinbase candidate, decode the rest,
    and finish the merkle root now (the codec's workspace goes back to its pool)."""
    from . import fastpath
    txs = info['transactions']
    hexes = txs if isinstance(txs, HexSpans) else list(txs)
    k = _coinbase_index(hexes)
    cb_hex = None
    if k is not None:
        cb_hex = hexes[k]
        hexes = hexes[:k] + hexes[k + 1:]
    # an empty block decodes too (n = 0): it then takes the native path like the others, and the plan models
    # its coinbase outputs instead of re-planning after it
    dec = fastpath.decode(hexes, threads=1 if len(hexes) < 512 else fastpath.THREADS)
    if dec is not None:
        dec['merkle_job'].result()
    return Item(info['block'], txs if isinstance(txs, HexSpans) else list(txs), hexes, cb_hex, dec)


def _key64(keys36: np.ndarray) -> np.ndarray:
    """A 64-bit hash of 36-byte outpoint keys (txid's first 8 bytes mixed with the index). Equal hashes are
    always confirmed on the full key; a collision only makes a block take the ordinary path."""
    k = np.ascontiguousarray(keys36[:, :32]).view('<u8')[:, 0]
    idx = np.ascontiguousarray(keys36[:, 32:36]).view('<u4')[:, 0].astype(np.uint64)
    with np.errstate(over='ignore'):
        return k ^ (idx + np.uint64(1)) * _HASH_MUL


def build_plan(db, items: List[Item], cbs: list, ctx=None) -> List[Optional[PageBlock]]:
    """Plan a chunk (see the module docstring). ``cbs[k]``: block k's parsed CoinbaseTransaction (or None).
    Returns one PageBlock per block, None for the blocks that take the ordinary path."""
    from ..parallel.verify_dp import shard_bounds, verify_records_dp, verify_shard_dp
    from .database import Database
    from .govcheck import OUTPUT_TABLE
    t0 = perf_counter()
    n_items = len(items)
    plan: List[Optional[PageBlock]] = [None] * n_items
    ks = [k for k, it in enumerate(items) if it.dec is not None and cbs[k] is not None]
    if not ks:
        return plan
    decs = [items[k].dec for k in ks]
    # ---- the chunk's columns, concatenated once: per-block slices of one array each, and one native call
    #      for all the chunk's output records (payloads exactly as the apply will insert them)
    tag_lut = np.full(256, MISSING, np.uint32)
    for t, table in OUTPUT_TABLE.items():
        tag_lut[t] = TAG_BY_TABLE[table]
    n_tx = np.array([int(d['n']) for d in decs], np.int64)
    n_out = np.array([len(d['out_type']) for d in decs], np.int64)
    tx_type = np.concatenate([np.asarray(d['_tx_type'], np.uint8) for d in decs])
    otype = np.concatenate([np.frombuffer(d['out_type'], np.uint8) for d in decs])
    tx_base = np.concatenate([[0], np.cumsum(n_tx)])
    out_base = np.concatenate([[0], np.cumsum(n_out)])
    # a block is governance-relevant when any tx type or any output type is not REGULAR (gov_block_mask)
    c_tt = np.concatenate([[0], np.cumsum(tx_type != 0)])
    c_ot = np.concatenate([[0], np.cumsum(otype != 0)])
    gov_blk = ((c_tt[tx_base[1:]] - c_tt[tx_base[:-1]]) + (c_ot[out_base[1:]] - c_ot[out_base[:-1]])) > 0
    cand = list(zip(ks, gov_blk.tolist()))
    txid_all = np.concatenate([np.frombuffer(d['txid'], np.uint8).reshape(-1, 32) for d in decs])
    out_tx_g = np.concatenate([_i32(d, 'out_tx').astype(np.int64) + tx_base[i] for i, d in enumerate(decs)])
    out_idx = np.concatenate([np.arange(len(d['out_type']), dtype=np.int64) - _i32(d, 'out_start')[_i32(d, 'out_tx')]
                              for d in decs])
    tags_o = tag_lut[otype]
    rb, pb = lib().output_index_records(
        np.ascontiguousarray(txid_all[out_tx_g]), out_idx, np.ascontiguousarray(tags_o, np.uint32),
        np.concatenate([np.frombuffer(d['out_amount'], np.uint64) for d in decs]),
        np.concatenate([np.frombuffer(d['out_addr'], np.uint8) for d in decs]),
        np.concatenate([np.frombuffer(d['out_len'], np.uint8) for d in decs]), (otype == int(OutputType.STAKE)).astype(np.uint8))
    out_keys = [np.frombuffer(rb, np.uint8).reshape(-1, 40)]
    out_pay = [np.frombuffer(pb, PAYLOAD_DTYPE)]
    out_tag = [tags_o]
    out_blk = [np.repeat(np.asarray(ks, np.int32), n_out)]
    # the coinbase outputs of the chunk (trusted coinbases: unspent_outputs, as the apply writes them)
    from .database import _addr_bytes
    cb_keys, cb_amt, cb_addr, cb_stake, cb_blk, cb_rows = [], [], [], [], [], []
    for k in ks:
        rows = Database.split_outputs([cbs[k]])['unspent_outputs']
        cb_rows.append((k, len(cb_keys), rows))
        for o in rows:
            cb_keys.append((o[0], o[1]))
            cb_amt.append(o[4])
            cb_addr.append(_addr_bytes(o[2]))
            cb_stake.append(bool(o[3]))
            cb_blk.append(k)
    if cb_keys:
        cb_recs, cb_pay = pack_records(cb_keys, TAG_U), make_payload(cb_amt, cb_addr, cb_stake)
        out_keys.append(cb_recs)
        out_pay.append(cb_pay)
        out_tag.append(np.full(len(cb_keys), TAG_U, np.uint32))
        out_blk.append(np.asarray(cb_blk, np.int32))
        # the apply of each block reuses its coinbase's rows and index records (fastpath apply)
        for k, at, rows in cb_rows:
            cbs[k].__dict__['_upow_cb_index'] = (rows, cb_recs[at:at + len(rows)], cb_pay[at:at + len(rows)])
    in_keys = [np.frombuffer(d['in_keys'], np.uint8).reshape(-1, 40) for d in decs]
    in_blk = [np.full(len(ik), k, np.int32) for k, ik in zip(ks, in_keys)]
    IK = np.ascontiguousarray(np.concatenate(in_keys))
    BI = np.concatenate(in_blk)
    OK_ = np.ascontiguousarray(np.concatenate(out_keys))
    OB = np.concatenate(out_blk)
    OT = np.concatenate(out_tag)
    OP = np.concatenate(out_pay)
    ni = len(IK)
    # ---- 1. the pre-chunk index: one lookup launch for every input
    tags_h, pay_h = db.utxo.lookup_records(IK) if ni else (np.zeros(0, np.uint8), np.zeros(0, PAYLOAD_DTYPE))
    tags = np.asarray(tags_h, np.uint32).copy()
    pay = np.array(pay_h, dtype=PAYLOAD_DTYPE)
    hit = (tags != MISSING) & (pay['len'] > 0)
    bad = np.zeros(ni, bool)
    # ---- 2. the rest from the chunk's own outputs, created by an EARLIER block
    miss = np.nonzero(~hit)[0]
    if len(miss) and len(OK_):
        ok64 = _key64(OK_)
        order = np.argsort(ok64, kind='stable')
        s64 = ok64[order]
        q = _key64(IK[miss])
        lo = np.searchsorted(s64, q, 'left')
        hi = np.searchsorted(s64, q, 'right')
        one = (hi - lo) == 1
        pos = order[np.minimum(lo, len(order) - 1)]
        same = one & np.all(OK_[pos, :36] == IK[miss, :36], axis=1)
        earlier = OB[pos] < BI[miss]
        res = same & earlier
        r = miss[res]
        tags[r] = OT[pos[res]]
        pay[r] = OP[pos[res]]
        hit[r] = True
        bad[miss[(hi - lo) > 1]] = True  # a hash collision among the outputs: no claim either way
    # ---- 3. every outpoint spent once in the chunk (a second spend is a double spend at its block)
    if ni > 1:
        k64 = _key64(IK)
        order = np.argsort(k64, kind='stable')  # stable: equal keys keep chunk order
        s = k64[order]
        eq = np.nonzero(s[1:] == s[:-1])[0]
        if len(eq):
            a, b = order[eq], order[eq + 1]
            bad[a] |= True  # conservative: both sides of a repeated (or colliding) key take the ordinary path
            bad[b] |= True
    ok_in = hit & ~bad & (tags == TAG_U)
    # ---- 4. eligible blocks: plain (no governance txs or outputs), every input resolved, live and unique
    starts = {}
    pos0 = 0
    for k, _ in cand:
        n_in = len(np.frombuffer(items[k].dec['in_keys'], np.uint8)) // 40
        starts[k] = (pos0, pos0 + n_in)
        pos0 += n_in
    elig = [k for k, anyg in cand if not anyg and bool(np.all(ok_in[starts[k][0]:starts[k][1]]))]
    if not elig:
        _record(t0, len(cand), 0, 0)
        return plan
    # ---- 5. the eligible blocks' signature jobs, records and ONE verify
    pa, pl, oa, ol, ji, sg, sid, dg, jt, per = [], [], [], [], [], [], [], [], [], []
    in_base = tx_base = sig_base = job_base = 0
    fees = {}
    keep = []
    for k in elig:
        d = items[k].dec
        a, b = starts[k]
        bpay = pay[a:b]
        in_start, out_start = _i32(d, 'in_start'), _i32(d, 'out_start')
        job_input = _i32(d, 'sig_first_in').astype(np.int64)
        grouped = np.nonzero(np.frombuffer(d['grouped'], dtype=np.uint8))[0] if 'grouped' in d else ()
        if len(grouped):
            from .fastpath import _resolve_groups
            job_input = _resolve_groups(grouped, job_input, bpay, in_start, _i32(d, 'sig_start'), d['_tx_type'])
            if job_input is None:
                continue
        n_tx = int(d['n'])
        in_tx = _i32(d, 'in_tx')
        amt_in = bpay['amount'].astype(np.int64)
        amt_out = np.frombuffer(d['out_amount'], np.uint64).astype(np.int64)
        cs_in = np.concatenate([[0], np.cumsum(amt_in)])
        cs_out = np.concatenate([[0], np.cumsum(amt_out)])
        fees[k] = (cs_in[in_start[1:]] - cs_in[in_start[:-1]]) - (cs_out[out_start[1:]] - cs_out[out_start[:-1]])
        nj = len(job_input)
        pa.append(np.ascontiguousarray(bpay['addr']))
        pl.append(bpay['len'].astype(np.uint8))
        oa.append(np.frombuffer(d['out_addr'], np.uint8).reshape(-1, 64))
        ol.append(np.frombuffer(d['out_len'], np.uint8))
        ji.append(in_base + job_input)
        jt.append(tx_base + in_tx[job_input].astype(np.int64))
        sg.append(np.frombuffer(d['sigs'], np.uint8).reshape(-1, 64))
        sid.append(sig_base + np.arange(nj, dtype=np.int64))
        dg.append(np.frombuffer(d['digest'], np.uint8).reshape(-1, 32))
        per.append((k, job_base, job_base + nj, a, b))
        keep.append(k)
        in_base += b - a
        tx_base += n_tx
        sig_base += len(sg[-1])
        job_base += nj
    if not keep:
        _record(t0, len(cand), 0, 0)
        return plan
    gpu_min = op.GPU_MIN_BATCH if gpu_available() else 1 << 62
    n_jobs = job_base
    cpu0 = process_time()  # host CPU of the P-256 work (key decompression, curve checks, verify) of the plan
    p_addr, p_len = np.ascontiguousarray(np.concatenate(pa)), np.concatenate(pl)
    o_addr, o_len = np.ascontiguousarray(np.concatenate(oa)), np.concatenate(ol)
    ji_all, sid_all, jt_all = np.concatenate(ji), np.concatenate(sid), np.concatenate(jt)
    sigs_all, dg_all = np.ascontiguousarray(np.concatenate(sg)), np.ascontiguousarray(np.concatenate(dg))
    sharded = ctx is not None and ctx.is_distributed and SHARD_KEYS
    if sharded:
        # each rank decompresses and curve-checks a shard of the chunk's keys only: the signer keys of its
        # verify shard, its shard of the spent outputs' owners and its shard of the new outputs. The shards
        # cover every key of the chunk, so the MIN of the ranks' verdicts below is the whole chunk's verdict;
        # each rank ends up with the records of its own verify shard, which is all it verifies
        lo, hi = shard_bounds(n_jobs, ctx.world, ctx.rank)
        ilo, ihi = shard_bounds(len(p_len), ctx.world, ctx.rank)
        olo, ohi = shard_bounds(len(o_len), ctx.world, ctx.rank)
        sub = np.concatenate([ji_all[lo:hi], np.arange(ilo, ihi, dtype=np.int64)])
        kst, rec_bytes = lib().block_signer_records(
            np.ascontiguousarray(p_addr[sub]), np.ascontiguousarray(p_len[sub]), np.ascontiguousarray(o_addr[olo:ohi]),
            np.ascontiguousarray(o_len[olo:ohi]), np.arange(hi - lo, dtype=np.int64), sigs_all, sid_all[lo:hi],
            dg_all, jt_all[lo:hi], gpu_min)
        # one 24-byte all-reduce: the replicas planned the same chunk (a difference would desynchronise the
        # sharded verify) and the chunk's key verdict (-1 a 64-byte address, 0 off the curve, 1 all good)
        mn = ctx.allreduce_min_vec([n_jobs, -n_jobs, kst])
        if mn[0] != -mn[1]:
            raise RuntimeError(f'page plan differs across cluster replicas ({n_jobs} jobs here)')
        kst = int(mn[2])
    elif n_jobs or len(o_len):
        kst, rec_bytes = lib().block_signer_records(p_addr, p_len, o_addr, o_len, ji_all, sigs_all, sid_all, dg_all,
                                                    jt_all, gpu_min)
        if ctx is not None and ctx.is_distributed:
            lo_hi = ctx.allreduce_min_vec([n_jobs * 4 + (kst + 1), -(n_jobs * 4 + (kst + 1))])
            if lo_hi[0] != -lo_hi[1]:
                raise RuntimeError(f'page plan differs across cluster replicas ({n_jobs} jobs, kst {kst} here)')
    else:  # empty blocks only: nothing to check or verify
        kst, rec_bytes = 1, b''
    if kst != 1:  # an off-curve key or a 64-byte address among the chunk's keys: the ordinary path decides
        _record(t0, len(cand), 0, n_jobs)
        return plan
    recs = np.frombuffer(rec_bytes, np.uint8).reshape(-1, 160)
    tv = perf_counter()
    if n_jobs == 0:
        status = np.zeros(0, np.uint8)
    elif sharded:
        status = verify_shard_dp(ctx, recs.reshape(-1), n_jobs)
    elif ctx is not None and ctx.is_distributed:
        status = verify_records_dp(ctx, recs.reshape(-1))
    else:
        status = op.verify_records(recs.reshape(-1))
    verify_s = perf_counter() - tv
    stats['plan_crypto_cpu_s'] = stats.get('plan_crypto_cpu_s', 0.0) + (process_time() - cpu0)
    tags_u = np.full(ni, TAG_U, np.uint8)
    for k, j0, j1, a, b in per:
        st = np.asarray(status[j0:j1], np.uint8)
        if sharded:
            if np.any(st != op.VALID):  # its retry needs records other ranks hold: the ordinary path decides
                continue
            rb = None
        else:
            rb = recs[j0:j1].tobytes()
        plan[k] = PageBlock(tags=tags_u[a:b], pay=pay[a:b], fee=fees[k], n_jobs=j1 - j0, recs=rb, status=st)
    _record(t0, len(cand), len(keep), n_jobs, verify_s)
    return plan


def _record(t0: float, cand: int, planned: int, sigs: int, verify_s: float = 0.0):
    stats['plans'] = stats.get('plans', 0) + 1
    stats['planned_blocks'] = stats.get('planned_blocks', 0) + planned
    stats['candidate_blocks'] = stats.get('candidate_blocks', 0) + cand
    stats['plan_signatures'] = stats.get('plan_signatures', 0) + sigs
    stats['plan_s'] = stats.get('plan_s', 0.0) + (perf_counter() - t0)
    stats['plan_verify_s'] = stats.get('plan_verify_s', 0.0) + verify_s


_POOL = None


def _pool():
    global _POOL
    if _POOL is None:
        from concurrent.futures import ThreadPoolExecutor
        _POOL = ThreadPoolExecutor(max_workers=1, thread_name_prefix='upow-page-decode')
    return _POOL


def _prepare_chunk(infos: List[dict]) -> List[Item]:
    return [prepare(i) for i in infos]


async def create_blocks(blocks: list, error_list: list = None, mirror: bool = True) -> bool:
    """node/main.py ``create_blocks`` (reference main.py:97-150) for a whole page; see the module docstring.
    On a cluster leader the page goes to the followers first as ONE 'page' op; every rank then runs this same
    procedure (its chunk plans sharding the signatures over the GPUs, every block agreed before it commits)."""
    from ..models.transaction import CoinbaseTransaction, Transaction
    from ..models.block import block_to_bytes, get_transactions_merkle_tree
    from ..parallel import cluster
    from . import fastpath, manager
    from .database import Database
    from ..constants import GENESIS_PREV_HASH
    if error_list is None:
        error_list = []
    c = cluster.get()
    ctx = None
    if c is not None and not c.replaying:
        ctx = c.op_ctx
        if c.leader and mirror:
            cluster.flush_txs()
            c.send_page(blocks)
    db: Database = Database.instance
    _, last_block = await manager.calculate_difficulty()
    last_block['id'] = last_block['id'] if last_block != {} else 0
    last_block['hash'] = last_block['hash'] if 'hash' in last_block else GENESIS_PREV_HASH
    i = last_block['id'] + 1
    loop = asyncio.get_running_loop()
    pool = _pool()
    chunks = [blocks[a:a + CHUNK] for a in range(0, len(blocks), CHUNK)]
    ahead = loop.run_in_executor(pool, _prepare_chunk, chunks[0]) if chunks else None
    page_stats = {'blocks': 0, 'page_path': 0, 'ordinary_path': 0, 'replans': 0}
    db.group_commit += 1
    db.utxo_defer = True
    try:
        for ci in range(len(chunks)):
            items = await ahead
            ahead = loop.run_in_executor(pool, _prepare_chunk, chunks[ci + 1]) if ci + 1 < len(chunks) else None
            cbs = []
            for it in items:
                cb = None
                if it.cb_hex is not None:
                    cand = await Transaction.from_hex(it.cb_hex)
                    if isinstance(cand, CoinbaseTransaction):
                        cb = cand
                    else:  # not what the scan assumed: the whole block goes through the ordinary decode
                        it.hexes = it.all_hexes[:]
                        it.dec = None
                cbs.append(cb)
            plan = build_plan(db, items, cbs, ctx)
            tc = perf_counter()
            n_page = page_stats['page_path']
            k = 0
            while k < len(items):
                it = items[k]
                block = it.block
                block_content = block.get('content')
                if not block_content:
                    txs = [await Transaction.from_hex(h) for h in it.hexes]
                    block['merkle_tree'] = get_transactions_merkle_tree([tx.hex() for tx in txs])
                    block_content = block_to_bytes(last_block['hash'], block)
                assert i == block['id'], (i, block['id'])
                if cbs[k] is None:
                    # a sync block carries its coinbase (create_block_in_syncing_old dereferences it,
                    # reference manager.py:790): without one the page stops here, as the reference's sync does.
                    # It never reaches the push variant, and the plan never modelled it (build_plan only plans
                    # blocks with a coinbase), so no later block of the chunk is applied on a stale plan
                    error_list.append(error := f'block {block["id"]} has no coinbase transaction')
                    logger.error(error)
                    return False
                pb = plan[k]
                if not await fastpath.create_block_from_hex(
                        block_content.hex() if isinstance(block_content, bytes) else block_content, it.hexes,
                        error_list=error_list, last_block=last_block, coinbase=cbs[k], mirror=False, decoded=it.dec,
                        page=pb):
                    return False
                page_stats['blocks'] += 1
                used = pb is not None and fastpath.last_path == 'native'
                page_stats['page_path' if used else 'ordinary_path'] += 1
                last_block = block
                i += 1
                k += 1
                if not used and (it.dec is None or fastpath.last_path != 'native') and k < len(items):
                    # the object path applied this block: its effects are not what the plan modelled, so the
                    # rest of the chunk is planned again against the settled index
                    page_stats['replans'] += 1
                    rest = build_plan(db, items[k:], cbs[k:], ctx)
                    plan = plan[:k] + rest
            logger.info(f'Synced blocks {items[0].block["id"]}..{items[-1].block["id"]} '
                        f'({page_stats["page_path"] - n_page} on the page plan) in {perf_counter() - tc:.3f} s')
        return True
    finally:
        if ahead is not None:  # a failed page: let the helper thread's decode finish before returning
            try:
                await ahead
            except Exception:
                pass
        db.utxo_defer = False
        db.group_commit -= 1
        db.utxo.settle()
        if db.group_commit == 0:
            db.wait_durable(force=True)  # the page's one fdatasync
        stats.update(page_stats)


__all__ = ['ENABLED', 'CHUNK', 'PageBlock', 'build_plan', 'create_blocks', 'prepare', 'stats']
