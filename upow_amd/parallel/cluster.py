"""Multi-GPU node: one process per GPU, every rank holds a full ledger replica in its own HBM.

SURVEY.md §2.6 "State replication" + "DP: tx-verify batch parallelism". The reference is one
process with one PostgreSQL; here ``torchrun --nproc-per-node G -m upow_amd.node --cluster``
starts G ranks:

* rank 0 (the leader) serves the REST/WebSocket API exactly like a single-GPU node;
* ranks 1..G-1 (followers) keep a file-backed ledger replica (``<data>/rank<N>/``: journal, undo segments,
  UTXO snapshot) plus their HBM UTXO index, and apply every ledger mutation the leader makes, in the
  same order, from an op stream the leader broadcasts over RCCL:

      resync    start-up: every rank reports (tip, tip hash); divergent replicas roll back to the last
                common block (``fork_window``: the leader's recent block hashes); then only the blocks
                above the lowest replica tip are re-sent (``replay_block``), each follower applying the
                ones above its own tip — a restart costs the missing tail, not the chain
      mempool_reset / txs   the leader's mempool rows (hex, input addresses, fees, propagation time,
                reserved inputs) replicated as they were ADMITTED on the leader: followers insert them
                without re-verifying (the leader already did), in one native index pass + one journal batch
      block     a block to validate + apply (push or sync form, tx hex + optional coinbase)
      gc        mempool garbage collection
      rollback / delete   fork handling (remove_blocks / delete_blocks)
      status    all-gather of every replica's (height, tip hash, UTXO-set K12 hash from the index)
      ping      idle heartbeat (keeps followers inside the op group's collective timeout)
      quit

Ordering and threads. Every collective of a rank is issued by ONE thread (``DistContext.bind_owner``):
the leader's ledger thread, the follower's op loop. ``/cluster_info`` and the idle heartbeat are routed
through the ledger thread; admissions on the HTTP loop only append to an outbox, which the ledger thread
ships as ONE 'txs' op every ``UPOW_CLUSTER_TX_FLUSH_MS`` and always right before any other op. A row
admitted on the leader while a block was being applied is edited in the outbox exactly as the block's
mempool confirm edited the leader's index (its tx dropped if the block confirmed it, confirmed inputs
stripped), so a follower that inserts it after that block ends in the leader's state.

Verification. Each replica validates every block itself; an all-reduce then checks that all replicas
reached the same verdict (a split raises: replica divergence). The signature batch is sharded across
the ranks only from ``UPOW_CLUSTER_SHARD_MIN`` signatures up (ledger/validate.py): a 2 MB block (~8,300
signatures) verifies in ~1.2 ms on one GPU, less than a sharded verify costs in collectives.
"""
from __future__ import annotations

import json
import os
import threading
import time
from typing import List, Optional

from ..utils.logger import get_logger
from .dist import DistContext

logger = get_logger(__name__)

_cluster: Optional['Cluster'] = None
HEARTBEAT_S = float(os.environ.get('UPOW_CLUSTER_HEARTBEAT_S', '5'))
FORK_WINDOW = 500  # remove_blocks' reach (reference database.py:146-169 pages of 500)


class Cluster:
    def __init__(self, ctx: DistContext, init_ctx: Optional[DistContext] = None):
        self.ctx = ctx  # op traffic (short timeout group)
        self.init_ctx = init_ctx or ctx  # start-up barrier (long timeout group)
        self.replaying = False
        self.closed = False  # after 'quit': no op is sent again (the heartbeat stops)
        self.last_send = time.monotonic()
        self.ops_sent = 0
        self.last_resync: Optional[dict] = None

    @property
    def leader(self) -> bool:
        return self.ctx.rank == 0

    # ------------------------------------------------------------------ op stream
    # One frame per op: u32 header length, a small JSON header, then a binary payload (a block's txs
    # travel as raw bytes, half the size of hex and no JSON string escaping): two broadcasts per op
    # (length, then frame) over RCCL, both from the owner thread.
    def send(self, op: str, payload: bytes = b'', **kw):
        assert self.leader
        head = json.dumps({'op': op, **kw}, separators=(',', ':')).encode()
        self.ctx.broadcast_bytes(len(head).to_bytes(4, 'little') + head + payload, src=0, max_len=0)
        self.last_send = time.monotonic()
        self.ops_sent += 1

    def recv(self) -> dict:
        raw = self.ctx.broadcast_bytes(None, src=0, max_len=0)
        n = int.from_bytes(raw[:4], 'little')
        msg = json.loads(raw[4:4 + n].decode())
        msg['_payload'] = raw[4 + n:]
        return msg

    def agree(self, ok: bool, what: str) -> bool:
        n = self.ctx.allreduce_sum(1 if ok else 0)
        if n not in (0, self.ctx.world):
            raise RuntimeError(f'cluster replicas diverged on {what}: {n}/{self.ctx.world} accepted')
        return bool(ok)

    def status(self, db, deep: bool = False, mempool: Optional[int] = None) -> List[dict]:
        """Collective: every rank's height, tip hash and UTXO-set hash. The hash comes from the HBM index
        (K12: compaction + radix sort on the device, host SHA tail), current at the commit point; ``deep``
        also hashes the SQL replica after the materialisers have caught up (the slow full-table audit)."""
        mine = {'rank': self.ctx.rank, 'height': db._tip_id(), 'tip_hash': _tip_hash(db),
                'utxo_hash': db.utxo.set_hash(_utxo_tag()), 'utxo_entries': len(db.utxo),
                'mempool': _mempool_size(db) if mempool is None else mempool}
        if deep:
            db.flush()
            mine['sql_utxo_hash'] = db.sql_unspent_outputs_hash()
        return [json.loads(b.decode()) for b in self.ctx.all_gather_bytes(json.dumps(mine).encode())]


def _utxo_tag() -> int:
    from ..ledger.utxo import TAG_BY_TABLE
    return TAG_BY_TABLE['unspent_outputs']


def _tip_hash(db) -> Optional[str]:
    tip = db._tip_id()
    if not tip:
        return None
    row = db._q1('SELECT hash FROM blocks WHERE id = ?', (tip,))
    return row[0] if row else None


def _mempool_size(db) -> int:
    mp = db._mempool()
    if mp is not None:
        return len(mp)
    return int(db._q1('SELECT COUNT(*) FROM pending_transactions')[0])


def pack_txs(tx_hexes) -> bytes:
    """Raw tx bytes of a block: u32 count, then u32 length + bytes per tx (hex-decoded natively on the
    host pool, csrc/txcodec.cpp ``pack_tx_hexes``)."""
    from ..ops.native import lib
    return lib().pack_tx_hexes(list(tx_hexes), _threads())


def unpack_txs(buf: bytes) -> List[str]:
    from ..ops.native import lib
    return lib().unpack_tx_hexes(bytes(buf), _threads())


def _threads() -> int:
    from ..ledger.fastpath import THREADS
    return THREADS


def init(ctx: DistContext, init_ctx: Optional[DistContext] = None) -> Optional[Cluster]:
    global _cluster
    _cluster = Cluster(ctx, init_ctx) if ctx.is_distributed else None
    return _cluster


def get() -> Optional[Cluster]:
    return _cluster


def active_leader() -> Optional[Cluster]:
    c = _cluster
    return c if (c is not None and c.leader and not c.replaying and not c.closed) else None


# ---------------------------------------------------------------------------------------------- leader hooks
# Replicated mempool rows: (tx_hex, inputs_addresses JSON, fees text, propagation time, [[txid, index], ...])
_outbox: List[list] = []
_outbox_lock = threading.Lock()
_flush_scheduled = False
FLUSH_S = float(os.environ.get('UPOW_CLUSTER_TX_FLUSH_MS', '20')) / 1000.0


def on_admit(row: list):
    """Database hook (``Database.on_admit``): a tx admitted to the leader's mempool, called under the
    mempool index lock on any thread. Queued for the next 'txs' op; never waits for a collective."""
    global _flush_scheduled
    if active_leader() is None:
        return
    with _outbox_lock:
        _outbox.append(row)
        if _flush_scheduled:
            return
        _flush_scheduled = True
    _on_ledger_loop(lambda loop: loop.call_later(FLUSH_S, _timed_flush), _timed_flush)


def on_confirm(hit_tx: list, hit_in: list):
    """Database hook (``Database.on_confirm``, under the mempool index lock): a block's confirm removed
    ``hit_tx`` (raw tx hashes) and ``hit_in`` (raw 36-byte outpoints) from the leader's index. Rows still
    in the outbox were admitted before that confirm, so the followers must see them as the confirm left
    them: the confirmed tx dropped, the confirmed inputs no longer reserved."""
    if not _outbox:
        return
    import hashlib
    txs = set(hit_tx)
    ins = {(k[:32].hex(), int.from_bytes(k[32:36], 'little')) for k in hit_in}
    with _outbox_lock:
        keep = []
        for row in _outbox:
            if hashlib.sha256(bytes.fromhex(row[0])).digest() in txs:
                continue
            if ins:
                row[4] = [p for p in row[4] if (p[0], int(p[1])) not in ins]
            keep.append(row)
        _outbox[:] = keep


def _on_ledger_loop(schedule, fallback):
    """Run ``schedule(loop)`` on the ledger thread's loop (the collective owner); without a ledger thread
    on the running loop; with no loop at all call ``fallback()`` now."""
    import asyncio
    from ..ledger import worker
    w = worker.get()
    if w is not None:
        w.loop.call_soon_threadsafe(lambda: schedule(w.loop))
        return
    try:
        schedule(asyncio.get_running_loop())
    except RuntimeError:
        fallback()


def _timed_flush():
    global _flush_scheduled
    with _outbox_lock:
        _flush_scheduled = False
    flush_txs()


def flush_txs() -> int:
    """Ship the queued mempool rows to the followers as one 'txs' op (owner thread)."""
    c = active_leader()
    with _outbox_lock:
        rows = list(_outbox)
        _outbox.clear()
    if c is None or not rows:
        return 0
    c.send('txs', json.dumps(rows, separators=(',', ':')).encode())
    return len(rows)


def _heartbeat():
    """Idle ping every HEARTBEAT_S on the owner thread, so followers waiting for the next op never reach
    the op group's collective timeout."""
    import asyncio
    c = active_leader()
    if c is None:
        return
    if time.monotonic() - c.last_send >= HEARTBEAT_S:
        c.send('ping')
    asyncio.get_running_loop().call_later(HEARTBEAT_S / 2, _heartbeat)


async def mirror_gc(pending):
    """Mempool GC on every replica (manager.clear_pending_transactions)."""
    from ..ledger.manager import clear_pending_transactions
    c = active_leader()
    if c is not None:
        flush_txs()
        c.send('gc', pending=list(pending) if pending is not None else None)
    return await clear_pending_transactions(pending)


async def mirror_rollback(db, block_no: int):
    c = active_leader()
    if c is not None:
        flush_txs()
        c.send('rollback', n=int(block_no))
    await db.remove_blocks(block_no)


async def mirror_delete(db, offset: int):
    c = active_leader()
    if c is not None:
        flush_txs()
        c.send('delete', n=int(offset))
    await db.delete_blocks(offset)


async def status_all(db, deep: bool = False) -> List[dict]:
    """``GET /cluster_info``: every replica's state (owner thread: the ledger thread)."""
    c = active_leader()
    if c is None:
        return [{'rank': 0, 'height': db._tip_id(), 'tip_hash': _tip_hash(db),
                 'utxo_hash': db.utxo.set_hash(_utxo_tag()), 'utxo_entries': len(db.utxo)}]
    # the leader's mempool keeps admitting on the HTTP loop: its size is read together with the outbox
    # drain, under the index lock the admissions hold, so it is the size the followers reach at this op
    mp = db._mempool()
    if mp is not None:
        with mp.lock:
            with _outbox_lock:
                rows = list(_outbox)
                _outbox.clear()
            size = len(mp)
        if rows:
            c.send('txs', json.dumps(rows, separators=(',', ':')).encode())
    else:
        flush_txs()
        size = None
    c.send('status', deep=bool(deep))
    return c.status(db, deep, mempool=size)


def _mempool_rows(db) -> List[list]:
    """The leader's mempool as replication rows, in admission (row) order."""
    spent = {(r[0], int(r[1])) for r in db._q('SELECT tx_hash, "index" FROM pending_spent_outputs')}
    rows = []
    for r in db._q('SELECT tx_hex, inputs_addresses, fees, propagation_time FROM pending_transactions ORDER BY rowid'):
        raw = bytes.fromhex(r[0])
        ins = [[raw[2 + 34 * k:34 + 34 * k].hex(), raw[34 + 34 * k]] for k in range(raw[1])] if len(raw) > 1 else []
        rows.append([r[0], r[1], str(r[2]), int(r[3]), [p for p in ins if (p[0], p[1]) in spent]])
    return rows


async def leader_start(db):
    """Leader start-up, ON the ledger thread: bind the collective owner, wait for every replica to open
    its ledger, resync them, then start the idle heartbeat."""
    import asyncio
    c = _cluster
    if c is None or not c.leader:
        return
    db.on_admit = on_admit
    db.on_confirm = on_confirm
    c.init_ctx.bind_owner()
    c.ctx.bind_owner()
    c.init_ctx.barrier()  # long-timeout group: followers may still be opening big ledgers
    await leader_resync(db)
    asyncio.get_running_loop().call_later(HEARTBEAT_S / 2, _heartbeat)


async def leader_resync(db) -> dict:
    """Bring every follower to the leader's chain and mempool, sending only what each lacks."""
    from ..ledger import validate
    c = _cluster
    tip = db._tip_id()
    c.replaying = True
    try:
        c.send('resync')
        st = _gather_tips(c, db)
        followers = [s for s in st if s['rank'] != 0]
        rolled_back = 0
        bad = [s for s in followers if s['tip'] > tip or (s['tip'] and _hash_at(db, s['tip']) != s['tip_hash'])]
        if bad:
            top = min(max(s['tip'] for s in bad), tip)
            lo = max(1, top - FORK_WINDOW + 1)
            win = db._q('SELECT id, hash FROM blocks WHERE id BETWEEN ? AND ? ORDER BY id', (lo, top)) if top else []
            c.send('fork_window', b''.join(bytes.fromhex(r[1]) for r in win), lo=lo, hi=top if win else 0)
            before = {s['rank']: s['tip'] for s in st}
            st = _gather_tips(c, db)
            rolled_back = sum(max(0, before[s['rank']] - s['tip']) for s in st)
            followers = [s for s in st if s['rank'] != 0]
            for s in followers:
                if s['tip'] > tip or (s['tip'] and _hash_at(db, s['tip']) != s['tip_hash']):
                    raise RuntimeError(f'cluster resync: rank {s["rank"]} still diverges after the fork window: {s}')
        start = min([s['tip'] for s in followers] + [tip])
        sent = 0
        rows = []
        offset = start + 1
        while offset <= tip:
            page = await db.get_blocks(offset, 200)
            if not page:
                break
            for info in page:
                h = info['block']['id']
                c.send('replay_block', pack_txs(info['transactions']), h=h, content=info['block']['content'])
                sent += 1
                offset = h + 1
        flush_txs()
        c.send('mempool_reset')
        rows = _mempool_rows(db)
        for k in range(0, len(rows), 512):
            c.send('txs', json.dumps(rows[k:k + 512], separators=(',', ':')).encode())
        c.send('replay_end')
    finally:
        c.replaying = False
    st = c.status(db)
    if any((s['height'], s['tip_hash'], s['utxo_hash']) != (st[0]['height'], st[0]['tip_hash'], st[0]['utxo_hash'])
           for s in st):
        raise RuntimeError(f'cluster resync left diverged replicas: {st}')
    validate.set_dist_context(c.ctx)
    c.last_resync = {'leader_tip': tip, 'follower_tips': {s['rank']: s['tip'] for s in followers},
                     'blocks_sent': sent, 'blocks_rolled_back': rolled_back, 'mempool_rows': len(rows)}
    logger.info(f'cluster: {c.ctx.world} replicas at height {tip}; resync sent {sent} block(s), '
                f'rolled back {rolled_back}, {len(rows)} mempool row(s)')
    return c.last_resync


def _hash_at(db, h: int) -> Optional[str]:
    row = db._q1('SELECT hash FROM blocks WHERE id = ?', (h,))
    return row[0] if row else None


def _gather_tips(c: Cluster, db) -> List[dict]:
    mine = json.dumps({'rank': c.ctx.rank, 'tip': db._tip_id(), 'tip_hash': _tip_hash(db)}).encode()
    return [json.loads(b.decode()) for b in c.ctx.all_gather_bytes(mine)]


async def leader_quit():
    """Tell the followers to stop (owner thread)."""
    c = _cluster
    if c is not None and c.leader and not c.closed:
        try:
            flush_txs()
            c.send('quit')
        except Exception as e:  # pragma: no cover - process group already gone
            logger.error(f'cluster quit: {e}')
        finally:
            c.closed = True


# ---------------------------------------------------------------------------------------------- follower
async def _split_coinbase(hexes):
    from ..models.transaction import CoinbaseTransaction, Transaction
    from ..ops.native import lib
    hexes = list(hexes)
    flags = lib().decode_block_txs(hexes, 1)['flags'] if hexes else b''
    for k, f in enumerate(flags):
        if f == 3:
            cand = await Transaction.from_hex(hexes[k])
            if isinstance(cand, CoinbaseTransaction):
                del hexes[k]
                return hexes, cand
    return hexes, None


async def _follower_fork_window(c: Cluster, db, msg):
    """Roll this replica back to the highest block of the window whose hash equals the leader's; with no
    common block in the window (or a rollback deeper than remove_blocks reaches) start from genesis."""
    lo, hi = int(msg['lo']), int(msg['hi'])
    ours = db._tip_id()
    leader = msg['_payload']
    common = 0
    if hi:
        mine = {int(r[0]): r[1] for r in db._q('SELECT id, hash FROM blocks WHERE id BETWEEN ? AND ?',
                                                (lo, min(hi, ours)))}
        for h in range(min(hi, ours), lo - 1, -1):
            if mine.get(h) == leader[32 * (h - lo):32 * (h - lo + 1)].hex():
                common = h
                break
    if common == ours:
        return
    if common and ours - common <= FORK_WINDOW:
        logger.info(f'cluster follower rank {c.ctx.rank}: rolling back {ours - common} block(s) to {common}')
        await db.remove_blocks(common + 1)
    else:
        logger.info(f'cluster follower rank {c.ctx.rank}: no common block in the window, rebuilding from genesis')
        await db.delete_blockchain()


async def follower_main(c: Cluster, db):
    """Apply the leader's op stream until 'quit'."""
    from ..ledger import fastpath, validate
    from ..ledger.manager import clear_pending_transactions
    from ..models.transaction import Transaction
    c.init_ctx.bind_owner()
    c.ctx.bind_owner()
    c.init_ctx.barrier()  # the leader has opened its ledger too
    logger.info(f'cluster follower rank {c.ctx.rank}/{c.ctx.world} ready at height {db._tip_id()}')
    last_block = None
    while True:
        msg = c.recv()
        op = msg['op']
        if op == 'ping':
            continue
        if op == 'quit':
            break
        if op == 'resync':
            c.replaying = True  # local verification, no agreement collectives: the leader is not applying
            validate.set_dist_context(None)
            last_block = None
            _gather_tips(c, db)
        elif op == 'fork_window':
            await _follower_fork_window(c, db, msg)
            _gather_tips(c, db)
        elif op == 'replay_block':
            if int(msg['h']) <= db._tip_id():
                continue  # this replica already holds it (same chain: checked by resync)
            hexes, cb = await _split_coinbase(unpack_txs(msg['_payload']))
            ok = await fastpath.create_block_from_hex(msg['content'], hexes, coinbase=cb, last_block=last_block,
                                                      mirror=False)
            if not ok:
                raise RuntimeError(f'cluster replay: block {msg["h"]} rejected on rank {c.ctx.rank}')
            last_block = await db.get_last_block()
        elif op == 'mempool_reset':
            db.clear_mempool()
        elif op == 'replay_end':
            c.replaying = False
            c.status(db)
            validate.set_dist_context(c.ctx)
        elif op == 'block':
            cb = None
            if msg.get('cb'):
                cb = await Transaction.from_hex(msg['cb'])
            # difficulty/last block come from this replica's own ledger (identical to the leader's)
            await fastpath.create_block_from_hex(msg['content'], unpack_txs(msg['_payload']), coinbase=cb, mirror=False)
        elif op == 'txs':
            db.admit_replicated(json.loads(msg['_payload'].decode()))
        elif op == 'gc':
            await clear_pending_transactions(msg.get('pending'))
        elif op == 'rollback':
            await db.remove_blocks(msg['n'])
        elif op == 'delete':
            await db.delete_blocks(msg['n'])
        elif op == 'status':
            c.status(db, bool(msg.get('deep')))
        else:  # pragma: no cover
            raise RuntimeError(f'unknown cluster op {op}')
    logger.info(f'cluster follower rank {c.ctx.rank} stopped at height {db._tip_id()}')


__all__ = ['Cluster', 'init', 'get', 'on_admit', 'on_confirm', 'flush_txs', 'mirror_gc', 'mirror_rollback',
           'mirror_delete', 'status_all', 'leader_start', 'leader_resync', 'leader_quit', 'follower_main']
