"""Multi-GPU node: one process per GPU, every rank holds a full ledger replica in its own HBM.

SURVEY.md §2.6 "State replication" + "DP: tx-verify batch parallelism". The reference is one
process with one PostgreSQL; here ``torchrun --nproc-per-node G -m upow_amd.node --cluster``
starts G ranks:

* rank 0 (the leader) serves the REST/WebSocket API exactly like a single-GPU node;
* ranks 1..G-1 (followers) keep an in-memory ledger + HBM UTXO replica and apply every ledger
  mutation the leader makes, in the same order, from an op stream the leader broadcasts over RCCL:

      block     a block to validate+apply (push or sync form, tx hex + optional coinbase)
      txs       the txs admitted to the leader's mempool since the last op (governance rules consult
                pending txs): /push_tx only appends to an outbox; the ledger thread ships the outbox as
                ONE op every ``UPOW_CLUSTER_TX_FLUSH_MS`` and always right before any other op, so a
                follower's mempool holds everything the leader's held when a block is applied
      tx        one mempool tx (start-up replay)
      gc        mempool garbage collection
      rollback  / delete   fork handling (remove_blocks / delete_blocks)
      status    all-gather of (height, UTXO-set hash) — replica audit (GET /cluster_info)
      quit

* block validation runs with the signature batch sharded across the ranks
  (``ledger.validate.set_dist_context``, parallel/verify_dp.py): each GPU verifies 1/G of the
  signatures, statuses are all-gathered, every replica reaches the same verdict, and an
  all-reduce checks that all replicas accepted or all rejected (a split is a replica divergence
  and raises).

At start the leader replays its chain (and mempool) to the followers (which verify locally during
the replay), then switches sharded verification on. Ops are processed strictly in broadcast order;
collectives block the leader's event loop for their (sub-millisecond) duration.
"""
from __future__ import annotations

import json
import os
import threading
from typing import List, Optional

from ..utils.logger import get_logger
from .dist import DistContext

logger = get_logger(__name__)

_cluster: Optional['Cluster'] = None


class Cluster:
    def __init__(self, ctx: DistContext):
        self.ctx = ctx
        self.replaying = False

    @property
    def leader(self) -> bool:
        return self.ctx.rank == 0

    # ------------------------------------------------------------------ op stream
    # One frame per op: u32 header length, a small JSON header, then a binary payload (a block's txs
    # travel as raw bytes, half the size of hex and no JSON string escaping): two broadcasts per op
    # (length, then frame) over RCCL.
    def send(self, op: str, payload: bytes = b'', **kw):
        assert self.leader
        head = json.dumps({'op': op, **kw}, separators=(',', ':')).encode()
        self.ctx.broadcast_bytes(len(head).to_bytes(4, 'little') + head + payload, src=0, max_len=0)

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

    def status(self, db) -> List[dict]:
        """Collective: every rank's (height, UTXO-set hash)."""
        mine = json.dumps({'rank': self.ctx.rank, 'height': db._tip_id(),
                           'utxo_hash': db.sql_unspent_outputs_hash(), 'utxo_entries': len(db.utxo)}).encode()
        return [json.loads(b.decode()) for b in self.ctx.all_gather_bytes(mine)]


def pack_txs(tx_hexes) -> bytes:
    """Raw tx bytes of a block: u32 count, then u32 length + bytes per tx."""
    parts = [len(tx_hexes).to_bytes(4, 'little')]
    for h in tx_hexes:
        raw = bytes.fromhex(h)
        parts.append(len(raw).to_bytes(4, 'little'))
        parts.append(raw)
    return b''.join(parts)


def unpack_txs(buf: bytes) -> List[str]:
    n = int.from_bytes(buf[:4], 'little')
    out, o = [], 4
    for _ in range(n):
        k = int.from_bytes(buf[o:o + 4], 'little')
        out.append(buf[o + 4:o + 4 + k].hex())
        o += 4 + k
    if o != len(buf):
        raise ValueError('cluster frame: trailing bytes after the tx list')
    return out


def init(ctx: DistContext) -> Optional[Cluster]:
    global _cluster
    _cluster = Cluster(ctx) if ctx.is_distributed else None
    return _cluster


def get() -> Optional[Cluster]:
    return _cluster


def active_leader() -> Optional[Cluster]:
    c = _cluster
    return c if (c is not None and c.leader and not c.replaying) else None


# ---------------------------------------------------------------------------------------------- leader hooks
_outbox: List[str] = []
_outbox_lock = threading.Lock()
_flush_scheduled = False
FLUSH_S = float(os.environ.get('UPOW_CLUSTER_TX_FLUSH_MS', '20')) / 1000.0


def mirror_tx(tx_hex: str):
    """A tx admitted by the leader (any thread): queued for the next 'txs' op, never waits for a collective."""
    global _flush_scheduled
    c = active_leader()
    if c is None:
        return
    with _outbox_lock:
        _outbox.append(tx_hex)
        if _flush_scheduled:
            return
        _flush_scheduled = True
    _schedule_flush()


def _schedule_flush():
    """Flush the outbox on the thread that issues every other collective (the ledger thread), after the
    flush interval: one broadcast pair per interval however many txs arrived."""
    import asyncio
    from ..ledger import worker
    w = worker.get()
    if w is not None:
        w.loop.call_soon_threadsafe(lambda: w.loop.call_later(FLUSH_S, _timed_flush))
        return
    try:
        asyncio.get_running_loop().call_later(FLUSH_S, _timed_flush)
    except RuntimeError:  # no loop (tests, tools): ship now
        _timed_flush()


def _timed_flush():
    global _flush_scheduled
    with _outbox_lock:
        _flush_scheduled = False
    flush_txs()


def flush_txs() -> int:
    """Ship the queued mempool txs to the followers as one 'txs' op (ledger thread / op-issuing thread)."""
    c = active_leader()
    with _outbox_lock:
        hexes = list(_outbox)
        _outbox.clear()
    if c is None or not hexes:
        return 0
    c.send('txs', pack_txs(hexes))
    return len(hexes)


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


async def leader_replay(db):
    """Ship the leader's chain and mempool to the followers (startup), then turn on sharded verify."""
    from ..ledger import validate
    c = _cluster
    if c is None or not c.leader:
        return
    tip = db._tip_id()
    c.send('replay_begin', tip=tip)
    offset = 1
    while offset <= tip:
        page = await db.get_blocks(offset, 200)
        if not page:
            break
        for info in page:
            c.send('replay_block', pack_txs(info['transactions']), content=info['block']['content'])
            offset = info['block']['id'] + 1
    pending = [r['tx_hex'] for r in db._q('SELECT tx_hex FROM pending_transactions ORDER BY rowid')]
    if pending:
        c.send('txs', pack_txs(pending))
    c.send('replay_end')
    st = c.status(db)
    bad = [s for s in st if (s['height'], s['utxo_hash']) != (st[0]['height'], st[0]['utxo_hash'])]
    if bad:
        raise RuntimeError(f'cluster replay left diverged replicas: {st}')
    validate.set_dist_context(c.ctx)
    logger.info(f'cluster: {c.ctx.world} replicas at height {tip}, sharded signature verification on')


def leader_quit():
    c = _cluster
    if c is not None and c.leader:
        try:
            flush_txs()
            c.send('quit')
        except Exception as e:  # pragma: no cover - process group already gone
            logger.error(f'cluster quit: {e}')


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


async def follower_main(c: Cluster, db):
    """Apply the leader's op stream until 'quit'."""
    from ..ledger import fastpath, validate
    from ..ledger.manager import clear_pending_transactions
    from ..models.transaction import Transaction
    logger.info(f'cluster follower rank {c.ctx.rank}/{c.ctx.world} ready')
    last_block = None
    while True:
        msg = c.recv()
        op = msg['op']
        if op == 'quit':
            break
        if op == 'replay_begin':
            c.replaying = True  # local verification, no agreement collectives: the leader is not applying
            validate.set_dist_context(None)
            await db.delete_blockchain()
            last_block = None
        elif op == 'replay_block':
            hexes, cb = await _split_coinbase(unpack_txs(msg['_payload']))
            ok = await fastpath.create_block_from_hex(msg['content'], hexes, coinbase=cb, last_block=last_block,
                                                      mirror=False)
            if not ok:
                raise RuntimeError('cluster replay: block rejected on a follower')
            last_block = await db.get_last_block()
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
        elif op == 'tx':
            try:
                await db.add_pending_transaction(await Transaction.from_hex(msg['h']))
            except Exception as e:
                logger.error(f'cluster follower: mempool insert failed: {e}')
        elif op == 'txs':
            for h in unpack_txs(msg['_payload']):
                try:
                    await db.add_pending_transaction(await Transaction.from_hex(h))
                except Exception as e:
                    logger.error(f'cluster follower: mempool insert failed: {e}')
        elif op == 'gc':
            await clear_pending_transactions(msg.get('pending'))
        elif op == 'rollback':
            await db.remove_blocks(msg['n'])
        elif op == 'delete':
            await db.delete_blocks(msg['n'])
        elif op == 'status':
            c.status(db)
        else:  # pragma: no cover
            raise RuntimeError(f'unknown cluster op {op}')
    logger.info(f'cluster follower rank {c.ctx.rank} stopped at height {db._tip_id()}')


__all__ = ['Cluster', 'init', 'get', 'mirror_tx', 'flush_txs', 'mirror_gc', 'mirror_rollback', 'mirror_delete', 'leader_replay',
           'leader_quit', 'follower_main']
