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
      page      a sync page: every block row and tx of a /get_blocks page (ledger/pagesync.py)
      gc        mempool garbage collection
      rollback / delete   fork handling (remove_blocks / delete_blocks)
      status    all-gather of every replica's (height, tip hash, UTXO-set K12 hash from the index)
      ping      idle heartbeat (keeps followers inside the op group's collective timeout)
      quit

Framing. An op is ONE fixed-capacity broadcast when it fits in 64 KB (everything but blocks and sync
pages), two otherwise (``DistContext.broadcast_frame``); mempool rows travel packed in binary.

Start-up resync runs on the long-timeout group (``init_ctx``): a replay of a long chain can outlast the op
timeout, and every ``ACK_EVERY`` replayed blocks the leader and the followers meet in an all-reduce that
also carries each follower's success, so no broadcast stays queued for long and a follower that cannot
apply the leader's chain stops the resync instead of hanging it.

Agree before commit. A block (push or sync form) is validated on every replica; right before its journal
write each replica votes in one all-reduce (``commit_point``, once the block's batch is encoded), and
writes only when every replica voted to. A replica that rejected the block votes no when it finishes. A
split vote is a replica divergence: nothing was committed anywhere, and every rank exits with status 70
(``DistContext._failed``); a relaunch resyncs the replicas from that common state. Rollbacks, chain
deletions and mempool GC end in an all-gather of (height, tip hash, mempool size) that must agree.

Ordering and threads. Every collective of a rank is issued by ONE thread (``DistContext.bind_owner``):
the leader's ledger thread, the follower's op loop. ``/cluster_info`` and the idle heartbeat are routed
through the ledger thread; admissions on the HTTP loop only append to an outbox, which the ledger thread
ships as ONE 'txs' op every ``UPOW_CLUSTER_TX_FLUSH_MS`` and always right before any other op. A row
admitted on the leader while a block was being applied is edited in the outbox exactly as the block's
mempool confirm edited the leader's index (its tx dropped if the block confirmed it, confirmed inputs
stripped), so a follower that inserts it after that block ends in the leader's state.

Verification. Each replica validates every block itself. A single pushed block's signature batch is sharded
across the ranks only from ``UPOW_CLUSTER_SHARD_MIN`` signatures up (ledger/validate.py): a 2 MB block
(~8,300 signatures) verifies in ~1.2 ms on one GPU, less than a sharded verify costs in collectives. Chain
sync sends a whole ``/get_blocks`` page as one 'page' op; every rank plans it in chunks (ledger/pagesync.py)
whose signature batches — thousands to hundreds of thousands of signatures — ARE sharded: rank r verifies
a contiguous shard, one all-gather of status bytes, then every replica applies the blocks in order.
"""
from __future__ import annotations

import contextvars
import json
import os
import struct
import threading
import time
from typing import List, Optional

import numpy as np

from ..utils.logger import get_logger
from .dist import DistContext

logger = get_logger(__name__)

_cluster: Optional['Cluster'] = None
HEARTBEAT_S = float(os.environ.get('UPOW_CLUSTER_HEARTBEAT_S', '5'))
FORK_WINDOW = 500  # remove_blocks' reach (reference database.py:146-169 pages of 500)
ACK_EVERY = int(os.environ.get('UPOW_CLUSTER_REPLAY_ACK', '32'))  # resync: replayed blocks per acknowledgement


class Cluster:
    def __init__(self, ctx: DistContext, init_ctx: Optional[DistContext] = None):
        self.ctx = ctx  # op traffic (short timeout group)
        self.init_ctx = init_ctx or ctx  # start-up barrier and resync (long timeout group)
        self.op_ctx = self.ctx  # the group the op stream runs on right now (init_ctx during resync)
        self.replaying = False
        self.closed = False  # after 'quit': no op is sent again (the heartbeat stops)
        self.last_send = time.monotonic()
        self.ops_sent = 0
        self.ops_received = 0
        self.commits_agreed = 0
        self.vote_s = 0.0  # wall time from a commit vote's start to its outcome (overlaps the block's batch encode)
        self.vote_issue_s = 0.0  # host time queueing the votes
        self.vote_issue_cpu_s = 0.0  # of which the thread was on a CPU (the rest: waiting for the GIL or a lock)
        self.vote_block_s = 0.0  # time the commit point waited for them: the per-block price of agreement
        self.last_resync: Optional[dict] = None

    @property
    def leader(self) -> bool:
        return self.ctx.rank == 0

    # ------------------------------------------------------------------ op stream
    # One frame per op: u32 header length, a small JSON header, then a binary payload (a block's txs travel as
    # raw bytes, half the size of hex and no JSON escaping), in one fixed-capacity broadcast when it fits.
    def send(self, op: str, payload: bytes = b'', **kw):
        assert self.leader
        head = json.dumps({'op': op, **kw}, separators=(',', ':'), default=str).encode()
        self.op_ctx.broadcast_frame(len(head).to_bytes(4, 'little') + head + payload, src=0)
        self.last_send = time.monotonic()
        self.ops_sent += 1

    def recv(self) -> dict:
        raw = self.op_ctx.broadcast_frame(None, src=0)
        n = int.from_bytes(raw[:4], 'little')
        msg = json.loads(raw[4:4 + n].decode())
        msg['_payload'] = raw[4 + n:]
        msg['_raw'] = raw  # a lean follower logs the frame as it arrived (ledger/lean.py)
        self.ops_received += 1
        return msg

    def send_page(self, blocks: list):
        """A /get_blocks page (block rows + every tx, coinbase included) as ONE 'page' op."""
        rows = [b['block'] for b in blocks]
        counts = [len(b['transactions']) for b in blocks]
        self.send('page', pack_groups([b['transactions'] for b in blocks]), rows=rows, counts=counts)

    @staticmethod
    def unpack_page(msg: dict) -> list:
        hexes = unpack_txs(msg['_payload'])
        out, at = [], 0
        for row, n in zip(msg['rows'], msg['counts']):
            out.append({'block': row, 'transactions': hexes[at:at + n]})
            at += n
        return out

    def agree(self, ok: bool, what: str) -> bool:
        n = self.op_ctx.allreduce_sum(1 if ok else 0)
        if n not in (0, self.ctx.world):
            self.diverged(f'{what}: {n}/{self.ctx.world} accepted')
        return bool(ok)

    def diverged(self, what: str):
        """Replica divergence: every rank detects it in the same collective, nothing was committed past the
        agreed state, and each rank exits (status 70; ``UPOW_DIST_FATAL=0`` raises instead)."""
        self.ctx._failed('replica agreement', RuntimeError(f'cluster replicas diverged on {what}'))

    def agree_state(self, db, what: str):
        """After a rollback, a chain deletion or a mempool GC: every replica at the same (height, tip hash,
        mempool size), checked in one fixed-size all-gather.

        The leader's HTTP loop keeps admitting txs while the op runs: an admission made after the op was sent
        sits in the leader's index but only in the outbox, not yet on the followers. So the leader counts what
        the followers hold at this op: its index minus the outbox rows still in it, read under the index lock
        the admissions take (outbox rows the op itself removed from the index are dropped, they never ship)."""
        tip = _tip_hash(db)
        size = _replicated_mempool_size(db) if self.leader else _mempool_size(db)
        mine = struct.pack('<qq', db._tip_id(), size) + (bytes.fromhex(tip) if tip else bytes(32))
        got = self.op_ctx.all_gather_fixed(mine)
        if any(g != got[0] for g in got):
            states = [(struct.unpack('<qq', g[:16]), g[16:].hex()[:16]) for g in got]
            self.diverged(f'{what}: replica states {states}')

    def replay_ack(self, ok: bool):
        """Resync checkpoint (long-timeout group): the leader learns that every follower applied the replayed
        blocks so far; a follower that failed votes 0 and the resync stops on every rank."""
        n = self.op_ctx.allreduce_sum(1 if ok else 0)
        if n != self.ctx.world:
            raise RuntimeError(f'cluster resync: {self.ctx.world - n} replica(s) could not apply the leader\'s chain')

    def status(self, db, deep: bool = False, mempool: Optional[int] = None) -> List[dict]:
        """Collective: every rank's height, tip hash and UTXO-set hash. The hash comes from the HBM index
        (K12: compaction + radix sort on the device, host SHA tail), current at the commit point; ``deep``
        also hashes the SQL replica after the materialisers have caught up (the slow full-table audit, on
        the long-timeout group: it may take longer than the op timeout on a big ledger)."""
        mine = {'rank': self.ctx.rank, 'height': db._tip_id(), 'tip_hash': _tip_hash(db),
                'utxo_hash': db.utxo.set_hash(_utxo_tag()), 'utxo_entries': len(db.utxo),
                'mempool': _mempool_size(db) if mempool is None else mempool,
                # process CPU seconds (every thread) so far: what each replica costs the host, per op stream
                'lean': bool(db.lean), 'cpu_s': round(time.process_time(), 4),
                'crypto_cpu_s': round(_pagesync_stats().get('plan_crypto_cpu_s', 0.0), 4)}
        if deep:
            db.flush()
            mine['sql_utxo_hash'] = db.sql_unspent_outputs_hash()
        g = self.init_ctx if deep else self.op_ctx
        return [json.loads(b.decode()) for b in g.all_gather_bytes(json.dumps(mine).encode())]

    def info(self) -> dict:
        """Op-stream counters for /cluster_info: collectives per op (framing + agreements + replies)."""
        ops = self.ops_sent if self.leader else self.ops_received
        coll = self.ctx.collectives
        return {'ops': ops, 'collectives': coll, 'collectives_per_op': round(coll / ops, 3) if ops else None,
                'commits_agreed': self.commits_agreed,
                # per agreed block: vote start to outcome (overlapping the batch encode), the host time spent
                # queueing it, and the time the commit point actually waited for it
                'vote_us_avg': round(self.vote_s / self.commits_agreed * 1e6, 1) if self.commits_agreed else None,
                'vote_issue_us_avg': round(self.vote_issue_s / self.commits_agreed * 1e6, 1) if self.commits_agreed else None,
                'vote_issue_cpu_us_avg': round(self.vote_issue_cpu_s / self.commits_agreed * 1e6, 1) if self.commits_agreed else None,
                'vote_wait_us_avg': round(self.vote_block_s / self.commits_agreed * 1e6, 1) if self.commits_agreed else None,
                **_native_vote_stats(self.op_ctx)}


def _native_vote_stats(ctx) -> dict:
    """Per-vote host time of the native vote's enqueues (csrc/rccl_vote.hip), when it is in use."""
    nv = ctx.__dict__.get('_nv')
    if not nv:
        return {}
    L, h = nv
    n, tg, tc, te = L.rccl_vote_stats(h)
    if not n:
        return {}
    return {'native_vote': {'votes': int(n), 'gather_us': round(tg / n * 1e6, 1), 'copy_us': round(tc / n * 1e6, 1),
                            'event_us': round(te / n * 1e6, 1), 'call_us': round(ctx.vote_call_s / n * 1e6, 1)}}


# ---------------------------------------------------------------------------------------------- commit gate
_GATE: contextvars.ContextVar = contextvars.ContextVar('upow_commit_gate', default=None)


class CommitGate:
    """Agree-before-commit for one block on a cluster node: :meth:`start` + :meth:`wait` at the commit point —
    right before the journal write (``commit_point``), once the block's batch is encoded — and :meth:`close`
    with the rank's final verdict. Exactly one all-reduce per block per rank; a rank that rejects the block, or
    fails before its commit point, votes no in :meth:`close`, so a failure every replica shares is a clean
    rejection and only a split is a divergence."""

    def __init__(self, c: Cluster, what: str):
        self.c, self.what = c, what
        self.ready = False  # passed validation (commit_gate); the vote itself is cast at the commit point
        self.voted: Optional[bool] = None
        self.n = 0
        self._pending = None
        self._t0 = 0.0

    def start(self):
        """This rank is ready to commit: queue the vote, do not wait for it."""
        if self.voted is not None:
            raise RuntimeError('commit gate: a block voted twice')
        self.voted = True
        self._t0 = time.perf_counter()
        c0 = time.thread_time()
        self._pending = self.c.op_ctx.vote_start(1)
        self.c.vote_issue_s += time.perf_counter() - self._t0
        self.c.vote_issue_cpu_s += time.thread_time() - c0

    def wait(self) -> bool:
        """The vote's outcome (waits for a queued one): True only when every replica is ready."""
        if self._pending is not None:
            pending, self._pending = self._pending, None
            tw = time.perf_counter()
            self.n = self.c.op_ctx.vote_finish(pending)
            t1 = time.perf_counter()
            self.c.vote_s += t1 - self._t0
            self.c.vote_block_s += t1 - tw
            if self.n == self.c.ctx.world:
                self.c.commits_agreed += 1
        return bool(self.voted) and self.n == self.c.ctx.world

    def vote(self, ok: bool) -> bool:
        """This rank is ready to commit (or not), voted and waited for at once; True only when every
        replica is."""
        if self.voted is not None:
            raise RuntimeError('commit gate: a block voted twice')
        if ok:
            self.start()
            return self.wait()
        self.voted = False
        self.n = self.c.op_ctx.vote_finish(self.c.op_ctx.vote_start(0))
        return False

    def close(self, ok: bool) -> bool:
        if self.voted is None:  # rejected (or failed) before reaching the commit point
            self.vote(False)
        self.wait()  # a queued vote always completes: the ranks' collectives pair up
        world = self.c.ctx.world
        if self.n not in (0, world):
            self.c.diverged(f'{self.what}: {self.n}/{world} replicas ready to commit (none committed)')
        if self.voted and self.n == world and not ok:
            self.c.diverged(f'{self.what}: agreed, but the ledger write failed on rank {self.c.ctx.rank}')
        return bool(ok) and self.n == world


def open_gate(what: str = 'block'):
    """(gate, token) for a block about to be validated; (None, token) outside an active cluster."""
    c = _cluster
    gate = CommitGate(c, what) if (c is not None and not c.replaying) else None
    return gate, _GATE.set(gate)


def close_gate(gate: Optional[CommitGate], token, ok: bool) -> bool:
    _GATE.reset(token)
    return gate.close(ok) if gate is not None else ok


def commit_gate() -> bool:
    """Called by the block paths once a block has passed validation, before they prepare its ledger writes.
    Casts no vote: the vote is taken at :func:`commit_point`, after every step that can still fail without
    writing (statement building and encoding). A vote queued here instead would let a replica vote yes and
    then fail before its journal write; a failure every replica shares would then look like a split (all
    voted yes, none committed) and stop the cluster on a block a single node simply rejects."""
    g = _GATE.get()
    if g is not None:
        g.ready = True
    return True


class CommitRefused(RuntimeError):
    """A replica is not ready to commit the block this rank prepared: nothing was written."""


def commit_point():
    """The ledger's commit point (right before a block's journal write): votes, waits for the outcome and
    raises :class:`CommitRefused` unless every replica is ready. Past this point the only failure is the
    journal write itself, which is a local I/O fault (a divergence, status 70). No-op outside an active
    cluster gate."""
    g = _GATE.get()
    if g is None:
        return
    g.start()
    if not g.wait():
        raise CommitRefused(f'{g.what}: {g.n}/{g.c.ctx.world} replicas ready to commit')


def _pagesync_stats() -> dict:
    from ..ledger import pagesync
    return pagesync.stats


def _utxo_tag() -> int:
    from ..ledger.utxo import TAG_BY_TABLE
    return TAG_BY_TABLE['unspent_outputs']


def _tip_hash(db) -> Optional[str]:
    return db.block_hash_at(db._tip_id())


def _mempool_size(db) -> int:
    mp = db._mempool()
    if mp is not None:
        return len(mp)
    return int(db._q1('SELECT COUNT(*) FROM pending_transactions')[0])


def _replicated_mempool_size(db) -> int:
    """The leader's mempool size as the followers see it at the current op (see ``Cluster.agree_state``)."""
    mp = db._mempool()
    if mp is None:
        with _outbox_lock:
            return _mempool_size(db) - len(_outbox)
    with mp.lock:
        with _outbox_lock:
            _outbox[:] = [row for row in _outbox if mp.has_tx(row[5])]
            return len(mp) - len(_outbox)


def pack_txs(tx_hexes) -> bytes:
    """Raw tx bytes of a block: u32 count, then u32 length + bytes per tx (hex-decoded natively on the
    host pool, csrc/txcodec.cpp ``pack_tx_hexes``)."""
    from ..ops.native import lib
    from ..utils.hexspans import HexSpans
    if isinstance(tx_hexes, HexSpans):  # read in place from the request / page body
        return lib().pack_tx_spans(tx_hexes.buf, np.ascontiguousarray(tx_hexes.spans).tobytes(),
                                   list(tx_hexes.extra), _threads())
    return lib().pack_tx_hexes(tx_hexes if isinstance(tx_hexes, list) else list(tx_hexes), _threads())


def pack_groups(groups) -> bytes:
    """``pack_txs`` of several blocks' tx lists in a row; the blocks of one page body stay spans of it."""
    from ..utils.hexspans import HexSpans
    if groups and all(isinstance(g, HexSpans) and g.buf is groups[0].buf and not g.extra for g in groups):
        return pack_txs(HexSpans(groups[0].buf, np.concatenate([g.spans for g in groups])))
    return pack_txs([h for g in groups for h in g])


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
# Replicated mempool rows: (tx_hex, inputs_addresses JSON, fees text, propagation time, [[txid, index], ...],
# tx hash hex); the hash stays on the leader (the outbox edit below), the rest travels packed in binary
_outbox: List[list] = []
_outbox_lock = threading.Lock()
_flush_scheduled = False
FLUSH_S = float(os.environ.get('UPOW_CLUSTER_TX_FLUSH_MS', '20')) / 1000.0


def pack_rows(rows: List[list]) -> bytes:
    """Mempool rows in binary: u32 count; per row u32 + raw tx bytes, u32 + inputs_addresses UTF-8,
    u8 + fees text, i64 propagation time, u16 count + (32-byte txid, u16 index) per reserved input."""
    out = bytearray(struct.pack('<I', len(rows)))
    for row in rows:
        raw = bytes.fromhex(row[0])
        ia = row[1].encode()
        fees = str(row[2]).encode()
        out += struct.pack('<I', len(raw)) + raw + struct.pack('<I', len(ia)) + ia
        out += struct.pack('<B', len(fees)) + fees + struct.pack('<qH', int(row[3]), len(row[4]))
        for h, i in row[4]:
            out += bytes.fromhex(h) + struct.pack('<H', int(i))
    return bytes(out)


def unpack_rows(buf: bytes) -> List[list]:
    mv = memoryview(buf)
    (n,), at = struct.unpack_from('<I', mv, 0), 4
    rows = []
    for _ in range(n):
        (ln,) = struct.unpack_from('<I', mv, at)
        tx_hex = mv[at + 4:at + 4 + ln].hex()
        at += 4 + ln
        (ln,) = struct.unpack_from('<I', mv, at)
        ia = bytes(mv[at + 4:at + 4 + ln]).decode()
        at += 4 + ln
        ln = mv[at]
        fees = bytes(mv[at + 1:at + 1 + ln]).decode()
        at += 1 + ln
        ptime, k = struct.unpack_from('<qH', mv, at)
        at += 10
        ins = []
        for _ in range(k):
            ins.append([mv[at:at + 32].hex(), struct.unpack_from('<H', mv, at + 32)[0]])
            at += 34
        rows.append([tx_hex, ia, fees, ptime, ins])
    return rows


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


def on_confirm(mp, hit_tx: list, hit_in: list):
    """Database hook (``Database.on_confirm``, under the mempool index lock): a block's confirm just removed
    ``hit_tx`` (raw tx hashes) and ``hit_in`` (raw 36-byte outpoints) from the leader's index ``mp``. Rows
    still in the outbox were admitted before that confirm, so the followers must see them as the confirm left
    them. With the index at hand that is one probe per outbox row, never a set over the block: a row whose
    tx left the index was confirmed; of its reserved inputs, only those the index still holds stay."""
    if not _outbox:
        return
    with _outbox_lock:
        keep = []
        if mp is not None:
            for row in _outbox:
                if not mp.has_tx(row[5]):
                    continue
                if row[4]:
                    live = {(h, int(i)) for h, i in mp.spent_of(row[4])}
                    row[4] = [p for p in row[4] if (p[0], int(p[1])) in live]
                keep.append(row)
        else:  # no mempool index (its SQL form): the block's own hit lists
            txs = set(hit_tx)
            ins = {(k[:32].hex(), int.from_bytes(k[32:36], 'little')) for k in hit_in}
            for row in _outbox:
                if bytes.fromhex(row[5]) in txs:
                    continue
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
    c.send('txs', pack_rows(rows))
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
    """Mempool GC on every replica (manager.clear_pending_transactions), then agreement on the result."""
    from ..ledger.database import Database
    from ..ledger.manager import clear_pending_transactions
    c = active_leader()
    if c is not None:
        flush_txs()
        c.send('gc', pending=list(pending) if pending is not None else None)
    res = await clear_pending_transactions(pending)
    if c is not None:
        c.agree_state(Database.instance, 'gc')
    return res


async def mirror_rollback(db, block_no: int):
    c = active_leader()
    if c is not None:
        flush_txs()
        c.send('rollback', n=int(block_no))
    await db.remove_blocks(block_no)
    if c is not None:
        c.agree_state(db, f'rollback to {block_no}')


async def mirror_delete(db, offset: int):
    c = active_leader()
    if c is not None:
        flush_txs()
        c.send('delete', n=int(offset))
    await db.delete_blocks(offset)
    if c is not None:
        c.agree_state(db, f'delete from {offset}')


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
            c.send('txs', pack_rows(rows))
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
    """Bring every follower to the leader's chain and mempool, sending only what each lacks. The whole resync
    runs on the long-timeout group, acknowledged every ACK_EVERY replayed blocks."""
    from ..ledger import validate
    c = _cluster
    tip = db._tip_id()
    c.replaying = True
    c.op_ctx = c.init_ctx
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
                if sent % ACK_EVERY == 0:
                    c.replay_ack(True)
        flush_txs()
        c.send('mempool_reset')
        rows = _mempool_rows(db)
        for k in range(0, len(rows), 512):
            c.send('txs', pack_rows(rows[k:k + 512]))
        c.send('replay_end', sent=sent)
        c.replay_ack(True)
        c.replaying = False
        st = c.status(db)
    finally:
        c.replaying = False
        c.op_ctx = c.ctx
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
    return db.block_hash_at(h)


def _gather_tips(c: Cluster, db) -> List[dict]:
    mine = json.dumps({'rank': c.ctx.rank, 'tip': db._tip_id(), 'tip_hash': _tip_hash(db)}).encode()
    return [json.loads(b.decode()) for b in c.op_ctx.all_gather_bytes(mine)]


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


LEDGER_OPS = ('block', 'page', 'replay_block')  # ops that move the chain tip: a lean follower logs them
SQL_OPS = ('rollback', 'delete', 'fork_window')  # ops that need the SQL tables: a lean follower materialises first


async def follower_main(c: Cluster, db):
    """Apply the leader's op stream until 'quit'. The first op is the start-up resync, on the long-timeout
    group; after 'replay_end' the stream moves to the op group.

    A lean follower (ledger/lean.py, the default) applies blocks to its indexes only and logs every
    tip-moving op as it arrived, with the tip it reached; ops that need its SQL tables (rollbacks, chain
    deletions, fork windows, deep audits) first materialise the log. It starts by materialising whatever a
    previous run logged."""
    from ..ledger import lean
    want_lean = lean.enabled()
    if lean.pending(db):
        await lean.materialise(db)
    if want_lean:
        db.enter_lean()
    c.init_ctx.bind_owner()
    c.ctx.bind_owner()
    c.op_ctx = c.init_ctx
    c.init_ctx.barrier()  # the leader has opened its ledger too
    logger.info(f'cluster follower rank {c.ctx.rank}/{c.ctx.world} ready at height {db._tip_id()}'
                f'{" (lean replica)" if db.lean else ""}')
    f = _Follower(c, db)
    while True:
        msg = c.recv()
        op = msg['op']
        if op == 'ping':
            continue
        if op == 'quit':
            break
        if db.lean and (op in SQL_OPS or (op == 'status' and msg.get('deep'))):
            await lean.materialise(db, online=True)
        if db.lean and op in LEDGER_OPS:
            db.lean_log.op(msg['_raw'])
        await f.apply(msg)
        if op in LEDGER_OPS and db.lean_log is not None and (db.lean or want_lean):
            db.lean_log.tip(db._tip_id(), _tip_hash(db))
        if want_lean and not db.lean and op not in ('resync', 'fork_window'):
            db.enter_lean()  # after an op that needed the full ledger (its log was materialised)
        elif op in ('status', 'replay_end') and db.lean_log is not None:
            db.lean_log.sync()
    if db.lean_log is not None:  # a graceful stop: the log ends on a durable tip marker
        db.lean_log.tip(db._tip_id(), _tip_hash(db))
        db.lean_log.sync()
    logger.info(f'cluster follower rank {c.ctx.rank} stopped at height {db._tip_id()}')


class _Follower:
    """One follower's op handlers (the replay state lives across the ops of a resync)."""

    def __init__(self, c: Cluster, db):
        self.c, self.db = c, db
        self.last_block = None
        self.replayed = 0
        self.replay_error = None

    async def apply(self, msg: dict):
        from ..ledger import fastpath, pagesync, validate
        from ..ledger.manager import clear_pending_transactions
        from ..models.transaction import Transaction
        c, db, op = self.c, self.db, msg['op']
        if op == 'resync':
            c.replaying = True  # local verification, no agreement collectives: the leader is not applying
            validate.set_dist_context(None)
            self.last_block = None
            self.replayed = 0
            self.replay_error = None
            _gather_tips(c, db)
        elif op == 'fork_window':
            await _follower_fork_window(c, db, msg)
            _gather_tips(c, db)
        elif op == 'replay_block':
            self.replayed += 1
            if self.replay_error is None and int(msg['h']) > db._tip_id():  # else: this replica already holds it
                try:
                    hexes, cb = await _split_coinbase(unpack_txs(msg['_payload']))
                    if cb is None:  # a replayed block is the sync form: it carries its coinbase
                        raise RuntimeError(f'block {msg["h"]} has no coinbase transaction')
                    if not await fastpath.create_block_from_hex(msg['content'], hexes, coinbase=cb,
                                                                last_block=self.last_block, mirror=False):
                        raise RuntimeError(f'block {msg["h"]} rejected')
                    self.last_block = await db.get_last_block()
                except Exception as e:  # reported at the next acknowledgement, on every rank
                    self.replay_error = e
                    logger.error(f'cluster replay on rank {c.ctx.rank}: {e}')
            if self.replayed % ACK_EVERY == 0:
                c.replay_ack(self.replay_error is None)
        elif op == 'mempool_reset':
            db.clear_mempool()
        elif op == 'replay_end':
            c.replay_ack(self.replay_error is None)
            c.replaying = False
            c.status(db)
            c.op_ctx = c.ctx
            validate.set_dist_context(c.ctx)
        elif op == 'block':
            cb = None
            if msg.get('cb'):
                cb = await Transaction.from_hex(msg['cb'])
            # difficulty/last block come from this replica's own ledger (identical to the leader's)
            await fastpath.create_block_from_hex(msg['content'], unpack_txs(msg['_payload']), coinbase=cb, mirror=False)
        elif op == 'page':
            await pagesync.create_blocks(Cluster.unpack_page(msg), mirror=False)
        elif op == 'txs':
            db.admit_replicated(unpack_rows(msg['_payload']))
        elif op == 'gc':
            await clear_pending_transactions(msg.get('pending'))
            c.agree_state(db, 'gc')
        elif op == 'rollback':
            await db.remove_blocks(msg['n'])
            c.agree_state(db, f'rollback to {msg["n"]}')
        elif op == 'delete':
            await db.delete_blocks(msg['n'])
            c.agree_state(db, f'delete from {msg["n"]}')
        elif op == 'status':
            c.status(db, bool(msg.get('deep')))
        else:  # pragma: no cover
            raise RuntimeError(f'unknown cluster op {op}')


__all__ = ['Cluster', 'CommitGate', 'init', 'get', 'on_admit', 'on_confirm', 'flush_txs', 'mirror_gc',
           'mirror_rollback', 'mirror_delete', 'status_all', 'leader_start', 'leader_resync', 'leader_quit',
           'follower_main', 'commit_gate', 'open_gate', 'close_gate', 'pack_rows', 'unpack_rows']
