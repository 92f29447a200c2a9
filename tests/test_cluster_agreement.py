"""Cluster agreement edge cases (parallel/cluster.py), on one process with a scripted peer.

The peer is a fake collective context: every other replica is taken to decide exactly as this one does
(``vote_finish`` returns world x this rank's vote), or to hold a given state (``all_gather_fixed``). That
isolates the two decisions the advisor flagged in round 5:

* a block that fails on EVERY replica after validation but before its journal write must be a clean
  rejection, not a divergence: the vote is cast at the commit point, after every step that can fail
  without writing (a vote queued at validation time saw "all ready" and then "all failed", which the gate
  read as a split and exited every rank with status 70);
* the leader's mempool size in a post-GC agreement counts only what the followers hold at that op: a tx
  the HTTP loop admitted after the op was sent is in the leader's index but still in the outbox.

Reference: the reference node has one store and no replicas (upow/database.py:36-43); a cluster must
reject what it would reject (upow/manager.py:650-757) and never diverge on it."""
import asyncio
from decimal import Decimal

import pytest

from upow_amd import devnet
from upow_amd.ledger import fastpath, manager
from upow_amd.ledger.database import Database
from upow_amd.parallel import cluster
from upow_amd.wallet.builders import address_of, create_transaction

GENESIS = 0xA11CE
KEYS = [0xC0FFEE + k for k in range(4)]


class Diverged(Exception):
    pass


class FakeCtx:
    """A collective context whose peers mirror this rank (votes) or hold ``peer_state`` (all-gathers)."""

    def __init__(self, rank=0, world=2):
        self.rank, self.world = rank, world
        self.is_distributed = True
        self.collectives = 0
        self.peer_state = None
        self.votes = []
        self.frames = []

    def _failed(self, what, e):
        raise Diverged(f'{what}: {e}')

    def vote_start(self, v):
        self.votes.append(int(v))
        return int(v)

    def vote_finish(self, handle):
        self.collectives += 1
        return handle * self.world

    def allreduce_sum(self, v):
        self.collectives += 1
        return int(v) * self.world

    def all_gather_fixed(self, data):
        self.collectives += 1
        return [data] + [self.peer_state if self.peer_state is not None else data] * (self.world - 1)

    def broadcast_frame(self, data, src):
        self.frames.append(data)
        return data


@pytest.fixture(autouse=True)
def _setup(monkeypatch):
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('1.0'))
    yield
    cluster._cluster = None
    cluster._outbox.clear()


def _use(db):
    Database.instance = db
    manager.Manager.difficulty = None


async def _chain(blocks):
    db = await Database.create()
    _use(db)
    base = 1_700_000_000
    for k in range(blocks):
        c = await devnet.mine_header(address_of(GENESIS), [], ts=base + 60 * k, device='cpu')
        assert await fastpath.create_block_from_hex(c, [])
    return db, base + 60 * blocks


def test_failure_on_every_replica_before_the_commit_point_is_a_clean_rejection(monkeypatch):
    async def go():
        db, ts = await _chain(3)
        ctx = FakeCtx()
        cluster.init(ctx)
        content = await devnet.mine_header(address_of(GENESIS), [], ts=ts, device='cpu')
        # every replica fails the same way while encoding the block's batch (after validation, before the
        # journal write): nothing was written anywhere, so the block is simply rejected
        orig = Database.encode_many, Database.encode

        def boom(self, *a, **kw):
            raise RuntimeError('injected encode failure')
        monkeypatch.setattr(Database, 'encode_many', boom)
        monkeypatch.setattr(Database, 'encode', boom)
        assert await fastpath.create_block_from_hex(content, [], mirror=False) is False
        assert ctx.votes == [0], ctx.votes  # one vote per block, a no
        assert db._tip_id() == 3
        # the same block once the fault is gone: every replica votes yes at the commit point and commits
        monkeypatch.setattr(Database, 'encode_many', orig[0])
        monkeypatch.setattr(Database, 'encode', orig[1])
        assert await fastpath.create_block_from_hex(content, [], mirror=False) is True
        assert ctx.votes == [0, 1]
        assert db._tip_id() == 4
        db.close()
    asyncio.run(go())


def test_a_split_vote_is_still_a_divergence():
    """One replica ready, another not (the peer votes the opposite way): every rank stops."""
    ctx = FakeCtx()
    ctx.vote_finish = lambda h: 1  # 1 of 2 replicas ready
    c = cluster.init(ctx)
    gate = cluster.CommitGate(c, 'block 9')
    with pytest.raises(Diverged):
        gate.close(False)


def test_gc_agreement_counts_a_late_admission_as_the_followers_see_it():
    async def go():
        db, _ = await _chain(6)
        ctx = FakeCtx()
        c = cluster.init(ctx)
        db.on_admit = cluster.on_admit
        txs = []
        for k in KEYS[:2]:
            txs.append(await create_transaction(GENESIS, address_of(k), '1.5'))
            assert await db.add_pending_transaction(txs[-1])
        assert cluster.flush_txs() == 2  # the followers hold both (the 'txs' op before the 'gc' op)
        mp = db._mempool()
        assert mp is not None and len(mp) == 2
        tip = cluster._tip_hash(db)
        import struct
        ctx.peer_state = struct.pack('<qq', db._tip_id(), 2) + bytes.fromhex(tip)
        c.send('gc', pending=None)
        # the HTTP loop admits a third tx after the 'gc' op went out: it waits in the outbox
        late = await create_transaction(GENESIS, address_of(KEYS[2]), '1.5')
        assert await db.add_pending_transaction(late)
        assert len(mp) == 3 and len(cluster._outbox) == 1
        c.agree_state(db, 'gc')  # the followers' 2 rows: no divergence
        assert cluster._outbox and cluster._outbox[0][5] == late.hash()  # still ships with the next op
        # the index without that row (e.g. a confirm removed it): it is dropped from the outbox, never shipped
        mp.confirm([late.hash()], [(i.tx_hash, i.index) for i in late.inputs])
        c.agree_state(db, 'gc')
        assert cluster._outbox == []
        # a real difference is still caught
        ctx.peer_state = struct.pack('<qq', db._tip_id(), 1) + bytes.fromhex(tip)
        with pytest.raises(Diverged):
            c.agree_state(db, 'gc')
        db.close()
    asyncio.run(go())
