"""Host mempool index (ledger/mempool.py): journaled /push_tx admission against the SQL-only path.

Two ledgers take the same admissions and blocks — one with the index (admission journals its rows, the
checks read host memory), one with ``mempool_index = False`` (the reference's SQL INSERT/SELECT path,
upow/database.py:93-115, 832-838) — and must give the same verdicts and the same mempool tables."""
import asyncio
import json
from datetime import timedelta
from decimal import Decimal

import pytest

from upow_amd import devnet
from upow_amd.ledger import database as dbmod
from upow_amd.ledger import fastpath, manager
from upow_amd.ledger.database import Database, UniqueViolationError
from upow_amd.utils.codec import sha256
from upow_amd.models.transaction import Transaction, TransactionInput, TransactionOutput
from upow_amd.wallet.builders import address_of, create_transaction

GENESIS = 0xA11CE
KEYS = [0x5EED + k for k in range(4)]


@pytest.fixture(autouse=True)
def _low_difficulty(monkeypatch):
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('1.0'))


def _use(db):
    Database.instance = db
    manager.Manager.difficulty = None


def _pending(db):
    db.flush()
    return (sorted(tuple(r) for r in db._q('SELECT tx_hash, tx_hex, inputs_addresses, fees FROM pending_transactions')),
            sorted(tuple(r) for r in db._q('SELECT tx_hash, "index" FROM pending_spent_outputs')))


async def _chain(blocks=6):
    a = await Database.create()
    b = await Database.create()
    b.mempool_index = False
    base = 1_700_000_000
    for k in range(blocks):
        for db in (a, b):
            _use(db)
            c = await devnet.mine_header(address_of(GENESIS), [], ts=base + 60 * k, device='cpu')
            assert await fastpath.create_block_from_hex(c, [])
    return a, b, base + 60 * blocks


async def _admit_both(a, b, tx):
    out = []
    for db in (a, b):
        _use(db)
        try:
            out.append(await db.add_pending_transaction(tx))
        except UniqueViolationError:
            out.append('dup')
    assert out[0] == out[1], out
    return out[0]


def test_admission_matches_sql_path():
    async def go():
        a, b, ts = await _chain()
        assert a.writer is not None and b.writer is not None
        _use(a)
        txs = []
        for k in KEYS:  # each built after the previous one is pending: spendable outputs skip its inputs
            _use(a)
            txs.append(await create_transaction(GENESIS, address_of(k), '1.5'))
            assert await _admit_both(a, b, txs[-1]) is True
        assert a._mp is not None and len(a._mp) == len(txs)
        assert await _admit_both(a, b, txs[0]) is False  # its own inputs are pending-spent (reference order)
        # same inputs, different outputs: a double spend against the mempool
        ins = [TransactionInput(i.tx_hash, i.index, amount=i.amount, public_key=i.public_key) for i in txs[1].inputs]
        ds = Transaction(ins, [TransactionOutput(address_of(KEYS[0]), Decimal('0.5'))])
        ds.sign([GENESIS])
        assert await _admit_both(a, b, ds) is False
        assert _pending(a) == _pending(b)
        assert await a.get_pending_spent_outputs([(i.tx_hash, i.index) for i in txs[2].inputs]) == \
            await b.get_pending_spent_outputs([(i.tx_hash, i.index) for i in txs[2].inputs])
        # a block confirming two of them: both leave the index and the tables
        for db in (a, b):
            _use(db)
            c = await devnet.mine_header(address_of(GENESIS), txs[:2], ts=ts, device='cpu')
            assert await fastpath.create_block_from_hex(c, [t.hex() for t in txs[:2]])
        assert len(a._mp) == 2
        assert _pending(a) == _pending(b)
        assert len(_pending(a)[0]) == 2
        reloads = a.mempool_reloads
        _use(a)
        assert await a.get_need_propagate_transactions() == []
        assert a.mempool_reloads == reloads  # blocks and admissions keep the index: no SQL reload
    asyncio.run(go())


def test_block_after_empty_decision_deletes_late_admission():
    """A tx admitted after a block found the mempool empty, and confirmed by that block: the block's
    batch carries no mempool deletes, so the confirm step journals a follow-up delete."""
    async def go():
        a, _, _ = await _chain(4)
        _use(a)
        tx = await create_transaction(GENESIS, address_of(KEYS[0]), '1')
        assert await a.add_pending_transaction(tx)
        a._mempool_confirm(False, hashes=[tx.hash()], inputs=[(i.tx_hash, i.index) for i in tx.inputs])
        assert a._mp.empty()
        assert _pending(a) == ([], [])
    asyncio.run(go())


def test_stale_propagation_and_python_write_invalidate(monkeypatch):
    async def go():
        a, _, _ = await _chain(4)
        _use(a)
        tx = await create_transaction(GENESIS, address_of(KEYS[1]), '1')
        assert await a.add_pending_transaction(tx)
        assert await a.get_need_propagate_transactions() == []
        real = dbmod._utcnow
        monkeypatch.setattr(dbmod, '_utcnow', lambda: real() + timedelta(seconds=700))
        assert await a.get_need_propagate_transactions() == [tx.hex()]
        await a.update_pending_transactions_propagation_time([tx.hash()])  # Python-side write: index dropped
        assert a._mp is None
        assert await a.get_need_propagate_transactions() == []
        assert a._mp is not None and a._mp.has_tx(tx.hash())
        await a.remove_pending_transaction(tx.hash())
        assert a._mp is None
        assert await a.get_pending_spent_outputs([(i.tx_hash, i.index) for i in tx.inputs]) == \
            [(i.tx_hash, i.index) for i in tx.inputs]  # the spent rows stay (reference behaviour)
    asyncio.run(go())


def test_template_and_hash_lookup_match_sql_path():
    async def go():
        a, b, _ = await _chain(6)
        txs = []
        for k in KEYS:
            _use(a)
            txs.append(await create_transaction(GENESIS, address_of(k), str(1 + k % 3)))
            assert await _admit_both(a, b, txs[-1]) is True
        ha, xa = a.pending_template()
        hb, xb = b.pending_template()
        assert (ha, xa) == (hb, xb) and xa == [t.hash() for t in map(lambda h: next(x for x in txs if x.hex() == h), ha)]
        assert await a.get_pending_transactions_limit(hex_only=True) == await b.get_pending_transactions_limit(hex_only=True)
        # /get_mining_info's template: native (index) vs Python (SQL) path, whole and cut by the hex limit
        for limit in (10 ** 9, sum(len(h) for h in ha[:4])):
            fa, sa, ja = a.mining_template(limit, 3)
            fb, sb, jb = b.mining_template(limit, 3)
            assert (fa, sa, ja) == (fb, sb, jb)
            hexes = sorted(h for h in ha if sum(len(x) for x in ha[:ha.index(h) + 1]) <= limit)
            assert fa == hexes[:3] and json.loads(b'[' + ja + b']') == sa == [sha256(h) for h in hexes]
        want = [txs[2].hash(), txs[0].hash(), '00' * 32, 'zz']
        assert await a.get_pending_transactions_hex_by_hash(want) == await b.get_pending_transactions_hex_by_hash(want[:3])
        assert await a.get_pending_transactions_hex_by_hash([txs[1].hash()]) == [txs[1].hex()]
    asyncio.run(go())


def test_coalescer_batches_concurrent_submissions():
    from upow_amd.utils import coalesce
    calls = []

    def fn(items):
        calls.append(list(items))
        return [x * 2 for x in items]

    async def go():
        c = coalesce.coalescer('test-double', fn)
        res = await asyncio.gather(*[c.submit(k) for k in range(10)])
        assert res == [2 * k for k in range(10)]
        assert sum(len(b) for b in calls) == 10 and len(calls) <= 2  # first item alone at most, rest together
    asyncio.run(go())


@pytest.mark.gpu
def test_admission_context_uses_batched_hbm_probe(gpu):
    """With the admission context set (as the node's /push_tx handler does), outpoint checks and
    signatures go through the coalescers: same verdicts as the synchronous path."""
    from upow_amd.utils import coalesce

    async def go():
        a = await Database.create(utxo_backend='gpu')
        b = await Database.create(utxo_backend='host')
        base = 1_700_000_000
        for k in range(4):
            for db in (a, b):
                _use(db)
                c = await devnet.mine_header(address_of(GENESIS), [], ts=base + 60 * k, device='cpu')
                assert await fastpath.create_block_from_hex(c, [])
        async def admit(db, tx):
            coalesce.ADMISSION.set(True)
            _use(db)
            return await db.add_pending_transaction(tx)
        txs = []
        for k in KEYS[:3]:  # each built after the previous one is pending on `a`
            _use(a)
            txs.append(await create_transaction(GENESIS, address_of(k), '1'))
            assert await asyncio.create_task(admit(a, txs[-1])) is True
            assert await asyncio.create_task(admit(b, txs[-1])) is True
        ins = [TransactionInput(i.tx_hash, i.index + 7, amount=i.amount, public_key=i.public_key) for i in txs[0].inputs]
        bad = Transaction(ins, [TransactionOutput(address_of(KEYS[0]), Decimal('0.5'))])
        bad.sign([GENESIS])
        assert await asyncio.create_task(admit(a, bad)) is False  # outpoint not in the HBM index
        assert coalesce.stats().get('utxo-probe', {}).get('items', 0) >= 4
        assert _pending(a) == _pending(b)
    asyncio.run(go())


def test_native_index_template_order_and_confirm():
    # the C++ index against the reference's ORDER BY fees / LENGTH(tx_hex) DESC, LENGTH(tx_hex), tx_hex
    # (Decimal arithmetic), and a block's raw confirm with the late-admission split
    import random
    import numpy as np
    from upow_amd.ledger.mempool import MempoolIndex, outpoint_key
    rng = random.Random(3)
    rows = []
    for k in range(400):
        hx = rng.randbytes(rng.choice([100, 120, 120, 200])).hex()
        fee = Decimal(rng.choice([0, 1, 2, 3, 10, 25])) / 1000000
        rows.append((rng.randbytes(32).hex(), 1_700_000_000 + k, hx, format(fee, 'f')))
    mp = MempoolIndex(rows, [])
    want = sorted(rows, key=lambda r: (-(Decimal(r[3]) / len(r[2])), len(r[2]), r[2]))
    got = mp.ordered(10 ** 9)
    assert [hx for hx, _ in got] == [r[2] for r in want]
    assert [h.hex() for _, h in got] == [r[0] for r in want]
    limit = sum(len(r[2]) for r in want[:37]) + 5
    assert len(mp.ordered(limit)) == 37
    assert mp.hex_in_order([rows[5][0], rows[2][0], 'zz', rows[2][0]]) == [rows[2][2], rows[5][2]]
    # admissions: duplicate, double spend, sequence; confirm splits hits by the block's sequence
    h1, h2 = rng.randbytes(32).hex(), rng.randbytes(32).hex()
    op = (rng.randbytes(32).hex(), 3)
    with mp.lock:
        assert mp.try_add(h1, 5, [op], 'ab' * 60, '0.000010') is None
        assert mp.try_add(h1, 5, [], 'ab' * 60, '0.000010') == 'duplicate'
        assert mp.try_add(h2, 5, [op], 'cd' * 60, '0.000010') == 'double spend'
        mp.set_seq(h1, [op], 9)
    assert mp.spent_of([op, op, (op[0], 4)]) == [op]
    txids = np.frombuffer(bytes.fromhex(h1) + bytes.fromhex(rows[0][0]), np.uint8).reshape(-1, 32)
    keys = np.zeros((1, 40), np.uint8)
    keys[0, :36] = np.frombuffer(outpoint_key(*op), np.uint8)
    hit_tx, hit_in, late_tx, late_in = mp.confirm_raw(txids, keys, 7)
    assert sorted(hit_tx) == sorted([bytes.fromhex(h1), bytes.fromhex(rows[0][0])])
    assert hit_in == [outpoint_key(*op)] and late_tx == [bytes.fromhex(h1)] and late_in == [outpoint_key(*op)]
    assert len(mp) == 399 and not mp.has_tx(h1) and mp.spent_of([op]) == []
    assert mp.maybe_stale(1_700_000_000 + 10_000, 100) and not mp.maybe_stale(1_700_000_000, 10 ** 6)


def test_lookups_concurrent_with_confirm_are_safe():
    """``spent_of``/``has_tx``/``len`` run on the HTTP loop while a block's ``confirm_raw``
    erases entries GIL-free on the ledger thread. The core's own reader/writer lock serialises them: hammer
    both sides from threads and check every lookup answer is one the index could have held."""
    import os
    import threading
    import numpy as np
    from upow_amd.ops.native import lib
    core = lib().MempoolIndexCore()
    core.load([], [])
    rng = np.random.default_rng(7)
    stop = threading.Event()
    errors = []
    rounds = 300

    def writer():
        try:
            for r in range(rounds):
                txids = rng.integers(0, 256, size=(64, 32), dtype=np.uint8)
                keys = np.zeros((128, 40), np.uint8)
                for j in range(64):
                    h = bytes(txids[j]).hex()
                    ins = [(os.urandom(32).hex(), 0), (os.urandom(32).hex(), 1)]
                    assert core.try_add(h, r, ins, 'ab' * (100 + j), '0.001') is None
                    for m, (ih, ii) in enumerate(ins):
                        keys[2 * j + m, :32] = np.frombuffer(bytes.fromhex(ih), np.uint8)
                        keys[2 * j + m, 32] = ii
                    core.set_seq(h, ins, r)
                probe.append((bytes(txids[0]).hex(), [(bytes(keys[0, :32]).hex(), 0)]))
                hit_tx, hit_in, _, _ = core.confirm_raw(txids, keys, None)
                assert len(hit_tx) == 64 and len(hit_in) == 128
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)
        finally:
            stop.set()

    probe = [('00' * 32, [('00' * 32, 0)])]

    def reader():
        try:
            while not stop.is_set():
                h, ins = probe[-1]
                assert core.has_tx(h) in (True, False)
                assert len(core.spent_of(ins + [('11' * 32, 3)])) <= 1
                assert 0 <= len(core) <= 64
                core.ordered(10_000)
                core.mining_template(10_000, 5)
                core.hex_in_order([h])
        except Exception as e:  # pragma: no cover
            errors.append(e)

    ts = [threading.Thread(target=reader) for _ in range(3)] + [threading.Thread(target=writer)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert not errors, errors
    assert len(core) == 0 and core.spent_count() == 0
