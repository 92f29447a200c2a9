"""Native block path (ledger/fastpath.py) vs the object path: same verdicts, same errors, same ledger.

Two ledgers receive the same blocks — one through ``manager.create_block`` with Transaction objects,
one through ``fastpath.create_block_from_hex`` — and every table, the UTXO index (with payloads)
and the UTXO-set hash must end up identical."""
import asyncio
import random
from decimal import Decimal

import numpy as np
import pytest

from upow_amd import devnet
from upow_amd.ledger import fastpath, manager
from upow_amd.ledger.database import OUTPUT_TABLES, Database
from upow_amd.models.transaction import Transaction, TransactionInput, TransactionOutput
from upow_amd.wallet.builders import address_of, create_stake_transaction, create_transaction

GENESIS = 0xA11CE
KEYS = [0xB0B + k for k in range(6)]
TABLES = ['blocks', 'transactions', 'pending_transactions', 'pending_spent_outputs', 'address_transactions',
          *OUTPUT_TABLES]


@pytest.fixture(autouse=True)
def _low_difficulty(monkeypatch):
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('1.0'))


def _dump(db):
    out = {}
    for t in TABLES:
        rows = db._q(f'SELECT * FROM {t}')
        out[t] = sorted(tuple(r) for r in rows)
    recs, pay = db.utxo.records_payload()
    out['index'] = (recs.tobytes(), pay.tobytes())
    return out


class Pair:
    def __init__(self, a, b):
        self.a, self.b = a, b

    def use(self, db):
        Database.instance = db
        manager.Manager.difficulty = None

    async def push(self, content, txs, expect=None):
        hexes = [t.hex() if not isinstance(t, str) else t for t in txs]
        self.use(self.a)
        ea = []
        ra = await manager.create_block(content, [await Transaction.from_hex(h) for h in hexes], error_list=ea)
        self.use(self.b)
        eb = []
        rb = await fastpath.create_block_from_hex(content, hexes, error_list=eb)
        assert ra == rb, (ra, rb, ea, eb)
        assert ea == eb
        if expect is not None:
            assert ra == expect, ea
        self.a.index_addresses()
        self.b.index_addresses()
        da, dbb = _dump(self.a), _dump(self.b)
        for k in da:
            assert da[k] == dbb[k], k
        self.use(self.a)
        h = self.a.sql_unspent_outputs_hash()
        assert h == self.b.sql_unspent_outputs_hash() == await self.a.get_unspent_outputs_hash() \
            == await self.b.get_unspent_outputs_hash()
        return ra, ea

    async def mine(self, txs=(), ts=None):
        self.use(self.a)
        return await devnet.mine_header(address_of(GENESIS), list(txs), ts=ts, device='cpu')


async def _setup(backend='host'):
    a = await Database.create(utxo_backend=backend)
    b = await Database.create(utxo_backend=backend)
    p = Pair(a, b)
    base = 1_700_000_000
    for k in range(8):
        c = await p.mine(ts=base + 60 * k)
        await p.push(c, [], expect=True)
    return p, base


def _off_curve_x() -> int:
    """Smallest x >= 5 with no curve point (x^3 - 3x + b is not a square mod p)."""
    from upow_amd.utils import p256 as o
    x = 5
    while o.is_on_curve(x, o.x_to_y(x, False)):
        x += 1
    return x


def _signed(inputs, outputs, keys, message=None):
    tx = Transaction(inputs, outputs, message)
    return tx.sign(keys)


@pytest.mark.parametrize('journal', [True, False], ids=['journal-writer', 'sync-executemany'])
@pytest.mark.parametrize('backend', ['host', pytest.param('gpu', marks=pytest.mark.gpu)])
def test_fast_path_matches_object_path(backend, journal, request):
    if backend == 'gpu':
        request.getfixturevalue('gpu')

    async def go():
        p, base = await _setup(backend)
        assert p.b.writer is not None  # csrc/ledger_writer.cpp owns a connection of its own
        if not journal:  # synchronous bulk writes on the Python connection (UPOW_LEDGER_WRITER=0)
            p.b.flush()
            p.b.writer.close()
            p.b.writer = None
        ts = base + 60 * 10
        p.use(p.a)
        txs = []
        for k in KEYS:  # fan out from the genesis coinbases: 1-in txs, change back to genesis
            tx = await create_transaction(GENESIS, address_of(k), '2.5')
            await p.a.add_pending_transaction(tx)
            txs.append(tx)
        txs.append(await create_transaction(GENESIS, address_of(KEYS[0]), '0.125', message=b'hello, block'))
        await p.a.add_pending_transaction(txs[-1])
        p.use(p.b)
        for t in txs:  # mirror the mempool so the pending-table cleanup is exercised on both sides
            await p.b.add_pending_transaction(t)
        c = await p.mine(txs, ts=ts)
        assert fastpath.decode([t.hex() for t in txs]) is not None
        await p.push(c, txs, expect=True)
        assert fastpath.last_path == 'native'
        # second block: multi-input spends with per-input signatures, one shared-signature tx
        p.use(p.a)
        txs2 = []
        for k in KEYS[:3]:
            tx = await create_transaction(k, address_of(KEYS[-1]), '1')
            txs2.append(tx)
        key = KEYS[4]
        outs = await p.a.get_spendable_outputs(address_of(key))
        tx = Transaction(outs, [TransactionOutput(address_of(GENESIS), Decimal('2.4'))])
        tx.sign([key])
        txs2.append(tx)
        c2 = await p.mine(txs2, ts=ts + 60)
        await p.push(c2, txs2, expect=True)
        assert fastpath.last_path == 'native'
        assert fastpath.last_path == 'native'
    asyncio.run(go())


@pytest.mark.parametrize('backend', ['host', pytest.param('gpu', marks=pytest.mark.gpu)])
def test_rejections_match(backend, request):
    if backend == 'gpu':
        request.getfixturevalue('gpu')

    async def go():
        p, base = await _setup(backend)
        ts = base + 60 * 10
        p.use(p.a)
        good = await create_transaction(GENESIS, address_of(KEYS[0]), '3')
        # double spend across two txs of the block
        dup = Transaction([TransactionInput(good.inputs[0].tx_hash, good.inputs[0].index)],
                          [TransactionOutput(address_of(KEYS[1]), Decimal('1'))])
        dup.inputs[0].public_key = good.inputs[0].public_key
        dup.sign([GENESIS])
        # forged signature
        forged, _ = Transaction.parse(good.hex())
        r, s = forged.inputs[0].signed
        forged.inputs[0].signed = (r, s ^ 0x10)
        # negative fee
        greedy = Transaction([TransactionInput(good.inputs[0].tx_hash, good.inputs[0].index)],
                             [TransactionOutput(address_of(KEYS[1]), Decimal('100'))])
        greedy.inputs[0].public_key = good.inputs[0].public_key
        greedy.sign([GENESIS])
        # unknown input
        ghost = Transaction([TransactionInput('ab' * 32, 0)], [TransactionOutput(address_of(KEYS[1]), Decimal('1'))])
        ghost.inputs[0].signed = good.inputs[0].signed
        # output to a 33-byte address whose x is not on the curve
        from upow_amd.utils import p256 as o
        from upow_amd.utils.codec import bytes_to_string
        x = _off_curve_x()
        off = bytes_to_string(bytes([42]) + x.to_bytes(32, 'little'))
        offc = await create_transaction(GENESIS, off, '1')
        for bad in ([good, dup], [greedy], [ghost], [offc]):
            c = await p.mine(bad, ts=ts)
            res, err = await p.push(c, bad, expect=False)
            assert fastpath.last_path == 'object' and err
        # plainly invalid signatures: decided on the native path with the object path's error (the first bad
        # tx in block order), whatever else the block holds
        spend = [o for o in await p.a.get_spendable_outputs(address_of(GENESIS))
                 if (o.tx_hash, o.index) != (good.inputs[0].tx_hash, good.inputs[0].index)]
        others = []
        for k, inp in zip((2, 3, 4), spend):  # each from its own genesis output: no double spend in the block
            t = Transaction([inp], [TransactionOutput(address_of(KEYS[k]), Decimal('0.5'))])
            t.sign([GENESIS])
            others.append(t)
        forged2, _ = Transaction.parse(others[2].hex())
        r2, s2 = forged2.inputs[0].signed
        forged2.inputs[0].signed = (r2 ^ 0x1, s2)
        for bad in ([forged], [others[0], forged, others[1], forged2], [others[0], forged2, others[1], forged]):
            c = await p.mine(bad, ts=ts)
            res, err = await p.push(c, bad, expect=False)
            assert fastpath.last_path == 'native' and len(err) == 1 and 'has been not verified' in err[0], err
        # merkle mismatch: header committed to other txs
        c = await p.mine([good], ts=ts)
        other = await create_transaction(GENESIS, address_of(KEYS[2]), '1')
        await p.push(c, [other], expect=False)
        # and the honest block still goes through on both
        c = await p.mine([good], ts=ts)
        await p.push(c, [good], expect=True)
        assert fastpath.last_path == 'native'
    asyncio.run(go())


def test_signer_records_native_matches_general():
    """csrc/txcodec.cpp block_signer_records (dedup + batched decompression + record assembly) against
    the numpy path that blocks with 64-byte addresses take: same 160-byte records; an off-curve key makes
    both refuse."""
    from upow_amd.ledger.utxo import PAYLOAD_DTYPE
    from upow_amd.ops.native import lib
    from upow_amd.utils import p256 as o
    rng = random.Random(7)
    pts = [o.get_public_key(rng.randrange(1, o.N)) for _ in range(12)]
    comp = [bytes([43 if q.y & 1 else 42]) + q.x.to_bytes(32, 'little') for q in pts]
    n_in, n_out, n_tx = 40, 30, 20
    pay = np.zeros(n_in, dtype=PAYLOAD_DTYPE)
    for i in range(n_in):
        pay['addr'][i, :33] = np.frombuffer(comp[rng.randrange(12)], np.uint8)
    pay['len'] = 33
    out_addr = np.zeros((n_out, 64), np.uint8)
    for i in range(n_out):
        out_addr[i, :33] = np.frombuffer(comp[rng.randrange(12)], np.uint8)
    out_len = np.full(n_out, 33, np.uint8)
    sigs = np.frombuffer(rng.randbytes(64 * 25), np.uint8).reshape(-1, 64)
    digest = np.frombuffer(rng.randbytes(32 * n_tx), np.uint8).reshape(-1, 32)
    job_input = np.array(sorted(rng.sample(range(n_in), 25)), np.int64)
    sig_ids = np.arange(25, dtype=np.int64)
    job_tx = np.array([rng.randrange(n_tx) for _ in range(25)], np.int64)
    args = (job_input, sigs, sig_ids, digest, job_tx)
    for gpu_min in (1 << 62,):  # host decompression (the GPU variant runs in the block tests)
        st, native = lib().block_signer_records(np.ascontiguousarray(pay['addr']), pay['len'].astype(np.uint8),
                                                out_addr, out_len, *args, gpu_min)
        general = fastpath._signer_records_general(pay, out_addr, out_len, *args, gpu_min)
        assert st == 1 and native == general
        want = comp[0]  # spot check: the first job's signer point
        rec = np.frombuffer(native, np.uint8).reshape(-1, 160)[0]
        signer = bytes(pay['addr'][job_input[0], :33])
        q = pts[comp.index(signer)]
        assert bytes(rec[:64]) == q.x.to_bytes(32, 'little') + q.y.to_bytes(32, 'little') and want
        bad = out_addr.copy()
        x = _off_curve_x()
        bad[3, 1:33] = np.frombuffer(x.to_bytes(32, 'little'), np.uint8)
        st, _ = lib().block_signer_records(np.ascontiguousarray(pay['addr']), pay['len'].astype(np.uint8),
                                           bad, out_len, *args, gpu_min)
        assert st == 0 and fastpath._signer_records_general(pay, bad, out_len, *args, gpu_min) is None
        full = out_len.copy()
        full[5] = 64
        st, _ = lib().block_signer_records(np.ascontiguousarray(pay['addr']), pay['len'].astype(np.uint8),
                                           out_addr, full, *args, gpu_min)
        assert st == -1


def test_stake_block_takes_native_path():
    """A stake tx (STAKE + DELEGATE_VOTING_POWER outputs) decodes natively and its block applies on the
    native path with the object path's ledger (tests/test_fastpath_governance.py has the full lifecycle)."""
    async def go():
        p, base = await _setup()
        p.use(p.a)
        st = await create_stake_transaction(GENESIS, '1')
        assert fastpath.decode([st.hex()]) is not None
        c = await p.mine([st], ts=base + 600)
        await p.push(c, [st], expect=True)
        assert fastpath.last_path == 'native'
    asyncio.run(go())


def test_sync_mode_matches_object_sync():
    """Replaying a chain page (blocks + their coinbase txs, as /get_blocks serves them) through the
    native sync path and through create_block_in_syncing_old gives identical ledgers."""
    async def go():
        p, base = await _setup()
        ts = base + 60 * 10
        p.use(p.a)
        for r in range(2):
            txs = []
            for k in KEYS[:4]:
                tx = await create_transaction(GENESIS, address_of(k), '0.75')
                await p.a.add_pending_transaction(tx)
                txs.append(tx)
            p.use(p.b)
            for t in txs:
                await p.b.add_pending_transaction(t)
            c = await p.mine(txs, ts=ts + 60 * r)
            await p.push(c, txs, expect=True)
        page = await p.a.get_blocks(1, 100)
        src = await Database.create(utxo_backend='host')
        dst = await Database.create(utxo_backend='host')
        from upow_amd.models.transaction import CoinbaseTransaction
        for db, native in ((src, False), (dst, True)):
            Database.instance = db
            last = {}
            for info in page:
                manager.Manager.difficulty = None
                hexes = list(info['transactions'])
                cb = None
                for k, h in enumerate(hexes):
                    t = await Transaction.from_hex(h, False)
                    if isinstance(t, CoinbaseTransaction):
                        cb = t
                        del hexes[k]
                        break
                if native:
                    ok = await fastpath.create_block_from_hex(info['block']['content'], hexes, last_block=last or None,
                                                              coinbase=cb)
                    if hexes:
                        assert fastpath.last_path == 'native'
                else:
                    txs = [await Transaction.from_hex(h) for h in hexes]
                    ok = await manager.create_block_in_syncing_old(info['block']['content'], txs, cb,
                                                                   last or None)
                assert ok
                last = info['block']
        da, dbb = _dump(src), _dump(dst)
        for k in da:
            assert da[k] == dbb[k], k
        assert _dump(src)['blocks'] == _dump(p.a)['blocks']
    asyncio.run(go())


def test_ascii_hex_signature_fallback_matches():
    """transaction_input.py:100-109: a signature over the ASCII hex string of ``hex(False)`` (legacy
    wallets) verifies through the retry pass. Both paths must accept it, with one signature per tx
    and with per-input signatures, and both must still reject a signature over neither form."""
    from upow_amd.ops import p256 as op

    async def go():
        p, base = await _setup()
        ts = base + 60 * 10
        p.use(p.a)
        txs = []
        for k in KEYS[:2]:
            tx = await create_transaction(GENESIS, address_of(k), '1.5')
            msg = tx.hex(False).encode()  # the ASCII form, not bytes.fromhex
            sig = op.sign(msg, GENESIS)
            for i in tx.inputs:
                i.signed = sig
            assert await p.a.add_pending_transaction(tx)  # mempool admission takes the fallback too
            txs.append(tx)
        p.use(p.b)
        for t in txs:
            assert await p.b.add_pending_transaction(t)
        c = await p.mine(txs, ts=ts)
        await p.push(c, txs, expect=True)
        assert fastpath.last_path == 'native'  # accepted by the native retry pass itself
        # a signature over some other message fails both forms on both paths
        p.use(p.a)
        bad = await create_transaction(GENESIS, address_of(KEYS[3]), '1')
        sig = op.sign(b'not the tx', GENESIS)
        for i in bad.inputs:
            i.signed = sig
        c = await p.mine([bad], ts=ts + 60)
        await p.push(c, [bad], expect=False)
    asyncio.run(go())


@pytest.mark.parametrize('seed,backend', [(1, 'host'), (2, 'host'), (3, 'host'),
                                          pytest.param(4, 'gpu', marks=pytest.mark.gpu),
                                          pytest.param(5, 'gpu', marks=pytest.mark.gpu)])
def test_random_blocks_differential(seed, backend, request):
    """Randomised blocks built from the live UTXO set, each carrying one randomly chosen fault (or
    none): both paths must return the same verdict and error and leave identical ledgers (Pair.push
    compares every table, the UTXO index with payloads and the UTXO-set hash). The gpu cases run both
    ledgers on the HBM table and the gfx950 verify/decompress kernels."""
    if backend == 'gpu':
        request.getfixturevalue('gpu')
    rng = random.Random(seed)

    async def go():
        p, base = await _setup(backend)
        ts = base + 60 * 10
        keys = [GENESIS] + KEYS
        # fan the genesis coinbases out to the test keys first (several small outputs each)
        p.use(p.a)
        fan = []
        for k in KEYS:
            tx = await create_transaction(GENESIS, address_of(k), '0.7')
            await p.a.add_pending_transaction(tx)
            fan.append(tx)
        c = await p.mine(fan, ts=ts)
        await p.push(c, fan, expect=True)
        accepted = 0
        for r in range(8):
            ts += 60
            p.use(p.a)
            owners = rng.sample(keys, 3)
            txs, used = [], set()
            for k in owners:
                outs = [o for o in await p.a.get_spendable_outputs(address_of(k))
                        if (o.tx_hash, o.index) not in used]
                if not outs:
                    continue
                ins = outs[:rng.randint(1, min(3, len(outs)))]
                used |= {(i.tx_hash, i.index) for i in ins}
                total = sum(i.amount for i in ins)
                pay = (total * Decimal(rng.randint(1, 9)) / 10).quantize(Decimal('0.00000001'))
                outs_ = [TransactionOutput(address_of(rng.choice(keys)), pay)]
                if total - pay > Decimal('0.01'):
                    outs_.append(TransactionOutput(address_of(k), total - pay - Decimal('0.001')))
                msg = rng.choice([None, None, b'memo %d' % r])
                tx = Transaction(ins, outs_, msg)
                tx.sign([k])
                txs.append(tx)
            if not txs:
                continue
            fault = rng.choice(['none', 'none', 'sig', 'dup_in_block', 'overspend', 'unknown_input', 'zero_out'])
            victim = txs[0]
            if fault == 'sig':
                a_, b_ = victim.inputs[0].signed
                for i in victim.inputs:
                    i.signed = (a_, (b_ ^ 0x5) or 1)
            elif fault == 'dup_in_block':
                twin = Transaction([victim.inputs[0]], [TransactionOutput(address_of(GENESIS), Decimal('0.0001'))])
                twin.sign([owners[0]] if owners else [GENESIS])
                txs.append(twin)
            elif fault == 'overspend':
                victim.outputs[0] = TransactionOutput(victim.outputs[0].address, Decimal('1000000'))
                victim.sign([o for o in owners])
            elif fault == 'unknown_input':
                ghost = Transaction([TransactionInput('cd' * 32, 1)], [TransactionOutput(address_of(GENESIS), Decimal('1'))])
                ghost.inputs[0].signed = victim.inputs[0].signed
                txs.append(ghost)
            elif fault == 'zero_out':
                victim.outputs.append(TransactionOutput(address_of(GENESIS), Decimal('0')))
                victim.sign([o for o in owners])
            hexes = [t.hex() for t in txs]
            c = await p.mine(hexes, ts=ts)
            ok, err = await p.push(c, hexes)
            accepted += bool(ok)
            if fault == 'none':
                assert ok, err
        assert accepted >= 1
    asyncio.run(go())


def test_block_trace_file(tmp_path, monkeypatch):
    """UPOW_TRACE_FILE: one JSON line per validated block with verdict, path, height and stage times."""
    import json
    trace = tmp_path / 'blocks.jsonl'
    monkeypatch.setattr(manager, '_TRACE_PATH', str(trace))

    async def go():
        p, base = await _setup()
        p.use(p.a)
        tx = await create_transaction(GENESIS, address_of(KEYS[0]), '1')
        c = await p.mine([tx], ts=base + 60 * 10)
        await p.push(c, [tx], expect=True)
    asyncio.run(go())
    recs = [json.loads(line) for line in trace.read_text().splitlines()]
    assert recs and all(r['ok'] for r in recs)
    last = recs[-1]
    assert last['path'] == 'native' and last['txs'] == 1 and last['height'] == 9
    assert {'decode_s', 'ecdsa_s', 'apply_commit_s'} <= set(last['stages_ms'])


@pytest.mark.parametrize('backend', ['host', pytest.param('gpu', marks=pytest.mark.gpu)])
def test_grouped_signature_txs_native_and_rejections(backend, request):
    """1 < k < n signatures (reference transaction.py:578-590: inputs grouped by owner key in order of first
    appearance, signature g for group g) on the native path: accepted blocks stay native and match the object
    path; a swapped signature order is rejected identically; more signatures than owner groups raises the
    parser's IndexError on both paths."""
    if backend == 'gpu':
        request.getfixturevalue('gpu')

    async def go():
        p, base = await _setup(backend)
        ts = base + 60 * 10
        p.use(p.a)
        fund = []
        from upow_amd.wallet.builders import create_transaction_to_send_multiple_wallet
        for k in KEYS[:3]:  # three outputs per key
            tx = await create_transaction_to_send_multiple_wallet(GENESIS, [address_of(k)] * 3, ['1.5'] * 3)
            await p.a.add_pending_transaction(tx)
            fund.append(tx)
        c = await p.mine(fund, ts=ts)
        await p.push(c, fund, expect=True)
        p.use(p.a)
        outs = {k: await p.a.get_spendable_outputs(address_of(k)) for k in KEYS[:3]}
        k0, k1, k2 = KEYS[:3]

        def grouped(ins, keys, amount):
            tx = Transaction(ins, [TransactionOutput(address_of(GENESIS), Decimal(amount))])
            return tx.sign(keys)
        a = grouped([outs[k0][0], outs[k1][0], outs[k0][1]], [k0, k1], '4.4')  # groups k0, k1: 2 sigs, 3 inputs
        b = grouped([outs[k1][1], outs[k2][0], outs[k2][1], outs[k1][2]], [k1, k2], '5.9')  # 2 sigs, 4 inputs
        plain = grouped([outs[k2][2]], [k2], '1.4')
        for t in (a, b):
            raw = bytes.fromhex(t.hex())
            assert len(raw) == len(bytes.fromhex(t.hex(False))) + 1 + 128  # two signatures on the wire
        assert fastpath.decode([a.hex(), b.hex()]) is not None
        # rejected: the two signatures swapped (group 0 gets group 1's signature)
        h = a.hex()
        swapped = h[:-256] + h[-128:] + h[-256:-128]
        c_bad = await p.mine([swapped], ts=ts + 60)
        ok, err = await p.push(c_bad, [swapped], expect=False)
        assert fastpath.last_path == 'native' and 'has been not verified' in err[0]  # same error on both paths
        # more signatures than owner groups: the parser's IndexError on both paths
        three = bytes.fromhex(b.hex()) + bytes.fromhex(b.hex())[-64:]
        p.use(p.b)
        c3 = await p.mine([three.hex()], ts=ts + 60)
        with pytest.raises(IndexError):
            await Transaction.from_hex(three.hex())
        with pytest.raises(IndexError):
            await fastpath.create_block_from_hex(c3, [three.hex()])
        c2 = await p.mine([a, b, plain], ts=ts + 60)
        await p.push(c2, [a, b, plain], expect=True)
        assert fastpath.last_path == 'native'
    asyncio.run(go())


def test_resolve_groups_native_matches_python():
    """csrc/txcodec.cpp resolve_groups vs the Python assignment: random owner layouts (33- and 64-byte
    addresses of the same points, repeated keys), matching and mismatching signature counts, governance types."""
    from upow_amd.ledger.utxo import PAYLOAD_DTYPE
    rng = random.Random(4)
    for _ in range(200):
        n_tx = rng.randint(1, 6)
        keys = [rng.randbytes(32) for _ in range(4)]
        in_start, sig_start, addrs, lens, tx_type = [0], [0], [], [], []
        for t in range(n_tx):
            n_in = rng.randint(3, 7)
            for _ in range(n_in):
                k, odd = rng.randrange(4), rng.randrange(2)
                if rng.random() < 0.5:
                    addrs.append(bytes([43 if odd else rng.choice([42, 44])]) + keys[k] + bytes(31)); lens.append(33)
                else:
                    addrs.append(keys[k] + bytes([odd]) + rng.randbytes(31)); lens.append(64)
            in_start.append(in_start[-1] + n_in)
            sig_start.append(sig_start[-1] + rng.randint(2, 4))
            tx_type.append(0 if rng.random() < 0.9 else 6)
        pay = np.zeros(len(addrs), dtype=PAYLOAD_DTYPE)
        pay['addr'] = np.frombuffer(b''.join(addrs), np.uint8).reshape(-1, 64)
        pay['len'] = lens
        grouped = np.array(sorted(rng.sample(range(n_tx), rng.randint(1, n_tx))), np.int64)
        job = np.full(sig_start[-1], -1, np.int64)
        args = (grouped, job, pay, np.array(in_start, np.int32), np.array(sig_start, np.int32), np.array(tx_type, np.uint8))
        a, b = fastpath._resolve_groups(*args), fastpath._resolve_groups_py(*args)
        assert (a is None) == (b is None) and (a is None or (a == b).all())
