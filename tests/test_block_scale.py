"""A full-size block of random-keypair traffic through both block paths.

BASELINE's verify workload: a 2 MB block of 8,300 two-in/two-out txs, each signed by its own fresh P-256
key and paying a fresh address (~8,300 distinct signers, ~16,600 distinct output addresses; built by
``bench_verify._setup(distinct_keys=True)``, the benchmark's own block builder). One ledger takes it through
the object path (``manager.create_block`` over ``Transaction.from_hex``; reference upow/manager.py:
create_block), the other through the native path (``fastpath.create_block_from_hex``): both must accept,
and every table, the UTXO index and both UTXO-set hashes must be identical afterwards. On the GPU this runs
the block-latency verify kernel, the decompression kernel and the HBM UTXO table at full block size."""
import asyncio
from decimal import Decimal

import pytest

from upow_amd import devnet
from upow_amd.ledger import fastpath, manager
from upow_amd.ledger.database import OUTPUT_TABLES, Database
from upow_amd.models.transaction import Transaction

TABLES = ['blocks', 'transactions', 'address_transactions', *OUTPUT_TABLES]


@pytest.fixture(autouse=True)
def _low_difficulty(monkeypatch):
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('1.0'))


def _dump(db):
    out = {t: sorted(tuple(r) for r in db._q(f'SELECT * FROM {t}')) for t in TABLES}
    recs, pay = db.utxo.records_payload()
    out['index'] = (recs.tobytes(), pay.tobytes())
    return out


def _use(db):
    Database.instance = db
    manager.Manager.difficulty = None


@pytest.mark.parametrize('backend', ['host', pytest.param('gpu', marks=pytest.mark.gpu)])
def test_full_size_distinct_key_block_both_paths(backend, request):
    if backend == 'gpu':
        request.getfixturevalue('gpu')
    from upow_amd.bench_verify import _setup
    n = 8300
    device = 'gpu' if backend == 'gpu' else 'cpu'

    async def go():
        # the same seed builds the same funding set, keys and block on both ledgers
        a, addr, blocks, base_ts = await _setup(1, n, 4242, utxo_backend=backend, device=device, distinct_keys=True)
        b, _, _, _ = await _setup(1, n, 4242, utxo_backend=backend, device=device, distinct_keys=True,
                                  make_blocks=False, base_ts=base_ts)
        hexes = blocks[0]
        assert len(hexes) == n
        assert sum(len(h) for h in hexes) // 2 > 1_750_000  # 8,300 x 214 B: the 2 MB block cap nearly full
        _use(a)
        content = await devnet.mine_header(addr, hexes, ts=base_ts + 10, device='cpu')
        ea = []
        ok_a = await manager.create_block(content, [await Transaction.from_hex(h) for h in hexes], error_list=ea)
        _use(b)
        eb = []
        ok_b = await fastpath.create_block_from_hex(content, hexes, error_list=eb)
        assert ok_a and ok_b, (ea, eb)
        assert fastpath.last_path == 'native'
        a.index_addresses()
        b.index_addresses()
        da, dbb = _dump(a), _dump(b)
        for k in da:
            assert da[k] == dbb[k], k
        _use(a)
        h = a.sql_unspent_outputs_hash()
        assert h == b.sql_unspent_outputs_hash() == await a.get_unspent_outputs_hash() \
            == await b.get_unspent_outputs_hash()
        # the block's ~8,300 signers and ~16,600 fresh outputs are all distinct
        assert len(da['blocks']) == 3
        a.close()
        b.close()
    asyncio.run(go())


@pytest.mark.parametrize('backend', ['host', pytest.param('gpu', marks=pytest.mark.gpu)])
def test_full_size_block_of_bad_signatures_rejected_natively(backend, request):
    """A hostile 2 MB block: every one of its 8,300 txs carries a signature that verifies under neither message
    form. The native path decides it (the object path's error: the first bad tx in block order) instead of
    handing 8,300 txs to the per-tx Python re-validation; the object path agrees, and neither ledger moves."""
    if backend == 'gpu':
        request.getfixturevalue('gpu')
    import time
    from upow_amd.bench_verify import _setup
    n = 8300
    device = 'gpu' if backend == 'gpu' else 'cpu'

    async def go():
        a, addr, blocks, base_ts = await _setup(1, n, 4343, utxo_backend=backend, device=device, distinct_keys=True)
        b, _, _, _ = await _setup(1, n, 4343, utxo_backend=backend, device=device, distinct_keys=True,
                                  make_blocks=False, base_ts=base_ts)
        # flip one bit of s in each tx's (only) signature: the last 64 bytes on the wire are (r, s)
        hexes = []
        for h in blocks[0]:
            raw = bytearray.fromhex(h)
            raw[-1] ^= 0x01
            hexes.append(raw.hex())
        _use(a)
        content = await devnet.mine_header(addr, hexes, ts=base_ts + 10, device='cpu')
        before = a.sql_unspent_outputs_hash()
        ea = []
        assert not await manager.create_block(content, [await Transaction.from_hex(h) for h in hexes], error_list=ea)
        _use(b)
        eb = []
        t = time.perf_counter()
        assert not await fastpath.create_block_from_hex(content, hexes, error_list=eb)
        native_s = time.perf_counter() - t
        assert fastpath.last_path == 'native'
        assert ea == eb and len(eb) == 1 and eb[0].endswith('has been not verified'), (ea, eb)
        assert a.sql_unspent_outputs_hash() == b.sql_unspent_outputs_hash() == before
        assert native_s < 30, native_s
        a.close()
        b.close()
    asyncio.run(go())
