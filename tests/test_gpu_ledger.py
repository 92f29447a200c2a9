"""End-to-end block validation with the GPU backends (HBM UTXO index + batched P-256 kernels)."""
import asyncio
import argparse

import pytest


@pytest.mark.gpu
def test_verify_bench_pipeline_on_gpu(gpu, monkeypatch):
    from decimal import Decimal
    from upow_amd import constants
    from upow_amd.ledger import manager
    monkeypatch.setattr(constants, 'START_DIFFICULTY', Decimal('4.0'))
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('4.0'))
    from upow_amd.bench_verify import run_verify_bench
    from upow_amd.parallel.dist import DistContext
    args = argparse.Namespace(steps=1, warmup=1, txs=600)
    out = run_verify_bench(args, DistContext())
    assert out['config']['utxo_backend'] == 'gpu' and out['config']['device'] == 'gpu'
    assert out['config']['block_path'] == 'native'
    assert out['value'] > 0


@pytest.mark.gpu
def test_gpu_index_snapshot_roundtrip(gpu, tmp_path, monkeypatch):
    """HBM index: dump -> canonical records -> K12 equals SQL; snapshot restore into a fresh table."""
    from decimal import Decimal
    from upow_amd import devnet
    from upow_amd.ledger import manager, snapshot
    from upow_amd.ledger.database import Database
    from upow_amd.wallet.builders import address_of, create_transaction
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('2.0'))

    async def go():
        path = str(tmp_path / 'g.sqlite3')
        db = await Database.create(path=path, utxo_backend='gpu')
        addr = address_of(0x4242)
        for b in range(6):
            await devnet.mine_block(addr, ts=1_700_000_000 + 60 * b)
        tx = await create_transaction(0x4242, address_of(0x99), '7')
        await devnet.mine_block(addr, [tx], ts=1_700_000_000 + 600)
        assert db.utxo.set_hash() == db.sql_unspent_outputs_hash() == await db.get_unspent_outputs_hash()
        # K12 off the block path: the snapshot is this state even when the table changes before the digest
        before = db.utxo.set_hash()
        digest = db.utxo.k12_snapshot(0)
        await devnet.mine_block(addr, ts=1_700_000_000 + 660)
        assert digest() == before != db.utxo.set_hash()
        snapshot.save(db)
        n = len(db.utxo)
        db.close()
        db2 = await Database.create(path=path, utxo_backend='gpu')
        assert db2.utxo_source == 'snapshot' and len(db2.utxo) == n and snapshot.verify(db2)['ok']
        db2.close()
    asyncio.run(go())


@pytest.mark.gpu
def test_sync_bench_pipeline_on_gpu(gpu, monkeypatch):
    """Chain sync replay (node.main.create_blocks: decode-ahead thread + native block path) on the
    HBM UTXO index: the replica reaches the source tip."""
    from decimal import Decimal
    from upow_amd import constants
    from upow_amd.ledger import manager
    monkeypatch.setattr(constants, 'START_DIFFICULTY', Decimal('4.0'))
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('4.0'))
    from upow_amd.bench_verify import run_sync_bench
    from upow_amd.parallel.dist import DistContext
    out = run_sync_bench(argparse.Namespace(steps=2, warmup=1, txs=500), DistContext())
    assert out['config']['utxo_backend'] == 'gpu' and out['config']['block_path'] == 'native'
    assert out['value'] > 0


def test_sync_bench_pipeline_host(monkeypatch):
    """Same replay on the host backend (CPU container): exercises the pipelined create_blocks."""
    from decimal import Decimal
    from upow_amd import constants
    from upow_amd.ledger import manager
    from upow_amd.ops import native
    monkeypatch.setattr(constants, 'START_DIFFICULTY', Decimal('2.0'))
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('2.0'))
    monkeypatch.setattr(native, 'gpu_available', lambda: False)
    from upow_amd.bench_verify import run_sync_bench
    from upow_amd.parallel.dist import DistContext
    # a /get_blocks page is capped at 8 x MAX_BLOCK_SIZE_HEX: shrink the cap so the replay needs
    # several pages, as 10 full 2 MB blocks do
    from upow_amd.ledger import database
    monkeypatch.setattr(database, 'MAX_BLOCK_SIZE_HEX', 120 * 560 // 8)
    out = run_sync_bench(argparse.Namespace(steps=3, warmup=1, txs=120), DistContext())
    assert out['config']['block_path'] == 'native' and out['value'] > 0
