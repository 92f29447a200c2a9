"""Wallet CLIs: key store, balance, send through the DB wallet (reference wallet.py / nodeless_wallet.py)."""
import asyncio
import json
from decimal import Decimal

import pytest

from upow_amd import devnet
from upow_amd.ledger import manager
from upow_amd.ledger.database import Database


@pytest.fixture
def env(tmp_path, monkeypatch):
    monkeypatch.setenv('UPOW_DATA_DIR', str(tmp_path))
    monkeypatch.setenv('UPOW_WALLET_NODE_URL', 'http://127.0.0.1:9/')  # unreachable -> direct mempool insert
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('1.0'))
    manager.Manager.difficulty = None
    db = asyncio.run(Database.create(utxo_backend='host'))
    yield tmp_path, db
    db.close()


def test_db_wallet_create_balance_send(env, capsys):
    tmp, db = env
    from upow_amd.wallet import cli
    asyncio.run(cli.main(['createwallet']))
    keys = json.loads((tmp / 'key_pair_list.json').read_text())['keys']
    assert len(keys) == 1
    addr = keys[0]['public_key']

    async def mine():
        for k in range(3):
            await devnet.mine_block(addr, ts=1_700_000_000 + k)
    asyncio.run(mine())
    asyncio.run(cli.main(['balance']))
    out = capsys.readouterr().out
    assert 'Balance: 18' in out and addr in out
    from upow_amd.wallet.builders import address_of
    tx = asyncio.run(cli.main(['send', '-to', address_of(0x77), '-a', '2']))
    assert tx is not None
    pend = asyncio.run(db.get_pending_transactions_limit())
    assert [t.hash() for t in pend] == [tx.hash()]
    asyncio.run(cli.main(['balance']))
    assert 'pending' in capsys.readouterr().out


def test_nodeless_createwallet(env, capsys):
    tmp, _ = env
    from upow_amd.wallet import nodeless
    nodeless.main(['createwallet'])
    data = json.loads((tmp / 'upow_wallet.json').read_text())
    assert len(data['private_keys']) == 1
    assert 'Address:' in capsys.readouterr().out
