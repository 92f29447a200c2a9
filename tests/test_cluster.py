"""Multi-GPU cluster node (parallel/cluster.py) under torchrun with 2 ranks (gloo on CPU here, RCCL
on a GPU node): rank 0 serves the API, rank 1 is a replica fed by the op stream; replay at start,
mirrored blocks/mempool, sharded signature verification, replica audit via /cluster_info."""
import asyncio
import hashlib
import os
import signal
import subprocess
import sys
import time
from decimal import Decimal

import httpx
import pytest

from test_multinode import ROOT, _port

KEY = 0xC1C1C1


def _prefill(path, blocks):
    from upow_amd import devnet
    from upow_amd.ledger import manager
    from upow_amd.ledger.database import Database
    from upow_amd.wallet.builders import address_of

    async def go():
        db = await Database.create(path=str(path), utxo_backend='host')
        manager.Manager.difficulty = None
        for b in range(blocks):
            await devnet.mine_block(address_of(KEY), ts=1_700_000_000 + 60 * b, device='cpu')
        db.close()
    asyncio.run(go())


def _mine_via_api(url, address, ts, tx_hexes):
    from upow_amd.models.block import PowTarget, get_transactions_merkle_tree, header_prefix
    from upow_amd.ops.pow import PowJob, search
    info = httpx.get(url + '/get_mining_info', timeout=10).json()['result']
    prev = info['last_block']['hash']
    merkle = get_transactions_merkle_tree(tx_hexes)
    hashes = [hashlib.sha256(bytes.fromhex(h)).hexdigest() for h in tx_hexes]
    job = PowJob.create(header_prefix(prev, address, merkle, ts, info['difficulty']),
                        PowTarget.from_difficulty(prev, info['difficulty']))
    r = search(job, 0, 1 << 20, device='cpu', threads=2)
    content = job.header_with_nonce(r.nonces[0]).hex()
    return httpx.post(url + '/push_block', json={'block_content': content, 'txs': sorted(hashes),
                                                 'block_no': info['last_block']['id'] + 1}, timeout=60).json()


@pytest.mark.slow
def test_cluster_node_replicates_and_shards(tmp_path, monkeypatch):
    from upow_amd.ledger import manager
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('1.0'))
    (tmp_path / 'n').mkdir()
    _prefill(tmp_path / 'n' / 'ledger.sqlite3', 4)
    import shutil
    from upow_amd.ledger.database import copy_ledger
    copy_ledger(tmp_path / 'n' / 'ledger.sqlite3', tmp_path / 'wallet.sqlite3')  # the test's own view
    port, mport = _port(), _port()
    env = dict(os.environ, UPOW_DATA_DIR=str(tmp_path / 'n'), UPOW_CORE_URL='', UPOW_START_DIFFICULTY='1.0',
               UPOW_UTXO_BACKEND='host', UPOW_DISABLE_GPU='1', UPOW_RATE_LIMIT='0', PYTHONPATH=ROOT,
               UPOW_LOG_LEVEL='WARNING', UPOW_SNAPSHOT='0')
    log = open(tmp_path / 'cluster.log', 'w')
    p = subprocess.Popen([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
                          '--master-addr', '127.0.0.1', '--master-port', str(mport), '-m', 'upow_amd.node',
                          '--cluster', '--host', '127.0.0.1', '--port', str(port), '--log-level', 'warning'],
                         env=env, cwd=ROOT, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    url = f'http://127.0.0.1:{port}'
    try:
        for _ in range(600):
            try:
                if httpx.get(url + '/get_nodes', timeout=1).status_code == 200:
                    break
            except Exception:
                time.sleep(0.2)
        else:
            raise AssertionError(open(tmp_path / 'cluster.log').read()[-3000:])
        info = httpx.get(url + '/cluster_info', timeout=30).json()['result']
        assert info['world'] == 2 and info['backend'] == 'gloo'
        r0, r1 = info['replicas']
        assert r0['height'] == r1['height'] == 4 and r0['utxo_hash'] == r1['utxo_hash']  # replayed at start

        from upow_amd.wallet.builders import address_of, create_transaction
        from upow_amd.ledger.database import Database

        async def build():  # txs built against a copy of the leader's ledger (same UTXO set)
            db = await Database.create(path=str(tmp_path / 'wallet.sqlite3'), utxo_backend='host')
            out = []
            for k in range(3):
                tx = await create_transaction(KEY, address_of(0xD00 + k), '1.25')
                await db.add_pending_transaction(tx)  # local only: keeps builder input selection disjoint
                out.append(tx)
            db.close()
            return out
        txs = asyncio.run(build())
        for tx in txs:
            assert httpx.post(url + '/push_tx', json={'tx_hex': tx.hex()}, timeout=30).json()['ok']
        res = _mine_via_api(url, address_of(KEY), 1_700_000_000 + 60 * 10, [tx.hex() for tx in txs])
        assert res == {'ok': True}, res
        res = _mine_via_api(url, address_of(KEY), 1_700_000_000 + 60 * 11, [])
        assert res == {'ok': True}, res
        info = httpx.get(url + '/cluster_info', timeout=30).json()['result']
        r0, r1 = info['replicas']
        assert r0['height'] == r1['height'] == 6
        assert r0['utxo_hash'] == r1['utxo_hash'] and r0['utxo_entries'] == r1['utxo_entries']
        assert httpx.get(url + '/get_address_info', params={'address': address_of(0xD01)}, timeout=10).json()[
            'result']['balance'] == '1.25'
    finally:
        try:
            os.killpg(p.pid, signal.SIGTERM)
            p.wait(20)
        except Exception:
            os.killpg(p.pid, signal.SIGKILL)
        log.close()
