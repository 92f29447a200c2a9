"""Fork resolution during sync (reference upow/node/main.py:153-227): two node processes share 520
blocks, then diverge; the node on the shorter branch rolls back to the common block and adopts the
longer chain, and the UTXO-set hashes agree afterwards."""
import asyncio
import os
import shutil
import subprocess
import sys
import time
from decimal import Decimal

import httpx
import pytest

from test_multinode import ROOT, _port

COMMON, A_EXTRA, B_EXTRA = 520, 3, 6


def _build_chain(path, n_blocks, key, start_ts, extend_from=None):
    from upow_amd import devnet
    from upow_amd.ledger import manager
    from upow_amd.ledger.database import Database
    from upow_amd.wallet.builders import address_of

    async def go():
        db = await Database.create(path=str(path), utxo_backend='host')
        manager.Manager.difficulty = None
        addr = address_of(key)
        h = await db.get_next_block_id()
        for k in range(n_blocks):
            await devnet.mine_block(addr, ts=start_ts + 60 * (h + k), device='cpu')
        tip = await db.get_last_block()
        db.close()
        return tip
    return asyncio.run(go())


@pytest.mark.slow
def test_fork_rollback_and_resync(tmp_path, monkeypatch):
    from upow_amd.ledger import manager
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('1.0'))
    start = int(time.time()) - 60 * 700
    (tmp_path / 'a').mkdir()
    (tmp_path / 'b').mkdir()
    a_db, b_db = tmp_path / 'a' / 'ledger.sqlite3', tmp_path / 'b' / 'ledger.sqlite3'
    _build_chain(a_db, COMMON, 0x61, start)
    from upow_amd.ledger.database import copy_ledger
    copy_ledger(a_db, b_db)
    tip_a = _build_chain(a_db, A_EXTRA, 0x61, start)     # branch A: 523 blocks
    tip_b = _build_chain(b_db, B_EXTRA, 0x61, start + 7)  # branch B: 526 blocks (same genesis miner, other timestamps)
    assert tip_a['id'] == COMMON + A_EXTRA and tip_b['id'] == COMMON + B_EXTRA and tip_a['hash'] != tip_b['hash']

    procs = []
    try:
        urls = []
        for name in ('a', 'b'):
            port = _port()
            env = dict(os.environ, UPOW_DATA_DIR=str(tmp_path / name), UPOW_CORE_URL='', UPOW_START_DIFFICULTY='1.0',
                       UPOW_UTXO_BACKEND='host', UPOW_DISABLE_GPU='1', UPOW_RATE_LIMIT='0', PYTHONPATH=ROOT,
                       UPOW_LOG_LEVEL='WARNING')
            procs.append(subprocess.Popen([sys.executable, '-m', 'upow_amd.node', '--host', '127.0.0.1', '--port',
                                           str(port), '--log-level', 'warning'], env=env, cwd=ROOT,
                                          stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL))
            urls.append(f'http://127.0.0.1:{port}')
        for u in urls:
            for _ in range(300):
                try:
                    if httpx.get(u + '/get_nodes', timeout=1).status_code == 200:
                        break
                except Exception:
                    time.sleep(0.1)
        a, b = urls
        assert httpx.get(a + '/get_block', params={'block': COMMON + A_EXTRA}).json()['result']['block']['hash'] == tip_a['hash']
        res = httpx.get(a + '/sync_blockchain', params={'node_url': b}, timeout=120).json()
        assert res == {'ok': True}, res
        ha = httpx.get(a + '/get_block', params={'block': COMMON + B_EXTRA}).json()['result']['block']['hash']
        assert ha == tip_b['hash']
        assert httpx.get(a + '/get_block', params={'block': COMMON + B_EXTRA + 1}).json()['ok'] is False
        assert httpx.get(a + '/').json()['unspent_outputs_hash'] == httpx.get(b + '/').json()['unspent_outputs_hash']
    finally:
        for p in procs:
            p.terminate()
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                p.kill()
