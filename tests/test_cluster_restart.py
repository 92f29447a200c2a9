"""Restart-safe cluster replicas (parallel/cluster.py resync): followers keep a durable ledger under
``<data>/rank<N>/``; on start the leader gathers every replica's (tip, tip hash), rolls divergent ones back
to the last common block and re-sends only the blocks above the lowest replica tip. Each case counts the
re-sent blocks (``/cluster_info`` ``last_resync``) and checks the replicas' K12 UTXO hashes agree.
Reference: the node resumes from durable state at startup (upow/node/main.py:246-257, database.py:34-85)."""
import asyncio
import os
import signal
import subprocess
import sys
import time
from decimal import Decimal

import httpx
import pytest

from test_cluster import KEY, _mine_via_api, _prefill
from test_multinode import ROOT, _port


def _start(tmp_path, world, tag):
    port, mport = _port(), _port()
    env = dict(os.environ, UPOW_DATA_DIR=str(tmp_path / 'n'), UPOW_CORE_URL='', UPOW_START_DIFFICULTY='1.0',
               UPOW_UTXO_BACKEND='host', UPOW_DISABLE_GPU='1', UPOW_RATE_LIMIT='0', PYTHONPATH=ROOT,
               UPOW_LOG_LEVEL='WARNING', OMP_NUM_THREADS='1', UPOW_CODEC_THREADS='1')
    log = open(tmp_path / f'cluster_{tag}.log', 'w')
    p = subprocess.Popen([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', str(world),
                          '--master-addr', '127.0.0.1', '--master-port', str(mport), '-m', 'upow_amd.node',
                          '--cluster', '--host', '127.0.0.1', '--port', str(port), '--log-level', 'warning'],
                         env=env, cwd=ROOT, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    url = f'http://127.0.0.1:{port}'
    for _ in range(900):
        try:
            if httpx.get(url + '/get_nodes', timeout=1).status_code == 200:
                return p, log, url
        except Exception:
            time.sleep(0.2)
    _stop(p, log)
    raise AssertionError(open(tmp_path / f'cluster_{tag}.log').read()[-3000:])


def _stop(p, log, follower_dir=None):
    """SIGTERM to the whole job (torchrun itself exits 1 on a signal); the follower must stop gracefully:
    the leader's shutdown sends 'quit', and the follower either snapshots its UTXO index at its tip (a full
    replica) or, a lean one (ledger/lean.py), closes its op log with a final tip marker."""
    snaps = [os.path.join(follower_dir, f) for f in ('utxo_snapshot.bin', 'ledger.sqlite3.oplog')] if follower_dir else []
    before = [os.path.getmtime(f) if os.path.exists(f) else None for f in snaps]
    try:
        os.killpg(p.pid, signal.SIGTERM)
        p.wait(60)
    except subprocess.TimeoutExpired:  # pragma: no cover
        os.killpg(p.pid, signal.SIGKILL)
        raise
    finally:
        log.close()
    if snaps:
        assert any(os.path.exists(f) and os.path.getmtime(f) != b for f, b in zip(snaps, before)), \
            'follower did not stop gracefully'


def _info(url):
    return httpx.get(url + '/cluster_info', timeout=60).json()['result']


def _edit_follower(path, fn):
    from upow_amd.ledger import manager

    async def go():
        from upow_amd.tools import open_ledger
        db = await open_ledger(str(path))  # a lean follower's op log is materialised first
        assert db.utxo.backend_name == 'host'
        manager.Manager.difficulty = None
        try:
            await fn(db)
        finally:
            db.close()
    asyncio.run(go())


@pytest.mark.slow
def test_cluster_restart_resends_only_the_missing_tail(tmp_path, monkeypatch):
    from upow_amd import devnet
    from upow_amd.ledger import manager
    from upow_amd.wallet.builders import address_of
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('1.0'))
    (tmp_path / 'n').mkdir()
    _prefill(tmp_path / 'n' / 'ledger.sqlite3', 4)
    follower = tmp_path / 'n' / 'rank1' / 'ledger.sqlite3'
    fdir = str(follower.parent)
    ts = 1_700_000_000 + 60 * 10

    # first start: the follower has nothing, the whole chain is sent
    p, log, url = _start(tmp_path, 2, 'a')
    try:
        info = _info(url)
        assert info['last_resync']['blocks_sent'] == 4 and info['last_resync']['follower_tips'] == {'1': 0}
        for b in range(2):
            assert _mine_via_api(url, address_of(KEY), ts + 60 * b, []) == {'ok': True}
        reps = _info(url)['replicas']
        assert reps[0]['height'] == reps[1]['height'] == 6 and reps[0]['utxo_hash'] == reps[1]['utxo_hash']
    finally:
        _stop(p, log, fdir)
    assert follower.exists()

    # restart with both replicas at the tip: nothing is re-sent
    p, log, url = _start(tmp_path, 2, 'b')
    try:
        info = _info(url)
        assert info['last_resync']['blocks_sent'] == 0 and info['last_resync']['follower_tips'] == {'1': 6}, info
        r0, r1 = info['replicas']
        assert r0['height'] == r1['height'] == 6 and r0['utxo_hash'] == r1['utxo_hash']
    finally:
        _stop(p, log, fdir)

    # the follower lost its last two blocks: exactly those two are re-sent
    async def behind(db):
        await db.remove_blocks(5)
        assert db._tip_id() == 4
    _edit_follower(follower, behind)
    p, log, url = _start(tmp_path, 2, 'c')
    try:
        info = _info(url)
        assert info['last_resync']['blocks_sent'] == 2 and info['last_resync']['follower_tips'] == {'1': 4}, info
        assert info['last_resync']['blocks_rolled_back'] == 0
        r0, r1 = info['replicas']
        assert (r0['height'], r0['tip_hash'], r0['utxo_hash']) == (r1['height'], r1['tip_hash'], r1['utxo_hash'])
    finally:
        _stop(p, log)

    # the follower holds a different block 6 (a fork): it rolls back one block and receives the leader's
    async def fork(db):
        await db.remove_blocks(6)
        await devnet.mine_block(address_of(KEY), ts=ts + 60 * 7 + 13, device='cpu')  # another block 6
        assert db._tip_id() == 6
    _edit_follower(follower, fork)
    p, log, url = _start(tmp_path, 2, 'd')
    try:
        info = _info(url)
        rs = info['last_resync']
        assert rs['blocks_rolled_back'] == 1 and rs['blocks_sent'] == 1 and rs['follower_tips'] == {'1': 5}, info
        r0, r1 = info['replicas']
        assert (r0['height'], r0['tip_hash'], r0['utxo_hash']) == (r1['height'], r1['tip_hash'], r1['utxo_hash'])
        deep = httpx.get(url + '/cluster_info', params={'deep': 'true'}, timeout=60).json()['result']['replicas']
        assert deep[0]['sql_utxo_hash'] == deep[1]['sql_utxo_hash'] == deep[0]['utxo_hash']
    finally:
        _stop(p, log)
