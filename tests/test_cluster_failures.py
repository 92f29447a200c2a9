"""Failure paths of the multi-GPU cluster node (parallel/cluster.py, parallel/dist.py), two ranks over gloo.

* A follower that rejects a block the leader accepts: the replicas vote right before committing
  (``commit_gate``), the split vote is a divergence, every rank exits with status 70 and no replica's tip
  passes the block before; a relaunch resyncs cleanly (nothing to re-send) and the chain continues.
* A follower killed with SIGKILL: the leader's next collective (its idle heartbeat) fails and the leader
  exits with status 70 within the op timeout plus a margin, instead of hanging; the relaunch re-sends only
  what the follower lacks and the replicas' K12 UTXO hashes agree.
* A start-up replay that lasts longer than the op timeout: it runs on the long-timeout group with periodic
  acknowledgements, so the node comes up.
* A collective issued from a thread other than the owner raises before touching the communicator.

Reference: the reference node reverts a failed sync to its cached chain (upow/node/main.py:218-226); a
cluster node's equivalent is that no replica ever commits a block the others do not."""
import asyncio
import os
import signal
import subprocess
import sys
import threading
import time
from decimal import Decimal

import httpx
import pytest

from test_cluster import KEY, _mine_via_api, _prefill
from test_multinode import ROOT, _port

LAUNCH = '''
import os, sys, time
sys.path.insert(0, {root!r})
if os.environ.get('RANK') == '1':
    from upow_amd.ledger import fastpath, manager
    reject_at = int(os.environ.get('TEST_REJECT_AT', '0'))
    delay = float(os.environ.get('TEST_REPLAY_DELAY', '0'))
    stall = [float(os.environ.get('TEST_REPLAY_STALL', '0'))]
    if reject_at:
        orig_hdr = manager.check_block_header

        async def check_block_header(block_content, mining_info, error_list):
            res = await orig_hdr(block_content, mining_info, error_list)
            if res is not None and res[0] == reject_at:
                error_list.append('injected rejection')
                return None
            return res
        manager.check_block_header = check_block_header
    if delay or stall[0]:
        orig_create = fastpath.create_block_from_hex

        async def create_block_from_hex(*a, **kw):
            time.sleep(delay + stall[0])
            stall[0] = 0.0
            return await orig_create(*a, **kw)
        fastpath.create_block_from_hex = create_block_from_hex
from upow_amd.node.__main__ import main
main()
'''


def _launch(tmp_path, tag, extra=None, world=2):
    """The ranks of a cluster node started directly (what torchrun does: RANK/WORLD_SIZE/MASTER_* per
    process), so each rank's own exit status is visible. Returns (procs, logs, url)."""
    script = tmp_path / 'launch.py'
    script.write_text(LAUNCH.format(root=ROOT))
    port, mport = _port(), _port()
    base = dict(os.environ, UPOW_DATA_DIR=str(tmp_path / 'n'), UPOW_CORE_URL='', UPOW_START_DIFFICULTY='1.0',
                UPOW_UTXO_BACKEND='host', UPOW_DISABLE_GPU='1', UPOW_RATE_LIMIT='0', PYTHONPATH=ROOT,
                UPOW_LOG_LEVEL='WARNING', OMP_NUM_THREADS='1', UPOW_CODEC_THREADS='1', MASTER_ADDR='127.0.0.1',
                MASTER_PORT=str(mport), WORLD_SIZE=str(world), **(extra or {}))
    procs, logs = [], []
    for r in range(world):
        log = open(tmp_path / f'{tag}_rank{r}.log', 'w')
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, str(script), '--cluster', '--host', '127.0.0.1', '--port',
                                       str(port), '--log-level', 'warning'], env=env, cwd=ROOT, stdout=log,
                                      stderr=subprocess.STDOUT, start_new_session=True))
        logs.append(log)
    url = f'http://127.0.0.1:{port}'
    for _ in range(900):
        try:
            if httpx.get(url + '/get_nodes', timeout=1).status_code == 200:
                return procs, logs, url
        except Exception:
            if any(p.poll() is not None for p in procs):
                break
            time.sleep(0.2)
    _kill(procs, logs)
    raise AssertionError(''.join(open(tmp_path / f'{tag}_rank{r}.log').read()[-2000:] for r in range(world)))


def _kill(procs, logs):
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait(30)
    for log in logs:
        log.close()


def _stop(procs, logs):
    """Graceful stop: SIGTERM to the leader (its shutdown sends 'quit'); the follower then exits on its own."""
    try:
        procs[0].send_signal(signal.SIGTERM)
        for p in procs:
            p.wait(60)
    finally:
        _kill(procs, logs)


def _tips(tmp_path):
    from upow_amd.ledger.database import Database

    async def go(path):
        from upow_amd.tools import open_ledger
        db = await open_ledger(str(path))  # a lean follower's op log is materialised first
        try:
            return db._tip_id()
        finally:
            db.close()
    return [asyncio.run(go(tmp_path / 'n' / 'ledger.sqlite3')),
            asyncio.run(go(tmp_path / 'n' / 'rank1' / 'ledger.sqlite3'))]


def _info(url):
    return httpx.get(url + '/cluster_info', timeout=60).json()['result']


def test_collective_from_a_non_owner_thread_raises():
    from upow_amd.parallel.dist import DistContext
    ctx = DistContext(rank=0, world=2)
    ctx.bind_owner()
    errors = []

    def other():
        for call in (lambda: ctx.allreduce_sum(1), lambda: ctx.broadcast_frame(b'x', src=0),
                     lambda: ctx.all_gather_fixed(b'abcd')):
            try:
                call()
            except RuntimeError as e:
                errors.append(str(e))
    t = threading.Thread(target=other, name='not-the-owner')
    t.start()
    t.join(30)
    assert len(errors) == 3 and all('not the owner thread' in e for e in errors), errors
    assert ctx.collectives == 0  # refused before anything was counted or sent


@pytest.mark.slow
def test_follower_rejecting_a_block_stops_every_rank_before_commit(tmp_path, monkeypatch):
    from upow_amd.ledger import manager
    from upow_amd.wallet.builders import address_of
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('1.0'))
    (tmp_path / 'n').mkdir()
    _prefill(tmp_path / 'n' / 'ledger.sqlite3', 4)
    ts = 1_700_000_000 + 60 * 10
    procs, logs, url = _launch(tmp_path, 'a', {'TEST_REJECT_AT': '6', 'UPOW_SNAPSHOT': '0'})
    try:
        assert _mine_via_api(url, address_of(KEY), ts, []) == {'ok': True}  # block 5: both replicas accept
        try:
            _mine_via_api(url, address_of(KEY), ts + 60, [])  # block 6: the follower rejects it
        except Exception:
            pass  # the leader exits while answering
        codes = [p.wait(60) for p in procs]
    finally:
        _kill(procs, logs)
    assert codes == [70, 70], codes
    text = open(tmp_path / 'a_rank0.log').read() + open(tmp_path / 'a_rank1.log').read()
    assert 'diverged' in text
    assert _tips(tmp_path) == [5, 5]  # nobody committed block 6
    # relaunch without the fault: the replicas agree, nothing is re-sent, and the chain continues
    procs, logs, url = _launch(tmp_path, 'b', {'UPOW_SNAPSHOT': '0'})
    try:
        info = _info(url)
        assert info['last_resync']['blocks_sent'] == 0 and info['last_resync']['follower_tips'] == {'1': 5}, info
        assert _mine_via_api(url, address_of(KEY), ts + 120, []) == {'ok': True}
        r0, r1 = _info(url)['replicas']
        assert (r0['height'], r0['tip_hash'], r0['utxo_hash']) == (6, r1['tip_hash'], r1['utxo_hash'])
    finally:
        _stop(procs, logs)


@pytest.mark.slow
def test_killed_follower_ends_the_leader_with_status_70(tmp_path, monkeypatch):
    import psutil
    from upow_amd.ledger import manager
    from upow_amd.wallet.builders import address_of
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('1.0'))
    (tmp_path / 'n').mkdir()
    _prefill(tmp_path / 'n' / 'ledger.sqlite3', 3)
    timeout_s = 5
    procs, logs, url = _launch(tmp_path, 'a', {'UPOW_DIST_TIMEOUT_S': str(timeout_s), 'UPOW_CLUSTER_HEARTBEAT_S': '1',
                                               'UPOW_SNAPSHOT': '0'})
    ts = 1_700_000_000 + 60 * 10
    try:
        for b in range(2):
            assert _mine_via_api(url, address_of(KEY), ts + 60 * b, []) == {'ok': True}
        psutil.Process(procs[1].pid).kill()  # SIGKILL mid-run
        t0 = time.monotonic()
        code = procs[0].wait(timeout_s + 10)
        dt = time.monotonic() - t0
    finally:
        _kill(procs, logs)
    assert code == 70 and dt <= timeout_s + 10, (code, dt)
    leader_tip, follower_tip = _tips(tmp_path)
    procs, logs, url = _launch(tmp_path, 'b', {'UPOW_SNAPSHOT': '0'})
    try:
        info = _info(url)
        assert info['last_resync']['blocks_sent'] == leader_tip - follower_tip == 0, info
        r0, r1 = info['replicas']
        assert (r0['height'], r0['tip_hash'], r0['utxo_hash']) == (5, r1['tip_hash'], r1['utxo_hash'])
    finally:
        _stop(procs, logs)


@pytest.mark.slow
def test_resync_longer_than_the_op_timeout(tmp_path, monkeypatch):
    from upow_amd.ledger import manager
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('1.0'))
    (tmp_path / 'n').mkdir()
    _prefill(tmp_path / 'n' / 'ledger.sqlite3', 40)
    # 40 replayed blocks at 0.1 s each on the follower (4 s of replay) and one 3 s stall, against a 2 s op
    # timeout: over gloo the leader's next collective waits out the stall, over RCCL its queued broadcasts
    # would; either exceeds the op timeout, neither the resync group's
    procs, logs, url = _launch(tmp_path, 'a', {'UPOW_DIST_TIMEOUT_S': '2', 'TEST_REPLAY_DELAY': '0.1',
                                               'TEST_REPLAY_STALL': '3', 'UPOW_SNAPSHOT': '0'})
    try:
        info = _info(url)
        assert info['last_resync']['blocks_sent'] == 40, info
        r0, r1 = info['replicas']
        assert (r0['height'], r0['utxo_hash']) == (40, r1['utxo_hash'])
    finally:
        _stop(procs, logs)
