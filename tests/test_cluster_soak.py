"""Cluster node soak (parallel/cluster.py, 4 ranks over gloo): /push_tx keeps answering while blocks are
validated and applied on all replicas. Admissions only queue their tx for the next batched 'txs' op
(no collective per tx, no hop through the ledger thread), so a push that lands while a block is being
applied does not wait for it. Reports push latency percentiles overall and during block application
into ``cluster_soak.json`` under the test's tmp dir, and checks every replica ends on the same state."""
import asyncio
import json
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


def _pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))] if xs else None


@pytest.mark.slow
def test_cluster_world4_push_latency_during_block_apply(tmp_path, monkeypatch):
    from upow_amd.ledger import manager
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('1.0'))
    (tmp_path / 'n').mkdir()
    _prefill(tmp_path / 'n' / 'ledger.sqlite3', 48)
    from upow_amd.ledger.database import copy_ledger
    copy_ledger(tmp_path / 'n' / 'ledger.sqlite3', tmp_path / 'wallet.sqlite3')
    from upow_amd.ledger.database import Database
    from upow_amd.wallet.builders import address_of, create_transaction

    async def build():
        db = await Database.create(path=str(tmp_path / 'wallet.sqlite3'), utxo_backend='host')
        out = []
        for k in range(40):
            tx = await create_transaction(KEY, address_of(0xE00 + k), '0.5')
            await db.add_pending_transaction(tx)
            out.append(tx)
        db.close()
        return out
    txs = asyncio.run(build())
    port, mport = _port(), _port()
    env = dict(os.environ, UPOW_DATA_DIR=str(tmp_path / 'n'), UPOW_CORE_URL='', UPOW_START_DIFFICULTY='1.0',
               UPOW_UTXO_BACKEND='host', UPOW_DISABLE_GPU='1', UPOW_RATE_LIMIT='0', PYTHONPATH=ROOT,
               UPOW_LOG_LEVEL='WARNING', UPOW_SNAPSHOT='0', OMP_NUM_THREADS='1', UPOW_CODEC_THREADS='1')
    log = open(tmp_path / 'cluster.log', 'w')
    p = subprocess.Popen([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '4',
                          '--master-addr', '127.0.0.1', '--master-port', str(mport), '-m', 'upow_amd.node',
                          '--cluster', '--host', '127.0.0.1', '--port', str(port), '--log-level', 'warning'],
                         env=env, cwd=ROOT, stdout=log, stderr=subprocess.STDOUT, start_new_session=True)
    url = f'http://127.0.0.1:{port}'
    try:
        for _ in range(900):
            try:
                if httpx.get(url + '/get_nodes', timeout=1).status_code == 200:
                    break
            except Exception:
                time.sleep(0.2)
        else:
            raise AssertionError(open(tmp_path / 'cluster.log').read()[-3000:])
        info = httpx.get(url + '/cluster_info', timeout=60).json()['result']
        assert info['world'] == 4
        pushed, lat, lock = [], [], threading.Lock()

        def pusher():
            c = httpx.Client(timeout=60)
            for tx in txs:
                t0 = time.time()
                ok = c.post(url + '/push_tx', json={'tx_hex': tx.hex()}).json().get('ok')
                t1 = time.time()
                with lock:
                    lat.append((t0, t1, ok))
                    if ok:
                        pushed.append(tx.hex())
                time.sleep(max(0.0, 0.05 - (t1 - t0)))
        th = threading.Thread(target=pusher)
        th.start()
        windows = []
        ts = 1_700_000_000 + 60 * 60
        for b in range(4):
            time.sleep(0.35)
            with lock:
                batch = list(pushed)
                pushed.clear()
            w0 = time.time()
            res = _mine_via_api(url, address_of(KEY), ts + 60 * b, batch)
            windows.append((w0, time.time()))
            assert res == {'ok': True}, res
        th.join()
        assert all(ok for _, _, ok in lat), lat
        during = [t1 - t0 for t0, t1, _ in lat if any(w0 <= t0 <= w1 for w0, w1 in windows)]
        every = [t1 - t0 for t0, t1, _ in lat]
        report = {'world': 4, 'backend': 'gloo', 'pushes': len(lat), 'pushes_during_block_apply': len(during),
                  'push_p50_ms': round(1e3 * _pct(every, 0.5), 2), 'push_p99_ms': round(1e3 * _pct(every, 0.99), 2),
                  'push_during_apply_p99_ms': round(1e3 * _pct(during, 0.99), 2) if during else None,
                  'block_apply_ms': [round(1e3 * (w1 - w0), 1) for w0, w1 in windows]}
        (tmp_path / 'cluster_soak.json').write_text(json.dumps(report))
        print('cluster soak', json.dumps(report))
        info = httpx.get(url + '/cluster_info', timeout=60).json()['result']
        reps = info['replicas']
        assert len(reps) == 4 and len({(r['height'], r['utxo_hash']) for r in reps}) == 1, reps
        assert report['push_p99_ms'] < 3000
    finally:
        try:
            os.killpg(p.pid, signal.SIGTERM)
            p.wait(30)
        except Exception:
            os.killpg(p.pid, signal.SIGKILL)
        log.close()
