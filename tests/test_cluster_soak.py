"""Cluster node soak (parallel/cluster.py, 4 ranks over gloo): /push_tx keeps answering while blocks are
validated and applied on all replicas, and ``/cluster_info`` is polled every 50 ms throughout. Admissions
only queue their row for the next batched 'txs' op (no collective per tx, no hop through the ledger
thread); ``/cluster_info`` is a 'status' op issued by the ledger thread like every other collective, so it
can never interleave with a block's or a tx batch's collectives — and because it is an op in the stream,
every replica answers it at the same point: each poll must show all four replicas at one (height, tip,
UTXO hash). Reports push latency percentiles overall and during block application into
``cluster_soak.json`` under the test's tmp dir.

The pushed txs spend a funding fan-out confirmed in the prefilled chain: a fresh key pair per tx, signed in
bulk (bench_verify.signed_spend_txs). ``UPOW_SOAK_RATE`` sets the offered push rate (default 200 tx/s on
this 8-CPU container; scripts run it at 1,200 tx/s on a GPU box's CPU share)."""
import asyncio
import json
import multiprocessing
import os
import random
import signal
import subprocess
import sys
import threading
import time
from decimal import Decimal

import httpx
import pytest

from test_cluster import KEY, _mine_via_api
from test_multinode import ROOT, _port


def _pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))] if xs else None


def _pusher(url, txs, k, step, t_start, rate, q):
    """Open-loop client (own process): tx j is due at t_start + j / rate; reports (t0, t1, ok, j)."""
    c = httpx.Client(timeout=60)
    for j in range(k, len(txs), step):
        time.sleep(max(0.0, t_start + j / rate - time.time()))
        t0 = time.time()
        ok = bool(c.post(url + '/push_tx', json={'tx_hex': txs[j]}).json().get('ok'))
        q.put((t0, time.time(), ok, j))
    q.put(None)


def prefill_funded(path, blocks: int, n_txs: int, seed: int = 11):
    """``blocks`` genesis-address blocks, then one block of fan-out txs giving each of ``n_txs`` fresh keys
    two 0.02-coin outputs. Returns the signed 2-in/2-out txs that spend them (one per key)."""
    from upow_amd import devnet
    from upow_amd.bench_verify import batch_keys, signed_spend_txs
    from upow_amd.ledger import manager
    from upow_amd.ledger.database import Database
    from upow_amd.utils.codec import bytes_to_string
    from upow_amd.wallet.builders import address_of, create_transaction_to_send_multiple_wallet
    rng = random.Random(seed)
    keys, _, owner33 = batch_keys(n_txs, rng)
    _, _, recip33 = batch_keys(n_txs, rng)
    owners = [bytes_to_string(a) for a in owner33]

    async def go():
        db = await Database.create(path=str(path), utxo_backend='host')
        manager.Manager.difficulty = None
        for b in range(blocks):
            await devnet.mine_block(address_of(KEY), ts=1_700_000_000 + 60 * b, device='cpu')
        fan, outs = [], []  # outs[i] = (fan-out tx index, output index) of output i
        for k in range(0, 2 * n_txs, 254):
            dests = [owners[i // 2] for i in range(k, min(2 * n_txs, k + 254))]
            tx = await create_transaction_to_send_multiple_wallet(KEY, dests, [Decimal('0.02')] * len(dests))
            assert await db.add_pending_transaction(tx)  # keeps the builder's input selection disjoint
            fan.append(tx)
        await devnet.mine_block(address_of(KEY), fan, ts=1_700_000_000 + 60 * blocks, device='cpu')
        for t in fan:
            # the builder may add a change output at the end: the fan-out outputs come first, in order
            outs.extend((t.hash(), j) for j in range(len(t.outputs)) if t.outputs[j].address != address_of(KEY))
        db.close()
        return outs
    outs = asyncio.run(go())
    assert len(outs) == 2 * n_txs
    spends = [(outs[2 * j], outs[2 * j + 1]) for j in range(n_txs)]
    return signed_spend_txs(spends, keys, owner33, recip33, amount_out=(2_500_000, 1_490_000))


@pytest.mark.slow
def test_cluster_world4_push_soak_with_cluster_info_polling(tmp_path, monkeypatch):
    from upow_amd.ledger import manager
    from upow_amd.wallet.builders import address_of
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('1.0'))
    rate = float(os.environ.get('UPOW_SOAK_RATE', '200'))
    seconds = float(os.environ.get('UPOW_SOAK_SECONDS', '5'))
    n = int(rate * seconds)
    (tmp_path / 'n').mkdir()
    txs = prefill_funded(tmp_path / 'n' / 'ledger.sqlite3', 48, n)
    port, mport = _port(), _port()
    env = dict(os.environ, UPOW_DATA_DIR=str(tmp_path / 'n'), UPOW_CORE_URL='', UPOW_START_DIFFICULTY='1.0',
               UPOW_UTXO_BACKEND='host', UPOW_DISABLE_GPU='1', UPOW_RATE_LIMIT='0', PYTHONPATH=ROOT,
               UPOW_LOG_LEVEL='WARNING', OMP_NUM_THREADS='1', UPOW_CODEC_THREADS='1')
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
        assert info['world'] == 4 and info['last_resync']['blocks_sent'] == 49
        pushed, lat = [], []
        stop = threading.Event()
        polls, bad_polls = [], []

        def poller():  # /cluster_info every 50 ms while txs and blocks flow
            c = httpx.Client(timeout=60)
            while not stop.is_set():
                t0 = time.time()
                reps = c.get(url + '/cluster_info').json()['result']['replicas']
                polls.append(time.time() - t0)
                if len({(r['height'], r['tip_hash'], r['utxo_hash'], r['mempool']) for r in reps}) != 1:
                    bad_polls.append(reps)
                stop.wait(max(0.0, 0.05 - (time.time() - t0)))

        n_procs = max(4, min(12, int(rate // 100)))  # pushing clients in processes of their own: the test process's GIL (block mining, the
        t_start = time.time() + 1.0  # poller) must not add to the latency they measure
        ctx = multiprocessing.get_context('fork')
        q = ctx.Queue()
        procs = [ctx.Process(target=_pusher, args=(url, txs, k, n_procs, t_start, rate, q)) for k in range(n_procs)]
        for pr in procs:
            pr.start()
        th_poll = threading.Thread(target=poller)
        th_poll.start()
        windows = []
        ts = 1_700_000_000 + 60 * 60
        b = 0
        done = 0
        while done < n_procs or pushed:
            time.sleep(0.5)
            while not q.empty():
                item = q.get()
                if item is None:
                    done += 1
                    continue
                lat.append(item)
                if item[2]:
                    pushed.append(txs[item[3]])
            batch = list(pushed)
            pushed.clear()
            w0 = time.time()
            res = _mine_via_api(url, address_of(KEY), ts + 60 * b, batch)
            windows.append((w0, time.time(), len(batch)))
            assert res == {'ok': True}, res
            b += 1
        for pr in procs:
            pr.join(30)
        stop.set()
        th_poll.join()
        assert len(lat) == n and all(x[2] for x in lat), [x for x in lat if not x[2]][:5]
        during = [t1 - t0 for t0, t1, _, _ in lat if any(w0 <= t0 <= w1 for w0, w1, _ in windows)]
        every = [t1 - t0 for t0, t1, _, _ in lat]
        span = max(x[1] for x in lat) - min(x[0] for x in lat)
        report = {'world': 4, 'backend': 'gloo', 'offered_rate': rate, 'pushes': len(lat),
                  'achieved_rate': round(len(lat) / span, 1), 'pushes_during_block_apply': len(during),
                  'push_p50_ms': round(1e3 * _pct(every, 0.5), 2), 'push_p99_ms': round(1e3 * _pct(every, 0.99), 2),
                  'push_during_apply_p99_ms': round(1e3 * _pct(during, 0.99), 2) if during else None,
                  'blocks': [(round(1e3 * (w1 - w0), 1), k) for w0, w1, k in windows],
                  'cluster_info_polls': len(polls), 'cluster_info_p99_ms': round(1e3 * _pct(polls, 0.99), 2)}
        (tmp_path / 'cluster_soak.json').write_text(json.dumps(report))
        print('cluster soak', json.dumps(report))
        assert not bad_polls, json.dumps(bad_polls[:3])
        assert len(polls) >= 20
        reps = httpx.get(url + '/cluster_info', params={'deep': 'true'}, timeout=60).json()['result']['replicas']
        assert len({(r['height'], r['utxo_hash'], r['sql_utxo_hash'], r['mempool']) for r in reps}) == 1, reps
        assert reps[0]['mempool'] == 0 and reps[0]['height'] == 49 + b
        # the target is push p99 < 50 ms. The 8-CPU container runs four ranks, the pushers and this process; when
        # its CPU share collapses (shared host) the pushers cannot even offer the rate, and every latency then
        # includes their own scheduling delay: such a run is reported, and held to a 3x looser bound only
        starved = report['achieved_rate'] < 0.9 * rate
        if starved:
            print(f"cluster soak: host CPU-starved (achieved {report['achieved_rate']} of {rate} tx/s)")
        assert report['push_p99_ms'] < (150 if starved else 50), report
    finally:
        try:
            os.killpg(p.pid, signal.SIGTERM)
            p.wait(60)
        except Exception:
            os.killpg(p.pid, signal.SIGKILL)
        log.close()
