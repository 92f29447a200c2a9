"""Steady-state node + miner soak on one MI355X (BASELINE.json config 5, scaled to one GPU):
a full node (REST, GPU UTXO set, native block path), the GPU miner CLI pointed at it, and a
synthetic wallet pushing ~40 tx/s through /push_tx.

    python scripts/node_soak.py [--rate 40] [--seconds 120] [--difficulty 9.5] [--out FILE] [--cluster N]

``--cluster N`` runs BASELINE config 5 as written: the multi-GPU node (``torchrun --nproc-per-node N -m
upow_amd.node --cluster``: rank 0 serves, ranks 1..N-1 are replicas) and the data-parallel miner
(``torchrun --nproc-per-node N -m upow_amd.miner``) co-located on the same N GPUs, both started as child
processes of this script before it touches a GPU. N = 1 forces the single-rank RCCL path (UPOW_FORCE_DIST).
The report adds per-rank MH/s and the replica agreement (``/cluster_info?deep=true``: height, tip, K12 UTXO
hash and SQL UTXO hash of every replica).

Prints one JSON line: confirmed tx/s, inclusion latency (push -> block) percentiles, block interval,
node-side block apply latency (from /metrics) and the miner's reported hashrate. Data: synthetic
(random keys; the miner's own coinbases are fanned out into ~5,000 spendable outputs first).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import random
import re
import socket
import subprocess
import sys
import tempfile
import threading
import time
from decimal import Decimal

import httpx

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


_PUSHER = r'''
import sys, threading, time, httpx
url, src, t0, rate, seconds, threads = sys.argv[1], sys.argv[2], float(sys.argv[3]), float(sys.argv[4]), float(sys.argv[5]), int(sys.argv[6])
jobs = [ln.split() for ln in open(src) if ln.strip()]
res, lock = [], threading.Lock()
def run(tid):
    c = httpx.Client(timeout=30)
    for j in range(tid, len(jobs), threads):
        k, hx = int(jobs[j][0]), jobs[j][1]
        target = t0 + k / rate
        delay = target - time.time()  # one clock read: the check and the sleep must agree
        if delay > 0:
            time.sleep(delay)
        if time.time() - t0 > seconds + 5:
            break
        ts = time.time()
        try:
            ok = c.post(url + '/push_tx', json={'tx_hex': hx}).json().get('ok')
        except Exception:
            ok = False
        with lock:
            res.append((k, time.time(), 1 if ok else 0, ts))
ts = [threading.Thread(target=run, args=(t,)) for t in range(threads)]
[t.start() for t in ts]
[t.join() for t in ts]
with open(src + '.out', 'w') as f:
    f.write(''.join(f'{k} {tp} {ok} {ts}\n' for k, tp, ok, ts in res))
'''


def _jsonl(path: str):
    """The records of a JSON-lines trace file; a line cut short (the node was stopped mid-write) is skipped."""
    with open(path) as f:
        for ln in f:
            try:
                yield json.loads(ln)
            except ValueError:
                continue


def _cpu_stat() -> dict:
    """The cgroup's CPU accounting (cgroup v2 cpu.stat): usage and CFS bandwidth throttling. A GPU box
    runs the job under a CPU quota far below its core count; a throttled period freezes every thread of the
    node (the HTTP loop included) until the next period, which reads as a loop stall of up to ~100 ms."""
    try:
        with open('/sys/fs/cgroup/cpu.stat') as f:
            return {k: int(v) for k, v in (ln.split() for ln in f if ln.strip())}
    except (OSError, ValueError):
        return {}


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--rate', type=float, default=40.0)
    ap.add_argument('--seconds', type=float, default=120.0)
    ap.add_argument('--difficulty', default='9.5')
    ap.add_argument('--out', default=None)
    ap.add_argument('--fanout1', type=int, default=25, help='coinbase -> N outputs')
    ap.add_argument('--fanout2', type=int, default=200, help='each of those -> M outputs (pool = N*M UTXOs)')
    ap.add_argument('--threads', type=int, default=1, help='concurrent /push_tx clients (per process)')
    ap.add_argument('--procs', type=int, default=1, help='client processes pushing txs')
    ap.add_argument('--cluster', type=int, default=0,
                    help='N > 0: multi-GPU node + DP miner on N GPUs under torchrun (N = 1: forced single-rank RCCL)')
    ap.add_argument('--client-cpus', default=None,
                    help="CPU list for the miner and the pushing clients (e.g. '16-47'), away from the node's")
    a = ap.parse_args()
    client_pin = None
    if a.client_cpus:
        from upow_amd.node.__main__ import parse_cpus
        cpus = set(parse_cpus(a.client_cpus)) & os.sched_getaffinity(0)
        client_pin = (lambda: os.sched_setaffinity(0, cpus)) if cpus else None

    from upow_amd.models.transaction import Transaction, TransactionInput, TransactionOutput
    from upow_amd.ops import p256 as op
    from upow_amd.ops.native import lib
    from upow_amd.utils.codec import point_to_string
    lib()
    rng = random.Random(7)
    key = rng.randrange(1, op.oracle.N)
    pub = op.public_key(key)
    addr = point_to_string(pub)
    sinks = [point_to_string(op.public_key(rng.randrange(1, op.oracle.N))) for _ in range(64)]

    data = tempfile.mkdtemp(prefix='soak')  # ledger files stay out of gpurun_out/ (size cap on the copy back)
    port = _port()
    url = f'http://127.0.0.1:{port}'
    trace = os.path.join(data, 'blocks.jsonl')  # per-block apply windows (UPOW_TRACE_FILE)
    env = dict(os.environ, UPOW_DATA_DIR=data, UPOW_CORE_URL='', UPOW_START_DIFFICULTY=a.difficulty,
               UPOW_RATE_LIMIT='0', PYTHONPATH=ROOT, UPOW_LOG_LEVEL='WARNING', UPOW_SNAPSHOT='0',
               UPOW_TRACE_FILE=trace)
    if os.environ.get('UPOW_SOAK_PROFILE') == '1':
        env['UPOW_PROFILE_OUT'] = os.path.join(data, 'node.prof')
    launch = []  # torchrun prefix of the node and the miner in --cluster mode
    if a.cluster:
        if a.cluster == 1:
            env['UPOW_FORCE_DIST'] = '1'
        launch = lambda: [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',  # noqa: E731
                          f'--nproc-per-node={a.cluster}', '--master-addr', '127.0.0.1', '--master-port', str(_port())]
    node_cmd = ([*launch(), '-m', 'upow_amd.node', '--cluster'] if a.cluster else [sys.executable, '-m', 'upow_amd.node'])
    node = subprocess.Popen([*node_cmd, '--host', '127.0.0.1', '--port', str(port), '--log-level', 'warning'],
                            env=env, cwd=ROOT, stdout=open(os.path.join(data, 'node.log'), 'w'), stderr=subprocess.STDOUT)
    client = httpx.Client(timeout=30)
    for _ in range(600):
        try:
            if client.get(url + '/get_nodes').status_code == 200:
                break
        except Exception:
            time.sleep(0.2)
    # an observer outside the node (csrc/stall_probe.cpp, sampling /proc/<node>/task every 2 ms): what each
    # node thread was doing in the kernel during a loop stall, even one that freezes the whole node process
    ext_probe = None
    node_pid = node.pid
    if a.cluster:  # the serving rank is a torchrun child: its loop thread id (= its pid) is in <trace>.threads
        node_pid = None
        for _ in range(100):
            try:
                with open(trace + '.threads') as tf:
                    node_pid = int(json.load(tf)['_loop'])
                break
            except (OSError, ValueError, KeyError):
                time.sleep(0.1)
    if node_pid is not None:
        try:
            from upow_amd.ops.native import lib as _lib
            ext_probe = _lib().StallProbe(trace + '.ext', None, node_pid, 10.0, 2000, node_pid)
        except (ImportError, AttributeError, RuntimeError) as e:
            print(f'external stall probe unavailable: {e}', flush=True)
    miner_log = open(os.path.join(data, 'miner.log'), 'w')
    from upow_amd.ops.native import gpu_available
    chunk = [] if gpu_available() else ['--chunk', '65536', '--device', 'cpu']
    miner_cmd = [*launch(), '-m', 'upow_amd.miner'] if a.cluster else [sys.executable, '-m', 'upow_amd.miner']
    miner = subprocess.Popen([*miner_cmd, addr, '1', url + '/', '--refresh', '10', *chunk],
                             preexec_fn=client_pin,
                             env=env, cwd=ROOT, stdout=miner_log, stderr=subprocess.STDOUT)
    t_start = time.time()
    phase = ['setup']

    def heartbeat():  # progress on stdout: a quiet minute-long setup must not look like a hang
        while node.poll() is None:
            time.sleep(15)
            print(f'[soak] {time.time() - t_start:.0f}s phase={phase[0]}', flush=True)
    threading.Thread(target=heartbeat, daemon=True).start()

    def height():
        return client.get(url + '/get_mining_info').json()['result']['last_block'].get('id', 0)

    def wait_height(h, limit=600):
        t = time.time()
        while height() < h:
            if time.time() - t > limit:
                raise RuntimeError(f'no block {h} within {limit} s')
            time.sleep(0.25)

    def spendable():
        r = client.get(url + '/get_address_info', params={'address': addr}).json()['result']
        return [(o['tx_hash'], o['index'], Decimal(str(o['amount']))) for o in r['spendable_outputs']]

    def push(tx):
        r = client.post(url + '/push_tx', json={'tx_hex': tx.hex()}).json()
        if not r.get('ok'):
            raise RuntimeError(f'push_tx rejected: {r}')

    def make_tx(h, i, amount, outs):
        inp = TransactionInput(h, i, amount=amount, public_key=pub)
        tx = Transaction([inp], [TransactionOutput(x, v) for x, v in outs])
        return tx.sign([key])

    # ---- fund: coinbase -> fanout1 outputs -> fanout1 x fanout2 outputs (the spendable pool)
    wait_height(2)
    cb = spendable()[0]
    v1 = (cb[2] / a.fanout1 - Decimal('0.0001')).quantize(Decimal('0.00000001'))
    push(make_tx(cb[0], cb[1], cb[2], [(addr, v1)] * a.fanout1))
    h0 = height()
    wait_height(h0 + 2)
    lvl1 = [u for u in spendable() if u[2] == v1]
    v2 = (v1 / a.fanout2 - Decimal('0.00000100')).quantize(Decimal('0.00000001'))
    for u in lvl1:
        push(make_tx(u[0], u[1], u[2], [(addr, v2)] * a.fanout2))
    h1 = height()
    wait_height(h1 + 2)
    pool = [u for u in spendable() if u[2] == v2]
    setup_s = time.time() - t_start

    # ---- steady state: one 1-in/1-out tx per pool UTXO at the target rate
    pushed = {}
    included = {}
    blocks = []
    stop = threading.Event()
    h_start = height()

    def watcher():
        c = httpx.Client(timeout=30)
        seen = h_start
        while not stop.is_set():
            # probe the next height with /get_block (an indexed lookup), not /get_mining_info: the
            # monitor must not load the node with a mempool-wide template build five times a second
            try:
                r = c.get(url + '/get_block', params={'block': seen + 1}).json()
            except Exception:
                time.sleep(0.2)
                continue
            if not r.get('ok'):
                time.sleep(0.2)
                continue
            seen += 1
            b = r['result']
            now = time.time()
            blocks.append((seen, now, len(b['transactions'])))
            for t in b['transactions']:
                th = hashlib.sha256(bytes.fromhex(t)).hexdigest()
                if th not in included:
                    included[th] = now  # every block tx; matched against the pushed set at the end

    w = threading.Thread(target=watcher, daemon=True)
    w.start()
    # pre-sign the whole pool (not part of the node's load)
    fee = min(Decimal('0.00001'), v2 / 2)
    signed = [make_tx(h, i, amount, [(sinks[k % len(sinks)], amount - fee)])
              for k, (h, i, amount) in enumerate(pool[:int(a.rate * a.seconds) + 1])]
    t0 = time.time()
    cpu0 = _cpu_stat()
    phase[0] = 'push'
    errors = [0]
    lock = threading.Lock()
    req = []  # (request start, request end) of every /push_tx

    def pusher(tid):
        c = httpx.Client(timeout=30)
        for k in range(tid, len(signed), a.threads):
            target = t0 + k / a.rate
            if time.time() < target:
                time.sleep(target - time.time())
            if time.time() - t0 > a.seconds + 5:
                break
            tx = signed[k]
            ts = time.time()
            try:
                r = c.post(url + '/push_tx', json={'tx_hex': tx.hex()}).json()
                with lock:
                    req.append((ts, time.time()))
                if not r.get('ok'):
                    raise RuntimeError(r)
                with lock:
                    pushed[tx.hash()] = time.time()
            except Exception:
                with lock:
                    errors[0] += 1

    if a.procs <= 1:
        ps = [threading.Thread(target=pusher, args=(t,), daemon=True) for t in range(a.threads)]
        for t in ps:
            t.start()
        for t in ps:
            t.join()
    else:
        # several client processes (one Python client tops out near ~600 req/s on the GIL): each
        # gets every procs-th tx, pushes it at its share of the schedule with its own threads and
        # reports (tx hash, push time, ok) lines back through a file
        hexes = [t.hex() for t in signed]
        hashes = [t.hash() for t in signed]
        kids = []
        for pidx in range(a.procs):
            src = os.path.join(data, f'push_{pidx}.txt')
            with open(src, 'w') as f:
                f.write('\n'.join(f'{k} {hexes[k]}' for k in range(pidx, len(hexes), a.procs)))
            kids.append((subprocess.Popen([sys.executable, '-c', _PUSHER, url, src, str(t0), str(a.rate),
                                           str(a.seconds), str(a.threads)], env=env, cwd=ROOT,
                                          preexec_fn=client_pin), src + '.out'))
        for proc, out in kids:
            proc.wait()
            for ln in open(out):
                k, tp, ok, ts = ln.split()
                req.append((float(ts), float(tp)))
                if ok == '1':
                    pushed[hashes[int(k)]] = float(tp)
                else:
                    errors[0] += 1
    n = len(pushed) + errors[0]
    t_push_end = time.time()
    if ext_probe is not None:
        ext_probe.stop()
    cpu1 = _cpu_stat()
    phase[0] = 'drain'
    # drain: wait until everything pushed is in a block (or 4 block intervals)
    deadline = time.time() + 120
    while sum(h in included for h in list(pushed)) < len(pushed) and time.time() < deadline:
        time.sleep(0.5)
    stop.set()
    w.join(5)
    metrics = client.get(url + '/metrics').text
    replicas = None
    if a.cluster:
        ci = client.get(url + '/cluster_info', params={'deep': 'true'}, timeout=120).json()['result']
        reps = ci['replicas']
        replicas = {'world': ci['world'], 'backend': ci['backend'], 'last_resync': ci.get('last_resync'),
                    'op_stream': ci.get('op_stream'),
                    'agree': len({(r['height'], r['tip_hash'], r['utxo_hash'], r.get('sql_utxo_hash')) for r in reps}) == 1,
                    'replicas': reps}
    miner.terminate()
    node.terminate()
    for p in (miner, node):
        try:
            p.wait(20)
        except subprocess.TimeoutExpired:
            p.kill()
    miner_log.close()
    prof = os.path.join(data, 'node.prof')
    if a.out and os.path.exists(prof):  # UPOW_SOAK_PROFILE=1: the event-loop thread's cProfile, top entries
        import io
        import pstats
        buf = io.StringIO()
        st = pstats.Stats(prof, stream=buf)
        st.sort_stats('tottime').print_stats(45)
        st.sort_stats('cumulative').print_stats(45)
        with open(os.path.splitext(a.out)[0] + '_loop_profile.txt', 'w') as f:
            f.write(buf.getvalue())
    included = {h: included[h] for h in pushed if h in included}
    lat = sorted(included[h] - pushed[h] for h in included)
    # the slowest 1 %: when they were pushed and when their block was seen (seconds from the push start),
    # and the heights that carried them -- a tail from one late block differs from txs a template skipped
    tail = sorted(included, key=lambda h: included[h] - pushed[h])[-max(1, len(included) // 100):] if included else []
    h_of = {}
    for ht, bt, _ in blocks:
        h_of.setdefault(round(bt, 3), ht)
    tail_info = {
        'n': len(tail),
        'pushed_s': [round(min(pushed[h] for h in tail) - t0, 2), round(max(pushed[h] for h in tail) - t0, 2)] if tail else None,
        'seen_s': [round(min(included[h] for h in tail) - t0, 2), round(max(included[h] for h in tail) - t0, 2)] if tail else None,
        'heights': sorted({h_of.get(round(included[h], 3)) for h in tail} - {None}),
        'block_seen_s': [[ht, round(bt - t0, 2), n] for ht, bt, n in blocks],
    }
    miner_text = open(os.path.join(data, 'miner.log')).read()
    rates = [float(x) for x in re.findall(r'([0-9.]+) MH/s \(', miner_text)]
    per_rank = [json.loads(x) for x in re.findall(r'per-rank MH/s: (\[[^\]]*\])', miner_text)]
    apply = {}
    for ln in metrics.splitlines():
        m = re.match(r'upow_block_apply_seconds_(sum|count)\{path="(\w+)"\} (\S+)', ln)
        if m:
            apply.setdefault(m.group(2), {})[m.group(1)] = float(m.group(3))
    steady_blocks = [b for b in blocks if b[1] <= t_push_end + 1]
    # /push_tx request latency, overall and for requests that overlapped a block application
    windows = []
    if os.path.exists(trace):
        for r in _jsonl(trace):
            if r.get('ok') and r.get('txs', 0) > 0:
                windows.append((r['t'] - r['ms'] / 1000.0, r['t']))
    windows.sort()

    def overlaps(a0, a1):
        return any(w0 < a1 and a0 < w1 for w0, w1 in windows)
    # where the HTTP loop stalled (node's UPOW_TRACE_FILE.lag) and what the block path spent its time on
    stalls = []
    if os.path.exists(trace + '.lag'):
        for r in _jsonl(trace + '.lag'):
            if t0 <= r['t'] <= t_push_end:
                stalls.append((r['t'] - r['ms'] / 1000.0, r['t'], r['ms']))
    in_blk = [s for s in stalls if overlaps(s[0], s[1])]
    stack_counts = {}
    other_counts = {}  # what the node's other Python threads were executing during loop stalls
    if os.path.exists(trace + '.stacks'):
        for r in _jsonl(trace + '.stacks'):
            if t0 <= r['t'] <= t_push_end:
                key = ' < '.join(reversed(r['stack'][-3:]))
                stack_counts[key] = stack_counts.get(key, 0) + 1
                for name, where in r.get('others', {}).items():
                    if any(w in where for w in ('wait', 'select', 'sleep', '_worker', 'get')):
                        continue  # parked threads
                    k2 = f'{name} @ {where}'
                    other_counts[k2] = other_counts.get(k2, 0) + 1
    # the native probe's samples (csrc/stall_probe.cpp: every thread's kernel state while the loop is late,
    # taken without the GIL): the loop thread's state / wait channel / syscall, and which threads ran (R)
    # or waited on the disk (D) meanwhile, by Python thread name where the node recorded one
    names = {}
    if os.path.exists(trace + '.threads'):
        with open(trace + '.threads') as tf:
            names = json.load(tf)
    loop_tid = str(names.get('_loop', ''))
    nat_loop, nat_busy, nat_n = {}, {}, 0
    if os.path.exists(trace + '.native'):
        for r in _jsonl(trace + '.native'):
            if not t0 <= r['t'] <= t_push_end:
                continue
            nat_n += 1
            for tid, comm, state, wchan, sc in r['threads']:
                if str(tid) == loop_tid:
                    k = f'{state} {wchan or "-"} sys={sc}'
                    nat_loop[k] = nat_loop.get(k, 0) + 1
                elif state in ('R', 'D'):
                    k = f'{names.get(str(tid), comm)} {state} {wchan or "-"} sys={sc}'
                    nat_busy[k] = nat_busy.get(k, 0) + 1
    ext_loop, ext_busy, ext_n = {}, {}, 0
    if os.path.exists(trace + '.ext'):
        for r in _jsonl(trace + '.ext'):
            if not any(s0 <= r['t'] <= s1 for s0, s1, _ in stalls if s1 - s0 > 0.02):
                continue  # only the samples inside a loop stall over 20 ms
            ext_n += 1
            for tid, comm, state, wchan, sc in r['threads']:
                if str(tid) == (loop_tid or str(node_pid)):
                    k = f'{state} {wchan or "-"} sys={sc}'
                    ext_loop[k] = ext_loop.get(k, 0) + 1
                elif state in ('R', 'D'):
                    k = f'{names.get(str(tid), comm)} {state} {wchan or "-"} sys={sc}'
                    ext_busy[k] = ext_busy.get(k, 0) + 1
    top_stacks = sorted(stack_counts.items(), key=lambda kv: -kv[1])[:12]
    top_others = sorted(other_counts.items(), key=lambda kv: -kv[1])[:12]
    gcs = []
    if os.path.exists(trace + '.gc'):
        for r in _jsonl(trace + '.gc'):
            if t0 <= r['t'] <= t_push_end:
                gcs.append(r)
    stages = {}
    if os.path.exists(trace):
        for r in _jsonl(trace):
            if r.get('ok') and r.get('txs', 0) > 0:
                for k, v in r.get('stages_ms', {}).items():
                    stages.setdefault(k, []).append(v)
    req_lat = sorted((b - a) * 1000 for a, b in req)
    req_lat_blk = sorted((b - a) * 1000 for a, b in req if overlaps(a, b))
    pq = lambda v, p: round(v[min(len(v) - 1, int(p * len(v)))], 2) if v else None
    intervals = [b2[1] - b1[1] for b1, b2 in zip(blocks, blocks[1:])]
    q = lambda p: round(lat[min(len(lat) - 1, int(p * len(lat)))], 2) if lat else None
    out = {
        'metric': 'node_soak_confirmed_tx_per_s', 'value': round(len(included) / max(1e-9, t_push_end - t0), 2),
        'unit': 'tx/s', 'target_rate': a.rate, 'pushed': len(pushed), 'push_errors': errors[0],
        'push_threads': a.threads, 'push_procs': a.procs, 'pool_utxos': len(pool),
        'confirmed': len(included), 'seconds': round(t_push_end - t0, 1),
        'inclusion_latency_s': {'p50': q(0.5), 'p90': q(0.9), 'p99': q(0.99), 'max': round(lat[-1], 2) if lat else None},
        'inclusion_tail_1pct': tail_info,
        'blocks': len(blocks), 'mean_block_interval_s': round(sum(intervals) / len(intervals), 2) if intervals else None,
        'txs_per_block_max': max((b[2] for b in blocks), default=0),
        'block_apply_ms_mean': {k: round(1000 * v['sum'] / v['count'], 2) for k, v in apply.items() if v.get('count')},
        'miner_mhs_median': sorted(rates)[len(rates) // 2] if rates else None,
        'push_tx_latency_ms': {'p50': pq(req_lat, 0.5), 'p99': pq(req_lat, 0.99), 'n': len(req_lat)},
        'push_tx_latency_during_block_apply_ms': {'p50': pq(req_lat_blk, 0.5), 'p99': pq(req_lat_blk, 0.99),
                                                  'n': len(req_lat_blk)},
        'block_apply_windows': len(windows),
        'block_apply_ms_max': round(max((w1 - w0) * 1000 for w0, w1 in windows), 1) if windows else None,
        'loop_stalls_over_2ms': {'n': len(stalls), 'total_ms': round(sum(s[2] for s in stalls), 1),
                                 'max_ms': round(max((s[2] for s in stalls), default=0), 1),
                                 'n_during_block_apply': len(in_blk),
                                 'total_ms_during_block_apply': round(sum(s[2] for s in in_blk), 1)},
        'loop_stall_samples_2ms': dict(top_stacks),
        'loop_stall_other_threads': dict(top_others),
        'loop_stall_native': {'samples': nat_n,
                              'loop_thread': dict(sorted(nat_loop.items(), key=lambda kv: -kv[1])[:8]),
                              'running_or_disk': dict(sorted(nat_busy.items(), key=lambda kv: -kv[1])[:16])},
        'loop_stall_external': {'samples_in_stalls_over_20ms': ext_n,
                                'loop_thread': dict(sorted(ext_loop.items(), key=lambda kv: -kv[1])[:8]),
                                'running_or_disk': dict(sorted(ext_busy.items(), key=lambda kv: -kv[1])[:16])},
        'gc_over_2ms': {'n': len(gcs), 'total_ms': round(sum(g['ms'] for g in gcs), 1),
                        'max_ms': round(max((g['ms'] for g in gcs), default=0), 1),
                        'gen2': sum(1 for g in gcs if g.get('gen') == 2)},
        'block_stage_ms_mean': {k: round(sum(v) / len(v), 2) for k, v in sorted(stages.items())},
        # the whole job's cgroup over the push window (node, miner and the pushing clients share it)
        'cgroup_cpu': {'cpus_used_mean': round((cpu1.get('usage_usec', 0) - cpu0.get('usage_usec', 0)) / 1e6
                                               / max(1e-9, t_push_end - t0), 2),
                       'nr_periods': cpu1.get('nr_periods', 0) - cpu0.get('nr_periods', 0),
                       'nr_throttled': cpu1.get('nr_throttled', 0) - cpu0.get('nr_throttled', 0),
                       'throttled_ms': round((cpu1.get('throttled_usec', 0) - cpu0.get('throttled_usec', 0)) / 1e3, 1)}
        if cpu0 and cpu1 else None,
        'difficulty': a.difficulty, 'setup_s': round(setup_s, 1), 'data': 'synthetic keys, miner coinbases fanned out',
    }
    if a.cluster:
        out['cluster'] = {'gpus': a.cluster, 'node': 'torchrun -m upow_amd.node --cluster',
                          'miner': 'torchrun -m upow_amd.miner (nonce-space DP)',
                          'miner_per_rank_mhs_median': [sorted(col)[len(col) // 2] for col in zip(*per_rank)] if per_rank else None,
                          **(replicas or {})}
    line = json.dumps(out)
    print(line, flush=True)
    if a.out:
        with open(a.out, 'w') as f:
            f.write(line + '\n')


if __name__ == '__main__':
    main()
