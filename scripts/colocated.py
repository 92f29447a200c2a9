"""Full node + miner sharing one MI355X (BASELINE config 5): block-apply GPU stages and hashrate, each
alone and side by side.

    python scripts/colocated.py [--blocks 8] [--dispatch-log2 24] [--prio high|normal] [--out FILE]

1. miner alone: a subprocess sweeps nonces in 2^30-nonce steps for a few seconds (hashrate alone);
2. node alone: the verify bench (native push_block path, file ledger) — per-stage times;
3. side by side: the miner subprocess runs while the verify bench applies its blocks; the miner's
   hashrate is taken over the verify bench's timed window only.
The miner uses the low-priority stream and UPOW_POW_DISPATCH_LOG2-sized dispatches; the node uses the
high-priority node stream (UPOW_NODE_STREAM_PRIORITY=normal for the A/B). Prints one JSON line."""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

MINER = r'''
import json, sys, time
sys.path.insert(0, sys.argv[1])
from upow_amd.ops.native import lib
lib()
from upow_amd.models.block import PowTarget, header_prefix
from upow_amd.ops.pow import PowJob, search
prev = '11' * 32
job = PowJob.create(header_prefix(prev, 'DgQKikeDqS2Fzue23KuA36L4eJSFh649zA9jJ6zwbzUMp', '22' * 32, 1790000000, '6.3'),
                    PowTarget.from_difficulty(prev, '6.3'))
step = 1 << 30
t_end = time.time() + float(sys.argv[2])
pos = 0
print(json.dumps({'t': time.time(), 'n': 0}), flush=True)
while time.time() < t_end:
    search(job, pos % (1 << 32), step, device='gpu')
    pos += step
    print(json.dumps({'t': time.time(), 'n': step}), flush=True)
'''


def miner(seconds: float, env):
    return subprocess.Popen([sys.executable, '-c', MINER, ROOT, str(seconds)], stdout=subprocess.PIPE, text=True,
                            env=env)


def rate(lines, t0=None, t1=None):
    """MH/s from the miner's step log, over [t0, t1] when given (steps wholly inside the window)."""
    recs = [json.loads(x) for x in lines if x.strip()]
    prev, total, span0, span1 = None, 0, None, None
    for r in recs:
        if prev is not None and (t0 is None or (prev >= t0 and r['t'] <= t1)):
            total += r['n']
            span0 = prev if span0 is None else span0
            span1 = r['t']
        prev = r['t']
    return total / (span1 - span0) / 1e6 if total else None


def verify(blocks: int):
    from upow_amd.bench_verify import run_verify_bench
    from upow_amd.parallel.dist import init_from_env
    ctx = init_from_env()
    tmp = tempfile.mkdtemp(prefix='coloc_')
    a = argparse.Namespace(steps=blocks, warmup=2, txs=8300, ledger=tmp, object_path=False, from_mempool=False)
    return run_verify_bench(a, ctx)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--blocks', type=int, default=8)
    ap.add_argument('--dispatch-log2', type=int, default=24)
    ap.add_argument('--prio', choices=['high', 'normal'], default='high')
    ap.add_argument('--out', default=None)
    a = ap.parse_args()
    os.environ['UPOW_POW_DISPATCH_LOG2'] = str(a.dispatch_log2)
    os.environ['UPOW_NODE_STREAM_PRIORITY'] = a.prio
    env = dict(os.environ)
    from upow_amd.ops.native import lib
    lib()
    # 1. miner alone
    p = miner(6.0, env)
    alone_lines = p.communicate()[0].splitlines()
    mhs_alone = rate(alone_lines[2:])  # skip the first (warm-up) step
    # 2. node alone
    v_alone = verify(a.blocks)
    # 3. side by side: the miner outlives the verify run
    p = miner(240.0, env)
    first = p.stdout.readline()
    p.stdout.readline()  # one full step done: the miner is warm
    v_co = verify(a.blocks)
    p.terminate()
    rest = p.communicate()[0].splitlines()
    t0, t1 = v_co['window_unix']
    mhs_co = rate([first] + rest, t0, t1)
    stages = ('utxo_s', 'decompress_s', 'ecdsa_s', 'block_s')

    def st(v):
        return {k: v['stage_ms_avg'].get(k) for k in stages}
    gpu_alone = sum(v_alone['stage_ms_avg'][k] for k in stages[:3])
    gpu_co = sum(v_co['stage_ms_avg'][k] for k in stages[:3])
    out = {'dispatch_log2': a.dispatch_log2, 'node_stream_priority': a.prio, 'blocks': a.blocks,
           'miner_mhs_alone': round(mhs_alone, 1), 'miner_mhs_colocated': round(mhs_co, 1) if mhs_co else None,
           'miner_kept': round(mhs_co / mhs_alone, 4) if mhs_co else None,
           'node_alone_ms': st(v_alone), 'node_colocated_ms': st(v_co),
           'gpu_stages_ms_alone': round(gpu_alone, 2), 'gpu_stages_ms_colocated': round(gpu_co, 2),
           'gpu_stage_slowdown': round(gpu_co / gpu_alone, 3),
           'verify_tx_per_s_alone': v_alone['value'], 'verify_tx_per_s_colocated': v_co['value']}
    line = json.dumps(out)
    print(line, flush=True)
    if a.out:
        with open(a.out, 'w') as f:
            f.write(line + '\n')


if __name__ == '__main__':
    main()
