"""Governance blocks vs plain blocks, interleaved in ONE process (A/B without box-to-box drift).

Two file ledgers are built with bench_verify's block builder: A holds plain 8,300-tx distinct-key blocks,
B the same blocks with 5 % governance txs (70 % delegate votes, 10 % validator votes, 20 % delegate
revokes on a seeded governance state; reference rules: transaction.py:240-479). The blocks are then
applied alternately A1 B1 A2 B2 ... through the native block path (``fastpath.create_block_from_hex``,
the push_block path), each timed to durability and with both ledgers' SQL writers drained before the next
block, so neither ledger's background work lands in the other's window. Separate runs of
``bench.py --mode verify`` vs ``--governance-txs 5%`` on the pool's boxes differ by ±15 % between runs
of the SAME config; interleaving cancels that.

    python scripts/gov_ab.py [--blocks 12] [--warmup 2] [--gov 0.05] [--out file.json]
"""
import argparse
import asyncio
import hashlib
import json
import os
import shutil
import statistics
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


async def main(args):
    from upow_amd import devnet
    from upow_amd.bench_verify import _setup
    from upow_amd.constants import START_DIFFICULTY
    from upow_amd.ledger import fastpath, manager, validate
    from upow_amd.ledger.database import Database
    from upow_amd.models.block import get_transactions_merkle_tree
    from upow_amd.ops.native import gpu_available
    device = 'gpu' if gpu_available() else 'cpu'
    backend = 'gpu' if device == 'gpu' else 'host'
    n_blocks = args.blocks + args.warmup
    root = tempfile.mkdtemp(prefix='gov_ab_', dir=os.environ.get('TMPDIR', '/tmp'))
    sides = {}
    try:
        for name, gov in (('plain', 0.0), ('gov', args.gov)):
            path = os.path.join(root, name)
            os.makedirs(path)
            db, addr, blocks, base_ts = await _setup(n_blocks, args.txs, 1234, backend, device,
                                                     ledger_path=os.path.join(path, 'ledger.sqlite3'),
                                                     gov_txs=gov, distinct_keys=True)
            db.flush()
            # the tx strings as a node holds them: parsed from one JSON body (/push_block, sync), i.e. allocated
            # together. The generator's strings are scattered over its setup heap, and that alone made the
            # native decode of the governance block ~10 % slower single-threaded (8 % of it gone after this
            # round trip, on one pinned CPU; docs/ROUND4.md section 8)
            blocks = [json.loads(json.dumps(b)) for b in blocks]
            last = await db.get_last_block()
            prev, headers = last['hash'], []
            for b, txs in enumerate(blocks):
                c = devnet.mine_header_raw(prev, addr, get_transactions_merkle_tree(txs), base_ts + 10 + b,
                                           START_DIFFICULTY, device=device)
                headers.append(c)
                prev = hashlib.sha256(bytes.fromhex(c)).hexdigest()
            sides[name] = {'db': db, 'blocks': blocks, 'headers': headers, 'ms': [], 'stages': []}
        for b in range(n_blocks):
            for name in ('plain', 'gov') if b % 2 == 0 else ('gov', 'plain'):
                s = sides[name]
                db = s['db']
                Database.instance = db
                manager.Manager.difficulty = None
                if db.gov is not None:
                    db.gov.lock.settle()
                t0 = time.perf_counter()
                ok = await fastpath.create_block_from_hex(s['headers'][b], s['blocks'][b])
                dt = time.perf_counter() - t0
                if not ok:
                    raise RuntimeError(f'{name} block {b} rejected')
                if fastpath.last_path != 'native':
                    raise RuntimeError(f'{name} block {b} left the native path')
                if b >= args.warmup:
                    s['ms'].append(dt * 1e3)
                    st = dict(validate.timings)
                    st.update(manager.last_block_timings)
                    st.update(fastpath.timings)
                    s['stages'].append(st)
                # the other ledger's turn starts with this one idle: SQL caught up, governance index applied
                db.flush()
                if db.gov is not None:
                    db.gov.lock.settle()
        out = {'metric': 'governance_block_time_ratio', 'blocks_per_side': args.blocks, 'txs_per_block': args.txs,
               'gov_share': args.gov, 'device': device, 'order': 'interleaved, alternating first side'}
        for name, s in sides.items():
            out[f'{name}_ms_median'] = round(statistics.median(s['ms']), 3)
            out[f'{name}_ms'] = [round(x, 3) for x in s['ms']]
            keys = sorted({k for st in s['stages'] for k, v in st.items() if isinstance(v, float)})
            out[f'{name}_stage_ms_median'] = {k: round(1e3 * statistics.median(st.get(k, 0.0) for st in s['stages']), 3)
                                              for k in keys}
        out['plain_over_gov_time'] = round(out['plain_ms_median'] / out['gov_ms_median'], 3)
        pairs = [p / g for p, g in zip(sides['plain']['ms'], sides['gov']['ms'])]
        out['pair_ratio_median'] = round(statistics.median(pairs), 3)
        line = json.dumps(out)
        print(line, flush=True)
        if args.out:
            with open(args.out, 'w') as f:
                f.write(line + '\n')
    finally:
        for s in sides.values():
            s['db'].close()
        shutil.rmtree(root, ignore_errors=True)


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('--blocks', type=int, default=12)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--txs', type=int, default=8300)
    ap.add_argument('--gov', type=float, default=0.05)
    ap.add_argument('--out', default=None)
    asyncio.run(main(ap.parse_args()))
