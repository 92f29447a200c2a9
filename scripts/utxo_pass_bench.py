"""Host-side cost of one 2 MB block's UTXO pass (K7 lookup + K10 duplicates + K11 fees in one round trip,
csrc/utxo_table.hip utxo_block_inputs) on the HBM table, outside the ledger.

    python scripts/utxo_pass_bench.py [--inputs 16600] [--txs 8300] [--live 1000000] [--reps 300]

A table holding --live outpoints; each rep passes a block whose 16,600 inputs all hit, 2 inputs and 2
outputs per tx. Prints one JSON line with the median / p10 / p90 wall time of the call (ms). Load an A/B
build with UPOW_NATIVE_SO=path/to/_native.so.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--inputs', type=int, default=16600)
    ap.add_argument('--txs', type=int, default=8300)
    ap.add_argument('--live', type=int, default=1_000_000)
    ap.add_argument('--reps', type=int, default=300)
    a = ap.parse_args()
    from upow_amd.ops.native import lib, require_gpu
    L = lib()
    require_gpu()
    rng = np.random.default_rng(7)
    log2 = max(16, int(np.ceil(np.log2(a.live * 3))))
    h = L.utxo_create(log2)
    try:
        recs = np.zeros((a.live, 40), dtype=np.uint8)
        recs[:, :32] = rng.integers(0, 256, size=(a.live, 32), dtype=np.uint8)
        # index 0 and tag 0 (the bytes after the txid stay zero): random txids are distinct
        pay = rng.integers(0, 256, size=(a.live, 80), dtype=np.uint8)
        pay[:, 0:16] = 0  # UtxoPayload: u64 amount, u32 addr_len, u32 flags, 64 B address
        pay[:, 0] = 100
        pay[:, 8] = 45
        for s in range(0, a.live, 1 << 18):
            L.utxo_insert(h, np.ascontiguousarray(recs[s:s + (1 << 18)]), np.ascontiguousarray(pay[s:s + (1 << 18)]))
        per_tx = a.inputs // a.txs
        in_start = (np.arange(a.txs + 1, dtype=np.int32) * per_tx)
        out_start = (np.arange(a.txs + 1, dtype=np.int32) * 2)
        out_amount = np.ones(2 * a.txs, dtype=np.uint64)
        times = []
        for r in range(a.reps + 10):
            pick = rng.choice(a.live, size=a.txs * per_tx, replace=False)
            keys = np.ascontiguousarray(recs[pick])
            t0 = time.perf_counter()
            tags, p, dup, fee, miss, nd = L.utxo_block_inputs(h, keys, in_start, out_amount, out_start, 0)
            dt = time.perf_counter() - t0
            if r >= 10:
                times.append(dt * 1e3)
            if r == 0:
                assert int(np.count_nonzero(tags == 0)) == len(pick), 'every input must hit'
                assert nd == 0 and int(miss.sum()) == 0
        t = np.array(times)
        print(json.dumps({'inputs': int(a.txs * per_tx), 'txs': a.txs, 'live': a.live, 'reps': a.reps,
                          'ms_median': round(float(np.median(t)), 4), 'ms_p10': round(float(np.percentile(t, 10)), 4),
                          'ms_p90': round(float(np.percentile(t, 90)), 4),
                          'so': os.environ.get('UPOW_NATIVE_SO') or 'in-tree'}), flush=True)
    finally:
        L.utxo_destroy(h)


if __name__ == '__main__':
    main()
