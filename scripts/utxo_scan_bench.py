"""K14 utxo_address_scan throughput on one MI355X: fill the HBM UTXO table to ~45 % load with random
outpoints owned by 1 000 addresses, then time address queries (one full-table scan each).

The figure of merit is slots/s. ``logical_key_GB_per_s`` = capacity x 48 B key slots per scan time: the
bytes a scan is DEFINED over, not the bytes it moves — the kernel reads only each slot's meta words (the
80 B payload line only for live slots whose tag matches), so the HBM traffic is lower; take that from
rocprofv3 ``--pmc FETCH_SIZE`` on this script, not from this figure."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from upow_amd.ledger.utxo import PAYLOAD_DTYPE, STAKE_ANY, UtxoIndex  # noqa: E402


def main(n=int(os.environ.get('N', 7_500_000)), queries=50):
    rng = np.random.default_rng(1)
    idx = UtxoIndex(backend='gpu')
    owners = np.zeros((1000, 64), np.uint8)
    owners[:, 0] = 42
    owners[:, 1:33] = rng.integers(0, 256, (1000, 32), dtype=np.uint8)
    done = 0
    while done < n:
        m = min(1_000_000, n - done)
        recs = np.zeros((m, 40), np.uint8)
        recs[:, :32] = rng.integers(0, 256, (m, 32), dtype=np.uint8)
        pay = np.zeros(m, PAYLOAD_DTYPE)
        pay['amount'] = rng.integers(1, 1 << 40, m)
        pay['len'] = 33
        pay['addr'] = owners[rng.integers(0, 1000, m)]
        idx.insert_records(recs, pay)
        done += m
    L, h = idx.be.L, idx.be.h
    cap = L.utxo_capacity(h)
    L.utxo_address_scan(h, bytes(owners[0, :33]), 1, STAKE_ANY)  # warm
    t = time.perf_counter()
    hits = 0
    for q in range(queries):
        raw, _, _ = L.utxo_address_scan(h, bytes(owners[q % 1000, :33]), 1, STAKE_ANY)
        hits += len(raw) // 40
    dt = (time.perf_counter() - t) / queries
    print(json.dumps({'live': len(idx), 'capacity': cap, 'ms_per_query': round(dt * 1e3, 3),
                      'slots_per_s': round(cap / dt / 1e9, 2), 'unit': 'G slots/s',
                      'logical_key_GB_per_s': round(cap * 48 / dt / 1e9, 1), 'avg_hits': hits / queries}))


if __name__ == '__main__':
    main()
