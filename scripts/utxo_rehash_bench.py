"""Time of one rebuild of the HBM UTXO table (csrc/utxo_table.hip): on the device (``utxo_rehash``, the
backend's path since round 6) against the dump to the host and re-insert it replaced, at 1 M / 5 M live
outpoints with payloads. One JSON line.

    python scripts/utxo_rehash_bench.py [millions=1,5]
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from upow_amd.ops.native import lib, require_gpu
    require_gpu()
    L = lib()
    sizes = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else '1,5').split(',')]
    rng = np.random.default_rng(7)
    out = {}
    for m in sizes:
        n = m * 1_000_000
        log2 = int(np.ceil(np.log2(3 * n)))
        recs = np.zeros((n, 40), np.uint8)
        recs[:, :32] = rng.integers(0, 256, (n, 32), dtype=np.uint8)
        recs[:, 32] = rng.integers(0, 4, n, dtype=np.uint8)
        pay = np.zeros((n, 80), np.uint8)
        pay[:, 8] = 33
        pay[:, 16:49] = rng.integers(0, 256, (n, 33), dtype=np.uint8)
        h = L.utxo_create(log2)
        assert L.utxo_insert(h, recs, pay) == (0, 0)
        t0 = time.perf_counter()
        moved, failed = L.utxo_rehash(h, log2)
        t_dev = time.perf_counter() - t0
        assert (moved, failed) == (n, 0), (moved, failed)
        t0 = time.perf_counter()
        raw, p = L.utxo_dump_payload(h)
        h2 = L.utxo_create(log2)
        assert L.utxo_insert(h2, np.frombuffer(raw, np.uint8).reshape(-1, 40), p) == (0, 0)
        t_host = time.perf_counter() - t0
        L.utxo_destroy(h)
        L.utxo_destroy(h2)
        out[f'{m}M'] = {'capacity': 1 << log2, 'device_rehash_ms': round(t_dev * 1e3, 2),
                        'dump_reinsert_ms': round(t_host * 1e3, 2)}
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
