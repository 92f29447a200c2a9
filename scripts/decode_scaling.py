"""Block decode (csrc/txcodec.cpp decode_block_txs) against the host-pool thread count.

One 8,300-tx distinct-key block (bench_verify's builder), decoded 15 times per thread count; prints the best
and median wall time per count and the native split (decode_one pass vs column fill) of the last call.
Runs on the CPU only."""
import json
import os
import random
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from upow_amd.bench_verify import batch_keys, signed_spend_txs
    from upow_amd.ops.native import lib
    rng = random.Random(1)
    n = 8300
    keys, _, a33 = batch_keys(n, rng)
    _, _, r33 = batch_keys(n, rng)
    spends = [((rng.randbytes(32).hex(), 0), (rng.randbytes(32).hex(), 1)) for _ in range(n)]
    txs = signed_spend_txs(spends, keys, a33, r33)
    L = lib()
    if '--tuned' in sys.argv:  # the node's allocator settings (utils/cpus.py tune_malloc)
        from upow_amd.utils.cpus import tune_malloc
        tune_malloc()
    out = {'txs': n, 'cpus': os.cpu_count(), 'affinity': len(os.sched_getaffinity(0)), 'tuned': '--tuned' in sys.argv}
    for th in (1, 2, 4, 8, 12, 16):
        ts = []
        for _ in range(15):
            t = time.perf_counter()
            d = L.decode_block_txs(txs, th)
            d['merkle_job'].result()
            ts.append(time.perf_counter() - t)
        out[f't{th}_best_ms'] = round(min(ts) * 1e3, 3)
        out[f't{th}_median_ms'] = round(statistics.median(ts) * 1e3, 3)
        print(json.dumps(out), flush=True)
    ts, tm = [], []
    for _ in range(15):  # 16 threads, the decode call alone (the merkle root is awaited outside the window)
        t = time.perf_counter()
        d = L.decode_block_txs(txs, 16)
        t1 = time.perf_counter()
        d['merkle_job'].result()
        ts.append(t1 - t)
        tm.append(time.perf_counter() - t1)
    out['t16_decode_only_median_ms'] = round(statistics.median(ts) * 1e3, 3)
    out['t16_merkle_wait_median_ms'] = round(statistics.median(tm) * 1e3, 3)
    print(json.dumps(out), flush=True)
    # the native split of a 16-thread call (decode_one pass / column fill / hex list), printed by txcodec
    os.environ['UPOW_TXCODEC_PROFILE'] = '1'
    for _ in range(3):
        L.decode_block_txs(txs, 16)['merkle_job'].result()
    sys.stderr.flush()


if __name__ == '__main__':
    main()
