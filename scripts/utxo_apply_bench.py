"""Block-path UTXO index update on the GPU: per 2 MB-block-shaped apply (16,600 created outputs with
payloads + 200 coinbase-like outputs in, 16,600 spent out), the host time of UtxoIndex.apply_block in async
mode (one pinned copy, one H2D, insert + erase queued, no wait) and in synchronous mode (insert, insert,
erase calls, each waiting), and the lookup that follows each apply. Prints one JSON line."""
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402


def main():
    from upow_amd.ledger import utxo as U
    rng = random.Random(5)
    n_out, n_cb, blocks = 16600, 200, 40

    def recs(n, seed):
        r = random.Random(seed)
        return U.pack_records([(r.randbytes(32).hex(), r.randrange(2)) for _ in range(n)], 0)

    def pay(n):
        return U.make_payload([rng.randrange(1, 1 << 40) for _ in range(n)], [bytes([42]) + rng.randbytes(32)] * n)
    pays = pay(n_out)
    out = {}
    for mode in ('async', 'sync', 'async', 'sync'):
        U.ASYNC_APPLY = mode == 'async'
        idx = U.UtxoIndex(backend='gpu')
        live = recs(n_out, 1)
        idx.apply_block([(live, pays)], np.zeros((0, 40), np.uint8))
        t_apply, t_look = [], []
        for b in range(blocks):
            new, cb = recs(n_out, 100 + b), recs(n_cb, 10000 + b)
            t0 = time.perf_counter()
            idx.apply_block([(new, pays), (cb, pays[:n_cb])], live)
            t1 = time.perf_counter()
            idx.lookup_records(new[:8300])  # the next block's input lookup, queued behind the apply
            t2 = time.perf_counter()
            live = new
            if b >= 5:
                t_apply.append(t1 - t0)
                t_look.append(t2 - t1)
        assert len(idx) == n_out + n_cb * blocks, len(idx)
        key = mode if mode not in out else mode + '_2'
        out[key] = {'apply_ms': round(1e3 * float(np.median(t_apply)), 3),
                    'next_lookup_ms': round(1e3 * float(np.median(t_look)), 3)}
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
