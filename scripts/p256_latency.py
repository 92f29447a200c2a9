"""Single-block (8,300 signatures) P-256 verify latency on the GPU for the kernel variants.

Wall time per launch (H2D of 1.3 MB records + kernel + D2H of the status bytes), median of 7; the
kernel-only time comes from a rocprofv3 --kernel-trace run of this script. Knobs read per call:
UPOW_P256_VARIANT (kernel variant), UPOW_P256_SPW (signatures per 64-lane wave). A config is
variant:spw[:n], n = signatures per launch (default all 8,300)."""
import hashlib
import json
import os
import random
import statistics
import sys
import time

sys.path.insert(0, '.')
from upow_amd.ops.native import lib  # noqa: E402
from upow_amd.ops import p256 as op  # noqa: E402

lib()
rng = random.Random(1)
keys = [rng.randrange(1, op.oracle.N) for _ in range(64)]
pubs = [op.public_key(k) for k in keys]
recs = []
for i in range(8300):
    msg = rng.randbytes(200)
    recs.append(op.record(pubs[i % 64], op.sign(msg, keys[i % 64]), hashlib.sha256(msg).digest()))
base = b''.join(recs)
configs = [c.split(':') for c in (','.join(sys.argv[1:]).split(',') if len(sys.argv) > 1 else ['1:64', '1:32', '1:16'])]
out = {}
rec_len = len(recs[0])
for cfg in configs:
    var, spw = cfg[:2]
    n = int(cfg[2]) if len(cfg) > 2 else len(recs)
    blk = base[:n * rec_len]
    os.environ['UPOW_P256_VARIANT'] = var
    os.environ['UPOW_P256_SPW'] = spw
    st = op.verify_records(blk, device='gpu')
    assert (st == 1).all(), (var, spw, st[:20])
    ts = []
    for _ in range(7):
        t = time.perf_counter()
        op.verify_records(blk, device='gpu')
        ts.append(time.perf_counter() - t)
    out[f'v{var}_spw{spw}' + (f'_n{n}' if n != len(recs) else '') + '_ms'] = round(statistics.median(ts) * 1e3, 3)
    print(json.dumps(out), flush=True)
