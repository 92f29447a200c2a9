"""Raw batch-verify throughput of the gfx950 P-256 kernel vs the host C++ path."""
import hashlib
import json
import random
import sys
import time

sys.path.insert(0, '.')
from upow_amd.ops.native import lib  # noqa: E402
from upow_amd.ops import p256 as op  # noqa: E402

lib()
import torch  # noqa: E402
torch.cuda.set_device(0)
rng = random.Random(1)
keys = [rng.randrange(1, op.oracle.N) for _ in range(64)]
pubs = [op.public_key(k) for k in keys]
recs = []
for i in range(8300):
    msg = rng.randbytes(200)
    recs.append(op.record(pubs[i % 64], op.sign(msg, keys[i % 64]), hashlib.sha256(msg).digest()))
base = b''.join(recs)
out = {}
import os
for var in ('0', '1', '2', '4'):
    os.environ['UPOW_P256_VARIANT'] = var
    buf = base * 16
    op.verify_records(buf[:160 * 512], device='gpu')
    t = time.perf_counter()
    st = op.verify_records(buf, device='gpu')
    out[f'variant{var}_gpu_{8300 * 16}'] = round(8300 * 16 / (time.perf_counter() - t), 1)
    assert (st == 1).all()
    t = time.perf_counter()
    st = op.verify_records(base, device='gpu')
    out[f'variant{var}_gpu_8300'] = round(8300 / (time.perf_counter() - t), 1)
os.environ['UPOW_P256_VARIANT'] = 'a'  # the default: pair kernel up to 32k signatures, then one lane
for n in (8300, 8300 * 4, 8300 * 16, 8300 * 64):  # 64 blocks = 8,300 waves: saturates the chip
    buf = base * (n // 8300)
    op.verify_records(buf[:160 * 512], device='gpu')
    t = time.perf_counter()
    st = op.verify_records(buf, device='gpu')
    dt = time.perf_counter() - t
    assert (st == 1).all(), st[:20]
    out[f'gpu_{n}'] = round(n / dt, 1)
t = time.perf_counter()
st = op.verify_records(base[:160 * 2000], device='cpu', threads=16)
out['cpu16_2000'] = round(2000 / (time.perf_counter() - t), 1)
print(json.dumps(out), flush=True)
