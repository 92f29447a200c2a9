"""Batch-verify throughput of the gfx950 P-256 kernels vs the host C++ path.

Every number is the median of three timed calls after one untimed call of the same size: the first call of a
size grows the pinned staging and the pooled device buffers (one-time allocations that are not throughput).
Records: 8,300 signatures by 64 keys, repeated to the batch size. Prints one JSON line of signatures/s."""
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


def rate(buf, reps: int = 3) -> float:
    n = len(buf) // 160
    st = op.verify_records(buf, device='gpu')  # untimed: sizes the buffers
    assert (st == 1).all(), st[:20]
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        op.verify_records(buf, device='gpu')
        ts.append(time.perf_counter() - t)
    return round(n / statistics.median(ts), 1)


for var in ('0', '1', '2', '4'):
    os.environ['UPOW_P256_VARIANT'] = var
    out[f'variant{var}_gpu_{8300 * 16}'] = rate(base * 16)
    out[f'variant{var}_gpu_8300'] = rate(base)
os.environ['UPOW_P256_VARIANT'] = 'a'  # the default: quad kernel up to 32k signatures, then one lane
for n in (8300, 8300 * 4, 8300 * 16, 8300 * 64):  # 64 blocks = 8,300 waves: saturates the chip
    out[f'gpu_{n}'] = rate(base * (n // 8300))
# the same 531,200 without the round-aligned split (one-lane kernel for everything: a third, 3 %-full round)
os.environ['UPOW_P256_TAIL'] = '0'
out['notail_split_gpu_531200'] = rate(base * 64)
os.environ.pop('UPOW_P256_TAIL')
# exactly two rounds (524,288) and a bigger batch (1,062,400 = 4 rounds + 14,024)
out['gpu_524288'] = rate((base * 64)[:160 * 524288])
out['gpu_1062400'] = rate(base * 128)
# the one-lane kernel's occupancy variants at the saturating size: 1 = 4 waves/SIMD (128 VGPRs, spills),
# 5 = 3 waves (168 VGPRs), 0 = the compiler's choice
for var in ('0', '1', '5'):
    os.environ['UPOW_P256_VARIANT'] = var
    out[f'variant{var}_gpu_531200'] = rate(base * 64)
os.environ['UPOW_P256_VARIANT'] = 'a'
# one-lane batch launches sliced (UPOW_P256_SLICE signatures per launch; 2^30 = one launch) at 531,200
for sl in (131072, 262144, 1 << 30):
    os.environ['UPOW_P256_SLICE'] = str(sl)
    out[f'slice{sl}_gpu_531200'] = rate(base * 64)
os.environ.pop('UPOW_P256_SLICE')
t = time.perf_counter()
st = op.verify_records(base[:160 * 2000], device='cpu', threads=16)
out['cpu16_2000'] = round(2000 / (time.perf_counter() - t), 1)
print(json.dumps(out), flush=True)
