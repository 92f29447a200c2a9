"""A/B the PoW kernel variants in one process (interleaved, n>=3 reps each)."""
import hashlib
import json
import sys
import time

sys.path.insert(0, '.')
from upow_amd.ops.native import lib  # noqa: E402
from upow_amd.models.block import PowTarget, header_prefix  # noqa: E402
from upow_amd.ops.pow import PowJob, search  # noqa: E402

L = lib()
import torch  # noqa: E402
torch.cuda.set_device(0)
prev = hashlib.sha256(b'x').hexdigest()
pre = header_prefix(prev, 'DgQKikeDqS2Fzue23KuA36L4eJSFh649zA9jJ6zwbzUMp', hashlib.sha256(b'm').hexdigest(),
                    1_790_000_000, '6.3')
job = PowJob.create(pre, PowTarget.from_difficulty(prev, '6.3'))
variants = [int(v) for v in (sys.argv[1].split(',') if len(sys.argv) > 1 else ['0', '1'])]
res = {v: [] for v in variants}
for v in variants:
    print('info', v, L.pow_kernel_info(v), flush=True)
    search(job, 0, 1 << 30, device='gpu', variant=v)  # warm
for rep in range(3):
    for v in variants:
        t = time.perf_counter()
        r = search(job, 0, 1 << 32, device='gpu', variant=v)
        dt = time.perf_counter() - t
        res[v].append((1 << 32) / dt / 1e6)
print(json.dumps({str(k): [round(x, 1) for x in v] for k, v in res.items()}), flush=True)
