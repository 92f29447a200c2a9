"""The cluster's native commit vote (csrc/rccl_vote.hip) on a real RCCL communicator: a single-rank job
under torch.distributed.run (UPOW_FORCE_DIST=1, the 1-GPU box), so the vote runs through ncclAllGather on
the runtime's own communicator next to PyTorch's process group. The outcome must be the sum of the votes,
for both values, and the latency script must report the native path."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROBE = r'''
import json, os, sys
sys.path.insert(0, sys.argv[1])
from upow_amd.ops.native import lib
lib()
from upow_amd.parallel.dist import init_from_env, op_context, shutdown
ctx = init_from_env()
assert ctx.is_distributed
op = op_context(ctx)
op.bind_owner()
outs = [op.vote_finish(op.vote_start(v)) for v in (1, 0, 1, 1, 0)]
print(json.dumps({'outs': outs, 'native': op.__dict__.get('_nv') is not None,
                  'stats': list(lib().rccl_vote_stats(op._nv[1])) if op.__dict__.get('_nv') else None}), flush=True)
shutdown(ctx)
'''


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.gpu
def test_native_vote_on_a_single_rank_rccl_job(gpu, tmp_path):
    script = tmp_path / 'probe.py'
    script.write_text(PROBE)
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_PORT')}
    env.update(UPOW_FORCE_DIST='1', HSA_ENABLE_IPC_MODE_LEGACY='0')
    p = subprocess.run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '1',
                        '--master-addr', '127.0.0.1', '--master-port', str(_port()), str(script), ROOT],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    res = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith('{')][-1]
    assert res['native'] is True
    assert res['outs'] == [1, 0, 1, 1, 0]
    assert int(res['stats'][0]) == 5  # five votes went through the native communicator
