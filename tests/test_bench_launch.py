"""bench.py rank launch: ``python bench.py --gpus N`` must run N ranks (driver contract), report them, and
refuse a mismatched WORLD_SIZE. CPU ranks over gloo, the same launcher path the driver takes on a node."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=300):
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_PORT')}
    env.update(env_extra or {})
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), *args], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{')]
    return p.returncode, (json.loads(lines[-1]) if lines else None), p


def test_bench_gpus2_launches_two_ranks():
    rc, out, p = _run(['--gpus', '2', '--nonces', str(1 << 20), '--steps', '2', '--warmup', '1'])
    assert rc == 0, p.stderr[-3000:]
    assert out['world'] == 2
    assert out['config']['parallelism'] == 'dp2'
    assert out['config']['global_batch'] == 2 * (1 << 20)
    assert out['metric'] == 'sha256_pow_hashrate_MH/s'


def test_bench_world_size_mismatch_refused():
    rc, out, p = _run(['--gpus', '4', '--nonces', str(1 << 16), '--steps', '1', '--warmup', '0'],
                      env_extra={'WORLD_SIZE': '1', 'RANK': '0', 'LOCAL_RANK': '0'})
    assert rc == 2 and out is None
    assert 'WORLD_SIZE=1' in p.stderr


def test_bench_cluster_verify_one_chain_two_ranks():
    """--mode verify at N=2 validates ONE chain on a two-replica cluster (sharded ECDSA); both replicas end
    at the same height and UTXO-set hash, and tx/s is the chain's, not a sum over ranks."""
    rc, out, p = _run(['--gpus', '2', '--mode', 'verify', '--txs', '120', '--steps', '2', '--warmup', '1'])
    assert rc == 0, p.stderr[-3000:]
    assert out['world'] == 2 and out['config']['parallelism'] == 'replica2+sigshard'
    assert out['config']['block_path'] == 'native'
    reps = out['replicas']
    assert len(reps) == 2 and reps[0]['utxo_hash'] == reps[1]['utxo_hash'] and reps[0]['height'] == reps[1]['height']
    assert abs(out['value'] - 2 * 120 / (out['ms_per_step'] * 2 / 1000)) / out['value'] < 0.02


def test_bench_cluster_sync_one_chain_two_ranks():
    """--mode sync at N=2: ONE chain synced page by page by a two-replica cluster node (chunk signatures sharded
    over the ranks, every block agreed before commit); both replicas end at the same height and UTXO hash."""
    rc, out, p = _run(['--gpus', '2', '--mode', 'sync', '--txs', '30', '--steps', '20', '--warmup', '2'],
                      env_extra={'UPOW_START_DIFFICULTY': '1.0'})
    assert rc == 0, p.stderr[-3000:]
    assert out['metric'] == 'sync_tx_per_s' and out['world'] == 2 and out['scaling'] == 'strong'
    assert len({(r['height'], r['utxo_hash']) for r in out['replicas']}) == 1
    assert out['page']['page_path'] == 20 and out['op_stream']['commits_agreed'] >= 22


def test_bench_sync_and_verify_hold_txs_as_body_spans():
    """The single-node sync and verify benches hold their txs as a node does after the native body parse
    (spans of the /get_blocks or /push_block body) and report the push body's parse times."""
    rc, out, p = _run(['--mode', 'sync', '--txs', '20', '--steps', '10', '--warmup', '1'],
                      env_extra={'UPOW_START_DIFFICULTY': '1.0'})
    assert rc == 0, p.stderr[-3000:]
    assert out['metric'] == 'sync_tx_per_s' and out['page']['page_path'] == 10
    rc, out, p = _run(['--mode', 'verify', '--txs', '60', '--steps', '2', '--warmup', '1'])
    assert rc == 0, p.stderr[-3000:]
    assert out['config']['block_path'] == 'native' and out['push_body_parse_ms']['native_spans'] > 0


GUARD = r'''
import os, sys, json
sys.path.insert(0, sys.argv[1])
import bench
from upow_amd.parallel.dist import init_from_env
ctx = init_from_env(backend='gloo', want_gpu=False)

def side(args, ctx):
    if ctx.rank == 1:
        raise RuntimeError('boom on rank 1')
    ctx.barrier()  # rank 0 waits in a collective rank 1 never joins
    return {'sync_tx_per_s': 1.0}
bench._sync_side_metrics = side
os.environ['UPOW_BENCH_SIDE_DEADLINE_S'] = '20'
res = bench._guarded_side_metric(None, ctx, {'metric': 'headline', 'value': 1})
print(json.dumps(res), flush=True)
'''


def test_side_metric_failure_keeps_the_headline_line(tmp_path):
    """A side metric that fails on one rank of N must still leave rank 0's one headline JSON line (with
    sync_error) and every rank exiting 0, not a job hung in a collective."""
    script = tmp_path / 'guard.py'
    script.write_text(GUARD)
    import socket
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_PORT')}
    p = subprocess.run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
                        '--master-addr', '127.0.0.1', '--master-port', str(port), str(script), ROOT],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    lines = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith('{')]
    assert p.returncode == 0, p.stderr[-2000:]
    assert len(lines) == 1 and lines[0]['metric'] == 'headline' and 'sync_error' in lines[0], p.stdout
