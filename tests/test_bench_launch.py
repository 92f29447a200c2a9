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
