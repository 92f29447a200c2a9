"""End to end on the MI355X: a node process (GPU validation backends) + the GPU miner CLI at the
mainnet start difficulty (6.0), then a wallet transfer mined into the next block."""
import os
import socket
import subprocess
import sys
import time

import httpx
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
def test_gpu_miner_against_node(gpu, tmp_path):
    env = dict(os.environ, UPOW_DATA_DIR=str(tmp_path / 'node'), UPOW_CORE_URL='', UPOW_RATE_LIMIT='0',
               PYTHONPATH=ROOT, UPOW_LOG_LEVEL='WARNING')
    port = _port()
    node = subprocess.Popen([sys.executable, '-m', 'upow_amd.node', '--host', '127.0.0.1', '--port', str(port),
                             '--log-level', 'warning'], env=env, cwd=ROOT, stdout=subprocess.DEVNULL,
                            stderr=subprocess.DEVNULL)
    url = f'http://127.0.0.1:{port}'
    try:
        for _ in range(600):
            try:
                if httpx.get(url + '/get_nodes', timeout=1).status_code == 200:
                    break
            except Exception:
                time.sleep(0.2)
        from upow_amd.wallet.builders import address_of
        addr = address_of(0x5151)
        r = subprocess.run([sys.executable, '-m', 'upow_amd.miner', addr, '1', url + '/', '--blocks', '3'],
                           env=dict(env, UPOW_DATA_DIR=str(tmp_path / 'miner')), cwd=ROOT, capture_output=True,
                           text=True, timeout=240)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        assert 'BLOCK MINED' in r.stdout and 'x gpu' in r.stdout
        info = httpx.get(url + '/get_mining_info', timeout=10).json()['result']
        assert info['last_block']['id'] == 3 and info['difficulty'] == 6.0
        bal = httpx.get(url + '/get_address_info', params={'address': addr}, timeout=10).json()['result']['balance']
        assert bal == '18'
    finally:
        node.terminate()
        try:
            node.wait(20)
        except subprocess.TimeoutExpired:
            node.kill()


@pytest.mark.gpu
def test_rccl_collectives_and_sharded_verify(gpu):
    """Every collective of parallel/ on a real RCCL process group (1 rank, forced)."""
    import subprocess
    import sys
    env = dict(os.environ, UPOW_FORCE_DIST='1', PYTHONPATH=ROOT + os.pathsep + os.environ.get('PYTHONPATH', ''))
    r = subprocess.run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '1',
                        '--master-addr', '127.0.0.1', '--master-port', '29541', 'scripts/rccl_selfcheck.py'],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert '"rccl_selfcheck": "ok"' in r.stdout and '"backend": "nccl"' in r.stdout
