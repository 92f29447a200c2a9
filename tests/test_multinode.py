"""Two real node processes (uvicorn on 127.0.0.1) + the miner CLI: mining, gossip, sync, and a WebSocket
subscriber receiving the new block over a real socket."""
import base64
import json
import os
import socket
import struct
import subprocess
import sys
import time

import httpx
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEY_A = 0x1111111111111111111111111111111111111111111111111111111111111111


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(tmp, name):
    env = dict(os.environ)
    env.update({'UPOW_DATA_DIR': str(tmp / name), 'UPOW_CORE_URL': '', 'UPOW_START_DIFFICULTY': '2.0',
                'UPOW_UTXO_BACKEND': 'host', 'UPOW_DISABLE_GPU': '1', 'UPOW_RATE_LIMIT': '0',
                'PYTHONPATH': ROOT, 'UPOW_LOG_LEVEL': 'WARNING'})
    return env


def _start(tmp, name, port):
    p = subprocess.Popen([sys.executable, '-m', 'upow_amd.node', '--host', '127.0.0.1', '--port', str(port),
                          '--log-level', 'warning'], env=_env(tmp, name), cwd=ROOT,
                         stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    url = f'http://127.0.0.1:{port}'
    for _ in range(300):
        try:
            if httpx.get(url + '/get_nodes', timeout=1).status_code == 200:
                return p, url
        except Exception:
            time.sleep(0.1)
    p.kill()
    raise RuntimeError('node did not start')


def _ws_connect(url):
    host, port = url.split('//')[1].split(':')
    c = socket.create_connection((host, int(port)), timeout=30)
    key = base64.b64encode(os.urandom(16))
    c.sendall(b'GET /ws HTTP/1.1\r\nHost: x\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n'
              b'Sec-WebSocket-Key: ' + key + b'\r\nSec-WebSocket-Version: 13\r\n\r\n')
    head = b''
    while b'\r\n\r\n' not in head:
        head += c.recv(1)
    assert head.startswith(b'HTTP/1.1 101'), head
    return c


def _ws_frame(payload: bytes) -> bytes:
    mask = os.urandom(4)
    n = len(payload)
    head = bytes([0x81]) + (bytes([0x80 | n]) if n < 126 else bytes([0x80 | 126]) + struct.pack('!H', n))
    return head + mask + bytes(b ^ mask[i % 4] for i, b in enumerate(payload))


def _ws_read(c) -> str:
    while True:  # text frames; server pings are skipped
        h = c.recv(2)
        op, n = h[0] & 15, h[1] & 127
        if n == 126:
            n = struct.unpack('!H', c.recv(2))[0]
        elif n == 127:
            n = struct.unpack('!Q', c.recv(8))[0]
        data = b''
        while len(data) < n:
            data += c.recv(n - len(data))
        if op == 1:
            return data.decode()


def _height(url):
    return httpx.get(url + '/get_mining_info', timeout=5).json()['result']['last_block'].get('id', 0)


@pytest.fixture
def two_nodes(tmp_path):
    procs = []
    try:
        pa, a = _start(tmp_path, 'a', _port())
        procs.append(pa)
        pb, b = _start(tmp_path, 'b', _port())
        procs.append(pb)
        yield a, b, tmp_path
    finally:
        for p in procs:
            p.terminate()
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                p.kill()


def test_mine_gossip_and_sync(two_nodes):
    a, b, tmp = two_nodes
    from upow_amd.wallet.builders import address_of
    addr = address_of(KEY_A)
    # node B mines 2 blocks on its own; node A then syncs them from B
    r = subprocess.run([sys.executable, '-m', 'upow_amd.miner', addr, '2', b + '/', '--device', 'cpu', '--blocks', '2',
                        '--chunk', '65536'], env=_env(tmp, 'miner'), cwd=ROOT, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert _height(b) == 2
    res = httpx.get(a + '/sync_blockchain', params={'node_url': b}, timeout=60).json()
    assert res == {'ok': True}, res
    assert _height(a) == 2
    ws = _ws_connect(a)  # the node's /ws endpoint over a real socket (node/http.py serves the upgrade)
    ws.sendall(_ws_frame(json.dumps({'type': 'subscribe_block'}).encode()))
    assert json.loads(_ws_read(ws))['message'] == 'Subscribed to block'
    assert json.loads(_ws_read(ws))['data'] == {'type': 'block_subscription'}
    ha = httpx.get(a + '/get_block', params={'block': 2}).json()['result']['block']['hash']
    hb = httpx.get(b + '/get_block', params={'block': 2}).json()['result']['block']['hash']
    assert ha == hb
    # register B as A's peer; a block mined on A is gossiped to B
    res = httpx.get(a + '/add_node', params={'url': b}, timeout=30).json()
    assert res['ok'] or res['error'] == 'Node already present', res  # sync already recorded B as a peer
    r = subprocess.run([sys.executable, '-m', 'upow_amd.miner', addr, '2', a + '/', '--device', 'cpu', '--blocks', '1',
                        '--chunk', '65536'], env=_env(tmp, 'miner'), cwd=ROOT, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    for _ in range(100):
        if _height(b) == 3:
            break
        time.sleep(0.1)
    assert _height(a) == 3 and _height(b) == 3
    ev = json.loads(_ws_read(ws))  # node A published its new block to the subscriber
    assert ev['type'] == 'new_block' and ev['data']['block_no'] == 3
    ws.close()
    assert httpx.get(a + '/').json()['unspent_outputs_hash'] == httpx.get(b + '/').json()['unspent_outputs_hash']
