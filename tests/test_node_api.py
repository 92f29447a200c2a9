"""Node REST + WebSocket API through starlette's TestClient (single node, in-process)."""
import asyncio
import hashlib
import os
from decimal import Decimal

import pytest

KEY_A = 0x1111111111111111111111111111111111111111111111111111111111111111
KEY_B = 0x2222222222222222222222222222222222222222222222222222222222222222


@pytest.fixture
def node(tmp_path, monkeypatch):
    monkeypatch.setenv('UPOW_DATA_DIR', str(tmp_path))
    monkeypatch.setenv('UPOW_CORE_URL', '')
    monkeypatch.setenv('UPOW_DATABASE_PATH', str(tmp_path / 'ledger.sqlite3'))
    monkeypatch.setenv('UPOW_UTXO_BACKEND', 'host')
    from upow_amd.ledger import manager
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('1.5'))
    manager.Manager.difficulty = None
    from upow_amd.node import main
    from upow_amd.node import peers
    peers.reset()
    main.limiter.reset()
    main.transactions_cache.clear()
    from starlette.testclient import TestClient
    with TestClient(main.app, base_url='http://testserver') as c:
        yield c, main
    main.db.close()


def _mine(client, address, ts, txs=()):
    from upow_amd.models.block import PowTarget, header_prefix
    from upow_amd.ops.pow import PowJob, search
    info = client.get('/get_mining_info').json()['result']
    last = info['last_block']
    prev = last.get('hash', (18_884_643).to_bytes(32, 'little').hex())
    hashes = info['pending_transactions_hashes'] if not txs else sorted(hashlib.sha256(bytes.fromhex(t)).hexdigest() for t in txs)
    merkle = hashlib.sha256(b''.join(bytes.fromhex(h) for h in hashes)).hexdigest()
    job = PowJob.create(header_prefix(prev, address, merkle, ts, info['difficulty']),
                        PowTarget.from_difficulty(prev, info['difficulty']))
    r = search(job, 0, 1 << 20, device='cpu', threads=2)
    content = job.header_with_nonce(r.nonces[0]).hex()
    return client.post('/push_block', json={'block_content': content, 'txs': hashes, 'block_no': last.get('id', 0) + 1}).json()


def test_mining_flow_and_queries(node):
    client, main = node
    from upow_amd.wallet.builders import address_of
    a, b = address_of(KEY_A), address_of(KEY_B)
    r = client.get('/get_mining_info').json()
    assert r['ok'] and r['result']['difficulty'] == 1.5 and r['result']['last_block'] == {}
    base = 1_700_000_000
    for k in range(1, 4):
        assert _mine(client, a, base + k) == {'ok': True}
    info = client.get('/get_address_info', params={'address': a}).json()
    assert info['result']['balance'] == '18'
    assert len(info['result']['spendable_outputs']) == 3
    blk = client.get('/get_block', params={'block': '2'}).json()['result']
    assert blk['block']['id'] == 2 and len(blk['transactions']) == 1
    assert client.get('/get_block', params={'block': blk['block']['hash']}).json()['result']['block']['id'] == 2
    blocks = client.get('/get_blocks', params={'offset': 1, 'limit': 10}).json()['result']
    assert [x['block']['id'] for x in blocks] == [1, 2, 3]
    # push a transfer and mine it by hash
    async def mk():
        from upow_amd.wallet.builders import create_transaction
        return await create_transaction(KEY_A, b, '1.25')
    tx = asyncio.run(mk())
    res = client.post('/push_tx', json={'tx_hex': tx.hex()}).json()
    assert res['ok'], res
    assert client.get('/push_tx', params={'tx_hex': tx.hex()}).json() == {'ok': False, 'error': 'Transaction just added'}
    assert client.get('/get_pending_transactions').json()['result'] == [tx.hex()]
    mi = client.get('/get_mining_info').json()['result']
    assert mi['pending_transactions_hashes'] == [tx.hash()]
    assert _mine(client, a, base + 10) == {'ok': True}
    assert client.get('/get_address_info', params={'address': b}).json()['result']['balance'] == '1.25'
    t = client.get('/get_transaction', params={'tx_hash': tx.hash()}).json()
    assert t['ok'] and t['result']['outputs'][0]['amount'] == 1.25
    txs = client.get('/get_address_transactions', params={'address': b}).json()['result']['transactions']
    assert [x['hash'] for x in txs] == [tx.hash()]
    root = client.get('/').json()
    assert root['ok'] and root['version'] == 2 and len(root['unspent_outputs_hash']) == 64
    sup = client.get('/get_supply_info').json()['result']
    assert sup['circulating_supply'] == 24 and sup['max_supply'] == 18884643.75
    # errors / envelopes
    assert client.get('/get_block', params={'block': '99'}).json() == {'ok': False, 'error': 'Block not found'}
    old = _mine(client, a, base + 5)
    assert old['ok'] is False
    assert client.get('/get_transaction', params={'tx_hash': '00' * 32}).json()['ok'] is False
    # observability: Prometheus text with the block/tx/signature counters
    m = client.get('/metrics')
    assert m.status_code == 200 and m.headers['content-type'].startswith('text/plain')
    series = {ln.split(' ')[0]: float(ln.split(' ')[1]) for ln in m.text.splitlines() if ln and not ln.startswith('#')}
    assert series['upow_chain_height'] == 4 and series['upow_mempool_size'] == 0
    assert sum(v for k, v in series.items() if k.startswith('upow_blocks_applied_total')) >= 4
    assert series['upow_blocks_applied_total{path="native"}'] >= 1  # the transfer block took the native path
    assert series['upow_signatures_verified_total'] >= 1
    assert series['upow_blocks_rejected_total{path="push"}'] >= 1


def test_push_tx_direct_path_matches_routed(node, monkeypatch):
    """POST /push_tx with a JSON body bypasses the framework router (node/main.py _push_tx_direct): the
    responses, status codes and error envelopes must be the routed endpoint's."""
    client, main = node
    from upow_amd.wallet.builders import address_of
    a, b = address_of(KEY_A), address_of(KEY_B)
    for k in range(1, 3):
        assert _mine(client, a, 1_700_000_000 + k) == {'ok': True}
    from starlette.testclient import TestClient
    raw = TestClient(main.app, base_url='http://testserver', raise_server_exceptions=False)  # 500s as responses
    cases = [{'tx_hex': 'zz'}, {'tx_hex': '00' * 40}, {'tx_hex': 'ab', 'extra': 1}]
    got = {}
    for fast in (True, False):
        monkeypatch.setattr(main, '_PUSH_FAST', fast)
        got[fast] = [(r.status_code, r.json()) for r in (raw.post('/push_tx', json=c) for c in cases)]
        got[fast].append((lambda r: (r.status_code, r.headers['access-control-allow-origin']))(
            raw.post('/push_tx', content=b'{not json', headers={'content-type': 'application/json'})))
    assert got[True] == got[False]
    assert got[True][0][0] == 500 and got[True][0][1]['ok'] is False

    async def mk():
        from upow_amd.wallet.builders import create_transaction
        return await create_transaction(KEY_A, b, '0.5')
    tx = asyncio.run(mk())
    monkeypatch.setattr(main, '_PUSH_FAST', True)
    r = client.post('/push_tx', json={'tx_hex': tx.hex()})
    assert r.status_code == 200 and r.json() == {'ok': True, 'result': 'Transaction has been accepted', 'tx_hash': tx.hash()}
    assert r.headers['access-control-allow-origin'] == '*'
    monkeypatch.setattr(main, '_PUSH_FAST', False)
    assert client.post('/push_tx', json={'tx_hex': tx.hex()}).json() == {'ok': False, 'error': 'Transaction just added'}


def test_rate_limit_and_ip_filter(node):
    client, main = node
    for _ in range(3):
        assert client.get('/').status_code == 200
    r = client.get('/')
    assert r.status_code == 429 and r.json()['error'].startswith('Rate limit exceeded')
    r = client.get('/get_nodes//', follow_redirects=False)
    assert r.status_code in (302, 307)
    from upow_amd.node.access import AccessPolicy
    main.access.install(AccessPolicy(blocked_paths=frozenset({'/get_nodes'})))
    r = client.get('/get_nodes')
    assert r.status_code == 403 and r.json() == {'ok': False, 'error': 'Access forbidden temporarily.'}
    main.access.install(AccessPolicy.from_json({'blocklist': ['10.1.0.0/16']}))
    r = client.get('/get_nodes', headers={'X-Forwarded-For': '10.1.2.3, 1.1.1.1'})
    assert r.status_code == 403 and r.json()['error'] == 'Access forbidden.'
    assert client.get('/get_nodes', headers={'X-Real-IP': '10.2.0.1'}).status_code == 200
    main.access.install(AccessPolicy.from_json({'whitelist': ['9.9.9.9'], 'blocklist': ['9.9.9.9']}))
    assert client.get('/get_nodes', headers={'X-Real-IP': '9.9.9.9'}).status_code == 200  # allow-list wins
    assert client.get('/get_nodes', headers={'X-Real-IP': '8.8.8.8'}).status_code == 403
    main.access.reload()  # back to the (empty) policy file
    assert client.get('/send_to_address', params={'to_address': 'x', 'amount': 1}).status_code == 403


def test_websocket_protocol(node):
    """/ws client contract on the node app: pong, the double success on subscribe, unsubscribe
    (subscribed and not), a published block, and close after a refused verb."""
    from starlette.websockets import WebSocketDisconnect
    client, main = node
    with client.websocket_connect('/ws') as ws:
        ws.send_json({'type': 'ping'})
        pong = ws.receive_json()
        assert pong['type'] == 'pong' and 'timestamp' in pong
        ws.send_json({'type': 'subscribe_block'})
        m1, m2 = ws.receive_json(), ws.receive_json()
        assert (m1['type'], m1['message'], m1['data']) == ('success', 'Subscribed to block', {'channel': 'block'})
        assert (m2['message'], m2['data']) == ('Subscribed to block updates', {'type': 'block_subscription'})
        ws.send_json({'type': 'unsubscribe_block'})
        u1, u2 = ws.receive_json(), ws.receive_json()
        assert (u1['message'], u1['data']) == ('Unsubscribed from block', {'channel': 'block'})
        assert (u2['message'], u2['data']) == ('Unsubscribed from block updates', {'type': 'block_unsubscription'})
        ws.send_json({'type': 'unsubscribe_block'})
        e, u3 = ws.receive_json(), ws.receive_json()
        assert (e['type'], e['error_code']) == ('error', 'NOT_SUBSCRIBED')
        assert e['message'] == "Not subscribed to channel 'block'"
        assert u3['type'] == 'success' and u3['data'] == {'type': 'block_unsubscription'}
        ws.send_json({'type': 'subscribe_block'})
        ws.receive_json(), ws.receive_json()
        ws.send_json({'type': 'pong'})  # accepted silently
        from upow_amd.wallet.builders import address_of
        assert _mine(client, address_of(KEY_A), 1_700_000_001) == {'ok': True}
        ev = ws.receive_json()
        assert ev['type'] == 'new_block' and ev['data']['block_no'] == 1 and 'timestamp' in ev
        assert isinstance(ev['data']['difficulty'], float)  # Decimal goes out as a JSON number
        ws.send_json({'type': 'subscribe_transaction'})  # not on the reference allow-list
        err = ws.receive_json()
        assert err['type'] == 'error' and err['error_code'] == 'INVALID_MESSAGE_TYPE'
        assert err['message'] == "Message type 'subscribe_transaction' not allowed"
        with pytest.raises(WebSocketDisconnect) as exc:
            ws.receive_json()
        assert exc.value.code == 1000
    assert main.websocket_router is not None


@pytest.mark.parametrize('ledger_thread', ['1', '0'])
def test_block_apply_does_not_block_the_http_loop(tmp_path, monkeypatch, ledger_thread):
    """While a block is validated/applied (here: held for 1.2 s on the ledger thread), other requests
    are served by the HTTP loop (ledger/worker.py). With UPOW_LEDGER_THREAD=0 the same request waits
    for the block — the reference's behaviour (main.py:521-652 on the single asyncio loop)."""
    import threading
    import time
    monkeypatch.setenv('UPOW_LEDGER_THREAD', ledger_thread)
    monkeypatch.setenv('UPOW_DATA_DIR', str(tmp_path))
    monkeypatch.setenv('UPOW_CORE_URL', '')
    monkeypatch.setenv('UPOW_DATABASE_PATH', str(tmp_path / 'ledger.sqlite3'))
    monkeypatch.setenv('UPOW_UTXO_BACKEND', 'host')
    from upow_amd.ledger import fastpath, manager
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('1.5'))
    manager.Manager.difficulty = None
    from upow_amd.node import main
    from upow_amd.node import peers
    from upow_amd.wallet.builders import address_of
    peers.reset()
    main.limiter.reset()
    inner = fastpath._create_block_from_hex
    ledger_threads = []

    async def slow(*a, **kw):
        ledger_threads.append(threading.current_thread().name)
        time.sleep(1.2)  # a long block: blocks whichever event loop runs it
        return await inner(*a, **kw)
    monkeypatch.setattr(fastpath, '_create_block_from_hex', slow)
    from starlette.testclient import TestClient
    with TestClient(main.app, base_url='http://testserver') as client:
        result = {}
        t = threading.Thread(target=lambda: result.setdefault('block', _mine(client, address_of(KEY_A), 1_700_000_001)))
        t.start()
        while not ledger_threads:
            time.sleep(0.01)
        t0 = time.perf_counter()
        assert client.get('/get_nodes').json()['ok']
        latency = time.perf_counter() - t0
        t.join()
        assert result['block'] == {'ok': True}
    main.db.close()
    if ledger_thread == '1':
        assert ledger_threads == ['upow-ledger'] and latency < 0.6, latency
    else:
        assert ledger_threads != ['upow-ledger'] and latency > 0.5, latency


def test_request_host_locality_matches_base_url_hostname():
    """The gate's cached Host-header test gives ``request.base_url.hostname``'s answer."""
    from starlette.requests import Request as StarletteRequest
    from upow_amd.node.main import _scope_host_is_local
    from upow_amd.node.utils import ip_is_local
    for host in (b'localhost:3006', b'127.0.0.1', b'192.168.1.7:80', b'example.org', b'8.8.8.8:3006', b'[::1]:80', None):
        scope = {'type': 'http', 'headers': [(b'host', host)] if host else [], 'server': ('10.0.0.5', 80),
                 'scheme': 'http', 'path': '/', 'query_string': b'', 'root_path': ''}
        name = StarletteRequest(scope).base_url.hostname
        assert _scope_host_is_local(scope) == (name == 'localhost' or ip_is_local(name)), host
