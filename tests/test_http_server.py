"""The node's server protocol (node/http.py over csrc/http_wire.cpp) on a real socket: HTTP/1.1 framing,
keep-alive, pipelining, chunked bodies both ways, Expect: 100-continue, bad requests, and WebSocket
(handshake, text/binary, fragmentation, ping/pong, close) through the ASGI scopes."""
import asyncio
import base64
import hashlib
import os
import socket
import struct
import threading
import time

import httpx
import pytest
from hypothesis import HealthCheck, given, settings, strategies as st
import uvicorn
from starlette.applications import Starlette
from starlette.responses import JSONResponse, PlainTextResponse, StreamingResponse
from starlette.routing import Route, WebSocketRoute

from upow_amd.node.http import NodeHttpProtocol


async def hello(request):
    return JSONResponse({'ok': True, 'q': request.query_params.get('q'), 'path': request.url.path})


async def echo(request):
    body = await request.body()
    return PlainTextResponse(body.decode(), headers={'x-len': str(len(body))})


async def stream(request):
    async def gen():
        for k in range(3):
            yield f'part{k};'.encode()
    return StreamingResponse(gen())


async def big(request):
    n = int(request.query_params['n'])
    return PlainTextResponse(bytes(range(97, 123)) * (n // 26) + b'z' * (n % 26))


async def ws_echo(websocket):
    await websocket.accept()
    while True:
        msg = await websocket.receive()
        if msg['type'] == 'websocket.disconnect':
            return
        if msg.get('text') == 'bye':
            await websocket.close(code=4000)
            return
        if msg.get('text') is not None:
            await websocket.send_text('echo:' + msg['text'])
        else:
            await websocket.send_bytes(b'echo:' + msg['bytes'])


app = Starlette(routes=[Route('/hello', hello), Route('/echo', echo, methods=['POST']), Route('/stream', stream), Route('/big', big),
                        WebSocketRoute('/ws', ws_echo)])


@pytest.fixture(scope='module')
def server():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    cfg = uvicorn.Config(app, host='127.0.0.1', port=port, log_level='warning', http=NodeHttpProtocol,
                         lifespan='off', timeout_keep_alive=5)
    srv = uvicorn.Server(cfg)
    t = threading.Thread(target=srv.run, daemon=True)
    t.start()
    for _ in range(200):
        if srv.started:
            break
        time.sleep(0.02)
    yield port
    srv.should_exit = True
    t.join(5)


def _raw(port, data: bytes, timeout: float = 5.0) -> bytes:
    """Send raw bytes and read until the server closes the connection (every caller's last request asks
    for that, or is one the server must close on)."""
    with socket.create_connection(('127.0.0.1', port), timeout=timeout) as c:
        c.sendall(data)
        out = b''
        while True:
            try:
                chunk = c.recv(65536)
            except socket.timeout:
                break
            if not chunk:
                break
            out += chunk
        return out


def test_keep_alive_requests_and_bodies(server):
    with httpx.Client(base_url=f'http://127.0.0.1:{server}') as c:
        for k in range(5):  # one pooled connection, several requests
            r = c.get('/hello', params={'q': str(k)})
            assert r.status_code == 200 and r.json() == {'ok': True, 'q': str(k), 'path': '/hello'}
        body = os.urandom(300_000).hex()
        r = c.post('/echo', content=body)
        assert r.text == body and r.headers['x-len'] == str(len(body))
        r = c.get('/stream')
        assert r.text == 'part0;part1;part2;' and r.headers.get('transfer-encoding') == 'chunked'
        assert c.get('/missing').status_code == 404
        assert c.head('/hello').status_code in (200, 405)


def test_pipelined_and_chunked_request(server):
    req = (b'GET /hello?q=a HTTP/1.1\r\nHost: x\r\n\r\n'
           b'POST /echo HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\n\r\n4\r\nabcd\r\n3;ext=1\r\nefg\r\n0\r\n\r\n'
           b'GET /hello?q=c HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n')
    out = _raw(server, req)
    parts = out.split(b'HTTP/1.1 ')[1:]
    assert len(parts) == 3 and all(p.startswith(b'200') for p in parts)
    assert b'"q":"a"' in parts[0] and parts[1].endswith(b'abcdefg') and b'"q":"c"' in parts[2]


def test_expect_continue_and_bad_requests(server):
    with socket.create_connection(('127.0.0.1', server), timeout=5) as c:
        c.sendall(b'POST /echo HTTP/1.1\r\nHost: x\r\nContent-Length: 5\r\nExpect: 100-continue\r\n\r\n')
        assert c.recv(100).startswith(b'HTTP/1.1 100 Continue')
        c.sendall(b'hello')
        got = b''
        while not got.endswith(b'hello'):
            chunk = c.recv(4096)
            assert chunk
            got += chunk
        assert got.startswith(b'HTTP/1.1 200')
    assert _raw(server, b'GARBAGE\r\n\r\n').startswith(b'HTTP/1.1 400')
    assert _raw(server, b'GET /hello HTTP/1.1\r\nContent-Length: 1\r\nContent-Length: 2\r\n\r\n').startswith(
        b'HTTP/1.1 400')
    out = _raw(server, b'GET /hello HTTP/1.0\r\n\r\n')  # HTTP/1.0: closed after the response
    assert out.startswith(b'HTTP/1.1 200') and b'connection: close' in out.lower()


def _ws_frame(op: int, payload: bytes, fin: bool = True) -> bytes:
    mask = os.urandom(4)
    n = len(payload)
    head = bytes([(0x80 if fin else 0) | op])
    head += bytes([0x80 | n]) if n < 126 else (bytes([0x80 | 126]) + struct.pack('!H', n))
    return head + mask + bytes(b ^ mask[i % 4] for i, b in enumerate(payload))


def _ws_read(c) -> tuple:
    h = c.recv(2)
    op, n = h[0] & 15, h[1] & 127
    if n == 126:
        n = struct.unpack('!H', c.recv(2))[0]
    data = b''
    while len(data) < n:
        data += c.recv(n - len(data))
    return op, data


def test_websocket_upgrade_echo_fragments_ping_close(server):
    key = base64.b64encode(os.urandom(16))
    with socket.create_connection(('127.0.0.1', server), timeout=5) as c:
        c.sendall(b'GET /ws HTTP/1.1\r\nHost: x\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n'
                  b'Sec-WebSocket-Key: ' + key + b'\r\nSec-WebSocket-Version: 13\r\n\r\n' + _ws_frame(1, b'early'))
        resp = b''
        while b'\r\n\r\n' not in resp:
            resp += c.recv(1)
        assert resp.startswith(b'HTTP/1.1 101')
        accept = base64.b64encode(hashlib.sha1(key + b'258EAFA5-E914-47DA-95CA-C5AB0DC85B11').digest())
        assert accept in resp
        assert _ws_read(c) == (1, b'echo:early')  # a frame sent with the handshake is not lost
        c.sendall(_ws_frame(1, 'héllo'.encode()))
        assert _ws_read(c) == (1, 'echo:héllo'.encode())
        c.sendall(_ws_frame(2, b'\x00\x01' * 200))
        assert _ws_read(c) == (2, b'echo:' + b'\x00\x01' * 200)
        c.sendall(_ws_frame(1, b'frag', fin=False) + _ws_frame(9, b'p') + _ws_frame(0, b'ment'))
        assert _ws_read(c) == (10, b'p')  # the ping is answered between the fragments
        assert _ws_read(c) == (1, b'echo:fragment')
        c.sendall(_ws_frame(1, b'bye'))
        op, data = _ws_read(c)
        assert op == 8 and struct.unpack('!H', data[:2])[0] == 4000


def test_large_response_to_a_slow_reader_arrives_whole(server):
    """A response larger than the socket buffer: the GIL-held direct send takes what fits and the
    transport sends the rest in order, also with a second response pipelined behind it."""
    n = 12 * 1024 * 1024
    partial = NodeHttpProtocol.partial_sends
    with socket.create_connection(('127.0.0.1', server), timeout=10) as c:
        c.sendall(b'GET /big?n=%d HTTP/1.1\r\nhost: x\r\n\r\nGET /big?n=30 HTTP/1.1\r\nhost: x\r\nconnection: close\r\n\r\n' % n)
        time.sleep(0.3)  # let the server fill the socket buffer first
        out = bytearray()
        while True:
            chunk = c.recv(1 << 16)
            if not chunk:
                break
            out += chunk
    want = bytes(range(97, 123)) * (n // 26) + b'z' * (n % 26)
    head, rest = bytes(out).split(b'\r\n\r\n', 1)
    assert b'content-length: %d' % n in head.lower()
    assert rest[:n] == want
    head2, body2 = rest[n:].split(b'\r\n\r\n', 1)
    assert head2.startswith(b'HTTP/1.1 200') and body2 == bytes(range(97, 123)) + b'zzzz'
    assert NodeHttpProtocol.partial_sends > partial


def test_client_gone_before_the_response_leaves_the_server_serving(server):
    """A client that closes (with a reset) before its response is written: the direct send fails, the
    transport reports the error and drops the connection, and the server keeps answering others."""
    for _ in range(3):
        c = socket.create_connection(('127.0.0.1', server), timeout=5)
        c.setsockopt(socket.SOL_SOCKET, socket.SO_LINGER, struct.pack('ii', 1, 0))  # close = RST
        c.sendall(b'GET /big?n=4000000 HTTP/1.1\r\nhost: x\r\n\r\n')
        c.close()
    time.sleep(0.2)
    r = httpx.get(f'http://127.0.0.1:{server}/hello', params={'q': 'still'}, timeout=5)
    assert r.status_code == 200 and r.json()['q'] == 'still'


_GOOD = [b'GET /hello?q=1 HTTP/1.1\r\nHost: x\r\n\r\n',
         b'POST /echo HTTP/1.1\r\nHost: x\r\nContent-Length: 3\r\n\r\nabc',
         b'POST /echo HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n2\r\nhi\r\n0\r\n\r\n',
         b'GET /missing HTTP/1.1\r\n\r\n']
_BAD = [b'GARBAGE\r\n\r\n', b'GET  HTTP/1.1\r\n\r\n', b'GET / HTTP/2.0\r\n\r\n', b'G\x00T / HTTP/1.1\r\n\r\n',
        b'GET / HTTP/1.1\r\n folded: x\r\n\r\n', b'GET / HTTP/1.1\r\nBad Header: 1\r\n\r\n',
        b'GET / HTTP/1.1\r\nX: a\x01b\r\n\r\n',
        b'POST /echo HTTP/1.1\r\nContent-Length: -5\r\n\r\n', b'POST /echo HTTP/1.1\r\nContent-Length: 99999999999999999999\r\n\r\n',
        b'POST /echo HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n-5\r\nhello\r\n0\r\n\r\n',
        b'POST /echo HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\nfffffffffffffffffff\r\n',
        b'POST /echo HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n3\r\nabcXY0\r\n\r\n',
        b'POST /echo HTTP/1.1\r\nTransfer-Encoding: gzip\r\n\r\n',
        b'POST /echo HTTP/1.1\r\nContent-Length: 1\r\nTransfer-Encoding: chunked\r\n\r\n',
        b'GET / HTTP/1.1\r\n' + b'X-Long: ' + b'a' * 70000 + b'\r\n\r\n']


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])
@given(st.lists(st.one_of(st.sampled_from(_GOOD), st.sampled_from(_BAD), st.binary(max_size=40)), min_size=1, max_size=5),
       st.lists(st.integers(1, 50), min_size=1, max_size=8))
def test_random_streams_get_400_or_close_never_a_crash(server, pieces, cuts):
    """Pipelined mixes of valid requests, malformed request lines and headers, oversized / negative /
    non-hex chunk sizes and random garbage, written in random segments: the server answers every complete
    valid request before the first bad one, answers the bad one with a 400 (or closes), and stays up."""
    data = b''.join(pieces)
    with socket.create_connection(('127.0.0.1', server), timeout=3) as c:
        at, k = 0, 0
        try:  # the server may answer 400 and close while the rest is still being written
            while at < len(data):
                n = cuts[k % len(cuts)]
                c.sendall(data[at:at + n])
                at += n
                k += 1
            c.shutdown(socket.SHUT_WR)
        except OSError:  # broken pipe, reset, or not connected any more
            pass
        out = b''
        while True:
            try:
                chunk = c.recv(65536)
            except OSError:
                break
            if not chunk:
                break
            out += chunk
    statuses = [int(p[:3]) for p in out.split(b'HTTP/1.1 ')[1:] if p[:3].isdigit()]
    assert all(s in (100, 200, 400, 404, 405, 413, 431) for s in statuses), (statuses, out[:300])
    if pieces[0] in _BAD:
        assert statuses[:1] in ([], [400], [413], [431]), (statuses, out[:300])
    with httpx.Client(base_url=f'http://127.0.0.1:{server}', timeout=5) as h:  # the server is still serving
        assert h.get('/hello').status_code == 200


def test_ws_64bit_length_with_msb_set_is_a_protocol_error(native):
    """RFC 6455 5.2: the most significant bit of a 64-bit payload length must be 0: the parser
    answers 1002 instead of reading a negative length."""
    p = native.WsParser(1 << 16)
    with pytest.raises(ValueError) as e:
        p.feed(b'\x81\xff' + b'\x80' + b'\x00' * 7 + b'\x01\x02\x03\x04')
    assert e.value.args[1] == 1002
    with pytest.raises(ValueError) as e:  # just over the limit: 1009, whatever the buffered bytes
        native.WsParser(100).feed(b'\x82\xff' + (101).to_bytes(8, 'big') + b'\x00' * 4)
    assert e.value.args[1] == 1009
