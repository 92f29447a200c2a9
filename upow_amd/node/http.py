"""The node's HTTP/1.1 + WebSocket server protocol for uvicorn (``uvicorn.run(app, http=NodeHttpProtocol)``).

reference: upow/node/run.py serves the FastAPI app with uvicorn (h11 or httptools) and its WebSocket
endpoint through the ``websockets`` library. Here:

* request framing is native (``csrc/http_wire.cpp`` ``HttpParser``): a connection's bytes go to one call
  that returns every complete request — method, target, version, lower-cased headers, de-chunked body,
  keep-alive and upgrade flags — so the event loop makes one Python call per request instead of a parser
  callback per header (h11 was about a third of the loop's CPU per ``/push_tx`` at 1,200 req/s,
  ``profiles/r3/node_soak_loop_cprofile_r3p.txt``);
* the request body is complete before the ASGI app runs (``receive()`` answers at once); responses are
  written with Content-Length or chunked framing as the app's headers ask;
* WebSocket upgrades (RFC 6455) are served in the same protocol — handshake, native frame parsing
  (``WsParser``: unmasking, size and control-frame checks), fragmentation, ping/pong, close handshake —
  bridged to the ASGI ``websocket`` scope, so the node's ``/ws`` endpoint works over a real socket
  without a WebSocket library.

Connection behaviour follows HTTP/1.1: keep-alive by default (``Connection: close`` and HTTP/1.0 honoured),
pipelined requests answered in order, ``Expect: 100-continue``, the server's keep-alive timeout, and a
graceful shutdown that lets an in-flight response finish.
"""
from __future__ import annotations

import asyncio
import base64
import hashlib
import http
import logging
import os
import struct
import urllib.parse
from collections import deque
from typing import Optional

from uvicorn.protocols.http.flow_control import FlowControl
from uvicorn.protocols.utils import get_local_addr, get_remote_addr, is_ssl

from ..ops.native import lib

_SEND_NOW = os.environ.get('UPOW_HTTP_SEND_NOW', '1') != '0'
_WS_GUID = b'258EAFA5-E914-47DA-95CA-C5AB0DC85B11'
_STATUS = {}


def _status_line(code: int) -> bytes:
    line = _STATUS.get(code)
    if line is None:
        try:
            phrase = http.HTTPStatus(code).phrase.encode()
        except ValueError:
            phrase = b''
        line = _STATUS[code] = b'HTTP/1.1 %d %s\r\n' % (code, phrase)
    return line


def _split_target(target: bytes):
    """(path str, raw path bytes, query bytes) of an origin- or absolute-form request target."""
    if target[:1] != b'/' and b'://' in target:  # absolute-form: drop scheme and authority
        rest = target.split(b'://', 1)[1]
        slash = rest.find(b'/')
        target = rest[slash:] if slash >= 0 else b'/'
    raw, _, query = target.partition(b'?')
    raw = raw.partition(b'#')[0]
    path = raw.decode('latin-1')
    if '%' in path:
        path = urllib.parse.unquote(path)
    return path, raw, query


class _Cycle:
    """One request/response exchange (the ASGI ``http`` scope's receive/send)."""

    __slots__ = ('proto', 'scope', 'body', 'keep_alive', 'body_sent', 'started', 'complete', 'disconnected',
                 'chunked', 'remaining', 'done', 'head', 'head_bytes')

    def __init__(self, proto: 'NodeHttpProtocol', scope: dict, body: bytes, keep_alive: bool):
        self.proto = proto
        self.scope = scope
        self.body = body
        self.keep_alive = keep_alive
        self.body_sent = False
        self.started = self.complete = self.disconnected = False
        self.chunked = False
        self.remaining = 0
        self.done = asyncio.Event()
        self.head = scope['method'] == 'HEAD'
        self.head_bytes = b''  # status line + headers, sent with the first body bytes (one write, one segment)

    async def run(self, app):
        try:
            await app(self.scope, self.receive, self.send)
        except BaseException as e:  # the app's own handlers answer every expected error
            self.proto.logger.error('Exception in ASGI application', exc_info=e)
            if not self.started:
                await self._plain(500, b'Internal Server Error', close=True)
            else:
                self.proto.transport.close()
        else:
            if not self.started and not self.disconnected:
                self.proto.logger.error('ASGI callable returned without starting response.')
                await self._plain(500, b'Internal Server Error', close=True)
            elif not self.complete and not self.disconnected:
                self.proto.logger.error('ASGI callable returned without completing response.')
                self.proto.transport.close()

    async def _plain(self, status: int, body: bytes, close: bool = False):
        headers = [(b'content-type', b'text/plain; charset=utf-8'), (b'content-length', b'%d' % len(body))]
        if close:
            headers.append((b'connection', b'close'))
        await self.send({'type': 'http.response.start', 'status': status, 'headers': headers})
        await self.send({'type': 'http.response.body', 'body': body})

    async def receive(self):
        if not self.body_sent:
            self.body_sent = True
            return {'type': 'http.request', 'body': self.body, 'more_body': False}
        if not (self.disconnected or self.complete):
            await self.done.wait()
        return {'type': 'http.disconnect'}

    async def send(self, message):
        p = self.proto
        if p.flow.write_paused and not self.disconnected:
            await p.flow.drain()
        if self.disconnected:
            return
        kind = message['type']
        if not self.started:
            if kind != 'http.response.start':
                raise RuntimeError(f"Expected ASGI message 'http.response.start', but got '{kind}'.")
            self.started = True
            status = message['status']
            out = [_status_line(status)]
            length = None
            for name, value in (*p.server_state.default_headers, *message.get('headers', ())):
                name = bytes(name).lower()
                value = bytes(value)
                if b'\r' in value or b'\n' in value or b'\r' in name or b'\n' in name or b':' in name:
                    raise RuntimeError('Invalid HTTP header.')
                if name == b'content-length' and length is None:
                    length = int(value)
                elif name == b'transfer-encoding' and value.lower() == b'chunked':
                    self.chunked = True
                elif name == b'connection' and value.lower() == b'close':
                    self.keep_alive = False
                out += (name, b': ', value, b'\r\n')
            if not self.keep_alive and b'connection: close' not in b''.join(out).lower():
                out.append(b'connection: close\r\n')
            if length is not None and not self.chunked:
                self.remaining = length
            elif not self.chunked and not self.head and status not in (204, 304) and status >= 200:
                self.chunked = True
                out.append(b'transfer-encoding: chunked\r\n')
            out.append(b'\r\n')
            self.head_bytes = b''.join(out)
            if p.access_log:
                p.access_logger.info('%s - "%s %s HTTP/%s" %d', self.scope['client'], self.scope['method'],
                                     self.scope['path'], self.scope['http_version'], status)
            return
        if self.complete:
            raise RuntimeError(f"Unexpected ASGI message '{kind}' sent, after response already completed.")
        if kind != 'http.response.body':
            raise RuntimeError(f"Expected ASGI message 'http.response.body', but got '{kind}'.")
        body = message.get('body', b'')
        more = message.get('more_body', False)
        out = [self.head_bytes] if self.head_bytes else []
        self.head_bytes = b''
        if self.head:
            pass
        elif self.chunked:
            if body:
                out += (b'%x\r\n' % len(body), body, b'\r\n')
            if not more:
                out.append(b'0\r\n\r\n')
        else:
            if len(body) > self.remaining:
                raise RuntimeError('Response content longer than Content-Length')
            self.remaining -= len(body)
            if body:
                out.append(body)
        if out:
            p.write(out[0] if len(out) == 1 else b''.join(out))
        if not more:
            if not self.head and not self.chunked and self.remaining:
                raise RuntimeError('Response content shorter than Content-Length')
            self.complete = True
            self.done.set()
            if not self.keep_alive:
                p.transport.close()
            p.response_complete(self)


class _WebSocket:
    """One upgraded connection: RFC 6455 framing under the ASGI ``websocket`` scope."""

    def __init__(self, proto: 'NodeHttpProtocol', scope: dict, key: bytes, leftover: bytes):
        self.proto = proto
        self.scope = scope
        self.key = key
        self.parser = lib().WsParser()
        self.inbox: asyncio.Queue = asyncio.Queue()
        self.accepted = self.closed_sent = self.closed = False
        self.frag_op = 0
        self.frag: list = []
        self.inbox.put_nowait({'type': 'websocket.connect'})
        self.pending = leftover

    async def run(self, app):
        if self.pending:
            data, self.pending = self.pending, b''
            self.feed(data)
        try:
            await app(self.scope, self.receive, self.send)
        except BaseException as e:
            self.proto.logger.error('Exception in ASGI application', exc_info=e)
            if not self.accepted:
                self._http_reject(500)
            else:
                self._close(1011, '')
            return
        if not self.accepted:
            self._http_reject(403)
        elif not self.closed_sent:
            self._close(1000, '')
        if not self.closed:  # the peer's close frame ends it; a silent peer is dropped after a second
            self.proto.loop.call_later(1.0, self._gone, 1006)

    # -- from the socket
    def feed(self, data: bytes):
        if self.closed:
            return
        try:
            frames = self.parser.feed(data)
        except ValueError as e:
            code = e.args[1] if len(e.args) > 1 else 1002
            self._close(int(code), '')
            self._gone(int(code))
            return
        for fin, op, payload in frames:
            if op == 9:  # ping -> pong
                self._frame(10, payload)
            elif op == 10:
                pass
            elif op == 8:
                code = struct.unpack('!H', payload[:2])[0] if len(payload) >= 2 else 1005
                if not self.closed_sent:
                    self._close(code if code not in (1005, 1006) else 1000, '')
                self._gone(code)
                return
            elif op == 0:  # continuation
                if not self.frag_op:
                    self._close(1002, '')
                    self._gone(1002)
                    return
                self.frag.append(payload)
                if fin:
                    self._deliver(self.frag_op, b''.join(self.frag))
                    self.frag_op, self.frag = 0, []
            else:
                if self.frag_op:
                    self._close(1002, '')
                    self._gone(1002)
                    return
                if fin:
                    self._deliver(op, payload)
                else:
                    self.frag_op, self.frag = op, [payload]

    def _deliver(self, op: int, payload: bytes):
        if op == 1:
            try:
                text = payload.decode('utf-8')
            except UnicodeDecodeError:
                self._close(1007, '')
                self._gone(1007)
                return
            self.inbox.put_nowait({'type': 'websocket.receive', 'text': text})
        else:
            self.inbox.put_nowait({'type': 'websocket.receive', 'bytes': payload})

    def _gone(self, code: int):
        if not self.closed:
            self.closed = True
            self.inbox.put_nowait({'type': 'websocket.disconnect', 'code': code})
            if not self.proto.transport.is_closing():
                self.proto.transport.close()

    def lost(self):
        self._gone(1006)

    # -- ASGI
    async def receive(self):
        return await self.inbox.get()

    async def send(self, message):
        kind = message['type']
        t = self.proto.transport
        if kind == 'websocket.accept':
            if self.accepted or self.closed:
                return
            self.accepted = True
            accept = base64.b64encode(hashlib.sha1(self.key + _WS_GUID).digest())
            out = [b'HTTP/1.1 101 Switching Protocols\r\nupgrade: websocket\r\nconnection: upgrade\r\n',
                   b'sec-websocket-accept: ', accept, b'\r\n']
            if message.get('subprotocol'):
                out += (b'sec-websocket-protocol: ', message['subprotocol'].encode(), b'\r\n')
            for name, value in message.get('headers', ()):
                out += (bytes(name).lower(), b': ', bytes(value), b'\r\n')
            out.append(b'\r\n')
            t.write(b''.join(out))
        elif kind == 'websocket.send':
            if not self.accepted:
                raise RuntimeError('websocket.send before websocket.accept')
            if self.closed or self.closed_sent:
                return
            if message.get('text') is not None:
                self._frame(1, message['text'].encode('utf-8'))
            else:
                self._frame(2, bytes(message.get('bytes') or b''))
            if self.proto.flow.write_paused:
                await self.proto.flow.drain()
        elif kind == 'websocket.close':
            if not self.accepted:
                self._http_reject(403)
                self._gone(1006)
                return
            self._close(int(message.get('code', 1000)), message.get('reason') or '')
            self._gone(int(message.get('code', 1000)))
        elif kind == 'websocket.http.response.start' and not self.accepted:
            self._http_reject(int(message['status']))

    def _frame(self, op: int, payload: bytes):
        n = len(payload)
        if n < 126:
            head = bytes((0x80 | op, n))
        elif n < 65536:
            head = struct.pack('!BBH', 0x80 | op, 126, n)
        else:
            head = struct.pack('!BBQ', 0x80 | op, 127, n)
        if not self.proto.transport.is_closing():
            self.proto.transport.write(head + payload)

    def _close(self, code: int, reason: str):
        if self.closed_sent:
            return
        self.closed_sent = True
        self._frame(8, struct.pack('!H', code) + reason.encode('utf-8')[:123])

    def _http_reject(self, status: int):
        t = self.proto.transport
        if not t.is_closing():
            t.write(_status_line(status) + b'content-length: 0\r\nconnection: close\r\n\r\n')
            t.close()


class NodeHttpProtocol(asyncio.Protocol):
    """uvicorn server protocol (``http=`` class): HTTP/1.1 on the native framer, WebSocket upgrades served
    in place. Constructor signature and server hooks (``connections``, ``tasks``, ``shutdown``) are the
    ones uvicorn's server drives its protocols with."""

    def __init__(self, config, server_state, app_state: dict, _loop: Optional[asyncio.AbstractEventLoop] = None):
        if not config.loaded:
            config.load()
        self.config = config
        self.app = config.loaded_app
        self.loop = _loop or asyncio.get_event_loop()
        self.logger = logging.getLogger('uvicorn.error')
        self.access_logger = logging.getLogger('uvicorn.access')
        self.access_log = self.access_logger.hasHandlers()
        self.root_path = config.root_path
        self.server_state = server_state
        self.connections = server_state.connections
        self.tasks = server_state.tasks
        self.app_state = app_state
        self.keep_alive_s = config.timeout_keep_alive
        self.parser = lib().HttpParser()
        self.transport = None
        self.flow = None
        self.cycle: Optional[_Cycle] = None
        self.queue: deque = deque()  # pipelined requests waiting for the current response
        self.ws: Optional[_WebSocket] = None
        self.ka_timer = None
        self.fd = -1

    # -- asyncio.Protocol
    partial_sends = 0  # direct sends the transport had to finish (tests)

    def connection_made(self, transport):
        self.connections.add(self)
        self.transport = transport
        self.flow = FlowControl(transport)
        self.server = get_local_addr(transport)
        self.client = get_remote_addr(transport)
        self.scheme = 'https' if is_ssl(transport) else 'http'
        sock = transport.get_extra_info('socket')
        self.fd = sock.fileno() if sock is not None and self.scheme == 'http' and _SEND_NOW else -1

    def write(self, data: bytes) -> None:
        """A response's bytes: sent at once from the loop thread without releasing the GIL while the
        transport has nothing queued (``send_now``), the rest (a full socket buffer, an error to report)
        through the transport, which keeps the order and the flow control."""
        t = self.transport
        if self.fd >= 0 and not t.get_write_buffer_size() and not t.is_closing():
            n = lib().send_now(self.fd, data)
            if n == len(data):
                return
            NodeHttpProtocol.partial_sends += 1
            if n > 0:
                data = memoryview(data)[n:]
        t.write(data)

    def connection_lost(self, exc):
        self.connections.discard(self)
        self._cancel_keep_alive()
        if self.cycle is not None:
            if not self.cycle.complete:
                self.cycle.disconnected = True
            self.cycle.done.set()
        for c in self.queue:
            c.disconnected = True
            c.done.set()
        if self.ws is not None:
            self.ws.lost()
        if self.flow is not None:
            self.flow.resume_writing()

    def eof_received(self):
        pass

    def pause_writing(self):
        self.flow.pause_writing()

    def resume_writing(self):
        self.flow.resume_writing()

    def data_received(self, data: bytes):
        self._cancel_keep_alive()
        if self.ws is not None:
            self.ws.feed(data)
            return
        try:
            reqs = self.parser.feed(data)
        except ValueError as e:
            self.logger.warning(f'Invalid HTTP request received: {e}')
            self._bad_request(str(e))
            return
        if self.parser.need_continue() and (self.cycle is None or self.cycle.complete):
            self.transport.write(b'HTTP/1.1 100 Continue\r\n\r\n')
            self.parser.ack_continue()
        for r in reqs:
            self._request(r)

    # -- requests
    def _scope(self, method: str, target: bytes, version: str, headers: list) -> dict:
        path, raw, query = _split_target(target)
        return {'type': 'http', 'asgi': {'version': self.config.asgi_version, 'spec_version': '2.3'},
                'http_version': version, 'server': self.server, 'client': self.client, 'scheme': self.scheme,
                'method': method, 'root_path': self.root_path, 'path': self.root_path + path,
                'raw_path': self.root_path.encode('ascii') + raw, 'query_string': query, 'headers': headers,
                'state': self.app_state.copy()}

    def _request(self, r):
        method, target, version, headers, body, keep_alive, upgrade, proto = r
        scope = self._scope(method, target, version, headers)
        if upgrade and proto == 'websocket' and method == 'GET' and self.cycle is None and not self.queue:
            key = next((v for k, v in headers if k == b'sec-websocket-key'), None)
            version_ok = any(k == b'sec-websocket-version' and v.strip() == b'13' for k, v in headers)
            if key and version_ok:
                self._websocket(scope, key, self.parser.rest())
                return
        if upgrade:  # an upgrade we do not serve: answer it as plain HTTP on a closing connection
            keep_alive = False
        cycle = _Cycle(self, scope, body, keep_alive)
        if self.cycle is None or self.cycle.complete:
            self._start(cycle)
        else:
            self.queue.append(cycle)
            self.flow.pause_reading()

    def _start(self, cycle: _Cycle):
        self.cycle = cycle
        task = self.loop.create_task(cycle.run(self.app))
        task.add_done_callback(self.tasks.discard)
        self.tasks.add(task)

    def response_complete(self, cycle: _Cycle):
        self.server_state.total_requests += 1
        if self.transport.is_closing():
            return
        self.flow.resume_reading()
        if self.queue:
            self._start(self.queue.popleft())
        else:
            if self.parser.need_continue():
                self.transport.write(b'HTTP/1.1 100 Continue\r\n\r\n')
                self.parser.ack_continue()
            self.ka_timer = self.loop.call_later(self.keep_alive_s, self._keep_alive_expired)

    def _websocket(self, scope: dict, key: bytes, leftover: bytes):
        scope = dict(scope, type='websocket', scheme='wss' if self.scheme == 'https' else 'ws')
        scope.pop('method', None)
        protos = next((v for k, v in scope['headers'] if k == b'sec-websocket-protocol'), b'')
        scope['subprotocols'] = [p.strip().decode('latin-1') for p in protos.split(b',') if p.strip()]
        self.connections.discard(self)  # a long-lived socket: not an HTTP connection for shutdown purposes
        self.ws = _WebSocket(self, scope, key, leftover)
        task = self.loop.create_task(self.ws.run(self.app))
        task.add_done_callback(self.tasks.discard)
        self.tasks.add(task)

    def _bad_request(self, msg: str):
        body = msg.encode('ascii', 'replace')
        self.transport.write(_status_line(400) + b'content-type: text/plain; charset=utf-8\r\ncontent-length: %d\r\n'
                             b'connection: close\r\n\r\n%s' % (len(body), body))
        self.transport.close()

    # -- server hooks
    def _cancel_keep_alive(self):
        if self.ka_timer is not None:
            self.ka_timer.cancel()
            self.ka_timer = None

    def _keep_alive_expired(self):
        if not self.transport.is_closing():
            self.transport.close()

    def shutdown(self):
        """Graceful shutdown: an idle connection closes now, a busy one after its response."""
        if self.ws is not None:
            self.ws._close(1012, '')
            self.transport.close()
        elif self.cycle is None or self.cycle.complete:
            self.transport.close()
        else:
            self.cycle.keep_alive = False


__all__ = ['NodeHttpProtocol']
