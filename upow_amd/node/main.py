"""uPow full-node HTTP service (reference: upow/node/main.py:55-1102).

Same routes, parameters, rate limits, response envelopes, middleware behaviour (IP filter, path
normalisation, Sender-Node peer learning, localhost-only /send_to_address, peer bootstrap,
re-propagation of stale mempool txs), gossip fan-out, chain sync with fork rollback and the /ws
WebSocket. The ledger is the embedded store + HBM UTXO index (:mod:`upow_amd.ledger.database`) and
block validation runs the batched GPU pipeline (:mod:`upow_amd.ledger.validate`).

Run: ``python -m upow_amd.node --host 0.0.0.0 --port 3006`` (uvicorn).
"""
from __future__ import annotations

import asyncio

import json
import os
import random
import re
import sys
import time
from asyncio import gather
from collections import OrderedDict, defaultdict, deque
from contextlib import asynccontextmanager
from functools import lru_cache
from decimal import Decimal
from typing import Annotated, Optional, Union
from urllib.parse import urlsplit

import numpy as np
from fastapi import Body, FastAPI, Header, Query
from fastapi.encoders import jsonable_encoder
from fastapi.exceptions import RequestValidationError
from fastapi.responses import PlainTextResponse, RedirectResponse
from starlette.background import BackgroundTasks
from starlette.middleware.cors import CORSMiddleware
from starlette.requests import Request
from starlette.responses import JSONResponse, Response

from .. import config
from ..constants import ENDIAN, GENESIS_PREV_HASH, MAX_SUPPLY, VERSION
from ..ledger import manager as mgr
from ..ledger.database import Database, UniqueViolationError
from ..ledger import fastpath, pagesync
from ..ledger.fastpath import create_block_from_hex
from ..ledger import worker as ledger_worker
from ..ledger.worker import on_ledger
from ..ops.native import lib
from ..utils import coalesce
from ..parallel import cluster
from ..ledger.manager import (Manager, block_to_bytes, calculate_difficulty, clear_pending_transactions, create_block,
                              ledger_lock,
                              create_block_in_syncing_old, get_circulating_supply, get_difficulty,
                              get_inodes_from_cache, get_transactions_merkle_tree, split_block_content)
from ..models.transaction import CoinbaseTransaction, Transaction
from ..utils import codec, hexspans
from ..utils.codec import sha256, timestamp
from ..utils.hexspans import HexSpans
from ..utils.logger import get_logger
from ..websocket.endpoint import (broadcast_new_block, broadcast_new_transaction, router as websocket_router,
                                  shutdown_websocket_manager, start_websocket_manager, transaction_listeners)
from .access import AccessControl
from . import peers
from .peers import PeerClient
from .ratelimit import Limiter, RateLimitExceeded, get_remote_address, rate_limit_exceeded_handler
from .utils import ip_is_local

logger = get_logger(__name__)
limiter = Limiter(key_func=get_remote_address, enabled=os.environ.get('UPOW_RATE_LIMIT', '1') == '1')

db: Database = None
started = False
is_syncing = False
self_url = None
access: AccessControl = None
transactions_cache = deque(maxlen=100)
LAST_PENDING_TRANSACTIONS_CLEAN = [0]
BANNED_SENDERS = ['DgQKikeDqS2Fzue23KuA36L4eJSFh649zA9jJ6zwbzUMp']  # main.py:426


@asynccontextmanager
async def lifespan(app: FastAPI):
    await startup()
    indexer = asyncio.create_task(_address_indexer())
    lag = asyncio.create_task(_loop_lag_monitor()) if os.environ.get('UPOW_TRACE_FILE') else None
    try:
        yield
    finally:
        indexer.cancel()
        if lag is not None:
            lag.cancel()
        if cluster.get() is not None:
            await on_ledger(cluster.leader_quit)  # the collective owner tells the replicas to stop
        ledger_worker.stop()
        peers.book().flush()
        await shutdown_websocket_manager()
        if db is not None and db.path != ':memory:' and os.environ.get('UPOW_SNAPSHOT', '1') != '0':
            try:  # checkpoint the UTXO index so the next start skips the SQL rebuild (ledger/snapshot.py)
                from ..ledger import snapshot
                snapshot.save(db)
            except Exception as e:
                logger.error(f'UTXO snapshot on shutdown failed: {e}')


async def _loop_lag_monitor(tick: float = 0.001, report_ms: float = 2.0):
    """With ``UPOW_TRACE_FILE``: how late the HTTP event loop runs a 1 ms timer, one JSON line per stall
    over ``report_ms`` (``<trace>.lag``: wall time at the end of the stall and its length), so a soak can
    tell which stalls overlap block application and which do not."""
    import threading
    import time as _time
    import traceback
    path = os.environ['UPOW_TRACE_FILE'] + '.lag'
    loop = asyncio.get_running_loop()
    beat = [_time.perf_counter()]
    loop_tid = threading.get_ident()
    stop = threading.Event()

    def watchdog():
        # while the loop is stalled past 5 ms, sample what the loop thread is executing (innermost
        # frames) every 2 ms: the .stacks file names the code that holds the event loop
        with open(os.environ['UPOW_TRACE_FILE'] + '.stacks', 'a') as out:
            while not stop.wait(0.002):
                if _time.perf_counter() - beat[0] > 0.005:
                    frames = sys._current_frames()
                    fr = frames.get(loop_tid)
                    if fr is not None:
                        st = traceback.extract_stack(fr)[-6:]
                        # the other Python threads' innermost frames at the same instant: a loop thread
                        # parked in an I/O call is usually waiting for the GIL that one of these holds
                        names = {t.ident: t.name for t in threading.enumerate()}
                        others = {}
                        for tid, f in frames.items():
                            if tid in (loop_tid, threading.get_ident()):
                                continue
                            others[names.get(tid, str(tid))] = \
                                f'{os.path.basename(f.f_code.co_filename)}:{f.f_lineno}:{f.f_code.co_name}'
                        out.write(json.dumps({'t': round(_time.time(), 4),
                                              'stack': [f'{os.path.basename(x.filename)}:{x.lineno}:{x.name}' for x in st],
                                              'others': others}) + '\n')
    threading.Thread(target=watchdog, name='upow-loop-watchdog', daemon=True).start()
    # the native probe (csrc/stall_probe.cpp) samples every thread's kernel state while the loop is late,
    # GIL or no GIL; <trace>.threads maps its tids to Python thread names
    import numpy as np
    hb = np.array([_time.perf_counter()])
    probe = None
    try:
        from ..ops.native import lib
        probe = lib().StallProbe(os.environ['UPOW_TRACE_FILE'] + '.native', hb, threading.get_native_id(), 10.0, 2000)
    except (ImportError, AttributeError) as e:
        logger.warning(f'native stall probe unavailable: {e}')

    def dump_thread_names():
        with open(os.environ['UPOW_TRACE_FILE'] + '.threads', 'w') as tf:
            json.dump({'_loop': threading.get_native_id(),
                       **{str(t.native_id): t.name for t in threading.enumerate() if t.native_id}}, tf)
    import gc
    gc_t0 = {}
    gc_out = open(os.environ['UPOW_TRACE_FILE'] + '.gc', 'a')

    def on_gc(phase, info):  # collections over 2 ms (they hold the GIL on whichever thread allocated)
        if phase == 'start':
            gc_t0['t'] = _time.perf_counter()
        elif 't' in gc_t0:
            ms = (_time.perf_counter() - gc_t0.pop('t')) * 1000.0
            if ms > 2.0:
                gc_out.write(json.dumps({'t': round(_time.time(), 4), 'gen': info.get('generation'),
                                         'ms': round(ms, 2)}) + '\n')
                gc_out.flush()
    gc.callbacks.append(on_gc)
    try:
        with open(path, 'a') as f:
            n = 0
            while True:
                t0 = loop.time()
                beat[0] = hb[0] = _time.perf_counter()
                await asyncio.sleep(tick)
                beat[0] = hb[0] = _time.perf_counter()
                n += 1
                if n % 2000 == 1:
                    dump_thread_names()
                late = (loop.time() - t0 - tick) * 1000.0
                if late > report_ms:
                    f.write(json.dumps({'t': round(_time.time(), 4), 'ms': round(late, 2)}) + '\n')
                    f.flush()
    finally:
        stop.set()
        gc.callbacks.remove(on_gc)
        if probe is not None:
            probe.stop()
        gc_out.close()


async def _address_indexer(period: float = 30.0):
    """Keep the lazily built per-address tx index near the tip (queries also catch it up on demand)."""
    while True:
        await asyncio.sleep(period)
        try:
            if db is not None:
                await db.asettle()  # block batches keep the index current; this only catches up a lag
                db.index_addresses()
        except Exception as e:
            logger.error(f'address indexer: {e}')


async def startup():
    """main.py:246-257: open the ledger (UPOW_DATABASE_PATH, default <data dir>/ledger.sqlite3)."""
    global db, access
    peers.book()
    access = AccessControl()
    path = os.environ.get('UPOW_DATABASE_PATH') or config.data_path('ledger.sqlite3')
    db = await Database.create(path=path)
    # block validation/apply and every cluster collective run on the ledger thread
    ledger_worker.start()
    from ..ledger import lean
    if lean.pending(db):  # a lean follower's ledger opened as this node's (promotion): its op log into SQL first
        await on_ledger(lean.materialise, db)
    if cluster.get() is not None:  # multi-GPU node: the replicas get only what they lack (parallel/cluster.py)
        await on_ledger(cluster.leader_start, db)
    # what exists now (ledger caches, indexes, modules) lives for the process: keep it out of the
    # cyclic collector's full passes, which run on whichever thread allocates and hold the GIL
    import gc
    gc.collect()
    gc.freeze()
    await start_websocket_manager()


app = FastAPI(lifespan=lifespan)
app.state.limiter = limiter
app.add_exception_handler(RateLimitExceeded, rate_limit_exceeded_handler)
app.add_middleware(CORSMiddleware, allow_origins=['*'], allow_methods=['GET', 'POST'], allow_headers=['*'])
app.include_router(websocket_router)


# ---------------------------------------------------------------------------------------------- gossip
async def propagate(path: str, args: dict, ignore_url=None, nodes: list = None):
    """main.py:79-94: fan out to <=10 recent + <=10 never-heard-from peers."""
    self_node = PeerClient(self_url or '')
    ignore_node = PeerClient(ignore_url or '')
    aws = []
    for node_url in nodes or peers.book().gossip_urls():
        ni = PeerClient(node_url)
        if ni.host == self_node.host or ni.host == ignore_node.host:
            continue
        aws.append(ni.call(path, args, self_node.url))
    await gather(*aws, return_exceptions=True)


# ---------------------------------------------------------------------------------------------- sync
def _scan_sync_block(hexes: list):
    """Host-thread half of a sync step (no ledger state involved): find the coinbase candidate
    (txcodec flag 3 = specifier 36) and decode the remaining txs for the native block path."""
    flags = fastpath.decode_raw(hexes, fastpath.THREADS)['flags'] if hexes else b''
    k = next((i for i, f in enumerate(flags) if f == 3), None)
    rest = hexes if k is None else hexes[:k] + hexes[k + 1:]
    return k, (fastpath.decode(rest) if rest else None)


_SYNC_DECODER = None


def _sync_decoder():
    global _SYNC_DECODER
    if _SYNC_DECODER is None:
        from concurrent.futures import ThreadPoolExecutor
        _SYNC_DECODER = ThreadPoolExecutor(max_workers=1, thread_name_prefix='upow-sync-decode')
    return _SYNC_DECODER


async def create_blocks(blocks: list, error_list=None) -> bool:
    """main.py:97-150 for a /get_blocks page: page-batched (ledger/pagesync.py: one UTXO lookup and one
    signature batch per chunk of blocks, deferred index writes, one fdatasync per page), or per block with
    ``UPOW_PAGE_SYNC=0``."""
    if pagesync.ENABLED:
        return await pagesync.create_blocks(blocks, error_list)
    return await create_blocks_per_block(blocks, error_list)


async def create_blocks_per_block(blocks: list, error_list=None) -> bool:
    """main.py:97-150, as a two-stage pipeline: while block k is validated and applied on the event
    loop (GPU passes + ledger writes, GIL released in the native parts), block k+1 is already being
    decoded on a host thread (``_scan_sync_block``: txids, canonical bytes, addresses, merkle)."""
    if error_list is None:
        error_list = []
    _, last_block = await calculate_difficulty()
    last_block['id'] = last_block['id'] if last_block != {} else 0
    last_block['hash'] = last_block['hash'] if 'hash' in last_block else GENESIS_PREV_HASH
    i = last_block['id'] + 1
    loop = asyncio.get_running_loop()
    pool = _sync_decoder()
    hexes_of = [b['transactions'][:] for b in blocks]  # a list, or a HexSpans read from the page body
    ahead = loop.run_in_executor(pool, _scan_sync_block, hexes_of[0]) if blocks else None
    for n, block_info in enumerate(blocks):
        block = block_info['block']
        hexes = hexes_of[n]
        cb_k, dec = await ahead
        ahead = loop.run_in_executor(pool, _scan_sync_block, hexes_of[n + 1]) if n + 1 < len(blocks) else None
        # the first coinbase among the txs is the trusted one (main.py:112-117); the rest go through
        # the native block path (ledger/fastpath.py) in sync mode
        cb_tx = None
        if cb_k is not None:
            cand = await Transaction.from_hex(hexes[cb_k])
            if isinstance(cand, CoinbaseTransaction):
                cb_tx = cand
                hexes = hexes[:cb_k] + hexes[cb_k + 1:]
            else:
                dec = None  # not what the scan assumed: decode inline below
        if cb_tx is None:
            # the reference's sync dereferences the coinbase (manager.py:790): a block without one ends the
            # sync; it never takes the push variant (which would mint its own coinbase)
            if ahead is not None:
                await ahead
            error_list.append(error := f'block {block["id"]} has no coinbase transaction')
            logger.error(error)
            return False
        block_content = block.get('content')
        if not block_content:
            txs = [await Transaction.from_hex(h) for h in hexes]
            block['merkle_tree'] = get_transactions_merkle_tree([tx.hex() for tx in txs])
            block_content = block_to_bytes(last_block['hash'], block)
        assert i == block['id']
        if not await create_block_from_hex(block_content.hex() if isinstance(block_content, bytes) else block_content,
                                           hexes, error_list=error_list, last_block=last_block, coinbase=cb_tx,
                                           decoded=dec):
            if ahead is not None:
                await ahead
            return False
        last_block = block
        i += 1
    return True


async def _locked(fn, *args):
    """``fn(*args)`` under the ledger lock (called on the ledger thread, where the lock lives)."""
    async with ledger_lock():
        return await fn(*args)


async def _on_ledger_sync(fn, *args):
    """A synchronous cluster call made from the ledger thread: every collective of a multi-GPU node is
    issued by that one thread, so ranks see them in one order."""
    async def call():
        return fn(*args)
    return await on_ledger(call)


async def _sync_blockchain(node_url: str = None):
    """main.py:153-227: pull pages of 1000 blocks; on a fork (height > 500) roll back to the last
    common block among the last 500 and re-apply; on failure restore the cached local chain."""
    logger.info('sync blockchain')
    error = []
    if not node_url:
        nodes = peers.book().recent_urls()
        if not nodes:
            logger.error(msg := 'No nodes found.')
            return msg
        node_url = random.choice(nodes)
    node_url = node_url.strip('/')
    _, last_block = await calculate_difficulty()
    starting_from = i = await db.get_next_block_id()
    node_interface = PeerClient(node_url)
    local_cache = None
    last_common_block = None
    if last_block != {} and last_block['id'] > 500:
        remote_last_block = (await node_interface.block(i - 1))['block']
        if remote_last_block['hash'] != last_block['hash']:
            offset, limit = i - 500, 500
            remote_blocks = await node_interface.blocks(offset, limit)
            local_blocks = await db.get_blocks(offset, limit)
            local_blocks = local_blocks[:len(remote_blocks)]
            local_blocks.reverse()
            remote_blocks.reverse()
            for n, local_block in enumerate(local_blocks):
                if local_block['block']['hash'] == remote_blocks[n]['block']['hash']:
                    last_common_block = local_block['block']['id']
                    local_cache = local_blocks[:n]
                    local_cache.reverse()
                    await on_ledger(_locked, cluster.mirror_rollback, db, last_common_block + 1)
                    break
    limit = 1000
    prefetch = None  # (offset, task): the next page, fetched over HTTP while this one is applied

    def drop_prefetch():
        nonlocal prefetch
        if prefetch is not None:
            prefetch[1].cancel()
            prefetch[1].add_done_callback(lambda t: t.cancelled() or t.exception())
            prefetch = None

    while True:
        i = await db.get_next_block_id()
        try:
            if prefetch is not None and prefetch[0] == i:
                task = prefetch[1]
                prefetch = None
                blocks = await task
            else:
                drop_prefetch()
                blocks = await node_interface.blocks(i, limit)
        except Exception as e:
            logger.error(e)
            peers.book().flush()
            break
        try:
            _, last_block = await calculate_difficulty()
            if not blocks:
                logger.info('syncing complete')
                if last_block['id'] > starting_from:
                    peers.book().seen(node_url)
                    if timestamp() - last_block['timestamp'] < 86400:
                        txs_hashes = await db.get_block_transaction_hashes(last_block['hash'])
                        await propagate('push_block', {'block_content': last_block['content'], 'txs': txs_hashes,
                                                       'block_no': last_block['id']}, node_url)
                return True
            nxt = i + len(blocks)
            prefetch = (nxt, asyncio.ensure_future(node_interface.blocks(nxt, limit)))
            assert await on_ledger(create_blocks, blocks, error_list=error)
        except Exception as e:
            drop_prefetch()
            logger.error(error[0] if error else e)
            if local_cache is not None:
                logger.info('sync failed, reverting back to previous chain')
                await on_ledger(_locked, cluster.mirror_delete, db, last_common_block)
                await on_ledger(create_blocks, local_cache)
            return error[0] if error else e


async def sync_blockchain(node_url: str = None):
    global is_syncing
    sync_status = None
    try:
        is_syncing = True
        codec.is_blockchain_syncing = True
        sync_status = await _sync_blockchain(node_url)
    except Exception as e:
        logger.error(f'sync_blockchain error: {e}')
    finally:
        is_syncing = False
        codec.is_blockchain_syncing = False
    return sync_status


# ---------------------------------------------------------------------------------------------- middleware
async def propagate_old_transactions(propagate_txs):
    await db.update_pending_transactions_propagation_time([sha256(tx_hex) for tx_hex in propagate_txs])
    for tx_hex in propagate_txs:
        await propagate('push_tx', {'tx_hex': tx_hex})


_SLASH_RUNS = re.compile('/+')


def client_address(request: Request):
    """Visitor address: first X-Forwarded-For hop, else X-Real-IP (both set by the NGINX front end the
    reference documents, NGINX.md:46-58), else the socket peer."""
    return _scope_client(request.scope)


def _scope_client(scope) -> Optional[str]:
    forwarded = real = None
    for k, v in scope['headers']:
        if k == b'x-forwarded-for':
            forwarded = forwarded or v
        elif k == b'x-real-ip':
            real = real or v
    if forwarded:
        return forwarded.decode('latin-1').split(',')[0].strip()
    if real:
        return real.decode('latin-1')
    client = scope.get('client')
    return client[0] if client else None


@lru_cache(maxsize=1024)
def _host_is_local(host_header: Optional[bytes], server_host: Optional[str]) -> bool:
    """Whether the request's host (``request.base_url.hostname``: the Host header without port and
    brackets, else the server address) is localhost or a private address. Cached per header value: the
    ``ipaddress`` parse and network scan would otherwise run on every request."""
    host = urlsplit('//' + host_header.decode('latin-1')).hostname if host_header else server_host
    return host == 'localhost' or (host is not None and ip_is_local(host))


def _scope_host_is_local(scope) -> bool:
    for k, v in scope['headers']:
        if k == b'host':
            return _host_is_local(v, None)
    server = scope.get('server')
    return _host_is_local(None, server[0] if server else None)


def _deny(text: str) -> JSONResponse:
    return JSONResponse(status_code=403, content={'ok': False, 'error': text})


async def _join_network(request: Request, local: bool) -> None:
    """First non-local request (reference main.py:327-361): pull the first known peer's peer list,
    learn our public URL from the request, and announce it to our peers and theirs. Best effort."""
    global started, self_url
    known = peers.book().recent_urls()
    if not known:
        return
    seed = known[0]
    try:
        listing = await peers.fetch_json(f'{seed}/get_nodes')
        known.extend(listing['result'])
        if local:
            return
        started = True
        self_url = str(request.base_url).strip('/')
        await propagate('add_node', {'url': self_url})
        await propagate('add_node', {'url': self_url}, nodes=await PeerClient(seed).peers())
    except Exception:
        pass


# requests that must not wait for the SQL materialiser: admission reads the mempool/UTXO indexes
# (ledger/mempool.py) and block pushes run on the ledger thread, which waits where it reads
_ADMISSION_BATCH = os.environ.get('UPOW_ADMISSION_BATCH', '1') != '0'
_NO_SETTLE = frozenset(('/push_tx', '/push_block'))
_STALE_CHECK_AT = [0.0]


class Gatekeeper:
    """Per-request gates, in order: access policy on the client address, path canonicalisation
    (redirect), blocked paths, Sender-Node peer learning, localhost-only /send_to_address, network
    join on the first request, and re-propagation of mempool txs that were not gossiped for 10 min
    (after the response is sent). reference: the ``@app.middleware("http")`` of upow/node/main.py:327-390.

    A plain ASGI middleware (starlette's BaseHTTPMiddleware runs the endpoint in a task of its own and
    re-streams the response through memory channels: ~0.3 ms per request at /push_tx rates). Before an
    endpoint that reads SQL, it awaits the journal materialiser on an executor thread
    (``Database.asettle``), so one request reading right after a block never blocks the event loop,
    and with it every /push_tx in flight."""

    def __init__(self, app):
        self.app = app

    async def __call__(self, scope, receive, send):
        if scope['type'] != 'http':
            await self.app(scope, receive, send)
            return
        request = Request(scope)
        policy = access.policy()
        if not policy.admits(_scope_client(scope)):
            await _deny('Access forbidden.')(scope, receive, send)
            return
        raw_path = scope['path']
        path = _SLASH_RUNS.sub('/', raw_path)
        if path != raw_path:
            await RedirectResponse(str(request.url).replace(raw_path, path))(scope, receive, send)
            return
        if policy.path_blocked(path):
            await _deny('Access forbidden temporarily.')(scope, receive, send)
            return
        sender = request.headers.get('Sender-Node')
        if sender:
            peers.book().add(sender)
        local = _scope_host_is_local(scope)
        if path == '/send_to_address' and not local:
            await _deny('Access forbidden. This endpoint can only be accessed from localhost.')(scope, receive, send)
            return
        if not started and path != '/get_nodes':
            await _join_network(request, local)
        # the reference asks on every request; an answer is only possible for txs not gossiped for
        # 10 min, so asking at most once a second changes nothing but the per-request cost
        stale = None
        now = time.monotonic()
        if now >= _STALE_CHECK_AT[0]:
            _STALE_CHECK_AT[0] = now + 1.0
            stale = await db.get_need_propagate_transactions()
        if path not in _NO_SETTLE:
            await db.asettle()

        async def send_cors(message):
            if message['type'] == 'http.response.start':
                headers = [(k, v) for k, v in message.get('headers', ()) if k.lower() != b'access-control-allow-origin']
                headers.append((b'access-control-allow-origin', b'*'))
                message = dict(message, headers=headers)
            await send(message)
        if path == '/push_tx' and scope['method'] == 'POST' and not scope.get('query_string') and _PUSH_FAST:
            receive = await _push_tx_direct(request, scope, receive, send_cors)
            if receive is None:
                if stale:
                    await propagate_old_transactions(stale)
                return
        await self.app(scope, receive, send_cors)
        if stale:
            await propagate_old_transactions(stale)


_PUSH_FAST = os.environ.get('UPOW_PUSH_FAST', '1') != '0'


async def _push_tx_direct(request: Request, scope, receive, send):
    """``POST /push_tx`` with a JSON body ``{"tx_hex": ...}`` — the only hot endpoint — answered without
    the framework's routing, dependency solving and body re-validation (about a quarter of a request's
    CPU at admission rates). Same handler (:func:`verify_and_push_tx`), same responses, same error
    envelope (:func:`exception_handler`), background tasks after the response. Anything else (other
    content types, malformed JSON, extra fields) returns a ``receive`` that replays the body, and the
    request takes the normal route. Returns None when the request was answered."""
    chunks = []
    more = True
    while more:
        msg = await receive()
        if msg['type'] != 'http.request':
            break
        chunks.append(msg.get('body', b''))
        more = msg.get('more_body', False)
    body = b''.join(chunks)
    ctype = request.headers.get('content-type', '')
    parsed = None
    if 'json' in ctype:
        try:
            parsed = json.loads(body)
        except ValueError:
            parsed = None
    if not (isinstance(parsed, dict) and len(parsed) == 1 and isinstance(parsed.get('tx_hex'), str)):
        replayed = False

        async def replay():
            nonlocal replayed
            if not replayed:
                replayed = True
                return {'type': 'http.request', 'body': body, 'more_body': False}
            return await receive()
        return replay
    tasks = BackgroundTasks()
    try:
        if is_syncing:
            logger.warning(error := 'Node is already syncing')
            result = {'ok': False, 'error': error}
        else:
            tx = await Transaction.from_hex(parsed['tx_hex'])
            result = await verify_and_push_tx(tx, request, tasks)
    except Exception as e:  # noqa: BLE001 - the app-wide handler's envelope
        result = await exception_handler(request, e)
    response = result if isinstance(result, Response) else JSONResponse(result)
    await response(scope, receive, send)
    await tasks()
    return None


app.add_middleware(Gatekeeper)


@app.exception_handler(Exception)
async def exception_handler(request: Request, e: Exception):
    """main.py:393-405."""
    logger.error(f"Error on {request.scope['path']}, {type(e).__name__}: {str(e)}")
    if type(e).__name__ in ('Exception', 'AssertionError'):
        return JSONResponse(status_code=500, content={'ok': False, 'error': f'Exception: {str(e)}'})
    return JSONResponse(status_code=500, content={'ok': False, 'error': f'Uncaught {type(e).__name__} exception'})


# ---------------------------------------------------------------------------------------------- endpoints
@app.get('/')
@limiter.limit('3/minute')
async def root(request: Request):
    unspent_outputs_hash = await db.get_unspent_outputs_hash()
    logger.info(f'unspent_outputs_hash: {unspent_outputs_hash}')
    return {'ok': True, 'version': VERSION, 'unspent_outputs_hash': unspent_outputs_hash}


async def verify_and_push_tx(tx: Transaction, request: Request, background_tasks: BackgroundTasks):
    """main.py:417-458."""
    tx_hash = tx.hash()
    if _ADMISSION_BATCH:  # checks of concurrent requests are batched off the loop (utils/coalesce.py)
        coalesce.ADMISSION.set(True)
    if tx_hash in transactions_cache:
        logger.error(error_msg := 'Transaction just added')
        return {'ok': False, 'error': error_msg}
    try:
        sender = await tx.inputs[0].get_address()
        if sender in BANNED_SENDERS:
            return JSONResponse(status_code=403, content={'ok': False, 'error': 'Access forbidden temporarily.'})
        if await db.add_pending_transaction(tx):  # a cluster leader queues the row for its replicas
            if 'Sender-Node' in request.headers:
                peers.book().seen(request.headers['Sender-Node'])
            background_tasks.add_task(propagate, 'push_tx', {'tx_hex': tx.hex()})
            if transaction_listeners():  # the event is only built for subscribed /ws sessions
                tx_data = {'tx_hash': tx_hash, 'from': await tx.inputs[0].get_address() if tx.inputs else None,
                           'to': [o.address for o in tx.outputs], 'amount': sum(o.amount for o in tx.outputs),
                           'fees': tx.fees}
                background_tasks.add_task(broadcast_new_transaction, tx_data)
            transactions_cache.append(tx_hash)
            logger.info(f'Transaction has been accepted: {tx_hash}')
            return {'ok': True, 'result': 'Transaction has been accepted', 'tx_hash': tx_hash}
        logger.error(error_msg := 'Transaction has not been added')
        return {'ok': False, 'error': error_msg}
    except UniqueViolationError:
        logger.error(error_msg := 'Transaction already present')
        return {'ok': False, 'error': error_msg}


@app.get('/push_tx')
@app.post('/push_tx')
async def push_tx(request: Request, background_tasks: BackgroundTasks, tx_hex: str = None, body=Body(False)):
    if is_syncing:
        logger.warning(error := 'Node is already syncing')
        return {'ok': False, 'error': error}
    if body and tx_hex is None:
        tx_hex = body['tx_hex']
    tx = await Transaction.from_hex(tx_hex)
    return await verify_and_push_tx(tx, request, background_tasks)


@app.get('/send_to_address')
@app.post('/send_to_address')
async def send_to_address(request: Request, background_tasks: BackgroundTasks, to_address: str = None, amount=None,
                          body=Body(False), authorization: Annotated[Union[str, None], Header()] = None):
    """main.py:481-518: spend from a key in key_pair_list.json (localhost only, see middleware)."""
    from ..wallet.builders import create_transaction
    if body:
        to_address = body.get('to_address', to_address)
        amount = body.get('amount', amount)
    if not to_address or not amount:
        return JSONResponse(status_code=422, content={'ok': False, 'error': 'Missing required params.'})
    amount = str(amount)
    selected_private_key = None
    key_file = os.environ.get('UPOW_KEY_FILE') or config.data_path('key_pair_list.json')
    with open(key_file) as f:
        data = json.load(f)
    for key in data.get('keys') or []:
        if key.get('public_key') == authorization:
            selected_private_key = key.get('private_key')
    if not selected_private_key:
        return {'ok': False, 'error': 'Unauthorized'}
    if isinstance(selected_private_key, str):
        selected_private_key = int(selected_private_key, 16) if not selected_private_key.isdigit() \
            else int(selected_private_key)
    tx = await create_transaction(selected_private_key, to_address, amount, None)
    return await verify_and_push_tx(tx, request, background_tasks)


async def _json_body(request: Request):
    """The request's JSON body as ``Body(False)`` gave it (False when there is none), parsed by
    ``utils.hexspans.loads``; a malformed body is the framework's 422."""
    raw = await request.body()
    if not raw:
        return False
    try:
        return hexspans.loads(raw)
    except ValueError as e:
        raise RequestValidationError([{'type': 'json_invalid', 'loc': ('body', 0), 'msg': 'JSON decode error',
                                       'input': {}, 'ctx': {'error': str(e)}}])


@app.post('/push_block')
@app.get('/push_block')
async def push_block(request: Request, background_tasks: BackgroundTasks, block_content: str = '', txs='',
                     block_no: int = None):
    """main.py:521-652. The JSON body is read here, not by the framework: its tx array stays inside the body
    bytes (utils/hexspans.py) and the native decoder reads the txs from there."""
    body = await _json_body(request)
    if is_syncing:
        return {'ok': False, 'error': 'Node is already syncing'}
    if codec.getting_active_inodes:
        return {'ok': False, 'error': 'Server is busy'}
    if body:
        txs = body['txs']
        if 'block_content' in body:
            block_content = body['block_content']
        if 'id' in body:
            return {'ok': False, 'error': 'Deprecated'}
        if 'block_no' in body:
            block_no = body['block_no']
    if isinstance(txs, str):
        txs = txs.split(',')
        if txs == ['']:
            txs = []
    previous_hash = split_block_content(block_content)[0]
    next_block_id = await db.get_next_block_id()
    sender = request.headers.get('Sender-Node')
    if block_no is None:
        previous_block = await db.get_block(previous_hash)
        if previous_block is None:
            if sender:
                background_tasks.add_task(sync_blockchain, sender)
                return {'ok': False, 'error': 'Previous hash not found, had to sync according to sender node, '
                                              'block may have been accepted'}
            return {'ok': False, 'error': 'Previous hash not found'}
        block_no = previous_block['id'] + 1
    if next_block_id < block_no:
        background_tasks.add_task(sync_blockchain, sender if sender else None)
        return {'ok': False, 'error': 'Blocks missing, had to sync according to sender node, block may have been '
                                      'accepted'}
    if next_block_id > block_no:
        return {'ok': False, 'error': 'Too old block'}
    # full tx hex and mempool hashes, in the reference's order (full txs first, main.py:587-600); the
    # block then goes through the native block path (ledger/fastpath.py), which defers to the object
    # path for anything beyond plain transfers
    if isinstance(txs, HexSpans):
        is_hash = txs.lengths == 64
        hashes = [txs[k] for k in np.nonzero(is_hash)[0].tolist()]
        final_hexes = txs.take(np.nonzero(~is_hash)[0])
    else:
        final_hexes, hashes = [], []
        for tx_hex in txs:
            if len(tx_hex) == 64:
                hashes.append(tx_hex)
            else:
                final_hexes.append(tx_hex)
    if hashes:
        # on a worker thread: the mempool index lock may be held by a block confirm on the ledger thread
        pending_hexes = await asyncio.to_thread(db.pending_hex_by_hash, hashes)
        if len(pending_hexes) < len(hashes):
            if sender:
                background_tasks.add_task(sync_blockchain, sender)
                return {'ok': False, 'error': 'Transaction hash not found, had to sync according to sender node, '
                                              'block may have been accepted'}
            return {'ok': False, 'error': 'Transaction hash not found'}
        final_hexes = final_hexes + list(pending_hexes)
    error_list = []
    if not await on_ledger(create_block_from_hex, block_content, final_hexes, error_list=error_list):
        return {'ok': False, 'error': error_list[0]} if error_list else {'ok': False}
    block_hash = sha256(block_content)
    Manager.difficulty = None
    difficulty, last_block = await get_difficulty()
    # the next template, from the mempool index in one call, on a worker thread: the index lock may be held
    # by the ledger thread confirming a block, and the event loop must not wait for it
    first, hashes_p, _ = await asyncio.to_thread(db.mining_template)
    _mirror_gc_when_due(background_tasks)
    block_data = {'block_no': block_no, 'block_hash': block_hash, 'transactions_count': len(final_hexes),
                  'timestamp': timestamp(), 'difficulty': difficulty, 'last_block': last_block,
                  'pending_transactions': first, 'pending_transactions_hashes': hashes_p,
                  'merkle_root': get_transactions_merkle_tree(first)}
    background_tasks.add_task(broadcast_new_block, block_data)
    if sender:
        peers.book().seen(sender)
    background_tasks.add_task(propagate, 'push_block', {
        'block_content': block_content,
        'txs': [(await Transaction.from_hex(h)).hex() for h in final_hexes] if len(final_hexes) < 10 else
        txs.tolist() if isinstance(txs, HexSpans) else txs,
        'block_no': block_no})
    return {'ok': True}


@app.get('/sync_blockchain')
@limiter.limit('10/minute')
async def sync(request: Request, node_url: str = None):
    if is_syncing:
        logger.warning(msg := 'Node is already syncing')
        return {'ok': False, 'error': msg}
    resp = await sync_blockchain(node_url)
    if isinstance(resp, str):
        return {'ok': False, 'error': resp}
    if isinstance(resp, Exception):
        return {'ok': False, 'error': str(resp)}
    return {'ok': resp}


def _mirror_gc_when_due(background_tasks: BackgroundTasks) -> None:
    """Every 10 min, drop cluster-mirrored mempool txs that left the template (reference main.py:686-688
    cleans the pending table on the same cadence)."""
    if LAST_PENDING_TRANSACTIONS_CLEAN[0] < timestamp() - 600:
        LAST_PENDING_TRANSACTIONS_CLEAN[0] = timestamp()
        background_tasks.add_task(on_ledger, cluster.mirror_gc, sorted(db.pending_template()[0]))


_HASHES_MARK = '@@upow-hashes@@'


@app.get('/get_mining_info')
@limiter.limit('30/minute')
async def get_mining_info(request: Request, background_tasks: BackgroundTasks):
    """main.py:675-695. The template comes from the mempool index in one native call (selection, hex
    order, hash strings and their JSON array); only the small fields go through the generic encoder."""
    Manager.difficulty = None
    difficulty, last_block = await get_difficulty()
    first, _, hashes_json = await asyncio.to_thread(db.mining_template)  # off the loop: see push_block
    _mirror_gc_when_due(background_tasks)
    head = jsonable_encoder({'ok': True, 'result': {
        'difficulty': difficulty, 'last_block': last_block, 'pending_transactions': first,
        'pending_transactions_hashes': _HASHES_MARK, 'merkle_root': get_transactions_merkle_tree(first)}})
    doc = json.dumps(head, ensure_ascii=False, allow_nan=False, separators=(',', ':')).encode()
    body = doc.replace(f'"{_HASHES_MARK}"'.encode(), b'[' + hashes_json + b']', 1)
    return Response(content=body, media_type='application/json')


@app.get('/get_validators_info')
async def get_validators_info(background_tasks: BackgroundTasks, inode: str = None, offset: int = 0,
                              limit: int = Query(default=100, le=1000)):
    ballot = await db.get_inode_ballot_by_address(offset, limit, inode=inode) if inode else \
        await db.get_inode_ballot(offset, limit)
    result = defaultdict(lambda: {'validator': '', 'vote': []})
    for tx_hash, inode_address, votes, validator, index in ballot:
        result[validator]['validator'] = validator
        result[validator]['vote'].append({'wallet': inode_address, 'vote_count': votes, 'tx_hash': tx_hash,
                                          'index': index})
        result[validator]['totalStake'] = await db.get_validators_stake(validator, check_pending_txs=True)
    return list(result.values())


@app.get('/get_delegates_info')
async def get_delegates_info(background_tasks: BackgroundTasks, validator: str = None, offset: int = 0,
                             limit: int = Query(default=100, le=1000)):
    ballot = await db.get_validator_ballot_by_address(offset, limit, validator=validator) if validator else \
        await db.get_validator_ballot(offset, limit)
    stakes = await db.get_multiple_address_stakes({d for _, _, _, d, _ in ballot}, check_pending_txs=True)
    result = defaultdict(lambda: {'delegate': '', 'vote': [], 'totalStake': Decimal(0)})
    for tx_hash, validator_address, votes, delegate, index in ballot:
        result[delegate]['delegate'] = delegate
        result[delegate]['vote'].append({'wallet': validator_address, 'vote_count': votes, 'tx_hash': tx_hash,
                                         'index': index})
        result[delegate]['totalStake'] = stakes.get(delegate, Decimal(0))
    return list(result.values())


def _outs(outputs):
    return [{'amount': '{:f}'.format(o.amount), 'tx_hash': o.tx_hash, 'index': o.index} for o in outputs]


@app.get('/get_address_info')
@limiter.limit('15/second')
async def get_address_info(request: Request, address: str, show_pending: bool = False, verify: bool = False,
                           stake_outputs: bool = False, delegate_spent_votes: bool = False,
                           delegate_unspent_votes: bool = False, address_state: bool = False,
                           inode_registration_outputs: bool = False, validator_unspent_votes: bool = False,
                           validator_spent_votes: bool = False):
    """main.py:768-921."""
    outputs = await db.get_spendable_outputs(address)
    stake = await db.get_address_stake(address)
    balance = sum(o.amount for o in outputs)
    pending_transactions = [await db.get_nice_transaction(tx.hash(), address if verify else None)
                            for tx in await db.get_address_pending_transactions(address, True)] \
        if show_pending else None
    pending_spent_outputs = await db.get_address_pending_spent_outputs(address) if show_pending else None
    is_inode = await db.is_inode_registered(address) if address_state else None
    is_inode_active = None
    if address_state:
        is_inode_active = any(e.get('wallet') == address for e in await get_inodes_from_cache()) if is_inode \
            else False
    is_validator = await db.is_validator_registered(address) if address_state else None
    return {'ok': True, 'result': {
        'balance': '{:f}'.format(balance),
        'stake': '{:f}'.format(stake),
        'spendable_outputs': _outs(outputs),
        'pending_transactions': pending_transactions,
        'pending_spent_outputs': pending_spent_outputs,
        'stake_outputs': _outs(await db.get_stake_outputs(address)) if stake_outputs else None,
        'delegate_spent_votes': _outs(await db.get_delegates_spent_votes(address)) if delegate_spent_votes else None,
        'delegate_unspent_votes': _outs(await db.get_delegates_voting_power(address))
        if delegate_unspent_votes else None,
        'inode_registration_outputs': _outs(await db.get_inode_registration_outputs(address))
        if inode_registration_outputs else None,
        'validator_unspent_votes': _outs(await db.get_validators_voting_power(address))
        if validator_unspent_votes else None,
        'validator_spent_votes': _outs(await db.get_validators_spent_votes(address))
        if validator_spent_votes else None,
        'is_inode': is_inode,
        'is_inode_active': is_inode_active,
        'is_validator': is_validator,
    }}


@app.get('/get_address_transactions')
async def get_address_transactions(request: Request, address: str, page: int = Query(default=1, ge=1),
                                   limit: int = Query(default=5, le=1000)):
    offset = (page - 1) * limit
    txs = await db.get_address_transactions(address, limit=limit, offset=offset, check_signatures=True) \
        if limit > 0 else []
    return {'ok': True, 'result': {'transactions': [await db.get_nice_transaction(tx.hash()) for tx in txs]}}


@app.get('/add_node')
@limiter.limit('10/minute')
async def add_node(request: Request, url: str, background_tasks: BackgroundTasks):
    nodes = peers.book().urls()
    url = url.strip('/')
    if url == self_url:
        return {'ok': False, 'error': 'Recursively adding node'}
    if url in nodes:
        return {'ok': False, 'error': 'Node already present'}
    try:
        assert await peers.is_alive(url)
        background_tasks.add_task(propagate, 'add_node', {'url': url}, url)
        peers.book().add(url)
        return {'ok': True, 'result': 'Node added'}
    except Exception:
        return {'ok': False, 'error': 'Could not add node'}


@app.get('/get_nodes')
async def get_nodes():
    return {'ok': True, 'result': peers.book().recent_urls()[:100]}


@app.get('/cluster_info')
async def cluster_info(deep: bool = False):
    """Multi-GPU node: every replica's height, tip hash and UTXO-set hash (a collective, issued by the
    ledger thread like every other one; the hash is the index's K12 digest, ``deep=true`` adds each SQL
    replica's table hash). Not in the reference."""
    c = cluster.get()
    replicas = await on_ledger(cluster.status_all, db, deep)
    if c is None:
        return {'ok': True, 'result': {'world': 1, 'replicas': replicas}}
    return {'ok': True, 'result': {'world': c.ctx.world, 'backend': c.ctx.backend, 'replicas': replicas,
                                   'last_resync': c.last_resync, 'ops_sent': c.ops_sent, 'op_stream': c.info()}}


@app.get('/metrics')
async def metrics_endpoint():
    """Prometheus text exposition of the node's counters (utils/metrics.py). Not in the reference."""
    from ..utils import metrics
    metrics.set_gauge('upow_mempool_size', db._q1('SELECT COUNT(*) FROM pending_transactions')[0],
                      help='pending transactions')
    metrics.set_gauge('upow_chain_height', db._tip_id(), help='id of the last applied block')
    db.publish_writer_metrics()
    return PlainTextResponse(metrics.prometheus_text(), media_type='text/plain; version=0.0.4')


@app.get('/get_pending_transactions')
async def get_pending_transactions():
    # the reference passes 1000 as the hex-size limit (main.py:982)
    return {'ok': True, 'result': [tx.hex() for tx in await db.get_pending_transactions_limit(1000)]}


@app.get('/get_transaction')
@limiter.limit('2/second')
async def get_transaction(request: Request, tx_hash: str, verify: bool = False):
    tx = await db.get_nice_transaction(tx_hash)
    if tx is None:
        return {'ok': False, 'error': 'Transaction not found'}
    return {'ok': True, 'result': tx}


async def _resolve_block(block: str):
    if block.isdecimal():
        info = await db.get_block_by_id(int(block))
        return (info['hash'], info) if info is not None else (None, None)
    return block, await db.get_block(block)


_BLOCK_BODIES: 'OrderedDict[str, bytes]' = OrderedDict()
_BLOCK_BODIES_KEEP = 8


def _block_body(block_hash: str, block_info: dict):
    """The ``/get_block`` document of a block (hex strings need no escaping: joined into the document
    instead of walked by the generic encoder). A block's content never changes under its hash, so the
    last few documents are kept: every peer and explorer asks for the new tip."""
    txs = db.block_tx_hexes(block_hash)
    if not all(t.isalnum() for t in txs):
        return None
    mark = '"@@upow-txs@@"'
    head = json.dumps(jsonable_encoder({'ok': True, 'result': {
        'block': block_info, 'transactions': '@@upow-txs@@', 'full_transactions': None}}),
        ensure_ascii=False, allow_nan=False, separators=(',', ':'))
    body = head.replace(mark, '["' + '","'.join(txs) + '"]' if txs else '[]', 1).encode()
    _BLOCK_BODIES[block_hash] = body
    while len(_BLOCK_BODIES) > _BLOCK_BODIES_KEEP:
        _BLOCK_BODIES.popitem(last=False)
    return body


@app.get('/get_block')
@limiter.limit('30/minute')
async def get_block(request: Request, block: str, full_transactions: bool = False):
    block_hash, block_info = await _resolve_block(block)
    if not block_info:
        return {'ok': False, 'error': 'Block not found'}
    if not full_transactions:
        body = _BLOCK_BODIES.get(block_hash)
        if body is None:
            # a full block is ~8k hex strings (4 MB of JSON): read and joined on a worker thread (the
            # read waits for the ledger's connection, which a block apply holds), never on the loop
            body = await asyncio.to_thread(_block_body, block_hash, block_info)
        if body is not None:
            return Response(content=body, media_type='application/json')
    return {'ok': True, 'result': {
        'block': block_info,
        'transactions': await db.get_block_transactions(block_hash, hex_only=True) if not full_transactions else None,
        'full_transactions': await db.get_block_nice_transactions(block_hash) if full_transactions else None}}


@app.get('/get_block_details')
@limiter.limit('10/minute')
async def get_block_details(request: Request, block: str):
    block_hash, block_info = await _resolve_block(block)
    if not block_info:
        return {'ok': False, 'error': 'Block not found'}
    return {'ok': True, 'result': {'block': block_info, 'transactions': [
        await db.get_nice_transaction(h) for h in await db.get_block_transactions_hashes(block_hash)]}}


@app.get('/get_blocks')
@limiter.limit('40/minute')
async def get_blocks(request: Request, offset: int, limit: int = Query(default=..., le=1000)):
    return {'ok': True, 'result': await db.get_blocks(offset, limit)}


@app.get('/get_blocks_details')
@limiter.limit('10/minute')
async def get_blocks_details(request: Request, offset: int, limit: int = Query(default=..., le=1000)):
    return {'ok': True, 'result': await db.get_blocks(offset, limit, tx_details=True)}


@app.get('/dobby_info')
@limiter.limit('20/minute')
async def dobby_info(request: Request):
    inodes = await get_inodes_from_cache()
    return {'ok': True, 'result': [{**item, 'emission': f"{item['emission']:.2f}%"
                                    if isinstance(item['emission'], Decimal) else str(item['emission']) + '%'}
                                   for item in inodes]}


@app.get('/get_supply_info')
@limiter.limit('20/minute')
async def get_supply_info(request: Request):
    last_block = await db.get_last_block()
    return {'ok': True, 'result': {'max_supply': MAX_SUPPLY, 'circulating_supply': get_circulating_supply(
        last_block['id']), 'last_block': last_block}}
