"""Page-batched chain sync (ledger/pagesync.py) against the per-block sync path (node/main.py
``create_blocks_per_block``, reference upow/node/main.py:97-150): the same /get_blocks pages must give the
same verdicts, the same error messages and the same ledgers — on chains with spends of outputs created
earlier in the same page (and chunk), a grouped-signature tx, a forged signature at either edge of a page, a
spend of a missing input and a double spend across two blocks of one page. The gloo test runs the page path on
a 4-rank cluster node (signatures sharded over the ranks, every block agreed before commit) and checks every
replica against the single-node per-block result."""
import asyncio
import hashlib
import json
import os
from decimal import Decimal

import pytest

KA, KB, KC = 0x5A1, 0x5B2, 0x5C3
START = 1_700_000_000
PATHS = []  # (blocks on the page path, blocks on the ordinary path) of each page synced in page mode


def _addr(k):
    from upow_amd.wallet.builders import address_of
    return address_of(k)


async def _mine(db, addr, txs, ts):
    from upow_amd import devnet
    from upow_amd.ledger import manager
    errors = []
    content = await devnet.mine_header(addr, txs, ts=ts, device='cpu')
    ok = await manager.create_block(content, txs, error_list=errors)
    assert ok, errors
    return content


async def _build_source(path):
    """A 24-block chain with intra-page spends, a grouped-signature tx and multi-tx blocks."""
    from upow_amd.bench_verify import signed_grouped_txs
    from upow_amd.ledger.database import Database
    from upow_amd.ledger import manager
    from upow_amd.utils.codec import string_to_bytes
    from upow_amd.wallet.builders import _spendable, create_transaction, create_transaction_to_send_multiple_wallet
    db = await Database.create(path=str(path), utxo_backend='host')
    manager.Manager.difficulty = None
    A, B, C = _addr(KA), _addr(KB), _addr(KC)
    h = 1
    for k in range(8):  # coinbases to A, the genesis miner (the only key that may mine without inodes)
        await _mine(db, A, [], START + 60 * h)
        h += 1
    # block 9: A pays C 2.5 and B three outputs
    tx = await create_transaction_to_send_multiple_wallet(KA, [C, B, B, B], [Decimal('2.5'), Decimal(5), Decimal(5),
                                                                              Decimal(4)])
    await _mine(db, A, [tx], START + 60 * h)
    h += 1
    tx = await create_transaction(KC, B, '1.0')  # block 10 spends block 9's output (same page)
    await _mine(db, A, [tx], START + 60 * h)
    h += 1
    # block 11: 4 inputs of two keys, two signatures (inputs grouped by owner key)
    ia = [i for i in await _spendable(db, A, Decimal(1)) if i.amount == 6][:2]
    ib = [i for i in await _spendable(db, B, Decimal(1)) if i.amount == 5][:2]
    assert len(ia) == 2 and len(ib) == 2
    grp = signed_grouped_txs([[(i.tx_hash, i.index) for i in ia + ib]], [KA], [KB], [string_to_bytes(A)],
                             [string_to_bytes(C)])
    from upow_amd.models.transaction import Transaction
    await _mine(db, A, [await Transaction.from_hex(grp[0])], START + 60 * h)
    h += 1
    for k in range(13):  # blocks 12..24: one to three txs each, spending what the page created
        txs = [await create_transaction(KA if k % 2 else KB, C, '0.5')]
        if k % 3 == 0:
            txs.append(await create_transaction(KC, A, '0.25'))
        await _mine(db, A, txs, START + 60 * h)
        h += 1
    page = await db.get_blocks(1, 100)
    db.close()
    return json.loads(json.dumps(page, default=str))


def _forge(page, at: int, txs_hex, miner_key=KA, tail: bool = False):
    """A copy of ``page[:at]`` plus a block ``at`` (index in the page) carrying ``txs_hex``, mined on the
    previous block with a fresh coinbase (what a hostile peer could serve); ``tail``: the page's original
    blocks after it follow (never reached: the sync stops at the forged block)."""
    from upow_amd import devnet
    from upow_amd.models.block import get_transactions_merkle_tree
    from upow_amd.models.transaction import CoinbaseTransaction
    prev = page[at - 1]['block']
    addr = _addr(miner_key)
    ts = int(prev['timestamp']) + 60
    content = devnet.mine_header_raw(prev['hash'], addr, get_transactions_merkle_tree(txs_hex), ts, Decimal('1.0'),
                                     device='cpu')
    bh = hashlib.sha256(bytes.fromhex(content)).hexdigest()
    cb = CoinbaseTransaction(bh, addr, Decimal(6))
    block = {'id': prev['id'] + 1, 'hash': bh, 'content': content, 'address': addr, 'random': 0,
             'difficulty': '1.0', 'reward': '6', 'timestamp': ts}
    return page[:at] + [{'block': block, 'transactions': [cb.hex()] + list(txs_hex)}] + (page[at + 1:] if tail else [])


def _bad_sig(tx_hex: str) -> str:
    raw = bytearray(bytes.fromhex(tx_hex))
    raw[-1] ^= 0x01  # s of the (only) signature
    return raw.hex()


def _missing_input_tx() -> str:
    from upow_amd.bench_verify import signed_spend_txs
    from upow_amd.utils.codec import string_to_bytes
    spend = [((hashlib.sha256(b'nowhere').hexdigest(), 0), (hashlib.sha256(b'nowhere').hexdigest(), 1))]
    return signed_spend_txs(spend, [KA], [string_to_bytes(_addr(KA))], [string_to_bytes(_addr(KC))])[0]


async def _sync(path, pages, mode: str, backend: str = 'host'):
    """Apply ``pages`` (each a list of /get_blocks entries) to a fresh ledger; returns (verdicts, errors,
    state)."""
    from upow_amd.ledger import manager, pagesync
    from upow_amd.ledger.database import Database
    from upow_amd.node import main as node_main
    db = await Database.create(path=str(path), utxo_backend=backend)
    assert db.utxo.backend_name == backend
    manager.Manager.difficulty = None
    verdicts, errors = [], []
    for page in pages:
        err = []
        if mode == 'page':
            ok = await pagesync.create_blocks(page, err)
            PATHS.append((pagesync.stats['page_path'], pagesync.stats['ordinary_path']))
        else:
            ok = await node_main.create_blocks_per_block(page, err)
        verdicts.append(ok)
        errors.append(err[:1])
        if not ok:
            break
    state = await _state(db)
    db.close()
    return verdicts, errors, state


async def _state(db):
    db.flush()
    tip = await db.get_last_block()
    rows = db._q('SELECT tx_hash, block_hash, inputs_addresses, outputs_addresses, outputs_amounts, fees '
                 'FROM transactions ORDER BY tx_hash')
    return {'height': tip['id'] if tip else 0, 'tip': tip['hash'] if tip else None,
            'sql_utxo': await db.get_unspent_outputs_hash(), 'index_utxo': db.utxo.set_hash(0),
            'utxo_entries': len(db.utxo),
            'txs': hashlib.sha256(json.dumps([tuple(r) for r in rows], default=str).encode()).hexdigest()}


@pytest.fixture(scope='module')
def source_page(tmp_path_factory):
    from upow_amd.ledger import manager
    old = manager.START_DIFFICULTY
    manager.START_DIFFICULTY = Decimal('1.0')
    try:
        yield asyncio.run(_build_source(tmp_path_factory.mktemp('src') / 'ledger.sqlite3'))
    finally:
        manager.START_DIFFICULTY = old


@pytest.fixture
def small_chunks(monkeypatch):
    from upow_amd.ledger import manager, pagesync
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('1.0'))
    monkeypatch.setattr(pagesync, 'CHUNK', 5)  # several chunks per page; spends cross chunk boundaries


@pytest.fixture(params=['host', pytest.param('gpu', marks=pytest.mark.gpu)])
def backend(request, monkeypatch):
    """The page path's UTXO table: host, or the HBM table with every signature batch on the GPU kernel."""
    if request.param == 'gpu':
        request.getfixturevalue('gpu')
        from upow_amd.ops import p256 as op
        monkeypatch.setattr(op, 'GPU_MIN_BATCH', 1)
    return request.param


def _both(tmp_path, pages, backend='host'):
    """(page path on ``backend``, per-block path on the host table: the reference's semantics)."""
    a = asyncio.run(_sync(tmp_path / 'page' / 'l.sqlite3', pages, 'page', backend))
    b = asyncio.run(_sync(tmp_path / 'block' / 'l.sqlite3', pages, 'block'))
    return a, b


def test_page_sync_equals_per_block_sync(tmp_path, source_page, small_chunks, backend):
    from upow_amd.ledger import pagesync
    pages = [source_page[:11], source_page[11:]]
    PATHS.clear()
    a, b = _both(tmp_path, pages, backend)
    assert a == b
    assert a[0] == [True, True] and a[2]['height'] == len(source_page)
    # the page path carried every block — empty ones, the genesis block and the grouped tx included
    assert PATHS == [(len(pages[0]), 0), (len(pages[1]), 0)], PATHS


@pytest.mark.parametrize('where', ['first', 'last', 'middle'])
def test_forged_signature_at_page_edges(tmp_path, source_page, small_chunks, where, backend):
    at = {'first': 12, 'last': 17, 'middle': 15}[where]
    victim = source_page[at]['transactions'][1]  # a plain tx (index 0 is the coinbase)
    forged = _forge(source_page, at, [_bad_sig(victim)], tail=where != 'last')
    pages = [forged[:12], forged[12:]]
    a, b = _both(tmp_path, pages, backend)
    assert a == b
    assert a[0][-1] is False and 'has been not verified' in a[1][-1][0]
    assert a[2]['height'] == at  # every block before the forged one applied, nothing after


def test_missing_input_and_cross_block_double_spend(tmp_path, source_page, small_chunks, backend):
    # a spend of an outpoint that never existed
    forged = _forge(source_page, 14, [_missing_input_tx()])
    a, b = _both(tmp_path / 'missing', [forged[:14], forged[14:]], backend)
    assert a == b and a[0] == [True, False] and a[2]['height'] == 14
    # block 16 re-spends an input block 15 (same page, same chunk) already spent
    spent_again = source_page[14]['transactions'][1]
    forged = _forge(source_page, 15, [spent_again])
    a, b = _both(tmp_path / 'double', [forged[:13], forged[13:]], backend)
    assert a == b and a[0] == [True, False] and a[2]['height'] == 15
    assert 'double spend' in a[1][-1][0]


def test_block_without_coinbase_stops_the_page(tmp_path, source_page, small_chunks, backend):
    """Block 15 carries no coinbase and spends a live output; block 16 spends it again. The reference's sync
    stops at block 15 (create_block_in_syncing_old dereferences the coinbase, manager.py:790): neither path
    may mint a coinbase for it (the push variant), and the page plan never applies block 16 on a plan that
    did not model block 15."""
    spend = source_page[15]['transactions'][1]
    forged = _forge(source_page, 14, [spend])
    forged[14]['transactions'] = forged[14]['transactions'][1:]  # the header's merkle root excludes the coinbase
    forged = _forge(forged, 15, [spend])
    a, b = _both(tmp_path, [forged[:12], forged[12:]], backend)
    assert a == b
    assert a[0] == [True, False] and a[2]['height'] == 14
    assert 'no coinbase' in a[1][-1][0]


def test_coinbase_with_trailing_bytes_is_split_off_on_both_paths(tmp_path, source_page, small_chunks, backend):
    """A coinbase (specifier 36) followed by extra bytes, placed after the block's txs: the codec flags it
    a coinbase (txdecode.h TX_COINBASE), so both sync paths split it off the same way."""
    from upow_amd.ledger.pagesync import _coinbase_index
    forged = _forge(source_page, 14, [source_page[14]['transactions'][1]])
    cb, *txs = forged[14]['transactions']
    odd = cb + 'abcd'
    forged[14]['transactions'] = txs + [odd]
    assert _coinbase_index(forged[14]['transactions']) == len(txs)
    # two coinbases: the trailing-bytes one comes first in the list, so it is the one the reference trusts
    assert _coinbase_index([odd, cb]) == 0
    a, b = _both(tmp_path, [forged[:12], forged[12:]], backend)
    assert a == b
    assert a[0][0] is True


def _cluster_worker(rank, world, port, tmp, q):
    os.environ.update({'RANK': str(rank), 'WORLD_SIZE': str(world), 'LOCAL_RANK': str(rank),
                       'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(port), 'UPOW_DISABLE_GPU': '1',
                       'UPOW_START_DIFFICULTY': '1.0', 'UPOW_CORE_URL': '', 'UPOW_SYNC_CHUNK': '4'})
    try:
        from upow_amd.ledger import pagesync
        from upow_amd.ledger.database import Database
        from upow_amd.parallel import cluster
        from upow_amd.parallel.dist import init_from_env, shutdown
        ctx = init_from_env(backend='gloo', want_gpu=False)
        c = cluster.init(ctx)
        with open(os.path.join(tmp, 'pages.json')) as f:
            pages = json.load(f)

        async def go():
            db = await Database.create(path=os.path.join(tmp, f'r{rank}', 'l.sqlite3'), utxo_backend='host')
            if rank != 0:
                await cluster.follower_main(c, db)
                from upow_amd.ledger import lean
                assert db.lean == lean.enabled()
                if db.lean:  # a lean replica: its SQL tables are materialised from its op log (promotion)
                    await lean.materialise(db)
            else:
                await cluster.leader_start(db)
                verdicts, errors = [], []
                for page in pages:
                    err = []
                    verdicts.append(await pagesync.create_blocks(page, err))
                    errors.append(err[:1])
                    if not verdicts[-1]:
                        break
                with open(os.path.join(tmp, 'leader.json'), 'w') as f:
                    json.dump([verdicts, errors, pagesync.stats], f)
                await cluster.leader_quit()
            st = await _state(db)
            db.close()
            return st
        st = asyncio.run(go())
        with open(os.path.join(tmp, f'state{rank}.json'), 'w') as f:
            json.dump(st, f)
        shutdown(ctx)
        q.put((rank, 'ok'))
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize('replica,shard', [('lean', '1'), ('full', '1'), ('lean', '0')],
                         ids=['lean', 'full', 'lean-unsharded-keys'])
def test_page_sync_on_a_gloo_cluster_matches_single_node(tmp_path, source_page, small_chunks, replica, shard,
                                                         monkeypatch):
    """Four ranks sync two pages (a forged signature in block 17) and reach the single node's ledger. With
    sharded keys (the default) each rank builds the records of its own verify shard only, and the block with the
    failing signature leaves the plan for the ordinary path on every rank."""
    from test_parallel import _spawn
    monkeypatch.setenv('UPOW_CLUSTER_LEAN', '1' if replica == 'lean' else '0')  # the followers' replica form
    monkeypatch.setenv('UPOW_SHARD_KEYS', shard)
    victim = source_page[17]['transactions'][1]
    forged = _forge(source_page, 17, [_bad_sig(victim)])
    pages = [forged[:9], forged[9:]]
    (tmp_path / 'c').mkdir()
    with open(tmp_path / 'c' / 'pages.json', 'w') as f:
        json.dump(pages, f)
    results = _spawn(_cluster_worker, 4, str(tmp_path / 'c'))
    assert results == {r: 'ok' for r in range(4)}, results
    states = [json.load(open(tmp_path / 'c' / f'state{r}.json')) for r in range(4)]
    verdicts, errors, stats = json.load(open(tmp_path / 'c' / 'leader.json'))
    ref = asyncio.run(_sync(tmp_path / 'ref' / 'l.sqlite3', pages, 'block'))
    assert [verdicts, errors] == [ref[0], ref[1]]
    assert all(s == ref[2] for s in states), (states, ref[2])
    assert ref[2]['height'] == 17 and stats['page_path'] > 0


RCCL_PAGE = r'''
import asyncio, json, os, sys
sys.path.insert(0, sys.argv[1])
tmp = sys.argv[2]
from upow_amd.ops.native import lib
lib()
from upow_amd.ledger import pagesync
from upow_amd.ledger.database import Database
from upow_amd.parallel import cluster
from upow_amd.parallel.dist import init_from_env, op_context, shutdown
from test_pagesync import _state
ctx = init_from_env()
assert ctx.is_distributed and ctx.backend == 'nccl', (ctx.is_distributed, ctx.backend)
c = cluster.init(op_context(ctx), ctx)  # as the node does: op traffic on its own group
with open(os.path.join(tmp, 'pages.json')) as f:
    pages = json.load(f)


async def go():
    db = await Database.create(path=os.path.join(tmp, 'r0', 'l.sqlite3'), utxo_backend='gpu')
    await cluster.leader_start(db)
    verdicts, errors = [], []
    for page in pages:
        err = []
        verdicts.append(await pagesync.create_blocks(page, err))
        errors.append(err[:1])
        if not verdicts[-1]:
            break
    info = c.info()
    await cluster.leader_quit()
    st = await _state(db)
    db.close()
    return {'verdicts': verdicts, 'errors': errors, 'state': st, 'info': info, 'stats': dict(pagesync.stats)}
res = asyncio.run(go())
print(json.dumps(res, default=str), flush=True)
shutdown(ctx)
'''


@pytest.mark.gpu
def test_page_sync_on_a_single_rank_rccl_cluster(gpu, tmp_path, source_page, small_chunks):
    """The page path of a cluster node on a real RCCL communicator (forced single-rank job): every chunk's
    signature batch through ``verify_records_dp`` (GPU kernel + status all-gather), the plan's all-reduce,
    and one native commit vote per block, against the host per-block reference."""
    import subprocess
    import sys
    from test_rccl_vote import _port
    victim = source_page[17]['transactions'][1]
    forged = _forge(source_page, 17, [_bad_sig(victim)])
    pages = [forged[:9], forged[9:]]
    (tmp_path / 'c').mkdir()
    with open(tmp_path / 'c' / 'pages.json', 'w') as f:
        json.dump(pages, f)
    script = tmp_path / 'rccl_page.py'
    script.write_text(RCCL_PAGE)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_PORT')}
    env.update(UPOW_FORCE_DIST='1', HSA_ENABLE_IPC_MODE_LEGACY='0', UPOW_START_DIFFICULTY='1.0', UPOW_CORE_URL='',
               UPOW_SYNC_CHUNK='5', UPOW_P256_GPU_MIN_BATCH='1',
               PYTHONPATH=os.pathsep.join([root, os.path.join(root, 'tests')]))
    p = subprocess.run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '1',
                        '--master-addr', '127.0.0.1', '--master-port', str(_port()), str(script), root,
                        str(tmp_path / 'c')], cwd=root, env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    res = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith('{')][-1]
    ref = asyncio.run(_sync(tmp_path / 'ref' / 'l.sqlite3', pages, 'block'))
    assert [res['verdicts'], res['errors']] == [ref[0], ref[1]]
    assert res['state'] == ref[2], (res['state'], ref[2])
    assert ref[2]['height'] == 17 and res['stats']['page_path'] > 0
    # every applied block of the sync was agreed on the native communicator
    assert res['info']['commits_agreed'] == 17 and res['info']['native_vote']['votes'] >= 17, res['info']
