"""Every ``UPOW_*`` switch that changes how the ledger is written, on its non-default branch.

Each case runs one scripted node history in a fresh interpreter (the switches are read at import or at ledger
open) and reduces the result to a digest: every SQL table that the reference keeps (upow/schema.sql: blocks,
transactions, unspent_outputs, pending_transactions, pending_spent_outputs, the six governance tables), the
address index, the chain tip and the HBM/host UTXO index's K12 hash (reference database.py:827-830). The
history covers what the switches touch: blocks through the native path (push form), a mempool admission
confirmed by a later block, a two-block rollback through the undo log and its re-application, and a second
ledger synced from the first one's /get_blocks page (reference upow/node/main.py:97-150). Every non-default
branch must reach the default's digest.

Switches and what their non-default branch changes:
  UPOW_FASTPATH=0              every block through the Transaction-object path (manager._create_block)
  UPOW_FUSED_VERIFY=0 / host   separate key + verify stages / the fused stages on the host
  UPOW_LEDGER_WRITER=0         synchronous SQL writes, no journal
  UPOW_JOURNAL_SYNC=off|group|commit   journal durability modes
  UPOW_JOURNAL_PATH            journal outside the ledger directory
  UPOW_WRITER_GROUP=1          one journal record per materialiser transaction
  UPOW_WRITER_MAX_QUEUE_MB=1   writer backpressure on every block
  UPOW_UNDO_KEEP=1             undo data of one block only: the rollback rebuilds the index instead
  UPOW_ENCODE_THREADS=1        statements encoded on one thread
  UPOW_CODEC_THREADS=1         block decode on one thread
  UPOW_ADDRESS_INDEX_INLINE=0  address index built by the lazy indexer, not inside the block batch
  UPOW_MEMPOOL_INDEX=0         mempool admission and confirm through SQL, no host index
  UPOW_GOV_INDEX=0             governance queries through SQL, no governance index
  UPOW_UTXO_ASYNC=0            the index update after a block as synchronous calls
  UPOW_WAL_CHECKPOINT_THREAD=0 / UPOW_WAL_AUTOCHECKPOINT=1   checkpoints inline / after every commit
  UPOW_SQLITE_PAGE_SIZE=4096, UPOW_SQLITE_CACHE_MB=8   B-tree page and cache sizes of a new ledger
  UPOW_SNAPSHOT_EVERY=2        UTXO snapshots on the block path
  UPOW_PAGE_SYNC=0, UPOW_SYNC_CHUNK=1   per-block sync / one-block page chunks
  UPOW_LEDGER_MIXED=0          the separate (non-mixed) file layout
(``UPOW_CLUSTER_LEAN=0``, the full follower replica, is the cluster test's second case:
tests/test_pagesync.py::test_page_sync_on_a_gloo_cluster_matches_single_node[full].)"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r'''
import asyncio, hashlib, json, os, sys
sys.path.insert(0, sys.argv[1])
from decimal import Decimal
from upow_amd import devnet
from upow_amd.ledger import fastpath, manager
from upow_amd.ledger.database import Database
from upow_amd.wallet.builders import address_of, create_transaction
manager.START_DIFFICULTY = Decimal('1.0')
G, K = 0xA11CE, [0x5EED + k for k in range(3)]
BASE = 1_700_000_000
TABLES = ['blocks', 'transactions', 'unspent_outputs', 'pending_transactions', 'pending_spent_outputs',
          'inode_registration_output', 'validators_voting_power', 'delegates_voting_power',
          'validator_registration_output', 'inodes_ballot', 'validators_ballot', 'address_transactions']


def use(db):
    Database.instance = db
    manager.Manager.difficulty = None


async def mine(db, txs, ts):
    use(db)
    c = await devnet.mine_header(address_of(G), txs, ts=ts, device='cpu')
    errs = []
    assert await fastpath.create_block_from_hex(c, [t.hex() for t in txs], error_list=errs), errs


async def digest(db):
    db.flush()
    try:
        db.index_addresses()
    except Exception:
        pass
    db.flush()
    out = {}
    for t in TABLES:
        cols = [r[1] for r in db._q(f'PRAGMA table_info({t})')]
        keep = [c for c in cols if c not in ('rowid', 'propagation_time')]
        order = ', '.join(str(i + 1) for i in range(len(keep)))  # every column: a total order, no row id
        rows = db._q(f'SELECT {", ".join(chr(34) + c + chr(34) for c in keep)} FROM {t} ORDER BY {order}')
        out[t] = hashlib.sha256(json.dumps([tuple(r) for r in rows], default=str).encode()).hexdigest()[:16]
    tip = await db.get_last_block()
    out['tip'] = tip['hash'] if tip else None
    out['k12'] = db.utxo.set_hash(0)
    out['sql_utxo'] = await db.get_unspent_outputs_hash()
    return out


async def go(tmp):
    a = await Database.create(path=os.path.join(tmp, 'a', 'ledger.sqlite3'))
    use(a)
    for k in range(6):
        await mine(a, [], BASE + 60 * k)
    tx1 = await create_transaction(G, address_of(K[0]), '2.5')
    await mine(a, [tx1], BASE + 60 * 6)
    use(a)
    tx2 = await create_transaction(G, address_of(K[1]), '1.25')
    assert await a.add_pending_transaction(tx2)
    late = await create_transaction(G, address_of(K[2]), '0.5')  # its coin selection skips tx2's pending inputs
    assert await a.add_pending_transaction(late)
    await mine(a, [tx2], BASE + 60 * 7)            # late stays pending
    await mine(a, [late], BASE + 60 * 8)           # ... and is confirmed here
    use(a)
    spend = await create_transaction(K[0], address_of(K[1]), '1')
    await mine(a, [spend], BASE + 60 * 9)
    use(a)
    await a.remove_blocks(9)                       # two blocks back through the undo log
    assert a._tip_id() == 8
    await mine(a, [late], BASE + 60 * 8 + 7)       # a different block 9, then block 10 again
    await mine(a, [spend], BASE + 60 * 9 + 7)
    use(a)
    keep = await create_transaction(G, address_of(K[0]), '0.75')
    assert await a.add_pending_transaction(keep)  # pending at the end
    da = await digest(a)
    page = await a.get_blocks(1, 100)
    page = json.loads(json.dumps(page, default=str))
    os.environ.pop('UPOW_JOURNAL_PATH', None)  # it names ONE ledger's journal: the synced ledger keeps its own
    b = await Database.create(path=os.path.join(tmp, 'b', 'ledger.sqlite3'))
    use(b)
    from upow_amd.node.main import create_blocks
    errs = []
    assert await create_blocks(page, errs), errs
    db_ = await digest(b)
    a.close(); b.close()
    return {'a': da, 'b': db_}

print(json.dumps(asyncio.run(go(sys.argv[2]))), flush=True)
'''

BASE_ENV = {'UPOW_DISABLE_GPU': '1', 'UPOW_UTXO_BACKEND': 'host', 'UPOW_START_DIFFICULTY': '1.0', 'UPOW_CORE_URL': '',
            'UPOW_LOG_LEVEL': 'WARNING', 'UPOW_CODEC_THREADS': '2', 'OMP_NUM_THREADS': '2'}
CASES = [('default', {}), ('fastpath_off', {'UPOW_FASTPATH': '0'}), ('fused_off', {'UPOW_FUSED_VERIFY': '0'}),
         ('fused_host', {'UPOW_FUSED_VERIFY': 'host'}), ('writer_off', {'UPOW_LEDGER_WRITER': '0'}),
         ('journal_sync_off', {'UPOW_JOURNAL_SYNC': 'off'}), ('journal_sync_group', {'UPOW_JOURNAL_SYNC': 'group'}),
         ('journal_sync_commit', {'UPOW_JOURNAL_SYNC': 'commit'}), ('journal_path', {'UPOW_JOURNAL_PATH': '{tmp}/elsewhere.journal'}),
         ('writer_group_1', {'UPOW_WRITER_GROUP': '1'}), ('writer_queue_1mb', {'UPOW_WRITER_MAX_QUEUE_MB': '1'}),
         ('undo_keep_1', {'UPOW_UNDO_KEEP': '1'}), ('encode_threads_1', {'UPOW_ENCODE_THREADS': '1'}),
         ('codec_threads_1', {'UPOW_CODEC_THREADS': '1'}), ('address_index_lazy', {'UPOW_ADDRESS_INDEX_INLINE': '0'}),
         ('mempool_index_off', {'UPOW_MEMPOOL_INDEX': '0'}), ('gov_index_off', {'UPOW_GOV_INDEX': '0'}),
         ('utxo_sync_apply', {'UPOW_UTXO_ASYNC': '0'}), ('checkpoint_inline', {'UPOW_WAL_CHECKPOINT_THREAD': '0'}),
         ('autocheckpoint_1', {'UPOW_WAL_AUTOCHECKPOINT': '1'}), ('page_4k_cache_8mb', {'UPOW_SQLITE_PAGE_SIZE': '4096',
                                                                                   'UPOW_SQLITE_CACHE_MB': '8'}),
         ('snapshot_every_2', {'UPOW_SNAPSHOT_EVERY': '2'}), ('page_sync_off', {'UPOW_PAGE_SYNC': '0'}),
         ('sync_chunk_1', {'UPOW_SYNC_CHUNK': '1'}), ('separate_layout', {'UPOW_LEDGER_MIXED': '0'})]


def _run(tmp_path, extra):
    script = tmp_path / 'history.py'
    script.write_text(SCRIPT)
    env = {**os.environ, **BASE_ENV, **{k: v.replace('{tmp}', str(tmp_path)) for k, v in extra.items()}}
    p = subprocess.run([sys.executable, str(script), ROOT, str(tmp_path)], env=env, capture_output=True, text=True,
                       timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-4000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


@pytest.fixture(scope='module')
def reference(tmp_path_factory):
    return _run(tmp_path_factory.mktemp('default'), {})


@pytest.mark.slow
@pytest.mark.parametrize('name,extra', CASES[1:], ids=[c[0] for c in CASES[1:]])
def test_switch_reaches_the_default_ledger(tmp_path, reference, name, extra):
    got = _run(tmp_path, extra)
    assert got == reference, {k: (got['a'].get(k), reference['a'].get(k)) for k in reference['a']
                              if got['a'].get(k) != reference['a'].get(k)}
    pending = ('pending_transactions', 'pending_spent_outputs')  # the mempool does not travel with a sync
    assert {k: v for k, v in got['a'].items() if k not in pending} == \
        {k: v for k, v in got['b'].items() if k not in pending}  # the synced ledger equals its source
