"""Operator tools.

``python -m upow_amd.tools rebuild-utxo``: rebuild the UTXO set by replaying every transaction in
block order (reference: create_unspent_outputs.py:9-45, database.py:846-862).
``python -m upow_amd.tools utxo-hash``: print the UTXO-set hash served at ``GET /``.
``python -m upow_amd.tools snapshot [--out FILE]``: checkpoint the UTXO index at the tip (ledger/snapshot.py).
``python -m upow_amd.tools verify-utxo``: audit the UTXO index against the SQL tables (K12 hash + sets).
``python -m upow_amd.tools address-utxos ADDRESS``: the address's live outputs in all seven output tables,
straight from the UTXO index (on a GPU node one ``utxo_address_scan`` over the HBM table, K14).
``python -m upow_amd.tools materialise --db <rankN ledger>``: bring a lean cluster follower's SQL tables to its
tip from its op log (ledger/lean.py); every other command does this first when the ledger has an op log.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import sys
from decimal import Decimal

from .constants import SMALLEST
from .ledger.database import Database


async def open_ledger(path: str = None) -> Database:
    """The ledger at ``path``, its SQL tables brought to the tip first when it is a lean follower's (op log)."""
    from .ledger import lean
    db = await Database.create(path=path)
    if lean.pending(db):
        n = await lean.materialise(db)
        print(f'materialised {n} block(s) from the op log', file=sys.stderr)
    return db


async def address_utxos(address: str, path: str = None, db: Database = None) -> dict:
    """Live outputs owned by ``address`` in all seven output tables, from the UTXO index (K14; one
    ``utxo_address_scan`` per address form on a GPU node). Both string forms of the key are matched
    (compressed 33 B and full 64 B, like the reference's ``address = ANY(addresses)``). ``spendable`` is
    the reference's ``get_address_balance`` (database.py:1138-1160: unspent_outputs rows with
    is_stake NULL/0); ``stake`` and each governance table are summed separately."""
    from .ledger.utxo import STAKE_ONLY, TABLE_BY_TAG
    from .utils.codec import address_search_hex
    db = db or await open_ledger(path)
    try:
        forms = [bytes.fromhex(h) for h in address_search_hex(address)]
    except Exception:
        raise SystemExit(f'not an address: {address}')
    outputs, sums = [], {'spendable': 0, 'stake': 0, **{t: 0 for t in TABLE_BY_TAG.values() if t != 'unspent_outputs'}}
    for raw in forms:
        recs, pay, _ = db.utxo.address_outputs(raw, TABLE_BY_TAG)
        idx = recs[:, 32:36].copy().view('<u4').ravel()
        tag = recs[:, 36:40].copy().view('<u4').ravel()
        for k in range(len(recs)):
            table = TABLE_BY_TAG[int(tag[k])]
            stake = table == 'unspent_outputs' and bool(int(pay['flags'][k]) & 1)
            amount = int(pay['amount'][k])
            key = ('stake' if stake else 'spendable') if table == 'unspent_outputs' else table
            sums[key] += amount
            outputs.append({'tx_hash': bytes(recs[k, :32]).hex(), 'index': int(idx[k]), 'table': table,
                            'is_stake': stake, 'amount': str(Decimal(amount) / SMALLEST), 'form': len(raw)})
    outputs.sort(key=lambda o: (o['tx_hash'], o['index']))
    return {'address': address, 'backend': db.utxo.backend_name,
            'spendable': str(Decimal(sums.pop('spendable')) / SMALLEST), 'stake': str(Decimal(sums.pop('stake')) / SMALLEST),
            'tables': {t: str(Decimal(v) / SMALLEST) for t, v in sums.items()},
            'total': str(Decimal(sum(int(Decimal(o['amount']) * SMALLEST) for o in outputs)) / SMALLEST),
            'outputs': outputs}


async def rebuild_utxo(path: str = None):
    db = await open_ledger(path)
    outputs = await db.get_unspent_outputs_from_all_transactions()
    with db.transaction():
        db._x('DELETE FROM unspent_outputs')
    await db.add_unspent_outputs(sorted(outputs))
    await db.set_unspent_outputs_addresses()
    db._rebuild_utxo_index()
    print(f'{len(outputs)} unspent outputs; hash {await db.get_unspent_outputs_hash()}')
    return len(outputs)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('command', choices=['rebuild-utxo', 'utxo-hash', 'snapshot', 'verify-utxo', 'address-utxos',
                                        'materialise'])
    ap.add_argument('address', nargs='?')
    ap.add_argument('--db', default=None)
    ap.add_argument('--out', default=None)
    a = ap.parse_args(argv)
    if a.command == 'address-utxos':
        if not a.address:
            ap.error('address-utxos needs an ADDRESS')
        print(json.dumps(asyncio.run(address_utxos(a.address, a.db))))
    elif a.command == 'rebuild-utxo':
        asyncio.run(rebuild_utxo(a.db))
    elif a.command in ('snapshot', 'verify-utxo'):
        from .ledger import snapshot

        async def s():
            db = await open_ledger(a.db)
            res = snapshot.save(db, a.out) if a.command == 'snapshot' else snapshot.verify(db)
            print(json.dumps(res))
            return 0 if res.get('ok', True) else 1
        return asyncio.run(s())
    elif a.command == 'materialise':
        async def m():
            db = await open_ledger(a.db)
            db.flush()
            print(json.dumps({'height': db._tip_id(), 'unspent_outputs_hash': await db.get_unspent_outputs_hash()}))
            db.close()
        asyncio.run(m())
    else:
        async def h():
            db = await open_ledger(a.db)
            print(await db.get_unspent_outputs_hash())
        asyncio.run(h())


if __name__ == '__main__':
    sys.exit(main())
