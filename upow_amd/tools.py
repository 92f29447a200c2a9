"""Operator tools.

``python -m upow_amd.tools rebuild-utxo``: rebuild the UTXO set by replaying every transaction in
block order (reference: create_unspent_outputs.py:9-45, database.py:846-862).
``python -m upow_amd.tools utxo-hash``: print the UTXO-set hash served at ``GET /``.
``python -m upow_amd.tools snapshot [--out FILE]``: checkpoint the UTXO index at the tip (ledger/snapshot.py).
``python -m upow_amd.tools verify-utxo``: audit the UTXO index against the SQL tables (K12 hash + sets).
``python -m upow_amd.tools address-utxos ADDRESS``: the address's live outputs in all seven output tables,
straight from the UTXO index (on a GPU node one ``utxo_address_scan`` over the HBM table, K14).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import sys
from decimal import Decimal

from .constants import SMALLEST
from .ledger.database import Database


async def address_utxos(address: str, path: str = None, db: Database = None) -> dict:
    from .ledger.database import _addr_bytes
    from .ledger.utxo import TABLE_BY_TAG
    db = db or await Database.create(path=path)
    raw = _addr_bytes(address)
    if raw is None:
        raise SystemExit(f'not an address: {address}')
    recs, pay, total = db.utxo.address_outputs(raw, TABLE_BY_TAG)
    idx = recs[:, 32:36].copy().view('<u4').ravel()
    tag = recs[:, 36:40].copy().view('<u4').ravel()
    return {'address': address, 'backend': db.utxo.backend_name, 'total': str(Decimal(total) / SMALLEST),
            'outputs': [{'tx_hash': bytes(recs[k, :32]).hex(), 'index': int(idx[k]), 'table': TABLE_BY_TAG[int(tag[k])],
                         'amount': str(Decimal(int(pay['amount'][k])) / SMALLEST)} for k in range(len(recs))]}


async def rebuild_utxo(path: str = None):
    db = await Database.create(path=path)
    outputs = await db.get_unspent_outputs_from_all_transactions()
    with db.transaction():
        db.conn.execute('DELETE FROM unspent_outputs')
    await db.add_unspent_outputs(sorted(outputs))
    await db.set_unspent_outputs_addresses()
    db._rebuild_utxo_index()
    print(f'{len(outputs)} unspent outputs; hash {await db.get_unspent_outputs_hash()}')
    return len(outputs)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('command', choices=['rebuild-utxo', 'utxo-hash', 'snapshot', 'verify-utxo', 'address-utxos'])
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
            db = await Database.create(path=a.db)
            res = snapshot.save(db, a.out) if a.command == 'snapshot' else snapshot.verify(db)
            print(json.dumps(res))
            return 0 if res.get('ok', True) else 1
        return asyncio.run(s())
    else:
        async def h():
            db = await Database.create(path=a.db)
            print(await db.get_unspent_outputs_hash())
        asyncio.run(h())


if __name__ == '__main__':
    sys.exit(main())
