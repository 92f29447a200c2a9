"""HTTP-only wallet (reference: upow/upow_wallet/nodeless_wallet.py:31-200).

``python -m upow_amd.wallet.nodeless {createwallet,send,balance} [-to R] [-d AMOUNT] [-m MSG]``.
Keys in ``<data dir>/upow_wallet.json`` ({"private_keys": [...]}). Coin selection follows the reference
(single covering input, else smallest-first up to 255 inputs). Unlike the reference, outputs listed
in ``pending_spent_outputs`` (dicts) are really skipped — the reference compared ``tuple(dict)``
(the key names) and never matched.
"""
from __future__ import annotations

import argparse
import os
import sys
from decimal import Decimal

import httpx

from .. import config
from ..models.transaction import Transaction, TransactionInput, TransactionOutput
from ..ops import p256 as op
from ..utils.codec import point_to_string, sha256, string_to_point
from ..utils.jsonstore import JsonStore
from .builders import string_to_bytes


def node_url() -> str:
    return (os.environ.get('UPOW_WALLET_NODE_URL') or os.environ.get('UPOW_CORE_URL') or 'http://localhost:3006/')\
        .rstrip('/') + '/'


def get_address_info(address: str):
    r = httpx.get(f'{node_url()}get_address_info', params={'address': address, 'transactions_count_limit': 0,
                                                           'show_pending': True}, timeout=10)
    result = r.json()['result']
    pending = {(o['tx_hash'], o['index']) for o in result['pending_spent_outputs'] or []}
    inputs = []
    for o in result['spendable_outputs']:
        if (o['tx_hash'], o['index']) in pending:
            continue
        i = TransactionInput(o['tx_hash'], o['index'])
        i.amount = Decimal(str(o['amount']))
        i.public_key = string_to_point(address)
        inputs.append(i)
    return Decimal(result['balance']), inputs


def create_transaction(private_keys, receiving_address, amount, message: bytes = None, send_back_address=None,
                       push: bool = True) -> Transaction:
    amount = Decimal(amount)
    inputs = []
    for d in private_keys:
        address = point_to_string(op.public_key(d))
        send_back_address = send_back_address or address
        _, addr_inputs = get_address_info(address)
        for i in addr_inputs:
            i.private_key = d
        inputs.extend(addr_inputs)
        if sum(i.amount for i in sorted(inputs, key=lambda x: x.amount)[:255]) >= amount:
            break
    if not inputs:
        raise Exception('No spendable outputs')
    if sum(i.amount for i in inputs) < amount:
        raise Exception("Error: You don't have enough funds")
    chosen = []
    if any(i.amount >= amount for i in inputs):
        for i in sorted(inputs, key=lambda x: x.amount):
            if i.amount >= amount:
                chosen.append(i)
                break
    else:
        for i in sorted(inputs, key=lambda x: x.amount):
            chosen.append(i)
            if sum(x.amount for x in chosen) >= amount:
                break
            if len(chosen) >= 255:
                chosen.pop(0)
    total = sum(i.amount for i in chosen)
    if total < amount:
        raise Exception(f'Consolidate outputs: send {total} upow to yourself')
    tx = Transaction(chosen, [TransactionOutput(receiving_address, amount=amount)], message)
    if total > amount:
        tx.outputs.append(TransactionOutput(send_back_address, total - amount))
    tx.sign(private_keys)
    if push:
        httpx.get(f'{node_url()}push_tx', params={'tx_hex': tx.hex()}, timeout=10)
    return tx


def main(argv=None):
    ap = argparse.ArgumentParser(description='UPOW wallet')
    ap.add_argument('command', choices=['createwallet', 'send', 'balance'])
    ap.add_argument('-to', dest='recipient', required=False)
    ap.add_argument('-d', dest='amount', required=False)
    ap.add_argument('-m', dest='message', required=False)
    args = ap.parse_args(argv)
    store = JsonStore(os.environ.get('UPOW_NODELESS_KEY_FILE') or config.data_path('upow_wallet.json'))
    keys = [int(k) for k in store.get('private_keys') or []]
    if args.command == 'createwallet':
        d = op.oracle.gen_private_key()
        store.set('private_keys', keys + [d])
        print(f'Private key: {hex(d)}\nAddress: {point_to_string(op.public_key(d))}')
    elif args.command == 'balance':
        total = 0
        for d in keys:
            address = point_to_string(op.public_key(d))
            bal, _ = get_address_info(address)
            total += bal
            print(f'\nAddress: {address}\nPrivate key: {hex(d)}\nBalance: {bal}')
        print(f'\nTotal Balance: {total}')
    else:
        if not args.recipient or not args.amount:
            ap.error('send needs -to and -d')
        tx = create_transaction(keys, args.recipient, args.amount, string_to_bytes(args.message))
        print(f'Transaction pushed. Transaction hash: {sha256(tx.hex())}')


if __name__ == '__main__':
    sys.exit(main())
