"""DB wallet CLI (reference: upow/upow_wallet/wallet.py:44-288).

``python -m upow_amd.wallet {createwallet,send,balance,stake,unstake,register_inode,de_register_inode,
register_validator,vote,revoke} [-to R] [-a AMOUNT] [-m MSG] [-r RANGE] [-from ADDR]``

Keys live in ``<data dir>/key_pair_list.json`` ({"keys": [{"private_key", "public_key"}]}); the wallet
reads the local ledger directly and pushes through the node's ``/push_tx`` (falling back to a direct
mempool insert, like the reference). The reference's single-key ``select_key`` bug (reads
``private_keys`` instead of ``keys``, wallet.py:282) is fixed.
"""
from __future__ import annotations

import argparse
import asyncio
import os
import sys

import httpx

from .. import config
from ..ledger.database import Database
from ..ops import p256 as op
from ..utils.codec import point_to_string, sha256
from ..utils.jsonstore import JsonStore
from . import builders
from .builders import string_to_bytes

COMMANDS = ['createwallet', 'send', 'balance', 'stake', 'unstake', 'register_inode', 'de_register_inode',
            'register_validator', 'vote', 'revoke']


def node_url() -> str:
    return (os.environ.get('UPOW_WALLET_NODE_URL') or os.environ.get('UPOW_CORE_URL') or 'http://localhost:3006/')\
        .rstrip('/') + '/'


def key_store() -> JsonStore:
    return JsonStore(os.environ.get('UPOW_KEY_FILE') or config.data_path('key_pair_list.json'))


def select_key(db: JsonStore, index: int = None) -> int:
    keys = db.get('keys') or []
    if not keys:
        raise Exception('No key. please create key')
    if len(keys) > 1:
        if index is None:
            for i, kp in enumerate(keys):
                print(i, kp['public_key'])
            try:
                index = int(input('Select key: '))
            except ValueError:
                raise Exception('Invalid input. Please enter a valid integer.')
        if index >= len(keys):
            raise Exception('Invalid input. Please enter a correct key number.')
        return int(keys[index]['private_key'])
    return int(keys[0]['private_key'])


async def push_tx(tx, database: Database):
    try:
        r = httpx.get(node_url() + 'push_tx', params={'tx_hex': tx.hex()}, timeout=10).json()
        print(f'Transaction pushed. Transaction hash: {sha256(tx.hex())}' if r.get('ok')
              else '\nTransaction has not been added')
    except Exception as e:
        print(f'Could not push transaction to local node: {e}')
        if await database.add_pending_transaction(tx):
            print(f'Transaction pushed. Transaction hash: {sha256(tx.hex())}')
        else:
            print('\nTransaction has not been added')


async def main(argv=None):
    ap = argparse.ArgumentParser(description='UPOW wallet')
    ap.add_argument('command', choices=COMMANDS)
    ap.add_argument('-to', dest='recipient', required=False)
    ap.add_argument('-a', dest='amount', required=False)
    ap.add_argument('-m', dest='message', required=False)
    ap.add_argument('-r', dest='range', required=False)
    ap.add_argument('-from', dest='revoke_from', required=False)
    ap.add_argument('-k', dest='key_index', type=int, required=False, help='key index (skips the prompt)')
    args = ap.parse_args(argv)
    store = key_store()
    database = await Database.get()
    cmd = args.command
    if cmd == 'createwallet':
        key_list = store.get('keys') or []
        d = op.oracle.gen_private_key()
        address = point_to_string(op.public_key(d))
        key_list.append({'private_key': d, 'public_key': address})
        store.set('keys', key_list)
        print(f'Private key: {hex(d)}\nAddress: {address}')
        return
    if cmd == 'balance':
        total = total_pending = 0
        for kp in store.get('keys') or []:
            address = point_to_string(op.public_key(int(kp['private_key'])))
            bal = await database.get_address_balance(address)
            stake = await database.get_address_stake(address)
            pbal = await database.get_address_balance(address, True)
            pstake = await database.get_address_stake(address, True)
            total += bal
            total_pending += pbal
            print(f'\nAddress: {address}\nPrivate key: {hex(int(kp["private_key"]))}'
                  f'\nBalance: {bal}{f" ({pbal - bal} pending)" if pbal - bal != 0 else ""}'
                  f'\nStake: {stake}{f" ({pstake - stake} pending)" if pstake - stake != 0 else ""}')
        print(f'\nTotal Balance: {total}{f" ({total_pending - total} pending)" if total_pending - total != 0 else ""}')
        return
    key = select_key(store, args.key_index)
    if cmd == 'send':
        if not args.recipient or not args.amount:
            ap.error('send needs -to and -a')
        recipients, amounts = args.recipient.split(','), args.amount.split(',')
        msg = string_to_bytes(args.message)
        if len(recipients) > 1 and len(amounts) > 1 and len(recipients) == len(amounts):
            tx = await builders.create_transaction_to_send_multiple_wallet(key, recipients, amounts, msg)
        else:
            tx = await builders.create_transaction(key, recipients[0], amounts[0], msg)
    elif cmd == 'stake':
        if not args.amount:
            ap.error('stake needs -a')
        tx = await builders.create_stake_transaction(key, args.amount)
    elif cmd == 'unstake':
        tx = await builders.create_unstake_transaction(key)
    elif cmd == 'register_inode':
        tx = await builders.create_inode_registration_transaction(key)
    elif cmd == 'de_register_inode':
        tx = await builders.create_inode_de_registration_transaction(key)
    elif cmd == 'register_validator':
        tx = await builders.create_validator_registration_transaction(key)
    elif cmd == 'vote':
        if not args.range or not args.recipient:
            ap.error('vote needs -r and -to')
        tx = await builders.create_voting_transaction(key, args.range, args.recipient)
    else:  # revoke
        if not args.revoke_from:
            ap.error('revoke needs -from')
        tx = await builders.create_revoke_transaction(key, args.revoke_from)
    await push_tx(tx, database)
    return tx


def run():
    return asyncio.run(main())


if __name__ == '__main__':
    sys.exit(run() and 0)
