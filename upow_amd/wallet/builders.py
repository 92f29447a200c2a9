"""Wallet core: coin selection and transaction builders for every tx type.

reference: upow/upow_wallet/utils.py:11-613 (create_transaction, multi-send, stake, unstake,
inode (de)registration, validator registration, voting as validator / delegate, revoking).
Same selection rule (smallest single input covering the amount, else largest-first), same outputs,
messages and error strings; signing uses the native RFC 6979 signer (csrc/p256.hip).
"""
from __future__ import annotations

from decimal import Decimal
from typing import List, Optional

from ..constants import MAX_INODES
from ..ledger.database import Database
from ..models.transaction import Transaction, TransactionInput, TransactionOutput
from ..ops import p256 as op
from ..utils.codec import OutputType, TransactionType, point_to_string


def address_of(private_key: int) -> str:
    return point_to_string(op.public_key(private_key))


def string_to_bytes(string: Optional[str]) -> Optional[bytes]:
    """utils.py:607-613 (tx-type messages are ASCII digits; hex strings are decoded)."""
    if string is None:
        return None
    try:
        return bytes.fromhex(string)
    except ValueError:
        return string.encode('utf-8')


def type_message(t: TransactionType) -> bytes:
    return string_to_bytes(str(t.value))


def select_transaction_input(inputs: List[TransactionInput], amount) -> List[TransactionInput]:
    """utils.py:594-604."""
    chosen = []
    for i in sorted(inputs, key=lambda x: x.amount):
        if i.amount >= amount:
            chosen.append(i)
            break
    for i in sorted(inputs, key=lambda x: x.amount, reverse=True):
        if sum(x.amount for x in chosen) >= amount:
            break
        chosen.append(i)
    return chosen


async def _spendable(db: Database, address: str, amount) -> List[TransactionInput]:
    inputs = await db.get_spendable_outputs(address, check_pending_txs=True)
    if not inputs:
        raise Exception('No spendable outputs')
    if sum(i.amount for i in inputs) < amount:
        raise Exception("Error: You don't have enough funds")
    return inputs


async def create_transaction(private_key, receiving_address, amount, message: bytes = None,
                             send_back_address=None) -> Transaction:
    db = await Database.get()
    amount = Decimal(amount)
    sender = address_of(private_key)
    send_back_address = send_back_address or sender
    chosen = select_transaction_input(await _spendable(db, sender, amount), amount)
    total = sum(i.amount for i in chosen)
    tx = Transaction(chosen, [TransactionOutput(receiving_address, amount=amount)], message)
    if total > amount:
        tx.outputs.append(TransactionOutput(send_back_address, total - amount))
    return tx.sign([private_key])


async def create_transaction_to_send_multiple_wallet(private_key, receiving_addresses, amounts,
                                                     message: bytes = None, send_back_address=None) -> Transaction:
    if len(receiving_addresses) != len(amounts):
        raise Exception('Receiving addresses length is different from amounts length')
    db = await Database.get()
    amounts = [Decimal(a) for a in amounts]
    total_amount = Decimal(sum(amounts))
    sender = address_of(private_key)
    send_back_address = send_back_address or sender
    inputs = await _spendable(db, sender, total_amount)
    chosen, acc = [], Decimal(0)
    for i in sorted(inputs, key=lambda x: x.amount, reverse=True):
        chosen.append(i)
        acc += i.amount
        if acc >= total_amount:
            break
    outputs = [TransactionOutput(a, amount=Decimal(v)) for a, v in zip(receiving_addresses, amounts)]
    if acc - total_amount > 0:
        outputs.append(TransactionOutput(send_back_address, amount=acc - total_amount))
    return Transaction(chosen, outputs, message).sign([private_key])


async def create_stake_transaction(private_key, amount, send_back_address=None) -> Transaction:
    db = await Database.get()
    amount = Decimal(amount)
    sender = address_of(private_key)
    send_back_address = send_back_address or sender
    inputs = await _spendable(db, sender, amount)
    if await db.get_stake_outputs(sender):
        raise Exception('Already staked')
    if await db.get_pending_stake_transaction(sender):
        raise Exception('Already staked. Transaction is in pending')
    chosen = select_transaction_input(inputs, amount)
    total = sum(i.amount for i in chosen)
    tx = Transaction(chosen, [TransactionOutput(sender, amount=amount, transaction_type=OutputType.STAKE)])
    if total > amount:
        tx.outputs.append(TransactionOutput(send_back_address, total - amount))
    if not await db.get_delegates_all_power(sender, check_pending_txs=True):
        tx.outputs.append(TransactionOutput(sender, Decimal(10), transaction_type=OutputType.DELEGATE_VOTING_POWER))
    return tx.sign([private_key])


async def create_unstake_transaction(private_key) -> Transaction:
    db = await Database.get()
    sender = address_of(private_key)
    stake_inputs = await db.get_stake_outputs(sender, check_pending_txs=True)
    if not stake_inputs:
        raise Exception('Error: There is nothing staked')
    amount = stake_inputs[0].amount
    if await db.get_delegates_spent_votes(sender):
        raise Exception('Kindly release the votes.')
    if await db.get_pending_vote_as_delegate_transaction(address=sender):
        raise Exception('Kindly release the votes. Vote transaction is in pending')
    tx = Transaction([stake_inputs[0]], [TransactionOutput(sender, amount=amount, transaction_type=OutputType.UN_STAKE)])
    return tx.sign([private_key])


async def create_inode_registration_transaction(private_key) -> Transaction:
    db = await Database.get()
    amount = Decimal(1000)
    address = address_of(private_key)
    inputs = await _spendable(db, address, amount)
    if not await db.get_stake_outputs(address, check_pending_txs=True):
        raise Exception('You are not a delegate. Become a delegate by staking.')
    if await db.is_inode_registered(address, check_pending_txs=True):
        raise Exception('This address is already registered as inode.')
    if await db.is_validator_registered(address, check_pending_txs=True):
        raise Exception('This address is registered as validator and a validator cannot be an inode.')
    if len(await db.get_active_inodes(check_pending_txs=True)) >= MAX_INODES:
        raise Exception(f'{MAX_INODES} inodes are already registered.')
    chosen = select_transaction_input(inputs, amount)
    total = sum(i.amount for i in chosen)
    tx = Transaction(chosen, [TransactionOutput(address, amount=amount, transaction_type=OutputType.INODE_REGISTRATION)])
    if total > amount:
        tx.outputs.append(TransactionOutput(address, total - amount))
    return tx.sign([private_key])


async def create_inode_de_registration_transaction(private_key) -> Transaction:
    db = await Database.get()
    address = address_of(private_key)
    inputs = await db.get_inode_registration_outputs(address, check_pending_txs=True)
    if not inputs:
        raise Exception('This address is not registered as an inode.')
    active = await db.get_active_inodes(check_pending_txs=True)
    if any(e.get('wallet') == address for e in active):
        raise Exception('This address is an active inode. Cannot de-register.')
    tx = Transaction(inputs, [TransactionOutput(address, amount=inputs[0].amount)],
                     type_message(TransactionType.INODE_DE_REGISTRATION))
    return tx.sign([private_key])


async def create_validator_registration_transaction(private_key) -> Transaction:
    db = await Database.get()
    amount = Decimal(100)
    address = address_of(private_key)
    inputs = await _spendable(db, address, amount)
    if not await db.get_stake_outputs(address, check_pending_txs=True):
        raise Exception('You are not a delegate. Become a delegate by staking.')
    if await db.is_validator_registered(address, check_pending_txs=True):
        raise Exception('This address is already registered as validator.')
    if await db.is_inode_registered(address, check_pending_txs=True):
        raise Exception('This address is registered as inode and an inode cannot be a validator.')
    chosen = select_transaction_input(inputs, amount)
    total = sum(i.amount for i in chosen)
    tx = Transaction(chosen, [TransactionOutput(address, amount=amount,
                                                transaction_type=OutputType.VALIDATOR_REGISTRATION)],
                     type_message(TransactionType.VALIDATOR_REGISTRATION))
    tx.outputs.append(TransactionOutput(address, Decimal(10), transaction_type=OutputType.VALIDATOR_VOTING_POWER))
    if total > amount:
        tx.outputs.append(TransactionOutput(address, total - amount))
    return tx.sign([private_key])


async def create_voting_transaction(private_key, vote_range, vote_receiving_address) -> Transaction:
    try:
        vote_range = int(vote_range)
    except Exception:
        raise Exception('Invalid voting range')
    if vote_range > 10:
        raise Exception('Voting should be in range of 10')
    if vote_range <= 0:
        raise Exception('Invalid voting range')
    db = await Database.get()
    address = address_of(private_key)
    if await db.is_inode_registered(address, check_pending_txs=True):
        raise Exception('This address is registered as inode. Cannot vote.')
    if await db.is_validator_registered(address, check_pending_txs=True):
        return await vote_as_validator(private_key, vote_range, vote_receiving_address)
    if await db.get_stake_outputs(address, check_pending_txs=True):
        return await vote_as_delegate(private_key, vote_range, vote_receiving_address)
    raise Exception('Not eligible to vote')


async def _vote(private_key, vote_range, receiver, power_inputs, receiver_check, not_registered_msg, left_msg,
                msg_type, vote_type, change_type) -> Transaction:
    address = address_of(private_key)
    vote_range = Decimal(vote_range)
    if not power_inputs:
        raise Exception('No voting outputs')
    if sum(i.amount for i in power_inputs) < vote_range:
        raise Exception(left_msg)
    if not await receiver_check(receiver, check_pending_txs=True):
        raise Exception(not_registered_msg)
    chosen = select_transaction_input(power_inputs, vote_range)
    total = sum(i.amount for i in chosen)
    tx = Transaction(chosen, [TransactionOutput(receiver, amount=vote_range, transaction_type=vote_type)],
                     type_message(msg_type))
    if total > vote_range:
        tx.outputs.append(TransactionOutput(address, total - vote_range, transaction_type=change_type))
    return tx.sign([private_key])


async def vote_as_validator(private_key, vote_range, vote_receiving_address) -> Transaction:
    db = await Database.get()
    inputs = await db.get_validators_voting_power(address_of(private_key), check_pending_txs=True)
    return await _vote(private_key, vote_range, vote_receiving_address, inputs, db.is_inode_registered,
                       'Vote recipient is not registered as an inode.',
                       "Error: You don't have enough voting power left. Kindly revoke some voting power.",
                       TransactionType.VOTE_AS_VALIDATOR, OutputType.VOTE_AS_VALIDATOR,
                       OutputType.VALIDATOR_VOTING_POWER)


async def vote_as_delegate(private_key, vote_range, vote_receiving_address) -> Transaction:
    db = await Database.get()
    inputs = await db.get_delegates_voting_power(address_of(private_key), check_pending_txs=True)
    return await _vote(private_key, vote_range, vote_receiving_address, inputs, db.is_validator_registered,
                       'Vote recipient is not registered as a validator.',
                       "Error: You don't have enough voting power left. Kindly release some voting power.",
                       TransactionType.VOTE_AS_DELEGATE, OutputType.VOTE_AS_DELEGATE,
                       OutputType.DELEGATE_VOTING_POWER)


async def create_revoke_transaction(private_key, revoke_from_address) -> Transaction:
    db = await Database.get()
    address = address_of(private_key)
    if await db.is_validator_registered(address, check_pending_txs=True):
        return await revoke_vote_as_validator(private_key, revoke_from_address)
    if await db.get_stake_outputs(address, check_pending_txs=True):
        return await revoke_vote_as_delegate(private_key, revoke_from_address)
    raise Exception('Not eligible to revoke')


async def _revoke(private_key, ballot_inputs, msg_type, out_type) -> Transaction:
    db = await Database.get()
    if not ballot_inputs:
        raise Exception('You have not voted.')
    if not any([await db.is_revoke_valid(i.tx_hash) for i in ballot_inputs]):
        raise Exception('You can revoke after 48 hrs of voting')
    total = sum(i.amount for i in ballot_inputs)
    tx = Transaction(ballot_inputs, [TransactionOutput(address_of(private_key), amount=total, transaction_type=out_type)],
                     type_message(msg_type))
    return tx.sign([private_key])


async def revoke_vote_as_validator(private_key, inode_address) -> Transaction:
    db = await Database.get()
    inputs = await db.get_inode_ballot_input_by_address(address_of(private_key), inode_address, check_pending_txs=True)
    return await _revoke(private_key, inputs, TransactionType.REVOKE_AS_VALIDATOR, OutputType.VALIDATOR_VOTING_POWER)


async def revoke_vote_as_delegate(private_key, validator_address) -> Transaction:
    db = await Database.get()
    inputs = await db.get_validator_ballot_input_by_address(address_of(private_key), validator_address,
                                                            check_pending_txs=True)
    return await _revoke(private_key, inputs, TransactionType.REVOKE_AS_DELEGATE, OutputType.DELEGATE_VOTING_POWER)
