"""Transaction data model and wire codec.

reference: upow/upow_transactions/{transaction_input,transaction_output,coinbase_transaction,
transaction}.py. Same constructor signatures, serialisation (``hex(full)``), txid (single SHA-256 of
the raw bytes), parsing (``from_hex`` incl. the signature->input assignment rules of
transaction.py:566-590) and the per-tx rule checker (``verify``), so wallets, miners and peers built
against the reference interoperate byte-for-byte.

Differences by design (MI355X build):
* addresses are kept as bytes/strings and only decompressed on demand, through a cache; a block's
  worth of decompressions and signature checks is batched on the GPU by
  :mod:`upow_amd.ledger.validate` instead of one ``fastecdsa`` call per input;
* the ledger is :class:`upow_amd.ledger.database.Database` (embedded store + HBM UTXO index).
"""
from __future__ import annotations

from decimal import Decimal
from operator import attrgetter
from io import BytesIO
from typing import List, Optional, Tuple

from .. import constants
from ..constants import ENDIAN, MAX_INODES, SMALLEST
from ..utils import codec
from ..utils.codec import (InputType, OutputType, TransactionType, bytes_to_string, byte_length,
                           get_transaction_type_from_message, point_to_string, sha256, string_to_bytes,
                           string_to_point)
from ..utils.logger import get_logger
from ..utils import p256
from ..utils.p256 import Point

logger = get_logger(__name__)
TRANSACTION_TAG = 'TRANSACTION'


def _db():
    from ..ledger.database import Database
    return Database.instance


def ecdsa_sign(msg: bytes, d: int) -> Tuple[int, int]:
    from ..ops import p256 as op
    return op.sign(msg, d)


def ecdsa_verify(sig: Tuple[int, int], msg, q: Point) -> bool:
    """fastecdsa.ecdsa.verify contract: raises p256.EcdsaError on bad key / r,s range."""
    from ..ops import p256 as op
    return op.verify(sig, msg, q)


async def ecdsa_verify_async(sig: Tuple[int, int], msg, q: Point) -> bool:
    """:func:`ecdsa_verify`, batched across concurrent /push_tx requests (ops/p256.py verify_async)."""
    from ..ops import p256 as op
    return await op.verify_async(sig, msg, q)


# C-level field getters for the hex() memo fingerprint (operator.attrgetter + map, no Python loop)
_IN_KEY = attrgetter('tx_hash', 'index', 'input_type')
_OUT_KEY = attrgetter('address_bytes', 'amount', 'transaction_type')
_SIG_KEY = attrgetter('signed')


class TransactionOutput:
    """reference: transaction_output.py:7-32."""
    __slots__ = ('address', 'address_bytes', '_public_key', 'amount', 'transaction_type', 'is_stake')

    def __init__(self, address: str, amount: Decimal, transaction_type: OutputType = OutputType.REGULAR):
        if isinstance(address, Point):
            raise Exception('TransactionOutput does not accept Point anymore. Pass the address string instead')
        self.address = address
        self.address_bytes = string_to_bytes(address)
        if len(self.address_bytes) not in (33, 64):
            raise NotImplementedError()
        self._public_key = None
        assert (amount * SMALLEST) % 1 == 0.0, 'too many decimal digits'
        self.amount = amount
        self.transaction_type = transaction_type
        self.is_stake = transaction_type == OutputType.STAKE

    @property
    def public_key(self) -> Point:
        if self._public_key is None:
            self._public_key = codec.bytes_to_point(self.address_bytes)
        return self._public_key

    def tobytes(self) -> bytes:
        amount = int(self.amount * SMALLEST)
        count = byte_length(amount)
        return (self.address_bytes + count.to_bytes(1, ENDIAN) + amount.to_bytes(count, ENDIAN)
                + int(self.transaction_type).to_bytes(1, ENDIAN))

    def point_valid(self) -> bool:
        try:
            pk = self.public_key
        except (ValueError, NotImplementedError):
            return False
        return p256.is_on_curve(pk.x, pk.y)

    def verify(self) -> bool:
        return self.amount > 0 and self.point_valid()

    @property
    def as_dict(self):
        return {'address': self.address, 'address_bytes': self.address_bytes, 'amount': self.amount,
                'transaction_type': self.transaction_type, 'is_stake': self.is_stake}


class TransactionInput:
    """reference: transaction_input.py:11-133."""

    def __init__(self, input_tx_hash: str, index: int, private_key: int = None, transaction=None,
                 amount: Decimal = None, public_key: Point = None, input_type: InputType = InputType.REGULAR):
        self.tx_hash = input_tx_hash
        self.index = index
        self.private_key = private_key
        self.transaction = transaction
        self.transaction_info = None
        self.amount = amount
        self.public_key = public_key
        self.input_type = input_type
        self.signed: Optional[Tuple[int, int]] = None
        if transaction is not None and amount is None:
            self.amount = transaction.outputs[index].amount

    async def get_transaction(self):
        if self.transaction is None:
            self.transaction = await _db().get_transaction(self.tx_hash, check_signatures=False)
            assert self.transaction is not None
        return self.transaction

    async def get_transaction_info(self):
        if self.transaction_info is None:
            self.transaction_info = await _db().get_transaction_info(self.tx_hash)
        assert self.transaction_info is not None
        return self.transaction_info

    async def get_related_output(self):
        tx = await self.get_transaction()
        related_output = tx.outputs[self.index]
        self.amount = related_output.amount
        return related_output

    async def get_related_input(self):
        tx = await self.get_transaction()
        return tx.inputs[0]

    async def get_related_input_info(self):
        tx = await self.get_transaction_info()
        return {'address': tx['inputs_addresses'][0]}

    async def get_related_output_info(self):
        tx = await self.get_transaction_info()
        related_output = {'address': tx['outputs_addresses'][self.index],
                          'amount': Decimal(tx['outputs_amounts'][self.index]) / SMALLEST}
        self.amount = related_output['amount']
        return related_output

    async def get_amount(self):
        if self.amount is None:
            if self.transaction is not None:
                return self.transaction.outputs[self.index].amount
            await self.get_related_output_info()
        return self.amount

    async def get_address(self):
        if self.transaction is not None:
            return (await self.get_related_output()).address
        return (await self.get_related_output_info())['address']

    async def get_voter_address(self):
        if self.transaction is not None:
            return (await self.get_related_input()).address
        return (await self.get_related_input_info())['address']

    def sign(self, tx_hex: str, private_key: int = None):
        private_key = private_key if private_key is not None else self.private_key
        self.signed = ecdsa_sign(bytes.fromhex(tx_hex), private_key)

    async def get_public_key(self):
        return self.public_key or string_to_point(await self.get_address())

    async def get_voter_public_key(self):
        return self.public_key or string_to_point(await self.get_voter_address())

    def tobytes(self) -> bytes:
        return bytes.fromhex(self.tx_hash) + self.index.to_bytes(1, ENDIAN) + int(self.input_type).to_bytes(1, ENDIAN)

    def get_signature(self) -> str:
        return self.signed[0].to_bytes(32, ENDIAN).hex() + self.signed[1].to_bytes(32, ENDIAN).hex()

    async def verify(self, input_tx: str) -> bool:
        try:
            public_key = await self.get_public_key()
        except AssertionError:
            return False
        # raw bytes first, then the ASCII-hex string (transaction_input.py:107-109)
        return await ecdsa_verify_async(self.signed, bytes.fromhex(input_tx), public_key) or \
            await ecdsa_verify_async(self.signed, input_tx, public_key)

    async def verify_revoke_tx(self, input_tx: str) -> bool:
        try:
            public_key = await self.get_voter_public_key()
        except AssertionError:
            return False
        return await ecdsa_verify_async(self.signed, bytes.fromhex(input_tx), public_key) or \
            await ecdsa_verify_async(self.signed, input_tx, public_key)

    @property
    def as_dict(self):
        d = {k: v for k, v in vars(self).items() if k not in ('transaction', 'private_key')}
        d['signed'] = d['signed'] is not None
        if d.get('public_key') is not None:
            d['public_key'] = point_to_string(d['public_key'])
        return d

    def __eq__(self, other):
        assert isinstance(other, self.__class__)
        return (self.tx_hash, self.index) == (other.tx_hash, other.index)

    __hash__ = object.__hash__


class CoinbaseTransaction:
    """reference: coinbase_transaction.py:8-47."""
    _hex: str = None

    def __init__(self, block_hash: str, address: str, amount: Decimal):
        self.block_hash = block_hash
        self.address = address
        self.amount = amount
        self.outputs = [TransactionOutput(address, amount)]
        self._hex = None

    async def verify(self):
        block = await _db().get_block(self.block_hash)
        return block['address'] == self.address and self.amount == block['reward']

    def hex(self) -> str:
        if self._hex is not None:
            return self._hex
        hex_inputs = (bytes.fromhex(self.block_hash) + (0).to_bytes(1, ENDIAN)).hex() + \
            int(InputType.REGULAR).to_bytes(1, ENDIAN).hex()
        hex_outputs = ''.join(o.tobytes().hex() for o in self.outputs)
        if all(len(o.address_bytes) == 64 for o in self.outputs):
            version = 1
        elif all(len(o.address_bytes) == 33 for o in self.outputs):
            version = 2
        else:
            raise NotImplementedError()
        self._hex = ''.join([version.to_bytes(1, ENDIAN).hex(), (1).to_bytes(1, ENDIAN).hex(), hex_inputs,
                             len(self.outputs).to_bytes(1, ENDIAN).hex(), hex_outputs,
                             (36).to_bytes(1, ENDIAN).hex()])
        return self._hex

    def hash(self) -> str:
        return sha256(self.hex())


class Transaction:
    """reference: transaction.py:21-601."""

    def __init__(self, inputs: List[TransactionInput], outputs: List[TransactionOutput], message: bytes = None,
                 version: int = None):
        if len(inputs) >= 256:
            raise Exception(f'You can spend max 255 inputs in a single transactions, not {len(inputs)}')
        if len(outputs) >= 256:
            raise Exception(f'You can have max 255 outputs in a single transactions, not {len(outputs)}')
        self.inputs = inputs
        self.outputs = outputs
        self.message = message
        self.transaction_type = get_transaction_type_from_message(message)
        if version is None:
            if all(len(o.address_bytes) == 64 for o in outputs):
                version = 1
            elif all(len(o.address_bytes) == 33 for o in outputs):
                version = 3
            else:
                raise NotImplementedError()
        if version > 3:
            raise NotImplementedError()
        self.version = version
        self._hex: Optional[str] = None
        self.fees: Optional[Decimal] = None
        self.tx_hash: Optional[str] = None
        self.block_hash = None

    # ------------------------------------------------------------------ codec
    def hex(self, full: bool = True) -> str:
        """transaction.py:46-83 (``full=False`` is the signed message).

        Memoised on a fingerprint of every serialised field (version, outpoints, outputs, message and,
        for ``full``, the signatures): a block's txs are serialised several times on the
        validation/apply path (txid, merkle, size check, storage), while a tx edited in place (an
        output replaced or re-valued, then re-signed) must never be signed or hashed from stale bytes."""
        fp = (full, self.version, self.message, tuple(map(_IN_KEY, self.inputs)), tuple(map(_OUT_KEY, self.outputs)),
              tuple(map(_SIG_KEY, self.inputs)) if full else None)
        memo = self.__dict__.setdefault('_hex_memo', {})
        c = memo.get(full)
        if c is not None and c[0] == fp:
            return c[1]
        h = self._hex_uncached(full)
        memo[full] = (fp, h)
        return h

    def _hex_uncached(self, full: bool = True) -> str:
        parts = [self.version.to_bytes(1, ENDIAN), len(self.inputs).to_bytes(1, ENDIAN)]
        parts += [i.tobytes() for i in self.inputs]
        parts.append(len(self.outputs).to_bytes(1, ENDIAN))
        parts += [o.tobytes() for o in self.outputs]
        h = b''.join(parts).hex()
        if not full and (self.version <= 2 or self.message is None):
            return h
        if self.message is not None:
            if self.version <= 2:
                h += bytes([1, len(self.message)]).hex()
            else:
                h += bytes([1]).hex() + len(self.message).to_bytes(2, ENDIAN).hex()
            h += self.message.hex()
            if not full:
                return h
        else:
            h += (0).to_bytes(1, ENDIAN).hex()
        signatures = []
        for tx_input in self.inputs:
            signed = tx_input.get_signature()
            if signed not in signatures:
                signatures.append(signed)
                h += signed
        self._hex = h
        return h

    def hash(self) -> str:
        if self.tx_hash is None:
            self.tx_hash = sha256(self.hex())
        return self.tx_hash

    @staticmethod
    def parse(hexstring: str):
        """Synchronous parse. Returns (tx, unresolved) where ``unresolved`` is True when the
        signature->input assignment needs public keys from the ledger (transaction.py:584-590)."""
        tx_bytes = BytesIO(bytes.fromhex(hexstring))
        version = int.from_bytes(tx_bytes.read(1), ENDIAN)
        if version > 3:
            raise NotImplementedError()
        inputs_count = int.from_bytes(tx_bytes.read(1), ENDIAN)
        inputs = []
        for _ in range(inputs_count):
            tx_hex = tx_bytes.read(32).hex()
            tx_index = int.from_bytes(tx_bytes.read(1), ENDIAN)
            input_type = int.from_bytes(tx_bytes.read(1), ENDIAN)
            inputs.append(TransactionInput(tx_hex, index=tx_index, input_type=InputType(input_type)))
        outputs_count = int.from_bytes(tx_bytes.read(1), ENDIAN)
        outputs = []
        for _ in range(outputs_count):
            pubkey = tx_bytes.read(64 if version == 1 else 33)
            amount_length = int.from_bytes(tx_bytes.read(1), ENDIAN)
            amount = int.from_bytes(tx_bytes.read(amount_length), ENDIAN) / Decimal(SMALLEST)
            transaction_type = int.from_bytes(tx_bytes.read(1), ENDIAN)
            outputs.append(TransactionOutput(bytes_to_string(pubkey), amount, OutputType(transaction_type)))
        specifier = int.from_bytes(tx_bytes.read(1), ENDIAN)
        if specifier == 36:
            assert len(inputs) == 1
            cb = CoinbaseTransaction(inputs[0].tx_hash, outputs[0].address, outputs[0].amount)
            if len(outputs) > 1:
                cb.outputs.extend(outputs[1:])
            return cb, None
        if specifier == 1:
            message_length = int.from_bytes(tx_bytes.read(1 if version <= 2 else 2), ENDIAN)
            message = tx_bytes.read(message_length)
        else:
            message = None
            assert specifier == 0
        signatures = []
        while True:
            signed = (int.from_bytes(tx_bytes.read(32), ENDIAN), int.from_bytes(tx_bytes.read(32), ENDIAN))
            if signed[0] == 0:
                break
            signatures.append(signed)
        tx = Transaction(inputs, outputs, message, version)
        if len(signatures) == 1:
            for i in inputs:
                i.signed = signatures[0]
            return tx, None
        if len(inputs) == len(signatures):
            for i, s in zip(inputs, signatures):
                i.signed = s
            return tx, None
        return tx, signatures

    @staticmethod
    async def from_hex(hexstring: str, check_signatures: bool = True):
        """transaction.py:520-592."""
        tx, pending = Transaction.parse(hexstring)
        if pending is None or not check_signatures:
            return tx
        index = {}
        for tx_input in tx.inputs:
            public_key = point_to_string(await tx_input.get_public_key())
            index.setdefault(public_key, []).append(tx_input)
        keys = list(index.keys())
        for i, signed in enumerate(pending):
            for tx_input in index[keys[i]]:
                tx_input.signed = signed
        return tx

    def __eq__(self, other):
        return isinstance(other, self.__class__) and self.hex() == other.hex()

    def __ne__(self, other):
        return not self.__eq__(other)

    __hash__ = object.__hash__

    # ------------------------------------------------------------------ rule checker
    def _verify_double_spend_same_transaction(self) -> bool:
        used = set()
        for i in self.inputs:
            k = f'{i.tx_hash}{i.index}'
            if k in used:
                return False
            used.add(k)
        return True

    async def verify_double_spend(self) -> bool:
        db = _db()
        check_inputs = [(i.tx_hash, i.index) for i in self.inputs]
        t = self.transaction_type
        if t == TransactionType.INODE_DE_REGISTRATION:
            found = await db.get_inode_outputs(check_inputs)
        elif t == TransactionType.VOTE_AS_VALIDATOR:
            found = await db.get_validator_voting_power_outputs(check_inputs)
        elif t == TransactionType.VOTE_AS_DELEGATE:
            found = await db.get_delegates_voting_power_outputs(check_inputs)
        elif t == TransactionType.REVOKE_AS_VALIDATOR:
            found = await db.get_inodes_ballot_outputs(check_inputs)
        elif t == TransactionType.REVOKE_AS_DELEGATE:
            found = await db.get_validators_ballot_outputs(check_inputs)
        else:
            found = await db.get_unspent_outputs(check_inputs)
        return set(check_inputs) == set(found)

    async def verify_double_spend_pending(self) -> bool:
        check_inputs = [(i.tx_hash, i.index) for i in self.inputs]
        spent = await _db().get_pending_spent_outputs(check_inputs)
        if spent:
            logger.error(f'Double spending in pending {spent}')
        return spent == []

    async def _fill_transaction_inputs(self, txs=None) -> None:
        check_inputs = [i.tx_hash for i in self.inputs if i.transaction is None and i.transaction_info is None]
        if not check_inputs:
            return
        if txs is None:
            txs = await _db().get_transactions_info(check_inputs)
        for i in self.inputs:
            if i.tx_hash in txs:
                i.transaction_info = txs[i.tx_hash]

    async def _check_signature(self, voter: bool = False) -> bool:
        tx_hex = self.hex(False)
        checked = []
        for i in self.inputs:
            if i.signed is None:
                logger.error('not signed')
                return False
            pk = await (i.get_voter_public_key() if voter else i.get_public_key())
            if voter:
                # reference: get_voter_public_key() result is not stored; the cache key uses .public_key
                sig_key = (i.public_key, i.signed)
            else:
                sig_key = (i.public_key, i.signed)
            if sig_key in checked:
                continue
            ok = await (i.verify_revoke_tx(tx_hex) if voter else i.verify(tx_hex))
            if not ok:
                logger.error('voter signature not valid' if voter else 'signature not valid')
                return False
            checked.append(sig_key)
            del pk
        return True

    async def _check_voter_revoke_signature(self) -> bool:
        return await self._check_signature(voter=True)

    def _verify_outputs(self) -> bool:
        return bool(self.outputs) and all(o.verify() for o in self.outputs)

    async def verify_rules(self, verifying_add_pending: bool = False) -> bool:
        """The governance rule checks of verify() (transaction.py:196-221), in reference order."""
        for check in (self.verify_stake_transaction, self.verify_un_stake_transaction,
                      self.verify_validator_transaction, self.verify_revoke_as_validator,
                      self.verify_revoke_as_delegate, self.verify_inode_de_register_transaction,
                      self.verify_inode_register_transaction, self.verify_vote_as_validator_transaction):
            if not await check():
                return False
        return await self.verify_vote_as_delegate_transaction(verifying_add_pending=verifying_add_pending)

    async def verify(self, check_double_spend: bool = True, verifying_add_pending: bool = False,
                     check_signatures: bool = True) -> bool:
        """transaction.py:185-238. ``check_signatures=False`` is used by the batched block validator,
        which verifies every signature of the block in one GPU pass instead."""
        tag = TRANSACTION_TAG if verifying_add_pending else ''
        if check_double_spend and not self._verify_double_spend_same_transaction():
            logger.error(f'{tag} Double spend inside same transaction')
            return False
        if check_double_spend and not await self.verify_double_spend():
            logger.error(f'{tag} Double spend')
            return False
        await self._fill_transaction_inputs()
        if not await self.verify_rules(verifying_add_pending):
            return False
        if check_signatures:
            if self.transaction_type in (TransactionType.REVOKE_AS_VALIDATOR, TransactionType.REVOKE_AS_DELEGATE):
                if not await self._check_voter_revoke_signature():
                    return False
            elif not await self._check_signature():
                return False
        if not self._verify_outputs():
            logger.error('invalid outputs')
            return False
        if await self.get_fees() < 0:
            logger.error('We are not the Federal Reserve')
            return False
        return True

    async def verify_inode_de_register_transaction(self) -> bool:
        if self.transaction_type == TransactionType.INODE_DE_REGISTRATION:
            db = _db()
            address = await self.inputs[0].get_address()
            if not await db.get_inode_registration_outputs(address):
                logger.error('This address is not registered as an inode.')
                return False
            active = await db.get_active_inodes()
            if any(e.get('wallet') == address for e in active):
                logger.error('This address is an active inode. Cannot de-register.')
                return False
        return True

    async def verify_vote_as_validator_transaction(self) -> bool:
        if self.transaction_type == TransactionType.VOTE_AS_VALIDATOR:
            vote_range = sum(o.amount for o in self.outputs if o.transaction_type == OutputType.VOTE_AS_VALIDATOR)
            if vote_range > 10:
                logger.error('Voting should be in range of 10')
                return False
            if vote_range <= 0:
                logger.error('Invalid voting range')
                return False
            db = _db()
            address = await self.inputs[0].get_address()
            if await db.is_inode_registered(address, check_pending_txs=True):
                logger.error('This address is registered as inode. Cannot vote.')
                return False
            if not await db.is_validator_registered(address, check_pending_txs=True):
                logger.error('This address is not registered as validator. Cannot vote.')
                return False
            receiver = ''
            for o in self.outputs:
                if o.transaction_type is OutputType.VOTE_AS_VALIDATOR:
                    receiver = o.address
            if not await db.is_inode_registered(receiver, check_pending_txs=True):
                logger.error('Vote recipient is not registered as an inode.')
                return False
        return True

    async def verify_vote_as_delegate_transaction(self, verifying_add_pending: bool = False) -> bool:
        if self.transaction_type == TransactionType.VOTE_AS_DELEGATE:
            vote_range = sum(o.amount for o in self.outputs if o.transaction_type == OutputType.VOTE_AS_DELEGATE)
            if vote_range > 10:
                logger.error('Voting should be in range of 10')
                return False
            if vote_range <= 0:
                logger.error('Invalid voting range')
                return False
            db = _db()
            address = await self.inputs[0].get_address()
            if await db.is_inode_registered(address, check_pending_txs=True):
                logger.error('This address is registered as inode. Cannot vote.')
                return False
            if not await db.get_stake_outputs(address, check_pending_txs=verifying_add_pending):
                logger.error('This address is not staked anything. Cannot vote.')
                return False
            receiver = ''
            for o in self.outputs:
                if o.transaction_type is OutputType.VOTE_AS_DELEGATE:
                    receiver = o.address
            if not await db.is_validator_registered(receiver, check_pending_txs=True):
                logger.error('Vote recipient is not registered as a validator.')
                return False
        return True

    async def verify_inode_register_transaction(self) -> bool:
        if any(o.transaction_type == OutputType.INODE_REGISTRATION for o in self.outputs):
            db = _db()
            address = await self.inputs[0].get_address()
            amount = sum(o.amount for o in self.outputs if o.transaction_type == OutputType.INODE_REGISTRATION)
            if amount != 1000:
                logger.error('Inode registration amount is in correct')
                return False
            if not await db.get_stake_outputs(address):
                logger.error('You are not a delegate. Become a delegate by staking.')
                return False
            if await db.is_inode_registered(address, check_pending_txs=True):
                logger.error('This address is already registered as inode.')
                return False
            if await db.is_validator_registered(address, check_pending_txs=True):
                logger.error('This address is registered as validator and a validator cannot be an inode.')
                return False
            if len(await db.get_active_inodes(check_pending_txs=True)) >= MAX_INODES:
                logger.error(f'{MAX_INODES} inodes are already registered.')
                return False
            active = await db.get_active_inodes()
            if any(e.get('wallet') == address for e in active):
                logger.error('This address is an active inode. Cannot de-register.')
                return False
        return True

    async def verify_validator_transaction(self) -> bool:
        if self.transaction_type == TransactionType.VALIDATOR_REGISTRATION:
            db = _db()
            address = await self.inputs[0].get_address()
            if not await db.get_stake_outputs(address):
                logger.error('You are not a delegate. Become a delegate by staking.')
                return False
            if await db.is_validator_registered(address, check_pending_txs=True):
                logger.error('validator already registered')
                return False
            if await db.is_inode_registered(address, check_pending_txs=True):
                logger.error('Already registered as an inode')
                return False
            amount = sum(o.amount for o in self.outputs if o.transaction_type == OutputType.VALIDATOR_REGISTRATION)
            if amount != 100:
                logger.error('validator reg amount is not correct')
                return False
            power = [o for o in self.outputs if o.transaction_type == OutputType.VALIDATOR_VOTING_POWER]
            if len(power) != 1:
                logger.error('Validator voting power input bug')
                return False
            if power[0].amount != 10:
                logger.error('Validator voting power bug')
                return False
        return True

    async def verify_revoke_as_validator(self) -> bool:
        if self.transaction_type == TransactionType.REVOKE_AS_VALIDATOR:
            db = _db()
            address = await self.inputs[0].get_voter_address()
            if not await db.is_validator_registered(address, check_pending_txs=True):
                logger.error('This address is not registered as validator.')
                return False
            if not await db.get_stake_outputs(address):
                logger.error('This address is not registered as delegate. Cannot revoke')
                return False
            valid = [await db.is_revoke_valid(i.tx_hash) for i in self.inputs]
            if not any(valid):
                logger.error('You can revoke after 48 hrs of voting')
                return False
        return True

    async def verify_revoke_as_delegate(self) -> bool:
        if self.transaction_type == TransactionType.REVOKE_AS_DELEGATE:
            db = _db()
            address = await self.inputs[0].get_voter_address()
            if not await db.get_stake_outputs(address):
                logger.error('This address is not registered as delegate. Cannot revoke')
                return False
            valid = [await db.is_revoke_valid(i.tx_hash) for i in self.inputs]
            if not any(valid):
                logger.error('You can revoke after 48 hrs of voting')
                return False
        return True

    async def verify_stake_transaction(self) -> bool:
        if any(o.transaction_type == OutputType.STAKE for o in self.outputs):
            db = _db()
            address = await self.inputs[0].get_address()
            stake_inputs = await db.get_stake_outputs(address)
            if stake_inputs and not codec.is_blockchain_syncing:
                logger.error('Already staked')
                return False
            pending = [t for t in await db.get_pending_stake_transaction(address) if t.tx_hash != self.tx_hash]
            if pending:
                logger.error('Already staked. Transaction is in pending')
                return False
            power = sum(o.amount for o in self.outputs if o.transaction_type == OutputType.DELEGATE_VOTING_POWER)
            if power > 0:
                if power != 10:
                    logger.error('Delegate voting power bug')
                    return False
                if await db.get_delegates_all_power(address):
                    logger.error('Delegate already have voting power')
                    return False
            elif not await db.get_delegates_all_power(address):
                logger.error('Delegate doesnt have voting power')
                return False
        return True

    async def verify_un_stake_transaction(self) -> bool:
        if any(o.transaction_type == OutputType.UN_STAKE for o in self.outputs):
            db = _db()
            address = await self.inputs[0].get_address()
            # consensus exception: revoke_as_delegate + unstake in the same block (transaction.py:472)
            if await db.get_delegates_spent_votes(address) and self.hash() not in [
                    '8befeb253bc6eddd8501f5b27a02b195f5c06a51ccf788213cbedafe7cc49c53']:
                logger.error('Kindly release the votes.')
                return False
            if await db.get_pending_vote_as_delegate_transaction(address=address):
                logger.error('Kindly release the votes. Vote transaction is in pending')
                return False
        return True

    async def verify_pending(self) -> bool:
        return await self.verify(verifying_add_pending=True) and await self.verify_double_spend_pending()

    def sign(self, private_keys=None):
        """transaction.py:484-497."""
        for private_key in private_keys or []:
            pub = None
            for i in self.inputs:
                if i.private_key is None and (i.public_key or i.transaction):
                    if pub is None:
                        from ..ops import p256 as op
                        pub = op.public_key(private_key)
                    input_public_key = i.public_key or i.transaction.outputs[i.index].public_key
                    if pub == input_public_key:
                        i.private_key = private_key
        msg = None
        for i in self.inputs:
            if i.private_key is not None:
                msg = msg or self.hex(False)
                i.sign(msg)
        return self

    async def get_fees(self) -> Decimal:
        """transaction.py:499-518 (only REGULAR txs carry fees)."""
        input_amount = 0
        output_amount = 0
        if self.transaction_type == TransactionType.REGULAR:
            for i in self.inputs:
                input_amount += await i.get_amount()
            output_amount = sum(o.amount for o in self.outputs if o.transaction_type not in
                                (OutputType.VALIDATOR_VOTING_POWER, OutputType.DELEGATE_VOTING_POWER))
        self.fees = input_amount - output_amount
        assert (self.fees * SMALLEST) % 1 == 0.0
        return self.fees


__all__ = ['Transaction', 'TransactionInput', 'TransactionOutput', 'CoinbaseTransaction', 'constants']
