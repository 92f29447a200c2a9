"""Protocol constants (reference: upow/constants.py:3-9, upow/manager.py:26-29).

The curve is NIST P-256 (secp256r1) exactly as the reference's ``CURVE = curve.P256``
(upow/constants.py:4); parameters live in :mod:`upow_amd.utils.p256`.
"""
from decimal import Decimal

ENDIAN = 'little'
SMALLEST = 100000000
MAX_SUPPLY = 18_884_643.75
VERSION = 2
MAX_BLOCK_SIZE_HEX = 4096 * 1024  # 4 MB hex == 2 MB raw
MAX_INODES = 12

# consensus (upow/manager.py:26-29)
BLOCK_TIME = 60
BLOCKS_COUNT = Decimal(100)
LAST_BLOCK_FOR_GENESIS_KEY = 10000
# 6.0 on mainnet; UPOW_START_DIFFICULTY overrides it for private devnets and tests only
START_DIFFICULTY = Decimal(__import__('os').environ.get('UPOW_START_DIFFICULTY', '6.0'))

# genesis "previous hash" used by miners/sync when the chain is empty (miner.py:40, main.py:105)
GENESIS_PREV_HASH = (18_884_643).to_bytes(32, ENDIAN).hex()

# reward schedule (upow/manager.py:154-168)
HALVING_INTERVAL = 1576800
NINE_HALVING_INTERVAL = 14191200
COINS_PER_BLOCK = 6
