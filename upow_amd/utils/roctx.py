"""Host stage ranges on the rocprofv3 timeline (roctx, ``rocprofv3 --marker-trace``).

With ``UPOW_ROCTX=1`` the block path brackets its host stages (decode, UTXO pass, governance rules, signer
records, ECDSA, ledger apply and its sub-stages) with roctx ranges, so one ``rocprofv3 --kernel-trace
--marker-trace`` run shows the device kernels inside the host stages that launch them on one clock
(``scripts/block_trace.py`` summarises it). Without it every call is a no-op.
"""
from __future__ import annotations

import ctypes
import os

ENABLED = os.environ.get('UPOW_ROCTX', '0') == '1'
_push = _pop = None


def _load():
    global _push, _pop, ENABLED
    for name in ('librocprofiler-sdk-roctx.so.1', 'librocprofiler-sdk-roctx.so', 'libroctx64.so.4'):
        try:
            lib = ctypes.CDLL(name)
        except OSError:
            continue
        _push, _pop = lib.roctxRangePushA, lib.roctxRangePop
        _push.argtypes, _push.restype = [ctypes.c_char_p], ctypes.c_int
        _pop.argtypes, _pop.restype = [], ctypes.c_int
        return
    ENABLED = False


if ENABLED:
    _load()


_depth = 0


def push(name: str):
    global _depth
    if ENABLED:
        _push(name.encode())
        _depth += 1


def pop():
    global _depth
    if ENABLED and _depth > 0:
        _pop()
        _depth -= 1


def depth() -> int:
    return _depth


def unwind(to: int):
    """Close the ranges opened since ``depth()`` returned ``to`` (a stage left early)."""
    while ENABLED and _depth > to:
        pop()


class stage:
    """``with stage('decode'): ...`` — one roctx range (no-op unless UPOW_ROCTX=1)."""
    __slots__ = ('name',)

    def __init__(self, name: str):
        self.name = name

    def __enter__(self):
        push(self.name)
        return self

    def __exit__(self, *exc):
        pop()
        return False


__all__ = ['ENABLED', 'push', 'pop', 'depth', 'unwind', 'stage']
