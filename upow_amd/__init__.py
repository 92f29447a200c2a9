"""uPow full node, miner and wallet for AMD MI355X (gfx950)."""


def _sqlite_no_memstatus() -> int:
    """Switch off SQLite's allocation statistics before the library initialises (``import sqlite3`` does
    that): the distribution build (OMIT_LOOKASIDE, MEMSTATUS=1) takes one process-wide mutex per
    malloc/free, which serialises the ledger's parallel materialiser threads (csrc/ledger_writer.cpp).
    Returns the sqlite3_config code: 0 applied, 21 too late (sqlite3 was imported first)."""
    import ctypes
    import sys
    if 'sqlite3' in sys.modules or '_sqlite3' in sys.modules:
        return 21
    try:
        lib = ctypes.CDLL('libsqlite3.so.0')
        return int(lib.sqlite3_config(ctypes.c_int(9), ctypes.c_int(0)))  # SQLITE_CONFIG_MEMSTATUS
    except OSError:
        return -1


SQLITE_MEMSTATUS_RC = _sqlite_no_memstatus()
