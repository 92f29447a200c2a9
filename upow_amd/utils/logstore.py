"""Append-only key-value log with the ``get``/``set``/``keys`` API of :class:`JsonStore`.

reference: ``emission_details`` is a pickledb file (upow/database.py:22) that ``create_block`` updates
once per block (manager.py:741-756); pickledb re-serialises the WHOLE file on every ``set``, so each
block costs O(chain length) I/O. Here each ``set`` appends one JSON line ``{"k": key, "v": value}``
(O(1)); memory holds only ``key -> (offset, length)``; ``get`` reads the one line back. A later line
for the same key supersedes the earlier one. On open, a torn final line (crash mid-append) is cut off,
and a legacy whole-file JSON object (``<name>.json``) is migrated into the log once. When the log
holds more than twice as many lines as live keys it is rewritten (amortised O(1)).
"""
from __future__ import annotations

import json
import os
import threading
from typing import Any, Dict, List, Optional, Tuple


class LogStore:
    def __init__(self, path: Optional[str], legacy_json: Optional[str] = None, fsync: bool = False):
        self.path = path
        self.fsync = fsync
        self.lock = threading.RLock()
        self.index: Dict[str, Tuple[int, int]] = {}
        self.mem: Dict[str, Any] = {}  # path None: in-memory only
        self.lines = 0
        self._f = None
        if path is None:
            return
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        fresh = not os.path.exists(path)
        self._f = open(path, 'a+b')
        self._scan()
        if fresh and legacy_json and os.path.exists(legacy_json):
            self._migrate(legacy_json)

    def _scan(self):
        self._f.seek(0)
        off = 0
        good = 0
        for line in self._f:
            n = len(line)
            if not line.endswith(b'\n'):
                break
            try:
                rec = json.loads(line)
                key = rec['k']
            except (ValueError, KeyError, TypeError):
                break
            self.index[key] = (off, n)
            self.lines += 1
            off += n
            good = off
        if good != self._f.seek(0, os.SEEK_END):
            self._f.truncate(good)
        self._f.seek(0, os.SEEK_END)

    def _migrate(self, legacy: str):
        try:
            with open(legacy) as f:
                txt = f.read()
            data = json.loads(txt) if txt.strip() else {}
        except (OSError, ValueError):
            return
        for k, v in data.items():
            self._append(str(k), v)
        self._flush()
        os.replace(legacy, legacy + '.migrated')

    def _append(self, key: str, value: Any):
        line = (json.dumps({'k': key, 'v': value}, separators=(',', ':')) + '\n').encode()
        off = self._f.seek(0, os.SEEK_END)
        self._f.write(line)
        self.index[key] = (off, len(line))
        self.lines += 1

    def _flush(self):
        self._f.flush()
        if self.fsync:
            os.fsync(self._f.fileno())

    def set(self, key: str, value: Any):
        key = str(key)
        with self.lock:
            if self._f is None:
                self.mem[key] = value
                return True
            self._append(key, value)
            self._flush()
            if self.lines > 2 * len(self.index) + 1024:
                self.compact()
        return True

    def get(self, key: str, default: Any = None):
        key = str(key)
        with self.lock:
            if self._f is None:
                return self.mem.get(key, default)
            loc = self.index.get(key)
            if loc is None:
                return default
            self._f.flush()
            self._f.seek(loc[0])
            rec = json.loads(self._f.read(loc[1]))
            self._f.seek(0, os.SEEK_END)
            return rec['v']

    def keys(self) -> List[str]:
        with self.lock:
            return list(self.mem if self._f is None else self.index)

    def compact(self):
        """Rewrite the log with one line per live key (atomic rename)."""
        with self.lock:
            if self._f is None:
                return
            tmp = self.path + '.tmp'
            new_index = {}
            with open(tmp, 'wb') as out:
                for key, (off, n) in self.index.items():
                    self._f.seek(off)
                    line = self._f.read(n)
                    new_index[key] = (out.tell(), n)
                    out.write(line)
                out.flush()
                os.fsync(out.fileno())
            self._f.close()
            os.replace(tmp, self.path)
            self._f = open(self.path, 'a+b')
            self.index = new_index
            self.lines = len(new_index)

    def close(self):
        with self.lock:
            if self._f is not None:
                self._flush()
                self._f.close()
                self._f = None


__all__ = ['LogStore']
