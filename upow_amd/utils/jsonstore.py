"""Tiny JSON key-value store (replaces the reference's pickledb files: nodes.json,
emission_details.json, key_pair_list.json; reference database.py:22, nodes_manager.py:28-43)."""
from __future__ import annotations

import json
import os
import threading
from typing import Any, Optional


class JsonStore:
    def __init__(self, path: Optional[str], auto_dump: bool = True):
        self.path = path
        self.auto_dump = auto_dump
        self.lock = threading.RLock()
        self.db = {}
        self.load()

    def load(self):
        with self.lock:
            self.db = {}
            if self.path and os.path.exists(self.path):
                try:
                    with open(self.path) as f:
                        txt = f.read()
                    self.db = json.loads(txt) if txt.strip() else {}
                except json.JSONDecodeError:
                    self.db = {}
                    self.dump()

    def dump(self):
        if not self.path:
            return
        with self.lock:
            tmp = self.path + '.tmp'
            d = os.path.dirname(os.path.abspath(self.path))
            os.makedirs(d, exist_ok=True)
            with open(tmp, 'w') as f:
                json.dump(self.db, f)
            os.replace(tmp, self.path)

    def get(self, key: str, default: Any = None):
        with self.lock:
            return self.db.get(key, default)

    def set(self, key: str, value: Any):
        with self.lock:
            self.db[key] = value
            if self.auto_dump:
                self.dump()
        return True

    def keys(self):
        with self.lock:
            return list(self.db.keys())
