"""IP allow/deny lists and blocked endpoints from ``ip_config.json``, re-read every cache_duration s.

reference: upow/node/ip_manager.py:8-56.
"""
from __future__ import annotations

import json
import os
import time
from typing import Dict, Optional, Set

from ..config import data_path


class Settings:
    CONFIG_FILE: str = 'ip_config.json'
    CACHE_DURATION: int = 300


class IPManager:
    def __init__(self, path: Optional[str] = None):
        self.whitelist: Set[str] = set()
        self.blocklist: Set[str] = set()
        self.block_endpoints: Set[str] = set()
        self.cache_duration: int = Settings.CACHE_DURATION
        self.last_update: float = 0
        self.config: Dict = {}
        self.path = path or data_path(Settings.CONFIG_FILE)
        self.ensure_config_exists()

    def update_config(self):
        now = time.time()
        if now - self.last_update > self.cache_duration:
            if os.path.exists(self.path):
                with open(self.path) as f:
                    self.config = json.load(f)
                self.whitelist = set(self.config.get('whitelist', []))
                self.blocklist = set(self.config.get('blocklist', []))
                self.block_endpoints = set(self.config.get('block_endpoints', []))
                self.cache_duration = self.config.get('cache_duration', Settings.CACHE_DURATION)
            self.last_update = now

    def ensure_config_exists(self):
        if not os.path.exists(self.path):
            with open(self.path, 'w') as f:
                json.dump({'whitelist': [], 'blocklist': [], 'block_endpoints': [],
                           'cache_duration': Settings.CACHE_DURATION}, f, indent=4)

    def is_ip_allowed(self, ip: str) -> bool:
        self.update_config()
        return ip in self.whitelist or (ip not in self.blocklist and not self.whitelist)

    def is_ip_whitelisted(self, ip: str) -> bool:
        self.update_config()
        return ip in self.whitelist

    def is_endpoint_blocked(self, endpoint: str) -> bool:
        return endpoint in self.block_endpoints
