"""Client access policy of the HTTP node: allow/deny lists and blocked paths.

Operator contract kept from the reference (upow/node/ip_manager.py:8-56): a JSON file
``ip_config.json`` with ``whitelist``, ``blocklist``, ``block_endpoints`` and ``cache_duration``
(seconds, default 300) is created with empty lists when missing and re-read once the loaded copy is
older than ``cache_duration``. A non-empty whitelist admits only its members; otherwise every client
not on the blocklist is admitted.

Design: the file is parsed into an immutable :class:`AccessPolicy` snapshot; a request takes one
snapshot and answers both questions (address, path) from it, so a reload in between cannot split a
decision. Entries may also be CIDR networks (``"10.0.0.0/8"``), an extension the reference lacks.
A malformed file keeps the previous policy instead of failing requests.
"""
from __future__ import annotations

import ipaddress
import json
import os
import time
from dataclasses import dataclass, field
from typing import FrozenSet, Iterable, Optional, Tuple

from ..config import data_path
from ..utils.logger import get_logger

logger = get_logger(__name__)

POLICY_FILE = 'ip_config.json'
DEFAULT_TTL = 300


def _split(entries: Iterable[str]) -> Tuple[FrozenSet[str], tuple]:
    exact, nets = set(), []
    for e in entries or ():
        e = str(e).strip()
        if '/' in e:
            try:
                nets.append(ipaddress.ip_network(e, strict=False))
                continue
            except ValueError:
                pass
        exact.add(e)
    return frozenset(exact), tuple(nets)


@dataclass(frozen=True)
class AccessPolicy:
    allow: FrozenSet[str] = frozenset()
    allow_nets: tuple = ()
    deny: FrozenSet[str] = frozenset()
    deny_nets: tuple = ()
    blocked_paths: FrozenSet[str] = frozenset()
    ttl: float = DEFAULT_TTL

    @classmethod
    def from_json(cls, doc: dict) -> 'AccessPolicy':
        allow, allow_nets = _split(doc.get('whitelist', []))
        deny, deny_nets = _split(doc.get('blocklist', []))
        return cls(allow, allow_nets, deny, deny_nets, frozenset(doc.get('block_endpoints', [])),
                   float(doc.get('cache_duration', DEFAULT_TTL)))

    @staticmethod
    def _hit(ip: Optional[str], exact, nets) -> bool:
        if ip is None:
            return False
        if ip in exact:
            return True
        if nets:
            try:
                addr = ipaddress.ip_address(ip)
            except ValueError:
                return False
            return any(addr in n for n in nets)
        return False

    @property
    def allowlist_active(self) -> bool:
        return bool(self.allow or self.allow_nets)

    def admits(self, ip: Optional[str]) -> bool:
        if self.allowlist_active:
            return self._hit(ip, self.allow, self.allow_nets)
        return not self._hit(ip, self.deny, self.deny_nets)

    def allowlisted(self, ip: Optional[str]) -> bool:
        return self._hit(ip, self.allow, self.allow_nets)

    def path_blocked(self, path: str) -> bool:
        return path in self.blocked_paths


class AccessControl:
    """Owns the policy file and hands out the current :class:`AccessPolicy`."""

    def __init__(self, path: Optional[str] = None, clock=time.monotonic):
        self.path = path or data_path(POLICY_FILE)
        self.clock = clock
        self._policy = AccessPolicy()
        self._loaded_at = None
        self._pinned = False
        if not os.path.exists(self.path):
            tmp = f'{self.path}.tmp'
            with open(tmp, 'w') as f:
                json.dump({'whitelist': [], 'blocklist': [], 'block_endpoints': [],
                           'cache_duration': DEFAULT_TTL}, f, indent=4)
            os.replace(tmp, self.path)

    def policy(self) -> AccessPolicy:
        now = self.clock()
        if not self._pinned and (self._loaded_at is None or now - self._loaded_at > self._policy.ttl):
            self._loaded_at = now
            try:
                with open(self.path) as f:
                    self._policy = AccessPolicy.from_json(json.load(f))
            except FileNotFoundError:
                self._policy = AccessPolicy()
            except (ValueError, TypeError, AttributeError) as e:
                logger.error(f'{self.path}: unreadable access policy ({e}); keeping the previous one')
        return self._policy

    def install(self, policy: AccessPolicy, pin: bool = True):
        """Replace the policy in memory (tests, admin tooling); pinned policies are not reloaded."""
        self._policy = policy
        self._loaded_at = self.clock()
        self._pinned = pin

    def reload(self):
        self._pinned = False
        self._loaded_at = None
        return self.policy()
