"""Structured counters for the node and miner (SURVEY.md §5 "Metrics / observability").

The reference only logs ad-hoc ``perf_counter`` timings (manager.py:655,732-736; database.py:628,661)
and the miner prints k hash/s (miner.py:89-95). Here the hot paths bump named series in one
process-wide registry, exposed as Prometheus text at ``GET /metrics`` on the node and as a dict for
benches/tests:

  upow_blocks_applied_total, upow_blocks_rejected_total, upow_block_apply_seconds (summary)
  upow_block_stage_seconds{stage=decompress|collect|ecdsa|rules}  (last validated block)
  upow_transactions_applied_total, upow_signatures_verified_total
  upow_pow_hashes_total, upow_pow_hashrate (gauge, H/s of the last search call)
  upow_mempool_size (gauge), upow_chain_height (gauge)
"""
from __future__ import annotations

import threading
from typing import Dict, Optional, Tuple

_lock = threading.Lock()
_counters: Dict[Tuple[str, Tuple], float] = {}
_gauges: Dict[Tuple[str, Tuple], float] = {}
_summaries: Dict[Tuple[str, Tuple], list] = {}  # [count, sum, max]
_help: Dict[str, str] = {}


def _key(name: str, labels: Optional[dict]) -> Tuple[str, Tuple]:
    return name, tuple(sorted((labels or {}).items()))


def inc(name: str, value: float = 1.0, labels: Optional[dict] = None, help: str = ''):
    k = _key(name, labels)
    with _lock:
        _counters[k] = _counters.get(k, 0.0) + value
        if help:
            _help.setdefault(name, help)


def set_gauge(name: str, value: float, labels: Optional[dict] = None, help: str = ''):
    with _lock:
        _gauges[_key(name, labels)] = float(value)
        if help:
            _help.setdefault(name, help)


def observe(name: str, value: float, labels: Optional[dict] = None, help: str = ''):
    k = _key(name, labels)
    with _lock:
        s = _summaries.setdefault(k, [0, 0.0, 0.0])
        s[0] += 1
        s[1] += value
        s[2] = max(s[2], value)
        if help:
            _help.setdefault(name, help)


def snapshot() -> dict:
    """Flat dict view: ``name{label=v}`` -> value (summaries as _count/_sum/_max)."""
    def fmt(name, labels):
        return name + ('{' + ','.join(f'{a}={b}' for a, b in labels) + '}' if labels else '')
    out = {}
    with _lock:
        for (n, l), v in list(_counters.items()) + list(_gauges.items()):
            out[fmt(n, l)] = v
        for (n, l), (c, s, m) in _summaries.items():
            out[fmt(n + '_count', l)] = c
            out[fmt(n + '_sum', l)] = s
            out[fmt(n + '_max', l)] = m
    return out


def reset():
    with _lock:
        _counters.clear()
        _gauges.clear()
        _summaries.clear()


def prometheus_text() -> str:
    """Prometheus text exposition format 0.0.4."""
    def lab(labels, extra=()):
        items = list(labels) + list(extra)
        return '{' + ','.join(f'{a}="{b}"' for a, b in items) + '}' if items else ''
    lines = []
    with _lock:
        seen = set()
        for kind, table in (('counter', _counters), ('gauge', _gauges)):
            for (n, l), v in sorted(table.items()):
                if n not in seen:
                    seen.add(n)
                    if n in _help:
                        lines.append(f'# HELP {n} {_help[n]}')
                    lines.append(f'# TYPE {n} {kind}')
                lines.append(f'{n}{lab(l)} {v:.17g}')
        for (n, l), (c, s, m) in sorted(_summaries.items()):
            if n not in seen:
                seen.add(n)
                if n in _help:
                    lines.append(f'# HELP {n} {_help[n]}')
                lines.append(f'# TYPE {n} summary')
            lines.append(f'{n}_count{lab(l)} {c}')
            lines.append(f'{n}_sum{lab(l)} {s:.17g}')
    return '\n'.join(lines) + '\n'


__all__ = ['inc', 'set_gauge', 'observe', 'snapshot', 'reset', 'prometheus_text']
