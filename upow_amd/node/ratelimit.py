"""Per-endpoint, per-client rate limits (replaces slowapi, which is not available).

reference: ``@limiter.limit("N/period")`` on the node endpoints (upow/node/main.py:266-1102) with
slowapi's default 429 handler body ``{"error": "Rate limit exceeded: N per 1 period"}``.
Fixed-window counters keyed by (endpoint, client address).
"""
from __future__ import annotations

import functools
import inspect
import time
from collections import defaultdict
from typing import Callable, Dict, Tuple

from starlette.requests import Request
from starlette.responses import JSONResponse

_PERIODS = {'second': 1, 'minute': 60, 'hour': 3600, 'day': 86400}


class RateLimitExceeded(Exception):
    def __init__(self, detail: str):
        super().__init__(detail)
        self.detail = detail


def get_remote_address(request: Request) -> str:
    return request.client.host if request.client else '127.0.0.1'


def parse_limit(spec: str) -> Tuple[int, int, str]:
    count, per = spec.split('/')
    per = per.strip().rstrip('s') if per.strip() not in _PERIODS else per.strip()
    return int(count), _PERIODS[per], per


class Limiter:
    def __init__(self, key_func: Callable[[Request], str] = get_remote_address, enabled: bool = True):
        self.key_func = key_func
        self.enabled = enabled
        self._windows: Dict[Tuple[str, str], Tuple[int, int]] = defaultdict(lambda: (0, 0))

    def reset(self):
        self._windows.clear()

    def hit(self, scope: str, request: Request, spec: str):
        if not self.enabled:
            return
        count, seconds, per = parse_limit(spec)
        key = (scope, self.key_func(request))
        window = int(time.time() // seconds)
        w, n = self._windows[key]
        if w != window:
            w, n = window, 0
        n += 1
        self._windows[key] = (w, n)
        if n > count:
            raise RateLimitExceeded(f'{count} per 1 {per}')

    def limit(self, spec: str):
        def deco(fn):
            sig = inspect.signature(fn)
            assert 'request' in sig.parameters, 'rate-limited endpoints need a `request: Request` parameter'

            @functools.wraps(fn)
            async def wrapper(*args, **kwargs):
                request = kwargs.get('request')
                if request is None:
                    request = next(a for a in args if isinstance(a, Request))
                self.hit(fn.__name__, request, spec)
                return await fn(*args, **kwargs)
            return wrapper
        return deco


async def rate_limit_exceeded_handler(request: Request, exc: RateLimitExceeded):
    return JSONResponse({'error': f'Rate limit exceeded: {exc.detail}'}, status_code=429)
