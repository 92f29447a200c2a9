"""Logging (reference: upow/my_logger.py:8-53, upow/helpers.py:20,24-28).

One process-wide ``'upow'`` logger: rotating file ``logs/app.log`` (5 MB x 100, DEBUG) plus console
(INFO; WARNING with ``--nologs``). The file handler is only attached when ``UPOW_LOG_DIR`` (default
``logs``) is writable, so library use (tests, benches) does not litter the working directory unless
``UPOW_FILE_LOG=1``.
"""
from __future__ import annotations

import logging
import os
import sys
from logging.handlers import RotatingFileHandler

_configured = False


def _configure():
    global _configured
    if _configured:
        return
    _configured = True
    logger = logging.getLogger('upow')
    logger.setLevel(logging.DEBUG)
    logger.propagate = False
    fmt = logging.Formatter('%(asctime)s - %(filename)s - %(levelname)s - %(message)s')
    console = logging.StreamHandler()
    level = os.environ.get('UPOW_LOG_LEVEL')
    if level:
        console.setLevel(getattr(logging, level.upper(), logging.INFO))
    else:
        console.setLevel(logging.WARNING if '--nologs' in sys.argv else logging.INFO)
    console.setFormatter(fmt)
    logger.addHandler(console)
    if os.environ.get('UPOW_FILE_LOG', '0') == '1':
        log_dir = os.environ.get('UPOW_LOG_DIR', 'logs')
        try:
            os.makedirs(log_dir, exist_ok=True)
            fh = RotatingFileHandler(os.path.join(log_dir, 'app.log'), maxBytes=5 * 1024 * 1024, backupCount=100)
            fh.setLevel(logging.DEBUG)
            fh.setFormatter(fmt)
            logger.addHandler(fh)
        except OSError:
            pass


def get_logger(name: str = 'upow') -> logging.Logger:
    _configure()
    return logging.getLogger('upow')


class CustomLogger:
    """API-compatible shim of the reference's singleton class."""

    def __init__(self, module_name: str = 'upow', *args, **kwargs):
        self.logger = get_logger(module_name)

    def get_logger(self):
        return self.logger
