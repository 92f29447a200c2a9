"""Logging (reference: upow/my_logger.py:8-53, upow/helpers.py:20,24-28).

One process-wide ``'upow'`` logger: rotating file ``app.log`` (5 MB x 100, DEBUG) plus console
(INFO; WARNING with ``--nologs``). The node and miner entry points turn the file on by default
(``UPOW_FILE_LOG=1``, as the reference always writes ``logs/app.log``); library use (tests, benches)
leaves it off unless asked. The directory is ``UPOW_LOG_DIR``, else ``<UPOW_DATA_DIR>/logs``, else
``./logs``.
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
    file_log = os.environ.get('UPOW_FILE_LOG', '0') == '1'
    # the logger's own level is the lowest level any of its handlers writes: without the DEBUG file a debug
    # call returns at isEnabledFor instead of building a record that every handler then drops (~15 us per call;
    # the sync path made one per block, profiles/r6/syncprof200_r6o.txt)
    logger.setLevel(logging.DEBUG if file_log else console.level)
    if not file_log and os.environ.get('UPOW_NATIVE_CONSOLE') == '1':
        # library use that asks for it (bench.py): the console lines go through the native writer thread, as
        # a node's do, instead of a format + write + flush of stderr on the calling thread
        native_console = _native_console(fmt, console.level)
        if native_console is not None:
            logger.removeHandler(console)
            logger.addHandler(native_console)
    if file_log:
        data = os.environ.get('UPOW_DATA_DIR')
        log_dir = os.environ.get('UPOW_LOG_DIR') or (os.path.join(data, 'logs') if data else 'logs')
        try:
            os.makedirs(log_dir, exist_ok=True)
            rank = int(os.environ.get('RANK', '0') or 0)  # cluster followers rotate files of their own
            name = 'app.log' if rank == 0 else f'app.rank{rank}.log'
            fh = RotatingFileHandler(os.path.join(log_dir, name), maxBytes=5 * 1024 * 1024, backupCount=100)
        except OSError:
            return
        fh.setLevel(logging.DEBUG)
        fh.setFormatter(fmt)
        native = _native_handler(fh.baseFilename, fmt)
        if native is not None:
            fh.close()
            logger.addHandler(native)
            # the console too: a synchronous write + flush of stderr per INFO line releases the GIL on the
            # HTTP loop thread at every /push_tx; the same writer thread batches them instead
            native_console = _native_console(fmt, console.level)
            if native_console is not None:
                logger.removeHandler(console)
                logger.addHandler(native_console)
            return
        # no native library: formatting and file I/O on a listener thread
        import atexit
        import queue
        from logging.handlers import QueueHandler, QueueListener
        q: queue.SimpleQueue = queue.SimpleQueue()
        listener = QueueListener(q, fh, respect_handler_level=True)
        listener.start()
        atexit.register(listener.stop)
        logger.addHandler(QueueHandler(q))


class NativeFileHandler(logging.Handler):
    """The rotating app.log through csrc/log_appender.cpp: the record is rendered here in the format above
    (the timestamp text cached per second) and handed to a C++ writer thread that batches, writes and
    rotates. /push_tx logs a line per request; no Python thread has to format or write them, so the HTTP
    loop does not lose the GIL to a logging thread at a four-digit tx rate."""

    def __init__(self, appender, fmt: logging.Formatter):
        super().__init__(logging.DEBUG)
        self.app = appender
        self.setFormatter(fmt)
        self._sec = None
        self._stamp = ''

    def emit(self, record):
        try:
            if record.exc_info or record.exc_text or record.stack_info:
                line = self.format(record)
            else:
                sec = int(record.created)
                if sec != self._sec:
                    import time
                    self._sec, self._stamp = sec, time.strftime('%Y-%m-%d %H:%M:%S', time.localtime(sec))
                line = (f'{self._stamp},{int(record.msecs):03d} - {record.filename} - {record.levelname} - '
                        f'{record.getMessage()}')
            if record.levelno >= logging.CRITICAL:
                # fatal paths (a failed collective, os._exit next): on disk before returning. ERROR lines
                # (rejected txs and blocks, fired on the HTTP loop, possibly at a client's flood rate) stay
                # asynchronous: a stalled disk must not stall the loop once per error
                self.app.write_sync(line + '\n')
            else:
                self.app.write(line + '\n')
        except Exception:
            self.handleError(record)

    def flush(self):
        self.app.flush()

    def close(self):
        try:
            self.app.close()
        finally:
            super().close()


def _native_handler(path: str, fmt: logging.Formatter):
    if os.environ.get('UPOW_NATIVE_LOG', '1') == '0':
        return None
    try:
        from ..ops.native import lib
        app = lib().LogAppender(path, 5 * 1024 * 1024, 100)
    except Exception:
        return None
    import atexit
    h = NativeFileHandler(app, fmt)
    atexit.register(h.close)
    return h


def _native_console(fmt: logging.Formatter, level: int):
    if os.environ.get('UPOW_NATIVE_LOG', '1') == '0' or os.environ.get('UPOW_NATIVE_CONSOLE', '1') == '0':
        return None
    try:
        from ..ops.native import lib
        fd = os.dup(sys.stderr.fileno())
    except Exception:
        return None
    try:
        app = lib().LogAppender(fd)
    except Exception:
        os.close(fd)
        return None
    import atexit
    h = NativeFileHandler(app, fmt)
    h.setLevel(level)
    atexit.register(h.close)
    return h


def get_logger(name: str = 'upow') -> logging.Logger:
    _configure()
    return logging.getLogger('upow')


class CustomLogger:
    """API-compatible shim of the reference's singleton class."""

    def __init__(self, module_name: str = 'upow', *args, **kwargs):
        self.logger = get_logger(module_name)

    def get_logger(self):
        return self.logger
