"""Native rotating app.log appender (csrc/log_appender.cpp) behind the node's file log handler."""
import logging
import os

from upow_amd.ops.native import lib
from upow_amd.utils.logger import NativeFileHandler


def test_appender_rotates_between_records(tmp_path):
    path = str(tmp_path / 'app.log')
    app = lib().LogAppender(path, 1000, 3)
    lines = [f'line {i:04d} ' + 'x' * 80 + '\n' for i in range(60)]  # 91 bytes each: ~10 lines per file
    for ln in lines:
        app.write(ln)
    app.flush()
    assert app.rotations >= 3
    app.close()
    files = [path + s for s in ('.3', '.2', '.1', '')]
    kept = ''.join(open(f).read() for f in files if os.path.exists(f))
    assert not os.path.exists(path + '.4')  # backups beyond the count are dropped
    assert kept.endswith(''.join(lines[-5:]))  # newest records last, whole lines, in order
    for f in files:
        if os.path.exists(f):
            data = open(f).read()
            assert len(data) < 1000 + 91 and data.endswith('\n')


def test_native_handler_format_matches_formatter(tmp_path):
    fmt = logging.Formatter('%(asctime)s - %(filename)s - %(levelname)s - %(message)s')
    h = NativeFileHandler(lib().LogAppender(str(tmp_path / 'a.log'), 1 << 20, 2), fmt)
    rec = logging.LogRecord('upow', logging.INFO, '/x/manager.py', 10, 'Added %d transactions', (5,), None)
    h.emit(rec)
    h.flush()
    h.close()
    assert open(tmp_path / 'a.log').read() == fmt.format(rec) + '\n'


def test_descriptor_appender_shares_the_offset_with_direct_writes(tmp_path):
    """The console appender writes through a dup of the descriptor: lines written directly to the
    original fd before and after land after them, never over them."""
    path = str(tmp_path / 'console.txt')
    fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)  # no O_APPEND, like a shell redirect
    os.write(fd, b'first\n')
    app = lib().LogAppender(os.dup(fd))
    for i in range(100):
        app.write(f'rec {i}\n')
    app.flush()
    os.write(fd, b'last\n')
    app.close()
    os.close(fd)
    assert open(path).read() == 'first\n' + ''.join(f'rec {i}\n' for i in range(100)) + 'last\n'


def test_pending_bytes_are_bounded_and_drops_are_reported(tmp_path):
    """the buffer in front of the writer is bounded; lines past it are dropped, counted, and the
    count is written to the log once the writer catches up. ERROR lines are written before write_sync returns."""
    from upow_amd.ops.native import lib
    path = str(tmp_path / 'b.log')
    app = lib().LogAppender(path, 1 << 30, 1)
    app.set_max_pending(4096)
    line = 'x' * 99 + '\n'
    ok = [app.write(line) for _ in range(200)]  # 20 KB in one burst: the writer drains every 20 ms
    assert not all(ok) and app.dropped == ok.count(False)
    app.write_sync('ERROR line\n')
    text = open(path).read()
    assert text.endswith('ERROR line\n') or 'ERROR line\n' in text
    app.flush()
    app.close()
    text = open(path).read()
    assert f'{app.dropped} line(s) dropped' in text and text.count(line) == ok.count(True)
