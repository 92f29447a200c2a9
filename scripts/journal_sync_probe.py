"""How long the journal's per-block fdatasync takes on this box's ledger filesystem, and how much of it an
early writeback start (sync_file_range(SYNC_FILE_RANGE_WRITE) right after each part of the record is written)
takes off the wait. The verify bench writes a ~8 MB journal record per 2 MB block (csrc/ledger_writer.cpp) and
then waits for its fdatasync (``block:durable`` in the block trace).

    python scripts/journal_sync_probe.py [dir=/tmp] [record_mb=8] [rounds=30]

Prints one JSON line: median ms of the write, and of the fdatasync after it, for
  plain   write the record, fdatasync
  early   write it in 1 MB parts, each followed by sync_file_range(WRITE), then fdatasync
  early+gap  as early, then 2 ms of other work (the verdict) before the fdatasync
"""
import ctypes
import json
import os
import statistics
import subprocess
import sys
import time

libc = ctypes.CDLL(None, use_errno=True)
SFR_WRITE = 2


def sfr(fd, off, n):
    if libc.sync_file_range(fd, ctypes.c_int64(off), ctypes.c_int64(n), SFR_WRITE) != 0:
        raise OSError(ctypes.get_errno(), 'sync_file_range')


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else '/tmp'
    mb = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    path = os.path.join(d, 'journal_sync_probe.bin')
    buf = os.urandom(mb << 20)
    part = 1 << 20
    fd = os.open(path, os.O_RDWR | os.O_CREAT | os.O_TRUNC, 0o644)
    res = {}
    try:
        for mode in ('plain', 'early', 'early+gap') * 1:
            w, s = [], []
            at = 0
            for _ in range(rounds):
                t0 = time.perf_counter()
                if mode == 'plain':
                    os.pwrite(fd, buf, at)
                else:
                    for o in range(0, len(buf), part):
                        os.pwrite(fd, buf[o:o + part], at + o)
                        sfr(fd, at + o, part)
                t1 = time.perf_counter()
                if mode == 'early+gap':
                    while time.perf_counter() - t1 < 0.002:
                        pass
                t2 = time.perf_counter()
                os.fdatasync(fd)
                t3 = time.perf_counter()
                w.append((t1 - t0) * 1e3)
                s.append((t3 - t2) * 1e3)
                at += len(buf)
                if at > (512 << 20):
                    os.ftruncate(fd, 0)
                    os.fdatasync(fd)
                    at = 0
            res[mode] = {'write_ms': round(statistics.median(w), 3), 'fdatasync_ms': round(statistics.median(s), 3),
                         'fdatasync_p90_ms': round(sorted(s)[int(0.9 * len(s))], 3)}
    finally:
        os.close(fd)
        os.unlink(path)
    try:
        fs = subprocess.run(['stat', '-f', '-c', '%T', d], capture_output=True, text=True).stdout.strip()
    except OSError:
        fs = None
    print(json.dumps({'dir': d, 'fs': fs, 'record_mb': mb, 'rounds': rounds, **res}), flush=True)


if __name__ == '__main__':
    main()
