"""Native tailer (csrc/runtime/tailer.cpp): the perl_tail.pl / File::Tail contract
(perl_tail.pl:13-42) plus what the reference lacked -- long lines, rotation without loss,
committed + fsync'd offsets, a read-ahead ring of caller-owned slots."""
import ctypes
import json
import os
import time

import pytest

from apmbackend_amd import _native

N = _native.load(build_if_missing=False)


def _drain(t, max_polls=50):
    out = []
    for _ in range(max_polls):
        buf, chunks = t.poll()
        if not chunks:
            break
        for fid, b, e in chunks:
            out.append((fid, buf[b:e]))
    return out


def _lines(parts, fid=None):
    data = b"".join(p for f, p in parts if fid is None or f == fid)
    return data.split(b"\n")[:-1]


def test_whole_lines_and_partial_tail(tmp_path):
    p = tmp_path / "a.log"
    p.write_bytes(b"one\ntwo\nthr")
    t = N.Tailer("", 1 << 20, 2)
    t.add(str(p), 0, True, 0)
    assert _lines(_drain(t)) == [b"one", b"two"]
    with open(p, "ab") as f:
        f.write(b"ee\nfour\n")
    assert _lines(_drain(t)) == [b"three", b"four"]


def test_line_longer_than_the_per_file_budget(tmp_path):
    """A 1 MiB line with a 256 KiB batch budget split over 4 files: the line is read whole
    (the budget stretches to its newline) instead of stalling the file forever."""
    files = [tmp_path / f"f{i}.log" for i in range(4)]
    big = b"X" * (1 << 20)
    files[0].write_bytes(b"a\n" + big + b"\nb\n")
    for f in files[1:]:
        f.write_bytes(b"small\n" * 1000)
    t = N.Tailer("", 4 << 20, 2)
    for i, f in enumerate(files):
        t.add(str(f), i, True, i)
    got = _drain(t)
    assert _lines(got, 0) == [b"a", big, b"b"]
    for i in range(1, 4):
        assert len(_lines(got, i)) == 1000


def test_large_reads_are_split_across_the_pool(tmp_path):
    """A file contributing megabytes to one batch is read in 1 MiB pieces by the pool (one pread
    per file left one thread copying most of the batch): the batch is byte-identical, lines
    straddling the piece boundaries included, for every pool size."""
    import random
    rng = random.Random(3)
    files = [tmp_path / f"f{i}.log" for i in range(3)]
    want = []
    for i, f in enumerate(files):
        rows = [(b"%d-%07d " % (i, k)) + b"y" * rng.randint(0, 700) for k in range(12000 if i != 1 else 40)]
        f.write_bytes(b"\n".join(rows) + b"\n")
        want.append(rows)
    assert files[0].stat().st_size > 3 << 20
    for threads in (0, 1, 5):
        t = N.Tailer("", 64 << 20, threads)
        for i, f in enumerate(files):
            t.add(str(f), i, True, i)
        got = _drain(t)
        for i in range(3):
            assert _lines(got, i) == want[i], (threads, i)


def test_line_longer_than_a_batch_is_skipped_and_counted(tmp_path):
    p = tmp_path / "a.log"
    p.write_bytes(b"x\n" + b"Y" * (300 << 10) + b"\nz\n")
    t = N.Tailer("", 256 << 10, 0)
    t.add(str(p), 0, True, 0)
    assert _lines(_drain(t)) == [b"x", b"z"]
    assert t.stats()["overlong_lines_skipped"] == 1


def test_rotation_drains_the_old_inode_first(tmp_path):
    """rename-rotation with unread data in the old file (some written after the rename, through
    the writer's still-open handle): nothing is lost, old lines come before the new file's."""
    p = tmp_path / "server.log"
    w = open(p, "ab", buffering=0)
    w.write(b"old1\nold2\n")
    t = N.Tailer("", 1 << 20, 1)
    t.add(str(p), 7, True, 0)
    assert _lines(_drain(t)) == [b"old1", b"old2"]
    w.write(b"old3\n")
    os.rename(p, tmp_path / "server.log.1")
    w.write(b"old4\nold5-unterminated")  # the writer still holds the old inode
    w.close()
    p.write_bytes(b"new1\nnew2\n")
    got = _lines(_drain(t))
    assert got == [b"old3", b"old4", b"old5-unterminated", b"new1", b"new2"]
    st = t.stats()
    assert st["rotations"] == 1 and st["unterminated_lines_closed"] == 1


def test_truncation_restarts_the_file(tmp_path):
    p = tmp_path / "a.log"
    p.write_bytes(b"aaaa\nbbbb\n")
    t = N.Tailer("", 1 << 20, 0)
    t.add(str(p), 0, True, 0)
    _drain(t)
    p.write_bytes(b"c\n")  # truncate + rewrite, same inode
    assert _lines(_drain(t)) == [b"c"]
    assert t.stats()["truncations"] == 1


def test_pause_file_holds_reads(tmp_path):
    p = tmp_path / "a.log"
    p.write_bytes(b"l1\n")
    pause = tmp_path / "PAUSE"
    pause.write_text("")
    t = N.Tailer(str(pause), 1 << 20, 0)
    t.add(str(p), 0, True, 0)
    assert t.paused() and _drain(t) == []
    pause.unlink()
    assert _lines(_drain(t)) == [b"l1"]


def test_batches_are_canonical_grouped_and_contiguous(tmp_path):
    """Chunks come out grouped by server (group), contiguous from byte 0, each ending in '\\n':
    the engine DMAs such a batch without re-layout (engine.cpp launch_parse fast path)."""
    files = []
    for i, grp in enumerate([2, 0, 1, 0, 2]):
        f = tmp_path / f"f{i}.log"
        f.write_bytes(b"".join(b"line %d %d\n" % (i, k) for k in range(50)))
        files.append((f, grp))
    t = N.Tailer("", 1 << 20, 3)
    for i, (f, g) in enumerate(files):
        t.add(str(f), i, True, g)
    buf, chunks = t.poll()
    groups = [files[fid][1] for fid, _, _ in chunks]
    assert groups == sorted(groups) and [c[0] for c in chunks] == [1, 3, 2, 0, 4]
    pos = 0
    for fid, b, e in chunks:
        assert b == pos and buf[e - 1:e] == b"\n"
        pos = e
    assert pos == len(buf)


def test_offsets_are_committed_escaped_and_persisted(tmp_path):
    d = tmp_path / 'we"ird\\dir'
    d.mkdir()
    p = d / "a.log"
    p.write_bytes(b"1\n2\n")
    t = N.Tailer("", 1 << 20, 0)
    t.add(str(p), 0, True, 0)
    slot = ctypes.create_string_buffer((1 << 20) + 256)
    n, chunks, bid = t.poll_into(ctypes.addressof(slot), 1 << 20)
    assert n == 4
    assert t.offsets()[0][1] == 0  # read but not committed yet
    t.commit(bid)
    assert t.offsets()[0][1] == 4
    out = tmp_path / "offs.json"
    t.save_offsets(str(out))
    assert json.load(open(out)) == {str(p): [4, os.stat(p).st_ino]}
    assert json.loads(t.offsets_json()) == json.load(open(out))
    # restoring a pre-rotation offset (inode gone) starts the new file from 0
    t2 = N.Tailer("", 1 << 20, 0)
    t2.add(str(p), 0, False, 0)
    t2.set_offset(str(p), 4, os.stat(p).st_ino + 12345)
    assert t2.offsets()[0][1] == 0


def test_readahead_ring_over_caller_slots(tmp_path):
    files = [tmp_path / f"f{i}.log" for i in range(3)]
    for f in files:
        f.write_bytes(b"")
    slots = [ctypes.create_string_buffer((64 << 10) + 256) for _ in range(3)]
    t = N.Tailer("", 64 << 10, 2)
    for i, f in enumerate(files):
        t.add(str(f), i, True, i)
    t.start([ctypes.addressof(s) for s in slots], 64 << 10, 5.0)
    want = {i: [] for i in range(3)}
    for k in range(3000):
        i = k % 3
        ln = b"file%d line %05d %s" % (i, k, b"p" * (k % 97))
        want[i].append(ln)
        with open(files[i], "ab") as f:
            f.write(ln + b"\n")
    got = {i: [] for i in range(3)}
    deadline = time.time() + 30
    total = sum(len(v) for v in want.values())
    while sum(len(v) for v in got.values()) < total and time.time() < deadline:
        r = t.next(200.0)
        if r is None:
            continue
        slot, ptr, n, chunks, bid = r
        data = ctypes.string_at(ptr, n)
        for fid, b, e in chunks:
            got[fid] += data[b:e].split(b"\n")[:-1]
        t.release(slot)
        t.commit(bid)
    t.stop()
    assert got == want
    assert [o[1] for o in t.offsets()] == [os.path.getsize(f) for f in files]


def test_idle_read_ahead_does_not_commit_a_waiting_batch(tmp_path):
    """the read-ahead thread's empty polls used to commit every earlier batch,
    including one still sitting in a ready slot, so a checkpoint could record offsets past lines
    the engine never processed.  Offsets now move only with commit(id) of the batch itself."""
    f = tmp_path / "a.log"
    f.write_bytes(b"")
    slots = [ctypes.create_string_buffer((64 << 10) + 256) for _ in range(2)]
    t = N.Tailer("", 64 << 10, 2)
    t.add(str(f), 0, True, 0)
    t.start([ctypes.addressof(s) for s in slots], 64 << 10, 2.0)
    with open(f, "ab") as fh:
        fh.write(b"alpha\nbeta\n")
    deadline = time.time() + 10
    r = None
    while r is None and time.time() < deadline:
        r = t.next(200.0)
    assert r is not None
    slot, ptr, n, chunks, bid = r
    assert ctypes.string_at(ptr, n) == b"alpha\nbeta\n"
    time.sleep(0.2)  # the read-ahead thread polls the idle file ~100 times meanwhile
    assert t.offsets()[0][1] == 0
    t.release(slot)
    time.sleep(0.05)
    assert t.offsets()[0][1] == 0
    t.commit(bid)
    assert t.offsets()[0][1] == 11
    t.stop()
