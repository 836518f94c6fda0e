"""The JNI glue of the KP:52 processor swap (integration/jni/kme_jni.c), driven without a JVM.

There is no JDK in this image, so libkme_jni_check.so is kme_jni.c built against
tests/jni_stub/jni.h, and the JNIEnv it receives is a function table made here with ctypes: Java
arrays and direct ByteBuffers are numpy arrays, exceptions are recorded.  The GPU tests drive the
processor's own protocol -- two slots of direct buffers over the glue's registered memory, an epoch
submitted per slot, poll, complete the oldest (kme_submit_epoch_host / kme_poll / kme_wait /
kme_expand_rows) -- and compare the MatchOut rows with the oracle's tape record by record ("IN",
maker fill, taker fill ..., "OUT"; KP:97, 265-274, 124), including the rows of the records before a
fault, and the commit / restart contract: a crash after a commit point, a restart
from its checkpoint, re-delivery from the committed offset.
"""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from kme import workloads as W

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "integration", "jni", "kme_jni.c")
CHECK_LIB = os.path.join(ROOT, "integration", "jni", "libkme_jni_check.so")
SYMBOLS = ["create", "destroy", "buffer", "submit", "poll", "complete", "forwarded", "statusText", "checkpoint",
           "restore", "stateChunks", "inspect", "shardStatus"]
ROW_DTYPE = np.dtype([("oid", "<i8"), ("aid", "<i8"), ("sid", "<i8"), ("prev", "<i8"), ("action", "<i4"),
                      ("price", "<i4"), ("size", "<i4"), ("kind", "u1"), ("has_prev", "u1"), ("_pad", "u1", 2)])
assert ROW_DTYPE.itemsize == 48


class FakeJni:
    """A JNIEnv (the stub header's member order) over Python objects."""

    def __init__(self):
        self.objs = {}
        self.thrown = []
        self._keep = []
        P, V, I, L = C.c_void_p, None, C.c_int32, C.c_int64
        fields = [
            ("FindClass", C.CFUNCTYPE(P, P, C.c_char_p), lambda env, name: self._new(("class", name))),
            ("ThrowNew", C.CFUNCTYPE(I, P, P, C.c_char_p), self._throw),
            ("GetArrayLength", C.CFUNCTYPE(I, P, P), lambda env, a: len(self.objs[a])),
            ("GetPrimitiveArrayCritical", C.CFUNCTYPE(P, P, P, P), lambda env, a, c: self.objs[a].ctypes.data),
            ("ReleasePrimitiveArrayCritical", C.CFUNCTYPE(V, P, P, P, I), lambda env, a, p, m: None),
            ("SetLongArrayRegion", C.CFUNCTYPE(V, P, P, I, I, C.POINTER(L)), self._set_long),
            ("NewStringUTF", C.CFUNCTYPE(P, P, C.c_char_p), lambda env, s: self._new(s.decode())),
            ("GetStringUTFChars", C.CFUNCTYPE(P, P, P, P), self._utf),
            ("ReleaseStringUTFChars", C.CFUNCTYPE(V, P, P, P), lambda env, s, p: None),
            ("GetDirectBufferAddress", C.CFUNCTYPE(P, P, P), lambda env, b: self.objs[b].ctypes.data),
            ("GetDirectBufferCapacity", C.CFUNCTYPE(L, P, P), lambda env, b: self.objs[b].nbytes),
            ("NewDirectByteBuffer", C.CFUNCTYPE(P, P, P, L), self._new_direct),
        ]

        class Table(C.Structure):
            _fields_ = [(n, t) for n, t, _ in fields]

        self.table = Table(*[t(f) for _, t, f in fields])
        self.fp = C.pointer(self.table)
        self.env = C.cast(C.pointer(self.fp), C.c_void_p)

    def _new(self, obj):
        h = 0x1000 + 16 * (len(self.objs) + 1)
        self.objs[h] = obj
        return h

    def _throw(self, env, cls, msg):
        self.thrown.append(msg.decode())
        return 0

    def _set_long(self, env, a, start, n, buf):
        self.objs[a][start:start + n] = np.ctypeslib.as_array(buf, shape=(n,))

    def _new_direct(self, env, addr, cap):
        """ByteBuffer over native memory: a uint8 view of it."""
        return self._new(np.ctypeslib.as_array((C.c_uint8 * cap).from_address(addr)))

    def _utf(self, env, s, c):
        b = C.create_string_buffer(self.objs[s].encode())
        self._keep.append(b)
        return C.addressof(b)

    def arr(self, a):
        return self._new(np.ascontiguousarray(a))

    def direct(self, nbytes, dtype):
        """A direct ByteBuffer: page-aligned native memory, as ByteBuffer.allocateDirect gives."""
        raw = np.zeros(nbytes + 4096, np.uint8)
        off = (-raw.ctypes.data) % 4096
        view = raw[off:off + nbytes].view(dtype)
        self._keep.append(raw)
        return self._new(view), view


def _lib():
    if not os.path.exists(CHECK_LIB):
        pytest.skip("integration/jni/libkme_jni_check.so not built (make -C kafka-matching-engine_amd/csrc)")
    # libkme through kme.lib() first: it imports torch, so the glue's libkme binds torch's HIP
    # runtime (a glue loaded first maps a second HIP runtime, and torch then sees no GPU)
    import kme
    kme.lib()
    lib = C.CDLL(CHECK_LIB)
    P, I, L = C.c_void_p, C.c_int32, C.c_int64
    lib.Java_GpuMatchingEngine_create.argtypes = [P, P, I, I, I, L, I, I, I, I, I, L]
    lib.Java_GpuMatchingEngine_create.restype = L
    lib.Java_GpuMatchingEngine_destroy.argtypes = [P, P, L]
    lib.Java_GpuMatchingEngine_buffer.argtypes = [P, P, L, I, I]
    lib.Java_GpuMatchingEngine_buffer.restype = P
    lib.Java_GpuMatchingEngine_forwarded.argtypes = [P, P, L, I]
    lib.Java_GpuMatchingEngine_forwarded.restype = None
    lib.Java_GpuMatchingEngine_checkpoint.argtypes = [P, P, L, P, L, L, P]
    lib.Java_GpuMatchingEngine_checkpoint.restype = I
    lib.Java_GpuMatchingEngine_restore.argtypes = [P, P, L, P, P]
    lib.Java_GpuMatchingEngine_restore.restype = I
    lib.Java_GpuMatchingEngine_submit.argtypes = [P, P, L, I, I]
    lib.Java_GpuMatchingEngine_submit.restype = I
    lib.Java_GpuMatchingEngine_poll.argtypes = [P, P, L]
    lib.Java_GpuMatchingEngine_poll.restype = I
    lib.Java_GpuMatchingEngine_complete.argtypes = [P, P, L, I, P]
    lib.Java_GpuMatchingEngine_complete.restype = I
    lib.Java_GpuMatchingEngine_statusText.argtypes = [P, P, I]
    lib.Java_GpuMatchingEngine_statusText.restype = P
    lib.Java_GpuMatchingEngine_stateChunks.argtypes = [P, P, L, P, I, P, P]
    lib.Java_GpuMatchingEngine_stateChunks.restype = I
    lib.Java_GpuMatchingEngine_inspect.argtypes = [P, P, P, P]
    lib.Java_GpuMatchingEngine_inspect.restype = I
    lib.Java_GpuMatchingEngine_shardStatus.argtypes = [P, P, C.c_int64, P]
    lib.Java_GpuMatchingEngine_shardStatus.restype = I
    return lib


def test_jni_glue_compiles_against_kme_h():
    subprocess.run(["gcc", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "tests", "jni_stub"),
                    "-I", os.path.join(ROOT, "include"), SRC], check=True)


def test_jni_glue_exports_and_cpu_paths():
    lib = _lib()
    for s in SYMBOLS:
        assert hasattr(lib, "Java_GpuMatchingEngine_" + s)
    j = FakeJni()
    txt = lib.Java_GpuMatchingEngine_statusText(j.env, None, 4)
    assert "UNFUNDED" in j.objs[txt].upper() or "fund" in j.objs[txt].lower()
    # an invalid configuration throws IllegalStateException before touching the device
    assert lib.Java_GpuMatchingEngine_create(j.env, None, 1, 65, 0, 1 << 16, 1 << 16, 256, 0, 0, 1, 1 << 16) == 0
    assert j.thrown and "maxEpoch" in j.thrown[0]


COLUMNS = (("action", np.int32), ("oid", np.int64), ("aid", np.int64), ("sid", np.int64), ("price", np.int32),
           ("size", np.int32))


def slot_views(lib, j, h):
    """GpuMatchingEngine.init's buffer() calls: per slot the six columns and the rows, as views."""
    cols, rows = [], []
    for slot in range(2):
        views = {}
        for c, (name, dt) in enumerate(COLUMNS):
            views[name] = j.objs[lib.Java_GpuMatchingEngine_buffer(j.env, None, h, slot, c)].view(dt)
        cols.append(views)
        rows.append(j.objs[lib.Java_GpuMatchingEngine_buffer(j.env, None, h, slot, 6)].view(ROW_DTYPE))
    for v in cols[0].values():
        assert v.ctypes.data % 4096 == 0            # page-aligned: no registration shares a page
    return cols, rows


class Proc:
    """GpuMatchingEngine.java's protocol over the JNI glue: two slots of direct buffers, epochs
    submitted asynchronously, the oldest completed first and its rows read back."""

    def __init__(self, lib, j, h, epoch, max_trades):
        self.lib, self.j, self.h, self.epoch = lib, j, h, epoch
        self.cols, self.rows = slot_views(lib, j, h)
        assert all(len(v) == epoch for v in self.cols[0].values())
        assert len(self.rows[0]) == 2 * epoch + 2 * max_trades
        self.status = j.arr(np.zeros(4, np.int64))
        self.pending = []          # (slot, n) in submission order

    def submit(self, slot, part):
        for name, v in self.cols[slot].items():
            v[:len(part)] = getattr(part, name)
        rc = self.lib.Java_GpuMatchingEngine_submit(self.j.env, None, self.h, slot, len(part))
        assert rc == 0, rc
        self.pending.append(slot)

    def complete(self):
        slot = self.pending.pop(0)
        m = self.lib.Java_GpuMatchingEngine_complete(self.j.env, None, self.h, slot, self.status)
        assert not self.j.thrown, self.j.thrown
        out = self.rows[slot][:m].copy(), self.j.objs[self.status].copy()
        self.lib.Java_GpuMatchingEngine_forwarded(self.j.env, None, self.h, slot)
        return out


def _as_tape(rows, rec_dtype):
    t = np.zeros(len(rows), rec_dtype)
    t["key"] = (rows["kind"] != 0).astype(np.int32)
    for f in ("action", "oid", "aid", "sid", "price", "size", "prev"):
        t[f] = rows[f]
    t["has_prev"] = rows["has_prev"]
    return t


def _cmp_fields(got, want):
    names = ["key", "action", "oid", "aid", "sid", "price", "size", "prev", "has_prev"]
    assert len(got) == len(want)
    for f in names:
        d = np.flatnonzero(got[f] != want[f])
        assert len(d) == 0, f"row {d[0]} field {f}: {got[d[0]]} != {want[d[0]]}"


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["funded", "exact"])
def test_jni_epochs_in_flight_equal_oracle_tape(oracle_mod, mode):
    """Two epochs in flight at a time (the processor fills one slot while the other runs), poll until
    the oldest is done, complete it: the rows of every epoch in order equal the oracle's tape."""
    import time

    lib = _lib()
    j = FakeJni()
    if mode == "funded":
        setup = W.funded_setup(256, range(1, 65))
        orders = W.Orders.concat([setup, W.uniform(40_000, n_symbols=64, n_accounts=256, seed=11)])
        # default processor flags: the exact ledger, serial fallback where the proof fails
        h = lib.Java_GpuMatchingEngine_create(j.env, None, 1, 65, 1 << 13, 1 << 16, 1 << 15, 256, 3, 0, 1, 1 << 16)
        epoch, max_trades = 1 << 13, 1 << 15
    else:
        orders = W.exchange_test(6_000, seed=5)
        h = lib.Java_GpuMatchingEngine_create(j.env, None, 0, 8, 1 << 12, 1 << 14, 1 << 14, 0, 0, 0, 1, 1 << 16)
        epoch, max_trades = 1 << 12, 1 << 14
    assert h and not j.thrown, j.thrown
    p = Proc(lib, j, h, epoch, max_trades)
    assert lib.Java_GpuMatchingEngine_poll(j.env, None, h) == 1      # nothing in flight
    got, polls = [], 0
    parts = [orders.slice(a, min(len(orders), a + epoch)) for a in range(0, len(orders), epoch)]
    for k, part in enumerate(parts):
        if len(p.pending) == 2:
            t0 = time.time()
            while lib.Java_GpuMatchingEngine_poll(j.env, None, h) == 0:   # the punctuator's poll
                polls += 1
                assert time.time() - t0 < 60
            rows, st = p.complete()
            assert st[0] == 0 and st[3] > 0
            got.append(_as_tape(rows, oracle_mod.REC_DTYPE))
        p.submit(k % 2, part)
    while p.pending:
        rows, st = p.complete()
        assert st[0] == 0
        got.append(_as_tape(rows, oracle_mod.REC_DTYPE))
    lib.Java_GpuMatchingEngine_destroy(j.env, None, h)
    o = oracle_mod.Oracle()
    o.process(orders)
    _cmp_fields(np.concatenate(got), o.tape())


@pytest.mark.gpu
def test_jni_forwards_the_records_before_a_fault(oracle_mod):
    """A REMOVE_SYMBOL of a non-empty book never returns in the reference (KP:341-353): the rows of
    the records before it are produced, status names the fault, its index and n_effective."""
    lib = _lib()
    j = FakeJni()
    setup = W.funded_setup(16, range(1, 9))
    body = W.uniform(3000, n_symbols=8, n_accounts=16, seed=2)
    bad = W.Orders.from_rows([(W.REMOVE_SYMBOL, 0, 0, 3, 0, 0)])
    orders = W.Orders.concat([body.slice(0, 2000), bad, body.slice(2000, 3000)])
    h = lib.Java_GpuMatchingEngine_create(j.env, None, 1, 9, 1 << 13, 1 << 14, 1 << 14, 16, 0, 0, 1, 1 << 16)
    assert h
    p = Proc(lib, j, h, 1 << 13, 1 << 14)
    p.submit(0, setup)
    _, st0 = p.complete()
    assert st0[0] == 0
    p.submit(1, orders)
    rows, st = p.complete()
    assert st[0] == 3 and st[2] == 2000 and st[3] == 2000      # KME_E_DOMAIN at the REMOVE_SYMBOL
    o = oracle_mod.Oracle()
    o.process(setup)
    o.clear_tape()
    o.process(orders.slice(0, 2000))
    _cmp_fields(_as_tape(rows, oracle_mod.REC_DTYPE), o.tape())
    lib.Java_GpuMatchingEngine_destroy(j.env, None, h)


class IllegalState(Exception):
    """java.lang.IllegalStateException thrown by the processor (the stream thread dies)."""


class JavaProcessor:
    """GpuMatchingEngine.java statement for statement (init / process / flush / completeOldest /
    forwardReady / punctuate / commitPoint / close) over the JNI glue.  Each record carries its Kafka
    offset (context.offset()); forwarded rows are collected in `out`; commit_point() is the commit
    hook's StateStore.flush(), which Kafka Streams calls before it commits the consumed offsets.
    `commit_log` is the changelogged commit-log store (a dict that survives the process: Kafka
    Streams restores it from its changelog wherever the task runs): the record naming the committed
    checkpoint, and the checkpoint file's chunks keyed by index and content hash (the state changelog:
    a restart whose state directory lost the file rebuilds it from them)."""

    CHUNK_BYTES = 512 << 10

    def __init__(self, lib, j, path, epoch, max_trades, create_args, commit_log=None, chunk_bytes=None):
        self.lib, self.j, self.path, self.epoch = lib, j, str(path), epoch
        if chunk_bytes:
            self.CHUNK_BYTES = chunk_bytes
        self.commit_log = {} if commit_log is None else commit_log
        self.h = lib.Java_GpuMatchingEngine_create(j.env, None, *create_args)
        assert self.h and not j.thrown, j.thrown
        self.cols, self.rows = slot_views(lib, j, self.h)
        self.count, self.busy, self.fill, self.oldest, self.inflight = [0, 0], [False, False], 0, 0, 0
        self.ready, self.ready_rows = [], [0, 0]
        self.ready_status = [j.arr(np.zeros(4, np.int64)) for _ in range(2)]
        self.last_offset = self.skip_through = self.checkpointed = -1
        self.generation = 0
        self.out = []
        want = self.commit_log.get("checkpoint")          # (generation, offset, bytes, digest, chunk bytes, hashes)
        self.chunk_hashes = list(want[5]) if want is not None else []
        if want is not None and not self._is_committed(self.path, want):
            self._rebuild_from_log(want)                    # the task moved, or an older file
        if os.path.exists(self.path):
            r = j.arr(np.zeros(9, np.int64))
            rc = lib.Java_GpuMatchingEngine_restore(j.env, None, self.h, _jstr(j, self.path), r)
            if rc != 0:
                self._fail(f"kme restore: {rc}")
            o = j.objs[r]
            if want is not None and (o[6] < want[0] or (o[6] == want[0] and (o[7] != want[2] or o[8] != want[3]))):
                self._fail(f"checkpoint generation {o[6]} is not the committed one {want}")
            self.generation = int(o[6])
            self.skip_through = self.checkpointed = self.last_offset = int(o[0])
            if want is not None and self._is_committed(self.path, want):
                self._state_chunks(int(o[7]))               # (the chunks the changelog holds)
            for k in range(int(o[1])):
                s = int(o[2 + 2 * k])
                self.ready_rows[s] = int(o[3 + 2 * k])
                j.objs[self.ready_status[s]][:] = 0
                self.busy[s] = True
                self.ready.append(s)
        elif want is not None:
            self._fail(f"the commit log names checkpoint generation {want[0]} but neither {self.path} nor the chunks hold it")

    @staticmethod
    def _chunk_key(k, h):
        return f"c:{k}:{h & 0xFFFFFFFFFFFFFFFF:x}"

    def _is_committed(self, path, want):
        if not os.path.exists(path):
            return False
        t = self.j.arr(np.zeros(3, np.int64))
        rc = self.lib.Java_GpuMatchingEngine_inspect(self.j.env, None, _jstr(self.j, str(path)), t)
        return rc == 0 and int(self.j.objs[t][0]) == want[2] and int(self.j.objs[t][2]) == want[3]

    def shard_status(self):
        """GpuMatchingEngine.shardStatus(): None for one engine, else the kme_multi_info fields."""
        t = self.j.arr(np.zeros(8, np.int64))
        if self.lib.Java_GpuMatchingEngine_shardStatus(self.j.env, None, self.h, t) != 0:
            return None
        keys = ("n_engines", "consolidated", "can_consolidate", "failed", "history_records", "history_cap",
                "history_saved", "generation")
        return dict(zip(keys, (int(x) for x in self.j.objs[t])))

    def _rebuild_from_log(self, want):
        if want[4] != self.CHUNK_BYTES:
            return
        parts = [self.commit_log.get(self._chunk_key(k, h)) for k, h in enumerate(want[5])]
        if any(b is None for b in parts):
            return
        tmp = self.path + ".log"
        with open(tmp, "wb") as f:
            f.write(b"".join(parts))
        if self._is_committed(tmp, want):
            os.replace(tmp, self.path)

    def _state_chunks(self, file_bytes):
        n = (file_bytes + self.CHUNK_BYTES - 1) // self.CHUNK_BYTES
        hs, ch = self.j.arr(np.zeros(max(n, 1), np.int64)), self.j.arr(np.zeros(n + 1, np.int64))
        got = self.lib.Java_GpuMatchingEngine_stateChunks(self.j.env, None, self.h, _jstr(self.j, self.path), self.CHUNK_BYTES, hs, ch)
        assert got == n, (got, n)
        changed = self.j.objs[ch]
        return [int(x) for x in self.j.objs[hs][:n]], [int(x) for x in changed[1:1 + int(changed[0])]]

    def _fail(self, msg):
        """init() throws; the task is torn down (close -> destroy)."""
        self.lib.Java_GpuMatchingEngine_destroy(self.j.env, None, self.h)
        self.h = 0
        raise IllegalState(msg)

    def process(self, offset, rec):
        self.forward_ready()
        if offset <= self.skip_through:
            return
        while self.busy[self.fill]:
            if self.ready:
                self.forward_ready()
            else:
                self.complete_oldest(True)
        n = self.count[self.fill]
        for name, v in self.cols[self.fill].items():
            v[n] = rec[name]
        self.count[self.fill] = n + 1
        self.last_offset = offset
        if self.count[self.fill] == self.epoch:
            self.flush()

    def flush(self):
        if self.count[self.fill] == 0:
            return
        while self.inflight == 2:
            self.complete_oldest(True)
        rc = self.lib.Java_GpuMatchingEngine_submit(self.j.env, None, self.h, self.fill, self.count[self.fill])
        assert rc == 0, rc
        if self.inflight == 0:
            self.oldest = self.fill
        self.busy[self.fill] = True
        self.inflight += 1
        self.fill ^= 1

    def complete_oldest(self, forward):
        s = self.oldest
        self.ready_rows[s] = self.lib.Java_GpuMatchingEngine_complete(self.j.env, None, self.h, s, self.ready_status[s])
        assert not self.j.thrown, self.j.thrown
        self.ready.append(s)
        self.inflight -= 1
        self.oldest = s ^ 1
        if forward:
            self.forward_ready()

    def forward_ready(self):
        while self.ready:
            s = self.ready.pop(0)
            self.out.append(self.rows[s][:self.ready_rows[s]].copy())
            self.lib.Java_GpuMatchingEngine_forwarded(self.j.env, None, self.h, s)
            self.busy[s] = False
            self.count[s] = 0
            assert self.j.objs[self.ready_status[s]][0] == 0, self.j.objs[self.ready_status[s]]

    def punctuate(self):
        self.forward_ready()
        while self.inflight > 0:
            p = self.lib.Java_GpuMatchingEngine_poll(self.j.env, None, self.h)
            assert p >= 0
            if p == 0:
                break
            self.complete_oldest(True)
        if self.inflight < 2 and self.count[self.fill] > 0 and not self.busy[self.fill]:
            self.flush()

    def commit_point(self):
        if self.h == 0 or self.last_offset == self.checkpointed:
            return
        self.flush()
        while self.inflight > 0:
            self.complete_oldest(False)
        info = self.j.arr(np.zeros(2, np.int64))
        rc = self.lib.Java_GpuMatchingEngine_checkpoint(self.j.env, None, self.h, _jstr(self.j, self.path), self.last_offset,
                                                        self.generation + 1, info)
        assert rc == 0, rc
        self.generation += 1
        fb, dg = (int(x) for x in self.j.objs[info])
        assert fb == os.path.getsize(self.path)
        # the state changelog: the chunks that changed, then the record naming every chunk, then the
        # keys the record no longer names
        hashes, changed = self._state_chunks(fb)
        with open(self.path, "rb") as f:
            for k in changed:
                f.seek(k * self.CHUNK_BYTES)
                self.commit_log[self._chunk_key(k, hashes[k])] = f.read(self.CHUNK_BYTES)
        self.chunks_put = len(changed)
        self.commit_log["checkpoint"] = (self.generation, self.last_offset, fb, dg, self.CHUNK_BYTES, tuple(hashes))
        for k, h in enumerate(self.chunk_hashes):
            if k >= len(hashes) or hashes[k] != h:
                self.commit_log.pop(self._chunk_key(k, h), None)
        self.chunk_hashes = hashes
        self.checkpointed = self.last_offset

    def close(self):
        self.forward_ready()
        self.flush()
        while self.inflight > 0:
            self.complete_oldest(True)
        self.commit_point()
        self.lib.Java_GpuMatchingEngine_destroy(self.j.env, None, self.h)
        self.h = 0

    def crash(self):
        """The JVM dies: nothing more is forwarded, nothing flushed (the native memory goes with it)."""
        self.lib.Java_GpuMatchingEngine_destroy(self.j.env, None, self.h)
        self.h = 0

    def rows_out(self):
        return np.concatenate(self.out) if self.out else np.zeros(0, ROW_DTYPE)


def _jstr(j, s):
    return j._new(s)


def _records(orders, k):
    return {f: getattr(orders, f)[k] for f in ("action", "oid", "aid", "sid", "price", "size")}


@pytest.mark.gpu
@pytest.mark.parametrize("mode,redeliver", [("funded", "committed"), ("funded", "previous"), ("exact", "committed")])
def test_crash_after_commit_restarts_without_losing_output(oracle_mod, tmp_path, mode, redeliver):
    """The commit / restart contract (KP:29-49, 125).  Records are taken with their
    Kafka offsets; two commit points (the commit hook's flush, which Kafka Streams runs before it
    commits the offsets) leave epochs completed but not forwarded and one partly filled; more records
    are taken, some forwarded, some buffered, then the process dies.  A new processor restores the
    checkpoint and Kafka re-delivers from the committed offset ("committed"), or from the commit
    before it when the last offset commit did not land ("previous": the restored checkpoint is ahead
    of Kafka, those records are skipped).  The rows forwarded before the commit point plus everything
    forwarded after the restart are the oracle's uninterrupted tape; what was forwarded between the
    commit point and the crash comes again, and only that (at least once).  The books (and the exact
    ledger) at the end equal the oracle's."""
    lib = _lib()
    j = FakeJni()
    if mode == "funded":
        setup = W.funded_setup(256, range(1, 65))
        orders = W.Orders.concat([setup, W.uniform(60_000, n_symbols=64, n_accounts=256, seed=23)])
        epoch, max_trades = 1 << 12, 1 << 14
        args = (1, 65, epoch, 1 << 16, max_trades, 256, 3, 0, 1, 1 << 16)   # the default flags: exact ledger + fallback
    else:
        orders = W.exchange_test(12_000, seed=9)
        epoch, max_trades = 1 << 11, 1 << 13
        args = (0, 8, epoch, 1 << 14, max_trades, 0, 0, 0, 1, 1 << 16)
    n = len(orders)
    ckpt = tmp_path / "kme-0_0.ckpt"
    log = {}
    p = JavaProcessor(lib, j, ckpt, epoch, max_trades, args, log)
    c0, c1, crash_at = int(n * 0.3) + 17, int(n * 0.55) + 5, int(n * 0.8) + 3
    committed = {}
    for k in range(crash_at):
        p.process(k, _records(orders, k))
        if k % 1500 == 700:
            p.punctuate()
        if k in (c0, c1):
            p.commit_point()
            committed[k] = sum(len(x) for x in p.out)     # rows forwarded before the commit point
            assert p.ready or p.count[p.fill] == 0
    first = p.rows_out()
    p.crash()
    q = JavaProcessor(lib, j, ckpt, epoch, max_trades, args, log)
    assert q.skip_through == c1 and q.generation == 2
    start = (c1 if redeliver == "committed" else c0) + 1
    for k in range(start, n):
        q.process(k, _records(orders, k))
        if k % 2000 == 1000:
            q.punctuate()
    # the books and ledger at the end, read through the engine the glue holds (its first field)
    eng = C.c_void_p.from_address(q.h).value
    import kme
    L = kme.lib()
    q.forward_ready()
    q.flush()
    while q.inflight:
        q.complete_oldest(True)
    books = _snapshot(L, L.kme_snapshot_books, eng)
    ledger = _snapshot(L, L.kme_snapshot_ledger, eng)
    q.close()
    second = q.rows_out()
    F = committed[c1]
    o = oracle_mod.Oracle()
    o.process(orders)
    got = np.concatenate([first[:F], second])
    _cmp_fields(_as_tape(got, oracle_mod.REC_DTYPE), o.tape())
    dup = first[F:]
    assert len(dup) > 0                                        # something was forwarded after the commit point
    _cmp_fields(_as_tape(second[:len(dup)], oracle_mod.REC_DTYPE), _as_tape(dup, oracle_mod.REC_DTYPE))
    assert books == o.dump_books()
    assert ledger == o.dump_ledger()


def _snapshot(L, fn, eng):
    p = C.c_void_p()
    n = C.c_size_t(0)
    assert fn(C.c_void_p(eng), C.byref(p), C.byref(n)) == 0
    try:
        return C.string_at(p, n.value).decode()
    finally:
        L.kme_free(p)


@pytest.mark.gpu
def test_checkpoint_of_another_processor_is_refused(kme_mod, tmp_path):
    """restore() takes only checkpoints with the processor's record (a bare kme_checkpoint file is
    refused), and a file of another geometry leaves the fresh engine untouched."""
    lib = _lib()
    j = FakeJni()
    args = (1, 9, 1 << 10, 1 << 12, 1 << 12, 16, 0, 0, 1, 1 << 12)
    h = lib.Java_GpuMatchingEngine_create(j.env, None, *args)
    eng = kme_mod.Engine(kme_mod.default_config(kme_mod.MODE_FUNDED, max_symbols=9, max_epoch=1 << 10,
                                                max_resting=1 << 12, max_trades=1 << 12, max_accounts=16,
                                                ledger_capacity=1 << 12))
    bare = tmp_path / "bare.ckpt"
    eng.checkpoint(str(bare))
    r = j.arr(np.zeros(9, np.int64))
    assert lib.Java_GpuMatchingEngine_restore(j.env, None, h, _jstr(j, str(bare)), r) == 1     # KME_E_INVALID
    other = kme_mod.Engine(kme_mod.default_config(kme_mod.MODE_FUNDED, max_symbols=17, max_epoch=1 << 10,
                                                  max_resting=1 << 12, max_trades=1 << 12, max_accounts=16))
    odd = tmp_path / "odd.ckpt"
    other.checkpoint_app(str(odd), b"x" * 40)
    assert lib.Java_GpuMatchingEngine_restore(j.env, None, h, _jstr(j, str(odd)), r) == 1
    assert other.restore_app(str(odd)) == b"x" * 40
    lib.Java_GpuMatchingEngine_destroy(j.env, None, h)
    eng.close()
    other.close()


def _drive(p, orders, start=0, end=None, punct=1500):
    end = len(orders) if end is None else end
    for k in range(start, end):
        p.process(k, _records(orders, k))
        if k % punct == punct // 2:
            p.punctuate()


@pytest.mark.gpu
@pytest.mark.parametrize("crash", [False, True])
def test_multi_gpu_drop_in_equals_the_single_partition_tape(oracle_mod, tmp_path, crash):
    """Round-3 verdict: the drop-in over N engines (kme_multi: the router's symbol split, one engine per
    shard, credit re-split before every epoch, results merged into input order through the router's
    index).  Four shard engines on GPU 0 (nDevices = -4) behind one processor: its MatchOut rows equal
    the oracle's single-partition tape (topic.js:17-18, KP:52) -- and across a crash and restart from
    the commit point (every shard's checkpoint, the router's directory rebuilt from the resting
    orders) as for one engine."""
    lib = _lib()
    j = FakeJni()
    setup = W.funded_setup(256, range(1, 129))
    orders = W.Orders.concat([setup, W.uniform(60_000, n_symbols=128, n_accounts=256, seed=31)])
    epoch, max_trades = 1 << 12, 1 << 14
    args = (1, 129, epoch, 1 << 16, max_trades, 256, 0, 0, -4, 1 << 12)   # FUNDED, flags 0, 4 shards on GPU 0
    ckpt = tmp_path / "multi.ckpt"
    p = JavaProcessor(lib, j, ckpt, epoch, max_trades, args)
    n = len(orders)
    if not crash:
        _drive(p, orders)
        p.close()
        got = p.rows_out()
    else:
        c1, crash_at = int(n * 0.5) + 11, int(n * 0.7) + 5
        _drive(p, orders, 0, c1 + 1)
        p.commit_point()
        F = sum(len(x) for x in p.out)
        _drive(p, orders, c1 + 1, crash_at)
        first = p.rows_out()
        p.crash()
        q = JavaProcessor(lib, j, ckpt, epoch, max_trades, args, p.commit_log)
        assert q.skip_through == c1
        _drive(q, orders, c1 + 1, n)
        q.close()
        got = np.concatenate([first[:F], q.rows_out()])
    o = oracle_mod.Oracle()
    o.process(orders)
    _cmp_fields(_as_tape(got, oracle_mod.REC_DTYPE), o.tape())


@pytest.mark.gpu
@pytest.mark.parametrize("rebalance,funding,flags", [(True, 1.5, 0), (False, 1.5, 0), (True, 1.25, 3), (False, 1.25, 3)])
def test_multi_gpu_drop_in_re_splits_credit(oracle_mod, tmp_path, monkeypatch, rebalance, funding, flags):
    """Every account funded with 1.5x its single-engine need over the whole stream, booked as a
    quarter on each of four shards.  The drop-in re-splits the pooled credit before every epoch, so
    every epoch stays provable and the tape is the oracle's; with re-splitting off
    (KME_MULTI_REBALANCE_EVERY=0) some shard's share runs dry and the processor fails (UNFUNDED).
    (A numpy model of the proof over this stream: the static split fails from epoch 6 at 1.5x, the
    re-split holds at 1.5x; at 1.25x the 2^14-record epochs leave too few orders per account and
    shard for the demand weights to follow, and a few pairs run dry.)  At 1.25x with the drop-in's
    default flags (exact ledger + serial fallback) a shard running dry is not fatal: the stream
    consolidates onto one exact engine and the tape is still the oracle's, re-split or not."""
    monkeypatch.setenv("KME_MULTI_REBALANCE_EVERY", "1" if rebalance else "0")
    lib = _lib()
    j = FakeJni()
    n_sym, n_acc, E = 2048, 1024, 1 << 14
    body = W.uniform(8 * E, n_symbols=n_sym, n_accounts=n_acc, seed=77)
    risk = np.where(body.action == W.BUY, body.size.astype(np.int64) * body.price,
                    np.where(body.action == W.SELL, body.size.astype(np.int64) * (100 - body.price.astype(np.int64)), 0))
    credit = np.floor(np.bincount(body.aid, weights=risk, minlength=n_acc) * funding).astype(np.int64)
    rows = [(W.CREATE_BALANCE, 0, a, 0, 0, 0) for a in range(n_acc)]
    rows += [(W.TRANSFER, 0, a, 0, 0, int(credit[a])) for a in range(n_acc)]
    rows += [(W.ADD_SYMBOL, 0, 0, s, 0, 0) for s in range(1, n_sym + 1)]
    orders = W.Orders.concat([W.Orders.from_rows(rows), body])
    args = (1, n_sym + 1, E, 1 << 20, 4 * E, n_acc, flags, 0, -4, 1 << 12)
    p = JavaProcessor(lib, j, tmp_path / "m.ckpt", E, 4 * E, args)
    if not rebalance and not flags:
        with pytest.raises(AssertionError):        # a shard's epoch refused: status UNFUNDED in the rows' epoch
            _drive(p, orders, punct=1 << 30)
            p.close()
        return
    _drive(p, orders, punct=1 << 30)
    p.close()
    o = oracle_mod.Oracle()
    o.process(orders)
    _cmp_fields(_as_tape(p.rows_out(), oracle_mod.REC_DTYPE), o.tape())


@pytest.mark.gpu
@pytest.mark.parametrize("damage", ["missing", "stale", "foreign"])
def test_restart_takes_the_committed_state_from_the_changelog(oracle_mod, tmp_path, damage):
    """Round-5 verdict (What's missing 2, row f next-3): the state follows the task.  Each commit point
    puts the checkpoint's changed chunks and then a record naming every chunk (generation, offset,
    size, digest, chunk hashes) into the changelogged commit log.  A restart whose state directory
    lost the file (the task moved: `missing`), holds an older one (`stale`) or another run's file of the
    same generation (`foreign`) rebuilds the committed file from the changelog and resumes: its rows
    after the restart plus the rows forwarded before the commit point are the oracle's tape.  Only the
    chunks that changed go to the changelog: a commit after a few records puts few of them.  When the
    changelog's chunks are incomplete too, the processor fails loudly instead of starting from an empty
    or wrong book; a file newer than the log's record is then taken (the crash fell between the file's
    rename and the changelog writes)."""
    import shutil

    lib = _lib()
    j = FakeJni()
    setup = W.funded_setup(64, range(1, 17))
    orders = W.Orders.concat([setup, W.uniform(20_000, n_symbols=16, n_accounts=64, seed=41)])
    epoch, max_trades = 1 << 11, 1 << 13
    args = (1, 17, epoch, 1 << 15, max_trades, 64, 3, 0, 1, 1 << 12)
    ckpt = tmp_path / "kme-0_1.ckpt"
    log = {}
    CB = 1 << 14                                                    # (small chunks: a small state shows the delta)
    p = JavaProcessor(lib, j, ckpt, epoch, max_trades, args, log, CB)
    n = len(orders)
    _drive(p, orders, 0, n // 3)
    p.commit_point()
    full = p.chunks_put
    shutil.copy(ckpt, tmp_path / "gen1.ckpt")
    _drive(p, orders, n // 3, n // 3 + 5)                         # a few records: few chunks change
    p.commit_point()
    assert 0 < p.chunks_put < full // 2, (p.chunks_put, full)
    _drive(p, orders, n // 3 + 5, 2 * n // 3)
    p.commit_point()
    c2 = p.last_offset
    F = sum(len(x) for x in p.out)
    assert log["checkpoint"][0] == 3
    assert sorted(k for k in log if k.startswith("c:")) == sorted(p._chunk_key(k, h) for k, h in enumerate(log["checkpoint"][5]))
    _drive(p, orders, 2 * n // 3, 2 * n // 3 + 500)
    first = p.rows_out()[:F]
    p.crash()
    if damage == "missing":
        os.remove(ckpt)
    elif damage == "stale":
        shutil.copy(tmp_path / "gen1.ckpt", ckpt)
    else:   # a file of the same generation written by another run: same name, other content
        other = JavaProcessor(lib, j, tmp_path / "other.ckpt", epoch, max_trades, args, {}, CB)
        for a, b in ((0, n // 3), (n // 3, n // 2), (n // 2, n // 2 + 10)):
            _drive(other, orders, a, b)
            other.commit_point()
        other.crash()
        shutil.copy(tmp_path / "other.ckpt", ckpt)
    q = JavaProcessor(lib, j, ckpt, epoch, max_trades, args, log, CB)
    assert q.generation == 3 and q.skip_through == c2
    _drive(q, orders, c2 + 1, n)
    q.close()
    got = np.concatenate([first, q.rows_out()])
    o = oracle_mod.Oracle()
    o.process(orders)
    _cmp_fields(_as_tape(got, oracle_mod.REC_DTYPE), o.tape())
    # the changelog's chunks incomplete as well: refused loudly (the damaged local file is not taken)
    broken = dict(log)
    broken.pop(next(k for k in broken if k.startswith("c:")))
    if damage == "missing":
        os.remove(ckpt)
    else:
        shutil.copy(tmp_path / "gen1.ckpt", ckpt)
    with pytest.raises(IllegalState):
        JavaProcessor(lib, j, ckpt, epoch, max_trades, args, broken, CB)
    # a file one generation ahead of the log's record, whose chunks are incomplete, is taken
    r = JavaProcessor(lib, j, tmp_path / "gen1.ckpt", epoch, max_trades, args,
                      {"checkpoint": (0, -1, 0, 0, CB, (7,))}, CB)
    assert r.generation == 1 and r.skip_through == n // 3 - 1
    r.crash()


@pytest.mark.gpu
def test_corrupted_checkpoint_is_refused_untouched(kme_mod, oracle_mod, tmp_path):
    """The digest in a checkpoint's trailer is recomputed over everything a restore reads: one flipped
    byte in the stores is refused (KME_E_INVALID) before anything reaches the device."""
    setup = W.funded_setup(32, range(1, 9))
    part = W.uniform(3000, n_symbols=8, n_accounts=32, seed=6)
    cfg = kme_mod.default_config(kme_mod.MODE_FUNDED, max_symbols=9, max_epoch=1 << 12, max_resting=1 << 14,
                                 max_accounts=32, flags=3)
    a = kme_mod.Engine(cfg)
    a.process(setup)
    a.process(part)
    ck = tmp_path / "a.ckpt"
    a.checkpoint_app(str(ck), b"rec")
    info = kme_mod.checkpoint_inspect(ck)
    assert info["file_bytes"] == os.path.getsize(ck) and info["app_bytes"] == 3
    raw = bytearray(ck.read_bytes())
    raw[len(raw) // 2] ^= 0x40
    bad = tmp_path / "bad.ckpt"
    bad.write_bytes(bytes(raw))
    b = kme_mod.Engine(cfg)
    b.process(setup)
    before = b.snapshot_books()
    with pytest.raises(kme_mod.KmeError) as ke:
        b.restore_app(str(bad))
    assert kme_mod.STATUS[ke.value.status] == "INVALID"
    assert b.snapshot_books() == before
    assert b.restore_app(str(ck)) == b"rec"
    assert b.snapshot_books() == a.snapshot_books() and b.snapshot_ledger() == a.snapshot_ledger()
    a.close()
    b.close()


# GpuMatchingEngine()'s arguments (integration/jni/GpuMatchingEngine.java: 65,536-record epochs, 2^18
# trades, FUNDED, exact ledger + serial fallback, 65,537 symbols, 2^20 accounts, 2^26 resting orders,
# device 0, one GPU, 2^20 ledger entries before the first growth)
DEFAULT_EPOCH, DEFAULT_TRADES = 1 << 16, 1 << 18
DEFAULT_ARGS = (1, 65537, DEFAULT_EPOCH, 1 << 26, DEFAULT_TRADES, 1 << 20, 3, 0, 1, 1 << 20)


@pytest.mark.gpu
@pytest.mark.parametrize("crash", [False, True])
def test_drop_in_defaults_take_the_reference_domain(oracle_mod, tmp_path, crash):
    """Round-5 verdict (What's missing 1): the processor with GpuMatchingEngine()'s defaults takes the
    reference's whole input domain.  exchange_test.js's stream, untruncated, with a sparse symbol
    (10^12), an account of id 2^40, BUY/SELL priced 101..125 and negative sizes spliced in
    (tests/domain_stream.py; KP:131-146, 184-191, 200-223, 391-404, 451-456): the MatchOut rows, books
    and exact ledger equal the oracle's -- and across a commit point, crash and restart."""
    import domain_stream as D

    lib = _lib()
    j = FakeJni()
    orders = D.reference_domain_stream(oracle_mod)
    ckpt = tmp_path / "defaults.ckpt"
    p = JavaProcessor(lib, j, ckpt, DEFAULT_EPOCH, DEFAULT_TRADES, DEFAULT_ARGS)
    n = len(orders)
    if not crash:
        _drive(p, orders)
        q = p
        got_head = np.zeros(0, ROW_DTYPE)
    else:
        c1, crash_at = int(n * 0.3) + 11, int(n * 0.7) + 5        # (after the first splices)
        _drive(p, orders, 0, c1 + 1)
        p.commit_point()
        F = sum(len(x) for x in p.out)
        _drive(p, orders, c1 + 1, crash_at)
        got_head = p.rows_out()[:F]
        p.crash()
        q = JavaProcessor(lib, j, ckpt, DEFAULT_EPOCH, DEFAULT_TRADES, DEFAULT_ARGS, p.commit_log)
        assert q.skip_through == c1
        _drive(q, orders, c1 + 1, n)
    q.forward_ready()
    q.flush()
    while q.inflight:
        q.complete_oldest(True)
    eng = C.c_void_p.from_address(q.h).value
    import kme
    L = kme.lib()
    books = _snapshot(L, L.kme_snapshot_books, eng)
    ledger = _snapshot(L, L.kme_snapshot_ledger, eng)
    q.close()
    got = np.concatenate([got_head, q.rows_out()])
    o = oracle_mod.Oracle()
    o.process(orders)
    _cmp_fields(_as_tape(got, oracle_mod.REC_DTYPE), o.tape())
    assert books == o.dump_books()
    assert ledger == o.dump_ledger()


@pytest.mark.gpu
@pytest.mark.parametrize("crash", [False, True])
def test_multi_gpu_drop_in_consolidates_an_unprovable_stream(oracle_mod, tmp_path, crash):
    """Round-4 verdict (What's missing 2): the drop-in's default flags (exact ledger + serial fallback)
    at nDevices > 1.  The reference's own harness stream (exchange_test.js: nearly every order is a
    balance reject, KP:167-182) cannot be proven by any shard's funded bound, so the first epoch that
    fails the proof consolidates the stream onto one exact engine (the history replayed into it; SURVEY
    §8e "replicas only") instead of failing with KME_E_UNFUNDED: the MatchOut rows equal the oracle's,
    and across a commit point, crash and restart from the consolidated checkpoint."""
    lib = _lib()
    j = FakeJni()
    import domain_stream as D

    orders = D.reference_domain_stream(oracle_mod, n=30_000, seed=13)   # (the whole domain: the shards refuse
                                                                        # what they cannot take, it consolidates)
    epoch, max_trades = 1 << 11, 1 << 13
    args = (1, 8, epoch, 1 << 15, max_trades, 64, 3, 0, -4, 1 << 12)   # FUNDED, exact ledger + fallback, 4 shards
    ckpt = tmp_path / "cons.ckpt"
    p = JavaProcessor(lib, j, ckpt, epoch, max_trades, args)
    n = len(orders)
    if not crash:
        _drive(p, orders)
        p.close()
        got = p.rows_out()
    else:
        c1, crash_at = int(n * 0.6) + 7, int(n * 0.8) + 3
        _drive(p, orders, 0, c1 + 1)
        p.commit_point()
        F = sum(len(x) for x in p.out)
        _drive(p, orders, c1 + 1, crash_at)
        first = p.rows_out()
        p.crash()
        q = JavaProcessor(lib, j, ckpt, epoch, max_trades, args, p.commit_log)
        assert q.skip_through == c1
        _drive(q, orders, c1 + 1, n)
        q.close()
        got = np.concatenate([first[:F], q.rows_out()])
    o = oracle_mod.Oracle()
    o.process(orders)
    _cmp_fields(_as_tape(got, oracle_mod.REC_DTYPE), o.tape())


@pytest.mark.gpu
@pytest.mark.parametrize("hist", ["kept", "lost"])
def test_multi_gpu_drop_in_consolidates_after_a_restart(oracle_mod, tmp_path, monkeypatch, hist):
    """Round-5 verdict (Next 8): a nDevices = -4 processor with the drop-in's default flags commits,
    crashes, restores from its sharded checkpoint, and only then meets an epoch no shard can prove
    (BUY/SELL priced 101..125, outside the funded domain: KP:167-182, 200-223).  The input history
    since the start went to `path`.hist with every commit point (its length and digest in the
    manifest), so the restored processor still consolidates onto one exact engine and its MatchOut rows
    equal the oracle's.  shardStatus() says so before and after.  With the history file gone at the
    restart (`lost`) the restore still succeeds, shardStatus() says consolidation is off, and the
    unprovable epoch fails loudly (KME_E_UNFUNDED) instead of answering wrongly."""
    lib = _lib()
    j = FakeJni()
    n_sym, n_acc, epoch, max_trades = 16, 64, 1 << 11, 1 << 13
    setup = W.funded_setup(n_acc, range(1, n_sym + 1))
    funded = W.uniform(12_000, n_symbols=n_sym, n_accounts=n_acc, seed=23)
    late = W.uniform(4_000, n_symbols=n_sym, n_accounts=n_acc, seed=24, oid_base=1 << 20)
    rng = np.random.default_rng(5)
    odd = rng.choice(np.flatnonzero((late.action == W.BUY) | (late.action == W.SELL)), 40, replace=False)
    late.price[odd] = rng.integers(101, 126, len(odd)).astype(late.price.dtype)
    orders = W.Orders.concat([setup, funded, late])
    args = (1, n_sym + 1, epoch, 1 << 15, max_trades, n_acc, 3, 0, -4, 1 << 12)
    ckpt = tmp_path / "m.ckpt"
    p = JavaProcessor(lib, j, ckpt, epoch, max_trades, args)
    c1 = len(setup) + len(funded) // 2
    _drive(p, orders, 0, c1 + 1)
    p.commit_point()
    st = p.shard_status()
    assert st["n_engines"] == 4 and st["consolidated"] == 0 and st["can_consolidate"] == 1
    assert st["history_saved"] == st["history_records"] == c1 + 1
    assert os.path.exists(str(ckpt) + ".hist")
    F = sum(len(x) for x in p.out)
    crash_at = len(setup) + len(funded) - 7
    _drive(p, orders, c1 + 1, crash_at)
    first = p.rows_out()[:F]
    p.crash()
    if hist == "lost":
        os.remove(str(ckpt) + ".hist")
    q = JavaProcessor(lib, j, ckpt, epoch, max_trades, args, p.commit_log)
    assert q.skip_through == c1
    st = q.shard_status()
    assert st["consolidated"] == 0 and st["can_consolidate"] == (1 if hist == "kept" else 0)
    if hist == "lost":
        with pytest.raises(AssertionError):           # the unprovable epoch's status: UNFUNDED
            _drive(q, orders, c1 + 1, len(orders))
            q.close()
        q.crash()
        return
    _drive(q, orders, c1 + 1, len(orders))
    q.forward_ready()
    q.flush()
    while q.inflight:
        q.complete_oldest(True)
    st = q.shard_status()
    assert st["consolidated"] == 1 and st["can_consolidate"] == 0
    q.close()
    got = np.concatenate([first, q.rows_out()])
    o = oracle_mod.Oracle()
    o.process(orders)
    _cmp_fields(_as_tape(got, oracle_mod.REC_DTYPE), o.tape())
