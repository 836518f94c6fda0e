"""ctypes wrapper of the CPU restatement (oracle/kme_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, always as the checker, never as the thing measured or shipped.
The restatement follows /root/reference/src/main/java/KProcessor.java:96-445 line by line;
parity is UNPINNED (the reference has no tests or golden vectors).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libkme_oracle.so")

KO_ERRORS = {
    1: "NPE position (KP:179-180/332)",
    2: "NPE bucket (KP:234-235/252-253)",
    3: "NPE order (KP:236-237/257)",
    4: "NPE balance (KP:157/286/331)",
    5: "removeAllOrders never terminates (KP:341-353)",
    6: "NPE book (KP:294/301)",
}

REC_DTYPE = np.dtype([
    ("key", "<i4"), ("action", "<i4"), ("oid", "<i8"), ("aid", "<i8"), ("sid", "<i8"),
    ("price", "<i4"), ("size", "<i4"), ("next", "<i8"), ("prev", "<i8"),
    ("has_next", "<i4"), ("has_prev", "<i4"),
])
assert REC_DTYPE.itemsize == 64


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        vp, sz, i32, i64 = C.c_void_p, C.c_size_t, C.c_int32, C.c_int64
        L.ko_create.restype = vp
        L.ko_destroy.argtypes = [vp]
        L.ko_process_batch.restype = C.c_int
        L.ko_process_batch.argtypes = [vp, sz, vp, vp, vp, vp, vp, vp, C.POINTER(sz)]
        L.ko_tape_len.restype = sz
        L.ko_tape_len.argtypes = [vp]
        L.ko_tape.restype = vp
        L.ko_tape.argtypes = [vp]
        L.ko_tape_clear.argtypes = [vp]
        L.ko_set_keep_tape.argtypes = [vp, C.c_int]
        L.ko_records_forwarded.restype = C.c_uint64
        L.ko_records_forwarded.argtypes = [vp]
        for f in (L.ko_tape_text, L.ko_dump_books, L.ko_dump_ledger):
            f.restype = C.c_void_p
            f.argtypes = [vp, C.POINTER(sz)]
        L.ko_free.argtypes = [vp]
        L.ko_first_set_bit_pos.restype = i32
        L.ko_first_set_bit_pos.argtypes = [i64]
        L.ko_last_set_bit_pos.restype = i32
        L.ko_last_set_bit_pos.argtypes = [i64]
        _lib = L
    return _lib


class OracleError(RuntimeError):
    def __init__(self, code: int, index: int):
        super().__init__(f"oracle domain error {code} ({KO_ERRORS.get(code, '?')}) at input {index}")
        self.code, self.index = code, index


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


class Oracle:
    """One `MatchingEngine` instance with fresh stores (KP:86-93)."""

    def __init__(self, keep_tape: bool = True):
        self._L = lib()
        self._e = self._L.ko_create()
        self._L.ko_set_keep_tape(self._e, 1 if keep_tape else 0)

    def close(self):
        if self._e:
            self._L.ko_destroy(self._e)
            self._e = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def process(self, orders) -> None:
        """`process()` over every record of an SoA batch (dict of arrays or kme.workloads.Orders)."""
        get = (lambda k: orders[k]) if isinstance(orders, dict) else (lambda k: getattr(orders, k))
        cols = {
            "action": np.ascontiguousarray(get("action"), dtype=np.int32),
            "oid": np.ascontiguousarray(get("oid"), dtype=np.int64),
            "aid": np.ascontiguousarray(get("aid"), dtype=np.int64),
            "sid": np.ascontiguousarray(get("sid"), dtype=np.int64),
            "price": np.ascontiguousarray(get("price"), dtype=np.int32),
            "size": np.ascontiguousarray(get("size"), dtype=np.int32),
        }
        n = len(cols["action"])
        done = C.c_size_t(0)
        rc = self._L.ko_process_batch(self._e, n, _ptr(cols["action"]), _ptr(cols["oid"]),
                                      _ptr(cols["aid"]), _ptr(cols["sid"]), _ptr(cols["price"]),
                                      _ptr(cols["size"]), C.byref(done))
        if rc:
            raise OracleError(rc, done.value)

    def tape(self) -> np.ndarray:
        n = self._L.ko_tape_len(self._e)
        if n == 0:
            return np.zeros(0, REC_DTYPE)
        buf = (C.c_char * (n * 64)).from_address(self._L.ko_tape(self._e))
        return np.frombuffer(bytes(buf), dtype=REC_DTYPE).copy()

    def clear_tape(self):
        self._L.ko_tape_clear(self._e)

    def records_forwarded(self) -> int:
        return int(self._L.ko_records_forwarded(self._e))

    def _text(self, fn) -> str:
        n = C.c_size_t(0)
        p = fn(self._e, C.byref(n))
        try:
            return C.string_at(p, n.value).decode()
        finally:
            self._L.ko_free(p)

    def tape_text(self) -> str:
        return self._text(self._L.ko_tape_text)

    def dump_books(self) -> str:
        return self._text(self._L.ko_dump_books)

    def dump_ledger(self) -> str:
        return self._text(self._L.ko_dump_ledger)


def first_set_bit_pos(n: int) -> int:
    return lib().ko_first_set_bit_pos(n)


def last_set_bit_pos(n: int) -> int:
    return lib().ko_last_set_bit_pos(n)
