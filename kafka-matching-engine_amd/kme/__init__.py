"""Python host layer of the MI355X matching core: ctypes bindings of include/kme.h and
include/kme_processor.h (libkme.so, built in-tree by __graft_entry__.build()).

The product path is the HIP engine in libkme.so; there is no CPU fallback.  Loading fails loudly
when the shared object is missing, and creating an engine fails when no HIP device is present.

Reference correspondence (KProcessor.java, "KP"):
    Engine            the five stores + MatchingEngine (KP:30-49, 63-445) for one stream task
    Engine.process    MatchingEngine.process (KP:96-126) over an epoch of records
    Processor         MatchingEngine as a Processor<String, Order> fed JSON records (KP:52, 96)
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

from .workloads import Orders  # noqa: F401  (re-export)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KME_LIB") or os.path.join(_HERE, "libkme.so")

MODE_EXACT, MODE_FUNDED = 0, 1
KME_OK = 0
STATUS = {0: "OK", 1: "INVALID", 2: "CAPACITY", 3: "DOMAIN", 4: "UNFUNDED", 5: "UNSUPPORTED", 6: "HIP",
          7: "FAILED"}
ABI_VERSION = 7
FLAG_EXACT_LEDGER = 1
FLAG_SERIAL_FALLBACK = 2   # FUNDED: an epoch whose funded proof fails (or that holds a record outside the
                           # parallel path's domain) runs serially (needs FLAG_EXACT_LEDGER)
FLAG_REFUSE_SERIAL = 4     # FUNDED: such an epoch is refused as unproven instead (kme_multi's shards)
SPARSE_NONE = 0xFFFFFFFF   # kme_config.max_sparse_symbols: no sparse symbols

TRADE_DTYPE = np.dtype([("maker_oid", "<i8"), ("maker_aid", "<i8"), ("maker_sid", "<i8"),
                        ("maker_price", "<i4"), ("size", "<i4")])
TOB_DTYPE = np.dtype([("bid_px", "<i4"), ("ask_px", "<i4"), ("bid_qty", "<i4"), ("ask_qty", "<i4")])
assert TRADE_DTYPE.itemsize == 32


class kme_config(C.Structure):
    _fields_ = [("abi_version", C.c_uint32), ("mode", C.c_uint32), ("max_symbols", C.c_uint32),
                ("max_accounts", C.c_uint32), ("max_epoch", C.c_uint32), ("max_trades", C.c_uint32),
                ("max_resting", C.c_uint64), ("ledger_capacity", C.c_uint64), ("device", C.c_int32),
                ("credit_shards", C.c_uint32), ("flags", C.c_uint32), ("light_max", C.c_int32),
                ("max_sparse_symbols", C.c_uint32), ("_reserved", C.c_uint32)]


assert C.sizeof(kme_config) == 64


class kme_orders(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in ("action", "oid", "aid", "sid", "price", "size")]


class kme_epoch_result(C.Structure):
    _fields_ = [("out_action", C.c_void_p), ("out_size", C.c_void_p), ("out_prev", C.c_void_p),
                ("out_flags", C.c_void_p), ("trade_off", C.c_void_p), ("trades", C.c_void_p),
                ("trades_cap", C.c_uint32)]


class kme_epoch_status(C.Structure):
    _fields_ = [("status", C.c_int32), ("detail", C.c_int32), ("error_index", C.c_int64),
                ("n_inputs", C.c_uint32), ("n_trades", C.c_uint32), ("n_orders", C.c_uint64),
                ("n_rests", C.c_uint64), ("n_maker_visits", C.c_uint64), ("n_cancel_ok", C.c_uint64),
                ("serial_fallback", C.c_uint32), ("n_effective", C.c_uint32), ("ledger_repaired", C.c_uint32),
                ("ledger_serial", C.c_uint32)]


class kme_checkpoint_info(C.Structure):
    _fields_ = [("file_bytes", C.c_uint64), ("app_bytes", C.c_uint64), ("digest", C.c_uint64)]


class kme_multi_status(C.Structure):
    _fields_ = [("n_engines", C.c_uint32), ("consolidated", C.c_uint32), ("can_consolidate", C.c_uint32),
                ("failed", C.c_uint32), ("history_records", C.c_uint64), ("history_cap", C.c_uint64),
                ("history_saved", C.c_uint64), ("generation", C.c_uint64)]


class kme_ledger_info(C.Structure):
    _fields_ = [("bal_slots", C.c_uint64), ("pos_slots", C.c_uint64), ("bal_used", C.c_uint64),
                ("pos_used", C.c_uint64), ("grows", C.c_uint32), ("_pad", C.c_uint32)]


FORWARD_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_char_p, C.c_void_p, C.c_size_t)
COMMIT_FN = C.CFUNCTYPE(None, C.c_void_p)

# Every symbol include/kme.h and include/kme_processor.h declare (checked by tests/test_abi.py).
EXPORTS = [
    "kme_create", "kme_destroy", "kme_set_stream", "kme_submit_epoch", "kme_submit_epoch_device",
    "kme_wait", "kme_device_results", "kme_snapshot_books", "kme_snapshot_ledger", "kme_free",
    "kme_top_of_book", "kme_top_of_book_groups", "kme_phase_times", "kme_phase_name", "kme_enable_timing", "kme_tape_json",
    "kme_tape_json_device", "kme_order_from_json", "kme_checkpoint", "kme_restore", "kme_checkpoint_app", "kme_restore_app", "kme_checkpoint_inspect", "kme_checkpoint_chunks", "kme_ledger_stats", "kme_shard_of", "kme_strerror", "kme_domain_str", "kme_debug_counters",
    "kme_processor_create", "kme_processor_process_json", "kme_processor_process",
    "kme_processor_punctuate", "kme_processor_close", "kme_processor_last_status",
    "kme_router_create", "kme_router_destroy", "kme_router_route", "kme_router_split", "kme_router_directory_size",
    "kme_host_register", "kme_host_unregister", "kme_submit_epoch_host", "kme_poll", "kme_expand_rows", "kme_expand_rows_mt", "kme_build_id",
    "kme_rccl_load", "kme_rccl_last_error", "kme_comm_unique_id", "kme_comm_init", "kme_comm_destroy", "kme_market_data_allgather", "kme_credit_state",
    "kme_credit_adjust", "kme_credit_rebalance",
    "kme_multi_create", "kme_multi_destroy", "kme_multi_submit_epoch_host", "kme_multi_poll", "kme_multi_wait",
    "kme_multi_checkpoint_app", "kme_multi_restore_app", "kme_multi_engine", "kme_multi_info",
]

_lib = None


def lib():
    """libkme.so with argtypes set.  Raises if the HIP extension was not built."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("KME_LIB") or LIB_PATH   # (diagnostic builds are selected at load time)
    if not os.path.exists(path):
        raise RuntimeError(f"libkme.so not built ({path}); run __graft_entry__.build()")
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64.so.7.  Loading torch first
    # makes libkme's NEEDED libamdhip64.so.7 resolve to that already-loaded copy (same SONAME);
    # loading libkme first would map a second HIP/HSA runtime and neither would see the GPU.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(path)
    vp, st, u32, i32, i64 = C.c_void_p, C.c_int, C.c_uint32, C.c_int32, C.c_int64
    sig = {
        "kme_create": (st, [C.POINTER(kme_config), C.POINTER(vp)]),
        "kme_destroy": (st, [vp]),
        "kme_set_stream": (st, [vp, vp]),
        "kme_submit_epoch": (st, [vp, C.POINTER(kme_orders), u32, C.POINTER(kme_epoch_result),
                                  C.POINTER(kme_epoch_status)]),
        "kme_submit_epoch_device": (st, [vp, C.POINTER(kme_orders), u32, C.POINTER(kme_epoch_result)]),
        "kme_wait": (st, [vp, C.POINTER(kme_epoch_status)]),
        "kme_device_results": (st, [vp, C.POINTER(kme_epoch_result)]),
        "kme_snapshot_books": (st, [vp, C.POINTER(vp), C.POINTER(C.c_size_t)]),
        "kme_snapshot_ledger": (st, [vp, C.POINTER(vp), C.POINTER(C.c_size_t)]),
        "kme_free": (None, [vp]),
        "kme_top_of_book": (st, [vp, vp]),
        "kme_top_of_book_groups": (st, [vp, vp, u32, vp]),
        "kme_phase_times": (st, [vp, C.POINTER(C.c_float), C.POINTER(C.c_int)]),
        "kme_phase_name": (C.c_char_p, [C.c_int]),
        "kme_enable_timing": (st, [vp, C.c_int]),
        "kme_tape_json": (st, [C.POINTER(kme_orders), u32, C.POINTER(kme_epoch_result), vp, C.c_size_t,
                               C.POINTER(C.c_size_t)]),
        "kme_tape_json_device": (st, [vp, C.POINTER(kme_orders), u32, C.POINTER(kme_epoch_result), vp, C.c_size_t,
                                      C.POINTER(C.c_size_t)]),
        "kme_checkpoint": (st, [vp, C.c_char_p]),
        "kme_restore": (st, [vp, C.c_char_p]),
        "kme_checkpoint_app": (st, [vp, C.c_char_p, vp, C.c_size_t]),
        "kme_restore_app": (st, [vp, C.c_char_p, vp, C.c_size_t, C.POINTER(C.c_size_t)]),
        "kme_checkpoint_inspect": (st, [C.c_char_p, C.POINTER(kme_checkpoint_info)]),
        "kme_checkpoint_chunks": (st, [C.c_char_p, C.c_uint32, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]),
        "kme_ledger_stats": (st, [vp, C.POINTER(kme_ledger_info)]),
        "kme_order_from_json": (st, [C.c_char_p, C.c_size_t, C.POINTER(i32), C.POINTER(i64), C.POINTER(i64),
                                     C.POINTER(i64), C.POINTER(i32), C.POINTER(i32)]),
        "kme_shard_of": (u32, [i64, u32]),
        "kme_debug_counters": (st, [vp, vp, C.c_size_t]),
        "kme_strerror": (C.c_char_p, [C.c_int]),
        "kme_domain_str": (C.c_char_p, [C.c_int]),
        "kme_processor_create": (st, [C.POINTER(kme_config), u32, FORWARD_FN, COMMIT_FN, vp, C.POINTER(vp)]),
        "kme_processor_process_json": (st, [vp, C.c_char_p, C.c_size_t]),
        "kme_processor_process": (st, [vp, i32, i64, i64, i64, i32, i32]),
        "kme_processor_punctuate": (st, [vp]),
        "kme_processor_close": (st, [vp]),
        "kme_processor_last_status": (st, [vp, C.POINTER(kme_epoch_status)]),
        "kme_router_create": (st, [u32, C.c_uint64, C.POINTER(vp)]),
        "kme_router_destroy": (st, [vp]),
        "kme_router_route": (st, [vp, C.POINTER(kme_orders), u32, vp]),
        "kme_router_split": (st, [vp, C.POINTER(kme_orders), u32, vp, vp, vp, vp]),
        "kme_router_directory_size": (C.c_uint64, [vp]),
        "kme_host_register": (st, [vp, vp, C.c_size_t]),
        "kme_host_unregister": (st, [vp, vp]),
        "kme_submit_epoch_host": (st, [vp, C.POINTER(kme_orders), u32, C.POINTER(kme_epoch_result)]),
        "kme_poll": (st, [vp, C.POINTER(C.c_int)]),
        "kme_expand_rows": (st, [C.POINTER(kme_orders), u32, C.POINTER(kme_epoch_result), vp, C.c_size_t,
                                 C.POINTER(C.c_size_t)]),
        "kme_expand_rows_mt": (st, [C.POINTER(kme_orders), u32, C.POINTER(kme_epoch_result), vp, C.c_size_t,
                                    C.POINTER(C.c_size_t), u32]),
        "kme_build_id": (C.c_char_p, []),
        "kme_rccl_load": (st, [C.c_char_p]),
        "kme_rccl_last_error": (C.c_char_p, []),
        "kme_comm_unique_id": (st, [vp]),
        "kme_comm_init": (st, [vp, u32, u32, vp, C.POINTER(vp)]),
        "kme_comm_destroy": (st, [vp]),
        "kme_market_data_allgather": (st, [vp, vp, vp, u32, u32, vp]),
        "kme_credit_state": (st, [vp, vp]),
        "kme_credit_adjust": (st, [vp, vp, u32, u32]),
        "kme_credit_rebalance": (st, [vp, vp]),
        "kme_multi_create": (st, [C.POINTER(kme_config), u32, vp, C.POINTER(vp)]),
        "kme_multi_destroy": (st, [vp]),
        "kme_multi_submit_epoch_host": (st, [vp, C.POINTER(kme_orders), u32, C.POINTER(kme_epoch_result)]),
        "kme_multi_poll": (st, [vp, C.POINTER(C.c_int)]),
        "kme_multi_wait": (st, [vp, C.POINTER(kme_epoch_status)]),
        "kme_multi_checkpoint_app": (st, [vp, C.c_char_p, vp, C.c_size_t]),
        "kme_multi_restore_app": (st, [vp, C.c_char_p, vp, C.c_size_t, C.POINTER(C.c_size_t)]),
        "kme_multi_engine": (st, [vp, u32, C.POINTER(vp)]),
        "kme_multi_info": (st, [vp, C.POINTER(kme_multi_status)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


class KmeError(RuntimeError):
    def __init__(self, status: int, what: str = "", st: kme_epoch_status | None = None):
        L = lib()
        detail = st.detail if st is not None else 0
        msg = f"{STATUS.get(status, status)}: {L.kme_strerror(status).decode()}"
        if detail:
            msg += f" [{L.kme_domain_str(detail).decode()}]"
        if st is not None and st.error_index >= 0:
            msg += f" at input {st.error_index}"
        if what:
            msg = f"{what}: {msg}"
        super().__init__(msg)
        self.status, self.detail = status, detail
        self.index = st.error_index if st is not None else -1
        self.n_effective = int(st.n_effective) if st is not None else 0


def _np_ptr(a: np.ndarray):
    return C.c_void_p(a.ctypes.data)


def _soa(orders: Orders):
    cols = dict(action=np.ascontiguousarray(orders.action, np.int32), oid=np.ascontiguousarray(orders.oid, np.int64),
                aid=np.ascontiguousarray(orders.aid, np.int64), sid=np.ascontiguousarray(orders.sid, np.int64),
                price=np.ascontiguousarray(orders.price, np.int32), size=np.ascontiguousarray(orders.size, np.int32))
    s = kme_orders(*[C.c_void_p(cols[k].ctypes.data) for k in ("action", "oid", "aid", "sid", "price", "size")])
    return s, cols


@dataclass
class EpochResult:
    """Per-input OUT fields and the ordered trades of one processed epoch (kme_epoch_result)."""
    out_action: np.ndarray
    out_size: np.ndarray
    out_prev: np.ndarray
    out_flags: np.ndarray
    trade_off: np.ndarray
    trades: np.ndarray
    status: kme_epoch_status

    def tape_json(self, orders: Orders) -> str:
        """The MatchOut tape as consumer.js prints it (consumer.js:19), via kme_tape_json."""
        L = lib()
        s, keep = _soa(orders)
        r = kme_epoch_result(_np_ptr(self.out_action), _np_ptr(self.out_size), _np_ptr(self.out_prev),
                             _np_ptr(self.out_flags), _np_ptr(self.trade_off), _np_ptr(self.trades),
                             len(self.trades))
        n = C.c_size_t(0)
        L.kme_tape_json(C.byref(s), len(orders), C.byref(r), None, 0, C.byref(n))
        buf = C.create_string_buffer(n.value + 1)
        rc = L.kme_tape_json(C.byref(s), len(orders), C.byref(r), buf, n.value + 1, C.byref(n))
        if rc:
            raise KmeError(rc, "kme_tape_json")
        del keep
        return buf.raw[: n.value].decode()


def default_config(mode: int, max_symbols: int, max_epoch: int, max_resting: int, max_trades: int | None = None,
                   max_accounts: int = 0, ledger_capacity: int = 1 << 16, device: int = 0,
                   flags: int = 0, light_max: int = 0, max_sparse_symbols: int = 0) -> kme_config:
    return kme_config(ABI_VERSION, mode, max_symbols, max_accounts, max_epoch,
                      max_trades if max_trades is not None else max(4 * max_epoch, 1 << 16),
                      max_resting, ledger_capacity, device, 0, flags, light_max, max_sparse_symbols, 0)


class Engine:
    """One device engine (kme_create).  `process` = host-buffer epochs (synchronous)."""

    def __init__(self, cfg: kme_config):
        L = lib()
        self._L = L
        self.cfg = cfg
        h = C.c_void_p()
        rc = L.kme_create(C.byref(cfg), C.byref(h))
        if rc:
            raise KmeError(rc, "kme_create")
        self._h = h

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None):
            self._L.kme_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def process(self, orders: Orders) -> EpochResult:
        n = len(orders)
        s, keep = _soa(orders)
        cap = max(1, int(self.cfg.max_trades))
        res = EpochResult(np.zeros(n, np.int32), np.zeros(n, np.int32), np.zeros(n, np.int64), np.zeros(n, np.uint8),
                          np.zeros(n + 1, np.uint32), np.zeros(cap, TRADE_DTYPE), kme_epoch_status())
        r = kme_epoch_result(_np_ptr(res.out_action), _np_ptr(res.out_size), _np_ptr(res.out_prev),
                             _np_ptr(res.out_flags), _np_ptr(res.trade_off), _np_ptr(res.trades), cap)
        st = kme_epoch_status()
        rc = self._L.kme_submit_epoch(self._h, C.byref(s), n, C.byref(r), C.byref(st))
        del keep
        res.status = st
        if rc:
            # the results of the records that took effect before the fault (kme.h, n_effective)
            k = int(st.n_effective)
            err = KmeError(rc, "kme_submit_epoch", st)
            err.result = EpochResult(res.out_action[:k].copy(), res.out_size[:k].copy(), res.out_prev[:k].copy(),
                                     res.out_flags[:k].copy(), res.trade_off[: k + 1].copy(),
                                     res.trades[: int(res.trade_off[k])].copy(), st)
            err.n_effective = k
            raise err
        res.trades = res.trades[: int(res.trade_off[n])].copy()
        return res

    # ---- device-resident epochs (bench): torch tensors or raw device pointers
    def submit_device(self, ptrs: dict, n: int, out: dict | None = None):
        """Device epoch; `out` (device pointers out_action, out_size, out_prev, out_flags, trade_off,
        trades, and trades_cap) receives the results instead of the engine-owned buffers."""
        s = kme_orders(*[C.c_void_p(int(ptrs[k])) for k in ("action", "oid", "aid", "sid", "price", "size")])
        r = None
        if out is not None:
            r = kme_epoch_result(*[C.c_void_p(int(out[k])) for k in ("out_action", "out_size", "out_prev", "out_flags",
                                                                      "trade_off", "trades")], int(out["trades_cap"]))
        rc = self._L.kme_submit_epoch_device(self._h, C.byref(s), n, C.byref(r) if r is not None else None)
        if rc:
            raise KmeError(rc, "kme_submit_epoch_device")

    # ---- host epochs at rate (kme_submit_epoch_host / kme_poll): numpy arrays registered once
    def host_register(self, arr: np.ndarray):
        rc = self._L.kme_host_register(self._h, C.c_void_p(arr.ctypes.data), arr.nbytes)
        if rc:
            raise KmeError(rc, "kme_host_register")

    def host_unregister(self, arr: np.ndarray):
        rc = self._L.kme_host_unregister(self._h, C.c_void_p(arr.ctypes.data))
        if rc:
            raise KmeError(rc, "kme_host_unregister")

    def submit_host(self, cols: dict, n: int, out: "EpochResult"):
        """cols: the six input columns (numpy, registered); out: an EpochResult whose arrays receive the
        results at wait()."""
        s = kme_orders(*[C.c_void_p(cols[k].ctypes.data) for k in ("action", "oid", "aid", "sid", "price", "size")])
        r = kme_epoch_result(_np_ptr(out.out_action), _np_ptr(out.out_size), _np_ptr(out.out_prev),
                             _np_ptr(out.out_flags), _np_ptr(out.trade_off), _np_ptr(out.trades), len(out.trades))
        rc = self._L.kme_submit_epoch_host(self._h, C.byref(s), n, C.byref(r))
        if rc:
            raise KmeError(rc, "kme_submit_epoch_host")

    def poll(self) -> bool:
        done = C.c_int(0)
        rc = self._L.kme_poll(self._h, C.byref(done))
        if rc:
            raise KmeError(rc, "kme_poll")
        return bool(done.value)

    # ---- multi-GPU: RCCL communicator, market data, credit between shards
    def comm_init(self, n_ranks: int, rank: int, uid: bytes) -> "Comm":
        return Comm(self, n_ranks, rank, uid)

    def credit_state(self, dev_ptr: int):
        rc = self._L.kme_credit_state(self._h, C.c_void_p(int(dev_ptr)))
        if rc:
            raise KmeError(rc, "kme_credit_state")

    def credit_adjust(self, dev_all_ptr: int, n_shards: int, my_shard: int):
        rc = self._L.kme_credit_adjust(self._h, C.c_void_p(int(dev_all_ptr)), n_shards, my_shard)
        if rc:
            raise KmeError(rc, "kme_credit_adjust")

    def wait(self) -> kme_epoch_status:
        st = kme_epoch_status()
        rc = self._L.kme_wait(self._h, C.byref(st))
        if rc:
            raise KmeError(rc, "kme_wait", st)
        return st

    def set_stream(self, stream_ptr: int | None):
        rc = self._L.kme_set_stream(self._h, C.c_void_p(stream_ptr) if stream_ptr else None)
        if rc:
            raise KmeError(rc, "kme_set_stream")

    def enable_timing(self, on=True):
        """True / "all": every phase; "match": the matching phase only; False: off."""
        mode = {"all": 1, "match": 2}.get(on, 1) if on else 0
        self._L.kme_enable_timing(self._h, mode)

    def phase_times(self) -> dict:
        ms = (C.c_float * 16)()
        n = C.c_int(0)
        self._L.kme_phase_times(self._h, ms, C.byref(n))
        return {self._L.kme_phase_name(i).decode(): float(ms[i]) for i in range(n.value)}

    def top_of_book(self, dev_ptr: int):
        rc = self._L.kme_top_of_book(self._h, C.c_void_p(int(dev_ptr)))
        if rc:
            raise KmeError(rc, "kme_top_of_book")

    def top_of_book_groups(self, groups_ptr: int, n: int, dev_ptr: int):
        """kme_top_of_book_groups: the snapshot of n groups (a device u32 array) into dev_ptr."""
        rc = self._L.kme_top_of_book_groups(self._h, C.c_void_p(int(groups_ptr)), int(n), C.c_void_p(int(dev_ptr)))
        if rc:
            raise KmeError(rc, "kme_top_of_book_groups")

    def _text(self, fn) -> str:
        p = C.c_void_p()
        n = C.c_size_t(0)
        rc = fn(self._h, C.byref(p), C.byref(n))
        if rc:
            raise KmeError(rc, fn.__name__)
        try:
            return C.string_at(p, n.value).decode()
        finally:
            self._L.kme_free(p)

    def debug_counters(self) -> np.ndarray:
        out = np.zeros(int(self.cfg.max_symbols) * 48, np.uint64)
        rc = self._L.kme_debug_counters(self._h, C.c_void_p(out.ctypes.data), out.size)
        if rc:
            raise KmeError(rc, "kme_debug_counters")
        return out.reshape(-1, 48)

    def checkpoint(self, path: str):
        rc = self._L.kme_checkpoint(self._h, str(path).encode())
        if rc:
            raise KmeError(rc, "kme_checkpoint")

    def restore(self, path: str):
        rc = self._L.kme_restore(self._h, str(path).encode())
        if rc:
            raise KmeError(rc, "kme_restore")

    def checkpoint_app(self, path: str, app: bytes):
        """kme_checkpoint_app: the state plus an application record (bytes), written atomically."""
        buf = C.create_string_buffer(bytes(app), max(1, len(app)))
        rc = self._L.kme_checkpoint_app(self._h, str(path).encode(), buf, len(app))
        if rc:
            raise KmeError(rc, "kme_checkpoint_app")

    def restore_app(self, path: str) -> bytes:
        """kme_restore_app: restores the state and returns the application record."""
        n = C.c_size_t(0)
        rc = self._L.kme_restore_app(self._h, str(path).encode(), None, 0, C.byref(n))
        if rc == 2:   # KME_E_CAPACITY: the record's size is known now
            buf = C.create_string_buffer(max(1, n.value))
            rc = self._L.kme_restore_app(self._h, str(path).encode(), buf, n.value, C.byref(n))
            if rc:
                raise KmeError(rc, "kme_restore_app")
            return buf.raw[:n.value]
        if rc:
            raise KmeError(rc, "kme_restore_app")
        return b""

    def ledger_stats(self) -> dict:
        """kme_ledger_stats: the exact ledger's table sizes, slots in use and rehashes so far."""
        info = kme_ledger_info()
        rc = self._L.kme_ledger_stats(self._h, C.byref(info))
        if rc:
            raise KmeError(rc, "kme_ledger_stats")
        return {k: int(getattr(info, k)) for k in ("bal_slots", "pos_slots", "bal_used", "pos_used", "grows")}

    def tape_json_device_into(self, ptrs: dict, n: int, out_ptr: int, cap: int) -> int:
        """kme_tape_json_device into a caller device buffer; returns the text length (nothing is
        written when it exceeds cap)."""
        s = kme_orders(*[C.c_void_p(int(ptrs[k])) for k in ("action", "oid", "aid", "sid", "price", "size")])
        got = C.c_size_t(0)
        rc = self._L.kme_tape_json_device(self._h, C.byref(s), n, None, C.c_void_p(int(out_ptr)), cap, C.byref(got))
        if rc:
            raise KmeError(rc, "kme_tape_json_device")
        return got.value

    def tape_json_device(self, ptrs: dict, n: int) -> bytes:
        """kme_tape_json_device over the last device epoch (inputs at `ptrs`, engine-owned results):
        the MatchOut tape printed by the GPU, copied back to the host."""
        import torch

        s = kme_orders(*[C.c_void_p(int(ptrs[k])) for k in ("action", "oid", "aid", "sid", "price", "size")])
        need = C.c_size_t(0)
        rc = self._L.kme_tape_json_device(self._h, C.byref(s), n, None, None, 0, C.byref(need))
        if rc:
            raise KmeError(rc, "kme_tape_json_device")
        buf = torch.empty(max(1, need.value), dtype=torch.uint8, device=f"cuda:{int(self.cfg.device)}")
        got = C.c_size_t(0)
        rc = self._L.kme_tape_json_device(self._h, C.byref(s), n, None, C.c_void_p(buf.data_ptr()), buf.numel(),
                                          C.byref(got))
        if rc:
            raise KmeError(rc, "kme_tape_json_device")
        return buf[: got.value].cpu().numpy().tobytes()

    def snapshot_books(self) -> str:
        return self._text(self._L.kme_snapshot_books)

    def snapshot_ledger(self) -> str:
        return self._text(self._L.kme_snapshot_ledger)


def rccl_load(path: str | None = None):
    """kme_rccl_load: the RCCL the kme_comm_* calls use (None: env KME_RCCL_LIB, else librccl.so.1)."""
    rc = lib().kme_rccl_load(path.encode() if path else None)
    if rc:
        raise KmeError(rc, f"kme_rccl_load({path}): {rccl_last_error()}")


def rccl_last_error() -> str:
    return (lib().kme_rccl_last_error() or b"").decode()


def torch_rccl_path() -> str | None:
    """The RCCL torch's collectives use (its wheel's own copy), if there is one."""
    import torch

    p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    return p if os.path.exists(p) else None


def comm_unique_id() -> bytes:
    """kme_comm_unique_id: 128 bytes for kme_comm_init, made on one rank and sent to all."""
    buf = C.create_string_buffer(128)
    rc = lib().kme_comm_unique_id(buf)
    if rc:
        raise KmeError(rc, f"kme_comm_unique_id: {rccl_last_error()}")
    return buf.raw


class Comm:
    """kme_comm: this engine's rank of an RCCL communicator over the node's engines."""

    def __init__(self, eng: "Engine", n_ranks: int, rank: int, uid: bytes):
        self._L, self.eng, self.n, self.rank = lib(), eng, n_ranks, rank
        h = C.c_void_p()
        b = C.create_string_buffer(bytes(uid), 128)
        rc = self._L.kme_comm_init(eng.handle, n_ranks, rank, b, C.byref(h))
        if rc:
            raise KmeError(rc, f"kme_comm_init: {rccl_last_error()}")
        self._h = h

    def market_data_allgather(self, groups_ptr: int, n_groups: int, rows_per_rank: int, dev_all_ptr: int):
        rc = self._L.kme_market_data_allgather(self.eng.handle, self._h, C.c_void_p(int(groups_ptr)), n_groups,
                                               rows_per_rank, C.c_void_p(int(dev_all_ptr)))
        if rc:
            raise KmeError(rc, f"kme_market_data_allgather: {rccl_last_error()}")

    def credit_rebalance(self):
        rc = self._L.kme_credit_rebalance(self.eng.handle, self._h)
        if rc:
            raise KmeError(rc, f"kme_credit_rebalance: {rccl_last_error()}")

    def close(self):
        if getattr(self, "_h", None):
            self._L.kme_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Processor:
    """kme_processor: the Processor<String, Order> mirror fed MatchIn JSON values.  Forwarded
    records are collected as (key, value) string pairs, as the MatchOut sink would emit them."""

    def __init__(self, cfg: kme_config, epoch_records: int):
        L = lib()
        self._L = L
        self.records: list[tuple[str, str]] = []
        self.commits = 0

        def _fwd(user, key, value, n):
            self.records.append((key.decode(), C.string_at(value, n).decode()))

        def _commit(user):
            self.commits += 1

        self._fwd = FORWARD_FN(_fwd)
        self._commit = COMMIT_FN(_commit)
        h = C.c_void_p()
        rc = L.kme_processor_create(C.byref(cfg), epoch_records, self._fwd, self._commit, None, C.byref(h))
        if rc:
            raise KmeError(rc, "kme_processor_create")
        self._h = h

    def process_json(self, value: str) -> int:
        b = value.encode()
        return self._L.kme_processor_process_json(self._h, b, len(b))

    def punctuate(self) -> int:
        return self._L.kme_processor_punctuate(self._h)

    def close(self) -> int:
        if not self._h:
            return 0
        rc = self._L.kme_processor_close(self._h)
        self._h = None
        return rc

    def last_status(self) -> kme_epoch_status:
        st = kme_epoch_status()
        self._L.kme_processor_last_status(self._h, C.byref(st))
        return st

    def tape_text(self) -> str:
        return "".join(f"{k} {v}\n" for k, v in self.records)


def checkpoint_inspect(path) -> dict:
    """kme_checkpoint_inspect: (file_bytes, app_bytes, digest) from a checkpoint file's trailer."""
    info = kme_checkpoint_info()
    rc = lib().kme_checkpoint_inspect(str(path).encode(), C.byref(info))
    if rc:
        raise KmeError(rc, "kme_checkpoint_inspect")
    return {"file_bytes": int(info.file_bytes), "app_bytes": int(info.app_bytes), "digest": int(info.digest)}


def checkpoint_chunks(path, chunk_bytes: int) -> np.ndarray:
    """kme_checkpoint_chunks: the content hash of each chunk_bytes chunk of a checkpoint file (the state
    changelog's unit)."""
    n = C.c_size_t(0)
    size = os.path.getsize(path)
    out = np.zeros(max(1, (size + chunk_bytes - 1) // chunk_bytes), np.uint64)
    rc = lib().kme_checkpoint_chunks(str(path).encode(), chunk_bytes, out.ctypes.data, len(out), C.byref(n))
    if rc:
        raise KmeError(rc, "kme_checkpoint_chunks")
    return out[: n.value]


def multi_info(m) -> dict:
    """kme_multi_info of a kme_multi handle (an address): whether an unprovable epoch is survivable now,
    the input history's size, cap and durable part, the checkpoint generation."""
    out = kme_multi_status()
    rc = lib().kme_multi_info(C.c_void_p(m), C.byref(out))
    if rc:
        raise KmeError(rc, "kme_multi_info")
    return {f: getattr(out, f) for f, _ in kme_multi_status._fields_}


def order_from_json(value: str):
    """JsonDeserializer<Order> (KP:513-520) of one MatchIn value -> 6-tuple (no device needed)."""
    L = lib()
    a, p, z = C.c_int32(), C.c_int32(), C.c_int32()
    o, ai, s = C.c_int64(), C.c_int64(), C.c_int64()
    b = value.encode()
    rc = L.kme_order_from_json(b, len(b), C.byref(a), C.byref(o), C.byref(ai), C.byref(s), C.byref(p), C.byref(z))
    if rc:
        raise KmeError(rc, "kme_order_from_json")
    return (a.value, o.value, ai.value, s.value, p.value, z.value)


ROW_DTYPE = np.dtype([("oid", "<i8"), ("aid", "<i8"), ("sid", "<i8"), ("prev", "<i8"), ("action", "<i4"),
                      ("price", "<i4"), ("size", "<i4"), ("kind", "u1"), ("has_prev", "u1"), ("_pad", "u1", 2)])
assert ROW_DTYPE.itemsize == 48   # kme_row


def new_result(n: int, trades_cap: int) -> EpochResult:
    """Result arrays of an n-record epoch (page-aligned, so that kme_host_register pins only them)."""
    def arr(count, dt):
        dt = np.dtype(dt)
        raw = np.zeros(count * dt.itemsize + 4096, np.uint8)
        off = (-raw.ctypes.data) % 4096
        return raw[off:off + count * dt.itemsize].view(dt)
    return EpochResult(arr(n, np.int32), arr(n, np.int32), arr(n, np.int64), arr(n, np.uint8), arr(n + 1, np.uint32),
                       arr(trades_cap, TRADE_DTYPE), kme_epoch_status())


def expand_rows(orders: Orders, res: EpochResult, n: int | None = None, threads: int = 1) -> np.ndarray:
    """kme_expand_rows (threads == 1) / kme_expand_rows_mt: the MatchOut rows (ROW_DTYPE) of records
    [0, n) -- IN, fills, OUT."""
    L = lib()
    n = len(orders) if n is None else n
    s, keep = _soa(orders)
    r = kme_epoch_result(_np_ptr(res.out_action), _np_ptr(res.out_size), _np_ptr(res.out_prev),
                         _np_ptr(res.out_flags), _np_ptr(res.trade_off), _np_ptr(res.trades), len(res.trades))
    need = C.c_size_t(0)
    L.kme_expand_rows(C.byref(s), n, C.byref(r), None, 0, C.byref(need))
    rows = np.zeros(need.value, ROW_DTYPE)
    if threads == 1:
        rc = L.kme_expand_rows(C.byref(s), n, C.byref(r), C.c_void_p(rows.ctypes.data), len(rows), C.byref(need))
    else:
        rc = L.kme_expand_rows_mt(C.byref(s), n, C.byref(r), C.c_void_p(rows.ctypes.data), len(rows), C.byref(need),
                                  threads)
    if rc:
        raise KmeError(rc, "kme_expand_rows")
    del keep
    return rows


def tape_json_from(orders: Orders, res: EpochResult) -> str:
    return res.tape_json(orders)


def shard_of(sid: int, n: int) -> int:
    return int(lib().kme_shard_of(int(sid), int(n)))


class kme_orders_buf(C.Structure):
    _fields_ = [("action", C.c_void_p), ("oid", C.c_void_p), ("aid", C.c_void_p), ("sid", C.c_void_p),
                ("price", C.c_void_p), ("size", C.c_void_p)]


class Router:
    """The C-ABI partition router (kme_router_*, include/kme.h): kme/sharding.py PartitionRouter's
    rules in native code, for the product path."""

    def __init__(self, n: int, directory_capacity: int = 1 << 20):
        self._L = lib()
        self.n = n
        h = C.c_void_p()
        rc = self._L.kme_router_create(n, directory_capacity, C.byref(h))
        if rc:
            raise KmeError(rc, "kme_router_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._L.kme_router_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def route(self, orders) -> np.ndarray:
        """Partition of every record (-1 = every partition); updates the oid directory."""
        ko, keep = _soa(orders)
        dest = np.empty(len(orders), np.int32)
        rc = self._L.kme_router_route(self._h, C.byref(ko), len(orders), dest.ctypes.data_as(C.c_void_p))
        if rc:
            raise KmeError(rc, "kme_router_route")
        return dest

    def split(self, orders):
        """-> (parts, echo, seqs) as PartitionRouter.route: per partition its Orders, the mask of
        the records it answers, and their input indices."""
        from .workloads import Orders

        n = len(orders)
        ko, keep = _soa(orders)
        bufs = [{"action": np.empty(n, np.int32), "oid": np.empty(n, np.int64), "aid": np.empty(n, np.int64),
                 "sid": np.empty(n, np.int64), "price": np.empty(n, np.int32), "size": np.empty(n, np.int32)}
                for _ in range(self.n)]
        parts_c = (kme_orders_buf * self.n)(*[kme_orders_buf(*[b[f].ctypes.data for f in
                                                               ("action", "oid", "aid", "sid", "price", "size")])
                                              for b in bufs])
        counts = np.zeros(self.n, np.uint32)
        echo = [np.empty(n, np.uint8) for _ in range(self.n)]
        index = [np.empty(n, np.uint32) for _ in range(self.n)]
        echo_p = (C.c_void_p * self.n)(*[e.ctypes.data for e in echo])
        index_p = (C.c_void_p * self.n)(*[x.ctypes.data for x in index])
        rc = self._L.kme_router_split(self._h, C.byref(ko), n, C.cast(parts_c, C.c_void_p),
                                      counts.ctypes.data_as(C.c_void_p), C.cast(echo_p, C.c_void_p),
                                      C.cast(index_p, C.c_void_p))
        if rc:
            raise KmeError(rc, "kme_router_split")
        parts, echos, seqs = [], [], []
        for k in range(self.n):
            c = int(counts[k])
            b = bufs[k]
            parts.append(Orders(b["action"][:c].copy(), b["oid"][:c].copy(), b["aid"][:c].copy(), b["sid"][:c].copy(),
                                b["price"][:c].copy(), b["size"][:c].copy(), None))
            echos.append(echo[k][:c].astype(bool))
            seqs.append(index[k][:c].astype(np.int64))
        return parts, echos, seqs

    def directory_size(self) -> int:
        return int(self._L.kme_router_directory_size(self._h))
