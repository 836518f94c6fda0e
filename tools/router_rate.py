"""The C partition router's rate (kme_router_route / kme_router_split, kme_router.cpp) on this host:
2^22-record epochs of the C3 stream (65,536 symbols, 30% cancels) into 8 partitions, the oid directory
carried over epochs, for several thread counts (KME_ROUTER_THREADS).  Host-only work.
Usage: python3 tools/router_rate.py [threads ...]"""
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))


def one(threads):
    sys.path.insert(0, os.path.join(HERE, "..", "kafka-matching-engine_amd"))
    import ctypes as C

    import numpy as np

    import kme
    from kme import workloads as W
    E, EP, P = 1 << 22, 6, 8
    L = kme.lib()
    orders = W.uniform(EP * E, n_symbols=65_536, n_accounts=65_536, seed=9)
    r = kme.Router(P, directory_capacity=1 << 24)
    # the C calls only, into buffers made (and touched) once, as kme_multi.cpp uses them
    dest = np.ones(E, np.int32)
    cols = [{f: np.ones(E, t) for f, t in (("action", np.int32), ("oid", np.int64), ("aid", np.int64),
                                            ("sid", np.int64), ("price", np.int32), ("size", np.int32))} for _ in range(P)]
    parts = (kme.kme_orders_buf * P)(*[kme.kme_orders_buf(*[b[f].ctypes.data for f in
                                                            ("action", "oid", "aid", "sid", "price", "size")])
                                       for b in cols])
    echo = [np.ones(E, np.uint8) for _ in range(P)]
    index = [np.ones(E, np.uint32) for _ in range(P)]
    echo_p = (C.c_void_p * P)(*[e.ctypes.data for e in echo])
    index_p = (C.c_void_p * P)(*[x.ctypes.data for x in index])
    counts = np.zeros(P, np.uint32)
    route, split = [], []
    for ep in range(EP):
        ko, keep = kme._soa(orders.slice(ep * E, (ep + 1) * E))
        t = time.perf_counter()
        if ep % 2 == 0:
            rc = L.kme_router_route(r._h, C.byref(ko), E, dest.ctypes.data_as(C.c_void_p))
            route.append(E / (time.perf_counter() - t))
        else:
            rc = L.kme_router_split(r._h, C.byref(ko), E, C.cast(parts, C.c_void_p), counts.ctypes.data_as(C.c_void_p),
                                    C.cast(echo_p, C.c_void_p), C.cast(index_p, C.c_void_p))
            split.append(E / (time.perf_counter() - t))
        assert rc == 0, rc
    return {"threads": threads, "route_M_per_s": round(max(route) / 1e6, 1), "split_M_per_s": round(max(split) / 1e6, 1),
            "epoch_records": E, "partitions": P, "directory": int(r.directory_size())}


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--one":
        print(json.dumps(one(int(os.environ["KME_ROUTER_THREADS"]))))
        sys.exit(0)
    for t in (sys.argv[1:] or ["1", "8", "16"]):
        env = dict(os.environ, KME_ROUTER_THREADS=t)
        subprocess.run([sys.executable, __file__, "--one"], env=env, check=True)
