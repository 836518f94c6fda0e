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
    import kme
    from kme import workloads as W
    E, EP = 1 << 22, 4
    orders = W.uniform(EP * E, n_symbols=65_536, n_accounts=65_536, seed=9)
    r = kme.Router(8, directory_capacity=1 << 24)
    route, split = [], []
    for ep in range(EP):
        part = orders.slice(ep * E, (ep + 1) * E)
        t = time.perf_counter()
        if ep % 2 == 0:
            r.route(part)
            route.append(E / (time.perf_counter() - t))
        else:
            r.split(part)
            split.append(E / (time.perf_counter() - t))
    return {"threads": threads, "route_M_per_s": round(max(route) / 1e6, 1), "split_M_per_s": round(max(split) / 1e6, 1)}


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--one":
        print(json.dumps(one(int(os.environ["KME_ROUTER_THREADS"]))))
        sys.exit(0)
    for t in (sys.argv[1:] or ["1", "8", "16"]):
        env = dict(os.environ, KME_ROUTER_THREADS=t)
        subprocess.run([sys.executable, __file__, "--one"], env=env, check=True)
