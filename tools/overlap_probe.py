"""Diagnostic: do two epochs' kernels gain from running at the same time?  Two independent FUNDED
engines (each half of the C3 symbols and records, own HIP stream) run their epochs either one after
the other or concurrently; the ratio bounds what overlapping consecutive epochs of one engine could
give.  Usage (through gpurun): python3 tools/overlap_probe.py [epochs]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kafka-matching-engine_amd"))

import torch  # noqa: E402

import kme  # noqa: E402
from kme import workloads as W  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    E = 1 << 21
    S = 32768
    dev = torch.device("cuda", 0)
    engines, inputs = [], []
    for part in range(2):
        setup = W.funded_setup(32768, range(1, S + 1))
        stream = W.uniform((K + 2) * E, n_symbols=S, n_accounts=32768, seed=100 + part)
        cfg = kme.default_config(kme.MODE_FUNDED, max_symbols=S + 1, max_epoch=E, max_resting=(K + 2) * E,
                                 max_trades=2 * E + (1 << 16), max_accounts=32768)
        eng = kme.Engine(cfg)
        st = torch.cuda.Stream(dev)
        eng.set_stream(st.cuda_stream)
        eng.process(setup)
        cols = {c: torch.from_numpy(np.ascontiguousarray(getattr(stream, c))).to(dev)
                for c in ("action", "oid", "aid", "sid", "price", "size")}
        engines.append(eng)
        inputs.append(cols)

    def ptrs(part, k):
        return {c: t.data_ptr() + k * E * t.element_size() for c, t in inputs[part].items()}

    for e in range(2):
        engines[e].submit_device(ptrs(e, 0), E)
        engines[e].wait()
    torch.cuda.synchronize()
    # sequential: A then B, each waited
    t = time.perf_counter()
    for k in range(1, 1 + K // 2):
        for e in range(2):
            engines[e].submit_device(ptrs(e, k), E)
            engines[e].wait()
    seq = time.perf_counter() - t
    # concurrent: A and B submitted together
    t = time.perf_counter()
    for k in range(1 + K // 2, 1 + K):
        for e in range(2):
            engines[e].submit_device(ptrs(e, k), E)
        for e in range(2):
            engines[e].wait()
    conc = time.perf_counter() - t
    n = (K // 2) * 2 * E
    print(f"sequential {n / seq / 1e6:.0f} M records/s, concurrent {n / conc / 1e6:.0f} M records/s, "
          f"ratio {seq / conc:.2f}")


if __name__ == "__main__":
    main()
