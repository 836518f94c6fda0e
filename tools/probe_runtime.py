"""Probe: which HIP runtime does libkme bind to when torch is imported first / second?"""
import ctypes, os, sys
order = sys.argv[1]
sys.path.insert(0, "kafka-matching-engine_amd")
if order == "torch_first":
    import torch
    print("torch", torch.__version__, torch.cuda.is_available(), torch.cuda.device_count())
import kme
kme.lib()
if order != "torch_first":
    import torch
    print("torch", torch.__version__, torch.cuda.is_available(), torch.cuda.device_count())
maps = open("/proc/self/maps").read()
print(sorted({l.split()[-1] for l in maps.splitlines() if "amdhip64" in l or "hsa-runtime" in l}))
from kme import workloads as W
eng = kme.Engine(kme.default_config(kme.MODE_FUNDED, max_symbols=9, max_epoch=1 << 14, max_resting=1 << 14, max_accounts=64))
r = eng.process(W.Orders.concat([W.funded_setup(64, range(1, 9)), W.uniform(5000, n_symbols=8, n_accounts=64, seed=2)]))
t = torch.zeros((9, 4), dtype=torch.int32, device="cuda")
eng.top_of_book(t.data_ptr()); torch.cuda.synchronize(); eng.wait()
print("tob", t.cpu().numpy()[1:3].tolist(), "trades", r.status.n_trades)
