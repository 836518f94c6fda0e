"""Test configuration: paths, the `gpu` marker, and session builds of the two libraries.

CPU tests (-m "not gpu") exercise the oracle against the committed golden vectors, host logic and
the C ABI surface; GPU tests (-m gpu) are the parity tests proper: HIP engine vs oracle.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "kafka-matching-engine_amd")
ORACLE = os.path.join(ROOT, "oracle")
for p in (PKG, ORACLE, ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); the parity tests proper")


@pytest.fixture(scope="session")
def oracle_mod():
    if not os.path.exists(os.path.join(ORACLE, "libkme_oracle.so")):
        subprocess.run(["make", "-s", "-C", ORACLE], check=True)
    import oracle

    return oracle


# the sources kme_build_id() hashes (kafka-matching-engine_amd/csrc/Makefile SRCS, same order)
LIB_SOURCES = ["kme_kernels.hip", "kme_serialize.hip", "kme_runtime.cpp", "kme_host.cpp", "kme_processor.cpp",
               "kme_router.cpp", "kme_device.h", "kme_launch.h", "kme_processor.hpp", "../../include/kme.h",
               "../../include/kme_processor.h", "kme_multi.cpp", "kme_internal.h", "kme_ledger.hip", "kme_jarith.h", "kme_maint.hip", "kme_ckpt.cpp"]


def source_hash() -> str:
    import hashlib

    h = hashlib.sha256()
    for f in LIB_SOURCES:
        with open(os.path.join(PKG, "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def built_id(path) -> str:
    """kme_build_id() of a built libkme.so, read from the file (loading it here would pin that copy
    in the process before a rebuild)."""
    import re

    with open(path, "rb") as fh:
        data = fh.read()
    want = source_hash().encode()
    return want.decode() if want in data else (re.findall(rb"[0-9a-f]{16}", data) or [b"?"])[0].decode()


@pytest.fixture(scope="session")
def kme_mod():
    """libkme.so built from THIS tree: rebuilt (make is incremental) when missing or when its
    kme_build_id() differs from the sources' hash, so a test run never uses a stale library."""
    so = os.path.join(PKG, "kme", "libkme.so")
    if not os.path.exists(so) or built_id(so) != source_hash():
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(PKG, "csrc")], check=True)
    import kme

    L = kme.lib()
    got = L.kme_build_id().decode()
    assert got == source_hash(), f"libkme.so was built from other sources ({got} != {source_hash()})"
    return kme
