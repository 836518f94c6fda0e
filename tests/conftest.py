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


@pytest.fixture(scope="session")
def kme_mod():
    if not os.path.exists(os.path.join(PKG, "kme", "libkme.so")):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(PKG, "csrc")], check=True)
    import kme

    kme.lib()
    return kme
