"""Shared pytest configuration.

Markers:
  gpu  -- needs a real MI355X (run on the GPU box: ``pytest -m gpu``).
Everything unmarked runs on CPU only and must stay within a few minutes.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs an AMD MI355X GPU")


GOLDEN = os.path.join(ROOT, "tests", "golden", "golden.npz")


def load_golden():
    """{name: dict(input, bwt, mtf, rle, lengths, payload, pi, orig_size, encoded_size)}."""
    z = np.load(GOLDEN, allow_pickle=False)
    out = {}
    for name in z["names"]:
        name = str(name)
        s = z[f"{name}/scalars"]
        out[name] = dict(
            input=z[f"{name}/input"].tobytes(),
            bwt=z[f"{name}/bwt"].tobytes(),
            mtf=z[f"{name}/mtf"].tobytes(),
            rle=z[f"{name}/rle"].tobytes(),
            lengths=z[f"{name}/lengths"].tobytes(),
            payload=z[f"{name}/payload"].tobytes(),
            pi=int(s[0]),
            orig_size=int(s[1]),
            encoded_size=int(s[2]),
        )
    return out


@pytest.fixture(scope="session")
def golden():
    return load_golden()


@pytest.fixture(scope="session")
def orc():
    from oracle import Oracle

    lib = os.path.join(ROOT, "oracle", "liboracle.so")
    if not os.path.exists(lib):
        import subprocess

        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle"), "liboracle.so"])
    return Oracle()
