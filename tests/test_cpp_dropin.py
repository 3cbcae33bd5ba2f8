"""The C++ drop-in adapter (include/rsvd.hpp, under include/rSVD.hpp) compiles against the C ABI
(CPU) and reproduces tests/rSVD_test.cpp's identity known answer through it (GPU)."""
import os
import subprocess

import pytest

from conftest import REPO

CPP = os.path.join(REPO, "tests", "cpp")


def _build():
    import rsvd_kamaneh_raganato_terrana_amd as R

    R.build()
    subprocess.run(["make", "-C", CPP, "-s"], check=True, capture_output=True)
    return os.path.join(CPP, "dropin_test")


def test_cpp_adapter_compiles_and_links():
    exe = _build()
    assert os.access(exe, os.X_OK)


@pytest.mark.gpu
def test_cpp_adapter_identity_known_answer():
    exe = _build()
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASSED" in r.stdout
