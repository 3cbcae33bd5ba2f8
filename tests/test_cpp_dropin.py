"""The C++ drop-in adapters compile against the C ABI (CPU) and reproduce the reference's call
shapes through it (GPU):

* tests/cpp/dropin_test.cpp -- the generic adapter include/rsvd.hpp on a minimal matrix type;
* tests/cpp/eigen_dropin_test.cpp -- the Eigen-typed headers include/rSVD.hpp, include/QR.hpp and
  include/SVD_class.hpp with the reference's exact signatures (rSVD_test.cpp:72, svd_test.cpp:58, a
  PCA_class.hpp:11-47-style subclass calling the protected setData), compiled over
  tests/cpp/eigen_shim (a minimal stand-in for the Eigen API slice they use: Eigen is absent from
  this image), plus the library-owned RCCL entry (rsvd::distributed_init) at world 1."""
import os
import subprocess

import pytest

from conftest import REPO

CPP = os.path.join(REPO, "tests", "cpp")


def _build():
    import rsvd_kamaneh_raganato_terrana_amd as R

    R.build(force=False)
    subprocess.run(["make", "-C", CPP, "-s"], check=True, capture_output=True)
    return os.path.join(CPP, "dropin_test"), os.path.join(CPP, "eigen_dropin_test")


def test_cpp_adapters_compile_and_link():
    for exe in _build():
        assert os.access(exe, os.X_OK), exe


@pytest.mark.gpu
def test_cpp_adapter_identity_known_answer():
    exe = _build()[0]
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASSED" in r.stdout


@pytest.mark.gpu
def test_eigen_typed_dropin_headers_run():
    exe = _build()[1]
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASSED" in r.stdout
