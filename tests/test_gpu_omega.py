"""The bf16 / e4m3 Omega (omega_lowp_kernel, two stream elements per thread for even n) is the fp64
Philox Gaussian stream (gauss_elem; util.hip, oracle/rsvd_oracle.c orc_philox_gaussian) rounded to
8 (bf16) / 4 (e4m3) significant bits, round-half-even -- bit for bit, for even and odd n."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _round_sig(x, bits, fp8):
    y = np.zeros_like(x)
    nz = (x != 0) & np.isfinite(x)
    e = np.floor(np.log2(np.abs(x[nz])))
    if fp8:
        e = np.maximum(e, -6.0)
    q = np.exp2(e - bits)
    y[nz] = np.rint(x[nz] / q) * q
    if fp8:
        y = np.clip(y, -448.0, 448.0)
    return y


@pytest.mark.parametrize("n,l", [(4096, 256), (1001, 96), (2048, 512)])
@pytest.mark.parametrize("fp8", [False, True])
def test_lowp_omega_is_the_rounded_fp64_stream(engine, n, l, fp8):
    import torch

    seed = 0x5EED0002
    o64 = engine.generate_omega(n, l, seed=seed, dtype=torch.float64).cpu().numpy()
    dt = torch.float8_e4m3fn if fp8 else torch.bfloat16
    olp = engine.generate_omega(n, l, seed=seed, dtype=dt).cpu().double().numpy()
    assert olp.shape == (n, l)
    assert np.array_equal(olp, _round_sig(o64, 3 if fp8 else 7, fp8))
