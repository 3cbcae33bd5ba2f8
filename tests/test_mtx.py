"""MatrixMarket I/O (rsvd_kamaneh_raganato_terrana_amd/mtx.py) and the reference harness mirror
(tools/rsvd_test.py): the inputs it regenerates equal the reference's input/*.mtx (compared
here when the reference tree is present), reads agree with the oracle's reader, writes round-trip
exactly.  GPU: the harness reproduces the known answers of SURVEY.md §8c on those inputs."""
import os
import sys

import numpy as np
import pytest

from conftest import REPO

sys.path.insert(0, os.path.join(REPO, "tools"))

import oracle  # noqa: E402  (test infrastructure)
import rsvd_test  # noqa: E402
from rsvd_kamaneh_raganato_terrana_amd.mtx import read_market, write_market  # noqa: E402

REF_INPUT = "/root/reference/input"


@pytest.fixture(scope="module")
def inputs(tmp_path_factory):
    d = str(tmp_path_factory.mktemp("input"))
    rsvd_test.make_inputs(d)
    return d


def test_generated_inputs_known_structure(inputs):
    for k in (100, 110, 140, 160):
        A = read_market(os.path.join(inputs, f"sparse_matrix{k}.mtx"))
        assert np.array_equal(A, np.eye(k))
    A = read_market(os.path.join(inputs, "sparse_matrix.mtx"))
    i, j = np.meshgrid(np.arange(100), np.arange(100), indexing="ij")
    assert np.array_equal(A, 100.0 * i + j + 1)
    assert np.linalg.matrix_rank(A) == 2


def test_reader_agrees_with_oracle_reader(inputs):
    for name in sorted(os.listdir(inputs)):
        p = os.path.join(inputs, name)
        assert np.array_equal(read_market(p), oracle.read_matrix_market(p))


@pytest.mark.skipif(not os.path.isdir(REF_INPUT), reason="reference tree absent")
def test_generated_inputs_equal_reference_files(inputs):
    for name in sorted(os.listdir(REF_INPUT)):
        ours = read_market(os.path.join(inputs, name))
        ref = read_market(os.path.join(REF_INPUT, name))
        assert np.array_equal(ours, ref), name


def test_write_read_round_trip(tmp_path):
    rng = np.random.default_rng(0)
    X = rng.standard_normal((13, 7)) * 10.0 ** rng.integers(-300, 300, (13, 7))
    p = str(tmp_path / "x.mtx")
    write_market(p, X)
    assert np.array_equal(read_market(p), X)
    s = rng.standard_normal(9)
    write_market(p, s)
    Y = read_market(p)
    assert Y.shape == (9, 1) and np.array_equal(Y[:, 0], s)
    with open(p) as f:
        assert f.readline().strip() == "%%MatrixMarket matrix coordinate real general"
        assert f.readline().split() == ["9", "1", "9"]


def test_reader_symmetric_array_and_pattern(tmp_path):
    p = str(tmp_path / "s.mtx")
    with open(p, "w") as f:
        f.write("%%MatrixMarket matrix coordinate real symmetric\n% comment\n3 3 4\n1 1 2\n2 1 5\n3 2 -1\n3 3 4\n")
    assert np.array_equal(read_market(p), np.array([[2, 5, 0], [5, 0, -1], [0, -1, 4.0]]))
    with open(p, "w") as f:
        f.write("%%MatrixMarket matrix array real general\n2 3\n1\n2\n3\n4\n5\n6\n")
    assert np.array_equal(read_market(p), np.array([[1, 3, 5], [2, 4, 6.0]]))
    with open(p, "w") as f:
        f.write("%%MatrixMarket matrix coordinate pattern general\n2 2 2\n1 2\n2 1\n")
    assert np.array_equal(read_market(p), np.array([[0, 1], [1, 0.0]]))


@pytest.mark.gpu
def test_rsvd_harness_known_answers(inputs, tmp_path):
    out = str(tmp_path / "out")
    res = {r["name"]: r for r in rsvd_test.run(inputs, out, "rsvd", 16, 0x5EED0001)}
    for k in (100, 110, 140, 160):
        r = res[f"sparse_matrix{k}.mtx"]
        assert np.abs(r["S"] - 1.0).max() < 1e-12
        assert abs(r["norm_of_diff"] - np.sqrt(k - 16)) < 1e-10
    r = res["sparse_matrix.mtx"]
    assert abs(r["S"][0] - 577391.767) / 577391.767 < 1e-9 and abs(r["S"][1] - 1443.12761) / 1443.12761 < 1e-8
    assert r["norm_of_diff"] < 1e-12 * np.linalg.norm(read_market(os.path.join(inputs, "sparse_matrix.mtx")))
    S = read_market(os.path.join(out, "sparse_matrix_S.mtx"))[:, 0]
    assert np.array_equal(S, r["S"])
    assert read_market(os.path.join(out, "sparse_matrix100_U.mtx")).shape == (100, 16)
    assert read_market(os.path.join(out, "sparse_matrix100_V.mtx")).shape == (100, 16)


@pytest.mark.gpu
def test_svd_harness_identity(inputs, tmp_path):
    out = str(tmp_path / "out")
    res = {r["name"]: r for r in rsvd_test.run(inputs, out, "svd", 16, 0)}
    for k in (100, 160):
        r = res[f"sparse_matrix{k}.mtx"]
        assert np.abs(r["S"] - 1.0).max() < 1e-13 and r["norm_of_diff"] < 1e-12
    assert read_market(os.path.join(out, "sparse_matrix140_U.mtx")).shape == (140, 140)
