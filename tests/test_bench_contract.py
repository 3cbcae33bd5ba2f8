"""bench.py's configurations are BASELINE.json's (configs[0..4]) and its metric helpers follow SURVEY.md
§8(d); CPU only (the bench itself needs a GPU)."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

import bench  # noqa: E402


def test_configs_are_the_baseline_ones():
    base = json.load(open(os.path.join(REPO, "BASELINE.json")))["configs"]
    assert len(base) == 5
    want = {  # name: (m, n, l, q, dtype, strong-scaled)
        "c1": (100, 100, 10, 2, "f64", False),         # rank-10 on sparse_matrix100.mtx (I_100)
        "c2": (4096, 4096, 64, 2, "f32", False),       # dense 4096^2 fp32, rank-64, q=2
        "c3": (1048576, 1024, 128, 1, "bf16", False),  # tall-skinny 2^20 x 1024 bf16, rank-128, q=1
        "c4": (65536, 65536, 256, 2, "bf16", True),    # dense 65536^2 bf16, rank-256, row-sharded
        "c5": (131072, 8192, 512, 2, "fp8", True),     # fp8 131072 x 8192, rank-512
    }
    for name, spec in want.items():
        assert bench.CONFIGS[name][:6] == spec, name
    assert "sparse_matrix100" in base[0] and "4096" in base[1] and "1048576" in base[2]
    assert "65536" in base[3] and "131072" in base[4]


def test_algorithmic_flops_formula():
    m, n, l, q = 4096, 4096, 64, 2
    f_proj, f_qr, f_small = bench.algorithmic_flops(m, n, l, q)
    assert f_proj == 2.0 * m * n * l * (2 * q + 2)
    assert f_qr == (q + 1) * (4.0 * m * l * l - 4.0 * l ** 3 / 3) + q * (4.0 * n * l * l - 4.0 * l ** 3 / 3)
    assert f_small == 4.0 * n * l * l - 4.0 * l ** 3 / 3 + 2.0 * n * l * l + 2.0 * m * l * l


def test_committed_evidence_lookups():
    # traffic and MFMA occupancy of the C4 headline kernel come from committed rocprofv3 passes
    tr = bench.pmc_traffic("c4_bf16_65536x65536_l256_q2", "wproj3tn2_kernel<true")
    assert tr is not None and tr[0] > 8.59e9 and tr[1].startswith("profiles/")
    mb = bench.pmc_mfma_busy("c4_bf16_65536x65536_l256_q2", "wproj3tn2_kernel<true")
    assert mb is not None and 0.5 < mb["frac"] < 1.0 and mb["clock_GHz"] <= 2.4
    # a short-dispatch pass (clock estimate above the peak) is priced against its duration at 2.4 GHz
    mb2 = bench.pmc_mfma_busy("c2_f32_4096x4096_l64_q2", "proj_nn_kernel")  # short dispatch: priced at 2.4 GHz
    assert mb2 is not None and mb2["bound"] == "lower" and mb2["clock_GHz"] is None and 0.3 < mb2["frac"] < 1.0


def test_self_launch_builds_torchrun_command(monkeypatch):
    """`python bench.py --gpus N` starts its own N ranks: torch.distributed.run
    with one process per GPU on 127.0.0.1, the bench's flags carried in RSVD_BENCH_ARGV (torchrun's
    own parser would take --m / --n placed after the script).  The GPU run of the same path is
    tests/test_gpu_bench_multirank.py."""
    import json
    import subprocess

    import bench

    seen = {}

    def fake_call(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return 0

    monkeypatch.setattr(subprocess, "call", fake_call)
    argv = ["--gpus", "2", "--config", "c5", "--m", "4096", "--backend", "gloo", "--comm", "torch"]
    monkeypatch.setattr(sys, "argv", ["bench.py"] + argv)
    assert bench.launch_ranks(2) == 0
    cmd = seen["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=2" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert any(c.startswith("--master-port=") for c in cmd)
    assert cmd[-1].endswith("bench.py")
    assert json.loads(seen["env"]["RSVD_BENCH_ARGV"]) == argv
