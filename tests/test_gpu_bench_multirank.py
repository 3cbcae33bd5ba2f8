"""bench.py's multi-rank path on the one-GPU test box (VERDICT r03 "do this" 1).

`python bench.py --gpus N` without torchrun starts its own N ranks (torch.distributed.run as a
child process, before the parent touches the GPU).  With `--backend gloo --comm torch` every rank
shares the box's GPU, so the whole N > 1 branch runs here: the row partition of
/root/reference/src/rSVD.cpp:20-23 (uneven at world 3), the n-side reduce-scatter / all-gather
hooks, the barriers around the timed region, the max-over-ranks time and the self-check's
all-reduce.  The line must carry n_gpus = N and a passing self-check.
"""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=300):
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, cwd=REPO, env=env,
                         capture_output=True, text=True, timeout=timeout)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-3000:]
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.parametrize("world,m,n,config", [(2, 8192, 8192, "c4"), (3, 8191, 8000, "c4"), (2, 8192, 4096, "c5")])
def test_bench_self_launches_ranks(world, m, n, config):
    line = _run(["--gpus", str(world), "--backend", "gloo", "--comm", "torch", "--config", config,
                 "--m", str(m), "--n", str(n), "--steps", "2", "--warmup", "1", "--cpu-budget", "0"])
    assert line["n_gpus"] == world
    assert line["steps"] == 2 and line["value"] > 0 and line["ms_per_step"] > 0
    assert line["config"]["m"] == m and line["config"]["n"] == n
    # rank 0's share by the reference's remainder rule (rank < m % world gets one row more)
    assert line["config"]["m_per_gpu"] == m // world + (1 if m % world else 0)
    assert line["check"]["ok"], line["check"]
    assert line["cpu_baseline"] is None  # the CPU leg runs at N = 1 only
