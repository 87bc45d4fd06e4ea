"""bench.py as the driver runs it: `python bench.py --gpus N` with NO torchrun variables must start its
N ranks itself (one process per GPU, rank 0 prints the one JSON line), and N = 1 must print the same
kind of line.  On the one-GPU box the two ranks share cuda:0 over gloo (`--same-device`), which
rehearses the code path (the numbers are not a measurement).  Replaces the reference's threaded
stripe loop as the unit of parallel work (multiply_1DVBC.jl:169-177)."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent
DIST_VARS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
             "GROUP_RANK", "ROLE_RANK", "TORCHELASTIC_RUN_ID")


def run_bench(*args, timeout=110):
    env = {k: v for k, v in os.environ.items() if k not in DIST_VARS}
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=str(ROOT))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]  # exactly one JSON line (rank 0 only)
    return json.loads(lines[0])


def test_bench_self_launches_two_ranks():
    d = run_bench("--gpus", "2", "--backend", "gloo", "--same-device", "--scale", "0.01", "--no-secondary",
                  "--no-abi-sharded", "--steps", "3", "--warmup", "1")
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["warmup"] == 1
    assert d["value"] > 0 and d["unit"] == "GB/s" and d["scaling"] == "strong"
    assert "stripe split x2" in d["config"]["parallelism"]
    assert d["parity"]["pass"] and d["parity"]["serial_bitwise_equal"]


def test_bench_multi_gpu_line_checks_itself():
    """the N > 1 line proves its numbers: the primary's gathered y, the C3 secondary's B'x
    and its forward all_reduce, and the one-process C-ABI sharded leg (vbc1d_create_sharded, devices
    [0, 0] on a one-GPU box) are all compared with the oracle."""
    d = run_bench("--gpus", "2", "--backend", "gloo", "--same-device", "--scale", "0.01", "--steps", "3",
                  "--warmup", "1", timeout=300)
    assert d["parity"]["pass"] and len(d["parity"]["slices_bitwise"]) == 2
    c3 = d["secondary"]["c3_ldoor"]
    assert c3["parity"]["pass"] and c3["forward_allreduce"]["parity"]["pass"]
    abi = d["secondary"]["abi_sharded"]
    assert abi["pass"] and abi["devices"] == [0, 0], abi
    for k in ("transposed", "forward"):
        assert abi[k]["parity"]["pass"] and abi[k]["value"] > 0


def test_bench_single_gpu_line():
    d = run_bench("--scale", "0.01", "--no-secondary", "--no-cpu-baseline", "--steps", "3", "--warmup", "1")
    assert d["n_gpus"] == 1 and d["value"] > 0
    assert d["roofline"]["frac"] > 0 and d["roofline"]["bound"] == "hbm"
    assert d["parity"]["pass"] and d["parity"]["rel_err"] <= 1e-10
    assert "cache" in d["config"]
