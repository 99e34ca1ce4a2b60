"""bench.py's multi-rank launcher: `python bench.py --gpus N` without torchrun
starts N rank processes itself, relays rank 0's line and fails when a rank fails; under a launcher
--gpus must equal WORLD_SIZE.  CPU only: the children stop at the USAC_BENCH_DRY_RUN hook, before
any torch / HIP import."""
import json
import os
import subprocess
import sys

import pytest

from tests.conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402

BENCH = os.path.join(ROOT, "bench.py")


def test_launch_plan():
    assert bench.launch_plan(1, {}) == ("self", 1)
    assert bench.launch_plan(4, {}) == ("spawn", 4)
    assert bench.launch_plan(2, {"WORLD_SIZE": "2"}) == ("rank", 2)
    assert bench.launch_plan(1, {"WORLD_SIZE": "1"}) == ("rank", 1)
    how, msg = bench.launch_plan(8, {"WORLD_SIZE": "2"})
    assert how == "refuse" and "WORLD_SIZE is 2" in msg
    assert bench.launch_plan(0, {})[0] == "refuse"
    assert bench.launch_plan(2, {"WORLD_SIZE": "x"})[0] == "refuse"


def _run(args, extra_env):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(extra_env)
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=120, env=env)


def test_spawn_relays_rank0_line():
    r = _run(["--gpus", "3", "--steps", "1"], {"USAC_BENCH_DRY_RUN": "1"})
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 3 and d["rank"] == 0 and d["local_rank"] == 0
    assert d["master"].startswith("127.0.0.1:")


def test_failing_rank_fails_the_launch():
    r = _run(["--gpus", "2"], {"USAC_BENCH_DRY_RUN": "1", "USAC_BENCH_FAIL_RANK": "1"})
    assert r.returncode == 5
    assert "rank 1 exited with status 5" in r.stderr


def test_failing_rank0_ends_waiting_ranks():
    r = _run(["--gpus", "2"], {"USAC_BENCH_DRY_RUN": "1", "USAC_BENCH_FAIL_RANK": "0",
                               "USAC_BENCH_DRY_SLEEP": "60"})
    assert r.returncode == 5  # the sleeping rank 1 was ended, not waited for


@pytest.mark.parametrize("flag", [[], ["--cfg5"]])
def test_mismatched_world_refused(flag):
    r = _run(["--gpus", "8"] + flag, {"WORLD_SIZE": "2", "RANK": "0", "USAC_BENCH_DRY_RUN": "1"})
    assert r.returncode == 2
    assert "WORLD_SIZE is 2" in r.stderr
