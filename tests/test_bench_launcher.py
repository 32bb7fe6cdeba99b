"""bench.py's multi-rank contract on CPU: `python bench.py --gpus N` with no RANK in the
environment starts N rank processes itself, times K steps between barriers, takes the max over
ranks and prints ONE JSON line on rank 0 with n_gpus = N and the whole-job value.

--selftest swaps the training step for its cross-rank part alone (a gloo all-reduce of a
gradient-sized buffer), so the launcher, rendezvous (127.0.0.1), timing and output line are
exercised without a GPU.  The GPU step itself is covered by tests/test_gpu_dp.py."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None):
    e = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, capture_output=True, text=True,
                         timeout=240, env=e, cwd="/tmp")
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout          # exactly one JSON line, from rank 0
    return json.loads(lines[0])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("n", [2, 4])
def test_bench_spawns_n_ranks(n):
    line = _run(["--gpus", str(n), "--selftest", "--steps", "3", "--warmup", "1", "--batch", "32"])
    assert line["n_gpus"] == n
    assert line["steps"] == 3 and line["warmup"] == 1
    assert line["config"]["global_batch"] == 32 * n and line["config"]["parallelism"] == f"dp{n}"
    assert line["grad_mean_ok"] is True          # every rank ended with the mean over ranks
    assert line["value"] == pytest.approx(n * 32 * 3 / (line["ms_per_step"] * 3 / 1e3), rel=1e-2)


@pytest.mark.timeout(120)
def test_bench_single_rank_default():
    line = _run(["--selftest", "--steps", "2", "--warmup", "0"])
    assert line["n_gpus"] == 1 and line["config"]["parallelism"] == "dp1"
