"""bench.py --gpus N with no launcher around it (the driver's command form):
the process starts N ranks itself before anything touches the GPU
(bench.launch_ranks).  CPU only: the ranks stop at --launch-check, which
reports the rank environment they were given before any GPU call."""
import json
import os
import re
import subprocess
import sys

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _env():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    return env


def test_gpus_n_starts_n_ranks_without_torch_in_the_parent():
    r = subprocess.run([sys.executable, "-X", "importtime", BENCH, "--gpus", "3", "--launch-check"],
                       capture_output=True, text=True, timeout=300, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    ranks = [json.loads(x) for x in r.stdout.splitlines() if x.startswith('{"rank"')]
    assert sorted(d["rank"] for d in ranks) == [0, 1, 2]
    assert sorted(d["local_rank"] for d in ranks) == [0, 1, 2]
    assert all(d["world"] == 3 and d["gpus"] == 3 for d in ranks)
    assert len({d["master"] for d in ranks}) == 1 and ranks[0]["master"].startswith("127.0.0.1:")
    assert not any(d["torch_cuda_initialized"] for d in ranks)
    # -X importtime applies to the parent only (the ranks are started without it): the parent
    # imported neither torch nor the engine package
    parent_imports = [ln.rsplit("|", 1)[-1].strip() for ln in r.stderr.splitlines() if ln.startswith("import time:")]
    assert parent_imports, "no import-time trace from the parent"
    assert not [m for m in parent_imports if re.match(r"(torch|numpy|plenum_amd)(\.|$)", m)]


def test_failing_rank_fails_the_launch():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--config", "c9"], capture_output=True, text=True,
                       timeout=300, env=_env(), cwd=ROOT)
    assert r.returncode == 2  # argparse's exit code in the ranks, relayed
    assert "invalid choice" in r.stderr  # (the other rank may have been stopped before it printed)


def test_one_gpu_runs_in_process():
    """--gpus 1 (the default) never launches: the launcher is not involved."""
    r = subprocess.run([sys.executable, BENCH, "--launch-check"], capture_output=True, text=True, timeout=300,
                       env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith('{"rank"')][0])
    assert d["world"] == 1 and d["rank"] == 0 and d["master"] == "None:None"
