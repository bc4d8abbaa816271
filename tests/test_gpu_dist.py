"""The N > 1 bench path with the HIP engine on every rank (test_dist_gloo.py
covers the sharding and collectives with the CPU oracle per rank): two ranks
of bench.py under torch.distributed.run, gloo, both on cuda:0 (the box's one
GPU), configs[4]'s step at a small size (160,000 requests per rank: a multiple of 64, and
of 100 / world so the 3PC keys cover every vote).  The all-gathered bitmask equals the
construction (every request valid) and the MAX-unioned ballots give the
expected per-key counts and quorum flags, primary-PREPARE rule included
(bench.py tally_check)."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_bench_two_ranks_one_gpu():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--dist-backend", "gloo", "--same-device", "--config", "c4", "--requests", "160000",
           "--signers", "64", "--key-window", "10", "--steps", "2", "--warmup", "1", "--no-cpu",
           "--general-steps", "0", "--dropin-steps", "0", "--e2e-n", "0", "--e2e-c0", "0"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=ROOT, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-8000:])
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith('{"metric')][-1])
    assert d["n_gpus"] == 2 and d["config"]["requests_per_gpu"] == 160000
    p = d["parity"]
    assert p["mismatches_vs_construction"] == 0 and p["accepted"] == p["expected"] == 2 * 160000
    assert p["accepted_in_gathered_bitmask"] == 2 * 160000
    assert d["tally"]["counts_match"] and d["tally"]["quorum_match"]
    assert d["tally"]["prepare_quorums"] > 0 and d["tally"]["commit_quorums"] > 0
    # near-threshold keys (synth.c4_votes): quorums missed by one vote, and keys whose prepare quorum
    # the primary-PREPARE rule decides, checked across the two ranks' unioned ballots
    assert d["tally"]["keys_below_prepare_quorum"] > 0 and d["tally"]["keys_below_commit_quorum"] > 0
    assert d["tally"]["keys_decided_by_primary_rule"] > 0


def test_bench_gpus_2_without_launcher():
    """The driver's bare command form: `python bench.py --gpus 2` starts its two
    ranks itself (bench.launch_ranks); both run the HIP engine (gloo, one GPU),
    the line reports n_gpus == 2, the all-gathered bitmask is exact, and the
    whole-node headline ran on both ranks (each its own authenticator over its
    own json-decoded batches, the host's CPUs split between them): value =
    both ranks' requests over the slower rank's time, every outcome exact."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo", "--same-device",
           "--requests", "131072", "--signers", "64", "--key-window", "10", "--steps", "2", "--warmup", "1",
           "--device-steps", "2", "--whole-node-n", "65536",
           "--no-cpu", "--general-steps", "0", "--dropin-steps", "0", "--e2e-n", "0", "--e2e-c0", "0"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=180, cwd=ROOT, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-8000:])
    lines = [x for x in r.stdout.splitlines() if x.startswith('{"metric')]
    assert len(lines) == 1  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["requests_per_gpu"] == 65536 and d["steps"] == 2
    p = d["parity"]
    assert p["mismatches_vs_construction"] == 0 and p["accepted"] == p["expected"] == 2 * 131072
    assert p["accepted_in_gathered_bitmask"] == 2 * 131072
    assert d["collective"]["all_gather_bitmask_ms"] > 0
    w = d["whole_node"]
    assert w["mismatches_all_ranks"] == 0 and p["whole_node_mismatches"] == 0
    assert w["synchronous"]["value"] == d["value"] and w["synchronous"]["value_per_rank"] * 2 == d["value"]
    assert w["pipelined"]["value"] > 0 and w["scan_threads"] != "auto"
    assert d["device_resident"]["value"] > 0


def test_bench_rccl_path_one_rank():
    """The RCCL exchange path of bench.py (nccl process group with device_id,
    the bitmask all-gather, the ballot all-reduce MAX on configs[4], barriers,
    the max-over-ranks timing) run as a one-rank group on this box's GPU
    (--force-dist): the calls SCALE makes at N = 2..8, exercised on ROCm."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--force-dist", "--config", "c4", "--requests", "131072",
           "--signers", "64", "--key-window", "10", "--steps", "2", "--warmup", "1", "--no-cpu",
           "--general-steps", "0", "--dropin-steps", "0", "--e2e-n", "0", "--e2e-c0", "0"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=ROOT, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-8000:])
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith('{"metric')][-1])
    assert d["n_gpus"] == 1 and d["parity"]["accepted_in_gathered_bitmask"] == 131072
    assert d["collective"]["all_gather_bitmask_ms"] > 0 and d["collective"]["all_reduce_max_ballots_ms"] > 0
    assert d["tally"]["counts_match"] and d["tally"]["quorum_match"]


def test_configs4_per_gpu_shard_at_full_size():
    """configs[4] at its per-GPU size: the 16M-request batch sharded over 8
    GPUs is a 2M-request shard per GPU (two 2^20-request chunks through the
    step) plus the full-K PREPARE/COMMIT tally of the whole job (K = 16M / 2 /
    50 keys would be 160,000 on 8 ranks; here the one rank's K = 20,000 keys x
    25 validators), through the RCCL exchange path as a one-rank group
    (--force-dist: nccl process group, bitmask all-gather, ballot all-reduce
    MAX).  Checked: the gathered bitmask accepts exactly the construction's 2M,
    the tally's counts and quorum flags equal the construction's (primary-PREPARE
    rule included, plenum/server/quorums.py:15-32, models.py:21-37,
    replica.py:1289-1291), and libsodium 1.0.18 agrees with the GPU on every
    one of the 2M verdicts and on a 6,000-request sample timed as the CPU leg."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--force-dist", "--config", "c4", "--requests", "2000000",
           "--key-window", "10", "--steps", "2", "--warmup", "1", "--cpu-sample", "6000",
           "--general-steps", "0", "--dropin-steps", "0", "--e2e-n", "0", "--e2e-c0", "0", "--whole-node-n", "0"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, cwd=ROOT, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-8000:])
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith('{"metric')][-1])
    assert d["n_gpus"] == 1 and d["config"]["requests_per_gpu"] == 2000000
    p = d["parity"]
    assert p["mismatches_vs_construction"] == 0 and p["accepted"] == p["expected"] == 2000000
    assert p["accepted_in_gathered_bitmask"] == 2000000
    assert p["mismatches_vs_libsodium_all_items"] == 0
    c = d["cpu_baseline"]
    assert c["agrees_with_gpu"] and c["all_items_check"]["items"] == 2000000
    t = d["tally"]
    assert t["counts_match"] and t["quorum_match"] and t["keys"] == 20000 and t["votes_per_gpu"] == 1000000
    assert t["prepare_quorums"] > 0 and t["commit_quorums"] > 0
    assert t["keys_below_prepare_quorum"] > 0 and t["keys_decided_by_primary_rule"] > 0
    assert d["collective"]["all_gather_bitmask_ms"] > 0 and d["collective"]["all_reduce_max_ballots_ms"] > 0
