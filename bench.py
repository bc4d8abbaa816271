"""Ed25519 request verifies/sec on MI355X -- the BASELINE.json headline metric.

One step = one pass of the verify path over this rank's batch, inputs already
resident in HBM.  Key-table path (default; the signers' verkeys registered
once, like SimpleAuthNr.addIdr): hash kernel (prechecks + SHA-512(R||A||M)
mod L) -> comb kernel ([h](-A) + [S]B from the key's and the base point's
fixed-base tables) -> encode kernel (16 results per lane share one inversion;
encode, compare with R, wave ballot) -> accept bitmask.  General path (any key
bytes per request): hash -> table (decode -A, [1..8](-A)) -> dsm -> encode.
For N > 1 the step ends with the RCCL all-gather of the bitmask words (the
path's one exchange step).  Weak scaling: each rank verifies its own shard of
`--n` requests.

Workload (BASELINE.json configs[1]): 1M single-signature NYM requests, ~200 B
signed payload (serialize_msg_for_signing of a NYM with an alias field), 1,000
signers, all valid.  `--config c2` adds the 10% corrupted / non-canonical /
small-order mix of configs[2].  Signatures are made on the GPU by the library's
own deterministic signer (bit-exact with libsodium, tests/test_gpu_parity.py).

Usage: python bench.py [--gpus N --steps K --warmup W]
  N > 1: either under torch.distributed.run (one rank per GPU, WORLD_SIZE set), or bare --
  the process then starts the N ranks itself (launch_ranks) before anything touches the GPU.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))


def _gpus_arg(argv):
    """--gpus N from the command line without argparse's full parse (stdlib only)."""
    for i, a in enumerate(argv):
        if a == "--gpus" and i + 1 < len(argv):
            return int(argv[i + 1])
        if a.startswith("--gpus="):
            return int(a.split("=", 1)[1])
    return 1


def launch_ranks(n, argv, poll_s=0.2):
    """`python bench.py --gpus N` with no launcher around it: start N child
    ranks of this script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1
    / a free MASTER_PORT in their environment, one per GPU), relay their output
    (rank 0 prints the JSON line), and return the worst child exit code.  This
    process imports neither torch nor the engine and never touches the GPU; if
    one rank fails, the others are terminated rather than left waiting in a
    collective."""
    import signal
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL across the rank processes
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rcs = [None] * n
    first_bad = None  # the first rank that failed: its exit code is the launch's (the others were stopped)

    def forward(signum, frame):  # a launcher stopped from outside stops its ranks too
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        raise SystemExit(128 + signum)
    signal.signal(signal.SIGTERM, forward)
    try:
        while any(rc is None for rc in rcs):
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    rcs[i] = p.poll()
            if any(rc not in (None, 0) for rc in rcs):  # one rank failed: the rest would wait forever
                first_bad = next(rc for rc in rcs if rc not in (None, 0))
                for i, p in enumerate(procs):
                    if rcs[i] is None:
                        p.send_signal(signal.SIGTERM)
                for i, p in enumerate(procs):
                    if rcs[i] is None:
                        try:
                            rcs[i] = p.wait(timeout=30)
                        except subprocess.TimeoutExpired:
                            p.kill()
                            rcs[i] = p.wait()
                break
            time.sleep(poll_s)
    except KeyboardInterrupt:
        for p in procs:
            p.kill()
        raise
    if first_bad is not None:
        return first_bad if first_bad > 0 else 128 - first_bad  # a signal -k as 128 + k
    bad = [rc for rc in rcs if rc]
    return max(bad, key=abs) if bad else 0


if __name__ == "__main__" and "WORLD_SIZE" not in os.environ and _gpus_arg(sys.argv[1:]) > 1:
    sys.exit(launch_ranks(_gpus_arg(sys.argv[1:]), sys.argv[1:]))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "indy-plenum_amd"))

from plenum_amd import EdVerifyEngine, pack_messages  # noqa: E402
from plenum_amd.engine import lengths_mixed  # noqa: E402
from plenum_amd import roofline as RL  # noqa: E402
from plenum_amd import synth  # noqa: E402

METRIC = "Ed25519 request verifies/sec (whole node) at 1/2/4/8 MI355X vs host libsodium"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", "--requests", dest="n", type=int, default=1_000_000, help="requests per GPU")
    ap.add_argument("--signers", type=int, default=1000)
    ap.add_argument("--alias-len", type=int, default=43, help="pads the NYM signing payload to ~200 B")
    ap.add_argument("--config", choices=["c1", "c2", "c3", "c4"], default="c1",
                    help="c1: configs[1] all-valid NYMs; c2: configs[2] 10%% corrupted; c3: configs[3] "
                         "multi-signature requests, 64 B - 4 KiB payloads; c4: configs[4] 2M NYMs per GPU "
                         "(16M on 8) + 25-validator PREPARE/COMMIT tally in the step")
    ap.add_argument("--cpu-sample", type=int, default=400_000, help="items timed on host libsodium (rank 0, N=1)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, affinity CPUs)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--path", choices=["keyed", "general"], default="keyed",
                    help="keyed: signers' verkeys registered once (fixed-base tables in HBM, like "
                         "SimpleAuthNr.addIdr); general: every request carries its own key bytes")
    ap.add_argument("--key-window", type=int, choices=[4, 6, 8, 10, 12, 13, 14, 16], default=14,
                    help="comb window of the key tables (edv_keys_set_window)")
    ap.add_argument("--pipeline", type=int, default=1, choices=[1, 2, 3, 4],
                    help="sub-batches per chunk (edv_set_pipeline; 1 = one launch per kernel, no overlap)")
    ap.add_argument("--length-buckets", choices=["auto", "on", "off", "packed"], default="auto",
                    help="hash lanes in SHA-512 block-count order (edv_set_length_buckets); auto = the "
                         "library's rule for host offsets, applied to this batch's lengths; packed = sorted "
                         "and packed into the length-bucketed SoA unit layout (mode 3)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl = RCCL over xGMI (the product); gloo only to rehearse N > 1 on one GPU")
    ap.add_argument("--same-device", action="store_true", help="every rank on cuda:0 (with --dist-backend gloo)")
    ap.add_argument("--general-steps", type=int, default=5,
                    help="also time the general path for this many steps (0 = skip)")
    ap.add_argument("--dropin-steps", type=int, default=10,
                    help="also time the keyed path at the drop-in authenticator's key window (0 = skip)")
    ap.add_argument("--whole-node-n", type=int, default=1_000_000,
                    help="requests per batch of the headline whole-node leg (configs[1] json-decoded request dicts "
                         "through GpuAuthNr.authenticate_batches, K = --steps batches timed; 0 = skip, value = the "
                         "device-resident step)")
    ap.add_argument("--device-steps", type=int, default=20,
                    help="timed steps of the device-resident kernel leg (device_resident; its roofline)")
    ap.add_argument("--e2e-n", type=int, default=1_000_000,
                    help="requests of the end-to-end authenticate_batch leg over configs[1] (0 = skip)")
    ap.add_argument("--e2e-c0", type=int, default=10_000, help="configs[0] end-to-end requests (0 = skip)")
    ap.add_argument("--key-order", choices=["arrival", "sorted"], default="arrival",
                    help="arrival: request i signed by signer i %% signers (the keys of a wave all differ); "
                         "sorted: requests grouped by signer (A/B of the comb's gather locality)")
    ap.add_argument("--key-sort", choices=["auto", "on", "off"], default="auto",
                    help="comb lanes in key-sorted order (edv_set_key_sort; auto = sub-batches >= 4096)")
    ap.add_argument("--bls-checks", type=int, default=25,
                    help="checks of the end_to_end.bls_commit_round leg (a 3PC batch's COMMIT BLS signatures in one "
                         "call; 0 = skip)")
    ap.add_argument("--drain-n", type=int, default=40,
                    help="drains of the end_to_end.node_drain leg (100 REQUESTs + 24 BATCHes of PROPAGATEs each; "
                         "0 = skip)")
    ap.add_argument("--churn-signers", type=int, default=100_000,
                    help="signers of the end_to_end.key_churn leg (all registered with addIdr; 0 = skip)")
    ap.add_argument("--churn-requests", type=int, default=1_000_000,
                    help="requests of the key_churn leg (4 batches, Zipf-distributed signers)")
    ap.add_argument("--launch-check", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--force-dist", action="store_true",
                    help="run the N > 1 exchange path (process group, all-gather, all-reduce) even at N = 1")
    ap.add_argument("--e2e-devices", type=int, default=1,
                    help="1: also run the end-to-end leg through MultiEngine over 1/2/4/8 of the visible devices "
                         "(one node process; rank 0 at world 1)")
    return ap.parse_args()


def cpu_baseline(sig, pk, msgs, off, threads):
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libcpu_baseline.so"))
    lib.cpu_baseline_sodium_version.restype = ctypes.c_char_p
    lib.cpu_baseline_run.restype = ctypes.c_int
    n = sig.shape[0]
    ok = np.zeros(n, np.uint8)
    secs = ctypes.c_double()
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    kind = lib.cpu_baseline_run(P(sig), P(pk), P(msgs), P(off), ctypes.c_uint64(n), threads, 1, P(ok),
                                ctypes.byref(secs))
    if kind < 0:
        raise RuntimeError("cpu baseline failed")
    ver = lib.cpu_baseline_sodium_version().decode()
    return n / secs.value, ok.astype(bool), ("reference" if kind == 1 else "port"), ver


def sodium_all_items(sig, pk, msgs, starts, ends, threads):
    """libsodium 1.0.18's verdict on EVERY item of the batch (spans into msgs;
    oracle/cpu_baseline.c, untimed, all of this job's CPUs): the full-batch
    parity check beside the construction's.  None when libsodium is absent."""
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "libcpu_baseline.so"))
    n = len(starts)
    ok = np.zeros(n, np.uint8)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    sig, pk, msgs = (np.ascontiguousarray(a, np.uint8) for a in (sig, pk, msgs))
    starts, ends = (np.ascontiguousarray(a, np.uint64) for a in (starts, ends))
    t0 = time.perf_counter()
    r = lib.cpu_baseline_verdicts_spans(P(sig), P(pk), P(msgs), P(starts), P(ends), ctypes.c_uint64(n), threads, P(ok))
    return (ok.astype(bool), time.perf_counter() - t0) if r == 1 else (None, 0.0)


def build_stamp(eng):
    """Which binaries this line was measured with: the library's version string and the
    sha256 (16 hex) of the loaded libplenum_edverify.so and _hostpack extension."""
    import hashlib
    from plenum_amd import _hostpack
    out = {"edv_version": eng._lib.edv_version().decode()}
    for key, path in (("lib", getattr(eng._lib, "_name", None)), ("hostpack", getattr(_hostpack, "__file__", None))):
        if path and os.path.exists(path):
            out[key] = os.path.relpath(path, ROOT)
            out[key + "_sha16"] = hashlib.sha256(open(path, "rb").read()).hexdigest()[:16]
    # provenance: the stamp __graft_entry__.build() wrote after its make, against the binaries loaded
    # here and the sources in this tree (recomputed now)
    try:
        import __graft_entry__ as GE
        src = GE.source_sha16()
        stamp = json.load(open(GE.STAMP)) if os.path.exists(GE.STAMP) else None
        prov = {"source_sha16": src, "stamp": stamp}
        if stamp:
            bins = stamp.get("binaries", {})
            prov["lib_matches_stamp"] = bins.get(out.get("lib")) == out.get("lib_sha16")
            prov["hostpack_matches_stamp"] = bins.get(out.get("hostpack")) == out.get("hostpack_sha16")
            prov["sources_match_stamp"] = stamp.get("source_sha16") == src
        out["provenance"] = prov
    except Exception as ex:  # (reported, never fatal to the measurement)
        out["provenance"] = {"error": "%s: %s" % (type(ex).__name__, ex)}
    return out


def host_cpus():
    """nproc / affinity / cgroup CPU quota of this host (the GPU box shows the
    whole machine in nproc; the quota is this job's share)."""
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        quota = None if q == "max" else float(q) / float(period)
    except (OSError, ValueError):
        pass
    return {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "cgroup_cpu_quota": quota}


def e2e_requests(eng, n, signers, alias_len, seed=1, spec=None, sig=None, pks=None, wire=True):
    """Signed NYM request dicts (the shape Node hands authenticate(),
    plenum/common/request.py:27-39) plus the signers' (identifier, '~'verkey).
    wire: each request json-encoded and decoded on its own, as the node gets
    it off the wire (ZStack -> json.loads per message), so every request owns
    its str / int objects like in a running node."""
    from plenum_amd import _hostpack
    from plenum_amd.base58 import b58encode
    if spec is None:
        pks, sks = eng.seed_keypair_batch(synth.signer_seeds(signers))
        msgs, kidx, spec = synth.nym_messages(n, pks, alias_len=alias_len, seed=seed)
        b, o = pack_messages(msgs)
        sig = eng.sign_batch(sks, kidx, b, o)
    sig_b58 = _hostpack.b58encode_rows(np.ascontiguousarray(sig[:n]).tobytes(), 64)
    reqs = []
    dumps, loads = json.dumps, json.loads
    for i in range(n):
        r = synth.nym_request_dict(spec, i, signers)
        r["signature"] = sig_b58[i]
        reqs.append(loads(dumps(r)) if wire else r)
    vks = ["~" + b58encode(bytes(pk[16:])) for pk in pks]
    return reqs, spec["idrs"], vks


def time_e2e(eng, reqs, idrs, vks):
    """GpuAuthNr.authenticate_batch end to end (host prepare -> pack -> pinned
    H2D -> kernels -> verdicts), the drop-in's default options; the signers'
    NYMs registered with addIdr like Node.addGenesisNyms (node.py:2476-2518)."""
    from plenum_amd.client_authn import GpuAuthNr
    a = GpuAuthNr(engine=eng)
    for idr, vk in zip(idrs, vks):
        a.addIdr(idr, vk)
    # genesis NYMs' key tables built before traffic (registrations on the request path build in the
    # background, their requests on the general path until built)
    a.keys_settle()
    a.authenticate_batch(reqs[:2048])
    t0 = time.perf_counter()
    res = a.authenticate_batch(reqs)  # first full-size batch: the scan's reused buffers grow (page faults)
    first = time.perf_counter() - t0
    ok = sum(1 for r, m in zip(res, reqs) if r == m["identifier"])
    del res
    reps, parts = [], []
    for _ in range(3):  # steady state: a node authenticates batch after batch
        t0 = time.perf_counter()
        res = a.authenticate_batch(reqs)
        reps.append(time.perf_counter() - t0)
        parts.append(getattr(a._g, "last_breakdown", None))
        assert sum(1 for r, m in zip(res, reqs) if r == m["identifier"]) == ok
        del res
    total = sorted(reps)[1]
    in_batch = parts[reps.index(total)]  # the median batch's own phases (streamed path)
    # the same batch four times through authenticate_batches: two batches in flight, batch k + 1's
    # scan (and PCIe copy) under batch k's kernels (median of 3 runs)
    pipe = []
    for _ in range(3):
        t0 = time.perf_counter()
        outs = list(a.authenticate_batches([reqs] * 4))
        pipe.append(time.perf_counter() - t0)
        for res in outs:  # every batch's verdicts, checked after the clock
            assert sum(1 for r, m in zip(res, reqs) if r == m["identifier"]) == ok
        del outs
    pipe_s = sorted(pipe)[1]
    from plenum_amd import _hostpack
    from plenum_amd.client_authn import _SIG_SLOT
    g = a._g
    n = len(reqs)
    slot = _SIG_SLOT if getattr(eng, "supports_sig_slots", False) else 64
    bufs = a._scan_buffers(eng, n, slot)
    # breakdown, separate passes: the native scan (one thread, then the default threads) into the
    # authenticator's output buffers (the engine's pinned memory), then the GPU call on its output
    t1 = time.perf_counter()
    _hostpack.scan_batch_u(reqs, ["signature"], 1, bufs, slot)
    t_scan1 = time.perf_counter() - t1
    t1 = time.perf_counter()
    fast, uidx_b, uniq, sig_o, msg_o, off, short = _hostpack.scan_batch_u(reqs, ["signature"], 0, bufs, slot)
    t_scan = time.perf_counter() - t1
    off_a = np.frombuffer(off, np.uint64)
    ks = a._key_store()
    ids = ks.lookup([a._key_for(i) for i in uniq])
    kid = np.asarray(ids, np.uint32)[np.frombuffer(uidx_b, np.uint32)]
    sig_a = np.frombuffer(sig_o, np.uint8, count=slot * n).reshape(-1, slot)
    msg_a = np.frombuffer(msg_o, np.uint8, count=int(off_a[-1]))
    kw = {"sig_slot": slot} if slot != 64 else {}
    calls = []
    for _ in range(3):
        t2 = time.perf_counter()
        eng.verify_batch_keyed(sig_a, kid, msg_a, off_a, **kw)
        calls.append(time.perf_counter() - t2)
    t_ver = sorted(calls)[1]
    hs = eng.last_host_stats() if hasattr(eng, "last_host_stats") else {}
    # the copy engine's rate for those bytes, pinned host -> HBM (torch, same device)
    h2d_ms = None
    if hs.get("h2d_bytes"):
        src = torch.empty(int(hs["h2d_bytes"]), dtype=torch.uint8).pin_memory()
        dst = torch.empty_like(src, device="cuda")
        dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        h2d_ms = (time.perf_counter() - t3) * 1e3
        del src, dst
    # a message the verify-ahead did not cover: authenticate() alone, one full host -> GPU -> host
    # round trip per call (node.py:2294-2318 calls it once per message)
    a.clear_verdicts()
    lat = []
    for r in reqs[:330]:
        t4 = time.perf_counter()
        a.authenticate(r)
        lat.append((time.perf_counter() - t4) * 1e6)
    lat = np.array(lat[30:])
    del sig_a, msg_a
    return {"requests": n, "value": n / total, "seconds": total, "accepted": ok,
            "pipelined": {"value": 4 * n / pipe_s, "batches": 4, "seconds": pipe_s,
                          "note": "authenticate_batches over 4 batches of these requests: two in flight (the "
                                  "engine's two staging sets), batch k + 1's host scan and PCIe copy under batch "
                                  "k's kernels; median of 3 runs, every batch's verdicts checked after the clock"},
            "first_batch_seconds": first, "first_batch_value": n / first,
            "in_batch_ms": in_batch,
            "host_scan_ms": t_scan * 1e3, "host_scan_us_per_request": t_scan / n * 1e6,
            "host_scan_us_per_request_1_thread": t_scan1 / n * 1e6,
            "gpu_call_ms": t_ver * 1e3, "gpu_call_rate": n / t_ver,
            "stage_ms": hs.get("stage_ms"), "h2d_bytes": hs.get("h2d_bytes"), "h2d_ms_copy_engine": h2d_ms,
            "inputs_direct_from_pinned": hs.get("direct"), "sig_slot": slot,
            "single_authenticate_us": {"p50": float(np.percentile(lat, 50)), "p99": float(np.percentile(lat, 99)),
                                       "calls": int(len(lat))},
            "key_window": g.key_window, "keyed_items_share": g.stats["keyed_items"] / max(1, g.stats["batch_items"]),
            "note": "requests json-decoded one by one as the node receives them; one Python thread (a Plenum node "
                    "is single-threaded asyncio); the native scan inside it runs "
                    "its checks, base58 length check and serialization on the process's CPU budget (scan_threads=0: one "
                    "per 2k requests, at most min(affinity, cgroup quota, 48); 16 on the GPU box) while the node thread waits, writing signature slots (base58 text, "
                    "decoded on the GPU) and messages into the engine's pinned host memory. Breakdown (separate "
                    "passes): host_scan = hostpack.scan_batch_u; gpu_call = edv_verify_batch_keyed_slots on its "
                    "output (H2D straight from pinned memory, stage_ms = CPU staging copies, 0 when every input "
                    "is direct; h2d_ms_copy_engine = the same bytes as one pinned torch copy) + base58 + kernels "
                    "+ D2H; the rest of value's time is per-identifier key resolution and the result list. "
                    "in_batch_ms: the median batch's own phases on the streamed path (scan with the pack deferred; "
                    "keys_and_ids = verkeys per distinct identifier + key ids per request; pack_and_submit = per "
                    "2^17-request chunk the pack into pinned memory and the async library call; collect_wait = waiting "
                    "for the last chunks' copies and kernels; verdicts = masks + the result list). "
                    "value = the median of 3 batches after the first full-size one (steady state); first_batch_* "
                    "= that first batch (buffers allocated). single_authenticate_us: authenticate() of one "
                    "request not in the verdict cache (300 calls after 30 warm-up)"}


def whole_node_sets(eng, n, pks, sks, alias_len, rank, sets=2):
    """`sets` distinct batches of n configs[1] NYM request dicts for this rank
    (distinct reqIds per set and rank, request i signed by signer i % signers),
    each json-encoded and decoded on its own as the node gets it off the wire;
    signed on the GPU (the library's libsodium-exact signer)."""
    out = []
    for s in range(sets):
        base = synth.REQ_ID_BASE + (1 << 44) + (rank * sets + s) * n
        msgs, kidx, spec = synth.nym_messages(n, pks, alias_len=alias_len, seed=101 + 7 * rank + s, req_id_base=base)
        b, o = pack_messages(msgs)
        del msgs
        sig = eng.sign_batch(sks, kidx, b, o)
        del b, o
        reqs, idrs, vks = e2e_requests(eng, n, len(pks), alias_len, spec=spec, sig=sig, pks=pks)
        out.append(reqs)
    return out, idrs, vks


def time_whole_node(eng, args, sets, idrs, vks, dist_on, dev, scan_threads):
    """The headline: BASELINE's "verifies/sec (whole node)" -- the drop-in
    authenticator (GpuAuthNr over this rank's engine, the signers' NYMs
    registered with addIdr as Node.addGenesisNyms does) verifying batches of
    json-decoded configs[1] request dicts: the native scan (checks, base58,
    signing serialization on the host's CPUs) with its PCIe copy and kernels
    under it, getVerkey per identifier, the GPU verdicts and the result list
    -- what replaces plenum/server/client_authn.py:67-107 per request.  A step
    is one batch of n requests.  Synchronous (the headline, value): K batches
    one authenticate_batch at a time; pipelined beside it: K batches through
    authenticate_batches (two in flight -- on a host-bound path the node
    thread scans one batch while the GPU finishes the other, so it measures
    level with synchronous).  The K batches alternate between the
    distinct request sets; the batch path keeps no verdicts (every step scans,
    serializes, copies and verifies all n).  The two forms are timed in
    alternating chunks (sync, pipelined, sync, ... over K / 4 batches each),
    so drift over the run weighs on both alike.  Each timed chunk is bracketed
    by a barrier and torch.cuda.synchronize() and takes the max over ranks;
    every outcome is checked after its chunk's clock."""
    from plenum_amd.client_authn import GpuAuthNr
    K, W = args.steps, args.warmup
    n = len(sets[0])
    want = [[m["identifier"] for m in reqs] for reqs in sets]
    a = GpuAuthNr(engine=eng, scan_threads=scan_threads)
    t0 = time.perf_counter()
    for idr, vk in zip(idrs, vks):
        a.addIdr(idr, vk)
    a.keys_settle()  # genesis NYMs' key tables built before traffic
    genesis_s = time.perf_counter() - t0
    order = [sets[k % len(sets)] for k in range(K)]
    wants = [want[k % len(sets)] for k in range(K)]
    for k in range(max(1, W)):  # scan buffers grown, kid_map built, both staging sets touched
        a.authenticate_batch(sets[k % len(sets)])
    for _ in a.authenticate_batches([sets[k % len(sets)] for k in range(max(2, W))]):
        pass

    def clocked(fn):
        torch.cuda.synchronize()
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize()
        t = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t
        if dist_on:
            e = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            el = float(e.item())
        return el, out

    def check(outs, ws):
        bad = 0
        for res, w in zip(outs, ws):
            if res != w:
                bad += sum(1 for r, x in zip(res, w) if r != x)
        return bad

    # the two forms alternate in R chunks (sync, pipelined, sync, ...): a host whose speed drifts
    # over the run (profiles/r10p: ~10 % over 90 batches, whatever the form) and the harness's own
    # collections over the results it keeps weigh on both alike
    R = max(1, min(4, K // 2))
    bounds = [K * r // R for r in range(R + 1)]
    per, parts, pipe_per, pipe_parts = [], [], [], []
    spec = {"sync": 0, "pipe": 0}

    def sync_run(chunk):
        res = []
        for batch in chunk:
            tb = time.perf_counter()
            res.append(a.authenticate_batch(batch))
            per.append(time.perf_counter() - tb)
            parts.append(a._g.last_breakdown)
        return res

    def pipe_run(chunk):
        res = []
        tb = time.perf_counter()
        for r in a.authenticate_batches(chunk):
            res.append(r)
            tn = time.perf_counter()
            pipe_per.append(tn - tb)
            pipe_parts.append(a._g.last_breakdown)
            tb = tn
        return res
    el_sync = el_pipe = 0.0
    bad_sync = bad_pipe = 0
    for r in range(R):
        chunk, cw = order[bounds[r]:bounds[r + 1]], wants[bounds[r]:bounds[r + 1]]
        for form in ("sync", "pipe"):
            s0 = a.stats.get("speculated", 0)
            el, outs = clocked(lambda: (sync_run if form == "sync" else pipe_run)(chunk))
            spec[form] += a.stats.get("speculated", 0) - s0
            bad = check(outs, cw)
            del outs
            if form == "sync":
                el_sync += el
                bad_sync += bad
            else:
                el_pipe += el
                bad_pipe += bad
    med = sorted(range(K), key=lambda k: per[k])[K // 2]
    pmed = sorted(range(len(pipe_per)), key=lambda k: pipe_per[k])[len(pipe_per) // 2] if pipe_per else None
    out = {"pipelined": {"value": n * K / el_pipe, "ms_per_batch": el_pipe / K * 1e3, "seconds": el_pipe,
                         "speculated_share": spec["pipe"] / (n * K),
                         "yield_ms": {"p50": float(np.median(pipe_per)) * 1e3, "min": min(pipe_per) * 1e3,
                                      "max": max(pipe_per) * 1e3} if pipe_per else None,
                         "each_ms": [round(x * 1e3, 2) for x in pipe_per],
                         "in_batch_ms": {k: (round(v, 3) if isinstance(v, float) else v)
                                         for k, v in ((pipe_parts[pmed] if pmed is not None else None) or {}).items()},
                         "mismatches": bad_pipe},
           "synchronous": {"value": n * K / el_sync, "ms_per_batch": el_sync / K * 1e3, "seconds": el_sync,
                           "batch_ms": {"p50": float(np.median(per)) * 1e3, "min": min(per) * 1e3,
                                        "max": max(per) * 1e3},
                           "each_ms": [round(x * 1e3, 2) for x in per],
                           "speculated_share": spec["sync"] / (n * K),
                           "in_batch_ms": {k: (round(v, 3) if isinstance(v, float) else v)
                                           for k, v in (parts[med] or {}).items()},
                           "mismatches": bad_sync},
           "requests_per_batch": n, "batches": K, "distinct_request_sets": len(sets), "signers": len(idrs),
           "interleaved_chunks": R,
           "scan_threads": scan_threads or "auto", "key_window": a._g.key_window,
           "keyed_items_share": a.stats["keyed_items"] / max(1, a.stats["batch_items"]),
           "genesis_addidr_and_builds_s": genesis_s}
    return out, a


def time_bls_commit_round(eng, checks=25, reps=5):
    """bls_commit_round: a 3PC batch's COMMIT BLS signatures (one per node, distinct keys, a
    state-root-sized message each) verified in one edv_bls_verify_batch call -- the wave form
    (one wave per check) and, for comparison, the four-lane form; median wall ms per call,
    H2D of the inputs included, every verdict checked."""
    from plenum_amd import pack_messages
    from plenum_amd.base58 import b58decode
    from plenum_amd.bls import GENERATOR, ORDER
    rng = np.random.default_rng(29)
    gen = np.frombuffer(b58decode(GENERATOR), np.uint8)
    sks = np.frombuffer(b"".join((int.from_bytes(rng.bytes(32), "big") % ORDER).to_bytes(32, "big")
                                 for _ in range(checks)), np.uint8).reshape(checks, 32)
    vks = eng.bls_keygen_batch(sks, gen)
    buf, off = pack_messages([rng.bytes(96) for _ in range(checks)])
    sigs = eng.bls_sign_batch(sks, buf, off)
    res = {"checks": checks}
    for form, wave, pair in (("wave", 8192, 32768), ("four_lane", 0, 32768)):
        eng.bls_set_wave_checks(wave)
        eng.bls_set_pair_lanes(pair)
        ok = eng.bls_verify_batch(sigs, buf, off, vks, gen)
        times = []
        for _ in range(reps if form == "wave" else 2):
            t0 = time.perf_counter()
            ok = eng.bls_verify_batch(sigs, buf, off, vks, gen)
            times.append((time.perf_counter() - t0) * 1e3)
            if not ok.all():
                raise SystemExit("bls_commit_round: a valid signature rejected (%s form)" % form)
        res[form + "_ms"] = float(np.median(times))
    eng.bls_set_wave_checks(8192)
    res["note"] = ("one edv_bls_verify_batch call over %d (signature, message, verkey) checks: wave = one wave per "
                   "check running the pairing check as a straight-line program (default for <= 8192 checks), "
                   "four_lane = the earlier latency form; median wall ms, inputs' H2D included" % checks)
    return res


def time_node_drain(eng, reqs, idrs, vks, drains=40, per_drain=100, n_nodes=25, ref_drains=16):
    """end_to_end.node_drain: the path a Plenum node actually runs
    (plenum_amd/nodeloop.py restates it).  Per drain of an n = 25 pool: 100
    client REQUESTs on the client stack and, on the node stack, 24 BATCH
    messages (one per other node) each wrapping that node's PROPAGATEs of the
    100 requests.  The stacks are the verify-ahead ones (batching.py
    verify_ahead_stack): processReceived prefetches the drain's requests in one
    GPU batch (native scan, one copy per distinct text) and hands the decoded
    objects to the reference loop, which calls authenticate() once per REQUEST
    and once per PROPAGATE (node.py:2294-2314, BATCH entries via
    unpackNodeMsg, node.py:1333-1337): 2,500 calls per drain, each a
    verdict-cache hit.  Beside it, the reference loop over the same drains on
    one core (oracle/ref_authn_port.py --drain: json per message, the
    reference authenticate() over libsodium), as a child process."""
    import subprocess
    import tempfile
    from plenum_amd.batching import verify_ahead_stack
    from plenum_amd.client_authn import GpuAuthNr
    from plenum_amd.nodeloop import NodeCounters, Stack, drain_texts
    a = GpuAuthNr(engine=eng)
    for idr, vk in zip(idrs, vks):
        a.addIdr(idr, vk)
    a.keys_settle()
    warm = 3
    need = (drains + warm) * per_drain
    assert len(reqs) >= need, (len(reqs), need)
    texts = [drain_texts(reqs[d * per_drain:(d + 1) * per_drain], n_nodes) for d in range(drains + warm)]
    nc = NodeCounters()
    ns = verify_ahead_stack(Stack, a)(a, "node", nc)
    cs = verify_ahead_stack(Stack, a)(a, "client", nc)
    per = []
    for d, (client, node) in enumerate(texts):
        if d == warm:
            nc.authenticated = nc.rejected = nc.messages = 0
            st0 = dict(a.stats)
            t0 = time.perf_counter()
        td = time.perf_counter()
        ns.rxMsgs.extend(node)
        cs.rxMsgs.extend(client)
        ns.processReceived(100)  # node stack first: its drain is the one that sees each request first
        cs.processReceived(100)
        if d >= warm:
            per.append(time.perf_counter() - td)
    el = time.perf_counter() - t0
    st1 = dict(a.stats)
    calls = nc.authenticated + nc.rejected
    rx = drains * (n_nodes - 1 + per_drain)
    # authenticate() alone on the node thread: a drain's PROPAGATE-shaped request dicts, prefetched
    last = [json.loads(json.dumps(r)) for r in reqs[:per_drain]]
    a.prefetch(last)
    msgs = [json.loads(json.dumps(r)) for r in last] * (n_nodes - 1)
    lat = []
    for k in range(0, len(msgs), 100):
        tk = time.perf_counter()
        for m in msgs[k:k + 100]:
            a.authenticate(m)
        lat.append((time.perf_counter() - tk) / 100 * 1e6)
    out = {"value": calls / el, "unit": "authenticate() calls/s (node thread, one process)",
           "requests_per_s": drains * per_drain / el, "rx_entries_per_s": rx / el,
           "drains": drains, "per_drain": {"requests": per_drain, "nodes": n_nodes, "rx_entries": n_nodes - 1 + per_drain,
                                           "authenticate_calls": calls // drains},
           "accepted": nc.authenticated, "rejected": nc.rejected,
           "us_per_authenticate_in_loop": el / calls * 1e6,
           "ms_per_drain": {"p50": float(np.percentile(per, 50)) * 1e3, "max": float(max(per)) * 1e3},
           "node_thread_us_per_authenticate": {"p50": float(np.percentile(lat, 50)), "mean": float(np.mean(lat))},
           "gpu_batches_per_drain": (st1["batches"] - st0["batches"]) / drains,
           "single_verifies": st1["single_verifies"] - st0["single_verifies"],
           "cache_hits": st1["cache_hits"] - st0["cache_hits"],
           "prefetched": st1["prefetched"] - st0["prefetched"]}
    # the reference loop over the same drains, one core
    if ref_drains:
        with tempfile.NamedTemporaryFile("w", suffix=".json", delete=False) as f:
            json.dump({"drains": [{"client": [t for t, _ in c], "node": [t for t, _ in nd]}
                                  for c, nd in texts[warm:warm + ref_drains]],
                       "verkeys": dict(zip(idrs, vks))}, f)
            path = f.name
        try:
            r = subprocess.run([sys.executable, os.path.join(ROOT, "oracle", "ref_authn_port.py"), path, "--drain"],
                               capture_output=True, text=True, timeout=900)
            if r.returncode == 0:
                ref = json.loads(r.stdout.strip().splitlines()[-1])
                out["reference_loop_1_core"] = ref
                out["vs_reference_per_core"] = out["value"] / ref["authenticate_per_s"]
            else:
                out["reference_loop_1_core"] = {"error": r.stderr[-500:]}
        finally:
            os.unlink(path)
    out["note"] = ("configs[1] requests (1,000 signers' NYMs, ~200 B signed payload) in drains of %d REQUESTs + %d "
                   "BATCHes of PROPAGATEs (n = %d); value = authenticate() calls per second of the whole loop (decode, "
                   "prefetch incl. the GPU batch, the node's handlers, authenticate); the scan's helper threads "
                   "join only for batches of 2k+ items (a drain's prefetch scans its ~100 distinct texts on the "
                   "node thread). reference_loop_1_core = the same drains through the reference's loop and "
                   "authenticate() chain over libsodium (oracle/ref_authn_port.py --drain)" % (per_drain, n_nodes - 1,
                                                                                            n_nodes))
    return out


def time_key_churn(eng, signers=100_000, n=1_000_000, batches=4, zipf=1.1, seed_offset=1 << 20, warm=3):
    """end_to_end.key_churn: a domain ledger's signer population through
    GpuAuthNr -- `signers` NYM owners all registered with addIdr
    (node.py:2476-2494), far more than the key store's max_keys slots, and
    requests whose signers follow a Zipf(zipf) law (synth.zipf_signers), in
    `batches` batches of n / batches json-decoded requests (0.5 % forged).
    Keys that verified hot_key_uses requests on the general path earn a slot
    and evict the least-recently-used (asynchronous table builds), so each
    batch reports its rate, its keyed / general shares and the registrations
    it triggered.  `warm` batches of the same stream run first, untimed (the
    node's steady state: its buffers sized and its hot signers' keys earned;
    reported as cold_start), then the `batches` timed ones.  Every outcome is
    checked after the clock."""
    from plenum_amd import _hostpack
    from plenum_amd.base58 import b58encode
    from plenum_amd.client_authn import GpuAuthNr
    pks, sks = eng.seed_keypair_batch(synth.signer_seeds(seed_offset + signers)[seed_offset:])
    idrs = [b58encode(bytes(pk[:16])) for pk in pks]
    vks = ["~" + b58encode(bytes(pk[16:])) for pk in pks]
    per = n // batches
    n = per * (batches + warm)  # (the warm-up batches first, then the timed ones: one request stream)
    kidx = synth.zipf_signers(n, signers, zipf)
    msgs, spec = synth.churn_messages(kidx, idrs, alias_len=43, req_id_base=synth.REQ_ID_BASE + (1 << 40))
    buf, off = pack_messages(msgs)
    del msgs
    sig = eng.sign_batch(sks, kidx, buf, off)
    sig_b58 = _hostpack.b58encode_rows(np.ascontiguousarray(sig).tobytes(), 64)
    del sig, buf, off
    dumps, loads = json.dumps, json.loads
    reqs = []
    for i in range(n):
        r = synth.churn_request_dict(spec, i)
        if i % 200 == 7:
            r["reqId"] += 1  # forged after signing
        r["signature"] = sig_b58[i]
        reqs.append(loads(dumps(r)))
    del sig_b58
    a = GpuAuthNr(engine=eng)
    t0 = time.perf_counter()
    for idr, vk in zip(idrs, vks):
        a.addIdr(idr, vk)
    a.keys_settle()  # genesis: the free slots take addIdr keys
    genesis_s = time.perf_counter() - t0
    out_b = []
    total = cold = 0.0
    bad = 0
    chunks = [reqs[b * per:(b + 1) * per] for b in range(batches + warm)]  # (the batch lists, made before the clock)
    for b in range(batches + warm):
        chunk = chunks[b]
        st0 = dict(a.stats)
        t0 = time.perf_counter()
        res = a.authenticate_batch(chunk)
        el = time.perf_counter() - t0
        if b >= warm:
            total += el
        else:
            cold += el
        st1 = dict(a.stats)
        for j, (r, m) in enumerate(zip(res, chunk)):
            forged = (b * per + j) % 200 == 7
            bad += (type(r).__name__ != "InvalidSignature") if forged else (r != m["identifier"])
        del res
        items = st1["batch_items"] - st0["batch_items"]
        keyed = st1["keyed_items"] - st0["keyed_items"]
        out_b.append({"requests": per, "value": per / el, "ms": el * 1e3, "timed": b >= warm,
                      "distinct_signers": int(len(np.unique(kidx[b * per:(b + 1) * per]))),
                      "keyed_share": keyed / max(1, items), "general_share": 1 - keyed / max(1, items),
                      "registrations": st1["keys_registered"] - st0["keys_registered"],
                      "in_batch_ms": {k: (round(v, 3) if isinstance(v, float) else v)
                                      for k, v in (a._g.last_breakdown or {}).items()}})
        a._g.last_breakdown = None
    ks = a._key_store()
    return {"signers": signers, "zipf_s": zipf, "requests": per * batches, "batches": out_b[warm:],
            "value": per * batches / total, "mismatches": int(bad), "key_slots": ks.capacity if ks else 0,
            "cold_start": {"batches": out_b[:warm], "value": per * warm / cold if warm else None},
            "key_window": a._g.key_window, "genesis_addidr_and_builds_s": genesis_s,
            "note": "%d signers registered with addIdr (more than the %d key slots), requests' signers Zipf(%.1f), "
                    "%d timed batches of %d json-decoded requests after %d untimed ones of the same stream "
                    "(cold_start: the authenticator's first batches -- buffers sized, hot keys not yet earned), "
                    "0.5%% forged; keys earn slots by verified use (hot_key_uses) and evict the "
                    "least-recently-used, tables built asynchronously; value = timed requests / summed batch "
                    "seconds; mismatches = outcomes != the construction's, every batch (checked after the clock)"
                    % (signers, ks.capacity if ks else 0, zipf, batches, per, warm)}


def time_e2e_devices(eng, reqs, idrs, vks, counts):
    """The node-shaped multi-GPU leg: one node process (looper.py:141-151),
    GpuAuthNr over MultiEngine with k engines (multi.py: every batch split by
    64-aligned request index, one host thread per device, key store
    replicated on every device), k in `counts`.  Per k: the steady-state
    authenticate_batch rate (median of 3 after two warm batches), the scan
    and the GPU call in the same process as configs1.  Engine 0 is this
    process's engine; the others are created here and closed after."""
    from plenum_amd.client_authn import GpuAuthNr
    from plenum_amd.multi import MultiEngine
    out = {}
    n = len(reqs)
    for k in counts:
        extra, me = [], None
        try:
            extra = [EdVerifyEngine(d) for d in range(1, k)]
            me = MultiEngine(engines=[eng] + extra)
            a = GpuAuthNr(engine=me)
            for idr, vk in zip(idrs, vks):
                a.addIdr(idr, vk)
            t0 = time.perf_counter()
            a.keys_settle()  # the signers' tables on every device (built concurrently, one thread each)
            keys_s = time.perf_counter() - t0
            a.authenticate_batch(reqs)
            a.authenticate_batch(reqs)
            reps = []
            for _ in range(3):
                t0 = time.perf_counter()
                res = a.authenticate_batch(reqs)
                reps.append(time.perf_counter() - t0)
            ok = sum(1 for r, m in zip(res, reqs) if r == m["identifier"])
            del res
            t = sorted(reps)[1]
            out[str(k)] = {"engines": k, "value": n / t, "seconds": t, "accepted": ok,
                           "keyed_items_share": a.stats["keyed_items"] / max(1, a.stats["batch_items"]),
                           "keys_build_s_all_devices": keys_s}
        except Exception as ex:  # (reported in the line; the headline and the other legs stand)
            out[str(k)] = {"engines": k, "error": "%s: %s" % (type(ex).__name__, ex)}
        finally:
            for e in extra:
                e.close()
            if me is not None and me._pool:
                me._pool.shutdown()
        if eng.keys_count():
            eng.keys_reset()
    return out


def reference_path_baseline(eng, n, host):
    """configs[0] on the CPU: the reference's authenticate() chain in plain
    Python over libsodium (oracle/ref_authn_port.py), 10k NYM requests from 100
    signers; one process, then one per core of this job's share.  Run as child
    processes (this process holds the GPU; it never forks)."""
    import subprocess
    import tempfile
    reqs, idrs, vks = e2e_requests(eng, n, 100, 0, seed=11)
    with tempfile.NamedTemporaryFile("w", suffix=".json", delete=False) as f:
        json.dump({"requests": reqs, "verkeys": dict(zip(idrs, vks))}, f)
        path = f.name
    out = {}
    try:
        procs = min(16, host["affinity"])
        for k in (1, procs):
            r = subprocess.run([sys.executable, os.path.join(ROOT, "oracle", "ref_authn_port.py"), path,
                                "--procs", str(k)], capture_output=True, text=True, timeout=600)
            if r.returncode != 0:
                out["error"] = r.stderr[-500:]
                break
            out["procs_%d" % k] = json.loads(r.stdout.strip().splitlines()[-1])
    finally:
        os.unlink(path)
    out["kind"] = "port"
    out["note"] = ("BASELINE configs[0]: %d NYM requests, 100 signers, the reference's authenticate() path "
                   "(client_authn.py:67-107 -> verifier.py -> nacl_wrappers.py -> libsodium crypto_sign_open) "
                   "restated in Python; value = requests/s" % n)
    return out


def general_dsm_roofline(eng, d_pk, n, o_ms):
    """The general path's ladder kernel against the MAD peak, priced at the
    implementation's own count for the split it ran (roofline.mad_dsm_kernel:
    K tables per distinct key, decided per sub-batch from its distinct-key
    count, reproduced here from the same keys)."""
    pk = d_pk.cpu().numpy()
    launches = eng.last_launch_count()
    per = -(-min(n, 1 << 20) // launches)
    splits = []
    for s0 in range(0, min(n, 1 << 20), per):
        sub = pk[s0:s0 + per]
        splits.append(RL.split_of(len(np.unique(sub.view(np.dtype((np.void, 32))))), len(sub)))
    k = splits[0]
    dsm_ms = float(np.mean(np.array(o_ms), axis=0)[2]) / launches
    mad = RL.mad_dsm_kernel(k)
    achieved = per * mad / (dsm_ms * 1e-3) / 1e12
    return {"split_tables": k, "dsm_kernel_mad_per_request": mad,
            "dsm_roofline": {"bound": "valu-mad", "achieved": achieved, "peak": RL.PEAK_MAD_PER_S / 1e12,
                             "unit": "T MAD/s", "frac": achieved / (RL.PEAK_MAD_PER_S / 1e12),
                             "work": "fe_dsm_split(%d) = %d field ops x 100 MAD" % (k, RL.fe_dsm_split(k))}}


def time_general_distinct(eng, args, n, d_msgs, d_ms, d_me, stream, steps=3):
    """General path with every request signed by a key of its own (n keys;
    the dedupe finds no sharing, K = 1): the worst case of the general path,
    on the same messages."""
    dev = d_msgs.device
    pks, sks = eng.seed_keypair_batch(synth.signer_seeds(n))
    d_k = torch.arange(n, dtype=torch.int32, device=dev)
    d_sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    eng.sign_spans_device(torch.from_numpy(sks).to(dev), d_k, d_msgs, d_ms, d_me, n, d_sig)
    d_pk = torch.from_numpy(pks).to(dev)
    words = torch.zeros((n + 63) // 64, dtype=torch.int64, device=dev)
    eng.verify_spans_device(d_sig, d_pk, False, d_msgs, d_ms, d_me, n, words, stream=stream)
    torch.cuda.synchronize()
    ms = []
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.verify_spans_device(d_sig, d_pk, False, d_msgs, d_ms, d_me, n, words, stream=stream)
        ms.append(eng.last_phases_ms())
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    bits = np.unpackbits(words.cpu().numpy().view(np.uint8), bitorder="little")[:n]
    out = {"value": n * steps / el, "keys": n, "all_accepted": bool(bits.all()),
           "phase_ms": dict(zip(("hash", "table", "dsm", "encode"),
                                (float(v) for v in np.mean(np.array(ms), axis=0))))}
    out.update(general_dsm_roofline(eng, d_pk, n, ms))
    return out


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.launch_check:  # the launcher's CPU test: what this rank was given, before any GPU call
        print(json.dumps({"rank": rank, "local_rank": local, "world": world, "gpus": args.gpus,
                          "master": "%s:%s" % (os.environ.get("MASTER_ADDR"), os.environ.get("MASTER_PORT")),
                          "torch_cuda_initialized": bool(torch.cuda.is_initialized())}), flush=True)
        return
    assert world == args.gpus, "WORLD_SIZE=%d ranks but --gpus %d" % (world, args.gpus)
    if args.same_device:  # rehearsal of the N > 1 logic on a one-GPU box (gloo)
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # the exchange path (process group, bitmask all-gather, ballot all-reduce): with N > 1 ranks, or
    # at N = 1 with --force-dist (exercises the RCCL calls on a one-GPU box)
    dist_on = world > 1 or args.force_dist
    if dist_on and "WORLD_SIZE" not in os.environ:  # --force-dist at N = 1: a one-rank group
        import socket
        so = socket.socket()
        so.bind(("127.0.0.1", 0))
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(so.getsockname()[1]), RANK="0", WORLD_SIZE="1")
        so.close()
    if dist_on:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)
    t_create = time.perf_counter()
    eng = EdVerifyEngine(local)
    create_s = time.perf_counter() - t_create  # includes the base comb's build (kBaseW)
    if hasattr(eng._lib, "edv_base_window"):
        RL.set_base_window(eng._lib.edv_base_window())
    eng.set_pipeline(args.pipeline)
    eng.set_key_sort(args.key_sort)
    n = args.n if not (args.config == "c4" and args.n == 1_000_000) else 2_000_000

    # ---- synthetic signed batch (not timed)
    seeds = synth.signer_seeds(args.signers)
    pks, sks = eng.seed_keypair_batch(seeds)
    d_sk = torch.from_numpy(sks).to(dev)
    expect = np.ones(n, dtype=bool)
    if args.config in ("c1", "c2", "c4"):
        msgs_l, key_idx, nym_spec = synth.nym_messages(n, pks, alias_len=args.alias_len, seed=1 + rank,
                                                req_id_base=synth.REQ_ID_BASE + rank * n)
        buf, off = pack_messages(msgs_l)
        del msgs_l
        item_start, item_end = off[:-1].copy(), off[1:].copy()
        req_desc = ""
    else:
        # configs[3]: multi-signature requests, 1-5 signatures each (distinct
        # signers), payloads log-uniform 64 B - 4 KiB; the k signatures of a
        # request share its one message copy (message spans)
        rng = np.random.default_rng(3 + rank)
        ks = rng.integers(1, 6, size=n)
        nreq = int(np.searchsorted(np.cumsum(ks), n)) + 1
        ks = ks[:nreq]
        ks[-1] -= int(ks.sum()) - n
        lens = np.exp(rng.uniform(np.log(64), np.log(4096), nreq)).astype(np.int64)
        roff = np.zeros(nreq + 1, np.uint64)
        roff[1:] = np.cumsum(lens)
        buf = rng.integers(33, 127, size=int(roff[-1]), dtype=np.uint8)  # printable serialized bytes
        item_req = np.repeat(np.arange(nreq), ks)
        slot = np.arange(n) - np.repeat(np.cumsum(ks) - ks, ks)
        key_idx = ((item_req * 7 + slot * 131) % args.signers).astype(np.uint32)  # distinct within a request
        item_start, item_end = roff[:-1][item_req], roff[1:][item_req]
        req_desc = ", %d requests x 1-5 signatures (mean %.2f), payload %d-%d B log-uniform" % (
            nreq, n / nreq, int(lens.min()), int(lens.max()))
    if args.key_order == "sorted":
        # requests grouped by signer (a batch sorted by key id; the messages stay, spans reordered)
        order = np.argsort(key_idx, kind="stable")
        key_idx, item_start, item_end = key_idx[order], item_start[order], item_end[order]
    mlen_mean = float(np.mean(item_end - item_start))
    buckets = args.length_buckets in ("on", "packed") or (args.length_buckets == "auto" and
                                                           lengths_mixed(item_start, item_end))
    eng.set_length_buckets(3 if args.length_buckets == "packed" else 1 if buckets else 0)
    d_kidx = torch.from_numpy(key_idx.astype(np.int32)).to(dev)
    d_msgs = torch.from_numpy(np.concatenate([buf, np.zeros(16, np.uint8)])).to(dev)
    d_ms = torch.from_numpy(item_start.astype(np.int64)).to(dev)
    d_me = torch.from_numpy(item_end.astype(np.int64)).to(dev)
    d_sig = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    eng.sign_spans_device(d_sk, d_kidx, d_msgs, d_ms, d_me, n, d_sig)
    d_pk = torch.from_numpy(pks).to(dev)[d_kidx.long()].contiguous()
    torch.cuda.synchronize()
    if args.config == "c2":
        off = np.concatenate([item_start, item_end[-1:]])
        sig_h, pk_h, buf_h = d_sig.cpu().numpy().copy(), d_pk.cpu().numpy().copy(), buf.copy()
        expect = synth.corrupt_configs2(sig_h, pk_h, buf_h, off, np.random.default_rng(2))
        d_sig = torch.from_numpy(sig_h).to(dev)
        d_pk = torch.from_numpy(pk_h).to(dev)
        buf = buf_h
        d_msgs = torch.from_numpy(np.concatenate([buf_h, np.zeros(16, np.uint8)])).to(dev)
    nwords = (n + 63) // 64
    d_words = torch.zeros(nwords, dtype=torch.int64, device=dev)
    gathered = [torch.zeros_like(d_words) for _ in range(world)] if dist_on else None
    stream = torch.cuda.current_stream(dev)

    # keyed path: register the signers' verkeys once (not per request)
    key_build_ms = None
    if args.config == "c2":
        # corrupted pks (small-order / non-canonical) become keys of their own
        pk_h = d_pk.cpu().numpy()
        uniq, inv = np.unique(pk_h, axis=0, return_inverse=True)
        reg_pks, d_kreq = uniq, torch.from_numpy(inv.reshape(-1).astype(np.int32)).to(dev)
    else:
        reg_pks, d_kreq = pks, d_kidx
    torch.cuda.synchronize()
    tk = time.perf_counter()
    eng.keys_reset()
    eng.keys_set_window(args.key_window)
    first = eng.keys_add(reg_pks)
    key_build_ms = (time.perf_counter() - tk) * 1e3
    assert first == 0

    def step_general():
        eng.verify_spans_device(d_sig, d_pk, False, d_msgs, d_ms, d_me, n, d_words, stream=stream)
        if dist_on:
            dist.all_gather(gathered, d_words)

    def step_keyed():
        eng.verify_spans_device(d_sig, d_kreq, True, d_msgs, d_ms, d_me, n, d_words, stream=stream)
        if dist_on:
            dist.all_gather(gathered, d_words)

    step = step_keyed if args.path == "keyed" else step_general

    tally_check = None
    if args.config == "c4":
        # configs[4]: votes of 3PC batches (Max3PCBatchSize = 100 requests,
        # plenum/config.py:185): K = all ranks' requests / 100 keys x 25
        # validators x {PREPARE, COMMIT}.  Vote j of this rank is backed by
        # request j's signature (its accept bit) and ~5% are missing/invalid.
        # Step += unpack bits -> ballot scatter -> RCCL all-reduce(MAX) of the
        # ballots (set union) -> counts + Quorums(25) flags (quorums.py:15-32).
        V = 25
        n_keys = -(-(n // 2) * world // (2 * V))  # every vote g // (2V) has its key (ceil)
        nv = n // 2
        g = np.arange(nv, dtype=np.int64) + rank * nv
        # which votes are present: per-key classes (synth.c4_votes) -- half the keys ~5% random drops,
        # the rest exactly at / one below the prepare (16) or commit (17) quorum of n = 25, the
        # prepare ones with the primary's PREPARE present (it must not count, replica.py:1289-1291)
        v_key, v_phase, v_voter, keep, _ = synth.c4_votes(g, V)
        d_vkey, d_vphase, d_vvoter = (torch.from_numpy(a).to(dev) for a in
                                      (v_key.astype(np.int32), v_phase.astype(np.uint8), v_voter.astype(np.uint8)))
        d_keep = torch.from_numpy(keep.astype(np.uint8)).to(dev)
        primary = synth.c4_primary(n_keys, V)
        d_primary = torch.from_numpy(primary).to(dev)
        d_ballot = torch.zeros(n_keys * 2 * V, dtype=torch.uint8, device=dev)
        d_counts = torch.zeros(n_keys * 2, dtype=torch.int32, device=dev)
        d_quorum = torch.zeros(n_keys, dtype=torch.uint8, device=dev)
        shifts = torch.arange(8, dtype=torch.uint8, device=dev)
        verify_step = step

        def step_c4():
            verify_step()
            bits = ((d_words.view(torch.uint8)[: (nv + 7) // 8].unsqueeze(1) >> shifts) & 1).reshape(-1)[:nv]
            d_valid = bits * d_keep
            eng.tally_device(d_vkey, d_vvoter, d_vphase, d_valid, nv, n_keys, V, d_ballot, d_counts, d_quorum,
                             stream=stream, d_primary=d_primary)
            if dist_on:
                dist.all_reduce(d_ballot, op=dist.ReduceOp.MAX)
            eng.tally_finish_device(d_ballot, n_keys, V, d_counts, d_quorum, stream=stream)

        step = step_c4

        def tally_check():
            # expected: every rank's present votes (all signatures valid here), the primary's PREPARE dropped
            cnt = np.zeros(n_keys * 2, np.int64)
            cnt_naive = np.zeros(n_keys, np.int64)
            cls_of = np.zeros(n_keys, np.int64)
            for r in range(world):
                kk, ph, vv, kr, cl = synth.c4_votes(np.arange(nv, dtype=np.int64) + r * nv, V)
                np.add.at(cnt_naive, kk[ph == 0], kr[ph == 0].astype(np.int64))
                cls_of[kk] = cl
                kr &= ~((ph == 0) & (vv == primary[kk]))
                np.add.at(cnt, kk * 2 + ph, kr.astype(np.int64))
            f = (V - 1) // 3
            q = ((cnt[0::2] >= V - f - 1).astype(np.uint8) | ((cnt[1::2] >= V - f).astype(np.uint8) << 1))
            got_c = d_counts.cpu().numpy().astype(np.int64)
            got_q = d_quorum.cpu().numpy()
            by_class = {}
            for c, name in enumerate(synth.C4_CLASSES):
                sel = cls_of == c
                d = by_class.setdefault(name, {"keys": 0, "prepare_quorums": 0, "commit_quorums": 0})
                d["keys"] += int(sel.sum())
                d["prepare_quorums"] += int((got_q[sel] & 1).sum())
                d["commit_quorums"] += int((got_q[sel] >> 1 & 1).sum())
            return {"keys": n_keys, "votes_per_gpu": nv, "validators": V,
                    "counts_match": bool((got_c == cnt).all()), "quorum_match": bool((got_q == q).all()),
                    "prepare_quorums": int((got_q & 1).sum()), "commit_quorums": int((got_q >> 1 & 1).sum()),
                    "keys_below_prepare_quorum": int((q & 1 == 0).sum()),
                    "keys_below_commit_quorum": int((q >> 1 & 1 == 0).sum()),
                    "keys_decided_by_primary_rule": int(((cnt_naive >= V - f - 1) != (cnt[0::2] >= V - f - 1)).sum()),
                    "by_class": by_class}

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.device_steps):
        step()  # (queued back to back: nothing in the loop waits on the device)
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # kernel phases (HIP events on the launch streams; every step is the same work): the last timed
    # step's and three more, each read after its step (untimed, so the timed loop never waits)
    phases = [eng.last_phases_ms()]
    for _ in range(3):
        step()
        phases.append(eng.last_phases_ms())
    torch.cuda.synchronize()
    if dist_on:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())

    tally_result = tally_check() if tally_check else None

    # the exchange step alone (RCCL cost reported apart from the
    # verify): the bitmask all-gather (+ the ballot all-reduce MAX on configs[4])
    # on the same buffers, timed with events on the compute stream, max over ranks
    collective = None
    if dist_on:
        reps = 20
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        dist.barrier()
        ev0.record(stream)
        for _ in range(reps):
            dist.all_gather(gathered, d_words)
        ev1.record(stream)
        torch.cuda.synchronize()
        ag = torch.tensor([ev0.elapsed_time(ev1) / reps], dtype=torch.float64, device=dev)
        dist.all_reduce(ag, op=dist.ReduceOp.MAX)
        collective = {"all_gather_bitmask_ms": float(ag.item()), "bitmask_bytes_per_rank": int(d_words.numel() * 8)}
        if args.config == "c4":
            dist.barrier()
            ev0.record(stream)
            for _ in range(reps):
                dist.all_reduce(d_ballot, op=dist.ReduceOp.MAX)
            ev1.record(stream)
            torch.cuda.synchronize()
            ar = torch.tensor([ev0.elapsed_time(ev1) / reps], dtype=torch.float64, device=dev)
            dist.all_reduce(ar, op=dist.ReduceOp.MAX)
            collective.update({"all_reduce_max_ballots_ms": float(ar.item()), "ballot_bytes": int(d_ballot.numel())})

    # ---- parity of the timed output against the construction
    words = d_words.cpu().numpy().view(np.uint64)
    got = np.unpackbits(words.view(np.uint8), bitorder="little")[:n].astype(bool)
    mismatches = int((got != expect).sum())
    accepted, expected = int(got.sum()), int(expect.sum())
    gathered_accepted = None
    if dist_on:  # every rank's parity, and the bitmask as the all-gather delivers it
        red = torch.tensor([mismatches, accepted, expected], dtype=torch.int64, device=dev)
        dist.all_reduce(red)
        mismatches, accepted, expected = (int(x) for x in red.tolist())
        parts = [torch.empty_like(d_words) for _ in range(world)]
        dist.all_gather(parts, d_words)
        gathered_accepted = sum(int(np.unpackbits(t.cpu().numpy().view(np.uint8), bitorder="little")[:n].sum())
                                for t in parts)

    # secondary: the other path on the same resident batch (same verdicts required)
    other = None
    if args.general_steps > 0:
        ostep = step_general if args.path == "keyed" else step_keyed
        ostep()
        torch.cuda.synchronize()
        if dist_on:
            dist.barrier()
        o_ms = []
        t1 = time.perf_counter()
        for _ in range(args.general_steps):
            ostep()
            o_ms.append(eng.last_phases_ms())
        torch.cuda.synchronize()
        if dist_on:
            dist.barrier()
        o_el = time.perf_counter() - t1
        if dist_on:
            e = torch.tensor([o_el], dtype=torch.float64, device=dev)
            dist.all_reduce(e, op=dist.ReduceOp.MAX)
            o_el = float(e.item())
        ow = d_words.cpu().numpy().view(np.uint64)
        og = np.unpackbits(ow.view(np.uint8), bitorder="little")[:n].astype(bool)
        other = {"path": "general" if args.path == "keyed" else "keyed",
                 "value": n * world * args.general_steps / o_el,
                 "phase_ms": dict(zip(("hash", "table", "dsm_or_comb", "encode"),
                                      (float(v) for v in np.mean(np.array(o_ms), axis=0)))),
                 "same_verdicts": bool((og == got).all())}
        if args.path == "keyed":
            other.update(general_dsm_roofline(eng, d_pk, n, o_ms))
            if args.config == "c1" and rank == 0:
                other["distinct_keys"] = time_general_distinct(eng, args, n, d_msgs, d_ms, d_me, stream)

    total = n * world * args.device_steps
    value = total / elapsed
    ms_per_step = elapsed / args.device_steps * 1e3
    ph = np.mean(np.array(phases), axis=0)  # per step: per-phase sums over the sub-batch launches
    launches = eng.last_launch_count()
    n_chunk = eng.last_chunk_items()  # the phase times cover the last 2^20-request chunk
    dsm_sum = float(ph[2])
    dsm_avg = dsm_sum / launches
    if args.path == "keyed":
        kernel_mad = RL.mad_comb_kernel(args.key_window)
    else:
        kernel_mad = general_dsm_roofline(eng, d_pk, n, phases)["dsm_kernel_mad_per_request"]
    kernel_name = "edv_comb_kernel" if args.path == "keyed" else "edv_dsm_kernel"
    achieved = (n_chunk / launches) * kernel_mad / (dsm_avg * 1e-3) / 1e12
    peak = RL.PEAK_MAD_PER_S / 1e12
    # HBM bytes per launch from the committed PMC pass (tools/pmc_passes.sh ->
    # tools/pmc_summary.py): 2 x FETCH_SIZE + WRITE_SIZE per request (gfx950
    # FETCH_SIZE correction), times the requests of one launch
    traffic = None
    utilisation = None
    key = "%s<%d>" % (kernel_name, args.key_window) if args.path == "keyed" else kernel_name
    tpath = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tpath):
        with open(tpath) as f:
            tj = json.load(f)
        kern = tj.get("kernels", {})
        row = kern.get(key)
        if row and "traffic_bytes_per_request" in row:
            traffic = row["traffic_bytes_per_request"] * (n_chunk / launches)
        # VALU busy / clock / HBM GB/s of the step's kernels: counters of the committed PMC pass
        # (same binary, same workload), durations from this run's HIP events
        per = n_chunk / launches
        hash_key = "edv_hash_keyed_kernel<false>" if args.path == "keyed" else "edv_hash_kernel<false>"
        legs = ((key, float(ph[2]) / launches, kernel_mad), (hash_key, float(ph[0]) / launches, None),
                ("edv_encode_kernel<16>", float(ph[3]) / launches, RL.mad_encode_kernel(16)))
        utilisation = {k: RL.pmc_utilisation(kern[k], ms, per, mad) for k, ms, mad in legs
                       if k in kern and ms > 0}
        utilisation["source"] = ("%s (run %s): counters per launch from the PMC passes, durations from this run's "
                                 "HIP events. clock = GRBM_GUI_ACTIVE/8/duration; valu_busy = SQ_ACTIVE_INST_VALU*4/"
                                 "(1024 SIMDs * GRBM_GUI_ACTIVE/8) (rocprof gfx94x VALUBusy); hbm_GBps = (2*FETCH_SIZE"
                                 " + WRITE_SIZE) bytes per request * requests / duration; mad_share_of_valu = MAD per "
                                 "request / VALU lane-instructions per request (roofline.pmc_utilisation)"
                                 % (os.path.relpath(tpath, ROOT), tj.get("run", "?")))

    # the dominant kernel alone on the GPU (one sub-batch, no overlap), one
    # untimed step: its own roofline fraction beside the overlapped one above
    eng.set_pipeline(1)
    step()
    solo = eng.last_phases_ms()
    eng.set_pipeline(args.pipeline)
    solo_ms = float(solo[2])
    solo_n = eng.last_chunk_items()
    standalone = {"avg_launch_ms": solo_ms, "n_per_launch": solo_n,
                  "achieved": solo_n * kernel_mad / (solo_ms * 1e-3) / 1e12,
                  "frac": solo_n * kernel_mad / (solo_ms * 1e-3) / RL.PEAK_MAD_PER_S,
                  "note": "same kernel, one launch over the whole batch with nothing else running (untimed step)"}

    # the keyed path at the key window the drop-in authenticator picks by
    # default (client_authn KEY_STORE_BYTES / max_keys): same resident batch
    dropin = None
    if args.dropin_steps > 0 and args.path == "keyed" and world == 1:
        from plenum_amd.client_authn import KEY_STORE_BYTES
        from plenum_amd.keystore import auto_window
        w_drop = auto_window(16384, KEY_STORE_BYTES)
        eng.keys_reset()
        eng.keys_set_window(w_drop)
        eng.keys_add(reg_pks)
        step_keyed()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.dropin_steps):
            step_keyed()
        torch.cuda.synchronize()
        d_el = time.perf_counter() - t1
        dw = d_words.cpu().numpy().view(np.uint64)
        dg = np.unpackbits(dw.view(np.uint8), bitorder="little")[:n].astype(bool)
        dropin = {"key_window": w_drop, "value": n * args.dropin_steps / d_el,
                  "ms_per_step": d_el / args.dropin_steps * 1e3, "same_verdicts": bool((dg == got).all()),
                  "note": "device-resident keyed step at the window GpuAuthNr picks for its default max_keys=16384 "
                          "in 32 GiB of key tables (the headline uses %d: %d keys)" % (args.key_window,
                                                                                          reg_pks.shape[0])}

    # ---- the headline: the whole node (GpuAuthNr over json-decoded request dicts), every rank
    whole, wn_sets, wn_idrs, wn_vks = None, None, None, None
    if args.whole_node_n > 0 and args.config == "c1" and args.path == "keyed":
        host0 = host_cpus()
        budget = host0["affinity"]
        if host0["cgroup_cpu_quota"]:
            budget = min(budget, int(host0["cgroup_cpu_quota"]))
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
        # one node process per GPU: the host's CPU share divided between the ranks (0 = the scan's own rule:
        # up to 16, one per 2k requests, within the affinity and the cgroup quota)
        scan_threads = 0 if local_world == 1 else max(1, min(16, budget // local_world))
        tw = time.perf_counter()
        wn_sets, wn_idrs, wn_vks = whole_node_sets(eng, args.whole_node_n, pks, sks, args.alias_len, rank)
        build_s = time.perf_counter() - tw
        whole, _wa = time_whole_node(eng, args, wn_sets, wn_idrs, wn_vks, dist_on, dev, scan_threads)
        del _wa
        whole["requests_built_s"] = build_s
        whole["host_cpus"] = host0
        if dist_on:
            bad = torch.tensor([whole["pipelined"]["mismatches"] + whole["synchronous"]["mismatches"]],
                               dtype=torch.int64, device=dev)
            dist.all_reduce(bad)
            whole["mismatches_all_ranks"] = int(bad.item())
        else:
            whole["mismatches_all_ranks"] = whole["pipelined"]["mismatches"] + whole["synchronous"]["mismatches"]
        for k in ("pipelined", "synchronous"):  # whole job: every rank's batches over the slowest rank's time
            whole[k]["value_per_rank"] = whole[k]["value"]
            whole[k]["value"] = whole[k]["value"] * world

    cpu = None
    lib_mis = 0 if whole is None else whole["mismatches_all_ranks"]
    if rank == 0 and world == 1 and not args.no_cpu:
        s = min(args.cpu_sample if args.config != "c3" else args.cpu_sample // 4, n)
        sig_h = d_sig[:s].cpu().numpy()
        pk_h = d_pk[:s].cpu().numpy()
        # contiguous copy of the sample's messages (the harness takes offsets)
        starts, ends = item_start[:s].astype(np.int64), item_end[:s].astype(np.int64)
        off_h = np.zeros(s + 1, np.uint64)
        off_h[1:] = np.cumsum(ends - starts)
        msg_h = np.concatenate([buf[a:b] for a, b in zip(starts, ends)] + [np.zeros(16, np.uint8)])
        host = host_cpus()
        runs = {}
        for threads in sorted({host["affinity"], min(16, host["affinity"])}):
            if args.cpu_threads:
                threads = args.cpu_threads
            rate, ok, kind, ver = cpu_baseline(sig_h, pk_h, msg_h, off_h, threads)
            runs[threads] = (rate, ok)
        best = max(runs, key=lambda t: runs[t][0])
        rate, ok = runs[best]
        cpu = {"value": rate, "unit": "verifies/s", "cores": best, "kind": kind,
               "sample": "first %d requests of this workload, libsodium %s crypto_sign_verify_detached, one pthread "
                         "per core; best of %s threads" % (s, ver or "(absent: oracle restatement)", sorted(runs)),
               "by_threads": {str(t): r for t, (r, _) in runs.items()},
               "host": host,
               "agrees_with_gpu": bool(all((o == got[:s]).all() for _, o in runs.values()))}
        # every item of the timed batch against libsodium (untimed): the step's bitmask == libsodium's
        lib_ok, lib_s = sodium_all_items(d_sig.cpu().numpy(), d_pk.cpu().numpy(), buf, item_start, item_end,
                                         min(16, host["affinity"]))
        if lib_ok is not None:
            lib_mis = int((lib_ok != got).sum())
            cpu["agrees_with_gpu_all_items"] = lib_mis == 0
            cpu["all_items_check"] = {"items": n, "mismatches": lib_mis, "accepted_by_libsodium": int(lib_ok.sum()),
                                      "threads": min(16, host["affinity"]), "seconds": lib_s}
        if args.e2e_c0 > 0:
            cpu["reference_path_configs0"] = reference_path_baseline(eng, args.e2e_c0, host)

    e2e = None
    if rank == 0 and world == 1 and args.config == "c1" and args.key_order == "arrival":
        e2e = {}
        if args.e2e_c0 > 0:
            reqs, idrs, vks = e2e_requests(eng, args.e2e_c0, 100, 0, seed=11)
            e2e["configs0"] = time_e2e(eng, reqs, idrs, vks)
            del reqs
        if args.e2e_n > 0:
            m = min(args.e2e_n, n)
            if wn_sets is not None and len(wn_sets[0]) == m:  # the headline's first request set
                reqs, idrs, vks = wn_sets[0], wn_idrs, wn_vks
            else:
                sig_all = d_sig[:m].cpu().numpy()
                reqs, idrs, vks = e2e_requests(eng, m, args.signers, args.alias_len, spec=nym_spec, sig=sig_all,
                                               pks=pks)
            e2e["configs1"] = time_e2e(eng, reqs, idrs, vks)
            if args.drain_n > 0:
                e2e["node_drain"] = time_node_drain(eng, reqs, idrs, vks, drains=args.drain_n)
            if args.e2e_devices:
                ndev = torch.cuda.device_count()
                counts = [k for k in (1, 2, 4, 8) if k <= ndev]
                e2e["by_devices"] = time_e2e_devices(eng, reqs, idrs, vks, counts)
                e2e["by_devices"]["note"] = (
                    "one node process over MultiEngine(k engines): configs1's %d requests per batch split by "
                    "64-aligned request index across k devices (one host thread each), the native scan as in "
                    "configs1 (up to 16 host threads); %d device(s) visible" % (m, ndev))
            del reqs
        if args.bls_checks > 0:
            e2e["bls_commit_round"] = time_bls_commit_round(eng, args.bls_checks)
        if args.churn_signers > 0:
            e2e["key_churn"] = time_key_churn(eng, args.churn_signers, args.churn_requests)
            if e2e["key_churn"]["mismatches"]:
                lib_mis += e2e["key_churn"]["mismatches"]

    # the metric's "whole node" reading is the headline (time_whole_node); beside it the same run's libsodium
    whole_vs = None
    if whole is not None and cpu:
        whole_vs = {"pipelined": whole["pipelined"]["value"] / cpu["value"],
                    "synchronous": whole["synchronous"]["value"] / cpu["value"],
                    "cpu": "cpu_baseline.value: libsodium %s crypto_sign_verify_detached on %d host threads" % (
                        cpu.get("sample", "").split("libsodium ")[-1].split(" ")[0] or "1.0.18", cpu["cores"])}
    device_resident = {
        "value": value, "unit": "verifies/s", "steps": args.device_steps, "warmup": args.warmup,
        "ms_per_step": ms_per_step, "path": args.path,
        "note": "one step = the verify kernels over this rank's %d requests already resident in HBM (hash -> comb "
                "-> encode on the keyed path), %d steps queued back to back; the roofline is this leg's dominant "
                "kernel" % (n, args.device_steps),
        "phase_ms": {"hash": float(ph[0]), "table": float(ph[1]),
                     ("comb" if args.path == "keyed" else "dsm"): dsm_sum, "encode": float(ph[3]),
                     "note": "per-phase sums over the %d sub-batch launches of the last %d-request chunk" % (
                         launches, n_chunk)},
        "length_buckets": "packed" if args.length_buckets == "packed" else bool(buckets),
        "key_window": args.key_window, "key_table_build_ms": key_build_ms, "keys": int(reg_pks.shape[0]),
        "base_window": RL.BASE_W, "engine_create_s": create_s,
        "value_incl_key_build_one_step": (n * world / (ms_per_step * 1e-3 + key_build_ms * 1e-3)
                                          if args.path == "keyed" else None),
        "ref10_equivalent_frac": (n * RL.MAD_PER_VERIFY / (ms_per_step * 1e-3)) / RL.PEAK_MAD_PER_S,
        "other_path": other, "dropin_window": dropin}
    if rank == 0:
        if whole is not None:
            head_value = whole["synchronous"]["value"]
            head_ms, head_steps = whole["synchronous"]["ms_per_batch"], args.steps
            workload = ("configs[1]: %d single-signature NYM requests per GPU per step, each a request dict json-decoded "
                        "on its own as the node receives it, %.0f B mean signed payload, %d signers (addIdr), all "
                        "valid; step = one GpuAuthNr.authenticate_batch of them, one batch at a time (synchronous): "
                        "native scan + serialization on the host CPUs with the PCIe copy and kernels under it, "
                        "getVerkey per identifier, result list -- the drop-in for client_authn.py:67-107, batch by "
                        "batch; authenticate_batches (two batches in flight) beside it (whole_node.pipelined)" % (
                            whole["requests_per_batch"], mlen_mean, args.signers))
        else:
            head_value, head_ms, head_steps = value, ms_per_step, args.device_steps
            workload = "configs[%d]: %d %s per GPU, %.0f B mean signed payload, %d signers%s%s; step = the verify " \
                       "kernels over HBM-resident inputs" % (
                           int(args.config[1]), n,
                           "signature verifications" if args.config == "c3" else "single-signature requests",
                           mlen_mean, args.signers,
                           ", 10% corrupted/non-canonical/small-order" if args.config == "c2" else ", all valid",
                           req_desc + (" + PREPARE/COMMIT tally of %d keys x 25 validators in the step (RCCL "
                                       "all-reduce MAX of the ballots)" % (-(-(n // 2) * world // 50))
                                       if args.config == "c4" else ""))
        out = {
            "metric": METRIC, "value": head_value, "unit": "verifies/s", "n_gpus": world, "steps": head_steps,
            "warmup": args.warmup, "ms_per_step": head_ms, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u32 (radix-2^25.5 GF(2^255-19), 64-bit MAD accumulators)",
            "data": ("synthetic NYM requests signed on-GPU (deterministic Ed25519, libsodium-exact)"
                     + (", json-encoded and decoded one by one" if whole is not None else "")),
            "config": {"workload": workload, "requests_per_gpu": (whole or {}).get("requests_per_batch", n),
                       "signers": args.signers, "parallelism": "dp%d (one node process per GPU; request-index shards)"
                                                               % world,
                       "path": ("keyed: the signers' verkeys registered once (comb tables; drop-in window %s for the "
                                "whole node, %d on the device-resident leg; base window %d)" % (
                                    (whole or {}).get("key_window"), args.key_window, RL.BASE_W)
                                if args.path == "keyed" else
                                "general: every request carries its key bytes, inputs HBM-resident")},
            "end_to_end": e2e,
            "device_resident": device_resident,
            "roofline": {"bound": "valu", "kernel": kernel_name, "achieved": achieved, "peak": peak,
                         "unit": "TMAD/s", "frac": achieved / peak, "traffic": traffic,
                         "leg": "device_resident (the whole node is host-bound; this is its dominant GPU kernel)",
                         "algorithmic": "%d MAD per verify (%s), %d launches per chunk of %d requests (n=%d each; "
                                        "%d requests per step), avg launch %.3f ms (HIP events on the launch streams)" % (
                             kernel_mad, RL.kernel_work(kernel_name, args.key_window), launches, n_chunk,
                             n_chunk // launches, n, dsm_avg),
                         "standalone": standalone,
                         "valu_busy": (utilisation or {}).get(key, {}).get("valu_busy"),
                         "hbm_GBps": (utilisation or {}).get(key, {}).get("hbm_GBps"),
                         "clock_GHz": (utilisation or {}).get(key, {}).get("clock_GHz"),
                         # the same achieved rate against the MAD peak at the clock the chip held under
                         # this kernel (GRBM_GUI_ACTIVE): what the instruction mix and issue leave
                         "frac_at_held_clock": (achieved / (peak * (utilisation or {}).get(key, {})["clock_GHz"] / 2.4)
                                                if (utilisation or {}).get(key, {}).get("clock_GHz") else None),
                         "utilisation": utilisation,
                         "frac_survey": (n * RL.MAD_PER_VERIFY / (ms_per_step * 1e-3)) / RL.PEAK_MAD_PER_S,
                         "frac_survey_note": "SURVEY 8(d)'s a-priori 305,000 MAD per verify (ref10: decode A + 253 "
                                             "doublings + ~86 additions + inversion) x requests / device step time / "
                                             "peak; > 1 on the keyed path because per-key comb tables built once at "
                                             "registration replace A's decode and every doubling (%d MAD per "
                                             "request in the step's dominant kernel)" % kernel_mad},
            "build": build_stamp(eng),
            "cpu_baseline": cpu,
            "parity": {"mismatches_vs_construction": mismatches, "accepted": accepted, "expected": expected,
                       "mismatches_vs_libsodium_all_items": (cpu or {}).get("all_items_check", {}).get("mismatches"),
                       "whole_node_mismatches": (whole or {}).get("mismatches_all_ranks"),
                       "ranks": world, "accepted_in_gathered_bitmask": gathered_accepted},
            "tally": tally_result,
            "collective": collective,
            # last, so the driver's tail of the line keeps them: the headline's two forms and their ratio
            "whole_node": whole,
            "whole_node_vs_cpu": whole_vs,
        }
        print(json.dumps(out), flush=True)
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()
    eng.close()
    if mismatches or lib_mis:
        sys.exit(3)


if __name__ == "__main__":
    main()
