"""One-screen summary of a bench.py log (its last JSON line): headline, roofline,
CPU baseline and the end-to-end / node-drain / BLS legs.  Usage: python tools/bench_summary.py LOG"""
import json
import sys


def r(x, k=1):
    return None if x is None else round(x, k)


def main(path):
    lines = [x for x in open(path) if x.startswith('{"metric')]
    if not lines:
        print("no bench line in", path)
        return
    d = json.loads(lines[-1])
    rl = d["roofline"]
    dr = d.get("device_resident") or d
    print("value %.2f M/s  %.3f ms/step  n_gpus %d | device-resident %.1f M/s  %.3f ms/step  frac %.3f  busy %s  "
          "GB/s %s  clk %s" % (d["value"] / 1e6, d["ms_per_step"], d["n_gpus"], dr["value"] / 1e6, dr["ms_per_step"],
                               rl["frac"], r(rl.get("valu_busy"), 3), r(rl.get("hbm_GBps"), 0),
                               r(rl.get("clock_GHz"), 3)))
    ph = dr.get("phase_ms") or {}
    print("phases", {k: r(v, 3) for k, v in ph.items() if k != "note"})
    cpu = d.get("cpu_baseline")
    if cpu:
        print("cpu %.1f k/s on %s cores (%s)  all items vs libsodium: %s" % (
            cpu["value"] / 1e3, cpu["cores"], cpu["kind"], (cpu.get("all_items_check") or {}).get("mismatches")))
    w, wv = d.get("whole_node"), d.get("whole_node_vs_cpu") or {}
    if w:
        print("whole node: sync %.2f M/s (%sx cpu), pipelined %.2f M/s (%sx cpu), mismatches %s" % (
            w["synchronous"]["value"] / 1e6, r(wv.get("synchronous")), w["pipelined"]["value"] / 1e6,
            r(wv.get("pipelined")), w.get("mismatches_all_ranks")))
        print("   sync batch ms", {k: r(v, 2) for k, v in w["synchronous"]["batch_ms"].items()},
              {k: r(v, 2) for k, v in (w["synchronous"].get("in_batch_ms") or {}).items()})
    for k, v in (d.get("end_to_end") or {}).items():
        if k == "by_devices":
            print(" ", k, {kk: (r(vv["value"] / 1e6, 2) if "value" in vv else vv.get("error"))
                           for kk, vv in v.items() if isinstance(vv, dict)})
        elif k in ("node_drain", "bls_commit_round"):
            print(" ", k, {kk: (r(vv, 2) if isinstance(vv, float) else vv) for kk, vv in v.items()
                           if not isinstance(vv, (dict, list, str))})
        else:
            s = v.get("single_authenticate_us") or {}
            print(" ", k, r(v["value"] / 1e6, 2), "M/s  pipelined", r((v.get("pipelined") or {}).get("value", 0) / 1e6, 2),
                  "single p50", r(s.get("p50")),
                  {kk: r(vv, 2) for kk, vv in (v.get("in_batch_ms") or {}).items()})


if __name__ == "__main__":
    main(sys.argv[1])
