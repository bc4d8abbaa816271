"""Summarise rocprofv3 --pmc passes (tools/pmc_passes.sh) per kernel.

usage: python tools/pmc_summary.py gpurun_out/pmc [n_requests] [out_json]
Per kernel: mean counter value per dispatch, per-request figures, and the HBM
traffic per launch used by bench.py's roofline.traffic:
  traffic = 2 * FETCH_SIZE + WRITE_SIZE   (kB -> bytes; FETCH_SIZE x 2 is the
  gfx950 correction of MI355X_MICROARCH.md 'HBM [CDNA4]': FETCH_SIZE counts
  128-B requests at 64 B).  SQ_* cycle counters count quad-cycles.
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def short(name):
    m = re.search(r"(edv_\w+?)(?:<(\w+)>)?\(", name)
    if m:
        return m.group(1) + ("<%s>" % m.group(2) if m.group(2) else "")
    return name[:60]


def load(root):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    grid = {}
    for path in glob.glob(os.path.join(root, "*", "*counter_collection.csv")):
        with open(path) as f:
            for row in csv.DictReader(f):
                k = short(row["Kernel_Name"])
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
                grid[k] = int(row["Grid_Size"])
    return acc, grid


def main():
    root = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    out_json = sys.argv[3] if len(sys.argv) > 3 else None
    acc, grid = load(root)
    summary = {"n": n, "kernels": {}, "run": sys.argv[4] if len(sys.argv) > 4 else os.path.basename(root)}
    for k in sorted(acc):
        c = {name: sum(v) / len(v) for name, v in acc[k].items()}
        row = {"grid": grid[k], "dispatches": max(len(v) for v in acc[k].values()), "mean": c, "n_requests": n}
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            row["traffic_bytes"] = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
            row["traffic_bytes_per_request"] = row["traffic_bytes"] / n
        if "SQ_INSTS_VALU" in c and "SQ_WAVES" in c:
            row["valu_insts_per_request"] = c["SQ_INSTS_VALU"] / n
            if "SQ_ACTIVE_INST_VALU" in c and "SQ_BUSY_CYCLES" in c:
                row["valu_active_quads_per_request"] = c["SQ_ACTIVE_INST_VALU"] / n
        summary["kernels"][k] = row
    for k, row in summary["kernels"].items():
        if row["grid"] < 1000:
            continue
        m = row["mean"]
        parts = ["%-28s grid=%8d" % (k, row["grid"])]
        if "traffic_bytes" in row:
            parts.append("traffic %.1f MB (%.0f B/req; fetch %.1f MB raw, write %.1f MB)" % (
                row["traffic_bytes"] / 1e6, row["traffic_bytes_per_request"], m["FETCH_SIZE"] * 1024 / 1e6,
                m["WRITE_SIZE"] * 1024 / 1e6))
        if "SQ_INSTS_VALU" in m:
            parts.append("VALU %.0f inst/req" % (m["SQ_INSTS_VALU"] / n))
        if "SQ_INSTS_VALU_INT64" in m:
            parts.append("int64 %.0f int32 %.0f /req" % (m["SQ_INSTS_VALU_INT64"] / n, m["SQ_INSTS_VALU_INT32"] / n))
        if "SQ_ACTIVE_INST_VALU" in m and "SQ_WAVE_CYCLES" in m:
            parts.append("VALU-active/wave-cycles %.2f" % (m["SQ_ACTIVE_INST_VALU"] / m["SQ_WAVE_CYCLES"]))
        if "SQ_WAIT_INST_ANY" in m and "SQ_WAVE_CYCLES" in m:
            parts.append("issue-stall/wave-cycles %.2f" % (m["SQ_WAIT_INST_ANY"] / m["SQ_WAVE_CYCLES"]))
        if "SQ_WAIT_ANY" in m and "SQ_WAVE_CYCLES" in m:
            parts.append("wait/wave-cycles %.2f" % (m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"]))
        print(" | ".join(parts))
    if out_json:
        with open(out_json, "w") as f:
            json.dump(summary, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
