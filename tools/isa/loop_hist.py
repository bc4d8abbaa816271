"""Instruction histogram of the loop bodies of one kernel in a hipcc -S listing.
usage: python tools/isa/loop_hist.py listing.s KERNEL_SUBSTRING
A loop body = the lines from a label to a later s_cbranch that jumps back to it."""
import collections, re, sys
path, name = sys.argv[1], sys.argv[2]
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and name in l and l.rstrip().endswith(":") is False or (l.startswith("_Z") and name in l and ":" in l))
end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith("s_endpgm"))
body = lines[start:end + 1]
labels = {l.split(":")[0]: i for i, l in enumerate(body) if re.match(r"^\.LBB\S+:", l)}
for i, l in enumerate(body):
    m = re.match(r"\s+s_cbranch_\w+\s+(\.LBB\S+)", l) or re.match(r"\s+s_branch\s+(\.LBB\S+)", l)
    if m and m.group(1) in labels and labels[m.group(1)] < i:
        j0 = labels[m.group(1)]
        ops = [x.split()[0] for x in body[j0 + 1:i + 1] if x.startswith("\t") and not x.strip().startswith(";") and not x.strip().startswith(".")]
        h = collections.Counter(ops)
        v = sum(c for o, c in h.items() if o.startswith("v_"))
        print("loop %s..%d: %d instructions, %d VALU" % (m.group(1), i, len(ops), v))
        for o, c in h.most_common(40):
            print("   %5d %s" % (c, o))
        # issue cycles per wave64 instruction on gfx950 (profiles/r02f/ubench_int*.txt: ~120 lane-ops
        # per clock per CU -> 2 cycles; ~60 -> 4); anything not listed counted at 4
        two = ("v_add_u32", "v_sub_u32", "v_and_b32", "v_or_b32", "v_xor_b32", "v_mov_b32", "v_bitop3_b32",
               "v_lshrrev_b32", "v_ashrrev_i32", "v_fma_f32")
        cyc = {o: (2 if o.split("_e32")[0].split("_e64")[0] in two else 4) for o in h if o.startswith("v_")}
        total = sum(cyc[o] * c for o, c in h.items() if o.startswith("v_"))
        mad = 4 * h.get("v_mad_u64_u32", 0)
        print("   v_mad_u64_u32: %.3f of the VALU instructions, %.3f of their issue cycles (%d of %d per wave)"
              % (h.get("v_mad_u64_u32", 0) / max(v, 1), mad / max(total, 1), mad, total))
