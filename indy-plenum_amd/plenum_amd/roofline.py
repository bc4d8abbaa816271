"""Algorithmic work per verification and the gfx950 peak it is priced against.

The path is 32-bit-integer VALU bound: neither HBM (about
300 B of input per verify) nor MFMA (not a dense contraction).  Work is fixed
a priori from libsodium's ref10 algorithm, not from this implementation:
  field multiplications/squarings per verify F = 3,050
    = 2,510 (double-scalar multiplication) + 270 (decode A) + 270 (encode's inversion)
  one field op = 100 32x32->64 multiply-adds  ->  305,000 MAD per verify
  SHA-512 = 5,000 32-bit ALU ops per 128-byte block, ceil((mlen + 81) / 128) blocks.
The general path's dominant kernel (edv_dsm_kernel) carries the double-scalar
multiplication: 2,510 * 100 = 251,000 MAD per verify; the encode's inversion
is shared by 16 requests in edv_encode_kernel (batch_encode.h).

Peak: v_mad_u64_u32 issues at half rate on gfx950 (64 lane-ops/clk/CU;
tools/microbench/ubench_int.hip measured 58.7 at 16 waves/CU), so
256 CUs * 64 * 2.4 GHz = 39.32 T MAD/s (MI355X_MICROARCH.md: 256 CUs, 2.4 GHz).
"""
MAD_PER_FE = 100
FE_DSM = 2510
FE_DECODE = 270
FE_ENCODE = 267
MAD_PER_VERIFY = 305_000
# General path: edv_dsm_kernel carries the double-scalar multiplication (the
# a-priori ref10 count); edv_table_kernel the decode of A.
MAD_DSM_KERNEL = FE_DSM * MAD_PER_FE  # 251,000
MAD_TABLE_KERNEL = FE_DECODE * MAD_PER_FE


# The implementation's edv_dsm_kernel with K split tables per distinct key
# (verify_core.h verify_phase_dsm_split_point): 64/K - 1 steps of 4 doublings
# (3 x (4 sq + 3 mul) + (4 sq + 4 mul) = 29 field ops), 64 cached additions
# (4 + 4 field ops), ceil(254 / kBaseW) = 11 base-comb mixed additions (7).
# K = 1: 2,416 field ops (ref10's 2,510 less its sliding-window bookkeeping);
# K = 4: 1,024; K = 8: 792.
def fe_dsm_split(k):
    return (64 // k - 1) * 29 + 64 * 8 + BASE_ROWS * 7


def mad_dsm_kernel(k):
    return fe_dsm_split(k) * MAD_PER_FE


def split_of(distinct, n):
    """edverify.hip split_of: tables per distinct key of a sub-batch."""
    return 8 if 16 * distinct <= n else 4 if 4 * distinct <= n else 1
# Key-table path (keys registered once): edv_comb_kernel<W> = fixed-base combs
# over both tables -- ceil(254 / W) rows of the key table + ceil(254 / kBaseW)
# rows of the base table (verify_core.h kBaseW = 24: 11 rows) -- one mixed
# addition (7 multiplications) per row, except the key comb's row 0, which is
# set with one multiplication (comb.h comb_set).  The base window is the
# library's (edv_base_window; set_base_window), so the price follows the build.
BASE_W = 24


def key_rows(w):
    return (254 + w - 1) // w


BASE_ROWS = key_rows(BASE_W)


def set_base_window(w):
    """Price the base comb at the window the loaded library was built with."""
    global BASE_W, BASE_ROWS
    BASE_W, BASE_ROWS = int(w), key_rows(int(w))


def mad_comb_kernel(w):
    return ((key_rows(w) - 1 + BASE_ROWS) * 7 + 1) * MAD_PER_FE  # base 24, W=14: 20,400; W=10: 25,300


# edv_encode_kernel<M>: per request 3 multiplications of Montgomery's trick +
# 2 (x, y) + the shared inversion (FE_ENCODE) / M.
def mad_encode_kernel(m):
    return (5 + FE_ENCODE / m) * MAD_PER_FE


def kernel_work(name, w=8):
    if name == "edv_comb_kernel":
        return ("((%d - 1 key rows (W=%d; row 0 set with 1 field op) + %d base rows (W=%d)) mixed additions "
                "x 7 field ops + 1) x 100 MAD" % (key_rows(w), w, BASE_ROWS, BASE_W))
    if name == "edv_dsm_kernel":
        return ("((64/K - 1) x 29 + 64 x 8 + %d x 7) field ops x 100 MAD (K split tables per distinct key, "
                "roofline.fe_dsm_split)" % BASE_ROWS)
    return ""


SHA_ALU_PER_BLOCK = 5_000

CUS = 256
CLOCK_HZ = 2.4e9
MAD_LANE_OPS_PER_CLK_CU = 64
PEAK_MAD_PER_S = CUS * MAD_LANE_OPS_PER_CLK_CU * CLOCK_HZ  # 39.32e12
MEASURED_MAD_PER_S = 36.1e12  # tools/microbench/ubench_int: 58.75 lane-ops/clk/CU at 16 waves/CU


SIMDS = CUS * 4
XCDS = 8


def pmc_utilisation(row, launch_ms, n_per_launch, mad_per_request=None):
    """VALU utilisation, clock and HBM rate of one kernel: its counters from the
    committed PMC pass (tools/pmc_passes.sh -> tools/pmc_summary.py; `row` is
    one kernel of pmc_traffic.json, counters per launch over n_req requests)
    and its launch duration measured live (HIP events).

      clock      = GRBM_GUI_ACTIVE / 8 / duration   (GRBM sums the 8 XCDs;
                   MI355X_MICROARCH.md 'DVFS give-back')
      valu_busy  = SQ_ACTIVE_INST_VALU * 4 / (SIMDs * GRBM_GUI_ACTIVE / 8)
                   (rocprof's gfx94x VALUBusy: SQ counts quad-cycles, one per
                   wave64 VALU issue; 1.0 = every SIMD issued a VALU op every
                   4 cycles of the kernel)
      hbm_GBps   = (2 * FETCH_SIZE + WRITE_SIZE) bytes per request (gfx950
                   FETCH_SIZE correction) * requests of the launch / duration
      mad_share  = v_mad_u64_u32 per request / 64 over VALU instructions per
                   request (wave64 instructions)
    """
    m = row.get("mean", {})
    n_req = float(row.get("n_requests", 1_000_000))
    sec = launch_ms * 1e-3
    # the PMC launch covered n_req requests; scale its cycle counts to this launch's size
    scale = n_per_launch / n_req
    out = {"launch_ms": launch_ms, "n_per_launch": n_per_launch}
    if "GRBM_GUI_ACTIVE" in m:
        gui = m["GRBM_GUI_ACTIVE"] * scale
        out["clock_GHz"] = gui / XCDS / sec / 1e9
        if "SQ_ACTIVE_INST_VALU" in m:
            out["valu_busy"] = m["SQ_ACTIVE_INST_VALU"] * scale * 4 / (SIMDS * gui / XCDS)
    if "traffic_bytes_per_request" in row:
        out["hbm_bytes_per_request"] = row["traffic_bytes_per_request"]
        out["hbm_GBps"] = row["traffic_bytes_per_request"] * n_per_launch / sec / 1e9
        out["hbm_frac_of_8TBps"] = out["hbm_GBps"] / 8000.0
    if "SQ_INSTS_VALU" in m:
        vpr = m["SQ_INSTS_VALU"] / n_req  # wave64 instructions per request
        out["valu_insts_per_request"] = vpr * 64  # lane-instructions
        if mad_per_request:
            out["mad_share_of_valu"] = mad_per_request / (vpr * 64)
    return out


def sha_blocks(mlen):
    return (mlen + 81 + 127) // 128


def algo_ops(mlen):
    """ALGO_OPS(mlen) = 305,000 MAD + 5,000 * ceil((mlen + 81) / 128) ALU."""
    return MAD_PER_VERIFY + SHA_ALU_PER_BLOCK * sha_blocks(mlen)
