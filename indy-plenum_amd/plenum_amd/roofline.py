"""Algorithmic work per verification and the gfx950 peak it is priced against.

The path is 32-bit-integer VALU bound: neither HBM (about
300 B of input per verify) nor MFMA (not a dense contraction).  Work is fixed
a priori from libsodium's ref10 algorithm, not from this implementation:
  field multiplications/squarings per verify F = 3,050
    = 2,510 (double-scalar multiplication) + 270 (decode A) + 270 (encode's inversion)
  one field op = 100 32x32->64 multiply-adds  ->  305,000 MAD per verify
  SHA-512 = 5,000 32-bit ALU ops per 128-byte block, ceil((mlen + 81) / 128) blocks.
The dominant kernel (edv_dsm_kernel) carries the double-scalar multiplication
and the encode: (2,510 + 267) * 100 = 277,700 MAD per verify.

Peak: v_mad_u64_u32 issues at half rate on gfx950 (64 lane-ops/clk/CU;
tools/microbench/ubench_int.hip measured 58.7 at 16 waves/CU), so
256 CUs * 64 * 2.4 GHz = 39.32 T MAD/s (MI355X_MICROARCH.md: 256 CUs, 2.4 GHz).
"""
MAD_PER_FE = 100
FE_DSM = 2510
FE_DECODE = 270
FE_ENCODE = 267
MAD_PER_VERIFY = 305_000
MAD_DSM_KERNEL = (FE_DSM + FE_ENCODE) * MAD_PER_FE  # 277,700
MAD_TABLE_KERNEL = FE_DECODE * MAD_PER_FE
# Key-table path (keys registered once): edv_comb_kernel = fixed-base comb over
# both tables -- 64 rows of the W=4 key table + 32 rows of the W=8 base table --
# 96 mixed additions x 7 multiplications, plus the encode inversion.
COMB_ADDS = 64 + 32
FE_COMB = COMB_ADDS * 7
MAD_COMB_KERNEL = (FE_COMB + FE_ENCODE) * MAD_PER_FE  # 93,900
KERNEL_WORK = {
    "edv_dsm_kernel": "(2510 DSM + 267 encode) field ops x 100, ref10 a-priori count",
    "edv_comb_kernel": "(96 mixed adds x 7 + 267 encode) field ops x 100, fixed-base comb: 64 key rows (W=4) + 32 base rows (W=8)",
}
SHA_ALU_PER_BLOCK = 5_000

CUS = 256
CLOCK_HZ = 2.4e9
MAD_LANE_OPS_PER_CLK_CU = 64
PEAK_MAD_PER_S = CUS * MAD_LANE_OPS_PER_CLK_CU * CLOCK_HZ  # 39.32e12
MEASURED_MAD_PER_S = 36.1e12  # tools/microbench/ubench_int: 58.75 lane-ops/clk/CU at 16 waves/CU


def sha_blocks(mlen):
    return (mlen + 81 + 127) // 128


def algo_ops(mlen):
    """ALGO_OPS(mlen) = 305,000 MAD + 5,000 * ceil((mlen + 81) / 128) ALU."""
    return MAD_PER_VERIFY + SHA_ALU_PER_BLOCK * sha_blocks(mlen)
