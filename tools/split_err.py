"""Accuracy of the split-f16 GEMM form (tts_amd/csrc/split16.h) against an fp64 reference, next to
a plain fp32 GEMM of the same operands. Emulated on the CPU with numpy's IEEE float16 (round to
nearest even, as v_cvt_f16_f32 / v_cvt_pk_f16_f32):

    hi = f16(v),  lo = f16((v - hi) * 2^11),   a.b ~ hi_a.hi_b + 2^-11 (hi_a.lo_b + lo_a.hi_b)

f16 x f16 products are exact in fp32; the sums are accumulated in fp32 over K in 32-wide k-steps
(one v_mfma_f32_16x16x32_f16 each), the main and correction sums in separate accumulators and
combined at the end, as the kernels do. The fp32 reference GEMM accumulates in fp32 in k order.

Usage: python tools/split_err.py   (prints max |error| relative to max |C| for a few shapes and
operand scales, including the small-magnitude range where lo is subnormal-adjacent)
"""
import numpy as np

SCALE = np.float32(2048.0)


def split(v):
    v = v.astype(np.float32)
    hi = v.astype(np.float16)
    lo = ((v - hi.astype(np.float32)) * SCALE).astype(np.float16)
    return hi, lo


def gemm_x3(a, b):
    """a (M, K), b (K, N) fp32 -> fp32, split-f16 with per-32 k-step fp32 accumulation."""
    ah, al = split(a)
    bh, bl = split(b)
    M, K = a.shape
    N = b.shape[1]
    main = np.zeros((M, N), np.float32)
    corr = np.zeros((M, N), np.float32)
    for k0 in range(0, K, 32):
        s = slice(k0, k0 + 32)
        # exact products, summed inside the k-step in fp64 then rounded once (an MFMA's internal
        # sum is at least as accurate as fp32 chained adds), accumulated across k-steps in fp32
        ahs, als, bhs, bls = (x[:, s].astype(np.float64) if x.shape[0] == M else x[s].astype(np.float64)
                              for x in (ah, al, bh, bl))
        main = (main + (ahs @ bhs).astype(np.float32)).astype(np.float32)
        corr = (corr + (ahs @ bls + als @ bhs).astype(np.float32)).astype(np.float32)
    return (main + corr / SCALE).astype(np.float32)


def gemm_f32(a, b):
    out = np.zeros((a.shape[0], b.shape[1]), np.float32)
    for k in range(a.shape[1]):
        out = (out + np.outer(a[:, k], b[k]).astype(np.float32)).astype(np.float32)
    return out


def main():
    rs = np.random.RandomState(0)
    print(f"{'M x K x N':>18s} {'scale':>8s} {'x3 err/max|C|':>15s} {'fp32 err/max|C|':>16s}")
    for (M, K, N) in [(64, 576, 64), (64, 2560, 32), (48, 160, 128)]:
        for sc in (1.0, 1e-3, 30.0):
            a = (rs.standard_normal((M, K)) * sc / np.sqrt(K)).astype(np.float32)
            b = rs.standard_normal((K, N)).astype(np.float32)
            ref = a.astype(np.float64) @ b.astype(np.float64)
            mx = np.abs(ref).max()
            e3 = np.abs(gemm_x3(a, b) - ref).max() / mx
            e32 = np.abs(gemm_f32(a, b) - ref).max() / mx
            print(f"{M:5d} x {K:4d} x {N:4d} {sc:8.0e} {e3:15.2e} {e32:16.2e}")


if __name__ == "__main__":
    main()
