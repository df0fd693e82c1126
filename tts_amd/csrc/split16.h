// Split-f16 operands for fp32-accurate GEMMs on the gfx950 f16 MFMA.
//
// Every fp32 operand v is carried as two f16 halves,
//   hi = f16(v),   lo = f16((v - hi) * 2^11),   v = hi + lo * 2^-11   (22 significant bits),
// and a product is formed from three MFMAs whose f16 x f16 products are exact in fp32:
//   a.b = hi_a.hi_b + 2^-11 (hi_a.lo_b + lo_a.hi_b)        (dropped: 2^-22 lo_a.lo_b)
// with the two sums accumulated in fp32 (v_mfma_f32_16x16x32_f16, 16 cycles per SIMD, 16x the
// rate of the fp32 v_mfma_f32_16x16x4_f32). Scaling lo by 2^11 keeps it a normal f16 for |v| down
// to ~6e-5 (below that its absolute error stays under 1e-11). Against an fp64 reference the error
// of this form matches the fp32 MFMA GEMM's (tools/split_err.py): the GEMM is
// fp32-accurate, not a reduced-precision shortcut. Range: |v| < 65504 (f16 max); producers flag
// anything outside it and the host re-runs that call on the fp32 kernels.
#pragma once
#include <cstdint>
#include <cstring>
#include <vector>

constexpr float SPLIT_SCALE = 2048.f;
constexpr float SPLIT_INV = 1.f / 2048.f;
constexpr float F16_RANGE = 65504.f;

// host: fp32 -> f16 bits, round to nearest even (normal, subnormal, overflow to inf)
inline uint16_t f32_to_f16_rne(float f) {
  uint32_t x;
  std::memcpy(&x, &f, 4);
  const uint32_t sign = (x >> 16) & 0x8000u;
  const uint32_t ax = x & 0x7fffffffu;
  if (ax >= 0x7f800000u) return (uint16_t)(sign | 0x7c00u | (ax > 0x7f800000u ? 0x200u : 0u));
  if (ax >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u);  // rounds past 65504
  if (ax < 0x38800000u) {                                      // f16 subnormal or zero
    if (ax < 0x33000000u) return (uint16_t)sign;               // below half the smallest subnormal
    const uint32_t m = (ax & 0x7fffffu) | 0x800000u;
    const int shift = 126 - (int)(ax >> 23);                   // 14 .. 24
    uint32_t r = m >> shift;
    const uint32_t rem = m & ((1u << shift) - 1), half = 1u << (shift - 1);
    if (rem > half || (rem == half && (r & 1u))) ++r;
    return (uint16_t)(sign | r);
  }
  uint32_t r = ((ax >> 13) - (112u << 10));
  const uint32_t rem = ax & 0x1fffu;
  if (rem > 0x1000u || (rem == 0x1000u && (r & 1u))) ++r;
  return (uint16_t)(sign | r);
}
inline float f16_to_f32(uint16_t h) {
  const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
  const uint32_t e = (h >> 10) & 0x1fu, m = h & 0x3ffu;
  uint32_t x;
  if (e == 0) {
    if (m == 0) x = sign;
    else {
      float v = (float)m * (1.f / 16777216.f);  // m * 2^-24
      std::memcpy(&x, &v, 4);
      x |= sign;
    }
  } else if (e == 31) x = sign | 0x7f800000u | (m << 13);
  else x = sign | ((e + 112u) << 23) | (m << 13);
  float f;
  std::memcpy(&f, &x, 4);
  return f;
}
inline void split_host(float v, uint16_t& hi, uint16_t& lo) {
  hi = f32_to_f16_rne(v);
  lo = f32_to_f16_rne((v - f16_to_f32(hi)) * SPLIT_SCALE);
}

// A-operand fragments of v_mfma_f32_16x16x32_f16 for a (rows x K) matrix given by f(m, k), split:
// for m-tile mt and k-step ks, 64 lanes x {8 hi halves, 8 lo halves} (32 bytes per lane);
// element j of lane l is W[16 mt + (l & 15)][32 ks + 8 (l >> 4) + j]. Blocks are ordered
// [mt][ks]; f returns 0 outside the matrix (padding).
template <class F>
std::vector<uint16_t> pack_split_a(int mtiles, int ksteps, F f) {
  std::vector<uint16_t> out((size_t)mtiles * ksteps * 64 * 16);
  for (int mt = 0; mt < mtiles; ++mt)
    for (int ks = 0; ks < ksteps; ++ks)
      for (int l = 0; l < 64; ++l) {
        uint16_t* o = &out[(((size_t)mt * ksteps + ks) * 64 + l) * 16];
        for (int j = 0; j < 8; ++j) split_host(f(16 * mt + (l & 15), 32 * ks + 8 * (l >> 4) + j), o[j], o[8 + j]);
      }
  return out;
}

#ifdef __HIPCC__
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));

// D += A.B on the f16 MFMA (16x16 output, K = 32); lane maps as for the bf16 form
// (cdna_hip_programming.md §3): A[m = l & 15][k = 8 (l >> 4) + j], B[k = 8 (l >> 4) + j][n = l & 15]
#define MFMA_H(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_f16((a), (b), (c), 0, 0, 0)

// acc_main += ah.bh; acc_corr += ah.bl + al.bh  (the value is acc_main + 2^-11 acc_corr)
__device__ __forceinline__ void mfma_x3(const h8& ah, const h8& al, const h8& bh, const h8& bl, f32x4& am,
                                        f32x4& ac) {
  am = MFMA_H(ah, bh, am);
  ac = MFMA_H(ah, bl, ac);
  ac = MFMA_H(al, bh, ac);
}
__device__ __forceinline__ float x3_value(float am, float ac) { return am + ac * SPLIT_INV; }

// device split of one value (no range check): v_cvt_f16_f32 for hi, and lo as one
// v_fma_mixlo_f16: 2^11 v - 2^11 hi is exact in fp32, so lo takes a single rounding
__device__ __forceinline__ void split_fast(float v, _Float16& hi, _Float16& lo) {
  hi = (_Float16)v;
  lo = (_Float16)__builtin_fmaf((float)hi, -SPLIT_SCALE, v * SPLIT_SCALE);
}
// two values at once: v_cvt_pk_f16_f32 (round to nearest even, as the scalar conversion) and
// packed fp32 math -- 3 VALU ops per pair instead of 5 per value; bit-identical to split_fast
typedef float f32x2_ __attribute__((ext_vector_type(2)));
typedef _Float16 h2_ __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void split2(f32x2_ v, h2_& hi, h2_& lo) {
  hi = __builtin_convertvector(v, h2_);
  const f32x2_ hf = __builtin_convertvector(hi, f32x2_);
  lo = __builtin_convertvector(v * SPLIT_SCALE - hf * SPLIT_SCALE, h2_);
}
// eight values (one B-operand octet): hi and lo halves as two h8
__device__ __forceinline__ void split8(const float (&v)[8], h8& hi, h8& lo) {
#pragma unroll
  for (int c = 0; c < 8; c += 2) {
    h2_ h, l;
    split2(f32x2_{v[c], v[c + 1]}, h, l);
    hi[c] = h[0];
    hi[c + 1] = h[1];
    lo[c] = l[0];
    lo[c + 1] = l[1];
  }
}

// split with a range check: `bad` collects operands outside the f16 range (and NaN)
__device__ __forceinline__ void split_dev(float v, _Float16& hi, _Float16& lo, bool& bad) {
  bad |= !(__builtin_fabsf(v) < F16_RANGE);
  split_fast(v, hi, lo);
}

// ---- packed epilogue forms for one MFMA output fragment (a lane's 4 consecutive rows of one
// column): v_pk_fma / v_pk_add / v_pk_mul / v_cvt_pk_f16_f32, half the VALU issues of the scalar
// forms and bit-identical to them (same operations in the same order per element)
// acc_main + 2^-11 acc_corr + bias
__device__ __forceinline__ f32x4 x3_value4(const f32x4& am, const f32x4& ac, const f32x4& b) {
  return am + ac * SPLIT_INV + b;
}
__device__ __forceinline__ f32x4 lrelu4(const f32x4& v) {
  const f32x4 s = v * 0.2f;
  return f32x4{fmaxf(v[0], s[0]), fmaxf(v[1], s[1]), fmaxf(v[2], s[2]), fmaxf(v[3], s[3])};
}
__device__ __forceinline__ void split4(const f32x4& v, h4& hi, h4& lo) {
  hi = __builtin_convertvector(v, h4);
  const f32x4 hf = __builtin_convertvector(hi, f32x4);
  lo = __builtin_convertvector(v * SPLIT_SCALE - hf * SPLIT_SCALE, h4);
}
// running maximum of |v| in place of a compare per value: GEMM outputs of finite, in-range
// operands are finite, so max < F16_RANGE at the end is the whole range check for them (inputs
// that may be NaN keep the ordered compare of split_dev / the staging check)
__device__ __forceinline__ float absmax4(float mx, const f32x4& v) {
  return fmaxf(fmaxf(mx, fmaxf(__builtin_fabsf(v[0]), __builtin_fabsf(v[1]))),
               fmaxf(__builtin_fabsf(v[2]), __builtin_fabsf(v[3])));
}
// LDS row swizzle of the position-major split-f16 tiles (resblock_x3 / resstack_x3): the 16-byte
// chunks of row r swap pairwise when bit 2 of r is set (an XOR of this value on the half offset
// within the row). Row strides there are 8 mod 16 dwords, which keeps the B-operand ds_read_b128 of
// 16 consecutive rows conflict-free with or without it; the swizzle takes the epilogues' 8-byte
// stores of 16 consecutive rows (banks mod 32) from 4-way to 2-way and the staging's 16-byte stores
// of 8 consecutive rows from 2-way to conflict-free. Every access of a tile's halves goes through
// it; offsets that are multiples of 16 halves (C, 2C, 32 ch) commute with the XOR.
__device__ __forceinline__ int lds_rsw(int r) {
#ifdef TTS_NO_LDS_SWZ  // A/B builds: the unswizzled layout
  return 0 * r;
#else
  return ((r >> 2) & 1) << 3;
#endif
}
#endif
