// MB-MelGAN output stage fused with PQMF synthesis (gfx950):
//   bands = tanh(Conv1d(C -> 4, k7)(ReflectionPad1d(3)(LeakyReLU(x))))   melgan_generator.py:75-81
//   wav   = conv1d(conv_transpose1d(bands, 4 I, stride 4), G, pad = taps/2)  pqmf.py:51-56
// One workgroup (256 threads) produces OP_TB = 1008 band positions (4032 waveform samples) of
// one utterance. The k7 conv computes OP_NB = 1024 band positions (8 of halo each side for the
// 63-tap synthesis filter), four consecutive positions x four bands per thread in packed fp32
// FMAs (v_pk_fma_f32: band pairs x a broadcast input), so one thread's 12-value input window
// serves 112 FMAs per channel. Channels stream through LDS in chunks of OP_CC: chunk c+1 is
// loaded into registers (coalesced, clamped, unguarded) while chunk c is computed. The 4 x 1024
// band tile then reuses the chunk buffer and the polyphase synthesis reads it from there: output
// samples 4m..4m+3 share their 16 band values per band (taps 3-r+4jj), so a thread does four
// samples per band read with the taps as one broadcast 16-byte LDS read. Weights and biases are
// wave-uniform (scalar loads). The band tensor never reaches HBM.
#include "common.h"

namespace {
constexpr int OP_N = 4;                  // bands
constexpr int OP_NB = 1024;              // band positions computed per workgroup (4 per thread)
constexpr int OP_HB = 8;                 // band halo on the left (7 used) and right (8 used)
constexpr int OP_TB = OP_NB - 2 * OP_HB;  // 1008 band positions of output
constexpr int OP_XW = OP_NB + 8;          // staged input positions [p0 - 12, p0 + 1020)
constexpr int OP_CC = 8;                  // channels per staged chunk
constexpr int OP_TAPS = 63;
constexpr int OP_PER = (OP_CC * OP_XW + 255) / 256;  // staged floats per thread per chunk
typedef float f32x2 __attribute__((ext_vector_type(2)));

// fp32 FMA kept out of v_pk_fma_f32: packed, the synthesis loop broadcasts the band value from
// the high dword of a ds_read2 register pair (op_sel:[0,1,0]), and those low-half results were
// wrong (runs of 16 lanes, output phases 0 / 2) in 4 of 30 runs beside a persistent BiLSTM launch
// of another context (tools/race_probe.py, profiles/r06/v26_pqmf_opsel.txt)
__device__ __forceinline__ float fma_nopk(float a, float b, float c) {
  float d;
  asm("v_fma_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
}
}  // namespace

template <int C>
__global__ __launch_bounds__(256) void out_pqmf_kernel(const float* __restrict__ x, long xb, long xc,
                                                       const float* __restrict__ Wo, const float* __restrict__ bo,
                                                       const float* __restrict__ G, const int* __restrict__ lens,
                                                       int len_add, int L_mul, int maxL, float* __restrict__ y,
                                                       long yb) {
  static_assert(C % OP_CC == 0, "channel chunking");
  constexpr int NCH = C / OP_CC;
  // chunk buffer [OP_CC][OP_XW]; after the conv it holds the band tile [4][OP_NB]
  __shared__ __attribute__((aligned(16))) float Xs[OP_CC * OP_XW];
  __shared__ __attribute__((aligned(16))) float Gr[OP_N][16][4];  // Gr[k][jj][r] = G[k][4jj + 3 - r]
  static_assert(OP_N * OP_NB <= OP_CC * OP_XW, "band tile fits the chunk buffer");
  const int b = blockIdx.y;
  const int L = (lens[b] + len_add) * L_mul;  // band length of this utterance
  const int p0 = blockIdx.x * OP_TB;
  const int tid = threadIdx.x;
  if (p0 >= L) {  // a tile past the utterance: its samples are the row's zero padding
    float* yp = y + (long)b * yb;
    for (int m = p0 + tid; m < min(p0 + OP_TB, maxL); m += 256)
      *reinterpret_cast<f32x4*>(yp + 4L * m) = f32x4{0.f, 0.f, 0.f, 0.f};
    return;
  }
  const float* xp = x + (long)b * xb;
  for (int i = tid; i < OP_N * 64; i += 256) {
    const int k = i >> 6, jj = (i >> 2) & 15, r = i & 3;
    const int j = 4 * jj + 3 - r;
    Gr[k][jj][r] = j < OP_TAPS ? G[k * OP_TAPS + j] : 0.f;
  }
  // staged element e -> (channel e / XW, position p0 - 12 + e % XW), ReflectionPad1d(3) at the
  // utterance edges, clamped beyond (positions whose bands are outside [0, L) are zeroed below)
  int off[OP_PER];
#pragma unroll
  for (int r = 0; r < OP_PER; ++r) {
    const int e = min(tid + 256 * r, OP_CC * OP_XW - 1);
    const int c = e / OP_XW;
    int q = p0 - 12 + (e - c * OP_XW);
    if (q < 0) q = -q;
    if (q >= L) q = 2 * (L - 1) - q;
    q = min(max(q, 0), L - 1);
    off[r] = c * (int)xc + q;
  }
  float v[OP_PER];
#pragma unroll
  for (int r = 0; r < OP_PER; ++r) v[r] = xp[off[r]];
  f32x2 acc01[4], acc23[4];  // [position][band pair]
  {
    const f32x2 b01 = {bo[0], bo[1]}, b23 = {bo[2], bo[3]};
#pragma unroll
    for (int j = 0; j < 4; ++j) acc01[j] = b01, acc23[j] = b23;
  }
  for (int ch = 0; ch < NCH; ++ch) {
    if (ch > 0) lds_barrier();  // the previous chunk's reads are done
#pragma unroll
    for (int r = 0; r < OP_PER; ++r) {
      const int e = tid + 256 * r;
      if (r < OP_PER - 1 || e < OP_CC * OP_XW) Xs[e] = lrelu02(v[r]);
    }
    lds_barrier();
    {  // next chunk's loads (the last iteration re-reads its own chunk: unconditional loads)
      const long nb = (long)min(ch + 1, NCH - 1) * OP_CC * xc;
#pragma unroll
      for (int r = 0; r < OP_PER; ++r) v[r] = xp[nb + off[r]];
    }
    const float* wc = Wo + (long)ch * OP_CC * 28;
#pragma unroll 2
    for (int c = 0; c < OP_CC; ++c) {
      const f32x4* xr = reinterpret_cast<const f32x4*>(Xs + c * OP_XW + 4 * tid);
      const f32x4 x0 = xr[0], x1 = xr[1], x2 = xr[2];
      const float xw[12] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3], x2[0], x2[1], x2[2], x2[3]};
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        const f32x2 w01 = {wc[c * 28 + 4 * k + 0], wc[c * 28 + 4 * k + 1]};
        const f32x2 w23 = {wc[c * 28 + 4 * k + 2], wc[c * 28 + 4 * k + 3]};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float xv = xw[1 + j + k];  // input position (p0 - 8 + 4 tid + j) - 3 + k
          const f32x2 xx = {xv, xv};
          acc01[j] = w01 * xx + acc01[j];
          acc23[j] = w23 * xx + acc23[j];
        }
      }
    }
  }
  lds_barrier();  // all chunk reads done: Xs becomes the band tile Bs[band][OP_NB]
  float* Bs = Xs;
  {
    f32x4 o[OP_N];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = p0 - OP_HB + 4 * tid + j;
      const bool valid = p >= 0 && p < L;  // the synthesis conv zero-pads outside the utterance
      o[0][j] = valid ? tanhf(acc01[j][0]) : 0.f;
      o[1][j] = valid ? tanhf(acc01[j][1]) : 0.f;
      o[2][j] = valid ? tanhf(acc23[j][0]) : 0.f;
      o[3][j] = valid ? tanhf(acc23[j][1]) : 0.f;
    }
#pragma unroll
    for (int k = 0; k < OP_N; ++k) *reinterpret_cast<f32x4*>(Bs + k * OP_NB + 4 * tid) = o[k];
  }
  lds_barrier();
  // y[4m + r] = 4 sum_k sum_jj G[k][4jj + 3 - r] bands_k[m + jj - 7]   (pqmf.py:51-56 restated)
  f32x4 out[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) out[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < OP_N; ++k) {
#pragma unroll 4
    for (int jj = 0; jj < 16; ++jj) {
      const f32x4 g = *reinterpret_cast<const f32x4*>(&Gr[k][jj][0]);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int mm = min(tid + 256 * i, OP_TB - 1);  // local band position of the output quad
        const float bv = Bs[k * OP_NB + mm + 1 + jj];
#pragma unroll
        for (int r = 0; r < 4; ++r) out[i][r] = fma_nopk(g[r], bv, out[i][r]);
      }
    }
  }
  float* yp = y + (long)b * yb;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int mm = tid + 256 * i;
    const int m = p0 + mm;
    if (mm < OP_TB && m < maxL)  // zeros past the utterance (the row is padded to maxL)
      *reinterpret_cast<f32x4*>(yp + 4L * m) = m < L ? (float)OP_N * out[i] : f32x4{0.f, 0.f, 0.f, 0.f};
  }
}

bool launch_out_pqmf(const float* x, long xb, long xc, int C, const float* Wo, const float* bo, const float* G,
                     int N, int taps, const int* lens, int len_add, int L_mul, int maxL, int B, float* y, long yb,
                     hipStream_t s) {
  if (N != OP_N || taps + 1 != OP_TAPS) return false;
  if (maxL <= 0 || B <= 0) return true;
  if (yb % 4 != 0 || (reinterpret_cast<uintptr_t>(y) & 15) != 0) return false;  // float4 output stores
  if ((long)C * xc >= (1L << 31)) return false;                                  // 32-bit staging offsets
  dim3 grid((maxL + OP_TB - 1) / OP_TB, B);
  switch (C) {
    case 48: out_pqmf_kernel<48><<<grid, 256, 0, s>>>(x, xb, xc, Wo, bo, G, lens, len_add, L_mul, maxL, y, yb); break;
    case 32: out_pqmf_kernel<32><<<grid, 256, 0, s>>>(x, xb, xc, Wo, bo, G, lens, len_add, L_mul, maxL, y, yb); break;
    default: return false;
  }
  HIP_OK(hipGetLastError());
  return true;
}

// Full-band MelGAN output stage (round 4): y = tanh(Conv1d(C -> 1, k7)(ReflectionPad1d(3)(LeakyReLU(x))))
// (melgan_generator.py:75-81) on the VALU. The generic MFMA conv pads the single output channel to
// a 16-row tile (16x the work, ~430 us at 2.35 M positions); here a thread makes OC1_P consecutive
// positions from an (OC1_P + 8)-value window per channel (16-byte loads away from the utterance
// ends, where ReflectionPad1d needs per-element indices), weights [c][k] wave-uniform.
constexpr int OC1_P = 16;

__global__ __launch_bounds__(256) void out_conv1_kernel(const float* __restrict__ x, long xb, long xc, int C,
                                                        const float* __restrict__ W, const float* __restrict__ bo,
                                                        const int* __restrict__ lens, int len_add, int L_mul,
                                                        float* __restrict__ y, long yb, int vec) {
  constexpr int P = OC1_P, NV = P + 8;
  const int b = blockIdx.y;
  const int L = (lens[b] + len_add) * L_mul;
  const int t0 = (blockIdx.x * 256 + threadIdx.x) * P;
  if (t0 >= L) return;
  const float* xr = x + b * xb;
  const float b0 = bo[0];
  float acc[P];
#pragma unroll
  for (int j = 0; j < P; ++j) acc[j] = b0;
  if (vec && t0 >= 4 && t0 + P + 4 <= L) {
    // v[i] = x[t0 - 4 + i]; position t0 + j, tap k reads x[t0 + j + k - 3] = v[j + k + 1]
    for (int c = 0; c < C; ++c) {
      const float4* p = reinterpret_cast<const float4*>(xr + (long)c * xc + t0 - 4);
      float v[NV];
#pragma unroll
      for (int i = 0; i < NV / 4; ++i) {
        const float4 q = p[i];
        v[4 * i] = lrelu02(q.x);
        v[4 * i + 1] = lrelu02(q.y);
        v[4 * i + 2] = lrelu02(q.z);
        v[4 * i + 3] = lrelu02(q.w);
      }
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        const float w = W[c * 7 + k];
#pragma unroll
        for (int j = 0; j < P; ++j) acc[j] = fmaf(w, v[j + k + 1], acc[j]);
      }
    }
  } else {
    int idx[P + 6];
#pragma unroll
    for (int i = 0; i < P + 6; ++i) {  // ReflectionPad1d(3), then clamped (positions past L are never stored)
      int p = t0 - 3 + i;
      if (p < 0) p = -p;
      if (p >= L) p = 2 * (L - 1) - p;
      idx[i] = p < 0 ? 0 : (p >= L ? L - 1 : p);
    }
    for (int c = 0; c < C; ++c) {
      const float* xc_ = xr + (long)c * xc;
      float v[P + 6];
#pragma unroll
      for (int i = 0; i < P + 6; ++i) v[i] = lrelu02(xc_[idx[i]]);
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        const float w = W[c * 7 + k];
#pragma unroll
        for (int j = 0; j < P; ++j) acc[j] = fmaf(w, v[j + k], acc[j]);
      }
    }
  }
  float* yr = y + b * yb + t0;
  if (vec && t0 + P <= L) {
#pragma unroll
    for (int j = 0; j < P; j += 4)
      *reinterpret_cast<float4*>(yr + j) = make_float4(tanhf(acc[j]), tanhf(acc[j + 1]), tanhf(acc[j + 2]), tanhf(acc[j + 3]));
  } else {
#pragma unroll
    for (int j = 0; j < P; ++j)
      if (t0 + j < L) yr[j] = tanhf(acc[j]);
  }
}

void launch_out_conv1(const float* x, long xb, long xc, int C, const float* W, const float* bo, const int* lens,
                      int len_add, int L_mul, int maxL, int B, float* y, long yb, hipStream_t s) {
  if (maxL <= 0 || B <= 0) return;
  const int vec = (reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(y) & 15) == 0 &&
                  xb % 4 == 0 && xc % 4 == 0 && yb % 4 == 0;
  const int per = 256 * OC1_P;
  out_conv1_kernel<<<dim3((maxL + per - 1) / per, B), 256, 0, s>>>(x, xb, xc, C, W, bo, lens, len_add, L_mul, y, yb,
                                                                    vec);
  HIP_OK(hipGetLastError());
}
