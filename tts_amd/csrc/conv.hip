// Generic fp32 MFMA Conv1d / polyphase ConvTranspose1d, and PQMF synthesis (gfx950).
//
// Replaces the ATen conv sequences of: ConvBNBlock (TTS/tts/layers/tacotron2.py:9-44),
// MelGAN generator convs (TTS/vocoder/models/melgan_generator.py:28-78),
// ResidualStack (TTS/vocoder/layers/melgan.py:5-39) and PQMF.synthesis
// (TTS/vocoder/layers/pqmf.py:51-56).
//
// Implicit GEMM: M = output channels, N = output time positions, K = Cin*taps.
// A (weights) is pre-swizzled into MFMA fragment order so every wave-load is one contiguous
// 1 KiB float4 read (L2-resident: the largest layer is 5 MB); B (activations) is staged per
// 16-channel chunk into LDS with padding / reflection / activation resolved at staging time,
// and read through a per-K offset table so dilation and taps cost no index math in the
// MFMA loop. v_mfma_f32_16x16x4_f32 keeps exact fp32 numerics.
#include "common.h"
#include <stdexcept>

__device__ __forceinline__ int map_pad_index(int i, int L, int mode, bool& valid) {
  if (i >= 0 && i < L) return i;
  if (mode == 0) {
    valid = false;
    return 0;
  }
  if (mode == 1) {  // torch ReflectionPad1d (edge not repeated)
    if (i < 0) i = -i;
    if (i >= L) i = 2 * (L - 1) - i;
  }
  return i < 0 ? 0 : (i >= L ? L - 1 : i);
}

template <int MI, int NI, int WM, int WN>
__global__ __launch_bounds__(256) void conv_mfma_kernel(ConvArgs a) {
  constexpr int TC = 16 * MI * WM;
  constexpr int TQ = 16 * NI * WN;
  static_assert(WM * WN == 4, "4 waves per workgroup");
  extern __shared__ __attribute__((aligned(16))) float smem[];

  const int ph = blockIdx.z % a.nphase;
  const int b = blockIdx.z / a.nphase;
  const int base = a.lens[b] + a.len_add;
  const int Lq = base * a.q_mul;
  const int q0 = blockIdx.x * TQ;
  if (q0 >= Lq) return;
  const int co0 = blockIdx.y * TC;
  const int Lin = base * a.in_mul;
  const int K = a.K, dil = a.dil;
  const int span = (K - 1) * dil;
  const int ROW = TQ + span + 1;
  float* X = smem;
  int* offs = reinterpret_cast<int*>(smem + ((16 * ROW + 3) & ~3));

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  for (int i = tid; i < 16 * K; i += 256) offs[i] = (i / K) * ROW + (i % K) * dil;

  const int i0 = q0 - a.pad_left[ph];
  const int nchunks = a.Cin / 16;
  const int nkc_total = a.Cin * K / 16;
  const f32x4* Wv = reinterpret_cast<const f32x4*>(a.W + (long)ph * a.w_phase_stride);
  const int mt0 = (co0 + wm * 16 * MI) / 16;
  const int qb = wn * 16 * NI + (lane & 15);
  const int g4 = 4 * (lane >> 4);
  const int rawL = a.lens[b];

  f32x4 acc[MI][NI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int chunk = 0; chunk < nchunks; ++chunk) {
    __syncthreads();
    {  // stage 16 channels x ROW positions
      const int cbase = chunk * 16;
      const ConvSrc& S = (cbase < a.src[0].C) ? a.src[0] : a.src[1];
      const int cs = (cbase < a.src[0].C) ? cbase : cbase - a.src[0].C;
      const float* sp = S.ptr + (long)b * S.sb;
      for (int c = wave * 4; c < wave * 4 + 4; ++c) {
        const float* rowp = sp + (long)(cs + c) * S.sc;
        for (int p = lane; p < ROW; p += 64) {
          float v = 0.f;
          if (p < TQ + span) {
            bool valid = true;
            int i = map_pad_index(i0 + p, Lin, a.pad_mode, valid);
            if (valid) {
              if (a.rep_pad) {
                i -= a.rep_pad;
                i = i < 0 ? 0 : (i >= rawL ? rawL - 1 : i);
              }
              v = rowp[(long)i * S.st];
              if (S.act) v = lrelu02(v);
            }
          }
          X[c * ROW + p] = v;
        }
      }
    }
    __syncthreads();
    for (int kq = 0; kq < K; ++kq) {
      const int kc = chunk * K + kq;
      f32x4 A[MI];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) A[mi] = Wv[((long)(mt0 + mi) * nkc_total + kc) * 64 + lane];
      const int4 o = *reinterpret_cast<const int4*>(offs + kq * 16 + g4);
      const int ov[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        float bv[NI];
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) bv[ni] = X[ov[s] + qb + ni * 16];
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni) acc[mi][ni] = MFMA16(A[mi][s], bv[ni], acc[mi][ni]);
      }
    }
  }

  // epilogue: bias, activation, optional residual, strided store
#pragma unroll
  for (int mi = 0; mi < MI; ++mi) {
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const int q = q0 + qb + ni * 16;
      if (q >= Lq) continue;
      const int t = q * a.out_mul + ph;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int co = co0 + wm * 16 * MI + mi * 16 + g4 + j;
        if (co >= a.Cout) continue;
        float v = acc[mi][ni][j] + a.bias[co];
        if (a.epi_act == 1) v = fmaxf(v, 0.f);
        else if (a.epi_act == 2) v = tanhf(v);
        if (a.resid) v += a.resid[(long)b * a.rb + (long)co * a.rc + (long)t * a.rt];
        a.out[(long)b * a.ob + (long)co * a.oc + (long)t * a.ot] = v;
      }
    }
  }
}

int conv_tile_tc(int tile) { return tile == TILE_64x64 ? 64 : (tile == TILE_32x128 ? 32 : 16); }
static int conv_tile_tq(int tile) { return tile == TILE_64x64 ? 64 : (tile == TILE_32x128 ? 128 : 256); }

int conv_tile_for_cout(int cout) {
  if (cout % 64 == 0) return TILE_64x64;
  if (cout % 32 == 0) return TILE_32x128;
  return TILE_16x256;
}

void launch_conv(const ConvArgs& a, int tile, hipStream_t s) {
  TTS_CHECK(a.Cin % 16 == 0, "conv: Cin must be a multiple of 16");
  TTS_CHECK(a.Cout_pad % conv_tile_tc(tile) == 0, "conv: Cout_pad / tile mismatch");
  TTS_CHECK(a.nphase >= 1 && a.nphase <= 8, "conv: nphase");
  if (a.max_q <= 0 || a.B <= 0) return;
  const int TQ = conv_tile_tq(tile);
  const int span = (a.K - 1) * a.dil;
  const int ROW = TQ + span + 1;
  const size_t lds = (size_t)(((16 * ROW + 3) & ~3) + 16 * a.K) * 4;
  TTS_CHECK(lds <= 64 * 1024, "conv: LDS tile too large");
  dim3 grid((a.max_q + TQ - 1) / TQ, a.Cout_pad / conv_tile_tc(tile), a.B * a.nphase);
  switch (tile) {
    case TILE_64x64: conv_mfma_kernel<2, 2, 2, 2><<<grid, 256, lds, s>>>(a); break;
    case TILE_32x128: conv_mfma_kernel<1, 4, 2, 2><<<grid, 256, lds, s>>>(a); break;
    default: conv_mfma_kernel<1, 4, 1, 4><<<grid, 256, lds, s>>>(a); break;
  }
  HIP_OK(hipGetLastError());
}

void swizzle_rows16(const float* Wm, int rows, int rows_pad, int Kdim, float* dst) {
  const int nkc = Kdim / 16;
  for (int m = 0; m < rows_pad / 16; ++m)
    for (int kc = 0; kc < nkc; ++kc)
      for (int l = 0; l < 64; ++l)
        for (int s = 0; s < 4; ++s) {
          const int r = m * 16 + (l & 15);
          const int k = kc * 16 + 4 * (l >> 4) + s;
          dst[(((size_t)m * nkc + kc) * 64 + l) * 4 + s] = r < rows ? Wm[(size_t)r * Kdim + k] : 0.f;
        }
}

// ------------------------------- PQMF synthesis --------------------------------------
// y[n] = sum_k sum_j G[k][j] * (N * x_k[(n + j - P) / N])  over (n + j - P) % N == 0,
// i.e. conv_transpose1d(x, N*I, stride N) followed by conv1d(G, padding P = taps/2).
__global__ __launch_bounds__(256) void pqmf_synth_kernel(const float* __restrict__ x, long xb, long xc,
                                                         const float* __restrict__ G, int N, int taps,
                                                         const int* lens, int len_add, int L_mul,
                                                         float* __restrict__ y, long yb) {
  __shared__ float g[8 * 128];
  const int b = blockIdx.y;
  const int L = (lens[b] + len_add) * L_mul;
  const int nt = taps + 1;
  for (int i = threadIdx.x; i < N * nt; i += blockDim.x) g[i] = G[i];
  __syncthreads();
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  const int NL = N * L;
  if (n >= NL) return;
  const int P = taps / 2;
  const float* xp = x + (long)b * xb;
  int j0 = (P - n) % N;
  if (j0 < 0) j0 += N;
  const float fN = (float)N;
  float acc = 0.f;
  for (int k = 0; k < N; ++k) {
    const float* xk = xp + (long)k * xc;
    for (int j = j0; j < nt; j += N) {
      const int m = n + j - P;
      if (m < 0 || m >= NL) continue;
      acc = fmaf(g[k * nt + j], fN * xk[m / N], acc);
    }
  }
  y[(long)b * yb + n] = acc;
}

void launch_pqmf_synthesis(const float* x, long xb, long xc, const float* G, int N, int taps, const int* lens,
                           int len_add, int L_mul, int maxL, int B, float* y, long yb, hipStream_t s) {
  TTS_CHECK(N * (taps + 1) <= 8 * 128, "pqmf: filter too large");
  if (maxL <= 0 || B <= 0) return;
  dim3 grid((N * maxL + 255) / 256, B);
  pqmf_synth_kernel<<<grid, 256, 0, s>>>(x, xb, xc, G, N, taps, lens, len_add, L_mul, y, yb);
  HIP_OK(hipGetLastError());
}
