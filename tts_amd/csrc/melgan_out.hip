// MB-MelGAN output stage fused with PQMF synthesis (gfx950):
//   bands = tanh(Conv1d(C -> 4, k7)(ReflectionPad1d(3)(LeakyReLU(x))))   melgan_generator.py:75-81
//   wav   = conv1d(conv_transpose1d(bands, 4 I, stride 4), G, pad = taps/2)  pqmf.py:51-56
// One workgroup produces TOUT = 960 waveform samples of one utterance. It stages the C input
// channels it needs (240 band positions + 8 each side for the 63-tap synthesis filter + 3 each
// side for the k7 conv) once in LDS, computes the 256 band positions x 4 bands on the VALU (4
// outputs per thread: M = 4 would waste 3/4 of a 16-wide MFMA tile), keeps them in LDS, and
// runs the polyphase synthesis from there. Versus the generic conv + a separate PQMF launch this
// removes the band tensor round trip and the padded-to-16 output tile.
#include "common.h"

namespace {
constexpr int OP_N = 4;                 // bands
constexpr int OP_NB = 256;              // band positions per workgroup (one per thread)
constexpr int OP_HB = 8;                // band halo each side (31 filter taps / 4, rounded up)
constexpr int OP_TB = OP_NB - 2 * OP_HB;  // 240 band positions of output
constexpr int OP_TOUT = OP_N * OP_TB;     // 960 waveform samples
constexpr int OP_NX = OP_NB + 6;          // input positions incl. the k7 halo
constexpr int OP_XLD = OP_NX + 1;         // LDS row stride
constexpr int OP_TAPS = 63;
}  // namespace

template <int C>
__global__ __launch_bounds__(256) void out_pqmf_kernel(const float* __restrict__ x, long xb, long xc,
                                                       const float* __restrict__ Wo, const float* __restrict__ bo,
                                                       const float* __restrict__ G, const int* lens, int len_add,
                                                       int L_mul, float* __restrict__ y, long yb) {
  __shared__ float Xs[C * OP_XLD];
  __shared__ __attribute__((aligned(16))) float Ws[C * 7 * 4];  // [c][k][o]
  __shared__ float Bs[OP_N][OP_NB];
  __shared__ float Gs[OP_N][OP_TAPS + 1];
  const int b = blockIdx.y;
  const int L = (lens[b] + len_add) * L_mul;  // band length of this utterance
  const int n0 = blockIdx.x * OP_TOUT;
  if (n0 >= OP_N * L) return;
  const int tid = threadIdx.x;
  const int p0 = n0 / OP_N - OP_HB;  // first band position held in Bs
  const float* xp = x + (long)b * xb;
  for (int i = tid; i < C * 7 * 4; i += 256) Ws[i] = Wo[i];
  for (int i = tid; i < OP_N * OP_TAPS; i += 256) Gs[i / OP_TAPS][i % OP_TAPS] = G[i];
  // input window [p0 - 3, p0 + NB + 3): ReflectionPad1d(3) at the utterance edges; positions a
  // band outside [0, L) would use are clamped (those bands are forced to zero below). All loads
  // of the window are issued before the first LDS store (clamped element index, no guards).
  constexpr int PER = (C * OP_NX + 255) / 256;
  float v[PER];
#pragma unroll
  for (int r = 0; r < PER; ++r) {
    const int e = min(tid + 256 * r, C * OP_NX - 1);
    const int c = e / OP_NX, i = e - c * OP_NX;
    int q = p0 - 3 + i;
    if (q < 0) q = -q;
    if (q >= L) q = 2 * (L - 1) - q;
    q = min(max(q, 0), L - 1);
    v[r] = xp[(long)c * xc + q];
  }
#pragma unroll
  for (int r = 0; r < PER; ++r) {
    const int e = tid + 256 * r;
    if (e < C * OP_NX) {
      const int c = e / OP_NX, i = e - c * OP_NX;
      Xs[c * OP_XLD + i] = lrelu02(v[r]);
    }
  }
  __syncthreads();
  {
    const int j = tid;  // band position p0 + j
    float a0 = bo[0], a1 = bo[1], a2 = bo[2], a3 = bo[3];
#pragma unroll 4
    for (int c = 0; c < C; ++c) {
      const float* xr = Xs + c * OP_XLD + j;
      const f32x4* wr = reinterpret_cast<const f32x4*>(Ws + c * 28);
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        const float xv = xr[k];
        const f32x4 w = wr[k];
        a0 = fmaf(w[0], xv, a0);
        a1 = fmaf(w[1], xv, a1);
        a2 = fmaf(w[2], xv, a2);
        a3 = fmaf(w[3], xv, a3);
      }
    }
    const int p = p0 + j;
    const bool valid = p >= 0 && p < L;  // the synthesis conv zero-pads outside the utterance
    Bs[0][j] = valid ? tanhf(a0) : 0.f;
    Bs[1][j] = valid ? tanhf(a1) : 0.f;
    Bs[2][j] = valid ? tanhf(a2) : 0.f;
    Bs[3][j] = valid ? tanhf(a3) : 0.f;
  }
  __syncthreads();
  // y[n] = sum_k sum_j G[k][j] * 4 * bands_k[(n + j - 31) / 4]   over j with n + j - 31 = 0 (mod 4)
  constexpr int P = OP_TAPS / 2;
  float* yp = y + (long)b * yb;
  for (int t = tid; t < OP_TOUT; t += 256) {
    const int n = n0 + t;
    if (n >= OP_N * L) break;
    const int j0 = (P - t) & (OP_N - 1);  // (P - n) mod 4; n0 is a multiple of 4
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < OP_N; ++k) {
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) {
        const int j = j0 + OP_N * jj;
        if (j < OP_TAPS) acc = fmaf(Gs[k][j], Bs[k][(t + j - P) / OP_N + OP_HB], acc);
      }
    }
    yp[n] = (float)OP_N * acc;
  }
}

bool launch_out_pqmf(const float* x, long xb, long xc, int C, const float* Wo, const float* bo, const float* G,
                     int N, int taps, const int* lens, int len_add, int L_mul, int maxL, int B, float* y, long yb,
                     hipStream_t s) {
  if (N != OP_N || taps + 1 != OP_TAPS) return false;
  if (maxL <= 0 || B <= 0) return true;
  dim3 grid((OP_N * maxL + OP_TOUT - 1) / OP_TOUT, B);
  switch (C) {
    case 48: out_pqmf_kernel<48><<<grid, 256, 0, s>>>(x, xb, xc, Wo, bo, G, lens, len_add, L_mul, y, yb); break;
    case 32: out_pqmf_kernel<32><<<grid, 256, 0, s>>>(x, xb, xc, Wo, bo, G, lens, len_add, L_mul, y, yb); break;
    default: return false;
  }
  HIP_OK(hipGetLastError());
  return true;
}
