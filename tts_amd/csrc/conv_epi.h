// Shared pieces of the generic conv kernels (conv.hip: fp32 MFMA, conv_x3.hip: split-f16 MFMA):
// index mapping of the padded input and the epilogue (bias, activation, pair / coupling forms,
// residual, strided store) applied to a wave's MI x NI 16x16 accumulator tiles.
#pragma once
#include "common.h"

constexpr int CONV_MAX_SPAN = 7;  // (K-1)*dil of the generic kernels (k <= 7, dilation 1)

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

// acc[mi][ni]: rows co0 + wm*16*MI + mi*16 + 4*(lane>>4) + j, columns (positions per phase)
// q0 + wn*16*NI + ni*16 + (lane&15) -- the 16x16 MFMA D layout
template <int MI, int NI, int WN>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a, f32x4 (&acc)[MI][NI], int b, int ph, int q0,
                                              int co0, int wm, int wn, int lane) {
  const int base = a.lens[b] + a.len_add;
  const int Lq = base * a.q_mul;
  const int qb = wn * 16 * NI + (lane & 15);
  const int g4 = 4 * (lane >> 4);
  // epilogue: bias, activation, optional residual, strided store
#pragma unroll
  for (int mi = 0; mi < MI; ++mi) {
    float bias4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int co = min(co0 + wm * 16 * MI + mi * 16 + g4 + j, a.Cout - 1);
      bias4[j] = a.bias[co];
    }
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      const int q = q0 + qb + ni * 16;
      if (q >= Lq) continue;
      const int t = q * a.out_mul + ph;
      if (a.epi_act == 5) {
        // coupling reverse for x1 channels (2m, 2m + 1), then the reverse InvConvNear (4 x 4 over
        // {x0[2m], x0[2m+1], x1[2m], x1[2m+1]}, glow.py:184-201) and ActNorm (glow.py:48-58):
        // the lane's 4 rows hold exactly one mixing group; resid = x, out = next x
        const int co = co0 + wm * 16 * MI + mi * 16 + g4;
        if (co >= a.Cout) continue;
        const int m2 = co >> 1, Ch = a.Cout >> 1;
        const float* xs = a.resid + (long)b * a.rb + (long)t * a.rt;
        float in[4];
        in[0] = xs[(long)m2 * a.rc];
        in[1] = xs[(long)(m2 + 1) * a.rc];
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const float u = acc[mi][ni][2 * p] + bias4[2 * p], g = acc[mi][ni][2 * p + 1] + bias4[2 * p + 1];
          in[2 + p] = (xs[(long)(Ch + m2 + p) * a.rc] - u) * expf(-g);
        }
        float* os = a.out + (long)b * a.ob + (long)t * a.ot;
#pragma unroll
        for (int o = 0; o < 4; ++o) {
          const int c = (o < 2 ? 0 : Ch) + m2 + (o & 1);
          const float* w = a.aux + c * 6;
          float v = w[0] * in[0];
          v = fmaf(w[1], in[1], v);
          v = fmaf(w[2], in[2], v);
          v = fmaf(w[3], in[3], v);
          os[(long)c * a.oc] = (v - w[4]) * w[5];
        }
        continue;
      }
      if (a.epi_act >= 3) {
        // row pairs (2c, 2c + 1) -> output channel c (weights interleaved at pack time):
        // 3 = WN gate tanh(u) * sigmoid(g); 4 = coupling reverse (resid - m) * exp(-logs)
#pragma unroll
        for (int j = 0; j < 4; j += 2) {
          const int co = co0 + wm * 16 * MI + mi * 16 + g4 + j;
          if (co >= a.Cout) continue;
          const int c = co >> 1;
          float u = acc[mi][ni][j] + bias4[j], g = acc[mi][ni][j + 1] + bias4[j + 1];
          if (a.epi_act == 3 && a.aux) {  // glow.py:125-131: x_in + g_l before the gate
            u += a.aux[(long)b * a.auxb + co];
            g += a.aux[(long)b * a.auxb + co + 1];
          }
          float v;
          if (a.epi_act == 3) v = tanhf(u) / (1.f + expf(-g));
          else if (a.epi_act == 6) v = u / (1.f + expf(-g));  // GLU
          else v = (a.resid[(long)b * a.rb + (long)c * a.rc + (long)t * a.rt] - u) * expf(-g);
          a.out[(long)b * a.ob + (long)c * a.oc + (long)t * a.ot] = v;
        }
        continue;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int co = co0 + wm * 16 * MI + mi * 16 + g4 + j;
        if (co >= a.Cout) continue;
        float v = acc[mi][ni][j] + bias4[j];
        if (a.epi_act == 1) v = fmaxf(v, 0.f);
        else if (a.epi_act == 2) v = tanhf(v);
        if (a.resid && (a.resid_rows == 0 || co < a.resid_rows))
          v += a.resid[(long)b * a.rb + (long)co * a.rc + (long)t * a.rt];
        a.out[(long)b * a.ob + (long)co * a.oc + (long)t * a.ot] = v;
      }
    }
  }
}
