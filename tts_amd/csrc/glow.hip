// Glow-TTS inference pieces that are not convolutions (gfx950), SURVEY.md §8f rank 3:
//   TTS/tts/layers/glow_tts/{gated_conv,normalization,duration_predictor,glow,decoder}.py and the
//   inference glue of TTS/tts/models/glow_tts.py:170-193 (durations -> monotonic path -> expanded
//   means + noise). Activations are channel-major (B, C, T); lanes run along time, so every channel
//   step is one coalesced row access per wave, and the 4 waves of a workgroup split the channels.
//   The WN gate and the coupling reverse are conv epilogues (conv.hip, epi 3 / 4). Only
//   positions t < length are written: the convolutions (conv.hip) read positions >= length as zero
//   padding, which is what the reference's masks produce.
#include "common.h"

// LayerNorm over the channel dim (normalization.py:4-27, eps 1e-4). A workgroup owns 64 time
// positions (one per lane, coalesced rows) x 4 channel groups (one per wave); the column's values
// stay in registers (NPT per thread) and the mean / variance partials meet in LDS.
//   GLU:  GatedConvBlock (gated_conv.py:31-42): out = res + a * sigmoid(g), [a | g] = LN(x), wave w
//         holds a-channels [w*NPT/2, (w+1)*NPT/2) and the matching g-channels (C2 = 4 * NPT)
//   !GLU: in-place LN (DurationPredictor norm_1 / norm_2 after the conv's ReLU), C = 4 * NPT
template <int NPT, bool GLU, bool RELU = false>
__global__ __launch_bounds__(256) void ln_chan_kernel(const float* x, long xb, const float* __restrict__ gamma,
                                                      const float* __restrict__ beta, const float* res, long rb,
                                                      float* out, long ob, const int* lens, int T) {
  constexpr int CN = 4 * NPT, HALF = NPT / 2;
  __shared__ float part[2][4][64];
  const int b = blockIdx.y, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int t = blockIdx.x * 64 + lane;
  const bool valid = t < T && t < lens[b];
  const float* xp = x + b * xb + (valid ? t : 0);
  auto chan = [&](int i) { return GLU ? (i < HALF ? w * HALF + i : CN / 2 + w * HALF + i - HALF) : w * NPT + i; };
  float v[NPT];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    v[i] = valid ? xp[(long)chan(i) * T] : 0.f;
    s += v[i];
  }
  part[0][w][lane] = s;
  __syncthreads();
  const float mean = (part[0][0][lane] + part[0][1][lane] + part[0][2][lane] + part[0][3][lane]) / (float)CN;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    const float d = v[i] - mean;
    q = fmaf(d, d, q);
  }
  part[1][w][lane] = q;
  __syncthreads();
  const float var = (part[1][0][lane] + part[1][1][lane] + part[1][2][lane] + part[1][3][lane]) / (float)CN;
  if (!valid) return;
  const float rs = rsqrtf(var + 1e-4f);
  if constexpr (GLU) {
#pragma unroll
    for (int i = 0; i < HALF; ++i) {
      const int ca = chan(i), cg = chan(i + HALF);
      const float a = (v[i] - mean) * rs * gamma[ca] + beta[ca];
      const float g = (v[i + HALF] - mean) * rs * gamma[cg] + beta[cg];
      out[b * ob + (long)ca * T + t] = res[b * rb + (long)ca * T + t] + a / (1.f + expf(-g));
    }
  } else {
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const int c = chan(i);
      const float y = (v[i] - mean) * rs * gamma[c] + beta[c];
      out[b * ob + (long)c * T + t] = RELU ? fmaxf(y, 0.f) : y;
    }
  }
}

// glow_tts.py:172-176: w = (exp(logw) - 1) * x_mask * length_scale, w_ceil = ceil(w),
// y_length = max(sum w_ceil, 1); cum = cumsum(w_ceil) (generate_path, monotonic_align:15-32);
// o_attn_dur = log(1 + sum_j path[t, j]) * x_mask. One workgroup (one wave) per utterance.
__global__ __launch_bounds__(64) void glow_durations_kernel(const float* __restrict__ logw, int T, const int* lens,
                                                            float length_scale, float* __restrict__ cum,
                                                            int* __restrict__ ylen, float* __restrict__ wceil_out) {
  const int b = blockIdx.x;
  if (threadIdx.x != 0) return;
  const int L = lens[b];
  float c = 0.f;
  for (int t = 0; t < T; ++t) {
    float w = 0.f;
    if (t < L) w = ceilf((expf(logw[(long)b * T + t]) - 1.f) * length_scale);
    wceil_out[(long)b * T + t] = w;
    c += w;
    cum[(long)b * T + t] = c;
  }
  ylen[b] = max((int)c, 1);  // clamp_min(sum, 1).long()
}

// path[t, j] = [j < cum_t] - [j < cum_{t-1}] (generate_path), masked by t < x_len, j < y_len.
// cum is not monotonic in general: with length_scale > 1 a token's ceil((exp(logw) - 1) * scale)
// can be -1, and the reference's path then holds -1 entries; so every (j, t) pair is evaluated
// (no search for a single t_j). y_mean[c, j] = sum_t path[t, j] o_mean[c, t]; z = (y_mean +
// noise * noise_scale) * y_mask (mean_only: y_log_scale = 0, glow_tts.py:184-186). A workgroup owns
// 64 frames: 4 threads per frame (a quarter of the channels each) accumulate over the nonzero
// path entries, then the 64 attn rows (B, T_y, T_x) are written with lanes along t.
__device__ __forceinline__ float glow_path(const float* cb, int t, int j, int xl, int yl) {
  if (t >= xl || j >= yl) return 0.f;
  const float jf = (float)j;
  return (jf < cb[t] ? 1.f : 0.f) - (t > 0 && jf < cb[t - 1] ? 1.f : 0.f);
}

__global__ __launch_bounds__(256) void glow_expand_kernel(const float* __restrict__ o_mean, int C, int Tx,
                                                          const int* xlens, const float* __restrict__ cum,
                                                          const int* ylens, int Ty, const float* noise,
                                                          float noise_scale, float* __restrict__ y_mean,
                                                          float* __restrict__ z, float* __restrict__ attn) {
  constexpr int CQ = 20;  // channels per thread (C = 80 = 4 x 20)
  const int b = blockIdx.y, j0 = blockIdx.x * 64, tid = threadIdx.x;
  const int xl = xlens[b], yl = ylens[b];
  const float* cb = cum + (long)b * Tx;
  {
    const int jj = tid & 63, q = tid >> 6, j = j0 + jj;
    if (j < Ty) {
      float acc[CQ];
#pragma unroll
      for (int i = 0; i < CQ; ++i) acc[i] = 0.f;
      for (int t = 0; t < xl; ++t) {
        const float p = glow_path(cb, t, j, xl, yl);
        if (p != 0.f) {
#pragma unroll
          for (int i = 0; i < CQ; ++i) acc[i] = fmaf(p, o_mean[((long)b * C + q * CQ + i) * Tx + t], acc[i]);
        }
      }
      const bool yv = j < yl;
#pragma unroll
      for (int i = 0; i < CQ; ++i) {
        const long ix = ((long)b * C + q * CQ + i) * Ty + j;
        y_mean[ix] = acc[i];
        const float nz = noise ? noise[ix] * noise_scale : 0.f;
        z[ix] = yv ? acc[i] + nz : 0.f;
      }
    }
  }
  const int nj = min(64, Ty - j0);
  for (int r = 0; r < nj; ++r) {
    float* arow = attn + ((long)b * Ty + j0 + r) * Tx;
    for (int t = tid; t < Tx; t += 256) arow[t] = glow_path(cb, t, j0 + r, xl, yl);
  }
}

// decoder.py:6-19: (B, C, T) -> (B, 2C, T/2), x_sqz[s*C + c][k] = x[c][2k + s], masked by
// y_mask[2k + 1]; unsqueeze (decoder.py:22-33) is the inverse, masked by the repeated mask.
// 64 positions x 4 channel groups per workgroup.
__global__ __launch_bounds__(256) void glow_squeeze_kernel(const float* __restrict__ x, int C, int T,
                                                           const int* ylens, float* __restrict__ y, int K) {
  const int b = blockIdx.y, k = blockIdx.x * 64 + (threadIdx.x & 63);
  if (k >= K) return;
  const bool v = 2 * k + 1 < ylens[b];
  for (int sc = threadIdx.x >> 6; sc < 2 * C; sc += 4) {
    const int s = sc / C, c = sc % C;
    y[((long)b * 2 * C + sc) * K + k] = v ? x[((long)b * C + c) * T + 2 * k + s] : 0.f;
  }
}
__global__ __launch_bounds__(256) void glow_unsqueeze_kernel(const float* __restrict__ x, int C2, int K,
                                                             const int* ylens, float* __restrict__ y, int T) {
  const int b = blockIdx.y, k = blockIdx.x * 64 + (threadIdx.x & 63);
  if (k >= K) return;
  const int C = C2 / 2;
  const bool v = 2 * k + 1 < ylens[b];
  for (int c = threadIdx.x >> 6; c < C; c += 4) {
    float2 o;
    o.x = v ? x[((long)b * C2 + c) * K + k] : 0.f;
    o.y = v ? x[((long)b * C2 + C + c) * K + k] : 0.f;
    *reinterpret_cast<float2*>(y + ((long)b * C + c) * T + 2 * k) = o;
  }
}

void launch_glu_ln_res(const float* x, long xb, int C2, const float* gamma, const float* beta, const float* res,
                       long rb, float* out, long ob, const int* lens, int B, int T, hipStream_t s) {
  TTS_CHECK(C2 == 384, "glow encoder LayerNorm: 2 * hidden must be 384");
  ln_chan_kernel<96, true><<<dim3((T + 63) / 64, B), 256, 0, s>>>(x, xb, gamma, beta, res, rb, out, ob, lens, T);
  HIP_OK(hipGetLastError());
}
void launch_ln(float* x, long xb, int C, const float* gamma, const float* beta, const int* lens, int B, int T,
               hipStream_t s, bool relu) {
  const dim3 grid((T + 63) / 64, B);
  if (C == 256 && !relu) ln_chan_kernel<64, false><<<grid, 256, 0, s>>>(x, xb, gamma, beta, nullptr, 0, x, xb, lens, T);
  else if (C == 192 && relu)
    ln_chan_kernel<48, false, true><<<grid, 256, 0, s>>>(x, xb, gamma, beta, nullptr, 0, x, xb, lens, T);
  else if (C == 192) ln_chan_kernel<48, false><<<grid, 256, 0, s>>>(x, xb, gamma, beta, nullptr, 0, x, xb, lens, T);
  else TTS_CHECK(false, "glow LayerNorm: unsupported channel count");
  HIP_OK(hipGetLastError());
}

// TimeDepthSeparableConv middle (time_depth_sep_conv.py:51-58): depthwise k5 conv (zero padding at
// the utterance's own length, as a B = 1 call sees it) with BatchNorm folded into w / bias, then
// x * sigmoid(x). 64 positions x 4 channel groups per workgroup.
__global__ __launch_bounds__(256) void tds_depthwise_kernel(const float* __restrict__ x, int C, int T,
                                                            const float* __restrict__ w,
                                                            const float* __restrict__ bias, const int* lens,
                                                            float* __restrict__ y) {
  const int b = blockIdx.y, t = blockIdx.x * 64 + (threadIdx.x & 63);
  const int L = lens[b];
  if (t >= T || t >= L) return;
  for (int c = threadIdx.x >> 6; c < C; c += 4) {
    const float* xp = x + ((long)b * C + c) * T;
    float acc = bias[c];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int u = t + k - 2;
      if (u >= 0 && u < L) acc = fmaf(w[c * 5 + k], xp[u], acc);
    }
    y[((long)b * C + c) * T + t] = acc / (1.f + expf(-acc));
  }
}
void launch_tds_depthwise(const float* x, int C, int T, const float* w, const float* bias, const int* lens, float* y,
                          int B, hipStream_t s) {
  tds_depthwise_kernel<<<dim3((T + 63) / 64, B), 256, 0, s>>>(x, C, T, w, bias, lens, y);
  HIP_OK(hipGetLastError());
}
void launch_glow_durations(const float* logw, int T, const int* lens, float length_scale, float* cum, int* ylen,
                           float* wceil, int B, hipStream_t s) {
  glow_durations_kernel<<<B, 64, 0, s>>>(logw, T, lens, length_scale, cum, ylen, wceil);
  HIP_OK(hipGetLastError());
}
void launch_glow_expand(const float* o_mean, int C, int Tx, const int* xlens, const float* cum, const int* ylens,
                        int Ty, const float* noise, float noise_scale, float* y_mean, float* z, float* attn, int B,
                        hipStream_t s) {
  TTS_CHECK(C == 80, "glow: 80 mel channels");
  glow_expand_kernel<<<dim3((Ty + 63) / 64, B), 256, 0, s>>>(o_mean, C, Tx, xlens, cum, ylens, Ty, noise,
                                                                noise_scale, y_mean, z, attn);
  HIP_OK(hipGetLastError());
}
void launch_glow_squeeze(const float* x, int C, int T, const int* ylens, float* y, int K, int B, hipStream_t s) {
  glow_squeeze_kernel<<<dim3((K + 63) / 64, B), 256, 0, s>>>(x, C, T, ylens, y, K);
  HIP_OK(hipGetLastError());
}
void launch_glow_unsqueeze(const float* x, int C2, int K, const int* ylens, float* y, int T, int B, hipStream_t s) {
  glow_unsqueeze_kernel<<<dim3((K + 63) / 64, B), 256, 0, s>>>(x, C2, K, ylens, y, T);
  HIP_OK(hipGetLastError());
}
// g = F.normalize(emb_g(speaker)) (glow_tts.py:159-161): x / max(||x||_2, 1e-12), one workgroup per
// utterance, written as (B, c_pad) with zeros in the padding channels [c_in, c_pad)
__global__ __launch_bounds__(256) void glow_speaker_kernel(const int* __restrict__ spk, const float* __restrict__ table,
                                                           int c_in, int c_pad, float* __restrict__ g) {
  __shared__ float part[4];
  const int b = blockIdx.x, tid = threadIdx.x;
  const float* row = table + (long)spk[b] * c_in;
  float ss = 0.f;
  for (int j = tid; j < c_in; j += 256) ss = fmaf(row[j], row[j], ss);
  for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
  if ((tid & 63) == 0) part[tid >> 6] = ss;
  __syncthreads();
  const float n = fmaxf(sqrtf(part[0] + part[1] + part[2] + part[3]), 1e-12f);
  for (int j = tid; j < c_pad; j += 256) g[(long)b * c_pad + j] = j < c_in ? row[j] / n : 0.f;
}
void launch_glow_speaker(const int* spk, const float* table, int c_in, int c_pad, float* g, int B, hipStream_t s) {
  glow_speaker_kernel<<<B, 256, 0, s>>>(spk, table, c_in, c_pad, g);
  HIP_OK(hipGetLastError());
}

// encoder.py:107: emb(x) * sqrt(hidden) (the scale is folded into the table), channel-major out
__global__ __launch_bounds__(256) void glow_embed_kernel(const int64_t* __restrict__ ids, int T, const float* table,
                                                         int rows, int D, const int* lens, float* __restrict__ out) {
  const int b = blockIdx.y, t = blockIdx.x * 64 + (threadIdx.x & 63);
  if (t >= T) return;
  const bool v = t < lens[b];
  long id = v ? ids[(long)b * T + t] : 0;
  if (id < 0 || id >= rows) id = 0;
  for (int c = threadIdx.x >> 6; c < D; c += 4) out[((long)b * D + c) * T + t] = v ? table[id * D + c] : 0.f;
}
void launch_glow_embed(const int64_t* ids, int T, const float* table, int rows, int D, const int* lens, float* out,
                       int B, hipStream_t s) {
  glow_embed_kernel<<<dim3((T + 63) / 64, B), 256, 0, s>>>(ids, T, table, rows, D, lens, out);
  HIP_OK(hipGetLastError());
}

// Self-attention of the Glow-TTS Transformer encoder (transformer.py:73-127; no relative-position
// tables, no proximal bias, as setup_model builds it): per (utterance, head) softmax(q k^T / sqrt(dk))
// v over the utterance's own keys (the reference's -1e4 mask makes padded keys exactly 0 after the
// softmax). One lane per query; keys and values staged through LDS in blocks of 32 and read as
// broadcasts; online softmax (running max / sum, rescaled accumulator).
constexpr int MHA_DK = 96, MHA_KB = 32;
__global__ __launch_bounds__(64) void glow_mha_kernel(const float* __restrict__ qkv, int H, int T, const int* lens,
                                                      float* __restrict__ out) {
  __shared__ float Ks[MHA_DK][MHA_KB];
  __shared__ float Vs[MHA_DK][MHA_KB];
  const int b = blockIdx.z, head = blockIdx.y, lane = threadIdx.x;
  const int t = blockIdx.x * 64 + lane;
  const int L = lens[b];
  if (blockIdx.x * 64 >= L) return;
  const float* qb = qkv + ((long)b * 3 * H + head * MHA_DK) * T;
  const float* kb = qb + (long)H * T;
  const float* vb = qb + (long)2 * H * T;
  const bool valid = t < L;
  float q[MHA_DK], o[MHA_DK];
  const float inv = 1.f / sqrtf((float)MHA_DK);
#pragma unroll
  for (int d = 0; d < MHA_DK; ++d) {
    q[d] = valid ? qb[(long)d * T + t] : 0.f;
    o[d] = 0.f;
  }
  float m = -INFINITY, l = 0.f;
  for (int s0 = 0; s0 < L; s0 += MHA_KB) {
    __syncthreads();
    for (int e = lane; e < MHA_DK * MHA_KB; e += 64) {
      const int d = e / MHA_KB, j = e % MHA_KB;
      const int sidx = min(s0 + j, L - 1);
      Ks[d][j] = kb[(long)d * T + sidx];
      Vs[d][j] = vb[(long)d * T + sidx];
    }
    __syncthreads();
    const int nb = min(MHA_KB, L - s0);
    for (int j = 0; j < nb; ++j) {
      float sc = 0.f;
#pragma unroll
      for (int d = 0; d < MHA_DK; ++d) sc = fmaf(q[d], Ks[d][j], sc);
      sc *= inv;
      const float mn = fmaxf(m, sc);
      const float r = expf(m - mn), p = expf(sc - mn);
      l = l * r + p;
#pragma unroll
      for (int d = 0; d < MHA_DK; ++d) o[d] = fmaf(o[d], r, p * Vs[d][j]);
      m = mn;
    }
  }
  if (!valid) return;
  const float il = 1.f / l;
  float* ob = out + ((long)b * H + head * MHA_DK) * T + t;
#pragma unroll
  for (int d = 0; d < MHA_DK; ++d) ob[(long)d * T] = o[d] * il;
}
void launch_glow_mha(const float* qkv, int H, int heads, int T, const int* lens, float* out, int B, hipStream_t s) {
  TTS_CHECK(H == heads * MHA_DK, "glow attention: head size must be 96");
  glow_mha_kernel<<<dim3((T + 63) / 64, heads, B), 64, 0, s>>>(qkv, H, T, lens, out);
  HIP_OK(hipGetLastError());
}
