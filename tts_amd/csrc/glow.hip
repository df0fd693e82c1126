// Glow-TTS inference pieces that are not convolutions (gfx950), SURVEY.md §8f rank 3:
//   TTS/tts/layers/glow_tts/{gated_conv,normalization,duration_predictor,glow,decoder}.py and the
//   inference glue of TTS/tts/models/glow_tts.py:170-193 (durations -> monotonic path -> expanded
//   means + noise). Activations are channel-major (B, C, T); a thread owns one time position and
//   walks the channels, so every channel step is one coalesced row access across the wave. Only
//   positions t < length are written: the convolutions (conv.hip) read positions >= length as zero
//   padding, which is what the reference's masks produce.
#include "common.h"

// LayerNorm over the channel dim (normalization.py:4-27, eps 1e-4), then GLU (dim 1) and the
// residual of GatedConvBlock (gated_conv.py:31-42): out = res + a * sigmoid(b), [a | b] = LN(x)
__global__ __launch_bounds__(256) void glu_ln_res_kernel(const float* __restrict__ x, long xb, int C2,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, const float* res,
                                                         long rb, float* out, long ob, const int* lens, int T) {
  const int b = blockIdx.y, t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T || t >= lens[b]) return;
  const float* xp = x + b * xb + t;
  float mean = 0.f;
  for (int c = 0; c < C2; ++c) mean += xp[(long)c * T];
  mean /= (float)C2;
  float var = 0.f;
  for (int c = 0; c < C2; ++c) {
    const float d = xp[(long)c * T] - mean;
    var = fmaf(d, d, var);
  }
  var /= (float)C2;
  const float rs = rsqrtf(var + 1e-4f);
  const int C = C2 / 2;
  for (int c = 0; c < C; ++c) {
    const float a = (xp[(long)c * T] - mean) * rs * gamma[c] + beta[c];
    const float g = (xp[(long)(c + C) * T] - mean) * rs * gamma[c + C] + beta[c + C];
    out[b * ob + (long)c * T + t] = res[b * rb + (long)c * T + t] + a / (1.f + expf(-g));
  }
}

// in-place LayerNorm over channels (DurationPredictor norm_1 / norm_2, after the conv's ReLU)
__global__ __launch_bounds__(256) void ln_kernel(float* x, long xb, int C, const float* __restrict__ gamma,
                                                 const float* __restrict__ beta, const int* lens, int T) {
  const int b = blockIdx.y, t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T || t >= lens[b]) return;
  float* xp = x + b * xb + t;
  float mean = 0.f;
  for (int c = 0; c < C; ++c) mean += xp[(long)c * T];
  mean /= (float)C;
  float var = 0.f;
  for (int c = 0; c < C; ++c) {
    const float d = xp[(long)c * T] - mean;
    var = fmaf(d, d, var);
  }
  var /= (float)C;
  const float rs = rsqrtf(var + 1e-4f);
  for (int c = 0; c < C; ++c) xp[(long)c * T] = (xp[(long)c * T] - mean) * rs * gamma[c] + beta[c];
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

// path[t, j] = [j < cum_t] - [j < cum_{t-1}] (generate_path), masked by t < x_len, j < y_len;
// y_mean[c, j] = sum_t path[t, j] o_mean[c, t]; z = (y_mean + noise * noise_scale) * y_mask
// (mean_only: y_log_scale = 0, glow_tts.py:184-186). Also writes attn (B, T_y, T_x) and y_mean.
__global__ __launch_bounds__(256) void glow_expand_kernel(const float* __restrict__ o_mean, int C, int Tx,
                                                          const int* xlens, const float* __restrict__ cum,
                                                          const int* ylens, int Ty, const float* noise,
                                                          float noise_scale, float* __restrict__ y_mean,
                                                          float* __restrict__ z, float* __restrict__ attn) {
  const int b = blockIdx.y, j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= Ty) return;
  const int xl = xlens[b], yl = ylens[b];
  const bool yv = j < yl;
  const float* cb = cum + (long)b * Tx;
  const float jf = (float)j;
  float* arow = attn + ((long)b * Ty + j) * Tx;
  for (int c = 0; c < C; ++c) y_mean[((long)b * C + c) * Ty + j] = 0.f;
  for (int t = 0; t < Tx; ++t) {
    const float hi = jf < cb[t] ? 1.f : 0.f;
    const float lo = t > 0 && jf < cb[t - 1] ? 1.f : 0.f;
    const float p = (yv && t < xl) ? hi - lo : 0.f;
    arow[t] = p;
    if (p != 0.f)
      for (int c = 0; c < C; ++c) y_mean[((long)b * C + c) * Ty + j] += p * o_mean[((long)b * C + c) * Tx + t];
  }
  for (int c = 0; c < C; ++c) {
    const long i = ((long)b * C + c) * Ty + j;
    const float nz = noise ? noise[i] * noise_scale : 0.f;
    z[i] = yv ? y_mean[i] + nz : 0.f;
  }
}

// decoder.py:6-19: (B, C, T) -> (B, 2C, T/2), x_sqz[s*C + c][k] = x[c][2k + s], masked by
// y_mask[2k + 1]; unsqueeze (decoder.py:22-33) is the inverse, masked by the repeated mask
__global__ __launch_bounds__(256) void glow_squeeze_kernel(const float* __restrict__ x, int C, int T,
                                                           const int* ylens, float* __restrict__ y, int K) {
  const int b = blockIdx.y, k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  const bool v = 2 * k + 1 < ylens[b];
  for (int s = 0; s < 2; ++s)
    for (int c = 0; c < C; ++c)
      y[((long)b * 2 * C + s * C + c) * K + k] = v ? x[((long)b * C + c) * T + 2 * k + s] : 0.f;
}
__global__ __launch_bounds__(256) void glow_unsqueeze_kernel(const float* __restrict__ x, int C2, int K,
                                                             const int* ylens, float* __restrict__ y, int T) {
  const int b = blockIdx.y, k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  const int C = C2 / 2;
  const bool v = 2 * k + 1 < ylens[b];
  for (int s = 0; s < 2; ++s)
    for (int c = 0; c < C; ++c)
      y[((long)b * C + c) * T + 2 * k + s] = v ? x[((long)b * C2 + s * C + c) * K + k] : 0.f;
}

// WN gate (glow.py fused_add_tanh_sigmoid_multiply, g = None): acts = tanh(a[:H]) * sigmoid(a[H:])
__global__ __launch_bounds__(256) void glow_gate_kernel(const float* __restrict__ a, int H, int K, const int* klens,
                                                        float* __restrict__ acts) {
  const int b = blockIdx.y, k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K || k >= klens[b]) return;
  for (int c = 0; c < H; ++c) {
    const float x = a[((long)b * 2 * H + c) * K + k], g = a[((long)b * 2 * H + c + H) * K + k];
    acts[((long)b * H + c) * K + k] = tanhf(x) / (1.f + expf(-g));
  }
}

// CouplingBlock reverse (glow.py:245-262, sigmoid_scale False): z1 = (x1 - m) * exp(-logs), in place
// on the second half of x; mo = end(wn(...)) = [m | logs]
__global__ __launch_bounds__(256) void glow_coupling_kernel(float* x, const float* __restrict__ mo, int Ch, int K,
                                                            const int* klens) {
  const int b = blockIdx.y, k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K || k >= klens[b]) return;
  for (int c = 0; c < Ch; ++c) {
    const long ix = ((long)b * 2 * Ch + Ch + c) * K + k;
    const float m = mo[((long)b * 2 * Ch + c) * K + k], ls = mo[((long)b * 2 * Ch + Ch + c) * K + k];
    x[ix] = (x[ix] - m) * expf(-ls);
  }
}

void launch_glu_ln_res(const float* x, long xb, int C2, const float* gamma, const float* beta, const float* res,
                       long rb, float* out, long ob, const int* lens, int B, int T, hipStream_t s) {
  glu_ln_res_kernel<<<dim3((T + 255) / 256, B), 256, 0, s>>>(x, xb, C2, gamma, beta, res, rb, out, ob, lens, T);
  HIP_OK(hipGetLastError());
}
void launch_ln(float* x, long xb, int C, const float* gamma, const float* beta, const int* lens, int B, int T,
               hipStream_t s) {
  ln_kernel<<<dim3((T + 255) / 256, B), 256, 0, s>>>(x, xb, C, gamma, beta, lens, T);
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
  glow_expand_kernel<<<dim3((Ty + 255) / 256, B), 256, 0, s>>>(o_mean, C, Tx, xlens, cum, ylens, Ty, noise,
                                                                noise_scale, y_mean, z, attn);
  HIP_OK(hipGetLastError());
}
void launch_glow_squeeze(const float* x, int C, int T, const int* ylens, float* y, int K, int B, hipStream_t s) {
  glow_squeeze_kernel<<<dim3((K + 255) / 256, B), 256, 0, s>>>(x, C, T, ylens, y, K);
  HIP_OK(hipGetLastError());
}
void launch_glow_unsqueeze(const float* x, int C2, int K, const int* ylens, float* y, int T, int B, hipStream_t s) {
  glow_unsqueeze_kernel<<<dim3((K + 255) / 256, B), 256, 0, s>>>(x, C2, K, ylens, y, T);
  HIP_OK(hipGetLastError());
}
void launch_glow_gate(const float* a, int H, int K, const int* klens, float* acts, int B, hipStream_t s) {
  glow_gate_kernel<<<dim3((K + 255) / 256, B), 256, 0, s>>>(a, H, K, klens, acts);
  HIP_OK(hipGetLastError());
}
void launch_glow_coupling(float* x, const float* mo, int Ch, int K, const int* klens, int B, hipStream_t s) {
  glow_coupling_kernel<<<dim3((K + 255) / 256, B), 256, 0, s>>>(x, mo, Ch, K, klens);
  HIP_OK(hipGetLastError());
}

// encoder.py:107: emb(x) * sqrt(hidden) (the scale is folded into the table), channel-major out
__global__ __launch_bounds__(256) void glow_embed_kernel(const int64_t* __restrict__ ids, int T, const float* table,
                                                         int rows, int D, const int* lens, float* __restrict__ out) {
  const int b = blockIdx.y, t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T) return;
  const bool v = t < lens[b];
  long id = v ? ids[(long)b * T + t] : 0;
  if (id < 0 || id >= rows) id = 0;
  for (int c = 0; c < D; ++c) out[((long)b * D + c) * T + t] = v ? table[id * D + c] : 0.f;
}
void launch_glow_embed(const int64_t* ids, int T, const float* table, int rows, int D, const int* lens, float* out,
                       int B, hipStream_t s) {
  glow_embed_kernel<<<dim3((T + 255) / 256, B), 256, 0, s>>>(ids, T, table, rows, D, lens, out);
  HIP_OK(hipGetLastError());
}
