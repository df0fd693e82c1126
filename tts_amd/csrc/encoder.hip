// Tacotron2 encoder pieces that are not convolutions (gfx950):
//  * embedding gather  (TTS/tts/models/tacotron2.py:61,144)
//  * BiLSTM recurrence (TTS/tts/layers/tacotron2.py:91-96,116-118, nn.LSTM bidirectional,
//    no packing at inference). The input projection x.W_ih^T + b_ih + b_hh for both directions
//    runs beforehand as one MFMA conv (K=1, Cout=2048); this kernel does the T sequential
//    steps with per-utterance lengths: the reverse direction starts at T_b - 1, never in the
//    padding (a padded reverse pass differs by 0.29 L-inf).
#include "common.h"

__global__ __launch_bounds__(256) void embed_gather_kernel(const int64_t* __restrict__ ids, int T_max,
                                                           const float* __restrict__ table, int num_rows,
                                                           int D, const int* lens,
                                                           float* __restrict__ out /* (B,T_max,D) */) {
  const int b = blockIdx.y, t = blockIdx.x;
  float* o = out + ((long)b * T_max + t) * D;
  const bool valid = t < lens[b];
  long id = valid ? ids[(long)b * T_max + t] : 0;
  if (id < 0 || id >= num_rows) id = 0;  // host validates ids; never read out of bounds
  for (int c = threadIdx.x; c < D; c += blockDim.x) o[c] = valid ? table[id * D + c] : 0.f;
}

void launch_embed_gather(const int64_t* ids, int T_max, const float* table, int num_rows, int D,
                         const int* lens, int B, float* out, hipStream_t s) {
  if (B <= 0 || T_max <= 0) return;
  embed_gather_kernel<<<dim3(T_max, B), 256, 0, s>>>(ids, T_max, table, num_rows, D, lens, out);
  HIP_OK(hipGetLastError());
}

// Gin: (B, 2048, T_max) channel-major gate pre-activations incl. b_ih + b_hh
//      rows [dir*1024 + gate*256 + j], gate order i, f, g, o.
// WhhT: per dir [gate][k/4][j][4] so thread j's float4 loads are contiguous across the wave.
// out: (B, T_max, 512) = [fwd h | bwd h]
__global__ __launch_bounds__(256) void bilstm_rec_kernel(const float* __restrict__ Gin,
                                                         const float* __restrict__ WhhT,
                                                         const int* lens, int T_max,
                                                         float* __restrict__ out) {
  const int b = blockIdx.x >> 1, dir = blockIdx.x & 1;
  const int j = threadIdx.x;
  const int T = lens[b];
  __shared__ __attribute__((aligned(16))) float h[256];
  h[j] = 0.f;
  float c = 0.f;
  __syncthreads();
  const f32x4* W = reinterpret_cast<const f32x4*>(WhhT) + (long)dir * 4 * 64 * 256 + j;
  const float* gbase = Gin + (long)b * 2048 * T_max + (long)dir * 1024 * T_max;
  for (int step = 0; step < T; ++step) {
    const int t = dir ? (T - 1 - step) : step;
    float a0 = gbase[(long)(0 * 256 + j) * T_max + t];
    float a1 = gbase[(long)(1 * 256 + j) * T_max + t];
    float a2 = gbase[(long)(2 * 256 + j) * T_max + t];
    float a3 = gbase[(long)(3 * 256 + j) * T_max + t];
#pragma unroll 8
    for (int k4 = 0; k4 < 64; ++k4) {
      const f32x4 hv = *reinterpret_cast<const f32x4*>(h + 4 * k4);
      const f32x4 w0 = W[(long)(0 * 64 + k4) * 256];
      const f32x4 w1 = W[(long)(1 * 64 + k4) * 256];
      const f32x4 w2 = W[(long)(2 * 64 + k4) * 256];
      const f32x4 w3 = W[(long)(3 * 64 + k4) * 256];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        a0 = fmaf(w0[e], hv[e], a0);
        a1 = fmaf(w1[e], hv[e], a1);
        a2 = fmaf(w2[e], hv[e], a2);
        a3 = fmaf(w3[e], hv[e], a3);
      }
    }
    const float ig = 1.f / (1.f + expf(-a0));
    const float fg = 1.f / (1.f + expf(-a1));
    const float gg = tanhf(a2);
    const float og = 1.f / (1.f + expf(-a3));
    c = fg * c + ig * gg;
    const float hn = og * tanhf(c);
    __syncthreads();
    h[j] = hn;
    __syncthreads();
    out[((long)b * T_max + t) * 512 + dir * 256 + j] = hn;
  }
}

void launch_bilstm_rec(const float* Gin, const float* WhhT, const int* lens, int T_max, int B, float* out,
                       hipStream_t s) {
  if (B <= 0 || T_max <= 0) return;
  bilstm_rec_kernel<<<2 * B, 256, 0, s>>>(Gin, WhhT, lens, T_max, out);
  HIP_OK(hipGetLastError());
}
