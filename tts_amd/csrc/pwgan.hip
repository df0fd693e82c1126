// ParallelWaveGAN generator inference (gfx950), SURVEY.md §8f rank 3 (config C4):
//   TTS/vocoder/models/parallel_wavegan_generator.py:90-125, layers/parallel_wavegan.py:56-87,
//   layers/upsample.py:5-101.
//
// Layout: every signal is channel-major (B, C, T) fp32 at the sample rate, T_b = hop * (M_b + 2p).
// The 30 WaveNet residual blocks are the cost (86 kFLOP per sample per block): one fused kernel per
// block, an implicit GEMM on v_mfma_f32_16x16x4_f32 with
//   GEMM1  a (128 x TQ) = Wd (128 x 3*64, the 3 dilated taps) . x  +  Wa (128 x 80) . c
//          (17 k-chunks of 16, staged through LDS with the dilation offsets and the zero padding
//          resolved at staging time; gate rows interleaved (tanh_j, sigmoid_j) so the gate
//          z = tanh * sigmoid is a lane-local epilogue written straight into LDS)
//   GEMM2  [out | skip] (128 x TQ) = W2 (128 x 64) . z   (z read from LDS, never from HBM)
//   epilogue  x' = (out + b + x) / 4  -> ping-pong buffer;  skip (+)= s + b  (in place)
// HBM per sample per block: x (+halo, L2) 256 B, c 320 B, skip r/w 512 B, x' 256 B.
#include "common.h"

#include <cstdlib>
#include "split16.h"

namespace {
constexpr int PW_TQ = 128;          // time columns per workgroup
constexpr int PW_ROW = PW_TQ + 4;   // LDS row stride (conflict-free B-operand reads)
constexpr int PW_R = 64, PW_G = 128, PW_A = 80, PW_S = 64;
constexpr int PW_KC1 = (3 * PW_R + PW_A) / 16;  // 17
constexpr int PW_KC2 = (PW_G / 2) / 16;         // 4
}  // namespace

// upsample.py:5-63: nearest stretch by S along time, then the (1, 2S + 1) Conv2d with zero padding
// S (one filter for every channel): out[t] = sum_k h[k] * in[(t + k - S) / S], 0 <= t + k - S < L*S.
// A thread makes S consecutive outputs, so its 2S + 1 taps touch 3 input samples; positions past
// the row's length are not written (every reader bounds its reads by the length).
template <int S>
__global__ __launch_bounds__(256) void pw_upsample_kernel(const float* __restrict__ in, long ib, int Lin_max,
                                                          const int* lens, int len_add, int in_mul,
                                                          const float* __restrict__ h, float* __restrict__ out,
                                                          long ob, int Lout_max) {
  const int b = blockIdx.z, ch = blockIdx.y, u = blockIdx.x * 256 + threadIdx.x;  // input sample u
  const int Lin = (lens[b] + len_add) * in_mul, Lout = Lin * S;
  if (u >= Lin) return;
  const float* ip = in + b * ib + (long)ch * Lin_max;
  const float xm = u > 0 ? ip[u - 1] : 0.f, x0 = ip[u], xp = u + 1 < Lin ? ip[u + 1] : 0.f;
  float hk[2 * S + 1];
#pragma unroll
  for (int k = 0; k <= 2 * S; ++k) hk[k] = h[k];
  float* op = out + b * ob + (long)ch * Lout_max + (long)u * S;
#pragma unroll
  for (int r = 0; r < S; ++r) {  // t = u S + r; tap k reads stretched sample t + k - S
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k <= 2 * S; ++k) {
      const int v = r + k - S;  // offset from u S, in [-S, 2S - 1]
      const float x = v < 0 ? xm : (v < S ? x0 : xp);
      const int tt = u * S + v;
      if (tt >= 0 && tt < Lout) acc = fmaf(hk[k], x, acc);
    }
    op[r] = acc;
  }
}

// first_conv (1 -> 64, k1) on the prior noise
__global__ __launch_bounds__(256) void pw_first_kernel(const float* __restrict__ noise, long nb,
                                                       const float* __restrict__ w, const float* __restrict__ bias,
                                                       const int* lens, int len_add, int hop,
                                                       float* __restrict__ x, int Tmax) {
  const int b = blockIdx.y, t = blockIdx.x * 64 + (threadIdx.x & 63);
  if (t >= Tmax) return;
  const int T = (lens[b] + len_add) * hop;
  const float n = t < T ? noise[b * nb + t] : 0.f;
  for (int ch = threadIdx.x >> 6; ch < PW_R; ch += 4)
    x[((long)b * PW_R + ch) * Tmax + t] = t < T ? fmaf(w[ch], n, bias[ch]) : 0.f;
}

// tanh(u) * sigmoid(g) on the hardware exp / rcp (common.h tanh_f / sigm_f: |error| < 2e-7 absolute).
// Round 4: __frcp_rn compiled to the IEEE division sequence (div_scale / div_fmas / div_fixup, ~10
// VALU per reciprocal), a third of the persistent residual-block kernel's VALU issue.
__device__ __forceinline__ float pw_gate(float u, float g) { return tanh_f(u) * sigm_f(g); }

struct PwLayerArgs {
  const float* x;      // (B, 64, Tmax)
  const float* c;      // (B, 80, Tmax) upsampled features
  float* xn;           // next x
  float* skip;         // (B, 64, Tmax)
  const f32x4* W1;     // [8 m16][17 kc][64] swizzled, rows interleaved (tanh_j, sigmoid_j)
  const float* b1;     // [128] interleaved
  const f32x4* W2;     // [8 m16][4 kc][64]: rows 0..63 conv1x1_out, 64..127 conv1x1_skip
  const float* b2;     // [128]
  const int* lens;
  const float* zeros;  // >= 64 zero floats: the source of out-of-range staging lanes (LDS-DMA path)
  int len_add, hop, Tmax, dil, first;
};

__global__ __launch_bounds__(256) void pw_layer_kernel(PwLayerArgs a) {
  __shared__ __attribute__((aligned(16))) float Xs[2][16 * PW_ROW];
  __shared__ __attribute__((aligned(16))) float Zs[(PW_G / 2) * PW_ROW];
  const int b = blockIdx.y;
  const int T = (a.lens[b] + a.len_add) * a.hop;
  const int t0 = blockIdx.x * PW_TQ;
  if (t0 >= T) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;  // 2 x 2 waves, each 64 rows x 64 columns
  const int g4 = 4 * (lane >> 4), col = lane & 15;
  const float* xb = a.x + (long)b * PW_R * a.Tmax;
  const float* cb = a.c + (long)b * PW_A * a.Tmax;

  // staging: chunk kc < 12 -> x rows 16*(kc%4).. at tap kc/4 (offset (tap-1)*dil); else c rows.
  // Two register sets, loads two chunks ahead: chunk kc+2's global loads go into the set chunk kc
  // vacated (written to LDS one iteration earlier) while chunk kc's MFMAs run; chunk kc+1's set
  // goes to LDS after them. Weight fragments run one chunk ahead (L2-resident).
  float st[2][8];
  auto stage_load = [&](float (&r8)[8], int kc) {
    const float* src;
    int off;
    if (kc < 12) {
      src = xb + (long)(16 * (kc & 3)) * a.Tmax;
      off = (kc / 4 - 1) * a.dil;
    } else {
      src = cb + (long)(16 * (kc - 12)) * a.Tmax;
      off = 0;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int e = tid + 256 * j;
      const int r = e >> 7, q = e & 127;
      const int t = t0 + q + off;
      const bool ok = t >= 0 && t < T;
      const float v = src[(long)r * a.Tmax + (ok ? t : 0)];
      r8[j] = ok ? v : 0.f;
    }
  };
  auto stage_store = [&](float* X, const float (&r8)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int e = tid + 256 * j;
      X[(e >> 7) * PW_ROW + (e & 127)] = r8[j];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int mt0 = wm * 4;
  f32x4 Ar[2][4];
  auto aload = [&](f32x4 (&r)[4], int kc) {
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) r[mi] = a.W1[((mt0 + mi) * PW_KC1 + kc) * 64 + lane];
  };
  aload(Ar[0], 0);
  stage_load(st[0], 0);
  stage_load(st[1], 1);
  stage_store(Xs[0], st[0]);
  __syncthreads();
#pragma unroll 2
  for (int kc = 0; kc < PW_KC1; ++kc) {
    const float* X = Xs[kc & 1];
    const int p = kc & 1, q = p ^ 1;
    if (kc + 2 < PW_KC1) stage_load(st[p], kc + 2);
    if (kc + 1 < PW_KC1) aload(Ar[q], kc + 1);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      float bv[4];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) bv[ni] = X[(g4 + s) * PW_ROW + wn * 64 + ni * 16 + col];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = MFMA16(Ar[p][mi][s], bv[ni], acc[mi][ni]);
    }
    if (kc + 1 < PW_KC1) stage_store(Xs[q], st[q]);
    __syncthreads();
  }

  // gate epilogue: rows R = wm*64 + mi*16 + g4 + j, (R even, R + 1) -> z[R / 2] into LDS
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
    const int R = wm * 64 + mi * 16 + g4;
    const float b0 = a.b1[R], b1 = a.b1[R + 1], b2 = a.b1[R + 2], b3 = a.b1[R + 3];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int q = wn * 64 + ni * 16 + col;
      const f32x4 v = acc[mi][ni];
      Zs[(R >> 1) * PW_ROW + q] = pw_gate(v[0] + b0, v[1] + b1);
      Zs[((R >> 1) + 1) * PW_ROW + q] = pw_gate(v[2] + b2, v[3] + b3);
    }
  }
  __syncthreads();

  // GEMM2: wave row half wm = 0 -> conv1x1_out rows, wm = 1 -> conv1x1_skip rows
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int kc = 0; kc < PW_KC2; ++kc) {
    f32x4 A[4];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) A[mi] = a.W2[((mt0 + mi) * PW_KC2 + kc) * 64 + lane];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      float bv[4];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) bv[ni] = Zs[(kc * 16 + g4 + s) * PW_ROW + wn * 64 + ni * 16 + col];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = MFMA16(A[mi][s], bv[ni], acc[mi][ni]);
    }
  }
  // x' = (out + b + x) * 0.25 (parallel_wavegan.py:85); skip (+)= s + b
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int t = t0 + wn * 64 + ni * 16 + col;
      if (t >= T) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ch = mi * 16 + g4 + j;
        const float v = acc[mi][ni][j] + a.b2[wm * 64 + ch];
        const long i = ((long)b * 64 + ch) * a.Tmax + t;
        if (wm == 0) a.xn[i] = (v + a.x[i]) * 0.25f;
        else a.skip[i] = a.first ? v : a.skip[i] + v;
      }
    }
  }
}

// s_waitcnt with vmcnt = n and no lgkm / exp wait (gfx9 encoding: vmcnt[3:0] | vmcnt[5:4] << 14)
#define PW_WAIT_VM(n) __builtin_amdgcn_s_waitcnt(((n) & 15) | (((n) >> 4) << 14) | (7 << 4) | (0xF << 8))

// The same residual block with LDS-DMA staging: both GEMM1 operands go global -> LDS with
// global_load_lds (no staging registers), through a 3-deep ring, two chunks ahead. Every wave
// issues exactly 10 LDS-DMA loads per chunk (8 x 4 B for its quarter of the 16 x 128 activation
// tile -- out-of-range lanes read a zero buffer --, 2 x 16 B for two of the 8 weight tiles), so a
// counted vmcnt(10) retires chunk kc while kc+1 stays in flight, and a raw s_barrier (no vmcnt(0)
// drain) publishes it. The weight fragments are read from LDS (ds_read_b128); GEMM2 and the
// epilogues are those of pw_layer_kernel, with z in LDS aliasing the ring.
constexpr int PW_RB = 16 * PW_ROW;  // activation slot (floats)
constexpr int PW_RA = 8 * 256;      // weight slot: 8 m16 tiles x 64 lanes x 4
template <int PW_NS>
__global__ __launch_bounds__(256, PW_NS == 3 ? 3 : 2) void pw_layer_glds_kernel(PwLayerArgs a) {
  constexpr int PW_LDS =
      PW_NS * (PW_RB + PW_RA) > (PW_G / 2) * PW_ROW ? PW_NS * (PW_RB + PW_RA) : (PW_G / 2) * PW_ROW;
  constexpr int AHEAD = PW_NS - 1;  // chunks in flight beyond the one being consumed
  __shared__ __attribute__((aligned(16))) float pool[PW_LDS];
  float* ringA = pool;                 // [NS][PW_RA]
  float* ringB = pool + PW_NS * PW_RA;  // [NS][PW_RB]
  float* Zs = pool;                    // after GEMM1
  const int b = blockIdx.y;
  const int T = (a.lens[b] + a.len_add) * a.hop;
  const int t0 = blockIdx.x * PW_TQ;
  if (t0 >= T) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int g4 = 4 * (lane >> 4), col = lane & 15;
  const float* xb = a.x + (long)b * PW_R * a.Tmax;
  const float* cb = a.c + (long)b * PW_A * a.Tmax;
  const float* W1f = reinterpret_cast<const float*>(a.W1);

  auto issue = [&](int kc) {
    const int sl = kc % PW_NS;
    const float* src;
    int off;
    if (kc < 12) {
      src = xb + (long)(16 * (kc & 3)) * a.Tmax;
      off = (kc / 4 - 1) * a.dil;
    } else {
      src = cb + (long)(16 * (kc - 12)) * a.Tmax;
      off = 0;
    }
    float* dstB = ringB + sl * PW_RB;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int e0 = j * 256 + wave * 64;  // this wave's 64 consecutive elements of the tile
      const int r = e0 >> 7, q = (e0 & 127) + lane;
      const int t = t0 + q + off;
      const float* g = (t >= 0 && t < T) ? src + (long)r * a.Tmax + t : a.zeros + lane;
      __builtin_amdgcn_global_load_lds(g, dstB + r * PW_ROW + (e0 & 127), 4, 0, 0);
    }
    float* dstA = ringA + sl * PW_RA;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int m16 = wave * 2 + i;
      __builtin_amdgcn_global_load_lds(W1f + ((long)(m16 * PW_KC1 + kc) * 64 + lane) * 4, dstA + m16 * 256, 16, 0,
                                       0);
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int mt0 = wm * 4;

#pragma unroll
  for (int k = 0; k < AHEAD; ++k) issue(k);
  for (int kc = 0; kc < PW_KC1; ++kc) {
    // chunks issued after kc: min(AHEAD - 1, PW_KC1 - 1 - kc), 10 LDS-DMA loads each
    const int after = min(AHEAD - 1, PW_KC1 - 1 - kc);
    if (after >= 2) PW_WAIT_VM(20);
    else if (after == 1) PW_WAIT_VM(10);
    else PW_WAIT_VM(0);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kc + AHEAD < PW_KC1) issue(kc + AHEAD);
    const int sl = kc % PW_NS;
    const float* X = ringB + sl * PW_RB;
    const f32x4* As = reinterpret_cast<const f32x4*>(ringA + sl * PW_RA);
    f32x4 A[4];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) A[mi] = As[(mt0 + mi) * 64 + lane];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      float bv[4];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) bv[ni] = X[(g4 + s) * PW_ROW + wn * 64 + ni * 16 + col];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = MFMA16(A[mi][s], bv[ni], acc[mi][ni]);
    }
  }
  __syncthreads();  // every wave is done with the ring before z overwrites it

#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
    const int R = wm * 64 + mi * 16 + g4;
    const float b0 = a.b1[R], b1 = a.b1[R + 1], b2 = a.b1[R + 2], b3 = a.b1[R + 3];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int q = wn * 64 + ni * 16 + col;
      const f32x4 v = acc[mi][ni];
      Zs[(R >> 1) * PW_ROW + q] = pw_gate(v[0] + b0, v[1] + b1);
      Zs[((R >> 1) + 1) * PW_ROW + q] = pw_gate(v[2] + b2, v[3] + b3);
    }
  }
  __syncthreads();
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int kc = 0; kc < PW_KC2; ++kc) {
    f32x4 A[4];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) A[mi] = a.W2[((mt0 + mi) * PW_KC2 + kc) * 64 + lane];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      float bv[4];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) bv[ni] = Zs[(kc * 16 + g4 + s) * PW_ROW + wn * 64 + ni * 16 + col];
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = MFMA16(A[mi][s], bv[ni], acc[mi][ni]);
    }
  }
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int t = t0 + wn * 64 + ni * 16 + col;
      if (t >= T) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ch = mi * 16 + g4 + j;
        const float v = acc[mi][ni][j] + a.b2[wm * 64 + ch];
        const long i = ((long)b * 64 + ch) * a.Tmax + t;
        if (wm == 0) a.xn[i] = (v + a.x[i]) * 0.25f;
        else a.skip[i] = a.first ? v : a.skip[i] + v;
      }
    }
  }
}

// parallel_wavegan_generator.py:111-116: skips * sqrt(1 / layers) -> ReLU -> 1x1 (64) -> ReLU -> 1x1 (1)
__global__ __launch_bounds__(256) void pw_out_kernel(const float* __restrict__ skip, float scale,
                                                     const float* __restrict__ W3, const float* __restrict__ b3,
                                                     const float* __restrict__ w4, const float* __restrict__ b4,
                                                     const int* lens, int len_add, int hop, int Tmax,
                                                     float* __restrict__ out) {
  const int b = blockIdx.y, t = blockIdx.x * 256 + threadIdx.x;
  if (t >= Tmax) return;
  const int T = (lens[b] + len_add) * hop;
  if (t >= T) {
    out[(long)b * Tmax + t] = 0.f;
    return;
  }
  float h[PW_S];
#pragma unroll
  for (int ch = 0; ch < PW_S; ++ch) h[ch] = fmaxf(skip[((long)b * PW_S + ch) * Tmax + t] * scale, 0.f);
  float y = b4[0];
  for (int o = 0; o < PW_S; ++o) {
    float v = b3[o];
#pragma unroll
    for (int ch = 0; ch < PW_S; ++ch) v = fmaf(W3[o * PW_S + ch], h[ch], v);
    y = fmaf(w4[o], fmaxf(v, 0.f), y);
  }
  out[(long)b * Tmax + t] = y;
}

void launch_pw_upsample(const float* in, long ib, int Lin_max, const int* lens, int len_add, int in_mul, int s,
                        const float* h, float* out, long ob, int Lout_max, int C, int B, hipStream_t st) {
  const dim3 grid((Lin_max + 255) / 256, C, B);
  switch (s) {
    case 2: pw_upsample_kernel<2><<<grid, 256, 0, st>>>(in, ib, Lin_max, lens, len_add, in_mul, h, out, ob, Lout_max); break;
    case 4: pw_upsample_kernel<4><<<grid, 256, 0, st>>>(in, ib, Lin_max, lens, len_add, in_mul, h, out, ob, Lout_max); break;
    case 8: pw_upsample_kernel<8><<<grid, 256, 0, st>>>(in, ib, Lin_max, lens, len_add, in_mul, h, out, ob, Lout_max); break;
    default: TTS_CHECK(false, "pwgan: upsample factors must be 2, 4 or 8");
  }
  HIP_OK(hipGetLastError());
}
void launch_pw_first(const float* noise, long nb, const float* w, const float* bias, const int* lens, int len_add,
                     int hop, float* x, int Tmax, int B, hipStream_t st) {
  pw_first_kernel<<<dim3((Tmax + 63) / 64, B), 256, 0, st>>>(noise, nb, w, bias, lens, len_add, hop, x, Tmax);
  HIP_OK(hipGetLastError());
}
void launch_pw_layer(const float* x, const float* c, float* xn, float* skip, const float* W1, const float* b1,
                     const float* W2, const float* b2, const int* lens, const float* zeros, int len_add, int hop,
                     int Tmax, int dil, int first, int B, int variant, hipStream_t st) {
  PwLayerArgs a{x, c, xn, skip, reinterpret_cast<const f32x4*>(W1), b1, reinterpret_cast<const f32x4*>(W2), b2,
                lens, zeros, len_add, hop, Tmax, dil, first};
  const dim3 grid((Tmax + PW_TQ - 1) / PW_TQ, B);
  if (variant == 1) pw_layer_glds_kernel<3><<<grid, 256, 0, st>>>(a);
  else if (variant == 2) pw_layer_glds_kernel<4><<<grid, 256, 0, st>>>(a);
  else pw_layer_kernel<<<grid, 256, 0, st>>>(a);
  HIP_OK(hipGetLastError());
}
void launch_pw_out(const float* skip, float scale, const float* W3, const float* b3, const float* w4,
                   const float* b4, const int* lens, int len_add, int hop, int Tmax, float* out, int B,
                   hipStream_t st) {
  pw_out_kernel<<<dim3((Tmax + 255) / 256, B), 256, 0, st>>>(skip, scale, W3, b3, w4, b4, lens, len_add, hop, Tmax,
                                                             out);
  HIP_OK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------
// The residual block on the f16 MFMA with split-f16 operands (split16.h), the
// same arithmetic as pw_layer_kernel at ~2x its speed:
//   GEMM1  9 k-steps of 32: the 3 dilated taps x 2 x-channel halves, then the 80 aux channels
//          padded to 96; each k-step staged as [pos][32 hi | 32 lo | 16 pad] (conflict-free
//          ds_read_b128 B operands), two steps ahead through two register sets
//   gate   z = tanh * sigmoid of the interleaved row pairs, split, into two [pos][32 | 32] planes
//   GEMM2  2 k-steps over the z planes; rows 0..63 conv1x1_out, 64..127 conv1x1_skip
// 4 waves (4 x 1): 32 gate rows x 64 positions each; weights (pre-split A fragments, L2-resident)
// through a 3-slot register ring that runs from GEMM1 straight into GEMM2.
namespace {
constexpr int PX_XR = 80;                 // staging row, halves
constexpr int PX_NK1 = 9, PX_NK2 = 2;     // k-steps
}  // namespace

// WN column groups of 64 positions: TQ = 64 WN positions, 4 WN waves (4 x WN)
template <int WN>
__global__ __launch_bounds__(256 * WN) void pw_layer_x3_kernel(PwLayerArgs a, const void* W1x, const void* W2x,
                                                               unsigned* oflow) {
  constexpr int TQ = 64 * WN;
  constexpr int PX_PLANE = TQ * PX_XR;  // one staged k-step / one z plane (halves)
  __shared__ __attribute__((aligned(16))) _Float16 Xs[2 * PX_PLANE];
  __shared__ __attribute__((aligned(16))) _Float16 Zs[2 * PX_PLANE];
  const int b = blockIdx.y;
  const int T = (a.lens[b] + a.len_add) * a.hop;
  const int t0 = blockIdx.x * TQ;
  if (t0 >= T) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;  // 4 x WN waves: 32 rows x 64 positions
  const int nb = wn * 64 + (lane & 15), kg = 8 * (lane >> 4);
  const float* xb = a.x + (long)b * PW_R * a.Tmax;
  const float* cb = a.c + (long)b * PW_A * a.Tmax;
  bool bad = false;

  // staging item of this thread: channel octet g (0..3) of the k-step, position q (0..127)
  const int sg = tid / TQ, sq = tid % TQ;
  float st[2][8];
  bool sok[2];  // validity applied at the LDS store, so no load is waited for where it is issued
  auto stage_load = [&](float (&r8)[8], bool& okr, int ks) {
    const float* src;
    int off, c0, cmax;
    if (ks < 6) {
      src = xb;
      c0 = 32 * (ks & 1) + 8 * sg;
      off = (ks / 2 - 1) * a.dil;
      cmax = PW_R;
    } else {
      src = cb;
      c0 = 32 * (ks - 6) + 8 * sg;
      off = 0;
      cmax = PW_A;
    }
    const int t = t0 + sq + off;
    okr = t >= 0 && t < T && c0 < cmax;
    const float* p = src + (long)min(c0, cmax - 8) * a.Tmax + (okr ? t : 0);
#pragma unroll
    for (int c = 0; c < 8; ++c) r8[c] = p[(long)c * a.Tmax];
  };
  auto stage_store = [&](_Float16* X, const float (&r8)[8], bool okr) {
    float mx = 0.f, v[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      v[c] = okr ? r8[c] : 0.f;
      mx = fmaxf(mx, __builtin_fabsf(v[c]));
    }
    bad |= !(mx < F16_RANGE);
    h8 hi, lo;
    split8(v, hi, lo);
    *reinterpret_cast<h8*>(X + sq * PX_XR + 8 * sg) = hi;
    *reinterpret_cast<h8*>(X + sq * PX_XR + 32 + 8 * sg) = lo;
  };

  // weights: A fragments [m16 (8)][k-step][lane][hi 8 | lo 8]; sequence 0..8 = GEMM1, 9..10 = GEMM2
  const __amdgpu_buffer_rsrc_t w1r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(W1x), 0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t w2r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(W2x), 0, 0x7fffffff, 0x00020000);
  const int mt0 = wm * 2;
  constexpr int RSL = 3;  // weight ring slots
  constexpr int SD = 2;   // staging depth (k-steps ahead)
  h8 ring[RSL][2][2];
  auto wload = [&](h8 (&r)[2][2], int seq) {
    seq = min(seq, PX_NK1 + PX_NK2 - 1);
    const bool g1 = seq < PX_NK1;
    const __amdgpu_buffer_rsrc_t wr = g1 ? w1r : w2r;
    const int nk = g1 ? PX_NK1 : PX_NK2, ks = g1 ? seq : seq - PX_NK1;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      const int so = ((mt0 + mi) * nk + ks) * 2048;
      r[mi][0] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(wr, lane * 32, so, 0));
      r[mi][1] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(wr, lane * 32 + 16, so, 0));
    }
  };

  // the epilogue's residual operands (x for the conv1x1_out rows, the running skip sum for the
  // skip rows), loaded now so their latency hides under the GEMMs
  float res[2][4][4];
  auto res_load = [&]() {
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int R = wm * 32 + mi * 16 + 4 * (lane >> 4) + j;
        const bool out_row = R < PW_R;
        const float* src = out_row ? a.x : a.skip;
        const long rowb = ((long)b * 64 + (out_row ? R : R - PW_R)) * a.Tmax;
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          const int t = min(t0 + nb + ni * 16, T - 1);
          res[mi][j][ni] = src[rowb + t];  // the skip rows' value is unused on the first block
        }
      }
  };
  res_load();
  f32x4 am[2][4], ac[2][4];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) am[mi][ni] = ac[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto kstep = [&](const _Float16* X, const h8 (&w)[2][2]) {
    h8 bh[4], bl[4];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const _Float16* q = X + (nb + ni * 16) * PX_XR + kg;
      bh[ni] = *reinterpret_cast<const h8*>(q);
      bl[ni] = *reinterpret_cast<const h8*>(q + 32);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) mfma_x3(w[mi][0], w[mi][1], bh[ni], bl[ni], am[mi][ni], ac[mi][ni]);
  };

  // GEMM1: staging two k-steps ahead (step s loaded into set s & 1 after step s - 3's MFMAs,
  // stored to LDS buffer s & 1 after step s - 1's)
  stage_load(st[0], sok[0], 0);
#pragma unroll
  for (int u = 0; u < RSL; ++u) wload(ring[u], u);
  if constexpr (SD == 2) {
    stage_load(st[1], sok[1], 1);
    stage_store(Xs, st[0], sok[0]);
    stage_load(st[0], sok[0], 2);
  } else {
    stage_store(Xs, st[0], sok[0]);
  }
  lds_barrier();
#pragma unroll
  for (int ks = 0; ks < PX_NK1; ++ks) {
    if constexpr (SD == 1) {
      if (ks + 1 < PX_NK1) stage_load(st[0], sok[0], ks + 1);
      __builtin_amdgcn_sched_barrier(0);
    }
    kstep(Xs + (ks & 1) * PX_PLANE, ring[ks % RSL]);
    wload(ring[ks % RSL], ks + RSL);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (SD == 2) {
      if (ks + 1 < PX_NK1) stage_store(Xs + ((ks + 1) & 1) * PX_PLANE, st[(ks + 1) & 1], sok[(ks + 1) & 1]);
      if (ks + 3 < PX_NK1) stage_load(st[(ks + 1) & 1], sok[(ks + 1) & 1], ks + 3);
    } else {
      if (ks + 1 < PX_NK1) stage_store(Xs + ((ks + 1) & 1) * PX_PLANE, st[0], sok[0]);
    }
    lds_barrier();
  }
  // gate: rows R = wm * 32 + mi * 16 + 4 (lane >> 4) + j, pairs (R, R + 1) -> z[R / 2]
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
    const int R = wm * 32 + mi * 16 + 4 * (lane >> 4);
    const float b0 = a.b1[R], b1 = a.b1[R + 1], b2 = a.b1[R + 2], b3 = a.b1[R + 3];
    const int zc = R >> 1;  // z channels zc, zc + 1
    _Float16* Z = Zs + (zc >> 5) * PX_PLANE + (zc & 31);
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int q = nb + ni * 16;
      f32x4 v;
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = x3_value(am[mi][ni][j], ac[mi][ni][j]);
      h2_ zh, zl;
      split2(f32x2_{pw_gate(v[0] + b0, v[1] + b1), pw_gate(v[2] + b2, v[3] + b3)}, zh, zl);
      *reinterpret_cast<h2_*>(Z + q * PX_XR) = zh;
      *reinterpret_cast<h2_*>(Z + q * PX_XR + 32) = zl;
      am[mi][ni] = ac[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  lds_barrier();
  // GEMM2 (weights 9, 10 already in the ring)
#pragma unroll
  for (int ks = 0; ks < PX_NK2; ++ks) kstep(Zs + ks * PX_PLANE, ring[(PX_NK1 + ks) % RSL]);
  // x' = (out + b + x) * 0.25 (parallel_wavegan.py:85); skip (+)= s + b
#pragma unroll
  for (int mi = 0; mi < 2; ++mi) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int R = wm * 32 + mi * 16 + 4 * (lane >> 4) + j;
      const float bias = a.b2[R];
      const bool out_row = R < PW_R;
      const int ch = out_row ? R : R - PW_R;
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int t = t0 + nb + ni * 16;
        if (t >= T) continue;
        const float v = x3_value(am[mi][ni][j], ac[mi][ni][j]) + bias;
        const long i = ((long)b * 64 + ch) * a.Tmax + t;
        if (out_row) a.xn[i] = (v + res[mi][j][ni]) * 0.25f;
        else a.skip[i] = a.first ? v : res[mi][j][ni] + v;
      }
    }
  }
  if (bad) __hip_atomic_fetch_or(oflow, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Persistent form (round 4): one 4-wave workgroup per CU loops over the (utterance, 64-position)
// tiles with every weight in registers. The register-ring kernel above spent most of a tile
// waiting: one workgroup per CU (320 VGPRs), a barrier per k-step and its operands two k-steps
// (~0.4 us of MFMA) ahead of ~2 us of load latency. Here
//   * a wave's 2 m-tiles x 11 k-steps of split A fragments (176 VGPRs) load once per launch;
//   * a tile's whole GEMM1 operand (9 k-steps, 32 floats per thread) is staged into 9 LDS planes at
//     once, and the next tile's is loaded into registers while this tile's GEMMs run (nothing
//     else is loaded between, so the in-order vmcnt waits of the GEMMs never wait for them);
//   * the epilogue operands (x, running skip) load before the next tile's operands.
// Same arithmetic, k-step order and epilogue as pw_layer_x3_kernel: bit-identical results.
template <int NW>
__global__ __launch_bounds__(64 * NW, 1) void pw_layer_x3p_kernel(PwLayerArgs a, const void* W1x, const void* W2x,
                                                                  unsigned* oflow, int B, int ntiles) {
  // NW = 4: 2 m-tiles per wave, one wave per SIMD; NW = 8: 1 m-tile per wave, two waves per SIMD
  constexpr int NTH = 64 * NW, MI = 8 / NW, CPI = 32 / NW;  // m-tiles per wave, staged channels per item
  static_assert(NW == 4 || NW == 8, "waves");
  constexpr int TQ = 64;
  constexpr int PLANE = TQ * PX_XR;  // halves
  extern __shared__ __attribute__((aligned(16))) _Float16 shp[];
  _Float16* Xs = shp;                   // PX_NK1 planes
  _Float16* Zs = shp + PX_NK1 * PLANE;  // 2 planes
  h8* W2s = reinterpret_cast<h8*>(shp + (PX_NK1 + 2) * PLANE);  // GEMM2 A fragments [m16][k-step][lane][2]
  __shared__ int tcum[65], tlen[64];
  __shared__ float b1s[PW_G], b2s[PW_G];
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave;  // NW x 1 waves: 16 MI rows x 64 positions each
  const int nb = lane & 15, kg = 8 * (lane >> 4);
  bool bad = false;
  if (wave == 0) {  // tiles per utterance, exclusive prefix sum
    const int L = lane < B ? (a.lens[lane] + a.len_add) * a.hop : 0;
    const int n = (L + TQ - 1) / TQ;
    int v = n;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(v, o, 64);
      if (lane >= o) v += y;
    }
    tcum[lane] = v - n;
    tlen[lane] = L;
    if (lane == 63) tcum[64] = v;
  }
  __syncthreads();
  struct Tile {
    int b, t0, T;
  };
  auto tile_of = [&](int i) {
    const bool hit = lane < B && tcum[lane] <= i && i < tcum[lane + 1];
    const unsigned long long m = __ballot(hit);
    Tile r;
    r.b = __builtin_amdgcn_readfirstlane(m ? __ffsll((long long)m) - 1 : 0);
    r.t0 = __builtin_amdgcn_readfirstlane((i - tcum[r.b]) * TQ);
    r.T = __builtin_amdgcn_readfirstlane(tlen[r.b]);
    return r;
  };

  // GEMM1 weights [m16 (8)][k-step][lane][hi 8 | lo 8] in registers (this wave's m-tiles MI wm ..
  // MI wm + MI - 1); GEMM2's (32 KB) and the biases in LDS
  h8 w1[PX_NK1][MI][2];
  {
    const __amdgpu_buffer_rsrc_t w1r = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(W1x), 0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int ks = 0; ks < PX_NK1; ++ks) {
        const int so = ((MI * wm + mi) * PX_NK1 + ks) * 2048;
        w1[ks][mi][0] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(w1r, lane * 32, so, 0));
        w1[ks][mi][1] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(w1r, lane * 32 + 16, so, 0));
      }
    const h8* w2g = reinterpret_cast<const h8*>(W2x);
    for (int i = tid; i < 8 * PX_NK2 * 64 * 2; i += NTH) W2s[i] = w2g[i];
    for (int i = tid; i < PW_G; i += NTH) {
      b1s[i] = a.b1[i];
      b2s[i] = a.b2[i];
    }
  }
  __syncthreads();

  // staging item of this thread: channel group sg (CPI channels) of a k-step, position sq (0..63)
  const int sg = tid / TQ, sq = tid % TQ;
  float st[PX_NK1][CPI];
  unsigned sok = 0;  // bit ks: k-step ks's item is inside the utterance
  // raw buffer loads: the utterance's rows as the resource (SGPRs), one 32-bit VGPR offset per
  // item and the channel inside the octet as an SGPR offset (64-bit flat addresses per load pushed
  // the kernel past its registers, and the spill reloads' vmcnt waits drained the prefetch)
  auto rsrc_rows = [&](const float* base, int rows) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, rows * a.Tmax * 4, 0x00020000);
  };
  auto stage_load = [&](const Tile& Tl, int ks) {
    const bool xs = ks < 6;
    const int c0 = xs ? 32 * (ks & 1) + CPI * sg : 32 * (ks - 6) + CPI * sg;
    const int off = xs ? (ks / 2 - 1) * a.dil : 0;
    const int cmax = xs ? PW_R : PW_A;
    const __amdgpu_buffer_rsrc_t r = xs ? rsrc_rows(a.x + (long)Tl.b * PW_R * a.Tmax, PW_R)
                                        : rsrc_rows(a.c + (long)Tl.b * PW_A * a.Tmax, PW_A);
    const int t = Tl.t0 + sq + off;
    const bool ok = t >= 0 && t < Tl.T && c0 < cmax;
    sok = ok ? (sok | (1u << ks)) : (sok & ~(1u << ks));
    const int vo = (min(c0, cmax - CPI) * a.Tmax + (ok ? t : 0)) * 4;
#pragma unroll
    for (int c = 0; c < CPI; ++c) st[ks][c] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, vo, c * a.Tmax * 4, 0));
  };
  auto stage_store = [&](int ks) {
    float mx = 0.f, v[CPI];
#pragma unroll
    for (int c = 0; c < CPI; ++c) {
      v[c] = ((sok >> ks) & 1u) ? st[ks][c] : 0.f;
      mx = fmaxf(mx, __builtin_fabsf(v[c]));
    }
    bad |= !(mx < F16_RANGE);
    _Float16* X = Xs + ks * PLANE + sq * PX_XR + CPI * sg;
    if constexpr (CPI == 8) {
      h8 hi, lo;
      split8(v, hi, lo);
      *reinterpret_cast<h8*>(X) = hi;
      *reinterpret_cast<h8*>(X + 32) = lo;
    } else {
      h4 hi, lo;
      split4(f32x4{v[0], v[1], v[2], v[3]}, hi, lo);  // bit-identical to split8 per element
      *reinterpret_cast<h4*>(X) = hi;
      *reinterpret_cast<h4*>(X + 32) = lo;
    }
  };
  float res[MI][4][4];
  auto res_load = [&](const Tile& Tl) {
    // the first half of the waves hold conv1x1_out rows (residual x), the rest skip rows (the
    // running skip sum)
    const bool outw = wm < NW / 2;
    const __amdgpu_buffer_rsrc_t r = rsrc_rows((outw ? a.x : a.skip) + (long)Tl.b * 64 * a.Tmax, 64);
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ch = wm * 16 * MI + mi * 16 + 4 * (lane >> 4) + j - (outw ? 0 : PW_R);
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          const int t = min(Tl.t0 + nb + ni * 16, Tl.T - 1);
          res[mi][j][ni] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (ch * a.Tmax + t) * 4, 0, 0));
        }
      }
  };
  f32x4 am[MI][4], ac[MI][4];
  // B operands two n-tiles at a time (16 VGPRs instead of 32: the kernel is at its register limit)
  auto kstep = [&](const _Float16* X, const h8 (&w)[MI][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int n2 = 0; n2 < 4; n2 += 2) {
      h8 bh[2], bl[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const _Float16* q = X + (nb + (n2 + u) * 16) * PX_XR + kg;
        bh[u] = *reinterpret_cast<const h8*>(q);
        bl[u] = *reinterpret_cast<const h8*>(q + 32);
      }
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int u = 0; u < 2; ++u) mfma_x3(w[mi][0], w[mi][1], bh[u], bl[u], am[mi][n2 + u], ac[mi][n2 + u]);
    }
  };

  int t = blockIdx.x;
  if (t >= ntiles) return;
  Tile cur = tile_of(t);
#pragma unroll
  for (int ks = 0; ks < PX_NK1; ++ks) stage_load(cur, ks);
  for (;;) {
#pragma unroll
    for (int ks = 0; ks < PX_NK1; ++ks) stage_store(ks);
    res_load(cur);
    lds_barrier();
    const int tn = t + (int)gridDim.x;
    const bool more = tn < ntiles;
    const Tile nxt = more ? tile_of(tn) : cur;
    // unconditional (the last tile reloads itself): a conditional load would make the compiler
    // count none of them at its merge, and the epilogue's waits for the residual operands would
    // then drain these too
#pragma unroll
    for (int ks = 0; ks < PX_NK1; ++ks) stage_load(nxt, ks);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) am[mi][ni] = ac[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < PX_NK1; ++ks) kstep(Xs + ks * PLANE, w1[ks]);
    // gate: rows R = 16 MI wm + 16 mi + 4 (lane >> 4) + j, pairs (R, R + 1) -> z[R / 2]
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      const int R = wm * 16 * MI + mi * 16 + 4 * (lane >> 4);
      const int zc = R >> 1;
      _Float16* Z = Zs + (zc >> 5) * PLANE + (zc & 31);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int q = nb + ni * 16;
        f32x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = x3_value(am[mi][ni][j], ac[mi][ni][j]);
        h2_ zh, zl;
        split2(f32x2_{pw_gate(v[0] + b1s[R], v[1] + b1s[R + 1]), pw_gate(v[2] + b1s[R + 2], v[3] + b1s[R + 3])}, zh,
               zl);
        *reinterpret_cast<h2_*>(Z + q * PX_XR) = zh;
        *reinterpret_cast<h2_*>(Z + q * PX_XR + 32) = zl;
        am[mi][ni] = ac[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    lds_barrier();
#pragma unroll
    for (int ks = 0; ks < PX_NK2; ++ks) {
      h8 w2[MI][2];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) {
        const h8* q = W2s + (((MI * wm + mi) * PX_NK2 + ks) * 64 + lane) * 2;
        w2[mi][0] = q[0];
        w2[mi][1] = q[1];
      }
      kstep(Zs + ks * PLANE, w2);
    }
    // x' = (out + b + x) * 0.25 (parallel_wavegan.py:85); skip (+)= s + b. Buffer stores: the
    // utterance's rows as the resource, one 32-bit offset per element (the 64-bit flat address
    // arithmetic per store was a sizeable share of the tile's VALU issue)
    {
      const bool outw = wm * 16 * MI < PW_R;  // a wave's rows are all x' rows or all skip rows
      const __amdgpu_buffer_rsrc_t orr = rsrc_rows((outw ? a.xn : a.skip) + (long)cur.b * 64 * a.Tmax, 64);
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int R = wm * 16 * MI + mi * 16 + 4 * (lane >> 4) + j;
          const int row = (outw ? R : R - PW_R) * a.Tmax;
#pragma unroll
          for (int ni = 0; ni < 4; ++ni) {
            const int tt = cur.t0 + nb + ni * 16;
            if (tt >= cur.T) continue;
            const float v = x3_value(am[mi][ni][j], ac[mi][ni][j]) + b2s[R];
            const float o = outw ? (v + res[mi][j][ni]) * 0.25f : (a.first ? v : res[mi][j][ni] + v);
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(o), orr, (row + tt) * 4, 0, 0);
          }
        }
      }
    }
    if (!more) break;
    lds_barrier();  // every wave is done with this tile's planes
    cur = nxt;
    t = tn;
  }
  if (bad) __hip_atomic_fetch_or(oflow, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

void launch_pw_layer_x3(const float* x, const float* c, float* xn, float* skip, const void* W1x, const float* b1,
                        const void* W2x, const float* b2, const int* lens, const int* h_lens, int len_add, int hop,
                        int Tmax, int dil, int first, int B, unsigned* oflow, hipStream_t st) {
  TTS_CHECK(W1x && W2x && oflow, "pwgan split-f16: weights / range flag missing");
  PwLayerArgs a{x, c, xn, skip, nullptr, b1, nullptr, b2, lens, nullptr, len_add, hop, Tmax, dil, first};
  static const int var = [] {
    const char* e = std::getenv("TTS_PWGAN_TILE");
    return e ? std::atoi(e) : 0;
  }();
  // the persistent kernel addresses a row block of the (B, 80, Tmax) features with 32-bit buffer
  // offsets: utterances past 2^31 bytes per row block (~26 k frames at hop 256) take the per-tile
  // kernel, whose offsets are 64-bit
  const bool off32 = (long)PW_A * Tmax * 4 < (1L << 31);
  if (B <= 64 && h_lens && var != 1 && off32) {  // persistent, weights in registers (TTS_PWGAN_TILE=1: the per-tile kernel)
    long ntiles = 0;
    for (int b = 0; b < B; ++b) ntiles += ((long)(h_lens[b] + len_add) * hop + 63) / 64;
    TTS_CHECK(ntiles < (1L << 30), "pwgan: too many tiles");
    if (ntiles == 0) return;
    constexpr int lds = (PX_NK1 + 2) * 64 * PX_XR * 2 + 8 * PX_NK2 * 64 * 32;
    const int grid = (int)std::min<long>(ntiles, device_cu_count());
    if (var == 2) {  // TTS_PWGAN_TILE=2: 4 waves, 2 m-tiles each
      ensure_dyn_lds((const void*)pw_layer_x3p_kernel<4>, lds);
      pw_layer_x3p_kernel<4><<<grid, 256, lds, st>>>(a, W1x, W2x, oflow, B, (int)ntiles);
    } else {
      ensure_dyn_lds((const void*)pw_layer_x3p_kernel<8>, lds);
      pw_layer_x3p_kernel<8><<<grid, 512, lds, st>>>(a, W1x, W2x, oflow, B, (int)ntiles);
    }
    HIP_OK(hipGetLastError());
    return;
  }
  // per-tile kernel (B > 64, very long utterances, or TTS_PWGAN_TILE=1): one 4-wave workgroup per tile of 64 positions
  constexpr int WN = 1;
  const dim3 grid((Tmax + 64 * WN - 1) / (64 * WN), B);
  pw_layer_x3_kernel<WN><<<grid, 256 * WN, 0, st>>>(a, W1x, W2x, oflow);
  HIP_OK(hipGetLastError());
}

// host packing: m1 (128 x 272: 3 taps x 64 x-channels, then 80 aux) and m2 (128 x 64)
void pack_pw_layer_x3(const std::vector<float>& m1, const std::vector<float>& m2, std::vector<uint16_t>& w1x,
                      std::vector<uint16_t>& w2x) {
  const int K1 = 3 * PW_R + PW_A;
  w1x = pack_split_a(8, PX_NK1, [&](int m, int k) -> float {
    const int ks = k / 32, kk = k % 32;
    if (ks < 6) return m1[(size_t)m * K1 + (ks / 2) * PW_R + 32 * (ks & 1) + kk];
    const int ch = 32 * (ks - 6) + kk;
    return ch < PW_A ? m1[(size_t)m * K1 + 3 * PW_R + ch] : 0.f;
  });
  w2x = pack_split_a(8, PX_NK2, [&](int m, int k) -> float { return m2[(size_t)m * (PW_G / 2) + k]; });
}
