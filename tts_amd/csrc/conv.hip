// Generic fp32 MFMA Conv1d / polyphase ConvTranspose1d, and PQMF synthesis (gfx950).
//
// Replaces the ATen conv sequences of: ConvBNBlock (TTS/tts/layers/tacotron2.py:9-44),
// MelGAN generator convs (TTS/vocoder/models/melgan_generator.py:28-78) and PQMF.synthesis
// (TTS/vocoder/layers/pqmf.py:51-56). (ResidualStack blocks have their own fused kernel,
// resblock.hip.)
//
// Implicit GEMM: M = output channels, N = output time positions, K = Cin*taps, on
// v_mfma_f32_16x16x4_f32 (exact fp32). A (weights) is pre-swizzled into MFMA fragment order:
// one contiguous 1 KiB float4 read per wave instruction, L2-resident, prefetched one k-chunk
// ahead. B (activations) is staged per 16-input-channel chunk into LDS with padding / reflection
// / activation resolved at staging time; weights are tap-major inside a chunk (k-chunk = tap,
// see pack_conv), so a tap is a column offset tap * dil into the staged rows; staging is
// register double-buffered -- the global loads of chunk
// c+1 are in flight while chunk c's MFMAs issue -- into two LDS buffers (one barrier per chunk).
// A wave owns MI x NI 16x16 tiles so each LDS read feeds MI MFMAs and each weight fragment NI.
#include "common.h"
#include "conv_epi.h"
#include <algorithm>
#include <stdexcept>


template <int MI, int NI, int WM, int WN>
struct ConvTileCfg {
  static constexpr int TC = 16 * MI * WM;
  static constexpr int TQ = 16 * NI * WN;
  static constexpr int ROWMAX = TQ + CONV_MAX_SPAN + 1;
  static constexpr int SPT = (16 * ROWMAX + 255) / 256;  // staged elements per thread
};

// KT > 0: the tap count is a compile-time constant and the weight fragments run in a ring of KT
// k-chunks (one staging chunk ahead, like the ResidualStack kernel); KT = 0: runtime taps, one
// k-chunk ahead.
template <int MI, int NI, int WM, int WN, int KT = 0>
__global__ __launch_bounds__(256) void conv_mfma_kernel(ConvArgs a) {
  using Cfg = ConvTileCfg<MI, NI, WM, WN>;
  constexpr int TC = Cfg::TC, TQ = Cfg::TQ, SPT = Cfg::SPT;
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
  const int K = KT > 0 ? KT : a.K, dil = a.dil;
  const int span = (K - 1) * dil;
  const int ROW = TQ + span + 1;
  const int XS = (16 * ROW + 3) & ~3;  // one LDS X buffer (floats)
  float* X0 = smem;
  float* X1 = smem + XS;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  const int i0 = q0 - a.pad_left[ph];
  const int nchunks = a.Cin / 16;
  const int nkc_total = a.Cin * K / 16;
  const f32x4* Wv = reinterpret_cast<const f32x4*>(a.W + (long)ph * a.w_phase_stride);
  const int mt0 = (co0 + wm * 16 * MI) / 16;
  const int qb = wn * 16 * NI + (lane & 15);
  const int g4 = 4 * (lane >> 4);
  const int rawL = a.lens[b];
  // interior tile: every staged position is inside [0, Lin) and needs no index remapping
  const bool interior = (a.rep_pad == 0) && i0 >= 0 && i0 + TQ + span <= Lin;

  // this thread's staged (channel, position) pairs, fixed for the whole kernel
  int sc_[SPT], sp_[SPT];
#pragma unroll
  for (int j = 0; j < SPT; ++j) {
    const int e = tid + 256 * j;
    sc_[j] = e / ROW;
    sp_[j] = e - sc_[j] * ROW;
  }
  float st[SPT];
  // every load address is clamped into the source (no per-element branch); zero padding is a
  // select after the load, slots past 16 x (TQ + span) are loaded but never stored
  auto stage_load = [&](int chunk) {
    const int cbase = chunk * 16;
    const bool first = cbase < a.src[0].C;
    const float* sp = first ? a.src[0].ptr : a.src[1].ptr;
    const long sb = first ? a.src[0].sb : a.src[1].sb;
    const int ssc = first ? a.src[0].sc : a.src[1].sc;
    const int sst = first ? a.src[0].st : a.src[1].st;
    const int cs = first ? cbase : cbase - a.src[0].C;
    const float* bp = sp + (long)b * sb + (long)cs * ssc;
    const int Lsrc = a.rep_pad ? rawL : Lin;
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      const int c = min(sc_[j], 15);
      int i = i0 + sp_[j];
      bool valid = true;
      if (!interior) {
        i = map_pad_index(i, Lin, a.pad_mode, valid);
        if (a.rep_pad) i -= a.rep_pad;
      }
      i = i < 0 ? 0 : (i >= Lsrc ? Lsrc - 1 : i);
      const float v = bp[(long)c * ssc + (long)i * sst];
      st[j] = valid ? v : 0.f;
    }
  };
  auto stage_store = [&](float* X, int chunk) {
    const int cbase = chunk * 16;
    const int act = cbase < a.src[0].C ? a.src[0].act : a.src[1].act;
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      const int e = tid + 256 * j;
      if (e < 16 * ROW) X[e] = act ? lrelu02(st[j]) : st[j];
    }
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};

  stage_load(0);
  if constexpr (KT > 0) {
    f32x4 ring[KT][MI];
    auto wload = [&](f32x4 (&r)[MI], int kc) {
      kc = min(kc, nkc_total - 1);
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) r[mi] = Wv[((long)(mt0 + mi) * nkc_total + kc) * 64 + lane];
    };
#pragma unroll
    for (int kq = 0; kq < KT; ++kq) wload(ring[kq], kq);
    stage_store(X0, 0);
    __syncthreads();
    for (int chunk = 0; chunk < nchunks; ++chunk) {
      float* X = (chunk & 1) ? X1 : X0;
      if (chunk + 1 < nchunks) stage_load(chunk + 1);  // in flight during this chunk's MFMAs
      // keep the scheduler from sinking the staging loads down to their LDS stores
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int kq = 0; kq < KT; ++kq) {
        // all 4 x NI operand reads of this k-chunk first (one LDS wait), tap offsets arithmetic
        float bv[4][NI];
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni) bv[s][ni] = X[(g4 + s) * ROW + kq * dil + qb + ni * 16];
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int mi = 0; mi < MI; ++mi)
#pragma unroll
            for (int ni = 0; ni < NI; ++ni) acc[mi][ni] = MFMA16(ring[kq][mi][s], bv[s][ni], acc[mi][ni]);
        // reload the slot in place after its MFMAs (no register rotation, no vmcnt(0))
        wload(ring[kq], (chunk + 1) * KT + kq);
      }
      if (chunk + 1 < nchunks) stage_store((chunk & 1) ? X0 : X1, chunk + 1);
      __syncthreads();
    }
  } else {
    f32x4 Anext[MI];
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) Anext[mi] = Wv[((long)(mt0 + mi) * nkc_total + 0) * 64 + lane];
    stage_store(X0, 0);
    __syncthreads();
    for (int chunk = 0; chunk < nchunks; ++chunk) {
      float* X = (chunk & 1) ? X1 : X0;
      if (chunk + 1 < nchunks) stage_load(chunk + 1);  // in flight during this chunk's MFMAs
      for (int kq = 0; kq < K; ++kq) {
        const int kc = chunk * K + kq;
        f32x4 A[MI];
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) A[mi] = Anext[mi];
        const int kn = min(kc + 1, nkc_total - 1);
#pragma unroll
        for (int mi = 0; mi < MI; ++mi) Anext[mi] = Wv[((long)(mt0 + mi) * nkc_total + kn) * 64 + lane];
        float bv[4][NI];
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni) bv[s][ni] = X[(g4 + s) * ROW + kq * dil + qb + ni * 16];
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int mi = 0; mi < MI; ++mi)
#pragma unroll
            for (int ni = 0; ni < NI; ++ni) acc[mi][ni] = MFMA16(A[mi][s], bv[s][ni], acc[mi][ni]);
      }
      if (chunk + 1 < nchunks) stage_store((chunk & 1) ? X0 : X1, chunk + 1);
      __syncthreads();
    }
  }

  conv_epilogue<MI, NI, WN>(a, acc, b, ph, q0, co0, wm, wn, lane);
}

// tile catalogue: {MI, NI, WM, WN} -> TC x TQ
//   TILE_128x64 : 4,2,2,2   (Cout % 128 == 0: 512, 384, 2048, 128)
//   TILE_64x64  : 2,2,2,2   (Cout % 64 == 0)
//   TILE_192x64 : 3,4,4,1   (Cout == 192)
//   TILE_96x64  : 3,2,2,2   (Cout == 96)
//   TILE_48x128 : 3,2,1,4   (Cout == 48)
//   TILE_80x64  : 5,1,1,4   (Cout == 80)
//   TILE_16x256 : 1,4,1,4   (anything else, Cout padded to 16)
int conv_tile_tc(int tile) {
  switch (tile) {
    case TILE_128x64: return 128;
    case TILE_64x64: return 64;
    case TILE_192x64: return 192;
    case TILE_96x64: return 96;
    case TILE_48x128: return 48;
    case TILE_80x64: return 80;
    default: return 16;
  }
}
static int conv_tile_tq(int tile) {
  switch (tile) {
    case TILE_48x128: return 128;
    case TILE_16x256: return 256;
    default: return 64;
  }
}

int conv_tile_for_cout(int cout) {
  if (cout % 128 == 0) return TILE_128x64;
  if (cout == 192) return TILE_192x64;
  if (cout == 96) return TILE_96x64;
  if (cout % 80 == 0) return TILE_80x64;
  if (cout == 48) return TILE_48x128;
  if (cout % 64 == 0) return TILE_64x64;
  return TILE_16x256;
}

void launch_conv(const ConvArgs& a, int tile, hipStream_t s) {
  TTS_CHECK(a.Cin % 16 == 0, "conv: Cin must be a multiple of 16");
  TTS_CHECK(a.Cout_pad % conv_tile_tc(tile) == 0, "conv: Cout_pad / tile mismatch");
  TTS_CHECK(a.nphase >= 1 && a.nphase <= 8, "conv: nphase");
  TTS_CHECK((a.K - 1) * a.dil <= CONV_MAX_SPAN, "conv: receptive span too large for the generic kernel");
  if (a.max_q <= 0 || a.B <= 0) return;
  int TQ = conv_tile_tq(tile), TC = conv_tile_tc(tile);
  // compile-time-tap variants with a weight ring (tools/conv_bench.hip, postnet 512->512 k5:
  // 128x64 one-ahead 642 us, 64x64 ring5 557 us)
  int variant = -1;
  if (a.K == 5 && tile == TILE_128x64) variant = 0, TC = 64;
  else if (a.K == 5 && tile == TILE_80x64) variant = 1;
  else if (a.K == 2 && tile == TILE_192x64) variant = 3;
  const int span = (a.K - 1) * a.dil;
  const int ROW = TQ + span + 1;
  const size_t lds = (size_t)2 * ((16 * ROW + 3) & ~3) * 4;
  dim3 grid((a.max_q + TQ - 1) / TQ, a.Cout_pad / TC, a.B * a.nphase);
  switch (variant) {
    case 0: conv_mfma_kernel<2, 2, 2, 2, 5><<<grid, 256, lds, s>>>(a); break;
    case 1: conv_mfma_kernel<5, 1, 1, 4, 5><<<grid, 256, lds, s>>>(a); break;
    case 3: conv_mfma_kernel<3, 4, 4, 1, 2><<<grid, 256, lds, s>>>(a); break;
    default:
      switch (tile) {
        case TILE_128x64: conv_mfma_kernel<4, 2, 2, 2><<<grid, 256, lds, s>>>(a); break;
        case TILE_64x64: conv_mfma_kernel<2, 2, 2, 2><<<grid, 256, lds, s>>>(a); break;
        case TILE_192x64: conv_mfma_kernel<3, 4, 4, 1><<<grid, 256, lds, s>>>(a); break;
        case TILE_96x64: conv_mfma_kernel<3, 2, 2, 2><<<grid, 256, lds, s>>>(a); break;
        case TILE_48x128: conv_mfma_kernel<3, 2, 1, 4><<<grid, 256, lds, s>>>(a); break;
        case TILE_80x64: conv_mfma_kernel<5, 1, 1, 4><<<grid, 256, lds, s>>>(a); break;
        default: conv_mfma_kernel<1, 4, 1, 4><<<grid, 256, lds, s>>>(a); break;
      }
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

// ------------------------------------------------------------------- FillList
__global__ __launch_bounds__(256) void fill_list_kernel(FillList f) {
  const int e = blockIdx.y;
  unsigned* p = static_cast<unsigned*>(f.p[e]);
  const long n = f.words[e];
  const unsigned v = f.val[e];
  const long stride = (long)gridDim.x * blockDim.x;
  const long i0 = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if ((reinterpret_cast<uintptr_t>(p) & 15) == 0) {  // 16-byte stores for the aligned bulk
    uint4* q = reinterpret_cast<uint4*>(p);
    const uint4 v4 = make_uint4(v, v, v, v);
    for (long i = i0; i < n / 4; i += stride) q[i] = v4;
    for (long i = (n / 4) * 4 + i0; i < n; i += stride) p[i] = v;
  } else {
    for (long i = i0; i < n; i += stride) p[i] = v;
  }
}

void launch_fills(const FillList& f, hipStream_t s) {
  if (!f.n) return;
  long mx = 0;
  for (int i = 0; i < f.n; ++i) mx = std::max(mx, f.words[i]);
  const int gx = (int)std::min<long>(512, std::max<long>(1, (mx / 4 + 255) / 256));
  fill_list_kernel<<<dim3(gx, f.n), 256, 0, s>>>(f);
  HIP_OK(hipGetLastError());
}
