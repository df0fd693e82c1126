// Generic Conv1d / polyphase ConvTranspose1d on the gfx950 f16 MFMA with split-f16 operands
// (split16.h): the fp32 conv of conv.hip at 5.3x the fp32 MFMA issue rate, fp32-accurate.
//
// Same implicit GEMM as conv.hip (M = output channels, N = output positions of one phase,
// K = Cin x taps) and the same epilogue (conv_epi.h), so every ConvBNBlock / MelGAN / Glow conv
// the library runs can take this path. Differences, all forced by v_mfma_f32_16x16x32_f16:
//   k-step     32 input channels of one tap (the fp32 kernel's k-chunk is 4 channels);
//              Cin is zero-padded to a multiple of 32 in the packed weights and at staging.
//   weights    pre-split on the host into A fragments [co16][k-step][lane][hi 8 | lo 8]
//              (32 B per lane per 16 x 32 block), streamed from L2 through an RS-slot register
//              ring over the flattened (chunk, tap) sequence, reloaded in place after use.
//   staging    per 32-channel chunk, TQ + span rows of the (padded, activated) input, split
//              into hi / lo and stored position-major [pos][32 hi | 32 lo | 16 pad] (160 B):
//              a lane's B operand (8 consecutive channels at one position) is one ds_read_b128
//              and a tap is a row offset. Double-buffered: chunk c+1's global loads are in
//              flight during chunk c's MFMAs, one barrier per chunk.
//   range      staged activations outside the f16 range set *oflow (split16.h); the host then
//              re-runs the call on the fp32 kernels. Weights are range-checked at pack time.
//   placement  a 1-D grid dealt so that the workgroups of one XCD (blockIdx % 8) take a
//              contiguous run of the output-channel-major tile list: each XCD's L2 holds the
//              weights of ~1/8 of the output channels instead of all of them.
#include "common.h"
#include "conv_epi.h"
#include "split16.h"

namespace {
constexpr int CX_XR = 80;  // staging row, halves: 32 hi | 32 lo | 16 pad (160 B)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t cx_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}
}  // namespace

template <int MI, int NI, int WM, int WN, int KT, int RS>
__global__ __launch_bounds__(64 * WM * WN) void conv_x3_kernel(ConvArgs a, int nq, int nco, int nz) {
  constexpr int NTHR = 64 * WM * WN;
  constexpr int TC = 16 * MI * WM, TQ = 16 * NI * WN;
  constexpr int SPT = (4 * (TQ + CONV_MAX_SPAN) + NTHR - 1) / NTHR;  // staging items per thread
  extern __shared__ __attribute__((aligned(16))) _Float16 shx[];

  // XCD-aware deal: physical block p runs logical tile (p % 8) * per + p / 8 of the
  // output-channel-major list (co, z, q)
  const int ntile = nq * nco * nz;
  const int per = (ntile + 7) / 8;
  const int w = (int)(blockIdx.x % 8) * per + (int)(blockIdx.x / 8);
  if (w >= ntile) return;
  const int cot = w / (nq * nz);
  const int rem = w - cot * nq * nz;
  const int z = rem / nq;
  const int qt = rem - z * nq;

  const int ph = z % a.nphase;
  const int b = z / a.nphase;
  const int base = a.lens[b] + a.len_add;
  const int Lq = base * a.q_mul;
  const int q0 = qt * TQ;
  if (q0 >= Lq) return;
  const int co0 = cot * TC;
  const int Lin = base * a.in_mul;
  const int dil = a.dil;
  const int span = (KT - 1) * dil;
  const int ROWS = TQ + span;
  _Float16* X0 = shx;
  _Float16* X1 = shx + ROWS * CX_XR;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int nb = wn * 16 * NI + (lane & 15);  // this lane's B column (position) for ni = 0
  const int kg = 8 * (lane >> 4);             // this lane's channel offset inside a k-step
  const int NCH = (a.Cin + 31) / 32;
  const int NKS = NCH * KT;
  const int mtiles = (a.Cout + 15) / 16;
  bool bad = false;

  // ---- staging: item e = (channel octet g, row), rows fastest (coalesced along time) ----
  const int i0 = q0 - a.pad_left[ph];
  const bool interior = (a.rep_pad == 0) && i0 >= 0 && i0 + ROWS <= Lin;
  const int rawL = a.lens[b];
  const int Lsrc = a.rep_pad ? rawL : Lin;
  int srow[SPT], sg[SPT];
#pragma unroll
  for (int j = 0; j < SPT; ++j) {
    const int e = tid + NTHR * j;
    sg[j] = e / ROWS;
    srow[j] = e - sg[j] * ROWS;
  }
  float st[SPT][8];
  auto stage_load = [&](int ch) {
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      const int g = min(sg[j], 3);
      int c0 = 32 * ch + 8 * g;
      c0 = min(c0, a.Cin - 8);  // past Cin: loaded (clamped) but stored as zero
      const bool first = c0 < a.src[0].C;
      const ConvSrc& S = first ? a.src[0] : a.src[1];
      const int cs = first ? c0 : c0 - a.src[0].C;
      int i = i0 + srow[j];
      bool valid = true;
      if (!interior) {
        i = map_pad_index(i, Lin, a.pad_mode, valid);
        if (a.rep_pad) i -= a.rep_pad;
      }
      i = i < 0 ? 0 : (i >= Lsrc ? Lsrc - 1 : i);
      const float* p = S.ptr + (long)b * S.sb + (long)cs * S.sc + (long)i * S.st;
      if (S.sc == 1 && ((S.st & 3) == 0) && ((reinterpret_cast<uintptr_t>(S.ptr) & 15) == 0)) {
        const float4 u = *reinterpret_cast<const float4*>(p);
        const float4 v = *reinterpret_cast<const float4*>(p + 4);
        st[j][0] = u.x, st[j][1] = u.y, st[j][2] = u.z, st[j][3] = u.w;
        st[j][4] = v.x, st[j][5] = v.y, st[j][6] = v.z, st[j][7] = v.w;
      } else {
#pragma unroll
        for (int c = 0; c < 8; ++c) st[j][c] = p[(long)c * S.sc];
      }
      if (!valid) {
#pragma unroll
        for (int c = 0; c < 8; ++c) st[j][c] = 0.f;
      }
    }
  };
  auto stage_store = [&](_Float16* X, int ch) {
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      const int g = sg[j], row = srow[j];
      if (g < 4) {
        const int c0 = 32 * ch + 8 * g;
        const bool real = c0 < a.Cin;
        const bool first = min(c0, a.Cin - 8) < a.src[0].C;
        const int act = first ? a.src[0].act : a.src[1].act;
        float mx = 0.f;
        h8 hi, lo;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          float v = real ? st[j][c] : 0.f;
          mx = fmaxf(mx, __builtin_fabsf(v));
          if (act) v = lrelu02(v);
          _Float16 h, l;
          split_fast(v, h, l);
          hi[c] = h;
          lo[c] = l;
        }
        bad |= !(mx < F16_RANGE);  // |lrelu(v)| <= |v|
        *reinterpret_cast<h8*>(X + row * CX_XR + 8 * g) = hi;
        *reinterpret_cast<h8*>(X + row * CX_XR + 32 + 8 * g) = lo;
      }
    }
  };

  // ---- weights: RS-slot ring over the flattened k-step sequence ----
  const __amdgpu_buffer_rsrc_t wr = cx_rsrc(reinterpret_cast<const char*>(a.W16) + (long)ph * a.w16_phase_stride);
  const int wlo = lane * 32;
  const int mt0 = co0 / 16 + wm * MI;
  h8 ring[RS][MI][2];
  auto wload = [&](h8 (&r)[MI][2], int seq) {
    const int ks = min(seq, NKS - 1);
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      const int mt = min(mt0 + mi, mtiles - 1);  // rows past Cout: discarded by the epilogue
      const int so = (mt * NKS + ks) * 2048;
      r[mi][0] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(wr, wlo, so, 0));
      r[mi][1] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(wr, wlo + 16, so, 0));
    }
  };

  f32x4 am[MI][NI], ac[MI][NI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) am[mi][ni] = ac[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
  stage_load(0);
#pragma unroll
  for (int u = 0; u < RS; ++u) wload(ring[u], u);
  stage_store(X0, 0);
  __syncthreads();
  for (int s0 = 0; s0 < NKS; s0 += RS) {
#pragma unroll
    for (int u = 0; u < RS; ++u) {
      const int seq = s0 + u;
      if (seq < NKS) {
        const int ch = seq / KT;
        const int kq = seq - ch * KT;
        const _Float16* X = (ch & 1) ? X1 : X0;
        if (kq == 0 && ch + 1 < NCH) stage_load(ch + 1);  // in flight during this chunk's MFMAs
        __builtin_amdgcn_sched_barrier(0);
        h8 bh[NI], bl[NI];
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) {
          const _Float16* p = X + (nb + ni * 16 + kq * dil) * CX_XR + kg;
          bh[ni] = *reinterpret_cast<const h8*>(p);
          bl[ni] = *reinterpret_cast<const h8*>(p + 32);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni)
            mfma_x3(ring[u][mi][0], ring[u][mi][1], bh[ni], bl[ni], am[mi][ni], ac[mi][ni]);
        wload(ring[u], seq + RS);  // reload the slot in place after its MFMAs
        if (kq == KT - 1) {
          if (ch + 1 < NCH) stage_store((ch & 1) ? X0 : X1, ch + 1);
          __syncthreads();
        }
      }
    }
  }
  f32x4 acc[MI][NI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[mi][ni][j] = x3_value(am[mi][ni][j], ac[mi][ni][j]);
  conv_epilogue<MI, NI, WN>(a, acc, b, ph, q0, co0, wm, wn, lane);
  if (bad) __hip_atomic_fetch_or(a.oflow, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// tiles {MI, NI, WM, WN}: every wave owns >= 32 output channels x >= 32 positions, so each
// ds_read_b128 of the B operand feeds >= 6 MFMAs and each weight fragment >= 6
//   128 x 64 : 2,4,4,1  (Cout % 128 == 0)      192 x 64 : 3,4,4,1  (Cout == 192)
//    96 x 128: 3,4,2,2  (Cout == 96)             64 x 128: 2,4,2,2  (Cout % 64 == 0)
//    80 x 128: 5,2,1,4  (Cout == 80)             48 x 128: 3,2,1,4  (Cout == 48)
enum { CX_T128 = 0, CX_T192, CX_T96, CX_T64, CX_T80, CX_T48, CX_NONE };

static int cx_tile(int Cout) {
  if (Cout % 128 == 0) return CX_T128;
  if (Cout == 192) return CX_T192;
  if (Cout == 96) return CX_T96;
  if (Cout == 80) return CX_T80;
  if (Cout == 48) return CX_T48;
  if (Cout % 64 == 0) return CX_T64;
  return CX_NONE;
}

bool conv_x3_supported(int Cin, int Cout, int K, int dil) {
  return Cin % 8 == 0 && Cin >= 8 && cx_tile(Cout) != CX_NONE && (K == 1 || K == 2 || K == 3 || K == 5 || K == 7) &&
         (K - 1) * dil <= CONV_MAX_SPAN;
}

template <int MI, int NI, int WM, int WN, int KT>
static void cx_launch(const ConvArgs& a, hipStream_t s) {
  constexpr int TC = 16 * MI * WM, TQ = 16 * NI * WN, RS = 3;
  static bool attr = false;
  if (!attr) {
    HIP_OK(hipFuncSetAttribute((const void*)conv_x3_kernel<MI, NI, WM, WN, KT, RS>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  const int nq = (a.max_q + TQ - 1) / TQ, nco = (a.Cout + TC - 1) / TC, nz = a.B * a.nphase;
  const long ntile = (long)nq * nco * nz;
  TTS_CHECK(ntile < (1L << 30), "conv_x3: grid too large");
  const int per = (int)((ntile + 7) / 8);
  const size_t lds = (size_t)2 * (TQ + (KT - 1) * a.dil) * CX_XR * 2;
  conv_x3_kernel<MI, NI, WM, WN, KT, RS><<<dim3(8 * per), 64 * WM * WN, lds, s>>>(a, nq, nco, nz);
}

template <int MI, int NI, int WM, int WN>
static void cx_taps(const ConvArgs& a, hipStream_t s) {
  switch (a.K) {
    case 1: cx_launch<MI, NI, WM, WN, 1>(a, s); break;
    case 2: cx_launch<MI, NI, WM, WN, 2>(a, s); break;
    case 3: cx_launch<MI, NI, WM, WN, 3>(a, s); break;
    case 5: cx_launch<MI, NI, WM, WN, 5>(a, s); break;
    case 7: cx_launch<MI, NI, WM, WN, 7>(a, s); break;
    default: TTS_CHECK(false, "conv_x3: unsupported tap count");
  }
}

void launch_conv_x3(const ConvArgs& a, hipStream_t s) {
  TTS_CHECK(conv_x3_supported(a.Cin, a.Cout, a.K, a.dil), "conv_x3: unsupported shape");
  TTS_CHECK(a.W16 && a.oflow, "conv_x3: split weights / overflow flag missing");
  TTS_CHECK(a.nphase >= 1 && a.nphase <= 8, "conv: nphase");
  TTS_CHECK(a.nsrc == 1 || a.src[0].C % 8 == 0, "conv_x3: first source's channels must be a multiple of 8");
  if (a.max_q <= 0 || a.B <= 0) return;
  switch (cx_tile(a.Cout)) {
    case CX_T128: cx_taps<2, 4, 4, 1>(a, s); break;
    case CX_T192: cx_taps<3, 4, 4, 1>(a, s); break;
    case CX_T96: cx_taps<3, 4, 2, 2>(a, s); break;
    case CX_T64: cx_taps<2, 4, 2, 2>(a, s); break;
    case CX_T80: cx_taps<5, 2, 1, 4>(a, s); break;
    case CX_T48: cx_taps<3, 2, 1, 4>(a, s); break;
    default: TTS_CHECK(false, "conv_x3: unsupported output channel count");
  }
  HIP_OK(hipGetLastError());
}

// k-step ks = chunk * K + tap covers input channels 32 chunk .. 32 chunk + 31 of that tap
std::vector<uint16_t> pack_conv_x3(const std::vector<float>& Wm, int Cin, int Cout, int K, int nphase,
                                   long* phase_stride_bytes) {
  const int nch = (Cin + 31) / 32, mtiles = (Cout + 15) / 16;
  const size_t per = (size_t)mtiles * nch * K * 64 * 16;  // halves
  std::vector<uint16_t> out(per * nphase);
  for (int ph = 0; ph < nphase; ++ph) {
    const float* w = Wm.data() + (size_t)ph * Cout * Cin * K;
    auto blk = pack_split_a(mtiles, nch * K, [&](int m, int k) -> float {
      const int step = k / 32, ch = step / K, tap = step % K, ci = 32 * ch + k % 32;
      return (m < Cout && ci < Cin) ? w[((size_t)m * Cin + ci) * K + tap] : 0.f;
    });
    std::copy(blk.begin(), blk.end(), out.begin() + per * ph);
  }
  *phase_stride_bytes = (long)(per * 2);
  return out;
}
