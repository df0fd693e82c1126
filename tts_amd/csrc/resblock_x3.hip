// Fused MelGAN ResidualStack block (TTS/vocoder/layers/melgan.py:5-39) on the f16 MFMA with
// split-f16 operands (split16.h): fp32-accurate at 5.3x the fp32 MFMA rate.
//   h = conv_k3_dil_d(ReflectionPad(d)(LeakyReLU(x))) + b_d
//   y = [W_1x1 | W_sc] . [lrelu(h); x] + (b_1x1 + b_sc)
// Same structure as the fp32 kernel (resblock.hip): one workgroup owns all C output channels of
// TQ positions, so h never leaves the CU.
//   staging   32 input channels x (TQ + 2d) positions of lrelu(x), reflect-padded per utterance,
//             split into hi / lo f16 and stored position-major ([pos][32 hi | 32 lo | 16 pad]):
//             one lane's B operand (8 consecutive channels of one position) is one ds_read_b128,
//             and the 160-byte row stride keeps those reads bank-conflict free for any tap offset.
//             The centre positions' raw x (shortcut input) go split into HX. Double-buffered:
//             chunk c+1's global loads are in flight during chunk c's MFMAs.
//   phase 1   h = Wd . X over K = 3 taps x C channels (3 MFMAs per product), weights (A operand,
//             pre-split on the host) streamed from L2 through a 3-slot register ring.
//   phase 2   lrelu(h + b_d) split into HX ([pos][2C hi | 2C lo]), then y = Wf . HX, K = 2C.
// Any operand outside the f16 range sets *oflow; the host then re-runs the call in fp32.
#include "common.h"
#include "split16.h"

namespace {
constexpr int X3_DMAX = 27;   // largest dilation (3^3, num_res_blocks <= 4)
constexpr int XR = 80;        // staging row, halves: 32 hi | 32 lo | 16 pad (160 B)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ float lrelu_x3(float v) { return fmaxf(v, 0.2f * v); }  // == lrelu02
}  // namespace

template <int C, int TQ, int WM, int WN>
__global__ __launch_bounds__(64 * WM * WN) void resblock_x3_kernel(ResArgs a) {
  constexpr int NTHR = 64 * WM * WN;
  constexpr int MI = C / 16 / WM;
  constexpr int NI = TQ / 16 / WN;
  static_assert(MI * 16 * WM == C && NI * 16 * WN == TQ, "tile split");
  constexpr int NCH = (C + 31) / 32;     // staging chunks of 32 input channels (C = 48: 16 zero channels)
  constexpr int NK1 = 3 * NCH;           // phase-1 k-steps: (chunk, tap)
  constexpr int NK2 = 2 * C / 32;        // phase-2 k-steps
  static_assert(NK2 * 32 == 2 * C && NK2 % 3 == 0, "phase-2 k-steps: multiple of the 3-slot ring");
  constexpr int HR = 4 * C + 16;         // HX row, halves: 2C hi | 2C lo | 16 pad (8C + 32 bytes)
  constexpr int SPT = (4 * (TQ + 2 * X3_DMAX) + NTHR - 1) / NTHR;  // staging items (8 channels x 1 pos) per thread
  extern __shared__ __attribute__((aligned(16))) _Float16 sh[];

  const int b = blockIdx.y;
  const int L = (a.lens[b] + a.len_add) * a.mul;
  const int q0 = blockIdx.x * TQ;
  if (q0 >= L) return;
  const int d = a.dil;
  const int ROWS = TQ + 2 * d;
  _Float16* X0 = sh;
  _Float16* X1 = sh + ROWS * XR;
  _Float16* HX = sh + 2 * ROWS * XR;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int nb = wn * 16 * NI + (lane & 15);  // this lane's position (B column) for ni = 0
  const int kg = 8 * (lane >> 4);             // this lane's k offset inside a k-step
  const int mt0 = wm * MI;
  bool bad = false;

  // ---- staging: item e = (channel octet g, row); rows fastest so that lanes read consecutive
  //      positions of one channel (coalesced); clamped addresses, no per-element guard
  const __amdgpu_buffer_rsrc_t xr = rsrc(a.x + (long)b * a.sb);  // one utterance: < 2^31 bytes
  const int i0 = q0 - d;
  const bool interior = i0 >= 0 && i0 + ROWS <= L;
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
      int i = i0 + srow[j];
      if (!interior) {  // reflection (torch ReflectionPad1d), then clamp
        if (i < 0) i = -i;
        if (i >= L) i = 2 * (L - 1) - i;
        i = i < 0 ? 0 : (i >= L ? L - 1 : i);
      }
      const int c0 = min(32 * ch + 8 * min(sg[j], 3), C - 8);
      const int vo = (c0 * a.Ls + i) * 4;  // per-lane offset; the 8 channel rows are SGPR offsets
#pragma unroll
      for (int c = 0; c < 8; ++c)
        st[j][c] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, vo, c * a.Ls * 4, 0));
    }
  };
  auto stage_store = [&](_Float16* X, int ch) {
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      const int g = sg[j], row = srow[j];
      if (g < 4) {
        const bool real = 32 * ch + 8 * g < C;  // C = 48: the second chunk's upper half is zero
        float v[8], mx = 0.f;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          v[c] = real ? st[j][c] : 0.f;
          mx = fmaxf(mx, __builtin_fabsf(v[c]));
        }
        bad |= !(mx < F16_RANGE);  // |lrelu(v)| <= |v|: one check covers both splits
        h8 hi, lo;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          _Float16 h, l;
          split_fast(lrelu_x3(v[c]), h, l);
          hi[c] = h;
          lo[c] = l;
        }
        *reinterpret_cast<h8*>(X + row * XR + 8 * g) = hi;
        *reinterpret_cast<h8*>(X + row * XR + 32 + 8 * g) = lo;
        const int p = row - d;
        if (real && p >= 0 && p < TQ) {  // raw x of the centre positions: the shortcut's operand
#pragma unroll
          for (int c = 0; c < 8; ++c) {
            _Float16 h, l;
            split_fast(v[c], h, l);
            hi[c] = h;
            lo[c] = l;
          }
          *reinterpret_cast<h8*>(HX + p * HR + C + 32 * ch + 8 * g) = hi;
          *reinterpret_cast<h8*>(HX + p * HR + 3 * C + 32 * ch + 8 * g) = lo;
        }
      }
    }
  };

  // ---- weights: A fragments [mt][k-step][lane][hi 8 | lo 8], phase 1 then phase 2 as one
  //      sequence through a 3-slot ring, so phase 2's first slots load during phase 1's last
  // buffer loads: the lane's 32 bytes are a VGPR offset, the (m-tile, k-step) block an SGPR one
  const __amdgpu_buffer_rsrc_t wdr = rsrc(a.Wd16), wfr = rsrc(a.Wf16);
  const int wlo = lane * 32;
  h8 ring[3][MI][2];
  auto wload = [&](h8 (&r)[MI][2], int seq) {
    const bool p1 = seq < NK1;
    const __amdgpu_buffer_rsrc_t wr = p1 ? wdr : wfr;
    const int nk = p1 ? NK1 : NK2;
    const int ks = p1 ? seq : min(seq - NK1, NK2 - 1);
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      const int so = ((mt0 + mi) * nk + ks) * 2048;
      r[mi][0] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(wr, wlo, so, 0));
      r[mi][1] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(wr, wlo + 16, so, 0));
    }
  };

  // ---------------- phase 1: h = Wd . lrelu(x) ----------------
  f32x4 am[MI][NI], ac[MI][NI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) am[mi][ni] = ac[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
  stage_load(0);
#pragma unroll
  for (int u = 0; u < 3; ++u) wload(ring[u], u);
  stage_store(X0, 0);
  __syncthreads();
  for (int ch = 0; ch < NCH; ++ch) {
    const _Float16* X = (ch & 1) ? X1 : X0;
    if (ch + 1 < NCH) stage_load(ch + 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kq = 0; kq < 3; ++kq) {
      h8 bh[NI], bl[NI];
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        const _Float16* p = X + (nb + ni * 16 + kq * d) * XR + kg;
        bh[ni] = *reinterpret_cast<const h8*>(p);
        bl[ni] = *reinterpret_cast<const h8*>(p + 32);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) mfma_x3(ring[kq][mi][0], ring[kq][mi][1], bh[ni], bl[ni], am[mi][ni], ac[mi][ni]);
      wload(ring[kq], (ch + 1) * 3 + kq);
    }
    if (ch + 1 < NCH) stage_store((ch & 1) ? X0 : X1, ch + 1);
    __syncthreads();
  }
  // lrelu(h + b_d), split, into HX[pos][0:C) (hi) and HX[pos][2C:3C) (lo)
#pragma unroll
  for (int mi = 0; mi < MI; ++mi) {
    const int co = (mt0 + mi) * 16 + 4 * (lane >> 4);
    float bd[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bd[j] = a.bd[co + j];
#pragma unroll
    for (int ni = 0; ni < NI; ++ni) {
      h4 hi, lo;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        _Float16 h, l;
        split_dev(lrelu_x3(x3_value(am[mi][ni][j], ac[mi][ni][j]) + bd[j]), h, l, bad);
        hi[j] = h;
        lo[j] = l;
      }
      const int p = nb + ni * 16;
      *reinterpret_cast<h4*>(HX + p * HR + co) = hi;
      *reinterpret_cast<h4*>(HX + p * HR + 2 * C + co) = lo;
      am[mi][ni] = ac[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  __syncthreads();
  // ---------------- phase 2: y = [W1 | Wsc] . [lrelu(h); x] ----------------
  for (int k0 = 0; k0 < NK2; k0 += 3) {
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int kc = k0 + u;
      h8 bh[NI], bl[NI];
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        const _Float16* p = HX + (nb + ni * 16) * HR + kc * 32 + kg;
        bh[ni] = *reinterpret_cast<const h8*>(p);
        bl[ni] = *reinterpret_cast<const h8*>(p + 2 * C);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) mfma_x3(ring[u][mi][0], ring[u][mi][1], bh[ni], bl[ni], am[mi][ni], ac[mi][ni]);
      wload(ring[u], NK1 + kc + 3);
    }
  }
  float* yb = a.y + (long)b * a.sb;
#pragma unroll
  for (int mi = 0; mi < MI; ++mi) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int co = (mt0 + mi) * 16 + 4 * (lane >> 4) + j;
      const float bf = a.bf[co];
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        const int q = q0 + nb + ni * 16;
        if (q < L) yb[(long)co * a.Ls + q] = x3_value(am[mi][ni][j], ac[mi][ni][j]) + bf;
      }
    }
  }
  if (bad) __hip_atomic_fetch_or(a.oflow, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int C, int TQ, int WM, int WN>
static void launch_rbx3(const ResArgs& a, hipStream_t s) {
  const int ROWS = TQ + 2 * a.dil;
  const size_t lds = ((size_t)2 * ROWS * XR + (size_t)TQ * (4 * C + 16)) * 2;
  static bool attr = false;
  if (!attr) {
    HIP_OK(hipFuncSetAttribute((const void*)resblock_x3_kernel<C, TQ, WM, WN>,
                               hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  TTS_CHECK(lds <= 160 * 1024, "resblock_x3: LDS tile too large");
  dim3 grid((a.max_q + TQ - 1) / TQ, a.B);
  resblock_x3_kernel<C, TQ, WM, WN><<<grid, 64 * WM * WN, lds, s>>>(a);
}

bool resblock_x3_supported(int C) { return C == 192 || C == 96 || C == 48; }

// host packing of one block's split weights: Wd (C, C, 3) [co][ci][k] and Wf (C, 2C) [co][k]
void pack_resblock_x3(const std::vector<float>& wd, const std::vector<float>& wf, int C,
                      std::vector<uint16_t>& wd16, std::vector<uint16_t>& wf16) {
  const int nch = (C + 31) / 32;
  wd16 = pack_split_a(C / 16, 3 * nch, [&](int m, int k) -> float {
    const int step = k / 32, ch = step / 3, kq = step % 3, ci = 32 * ch + k % 32;
    return ci < C ? wd[((size_t)m * C + ci) * 3 + kq] : 0.f;
  });
  wf16 = pack_split_a(C / 16, 2 * C / 32, [&](int m, int k) -> float { return wf[(size_t)m * 2 * C + k]; });
}

void launch_resblock_x3(const ResArgs& a, int C, hipStream_t s) {
  TTS_CHECK(a.dil >= 1 && a.dil <= X3_DMAX, "resblock: dilation must be in [1, 27] (num_res_blocks <= 4)");
  TTS_CHECK(a.Wd16 && a.Wf16 && a.oflow, "resblock_x3: split weights / overflow flag missing");
  if (a.max_q <= 0 || a.B <= 0) return;
  switch (C) {
    // tiles from tools/rbx3_bench.hip (C2 shapes): 12 waves, one m-tile (or two) per wave
    case 192: launch_rbx3<192, 64, 12, 1>(a, s); break;
    case 96: launch_rbx3<96, 128, 6, 2>(a, s); break;
    case 48: launch_rbx3<48, 128, 3, 4>(a, s); break;
    default: TTS_CHECK(false, "resblock_x3: unsupported channel count");
  }
  HIP_OK(hipGetLastError());
}
