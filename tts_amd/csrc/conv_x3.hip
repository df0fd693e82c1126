// Generic Conv1d / polyphase ConvTranspose1d on the gfx950 f16 MFMA with split-f16 operands
// (split16.h): the fp32 conv of conv.hip at 5.3x the fp32 MFMA issue rate, fp32-accurate.
//
// Same implicit GEMM as conv.hip (M = output channels, N = output positions of one phase,
// K = Cin x taps) and the same epilogue (conv_epi.h), so every ConvBNBlock / MelGAN / Glow conv
// the library runs can take this path. Differences, all forced by v_mfma_f32_16x16x32_f16:
//   k-step     32 input channels of one tap (the fp32 kernel's k-chunk is 4 channels);
//              Cin is zero-padded to a multiple of 32 in the packed weights and at staging.
//   weights    pre-split on the host into A fragments [co16][k-step][lane][hi 8 | lo 8]
//              (32 B per lane per 16 x 32 block), streamed from L2 through a register ring of
//              one (k >= 5) or two (k <= 3) chunks of taps, each slot reloaded in place after use.
//   staging    per 32-channel chunk (one source), TQ + span rows of the (padded, activated) input, split
//              into hi / lo and stored position-major [pos][32 hi | 32 lo | 16 pad] (160 B):
//              a lane's B operand (8 consecutive channels at one position) is one ds_read_b128
//              and a tap is a row offset. Two LDS buffers and two register sets: chunk c+2's
//              global loads are in flight during chunk c's MFMAs, one barrier per chunk.
//   range      staged activations outside the f16 range set *oflow (split16.h); the host then
//              re-runs the call on the fp32 kernels. Weights are range-checked at pack time.
//   ConvT      merged_u > 0: the u phases of a ConvTranspose1d(k = 2u, stride u, padding u/2) as
//              ONE GEMM (rows co * u + phase, both tap pairs expressed as input q - 1, q): the
//              input is staged once instead of u times and a workgroup writes whole runs of
//              consecutive output samples instead of every u-th one.
//   placement  a 1-D grid dealt so that the workgroups of one XCD (blockIdx % 8) take a
//              contiguous run of the output-channel-major tile list: each XCD's L2 holds the
//              weights of ~1/8 of the output channels instead of all of them.
#include "common.h"
#include "conv_epi.h"
#include "split16.h"

#include <cstdlib>
#include <algorithm>
#include <mutex>
#include <map>

namespace {
constexpr int CX_XR = 80;  // staging row, halves: 32 hi | 32 lo | 16 pad (160 B)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t cx_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}
}  // namespace

template <int MI, int NI, int WM, int WN, int KT, int RS, int SD>
__global__ __launch_bounds__(64 * WM * WN) void conv_x3_kernel(ConvArgs a, int nq, int nco, int nz) {
  constexpr int NTHR = 64 * WM * WN;
  constexpr int TC = 16 * MI * WM, TQ = 16 * NI * WN;
  constexpr int SPT = (4 * (TQ + CONV_MAX_SPAN) + NTHR - 1) / NTHR;  // staging items per thread
  static_assert(RS == KT || RS == 2 * KT, "weight ring: one or two chunks of taps");
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
  const int Lq = base * a.q_mul + (a.merged_u ? 1 : 0);
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
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int nb = wn * 16 * NI + (lane & 15);  // this lane's B column (position) for ni = 0
  const int kg = 8 * (lane >> 4);             // this lane's channel offset inside a k-step
  const int NCH = (a.Cin + 31) / 32;
  const int NKS = NCH * KT;
  const int mtiles = (a.Cout + 15) / 16;
  bool bad = false;

  // ---- staging: item e = (channel octet g, row), rows fastest (coalesced along time). An item's
  //      position (and its padding) is fixed for the whole kernel: one VGPR byte offset per item;
  //      the chunk and the channel inside the octet are SGPR offsets of raw buffer loads whose
  //      range is this utterance's source (channels past Cin are zeroed at the store) ----
  const ConvSrc& S = a.src[0];
  const int i0 = q0 - a.pad_left[ph];
  const bool interior = (a.rep_pad == 0) && i0 >= 0 && i0 + ROWS <= Lin;
  const int rawL = a.lens[b];
  const int Lsrc = a.rep_pad ? rawL : Lin;
  const bool tmajor = S.sc == 1;  // 8 channels of a position are contiguous: two 16-byte loads
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(S.ptr + (long)b * S.sb), 0,
      (int)min((long)0x7fffffff, ((long)(S.C - 1) * S.sc + (long)(Lsrc - 1) * S.st + 1) * 4), 0x00020000);
  int voff[SPT], sgv[SPT], srow[SPT];
  bool sval[SPT];
#pragma unroll
  for (int j = 0; j < SPT; ++j) {
    const int e = tid + NTHR * j;
    const int g = e / ROWS;
    srow[j] = e - g * ROWS;
    sgv[j] = g;
    int i = i0 + srow[j];
    bool valid = true;
    if (!interior) {
      i = map_pad_index(i, Lin, a.pad_mode, valid);
      if (a.rep_pad) i -= a.rep_pad;
    }
    i = i < 0 ? 0 : (i >= Lsrc ? Lsrc - 1 : i);
    sval[j] = valid && g < 4;
    voff[j] = (min(g, 3) * 8 * S.sc + i * S.st) * 4;
  }
  const int act = S.act;
  float st[SD][SPT][8];
  auto stage_load = [&](float (&sr)[SPT][8], int ch) {
    const int cb = 32 * ch * S.sc * 4;  // uniform
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      if (tmajor) {
        const f32x4 u = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, voff[j], cb, 0));
        const f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, voff[j] + 16, cb, 0));
#pragma unroll
        for (int c = 0; c < 4; ++c) sr[j][c] = u[c], sr[j][4 + c] = v[c];
      } else {
#pragma unroll
        for (int c = 0; c < 8; ++c)
          sr[j][c] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, voff[j], cb + c * S.sc * 4, 0));
      }
    }
  };
  auto stage_store = [&](_Float16* X, const float (&sr)[SPT][8], int ch) {
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      if (sgv[j] < 4) {
        const bool keep = sval[j] && 32 * ch + 8 * sgv[j] < a.Cin;  // zero padding; channels past Cin
        float mx = 0.f, v[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          v[c] = keep ? sr[j][c] : 0.f;
          mx = fmaxf(mx, __builtin_fabsf(v[c]));
          if (act) v[c] = lrelu02(v[c]);
        }
        bad |= !(mx < F16_RANGE);  // |lrelu(v)| <= |v|
        h8 hi, lo;
        split8(v, hi, lo);
        *reinterpret_cast<h8*>(X + srow[j] * CX_XR + 8 * sgv[j]) = hi;
        *reinterpret_cast<h8*>(X + srow[j] * CX_XR + 32 + 8 * sgv[j]) = lo;
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
  // SD = 2: staging runs two chunks ahead (chunk c's global loads are issued after chunk c - 3's
  // MFMAs into register set c & 1 and stored to LDS buffer c & 1 after chunk c - 1's);
  // SD = 1: one chunk ahead (loads issued before chunk c - 1's MFMAs), one register set
  stage_load(st[0], 0);
#pragma unroll
  for (int u = 0; u < RS; ++u) wload(ring[u], u);
  stage_store(X0, st[0], 0);
  if constexpr (SD == 2) {
    if (NCH > 1) stage_load(st[1], 1);
    if (NCH > 2) stage_load(st[0], 2);
  }
  lds_barrier();
  for (int ch0 = 0; ch0 < NCH; ch0 += 2) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int ch = ch0 + p;
      if (ch < NCH) {
        const _Float16* X = p ? X1 : X0;
        if constexpr (SD == 1) {
          if (ch + 1 < NCH) stage_load(st[0], ch + 1);
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int kq = 0; kq < KT; ++kq) {
          constexpr bool TWO = RS == 2 * KT;
          const int slot = TWO ? p * KT + kq : kq;
          h8 bh[NI], bl[NI];
#pragma unroll
          for (int ni = 0; ni < NI; ++ni) {
            const _Float16* q = X + (nb + ni * 16 + kq * dil) * CX_XR + kg;
            bh[ni] = *reinterpret_cast<const h8*>(q);
            bl[ni] = *reinterpret_cast<const h8*>(q + 32);
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int mi = 0; mi < MI; ++mi)
#pragma unroll
            for (int ni = 0; ni < NI; ++ni)
              mfma_x3(ring[slot][mi][0], ring[slot][mi][1], bh[ni], bl[ni], am[mi][ni], ac[mi][ni]);
          wload(ring[slot], ch * KT + kq + RS);  // reload the slot in place after its MFMAs
          __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (SD == 2) {
          if (ch + 1 < NCH) stage_store(p ? X0 : X1, st[p ^ 1], ch + 1);
          if (ch + 3 < NCH) stage_load(st[p ^ 1], ch + 3);
        } else {
          if (ch + 1 < NCH) stage_store(p ? X0 : X1, st[0], ch + 1);
        }
        lds_barrier();
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
  // phase-merged ConvTranspose, row m = co * u + phase; a lane's 4 rows (j) are 4 consecutive
  // phases of one co (u >= 4) or phases 0, 1 of two co (u = 2), written as vectors of consecutive
  // output samples (the scalar form spent a third of the u = 2 kernel on its stores)
  const bool vec = a.merged_u && a.ot == 1 && (a.oc & 3) == 0 && (a.ob & 3) == 0 &&
                   (reinterpret_cast<uintptr_t>(a.out) & 15) == 0 && a.Cout % 16 == 0;
  if (vec && a.merged_u % 4 == 0) {
    // u % 8 == 0: phases phs0 .. phs0 + 3 all on one side of u / 2 -> one 16-byte store;
    // u == 4: two pairs (0, 1 at q) and (2, 3 at q - 1) -> two 8-byte stores
    const int u = a.merged_u, L = Lin;
    float* ob = a.out + (long)b * a.ob;
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      const int m0 = co0 + wm * 16 * MI + mi * 16 + 4 * (lane >> 4);
      if (m0 >= a.Cout) continue;
      const int co = m0 / u, phs0 = m0 - co * u;
      const int hi0 = 2 * phs0 >= u, hi1 = 2 * (phs0 + 2) >= u;
      const f32x4 bias{a.bias[m0], a.bias[m0 + 1], a.bias[m0 + 2], a.bias[m0 + 3]};
      float* orow = ob + (long)co * a.oc;
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        const int q = q0 + nb + ni * 16;
        const f32x4 v = acc[mi][ni] + bias;
        if (u % 8 == 0) {
          if (q - hi0 >= 0 && q - hi0 < L) *reinterpret_cast<f32x4*>(orow + (long)(q - hi0) * u + phs0) = v;
        } else {
          typedef float f2 __attribute__((ext_vector_type(2)));
          if (q - hi0 >= 0 && q - hi0 < L) *reinterpret_cast<f2*>(orow + (long)(q - hi0) * u + phs0) = f2{v[0], v[1]};
          if (q - hi1 >= 0 && q - hi1 < L) *reinterpret_cast<f2*>(orow + (long)(q - hi1) * u + phs0 + 2) = f2{v[2], v[3]};
        }
      }
    }
  } else if (vec && a.merged_u == 2) {
    // u = 2: position q holds out[2q] (phase 0) and out[2q - 1] (phase 1). The aligned pair
    // (2q, 2q + 1) takes phase 1 from the next position: the next lane of the 16-lane row, or
    // lane 0 of the next n-tile; a wave's last position stores out[2q] alone and its first
    // position out[2q - 1] alone (the neighbouring wave / workgroup holds their partners)
    typedef float f2 __attribute__((ext_vector_type(2)));
    const int L = Lin;
    float* ob = a.out + (long)b * a.ob;
    const int r = lane & 15;
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      const int m0 = co0 + wm * 16 * MI + mi * 16 + 4 * (lane >> 4);
      if (m0 >= a.Cout) continue;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int co = m0 / 2 + c;
        const float b0 = a.bias[m0 + 2 * c], b1 = a.bias[m0 + 2 * c + 1];
        float* orow = ob + (long)co * a.oc;
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) {
          const float v0 = acc[mi][ni][2 * c] + b0;
          const float v1 = acc[mi][ni][2 * c + 1] + b1;
          const float down = __shfl_down(v1, 1, 16);
          const float wrap = ni + 1 < NI ? __shfl(acc[mi][ni + 1 < NI ? ni + 1 : ni][2 * c + 1] + b1, lane & ~15) : 0.f;
          const int q = q0 + nb + ni * 16;
          const bool last = r == 15 && ni == NI - 1;
          if (q >= 0 && q < L) {
            if (last) orow[2 * q] = v0;
            else *reinterpret_cast<f2*>(orow + 2 * q) = f2{v0, r < 15 ? down : wrap};
          }
          if (r == 0 && ni == 0 && q - 1 >= 0 && q - 1 < L) orow[2 * q - 1] = v1;
        }
      }
    }
  } else if (a.merged_u) {
    const int u = a.merged_u, L = Lin;
    float* ob = a.out + (long)b * a.ob;
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = co0 + wm * 16 * MI + mi * 16 + 4 * (lane >> 4) + j;
        if (m >= a.Cout) continue;
        const int co = m / u, phs = m - co * u;
        const int hi = 2 * phs >= u;  // taps (q, q + 1) of the polyphase form, i.e. this q - 1
        const float bias = a.bias[m];
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) {
          const int qq = q0 + nb + ni * 16 - hi;
#ifdef CX_PROBE_NOSTORE  // tools/cx3_bench.hip probe: the epilogue without its stores
          if (qq >= 0 && qq < L && acc[mi][ni][j] + bias == 12345.f) ob[(long)co * a.oc + (long)(qq * u + phs) * a.ot] = 0.f;
#else
          if (qq >= 0 && qq < L) ob[(long)co * a.oc + (long)(qq * u + phs) * a.ot] = acc[mi][ni][j] + bias;
#endif
        }
      }
  } else {
    conv_epilogue<MI, NI, WN>(a, acc, b, ph, q0, co0, wm, wn, lane);
  }
  if (bad) __hip_atomic_fetch_or(a.oflow, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// tiles {MI, NI, WM, WN}: every wave owns >= 32 output channels x >= 32 positions, so each
// ds_read_b128 of the B operand feeds >= 6 MFMAs and each weight fragment >= 6
//   128 x 64 : 2,4,4,1  (Cout % 128 == 0, 1x1) 192 x 64 : 3,4,4,1  (Cout == 192)
//   128 x 48 : 2,3,4,1  (Cout % 128 == 0, K >= 2)
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
  if (Cout % 80 == 0) return CX_T80;  // several 80-row tiles (Glow-TTS end convs: 160 rows)
  return CX_NONE;
}

bool conv_x3_supported(int Cin, int Cout, int K, int dil) {
  return Cin % 8 == 0 && Cin >= 8 && cx_tile(Cout) != CX_NONE && (K == 1 || K == 2 || K == 3 || K == 5 || K == 7) &&
         (K - 1) * dil <= CONV_MAX_SPAN;
}

// RS weight-ring slots (one or two chunks of taps), SD staging depth in chunks: per shape from
// tools/cx3_bench.hip (two chunks ahead wins where a chunk's MFMAs are long enough to keep two
// register sets without losing occupancy)
template <int MI, int NI, int WM, int WN, int KT, int RS, int SD>
static void cx_launch(const ConvArgs& a, hipStream_t s) {
  constexpr int TC = 16 * MI * WM, TQ = 16 * NI * WN;
  ensure_dyn_lds((const void*)conv_x3_kernel<MI, NI, WM, WN, KT, RS, SD>, 160 * 1024);
  const int nq = (a.max_q + TQ - 1) / TQ, nco = (a.Cout + TC - 1) / TC, nz = a.B * a.nphase;
  const long ntile = (long)nq * nco * nz;
  TTS_CHECK(ntile < (1L << 30), "conv_x3: grid too large");
  const int per = (int)((ntile + 7) / 8);
  const size_t lds = (size_t)2 * (TQ + (KT - 1) * a.dil) * CX_XR * 2;
  conv_x3_kernel<MI, NI, WM, WN, KT, RS, SD><<<dim3(8 * per), 64 * WM * WN, lds, s>>>(a, nq, nco, nz);
}

// estimated cost of a call on one tile shape: rounds of resident workgroups x positions per tile
// (host-side tile count from max_q, an upper bound for ragged batches; residency from the
// occupancy query of the instantiation the call would launch, cached per kernel and LDS size)
template <int MI, int NI, int WM, int WN, int KT, int RS, int SD>
static long cx_cost_k(const ConvArgs& a) {
  constexpr int TC = 16 * MI * WM, TQ = 16 * NI * WN;
  const void* f = (const void*)conv_x3_kernel<MI, NI, WM, WN, KT, RS, SD>;
  const size_t lds = (size_t)2 * (TQ + (KT - 1) * a.dil) * CX_XR * 2;
  static std::mutex mu;
  static std::map<size_t, long> slots_by_lds;
  long slots;
  ensure_dyn_lds(f, 160 * 1024);
  const int cus = device_cu_count();
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = slots_by_lds.find(lds);
    if (it == slots_by_lds.end()) {
      int nb = 0;
      HIP_OK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, f, 64 * WM * WN, lds));
      it = slots_by_lds.emplace(lds, std::max(1L, (long)nb * cus)).first;
    }
    slots = it->second;
  }
  const long tiles = (long)((a.max_q + TQ - 1) / TQ) * ((a.Cout + TC - 1) / TC) * a.B * a.nphase;
  return (tiles + slots - 1) / slots * TQ;
}
template <int MI, int NI, int WM, int WN, int SD12>
static long cx_cost(const ConvArgs& a) {
  switch (a.K) {
    case 1: return cx_cost_k<MI, NI, WM, WN, 1, 2, SD12>(a);
    case 2: return cx_cost_k<MI, NI, WM, WN, 2, 2 * SD12, SD12>(a);
    case 3: return cx_cost_k<MI, NI, WM, WN, 3, 3, 1>(a);
    case 5: return cx_cost_k<MI, NI, WM, WN, 5, 5, 2>(a);
    case 7: return cx_cost_k<MI, NI, WM, WN, 7, 7, 1>(a);
    default: return 0;
  }
}

template <int MI, int NI, int WM, int WN, int SD12>
static void cx_taps(const ConvArgs& a, hipStream_t s) {
  switch (a.K) {
    case 1: cx_launch<MI, NI, WM, WN, 1, 2, SD12>(a, s); break;
    case 2: cx_launch<MI, NI, WM, WN, 2, 2 * SD12, SD12>(a, s); break;
    case 3: cx_launch<MI, NI, WM, WN, 3, 3, 1>(a, s); break;
    case 5: cx_launch<MI, NI, WM, WN, 5, 5, 2>(a, s); break;
    case 7: cx_launch<MI, NI, WM, WN, 7, 7, 1>(a, s); break;
    default: TTS_CHECK(false, "conv_x3: unsupported tap count");
  }
}

void launch_conv_x3(const ConvArgs& a, hipStream_t s) {
  TTS_CHECK(conv_x3_supported(a.Cin, a.Cout, a.K, a.dil), "conv_x3: unsupported shape");
  TTS_CHECK(a.W16 && a.oflow, "conv_x3: split weights / overflow flag missing");
  TTS_CHECK(a.nphase >= 1 && a.nphase <= 8, "conv: nphase");
  TTS_CHECK(a.nsrc == 1 && a.src[0].C == a.Cin, "conv_x3: one source");
  TTS_CHECK(!a.merged_u || (a.nphase == 1 && a.K == 2 && a.pad_left[0] == 1 && a.pad_mode == 0 && a.epi_act == 0 &&
                            a.rep_pad == 0 && a.Cout % a.merged_u == 0 && a.merged_u % 2 == 0),
            "conv_x3: phase-merged ConvTranspose arguments");
  TTS_CHECK(a.src[0].sc != 1 || (a.src[0].st % 4 == 0 && (reinterpret_cast<uintptr_t>(a.src[0].ptr) & 15) == 0),
            "conv_x3: time-major source rows must be 16-byte aligned");
  if (a.max_q <= 0 || a.B <= 0) return;
  switch (cx_tile(a.Cout)) {
    case CX_T128: {
      // 128 x 48 or 128 x 64 tiles, whichever the round-quantised cost model prefers (ties: 64);
      // 1x1 convs keep 128 x 64.
      // tools/cx3_bench.hip (C2 shapes, 48 / 64 wide): encoder conv 45.5 / 55.8 us, postnet
      // 512 -> 512 176.1 / 180.5 us, upsample 1 173.2 / 197.4 us, upsample 2 208.6 / 226.7 us;
      // Glow-TTS (WN convs 192 -> 384, 8 k squeezed frames: 513 tiles on 512 slots at 48 wide)
      // 4.75 / 4.44 ms per call. TTS_CX_NI128 = 3 / 4 forces one width (A/B builds).
      static const int force = [] {
        const char* e = std::getenv("TTS_CX_NI128");
        return e ? std::atoi(e) : 0;
      }();
      bool narrow = force == 3;
      if (!force && a.K >= 2) narrow = cx_cost<2, 3, 4, 1, 2>(a) < cx_cost<2, 4, 4, 1, 2>(a);
      if (narrow) cx_taps<2, 3, 4, 1, 2>(a, s);
      else cx_taps<2, 4, 4, 1, 2>(a, s);
      break;
    }
    case CX_T192: cx_taps<3, 4, 4, 1, 2>(a, s); break;
    case CX_T96: cx_taps<3, 4, 2, 2, 1>(a, s); break;
    case CX_T64: cx_taps<2, 4, 2, 2, 1>(a, s); break;
    case CX_T80: cx_taps<5, 2, 1, 4, 2>(a, s); break;
    case CX_T48: cx_taps<3, 2, 1, 4, 1>(a, s); break;
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

std::vector<float> merge_convT_phases(const std::vector<float>& Wm, int u, int Cin, int Cout) {
  std::vector<float> out((size_t)u * Cout * Cin * 2);
  for (int ph = 0; ph < u; ++ph)
    for (int co = 0; co < Cout; ++co)
      std::copy_n(&Wm[(((size_t)ph * Cout + co) * Cin) * 2], (size_t)Cin * 2, &out[(((size_t)co * u + ph) * Cin) * 2]);
  return out;
}
