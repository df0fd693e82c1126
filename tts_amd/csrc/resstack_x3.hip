// The first three MelGAN ResidualStack blocks (dilations 1, 3, 9; TTS/vocoder/layers/melgan.py:5-39,
// stacked by vocoder/models/melgan_generator.py:60-68) fused per time tile, split-f16 as in
// resblock_x3.hip. A tile of TQ output positions is staged once with a halo of OFF = 16 >=
// 1 + 3 + 9 positions on each side; block k's output is computed on the tile widened by the
// dilations of the blocks after it (ext[k]), so x_1 and x_2 stay in LDS and the stage's HBM traffic
// for those three blocks is one read of x_0 and one write of x_3 instead of three of each.
// Block 3 (dilation 27: a 27-position halo per side would cost more recompute than its traffic)
// stays on resblock_x3_kernel.
//
// LDS rows (position-major, row r <-> position q0 - OFF + r, ROWS = TQ + 2 OFF; 16-byte chunks
// swizzled per row, split16.h lds_rsw):
//   XL  lrelu(x_k) split: [C hi | C lo | 16 pad] -- the phase-1 operand (3 taps read each row)
//   HX  [lrelu(h) hi | x_k hi | lrelu(h) lo | x_k lo | 16 pad] -- the phase-2 operand, as resblock_x3
// Per block: phase 1 h = Wd . XL over 3 taps (rows reflected at the utterance ends), epilogue
// lrelu(h + b_d) into HX; phase 2 y = Wf . HX; y (block < 2) goes back into XL / HX as x_{k+1},
// the last block's y to HBM. Rows outside a block's valid range are written as zeros, so nothing
// but finite values is ever split. The next tile's x_0 loads into registers during the last block's
// phase 2. Waves: one m-tile each (C / 16 of them) x WN n-groups; n-tile j of a block goes to
// group j % WN.
#include "common.h"
#include "split16.h"

#include <algorithm>
#include <type_traits>

namespace {
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_s(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ float lrelu_s(float v) { return fmaxf(v, 0.2f * v); }
template <class T>
__device__ __forceinline__ T pick3(T v0, T v1, T v2, int i) {  // wave-uniform select, no indexed kernarg
  return i == 0 ? v0 : (i == 1 ? v1 : v2);
}
constexpr int ST_OFF = 16;  // halo rows per side (>= the sum of the fused dilations)
}  // namespace

// bottleneck probes for tools/rsx3_bench.hip only: RS_NO_LDS (MFMAs on register operands),
// RS_NO_MFMA (operand reads, no MFMAs)
#ifdef RS_NO_LDS
#define RS_LD(ptr) (ring[0][1])
#else
#define RS_LD(ptr) (*reinterpret_cast<const h8*>(ptr))
#endif
#ifdef RS_TRACE  // s_memrealtime (100 MHz) stamps of wave 0, first RS_TRACE_TILES tiles of every workgroup
#define RS_TRACE_TILES 4
#define RS_STAMP(k)                                                                               \
  if (threadIdx.x == 0 && it_ < RS_TRACE_TILES && blockIdx.x < 256 && rs_trace)                  \
  rs_trace[((long)blockIdx.x * RS_TRACE_TILES + it_) * 16 + (k)] = __builtin_amdgcn_s_memrealtime()
#else
#define RS_STAMP(k)
#endif
#ifndef RS_STAGE_AT
#define RS_STAGE_AT 1
#endif
#ifdef RS_NO_SB
#define RS_SB()
#else
#define RS_SB() __builtin_amdgcn_sched_barrier(0)
#endif
#ifdef RS_NO_MFMA
#define RS_MMA(ah, al, bh, bl, am, ac) ((am)[0] += (float)(bh)[0] + (float)(bl)[7])
#else
#define RS_MMA(ah, al, bh, bl, am, ac) mfma_x3(ah, al, bh, bl, am, ac)
#endif

template <int C, int TQ, int WN, int NI, int CTU>
__global__ __launch_bounds__(64 * (C / 16) * WN) void resstack_x3_kernel(StackArgs a, int ntiles) {
  constexpr int NB = 3;
  constexpr int WM = C / 16;
  constexpr int NTHR = 64 * WM * WN;
  constexpr int OFF = ST_OFF;
  constexpr int ROWS = TQ + 2 * OFF;
  static_assert(ROWS % 16 == 0 && ROWS / 16 <= WN * NI, "n-tiles per wave group");
  constexpr int NCH = (C + 31) / 32;  // phase-1 chunks of 32 input channels
  // phase-1 k-steps: 3 taps per full chunk; a half chunk (C % 32 == 16: C = 48) packs its 2 channel
  // octets x 3 taps into 2 k-steps instead of 3 (pack_resblock_x3p; k-step 3K: taps 0 | 1 by lane
  // group pair, 3K + 1: tap 2 | zero weights), 5 k-steps instead of 6 at C = 48
  constexpr bool HALF = C % 32 == 16;
  constexpr int NK1 = HALF ? 3 * (NCH - 1) + 2 : 3 * NCH, NK2 = 2 * C / 32, NKB = NK1 + NK2;
  constexpr int R = 3;  // weight ring; the blocks are unrolled, so a k-step's slot is the compile-time
                        // (its index in the tile's weight sequence) % R
  static_assert(NK2 * 32 == 2 * C && (C % 32 == 0 || HALF), "weight ring / channel chunks");
  // XL row stride 2C + 16 halves (C = 48: 56 dwords): the 16 lanes of each ds_read_b128 group
  // (16 consecutive rows, two k-octets) land on distinct banks
  constexpr int XLR = 2 * C + 16;
  constexpr int HR = 4 * C + 16;
  constexpr int NG = C / 8;  // channel octets of a staged row
  // fused ConvTranspose geometry: CIN input channels in CROWS staged rows of CRS halves; CMT m-tiles
  // of merged rows, CNT n-tiles of input columns, CKS k-steps (32 channels x 2 taps). Row stride
  // 104 dwords (8 mod 16, as XL / HX): the B-operand ds_read_b128 is conflict-free in each of the
  // instruction's four lane groups ({0-3, 12-15, 20-27}, ...: rows 0-3 and 12-15 at k-group 0 beside
  // rows 4-11 at k-group 1). Round 5's 100-dword stride kept 16 consecutive rows on distinct banks
  // but put every group's two k-groups 2-way on the same banks (PMC LDS_conflict 0.29).
  constexpr int CIN = 2 * C, NGI = CIN / 8, CROWS = 128, CRS = 2 * CIN + 16;
  constexpr int CMT = CTU ? C * CTU / 16 : 1, CNT = CROWS / 16, CKS = CIN / 32 * 2;
  static_assert(CTU == 0 || (C == 48 && CTU == 2 && ROWS / 2 + 2 <= CROWS && CROWS * CRS <= ROWS * (2 * C + 16) &&
                             WM * WN == 2 * CMT && CNT == 2 * NI),
                "fused ConvTranspose geometry");
  constexpr int SPT0 = (NG * ROWS + NTHR - 1) / NTHR, SPT1 = (NGI * CROWS + NTHR - 1) / NTHR;
  constexpr int SPT = CTU ? SPT1 : SPT0;
  extern __shared__ __attribute__((aligned(16))) _Float16 sh[];
  _Float16* XL = sh;
  _Float16* HX = sh + ROWS * XLR;
  __shared__ float bias[NB][2][C];
  __shared__ __attribute__((aligned(16))) float bct[CTU ? C * CTU : 4];  // fused ConvTranspose bias per merged row
  __shared__ int tcum[65], tlen[64];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int kg = 8 * (lane >> 4);
  const int co = wm * 16 + 4 * (lane >> 4);  // first of this lane's 4 output channels
  // rows nt * 16 + (lane & 15) (epilogues, phase 2): the swizzled channel / k offsets
  const int lsw = lds_rsw(lane & 15);
  const int cosw = co ^ lsw, kgsw = kg ^ lsw;
  bool bad = false;   // staged inputs: ordered compare (catches NaN)
  float vmax = 0.f;   // produced values: running max of |v| (split16.h absmax4)
  int t = blockIdx.x;

  if (wave == 0) {
    const int L = lane < a.B ? (a.lens[lane] + a.len_add) * a.mul : 0;
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
  // zero the whole tile once: pads and never-written rows hold finite values for the
  // unconditional operand reads
  for (int i = tid; i < ROWS * (XLR + HR) / 8; i += NTHR) reinterpret_cast<h8*>(sh)[i] = h8{};
  for (int i = tid; i < NB * 2 * C; i += NTHR) {
    const int blk = i / (2 * C), w = (i / C) & 1, c = i % C;
    const float* p = w ? pick3(a.bf[0], a.bf[1], a.bf[2], blk) : pick3(a.bd[0], a.bd[1], a.bd[2], blk);
    bias[blk][w][c] = p[c];
  }
  if constexpr (CTU) {
    for (int i = tid; i < C * CTU; i += NTHR) bct[i] = a.ct_bias[i];
  }
  lds_barrier();
  // the host's count may be an upper bound (lengths decoded on the device): the tiles that exist
  ntiles = min(ntiles, __builtin_amdgcn_readfirstlane(tcum[64]));
  struct Tile {
    int b, q0, L;
  };
  auto tile_of = [&](int i) {
    const bool hit = lane < a.B && tcum[lane] <= i && i < tcum[lane + 1];
    const unsigned long long m = __ballot(hit);
    const int b = __builtin_amdgcn_readfirstlane(m ? __ffsll((long long)m) - 1 : 0);
    Tile r;
    r.b = b;
    r.q0 = __builtin_amdgcn_readfirstlane((i - tcum[b]) * TQ);
    r.L = __builtin_amdgcn_readfirstlane(tlen[b]);
    return r;
  };

  // ---- staging of x_0: item = (channel octet, row), rows fastest (coalesced per channel)
  constexpr int SROWS = CTU ? CROWS : ROWS;
  int srow[SPT], sg[SPT];
#pragma unroll
  for (int j = 0; j < SPT; ++j) {
    const int e = tid + NTHR * j;
    sg[j] = e / SROWS;
    srow[j] = e - sg[j] * SROWS;
  }
  float st[SPT][8];
  // CTU: the ConvTranspose input of a tile, rows = input positions (q0 - OFF) / CTU - 1 + row
  auto stage_load_ct = [&](const Tile& T) {
    const __amdgpu_buffer_rsrc_t xr = rsrc_s(a.xin + (long)T.b * a.sb_in);
    constexpr int U = CTU ? CTU : 1;
    const int Lin = T.L / U, qb = (T.q0 - OFF) / U - 1;
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      int p = qb + srow[j];
      p = p < 0 ? 0 : (p >= Lin ? Lin - 1 : p);
      const int vo = (8 * min(sg[j], NGI - 1) * a.Ls_in + p) * 4;
#pragma unroll
      for (int c = 0; c < 8; ++c)
        st[j][c] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, vo, c * a.Ls_in * 4, 0));
    }
  };
  auto stage_store_ct = [&](const Tile& T) {
    constexpr int U = CTU ? CTU : 1;
    const int Lin = T.L / U, qb = (T.q0 - OFF) / U - 1;
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      if (sg[j] >= NGI) continue;
      const int p = qb + srow[j];
      const bool in = p >= 0 && p < Lin;  // the ConvTranspose's zero padding
      float lv[8], mx = 0.f;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const float v = in ? st[j][c] : 0.f;
        mx = fmaxf(mx, __builtin_fabsf(v));
        lv[c] = lrelu_s(v);
      }
      bad |= !(mx < F16_RANGE);
      h8 hi, lo;
      split8(lv, hi, lo);
      _Float16* xl = XL + srow[j] * CRS + 8 * sg[j];
      *reinterpret_cast<h8*>(xl) = hi;
      *reinterpret_cast<h8*>(xl + CIN) = lo;
    }
  };
  auto stage_load = [&](const Tile& T) {
    const __amdgpu_buffer_rsrc_t xr = rsrc_s(a.x + (long)T.b * a.sb);
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      int p = T.q0 - OFF + srow[j];
      p = p < 0 ? 0 : (p >= T.L ? T.L - 1 : p);
      const int vo = (8 * min(sg[j], NG - 1) * a.Ls + p) * 4;
#pragma unroll
      for (int c = 0; c < 8; ++c) st[j][c] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, vo, c * a.Ls * 4, 0));
    }
  };
  auto stage_store = [&](const Tile& T) {
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      if (sg[j] >= NG) continue;
      const int p = T.q0 - OFF + srow[j];
      const bool in = p >= 0 && p < T.L;
      float v[8], lv[8], mx = 0.f;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        v[c] = in ? st[j][c] : 0.f;
        mx = fmaxf(mx, __builtin_fabsf(v[c]));
        lv[c] = lrelu_s(v[c]);
      }
      bad |= !(mx < F16_RANGE);
      h8 hi, lo;
      split8(lv, hi, lo);
      const int sx = (8 * sg[j]) ^ lds_rsw(srow[j]);
      _Float16* xl = XL + srow[j] * XLR + sx;
      *reinterpret_cast<h8*>(xl) = hi;
      *reinterpret_cast<h8*>(xl + C) = lo;
      split8(v, hi, lo);
      _Float16* hx = HX + srow[j] * HR + C + sx;
      *reinterpret_cast<h8*>(hx) = hi;
      *reinterpret_cast<h8*>(hx + 2 * C) = lo;
    }
  };

  auto load_tile = [&](const Tile& T) {
    if constexpr (CTU) stage_load_ct(T);
    else stage_load(T);
  };
  auto store_tile = [&](const Tile& T) {
    if constexpr (CTU) stage_store_ct(T);
    else stage_store(T);
  };
  // ---- weights: block k's phase-1 then phase-2 fragments ([mt][k-step][lane][hi | lo], the
  //      resblock_x3 packing) through a 3-slot ring that runs on across blocks and tiles
  const int wlo = lane * 32;
  h8 ring[R][2];
  // CTU: the fused ConvTranspose is "block -1" of every tile, CKS k-steps of this wave's merged-row
  // m-tile (wave % CMT) ahead of block 0 in the ring sequence (CKS % R == 0 keeps slots fixed)
  constexpr int SEQ0 = CTU ? CKS : 0;  // index of block 0's first k-step in the tile's weight sequence
  static_assert((SEQ0 + NB * NKB) % R == 0, "weight ring: a tile's weight sequence must be a multiple of R");
  auto wload = [&](h8 (&r)[2], int blk, int s) {  // s: k-step within block blk (compile-time)
    if (CTU && blk < 0) {
      const __amdgpu_buffer_rsrc_t wr = rsrc_s(a.ct16);
      const int so = ((wave % CMT) * CKS + s) * 2048;
      r[0] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(wr, wlo, so, 0));
      r[1] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(wr, wlo + 16, so, 0));
      return;
    }
    const bool p1 = s < NK1;
    const __amdgpu_buffer_rsrc_t wr = rsrc_s(p1 ? pick3(a.wd16[0], a.wd16[1], a.wd16[2], blk) : pick3(a.wf16[0], a.wf16[1], a.wf16[2], blk));
    const int so = (wm * (p1 ? NK1 : NK2) + (p1 ? s : s - NK1)) * 2048;
    r[0] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(wr, wlo, so, 0));
    r[1] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(wr, wlo + 16, so, 0));
  };
  // after k-step s of block blk: load the k-step R ahead (into the next block past its end)
  auto wnext = [&](h8 (&r)[2], int blk, int s) {
#ifdef RS_NO_WLOAD
    return;
#endif
    const int nk = (CTU && blk < 0) ? CKS : NKB;
    if (s + R < nk) wload(r, blk, s + R);
    else wload(r, blk + 1 == NB ? (CTU ? -1 : 0) : blk + 1, s + R - nk);
  };

  f32x4 am[NI], ac[NI];
  // CTU prologue (after store_tile + barrier): x_0 of every row of the tile from the staged input.
  // Wave w: merged-row m-tile w % CMT, input-column n-tiles w / CMT + 2 n (the 4 accumulator pairs
  // of a block's n-tiles); the epilogue waits until every wave is done with the staging (it shares
  // the XL region)
  auto ct_prologue = [&](const Tile& T) __attribute__((always_inline)) {
    const int mt = wave % CMT, g = wave / CMT;
    // the row / column index of this lane, opaque per tile: the LDS addresses derived from it are
    // recomputed here instead of hoisted out of the tile loop (where they spilled)
    int lrow = lane & 15;
    asm volatile("" : "+v"(lrow));
#pragma unroll
    for (int n = 0; n < NI; ++n) am[n] = ac[n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < CKS; ++ks) {  // k-step = chunk * 2 + tap, as pack_conv_x3 (K = 2)
      const int ch = ks >> 1, tap = ks & 1;
      h8 bh[NI], bl[NI];
#pragma unroll
      for (int n = 0; n < NI; ++n) {
        const int j = min((g + 2 * n) * 16 + lrow + tap, CROWS - 1);
        const _Float16* p = XL + j * CRS + 32 * ch + kg;
        bh[n] = RS_LD(p);
        bl[n] = RS_LD(p + CIN);
      }
      RS_SB();
#pragma unroll
      for (int n = 0; n < NI; ++n) RS_MMA(ring[ks % R][0], ring[ks % R][1], bh[n], bl[n], am[n], ac[n]);
      wnext(ring[ks % R], -1, ks);
      RS_SB();
    }
    lds_barrier();  // the staged input (XL region) is dead from here
    const int m0 = mt * 16 + 4 * (lane >> 4), co0 = m0 / 2;  // rows m0 .. m0 + 3 = (co0, co0 + 1) x phases 0, 1
    const f32x4 b4 = *reinterpret_cast<const f32x4*>(bct + m0);
    const int P0 = T.q0 - OFF;
#pragma unroll
    for (int n = 0; n < NI; ++n) {
      const int c = (g + 2 * n) * 16 + lrow;  // input column q' = P0 / 2 + c
      const f32x4 v = x3_value4(am[n], ac[n], b4);
      vmax = absmax4(vmax, v);
#pragma unroll
      for (int ph = 0; ph < 2; ++ph) {
        const int r = 2 * c - ph;  // phase 0: output 2 q', phase 1: 2 q' - 1
        if (r < 0 || r >= ROWS) continue;
        const int p = P0 + r;
        const bool in = p >= 0 && p < T.L;
        const f32x2_ x2{in ? v[ph] : 0.f, in ? v[2 + ph] : 0.f};
        const int cs = co0 ^ lds_rsw(r);
        h2_ hi, lo;
        split2(x2, hi, lo);
        *reinterpret_cast<h2_*>(HX + r * HR + C + cs) = hi;
        *reinterpret_cast<h2_*>(HX + r * HR + 3 * C + cs) = lo;
        split2(f32x2_{lrelu_s(x2[0]), lrelu_s(x2[1])}, hi, lo);
        *reinterpret_cast<h2_*>(XL + r * XLR + cs) = hi;
        *reinterpret_cast<h2_*>(XL + r * XLR + C + cs) = lo;
      }
    }
    lds_barrier();
  };

  if (t >= ntiles) return;
  Tile cur = tile_of(t);
  load_tile(cur);
#pragma unroll
  for (int u = 0; u < R; ++u) wload(ring[u], CTU ? -1 : 0, u);
  store_tile(cur);
  lds_barrier();
  if constexpr (CTU) ct_prologue(cur);

#ifdef RS_TRACE
  int it_ = 0;
#endif
  for (;;) {
    RS_STAMP(0);
    const int tn = t + gridDim.x;
    const bool more = tn < ntiles;
    const Tile nxt = more ? tile_of(tn) : cur;
    const int base = cur.q0 - OFF;  // position of row 0
    // one ResidualStack block; the last is peeled (a second inlined copy) so that the next tile's
    // staging loads are issued on a path the compiler sees whole: its vmcnt waits for the weight
    // ring then count them instead of draining them
    auto block = [&](auto BI, const bool last) __attribute__((always_inline)) {
      constexpr int bi = decltype(BI)::value;
      constexpr int g0 = SEQ0 + bi * NKB;  // weight-sequence index of this block's k-step 0
      const int d = pick3(a.dil[0], a.dil[1], a.dil[2], bi), E = pick3(a.ext[0], a.ext[1], a.ext[2], bi);
      const int vlo = max(OFF - E, -base), vhi = min(OFF + TQ + E, cur.L - base);
      const int tlo = vlo >> 4, thi = (vhi + 15) >> 4;
      // every tap of every row of the tile lies inside the utterance
      const bool interior = base - d >= 0 && base + ROWS + d <= cur.L;
      int nt[NI], trow[NI][3];
      bool act[NI];
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        nt[ni] = tlo + wn + WN * ni;
        act[ni] = nt[ni] < thi;
        const int r = nt[ni] * 16 + (lane & 15);
        if (interior) {  // no reflection: rows r - d, r, r + d (past ROWS: finite HX bytes, dropped)
#pragma unroll
          for (int kq = 0; kq < 3; ++kq) trow[ni][kq] = max(r + (kq - 1) * d, 0);
        } else {
#pragma unroll
          for (int kq = 0; kq < 3; ++kq) {  // tap rows: ReflectionPad1d(d) at the utterance ends
            int pp = base + r + (kq - 1) * d;
            if (pp < 0) pp = -pp;
            if (pp >= cur.L) pp = 2 * (cur.L - 1) - pp;
            pp = pp < 0 ? 0 : (pp >= cur.L ? cur.L - 1 : pp);
            const int rr = pp - base;
            trow[ni][kq] = rr < 0 ? 0 : (rr >= ROWS ? ROWS - 1 : rr);
          }
        }
      }
      RS_STAMP(4 * bi + 1);
      if (RS_STAGE_AT == 1 && last) load_tile(nxt);
      // ---------------- phase 1: h = Wd . lrelu(x_k) ----------------
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) am[ni] = ac[ni] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < NK1; ++s) {
        const int ch = HALF && s >= 3 * (NCH - 1) ? NCH - 1 : s / 3;
        h8 bh[NI], bl[NI];
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) {
          // unconditional: an inactive slot reads a clamped row and its result is dropped
          int r, col;
          if (!HALF || s < 3 * (NCH - 1)) {  // full chunk ch, tap s % 3, the lane's k octet kg
            r = trow[ni][s % 3];
            col = 32 * ch + kg;
          } else {  // half chunk: lane-group pair gp = lane >> 5 picks the tap, octet 4 + (lane >> 4 & 1)
            const int gp = lane >> 5;
            r = s == 3 * (NCH - 1) ? (gp ? trow[ni][1] : trow[ni][0]) : trow[ni][2];
            col = 32 * ch + 8 * ((lane >> 4) & 1);  // the second lane-group pair of the last
                                                     // k-step reads these finite halves against
                                                     // zero weights
          }
          const _Float16* p = XL + r * XLR + (col ^ lds_rsw(r));
          bh[ni] = RS_LD(p);
          bl[ni] = RS_LD(p + C);
        }
        RS_SB();
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          RS_MMA(ring[(g0 + s) % R][0], ring[(g0 + s) % R][1], bh[ni], bl[ni], am[ni], ac[ni]);
        wnext(ring[(g0 + s) % R], bi, s);
        RS_SB();
      }
      // lrelu(h + b_d) into HX's h columns; rows outside [vlo, vhi) as zeros
      {
        const f32x4 bd = *reinterpret_cast<const f32x4*>(bias[bi][0] + co);
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) {
          if (!act[ni]) continue;
          const int r = nt[ni] * 16 + (lane & 15);
          const bool in = r >= vlo && r < vhi;
          f32x4 v = lrelu4(x3_value4(am[ni], ac[ni], bd));
          if (!in) v = f32x4{0.f, 0.f, 0.f, 0.f};
          vmax = absmax4(vmax, v);
          h4 hi, lo;
          split4(v, hi, lo);
          *reinterpret_cast<h4*>(HX + r * HR + cosw) = hi;
          *reinterpret_cast<h4*>(HX + r * HR + 2 * C + cosw) = lo;
          am[ni] = ac[ni] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
      lds_barrier();
      RS_STAMP(4 * bi + 2);
      if (RS_STAGE_AT == 0 && last) load_tile(nxt);  // in flight during the last phase 2 and the stores
      // ---------------- phase 2: y = [W1 | Wsc] . [lrelu(h); x_k] ----------------
#pragma unroll
      for (int kc = 0; kc < NK2; ++kc) {
        const int s = NK1 + kc;
        h8 bh[NI], bl[NI];
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) {
          {
            const _Float16* p = HX + (min(nt[ni], ROWS / 16 - 1) * 16 + (lane & 15)) * HR + kc * 32 + kgsw;
            bh[ni] = RS_LD(p);
            bl[ni] = RS_LD(p + 2 * C);
          }
        }
        RS_SB();
#pragma unroll
        for (int ni = 0; ni < NI; ++ni)
          if (last)  // transposed (D = HX^T . Wf^T): the stores below write 4 positions of one channel
            RS_MMA(bh[ni], bl[ni], ring[(g0 + s) % R][0], ring[(g0 + s) % R][1], am[ni], ac[ni]);
          else
            RS_MMA(ring[(g0 + s) % R][0], ring[(g0 + s) % R][1], bh[ni], bl[ni], am[ni], ac[ni]);
        wnext(ring[(g0 + s) % R], bi, s);
        RS_SB();
      }
      const f32x4 bf = *reinterpret_cast<const f32x4*>(bias[bi][1] + co);
      RS_STAMP(4 * bi + 3);
      if (RS_STAGE_AT == 2 && last) load_tile(nxt);
      if (!last) {
        lds_barrier();  // every wave is done reading x_k
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) {
          if (!act[ni]) continue;
          const int r = nt[ni] * 16 + (lane & 15);
          const bool in = r >= vlo && r < vhi;
          f32x4 v = x3_value4(am[ni], ac[ni], bf);
          if (!in) v = f32x4{0.f, 0.f, 0.f, 0.f};
          vmax = absmax4(vmax, v);  // |lrelu(v)| <= |v|: one maximum covers both
          h4 xh, xlo, lh, llo;
          split4(v, xh, xlo);
          split4(lrelu4(v), lh, llo);
          *reinterpret_cast<h4*>(XL + r * XLR + cosw) = lh;
          *reinterpret_cast<h4*>(XL + r * XLR + C + cosw) = llo;
          *reinterpret_cast<h4*>(HX + r * HR + C + cosw) = xh;
          *reinterpret_cast<h4*>(HX + r * HR + 3 * C + cosw) = xlo;
        }
        lds_barrier();
        RS_STAMP(4 * bi + 4);
      } else {
        // lane: channel wm * 16 + (lane & 15), rows r .. r + 3 (OFF and TQ are multiples of 4,
        // so a 4-row group is wholly inside or outside the tile's own positions)
        const int cl = wm * 16 + (lane & 15);
        const float b1 = bias[bi][1][cl];
        const f32x4 bf1{b1, b1, b1, b1};
        float* yr = a.y + (long)cur.b * a.sb + (long)cl * a.Ls;
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) {
          if (!act[ni]) continue;
          const int r = nt[ni] * 16 + 4 * (lane >> 4);
          const int q = base + r;
          if (r >= OFF && r < OFF + TQ) {
            const f32x4 v = x3_value4(am[ni], ac[ni], bf1);
            if (q + 3 < cur.L) {
              *reinterpret_cast<f32x4*>(yr + q) = v;
            } else {
#pragma unroll
              for (int j = 0; j < 4; ++j)
                if (q + j < cur.L) yr[q + j] = v[j];
            }
          }
        }
      }
    };
    static_assert(NB == 3, "three fused blocks");
    block(std::integral_constant<int, 0>{}, false);
    block(std::integral_constant<int, 1>{}, false);
    block(std::integral_constant<int, 2>{}, true);
    if (!more) break;
    RS_STAMP(14);
    lds_barrier();  // every wave is done with this tile's XL / HX
    cur = nxt;
    t = tn;
    store_tile(cur);
    lds_barrier();
    if constexpr (CTU) ct_prologue(cur);
    RS_STAMP(15);
#ifdef RS_TRACE
    ++it_;
#endif
  }
  if (bad || !(vmax < F16_RANGE)) __hip_atomic_fetch_or(a.oflow, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int C, int TQ, int WN, int NI, int CTU = 0>
static void launch_rsx3(const StackArgs& a, const int* h_lens, hipStream_t s) {
  constexpr int ROWS = TQ + 2 * ST_OFF;
  constexpr size_t lds = (size_t)ROWS * ((2 * C + 16) + (4 * C + 16)) * 2;
  static_assert(lds + 3 * 2 * C * 4 + 65 * 4 + 64 * 4 <= 160 * 1024, "LDS");
  ensure_dyn_lds((const void*)resstack_x3_kernel<C, TQ, WN, NI, CTU>, (int)lds);
  const int ncu = device_cu_count();
  long ntiles = 0;
  for (int b = 0; b < a.B; ++b) ntiles += ((long)(h_lens[b] + a.len_add) * a.mul + TQ - 1) / TQ;
  TTS_CHECK(ntiles < (1L << 30), "resstack_x3: too many tiles");
  if (ntiles == 0) return;
  const int grid = (int)std::min<long>(ntiles, ncu);
  resstack_x3_kernel<C, TQ, WN, NI, CTU><<<grid, 64 * (C / 16) * WN, lds, s>>>(a, (int)ntiles);
}

bool resstack_x3_supported(int C, const int* dil, int n) {
  if ((C != 48 && C != 96) || n < 3) return false;
  int sum = 0;
  for (int k = 0; k < 3; ++k) {
    if (dil[k] < 1) return false;
    sum += dil[k];
  }
  return sum <= ST_OFF;
}

// the call-dependent conditions: 16-byte aligned output rows and every utterance longer than the
// stack's reflection reach (callers fall back to the per-block kernels otherwise)
bool resstack_x3_fits(const StackArgs& a, const int* h_lens) {
  if (a.B > 64 || a.Ls % 4 != 0 || a.sb % 4 != 0 || (reinterpret_cast<uintptr_t>(a.y) & 15) != 0) return false;
  for (int b = 0; b < a.B; ++b)
    if ((long)(h_lens[b] + a.len_add) * a.mul <= ST_OFF) return false;
  return true;
}

void launch_resstack_x3(const StackArgs& a0, const int* h_lens, int C, hipStream_t s) {
  TTS_CHECK(resstack_x3_supported(C, a0.dil, 3), "resstack_x3: shape not covered");
  TTS_CHECK(a0.oflow, "resstack_x3: overflow flag missing");
  TTS_CHECK(resstack_x3_fits(a0, h_lens), "resstack_x3: unaligned rows, more than 64 utterances or an utterance "
                                          "shorter than the reflection pad");
  StackArgs a = a0;
  a.ext[2] = 0;
  a.ext[1] = a.dil[2];
  a.ext[0] = a.dil[1] + a.dil[2];
  if (C == 48 && a.ct16) {
    TTS_CHECK(a.xin && a.ct_bias && a.mul % 2 == 0, "resstack_x3: fused ConvTranspose arguments");
    launch_rsx3<48, 208, 4, 4, 2>(a, h_lens, s);
  } else if (C == 48) {
    // 3 m-tile waves x 4 n-groups; ROWS = 240 = 15 n-tiles, <= 4 per wave
    launch_rsx3<48, 208, 4, 4>(a, h_lens, s);
  } else {
    TTS_CHECK(!a.ct16, "resstack_x3: fused ConvTranspose only at C = 48");
    // C = 96: 6 m-tile waves x 2 n-groups; ROWS = 128 = 8 n-tiles, 4 per wave (158.5 KB LDS)
    launch_rsx3<96, 96, 2, 4>(a, h_lens, s);
  }
  HIP_OK(hipGetLastError());
}
