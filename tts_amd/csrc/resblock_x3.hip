// Fused MelGAN ResidualStack block (TTS/vocoder/layers/melgan.py:5-39) on the f16 MFMA with
// split-f16 operands (split16.h): fp32-accurate at 5.3x the fp32 MFMA rate.
//   h = conv_k3_dil_d(ReflectionPad(d)(LeakyReLU(x))) + b_d
//   y = [W_1x1 | W_sc] . [lrelu(h); x] + (b_1x1 + b_sc)
// Same structure as the fp32 kernel (resblock.hip): one workgroup owns all C output channels of
// TQ positions, so h never leaves the CU. Persistent: one workgroup per CU (the LDS tile allows no
// more) loops over the (utterance, position) tiles; the next tile's first two staging chunks and
// phase-1 weights load during this tile's phase 2, so neither the staging latency of a tile's
// start nor its output stores sit on the critical path (a launch-per-tile grid spent ~2 us of a
// 7-21 us tile in its prologue, tools/rbx3_bench.hip).
//   staging   32 input channels x (TQ + 2d) positions of lrelu(x), reflect-padded per utterance,
//             split into hi / lo f16 and stored position-major ([pos][32 hi | 32 lo | 16 pad]):
//             one lane's B operand (8 consecutive channels of one position) is one ds_read_b128,
//             and the 160-byte row stride keeps those reads bank-conflict free for any tap offset
//             (16-byte chunks swizzled per row for the stores, split16.h lds_rsw).
//             The centre positions' raw x (shortcut input) go split into HX. Two LDS buffers and
//             two register sets: chunk c+2's global loads are in flight during chunk c's MFMAs.
//   phase 1   h = Wd . X over K = 3 taps x C channels (3 MFMAs per product), weights (A operand,
//             pre-split on the host) streamed from L2 through a 3-slot register ring.
//   phase 2   lrelu(h + b_d) split into HX ([pos][2C hi | 2C lo]), then y = Wf . HX, K = 2C.
// Any operand outside the f16 range sets *oflow; the host then re-runs the call in fp32.
#include "common.h"
#include "split16.h"

#include <algorithm>
#include <cstdlib>

// bottleneck probes for tools/rbx3_bench.hip only (results are wrong in these builds):
// RB_NO_WLOAD (the weight ring is loaded once and never refilled), RB_NO_LDS (MFMAs on register
// operands instead of the LDS reads), RB_NO_MFMA (operand traffic only), RB_NO_XLOAD (tiles staged
// from stale registers: no activation loads after the first tile). Every probe also makes the MFMA
// operands repeat from tile to tile, which lets the chip clock higher (DVFS, MI355X_MICROARCH.md):
// their speedups (profiles/r06/v3_rb_probes.txt) overstate the removed resource's share; loader
// waves that took the HBM staging off the MFMA waves measured no faster (v4_rb_ws_rejected.txt)
#ifdef RB_NO_LDS
#define RB_LD(ptr) (ring[0][0][1])
#else
#define RB_LD(ptr) (*reinterpret_cast<const h8*>(ptr))
#endif
#ifdef RB_NO_MFMA
#define RB_MMA(ah, al, bh, bl, am, ac) ((am)[0] += (float)(bh)[0] + (float)(bl)[7])
#else
#define RB_MMA(ah, al, bh, bl, am, ac) mfma_x3(ah, al, bh, bl, am, ac)
#endif

namespace {
constexpr int X3_DMAX = 27;   // largest dilation (3^3, num_res_blocks <= 4)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ float lrelu_x3(float v) { return fmaxf(v, 0.2f * v); }  // == lrelu02
}  // namespace

// Tile of the persistent loop: utterance b, positions [q0, q0 + TQ) of its L = (lens + len_add) * mul
struct RbTile {
  int b, q0, L;
};

// CPB (round 6): channel chunks of 32 staged per barrier interval. The staging row holds CPB chunks
// ([32 CPB hi | 32 CPB lo | 16 pad]: a stride of 8 mod 16 dwords, conflict-free as the 1-chunk row),
// so phase 1 runs 3 CPB k-steps between barriers instead of 3; the weights keep their k-step order
// (chunk-major, tap-minor), so results are bit-identical for every CPB.
template <int C, int TQ, int WM, int WN, int R, int CPB = 1>
__global__ __launch_bounds__(64 * WM * WN) void resblock_x3_kernel(ResArgs a, int ntiles, bool vec) {
  constexpr int NTHR = 64 * WM * WN;
  constexpr int MI = C / 16 / WM;
  constexpr int NI = TQ / 16 / WN;
  static_assert(MI * 16 * WM == C && NI * 16 * WN == TQ, "tile split");
  constexpr int NCH = (C + 31) / 32;     // staging chunks of 32 input channels (C = 48: 16 zero channels)
  constexpr int NK1 = 3 * NCH;           // phase-1 k-steps: (chunk, tap)
  constexpr int W32 = 32 * CPB;          // channels staged per barrier interval ("super-chunk")
  constexpr int NSC = NCH / CPB;         // super-chunks
  constexpr int XRW = 2 * W32 + 16;      // staging row, halves
  static_assert(NSC * CPB == NCH && (CPB == 1 || C % W32 == 0), "chunks per barrier");
  constexpr int NK2 = 2 * C / 32;        // phase-2 k-steps
  constexpr int NTOT = NK1 + NK2;        // weight sequence of one tile (the ring runs on across tiles)
  // R-slot weight ring: k-step s of a tile's sequence uses slot s % R, so R must divide both
  // phases' lengths for the slots to line up across phases and tiles (C = 192 / 96 / 48: R = 3;
  // C = 256 / 128: 4; C = 64 / 32: 2 / 1)
  static_assert(NK2 * 32 == 2 * C && NK1 % R == 0 && NK2 % R == 0, "weight ring: R must divide both phases");
  constexpr int HR = 4 * C + 16;         // HX row, halves: 2C hi | 2C lo | 16 pad (8C + 32 bytes)
  constexpr int NO = 4 * CPB;  // channel octets per staged row
  constexpr int SPT = (NO * (TQ + 2 * X3_DMAX) + NTHR - 1) / NTHR;  // staging items (8 channels x 1 pos) per thread
  extern __shared__ __attribute__((aligned(16))) _Float16 sh[];

  int t = blockIdx.x;
  const int d = a.dil;
  const int ROWS = TQ + 2 * d;
  _Float16* X0 = sh;
  _Float16* X1 = sh + ROWS * XRW;
  _Float16* HX = sh + 2 * ROWS * XRW;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int nb = wn * 16 * NI + (lane & 15);  // this lane's position (B column) for ni = 0
  const int kg = 8 * (lane >> 4);             // this lane's k offset inside a k-step
  // swizzled (split16.h lds_rsw) k offsets of this lane's rows: HX rows nb + 16 i, X rows
  // nb + 16 i + kq d (tap kq)
  const int lsw = lds_rsw(lane & 15);
  const int kgsw = kg ^ lsw;
  const int kgx[3] = {kgsw, kg ^ lds_rsw((lane & 15) + d), kg ^ lds_rsw((lane & 15) + 2 * d)};
  const int mt0 = wm * MI;
  bool bad = false;   // staged inputs: ordered compare (catches NaN)
  float vmax = 0.f;   // h values: running max of |h| (split16.h absmax4)

  // tile index -> (utterance, first position): per-utterance tile offsets (exclusive scan over the
  // <= 64 lengths, once per workgroup, in LDS); a lookup is one LDS read per lane and a ballot
  __shared__ int tcum[65], tlen[64];
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
  lds_barrier();
  // the host's count may be an upper bound (lengths decoded on the device): the tiles that exist
  ntiles = min(ntiles, __builtin_amdgcn_readfirstlane(tcum[64]));
  auto tile_of = [&](int i) {
    const bool hit = lane < a.B && tcum[lane] <= i && i < tcum[lane + 1];
    const unsigned long long m = __ballot(hit);
    const int b = __builtin_amdgcn_readfirstlane(m ? __ffsll((long long)m) - 1 : 0);
    RbTile r;
    r.b = b;
    r.q0 = __builtin_amdgcn_readfirstlane((i - tcum[b]) * TQ);
    r.L = __builtin_amdgcn_readfirstlane(tlen[b]);
    return r;
  };

  // ---- staging: item e = (channel octet g, row); rows fastest so that lanes read consecutive
  //      positions of one channel (coalesced); clamped addresses, no per-element guard
  int srow[SPT], sg[SPT];
#pragma unroll
  for (int j = 0; j < SPT; ++j) {
    const int e = tid + NTHR * j;
    sg[j] = e / ROWS;
    srow[j] = e - sg[j] * ROWS;
  }
  float st[2][SPT][8];
  auto stage_load = [&](const RbTile& T, float (&sr)[SPT][8], int ch) {
#ifdef RB_NO_XLOAD
    if (T.q0 + T.b + ch > 0 || blockIdx.x > 0) return;
#endif
    const __amdgpu_buffer_rsrc_t xr = rsrc(a.x + (long)T.b * a.sb);  // one utterance: < 2^31 bytes
    const int i0 = T.q0 - d;
    const bool interior = i0 >= 0 && i0 + ROWS <= T.L;
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      int i = i0 + srow[j];
      if (!interior) {  // reflection (torch ReflectionPad1d), then clamp
        if (i < 0) i = -i;
        if (i >= T.L) i = 2 * (T.L - 1) - i;
        i = i < 0 ? 0 : (i >= T.L ? T.L - 1 : i);
      }
      // the channel octet passes through an opaque copy: otherwise the compiler hoists c0 * Ls of
      // every chunk out of the tile loop, and at C = 192 (168 VGPRs for 12 waves) spills them; each
      // scratch reload then came with a vmcnt(0) that drained the weight ring's prefetches
      int g8 = min(sg[j], NO - 1);
      asm volatile("" : "+v"(g8));
      const int c0 = min(W32 * ch + 8 * g8, C - 8);
      const int vo = (c0 * a.Ls + i) * 4;  // per-lane offset; the 8 channel rows are SGPR offsets
#pragma unroll
      for (int c = 0; c < 8; ++c)
        sr[j][c] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(xr, vo, c * a.Ls * 4, 0));
    }
  };
  auto stage_store = [&](_Float16* X, const float (&sr)[SPT][8], int ch) {
#pragma unroll
    for (int j = 0; j < SPT; ++j) {
      const int g = sg[j], row = srow[j];
      if (g < NO) {
        const bool real = W32 * ch + 8 * g < C;  // C = 48: the second chunk's upper half is zero
        float v[8], mx = 0.f;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          v[c] = real ? sr[j][c] : 0.f;
          mx = fmaxf(mx, __builtin_fabsf(v[c]));
        }
        bad |= !(mx < F16_RANGE);  // |lrelu(v)| <= |v|: one check covers both splits
        float lv[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) lv[c] = lrelu_x3(v[c]);
        h8 hi, lo;
        split8(lv, hi, lo);
        const int sx = (8 * g) ^ lds_rsw(row);
        *reinterpret_cast<h8*>(X + row * XRW + sx) = hi;
        *reinterpret_cast<h8*>(X + row * XRW + W32 + sx) = lo;
        const int p = row - d;
        if (real && p >= 0 && p < TQ) {  // raw x of the centre positions: the shortcut's operand
          split8(v, hi, lo);
          const int hx = C + W32 * ch + ((8 * g) ^ lds_rsw(p));
          *reinterpret_cast<h8*>(HX + p * HR + hx) = hi;
          *reinterpret_cast<h8*>(HX + p * HR + 2 * C + hx) = lo;
        }
      }
    }
  };

  // ---- weights: A fragments [mt][k-step][lane][hi 8 | lo 8]; phase 1 then phase 2 as one
  //      sequence through a 3-slot ring that wraps into the next tile's phase 1, so every slot
  //      is reloaded in place right after its MFMAs and never waits at a tile boundary
  // buffer loads: the lane's 32 bytes are a VGPR offset, the (m-tile, k-step) block an SGPR one
  const __amdgpu_buffer_rsrc_t wdr = rsrc(a.Wd16), wfr = rsrc(a.Wf16);
  const int wlo = lane * 32;
  h8 ring[R][MI][2];
  auto wload = [&](h8 (&r)[MI][2], int seq) {
#ifdef RB_NO_WLOAD
    if (seq >= R) return;
#endif
    if (seq >= NTOT) seq -= NTOT;
    const bool p1 = seq < NK1;
    const __amdgpu_buffer_rsrc_t wr = p1 ? wdr : wfr;
    const int nk = p1 ? NK1 : NK2;
    const int ks = p1 ? seq : seq - NK1;
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      const int so = ((mt0 + mi) * nk + ks) * 2048;
      r[mi][0] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(wr, wlo, so, 0));
      r[mi][1] = __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(wr, wlo + 16, so, 0));
    }
  };

  if (t >= ntiles) return;
  // first tile's prologue; later tiles stage chunks 0 and 1 during the previous tile's phase 2.
  // Staging runs two chunks ahead: chunk c is loaded into register set c & 1 after chunk c - 3's
  // MFMAs and stored to LDS buffer c & 1 after chunk c - 1's.
  RbTile cur = tile_of(t);
  stage_load(cur, st[0], 0);
#pragma unroll
  for (int u = 0; u < R; ++u) wload(ring[u], u);
  if (NSC > 1) stage_load(cur, st[1], 1);
  stage_store(X0, st[0], 0);
  if (NSC > 2) stage_load(cur, st[0], 2);
  lds_barrier();
  f32x4 am[MI][NI], ac[MI][NI];
  // EARLY (an even chunk count): the next tile's chunk k loads into the register set this tile's
  // chunk NCH - 2 + k vacates, i.e. during phase 1, a whole tile ahead of its use; with an odd
  // count the set parity would flip every tile, so those loads wait for phase 2
  constexpr bool EARLY = NSC % 2 == 0;
  // per-channel biases, loaded once (a load inside the tile loop would be the youngest in the
  // vmcnt order and make its wait drain every prefetch)
  float bdv[MI][4], bfv[MI];
#pragma unroll
  for (int mi = 0; mi < MI; ++mi) {
#pragma unroll
    for (int j = 0; j < 4; ++j) bdv[mi][j] = a.bd[(mt0 + mi) * 16 + 4 * (lane >> 4) + j];
    bfv[mi] = a.bf[(mt0 + mi) * 16 + (lane & 15)];  // phase 2 is transposed: one channel per lane
  }
#ifdef RB_TRACE  // tools/rbx3_bench.hip trace mode: s_memrealtime per phase, first 4 tiles of a workgroup
  int it = 0;
#define RB_STAMP(k)                                                                             \
  if (threadIdx.x == 0 && it < 4) rb_trace[((long)blockIdx.x * 4 + it) * 8 + (k)] = __builtin_amdgcn_s_memrealtime()
#else
#define RB_STAMP(k)
#endif
  for (;;) {
    RB_STAMP(0);
    const int tn = t + gridDim.x;
    const bool more = tn < ntiles;
    const RbTile nxt = more ? tile_of(tn) : cur;
    // the prefetch loads are issued unconditionally (a last tile re-loads itself): vmcnt is an
    // in-order counter, and a conditional load makes the compiler wait for everything (vmcnt(0))
    if (EARLY && NSC == 2) stage_load(nxt, st[0], 0);
    // ---------------- phase 1: h = Wd . lrelu(x) ----------------
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) am[mi][ni] = ac[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ch = 0; ch < NSC; ++ch) {
      const _Float16* X = (ch & 1) ? X1 : X0;
#pragma unroll
      for (int jk = 0; jk < 3 * CPB; ++jk) {
        const int jc = jk / 3, kq = jk % 3;                // chunk jc of the super-chunk, tap kq
        const int sl = ((ch * CPB + jc) * 3 + kq) % R;     // compile-time after unrolling
        h8 bh[NI], bl[NI];
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) {
          const _Float16* p = X + (nb + ni * 16 + kq * d) * XRW + 32 * jc + kgx[kq];
          bh[ni] = RB_LD(p);
          bl[ni] = RB_LD(p + W32);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni) RB_MMA(ring[sl][mi][0], ring[sl][mi][1], bh[ni], bl[ni], am[mi][ni], ac[mi][ni]);
        wload(ring[sl], (ch * CPB + jc) * 3 + kq + R);
        __builtin_amdgcn_sched_barrier(0);
      }
      if (ch + 1 < NSC) stage_store((ch & 1) ? X0 : X1, st[(ch + 1) & 1], ch + 1);
      if (ch + 3 < NSC) stage_load(cur, st[(ch + 1) & 1], ch + 3);
      else if (EARLY && ch + 3 - NSC < 2) stage_load(nxt, st[(ch + 1) & 1], ch + 3 - NSC);
      lds_barrier();
    }
    RB_STAMP(1);
    // lrelu(h + b_d), split, into HX[pos][0:C) (hi) and HX[pos][2C:3C) (lo)
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      const int co = ((mt0 + mi) * 16 + 4 * (lane >> 4)) ^ lsw;
      const f32x4 bd{bdv[mi][0], bdv[mi][1], bdv[mi][2], bdv[mi][3]};
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        const f32x4 v = lrelu4(x3_value4(am[mi][ni], ac[mi][ni], bd));
        vmax = absmax4(vmax, v);
        h4 hi, lo;
        split4(v, hi, lo);
        const int p = nb + ni * 16;
        *reinterpret_cast<h4*>(HX + p * HR + co) = hi;
        *reinterpret_cast<h4*>(HX + p * HR + 2 * C + co) = lo;
        am[mi][ni] = ac[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    lds_barrier();
    // odd chunk count: the next tile's first two chunks load during phase 2
    if (!EARLY) {
      stage_load(nxt, st[0], 0);
      if (NSC > 1) stage_load(nxt, st[1], 1);
    }
    RB_STAMP(2);
    // ---------------- phase 2: y = [W1 | Wsc] . [lrelu(h); x] ----------------
#pragma unroll
    for (int k0 = 0; k0 < NK2; k0 += R) {
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const int kc = k0 + u;  // slot (NK1 + kc) % R == u since R divides NK1
        h8 bh[NI], bl[NI];
#pragma unroll
        for (int ni = 0; ni < NI; ++ni) {
          const _Float16* p = HX + (nb + ni * 16) * HR + kc * 32 + kgsw;
          bh[ni] = RB_LD(p);
          bl[ni] = RB_LD(p + 2 * C);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int mi = 0; mi < MI; ++mi)
#pragma unroll
          for (int ni = 0; ni < NI; ++ni) RB_MMA(bh[ni], bl[ni], ring[u][mi][0], ring[u][mi][1], am[mi][ni], ac[mi][ni]);
        wload(ring[u], NK1 + kc + R);  // past NK2: the next tile's phase-1 weights
      }
    }
    RB_STAMP(3);
    float* yb = a.y + (long)cur.b * a.sb;
    // transposed phase 2 (operands swapped: D = [lrelu(h); x]^T . Wf^T): a lane holds positions
    // q .. q + 3 of channel co, one 16-byte store instead of four 4-byte ones where the rows are
    // 16-byte aligned (vec: Ls, sb multiples of 4 and y aligned), per-position stores otherwise
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      const int co = (mt0 + mi) * 16 + (lane & 15);
      const f32x4 bf{bfv[mi], bfv[mi], bfv[mi], bfv[mi]};
      float* yr = yb + (long)co * a.Ls;
#pragma unroll
      for (int ni = 0; ni < NI; ++ni) {
        const f32x4 v = x3_value4(am[mi][ni], ac[mi][ni], bf);
        const int q = cur.q0 + wn * 16 * NI + ni * 16 + 4 * (lane >> 4);
        if (vec && q + 3 < cur.L) {
          *reinterpret_cast<f32x4*>(yr + q) = v;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (q + j < cur.L) yr[q + j] = v[j];
        }
      }
    }
    RB_STAMP(4);
    if (!more) break;
    lds_barrier();  // every wave is done with this tile's X / HX
    RB_STAMP(5);
    cur = nxt;
    t = tn;
    stage_store(X0, st[0], 0);
    if (NSC > 2) stage_load(cur, st[0], 2);
    lds_barrier();
#ifdef RB_TRACE
    ++it;
#endif
  }
#undef RB_STAMP
  if (bad || !(vmax < F16_RANGE)) __hip_atomic_fetch_or(a.oflow, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// one resident workgroup per CU (the LDS tile allows no more), each looping over tiles; the
// dynamic LDS leaves 1 KiB of the CU's 160 KiB for the kernel's static tile tables
constexpr int RB_DYN_LDS = 159 * 1024;
template <int C, int TQ, int WM, int WN, int R, int CPB = 1>
static void launch_rbx3(const ResArgs& a, const int* h_lens, hipStream_t s) {
  const int ROWS = TQ + 2 * a.dil;
  const size_t lds = ((size_t)2 * ROWS * (64 * CPB + 16) + (size_t)TQ * (4 * C + 16)) * 2;
  ensure_dyn_lds((const void*)resblock_x3_kernel<C, TQ, WM, WN, R, CPB>, RB_DYN_LDS);
  const int ncu = device_cu_count();
  TTS_CHECK(lds <= RB_DYN_LDS, "resblock_x3: LDS tile too large");
  long ntiles = 0;
  for (int b = 0; b < a.B; ++b) ntiles += ((long)(h_lens[b] + a.len_add) * a.mul + TQ - 1) / TQ;
  TTS_CHECK(ntiles < (1L << 30), "resblock_x3: too many tiles");
  if (ntiles == 0) return;
  const int grid = (int)std::min<long>(ntiles, ncu);
  const bool vec = a.Ls % 4 == 0 && a.sb % 4 == 0 && (reinterpret_cast<uintptr_t>(a.y) & 15) == 0;
  resblock_x3_kernel<C, TQ, WM, WN, R, CPB><<<grid, 64 * WM * WN, lds, s>>>(a, (int)ntiles, vec);
}

bool resblock_x3_supported(int C) { return C == 256 || C == 192 || C == 128 || C == 96 || C == 64 || C == 48 || C == 32; }

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

// the phase-1 weights in resstack_x3's packed k-step order for a half last chunk (C % 32 == 16):
// full chunks as pack_resblock_x3 (k-step 3 ch + tap), then the half chunk's 2 octets x 3 taps in
// 2 k-steps: k-step 3K lane groups 0-1 tap 0 / 2-3 tap 1, k-step 3K + 1 groups 0-1 tap 2 / 2-3 zero
// (group g reads channel octet 4 (K) + (g & 1), i.e. channels 32 K + 8 (g & 1) + j)
void pack_resblock_x3p(const std::vector<float>& wd, int C, std::vector<uint16_t>& wd16) {
  TTS_CHECK(C % 32 == 16, "pack_resblock_x3p: half last chunk only");
  const int K = C / 32;  // full chunks
  wd16 = pack_split_a(C / 16, 3 * K + 2, [&](int m, int k) -> float {
    const int step = k / 32, g = (k % 32) / 8, j = k % 8;
    int kq, ci;
    if (step < 3 * K) {
      kq = step % 3;
      ci = 32 * (step / 3) + 8 * g + j;
    } else if (step == 3 * K) {
      kq = g >> 1;
      ci = 32 * K + 8 * (g & 1) + j;
    } else {
      if (g >= 2) return 0.f;
      kq = 2;
      ci = 32 * K + 8 * g + j;
    }
    return wd[((size_t)m * C + ci) * 3 + kq];
  });
}

void launch_resblock_x3(const ResArgs& a, const int* h_lens, int C, hipStream_t s) {
  TTS_CHECK(a.dil >= 1 && a.dil <= X3_DMAX, "resblock: dilation must be in [1, 27] (num_res_blocks <= 4)");
  TTS_CHECK(a.Wd16 && a.Wf16 && a.oflow, "resblock_x3: split weights / overflow flag missing");
  TTS_CHECK(a.B <= 64, "resblock_x3: at most 64 utterances per call");
  if (a.max_q <= 0 || a.B <= 0) return;
  switch (C) {
    // tiles from tools/rbx3_bench.hip (C2 shapes): 12 waves, one m-tile (or two) per wave
    case 192: launch_rbx3<192, 64, 12, 1, 3>(a, h_lens, s); break;
    case 96: launch_rbx3<96, 128, 6, 2, 3>(a, h_lens, s); break;  // round 3: 4 blocks 926 -> 879 us
    case 48: launch_rbx3<48, 192, 3, 4, 3>(a, h_lens, s); break;
    // full-band MelGAN stages (base 512): tiles sized to the 159 KB LDS budget, 8 waves
    case 256: launch_rbx3<256, 32, 8, 1, 4>(a, h_lens, s); break;
    case 128: launch_rbx3<128, 64, 8, 1, 4>(a, h_lens, s); break;
    case 64: launch_rbx3<64, 128, 4, 2, 2>(a, h_lens, s); break;
    case 32: launch_rbx3<32, 192, 2, 4, 1>(a, h_lens, s); break;
    default: TTS_CHECK(false, "resblock_x3: unsupported channel count");
  }
  HIP_OK(hipGetLastError());
}
