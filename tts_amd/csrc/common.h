// Shared definitions for the ttship HIP library (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <atomic>
#include <cstdint>
#include <mutex>
#include <set>
#include <string>
#include <tuple>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

// 16x16x4 f32-in / f32-accumulate MFMA (exact f32, k-ordered fma chain).
// Operand lane maps (cdna_hip_programming.md §3): A[i=l&15][k=l>>4], B[k=l>>4][j=l&15];
// D: col j = l&15, row i = 4*(l>>4) + reg.
#define MFMA16(a, b, c) __builtin_amdgcn_mfma_f32_16x16x4f32((a), (b), (c), 0, 0, 0)

// Error plumbing: every C-ABI entry returns 0 on success, nonzero on failure, and stores a
// message retrievable with tts_last_error().
void tts_set_error(const std::string& msg);

#define HIP_OK(expr)                                                                   \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    if (_e != hipSuccess) {                                                            \
      throw std::runtime_error(std::string(#expr) + ": " + hipGetErrorString(_e));     \
    }                                                                                  \
  } while (0)

#define TTS_CHECK(cond, msg)                                                           \
  do {                                                                                 \
    if (!(cond)) throw std::runtime_error(std::string(msg));                           \
  } while (0)

// Kernel attributes and device facts, per device and thread-safe: contexts on several devices
// (one host thread each) launch the same templates concurrently
inline void ensure_dyn_lds(const void* f, int bytes) {
  static std::mutex m;
  static std::set<std::tuple<const void*, int, int>> done;
  int dev = 0;
  HIP_OK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> g(m);
  if (done.count({f, dev, bytes})) return;
  HIP_OK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  done.insert({f, dev, bytes});
}
inline int device_cu_count() {
  static std::mutex m;
  static int ncu[64] = {};
  int dev = 0;
  HIP_OK(hipGetDevice(&dev));
  TTS_CHECK(dev >= 0 && dev < 64, "device index out of range");
  std::lock_guard<std::mutex> g(m);
  if (!ncu[dev]) HIP_OK(hipDeviceGetAttribute(&ncu[dev], hipDeviceAttributeMultiprocessorCount, dev));
  return ncu[dev];
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its
// global loads and stores (__syncthreads also drains vmcnt, which would complete every prefetch
// issued before it and stall on every store)
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }
__device__ __forceinline__ float lrelu02(float x) { return x >= 0.f ? x : 0.2f * x; }
// Short forms for the recurrent cells and the attention energies (on the steps' critical paths):
// v_exp_f32 / v_rcp_f32 (1 ulp each) instead of the libm sequences. Absolute error below 2e-7
// over the whole range (tools/fast_math_err.py); tanh takes an odd Taylor polynomial below 0.25,
// where 1 - e^-2x would cancel.
__device__ __forceinline__ float sigm_f(float x) {
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-1.4426950408889634f * x));
}
__device__ __forceinline__ float tanh_f(float x) {
  const float ax = __builtin_fabsf(x);
  const float e = __builtin_amdgcn_exp2f(-2.8853900817779268f * ax);  // exp(-2|x|)
  const float big = (1.f - e) * __builtin_amdgcn_rcpf(1.f + e);
  const float x2 = ax * ax;
  const float small =
      __builtin_fmaf(ax * x2, __builtin_fmaf(x2, __builtin_fmaf(x2, __builtin_fmaf(x2, 0.021869488f, -0.053968254f),
                                                               0.13333334f), -0.33333334f), ax);
  return __builtin_copysignf(ax < 0.25f ? small : big, x);
}

// tanh for the attention energies: the same form without the small-argument polynomial. Near 0,
// (1 - e) / (1 + e) loses relative accuracy but not absolute: its error stays below ~1.5e-7 over the
// whole range (tools/fast_math_err.py), the size that matters in e = v . tanh(..), a sum of 128
// such terms. Half the instructions of tanh_f on the attention items' VALU-bound energy stage.
__device__ __forceinline__ float tanh_e(float x) {
  const float e = __builtin_amdgcn_exp2f(-2.8853900817779268f * __builtin_fabsf(x));  // exp(-2|x|)
  return __builtin_copysignf((1.f - e) * __builtin_amdgcn_rcpf(1.f + e), x);
}

// ---------------------------------------------------------------------------------------
// Generic fp32 MFMA Conv1d (implicit GEMM): out[b][co][q*out_mul+ph] =
//   epi( sum_{ci,tap} W[co][ci][tap] * in_act(src[b][ci][pad_map(q + tap*dil - pad_left[ph])]) )
// Used for: encoder convs (BN folded), LSTM input projection, processed_inputs, postnet,
// every MelGAN conv, and ConvTranspose1d as `nphase` polyphase 2-tap convs.
// ---------------------------------------------------------------------------------------
struct ConvSrc {
  const float* ptr;
  long sb;     // batch stride (elements)
  int sc, st;  // channel / time strides (elements)
  int C;       // channels contributed by this source
  int act;     // 0 none, 1 leaky-relu(0.2) applied on load
};

struct ConvArgs {
  ConvSrc src[2];
  int nsrc;
  int Cin;            // total input channels (multiple of 16)
  int K, dil;
  int pad_mode;       // 0 zero, 1 reflect, 2 clamp (replicate)
  const int* lens;    // per-utterance base length (device)
  int len_add;        // base' = lens[b] + len_add (vocoder: 2*inference_padding)
  int in_mul;         // input length  = base' * in_mul
  int q_mul;          // output positions per phase = base' * q_mul
  int rep_pad;        // virtual replicate padding of the raw source (first vocoder conv)
  int nphase;         // 1, or stride of a ConvTranspose1d
  int pad_left[8];    // per phase
  long w_phase_stride;
  const float* W;     // swizzled [co16][kc][64][4] per phase
  const float* bias;  // [Cout]
  int Cout, Cout_pad;
  float* out;
  long ob;
  int oc, ot;
  int out_mul;        // t_out = q*out_mul + phase
  int epi_act;        // 0 none, 1 relu, 2 tanh, 3 gate pair, 4 coupling pair, 5 coupling +
                      // inverse InvConvNear / ActNorm, 6 GLU pair (see conv.hip)
  const float* resid; // optional residual added after activation
  long rb;
  int rc, rt;
  int resid_rows;     // > 0: the residual applies to output rows < resid_rows only
  const float* aux;   // epi 5: per output channel {w[4], actnorm bias, exp(-logs)}; epi 3 (optional):
                      // per-utterance gate bias aux[b * auxb + co] (Glow WN speaker conditioning)
  long auxb;
  int max_q;          // max over batch of output positions per phase (grid x extent)
  int B;
  // split-f16 variant (conv_x3.hip): pre-split A fragments [co16][k-step][64][hi 8 | lo 8] per
  // phase (k-step = 32 input channels of one tap), and the range flag
  const void* W16 = nullptr;
  long w16_phase_stride = 0;  // bytes
  unsigned* oflow = nullptr;
  // > 0: phase-merged ConvTranspose1d of stride merged_u (conv_x3.hip only): GEMM row
  // m = co * merged_u + phase, 2 taps at input q - 1 and q for q in [0, L] (nphase = 1,
  // pad_left 1, zero padding), bias per row; phases >= merged_u / 2 write output position
  // (q - 1) * merged_u + phase, the others q * merged_u + phase
  int merged_u = 0;
};

// tile configs: TC = output channels per workgroup, TQ = output positions per workgroup
enum ConvTile { TILE_128x64 = 0, TILE_64x64, TILE_192x64, TILE_96x64, TILE_48x128, TILE_80x64, TILE_16x256 };
int conv_tile_tc(int tile);
int conv_tile_for_cout(int cout);
void launch_conv(const ConvArgs& a, int tile, hipStream_t s);
// split-f16 form of the same conv (conv_x3.hip); false when the shape is not covered
bool conv_x3_supported(int Cin, int Cout, int K, int dil);
void launch_conv_x3(const ConvArgs& a, hipStream_t s);
// host packing of the split weights: Wm = nphase blocks of [Cout][Cin*K] row-major
std::vector<uint16_t> pack_conv_x3(const std::vector<float>& Wm, int Cin, int Cout, int K, int nphase,
                                   long* phase_stride_bytes);
// merged ConvTranspose weights from the polyphase form Wm [u][Cout][Cin][2] (merged_u above)
std::vector<float> merge_convT_phases(const std::vector<float>& Wm, int u, int Cin, int Cout);

// host-side swizzle of a row-major weight matrix Wm[Cout][Kdim] (Kdim % 16 == 0) into the
// MFMA fragment order: dst[((m*nkc + kc)*64 + l)*4 + s] = Wm[m*16 + (l&15)][kc*16 + 4*(l>>4) + s]
void swizzle_rows16(const float* Wm, int rows, int rows_pad, int Kdim, float* dst);

// Several buffer fills as ONE launch (each hipMemsetAsync is a ~5 us kernel of its own): entries
// are (pointer, bytes, 32-bit fill word); bytes a multiple of 4, entries must not overlap.
struct FillList {
  static constexpr int N = 32;  // the decoder state fill: 14 buffers + 3 per barrier block (4 launches)
  int n = 0;
  void* p[N];
  long words[N];
  unsigned val[N];
  void add(void* ptr, size_t bytes, unsigned v = 0) {
    TTS_CHECK(n < N && bytes % 4 == 0, "FillList: too many entries or unaligned size");
    if (!bytes) return;
    p[n] = ptr;
    words[n] = (long)(bytes / 4);
    val[n] = v;
    ++n;
  }
};
void launch_fills(const FillList& f, hipStream_t s);

// PQMF synthesis (pqmf.py:51-56): x (B, N, L) -> y (B, 1, N*L)
void launch_pqmf_synthesis(const float* x, long xb, long xc, const float* G, int N, int taps,
                           const int* lens, int len_add, int L_mul, int maxL, int B, float* y, long yb,
                           hipStream_t s);

// Fused MelGAN ResidualStack block (TTS/vocoder/layers/melgan.py:35-39):
//   y = [W_1x1 | W_sc] . [lrelu(conv_k3_dil(reflectpad(lrelu(x))) + b_d); x] + (b_1x1 + b_sc)
struct ResArgs {
  const float* x;   // (B, C, Ls)
  float* y;         // (B, C, Ls)
  long sb;          // batch stride (C * Ls)
  int Ls;           // channel stride
  const int* lens;  // base length per utterance
  int len_add, mul; // L = (lens[b] + len_add) * mul
  int dil;
  const float* Wd;  // dilated conv, swizzled rows C, K = 3C
  const float* bd;
  const float* Wf;  // [W_1x1 | W_sc], swizzled rows C, K = 2C
  const float* bf;
  int max_q, B;
  // split-f16 variant (resblock_x3.hip): pre-split A fragments of Wd / Wf and the range flag
  const void* Wd16 = nullptr;
  const void* Wf16 = nullptr;
  unsigned* oflow = nullptr;
};
void launch_resblock(const ResArgs& a, int C, hipStream_t s);
bool resblock_x3_supported(int C);
// persistent: one workgroup per CU loops over the (utterance, position) tiles; h_lens = the
// host copy of lens, or per-row upper bounds of the device lens (grid size; the kernel counts
// the tiles from the device lens)
void launch_resblock_x3(const ResArgs& a, const int* h_lens, int C, hipStream_t s);
void pack_resblock_x3(const std::vector<float>& wd, const std::vector<float>& wf, int C,
                      std::vector<uint16_t>& wd16, std::vector<uint16_t>& wf16);
// phase-1 weights in resstack_x3's packed order for C % 32 == 16 (C = 48: 5 k-steps, not 6)
void pack_resblock_x3p(const std::vector<float>& wd, int C, std::vector<uint16_t>& wd16);

// Blocks 0-2 of a ResidualStack fused per time tile (resstack_x3.hip), split-f16 weights in the
// pack_resblock_x3 layout (phase 1 in the pack_resblock_x3p order when C % 32 == 16);
// y = block2(block1(block0(x)))
struct StackArgs {
  const float* x;
  float* y;
  long sb;
  int Ls;
  const int* lens;
  int len_add, mul, B;
  int dil[3];
  int ext[3];  // filled by the launcher
  const void* wd16[3];
  const void* wf16[3];
  const float* bd[3];
  const float* bf[3];  // b_1x1 + b_sc
  unsigned* oflow;
  // fused ConvTranspose (resstack_x3 with CTU = 2, C = 48): x_0 = ConvT(lrelu(xin)) computed per
  // tile from the 2C-channel input at half the rate (x is then unused); ct16 / ct_bias: the
  // phase-merged split weights and per-merged-row bias of conv_x3.hip (merged_u = 2)
  const float* xin;
  long sb_in;
  int Ls_in;
  const void* ct16;
  const float* ct_bias;
};
bool resstack_x3_supported(int C, const int* dil, int n);
bool resstack_x3_fits(const StackArgs& a, const int* h_lens);
void launch_resstack_x3(const StackArgs& a, const int* h_lens, int C, hipStream_t s);

// fused MB-MelGAN output conv (C -> 4, k7, LReLU + reflect pad 3 + tanh) and PQMF synthesis
// (melgan_out.hip); returns false when the shape is not covered (N != 4, 63 taps, C not 32/48).
// launch_out_pqmf writes every row's band positions [0, maxL): zeros past its own length
void launch_out_conv1(const float* x, long xb, long xc, int C, const float* W, const float* bo, const int* lens,
                      int len_add, int L_mul, int maxL, int B, float* y, long yb, hipStream_t s);
bool launch_out_pqmf(const float* x, long xb, long xc, int C, const float* Wo, const float* bo, const float* G,
                     int N, int taps, const int* lens, int len_add, int L_mul, int maxL, int B, float* y, long yb,
                     hipStream_t s);
// test hook of the persistent BiLSTM (tts_test_stall_lstm): recurrence to stall, -1 = off
extern std::atomic<int> g_test_stall_lstm;

