// Latency skeleton of the persistent decoder's step (decoder_persist.hip): the same 256 x 512-thread
// grid, workgroup roles and hand-off sizes, no arithmetic (optional spin delays stand in for each
// role's compute). Measures the step's hand-off chain under two synchronisation schemes:
//   mode 0: a grid barrier after every phase (gsync.h, as the decoder runs)
//   mode 1: edge-scoped counters, each consumer waits only for the workgroups it reads
// Not part of the library:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/chain_bench.hip -o tools/chain_bench
#include "../tts_amd/csrc/gsync.h"
// -DCB_FLAG: the flag barrier the decoder runs since round 5 (gsync.h gflag_*) in place of the
// counter form; argv[2] picks the barrier block among 16 of one allocation (its placement matters,
// DESIGN.md 4.1d)
#ifdef CB_FLAG
#define gsync_arrive(b, g) gflag_arrive(b, g)
#define gsync_wait(b, g, f) gflag_wait(b, g, f)
#endif

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace {
constexpr int PW = 256, PT = 512, NATT = 64, IW0 = 64, NPRE = 32, NPJ = 54, NB = 32, NCH = 6, YP = 432;
constexpr int STOP_WG = 63;

struct CArgs {
  float *ypart, *pb, *hatt, *pq, *part_u, *ctx, *hd0, *hd1, *alpha, *sink;
  unsigned* bar;   // grid barrier block (mode 0)
  unsigned* ctr;   // edge counters (mode 1), each on its own 128-byte line: [0] y, [32] pb, [64] h, [96] ctx,
                   // [128] d, [160 + 32 b] per-utterance alignment, [2048 + 32 b] tickets
  int steps;
  int dl[6];       // spin delays (100 MHz ticks) per role: prenet, att P3, item P4, P5, pj P6, item P3
  unsigned* err;
};

__device__ __forceinline__ void spin(int ticks) {
  if (ticks <= 0) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)ticks) {}
}

// every wave drains its stores, then one lane counts the workgroup in
__device__ __forceinline__ void edge_arrive(unsigned* c) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool edge_wait(unsigned* c, unsigned target, unsigned* err, int* flag) {
  if (threadIdx.x == 0) {
    int good = 1;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {
        __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        good = 0;
        break;
      }
      if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
        good = 0;
        break;
      }
    }
    *flag = good;
  }
  lds_barrier();
  return *flag;
}

// hierarchical edge (mode 2): P producers per step, producer i counts in at first-level counter
// i % nc (each on its own 128-byte line); the last arrival at a counter counts it in at the top
// counter, the last of those writes the go word (t + 1); consumers poll only the go word
struct Edge {
  unsigned* blk;  // [0] top, [32] go, [64 + 32 c] first-level counters
  int P, nc;
};
__device__ __forceinline__ void hedge_arrive(const Edge& e, int i, int t) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned per = (unsigned)(e.P / e.nc), gen = (unsigned)(t + 1);
    unsigned* c = e.blk + 64 + (i % e.nc) * 32;
    if (__hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == per * gen - 1)
      if (__hip_atomic_fetch_add(e.blk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)e.nc * gen - 1)
        __hip_atomic_store(e.blk + 32, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// load n 16-byte granules per thread from base (coherent), fold them into a register sum
__device__ int g_noload;
__device__ int g_rep;  // copies of each broadcast buffer (hatt, ctx, h_dec, pb); consumer wg g reads copy g % rep
constexpr long S_HATT = 64 * 1024, S_CTX = 32 * 1024, S_HD = 64 * 1024, S_PB = 16 * 1024;  // floats per copy
__device__ __forceinline__ float load_sum(const float* base, int n, int stride_bytes) {
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (g_noload) return 0.f;
  f32x4 v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (i < n) v[i] = ldc4(base, (int)threadIdx.x * 16 + i * stride_bytes);
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (i < n) s += v[i];
  return s[0] + s[1] + s[2] + s[3];
}
}  // namespace

template <int MODE>
__global__ __launch_bounds__(PT) void chain_kernel(CArgs a) {
  __shared__ int flag, is_last;
  __shared__ float red[PT];
  const int g = blockIdx.x, tid = threadIdx.x;
  unsigned gen = 0;
  float acc = 0.f;
  unsigned* Cy = a.ctr;
  unsigned* Cpb = a.ctr + 32;
  unsigned* Ch = a.ctr + 64;
  unsigned* Cctx = a.ctr + 96;
  unsigned* Cd = a.ctr + 128;
  const int it = g - IW0, ib = it / NCH, ich = it % NCH;
  // mode 2: hierarchical edges, one 1024-word block each (ctr + 4096 + 1024 k)
  const Edge Ey{a.ctr + 4096, NPJ, 6}, Epb{a.ctr + 4096 + 1024, NPRE + 1, 3}, Eh{a.ctr + 4096 + 2048, NATT, 8},
      Ectx{a.ctr + 4096 + 3072, NB, 8}, Ed{a.ctr + 4096 + 4096, PW, 16};
  auto go = [&](const Edge& e) { return e.blk + 32; };
  auto sync = [&](unsigned* c, unsigned target) -> bool {  // mode 0: grid barrier, mode 1/2: edge wait
    if (MODE == 0) {
      gsync_arrive(a.bar, gen);
      return gsync_wait(a.bar, gen, &flag);
    }
    return edge_wait(c, target, a.err, &flag);
  };
  auto arrive = [&](unsigned* c, const Edge& e, int i, int t_) {
    if (MODE == 1) edge_arrive(c);
    if (MODE == 2) hedge_arrive(e, i, t_);
  };
  for (int t = 0; t < a.steps; ++t) {
    float* hd_cur = (t & 1) ? a.hd1 : a.hd0;
    float* hd_nxt = (t & 1) ? a.hd0 : a.hd1;
    // ---- P1: prenet layer 2 (wg 0..31) || stop (wg 63) || items' location window
    if (MODE == 1 && (g < NPRE || g == STOP_WG) && t > 0 && !edge_wait(Cy, NPJ * t, a.err, &flag)) return;
    if (MODE == 2 && (g < NPRE || g == STOP_WG) && t > 0 && !edge_wait(go(Ey), t, a.err, &flag)) return;
    if (g < NPRE) {
      acc += load_sum(a.ypart + (g & 1) * 16 * YP, 2, PT * 16);  // 16 rows x 256 columns
      spin(a.dl[0]);
      if (tid < 64) for (int c = 0; c < g_rep; ++c) stc4(a.pb + c * S_PB, ((g * 64 + tid) * 4) * 4, f32x4{acc, acc, acc, acc});
    } else if (g == STOP_WG) {
      acc += tid < 32 ? ldc(a.ypart + tid * YP) : 0.f;
    } else if (it >= 0 && it < NB * NCH) {
      if (MODE >= 1 && t > 0 && !edge_wait(a.ctr + 160 + 32 * ib, NCH * t, a.err, &flag)) return;
      acc += tid < 128 ? ldc(a.alpha + ib * 256 + min(max(ich * 32 - 15 + (tid & 63), 0), 191)) : 0.f;
    }
    if (g < NPRE || g == STOP_WG) arrive(Cpb, Epb, g < NPRE ? g : NPRE, t);
    if (!sync(MODE == 2 ? go(Epb) : Cpb, MODE == 2 ? t + 1 : (NPRE + 1) * (t + 1))) return;
    // ---- P3: attention_rnn (wg 0..63) || h_dec part (items)
    if (g < NATT) {
      acc += load_sum(a.pb + (g % g_rep) * S_PB, 4, PT * 16);  // 32 rows x 256
      spin(a.dl[1]);
      if (tid < 128) for (int c = 0; c < g_rep; ++c) stc4(a.hatt + c * S_HATT, ((g * 128 + tid) * 4) * 4, f32x4{acc, acc, acc, acc});  // 2 KB
      stc4(a.pq, ((g * 1024 + tid) * 4) * 4, f32x4{acc, acc, acc, acc});                 // 16 KB
      stc4(a.pq, ((g * 1024 + 512 + tid) * 4) * 4, f32x4{acc, acc, acc, acc});
      arrive(Ch, Eh, g, t);
    } else {
      acc += load_sum(hd_cur + (g % g_rep) * S_HD, 16, PT * 16);  // 128 KB
      spin(a.dl[5]);
    }
    if (!sync(MODE == 2 ? go(Eh) : Ch, MODE == 2 ? t + 1 : NATT * (t + 1))) return;
    // ---- P4: attention items || h_att parts (wg 0..63)
    if (g >= IW0 && it < NB * NCH) {
      acc += load_sum(a.pq + ib * 128, 4, 32 * 128 * 4 * 4);  // 64 partials x 128 dims of row ib (16 per group)
      spin(a.dl[2]);
      stc4(a.part_u, ((it * 128 + (tid & 127)) * 4) * 4, f32x4{acc, acc, acc, acc});
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        const unsigned prev = __hip_atomic_fetch_add(a.ctr + 2048 + 32 * ib, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        is_last = prev == (unsigned)(NCH * (t + 1) - 1);
      }
      lds_barrier();
      if (is_last) {
        acc += load_sum(a.part_u + ib * NCH * 512, 6, 512 * 4) ;
        for (int c = 0; c < g_rep; ++c) stc(a.ctx + c * S_CTX + ib * 512 + tid, acc);
        arrive(Cctx, Ectx, ib, t);
      }
    } else if (g < IW0) {
      acc += load_sum(a.hatt + (g % g_rep) * S_HATT, 16, PT * 16);
      acc += load_sum(hd_cur + (g % g_rep) * S_HD, 16, PT * 16);
    }
    if (!sync(MODE == 2 ? go(Ectx) : Cctx, MODE == 2 ? t + 1 : NB * (t + 1))) return;
    // ---- P5: ctx parts (+ h_att parts on the items), decoder_rnn cell
    acc += load_sum(a.ctx + (g % g_rep) * S_CTX, 8, PT * 16);
    if (g >= IW0) acc += load_sum(a.hatt + (g % g_rep) * S_HATT, 16, PT * 16);
    spin(a.dl[3]);
    if (tid < 32) for (int c = 0; c < g_rep; ++c) stc4(hd_nxt + c * S_HD, ((g * 32 + tid) * 4) * 4, f32x4{acc, acc, acc, acc});
    arrive(Cd, Ed, g, t);
    if (MODE == 0) {
      if (!sync(Cd, 0)) return;
    }
    // ---- P6: projection jobs (wg 0..53) || alignment pass (items)
    if (g < NPJ) {
      if (MODE == 1 && !edge_wait(Cd, PW * (t + 1), a.err, &flag)) return;
      if (MODE == 2 && !edge_wait(go(Ed), t + 1, a.err, &flag)) return;
      acc += load_sum(hd_nxt + (g % g_rep) * S_HD + (g & 1) * 16 * 1024, 8, PT * 16);   // 16 rows x 1024
      acc += load_sum(a.ctx + (g % g_rep) * S_CTX + (g & 1) * 16 * 512, 4, PT * 16);     // 16 rows x 512
      spin(a.dl[4]);
      if (tid < 64) stc4(a.ypart, (((g & 1) * 16 * YP + (g >> 1) * 16) + tid * 4) * 4, f32x4{acc, acc, acc, acc});
      arrive(Cy, Ey, g, t);
    } else if (g >= IW0 && it < NB * NCH) {
      if (tid < 32) stc(a.alpha + ib * 256 + ich * 32 + tid, acc);
      if (MODE >= 1) edge_arrive(a.ctr + 160 + 32 * ib);
    }
    if (MODE == 0 && !sync(nullptr, 0)) return;
  }
  if (tid == 0) a.sink[g] = acc;
}

// mode 3: grid barriers, but a workgroup whose phase work feeds nothing in the next phase arrives
// BEFORE that work (its stores are covered by a later barrier it arrives at afterwards): each
// barrier completes when its real producers arrive. Items' location window moves from P1 to P3,
// items' P6 stores (alignment) are covered by the next step's P1 barrier.
__global__ __launch_bounds__(PT) void early_kernel(CArgs a) {
  __shared__ int flag, is_last;
  const int g = blockIdx.x, tid = threadIdx.x;
  unsigned gen = 0;
  float acc = 0.f;
  const int it = g - IW0, ib = it / NCH, ich = it % NCH;
  const bool item = g >= IW0 && it < NB * NCH;
  auto wait = [&]() { return gsync_wait(a.bar, gen, &flag); };
  for (int t = 0; t < a.steps; ++t) {
    float* hd_cur = (t & 1) ? a.hd1 : a.hd0;
    float* hd_nxt = (t & 1) ? a.hd0 : a.hd1;
    // P1: producers prenet + stop
    const bool p1 = g < NPRE || g == STOP_WG;
    if (!p1) gsync_arrive(a.bar, gen);
    if (g < NPRE) {
      acc += load_sum(a.ypart + (g & 1) * 16 * YP, 2, PT * 16);
      spin(a.dl[0]);
      if (tid < 64) for (int c = 0; c < g_rep; ++c) stc4(a.pb + c * S_PB, ((g * 64 + tid) * 4) * 4, f32x4{acc, acc, acc, acc});
    } else if (g == STOP_WG) {
      acc += tid < 32 ? ldc(a.ypart + tid * YP) : 0.f;
    }
    if (p1) gsync_arrive(a.bar, gen);
    if (!wait()) return;
    // P3: producers att
    if (g >= NATT) gsync_arrive(a.bar, gen);
    if (g < NATT) {
      acc += load_sum(a.pb + (g % g_rep) * S_PB, 4, PT * 16);
      spin(a.dl[1]);
      if (tid < 128) for (int c = 0; c < g_rep; ++c) stc4(a.hatt + c * S_HATT, ((g * 128 + tid) * 4) * 4, f32x4{acc, acc, acc, acc});
      stc4(a.pq, ((g * 1024 + tid) * 4) * 4, f32x4{acc, acc, acc, acc});
      stc4(a.pq, ((g * 1024 + 512 + tid) * 4) * 4, f32x4{acc, acc, acc, acc});
      gsync_arrive(a.bar, gen);
    } else {
      if (item) acc += tid < 128 ? ldc(a.alpha + ib * 256 + min(max(ich * 32 - 15 + (tid & 63), 0), 191)) : 0.f;
      acc += load_sum(hd_cur + (g % g_rep) * S_HD, 16, PT * 16);
      spin(a.dl[5]);
    }
    if (!wait()) return;
    // P4: producers items
    if (g < IW0) gsync_arrive(a.bar, gen);
    if (item) {
      acc += load_sum(a.pq + ib * 128, 4, 32 * 128 * 4 * 4);
      spin(a.dl[2]);
      stc4(a.part_u, ((it * 128 + (tid & 127)) * 4) * 4, f32x4{acc, acc, acc, acc});
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        const unsigned prev = __hip_atomic_fetch_add(a.ctr + 2048 + 32 * ib, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        is_last = prev == (unsigned)(NCH * (t + 1) - 1);
      }
      lds_barrier();
      if (is_last) {
        acc += load_sum(a.part_u + ib * NCH * 512, 6, 512 * 4);
        for (int c = 0; c < g_rep; ++c) stc(a.ctx + c * S_CTX + ib * 512 + tid, acc);
      }
    } else {
      acc += load_sum(a.hatt + (g % g_rep) * S_HATT, 16, PT * 16);
      acc += load_sum(hd_cur + (g % g_rep) * S_HD, 16, PT * 16);
    }
    if (g >= IW0) gsync_arrive(a.bar, gen);
    if (!wait()) return;
    // P5: everyone
    acc += load_sum(a.ctx + (g % g_rep) * S_CTX, 8, PT * 16);
    if (g >= IW0) acc += load_sum(a.hatt + (g % g_rep) * S_HATT, 16, PT * 16);
    spin(a.dl[3]);
    if (tid < 32) for (int c = 0; c < g_rep; ++c) stc4(hd_nxt + c * S_HD, ((g * 32 + tid) * 4) * 4, f32x4{acc, acc, acc, acc});
    gsync_arrive(a.bar, gen);
    if (!wait()) return;
    // P6: producers pj
    if (g >= NPJ) gsync_arrive(a.bar, gen);
    if (g < NPJ) {
      acc += load_sum(hd_nxt + (g % g_rep) * S_HD + (g & 1) * 16 * 1024, 8, PT * 16);
      acc += load_sum(a.ctx + (g % g_rep) * S_CTX + (g & 1) * 16 * 512, 4, PT * 16);
      spin(a.dl[4]);
      if (tid < 64) stc4(a.ypart, (((g & 1) * 16 * YP + (g >> 1) * 16) + tid * 4) * 4, f32x4{acc, acc, acc, acc});
      gsync_arrive(a.bar, gen);
    } else if (item) {
      if (tid < 32) stc(a.alpha + ib * 256 + ich * 32 + tid, acc);
    }
    if (!wait()) return;
  }
  if (tid == 0) a.sink[g] = acc;
}

static hipStream_t S;

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  HIP_OK(hipStreamCreate(&S));
  auto alloc = [](size_t n) {
    float* p;
    HIP_OK(hipMalloc(&p, n * 4));
    HIP_OK(hipMemset(p, 0, n * 4));
    return p;
  };
  CArgs a{};
  a.ypart = alloc(64 * YP);
  a.pb = alloc(8 * S_PB);
  a.hatt = alloc(8 * S_HATT);
  a.pq = alloc(64 * 32 * 128 * 2);
  a.part_u = alloc(NB * NCH * 512 * 2);
  a.ctx = alloc(8 * S_CTX);
  a.hd0 = alloc(8 * S_HD);
  a.hd1 = alloc(8 * S_HD);
  a.alpha = alloc(NB * 256);
  a.sink = alloc(PW);
  unsigned* bar_pool;
  HIP_OK(hipMalloc(&bar_pool, 16 * BAR_WORDS * 4));
  a.bar = bar_pool + (argc > 2 ? std::atoi(argv[2]) % 16 : 0) * BAR_WORDS;
  HIP_OK(hipMalloc(&a.ctr, 16384 * 4));
  HIP_OK(hipMalloc(&a.err, 4));
  const int steps = 400;
  a.steps = steps;
  const unsigned tmo = 200000000u;
  struct Cfg {
    const char* name;
    int dl[6];
  } cfgs[] = {{"no compute", {0, 0, 0, 0, 0, 0}},
              // compute stand-ins near the MT = 2 kernel's per-role work (us x 100 ticks)
              {"compute stand-ins", {60, 150, 180, 150, 80, 60}}};
  std::string js = "{";
  for (int rep : {1, 2, 4, 8})
  for (int noload : {0, 1})
  for (const Cfg& c : cfgs) {
    if (rep > 1 && noload) continue;
    HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(g_noload), &noload, 4));
    HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(g_rep), &rep, 4));
    for (int mode : {0, 1, 2, 3}) {
      if (rep > 1 && (mode == 1 || mode == 2)) continue;
      std::memcpy(a.dl, c.dl, sizeof(a.dl));
      const void* f = mode == 0 ? (const void*)chain_kernel<0> : mode == 1 ? (const void*)chain_kernel<1>
                    : mode == 2 ? (const void*)chain_kernel<2> : (const void*)early_kernel;
      ensure_dyn_lds(f, 128 * 1024);
      float best = 1e30f;
      for (int rep = 0; rep < 3; ++rep) {
        HIP_OK(hipMemsetAsync(a.bar, 0, BAR_WORDS * 4, S));
        HIP_OK(hipMemcpyAsync(a.bar + BAR_TMO, &tmo, 4, hipMemcpyHostToDevice, S));
        HIP_OK(hipMemsetAsync(a.ctr, 0, 16384 * 4, S));
        HIP_OK(hipMemsetAsync(a.err, 0, 4, S));
        hipEvent_t e0, e1;
        HIP_OK(hipEventCreate(&e0));
        HIP_OK(hipEventCreate(&e1));
        HIP_OK(hipEventRecord(e0, S));
        CArgs cp = a;
        void* args[] = {&cp};
        launch_resident(f, dim3(PW), dim3(PT), args, 128 * 1024, S);
        HIP_OK(hipEventRecord(e1, S));
        HIP_OK(hipEventSynchronize(e1));
        float ms;
        HIP_OK(hipEventElapsedTime(&ms, e0, e1));
        unsigned e = 0, eb = 0;
        HIP_OK(hipMemcpy(&e, a.err, 4, hipMemcpyDeviceToHost));
        HIP_OK(hipMemcpy(&eb, a.bar + 16, 4, hipMemcpyDeviceToHost));
        if (e || eb) {
          printf("%s mode %d: wait timeout\n", c.name, mode);
          return 1;
        }
        best = std::min(best, ms);
      }
      printf("rep %d %-18s %-9s %s: %.2f us per step\n", rep, c.name, noload ? "no loads" : "loads",
             mode == 0 ? "grid barriers     " : mode == 1 ? "edge counters     " : mode == 2 ? "hierarchical edges" : "early arrivals    ",
             best * 1000.f / steps);
      js += std::string(js.size() > 1 ? ", " : "") + "\"" + (rep > 1 ? "rep" + std::to_string(rep) + "_" : std::string()) +
            (c.dl[0] ? "compute_" : "") + (noload ? "noload_" : "loads_") +
            (mode == 0 ? "barriers" : mode == 1 ? "edge_counters" : mode == 2 ? "hier_edges" : "early_arrival") + "_us\": " +
            std::to_string(best * 1000.f / steps);
    }
  }
  js += "}";
  if (argc > 1) {
    if (FILE* f = std::fopen(argv[1], "w")) {
      std::fprintf(f, "%s\n", js.c_str());
      std::fclose(f);
    }
  }
  printf("%s\ndone\n", js.c_str());
  return 0;
}
