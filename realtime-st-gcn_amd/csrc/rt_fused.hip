// RT-ST-GCN per-frame inference (config 3: models/rtstgcn/rtstgcn.py OnlineLayer / AggregateStgcn / Model
// after _swap_layers_for_inference), fp32, batch 1, one frame per call: the per-frame step as 2 launches
// per layer + 1 for the input head + 1 for the output head (the eager op-by-op path took ~60 launches and
// ~1 ms per frame, most of it tile-GEMM kernels sized for batches running a 25-row GEMM).
//
//   rt_in     : x (1,3,1,V) -> LayerNorm([3,1,V]) (per frame, unbiased var; layernorm.py:22-28) -> fcn_in
//               (1x1 conv + bias; rtstgcn.py:103) -> rows [V][C0]                               (1 block)
//   rt_gcn    : z = conv1x1(x) (+bias) mixed by A (tgcn as the online layer applies it, rtstgcn.py:531-537)
//               evaluated as z[v][co] = bias2d[v][co] + sum_{p,ci} W[p*Cout+co][ci] * XA_p[v][ci],
//               XA_p[v][ci] = sum_u A[p][u][v] x[u][ci] (A = graph * importance, OnlineLayer.eval_);
//               FIFO aggregation (AggregateStgcn.forward, rtstgcn.py:591-627): a = acc[ai] + z - fifo[fi],
//               acc[ai] = a, fifo[fi] = z; and the residual 1x1 conv (no bias) when the layer has one.
//               Grid over pairs of output channels; conv first (P*V*2 dot products), then the A-mix.
//   rt_norm   : y = relu(relu(LN(a)) + res) (residual; res = LN_r(r) | x) or relu(LN(a)) (rtstgcn.py:538-553),
//               LN over the frame's C*V values (two-pass mean / unbiased variance, fixed-order sums);
//               advances the FIFO indices.                                                    (1 block)
//   rt_out    : AvgPool over the V joints (rtstgcn.py:149) -> fcn_out (+ bias) -> (classes)      (1 block)
// Rows are channels-last [V][C] fp32 (the layout of the rest of the package); FIFO state [fifo][V][C],
// accumulators [S][V][C], indices int[2] (fifo, acc) — device buffers, so a HIP graph can replay frames.
#include "common.h"
#include "../../include/stgcn_amd.h"

namespace {

constexpr int NT = 256;
constexpr int CB = 2;        // output channels per rt_gcn block (Cout / 2 blocks: the weight rows stream in parallel)
constexpr int VMAX = 32;
constexpr int CMAX = 256;
constexpr int PMAX = 3;

// fixed-order block sum (NT threads): every thread gets the total
DEV float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
  return t;
}

// LayerNorm statistics (mean, 1/sqrt(unbiased var + eps)) of n values (two passes over the data)
DEV float2 ln_stats(const float* x, int n, float eps, float* red) {
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += x[i];
  const float mean = block_sum(s, red) / (float)n;
  float q = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float d = x[i] - mean;
    q = fmaf(d, d, q);
  }
  const float var = block_sum(q, red) / (float)(n - 1);
  return make_float2(mean, 1.f / sqrtf(var + eps));
}

__global__ __launch_bounds__(NT) void rt_in_kernel(const float* __restrict__ x, int V, const float* __restrict__ g,
                                                   const float* __restrict__ b, const float* __restrict__ W,
                                                   const float* __restrict__ bias, int C0, float eps,
                                                   float* __restrict__ out) {
  __shared__ float xs[3 * VMAX];
  __shared__ float red[NT / 64];
  const int n = 3 * V;  // (3, 1, V) per frame, element c*V + v
  for (int i = threadIdx.x; i < n; i += NT) xs[i] = x[i];
  __syncthreads();
  const float2 st = ln_stats(xs, n, eps, red);
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += NT) xs[i] = fmaf(g[i], (xs[i] - st.x) * st.y, b[i]);
  __syncthreads();
  for (int i = threadIdx.x; i < V * C0; i += NT) {
    const int v = i / C0, co = i - v * C0;
    float s = bias[co];
#pragma unroll
    for (int c = 0; c < 3; ++c) s = fmaf(W[co * 3 + c], xs[c * V + v], s);
    out[i] = s;
  }
}

// 8 lanes per dot product of length Cin (float4 k = kk + 8j: one contiguous 128-B piece per step),
// butterfly-summed; w from global (L2), x from LDS
DEV float dot8(const float* __restrict__ w, const float* x, int K4, int kk) {
  const float4* w4 = reinterpret_cast<const float4*>(w);
  const float4* x4 = reinterpret_cast<const float4*>(x);
  float s = 0.f;
  for (int k = kk; k < K4; k += 8) {
    const float4 a = w4[k], b = x4[k];
    s = fmaf(a.x, b.x, s);
    s = fmaf(a.y, b.y, s);
    s = fmaf(a.z, b.z, s);
    s = fmaf(a.w, b.w, s);
  }
#pragma unroll
  for (int m = 1; m < 8; m <<= 1) s += __shfl_xor(s, m);
  return s;
}

// conv first, as the reference (tgcn: conv1x1 then @A): y_p[u][co] = W_p[co] . x[u] for the block's CB
// channels (P*V*CB dot products), then z[v][co] = bias2d[v][co] + sum_{p,u} A[p][u][v] y_p[u][co]
__global__ __launch_bounds__(NT) void rt_gcn_kernel(const float* __restrict__ x, int V, int Cin, int Cout, int P,
                                                    const float* __restrict__ A, const float* __restrict__ W,
                                                    const float* __restrict__ bias2d, float* fifo, float* acc,
                                                    const int* __restrict__ idx, const float* __restrict__ Wr,
                                                    float* __restrict__ a_out, float* __restrict__ r_out) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* xs = sm;                 // [V][Cin]
  float* ys = xs + V * Cin;       // [P][V][CB]
  float* As = ys + P * V * CB;    // [P][V][V]
  const int tid = threadIdx.x, kk = tid & 7, K4 = Cin / 4;
  for (int i = tid; i < V * Cin / 4; i += NT) reinterpret_cast<float4*>(xs)[i] = reinterpret_cast<const float4*>(x)[i];
  for (int i = tid; i < P * V * V; i += NT) As[i] = A[i];
  __syncthreads();
  const int co0 = blockIdx.x * CB;
  for (int t0 = 0; t0 < P * V * CB; t0 += NT / 8) {
    const int t = t0 + (tid >> 3);
    const int cl = t % CB, pu = t / CB, u = pu % V, p = pu / V;
    const bool ok = t < P * V * CB && co0 + cl < Cout;
    const int co = ok ? co0 + cl : co0;
    const float y = dot8(W + ((long)(ok ? p : 0) * Cout + co) * Cin, xs + (ok ? u : 0) * Cin, K4, kk);
    if (ok && kk == 0) ys[t] = y;  // t = (p * V + u) * CB + cl
  }
  __syncthreads();
  const int fi = idx[0], ai = idx[1];
  const long E = (long)V * Cout;
  for (int t0 = 0; t0 < V * CB; t0 += NT / 8) {  // (v, cl) outputs, 8 lanes each
    const int tr = t0 + (tid >> 3);
    const int cl = tr % CB, v = tr / CB, co = co0 + cl;
    const bool ok = v < V && co < Cout;
    float r = 0.f;
    if (Wr) r = dot8(Wr + (long)(ok ? co : co0) * Cin, xs + (ok ? v : 0) * Cin, K4, kk);  // residual (no bias)
    if (ok && kk == 0) {
      float s = bias2d ? bias2d[v * Cout + co] : 0.f;
      for (int p = 0; p < P; ++p)
        for (int u = 0; u < V; ++u) s = fmaf(As[(p * V + u) * V + v], ys[(p * V + u) * CB + cl], s);
      const long e = (long)v * Cout + co;
      const float a = acc[ai * E + e] + s - fifo[fi * E + e];
      acc[ai * E + e] = a;
      fifo[fi * E + e] = s;
      a_out[e] = a;
      if (Wr) r_out[e] = r;
    }
  }
}

// LayerNorm statistics of n <= R * blockDim values held in registers (one global read; two-pass from registers)
template <int R>
DEV float2 ln_stats_regn(const float (&v)[R], int cnt, int n, float eps, float* red) {
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < R; ++j) s += j < cnt ? v[j] : 0.f;
  const float mean = block_sum(s, red) / (float)n;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const float d = j < cnt ? v[j] - mean : 0.f;
    q = fmaf(d, d, q);
  }
  const float var = block_sum(q, red) / (float)(n - 1);
  return make_float2(mean, 1.f / sqrtf(var + eps));
}

// res_mode: 0 none, 1 identity (x), 2 LN_r(r).  Element e = i * 1024 + thread.
__global__ __launch_bounds__(1024) void rt_norm_kernel(const float* __restrict__ a, const float* __restrict__ g,
                                                       const float* __restrict__ b, int res_mode,
                                                       const float* __restrict__ res, const float* __restrict__ gr,
                                                       const float* __restrict__ br, int V, int C, float eps,
                                                       int* idx, int fifo_size, int S, float* __restrict__ y) {
  __shared__ float red[16];
  const int n = V * C, tid = threadIdx.x;
  const int cnt = (n - tid + 1023) / 1024;
  float va[8], vr[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int e = j * 1024 + tid;
    va[j] = j < cnt ? a[e] : 0.f;
    vr[j] = (res_mode && j < cnt) ? res[e] : 0.f;
  }
  const float2 st = ln_stats_regn(va, cnt, n, eps, red);
  float2 sr = make_float2(0.f, 1.f);
  if (res_mode == 2) sr = ln_stats_regn(vr, cnt, n, eps, red);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (j >= cnt) break;
    const int e = j * 1024 + tid;
    const int v = e / C, c = e - v * C, gi = c * V + v;  // affine (C,1,V): element c*V + v
    float o = fmaxf(fmaf(g[gi], (va[j] - st.x) * st.y, b[gi]), 0.f);
    if (res_mode == 1) o = fmaxf(o + vr[j], 0.f);
    if (res_mode == 2) o = fmaxf(o + fmaf(gr[gi], (vr[j] - sr.x) * sr.y, br[gi]), 0.f);
    y[e] = o;
  }
  if (tid == 0) {
    idx[0] = (idx[0] + 1) % fifo_size;
    idx[1] = (idx[1] + 1) % S;
  }
}

__global__ __launch_bounds__(1024) void rt_out_kernel(const float* __restrict__ x, int V, int C,
                                                      const float* __restrict__ W, const float* __restrict__ bias,
                                                      int K, float* __restrict__ out) {
  __shared__ float pool[CMAX];
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float s = 0.f;
    for (int v = 0; v < V; ++v) s += x[v * C + c];
    pool[c] = s / (float)V;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int k = w; k < K; k += nw) {  // one wave per class, the channels over the lanes
    float s = 0.f;
    for (int c = lane; c < C; c += 64) s = fmaf(W[(long)k * C + c], pool[c], s);
    s = wave_sum(s);
    if (lane == 0) out[k] = s + (bias ? bias[k] : 0.f);
  }
}

// ------------------------------------------------------------------ the whole frame in one launch
// rt_frame_kernel: G persistent workgroups (all resident: G <= 256 and ~120 KB of LDS each, so one per CU).
// Every workgroup computes the input head into LDS, then per layer: (1) its channel pairs t = b, b + G, ... of
// the layer's conv1x1 + A-mix + FIFO step (+ residual conv) with x, the pair's weight rows and A in LDS, a / r
// stored to the layer's a_buf / r_buf; (2) a grid barrier; (3) the layer's norms over ALL channels from a_buf /
// r_buf, redundantly in every workgroup (a 25 KB read), written into LDS as the next layer's input — the only
// cross-workgroup traffic is a_buf / r_buf.  Everything the next layer needs that does not depend on the barrier
// (its first pair's weight rows, A, the pair's FIFO / accumulator values) is loaded into registers before the
// barrier, so those loads fly during the wait.  Workgroup 0 advances the FIFO indices of layer l after barrier l
// (every read of them precedes a workgroup's arrival; all of them are read at the start) and runs the output head.
// Hand-off (cdna_hip_programming.md Guideline 16, MI355X_MICROARCH.md "Valid forms", first table row): a_buf /
// r_buf are stored write-through (sc1: agent-scope relaxed atomic stores) and read with sc1 loads only, every
// storing wave drains (s_waitcnt vmcnt(0)) before a workgroup barrier, then ONE lane adds to one counter (relaxed
// agent atomic) and polls it (relaxed sc1 loads + s_sleep) until it reaches (phase + 1) * G; the other waves load
// after a workgroup barrier — so neither an L2 write-back nor an L1 invalidate is needed.  The counter is zeroed by a
// memset ahead of every launch; the spin is bounded (a wait that gives up sets *status; the launch still ends).
constexpr int RF_NT = 1024;
// per-phase s_memtime stamps of thread 0 of every workgroup (-DSTGCN_RT_PROF=1 builds only: tools/rt_prof.py)
#ifndef STGCN_RT_PROF
#define STGCN_RT_PROF 0
#endif
__device__ long long g_rt_prof[STGCN_RT_PROF ? 256 * STGCN_RT_MAX_LAYERS * 8 : 1];
#define RF_STAMP(l, k)                                                                              \
  do {                                                                                              \
    if (STGCN_RT_PROF && threadIdx.x == 64)                                                         \
      g_rt_prof[((long)blockIdx.x * STGCN_RT_MAX_LAYERS + (l)) * 8 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)

// The caller drains every wave's write-through stores (s_waitcnt vmcnt(0)) BEFORE issuing the loads it wants in flight
// across the barrier; the polling lane (wave 0) issues no such loads, so its sc1 polls wait for nothing else.
DEV void rf_grid_sync(unsigned* ctr, unsigned target, int* status) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
      unsigned spins = 0;
      while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins == (1u << 22)) {  // ~0.1 s: a workgroup never arrived
          __hip_atomic_store(status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
  }
  __syncthreads();
}

DEV void st_wt(float* p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
DEV float ld_wt(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Waves 1..15 issue every load that stays in flight across a barrier (wave 0 polls): worker index pt = tid - 64.
constexpr int RF_PT = RF_NT - 64;

// DPP sums (VALU only, fixed order; layer_fused.hip's half_sum): over the 32 lanes of each wave half, the totals
// in lanes 31 and 63; and over a whole block of RF_NT threads through red[RF_NT / 64]
template <int CTRL, int ROWS>
DEV float rf_dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROWS, 0xf, false));
}
DEV float rf_half_sum(float v) {
  v += rf_dpp<0xB1, 0xf>(v);   // quad_perm [1,0,3,2]
  v += rf_dpp<0x4E, 0xf>(v);   // quad_perm [2,3,0,1]
  v += rf_dpp<0x141, 0xf>(v);  // row_half_mirror: 8-lane sums
  v += rf_dpp<0x140, 0xf>(v);  // row_mirror: 16-lane (row) sums
  v += rf_dpp<0x142, 0xa>(v);  // row_bcast15 into rows 1 and 3
  return v;
}
DEV float rf_block_sum(float v, float* red) {
  v = rf_half_sum(v);
  v = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 31)) +
      __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
  __syncthreads();  // the previous reduction's reads of red are done
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < RF_NT / 64; ++i) t += red[i];
  return t;
}

DEV float2 rf_block_sum2(float2 v, float* red) {  // two sums at once; red holds 2 * RF_NT / 64 floats
  float a = rf_half_sum(v.x), b = rf_half_sum(v.y);
  a = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, a), 31)) +
      __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, a), 63));
  b = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, b), 31)) +
      __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, b), 63));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x >> 6] = a;
    red[RF_NT / 64 + (threadIdx.x >> 6)] = b;
  }
  __syncthreads();
  float2 t = make_float2(0.f, 0.f);
#pragma unroll
  for (int i = 0; i < RF_NT / 64; ++i) {
    t.x += red[i];
    t.y += red[RF_NT / 64 + i];
  }
  return t;
}

// output channels per task of the one-launch kernel (build flag for A/B: 4 channels, one task per workgroup at
// G = 64 up to C = 256, measured 0.127 vs 0.109 ms/frame: the 12-row conv spills)
#ifndef STGCN_RT_CB
#define STGCN_RT_CB 2
#endif
constexpr int RF_CB = STGCN_RT_CB;
// W rows of one channel-group task, staged in LDS: rows [0, P*RF_CB) = conv rows (p, cl) -> w[(p*Cout + co0 + cl)],
// then RF_CB residual rows (res_mode 2); each thread moves at most RF_WU float4 units
constexpr int RF_WROWS = PMAX * RF_CB + RF_CB;
constexpr int RF_WU = (RF_WROWS * CMAX / 4 + RF_PT - 1) / RF_PT;
constexpr int RF_AU = (PMAX * VMAX * VMAX + RF_PT - 1) / RF_PT;  // A floats per worker
constexpr int RF_FU = (VMAX * RF_CB + RF_PT / 8 - 1) / (RF_PT / 8);  // FIFO outputs per 8-lane group

// everything a task needs from memory before its arithmetic: weight rows, A (first task of a layer only), and the
// FIFO / accumulator values of its outputs
struct RfPre {
  float4 w[RF_WU];
  float a[RF_AU];
  float acc[RF_FU], fifo[RF_FU], bias[RF_FU];
};

DEV int rf_nrows(const stgcn_rt_layer& ly) { return ly.P * RF_CB + (ly.res_mode == 2 ? RF_CB : 0); }

DEV void rf_prefetch(const stgcn_rt_layer& ly, int co0, int V, int fi, int ai, bool withA, RfPre& r) {
  const int K4 = ly.Cin / 4, n = rf_nrows(ly) * K4;
  const int pt = (int)threadIdx.x - 64;  // < 0: wave 0, no loads
#pragma unroll
  for (int u = 0; u < RF_WU; ++u) {
    const int i = pt < 0 ? n : pt + RF_PT * u;
    r.w[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (i < n) {
      const int row = i / K4, k4 = i - row * K4;
      const bool res = row >= ly.P * RF_CB;
      const int cl = res ? row - ly.P * RF_CB : row % RF_CB, p = res ? 0 : row / RF_CB, co = co0 + cl;
      if (co < ly.Cout) {
        const float* src = res ? ly.wr + (long)co * ly.Cin : ly.w + ((long)p * ly.Cout + co) * ly.Cin;
        r.w[u] = reinterpret_cast<const float4*>(src)[k4];
      }
    }
  }
  if (withA) {
#pragma unroll
    for (int u = 0; u < RF_AU; ++u) {
      const int i = pt + RF_PT * u;
      r.a[u] = pt >= 0 && i < ly.P * V * V ? ly.A[i] : 0.f;
    }
  }
  const long E = (long)V * ly.Cout;
#pragma unroll
  for (int u = 0; u < RF_FU; ++u) {
    const int tr = (pt >> 3) + (RF_PT / 8) * u;
    const int cl = tr % RF_CB, v = tr / RF_CB, co = co0 + cl;
    const bool ok = pt >= 0 && (pt & 7) == 0 && v < V && co < ly.Cout;
    const long e = (long)v * ly.Cout + co;
    r.acc[u] = ok ? ly.acc[ai * E + e] : 0.f;
    r.fifo[u] = ok ? ly.fifo[fi * E + e] : 0.f;
    r.bias[u] = ok && ly.bias2d ? ly.bias2d[e] : 0.f;
  }
}

DEV void rf_stage(const stgcn_rt_layer& ly, int V, bool withA, const RfPre& r, float* wsm, float* As) {
  const int n = rf_nrows(ly) * (ly.Cin / 4);
  const int pt = (int)threadIdx.x - 64;
  if (pt < 0) return;
#pragma unroll
  for (int u = 0; u < RF_WU; ++u) {
    const int i = pt + RF_PT * u;
    if (i < n) reinterpret_cast<float4*>(wsm)[i] = r.w[u];
  }
  if (withA) {
#pragma unroll
    for (int u = 0; u < RF_AU; ++u) {
      const int i = pt + RF_PT * u;
      if (i < ly.P * V * V) As[i] = r.a[u];
    }
  }
}

// 8-lane dot product of two LDS rows of K4 float4 (lane kk takes k = kk, kk + 8, ...), butterfly-summed
DEV float rf_dot8(const float* w, const float* x, int K4, int kk) {
  const float4* w4 = reinterpret_cast<const float4*>(w);
  const float4* x4 = reinterpret_cast<const float4*>(x);
  float s = 0.f;
#pragma unroll 4
  for (int k = kk; k < K4; k += 8) {
    const float4 a = w4[k], b = x4[k];
    s = fmaf(a.x, b.x, s);
    s = fmaf(a.y, b.y, s);
    s = fmaf(a.z, b.z, s);
    s = fmaf(a.w, b.w, s);
  }
#pragma unroll
  for (int m = 1; m < 8; m <<= 1) s += __shfl_xor(s, m);
  return s;
}

// the norm phase: 16-B unit e4 = pt + RF_PT * j (elements 4*e4 .. 4*e4+3) of the frame's [V][Cout] rows, j < RF_U4,
// in the workers' registers
constexpr int RF_U4 = 2;
constexpr int RF_MAXE = RF_U4 * RF_PT * 4;  // V * Cout limit of the one-launch kernel (7680: V = 25 at C = 256)
struct RfLn {
  float4 w[RF_U4], b[RF_U4], rw[RF_U4], rb[RF_U4];
};
// the layer's LayerNorm affine(s) in the rows' [V][Cout] layout (coalesced 16-B loads), issued before the barrier
DEV float4 ld4(__amdgpu_buffer_rsrc_t r, int e4) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, e4 * 16, 0, 0));
}
DEV void rf_ln_prefetch(const stgcn_rt_layer& ly, int n4, RfLn& p) {
  const int pt = (int)threadIdx.x - 64;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  const bool two = ly.res_mode == 2;
  const __amdgpu_buffer_rsrc_t rw_ = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(ly.ln_w), 0, n4 * 16, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb_ = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(ly.ln_b), 0, n4 * 16, 0x00020000);
  const __amdgpu_buffer_rsrc_t rrw_ =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(two ? ly.lnr_w : ly.ln_w), 0, n4 * 16, 0x00020000);
  const __amdgpu_buffer_rsrc_t rrb_ =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(two ? ly.lnr_b : ly.ln_b), 0, n4 * 16, 0x00020000);
#pragma unroll
  for (int j = 0; j < RF_U4; ++j) {
    const int e4 = pt + RF_PT * j;
    const bool ok = pt >= 0 && e4 < n4, r2 = ok && ly.res_mode == 2;
    p.w[j] = ok ? ld4(rw_, e4) : z;
    p.b[j] = ok ? ld4(rb_, e4) : z;
    p.rw[j] = r2 ? ld4(rrw_, e4) : z;
    p.rb[j] = r2 ? ld4(rrb_, e4) : z;
  }
}

// 16-B write-through (sc1) load of a handed-off unit: buffer load with aux 16 = sc1, the descriptor built from
// kernel-argument (wave-uniform) values
DEV float4 ld_wt4(__amdgpu_buffer_rsrc_t r, int e4) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, e4 * 16, 0, 16));
}
DEV float sum4(float4 v) { return (v.x + v.y) + (v.z + v.w); }
DEV float sq4(float4 v, float m) {
  const float a = v.x - m, b = v.y - m, c = v.z - m, d = v.w - m;
  return fmaf(a, a, fmaf(b, b, fmaf(c, c, d * d)));
}

// dynamic LDS carve (floats): xs [VMAX*CMAX] (the current layer's input), wsm, ys, As, red, idx
constexpr int RF_LDS_FLOATS = VMAX * CMAX + RF_WROWS * CMAX + PMAX * VMAX * RF_CB + PMAX * VMAX * VMAX + 64 +
                              2 * STGCN_RT_MAX_LAYERS;

__global__ __launch_bounds__(RF_NT) void rt_frame_kernel(const stgcn_rt_frame_desc d) {
  extern __shared__ __attribute__((aligned(16))) float rf_sm[];
  float* xs = rf_sm;                     // [V][C] the current layer's input
  float* wsm = xs + VMAX * CMAX;         // [RF_WROWS][Cin] weight rows of the current task
  float* ys = wsm + RF_WROWS * CMAX;     // [P][V][RF_CB]
  float* As = ys + PMAX * VMAX * RF_CB;     // [P][V][V]
  float* red = As + PMAX * VMAX * VMAX;  // [RF_NT / 64]
  int* sidx = reinterpret_cast<int*>(red + 64);  // (fifo, acc) index of every layer, read once at the start
  const int tid = threadIdx.x, kk = tid & 7, G = gridDim.x, V = d.V;
  if (tid < 2 * d.L) sidx[tid] = d.layers[tid >> 1].idx[tid & 1];
  __syncthreads();
  RfPre pre;
  // layer 0's first task: in flight during the input head
  if ((int)blockIdx.x * RF_CB < d.layers[0].Cout) rf_prefetch(d.layers[0], blockIdx.x * RF_CB, V, sidx[0], sidx[1], true, pre);
  else rf_prefetch(d.layers[0], 0, V, sidx[0], sidx[1], true, pre);  // A only is used

  // input head: LayerNorm([3,1,V]) + fcn_in (rt_in_kernel's arithmetic), every workgroup
  {
    float* xi = ys;  // 3 * V <= 96 < PMAX * VMAX * RF_CB
    const int n = 3 * V;
    for (int i = tid; i < n; i += RF_NT) xi[i] = d.x[i];
    __syncthreads();
    const float2 st = ln_stats(xi, n, 1e-5f, red);
    __syncthreads();
    for (int i = tid; i < n; i += RF_NT) xi[i] = fmaf(d.ln_w[i], (xi[i] - st.x) * st.y, d.ln_b[i]);
    __syncthreads();
    for (int i = tid; i < V * d.C0; i += RF_NT) {
      const int v = i / d.C0, co = i - v * d.C0;
      float s = d.b_in[co];
#pragma unroll
      for (int c = 0; c < 3; ++c) s = fmaf(d.w_in[co * 3 + c], xi[c * V + v], s);
      xs[i] = s;
    }
  }

  for (int l = 0; l < d.L; ++l) {
    // this layer's and the next layer's descriptors as whole-struct copies at the top: their scalar loads are issued
    // together here instead of one dependent s_load + wait per field use deep inside the phases
    const stgcn_rt_layer ly = d.layers[l];
    const stgcn_rt_layer nx = d.layers[l + 1 < d.L ? l + 1 : l];
    const int Cin = ly.Cin, Cout = ly.Cout, P = ly.P, K4 = Cin / 4;
    const int fi = sidx[2 * l], ai = sidx[2 * l + 1];
    const long E = (long)V * Cout;
    RF_STAMP(l, 0);
    // (1) conv1x1 + A-mix + FIFO (+ residual conv) of this workgroup's channel pairs
    bool first = true;
    for (int task = blockIdx.x; task * RF_CB < Cout || first; task += G) {
      const int co0 = task * RF_CB;
      if (!first) {  // the first task's operands were prefetched (and staged during the previous norm phase)
        __syncthreads();  // every read of wsm by the previous task
        rf_prefetch(ly, co0, V, fi, ai, false, pre);
        rf_stage(ly, V, false, pre, wsm, As);
      } else if (l == 0) {
        rf_stage(ly, V, true, pre, wsm, As);
      }
      first = false;
      if (co0 >= Cout) break;  // no pair here: A staged only (kept for uniformity)
      __syncthreads();
      // conv rows: ys[(p*V + u)*RF_CB + cl] = w_(p, co0+cl) . x[u]; half-wave h = joint u, its 32 lanes split Cin
      // (k = lane, lane + 32, ...) and keep all P*RF_CB rows' sums (one x read per k for the pair's rows), DPP-summed
      {
        const int h = tid >> 5, l32 = tid & 31, u = h < V ? h : 0;
        const float4* x4 = reinterpret_cast<const float4*>(xs) + u * K4;
        const float4* w4 = reinterpret_cast<const float4*>(wsm);
        float acc[PMAX * RF_CB];
#pragma unroll
        for (int r = 0; r < PMAX * RF_CB; ++r) acc[r] = 0.f;
        for (int k = l32; k < K4; k += 32) {
          const float4 xv = x4[k];
#pragma unroll
          for (int r = 0; r < PMAX * RF_CB; ++r) {
            if (r < P * RF_CB) {
              const float4 wv = w4[r * K4 + k];
              acc[r] = fmaf(wv.x, xv.x, fmaf(wv.y, xv.y, fmaf(wv.z, xv.z, fmaf(wv.w, xv.w, acc[r]))));
            }
          }
        }
#pragma unroll
        for (int r = 0; r < PMAX * RF_CB; ++r) {
          if (r < P * RF_CB) {
            const float t = rf_half_sum(acc[r]);
            if (l32 == 31 && h < V) ys[((r / RF_CB) * V + u) * RF_CB + r % RF_CB] = t;
          }
        }
      }
      __syncthreads();
      RF_STAMP(l, 1);
      // A-mix over (p, u) split over the 8 lanes of an output (u = kk, kk + 8, ...), FIFO step, residual conv
      // (workers only: the FIFO values were prefetched by the worker that uses them)
#pragma unroll
      for (int q = 0; q < RF_FU; ++q) {
        if (tid < 64) break;  // wave-uniform
        const int tr = ((tid - 64) >> 3) + (RF_PT / 8) * q;
        const int cl = tr % RF_CB, v = tr / RF_CB, co = co0 + cl;
        const bool ok = v < V && co < Cout;
        float r = 0.f;
        if (ly.res_mode == 2) r = rf_dot8(wsm + (P * RF_CB + cl) * Cin, xs + (ok ? v : 0) * Cin, K4, kk);
        float s = 0.f;
        if (ok)
          for (int p = 0; p < P; ++p)
            for (int u = kk; u < V; u += 8) s = fmaf(As[(p * V + u) * V + v], ys[(p * V + u) * RF_CB + cl], s);
#pragma unroll
        for (int m = 1; m < 8; m <<= 1) s += __shfl_xor(s, m);
        if (ok && kk == 0) {
          s += pre.bias[q];
          const long e = (long)v * Cout + co;
          const float a = pre.acc[q] + s - pre.fifo[q];
          ly.acc[ai * E + e] = a;
          ly.fifo[fi * E + e] = s;
          st_wt(ly.a_buf + e, a);
          if (ly.res_mode == 2) st_wt(ly.r_buf + e, r);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave: its write-through stores have completed
    RF_STAMP(l, 2);
    // the next layer's first task (weight rows, A, FIFO values): in flight across the barrier
    if (l + 1 < d.L) {
      rf_prefetch(nx, (int)blockIdx.x * RF_CB < nx.Cout ? blockIdx.x * RF_CB : 0, V, sidx[2 * l + 2], sidx[2 * l + 3], true,
                  pre);
    }
    RfLn lnp;
    rf_ln_prefetch(ly, V * Cout / 4, lnp);
    RF_STAMP(l, 3);
    // (2) every workgroup's a_buf / r_buf slice published
    rf_grid_sync(d.sync, (unsigned)(l + 1) * (unsigned)G, d.status);
    RF_STAMP(l, 4);
    if (blockIdx.x == 0 && tid == 0) {  // no workgroup reads layer l's indices after barrier l
      ly.idx[0] = (fi + 1) % ly.fifo_size;
      ly.idx[1] = (ai + 1) % ly.S;
    }
    // (3) y = relu(relu(LN(a)) + res) over the whole frame, into xs (the next layer's input): a (and r) in the
    // workers' registers by 16-B write-through (sc1) loads; two-pass statistics of both norms from registers with one
    // block reduction per pass (rt_norm_kernel's math, another fixed order)
    {
      const int n = V * Cout, n4 = n / 4, pt = tid - 64;
      const int cnt = pt >= 0 && pt < n4 ? (n4 - pt + RF_PT - 1) / RF_PT : 0;
      const __amdgpu_buffer_rsrc_t ra_ = __builtin_amdgcn_make_buffer_rsrc(ly.a_buf, 0, n * 4, 0x00020000);
      const __amdgpu_buffer_rsrc_t rr_ =
          __builtin_amdgcn_make_buffer_rsrc(ly.res_mode == 2 ? ly.r_buf : ly.a_buf, 0, n * 4, 0x00020000);
      const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
      float4 va[RF_U4], vr[RF_U4];
#pragma unroll
      for (int j = 0; j < RF_U4; ++j) {
        const int e4 = pt + RF_PT * j;
        va[j] = j < cnt ? ld_wt4(ra_, e4) : z;
        vr[j] = j >= cnt ? z : ly.res_mode == 2 ? ld_wt4(rr_, e4)
                             : ly.res_mode == 1 ? reinterpret_cast<const float4*>(xs)[e4] : z;
      }
      RF_STAMP(l, 5);
      const bool two = ly.res_mode == 2;
      float sa = 0.f, sb = 0.f;
#pragma unroll
      for (int j = 0; j < RF_U4; ++j) {
        sa += sum4(va[j]);
        sb += sum4(vr[j]);
      }
      // the next layer's prefetched operands have landed (loads complete in order, before these a loads): stage them
      // now (wsm / As are free after the barrier) so their registers are free for the rest of this phase
      if (l + 1 < d.L) rf_stage(nx, V, true, pre, wsm, As);
      const float2 m = rf_block_sum2(make_float2(sa, two ? sb : 0.f), red);
      const float ma = m.x / (float)n, mb = m.y / (float)n;
      float qa = 0.f, qb = 0.f;
#pragma unroll
      for (int j = 0; j < RF_U4; ++j) {
        if (j < cnt) {
          qa += sq4(va[j], ma);
          qb += sq4(vr[j], mb);
        }
      }
      const float2 q = rf_block_sum2(make_float2(qa, two ? qb : 0.f), red);
      const float ra = 1.f / sqrtf(q.x / (float)(n - 1) + 1e-5f), rb = 1.f / sqrtf(q.y / (float)(n - 1) + 1e-5f);
      RF_STAMP(l, 6);
      __syncthreads();  // every read of xs (the residual x) before the overwrite
#pragma unroll
      for (int j = 0; j < RF_U4; ++j) {
        if (j < cnt) {
          const float4 a = va[j], r = vr[j], w = lnp.w[j], b = lnp.b[j];
          float o[4] = {fmaxf(fmaf(w.x, (a.x - ma) * ra, b.x), 0.f), fmaxf(fmaf(w.y, (a.y - ma) * ra, b.y), 0.f),
                        fmaxf(fmaf(w.z, (a.z - ma) * ra, b.z), 0.f), fmaxf(fmaf(w.w, (a.w - ma) * ra, b.w), 0.f)};
          const float rv[4] = {r.x, r.y, r.z, r.w};
          if (ly.res_mode == 1) {
#pragma unroll
            for (int c = 0; c < 4; ++c) o[c] = fmaxf(o[c] + rv[c], 0.f);
          }
          if (two) {
            const float gw[4] = {lnp.rw[j].x, lnp.rw[j].y, lnp.rw[j].z, lnp.rw[j].w};
            const float gb[4] = {lnp.rb[j].x, lnp.rb[j].y, lnp.rb[j].z, lnp.rb[j].w};
#pragma unroll
            for (int c = 0; c < 4; ++c) o[c] = fmaxf(o[c] + fmaf(gw[c], (rv[c] - mb) * rb, gb[c]), 0.f);
          }
          reinterpret_cast<float4*>(xs)[pt + RF_PT * j] = make_float4(o[0], o[1], o[2], o[3]);
        }
      }
      __syncthreads();
      RF_STAMP(l, 7);
    }
  }

  // output head (rt_out_kernel's arithmetic) on workgroup 0
  if (blockIdx.x == 0) {
    const int C = d.layers[d.L - 1].Cout;
    float* pool = As;
    for (int c = tid; c < C; c += RF_NT) {
      float s = 0.f;
      for (int v = 0; v < V; ++v) s += xs[v * C + c];
      pool[c] = s / (float)V;
    }
    __syncthreads();
    const int lane = tid & 63, w = tid >> 6;
    for (int k = w; k < d.K; k += RF_NT / 64) {
      float s = 0.f;
      for (int c = lane; c < C; c += 64) s = fmaf(d.w_out[(long)k * C + c], pool[c], s);
      s = wave_sum(s);
      if (lane == 0) d.out[k] = s + (d.b_out ? d.b_out[k] : 0.f);
    }
  }
}

}  // namespace

int rt_frame_launch(const stgcn_rt_frame_desc& d, hipStream_t s) {
  if (!d.x || !d.ln_w || !d.ln_b || !d.w_in || !d.b_in || !d.w_out || !d.out || !d.sync || !d.status)
    return STGCN_EBADSHAPE;
  if (d.V < 2 || d.V > VMAX || d.L < 1 || d.L > STGCN_RT_MAX_LAYERS || d.C0 < 4 || d.C0 > CMAX || d.C0 % 4 || d.K < 1 ||
      d.blocks < 0 || d.blocks > 256)
    return STGCN_EBADSHAPE;
  int cin = d.C0;
  for (int l = 0; l < d.L; ++l) {
    const stgcn_rt_layer& y = d.layers[l];
    if (y.Cin != cin || y.Cout < 4 || y.Cout > CMAX || y.Cout % 4 || d.V * y.Cout > RF_MAXE || y.P < 1 || y.P > PMAX ||
        y.fifo_size < 1 ||
        y.S < 1 || y.res_mode < 0 || y.res_mode > 2 || (y.res_mode == 1 && y.Cin != y.Cout))
      return STGCN_EBADSHAPE;
    if (!y.A || !y.w || !y.ln_w || !y.ln_b || !y.fifo || !y.acc || !y.idx || !y.a_buf ||
        (y.res_mode == 2 && (!y.wr || !y.lnr_w || !y.lnr_b || !y.r_buf)))
      return STGCN_EBADSHAPE;
    cin = y.Cout;
  }
  const int G = d.blocks ? d.blocks : 64;
  constexpr int lds = RF_LDS_FLOATS * (int)sizeof(float);
  if (stgcn_lds_attr((const void*)rt_frame_kernel, lds, s)) return STGCN_EHIP;
  if (hipMemsetAsync(d.sync, 0, 16, s) != hipSuccess) return STGCN_EHIP;
  hipLaunchKernelGGL(rt_frame_kernel, dim3((unsigned)G), dim3(RF_NT), lds, s, d);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

extern "C" int stgcn_rt_prof(void* dst, long n) {
  if (!STGCN_RT_PROF || n > 256L * STGCN_RT_MAX_LAYERS * 8) return -1;
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_rt_prof), n * sizeof(long long), 0, hipMemcpyDeviceToHost) == hipSuccess
             ? 0 : -1;
}

int rt_in_launch(const float* x, int V, const float* g, const float* b, const float* W, const float* bias, int C0,
                 float* out, hipStream_t s) {
  if (!x || !g || !b || !W || !bias || !out || V < 2 || V > VMAX || C0 < 1) return STGCN_EBADSHAPE;
  hipLaunchKernelGGL(rt_in_kernel, dim3(1), dim3(NT), 0, s, x, V, g, b, W, bias, C0, 1e-5f, out);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

int rt_gcn_launch(const float* x, int V, int Cin, int Cout, int P, const float* A, const float* W, const float* bias2d,
                  float* fifo, float* acc, const int* idx, const float* Wr, float* a_out, float* r_out,
                  hipStream_t s) {
  if (!x || !A || !W || !fifo || !acc || !idx || !a_out || (Wr && !r_out)) return STGCN_EBADSHAPE;
  if (V < 1 || V > VMAX || Cin < 4 || Cin > CMAX || Cin % 4 || Cout < 1 || P < 1 || P > PMAX) return STGCN_EBADSHAPE;
  const size_t lds = ((size_t)V * Cin + (size_t)P * V * CB + (size_t)P * V * V) * sizeof(float);
  if (lds > 160 * 1024) return STGCN_EBADSHAPE;
  if (stgcn_lds_attr((const void*)rt_gcn_kernel, 160 * 1024, s)) return STGCN_EHIP;
  hipLaunchKernelGGL(rt_gcn_kernel, dim3((unsigned)((Cout + CB - 1) / CB)), dim3(NT), lds, s, x, V, Cin, Cout, P, A, W,
                     bias2d, fifo, acc, idx, Wr, a_out, r_out);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

int rt_norm_launch(const float* a, const float* g, const float* b, int res_mode, const float* res, const float* gr,
                   const float* br, int V, int C, int* idx, int fifo_size, int S, float* y, hipStream_t s) {
  if (!a || !g || !b || !idx || !y || V * C < 2 || V * C > 8 * 1024 || fifo_size < 1 || S < 1 || res_mode < 0 ||
      res_mode > 2 ||
      (res_mode && !res) || (res_mode == 2 && (!gr || !br)))
    return STGCN_EBADSHAPE;
  hipLaunchKernelGGL(rt_norm_kernel, dim3(1), dim3(1024), 0, s, a, g, b, res_mode, res, gr, br, V, C, 1e-5f, idx,
                     fifo_size, S, y);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

int rt_out_launch(const float* x, int V, int C, const float* W, const float* bias, int K, float* out, hipStream_t s) {
  if (!x || !W || !out || V < 1 || C < 1 || C > CMAX || K < 1) return STGCN_EBADSHAPE;
  hipLaunchKernelGGL(rt_out_kernel, dim3(1), dim3(1024), 0, s, x, V, C, W, bias, K, out);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
