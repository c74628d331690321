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

// LayerNorm statistics of n <= 8 * 1024 values held in registers (one global read; two-pass from registers)
DEV float2 ln_stats_reg(const float (&v)[8], int cnt, int n, float eps, float* red) {
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += j < cnt ? v[j] : 0.f;
  const float mean = block_sum(s, red) / (float)n;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
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
  const float2 st = ln_stats_reg(va, cnt, n, eps, red);
  float2 sr = make_float2(0.f, 1.f);
  if (res_mode == 2) sr = ln_stats_reg(vr, cnt, n, eps, red);
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

}  // namespace

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
