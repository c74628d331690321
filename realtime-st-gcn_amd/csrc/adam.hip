// Adam over every parameter of a model in ONE launch (include/stgcn_amd.h, stgcn_adam_*).
// Replaces the reference's optimizer step (processor.py:561; torch.optim.Adam built at processor.py:579,
// config learning_rate 5e-4): torch's fused multi-tensor Adam needs three launches for the 96 tensors of the config-2
// model (its kernel-argument chunks) plus the step-counter increments; this is one grid that streams
// p, g, m, v once (HBM-bound: 28 B per element, 3.06 M elements -> ~86 MB per step).
// Layout: the moments m, v live in two flat fp32 buffers (16-B aligned slice per tensor); a static device
// table holds per tensor (p, m, v, n, first block); the gradient pointers change every step and travel
// as kernel arguments.  Each block owns a private step counter slot (read and rewritten by that block
// only, so no cross-block ordering and no atomics): all slots of a tensor advance together, and a tensor
// whose gradient is NULL is skipped with its counters unchanged, as torch skips params without grads.
#include "common.h"
#include "../../include/stgcn_amd.h"

namespace {

constexpr int EPB = 2048;  // elements per block: 256 threads x 2 float4

struct AdamGrads {
  const float* g[STGCN_ADAM_MAXT];
};

__global__ __launch_bounds__(256) void adam_kernel(const stgcn_adam_entry* __restrict__ tab, int nt,
                                                   const AdamGrads gr, float* __restrict__ steps, double lr,
                                                   double beta1, double beta2, double eps, double wd) {
  const long b = blockIdx.x;
  int lo = 0, hi = nt - 1;  // last tensor with b0 <= b
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (tab[mid].b0 <= b) lo = mid;
    else hi = mid - 1;
  }
  const float* __restrict__ g = gr.g[lo];
  if (!g) return;  // block-uniform
  const stgcn_adam_entry e = tab[lo];
  const float t = steps[b] + 1.f;
  // torch.optim.Adam's default (foreach) update, hyper-parameters as Python floats (double) cast to fp32 where
  // the foreach kernels take them: m = lerp(m, g, 1 - b1); v = v * b2 + (1 - b2) * g * g;
  // p += (-lr / (1 - b1^t)) * (m / (sqrt(v) / sqrt(1 - b2^t) + eps))
  const double bc1 = 1.0 - pow(beta1, (double)t);
  const float nstep = (float)(-lr / bc1);
  const float bc2s = (float)sqrt(1.0 - pow(beta2, (double)t));
  const float wl = (float)(1.0 - beta1), b2 = (float)beta2, ob2 = (float)(1.0 - beta2), ep = (float)eps;
  const float wdf = (float)wd;
  auto upd = [&](float& p, float gv, float& m, float& v) {
    if (wdf != 0.f) gv = gv + wdf * p;  // grad.add(param, alpha=weight_decay)
    m = m + wl * (gv - m);              // lerp, weight < 0.5
    v = v * b2 + ob2 * gv * gv;         // addcmul(g, g, value=1 - b2)
    const float denom = sqrtf(v) / bc2s + ep;
    p = p + nstep * (m / denom);        // addcdiv(m, denom, value=-step_size)
  };
  const long base = (b - e.b0) * EPB;
  // every pointer 16-B aligned: float4 units, the loads of both units issued first
  if (e.vec && (reinterpret_cast<unsigned long>(g) & 15) == 0) {
    float4 P[2], G[2], M[2], Vv[2];
    bool ok[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const long i = base + (long)(u * 256 + threadIdx.x) * 4;
      ok[u] = i + 4 <= e.n;
      if (ok[u]) {
        P[u] = *reinterpret_cast<const float4*>(e.p + i);
        G[u] = *reinterpret_cast<const float4*>(g + i);
        M[u] = *reinterpret_cast<const float4*>(e.m + i);
        Vv[u] = *reinterpret_cast<const float4*>(e.v + i);
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const long i = base + (long)(u * 256 + threadIdx.x) * 4;
      if (ok[u]) {
        upd(P[u].x, G[u].x, M[u].x, Vv[u].x);
        upd(P[u].y, G[u].y, M[u].y, Vv[u].y);
        upd(P[u].z, G[u].z, M[u].z, Vv[u].z);
        upd(P[u].w, G[u].w, M[u].w, Vv[u].w);
        *reinterpret_cast<float4*>(e.p + i) = P[u];
        *reinterpret_cast<float4*>(e.m + i) = M[u];
        *reinterpret_cast<float4*>(e.v + i) = Vv[u];
      } else {  // tail of the tensor: scalar
        for (long k = i; k < min(i + 4, e.n); ++k) {
          float p = e.p[k], m = e.m[k], v = e.v[k];
          upd(p, g[k], m, v);
          e.p[k] = p;
          e.m[k] = m;
          e.v[k] = v;
        }
      }
    }
  } else {
    for (long k = base + threadIdx.x; k < min(base + EPB, e.n); k += 256) {
      float p = e.p[k], m = e.m[k], v = e.v[k];
      upd(p, g[k], m, v);
      e.p[k] = p;
      e.m[k] = m;
      e.v[k] = v;
    }
  }
  __syncthreads();  // every thread has read steps[b]
  if (threadIdx.x == 0) steps[b] = t;
}

}  // namespace

extern "C" long stgcn_adam_blocks(long n) { return (n + EPB - 1) / EPB; }

extern "C" int stgcn_adam_step(const stgcn_adam_entry* table_dev, int ntensors, long nblocks,
                               const float* const* grads, float* steps, double lr, double beta1, double beta2,
                               double eps, double weight_decay, void* stream) {
  if (!table_dev || !grads || !steps || ntensors <= 0 || ntensors > STGCN_ADAM_MAXT || nblocks <= 0 ||
      nblocks > 0x7fffffffL)
    return STGCN_EBADSHAPE;
  AdamGrads gr;
  for (int i = 0; i < STGCN_ADAM_MAXT; ++i) gr.g[i] = i < ntensors ? grads[i] : nullptr;
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)nblocks), dim3(256), 0, (hipStream_t)stream, table_dev, ntensors,
                     gr, steps, lr, beta1, beta2, eps, weight_decay);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
