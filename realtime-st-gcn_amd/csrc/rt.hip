// RT-ST-GCN temporal aggregation (models/rtstgcn/rtstgcn.py).
//
// OfflineLayer (rtstgcn.py:366-379) sums the A-mixed features over a causal window by a dense
// L x L Toeplitz matmul (O(L^2)).  Its algorithm is a causal, unweighted box sum of K/S taps at
// dilation S; we evaluate exactly that in O(K/S) per output:
//     y[(n,t,v)][c] = sum_{i < K/S, t - i*S >= 0} x[(n, t - i*S, v)][c]          (trans = 0)
//     y[(n,t,v)][c] = sum_{i < K/S, t + i*S <  T} x[(n, t + i*S, v)][c]          (trans = 1, adjoint)
//
// OnlineLayer/AggregateStgcn (rtstgcn.py:591-627) keeps a FIFO of the last S*(K-1)+1 frames and
// S running accumulators; one step:  acc[ai] += z - fifo[fi];  out = acc[ai];  fifo[fi] = z;
// ai = (ai+1) % S;  fi = (fi+1) % fifo_size.  The state lives in device buffers (the reference
// keeps it in CPU tensors, rtstgcn.py:576-579) and the indices in a device int[2], so the step can
// be replayed from a HIP graph.
#include "common.h"

namespace {

template <typename T>
__global__ __launch_bounds__(256) void box_sum_kernel(const T* __restrict__ x, int ldx, T* __restrict__ y, int ldy,
                                                      int N, int T_, int V, int C, int K, int S, int trans,
                                                      int accumulate) {
  const long total = (long)N * T_ * V * C;
  const int taps = K / S;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long m = i / C;
    const int c = (int)(i % C);
    const int v = (int)(m % V);
    const long nt = m / V;
    const int t = (int)(nt % T_);
    const long n = nt / T_;
    float s = 0.f;
    for (int k = 0; k < taps; ++k) {
      const int tt = trans ? t + k * S : t - k * S;
      if (tt < 0 || tt >= T_) break;
      s += Tr<T>::to_f(x[((n * T_ + tt) * V + v) * ldx + c]);
    }
    T* p = y + m * ldy + c;
    if (accumulate) s += Tr<T>::to_f(*p);
    *p = Tr<T>::from_f(s);
  }
}

__global__ __launch_bounds__(256) void rt_online_kernel(const float* __restrict__ z, float* fifo, float* acc, int* idx,
                                                        int E, int fifo_size, int S, float* out) {
  const int fi = idx[0], ai = idx[1];
  for (int e = threadIdx.x; e < E; e += 256) {
    const float zv = z[e];
    float a = acc[(long)ai * E + e] + zv - fifo[(long)fi * E + e];
    acc[(long)ai * E + e] = a;
    out[e] = a;
    fifo[(long)fi * E + e] = zv;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    idx[0] = (fi + 1) % fifo_size;
    idx[1] = (ai + 1) % S;
  }
}

}  // namespace

int box_sum_launch(const void* x, int ldx, void* y, int ldy, int N, int T_, int V, int C, int K, int S, int trans,
                   int accumulate, int dtype, hipStream_t s) {
  if (S < 1 || K < 1) return STGCN_EBADSHAPE;
  long total = (long)N * T_ * V * C;
  long g = (total + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  if (dtype)
    hipLaunchKernelGGL(box_sum_kernel<bf16>, dim3((unsigned)g), dim3(256), 0, s, (const bf16*)x, ldx, (bf16*)y, ldy,
                       N, T_, V, C, K, S, trans, accumulate);
  else
    hipLaunchKernelGGL(box_sum_kernel<float>, dim3((unsigned)g), dim3(256), 0, s, (const float*)x, ldx, (float*)y,
                       ldy, N, T_, V, C, K, S, trans, accumulate);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

int rt_online_launch(const float* z, float* fifo, float* acc, int* idx, int C, int V, int fifo_size, int S,
                     float* out, hipStream_t s) {
  hipLaunchKernelGGL(rt_online_kernel, dim3(1), dim3(256), 0, s, z, fifo, acc, idx, C * V, fifo_size, S, out);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
