// Spatial (joint-axis) mixing of the graph convolution, ConvTemporalGraphical (tgcn.py:58-79).
//
// The reference computes conv1x1(x) -> view(N,P,C*T,V) @ A -> sum_P.  We evaluate the same
// contraction with A applied FIRST (exact, incl. the bias, which becomes a (V x C) bias matrix
// bias2d[w][c] = sum_p b[p*C+c] * colsum_p[w]):
//
//   amix_fwd  : XA[(n,t,w)][p*Cin+ci] = sum_v A[(n),p][v][w] * x[(n,t,v)][ci]
//   amix_trans: dx[(n,t,v)][ci]      (+)= sum_p sum_w A[(n),p][v][w] * DW[(n,t,w)][p*Cin+ci]
//   amix_dA   : dA[(n),p][v][w]       += sum_t sum_ci x[(n,t,v)][ci] * DW[(n,t,w)][p*Cin+ci]
//   gcn_bias  : bias2d[(n),w][c]        = sum_p b[p*C+c] * sum_v A[(n),p][v][w]
//
// A is shared (P,V,V) or per sample (N,P,V,V) (AAGCN, aagcn.py:148).  The channel GEMM on XA
// (K = P*Cin) runs on the MFMA row-conv kernel (conv_rows.hip).  amix_dA is a batched GEMM with
// K = (t, ci) and both operands contiguous along ci, so it runs on MFMA straight from HBM.
#include "common.h"

#include "../../include/stgcn_amd.h"
typedef stgcn_amix_desc AmixArgs;

namespace {
constexpr int VMAX = 32;

template <typename T>
__global__ __launch_bounds__(256) void amix_fwd_kernel(const AmixArgs a, int tpf, int fpb) {
  __shared__ float sA[4 * VMAX * VMAX];
  const int n = blockIdx.y;
  const float* A = a.A + (a.per_sample ? (long)n * a.P * a.V * a.V : 0);
  for (int i = threadIdx.x; i < a.P * a.V * a.V; i += 256) sA[i] = A[i];
  __syncthreads();
  const int f = threadIdx.x / tpf, ct = threadIdx.x % tpf;
  const int t = blockIdx.x * fpb + f;
  if (f >= fpb || t >= a.T) return;
  const T* __restrict__ x = reinterpret_cast<const T*>(a.x);
  T* __restrict__ out = reinterpret_cast<T*>(a.out);
  const long row0 = ((long)n * a.T + t) * a.V;
  const int ld_out = a.P * a.Cin;
  for (int ci = ct; ci < a.Cin; ci += tpf) {
    float xv[VMAX];
#pragma unroll
    for (int v = 0; v < VMAX; ++v) xv[v] = v < a.V ? Tr<T>::to_f(x[(row0 + v) * a.x_ld + ci]) : 0.f;
    for (int p = 0; p < a.P; ++p) {
      const float* Ap = sA + p * a.V * a.V;
      for (int w = 0; w < a.V; ++w) {
        float s = 0.f;
#pragma unroll
        for (int v = 0; v < VMAX; ++v)
          if (v < a.V) s += Ap[v * a.V + w] * xv[v];
        out[(row0 + w) * ld_out + p * a.Cin + ci] = Tr<T>::from_f(s);
      }
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void amix_trans_kernel(const AmixArgs a, int tpf, int fpb) {
  __shared__ float sA[4 * VMAX * VMAX];
  const int n = blockIdx.y;
  const float* A = a.A + (a.per_sample ? (long)n * a.P * a.V * a.V : 0);
  for (int i = threadIdx.x; i < a.P * a.V * a.V; i += 256) sA[i] = A[i];
  __syncthreads();
  const int f = threadIdx.x / tpf, ct = threadIdx.x % tpf;
  const int t = blockIdx.x * fpb + f;
  if (f >= fpb || t >= a.T) return;
  const T* __restrict__ dw = reinterpret_cast<const T*>(a.x);
  T* __restrict__ out = reinterpret_cast<T*>(a.out);
  const long row0 = ((long)n * a.T + t) * a.V;
  const int ld_in = a.P * a.Cin;
  for (int ci = ct; ci < a.Cin; ci += tpf) {
    float acc[VMAX];
#pragma unroll
    for (int v = 0; v < VMAX; ++v) acc[v] = 0.f;
    for (int p = 0; p < a.P; ++p) {
      const float* Ap = sA + p * a.V * a.V;
      for (int w = 0; w < a.V; ++w) {
        const float d = Tr<T>::to_f(dw[(row0 + w) * ld_in + p * a.Cin + ci]);
#pragma unroll
        for (int v = 0; v < VMAX; ++v)
          if (v < a.V) acc[v] += Ap[v * a.V + w] * d;
      }
    }
#pragma unroll
    for (int v = 0; v < VMAX; ++v) {
      if (v < a.V) {
        T* p = out + (row0 + v) * a.out_ld + ci;
        float r = acc[v];
        if (a.accumulate) r += Tr<T>::to_f(*p);
        *p = Tr<T>::from_f(r);
      }
    }
  }
}

// dA via MFMA: per frame, C_p[v][w] += sum_ci X[v][ci] * DW[w][p][ci]  (A-operand rows v, B-operand
// cols w, both 8-consecutive-ci per lane => plain 16B loads).  One wave per frame stream; waves of
// a block reduce through LDS, then one atomicAdd per element per block.
template <typename T>
__global__ __launch_bounds__(256) void amix_dA_kernel(const AmixArgs a, const void* dwp, float* dA, int frames_per_block) {
  constexpr int VEC = 16 / sizeof(T);
  __shared__ float red[4][VMAX * VMAX];
  const int n = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const T* __restrict__ x = reinterpret_cast<const T*>(a.x);
  const T* __restrict__ dw = reinterpret_cast<const T*>(dwp);
  const int ld_dw = a.P * a.Cin;
  const bool vec_ok = a.Cin % 8 == 0 && a.x_ld % 8 == 0;
  const int t0 = blockIdx.x * frames_per_block;
  const int t1 = min(a.T, t0 + frames_per_block);
  for (int p = 0; p < a.P; ++p) {
    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    for (int t = t0 + wave; t < t1; t += 4) {
      const long row0 = ((long)n * a.T + t) * a.V;
      for (int k0 = 0; k0 < a.Cin; k0 += 16) {
        typename Tr<T>::frag fa, fb;
        const int ci = k0 + 8 * h;
        float fx[8], fd[8];
        if (r < a.V && ci < a.Cin) {
          const T* px = x + (row0 + r) * a.x_ld + ci;
          const T* pd = dw + (row0 + r) * ld_dw + p * a.Cin + ci;
          if (vec_ok) {
#pragma unroll
            for (int u = 0; u < 8; u += VEC) {
              unpack16(*reinterpret_cast<const uint4*>(px + u), fx + u, (T*)nullptr);
              unpack16(*reinterpret_cast<const uint4*>(pd + u), fd + u, (T*)nullptr);
            }
          } else {  // ragged channel count: element loads
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const bool in = ci + j < a.Cin;
              fx[j] = in ? Tr<T>::to_f(px[j]) : 0.f;
              fd[j] = in ? Tr<T>::to_f(pd[j]) : 0.f;
            }
          }
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) fx[j] = fd[j] = 0.f;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          fa[j] = Tr<T>::from_f(fx[j]);
          fb[j] = Tr<T>::from_f(fd[j]);
        }
        Tr<T>::mma(acc, fa, fb);
      }
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) red[wave][acc_row(i, lane) * VMAX + r] = acc[i];
    __syncthreads();
    float* dst = dA + ((a.per_sample ? (long)n * a.P : 0) + p) * a.V * a.V;
    for (int i = threadIdx.x; i < a.V * a.V; i += 256) {
      const int v = i / a.V, w = i % a.V;
      const float s = red[0][v * VMAX + w] + red[1][v * VMAX + w] + red[2][v * VMAX + w] + red[3][v * VMAX + w];
      atomicAdd(dst + i, s);
    }
    __syncthreads();
  }
}

__global__ void gcn_bias_kernel(const float* A, const float* b, float* out, int P, int V, int C, int per_sample) {
  // out[(n), w, c] = sum_p b[p*C + c] * sum_v A[(n), p, v, w]
  const int n = blockIdx.y;
  const float* An = A + (per_sample ? (long)n * P * V * V : 0);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < V * C; i += gridDim.x * blockDim.x) {
    const int w = i / C, c = i % C;
    float s = 0.f;
    for (int p = 0; p < P; ++p) {
      float cs = 0.f;
      for (int v = 0; v < V; ++v) cs += An[(p * V + v) * V + w];
      s += b[p * C + c] * cs;
    }
    out[(long)n * V * C + i] = s;
  }
}

void tpf_fpb(int cin, int& tpf, int& fpb) {
  tpf = cin < 256 ? cin : 256;
  fpb = 256 / tpf;
}
}  // namespace

int amix_fwd_launch(const AmixArgs& a, int dtype, hipStream_t s) {
  if (a.V > VMAX || a.P > 4) return STGCN_EBADSHAPE;
  int tpf, fpb;
  tpf_fpb(a.Cin, tpf, fpb);
  dim3 grid((a.T + fpb - 1) / fpb, a.N);
  if (dtype)
    hipLaunchKernelGGL(amix_fwd_kernel<bf16>, grid, dim3(256), 0, s, a, tpf, fpb);
  else
    hipLaunchKernelGGL(amix_fwd_kernel<float>, grid, dim3(256), 0, s, a, tpf, fpb);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

int amix_trans_launch(const AmixArgs& a, int dtype, hipStream_t s) {
  if (a.V > VMAX || a.P > 4) return STGCN_EBADSHAPE;
  int tpf, fpb;
  tpf_fpb(a.Cin, tpf, fpb);
  dim3 grid((a.T + fpb - 1) / fpb, a.N);
  if (dtype)
    hipLaunchKernelGGL(amix_trans_kernel<bf16>, grid, dim3(256), 0, s, a, tpf, fpb);
  else
    hipLaunchKernelGGL(amix_trans_kernel<float>, grid, dim3(256), 0, s, a, tpf, fpb);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

int amix_dA_launch(const AmixArgs& a, const void* dw, float* dA, int dtype, hipStream_t s) {
  if (a.V > VMAX || a.P > 4) return STGCN_EBADSHAPE;
  // ~1024 blocks overall
  int fpb = (int)(((long)a.N * a.T + 1023) / 1024);
  if (fpb < 8) fpb = 8;
  dim3 grid((a.T + fpb - 1) / fpb, a.N);
  if (dtype)
    hipLaunchKernelGGL(amix_dA_kernel<bf16>, grid, dim3(256), 0, s, a, dw, dA, fpb);
  else
    hipLaunchKernelGGL(amix_dA_kernel<float>, grid, dim3(256), 0, s, a, dw, dA, fpb);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

int gcn_bias_launch(const float* A, const float* b, float* out, int N, int P, int V, int C, int per_sample,
                    hipStream_t s) {
  dim3 grid((V * C + 255) / 256, per_sample ? N : 1);
  hipLaunchKernelGGL(gcn_bias_kernel, grid, dim3(256), 0, s, A, b, out, P, V, C, per_sample);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
