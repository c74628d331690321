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

// Neighbour lists of A built in LDS by every block (A's zero pattern is exploited exactly: a zero
// coefficient contributes nothing).  The ST-GCN spatial graph has 73 non-zeros of 3*25*25, so the
// mixing is ~1 FMA per output element and both kernels are HBM-bound gathers; a dense A (AAGCN's
// A+B+C) simply yields full lists.
struct MixLists {
  float A[4 * VMAX * VMAX];
  float fco[4 * VMAX * VMAX];     // fwd: per (p,w) coefficients, stride V
  unsigned char fv[4 * VMAX * VMAX];
  int fcnt[4 * VMAX];
  float tco[4 * VMAX * VMAX];     // trans: per v, entries (p,w), stride P*V
  short tpw[4 * VMAX * VMAX];
  int tcnt[VMAX];
};

DEV void build_lists(MixLists& L, const float* A, int P, int V, bool fwd) {
  for (int i = threadIdx.x; i < P * V * V; i += blockDim.x) L.A[i] = A[i];
  __syncthreads();
  if (fwd) {
    for (int pw = threadIdx.x; pw < P * V; pw += blockDim.x) {
      const int p = pw / V, w = pw % V;
      int c = 0;
      for (int v = 0; v < V; ++v) {
        const float a = L.A[(p * V + v) * V + w];
        if (a != 0.f) {
          L.fco[pw * V + c] = a;
          L.fv[pw * V + c] = (unsigned char)v;
          ++c;
        }
      }
      L.fcnt[pw] = c;
    }
  } else {
    for (int v = threadIdx.x; v < V; v += blockDim.x) {
      int c = 0;
      for (int p = 0; p < P; ++p)
        for (int w = 0; w < V; ++w) {
          const float a = L.A[(p * V + v) * V + w];
          if (a != 0.f) {
            L.tco[v * P * V + c] = a;
            L.tpw[v * P * V + c] = (short)(p * V + w);
            ++c;
          }
        }
      L.tcnt[v] = c;
    }
  }
  __syncthreads();
}

template <typename T, int VEC>
DEV void ld_unit(const T* p, float* f) {
  if constexpr (VEC == 1) f[0] = Tr<T>::to_f(*p);
  else unpack16(*reinterpret_cast<const uint4*>(p), f, (T*)nullptr);
}
template <typename T, int VEC>
DEV void st_unit(T* p, const float* f) {
  if constexpr (VEC == 1) *p = Tr<T>::from_f(f[0]);
  else *reinterpret_cast<uint4*>(p) = pack16(f, (T*)nullptr);
}

// XA[(n,t,w)][p*Cin + ci] = sum_{v in nbr(p,w)} A[p][v][w] x[(n,t,v)][ci]; work item = (frame, w, p, unit)
template <typename T, int VEC>
__global__ __launch_bounds__(256) void amix_fwd_kernel(const AmixArgs a, int fpb) {
  __shared__ MixLists L;
  const int n = blockIdx.y;
  build_lists(L, a.A + (a.per_sample ? (long)n * a.P * a.V * a.V : 0), a.P, a.V, true);
  const int CU = a.Cin / VEC;
  const int per_frame = a.V * a.P * CU;
  const int t0 = blockIdx.x * fpb;
  const int nf = min(fpb, a.T - t0);
  const T* __restrict__ x = reinterpret_cast<const T*>(a.x);
  T* __restrict__ out = reinterpret_cast<T*>(a.out);
  const int ldo = a.P * a.Cin;
  for (int it = threadIdx.x; it < nf * per_frame; it += 256) {
    const int f = it / per_frame;
    int r = it - f * per_frame;
    const int w = r / (a.P * CU);
    r -= w * a.P * CU;
    const int p = r / CU, u = r - p * CU;
    const long row0 = ((long)n * a.T + t0 + f) * a.V;
    float acc[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] = 0.f;
    const int pw = p * a.V + w;
    const int cnt = L.fcnt[pw];
    for (int k = 0; k < cnt; ++k) {
      const float c = L.fco[pw * a.V + k];
      float f8[VEC];
      ld_unit<T, VEC>(x + (row0 + L.fv[pw * a.V + k]) * a.x_ld + u * VEC, f8);
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[j] += c * f8[j];
    }
    st_unit<T, VEC>(out + (row0 + w) * ldo + p * a.Cin + u * VEC, acc);
  }
}

// dx[(n,t,v)][ci] (+)= sum_{(p,w) in nbr^T(v)} A[p][v][w] DW[(n,t,w)][p*Cin+ci]; item = (frame, v, unit)
template <typename T, int VEC>
__global__ __launch_bounds__(256) void amix_trans_kernel(const AmixArgs a, int fpb) {
  __shared__ MixLists L;
  const int n = blockIdx.y;
  build_lists(L, a.A + (a.per_sample ? (long)n * a.P * a.V * a.V : 0), a.P, a.V, false);
  const int CU = a.Cin / VEC;
  const int per_frame = a.V * CU;
  const int t0 = blockIdx.x * fpb;
  const int nf = min(fpb, a.T - t0);
  const T* __restrict__ dw = reinterpret_cast<const T*>(a.x);
  T* __restrict__ out = reinterpret_cast<T*>(a.out);
  const int ldi = a.P * a.Cin;
  for (int it = threadIdx.x; it < nf * per_frame; it += 256) {
    const int f = it / per_frame;
    int r = it - f * per_frame;
    const int v = r / CU, u = r - v * CU;
    const long row0 = ((long)n * a.T + t0 + f) * a.V;
    float acc[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] = 0.f;
    const int cnt = L.tcnt[v];
    const int PV = a.P * a.V;
    for (int k = 0; k < cnt; ++k) {
      const float c = L.tco[v * PV + k];
      const int pw = L.tpw[v * PV + k];
      const int p = pw / a.V, w = pw - p * a.V;
      float f8[VEC];
      ld_unit<T, VEC>(dw + (row0 + w) * ldi + p * a.Cin + u * VEC, f8);
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[j] += c * f8[j];
    }
    T* po = out + (row0 + v) * a.out_ld + u * VEC;
    if (a.accumulate) {
      float prev[VEC];
      ld_unit<T, VEC>(po, prev);
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[j] += prev[j];
    }
    st_unit<T, VEC>(po, acc);
  }
}

// dA via MFMA: per frame, C_p[v][w] += sum_ci X[v][ci] * DW[w][p][ci]  (A-operand rows v, B-operand
// cols w, both 8-consecutive-ci per lane => plain 16B loads).  One wave per frame stream; waves of
// a block reduce through LDS, then one atomicAdd per element per block.
template <typename T>
__global__ __launch_bounds__(256) void amix_dA_kernel(const AmixArgs a, const void* dwp, float* dA, float* work,
                                                      int frames_per_block) {
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
    // work: this block's partial in slab row (n * gridDim.x + blockIdx.x) of width P*V*V (fixed-order
    // reduction afterwards -> deterministic); no work: atomics
    float* dst = work ? work + ((long)n * gridDim.x + blockIdx.x) * a.P * a.V * a.V + (long)p * a.V * a.V
                      : dA + ((a.per_sample ? (long)n * a.P : 0) + p) * a.V * a.V;
    for (int i = threadIdx.x; i < a.V * a.V; i += 256) {
      const int v = i / a.V, w = i % a.V;
      const float s = red[0][v * VMAX + w] + red[1][v * VMAX + w] + red[2][v * VMAX + w] + red[3][v * VMAX + w];
      if (work) dst[i] = s; else atomicAdd(dst + i, s);
    }
    __syncthreads();
  }
}

// The same products with 16-B rows (Cin % 8 == 0): x's fragment is loaded once for all P partitions
// (P accumulators), and KC k-steps' fragments of x and of the P DW blocks are issued before their MFMAs — the
// generic kernel above re-read x per partition and waited for every 16-channel step's two loads.
template <typename T>
__global__ __launch_bounds__(256) void amix_dA_vec_kernel(const AmixArgs a, const void* dwp, float* dA, float* work,
                                                          int frames_per_block) {
  constexpr int VEC = 16 / sizeof(T);
  constexpr int NU = 8 / VEC;                 // 16-B units per 8-channel fragment
  constexpr int KC = sizeof(T) == 2 ? 4 : 2;  // k-steps per load batch
  constexpr int PM = 4;
  __shared__ float red[4][VMAX * VMAX];
  const int n = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const T* __restrict__ x = reinterpret_cast<const T*>(a.x);
  const T* __restrict__ dw = reinterpret_cast<const T*>(dwp);
  const int ld_dw = a.P * a.Cin;
  const int t0 = blockIdx.x * frames_per_block;
  const int t1 = min(a.T, t0 + frames_per_block);
  const bool rok = r < a.V;
  f32x16 acc[PM];
#pragma unroll
  for (int p = 0; p < PM; ++p)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[p][i] = 0.f;
  for (int t = t0 + wave; t < t1; t += 4) {
    const long row = ((long)n * a.T + t) * a.V + (rok ? r : 0);
    const T* px = x + row * a.x_ld + 8 * h;
    const T* pd = dw + row * ld_dw + 8 * h;
    for (int k0 = 0; k0 < a.Cin; k0 += 16 * KC) {
      uint4 ux[KC][NU], ud[KC][PM][NU];
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        const int ci = k0 + 16 * kc;
        const bool ok = rok && ci + 8 * h < a.Cin;  // this lane's 8 channels (Cin % 8 == 0: all or none)
#pragma unroll
        for (int u = 0; u < NU; ++u) {
          ux[kc][u] = ok ? *reinterpret_cast<const uint4*>(px + ci + u * VEC) : make_uint4(0, 0, 0, 0);
#pragma unroll
          for (int p = 0; p < PM; ++p)
            ud[kc][p][u] = ok && p < a.P ? *reinterpret_cast<const uint4*>(pd + p * a.Cin + ci + u * VEC)
                                         : make_uint4(0, 0, 0, 0);
        }
      }
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        if (k0 + 16 * kc >= a.Cin) break;  // wave-uniform
        float fx[8];
        typename Tr<T>::frag fa;
#pragma unroll
        for (int u = 0; u < NU; ++u) unpack16(ux[kc][u], fx + u * VEC, (T*)nullptr);
#pragma unroll
        for (int j = 0; j < 8; ++j) fa[j] = Tr<T>::from_f(fx[j]);
#pragma unroll
        for (int p = 0; p < PM; ++p) {
          if (p >= a.P) break;
          float fd[8];
          typename Tr<T>::frag fb;
#pragma unroll
          for (int u = 0; u < NU; ++u) unpack16(ud[kc][p][u], fd + u * VEC, (T*)nullptr);
#pragma unroll
          for (int j = 0; j < 8; ++j) fb[j] = Tr<T>::from_f(fd[j]);
          Tr<T>::mma(acc[p], fa, fb);
        }
      }
    }
  }
#pragma unroll
  for (int p = 0; p < PM; ++p) {
    if (p >= a.P) break;
#pragma unroll
    for (int i = 0; i < 16; ++i) red[wave][acc_row(i, lane) * VMAX + r] = acc[p][i];
    __syncthreads();
    float* dst = work ? work + ((long)n * gridDim.x + blockIdx.x) * a.P * a.V * a.V + (long)p * a.V * a.V
                      : dA + ((a.per_sample ? (long)n * a.P : 0) + p) * a.V * a.V;
    for (int i = threadIdx.x; i < a.V * a.V; i += 256) {
      const int v = i / a.V, w = i % a.V;
      const float s = red[0][v * VMAX + w] + red[1][v * VMAX + w] + red[2][v * VMAX + w] + red[3][v * VMAX + w];
      if (work) dst[i] = s; else atomicAdd(dst + i, s);
    }
    __syncthreads();
  }
}

// out[b][r2][e] (+)= sum_{r in group r2} in[b][r][e], rows summed in a fixed order (deterministic).
// Block: 64 columns x 4 row-interleaved waves, LDS combine in wave order.
__global__ __launch_bounds__(256) void slab_sum_kernel(const float* __restrict__ in, long R, long E, int rpb,
                                                       float* out, int accumulate) {
  const int g = threadIdx.x >> 6;
  const long e = (long)blockIdx.x * 64 + (threadIdx.x & 63);
  const long b = blockIdx.z;
  const long r0 = (long)blockIdx.y * rpb, r1 = min(R, r0 + rpb);
  const float* src = in + b * R * E + e;
  float acc = 0.f;
  if (e < E)
    for (long r = r0 + g; r < r1; r += 4) acc += src[r * E];
  __shared__ float part[4][64];
  part[g][threadIdx.x & 63] = acc;
  __syncthreads();
  if (g == 0 && e < E) {
    const int l = threadIdx.x;
    const float t = ((part[0][l] + part[1][l]) + part[2][l]) + part[3][l];
    float* o = out + (b * gridDim.y + blockIdx.y) * E + e;
    *o = accumulate ? *o + t : t;
  }
}

__global__ __launch_bounds__(256) void gcn_bias_kernel(const float* A, const float* b, float* out, int P, int V, int C,
                                                       int per_sample) {
  // out[(n), w, c] = sum_p b[p*C + c] * colsum_p[w],  colsum_p[w] = sum_v A[(n), p, v, w] (staged in LDS)
  // A is staged in LDS by coalesced loads first: a per-thread loop of V dependent global loads was the
  // whole cost of this kernel
  __shared__ float cs[4 * VMAX];
  __shared__ float sA[4 * VMAX * VMAX];
  const int n = blockIdx.y;
  const float* An = A + (per_sample ? (long)n * P * V * V : 0);
  for (int i = threadIdx.x; i < P * V * V; i += blockDim.x) sA[i] = An[i];
  __syncthreads();
  for (int i = threadIdx.x; i < P * V; i += blockDim.x) {
    const int p = i / V, w = i % V;
    float t = 0.f;
    for (int v = 0; v < V; ++v) t += sA[(p * V + v) * V + w];
    cs[i] = t;
  }
  __syncthreads();
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < V * C; i += gridDim.x * blockDim.x) {
    const int w = i / C, c = i % C;
    float s = 0.f;
    for (int p = 0; p < P; ++p) s += b[p * C + c] * cs[p * V + w];
    out[(long)n * V * C + i] = s;
  }
}

// Gradients of the conv bias pushed through a shared A, from S[w][c] = sum over rows of joint w of dg:
//   dA[p][v][w] += sum_c b[p][c] S[w][c]   (independent of v)
//   db[p][c]     = sum_w colsum_p[w] S[w][c]
// Block x < P*V: one (p, w) dot over c, broadcast along v; blocks >= P*V: db columns.
__global__ __launch_bounds__(256) void gcn_bias_bwd_kernel(const float* A, const float* b, const float* S, int P, int V,
                                                           int C, float* dA, float* db) {
  const int bx = blockIdx.x;
  if (bx < P * V) {
    const int p = bx / V, w = bx % V;
    float t = 0.f;
    for (int c = threadIdx.x; c < C; c += 256) t += b[p * C + c] * S[w * C + c];
    t = wave_sum(t);
    __shared__ float red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = t;
    __syncthreads();
    const float tot = ((red[0] + red[1]) + red[2]) + red[3];
    for (int v = threadIdx.x; v < V; v += 256) dA[(p * V + v) * V + w] += tot;
    return;
  }
  __shared__ float cs[4 * VMAX];
  __shared__ float sA[4 * VMAX * VMAX];
  for (int i = threadIdx.x; i < P * V * V; i += 256) sA[i] = A[i];
  __syncthreads();
  for (int i = threadIdx.x; i < P * V; i += 256) {
    const int p = i / V, w = i % V;
    float t = 0.f;
    for (int v = 0; v < V; ++v) t += sA[(p * V + v) * V + w];
    cs[i] = t;
  }
  __syncthreads();
  const int i = (bx - P * V) * 256 + threadIdx.x;  // (p, c)
  if (i >= P * C) return;
  const int p = i / C, c = i % C;
  float t = 0.f;
  for (int w = 0; w < V; ++w) t += cs[p * V + w] * S[w * C + c];
  db[i] = t;
}

// frames per block so that a block has ~16 work items per thread
int frames_per_block(int items_per_frame) {
  int f = (4096 + items_per_frame - 1) / items_per_frame;
  return f < 1 ? 1 : f;
}
}  // namespace

#define AMIX_DISPATCH(KERNEL, a, per_frame_units, dtype, s)                                          \
  do {                                                                                              \
    const bool v8 = (a.Cin % 8 == 0) && (a.x_ld % 8 == 0) && (a.out_ld % 8 == 0);                   \
    const bool v4 = (a.Cin % 4 == 0) && (a.x_ld % 4 == 0) && (a.out_ld % 4 == 0);                   \
    const int vec = dtype ? (v8 ? 8 : 1) : (v4 ? 4 : 1);                                           \
    const int fpb = frames_per_block((per_frame_units) * (a.Cin / vec));                           \
    dim3 grid((a.T + fpb - 1) / fpb, a.N);                                                          \
    if (dtype) {                                                                                    \
      if (vec == 8) hipLaunchKernelGGL((KERNEL<bf16, 8>), grid, dim3(256), 0, s, a, fpb);           \
      else hipLaunchKernelGGL((KERNEL<bf16, 1>), grid, dim3(256), 0, s, a, fpb);                    \
    } else {                                                                                        \
      if (vec == 4) hipLaunchKernelGGL((KERNEL<float, 4>), grid, dim3(256), 0, s, a, fpb);          \
      else hipLaunchKernelGGL((KERNEL<float, 1>), grid, dim3(256), 0, s, a, fpb);                   \
    }                                                                                               \
  } while (0)

int jmix_launch(const void* in, int in_ld, void* out, int out_ld, const float* M, int N, int T, int V, int P, int C,
                int mode, int bt, int per_sample, int accumulate, int dtype, hipStream_t s);

int amix_fwd_launch(const AmixArgs& a0, int dtype, hipStream_t s) {
  if (a0.V > VMAX || a0.P > 4) return STGCN_EBADSHAPE;
  AmixArgs a = a0;
  a.out_ld = a.P * a.Cin;
  // dense joint mixing on MFMA (jmix.hip) where the shape allows; the gather kernel otherwise
  const int r = jmix_launch(a.x, a.x_ld, a.out, a.out_ld, a.A, a.N, a.T, a.V, a.P, a.Cin, 0, 0, a.per_sample, 0,
                            dtype, s);
  if (r >= 0) return r;
  AMIX_DISPATCH(amix_fwd_kernel, a, a.V * a.P, dtype, s);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

int amix_trans_launch(const AmixArgs& a0, int dtype, hipStream_t s) {
  if (a0.V > VMAX || a0.P > 4) return STGCN_EBADSHAPE;
  AmixArgs a = a0;
  a.x_ld = a.P * a.Cin;  // DW rows
  const int r = jmix_launch(a.x, a.x_ld, a.out, a.out_ld, a.A, a.N, a.T, a.V, a.P, a.Cin, 1, 0, a.per_sample,
                            a.accumulate, dtype, s);
  if (r >= 0) return r;
  AMIX_DISPATCH(amix_trans_kernel, a, a.V, dtype, s);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

namespace {
constexpr int SLAB_RPB = 32;  // rows per block of a slab_sum level
int amix_dA_chunks(const AmixArgs& a, int* fpb_out) {
  // ~1024 blocks overall
  int fpb = (int)(((long)a.N * a.T + 1023) / 1024);
  if (fpb < 8) fpb = 8;
  if (fpb_out) *fpb_out = fpb;
  return (a.T + fpb - 1) / fpb;
}
}  // namespace

// Deterministic fixed-order sum of a slab in[B][R][E] into out[B][E] (+=: accumulate); two levels when R
// is large.  tmp: ceil(R / SLAB_RPB) * B * E floats (only when R > SLAB_RPB).
void slab_sum_launch(const float* in, long B, long R, long E, float* tmp, float* out, int accumulate, hipStream_t s) {
  const unsigned cb = (unsigned)((E + 63) / 64);
  if (R > SLAB_RPB) {
    const long R2 = (R + SLAB_RPB - 1) / SLAB_RPB;
    hipLaunchKernelGGL(slab_sum_kernel, dim3(cb, (unsigned)R2, (unsigned)B), dim3(256), 0, s, in, R, E, SLAB_RPB, tmp, 0);
    in = tmp;
    R = R2;
  }
  hipLaunchKernelGGL(slab_sum_kernel, dim3(cb, 1, (unsigned)B), dim3(256), 0, s, in, R, E, (int)R, out, accumulate);
}

long slab_sum_tmp_floats(long B, long R, long E) { return R > SLAB_RPB ? ((R + SLAB_RPB - 1) / SLAB_RPB) * B * E : 0; }

long amix_dA_workspace(const AmixArgs& a) {
  if (a.V > VMAX || a.P > 4) return 0;
  const long rows = (long)a.N * amix_dA_chunks(a, nullptr);
  const long E = (long)a.P * a.V * a.V;
  const long B = a.per_sample ? a.N : 1, R = a.per_sample ? rows / a.N : rows;
  return (long)sizeof(float) * (rows * E + slab_sum_tmp_floats(B, R, E));
}

int amix_dA_launch(const AmixArgs& a, const void* dw, float* dA, void* work, int dtype, hipStream_t s) {
  if (a.V > VMAX || a.P > 4) return STGCN_EBADSHAPE;
  int fpb;
  const int chunks = amix_dA_chunks(a, &fpb);
  dim3 grid(chunks, a.N);
  float* w = reinterpret_cast<float*>(work);
  const bool vec = a.Cin % 8 == 0 && a.x_ld % 8 == 0 && (a.P * a.Cin) % 8 == 0 && ((size_t)a.x & 15) == 0 &&
                   ((size_t)dw & 15) == 0;
  if (dtype) {
    if (vec) hipLaunchKernelGGL(amix_dA_vec_kernel<bf16>, grid, dim3(256), 0, s, a, dw, dA, w, fpb);
    else hipLaunchKernelGGL(amix_dA_kernel<bf16>, grid, dim3(256), 0, s, a, dw, dA, w, fpb);
  } else {
    if (vec) hipLaunchKernelGGL(amix_dA_vec_kernel<float>, grid, dim3(256), 0, s, a, dw, dA, w, fpb);
    else hipLaunchKernelGGL(amix_dA_kernel<float>, grid, dim3(256), 0, s, a, dw, dA, w, fpb);
  }
  if (w) {
    const long E = (long)a.P * a.V * a.V;
    const long B = a.per_sample ? a.N : 1, R = a.per_sample ? chunks : (long)a.N * chunks;
    slab_sum_launch(w, B, R, E, w + (long)a.N * chunks * E, dA, 1, s);
  }
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

int gcn_bias_bwd_launch(const float* A, const float* b, const float* S, int P, int V, int C, float* dA, float* db,
                        hipStream_t s) {
  if (V > VMAX || P > 4) return STGCN_EBADSHAPE;
  hipLaunchKernelGGL(gcn_bias_bwd_kernel, dim3((unsigned)(P * V + (P * C + 255) / 256)), dim3(256), 0, s, A, b, S, P,
                     V, C, dA, db);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

int gcn_bias_launch(const float* A, const float* b, float* out, int N, int P, int V, int C, int per_sample,
                    hipStream_t s) {
  if (V > VMAX || P > 4) return STGCN_EBADSHAPE;
  dim3 grid((V * C + 255) / 256, per_sample ? N : 1);
  hipLaunchKernelGGL(gcn_bias_kernel, grid, dim3(256), 0, s, A, b, out, P, V, C, per_sample);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
