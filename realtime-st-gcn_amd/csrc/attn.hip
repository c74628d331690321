// AAGCN self-attention adjacency (models/aagcn/aagcn.py:139-145):
//
//   theta, phi = conv1x1(x) -> (N, P*ce, T, V)  (rows, channels-last)
//   S[n,p,v,w] = sum_{t,c<ce} theta[(n,t,v)][p*ce+c] * phi[(n,t,w)][p*ce+c]      (matmul, :145)
//   C[n,p,v,:] = softmax_w(S[n,p,v,:])                                            (softmax dim=3)
// Backward: dS = C * (dC - sum_w dC*C);  dtheta[(n,t,v)][p*ce+c] = sum_w dS[v][w] phi[(n,t,w)][.]
//                                        dphi[(n,t,w)][p*ce+c]   = sum_v dS[v][w] theta[(n,t,v)][.]
// The score GEMM (K = T*ce, up to 4800) runs on MFMA with both operands loaded straight from the rows
// (8 consecutive channels per lane = 16 B); blocks split T and add fp32 partials.
#include "common.h"

void slab_sum_launch(const float* in, long B, long R, long E, float* tmp, float* out, int accumulate, hipStream_t s);
long slab_sum_tmp_floats(long B, long R, long E);

namespace {
constexpr int VMAX = 32;

template <typename T>
__global__ __launch_bounds__(256) void attn_scores_kernel(const T* __restrict__ th, const T* __restrict__ ph,
                                                          int ld, int T_, int V, int P, int ce, int tpb, float* S,
                                                          float* work) {
  constexpr int VEC = 16 / sizeof(T);
  __shared__ float red[4][VMAX * VMAX];
  const int n = blockIdx.z, p = blockIdx.y;
  const int t0 = blockIdx.x * tpb, t1 = min(T_, t0 + tpb);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 31, h = lane >> 5;
  const bool vec = (ce % 8 == 0) && (ld % VEC == 0);
  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  const long K = (long)(t1 - t0) * ce;
  // k = (t - t0)*ce + c ; each wave takes k-steps of 16 round-robin
  for (long k0 = (long)wave * 16; k0 < K; k0 += 64) {
    typename Tr<T>::frag fa, fb;
    float fx[8], fy[8];
    if (vec && r < V) {
      const long k = k0 + 8 * h;
      const int t = t0 + (int)(k / ce), c = (int)(k % ce);
      if (k < K) {
        const long base = ((long)n * T_ + t) * V;
        const T* pa = th + (base + r) * ld + p * ce + c;
        const T* pb = ph + (base + r) * ld + p * ce + c;
#pragma unroll
        for (int u = 0; u < 8; u += VEC) {
          unpack16(*reinterpret_cast<const uint4*>(pa + u), fx + u, (T*)nullptr);
          unpack16(*reinterpret_cast<const uint4*>(pb + u), fy + u, (T*)nullptr);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) fx[j] = fy[j] = 0.f;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const long k = k0 + 8 * h + j;
        fx[j] = fy[j] = 0.f;
        if (r < V && k < K) {
          const int t = t0 + (int)(k / ce), c = (int)(k % ce);
          const long row = ((long)n * T_ + t) * V + r;
          fx[j] = Tr<T>::to_f(th[row * ld + p * ce + c]);
          fy[j] = Tr<T>::to_f(ph[row * ld + p * ce + c]);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      fa[j] = Tr<T>::from_f(fx[j]);
      fb[j] = Tr<T>::from_f(fy[j]);
    }
    Tr<T>::mma(acc, fa, fb);  // rows v (theta), cols w (phi)
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) red[wave][acc_row(i, lane) * VMAX + r] = acc[i];
  __syncthreads();
  // work: partial of T-chunk blockIdx.x in slab row ((n*P + p) * chunks + chunk) (ordered sum afterwards)
  float* dst = work ? work + (((long)n * P + p) * gridDim.x + blockIdx.x) * V * V : S + ((long)n * P + p) * V * V;
  for (int i = threadIdx.x; i < V * V; i += 256) {
    const int v = i / V, w = i % V;
    const float s = red[0][v * VMAX + w] + red[1][v * VMAX + w] + red[2][v * VMAX + w] + red[3][v * VMAX + w];
    if (work) dst[i] = s; else atomicAdd(dst + i, s);
  }
}

// in-place row softmax over w of S (N*P*V rows of V)
__global__ void attn_softmax_kernel(float* S, long rows, int V) {
  const long r = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  float* s = S + r * V;
  float m = -INFINITY;
  for (int w = 0; w < V; ++w) m = fmaxf(m, s[w]);
  float z = 0.f;
  for (int w = 0; w < V; ++w) z += __expf(s[w] - m);
  const float iz = 1.f / z;
  for (int w = 0; w < V; ++w) s[w] = __expf(s[w] - m) * iz;
}

// dS = C * (dC - sum_w dC*C), per row
__global__ void attn_softmax_bwd_kernel(const float* C, const float* dC, float* dS, long rows, int V) {
  const long r = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  const float* c = C + r * V;
  const float* g = dC + r * V;
  float s = 0.f;
  for (int w = 0; w < V; ++w) s += g[w] * c[w];
  for (int w = 0; w < V; ++w) dS[r * V + w] = c[w] * (g[w] - s);
}

// out[(n,t,a)][p*ce+c] = sum_b Mt[n][p][a][b] in[(n,t,b)][p*ce+c], Mt = dS (trans=0) or dS^T (trans=1)
template <typename T>
__global__ __launch_bounds__(256) void attn_mix_kernel(const T* __restrict__ in, int ld, const float* M, int T_,
                                                       int V, int P, int ce, int trans, int fpb,
                                                       T* __restrict__ out) {
  __shared__ float sM[4 * VMAX * VMAX];
  const int n = blockIdx.y;
  for (int i = threadIdx.x; i < P * V * V; i += 256) {
    const int p = i / (V * V), rem = i % (V * V), a = rem / V, b = rem % V;
    const float v = M[((long)n * P + p) * V * V + rem];
    if (trans) sM[(p * V + b) * V + a] = v; else sM[(p * V + a) * V + b] = v;
  }
  __syncthreads();
  const int CH = P * ce;
  const int per_frame = V * CH;
  const int t0 = blockIdx.x * fpb;
  const int nf = min(fpb, T_ - t0);
  for (int it = threadIdx.x; it < nf * per_frame; it += 256) {
    const int f = it / per_frame, rem = it % per_frame;
    const int a = rem / CH, ch = rem % CH;
    const int p = ch / ce;
    const long row0 = ((long)n * T_ + t0 + f) * V;
    const float* m = sM + (p * V + a) * V;
    float s = 0.f;
    for (int b = 0; b < V; ++b) s += m[b] * Tr<T>::to_f(in[(row0 + b) * ld + ch]);
    out[(row0 + a) * ld + ch] = Tr<T>::from_f(s);
  }
}
}  // namespace

namespace {
int attn_chunks(int N, int T_, int P, int* tpb_out) {
  int tpb = (int)(((long)T_ * N * P + 1023) / 1024);  // ~1024 blocks
  if (tpb < 8) tpb = 8;
  if (tpb_out) *tpb_out = tpb;
  return (T_ + tpb - 1) / tpb;
}
}  // namespace

long attn_scores_workspace(int N, int T_, int V, int P) {
  const long chunks = attn_chunks(N, T_, P, nullptr), E = (long)V * V;
  return (long)sizeof(float) * ((long)N * P * chunks * E + slab_sum_tmp_floats((long)N * P, chunks, E));
}

int attn_scores_launch(const void* th, const void* ph, int ld, int N, int T_, int V, int P, int ce, float* S,
                       void* work, int dtype, hipStream_t s) {
  if (V > VMAX || P > 4) return STGCN_EBADSHAPE;
  int tpb;
  const int chunks = attn_chunks(N, T_, P, &tpb);
  float* w = reinterpret_cast<float*>(work);
  if (!w) (void)hipMemsetAsync(S, 0, sizeof(float) * N * P * V * V, s);
  dim3 grid(chunks, P, N);
  if (dtype)
    hipLaunchKernelGGL(attn_scores_kernel<bf16>, grid, dim3(256), 0, s, (const bf16*)th, (const bf16*)ph, ld, T_, V,
                       P, ce, tpb, S, w);
  else
    hipLaunchKernelGGL(attn_scores_kernel<float>, grid, dim3(256), 0, s, (const float*)th, (const float*)ph, ld, T_,
                       V, P, ce, tpb, S, w);
  if (w) slab_sum_launch(w, (long)N * P, chunks, (long)V * V, w + (long)N * P * chunks * V * V, S, 0, s);
  const long rows = (long)N * P * V;
  hipLaunchKernelGGL(attn_softmax_kernel, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, s, S, rows, V);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

int jmix_launch(const void* in, int in_ld, void* out, int out_ld, const float* M, int N, int T, int V, int P, int C,
                int mode, int bt, int per_sample, int accumulate, int dtype, hipStream_t s);

int attn_bwd_launch(const void* th, const void* ph, int ld, int N, int T_, int V, int P, int ce, const float* C,
                    const float* dC, float* dS, void* dth, void* dph, int dtype, hipStream_t s) {
  if (V > VMAX || P > 4) return STGCN_EBADSHAPE;
  const long rows = (long)N * P * V;
  hipLaunchKernelGGL(attn_softmax_bwd_kernel, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, s, C, dC, dS, rows,
                     V);
  // dth = dS-mix of phi, dph = dS^T-mix of theta, per (sample, partition) channel group: MFMA (jmix.hip)
  const int r1 = jmix_launch(ph, ld, dth, ld, dS, N, T_, V, P, ce, 2, 1, 1, 0, dtype, s);
  if (r1 > 0) return r1;
  if (r1 == 0) {
    const int r2 = jmix_launch(th, ld, dph, ld, dS, N, T_, V, P, ce, 2, 0, 1, 0, dtype, s);
    if (r2 >= 0) return r2;
  }
  int fpb = (4096 + V * P * ce - 1) / (V * P * ce);
  if (fpb < 1) fpb = 1;
  dim3 grid((T_ + fpb - 1) / fpb, N);
  if (dtype) {
    hipLaunchKernelGGL(attn_mix_kernel<bf16>, grid, dim3(256), 0, s, (const bf16*)ph, ld, dS, T_, V, P, ce, 0, fpb,
                       (bf16*)dth);
    hipLaunchKernelGGL(attn_mix_kernel<bf16>, grid, dim3(256), 0, s, (const bf16*)th, ld, dS, T_, V, P, ce, 1, fpb,
                       (bf16*)dph);
  } else {
    hipLaunchKernelGGL(attn_mix_kernel<float>, grid, dim3(256), 0, s, (const float*)ph, ld, dS, T_, V, P, ce, 0, fpb,
                       (float*)dth);
    hipLaunchKernelGGL(attn_mix_kernel<float>, grid, dim3(256), 0, s, (const float*)th, ld, dS, T_, V, P, ce, 1, fpb,
                       (float*)dph);
  }
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

// ---------------------------------------------------------------- attention projections (bf16 path)
// out[r][o] = bias[o] + sum_c W[o][c] x[r][c]  for theta and phi stacked (o < Nout): x bf16 rows (exact
// values), W fp32 split as W_hi + W_lo (two bf16 MFMAs, ~2^-17 relative coefficient error) and fp32
// outputs: the attention logits contract theta^T phi over C'*T terms and then a softmax, so theta/phi
// must not be rounded to bf16 (aagcn.py:142-145), but they need no fp32 MFMA either.
// D^T = W x^T on 32x32x16 MFMAs: A = W rows (m = output channel) from LDS (hi/lo staged once per block for
// its group of <= 128 output channels), B = x rows (n = row) straight from global as 16-B fragments held
// in registers for all channel tiles; D lane = row, 4 consecutive channels per float4 store.
namespace {
constexpr int PJ_CG = 128;  // output channels per block group
template <int KSN>
__global__ __launch_bounds__(256) void attn_proj_kernel(const bf16* __restrict__ x, int ldx, long M, int Cin,
                                                        const float* __restrict__ W, const float* __restrict__ bias,
                                                        int Nout, float* __restrict__ out, int ldo, int rt_per_block) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int RS = Cin * 2 + 16;  // padded LDS row bytes
  char* const sHi = smem;
  char* const sLo = smem + PJ_CG * RS;
  const int g = blockIdx.y;
  const int o0 = g * PJ_CG, og = min(PJ_CG, Nout - o0);
  for (int e = threadIdx.x; e < PJ_CG * Cin / 4; e += 256) {  // stage W_hi / W_lo, 4 weights per thread (rows >= og: 0)
    const int o = (4 * e) / Cin, c = 4 * e - o * Cin;
    const float4 w = o < og ? *reinterpret_cast<const float4*>(W + (long)(o0 + o) * Cin + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float wv[4] = {w.x, w.y, w.z, w.w};
    bf16x4 h, l;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      h[j] = (bf16)wv[j];
      l[j] = (bf16)(wv[j] - (float)h[j]);
    }
    *reinterpret_cast<bf16x4*>(sHi + o * RS + c * 2) = h;
    *reinterpret_cast<bf16x4*>(sLo + o * RS + c * 2) = l;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, lr = lane & 31, lh = lane >> 5;
  const int ntile = (og + 31) / 32;
  const long rt_total = (M + 31) / 32;
  const long rt0 = (long)blockIdx.x * rt_per_block, rt1 = min(rt_total, rt0 + rt_per_block);
  for (long rt = rt0 + wave; rt < rt1; rt += 4) {
    const long row = rt * 32 + lr;
    const bool rok = row < M;
    bf16x8 xf[KSN];
#pragma unroll
    for (int ks = 0; ks < KSN; ++ks) {
      const uint4 u = rok ? *reinterpret_cast<const uint4*>(x + row * ldx + 16 * ks + 8 * lh) : make_uint4(0, 0, 0, 0);
      xf[ks] = __builtin_bit_cast(bf16x8, u);
    }
    for (int ct = 0; ct < ntile; ++ct) {
      f32x16 acc = {};
      const char* ah = sHi + (ct * 32 + lr) * RS + lh * 16;
      const char* al = sLo + (ct * 32 + lr) * RS + lh * 16;
#pragma unroll
      for (int ks = 0; ks < KSN; ++ks) {
        const bf16x8 wh = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(ah + ks * 32));
        const bf16x8 wl = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(al + ks * 32));
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wh, xf[ks], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wl, xf[ks], acc, 0, 0, 0);
      }
      if (rok) {
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
          const int o = ct * 32 + 8 * q4 + 4 * lh;  // within the group
          if (o >= og) continue;
          float4 v = make_float4(acc[4 * q4], acc[4 * q4 + 1], acc[4 * q4 + 2], acc[4 * q4 + 3]);
          if (bias) {
            const float4 b = *reinterpret_cast<const float4*>(bias + o0 + o);
            v.x += b.x; v.y += b.y; v.z += b.z; v.w += b.w;
          }
          *reinterpret_cast<float4*>(out + row * ldo + o0 + o) = v;
        }
      }
    }
  }
}
}  // namespace

int attn_proj_launch(const void* x, int ldx, long M, int Cin, const float* W, const float* bias, int Nout, float* out,
                     int ldo, hipStream_t s) {
  if (!x || !W || !out || M < 1 || Nout < 1 || Nout % 4 || ldo < Nout || ldo % 4 || Cin % 16 || Cin < 16 ||
      Cin > 256 || ldx < Cin || ldx % 8 || ((size_t)W & 15))
    return STGCN_EBADSHAPE;
  const int KSN = Cin / 16;
  const long rt_total = (M + 31) / 32;
  const int groups = (Nout + PJ_CG - 1) / PJ_CG;
  const int ncu = stgcn_cu_count(s);
  // one round of resident blocks (each stages its group's W_hi / W_lo, up to 132 KB: more blocks only repeat that)
  const size_t lds0 = (size_t)2 * PJ_CG * (Cin * 2 + 16);
  const long bpc = lds0 > 80 * 1024 ? 1 : (lds0 > 53 * 1024 ? 2 : 4);
  long blocks = (long)(ncu > 0 ? ncu : 256) * bpc / groups;
  if (blocks < 1) blocks = 1;
  long rpb = (rt_total + blocks - 1) / blocks;
  if (rpb < 4) rpb = 4;
  blocks = (rt_total + rpb - 1) / rpb;
  const size_t lds = (size_t)2 * PJ_CG * (Cin * 2 + 16);
  const dim3 grid((unsigned)blocks, (unsigned)groups);
  switch (KSN) {
#define PJ_CASE(K)                                                                                            \
  case K:                                                                                                     \
    if (stgcn_lds_attr((const void*)attn_proj_kernel<K>, (int)lds, s)) return STGCN_EHIP;                      \
    hipLaunchKernelGGL(attn_proj_kernel<K>, grid, dim3(256), lds, s, (const bf16*)x, ldx, M, Cin, W, bias, Nout, \
                       out, ldo, (int)rpb);                                                                   \
    break;
    PJ_CASE(1) PJ_CASE(2) PJ_CASE(3) PJ_CASE(4) PJ_CASE(5) PJ_CASE(6) PJ_CASE(7) PJ_CASE(8)
    PJ_CASE(9) PJ_CASE(10) PJ_CASE(11) PJ_CASE(12) PJ_CASE(13) PJ_CASE(14) PJ_CASE(15) PJ_CASE(16)
#undef PJ_CASE
    default:
      return STGCN_EBADSHAPE;
  }
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
