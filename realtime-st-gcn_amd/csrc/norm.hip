// Normalisation, activation and reduction kernels of the ST-GCN layer (channels-last rows).
//
//  BatchNorm2d(C, track_running_stats=False)  (stgcn.py:152,160,171): batch statistics over
//    all N*T*V rows even in eval(), biased variance, eps 1e-5.  Forward statistics come as
//    (count, mean, M2) partials from the producing GEMM's epilogue (conv_rows.hip) or from
//    bn_stats_partial; bn_finalize merges them (Chan, fp64) and emits mean/rstd and the folded
//    affine (scale, shift) that the consumer's prologue applies.
//  BatchNorm1d(V*C) input norm (batchnorm.py:13-23): the same kernels viewing the NTVC input as
//    [N*T rows][V*C channels].
//  Custom LayerNorm([C,1,V]) (layernorm.py:22-28): per-frame statistics over the V*C contiguous
//    elements of an (n,t) frame, UNBIASED variance, per-(c,v) affine.
//  Backward: dz = dy * relu-mask; BN: dx = g*rstd*(dz - E[dz] - xhat*E[dz*xhat]);
//    LN: dx = rstd*(gz - mean(gz) - xhat*sum(gz*xhat)/(F-1)), gz = dz*gamma.
#include "common.h"
#include <type_traits>

namespace {

template <typename T, int VEC>
DEV void ldv(const T* p, float* f) {
  if constexpr (VEC == 1) {
    f[0] = Tr<T>::to_f(*p);
  } else {
    unpack16(*reinterpret_cast<const uint4*>(p), f, (T*)nullptr);
  }
}
template <typename T, int VEC>
DEV void stv(T* p, const float* f) {
  if constexpr (VEC == 1) {
    *p = Tr<T>::from_f(f[0]);
  } else {
    *reinterpret_cast<uint4*>(p) = pack16(f, (T*)nullptr);
  }
}

// rows per block for the channel-wise row kernels
DEV void row_layout(int C, int VEC, int& cu_n, int& rpi) {
  cu_n = C / VEC;
  rpi = 256 / cu_n;
  if (rpi < 1) rpi = 1;
}

// ------------------------------------------------------------------ BN forward statistics
template <typename T, int VEC>
__global__ __launch_bounds__(256) void bn_stats_partial_kernel(const T* __restrict__ x, int ld, long M, int C,
                                                                long rpb, float4* part) {
  __shared__ float4 red[256 * 8];
  int CU, RPI;
  row_layout(C, VEC, CU, RPI);
  const int tid = threadIdx.x;
  const int cu = tid % CU, rs = tid / CU;
  const long mb = blockIdx.x * rpb, me = min(M, mb + rpb);
  float k[VEC], s1[VEC], s2[VEC];
  float n = 0.f;
#pragma unroll
  for (int j = 0; j < VEC; ++j) k[j] = s1[j] = s2[j] = 0.f;
  if (rs < RPI && cu < CU) {
    for (long m = mb + rs; m < me; m += RPI) {
      float f[VEC];
      ldv<T, VEC>(x + m * ld + cu * VEC, f);
      if (n == 0.f) {
#pragma unroll
        for (int j = 0; j < VEC; ++j) k[j] = f[j];
      }
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        const float d = f[j] - k[j];
        s1[j] += d;
        s2[j] += d * d;
      }
      n += 1.f;
    }
  }
  // per-thread (n, mean, M2)
  if (rs < RPI && cu < CU) {
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const float mean = n > 0.f ? k[j] + s1[j] / n : 0.f;
      const float m2 = n > 0.f ? fmaxf(s2[j] - s1[j] * s1[j] / n, 0.f) : 0.f;
      red[rs * C + cu * VEC + j] = make_float4(n, mean, m2, 0.f);
    }
  }
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    Welford w = {0.f, 0.f, 0.f};
    for (int r = 0; r < RPI; ++r) {
      const float4 g = red[r * C + c];
      w = welford_merge(w, Welford{g.x, g.y, g.z});
    }
    part[(long)blockIdx.x * C + c] = make_float4(w.n, w.mean, w.m2, 0.f);
  }
}

// one block per channel: merge nb (count, mean, M2) partials in fp64
__global__ __launch_bounds__(1024) void bn_finalize_kernel(const float4* part, int nb, int ldp, int C,
                                                          const float* gamma, const float* beta, float eps,
                                                          float2* mean_rstd, float* scale, float* shift,
                                                          float4* merged) {
  // fp64 power sums (n, sum n*mean, sum M2 + n*mean^2) instead of pairwise Chan merges: adds only (no
  // division chain), a wave reduction and one LDS step; at fp64 the final var = S2/n - mean^2 loses
  // ~1e-16 * mean^2/var, far below the fp32 result
  __shared__ double sred[3][16];
  const int nt = blockDim.x;  // 256, or 1024 for long partial lists (the C = 64 layers' conv-epilogue partials)
  const int c = xcd_channel(blockIdx.x, C);
  double n = 0, s1 = 0, s2 = 0;
  for (int b0 = 0; b0 < nb; b0 += nt * 8) {
    float4 gv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int b = b0 + threadIdx.x + nt * u;
      gv[u] = b < nb ? part[(long)b * ldp + c] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const double cnt = gv[u].x, mu = gv[u].y;
      n += cnt;
      s1 += cnt * mu;
      s2 += (double)gv[u].z + cnt * mu * mu;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    n += __shfl_xor(n, o);
    s1 += __shfl_xor(s1, o);
    s2 += __shfl_xor(s2, o);
  }
  if ((threadIdx.x & 63) == 0) {
    sred[0][threadIdx.x >> 6] = n;
    sred[1][threadIdx.x >> 6] = s1;
    sred[2][threadIdx.x >> 6] = s2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double tn = 0, t1 = 0, t2 = 0;
    for (int w = 0; w < nt / 64; ++w) {
      tn += sred[0][w];
      t1 += sred[1][w];
      t2 += sred[2][w];
    }
    const double m = tn > 0 ? t1 / tn : 0.0;
    double var = tn > 0 ? t2 / tn - m * m : 0.0;  // biased (BatchNorm)
    if (var < 0) var = 0;
    if (merged) {  // merge-only mode (SyncBN): this rank's channel statistics as ONE (count, mean, M2) partial
      merged[c] = make_float4((float)tn, (float)m, (float)(var * tn), 0.f);
      return;
    }
    const float rstd = (float)(1.0 / sqrt(var + (double)eps));
    const float mu = (float)m;
    mean_rstd[c] = make_float2(mu, rstd);
    if (scale) {
      const float g = gamma ? gamma[c] : 1.f;
      const float b = beta ? beta[c] : 0.f;
      scale[c] = g * rstd;
      shift[c] = b - mu * g * rstd;
    }
  }
}

// ------------------------------------------------------------------ BN apply (+res) (+ReLU)
// y = act(u*sc + sh + res), res: 0 none | 1 r | 2 r*rsc + rsh
template <typename T, int VEC>
__global__ __launch_bounds__(256) void bn_apply_kernel(const T* __restrict__ u, int ldu, const float* sc,
                                                       const float* sh, int res_mode, const T* __restrict__ r,
                                                       int ldr, const float* rsc, const float* rsh, int relu,
                                                       T* __restrict__ y, int ldy, long M, int C, long rpb,
                                                       unsigned char* __restrict__ bits) {
  int CU, RPI;
  row_layout(C, VEC, CU, RPI);
  const int cu = threadIdx.x % CU, rs = threadIdx.x / CU;
  if (rs >= RPI) return;
  const int c0 = cu * VEC;
  float a[VEC], b[VEC], ra[VEC], rb[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    a[j] = sc[c0 + j];
    b[j] = sh[c0 + j];
    ra[j] = res_mode == 2 ? rsc[c0 + j] : 1.f;
    rb[j] = res_mode == 2 ? rsh[c0 + j] : 0.f;
  }
  const long mb = blockIdx.x * rpb, me = min(M, mb + rpb);
  // AU rows per thread and iteration, all loads issued before any use (a one-row loop kept two 16-B loads in
  // flight per thread: 4.5 TB/s at config 2); the next iteration's loads (raw 16-B units) are issued before this
  // iteration's stores — vmcnt completes in order, so loads issued after the stores would wait for their writes
  constexpr int AU = VEC == 1 ? 1 : 4;
  typedef typename std::conditional<VEC == 1, T, uint4>::type Raw;
  auto ld_raw = [&](const T* p) -> Raw {
    if constexpr (VEC == 1) return *p;
    else return *reinterpret_cast<const uint4*>(p);
  };
  auto unraw = [&](const Raw& v, float* f) {
    if constexpr (VEC == 1) f[0] = Tr<T>::to_f(v);
    else unpack16(v, f, (T*)nullptr);
  };
  Raw fu[AU], gu[AU], fn[AU], gn[AU];
  auto load = [&](long m0, Raw* fr, Raw* gr) {
#pragma unroll
    for (int k = 0; k < AU; ++k) {
      const long m = min(m0 + (long)k * RPI, me - 1);  // rows past the block's end re-read its last row
      fr[k] = ld_raw(u + m * ldu + c0);
      if (res_mode) gr[k] = ld_raw(r + m * ldr + c0);
    }
  };
  if (mb + rs < me) load(mb + rs, fu, gu);
  for (long m0 = mb + rs; m0 < me; m0 += (long)RPI * AU) {
    const bool more = m0 + (long)RPI * AU < me;
    if (more) load(m0 + (long)RPI * AU, fn, gn);
#pragma unroll
    for (int k = 0; k < AU; ++k) {
      const long m = m0 + (long)k * RPI;
      if (m >= me) break;
      float f[VEC], g[VEC];
      unraw(fu[k], f);
      if (res_mode) unraw(gu[k], g);
#pragma unroll
      for (int j = 0; j < VEC; ++j) f[j] = f[j] * a[j] + b[j];
      if (relu & 2) {  // inner ReLU on the normalised branch (RT-ST-GCN bn_relu, rtstgcn.py:319-321)
#pragma unroll
        for (int j = 0; j < VEC; ++j) f[j] = fmaxf(f[j], 0.f);
      }
      if (res_mode) {
#pragma unroll
        for (int j = 0; j < VEC; ++j) f[j] += g[j] * ra[j] + rb[j];
      }
      if (relu & 1) {
#pragma unroll
        for (int j = 0; j < VEC; ++j) f[j] = fmaxf(f[j], 0.f);
      }
      if constexpr (VEC == 8 && sizeof(T) == 2) {
        if (bits) {  // the stored values' sign bits (> 0: nonzero, sign clear), one byte per 8 channels
          const uint4 p = pack16(f, (T*)nullptr);
          *reinterpret_cast<uint4*>(y + m * ldy + c0) = p;
          const unsigned w[4] = {p.x, p.y, p.z, p.w};
          unsigned b = 0;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const unsigned h = (w[j >> 1] >> (16 * (j & 1))) & 0xffffu;
            b |= ((h & 0x8000u) == 0u && h != 0u) ? (1u << j) : 0u;
          }
          bits[m * (C / 8) + cu] = (unsigned char)b;
          continue;
        }
      }
      stv<T, VEC>(y + m * ldy + c0, f);
    }
    if (more) {
#pragma unroll
      for (int k = 0; k < AU; ++k) {
        fu[k] = fn[k];
        gu[k] = gn[k];
      }
    }
  }
}

// ------------------------------------------------------------------ BN backward
// partial sums per channel of dz and dz*xhat, dz = dy * mask.
// mask: 0 none | 1 (mref > 0) | 2 (mref*msc + msh > 0)
template <typename T, int VEC>
DEV void dz_load(const T* dy, int lddy, int mask, const T* mref, int ldm, const float* msc, const float* msh,
                 long m, int c0, float* dz) {
  ldv<T, VEC>(dy + m * lddy + c0, dz);
  if (mask) {
    float g[VEC];
    ldv<T, VEC>(mref + m * ldm + c0, g);
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const float pre = mask == 1 ? g[j] : g[j] * msc[c0 + j] + msh[c0 + j];
      if (!(pre > 0.f)) dz[j] = 0.f;
    }
  }
}

template <typename T, int VEC>
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(const T* __restrict__ dy, int lddy, int mask,
                                                            const T* __restrict__ mref, int ldm, const float* msc,
                                                            const float* msh, const T* __restrict__ x, int ldx,
                                                            const float2* mean_rstd, long M, int C, long rpb,
                                                            float2* part) {
  __shared__ float2 red[256 * 8];
  int CU, RPI;
  row_layout(C, VEC, CU, RPI);
  const int tid = threadIdx.x;
  const int cu = tid % CU, rs = tid / CU;
  const long mb = blockIdx.x * rpb, me = min(M, mb + rpb);
  float s1[VEC], s2[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) s1[j] = s2[j] = 0.f;
  if (rs < RPI) {
    const int c0 = cu * VEC;
    float mu[VEC], rsd[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const float2 st = x ? mean_rstd[c0 + j] : make_float2(0.f, 0.f);
      mu[j] = st.x;
      rsd[j] = st.y;
    }
    for (long m = mb + rs; m < me; m += RPI) {
      float dz[VEC];
      dz_load<T, VEC>(dy, lddy, mask, mref, ldm, msc, msh, m, c0, dz);
      float xv[VEC];
      if (x) ldv<T, VEC>(x + m * ldx + c0, xv);
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        s1[j] += dz[j];
        if (x) s2[j] += dz[j] * (xv[j] - mu[j]) * rsd[j];
      }
    }
#pragma unroll
    for (int j = 0; j < VEC; ++j) red[rs * C + c0 + j] = make_float2(s1[j], s2[j]);
  }
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    float a = 0.f, b = 0.f;
    for (int r = 0; r < RPI; ++r) {
      a += red[r * C + c].x;
      b += red[r * C + c].y;
    }
    part[(long)blockIdx.x * C + c] = make_float2(a, b);
  }
}

// column sums of float2 partials -> out[c] (double accumulation), one block per channel
__global__ __launch_bounds__(256) void sum_partials_kernel(const float2* part, int nb, int C, float2* out) {
  __shared__ double sa[256], sb[256];
  const int c = xcd_channel(blockIdx.x, C);
  double a = 0, b = 0;
  for (int i = threadIdx.x; i < nb; i += 256) {
    const float2 g = part[(long)i * C + c];
    a += g.x;
    b += g.y;
  }
  sa[threadIdx.x] = a;
  sb[threadIdx.x] = b;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      sa[threadIdx.x] += sa[threadIdx.x + s];
      sb[threadIdx.x] += sb[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) out[c] = make_float2((float)sa[0], (float)sb[0]);
}

// dx (+)= gamma*rstd*(dz - S1/M - xhat*S2/M); with x == nullptr: dx (+)= dz (identity branch)
template <typename T, int VEC>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const T* __restrict__ dy, int lddy, int mask,
                                                           const T* __restrict__ mref, int ldm, const float* msc,
                                                           const float* msh, const T* __restrict__ x, int ldx,
                                                           const float2* mean_rstd, const float* gamma,
                                                           const float2* sums, long M, int C, T* __restrict__ dx,
                                                           int lddx, int accumulate, long rpb) {
  int CU, RPI;
  row_layout(C, VEC, CU, RPI);
  const int cu = threadIdx.x % CU, rs = threadIdx.x / CU;
  if (rs >= RPI) return;
  const int c0 = cu * VEC;
  const float invM = 1.f / (float)M;
  // dx = k1*dz + k2*x + k3  with k1 = g*rstd, k2 = -g*rstd^2*S2/M, k3 = -g*rstd*S1/M + g*rstd^2*S2/M*mean
  float k1[VEC], k2[VEC], k3[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    if (x) {
      const float2 st = mean_rstd[c0 + j];
      const float2 sm = sums[c0 + j];
      const float g = gamma ? gamma[c0 + j] : 1.f;
      k1[j] = g * st.y;
      k2[j] = -g * st.y * st.y * sm.y * invM;
      k3[j] = -g * st.y * sm.x * invM - k2[j] * st.x;
    } else {
      k1[j] = 1.f;
      k2[j] = k3[j] = 0.f;
    }
  }
  const long mb = blockIdx.x * rpb, me = min(M, mb + rpb);
  for (long m = mb + rs; m < me; m += RPI) {
    float dz[VEC];
    dz_load<T, VEC>(dy, lddy, mask, mref, ldm, msc, msh, m, c0, dz);
    float o[VEC];
    if (x) {
      float xv[VEC];
      ldv<T, VEC>(x + m * ldx + c0, xv);
#pragma unroll
      for (int j = 0; j < VEC; ++j) o[j] = k1[j] * dz[j] + k2[j] * xv[j] + k3[j];
    } else {
#pragma unroll
      for (int j = 0; j < VEC; ++j) o[j] = dz[j];
    }
    if (accumulate) {
      float p[VEC];
      ldv<T, VEC>(dx + m * lddx + c0, p);
#pragma unroll
      for (int j = 0; j < VEC; ++j) o[j] += p[j];
    }
    stv<T, VEC>(dx + m * lddx + c0, o);
  }
}

// S[w][c] += sum_f x[(f*V + w)][c] over the block's frames; thread item = (w, channel unit), registers
// accumulate over frames, one atomicAdd per item per block.  period > 0: per-sample S[n][w][c].
template <typename T, int VEC>
__global__ __launch_bounds__(256) void rowgroup_sum_kernel(const T* __restrict__ x, int ld, long F, int C, int G,
                                                           long fpb, long frames_per_sample, float* part) {
  const int CU = C / VEC;
  const long fb0 = frames_per_sample > 0 ? (long)blockIdx.y * frames_per_sample : 0;
  const long flim = frames_per_sample > 0 ? fb0 + frames_per_sample : F;
  const long fb = fb0 + blockIdx.x * fpb, fe = min(flim, fb + fpb);
  for (int item = threadIdx.x; item < G * CU; item += 256) {
    const int w = item / CU, cu = item - w * CU;
    float acc[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] = 0.f;
    const T* base = x + w * (long)ld + cu * VEC;
    long f = fb;
    for (; f + 4 <= fe; f += 4) {  // 4 independent loads in flight
      float v0[VEC], v1[VEC], v2[VEC], v3[VEC];
      ldv<T, VEC>(base + (f + 0) * G * (long)ld, v0);
      ldv<T, VEC>(base + (f + 1) * G * (long)ld, v1);
      ldv<T, VEC>(base + (f + 2) * G * (long)ld, v2);
      ldv<T, VEC>(base + (f + 3) * G * (long)ld, v3);
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[j] += (v0[j] + v1[j]) + (v2[j] + v3[j]);
    }
    for (; f < fe; ++f) {
      float v[VEC];
      ldv<T, VEC>(base + f * G * (long)ld, v);
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[j] += v[j];
    }
    float* slab = part + ((long)blockIdx.y * gridDim.x + blockIdx.x) * G * C;  // per-block partial
#pragma unroll
    for (int j = 0; j < VEC; ++j) slab[w * C + cu * VEC + j] = acc[j];
  }
}


// ------------------------------------------------------------------ fp32 -> bf16 rows + column sums
// out16[m][c] = bf16(x[m][c]); part[b][c] = sum over block b's rows of x[m][c] (fp32, before the rounding).
// The attention projections' backward (aagcn.py:139-141 autograd): the bf16 operand of the data / weight
// gradient GEMMs and the bias gradient from one read of the fp32 gradient.  Thread = one 16-B unit (4
// channels) of a row, rows strided by the block's row groups; four rows' loads issued before their use.
__global__ __launch_bounds__(256) void cast_colsum_kernel(const float* __restrict__ x, int ldx, long M, int C,
                                                          bf16* __restrict__ out, int ldo, long rpb,
                                                          float* __restrict__ part) {
  __shared__ float red[256 * 4];
  const int cun = C / 4, rpi = 256 / cun;
  const int tid = threadIdx.x, cu = tid % cun, rs = tid / cun;
  float s[4] = {0.f, 0.f, 0.f, 0.f};
  if (rs < rpi) {
    const long mb = (long)blockIdx.x * rpb, me = min(M, mb + rpb);
    // four rows per thread per iteration; the next iteration's loads are issued before this one's stores
    // (vmcnt completes in order: loads issued after a store wait for its write to finish)
    auto ld4 = [&](long m0, float4* v) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long m = m0 + (long)u * rpi;
        v[u] = m < me ? *reinterpret_cast<const float4*>(x + m * ldx + cu * 4) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    };
    float4 v[4], nv[4];
    ld4(mb + rs, v);
    for (long m0 = mb + rs; m0 < me; m0 += 4L * rpi) {
      ld4(m0 + 4L * rpi, nv);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long m = m0 + (long)u * rpi;
        if (m >= me) continue;
        s[0] += v[u].x; s[1] += v[u].y; s[2] += v[u].z; s[3] += v[u].w;
        bf16x4 r;
        r[0] = (bf16)v[u].x; r[1] = (bf16)v[u].y; r[2] = (bf16)v[u].z; r[3] = (bf16)v[u].w;
        *reinterpret_cast<bf16x4*>(out + m * ldo + cu * 4) = r;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = nv[u];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) red[rs * C + cu * 4 + j] = s[j];
  }
  __syncthreads();
  for (int c = tid; c < C; c += 256) {
    float t = 0.f;
    for (int r = 0; r < rpi; ++r) t += red[r * C + c];  // fixed order
    part[(long)blockIdx.x * C + c] = t;
  }
}

// LayerNorm([C,1,V]): ln.hip

// ------------------------------------------------------------------ head: global average pool
// out[n][c] = mean_{r < R} x[(n*R + r)][c].  Block = (sample n, 64 channels); 256 threads = 8 units of
// 8 channels x 32 row groups, 16-B loads (bf16) four rows in flight per thread, fixed-order LDS combine.
template <typename T>
__global__ __launch_bounds__(256) void pool_rows_kernel(const T* __restrict__ x, int ld, int R, int C,
                                                        T* __restrict__ out, int ldo) {
  constexpr int VEC = 16 / (int)sizeof(T);  // channels per 16-B unit
  constexpr int UPB = 64 / VEC;             // units per 64-channel block
  constexpr int RG = 256 / UPB;             // row groups
  __shared__ float red[RG][64];
  const int n = blockIdx.y;
  const int u = threadIdx.x % UPB, rg = threadIdx.x / UPB;
  const int c0 = blockIdx.x * 64 + u * VEC;
  const bool vec = (ld % VEC) == 0 && c0 + VEC <= C;
  float s[VEC];
#pragma unroll
  for (int e = 0; e < VEC; ++e) s[e] = 0.f;
  const T* base = x + (long)n * R * ld + c0;
  if (vec) {
    int r = rg;
    for (; r + 3 * RG < R; r += 4 * RG) {
      uint4 q[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) q[k] = *reinterpret_cast<const uint4*>(base + (long)(r + k * RG) * ld);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        float f[VEC];
        unpack16(q[k], f, (T*)nullptr);
#pragma unroll
        for (int e = 0; e < VEC; ++e) s[e] += f[e];
      }
    }
    for (; r < R; r += RG) {
      float f[VEC];
      unpack16(*reinterpret_cast<const uint4*>(base + (long)r * ld), f, (T*)nullptr);
#pragma unroll
      for (int e = 0; e < VEC; ++e) s[e] += f[e];
    }
  } else {
    for (int r = rg; r < R; r += RG)
#pragma unroll
      for (int e = 0; e < VEC; ++e)
        if (c0 + e < C) s[e] += Tr<T>::to_f(base[(long)r * ld + e]);
  }
#pragma unroll
  for (int e = 0; e < VEC; ++e) red[rg][u * VEC + e] = s[e];
  __syncthreads();
  if (threadIdx.x < 64) {
    const int c = blockIdx.x * 64 + threadIdx.x;
    float t = 0.f;
    for (int k = 0; k < RG; ++k) t += red[k][threadIdx.x];
    if (c < C) out[(long)n * ldo + c] = Tr<T>::from_f(t / (float)R);
  }
}

// dx[m][c] = dp[m / R][c] / R; one thread per 16-B unit of a row when aligned
template <typename T>
__global__ __launch_bounds__(256) void unpool_rows_kernel(const T* __restrict__ dp, int ldp, int R, int C, long M,
                                                          T* __restrict__ dx, int ldx) {
  constexpr int VEC = 16 / (int)sizeof(T);
  const float inv = 1.f / (float)R;
  if ((C % VEC) == 0 && (ldp % VEC) == 0 && (ldx % VEC) == 0) {
    const int CU = C / VEC;
    const long total = M * CU;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
      const long m = i / CU;
      const int c = (int)(i - m * CU) * VEC;
      float f[VEC];
      unpack16(*reinterpret_cast<const uint4*>(dp + (m / R) * ldp + c), f, (T*)nullptr);
#pragma unroll
      for (int e = 0; e < VEC; ++e) f[e] *= inv;
      *reinterpret_cast<uint4*>(dx + m * ldx + c) = pack16(f, (T*)nullptr);
    }
    return;
  }
  const long total = M * C;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long m = i / C;
    const int c = (int)(i % C);
    dx[m * ldx + c] = Tr<T>::from_f(Tr<T>::to_f(dp[(m / R) * ldp + c]) * inv);
  }
}

int grid_for(long work) {
  long g = (work + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

// elementwise kernels: ~2048 blocks (one resident wave of 8 blocks per CU).  bn_apply at C=64..256 measured
// 41 us at 1024-2048 blocks, 43 at 3072, 45.6 at 4096, 56.5 at 8192.
long elt_rows_per_block(long M) {
  constexpr long nb = 2048;
  long rpb = (M + nb - 1) / nb;
  return rpb < 32 ? 32 : rpb;
}

long rows_per_block(long M) {
  long rpb = (M + 1023) / 1024;
  return rpb < 64 ? 64 : rpb;
}

}  // namespace

#define DISPATCH_VEC(dtype, C, ...)                                   \
  if (dtype == 1) {                                                   \
    typedef bf16 T;                                                   \
    if (C % 8 == 0) { constexpr int VEC = 8; __VA_ARGS__; }           \
    else { constexpr int VEC = 1; __VA_ARGS__; }                      \
  } else {                                                            \
    typedef float T;                                                  \
    if (C % 4 == 0) { constexpr int VEC = 4; __VA_ARGS__; }           \
    else { constexpr int VEC = 1; __VA_ARGS__; }                      \
  }

#define DISPATCH_T(dtype, ...)                  \
  if (dtype == 1) { typedef bf16 T; __VA_ARGS__; } \
  else { typedef float T; __VA_ARGS__; }

#define RET_HIP return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP

long norm_stats_num_blocks(long M) { return (M + rows_per_block(M) - 1) / rows_per_block(M); }

static bool rows_fit(int C, int dtype) {  // one row of C channels must fit the 256 threads
  const int vec = dtype == 1 ? (C % 8 == 0 ? 8 : 1) : (C % 4 == 0 ? 4 : 1);
  return C / vec <= 256;
}

int bn_stats_partial_launch(const void* x, int ld, long M, int C, float4* part, int dtype, hipStream_t s) {
  if (!rows_fit(C, dtype)) return STGCN_EBADSHAPE;
  const long rpb = rows_per_block(M);
  const int nb = (int)((M + rpb - 1) / rpb);
  DISPATCH_VEC(dtype, C, hipLaunchKernelGGL((bn_stats_partial_kernel<T, VEC>), dim3(nb), dim3(256), 0, s,
                                            (const T*)x, ld, M, C, rpb, part));
  RET_HIP;
}

int bn_finalize_launch(const float4* part, int nb, int ldp, int C, const float* gamma, const float* beta, float eps,
                       float2* mean_rstd, float* scale, float* shift, hipStream_t s) {
  const int nt = nb > 2048 ? 1024 : 256;  // one 8-load batch per thread where the list allows
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(C), dim3(nt), 0, s, part, nb, ldp, C, gamma, beta, eps, mean_rstd,
                     scale, shift, (float4*)nullptr);
  RET_HIP;
}

// the nb partials of each channel merged into one (count, mean, M2, 0) entry [C] — what a SyncBatchNorm rank
// contributes; the gathered [ranks][C] entries are finalized by bn_finalize_launch(nb = ranks, ldp = C)
int bn_merge_launch(const float4* part, int nb, int ldp, int C, float4* merged, hipStream_t s) {
  if (!part || !merged || nb < 1 || C < 1 || ldp < C) return STGCN_EBADSHAPE;
  const int nt = nb > 2048 ? 1024 : 256;
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(C), dim3(nt), 0, s, part, nb, ldp, C, (const float*)nullptr,
                     (const float*)nullptr, 0.f, (float2*)nullptr, (float*)nullptr, (float*)nullptr, merged);
  RET_HIP;
}

int bn_apply_launch(const void* u, int ldu, const float* sc, const float* sh, int res_mode, const void* r, int ldr,
                    const float* rsc, const float* rsh, int relu, void* y, int ldy, long M, int C, int dtype,
                    hipStream_t s, unsigned char* bits) {
  if (!rows_fit(C, dtype)) return STGCN_EBADSHAPE;
  // bit-mask output: the 16-B (8 x bf16) path only
  if (bits && (dtype != 1 || C % 8 || ldu % 8 || ldy % 8 || (res_mode && ldr % 8))) return STGCN_EBADSHAPE;
  const long rpb = elt_rows_per_block(M);
  const int nb = (int)((M + rpb - 1) / rpb);
  DISPATCH_VEC(dtype, C, hipLaunchKernelGGL((bn_apply_kernel<T, VEC>), dim3(nb), dim3(256), 0, s,
                                            (const T*)u, ldu, sc, sh, res_mode, (const T*)r, ldr, rsc, rsh, relu,
                                            (T*)y, ldy, M, C, rpb, bits));
  RET_HIP;
}

int bn_bwd_reduce_launch(const void* dy, int lddy, int mask, const void* mref, int ldm, const float* msc,
                         const float* msh, const void* x, int ldx, const float2* mean_rstd, long M, int C,
                         float2* part, float2* out, int dtype, hipStream_t s) {
  if (!rows_fit(C, dtype)) return STGCN_EBADSHAPE;
  const long rpb = rows_per_block(M);
  const int nb = (int)((M + rpb - 1) / rpb);
  DISPATCH_VEC(dtype, C, hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, VEC>), dim3(nb), dim3(256), 0, s,
                                            (const T*)dy, lddy, mask, (const T*)mref, ldm, msc, msh, (const T*)x,
                                            ldx, mean_rstd, M, C, rpb, part));
  hipLaunchKernelGGL(sum_partials_kernel, dim3(C), dim3(256), 0, s, part, nb, C, out);
  RET_HIP;
}

int bn_bwd_apply_launch(const void* dy, int lddy, int mask, const void* mref, int ldm, const float* msc,
                        const float* msh, const void* x, int ldx, const float2* mean_rstd, const float* gamma,
                        const float2* sums, long M, int C, void* dx, int lddx, int accumulate, int dtype,
                        hipStream_t s) {
  if (!rows_fit(C, dtype)) return STGCN_EBADSHAPE;
  const long rpb = elt_rows_per_block(M);
  const int nb = (int)((M + rpb - 1) / rpb);
  DISPATCH_VEC(dtype, C, hipLaunchKernelGGL((bn_bwd_apply_kernel<T, VEC>), dim3(nb), dim3(256), 0, s,
                                            (const T*)dy, lddy, mask, (const T*)mref, ldm, msc, msh, (const T*)x,
                                            ldx, mean_rstd, gamma, sums, M, C, (T*)dx, lddx, accumulate, rpb));
  RET_HIP;
}

static void rowgroup_geometry(long M, int G, long period, long& F, long& fps, long& nsamp, long& fpb, int& nb) {
  F = M / G;
  fps = period > 0 ? period / G : 0;
  nsamp = period > 0 ? M / period : 1;
  const long span = period > 0 ? fps : F;
  // ~1024 blocks over the whole tensor (enough loads in flight to stream it at HBM rate)
  fpb = (span * nsamp + 1023) / 1024;
  if (fpb < 4) fpb = 4;
  nb = (int)((span + fpb - 1) / fpb);
}

void slab_sum_launch(const float* in, long B, long R, long E, float* tmp, float* out, int accumulate, hipStream_t s);
long slab_sum_tmp_floats(long B, long R, long E);

long rowgroup_sum_workspace(long M, int C, int G, long period) {
  long F, fps, nsamp, fpb;
  int nb;
  rowgroup_geometry(M, G, period, F, fps, nsamp, fpb, nb);
  return (long)nb * nsamp * G * C + slab_sum_tmp_floats(nsamp, nb, (long)G * C);
}

int rowgroup_sum_launch(const void* x, int ld, long M, int C, int G, long period, float* S, float* work, int dtype,
                        hipStream_t s) {
  if (M % G || (period > 0 && (period % G || M % period))) return STGCN_EBADSHAPE;
  long F, fps, nsamp, fpb;
  int nb;
  rowgroup_geometry(M, G, period, F, fps, nsamp, fpb, nb);
  DISPATCH_VEC(dtype, C, hipLaunchKernelGGL((rowgroup_sum_kernel<T, VEC>), dim3(nb, (unsigned)nsamp), dim3(256), 0, s,
                                            (const T*)x, ld, F, C, G, fpb, fps, work));
  const long E = (long)G * C;
  slab_sum_launch(work, nsamp, nb, E, work + (long)nb * nsamp * E, S, 1, s);  // fixed-order, two levels
  RET_HIP;
}

static long cast_colsum_rpb(long M) {
  long rpb = (M + 2047) / 2048;  // ~2048 blocks
  return rpb < 64 ? 64 : rpb;
}
long cast_colsum_workspace(long M, int C) {
  const long nb = (M + cast_colsum_rpb(M) - 1) / cast_colsum_rpb(M);
  return nb * C + slab_sum_tmp_floats(1, nb, C);
}
int cast_colsum_launch(const float* x, int ldx, long M, int C, void* out16, int ldo, float* colsum, float* work,
                       hipStream_t s) {
  if (M <= 0) return STGCN_OK;
  if (C % 4 || C / 4 > 256 || ldx % 4 || ldo % 4 || ((size_t)x & 15) || ((size_t)out16 & 7)) return STGCN_EBADSHAPE;
  const long rpb = cast_colsum_rpb(M), nb = (M + rpb - 1) / rpb;
  hipLaunchKernelGGL(cast_colsum_kernel, dim3((unsigned)nb), dim3(256), 0, s, x, ldx, M, C, (bf16*)out16, ldo, rpb,
                     work);
  slab_sum_launch(work, 1, nb, C, work + nb * C, colsum, 0, s);
  RET_HIP;
}

int pool_rows_launch(const void* x, int ld, int N, int R, int C, void* out, int ldo, int dtype, hipStream_t s) {
  DISPATCH_T(dtype, hipLaunchKernelGGL(pool_rows_kernel<T>, dim3((C + 63) / 64, N), dim3(256), 0, s, (const T*)x, ld,
                                       R, C, (T*)out, ldo));
  RET_HIP;
}

int unpool_rows_launch(const void* dp, int ldp, int R, int C, long M, void* dx, int ldx, int dtype, hipStream_t s) {
  DISPATCH_T(dtype, hipLaunchKernelGGL(unpool_rows_kernel<T>, dim3(grid_for(M * C / 8 + 1)), dim3(256), 0, s, (const T*)dp,
                                       ldp, R, C, M, (T*)dx, ldx));
  RET_HIP;
}
