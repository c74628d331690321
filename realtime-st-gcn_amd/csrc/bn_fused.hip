// Fused BatchNorm backward of the ST-GCN layer tail (stgcn.py:160-193, autograd of
//   y = relu(BN2(u) + res),  res = BN_r(r) | x | 0          and of  h = relu(BN1(g))).
//
// Two passes over the rows instead of the four-to-six of the unfused path:
//   reduce : dz = dy * mask;  per channel  S = (sum dz, sum dz*xhat1, sum dz*xhat2)
//            (xhat2 = the residual branch's BN input r, sharing dz with BN2)
//   apply  : out1 = g1*rstd1*(dz - S0/M - xhat1*S1/M)          (du, or dg for BN1)
//            out2 = g2*rstd2*(dz - S0/M - xhat2*S2/M)          (dr)   | out2 (+)= dz (identity residual)
//            + per-channel column sums of out1 / out2 = the conv-bias gradients (tcn.2.bias,
//              residual.0.bias), which the unfused path took with two more passes.
// mask: 0 none | 1 (mref > 0) | 2 (mref*msc + msh > 0).  Rows are processed UNR at a time with all
// loads issued first (16-B units, channels-last), so every thread keeps several HBM requests in
// flight; partial sums go to a workspace [blocks][C] and are folded in fp64 by a second kernel.
#include "common.h"
#include "../../include/stgcn_amd.h"

namespace {

// rows per thread per iteration (raw 16-B units held until use, all loads issued first): 4 for the passes
// with at most three input streams, 2 for the four-stream ones (register budget)
constexpr int UNR_MAX = 4;
constexpr int ur_for(int streams) { return streams <= 3 ? 4 : 2; }

template <typename T, int VEC>
DEV void ld8(const T* p, float* f) {
  unpack16(*reinterpret_cast<const uint4*>(p), f, (T*)nullptr);
}
template <typename T, int VEC>
DEV void st8(T* p, const float* f) {
  *reinterpret_cast<uint4*>(p) = pack16(f, (T*)nullptr);
}

struct Geo {
  int CU;    // 16-B units per row
  int RPI;   // rows per block iteration (256 / CU)
  long rpb;  // rows per block
  int nb;
};

template <typename T, int VEC, int MASK, bool X2, int UNR>
__global__ __launch_bounds__(256) void bn_bwd_reduce_fused_kernel(const stgcn_bn_bwd_desc a, const Geo g) {
  __shared__ float4 red[256 * 8];  // [RPI][C]
  const int tid = threadIdx.x;
  const int cu = tid % g.CU, rs = tid / g.CU;
  const int c0 = cu * VEC;
  const T* dy = reinterpret_cast<const T*>(a.dy);
  const T* mref = reinterpret_cast<const T*>(a.mref);
  const T* x1 = reinterpret_cast<const T*>(a.x1);
  // BN1 backward: the mask reference and the normalised input are the same tensor (g): load it once
  const bool same_x = MASK == 2 && (const void*)x1 == (const void*)mref && a.ldx1 == a.ldm;
  const T* x2 = reinterpret_cast<const T*>(a.x2);
  float s0[VEC], s1[VEC], s2[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) s0[j] = s1[j] = s2[j] = 0.f;
  if (rs < g.RPI) {
    float mu1[VEC], rs1[VEC], mu2[VEC], rs2[VEC], msc[VEC], msh[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const float2 m1 = reinterpret_cast<const float2*>(a.mean_rstd1)[c0 + j];
      const float2 m2 = X2 ? reinterpret_cast<const float2*>(a.mean_rstd2)[c0 + j] : make_float2(0.f, 0.f);
      mu1[j] = m1.x; rs1[j] = m1.y; mu2[j] = m2.x; rs2[j] = m2.y;
      msc[j] = MASK == 2 ? a.msc[c0 + j] : 0.f;
      msh[j] = MASK == 2 ? a.msh[c0 + j] : 0.f;
    }
    const long mb = (long)blockIdx.x * g.rpb, me = min(a.M, mb + g.rpb);
    for (long m0 = mb + rs; m0 < me; m0 += (long)g.RPI * UNR) {
      uint4 Udz[UNR], Umr[UNR], Uxa[UNR], Uxb[UNR];
      bool ok[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const long m = m0 + (long)u * g.RPI;
        ok[u] = m < me;
        const long mm = ok[u] ? m : mb;
        Udz[u] = *reinterpret_cast<const uint4*>(dy + mm * a.lddy + c0);
        if constexpr (MASK == 3)  // the forward's sign bits: one byte per 8 channels
          Umr[u].x = reinterpret_cast<const unsigned char*>(a.mref)[mm * a.ldm + cu];
        else
          Umr[u] = *reinterpret_cast<const uint4*>(mref + mm * a.ldm + c0);
        if (!same_x) Uxa[u] = *reinterpret_cast<const uint4*>(x1 + mm * a.ldx1 + c0);
        if (X2) Uxb[u] = *reinterpret_cast<const uint4*>(x2 + mm * a.ldx2 + c0);
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        if (!ok[u]) continue;
        float dz[1][VEC], mr[1][VEC], xa[1][VEC], xb[1][VEC];
        unpack16(Udz[u], dz[0], (T*)nullptr);
        if constexpr (MASK != 3) unpack16(Umr[u], mr[0], (T*)nullptr);
        unpack16(same_x ? Umr[u] : Uxa[u], xa[0], (T*)nullptr);
        if (X2) unpack16(Uxb[u], xb[0], (T*)nullptr);
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          float d = dz[0][j];
          if (MASK == 1 && !(mr[0][j] > 0.f)) d = 0.f;
          if (MASK == 2 && !(mr[0][j] * msc[j] + msh[j] > 0.f)) d = 0.f;
          if (MASK == 3 && !((Umr[u].x >> j) & 1u)) d = 0.f;
          s0[j] += d;
          s1[j] += d * (xa[0][j] - mu1[j]) * rs1[j];
          if (X2) s2[j] += d * (xb[0][j] - mu2[j]) * rs2[j];
        }
      }
    }
#pragma unroll
    for (int j = 0; j < VEC; ++j) red[rs * a.C + c0 + j] = make_float4(s0[j], s1[j], s2[j], 0.f);
  }
  __syncthreads();
  float4* part = reinterpret_cast<float4*>(a.work);
  for (int c = tid; c < a.C; c += 256) {
    float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int r = 0; r < g.RPI; ++r) {
      const float4 v = red[r * a.C + c];
      t.x += v.x; t.y += v.y; t.z += v.z;
    }
    part[(long)blockIdx.x * a.C + c] = t;
  }
}

// column sums of float4 partials [nb][C] -> out [C] (fp64 accumulation); one block per channel.
// The same values also go planar to ((float*)(out + C))[k*C + c], k < 3, so per-channel parameter
// gradients are contiguous views (no gather copies on the host side).
__global__ __launch_bounds__(256) void sum4_kernel(const float4* part, int nb, int C, float4* out) {
  // the partials of a thread are loaded together, then a wave reduction and one LDS step (an 8-level LDS
  // tree with a barrier per level was most of this ~5 us launch, 27 of them per config-2 step)
  __shared__ double sred[3][4];
  const int c = xcd_channel(blockIdx.x, C);
  double x = 0, y = 0, z = 0;
  for (int i0 = 0; i0 < nb; i0 += 256 * 4) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + threadIdx.x + 256 * u;
      v[u] = i < nb ? part[(long)i * C + c] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      x += v[u].x; y += v[u].y; z += v[u].z;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    x += __shfl_xor(x, o);
    y += __shfl_xor(y, o);
    z += __shfl_xor(z, o);
  }
  if ((threadIdx.x & 63) == 0) {
    sred[0][threadIdx.x >> 6] = x;
    sred[1][threadIdx.x >> 6] = y;
    sred[2][threadIdx.x >> 6] = z;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const double sx0 = ((sred[0][0] + sred[0][1]) + sred[0][2]) + sred[0][3];
    const double sy0 = ((sred[1][0] + sred[1][1]) + sred[1][2]) + sred[1][3];
    const double sz0 = ((sred[2][0] + sred[2][1]) + sred[2][2]) + sred[2][3];
    const float4 r = make_float4((float)sx0, (float)sy0, (float)sz0, 0.f);
    out[c] = r;
    float* pl = reinterpret_cast<float*>(out + C);
    pl[c] = r.x;
    pl[C + c] = r.y;
    pl[2 * C + c] = r.z;
  }
}

template <typename T, int VEC, int MASK, int O2, bool OSUM, int UNR>
__global__ __launch_bounds__(256) void bn_bwd_apply_fused_kernel(const stgcn_bn_bwd_desc a, const Geo g) {
  __shared__ float2 red[256 * 8];
  const int tid = threadIdx.x;
  const int cu = tid % g.CU, rs = tid / g.CU;
  const int c0 = cu * VEC;
  const T* dy = reinterpret_cast<const T*>(a.dy);
  const T* mref = reinterpret_cast<const T*>(a.mref);
  const T* x1 = reinterpret_cast<const T*>(a.x1);
  // BN1 backward: the mask reference and the normalised input are the same tensor (g): load it once
  const bool same_x = MASK == 2 && (const void*)x1 == (const void*)mref && a.ldx1 == a.ldm;
  const T* x2 = reinterpret_cast<const T*>(a.x2);
  T* o1 = reinterpret_cast<T*>(a.out1);
  T* o2 = reinterpret_cast<T*>(a.out2);
  const float invM = 1.f / (float)a.M;
  float q1[VEC], q2[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) q1[j] = q2[j] = 0.f;
  if (rs < g.RPI) {
    // out = k1*dz + k2*x + k3 (k2 = -g*rstd^2*S/M, k3 = -g*rstd*S0/M - k2*mean)
    float k11[VEC], k21[VEC], k31[VEC], k12[VEC], k22[VEC], k32[VEC], msc[VEC], msh[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      const float4 sm = reinterpret_cast<const float4*>(a.sums)[c0 + j];
      {
        const float2 st = reinterpret_cast<const float2*>(a.mean_rstd1)[c0 + j];
        const float gm = a.gamma1 ? a.gamma1[c0 + j] : 1.f;
        k11[j] = gm * st.y;
        k21[j] = -gm * st.y * st.y * sm.y * invM;
        k31[j] = -gm * st.y * sm.x * invM - k21[j] * st.x;
      }
      if (O2 == 1) {
        const float2 st = reinterpret_cast<const float2*>(a.mean_rstd2)[c0 + j];
        const float gm = a.gamma2 ? a.gamma2[c0 + j] : 1.f;
        k12[j] = gm * st.y;
        k22[j] = -gm * st.y * st.y * sm.z * invM;
        k32[j] = -gm * st.y * sm.x * invM - k22[j] * st.x;
      } else {
        k12[j] = 1.f; k22[j] = k32[j] = 0.f;
      }
      msc[j] = MASK == 2 ? a.msc[c0 + j] : 0.f;
      msh[j] = MASK == 2 ? a.msh[c0 + j] : 0.f;
    }
    const long mb = (long)blockIdx.x * g.rpb, me = min(a.M, mb + g.rpb);
    // the next iteration's loads are issued before this iteration's stores (vmcnt completes in order: loads
    // issued after the stores would wait for their writes)
    uint4 Udz[UNR], Umr[UNR], Uxa[UNR], Uxb[UNR], Upa[UNR];
    uint4 Ndz[UNR], Nmr[UNR], Nxa[UNR], Nxb[UNR], Npa[UNR];
    bool ok[UNR], nok[UNR];
    auto load = [&](long m0, uint4* Ldz, uint4* Lmr, uint4* Lxa, uint4* Lxb, uint4* Lpa, bool* lok) {
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const long m = m0 + (long)u * g.RPI;
        lok[u] = m < me;
        const long mm = lok[u] ? m : mb;
        Ldz[u] = *reinterpret_cast<const uint4*>(dy + mm * a.lddy + c0);
        if constexpr (MASK == 3)
          Lmr[u].x = reinterpret_cast<const unsigned char*>(a.mref)[mm * a.ldm + cu];
        else
          Lmr[u] = *reinterpret_cast<const uint4*>(mref + mm * a.ldm + c0);
        if (!same_x) Lxa[u] = *reinterpret_cast<const uint4*>(x1 + mm * a.ldx1 + c0);
        if (O2 == 1) Lxb[u] = *reinterpret_cast<const uint4*>(x2 + mm * a.ldx2 + c0);
        if (O2 && a.acc2) Lpa[u] = *reinterpret_cast<const uint4*>(o2 + mm * a.ldo2 + c0);
      }
    };
    if (mb + rs < me) load(mb + rs, Udz, Umr, Uxa, Uxb, Upa, ok);
    for (long m0 = mb + rs; m0 < me; m0 += (long)g.RPI * UNR) {
      const bool more = m0 + (long)g.RPI * UNR < me;
      if (more) load(m0 + (long)g.RPI * UNR, Ndz, Nmr, Nxa, Nxb, Npa, nok);
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        if (!ok[u]) continue;
        const long m = m0 + (long)u * g.RPI;
        float dz[VEC], mr[VEC], xa[VEC], xb[VEC], pa[VEC];
        unpack16(Udz[u], dz, (T*)nullptr);
        if constexpr (MASK != 3) unpack16(Umr[u], mr, (T*)nullptr);
        unpack16(same_x ? Umr[u] : Uxa[u], xa, (T*)nullptr);
        if (O2 == 1) unpack16(Uxb[u], xb, (T*)nullptr);
        if (O2 && a.acc2) unpack16(Upa[u], pa, (T*)nullptr);
        float r1[VEC], r2[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          float d = dz[j];
          if (MASK == 1 && !(mr[j] > 0.f)) d = 0.f;
          if (MASK == 2 && !(mr[j] * msc[j] + msh[j] > 0.f)) d = 0.f;
          if (MASK == 3 && !((Umr[u].x >> j) & 1u)) d = 0.f;
          r1[j] = k11[j] * d + k21[j] * xa[j] + k31[j];
          r2[j] = O2 == 1 ? k12[j] * d + k22[j] * xb[j] + k32[j] : d;
          if (O2 && a.acc2) r2[j] += pa[j];
        }
        st8<T, VEC>(o1 + m * a.ldo1 + c0, r1);
        if (O2) st8<T, VEC>(o2 + m * a.ldo2 + c0, r2);
        if (OSUM) {
          // bias gradients from the fp32 values before the storage rounding: for a bias that feeds a
          // batch-statistics BatchNorm the exact sum is ~0, and summing 480 000 bf16-rounded values would
          // add a random walk of rounding errors (~1 % of the paired weight gradient at config 2)
#pragma unroll
          for (int j = 0; j < VEC; ++j) {
            q1[j] += r1[j];
            q2[j] += r2[j];
          }
        }
      }
      if (more) {
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          Udz[u] = Ndz[u];
          Umr[u] = Nmr[u];
          Uxa[u] = Nxa[u];
          Uxb[u] = Nxb[u];
          Upa[u] = Npa[u];
          ok[u] = nok[u];
        }
      }
    }
    if (OSUM) {
#pragma unroll
      for (int j = 0; j < VEC; ++j) red[rs * a.C + c0 + j] = make_float2(q1[j], q2[j]);
    }
  }
  if (OSUM) {
    __syncthreads();
    float4* part = reinterpret_cast<float4*>(a.work);
    for (int c = tid; c < a.C; c += 256) {
      float2 t = make_float2(0.f, 0.f);
      for (int r = 0; r < g.RPI; ++r) {
        const float2 v = red[r * a.C + c];
        t.x += v.x; t.y += v.y;
      }
      part[(long)blockIdx.x * a.C + c] = make_float4(t.x, t.y, 0.f, 0.f);
    }
  }
}

// block target of the apply pass (the reduce pass keeps 1024: its partials are folded by sum4_kernel, and it
// measured slower with fewer blocks); A/B build flag
#ifndef STGCN_BN_APPLY_TB
#define STGCN_BN_APPLY_TB 512
#endif
Geo geo(long M, int C, int vec, long tb = 1024) {
  Geo g;
  g.CU = C / vec;
  g.RPI = 256 / g.CU;
  // >= 2 iterations of UNR_MAX rows per thread and at most ~tb blocks
  const long step = (long)g.RPI * UNR_MAX;
  // block target (both passes): 512 / 1024 / 2048 measured 1.67 / 1.68 / 1.8 ms per step for all fused BN
  // backward passes + sum4 folds (512 speeds up apply, slows reduce)
  long it = (M + step * tb - 1) / (step * tb);
  if (it < 2) it = 2;
  g.rpb = step * it;
  g.nb = (int)((M + g.rpb - 1) / g.rpb);
  return g;
}

bool fits(const stgcn_bn_bwd_desc& a, int dtype, int& vec) {
  vec = dtype == 1 ? 8 : 4;
  if (a.C % vec || a.C / vec > 256 || a.C > 2048) return false;
  auto al = [&](int ld) { return ld % vec == 0; };
  if (a.mask == 3 && dtype != 1) return false;
  return al(a.lddy) && (!a.mask || a.mask == 3 || al(a.ldm)) && (!a.x1 || al(a.ldx1)) && (!a.x2 || al(a.ldx2)) &&
         (!a.out1 || al(a.ldo1)) && (!a.out2 || al(a.ldo2));
}

long bn_bwd_fused_work_floats_impl(long M, int C, int dtype) {
  const Geo g = geo(M, C, dtype == 1 ? 8 : 4), ga = geo(M, C, dtype == 1 ? 8 : 4, STGCN_BN_APPLY_TB);
  return (long)(g.nb > ga.nb ? g.nb : ga.nb) * C * 4;
}

template <typename T, int VEC, int MASK, bool X2>
void launch_reduce(const stgcn_bn_bwd_desc& a, const Geo& g, hipStream_t s) {
  // input streams: dy, the mask reference, x1 (shared with the mask reference for BN1), x2
  constexpr int UR = ur_for(2 + (MASK == 1 ? 1 : 0) + (X2 ? 1 : 0));  // mask 2 reads x1, mask 3 one byte
  hipLaunchKernelGGL((bn_bwd_reduce_fused_kernel<T, VEC, MASK, X2, UR>), dim3(g.nb), dim3(256), 0, s, a, g);
}
template <typename T, int VEC>
void reduce_dispatch(const stgcn_bn_bwd_desc& a, const Geo& g, hipStream_t s) {
  if (a.mask == 1) {
    if (a.x2) launch_reduce<T, VEC, 1, true>(a, g, s);
    else launch_reduce<T, VEC, 1, false>(a, g, s);
  } else if (a.mask == 3) {
    if constexpr (VEC == 8) {
      if (a.x2) launch_reduce<T, VEC, 3, true>(a, g, s);
      else launch_reduce<T, VEC, 3, false>(a, g, s);
    }
  } else {
    if (a.x2) launch_reduce<T, VEC, 2, true>(a, g, s);
    else launch_reduce<T, VEC, 2, false>(a, g, s);
  }
}

template <typename T, int VEC, int MASK, int O2>
void launch_apply(const stgcn_bn_bwd_desc& a, const Geo& g, hipStream_t s) {
  constexpr int UR = ur_for(2 + (MASK == 1 ? 1 : 0) + (O2 == 1 ? 1 : 0));  // (+ out2 read-back when acc2)
  if (a.osum)
    hipLaunchKernelGGL((bn_bwd_apply_fused_kernel<T, VEC, MASK, O2, true, UR>), dim3(g.nb), dim3(256), 0, s, a, g);
  else
    hipLaunchKernelGGL((bn_bwd_apply_fused_kernel<T, VEC, MASK, O2, false, UR>), dim3(g.nb), dim3(256), 0, s, a, g);
}
template <typename T, int VEC>
void apply_dispatch(const stgcn_bn_bwd_desc& a, const Geo& g, hipStream_t s) {
  const int o2 = a.out2 ? (a.x2 ? 1 : 2) : 0;
  if (a.mask == 1) {
    if (o2 == 1) launch_apply<T, VEC, 1, 1>(a, g, s);
    else if (o2 == 2) launch_apply<T, VEC, 1, 2>(a, g, s);
    else launch_apply<T, VEC, 1, 0>(a, g, s);
  } else if (a.mask == 3) {
    if constexpr (VEC == 8) {
      if (o2 == 1) launch_apply<T, VEC, 3, 1>(a, g, s);
      else if (o2 == 2) launch_apply<T, VEC, 3, 2>(a, g, s);
      else launch_apply<T, VEC, 3, 0>(a, g, s);
    }
  } else {
    if (o2 == 1) launch_apply<T, VEC, 2, 1>(a, g, s);
    else if (o2 == 2) launch_apply<T, VEC, 2, 2>(a, g, s);
    else launch_apply<T, VEC, 2, 0>(a, g, s);
  }
}

}  // namespace

long bn_bwd_fused_work_floats(long M, int C, int dtype) { return bn_bwd_fused_work_floats_impl(M, C, dtype); }

int bn_bwd_fused_reduce_launch(const stgcn_bn_bwd_desc& a, int dtype, hipStream_t s) {
  int vec;
  if (!fits(a, dtype, vec) || !a.work || !a.sums || !a.x1 || !a.mref || a.mask < 1 || a.mask > 3)
    return STGCN_EBADSHAPE;
  const Geo g = geo(a.M, a.C, vec);
  if (dtype == 1) reduce_dispatch<bf16, 8>(a, g, s);
  else reduce_dispatch<float, 4>(a, g, s);
  hipLaunchKernelGGL(sum4_kernel, dim3(a.C), dim3(256), 0, s, (const float4*)a.work, g.nb, a.C, (float4*)a.sums);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

int bn_bwd_fused_apply_launch(const stgcn_bn_bwd_desc& a, int dtype, hipStream_t s) {
  int vec;
  if (!fits(a, dtype, vec) || !a.out1 || !a.sums || !a.x1 || !a.mref || (a.osum && !a.work) || a.mask < 1 ||
      a.mask > 3)
    return STGCN_EBADSHAPE;
  const Geo g = geo(a.M, a.C, vec, STGCN_BN_APPLY_TB);
  if (dtype == 1) apply_dispatch<bf16, 8>(a, g, s);
  else apply_dispatch<float, 4>(a, g, s);
  if (a.osum)
    hipLaunchKernelGGL(sum4_kernel, dim3(a.C), dim3(256), 0, s, (const float4*)a.work, g.nb, a.C,
                       (float4*)a.osum);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
