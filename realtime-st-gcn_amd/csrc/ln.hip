// LayerNorm([C,1,V]) of the ln/ configs (models/utils/layernorm.py:4-28): per (n,t) frame over its V rows x C
// channels, UNBIASED variance, per-(c,v) affine gamma/beta[c*V + v], eps 1e-5.  Channels-last rows: frame f is
// rows f*V .. f*V+V-1 (row stride ld), so the kernels move 16-B units (8 bf16 / 4 fp32 channels of one row;
// 1 element when the rows do not allow it).  U = V*C/VEC units per frame; unit p -> row v = p / (C/VEC),
// channels c0 = (p % (C/VEC))*VEC.
//
//  ln_stats : one wave per frame, shifted one-pass sums (shift = the frame's first element, so the
//             sum of squares carries no mean^2 cancellation), (mean, rstd) per frame.
//  ln_apply : y = act((u-mu)*rstd*g + b [+ r | + LN_r(r)]).  The grid's thread count is a multiple of U, so a
//             thread visits the SAME unit position of every frame it handles: its 2*VEC (4*VEC with an LN
//             residual) affine parameters are loaded once, and the frame index steps without a division.
//  ln_bwd   : dx (+)= rstd*(gz - mean(gz) - xhat*sum(gz*xhat)/(E-1)), gz = dz*g, dz = dy*mask.  A block walks a
//             contiguous run of frames, one thread per unit of a frame (blocks of 256, 512 or 1024 threads; a
//             unit is 1, 2 or 4 16-B vectors of a row, the fewest that keep a frame within 1024 units);
//             the two frame sums are a wave reduction + an LDS exchange per frame (double-buffered, one
//             barrier); the raw loads of the next PF frames are in flight in a register ring meanwhile.  dgamma/dbeta (sum over frames of dz*xhat, dz) accumulate in
//             registers over the run — each thread always holds the same units — and go to a per-block slab,
//             summed over the blocks in a fixed order (deterministic; slab_sum_launch).
// Bound: HBM (stats 1 read, apply 2-3 reads + 1 write, bwd 2-3 reads + 1 write of the activation).
#include "common.h"

void slab_sum_launch(const float* in, long B, long R, long E, float* tmp, float* out, int accumulate, hipStream_t s);
long slab_sum_tmp_floats(long B, long R, long E);

namespace {

template <typename T, int VEC>
DEV void ldu(const T* p, float* f) {
  if constexpr (VEC == 1) {
    f[0] = Tr<T>::to_f(*p);
  } else {
    unpack16(*reinterpret_cast<const uint4*>(p), f, (T*)nullptr);
  }
}
template <typename T, int VEC>
DEV void stu(T* p, const float* f) {
  if constexpr (VEC == 1) {
    *p = Tr<T>::from_f(f[0]);
  } else {
    *reinterpret_cast<uint4*>(p) = pack16(f, (T*)nullptr);
  }
}

// ------------------------------------------------------------------ statistics
template <typename T, int VEC>
__global__ __launch_bounds__(256) void ln_stats_kernel(const T* __restrict__ x, int ld, long F, int V, int C,
                                                       float eps, float2* __restrict__ st) {
  const int lane = threadIdx.x & 63;
  const long f = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (f >= F) return;
  const int cun = C / VEC, U = V * cun;
  const T* base = x + f * V * (long)ld;
  const float K = Tr<T>::to_f(base[0]);
  float s1 = 0.f, s2 = 0.f;
  for (int p0 = lane; p0 < U; p0 += 4 * 64) {  // four units in flight per lane
    float a[4][VEC];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int p = p0 + 64 * k;
      if (p < U) {
        const int v = p / cun;
        ldu<T, VEC>(base + (long)v * ld + (p - v * cun) * VEC, a[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (p0 + 64 * k < U) {
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          const float d = a[k][j] - K;
          s1 += d;
          s2 += d * d;
        }
      }
  }
  s1 = wave_sum(s1);
  s2 = wave_sum(s2);
  const float E = (float)(V * C);
  const float md = s1 / E;
  const float var = fmaxf((s2 - s1 * md) / (E - 1.f), 0.f);  // unbiased (torch.var default, layernorm.py:24)
  if (lane == 0) st[f] = make_float2(K + md, 1.f / sqrtf(var + eps));
}

// ------------------------------------------------------------------ apply
struct LnApplyArgs {
  const void* u;
  const float2* st;
  const float* g;
  const float* b;
  const void* r;
  const float2* rst;
  const float* rg;
  const float* rb;
  void* y;
  long F;
  int ldu, ldr, ldy, V, C, res_mode, relu;
};

template <typename T, int VEC>
DEV void apply_unit(const LnApplyArgs& a, long f, int v, int c0, const float* ga, const float* ba, const float* rga,
                    const float* rba, const float* uu, const float* rr) {
  const float2 s = a.st[f];
  float o[VEC];
  float2 q = make_float2(0.f, 0.f);
  if (a.res_mode == 2) q = a.rst[f];
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    float t = (uu[j] - s.x) * s.y * ga[j] + ba[j];
    if (a.relu & 2) t = fmaxf(t, 0.f);
    if (a.res_mode == 1) t += rr[j];
    if (a.res_mode == 2) t += (rr[j] - q.x) * q.y * rga[j] + rba[j];
    if (a.relu & 1) t = fmaxf(t, 0.f);
    o[j] = t;
  }
  stu<T, VEC>(reinterpret_cast<T*>(a.y) + (f * a.V + v) * (long)a.ldy + c0, o);
}

template <typename T, int VEC>
__global__ __launch_bounds__(256) void ln_apply_kernel(const LnApplyArgs a) {
  const int cun = a.C / VEC, U = a.V * cun;
  const long i0 = (long)blockIdx.x * 256 + threadIdx.x;
  const long fstep = (long)gridDim.x * 256 / U;  // the host makes gridDim.x * 256 a multiple of U
  const int p = (int)(i0 % U);
  const int v = p / cun, c0 = (p - v * cun) * VEC;
  float ga[VEC], ba[VEC], rga[VEC], rba[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    const int gi = (c0 + j) * a.V + v;
    ga[j] = a.g[gi];
    ba[j] = a.b[gi];
    rga[j] = a.res_mode == 2 ? a.rg[gi] : 0.f;
    rba[j] = a.res_mode == 2 ? a.rb[gi] : 0.f;
  }
  const T* u = reinterpret_cast<const T*>(a.u);
  const T* r = reinterpret_cast<const T*>(a.r);
  const long ou = (long)v * a.ldu + c0, orr = (long)v * a.ldr + c0;
  long f = i0 / U;
  for (; f + fstep < a.F; f += 2 * fstep) {  // two frames' loads in flight
    float u0[VEC], u1[VEC], r0[VEC], r1[VEC];
    ldu<T, VEC>(u + f * a.V * (long)a.ldu + ou, u0);
    ldu<T, VEC>(u + (f + fstep) * a.V * (long)a.ldu + ou, u1);
    if (a.res_mode) {
      ldu<T, VEC>(r + f * a.V * (long)a.ldr + orr, r0);
      ldu<T, VEC>(r + (f + fstep) * a.V * (long)a.ldr + orr, r1);
    }
    apply_unit<T, VEC>(a, f, v, c0, ga, ba, rga, rba, u0, r0);
    apply_unit<T, VEC>(a, f + fstep, v, c0, ga, ba, rga, rba, u1, r1);
  }
  if (f < a.F) {
    float u0[VEC], r0[VEC];
    ldu<T, VEC>(u + f * a.V * (long)a.ldu + ou, u0);
    if (a.res_mode) ldu<T, VEC>(r + f * a.V * (long)a.ldr + orr, r0);
    apply_unit<T, VEC>(a, f, v, c0, ga, ba, rga, rba, u0, r0);
  }
}

// ------------------------------------------------------------------ backward
struct LnBwdArgs {
  const void* dy;
  const void* mref;
  const void* x;
  const float2* st;
  const float* g;
  const float* b;
  void* dx;
  float* slab;  // [nb][2][E] (dgamma | dbeta, element c*V+v) or NULL
  long F;
  long fpb;  // frames per block
  int lddy, ldm, ldx, lddx, V, C, mask, accumulate;
};

// raw (packed) storage of one 16-B vector, or of one element on the scalar path
template <typename T, int VEC1> struct RawOf { typedef uint4 type; };
template <typename T> struct RawOf<T, 1> { typedef T type; };

template <typename T, int VEC1>
DEV typename RawOf<T, VEC1>::type ld_raw(const T* p) {
  if constexpr (VEC1 == 1) return *p;
  else return *reinterpret_cast<const uint4*>(p);
}
template <typename T, int VEC1>
DEV void unpack_raw(const typename RawOf<T, VEC1>::type& r, float* f) {
  if constexpr (VEC1 == 1) f[0] = Tr<T>::to_f(r);
  else unpack16(r, f, (T*)nullptr);
}

// NT threads (one per unit of R vectors), PF frames of raw loads in flight per thread: the loads of frame f + PF
// are issued as soon as frame f's have been unpacked, so they fly under f's reduction barrier and its stores —
// a thread without the ring waits out the full load latency once per frame (measured 2.3 us/frame).
template <typename T, int VEC1, int R, int NT, int PF, int MASK>
__global__ __launch_bounds__(NT) void ln_bwd_kernel(const LnBwdArgs a) {
  constexpr int VEC = VEC1 * R;  // elements per unit
  constexpr int NW = NT / 64;
  typedef typename RawOf<T, VEC1>::type Raw;
  __shared__ float red[2][NW][2];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int cun = a.C / VEC, U = a.V * cun, E = a.V * a.C;
  const long f0 = (long)blockIdx.x * a.fpb;
  const long f1 = f0 + a.fpb < a.F ? f0 + a.fpb : a.F;
  const T* dy = reinterpret_cast<const T*>(a.dy);
  const T* mref = reinterpret_cast<const T*>(a.mref);
  const T* x = reinterpret_cast<const T*>(a.x);
  T* dx = reinterpret_cast<T*>(a.dx);
  const bool on = t < U;
  const int pp = on ? t : 0;
  const int v = pp / cun, c0 = (pp - v * cun) * VEC;
  float ga[VEC], ba[VEC], dgam[VEC], dbet[VEC];
#pragma unroll
  for (int k = 0; k < VEC; ++k) {
    const int gi = (c0 + k) * a.V + v;
    ga[k] = a.g[gi];
    ba[k] = MASK == 2 ? a.b[gi] : 0.f;
    dgam[k] = 0.f;
    dbet[k] = 0.f;
  }
  Raw rdy[PF][R], rx[PF][R], rm[PF][R];
  auto issue = [&](int q, long f) {
    if (on && f < f1) {
      const long row = f * a.V + v;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        rdy[q][r] = ld_raw<T, VEC1>(dy + row * a.lddy + c0 + r * VEC1);
        rx[q][r] = ld_raw<T, VEC1>(x + row * a.ldx + c0 + r * VEC1);
        if (MASK == 1) rm[q][r] = ld_raw<T, VEC1>(mref + row * a.ldm + c0 + r * VEC1);
      }
    }
  };
#pragma unroll
  for (int q = 0; q < PF; ++q) issue(q, f0 + q);
  int par = 0;
  for (long fb = f0; fb < f1; fb += PF) {
#pragma unroll
    for (int q = 0; q < PF; ++q) {
      const long f = fb + q;
      if (f >= f1) break;  // block-uniform
      const float2 s = a.st[f];
      float dz[VEC], xh[VEC];
      float p1 = 0.f, p2 = 0.f;
      if (on) {
        float m[VEC];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          unpack_raw<T, VEC1>(rdy[q][r], dz + r * VEC1);
          unpack_raw<T, VEC1>(rx[q][r], xh + r * VEC1);
          if (MASK == 1) unpack_raw<T, VEC1>(rm[q][r], m + r * VEC1);
        }
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
          xh[k] = (xh[k] - s.x) * s.y;
          if (MASK == 1 && !(m[k] > 0.f)) dz[k] = 0.f;
          if (MASK == 2 && !(xh[k] * ga[k] + ba[k] > 0.f)) dz[k] = 0.f;
          const float gz = dz[k] * ga[k];
          p1 += gz;
          p2 += gz * xh[k];
          dgam[k] += dz[k] * xh[k];
          dbet[k] += dz[k];
        }
      }
      issue(q, f + PF);  // the slot is free: its frame is in registers
      p1 = wave_sum(p1);
      p2 = wave_sum(p2);
      if (lane == 0) {
        red[par][wave][0] = p1;
        red[par][wave][1] = p2;
      }
      __syncthreads();
      float a1 = 0.f, a2 = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) {  // fixed order
        a1 += red[par][w][0];
        a2 += red[par][w][1];
      }
      par ^= 1;  // the other slot is written next frame: every wave has passed this frame's barrier by then
      if (on) {
        const float k1 = a1 / (float)E, k2 = a2 / (float)(E - 1);
        T* p = dx + (f * a.V + v) * a.lddx + c0;
        float o[VEC], old[VEC];
        if (a.accumulate) {
#pragma unroll
          for (int r = 0; r < R; ++r) ldu<T, VEC1>(p + r * VEC1, old + r * VEC1);
        }
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
          o[k] = s.y * (dz[k] * ga[k] - k1 - xh[k] * k2);
          if (a.accumulate) o[k] += old[k];
        }
#pragma unroll
        for (int r = 0; r < R; ++r) stu<T, VEC1>(p + r * VEC1, o + r * VEC1);
      }
    }
  }
  if (a.slab && on) {
    float* sl = a.slab + (long)blockIdx.x * 2 * E;
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      const int gi = (c0 + k) * a.V + v;
      sl[gi] = dgam[k];
      sl[E + gi] = dbet[k];
    }
  }
}

int vec_of(int dtype, int C, std::initializer_list<long> lds, std::initializer_list<const void*> ptrs) {
  const int vec = dtype == 1 ? 8 : 4;
  if (C % vec) return 1;
  for (long l : lds)
    if (l % vec) return 1;
  for (const void* p : ptrs)
    if (p && ((size_t)p & 15)) return 1;
  return vec;
}

int bwd_threads(int U) {  // threads per block of ln_bwd (one per unit): 256, 512 or 1024; 0 = too many units
  const int n = (U + 255) / 256 * 256;
  return n <= 256 ? 256 : (n <= 512 ? 512 : (n <= 1024 ? 1024 : 0));
}

// vectors per ln_bwd unit (1, 2, 4, 8; 16-B vectors: 1, 2): the fewest that bring a frame to <= 512 units (the
// 1024-thread blocks' 128-VGPR cap spills the prefetch ring), else to <= 1024; 0 = none (the scalar path's 8
// elements per unit cover every C that is a multiple of 8 up to 1024 / V * 8: C = 256 at V = 25 on a misaligned view)
int bwd_r(int V, int C, int vec) {
  const int rmax = vec > 1 ? 2 : 8;
  for (int lim = 512; lim <= 1024; lim *= 2)
    for (int r = 1; r <= rmax; r *= 2)
      if ((C / vec) % r == 0 && V * (C / vec / r) <= lim) return r;
  return 0;
}

// blocks of ln_bwd: whole rounds of the resident blocks (2 per CU of 256 threads, 1 of 512 / 1024 at the kernels'
// VGPR counts; a partial last round costs a full block time), one round with gamma/beta gradients (the per-block
// slab stays <= ~13 MB), two without
long bwd_blocks(long F, int nt, bool slab) {
  const long nb = (nt == 256 ? 512L : 256L) * (slab ? 1 : 2);
  return nb > F ? F : nb;
}

long gcd_l(long a, long b) {
  while (b) {
    const long t = a % b;
    a = b;
    b = t;
  }
  return a;
}

}  // namespace

#define LN_DISPATCH(dtype, vec, ...)                            \
  if (dtype == 1) {                                             \
    typedef bf16 T;                                             \
    if (vec == 8) { constexpr int VEC = 8; __VA_ARGS__; }       \
    else { constexpr int VEC = 1; __VA_ARGS__; }                \
  } else {                                                      \
    typedef float T;                                            \
    if (vec == 4) { constexpr int VEC = 4; __VA_ARGS__; }       \
    else { constexpr int VEC = 1; __VA_ARGS__; }                \
  }

int ln_stats_launch(const void* x, int ld, long F, int V, int C, float eps, float2* stats, int dtype, hipStream_t s) {
  if (F <= 0) return STGCN_OK;
  const int vec = vec_of(dtype, C, {ld}, {x});
  LN_DISPATCH(dtype, vec, hipLaunchKernelGGL((ln_stats_kernel<T, VEC>), dim3((unsigned)((F + 3) / 4)), dim3(256), 0, s,
                                             (const T*)x, ld, F, V, C, eps, stats));
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

int ln_apply_launch(const void* u, int ldu, const float2* st, const float* g, const float* b, int res_mode,
                    const void* r, int ldr, const float2* rst, const float* rg, const float* rb, int relu, void* y,
                    int ldy, long M, int V, int C, int dtype, hipStream_t s) {
  if (M <= 0) return STGCN_OK;
  if (M % V) return STGCN_EBADSHAPE;
  LnApplyArgs a{u, st, g, b, res_mode ? r : nullptr, rst, rg, rb, y, M / V, ldu, res_mode ? ldr : 0, ldy, V, C,
                res_mode, relu};
  const int vec = vec_of(dtype, C, {ldu, a.ldr, ldy}, {u, a.r, y});
  const long U = (long)V * (C / vec);
  // gridDim * 256 a multiple of U: grid = G0 * k with G0 = U / gcd(U, 256), ~2048 blocks
  const long G0 = U / gcd_l(U, 256);
  long k = 2048 / G0;
  if (k < 1) k = 1;
  const long need = (a.F * U + 255) / 256;  // no more blocks than one sweep needs
  while (k > 1 && G0 * (k - 1) >= need) --k;
  LN_DISPATCH(dtype, vec, hipLaunchKernelGGL((ln_apply_kernel<T, VEC>), dim3((unsigned)(G0 * k)), dim3(256), 0, s, a));
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

static void bwd_geometry(long F, int V, int C, int vec, bool slab, long& nb, long& fpb, int& nt) {
  const int r = bwd_r(V, C, vec);
  nt = r ? bwd_threads(V * (C / vec / r)) : 0;
  nb = bwd_blocks(F, nt, slab);
  fpb = (F + nb - 1) / nb;
  nb = (F + fpb - 1) / fpb;
}

long ln_bwd_workspace(long F, int V, int C, int dtype) {
  if (F <= 0) return 0;
  const long nb = F < 512 ? F : 512;  // the most blocks any unit width takes with a slab (bwd_blocks)
  const long E2 = 2L * V * C;
  return (long)sizeof(float) * (nb * E2 + slab_sum_tmp_floats(1, nb, E2));
}

int ln_bwd_launch(const void* dy, int lddy, int mask, const void* mref, int ldm, const void* x, int ldx,
                  const float2* st, const float* g, const float* b, long F, int V, int C, void* dx, int lddx,
                  int accumulate, float* dgb, void* work, long work_bytes, int dtype, hipStream_t s) {
  if (F <= 0) return STGCN_OK;
  if (dgb && (!work || work_bytes < ln_bwd_workspace(F, V, C, dtype))) return STGCN_EBADSHAPE;
  const int vec = vec_of(dtype, C, {lddy, mask == 1 ? ldm : 0, ldx, lddx}, {dy, mask == 1 ? mref : nullptr, x, dx});
  long nb, fpb;
  int nt;
  bwd_geometry(F, V, C, vec, dgb != nullptr, nb, fpb, nt);
  if (!nt) return STGCN_EBADSHAPE;  // > 4096 vectors per frame
  const int R = bwd_r(V, C, vec);
  LnBwdArgs a{dy, mask == 1 ? mref : nullptr, x, st, g, b, dx, dgb ? (float*)work : nullptr, F, fpb,
              lddy, mask == 1 ? ldm : 0, ldx, lddx, V, C, mask, accumulate};
#define LN_BWD_GO(R_, NT_, PF_)                                                                                  \
  do {                                                                                                          \
    if (mask == 1) hipLaunchKernelGGL((ln_bwd_kernel<T, VEC, R_, NT_, PF_, 1>), dim3((unsigned)nb), dim3(NT_), 0, s, a); \
    else if (mask == 2) hipLaunchKernelGGL((ln_bwd_kernel<T, VEC, R_, NT_, PF_, 2>), dim3((unsigned)nb), dim3(NT_), 0, s, a); \
    else hipLaunchKernelGGL((ln_bwd_kernel<T, VEC, R_, NT_, PF_, 0>), dim3((unsigned)nb), dim3(NT_), 0, s, a);     \
  } while (0)
#define LN_BWD_NT(R_, PF_)                    \
  do {                                        \
    if (nt == 256) LN_BWD_GO(R_, 256, PF_);   \
    else if (nt == 512) LN_BWD_GO(R_, 512, PF_); \
    else LN_BWD_GO(R_, 1024, (PF_ > 2 ? 2 : PF_)); \
  } while (0)
  LN_DISPATCH(dtype, vec, {
    if (R == 1) LN_BWD_NT(1, 4);
    else if constexpr (VEC > 1) LN_BWD_NT(2, 2);
    else if (R == 2) LN_BWD_NT(2, 2);
    else if (R == 4) LN_BWD_NT(4, 1);
    else LN_BWD_NT(8, 1);
  });
#undef LN_BWD_NT
#undef LN_BWD_GO
  if (hipGetLastError() != hipSuccess) return STGCN_EHIP;
  if (dgb) {
    const long E2 = 2L * V * C;
    float* slab = (float*)work;
    slab_sum_launch(slab, 1, nb, E2, slab + nb * E2, dgb, 1, s);
  }
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
