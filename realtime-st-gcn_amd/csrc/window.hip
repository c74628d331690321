// Window staging: the first activation of a batch of sliding windows, built straight
// from the padded capture.  The reference (WindowSegment, utils/segment_generator.py:132-145) unfolds the
// padded capture (1, Cin, Lp, V) into nw windows of W frames — a W-fold copy, (nw, Cin, W, V) — then
// runs norm_in (BatchNorm1d(V*Cin) over the batch, batchnorm.py:13-23, or the per-frame LayerNorm,
// layernorm.py:22-28) and fcn_in (1x1 conv Cin -> Cout, stgcn.py:82-85) over every copy.
//
// Window n holds padded frames [n, n+W): row (n, t, v) of every one of these tensors is a function of
// padded frame p = n + t alone.  So nothing here forms the windows:
//   * BatchNorm statistics of the windowed batch = statistics over the distinct frames weighted by their
//     multiplicity m(p) = #windows holding p (win_bn_stats_kernel -> (count, mean, M2) partials merged by
//     the existing bn_finalize); LayerNorm statistics are per frame (win_ln_stats_kernel);
//   * the first activation is written once: each (frame, joint) unit is computed once from the frame's Cin
//     values and stored into every window holding the frame (win_expand_kernel; HBM-write bound);
//   * backward (the capture takes no gradient): dy is folded back onto frames, D(p) = sum over the windows
//     holding p, and every parameter gradient is a sum over frames of D(p) against the frame's values
//     (win_grad_kernel: one pass over dy; deterministic per-block partials + win_grad_finish_kernel).
// Layouts: capture fp32 [Cin][Lp][V] (batch 1, as the reference's trial loader gives it); activation rows
// channels-last [nw][W][V][Cout] (bf16 or fp32), row stride ld.
#include "common.h"

namespace {

constexpr int STAT_FB = 8;       // frames per statistics block
constexpr int GRAD_BLOCKS = 4096;  // at most this many frame runs in the gradient pass

// windows n in [n0, n1) that hold padded frame p
DEV int win_mult(int p, int n0, int n1, int W) { return min(p, n1 - 1) - max(n0, p - W + 1) + 1; }

__global__ __launch_bounds__(256) void win_bn_stats_kernel(const float* __restrict__ X, int Cin, int Lp, int V, int W,
                                                           int n0, int nw, float4* __restrict__ part) {
  const int F = nw + W - 1;
  const int f0 = blockIdx.x * STAT_FB, f1 = min(F, f0 + STAT_FB);
  const int KC = V * Cin;
  for (int k = threadIdx.x; k < KC; k += blockDim.x) {  // k = v*Cin + c: the reference's BatchNorm1d channel
    const int v = k / Cin, c = k - v * Cin;
    const float* xp = X + (long)c * Lp * V + v;
    float s0 = 0.f, s1 = 0.f;
    for (int f = f0; f < f1; ++f) {
      const float m = (float)win_mult(n0 + f, n0, n0 + nw, W);
      s0 += m;
      s1 += m * xp[(long)(n0 + f) * V];
    }
    const float mean = s1 / s0;
    float m2 = 0.f;
    for (int f = f0; f < f1; ++f) {
      const float m = (float)win_mult(n0 + f, n0, n0 + nw, W);
      const float d = xp[(long)(n0 + f) * V] - mean;
      m2 += m * d * d;
    }
    part[(long)blockIdx.x * KC + k] = make_float4(s0, mean, m2, 0.f);
  }
}

// LayerNorm([Cin,1,V]) statistics of each frame: mean and 1/sqrt(unbiased var + eps); one wave per frame
__global__ __launch_bounds__(256) void win_ln_stats_kernel(const float* __restrict__ X, int Cin, int Lp, int V, int n0,
                                                           int F, float eps, float2* __restrict__ fst) {
  const int f = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (f >= F) return;  // whole waves
  const int p = n0 + f, KC = Cin * V;
  float s = 0.f;
  for (int k = lane; k < KC; k += 64) s += X[((long)(k / V) * Lp + p) * V + k % V];
  const float mean = wave_sum(s) / (float)KC;
  float q = 0.f;
  for (int k = lane; k < KC; k += 64) {
    const float d = X[((long)(k / V) * Lp + p) * V + k % V] - mean;
    q += d * d;
  }
  const float var = wave_sum(q) / (float)(KC - 1);
  if (lane == 0) fst[f] = make_float2(mean, 1.f / sqrtf(var + eps));
}

// normalised values of (frame p = n0 + f, joint v): xh = standardised, xn = gamma * xh + beta
// mode 0 (BatchNorm1d): st = (mean, rstd) per channel v*Cin + c; gamma/beta index v*Cin + c
// mode 1 (LayerNorm):   st = (mean, rstd) per frame f;          gamma/beta index c*V + v
template <int CIN>
DEV void win_norm(const float* __restrict__ X, int Lp, int V, int p, int f, int v, int mode,
                  const float2* __restrict__ st, const float* __restrict__ g, const float* __restrict__ b,
                  float* xh, float* xn) {
  float2 fs = make_float2(0.f, 1.f);
  if (mode == 1) fs = st[f];
#pragma unroll
  for (int c = 0; c < CIN; ++c) {
    const float x = X[((long)c * Lp + p) * V + v];
    const int k = mode == 0 ? v * CIN + c : c * V + v;
    const float2 s = mode == 0 ? st[k] : fs;
    xh[c] = (x - s.x) * s.y;
    xn[c] = xh[c] * g[k] + b[k];
  }
}

// One thread = one 16-byte unit (joint v, channels [u*VEC, u*VEC + VEC)) of one frame f: the unit is
// computed once and stored into every window holding the frame (rows (n*W + f - n)*V + v).  Consecutive
// lanes take consecutive units of a frame, so each store instruction writes one contiguous run of a row
// block.  mode 0 takes the FOLDED affine (sc = gamma*rstd, sh = beta - mean*sc, from bn_finalize) as g/b
// with fst = NULL; mode 1 takes the frame statistics and gamma/beta.
template <typename T, int CIN>
__global__ __launch_bounds__(256) void win_expand_kernel(const float* __restrict__ X, int Lp, int V, int W,
                                                         int n0, int nw, int units, int mode,
                                                         const float2* __restrict__ fst, const float* __restrict__ g,
                                                         const float* __restrict__ b, const float* __restrict__ w,
                                                         const float* __restrict__ bias, int Cout,
                                                         T* __restrict__ out, int ldo) {
  constexpr int VEC = Tr<T>::VEC;
  const int U = Cout / VEC;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= units) return;
  const int VU = V * U;
  const int f = i / VU, r = i - f * VU;
  const int v = r / U, u = r - v * U;
  const int p = n0 + f;
  float xn[CIN];
  if (mode == 0) {
#pragma unroll
    for (int c = 0; c < CIN; ++c) xn[c] = X[((long)c * Lp + p) * V + v] * g[v * CIN + c] + b[v * CIN + c];
  } else {
    float xh[CIN];
    win_norm<CIN>(X, Lp, V, p, f, v, 1, fst, g, b, xh, xn);
  }
  float y[8];
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    const int co = u * VEC + j;
    float a = bias ? bias[co] : 0.f;
#pragma unroll
    for (int c = 0; c < CIN; ++c) a = fmaf(w[co * CIN + c], xn[c], a);
    y[j] = a;
  }
  const uint4 val = pack16(y, (T*)nullptr);
  const int na = max(0, f - W + 1), nb = min(nw - 1, f);
  T* o = out + ((long)f * V + v) * ldo + u * VEC;  // window n: + n*(W-1)*V rows
  const long step = (long)(W - 1) * V * ldo;
  for (int n = na; n <= nb; ++n) *reinterpret_cast<uint4*>(o + n * step) = val;
}

// One block = a run of frames; thread (v, u) owns joint v and output channels [u*VEC, u*VEC + VEC).
// Partials per block: [Cout][Cin + 1] (dW, then db in column Cin), dgamma [V*Cin], dbeta [V*Cin] (in the
// norm's own parameter order).  dy rows of window n, frame t: (n*W + t)*V + v.
template <typename T, int CIN>
__global__ __launch_bounds__(512) void win_grad_kernel(const T* __restrict__ dy, int ldd, const float* __restrict__ X,
                                                        int Lp, int V, int W, int n0, int nw, int FB, int mode,
                                                        const float2* __restrict__ st, const float* __restrict__ g,
                                                        const float* __restrict__ b, const float* __restrict__ w,
                                                        int Cout, float* __restrict__ work, int E) {
  constexpr int VEC = Tr<T>::VEC;
  extern __shared__ float red[];  // [V][Cout][Cin + 1]
  const int U = Cout / VEC;
  const int tid = threadIdx.x;
  const int v = tid / U, u = tid - v * U;
  const bool act = v < V;
  const int F = nw + W - 1;
  const int f0 = blockIdx.x * FB, f1 = min(F, f0 + FB);
  float dwa[VEC][CIN], dba[VEC], dga[CIN], dbb[CIN], wc[VEC][CIN];
#pragma unroll
  for (int j = 0; j < VEC; ++j) {
    dba[j] = 0.f;
#pragma unroll
    for (int c = 0; c < CIN; ++c) {
      dwa[j][c] = 0.f;
      wc[j][c] = act ? w[(u * VEC + j) * CIN + c] : 0.f;
    }
  }
#pragma unroll
  for (int c = 0; c < CIN; ++c) dga[c] = dbb[c] = 0.f;

  for (int f = f0; f < f1; ++f) {
    float D[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) D[j] = 0.f;
    if (act) {
      const int na = max(0, f - W + 1), nb = min(nw - 1, f);
      const T* base = dy + ((long)f * V + v) * ldd + u * VEC;  // row of (n, t = f - n) = (n*(W-1) + f)*V + v
      const long step = (long)(W - 1) * V * ldd;
      int n = na;
      for (; n + 7 <= nb; n += 8) {
        uint4 q[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) q[k] = *reinterpret_cast<const uint4*>(base + (n + k) * step);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float e[8];
          unpack16(q[k], e, (T*)nullptr);
#pragma unroll
          for (int j = 0; j < VEC; ++j) D[j] += e[j];
        }
      }
      for (; n <= nb; ++n) {
        float e[8];
        unpack16(*reinterpret_cast<const uint4*>(base + n * step), e, (T*)nullptr);
#pragma unroll
        for (int j = 0; j < VEC; ++j) D[j] += e[j];
      }
    }
    float xh[CIN], xn[CIN];
    if (act) {
      win_norm<CIN>(X, Lp, V, n0 + f, f, v, mode, st, g, b, xh, xn);
    } else {
#pragma unroll
      for (int c = 0; c < CIN; ++c) xh[c] = xn[c] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      dba[j] += D[j];
#pragma unroll
      for (int c = 0; c < CIN; ++c) dwa[j][c] = fmaf(D[j], xn[c], dwa[j][c]);
    }
    // d(norm output) of this (frame, joint): sum over all Cout channels = over the U lanes of joint v
#pragma unroll
    for (int c = 0; c < CIN; ++c) {
      float d = 0.f;
#pragma unroll
      for (int j = 0; j < VEC; ++j) d = fmaf(wc[j][c], D[j], d);
      for (int o = U >> 1; o > 0; o >>= 1) d += __shfl_xor(d, o);
      dga[c] = fmaf(d, xh[c], dga[c]);
      dbb[c] += d;
    }
  }

  // block partials: dW/db reduced over joints through LDS in a fixed order; dgamma/dbeta from lane u == 0
  constexpr int CE = CIN + 1;
  if (act) {
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      float* r = red + ((long)v * Cout + u * VEC + j) * CE;
#pragma unroll
      for (int c = 0; c < CIN; ++c) r[c] = dwa[j][c];
      r[CIN] = dba[j];
    }
  }
  float* wb = work + (long)blockIdx.x * E;
  if (act && u == 0) {
    float* dgp = wb + Cout * CE;
#pragma unroll
    for (int c = 0; c < CIN; ++c) {
      const int k = mode == 0 ? v * CIN + c : c * V + v;
      dgp[k] = dga[c];
      dgp[V * CIN + k] = dbb[c];
    }
  }
  __syncthreads();
  for (int e = tid; e < Cout * CE; e += blockDim.x) {
    float s = 0.f;
    for (int vv = 0; vv < V; ++vv) s += red[(long)vv * Cout * CE + e];
    wb[e] = s;
  }
}

// 64 entries per block, 16 interleaved groups of partial rows per entry, combined in a fixed order
__global__ __launch_bounds__(1024) void win_grad_finish_kernel(const float* __restrict__ work, int nb, int E, int Cin,
                                                               int Cout, int VC, float* __restrict__ dw,
                                                               float* __restrict__ db, float* __restrict__ dg,
                                                               float* __restrict__ dbeta) {
  __shared__ float part[16][64];
  const int le = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + le;
  float s = 0.f;
  if (e < E) {
    int k = q;
    for (; k + 48 < nb; k += 64) {
      const float a0 = work[(long)k * E + e], a1 = work[(long)(k + 16) * E + e];
      const float a2 = work[(long)(k + 32) * E + e], a3 = work[(long)(k + 48) * E + e];
      s += (a0 + a1) + (a2 + a3);
    }
    for (; k < nb; k += 16) s += work[(long)k * E + e];
  }
  part[q][le] = s;
  __syncthreads();
  if (q != 0 || e >= E) return;
  s = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) s += part[j][le];
  const int CE = Cin + 1;
  if (e < Cout * CE) {
    const int co = e / CE, c = e - co * CE;
    if (c < Cin) {
      if (dw) dw[co * Cin + c] = s;
    } else if (db) {
      db[co] = s;
    }
  } else if (e < Cout * CE + VC) {
    if (dg) dg[e - Cout * CE] = s;
  } else if (dbeta) {
    dbeta[e - Cout * CE - VC] = s;
  }
}

bool win_shape_ok(int Cin, int Lp, int V, int W, int n0, int nw) {
  return Cin >= 1 && Cin <= 8 && V >= 1 && W >= 1 && nw >= 1 && n0 >= 0 && (long)n0 + nw + W - 1 <= Lp;
}

int grad_fb(int F) { return (F + GRAD_BLOCKS - 1) / GRAD_BLOCKS; }

// instantiate per input-channel count (the capture's features: 3 for xyz skeletons) and element type
#define WIN_CASE_T(CV, ...)           \
  case CV: {                          \
    constexpr int CIN = CV;           \
    if (dtype == 1) {                 \
      typedef bf16 T;                 \
      __VA_ARGS__;                    \
    } else {                          \
      typedef float T;                \
      __VA_ARGS__;                    \
    }                                 \
  } break;
#define WIN_DISPATCH(cin, dtype, ...)                                                                     \
  switch (cin) {                                                                                          \
    WIN_CASE_T(1, __VA_ARGS__) WIN_CASE_T(2, __VA_ARGS__) WIN_CASE_T(3, __VA_ARGS__)                      \
    WIN_CASE_T(4, __VA_ARGS__) WIN_CASE_T(6, __VA_ARGS__) WIN_CASE_T(8, __VA_ARGS__)                      \
    default: return STGCN_EBADSHAPE;                                                                      \
  }

}  // namespace

int window_stat_blocks_launch(int nw, int W) { return (nw + W - 1 + STAT_FB - 1) / STAT_FB; }

int window_stats_launch(const float* x, int Cin, int Lp, int V, int W, int n0, int nw, int mode, float eps, float* out,
                        hipStream_t s) {
  if (!x || !out || !win_shape_ok(Cin, Lp, V, W, n0, nw) || (mode != 0 && mode != 1)) return STGCN_EBADSHAPE;
  const int F = nw + W - 1;
  if (mode == 0)
    hipLaunchKernelGGL(win_bn_stats_kernel, dim3(window_stat_blocks_launch(nw, W)), dim3(256), 0, s, x, Cin, Lp, V, W,
                       n0, nw, reinterpret_cast<float4*>(out));
  else {
    if (Cin * V < 2) return STGCN_EBADSHAPE;
    hipLaunchKernelGGL(win_ln_stats_kernel, dim3((F + 3) / 4), dim3(256), 0, s, x, Cin, Lp, V, n0, F, eps,
                       reinterpret_cast<float2*>(out));
  }
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

int window_expand_launch(const float* x, int Cin, int Lp, int V, int W, int n0, int nw, int mode, const float* g,
                         const float* b, const float* fst, const float* w, const float* bias, int Cout, void* out,
                         int ldo, int dtype, hipStream_t s) {
  if (!x || !g || !b || !w || !out || !win_shape_ok(Cin, Lp, V, W, n0, nw) || (mode != 0 && mode != 1) ||
      (mode == 1 && !fst) || (dtype != 0 && dtype != 1))
    return STGCN_EBADSHAPE;
  const int VEC = dtype == 1 ? 8 : 4;
  if (Cout < VEC || Cout % VEC || ldo < Cout || ldo % VEC) return STGCN_EBADSHAPE;
  const long units = (long)(nw + W - 1) * V * (Cout / VEC);
  if (units > 0x7fffffffL) return STGCN_EBADSHAPE;
  const dim3 grid((unsigned)((units + 255) / 256));
  const float2* st = reinterpret_cast<const float2*>(fst);
  WIN_DISPATCH(Cin, dtype,
               hipLaunchKernelGGL((win_expand_kernel<T, CIN>), grid, dim3(256), 0, s, x, Lp, V, W, n0, nw, (int)units,
                                  mode, st, g, b, w, bias, Cout, (T*)out, ldo));
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

long window_grad_workspace_launch(int nw, int W, int V, int Cin, int Cout) {
  const int F = nw + W - 1;
  const long nb = (F + grad_fb(F) - 1) / grad_fb(F);
  return nb * ((long)Cout * (Cin + 1) + 2L * V * Cin) * 4;
}

int window_grad_launch(const void* dy, int ldd, int dtype, const float* x, int Cin, int Lp, int V, int W, int n0, int nw,
                       int mode, const float* st, const float* g, const float* b, const float* w, int Cout, float* work,
                       float* dg, float* dbeta, float* dw, float* db, hipStream_t s) {
  if (!dy || !x || !st || !g || !b || !w || !work || !win_shape_ok(Cin, Lp, V, W, n0, nw) ||
      (mode != 0 && mode != 1) || (dtype != 0 && dtype != 1))
    return STGCN_EBADSHAPE;
  const int VEC = dtype == 1 ? 8 : 4;
  const int U = Cout / VEC;
  if (Cout < VEC || Cout % VEC || ldd < Cout || ldd % VEC || (U & (U - 1)) || U > 64) return STGCN_EBADSHAPE;
  const int threads = (V * U + 63) / 64 * 64;
  if (threads > 512) return STGCN_EBADSHAPE;
  const size_t lds = (size_t)V * Cout * (Cin + 1) * sizeof(float);
  if (lds > 160 * 1024) return STGCN_EBADSHAPE;
  const int F = nw + W - 1, FB = grad_fb(F), nb = (F + FB - 1) / FB;
  const int E = Cout * (Cin + 1) + 2 * V * Cin;
  const float2* st2 = reinterpret_cast<const float2*>(st);
  int rc = STGCN_OK;
  WIN_DISPATCH(Cin, dtype, {
    if (stgcn_lds_attr((const void*)win_grad_kernel<T, CIN>, 160 * 1024, s)) {
      rc = STGCN_EHIP;
    } else {
      hipLaunchKernelGGL((win_grad_kernel<T, CIN>), dim3(nb), dim3(threads), lds, s, (const T*)dy, ldd, x, Lp, V, W,
                         n0, nw, FB, mode, st2, g, b, w, Cout, work, E);
    }
  });
  if (rc != STGCN_OK || hipGetLastError() != hipSuccess) return STGCN_EHIP;
  hipLaunchKernelGGL(win_grad_finish_kernel, dim3((E + 63) / 64), dim3(1024), 0, s, work, nb, E, Cin, Cout, V * Cin,
                     dw, db, dg, dbeta);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
