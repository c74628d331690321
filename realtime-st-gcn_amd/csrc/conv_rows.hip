// Implicit-GEMM temporal convolution over channels-last skeleton rows (MFMA, gfx950).
//
// Covers every (Kt x 1) convolution on the ST-GCN hot path:
//   * tcn.2           Conv2d(C, C, (Kt,1), stride (s,1), pad ((Kt-1)/2,0))   stgcn.py:154-159
//   * residual.0      Conv2d(Cin, Cout, 1, stride (s,1))                     stgcn.py:165-170
//   * gcn.conv        Conv2d(Cin, P*Cout, 1) on the A-mixed rows (K = P*Cin)  tgcn.py:48-55,71
//   * fcn_in/fcn_out  1x1 convs                                              stgcn.py:49,74
//   * the data-gradients of all of the above (trans = 1: transposed conv, any stride).
//
//   out[m, co] = epi( sum_{dt, ci} W[dt][co][ci] * pro(in[src(m, dt), ci]) )
//   m = (n*T_out + t)*V + v;  src = (n*T_in + t_in)*V + v with
//     trans = 0:  t_in = t*stride + dt - pad
//     trans = 1:  t_in = (t + pad - dt) / stride   (only when divisible)
//   rows with t_in outside [0, T_in) contribute zero (zero padding AFTER the prologue).
//   pro : 0 none | 1 relu(x*a[ci] + b[ci]) (BatchNorm apply + ReLU, stgcn.py:152-153)
//         | 2 relu((x-mu[n,t])*rs[n,t]*a[ci*V+v] + b[ci*V+v]) (custom LayerNorm + ReLU, layernorm.py:22-28)
//   epi : + bias[co] | + bias2d[v][co] | + bias3d[n][v][co] ; optional += existing out ; optional BatchNorm partial
//         statistics (count, mean, M2) per column per row-block for a later finalize (Chan merge).
//
// Tiling: 256 threads = 4 waves as WM x WN; each wave owns TM x TN tiles of 32x32
// (v_mfma_f32_32x32x16_bf16 or 8x v_mfma_f32_32x32x2_f32).  K is walked as (ci-chunk of KC=32,
// tap dt) pairs; A (gathered rows) and B (packed weights) tiles are double-buffered in LDS with
// register prefetch of the next pair, XOR-swizzled so fragment reads are bank-conflict free.
#include "common.h"
#include "pack.h"
#include <stdlib.h>

#include "../../include/stgcn_amd.h"
typedef stgcn_conv_desc ConvArgs;

namespace {

constexpr int KC = 32;  // k-chunk (elements) staged per LDS tile

template <typename T>
struct Layout {
  static constexpr int RB = KC * sizeof(T);        // bytes per tile row
  static constexpr int UPR = RB / 16;              // 16-byte units per row
  static constexpr int RPB = (256 / RB) > 0 ? 256 / RB : 1;  // rows per 256-byte bank row
  static DEV int off(int r, int u) {               // swizzled byte offset of unit u of row r
    return r * RB + ((u ^ ((r / RPB) & (UPR - 1))) << 4);
  }
};

template <typename T>
DEV typename Tr<T>::frag read_frag(const char* base, int r, int ks, int h) {
  typedef Layout<T> L;
  if constexpr (sizeof(T) == 2) {
    const int u = 2 * ks + h;
    uint4 v = *reinterpret_cast<const uint4*>(base + L::off(r, u));
    return __builtin_bit_cast(bf16x8, v);
  } else {
    const int u = 4 * ks + 2 * h;
    uint4 v0 = *reinterpret_cast<const uint4*>(base + L::off(r, u));
    uint4 v1 = *reinterpret_cast<const uint4*>(base + L::off(r, u + 1));
    f32x4 a = __builtin_bit_cast(f32x4, v0), b = __builtin_bit_cast(f32x4, v1);
    f32x8 f;
    f[0] = a[0]; f[1] = a[1]; f[2] = a[2]; f[3] = a[3];
    f[4] = b[0]; f[5] = b[1]; f[6] = b[2]; f[7] = b[3];
    return f;
  }
}

template <typename T, int WM, int WN, int TM, int TN>
__global__ __launch_bounds__(256) void conv_rows_kernel(const ConvArgs a) {
  typedef Layout<T> L;
  constexpr int BM = WM * TM * 32;
  constexpr int BN = WN * TN * 32;
  constexpr int VEC = 16 / sizeof(T);
  constexpr int A_UNITS = BM * L::UPR / 256;  // 16B units per thread for the A tile
  constexpr int B_UNITS = (BN * L::UPR + 255) / 256;
  constexpr int A_BYTES = BM * L::RB;
  constexpr int B_BYTES = BN * L::RB;
  static_assert(A_UNITS >= 1, "tile too small");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  auto sA = [&](int b) -> char* { return smem + b * A_BYTES; };
  auto sB = [&](int b) -> char* { return smem + 2 * A_BYTES + b * B_BYTES; };

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const long M = (long)a.N * a.T_out * a.V;
  const long m0 = (long)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;

  const T* __restrict__ in = reinterpret_cast<const T*>(a.in);
  const T* __restrict__ wp = reinterpret_cast<const T*>(a.w);

  // Per-thread A rows (fixed for the block): decompose once.
  int a_row[A_UNITS], a_u[A_UNITS], a_n[A_UNITS], a_t[A_UNITS], a_v[A_UNITS];
  bool a_ok[A_UNITS];
#pragma unroll
  for (int i = 0; i < A_UNITS; ++i) {
    const int id = tid + i * 256;
    a_row[i] = id / L::UPR;
    a_u[i] = id % L::UPR;
    const long m = m0 + a_row[i];
    a_ok[i] = m < M;
    const long mm = a_ok[i] ? m : 0;
    a_v[i] = (int)(mm % a.V);
    const long nt = mm / a.V;
    a_t[i] = (int)(nt % a.T_out);
    a_n[i] = (int)(nt / a.T_out);
  }

  const bool vec_ok = (a.in_ld % VEC) == 0;
  const int nchunks = a.Cin_pad / KC;
  const int NIT = nchunks * a.Kt;

  uint4 ra[A_UNITS];
  uint4 rb[B_UNITS];
  int rsrc_t[A_UNITS];  // t_in per unit for the prologue (LN stats), -1 = invalid

  auto load = [&](int it) {
    const int chunk = it / a.Kt;
    const int dt = it % a.Kt;
#pragma unroll
    for (int i = 0; i < A_UNITS; ++i) {
      int t_in;
      bool ok = a_ok[i];
      if (!a.trans) {
        t_in = a_t[i] * a.stride + dt - a.pad;
      } else {
        const int num = a_t[i] + a.pad - dt;
        t_in = num >= 0 ? num / a.stride : -1;
        ok = ok && num >= 0 && (num % a.stride) == 0;
      }
      ok = ok && t_in >= 0 && t_in < a.T_in;
      const int ci = chunk * KC + a_u[i] * VEC;
      ok = ok && ci < a.Cin;
      rsrc_t[i] = ok ? t_in : -1;
      if (ok) {
        const long src = ((long)a_n[i] * a.T_in + t_in) * a.V + a_v[i];
        const T* p = in + src * a.in_ld + ci;
        if (vec_ok && ci + VEC <= a.Cin) {
          ra[i] = *reinterpret_cast<const uint4*>(p);
        } else {  // ragged channel tail / unaligned rows: element loads, zero fill
          T tmp[VEC];
#pragma unroll
          for (int j = 0; j < VEC; ++j) tmp[j] = ci + j < a.Cin ? p[j] : Tr<T>::from_f(0.f);
          ra[i] = *reinterpret_cast<const uint4*>(tmp);
        }
      } else {
        ra[i] = make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < B_UNITS; ++i) {
      const int id = tid + i * 256;
      if (id < BN * L::UPR) {
        const int r = id / L::UPR, u = id % L::UPR;
        const long off = ((long)dt * a.Cout_pad + n0 + r) * a.Cin_pad + chunk * KC + u * VEC;
        rb[i] = *reinterpret_cast<const uint4*>(wp + off);
      }
    }
  };

  auto store = [&](int it, int buf) {
    const int chunk = it / a.Kt;
#pragma unroll
    for (int i = 0; i < A_UNITS; ++i) {
      uint4 v = ra[i];
      if (a.pro != 0 && rsrc_t[i] >= 0) {
        float f[VEC];
        unpack16(v, f, (T*)nullptr);
        const int ci = chunk * KC + a_u[i] * VEC;
        if (a.pro == 1) {
#pragma unroll
          for (int j = 0; j < VEC; ++j) f[j] = fmaxf(f[j] * a.pro_a[ci + j] + a.pro_b[ci + j], 0.f);
        } else {
          const float2 st = reinterpret_cast<const float2*>(a.pro_stats)[(long)a_n[i] * a.T_in + rsrc_t[i]];
#pragma unroll
          for (int j = 0; j < VEC; ++j) {
            const int g = (ci + j) * a.V + a_v[i];
            f[j] = fmaxf((f[j] - st.x) * st.y * a.pro_a[g] + a.pro_b[g], 0.f);
          }
        }
        v = pack16(f, (T*)nullptr);
      }
      *reinterpret_cast<uint4*>(sA(buf) + L::off(a_row[i], a_u[i])) = v;
    }
#pragma unroll
    for (int i = 0; i < B_UNITS; ++i) {
      const int id = tid + i * 256;
      if (id < BN * L::UPR) {
        const int r = id / L::UPR, u = id % L::UPR;
        *reinterpret_cast<uint4*>(sB(buf) + L::off(r, u)) = rb[i];
      }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  load(0);
  store(0, 0);
  __syncthreads();
  int cur = 0;
  const int lr = lane & 31, lh = lane >> 5;
  for (int it = 0; it < NIT; ++it) {
    const bool more = it + 1 < NIT;
    if (more) load(it + 1);
#pragma unroll
    for (int ks = 0; ks < KC / 16; ++ks) {
      typename Tr<T>::frag fa[TM], fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[i] = read_frag<T>(sA(cur), (wm * TM + i) * 32 + lr, ks, lh);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[j] = read_frag<T>(sB(cur), (wn * TN + j) * 32 + lr, ks, lh);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) Tr<T>::mma(acc[i][j], fa[i], fb[j]);
    }
    if (more) store(it + 1, cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  // ---------------------------------------------------------------- epilogue
  T* __restrict__ out = reinterpret_cast<T*>(a.out);
  Welford ws[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + (wn * TN + j) * 32 + lr;
    const bool cok = col < a.Cout;
    float b1 = (a.bias_mode == 1 && cok) ? a.bias[col] : 0.f;
    float s = 0.f, cnt = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long m = m0 + (wm * TM + i) * 32 + acc_row(r, lane);
        float v = acc[i][j][r] + b1;
        if (a.bias_mode >= 2 && cok && m < M) {
          long bi = (m % a.V);
          if (a.bias_mode == 3) bi += (m / ((long)a.T_out * a.V)) * a.V;  // per-sample [N][V][Cout]
          v += a.bias[bi * a.Cout + col];
        }
        if (cok && m < M) {
          T* p = out + m * a.out_ld + col;
          if (a.accumulate) v += Tr<T>::to_f(*p);
          *p = Tr<T>::from_f(v);
          s += v;
          cnt += 1.f;
        }
        acc[i][j][r] = v;
      }
    }
    Welford w;
    w.n = cnt;
    w.mean = cnt > 0.f ? s / cnt : 0.f;
    float m2 = 0.f;
    if (a.stats) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const long m = m0 + (wm * TM + i) * 32 + acc_row(r, lane);
          const float d = acc[i][j][r] - w.mean;
          if (cok && m < M) m2 += d * d;
        }
    }
    w.m2 = m2;
    ws[j] = w;
  }
  if (a.stats) {
    // lanes l and l^32 hold the same column: merge, then merge across the WM waves via LDS.
    __syncthreads();
    float4* red = reinterpret_cast<float4*>(smem);  // [WM][BN]
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      Welford o;
      o.n = __shfl_xor(ws[j].n, 32);
      o.mean = __shfl_xor(ws[j].mean, 32);
      o.m2 = __shfl_xor(ws[j].m2, 32);
      Welford w = welford_merge(ws[j], o);
      if (lh == 0) red[wm * BN + (wn * TN + j) * 32 + lr] = make_float4(w.n, w.mean, w.m2, 0.f);
    }
    __syncthreads();
    for (int c = tid; c < BN; c += 256) {
      float4 f = red[c];
      Welford w = {f.x, f.y, f.z};
      for (int k = 1; k < WM; ++k) {
        float4 g = red[k * BN + c];
        w = welford_merge(w, Welford{g.x, g.y, g.z});
      }
      if (n0 + c < a.Cout_pad)
        reinterpret_cast<float4*>(a.stats)[(long)blockIdx.x * a.Cout_pad + n0 + c] = make_float4(w.n, w.mean, w.m2, 0.f);
    }
  }
}

template <typename T, int WM, int WN, int TM, int TN>
int launch_conv(const ConvArgs& a, hipStream_t s) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  const long M = (long)a.N * a.T_out * a.V;
  dim3 grid((unsigned)((M + BM - 1) / BM), (unsigned)(a.Cout_pad / BN));
  const size_t lds = 2 * (BM + BN) * KC * sizeof(T);
  const size_t red = (a.stats ? (size_t)WM * BN * 16 : 0);
  const size_t bytes = lds > red ? lds : red;
  if (stgcn_lds_attr((const void*)conv_rows_kernel<T, WM, WN, TM, TN>, 160 * 1024, s)) return STGCN_EHIP;
  hipLaunchKernelGGL((conv_rows_kernel<T, WM, WN, TM, TN>), grid, dim3(256), bytes, s, a);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

template <typename T>
__global__ void pack_weight_kernel(const float* __restrict__ src, long s0, long s1, long s2, int Co, int Ci, int cp,
                                   int kp, long total, T* __restrict__ dst, T* __restrict__ dst_frag) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < total) pack_weight_elem<T>(src, s0, s1, s2, Co, Ci, cp, kp, i, dst, dst_frag);
}

}  // namespace

int pack_weight_launch(const float* src, long s0, long s1, long s2, int Kt, int Co, int Ci, void* dst, int cp, int kp,
                       int dtype, hipStream_t s, void* dst_frag) {
  const long total = (long)Kt * cp * kp / 8;  // threads: 8 consecutive ci each
  const unsigned blocks = (unsigned)((total + 255) / 256);
  if (kp % 8 || (dst_frag && (cp % 32 || kp % 16))) return STGCN_EBADSHAPE;
  if (dtype == 1)
    hipLaunchKernelGGL(pack_weight_kernel<bf16>, dim3(blocks), dim3(256), 0, s, src, s0, s1, s2, Co, Ci, cp, kp, total,
                       (bf16*)dst, (bf16*)dst_frag);
  else
    hipLaunchKernelGGL(pack_weight_kernel<float>, dim3(blocks), dim3(256), 0, s, src, s0, s1, s2, Co, Ci, cp, kp,
                       total, (float*)dst, (float*)dst_frag);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

// Column tile = 64 for Cout <= 64, 128 otherwise; weights are packed to a multiple of it.
int conv_rows_bn_tile(int cout) { return cout <= 64 ? 64 : 128; }
// upper bound over both kernels (smallest row tile = 128); unused partial slots must be zeroed
long conv_rows_num_row_blocks(long M, int cout) { (void)cout; return (M + 127) / 128; }

int conv_tile_launch(const ConvArgs& a, int dtype, hipStream_t s);

int conv_rows_launch(const ConvArgs& a, int dtype, hipStream_t s) {
  {  // frame-tiled kernels (conv_tile.hip and the kernels it dispatches to) for the shapes they cover
    const int r = conv_tile_launch(a, dtype, s);
    if (r >= 0) return r;
  }
  const int bn = conv_rows_bn_tile(a.Cout);
  if (a.Cout_pad % bn || a.Cin_pad % KC) return STGCN_EBADSHAPE;
  if (dtype == 1) {
    return bn == 64 ? launch_conv<bf16, 4, 1, 2, 2>(a, s) : launch_conv<bf16, 2, 2, 2, 2>(a, s);
  } else {
    return bn == 64 ? launch_conv<float, 4, 1, 2, 2>(a, s) : launch_conv<float, 2, 2, 2, 2>(a, s);
  }
}
