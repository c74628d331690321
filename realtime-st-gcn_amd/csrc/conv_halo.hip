// Halo implicit-GEMM for stride-1 (Kt x 1) row convolutions (temporal conv fwd + its data
// gradient, and all 1x1 convs), MFMA on gfx950.
//
// Same contract as conv_rows.hip (stgcn_conv_desc) restricted to stride == 1.  For stride 1 the
// input row of output row m and tap dt is the flattened row m + o(dt)*V, o(dt) = dt - pad (fwd) or
// pad - dt (trans).  So instead of re-gathering a BM-row tile per tap (conv_rows.hip), each block
// stages ONE halo tile of BM + 2*pad*V input rows per K-chunk (prologue BN/LN+ReLU applied once per
// element) and all Kt taps read it at a row offset.  Rows whose tap falls outside the sequence (or
// into the neighbouring sample) are zeroed per MFMA fragment (one condition per lane and tap).
//
// Block: WAVES x 64 threads; wave w owns output rows [64w, 64w+64) x all BN columns (2 x BN/32 tiles
// of 32x32).  K loop over chunks of KC input channels; A halo + B (all taps) double-buffered in LDS,
// next chunk prefetched into registers while the current chunk's Kt*KC/16*2*BN/32 MFMAs run.
#include "common.h"
#include "../../include/stgcn_amd.h"

namespace {

template <typename T, int KC>
struct HLayout {
  static constexpr int RB = KC * sizeof(T);                  // bytes per LDS row
  static constexpr int UPR = RB / 16;                        // 16-B units per row
  static constexpr int RPB = (256 / RB) > 0 ? 256 / RB : 1;  // rows per 256-B bank row
  static DEV int off(int r, int u) { return r * RB + ((u ^ ((r / RPB) & (UPR - 1))) << 4); }
};

template <typename T, int KC>
DEV typename Tr<T>::frag hread(const char* base, int r, int ks, int h) {
  typedef HLayout<T, KC> L;
  if constexpr (sizeof(T) == 2) {
    return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(base + L::off(r, 2 * ks + h)));
  } else {
    const int u = 4 * ks + 2 * h;
    const f32x4 a = __builtin_bit_cast(f32x4, *reinterpret_cast<const uint4*>(base + L::off(r, u)));
    const f32x4 b = __builtin_bit_cast(f32x4, *reinterpret_cast<const uint4*>(base + L::off(r, u + 1)));
    f32x8 f;
    f[0] = a[0]; f[1] = a[1]; f[2] = a[2]; f[3] = a[3];
    f[4] = b[0]; f[5] = b[1]; f[6] = b[2]; f[7] = b[3];
    return f;
  }
}

// 16-byte LDS-DMA (global_load_lds_dwordx4): lane l writes lds_base + 16*l (device-only builtin)
DEV void glds16(const void* src, char* lds_base) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
#endif
}

template <typename T>
DEV typename Tr<T>::frag zero_if(typename Tr<T>::frag f, bool ok) {
  if constexpr (sizeof(T) == 2) {
    uint4 u = __builtin_bit_cast(uint4, f);
    u.x = ok ? u.x : 0u; u.y = ok ? u.y : 0u; u.z = ok ? u.z : 0u; u.w = ok ? u.w : 0u;
    return __builtin_bit_cast(bf16x8, u);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = ok ? f[j] : 0.f;
    return f;
  }
}

template <typename T, int BN, int WAVES, int KC, int KT>
__global__ __launch_bounds__(WAVES * 64) void conv_halo_kernel(const stgcn_conv_desc a) {
  typedef HLayout<T, KC> L;
  constexpr int NT = WAVES * 64;
  constexpr int BM = WAVES * 64;
  constexpr int TM = 2, TN = BN / 32;
  constexpr int VEC = 16 / sizeof(T);
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int V = a.V;
  const int pad = a.pad;
  const int hs = pad * V;                 // halo rows on each side
  const int HR = BM + 2 * hs;             // halo tile rows
  const int A_BYTES = ((HR * L::RB) + 1023) & ~1023;
  const int B_BYTES = KT * BN * L::RB;
  auto sA = [&](int b) -> char* { return smem + b * (A_BYTES + B_BYTES); };
  auto sB = [&](int b) -> char* { return smem + b * (A_BYTES + B_BYTES) + A_BYTES; };

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long M = (long)a.N * a.T_out * V;           // == input rows (stride 1)
  const long m0 = (long)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const T* __restrict__ in = reinterpret_cast<const T*>(a.in);
  const T* __restrict__ wp = reinterpret_cast<const T*>(a.w);
  const bool vec_ok = (a.in_ld % VEC) == 0;

  // ---- per-lane output-row info for the fragment validity test
  const int lr = lane & 31, lh = lane >> 5;
  int trow[TM];
  bool rok[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const long m = m0 + wave * 64 + i * 32 + lr;
    rok[i] = m < M;
    trow[i] = (int)((m / V) % a.T_out);
  }

  // ---- staging assignment: A halo units (HR * UPR), B units (KT * BN * UPR)
  const int a_units = HR * L::UPR;
  constexpr int B_PIECES = KT * BN * L::RB / 1024;        // 1-KiB LDS-DMA pieces per chunk
  static_assert((KT * BN * L::RB) % 1024 == 0, "B tile must be whole 1-KiB pieces");
  // halo rows HR <= BM + (KT-1)*32 for V <= 32
  constexpr int A_MAX = ((BM + (KT - 1) * 32) * L::UPR + NT - 1) / NT;
  uint4 ra[A_MAX];
  int a_src[A_MAX];         // input row index (or -1); rows < 2^31
#pragma unroll
  for (int i = 0; i < A_MAX; ++i) {
    const int id = tid + i * NT;
    a_src[i] = -1;
    if (id < a_units) {
      const long mi = m0 - hs + id / L::UPR;
      if (mi >= 0 && mi < M) a_src[i] = (int)mi;
    }
  }

  const int nchunks = a.Cin_pad / KC;

  auto load = [&](int c, int buf) {
#pragma unroll
    for (int i = 0; i < A_MAX; ++i) {
      const int id = tid + i * NT;
      ra[i] = make_uint4(0, 0, 0, 0);
      if (id < a_units && a_src[i] >= 0) {
        const int ci = c * KC + (id % L::UPR) * VEC;
        if (ci < a.Cin) {
          const T* p = in + (long)a_src[i] * a.in_ld + ci;
          if (vec_ok && ci + VEC <= a.Cin) {
            ra[i] = *reinterpret_cast<const uint4*>(p);
          } else {
            float f[VEC];
#pragma unroll
            for (int j = 0; j < VEC; ++j) f[j] = ci + j < a.Cin ? Tr<T>::to_f(p[j]) : 0.f;
            ra[i] = pack16(f, (T*)nullptr);
          }
        }
      }
    }
    // B (all taps of this chunk) straight to LDS by LDS-DMA: lane-linear destination, XOR swizzle
    // applied on the SOURCE unit so that hread's swizzled read finds logical unit u.
    char* B_ = sB(buf);
    for (int piece = wave; piece < B_PIECES; piece += WAVES) {
      const int byte = piece * 1024 + lane * 16;
      const int row = byte / L::RB, pu = (byte % L::RB) >> 4;
      const int u = pu ^ ((row / L::RPB) & (L::UPR - 1));
      const int dt = row / BN, col = row % BN;
      const T* src = wp + ((long)dt * a.Cout_pad + n0 + col) * a.Cin_pad + c * KC + u * VEC;
      glds16(src, B_ + piece * 1024);
    }
  };

  auto store = [&](int c, int buf) {
    char* A_ = sA(buf);
#pragma unroll
    for (int i = 0; i < A_MAX; ++i) {
      const int id = tid + i * NT;
      if (id < a_units) {
        uint4 v = ra[i];
        if (a.pro != 0 && a_src[i] >= 0) {
          float f[VEC];
          unpack16(v, f, (T*)nullptr);
          const int ci = c * KC + (id % L::UPR) * VEC;
          if (a.pro == 1) {
#pragma unroll
            for (int j = 0; j < VEC; ++j)
              f[j] = ci + j < a.Cin ? fmaxf(f[j] * a.pro_a[ci + j] + a.pro_b[ci + j], 0.f) : 0.f;
          } else {
            const float2 st = reinterpret_cast<const float2*>(a.pro_stats)[a_src[i] / V];
            const int av = a_src[i] % V;
#pragma unroll
            for (int j = 0; j < VEC; ++j) {
              const int g = (ci + j) * V + av;
              f[j] = ci + j < a.Cin ? fmaxf((f[j] - st.x) * st.y * a.pro_a[g] + a.pro_b[g], 0.f) : 0.f;
            }
          }
          v = pack16(f, (T*)nullptr);
        }
        *reinterpret_cast<uint4*>(A_ + L::off(id / L::UPR, id % L::UPR)) = v;
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

  load(0, 0);
  store(0, 0);
  __syncthreads();
  int cur = 0;
  for (int c = 0; c < nchunks; ++c) {
    const bool more = c + 1 < nchunks;
    if (more) load(c + 1, cur ^ 1);
    const char* A_ = sA(cur);
    const char* B_ = sB(cur);
#pragma unroll 1
    for (int dt = 0; dt < KT; ++dt) {
      const int o = a.trans ? pad - dt : dt - pad;   // input row offset in frames
      bool ok[TM];
      int arow[TM];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int tin = trow[i] + o;
        ok[i] = rok[i] && tin >= 0 && tin < a.T_in;
        arow[i] = hs + wave * 64 + i * 32 + lr + o * V;
      }
#pragma unroll
      for (int ks = 0; ks < KC / 16; ++ks) {
        typename Tr<T>::frag fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = zero_if<T>(hread<T, KC>(A_, arow[i], ks, lh), ok[i]);
#pragma unroll
        for (int j = 0; j < TN; ++j) fb[j] = hread<T, KC>(B_, dt * BN + j * 32 + lr, ks, lh);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) Tr<T>::mma(acc[i][j], fa[i], fb[j]);
      }
    }
    if (more) store(c + 1, cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  // ---------------------------------------------------------------- epilogue (as conv_rows.hip)
  T* __restrict__ out = reinterpret_cast<T*>(a.out);
  Welford ws[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + j * 32 + lr;
    const bool cok = col < a.Cout;
    const float b1 = (a.bias_mode == 1 && cok) ? a.bias[col] : 0.f;
    float s = 0.f, cnt = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long m = m0 + wave * 64 + i * 32 + acc_row(r, lane);
        float v = acc[i][j][r] + b1;
        if (a.bias_mode >= 2 && cok && m < M) {
          long bi = m % V;
          if (a.bias_mode == 3) bi += (m / ((long)a.T_out * V)) * V;
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
          const long m = m0 + wave * 64 + i * 32 + acc_row(r, lane);
          const float d = acc[i][j][r] - w.mean;
          if (cok && m < M) m2 += d * d;
        }
    }
    w.m2 = m2;
    ws[j] = w;
  }
  if (a.stats) {
    __syncthreads();
    float4* red = reinterpret_cast<float4*>(smem);  // [WAVES][BN]
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      Welford o;
      o.n = __shfl_xor(ws[j].n, 32);
      o.mean = __shfl_xor(ws[j].mean, 32);
      o.m2 = __shfl_xor(ws[j].m2, 32);
      const Welford w = welford_merge(ws[j], o);
      if (lh == 0) red[wave * BN + j * 32 + lr] = make_float4(w.n, w.mean, w.m2, 0.f);
    }
    __syncthreads();
    for (int c = tid; c < BN; c += NT) {
      const float4 f = red[c];
      Welford w = {f.x, f.y, f.z};
      for (int k = 1; k < WAVES; ++k) {
        const float4 g = red[k * BN + c];
        w = welford_merge(w, Welford{g.x, g.y, g.z});
      }
      if (n0 + c < a.Cout_pad)
        reinterpret_cast<float4*>(a.stats)[(long)blockIdx.x * a.Cout_pad + n0 + c] =
            make_float4(w.n, w.mean, w.m2, 0.f);
    }
  }
}

template <typename T, int BN, int WAVES, int KC, int KT>
int launch_halo(const stgcn_conv_desc& a, hipStream_t s) {
  typedef HLayout<T, KC> L;
  constexpr int BM = WAVES * 64;
  const int hs = a.pad * a.V;
  const int HR = BM + 2 * hs;
  if (a.V > 32) return -1;
  (void)HR;
  const long M = (long)a.N * a.T_out * a.V;
  const int A_BYTES = ((HR * L::RB) + 1023) & ~1023;
  const int B_BYTES = KT * BN * L::RB;
  size_t lds = 2 * (size_t)(A_BYTES + B_BYTES);
  const size_t red = a.stats ? (size_t)WAVES * BN * 16 : 0;
  if (red > lds) lds = red;
  if (lds > 160 * 1024) return -1;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv_halo_kernel<T, BN, WAVES, KC, KT>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  dim3 grid((unsigned)((M + BM - 1) / BM), (unsigned)(a.Cout_pad / BN));
  hipLaunchKernelGGL((conv_halo_kernel<T, BN, WAVES, KC, KT>), grid, dim3(WAVES * 64), lds, s, a);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

}  // namespace

// Row blocks of the halo kernel (first dim of the BN partial-stat buffer)
long conv_halo_row_blocks(long M, int dtype) { (void)dtype; return (M + 255) / 256; }

// returns -1 when the shape is not handled by the halo kernel (caller falls back to conv_rows)
int conv_halo_launch(const stgcn_conv_desc& a, int dtype, hipStream_t s) {
  if (a.stride != 1 || !(a.Kt == 1 || a.Kt == 9) || a.T_in != a.T_out || a.pad != (a.Kt - 1) / 2) return -1;
  if (a.Cout_pad % 64) return -1;
  if (dtype == 1) {
    const bool wide = a.Cout_pad % 128 == 0 && a.Cout > 64;
    if (a.Kt == 9) {
      if (a.Cin_pad % 16) return -1;
      return wide ? launch_halo<bf16, 128, 4, 16, 9>(a, s) : launch_halo<bf16, 64, 4, 16, 9>(a, s);
    }
    if (a.Cin_pad % 32) return -1;
    return wide ? launch_halo<bf16, 128, 4, 32, 1>(a, s) : launch_halo<bf16, 64, 4, 32, 1>(a, s);
  }
  if (a.Cin_pad % 16) return -1;
  if (a.Kt == 9) return launch_halo<float, 64, 4, 16, 9>(a, s);
  return launch_halo<float, 64, 4, 16, 1>(a, s);
}
