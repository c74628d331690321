// Graph convolution of ST-GCN (ConvTemporalGraphical, models/utils/tgcn.py:58-79) as a
// joint-gathered GEMM, for a graph shared by the batch.
//
// The reference computes  y = conv1x1(x) (P*Cout channels) ; g = einsum('nkctv,kvw->nctw', y, A).
// Writing W_p = conv weight rows [p*Cout, (p+1)*Cout) and S(w) = {v : A_p[v][w] != 0 for some p}
// (the joints feeding output joint w; <= 5 for the skeleton graphs), the same thing is
//
//   g[(i,w)][co] = sum_{j < |S(w)|} sum_ci x[(i, S(w)_j)][ci] * Weff[w][j][co][ci] + bias2d[w][co]
//   Weff[w][j][co][ci] = sum_p A_p[S(w)_j][w] * W_p[co][ci]            (i = n*T + t)
//
// i.e. for every output joint w a GEMM over the frame rows i whose K axis gathers the |S(w)|
// neighbour rows of the same frame.  Total MFMA work = sum_w |S(w)| * Cin * Cout per frame
// (73 * Cin * Cout for the 25-joint graphs, vs P*V = 75 for the A-first form) and no A-mixed
// intermediate ever touches HBM: the old path wrote and re-read an M x P*Cin tensor three times
// (forward, data grad, weight grad).  The data gradient is the same kernel on dg with the
// transposed effective weights  WeffT[v][j][ci][co] = sum_p A_p[v][R(v)_j] W_p[co][ci]  over the
// reverse lists R(v) = {w : v in S(w)}; the weight/adjacency gradients come from
//   dWeff[w][j][co][ci] = sum_i dg[(i,w)][co] * x[(i, S(w)_j)][ci]          (gconv_wgrad)
//   dW_p[co][ci] = sum_{w,j} A_p[S(w)_j][w] dWeff[w][j][co][ci],
//   dA_p[S(w)_j][w] = sum_{co,ci} W_p[co][ci] dWeff[w][j][co][ci]            (gconv_wgrad_finish)
//
// Kernel layout follows conv_tile.hip (flat mode): block = (row tile of BM frames, joint a, column
// tile); A rows staged through registers into padded LDS rows, B (packed Weff) by LDS-DMA with the
// XOR swizzle on the source, fragment double-buffering, BN partial statistics in the epilogue.
#include "common.h"
#include "pack.h"
#include <stdlib.h>
#include <utility>
#include "../../include/stgcn_amd.h"

#ifndef GCONV_NSTG_N
#define GCONV_NSTG_N 2
#endif
#ifndef GCONV_NSTG_M
#define GCONV_NSTG_M 2
#endif
#ifndef GCONV_NSTG_W
#define GCONV_NSTG_W 2
#endif
// row tiles of the wide DMA forms (A/B build flags): BM = 4 * TM * 32 rows; a taller tile re-reads each joint's
// effective weights (deg x 64-channel chunks x 128 columns) fewer times per launch
#ifndef GCONV_TM_W
#define GCONV_TM_W 2
#endif
#ifndef GCONV_TM_M
#define GCONV_TM_M 1
#endif

namespace {

template <typename T, int KC>
struct GL {
  static constexpr int RB = KC * (int)sizeof(T);
  static constexpr int UPR = RB / 16;
  static constexpr int RPB = RB >= 256 ? 1 : 256 / RB;
  static constexpr int RS = RB + 16;
  static DEV int swz(int row) { return (row / RPB) & (UPR - 1); }
};

DEV void glds16(const void* src, char* lds_base) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
#endif
}

// global -> LDS DMA of 16 B per lane at a wave-uniform LDS offset, through asm so the compiler inserts no
// alias-driven vmcnt drains (the DMA K loop counts its own); m0 saved / restored
DEV void gdma16(const void* src, unsigned lds_off) {
  unsigned saved;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(saved) : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds_off)) : "memory");
}
DEV unsigned glds_off(const void* p) { return (unsigned)(size_t)(const __attribute__((address_space(3))) char*)p; }
// s_waitcnt vmcnt(n) for the counts the DMA K loop uses (n = steps in flight x instructions per step)
DEV void gwait_vm(int n) {
  switch (n) {
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

template <typename T>
DEV typename Tr<T>::frag frag2(const char* p0, const char* p1) {
  if constexpr (sizeof(T) == 2) {
    (void)p1;
    return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(p0));
  } else {
    const f32x4 a = __builtin_bit_cast(f32x4, *reinterpret_cast<const uint4*>(p0));
    const f32x4 b = __builtin_bit_cast(f32x4, *reinterpret_cast<const uint4*>(p1));
    f32x8 f;
    f[0] = a[0]; f[1] = a[1]; f[2] = a[2]; f[3] = a[3];
    f[4] = b[0]; f[5] = b[1]; f[6] = b[2]; f[7] = b[3];
    return f;
  }
}

struct GGeom {
  int ntile;  // row tiles
  int ncol;   // column tiles
  int nblk;
};

// ------------------------------------------------------------------ gather GEMM (fwd and data grad)
// ACCV: stores (and accumulate, out +=) through the vectorised LDS-scratch epilogue; a separate instantiation so
// the plain-store kernel keeps its register budget (<= 128 VGPRs: 2 blocks per CU)
// NSTG > 0 (bf16, KC = 64): the K loop DMAs both operands (gathered x rows and the effective weights,
// XOR-swizzled 128-B rows) into an NSTG-deep LDS ring, NSTG - 1 K steps ahead, with counted vmcnt waits
// (every wave issues the same number of DMA instructions per step) and one LDS-only barrier per step;
// NSTG = 0: rows staged through registers, double-buffered.
template <typename T, int WM, int WN, int TM, int TN, int KC, bool ACCV, int NSTG = 0>
__global__ __launch_bounds__(WM * WN * 64, (NSTG && (WM * TM + WN * TN) * 32 * 128 * NSTG > 80 * 1024) ? 1 : 2) void gconv_kernel(const stgcn_gconv_desc a, const GGeom g) {
  typedef GL<T, KC> L;
  constexpr int NW = WM * WN, NT = NW * 64;
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  constexpr int VEC = 16 / (int)sizeof(T);
  constexpr int KS = KC / 16;
  constexpr int A_UNITS = BM * L::UPR / NT;
  constexpr int A_BYTES = BM * L::RS;
  constexpr int B_BYTES = BN * L::RB;
  constexpr int B_PIECES = (B_BYTES + 1023) / 1024;
  constexpr int STAGE = ((A_BYTES + B_BYTES) + 1023) & ~1023;
  static_assert(BM * L::UPR % NT == 0, "A units");
  static_assert(B_BYTES % 1024 == 0, "B pieces");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int lr = lane & 31, lh = lane >> 5;
  const int V = a.V;

  // XCD-aware order: consecutive ids (column tile fastest, then joint) share the row tile's x rows
  int wg;
  {
    const int id = blockIdx.x, x = id & 7, q = g.nblk >> 3, r = g.nblk & 7;
    wg = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (id >> 3);
  }
  const int ct = wg % g.ncol;
  const int jt = (wg / g.ncol) % V;  // output joint
  const int it = wg / (g.ncol * V);
  const int n0 = ct * BN;
  const int i0 = it * BM;
  const int rows_valid = min(BM, a.NT - i0);
  const int deg = a.deg[jt];

  const T* __restrict__ in = reinterpret_cast<const T*>(a.in);
  const T* __restrict__ wp = reinterpret_cast<const T*>(a.w);
  const int ucol = tid % L::UPR;
  long a_row[A_UNITS];  // element offset of frame row (i, joint 0) ; -1 = zero row
  int a_lds[A_UNITS];
#pragma unroll
  for (int u = 0; u < A_UNITS; ++u) {
    const int row = (tid + u * NT) / L::UPR;
    a_lds[u] = row * L::RS + ucol * 16;
    a_row[u] = row < rows_valid ? (long)(i0 + row) * V * a.in_ld + ucol * VEC : -1;
  }
  const bool fast_ld = (a.in_ld % VEC) == 0 && (a.Cin % KC) == 0;

  int a_off[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) a_off[i] = ((wm * TM + i) * 32 + lr) * L::RS + lh * 16 * (int)(sizeof(T) / 2);
  int b_off[KS][2];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int f = L::swz(lr);
    if constexpr (sizeof(T) == 2) {
      b_off[ks][0] = lr * L::RB + (((2 * ks + lh) ^ f) << 4);
      b_off[ks][1] = b_off[ks][0];
    } else {
      b_off[ks][0] = lr * L::RB + (((4 * ks + 2 * lh) ^ f) << 4);
      b_off[ks][1] = lr * L::RB + (((4 * ks + 2 * lh + 1) ^ f) << 4);
    }
  }

  const int nch = a.Cin_pad / KC;
  const int nk = deg * nch;  // K chunks: (neighbour j, channel chunk c)
  uint4 ra[A_UNITS];

  auto load = [&](int k, int buf) {
    const int j = k / nch, c = k - j * nch;
    const int src = a.nbr[jt * a.J + j];
    const long joff = (long)src * a.in_ld + c * KC;
    const int ci = c * KC + ucol * VEC;
#pragma unroll
    for (int u = 0; u < A_UNITS; ++u) {
      ra[u] = make_uint4(0, 0, 0, 0);
      if (a_row[u] >= 0) {
        const T* p = in + a_row[u] + joff;
        if (fast_ld) {
          ra[u] = *reinterpret_cast<const uint4*>(p);
        } else if (ci < a.Cin) {
          float f[VEC];
#pragma unroll
          for (int e = 0; e < VEC; ++e) f[e] = ci + e < a.Cin ? Tr<T>::to_f(p[e]) : 0.f;
          ra[u] = pack16(f, (T*)nullptr);
        }
      }
    }
    char* B_ = smem + buf * STAGE + A_BYTES;
    const T* wsrc = wp + ((long)(jt * a.J + j) * a.Cout_pad + n0) * a.Cin_pad + c * KC;
#pragma unroll
    for (int kk = 0; kk < (B_PIECES + NW - 1) / NW; ++kk) {
      const int piece = wave + kk * NW;
      if (piece < B_PIECES) {
        const int byte = piece * 1024 + lane * 16;
        const int br = byte / L::RB, pu = (byte % L::RB) >> 4;
        glds16(wsrc + (long)br * a.Cin_pad + (pu ^ L::swz(br)) * VEC, B_ + piece * 1024);
      }
    }
  };
  auto store = [&](int buf) {
    char* A_ = smem + buf * STAGE;
#pragma unroll
    for (int u = 0; u < A_UNITS; ++u) *reinterpret_cast<uint4*>(A_ + a_lds[u]) = ra[u];
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  typedef typename Tr<T>::frag Frag;
  if constexpr (NSTG > 0) {
    static_assert(sizeof(T) == 2 && KC == 64, "DMA K loop: bf16, 64-channel chunks");
    constexpr int RBD = 128, A_B = BM * RBD, STG = A_B + BN * RBD;
    constexpr int AI = BM / 8 / NW, BI = BN / 8 / NW, OPS = AI + BI;  // DMA instructions per wave and step
    static_assert(BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "DMA rows");
    int* const snbr = reinterpret_cast<int*>(smem + NSTG * STG);  // this joint's neighbour list
    if (tid < a.J) snbr[tid] = a.nbr[jt * a.J + tid];
    __syncthreads();
    // lane -> (row rr of the instruction's 8 rows, 16-B slot); the slot holds unit slot ^ swz(row)
    const int rr = lane >> 3, slot = lane & 7;
    long a_src[AI];
    int b_src[BI];
#pragma unroll
    for (int q = 0; q < AI; ++q) {
      const int r = (wave * AI + q) * 8 + rr;
      const int rc = min(r, max(rows_valid, 1) - 1);  // rows past the tile's end read a valid row (discarded)
      a_src[q] = (long)(i0 + rc) * V * a.in_ld + (slot ^ ((r >> 1) & 7)) * 8;
    }
#pragma unroll
    for (int q = 0; q < BI; ++q) {
      const int r = (wave * BI + q) * 8 + rr;
      b_src[q] = (n0 + r) * a.Cin_pad + (slot ^ ((r >> 1) & 7)) * 8;
    }
    auto issue = [&](int k, int stage) {
      const int j = k / nch, c = k - j * nch;
      const long joff = (long)snbr[j] * a.in_ld + c * KC;
      const T* wsrc = wp + (long)(jt * a.J + j) * a.Cout_pad * a.Cin_pad + c * KC;
      char* base = smem + stage * STG;
#pragma unroll
      for (int q = 0; q < AI; ++q) gdma16(in + a_src[q] + joff, glds_off(base + (wave * AI + q) * 1024));
#pragma unroll
      for (int q = 0; q < BI; ++q) gdma16(wsrc + b_src[q], glds_off(base + A_B + (wave * BI + q) * 1024));
    };
#pragma unroll
    for (int sidx = 0; sidx < NSTG - 1; ++sidx)
      if (sidx < nk) issue(sidx, sidx);
    for (int k = 0; k < nk; ++k) {
      const int younger = min(NSTG - 2, nk - 1 - k);  // own DMA steps allowed to stay in flight
      gwait_vm(younger * OPS);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // every wave's DMAs of step k landed
      if (k + NSTG - 1 < nk) issue(k + NSTG - 1, (k + NSTG - 1) % NSTG);  // that stage was read in step k-1
      const char* A_ = smem + (k % NSTG) * STG;
      const char* B_ = A_ + A_B;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        Frag fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int r = (wm * TM + i) * 32 + lr;
          fa[i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(A_ + r * RBD + (((2 * ks + lh) ^ ((r >> 1) & 7)) << 4)));
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int r = (wn * TN + j) * 32 + lr;
          fb[j] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(B_ + r * RBD + (((2 * ks + lh) ^ ((r >> 1) & 7)) << 4)));
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) Tr<T>::mma(acc[i][j], fa[i], fb[j]);
      }
    }
    __syncthreads();  // every wave is done with the ring before the epilogue reuses it
  } else {
  int cur = 0;
  if (nk > 0) {
    load(0, 0);
    store(0);
  }
  __syncthreads();
  for (int k = 0; k < nk; ++k) {
    const bool more = k + 1 < nk;
    if (more) load(k + 1, cur ^ 1);
    const char* A_ = smem + cur * STAGE;
    const char* B_ = A_ + A_BYTES;
    Frag fa[2][TM], fb[2][TN];
    auto rd = [&](int ks, int b) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const char* p = A_ + a_off[i] + ks * 16 * (int)sizeof(T);
        fa[b][i] = frag2<T>(p, p + 16);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const char* p = B_ + ((wn * TN + j) * 32) * L::RB;
        fb[b][j] = frag2<T>(p + b_off[ks][0], p + b_off[ks][1]);
      }
    };
    rd(0, 0);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + 1 < KS) rd(ks + 1, (ks + 1) & 1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) Tr<T>::mma(acc[i][j], fa[ks & 1][i], fb[ks & 1][j]);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (more) store(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }
  }  // NSTG == 0

  // ---------------------------------------------------------------- epilogue
  // bias + BN partials on the fp32 accumulators.  accumulate: the values go through a per-wave LDS
  // scratch (one 32x32 tile at a time) so that every lane read-modify-writes 16-B units of an output
  // row instead of scattered 2/4-byte elements (a dependent load per element before its store).  The main loop's last barrier
  // retired every read of the stage buffers, which the scratch reuses.
  T* __restrict__ out = reinterpret_cast<T*>(a.out);
  const long ldv = (long)a.out_ld * V;  // row stride between consecutive frames of joint jt
  constexpr int SROW = 32 * (int)sizeof(T) + 16;  // padded scratch row (bytes)
  constexpr int UR = 32 * (int)sizeof(T) / 16;     // 16-B units per 32-column row
  char* scratch = smem + wave * 32 * SROW;
  constexpr bool vec_out = ACCV;  // launcher: ACCV when rows are 16-B aligned
  Welford ws[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int c0 = n0 + (wn * TN + j) * 32;
    const int col = c0 + lr;
    const bool cok = col < a.Cout;
    const float b1 = (a.bias && cok) ? a.bias[jt * a.Cout + col] : 0.f;
    float s = 0.f, cnt = 0.f;
    if constexpr (!vec_out) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int lb = (wm * TM + i) * 32 + 4 * lh;
        T* pb = out + ((long)(i0 + lb) * V + jt) * a.out_ld + col;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int ro = (r & 3) + 8 * (r >> 2);
          const bool ok = cok && lb + ro < rows_valid;
          float v = acc[i][j][r] + b1;
          if (ok) {
            T* p = pb + ro * ldv;
            if (a.accumulate) v += Tr<T>::to_f(*p);
            *p = Tr<T>::from_f(v);
            s += v;
            cnt += 1.f;
          }
          acc[i][j][r] = v;
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int rb = (wm * TM + i) * 32;  // tile's first row (frame index within the row tile)
        const int lb = rb + 4 * lh;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int ro = (r & 3) + 8 * (r >> 2);
          const float v = acc[i][j][r] + b1;
          acc[i][j][r] = v;
          if (cok && lb + ro < rows_valid) {
            s += v;
            cnt += 1.f;
          }
          *reinterpret_cast<T*>(scratch + (4 * lh + ro) * SROW + lr * (int)sizeof(T)) = Tr<T>::from_f(v);
        }
        // 32 rows x UR units, lane -> (row, unit): 16-B read-modify-write of the output (wave-private
        // scratch: no block barrier needed)
#pragma unroll
        for (int q = 0; q < 32 * UR / 64; ++q) {
          const int idx = q * 64 + lane, row = idx / UR, u = idx % UR;
          if (rb + row < rows_valid && c0 + u * VEC < a.Cout) {
            T* p = out + ((long)(i0 + rb + row) * V + jt) * a.out_ld + c0 + u * VEC;
            float f[VEC], o[VEC];
            if (a.accumulate) {
              unpack16(*reinterpret_cast<const uint4*>(scratch + row * SROW + u * 16), f, (T*)nullptr);
              unpack16(*reinterpret_cast<const uint4*>(p), o, (T*)nullptr);
#pragma unroll
              for (int e = 0; e < VEC; ++e) f[e] += o[e];
              *reinterpret_cast<uint4*>(p) = pack16(f, (T*)nullptr);
            } else if (sizeof(T) == 2 && a.res) {  // masked residual (launcher: bf16, VEC = 8 = one mask byte)
              const long grow = (long)(i0 + rb + row) * V + jt;
              const int cc = c0 + u * VEC;
              unpack16(*reinterpret_cast<const uint4*>(scratch + row * SROW + u * 16), f, (T*)nullptr);
              unpack16(*reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(a.res) + grow * a.res_ld + cc), o,
                       (T*)nullptr);
              const unsigned mb = reinterpret_cast<const unsigned char*>(a.res_bits)[grow * (a.Cout / 8) + cc / 8];
#pragma unroll
              for (int e = 0; e < VEC; ++e) f[e] += ((mb >> e) & 1u) ? o[e] : 0.f;
              *reinterpret_cast<uint4*>(p) = pack16(f, (T*)nullptr);
            } else {
              *reinterpret_cast<uint4*>(p) = *reinterpret_cast<const uint4*>(scratch + row * SROW + u * 16);
            }
          }
        }
      }
    }
    Welford w;
    w.n = cnt;
    w.mean = cnt > 0.f ? s / cnt : 0.f;
    float m2 = 0.f;
    if (a.stats) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int lb = (wm * TM + i) * 32 + 4 * lh;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float d = acc[i][j][r] - w.mean;
          if (cok && lb + (r & 3) + 8 * (r >> 2) < rows_valid) m2 += d * d;
        }
      }
    }
    w.m2 = m2;
    ws[j] = w;
  }
  if (a.stats) {
    __syncthreads();
    float4* red = reinterpret_cast<float4*>(smem);  // [WM][BN]
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      Welford o;
      o.n = __shfl_xor(ws[j].n, 32);
      o.mean = __shfl_xor(ws[j].mean, 32);
      o.m2 = __shfl_xor(ws[j].m2, 32);
      const Welford w = welford_merge(ws[j], o);
      if (lh == 0) red[wm * BN + (wn * TN + j) * 32 + lr] = make_float4(w.n, w.mean, w.m2, 0.f);
    }
    __syncthreads();
    for (int c = tid; c < BN; c += NT) {
      const float4 f = red[c];
      Welford w = {f.x, f.y, f.z};
      for (int k = 1; k < WM; ++k) {
        const float4 h = red[k * BN + c];
        w = welford_merge(w, Welford{h.x, h.y, h.z});
      }
      if (n0 + c < a.Cout_pad)
        reinterpret_cast<float4*>(a.stats)[((long)it * V + jt) * a.Cout_pad + n0 + c] =
            make_float4(w.n, w.mean, w.m2, 0.f);
    }
  }
}

template <typename T, int WM, int WN, int TM, int TN, int KC, int NSTG = 0>
int launch_gconv(const stgcn_gconv_desc& a, hipStream_t s) {
  constexpr int VEC = 16 / (int)sizeof(T);
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  typedef GL<T, KC> L;
  if (a.Cout_pad % BN || a.Cin_pad % KC) return STGCN_EBADSHAPE;
  if (NSTG && (a.in_ld % VEC || a.Cin != a.Cin_pad || a.J > 64)) return STGCN_EBADSHAPE;
  GGeom g;
  g.ntile = (a.NT + BM - 1) / BM;
  g.ncol = a.Cout_pad / BN;
  const long nblk = (long)g.ntile * a.V * g.ncol;
  if (nblk <= 0 || nblk > 0x7fffffffL) return STGCN_EBADSHAPE;
  g.nblk = (int)nblk;
  const int STAGE = ((BM * L::RS + BN * L::RB) + 1023) & ~1023;
  size_t lds = NSTG ? (size_t)NSTG * (BM + BN) * 128 + 256 : 2 * (size_t)STAGE;
  const size_t red = a.stats ? (size_t)WM * BN * 16 : 0;
  if (red > lds) lds = red;
  if (stgcn_lds_attr((const void*)gconv_kernel<T, WM, WN, TM, TN, KC, false, NSTG>, 160 * 1024, s) ||
      stgcn_lds_attr((const void*)gconv_kernel<T, WM, WN, TM, TN, KC, true, NSTG>, 160 * 1024, s))
    return STGCN_EHIP;
  // 16-B row stores through the LDS scratch whenever rows are 16-B aligned (per-element stores otherwise)
  const bool accv = (a.out_ld % VEC) == 0 && (a.Cout % VEC) == 0;
  if (a.res && (!accv || sizeof(T) != 2 || a.accumulate || !a.res_bits || a.Cout % 8 || a.res_ld % 8))
    return STGCN_EBADSHAPE;  // the masked residual rides on the 16-B bf16 epilogue only
  if (accv)
    hipLaunchKernelGGL((gconv_kernel<T, WM, WN, TM, TN, KC, true, NSTG>), dim3((unsigned)nblk), dim3(WM * WN * 64),
                       lds, s, a, g);
  else
    hipLaunchKernelGGL((gconv_kernel<T, WM, WN, TM, TN, KC, false, NSTG>), dim3((unsigned)nblk), dim3(WM * WN * 64),
                       lds, s, a, g);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

// ------------------------------------------------------------------ effective weights (pack.h)
template <typename T>
__global__ void gconv_weights_kernel(const float* __restrict__ A, const float* __restrict__ W, const int* nbr,
                                     const int* deg, int P, int V, int J, int Cout, int Cin, int trans, T* out,
                                     int R_pad, int C_pad, const float* __restrict__ bconv, float* __restrict__ bias2d) {
  __shared__ float colsum[GW_COLSUM_MAX];
  if (bias2d) gconv_colsum_block(A, nullptr, P, V, colsum);  // block-uniform
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx < (long)V * R_pad * (C_pad / 8))
    gconv_weights_elem<T>(A, nullptr, W, nbr, deg, P, V, J, Cout, Cin, trans, out, R_pad, C_pad, bconv, bias2d, colsum,
                          idx);
}

// ------------------------------------------------------------------ weight gradient (bf16 + fp32)
// dWeff[w][j][co][ci] += sum_i dy[(i,w)][co] * x[(i, nbr[w][j])][ci].  Block = (pair (w,j), 64-co x
// 64-ci block, row range); the 4 waves split the k-steps of each 128-row tile and are summed in LDS
// at the end; per-block partials go to a slab and are reduced deterministically.
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
constexpr int WKM = 128;  // rows per tile
constexpr int WPR = 64;   // bytes per bf16 panel row (32 channels)

DEV bf16x8 trfrag(const char* panel, int row0, int lane) {
  const int i = lane & 15, gq = lane >> 4;
  const int q = i >> 2, p = i & 3, h = gq >> 1;
  const char* a0 = panel + (row0 + 8 * h + q) * WPR + (16 * (gq & 1) + 4 * p) * 2;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 4 * WPR));
  s16x8 v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return __builtin_bit_cast(bf16x8, v);
}

struct WGG {
  int ntile, tpb, R, nco, nci;
  float* slab;     // [R][V*J][Cout][Cin]
  float* rowpart;  // joint-grouped kernel: [R][V][Cout] partial row sums of dy per joint, or NULL
  int zero_unused;  // direct plan (slab = dWeff): also write zeros into the slots j in [deg, J)
  // direct plan, degree-balanced: the joints whose ring is shallow (deg >= W3_SPLIT_DEG) run as two half-row-range
  // blocks that merge in-kernel; part = [V][ngrp][2][J*4096 + 64] half partials, cnt = [V*ngrp] arrival counters
  // (zeroed ahead of every launch)
  float* part;
  unsigned* cnt;
};
constexpr int W3_SPLIT_DEG = 4;  // at 80 KB: ring depth 4 (deg 4) / 3 (deg 5) vs 5 at deg 3 (w3d)

__global__ __launch_bounds__(256, 2) void gconv_wgrad_kernel(const stgcn_gconv_wgrad_desc a, const WGG g) {
  constexpr int PANEL = WKM * WPR;   // one 32-channel panel of a tile
  constexpr int STAGE = 4 * PANEL;   // dy: 2 panels, x: 2 panels
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int V = a.V;
  const int ngrp = g.nco * g.nci;
  const int pair = blockIdx.x / (ngrp * g.R);
  const int rem = blockIdx.x % (ngrp * g.R);
  const int rr = rem / ngrp, grp = rem % ngrp;
  const int w = pair / a.J, j = pair % a.J;
  if (j >= a.deg[w]) return;  // unused (joint, neighbour) slot: block-uniform exit before any barrier
  const int src = a.nbr[pair];
  const int co0 = (grp % g.nco) * 64, ci0 = (grp / g.nco) * 64;
  const int t0 = rr * g.tpb, t1 = min(g.ntile, t0 + g.tpb);

  const bf16* __restrict__ dy = reinterpret_cast<const bf16*>(a.dy);
  const bf16* __restrict__ x = reinterpret_cast<const bf16*>(a.x);
  // staging: 128 rows x 8 units (64 channels) per operand -> 4 units per thread per operand
  const int uc = tid & 7;
  const int co = co0 + uc * 8, ci = ci0 + uc * 8;
  uint4 ry[4], rx[4];
  auto load = [&](int t) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int row = (tid >> 3) + u * 32;
      const int i = t * WKM + row;
      ry[u] = make_uint4(0, 0, 0, 0);
      rx[u] = make_uint4(0, 0, 0, 0);
      if (i < a.NT) {
        if (co < a.Cout) ry[u] = *reinterpret_cast<const uint4*>(dy + ((long)i * V + w) * a.dy_ld + co);
        if (ci < a.Cin) rx[u] = *reinterpret_cast<const uint4*>(x + ((long)i * V + src) * a.x_ld + ci);
      }
    }
  };
  auto store = [&](int buf) {
    char* base = smem + buf * STAGE;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int row = (tid >> 3) + u * 32;
      const int off = (uc >> 2) * PANEL + row * WPR + (uc & 3) * 16;
      *reinterpret_cast<uint4*>(base + off) = ry[u];
      *reinterpret_cast<uint4*>(base + 2 * PANEL + off) = rx[u];
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int a2 = 0; a2 < 2; ++a2)
#pragma unroll
    for (int b2 = 0; b2 < 2; ++b2)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a2][b2][r] = 0.f;

  int cur = 0;
  if (t0 < t1) {
    load(t0);
    store(0);
  }
  __syncthreads();
  for (int t = t0; t < t1; ++t) {
    const bool more = t + 1 < t1;
    if (more) load(t + 1);
    const char* base = smem + cur * STAGE;
#pragma unroll
    for (int kk = 0; kk < WKM / 16 / 4; ++kk) {  // this wave's k-steps: ks = wave + 4*kk
      const int ks = wave + 4 * kk;
      bf16x8 fa[2], fb[2];
#pragma unroll
      for (int a2 = 0; a2 < 2; ++a2) fa[a2] = trfrag(base + a2 * PANEL, ks * 16, lane);
#pragma unroll
      for (int b2 = 0; b2 < 2; ++b2) fb[b2] = trfrag(base + (2 + b2) * PANEL, ks * 16, lane);
#pragma unroll
      for (int a2 = 0; a2 < 2; ++a2)
#pragma unroll
        for (int b2 = 0; b2 < 2; ++b2)
          acc[a2][b2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[a2], fb[b2], acc[a2][b2], 0, 0, 0);
    }
    if (more) store(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  // sum the 4 waves' accumulators (LDS), wave 0 writes this block's partial
  float* red = reinterpret_cast<float*>(smem);  // [3][4 tiles][16][64]
  if (wave > 0) {
#pragma unroll
    for (int a2 = 0; a2 < 2; ++a2)
#pragma unroll
      for (int b2 = 0; b2 < 2; ++b2)
#pragma unroll
        for (int r = 0; r < 16; ++r) red[(((wave - 1) * 4 + a2 * 2 + b2) * 16 + r) * 64 + lane] = acc[a2][b2][r];
  }
  __syncthreads();
  if (wave == 0) {
    float* slab = g.slab + ((long)rr * V * a.J + pair) * a.Cout * a.Cin;
#pragma unroll
    for (int a2 = 0; a2 < 2; ++a2)
#pragma unroll
      for (int b2 = 0; b2 < 2; ++b2) {
        const int cc = ci0 + b2 * 32 + (lane & 31);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float v = acc[a2][b2][r];
          for (int k = 0; k < 3; ++k) v += red[((k * 4 + a2 * 2 + b2) * 16 + r) * 64 + lane];
          const int oc = co0 + a2 * 32 + acc_row(r, lane);
          if (oc < a.Cout && cc < a.Cin) slab[(long)oc * a.Cin + cc] = v;
        }
      }
  }
}

// Joint-grouped variant: block = (output joint w, COB output channels, 64 input channels, row range).
// Every pair (w, j < deg[w]) shares the dy[:, w] panel, so a 64-row tile stages dy once plus deg x
// panels (one per neighbour) instead of deg (dy, x) pairs: (1 + deg) / (2 deg) of the L2 -> LDS traffic
// at COB = 64 and (COB/64 + deg) / (2 deg COB/64) at COB = 128.  Waves = (32-co quarter, 32-ci half);
// each keeps one 32x32 accumulator per neighbour (J2 <= 5) and per k-step reads one dy fragment and
// deg x fragments (ds_read_b64_tr_b16) for deg MFMAs.  Partials go to the same slab as above.
constexpr int w2m(int cob) { return cob == 128 ? 64 : 32; }  // rows per tile (LDS: 112 / 48 KB double-buffered)
constexpr int J2 = 5;     // max neighbours per joint
template <int COB>
__global__ __launch_bounds__(COB / 16 * 64, COB == 64 ? 3 : 1) void gconv_wgrad2_kernel(const stgcn_gconv_wgrad_desc a, const WGG g) {
  constexpr int NW = COB / 16, NT = NW * 64;
  constexpr int W2M = w2m(COB);
  constexpr int PANEL = W2M * WPR;           // 32 channels x W2M rows
  constexpr int DYP = COB / 32;              // dy panels
  constexpr int STAGE = (DYP + 2 * J2) * PANEL;
  constexpr int DYU = COB * W2M / 8 / NT;    // dy 16-B units per thread (2)
  constexpr int XU = 64 * W2M / 8 / NT;      // x units per thread per neighbour (2 at COB 64, 1 at 128)
  static_assert(DYU >= 1 && XU >= 1, "units");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cq = wave % DYP, ch = wave / DYP;  // co quarter (32), ci half (32)
  const int V = a.V;
  const int ngrp = g.nco * g.nci;
  const int w = blockIdx.x / (ngrp * g.R);
  const int rem = blockIdx.x % (ngrp * g.R);
  const int rr = rem / ngrp, grp = rem % ngrp;
  const int deg = a.deg[w];
  const int co0 = (grp % g.nco) * COB, ci0 = (grp / g.nco) * 64;
  const int t0 = rr * g.tpb, t1 = min(g.ntile, t0 + g.tpb);
  int src[J2];
#pragma unroll
  for (int j = 0; j < J2; ++j) src[j] = j < deg ? a.nbr[w * a.J + j] : 0;

  const bf16* __restrict__ dy = reinterpret_cast<const bf16*>(a.dy);
  const bf16* __restrict__ x = reinterpret_cast<const bf16*>(a.x);
  uint4 ry[DYU], rx[J2][XU];
  // dy unit e = tid + NT*u: row e / (COB/8), 8 channels at (e % (COB/8)) * 8; x unit: row e / 8, ch (e % 8) * 8
  auto load = [&](int t) {
#pragma unroll
    for (int u = 0; u < DYU; ++u) {
      const int e = tid + NT * u, row = e / (COB / 8), cu = e % (COB / 8);
      const int i = t * W2M + row;
      ry[u] = make_uint4(0, 0, 0, 0);
      if (i < a.NT && co0 + cu * 8 < a.Cout) ry[u] = *reinterpret_cast<const uint4*>(dy + ((long)i * V + w) * a.dy_ld + co0 + cu * 8);
    }
#pragma unroll
    for (int j = 0; j < J2; ++j)
#pragma unroll
      for (int u = 0; u < XU; ++u) {
        const int e = tid + NT * u, row = e >> 3, cu = e & 7;
        const int i = t * W2M + row;
        rx[j][u] = make_uint4(0, 0, 0, 0);
        if (j < deg && i < a.NT && ci0 + cu * 8 < a.Cin)
          rx[j][u] = *reinterpret_cast<const uint4*>(x + ((long)i * V + src[j]) * a.x_ld + ci0 + cu * 8);
      }
  };
  auto store = [&](int buf) {
    char* base = smem + buf * STAGE;
#pragma unroll
    for (int u = 0; u < DYU; ++u) {
      const int e = tid + NT * u, row = e / (COB / 8), cu = e % (COB / 8);
      *reinterpret_cast<uint4*>(base + (cu >> 2) * PANEL + row * WPR + (cu & 3) * 16) = ry[u];
    }
#pragma unroll
    for (int j = 0; j < J2; ++j)
#pragma unroll
      for (int u = 0; u < XU; ++u) {
        const int e = tid + NT * u, row = e >> 3, cu = e & 7;
        if (j < deg)
          *reinterpret_cast<uint4*>(base + (DYP + 2 * j + (cu >> 2)) * PANEL + row * WPR + (cu & 3) * 16) = rx[j][u];
      }
  };

  f32x16 acc[J2];
#pragma unroll
  for (int j = 0; j < J2; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  // per-joint row sums of dy (the bias-through-A gradient) ride along in the first ci-group's blocks
  const bool rsum = g.rowpart != nullptr && grp / g.nco == 0;
  float sacc[DYU][8];
#pragma unroll
  for (int u = 0; u < DYU; ++u)
#pragma unroll
    for (int e = 0; e < 8; ++e) sacc[u][e] = 0.f;
  auto add_rows = [&]() {
    if (rsum) {
#pragma unroll
      for (int u = 0; u < DYU; ++u) {
        float f[8];
        unpack16(ry[u], f, (bf16*)nullptr);
#pragma unroll
        for (int e = 0; e < 8; ++e) sacc[u][e] += f[e];
      }
    }
  };

  int cur = 0;
  if (t0 < t1) {
    load(t0);
    add_rows();
    store(0);
  }
  __syncthreads();
  for (int t = t0; t < t1; ++t) {
    const bool more = t + 1 < t1;
    if (more) load(t + 1);
    const char* base = smem + cur * STAGE;
#pragma unroll
    for (int ks = 0; ks < W2M / 16; ++ks) {
      const bf16x8 fa = trfrag(base + cq * PANEL, ks * 16, lane);
#pragma unroll
      for (int j = 0; j < J2; ++j)
        if (j < deg) {
          const bf16x8 fb = trfrag(base + (DYP + 2 * j + ch) * PANEL, ks * 16, lane);
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb, acc[j], 0, 0, 0);
        }
    }
    if (more) {
      add_rows();
      store(cur ^ 1);
    }
    __syncthreads();
    cur ^= 1;
  }
  if (rsum) {  // [row slot][COB] in LDS (the stages are free after the last barrier), fixed-order sum
    float* red = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int u = 0; u < DYU; ++u) {
      const int e = tid + NT * u, row = e / (COB / 8), cu = e % (COB / 8);
#pragma unroll
      for (int k = 0; k < 8; ++k) red[row * COB + cu * 8 + k] = sacc[u][k];
    }
    __syncthreads();
    if (tid < COB && co0 + tid < a.Cout) {
      float t = 0.f;
      for (int r = 0; r < W2M; ++r) t += red[r * COB + tid];
      g.rowpart[((long)rr * V + w) * a.Cout + co0 + tid] = t;
    }
  }

  // block partial of each pair (w, j) -> slab[rr][w*J + j][co][ci]
  const int cc = ci0 + ch * 32 + (lane & 31);
#pragma unroll
  for (int j = 0; j < J2; ++j) {
    if (j >= deg) continue;
    float* slab = g.slab + ((long)rr * V * a.J + w * a.J + j) * a.Cout * a.Cin;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int oc = co0 + cq * 32 + acc_row(r, lane);
      if (oc < a.Cout && cc < a.Cin) slab[(long)oc * a.Cin + cc] = acc[j][r];
    }
  }
}

// DMA-ring variant of gconv_wgrad2_kernel<64> (the default): the same block = (joint w, 64 co, 64 ci,
// row range) and wave split, but the 32-row tiles go global -> LDS with global_load_lds (no register
// staging) into a ring of W3D(DEG) slots sized by the joint's degree, so D - 1 tiles are in flight
// while one is consumed instead of one.  The register-staged kernel kept at most one tile (~16 KB)
// per block in flight and sat at ~13 % of the MFMA peak, latency-bound on L2/MALL.  Body per degree
// (DEG = deg[w], a block-uniform value) so the vmcnt counts are immediates.
// LDS per block: 80 KB (two blocks per CU) or, for the direct plans (R = 1: fewer, longer blocks), 160 KB for a
// deeper ring (one block per CU)
constexpr int w3_stage(int deg) { return (2 + 2 * deg) * 32 * WPR; }
constexpr int w3d(int deg, int lds) { return lds / w3_stage(deg) > 8 ? 8 : lds / w3_stage(deg); }

template <int N, typename F>
DEV void sfor(F&& f) {
  [&]<int... I>(std::integer_sequence<int, I...>) { (f.template operator()<I>(), ...); }(
      std::make_integer_sequence<int, N>{});
}

DEV unsigned lds_u32(const void* p) { return (unsigned)(size_t)(const __attribute__((address_space(3))) char*)p; }

// 16 B per lane, global -> LDS at M0 = lds_off (lane-linear).  m0 is a reserved register, so it is not
// declared clobbered: the asm saves the compiler's m0 in an SGPR it owns and restores it after the
// issue (the DMA samples M0 when it is issued).
DEV void glds16m(const void* src, unsigned lds_off) {
  unsigned saved;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(saved) : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds_off)) : "memory");
}

// half: -1 = a whole (joint, group, row range) block; 0 / 1 = one half of a split direct-plan block (tiles t0..t1)
template <int DEG, int LDSB>
DEV void wgrad3_body(const stgcn_gconv_wgrad_desc& a, const WGG& g, char* smem, int w, int rr, int grp, int t0,
                     int t1, int half) {
  constexpr int D = w3d(DEG, LDSB), PANEL = 32 * WPR, STAGE = w3_stage(DEG), NU = 1 + DEG;
  static_assert(D >= 3 && (D - 2) * NU <= 63, "ring");
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cq = wave & 1, ch = wave >> 1;  // co half (32), ci half (32)
  const int V = a.V;
  const int co0 = (grp % g.nco) * 64, ci0 = (grp / g.nco) * 64;
  const bf16* __restrict__ dy = reinterpret_cast<const bf16*>(a.dy);
  const bf16* __restrict__ x = reinterpret_cast<const bf16*>(a.x);
  // this wave's DMA share of a tile: dy panel (wave >> 1) rows 16 (wave & 1) .. +15, and the same
  // (panel, half) of every neighbour's x; lane -> (row lane / 4, 16-B unit lane % 4)
  const int prow = 16 * (wave & 1) + (lane >> 2), pu = lane & 3, pp = wave >> 1;
  const bf16* ysrc = dy + (long)w * a.dy_ld + co0 + pp * 32 + pu * 8;
  const bf16* xsrc[DEG];
#pragma unroll
  for (int j = 0; j < DEG; ++j) xsrc[j] = x + (long)a.nbr[w * a.J + j] * a.x_ld + ci0 + pp * 32 + pu * 8;
  const long ystep = (long)V * a.dy_ld, xstep = (long)V * a.x_ld;
  const unsigned ring = lds_u32(smem);
  const unsigned woff = (unsigned)(pp * PANEL + (wave & 1) * 1024);
  auto issue = [&](int t) {
    const int i = min(t * 32 + prow, a.NT - 1);  // rows past NT: clamped here, zeroed in LDS below
    const unsigned slot = ring + (unsigned)(((t - t0) % D) * STAGE) + woff;
    glds16m(ysrc + i * ystep, slot);
#pragma unroll
    for (int j = 0; j < DEG; ++j) glds16m(xsrc[j] + i * xstep, slot + (unsigned)((2 + 2 * j) * PANEL));
  };
#pragma unroll
  for (int k = 0; k < D - 1; ++k)
    if (t0 + k < t1) issue(t0 + k);

  f32x16 acc[DEG];
#pragma unroll
  for (int j = 0; j < DEG; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  const bool rsum = g.rowpart != nullptr && grp / g.nco == 0;
  float sacc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) sacc[e] = 0.f;
  // row-sum unit of this thread: row tid / 8, 8 channels at (tid % 8) * 8
  const int srow = tid >> 3, scu = tid & 7;
  const int soff = (scu >> 2) * PANEL + srow * WPR + (scu & 3) * 16;

  for (int t = t0; t < t1; ++t) {
    const int after = min(D - 2, t1 - 1 - t);  // tiles issued after t
    sfor<D - 1>([&]<int m>() {
      if (after == m) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(m * NU) : "memory");
    });
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (t + D - 1 < t1) issue(t + D - 1);  // into the slot of tile t - 1, free after the barrier
    char* base = smem + ((t - t0) % D) * STAGE;
    if (t * 32 + 32 > a.NT) {  // last, partial tile: zero dy rows >= NT (block-uniform branch)
      if (t * 32 + srow >= a.NT) *reinterpret_cast<uint4*>(base + soff) = make_uint4(0, 0, 0, 0);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    if (rsum) {
      float f[8];
      unpack16(*reinterpret_cast<const uint4*>(base + soff), f, (bf16*)nullptr);
#pragma unroll
      for (int e = 0; e < 8; ++e) sacc[e] += f[e];
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 fa = trfrag(base + cq * PANEL, ks * 16, lane);
#pragma unroll
      for (int j = 0; j < DEG; ++j) {
        const bf16x8 fb = trfrag(base + (2 + 2 * j + ch) * PANEL, ks * 16, lane);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb, acc[j], 0, 0, 0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  float rs = 0.f;  // this block's row sum of column co0 + tid (tid < 64)
  if (rsum) {  // [row][64] in LDS, fixed-order column sums
    float* red = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int k = 0; k < 8; ++k) red[srow * 64 + scu * 8 + k] = sacc[k];
    __syncthreads();
    if (tid < 64)
      for (int r = 0; r < 32; ++r) rs += red[r * 64 + tid];
  }
  if (half >= 0) {
    // split block: publish this half's partial write-through (sc1), drain, one arrival; the second arriver reads the
    // other half (sc1) and adds it (a + b == b + a: the result does not depend on which half came last) and writes
    // the outputs (MI355X_MICROARCH "Valid forms" row 1: sc1 stores and loads on both sides, no fences)
    constexpr int PSZ_J = 4096;
    const int ngrp = g.nco * g.nci;
    const long PSZ = (long)a.J * PSZ_J + 64;
    float* mine = g.part + (((long)w * ngrp + grp) * 2 + half) * PSZ;
    const float* other = g.part + (((long)w * ngrp + grp) * 2 + (1 - half)) * PSZ;
    const int el = (cq * 32) * 64 + ch * 32 + (lane & 31);  // + acc_row(r, lane) * 64
#pragma unroll
    for (int j = 0; j < DEG; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        __hip_atomic_store(mine + j * PSZ_J + el + acc_row(r, lane) * 64, acc[j][r], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    if (rsum && tid < 64) __hip_atomic_store(mine + a.J * PSZ_J + tid, rs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(smem);
    if (tid == 0)
      *flag = (int)__hip_atomic_fetch_add(g.cnt + (long)w * ngrp + grp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (*flag == 0) return;  // first arriver: the partner merges
#pragma unroll
    for (int j = 0; j < DEG; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        acc[j][r] += __hip_atomic_load(const_cast<float*>(other) + j * PSZ_J + el + acc_row(r, lane) * 64,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (rsum && tid < 64)
      rs += __hip_atomic_load(const_cast<float*>(other) + a.J * PSZ_J + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (rsum && tid < 64) g.rowpart[((long)rr * V + w) * a.Cout + co0 + tid] = rs;
  const int cc = ci0 + ch * 32 + (lane & 31);
#pragma unroll
  for (int j = 0; j < DEG; ++j) {
    float* slab = g.slab + ((long)rr * V * a.J + w * a.J + j) * a.Cout * a.Cin;
#pragma unroll
    for (int r = 0; r < 16; ++r) slab[(long)(co0 + cq * 32 + acc_row(r, lane)) * a.Cin + cc] = acc[j][r];
  }
  if (g.zero_unused)
    for (int j = DEG; j < a.J; ++j) {
      float* slab = g.slab + ((long)w * a.J + j) * a.Cout * a.Cin;
#pragma unroll
      for (int r = 0; r < 16; ++r) slab[(long)(co0 + cq * 32 + acc_row(r, lane)) * a.Cin + cc] = 0.f;
    }
}

// STGCN_W3_XCD (A/B build flag): row-range-major block order remapped so that consecutive logical blocks share an
// XCD (all joints of one row range on one XCD: the x rows a joint's neighbours also read stay in that XCD's L2)
#ifndef STGCN_W3_XCD
#define STGCN_W3_XCD 0
#endif
// STGCN_W3_SPLIT: degree-balanced direct plan (W3_SPLIT_DEG); the XCD-order A/B build keeps the plain direct plan
#if STGCN_W3_XCD
#undef STGCN_W3_SPLIT
#define STGCN_W3_SPLIT 0
#endif
#ifndef STGCN_W3_SPLIT
#define STGCN_W3_SPLIT 1
#endif
template <int LDSB>
__global__ __launch_bounds__(256, LDSB > 80 * 1024 ? 1 : 2) void gconv_wgrad3_kernel(const stgcn_gconv_wgrad_desc a,
                                                                                    const WGG g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int ngrp = g.nco * g.nci;
#if STGCN_W3_XCD
  int wgi;
  {
    const int id = blockIdx.x, nblk = gridDim.x, x = id & 7, q = nblk >> 3, r = nblk & 7;
    wgi = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (id >> 3);
  }
  const int rr = wgi / (a.V * ngrp), rem = wgi % (a.V * ngrp);
  const int w = rem / ngrp, grp = rem % ngrp;
#else
  const int bid = g.part ? (int)(blockIdx.x % (a.V * ngrp)) : (int)blockIdx.x;  // split plan: slot 1 repeats slot 0
  const int w = bid / (ngrp * g.R);
  const int rem = bid % (ngrp * g.R);
  const int rr = rem / ngrp, grp = rem % ngrp;
#endif
  // joints in decreasing-degree order (ties by index): the heaviest blocks are dispatched first and the
  // light ones fill the tail.  Scratch in the ring's first bytes, before any DMA is issued.
  int* sdeg = reinterpret_cast<int*>(smem);
  int* order = sdeg + 64;
  int wj = w;
  if (a.V <= 64) {
    const int tid = threadIdx.x;
    if (tid < a.V) sdeg[tid] = a.deg[tid];
    __syncthreads();
    if (tid < a.V) {
      const int d = sdeg[tid];
      int r = 0;
      for (int u = 0; u < a.V; ++u) r += (sdeg[u] > d) | ((sdeg[u] == d) & (u < tid));
      order[r] = tid;
    }
    __syncthreads();
    wj = order[w];
    __syncthreads();
  }
  int t0 = rr * g.tpb, t1 = min(g.ntile, t0 + g.tpb), half = -1;
  if (g.part) {  // degree-balanced direct plan: grid = 2 x V x ngrp, slot 1 only for the split joints
    const int slot = blockIdx.x / (a.V * ngrp);
    const bool split = a.deg[wj] >= W3_SPLIT_DEG;
    if (slot == 1 && !split) return;  // block-uniform exit before any barrier
    if (split) {
      half = slot;
      const int tm = g.ntile / 2;
      t0 = half ? tm : 0;
      t1 = half ? g.ntile : tm;
    }
  }
  switch (a.deg[wj]) {
    case 1: wgrad3_body<1, LDSB>(a, g, smem, wj, rr, grp, t0, t1, half); break;
    case 2: wgrad3_body<2, LDSB>(a, g, smem, wj, rr, grp, t0, t1, half); break;
    case 3: wgrad3_body<3, LDSB>(a, g, smem, wj, rr, grp, t0, t1, half); break;
    case 4: wgrad3_body<4, LDSB>(a, g, smem, wj, rr, grp, t0, t1, half); break;
    case 5: wgrad3_body<5, LDSB>(a, g, smem, wj, rr, grp, t0, t1, half); break;
    default:  // deg 0: no pairs (the reduction skips j >= deg); the row sums still come from here
      if (g.rowpart != nullptr && grp / g.nco == 0 && threadIdx.x < 64) {
        const int co = (grp % g.nco) * 64 + threadIdx.x;
        const int i1 = min(a.NT, min(g.ntile, (rr + 1) * g.tpb) * 32);
        const bf16* dy = reinterpret_cast<const bf16*>(a.dy);
        float s = 0.f;
        for (int i = rr * g.tpb * 32; i < i1; ++i) s += (float)dy[((long)i * a.V + wj) * a.dy_ld + co];
        g.rowpart[((long)rr * a.V + wj) * a.Cout + co] = s;
      }
      if (g.zero_unused) {  // direct plan: this joint's J slots of the (64 co, 64 ci) group are zero
        const int co0 = (grp % g.nco) * 64, ci0 = (grp / g.nco) * 64;
        for (int i = threadIdx.x; i < a.J * 64 * 64; i += blockDim.x) {
          const int j = i >> 12, co = (i >> 6) & 63, ci = i & 63;
          g.slab[(((long)wj * a.J + j) * a.Cout + co0 + co) * a.Cin + ci0 + ci] = 0.f;
        }
      }
      break;
  }
}

// ---- wide plan (Cin, Cout % 128 == 0): block = (joint, 128 co x 128 ci group, row part), 4 waves (one per SIMD, 2 x 2
// output tiles per neighbour each: 64*DEG accumulators, up to 512 registers per lane) and a 160 KB ring.  Against the 64 x 64 blocks above it halves the panels every block stages per MFMA (dy read by
// Cin/128 instead of Cin/64 blocks, x by Cout/128) and gives each barrier twice the matrix work per SIMD.  Row
// parts of one group merge in-kernel: every part publishes its partial write-through (sc1), takes a ticket, and
// the last arriver sums the R partials in part-index order (a fixed order: the result does not depend on
// arrival), then writes dWeff, the zero slots and the row sums.
#ifndef STGCN_W3W
#define STGCN_W3W 1
#endif
#ifndef STGCN_W3W_TARGET
#define STGCN_W3W_TARGET 256
#endif
constexpr int W3W_LDS = 160 * 1024;
constexpr int W3W_PSZ_J = 128 * 128;
constexpr int W3W_JE = 3;  // neighbours per entry at most: joints of degree >= 4 run as two entries
constexpr int w3w_stage(int deg) { return (4 + 4 * deg) * 32 * WPR; }
constexpr int w3w_d(int deg) { return W3W_LDS / w3w_stage(deg) > 8 ? 8 : W3W_LDS / w3w_stage(deg); }

template <int DEG>
DEV void wgrad3w_body(const stgcn_gconv_wgrad_desc& a, const WGG& g, char* smem, int w, int e, int j0, int dtot, int rr,
                      int grp, int t0, int t1) {
  constexpr int D = w3w_d(DEG), PANEL = 32 * WPR, STAGE = w3w_stage(DEG), NU = 2 * (1 + DEG);
  static_assert(D >= 3 && (D - 2) * NU <= 63, "ring");
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cp = wave & 1, ip = wave >> 1;  // co tiles 2cp, 2cp+1 and ci tiles 2ip, 2ip+1 (32 each) of the group
  const int V = a.V;
  const int co0 = (grp % g.nco) * 128, ci0 = (grp / g.nco) * 128;
  const bf16* __restrict__ dy = reinterpret_cast<const bf16*>(a.dy);
  const bf16* __restrict__ x = reinterpret_cast<const bf16*>(a.x);
  // DMA share of a tile: panel `wave` of dy and of every neighbour's x, both 16-row halves;
  // lane -> (row lane / 4 (+16), 16-B unit lane % 4)
  const int prow = lane >> 2, pu = lane & 3;
  const bf16* ysrc = dy + (long)w * a.dy_ld + co0 + wave * 32 + pu * 8;
  const bf16* xsrc[DEG];
#pragma unroll
  for (int j = 0; j < DEG; ++j) xsrc[j] = x + (long)a.nbr[w * a.J + j0 + j] * a.x_ld + ci0 + wave * 32 + pu * 8;
  const long ystep = (long)V * a.dy_ld, xstep = (long)V * a.x_ld;
  const unsigned ring = lds_u32(smem);
  const unsigned woff = (unsigned)(wave * PANEL);
  auto issue = [&](int t) {
    const unsigned slot = ring + (unsigned)(((t - t0) % D) * STAGE) + woff;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int i = min(t * 32 + 16 * h + prow, a.NT - 1);  // rows past NT: clamped here, dy zeroed in LDS below
      glds16m(ysrc + i * ystep, slot + (unsigned)(h * 1024));
#pragma unroll
      for (int j = 0; j < DEG; ++j) glds16m(xsrc[j] + i * xstep, slot + (unsigned)((4 + 4 * j) * PANEL + h * 1024));
    }
  };
#pragma unroll
  for (int k = 0; k < D - 1; ++k)
    if (t0 + k < t1) issue(t0 + k);

  f32x16 acc[DEG][2][2];
#pragma unroll
  for (int j = 0; j < DEG; ++j)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][u][c][r] = 0.f;
  const bool rsum = g.rowpart != nullptr && grp / g.nco == 0 && j0 == 0;  // an entry's first neighbour slot: row sums
  float sacc[2][8];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int e = 0; e < 8; ++e) sacc[h][e] = 0.f;
  // dy units of this thread (row sums, zeroing past NT): unit tid + 256 h -> row (unit / 16), channels (unit % 16) * 8
  auto soff = [&](int h) {
    const int u = tid + 256 * h, sr = u >> 4, sc = u & 15;
    return (sc >> 2) * PANEL + sr * WPR + (sc & 3) * 16;
  };

  for (int t = t0; t < t1; ++t) {
    const int after = min(D - 2, t1 - 1 - t);  // tiles issued after t
    sfor<D - 1>([&]<int m>() {
      if (after == m) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(m * NU) : "memory");
    });
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (t + D - 1 < t1) issue(t + D - 1);  // into the slot of tile t - 1, free after the barrier
    char* base = smem + ((t - t0) % D) * STAGE;
    if (t * 32 + 32 > a.NT) {  // last, partial tile: zero dy rows >= NT (block-uniform branch)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        if (t * 32 + ((tid + 256 * h) >> 4) >= a.NT) *reinterpret_cast<uint4*>(base + soff(h)) = make_uint4(0, 0, 0, 0);
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    if (rsum) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float f[8];
        unpack16(*reinterpret_cast<const uint4*>(base + soff(h)), f, (bf16*)nullptr);
#pragma unroll
        for (int e = 0; e < 8; ++e) sacc[h][e] += f[e];
      }
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 fa[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) fa[u] = trfrag(base + (2 * cp + u) * PANEL, ks * 16, lane);
#pragma unroll
      for (int j = 0; j < DEG; ++j) {
        bf16x8 fb[2];
#pragma unroll
        for (int c = 0; c < 2; ++c) fb[c] = trfrag(base + (4 + 4 * j + 2 * ip + c) * PANEL, ks * 16, lane);
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int c = 0; c < 2; ++c)
            acc[j][u][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[u], fb[c], acc[j][u][c], 0, 0, 0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  float rs = 0.f;  // this block's row sum of column co0 + tid (tid < 128)
  if (rsum) {      // [row][128] in LDS (first 16 KB), fixed-order column sums
    float* red = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int u = tid + 256 * h;
#pragma unroll
      for (int k = 0; k < 8; ++k) red[(u >> 4) * 128 + (u & 15) * 8 + k] = sacc[h][k];
    }
    __syncthreads();
    if (tid < 128)
      for (int r = 0; r < 32; ++r) rs += red[r * 128 + tid];
  }
  // Epilogue through LDS, one neighbour at a time: the 128 x 128 tile staged as fp32 rows [co][132], then whole
  // 512-B rows leave as 16-B stores (every address an LDS immediate or one running pointer: no per-element
  // address registers next to the 64*DEG accumulators)
  constexpr int SRS = 132;
  float* stg = reinterpret_cast<float*>(smem + 20 * 1024);  // after the row sums and the ticket word
  int* flag = reinterpret_cast<int*>(smem + 16 * 1024);
  const bool merged = g.R > 1;
  const int ngrp = g.nco * g.nci;
  const long PSZ = (long)W3W_JE * W3W_PSZ_J + 128;
  float* gp = merged ? g.part + ((long)e * ngrp + grp) * g.R * PSZ : nullptr;
  const __amdgpu_buffer_rsrc_t prs =
      __builtin_amdgcn_make_buffer_rsrc(merged ? gp : g.slab, 0, merged ? (int)(g.R * PSZ * 4) : 0, 0x00020000);
  float* o0 = g.slab + (long)w * a.J * a.Cout * a.Cin + (long)co0 * a.Cin + ci0;  // dWeff[w][0][co0][ci0]
  const long ojs = (long)a.Cout * a.Cin;
#pragma unroll
  for (int j = 0; j < DEG; ++j) {
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          stg[(cp * 64 + u * 32 + acc_row(r, lane)) * SRS + ip * 64 + c * 32 + (lane & 31)] = acc[j][u][c][r];
    __syncthreads();
    for (int e = tid; e < 128 * 32; e += 256) {
      const int row = e >> 5, q4 = e & 31;
      const float4 v = *reinterpret_cast<const float4*>(stg + row * SRS + q4 * 4);
      if (!merged)
        *reinterpret_cast<float4*>(o0 + (j0 + j) * ojs + (long)row * a.Cin + q4 * 4) = v;
      else  // this part's partial, write-through (sc1): the last arriver reads it from another CU / XCD
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v), prs,
                                               (int)(((long)rr * PSZ + j * W3W_PSZ_J + row * 128 + q4 * 4) * 4), 0, 16);
    }
  }
  if (merged) {
    if (rsum && tid < 128)
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, rs), prs,
                                            (int)(((long)rr * PSZ + W3W_JE * W3W_PSZ_J + tid) * 4), 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0)
      *flag = (int)__hip_atomic_fetch_add(g.cnt + (long)e * ngrp + grp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (*flag != g.R - 1) return;  // not the last part: the last arriver merges
    // the R partials summed in part-index order (a fixed order: the result does not depend on arrival)
    for (int j = 0; j < DEG; ++j)
      for (int e = tid; e < 128 * 32; e += 256) {
        const int row = e >> 5, q4 = e & 31;
        const int off = (j * W3W_PSZ_J + row * 128 + q4 * 4) * 4;
        float4 sum = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(prs, off, 0, 16));
        for (int k = 1; k < g.R; ++k) {
          const float4 v =
              __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(prs, (int)(off + k * PSZ * 4), 0, 16));
          sum.x += v.x;
          sum.y += v.y;
          sum.z += v.z;
          sum.w += v.w;
        }
        *reinterpret_cast<float4*>(o0 + (j0 + j) * ojs + (long)row * a.Cin + q4 * 4) = sum;
      }
    if (rsum && tid < 128) {
      rs = 0.f;
      for (int k = 0; k < g.R; ++k) {
        const float v = __builtin_bit_cast(
            float, __builtin_amdgcn_raw_buffer_load_b32(prs, (int)((k * PSZ + W3W_JE * W3W_PSZ_J + tid) * 4), 0, 16));
        rs = k == 0 ? v : rs + v;
      }
    }
  }
  if (rsum && tid < 128) g.rowpart[(long)w * a.Cout + co0 + tid] = rs;
  if (j0 == 0)
  for (int j = dtot; j < a.J; ++j)  // the unused slots of this joint and group: zero (by the joint's first entry)
    for (int e = tid; e < 128 * 32; e += 256)
      *reinterpret_cast<float4*>(o0 + j * ojs + (long)(e >> 5) * a.Cin + (e & 31) * 4) = make_float4(0.f, 0.f, 0.f, 0.f);
}

__global__ __launch_bounds__(256, 1) void gconv_wgrad3w_kernel(const stgcn_gconv_wgrad_desc a, const WGG g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int ngrp = g.nco * g.nci;
  const int bid = blockIdx.x;
  const int e = bid / (ngrp * g.R), rem = bid % (ngrp * g.R);
  const int rr = rem / ngrp, grp = rem % ngrp;
  // entries (joint, first neighbour slot, neighbour count) in decreasing-degree joint order (the heaviest blocks
  // are dispatched first); a joint of degree >= 4 runs as two entries of <= 3 neighbours (its dy panels are staged
  // twice, but 64*deg accumulators would exceed the register file and its ring would be shallow).  Scratch in the
  // ring's first bytes, read before any DMA is issued.  Grid: 2V entries (the ones past the count exit at once).
  int* sdeg = reinterpret_cast<int*>(smem);
  int* order = sdeg + 64;
  int* ent = order + 64;  // [0] = count, then (joint, j0, n) triples
  const int tid = threadIdx.x;
  if (tid < a.V) sdeg[tid] = a.deg[tid];
  __syncthreads();
  if (tid < a.V) {
    const int d = sdeg[tid];
    int r = 0;
    for (int u = 0; u < a.V; ++u) r += (sdeg[u] > d) | ((sdeg[u] == d) & (u < tid));
    order[r] = tid;
  }
  __syncthreads();
  if (tid == 0) {
    int E = 0;
    for (int r = 0; r < a.V; ++r) {
      const int w = order[r], d = sdeg[w];
      if (d > W3W_JE) {
        const int h = (d + 1) / 2;
        ent[1 + 3 * E] = w, ent[2 + 3 * E] = 0, ent[3 + 3 * E] = h, ++E;
        ent[1 + 3 * E] = w, ent[2 + 3 * E] = h, ent[3 + 3 * E] = d - h, ++E;
      } else {
        ent[1 + 3 * E] = w, ent[2 + 3 * E] = 0, ent[3 + 3 * E] = d, ++E;
      }
    }
    ent[0] = E;
  }
  __syncthreads();
  const int E = ent[0];
  const int wj = e < E ? ent[1 + 3 * e] : 0, j0 = e < E ? ent[2 + 3 * e] : 0, n = e < E ? ent[3 + 3 * e] : 0;
  const int dtot = e < E ? sdeg[wj] : 0;
  __syncthreads();  // every thread has its entry: the ring may overwrite the scratch
  if (e >= E) return;
  const int t0 = rr * g.tpb, t1 = min(g.ntile, t0 + g.tpb);
  switch (n) {
    case 1: wgrad3w_body<1>(a, g, smem, wj, e, j0, dtot, rr, grp, t0, t1); break;
    case 2: wgrad3w_body<2>(a, g, smem, wj, e, j0, dtot, rr, grp, t0, t1); break;
    case 3: wgrad3w_body<3>(a, g, smem, wj, e, j0, dtot, rr, grp, t0, t1); break;
    default:  // deg 0: no pairs; part 0 writes the zero slots and the row sums
      if (rr != 0) break;
      const int co0 = (grp % g.nco) * 128, ci0 = (grp / g.nco) * 128;
      if (g.rowpart != nullptr && grp / g.nco == 0 && tid < 128) {
        const bf16* dy = reinterpret_cast<const bf16*>(a.dy);
        float s = 0.f;
        for (int i = 0; i < a.NT; ++i) s += (float)dy[((long)i * a.V + wj) * a.dy_ld + co0 + tid];
        g.rowpart[(long)wj * a.Cout + co0 + tid] = s;
      }
      for (int i = tid; i < a.J * 128 * 128; i += blockDim.x) {
        const int j = i >> 14, co = (i >> 7) & 127, ci = i & 127;
        g.slab[(((long)wj * a.J + j) * a.Cout + co0 + co) * a.Cin + ci0 + ci] = 0.f;
      }
      break;
  }
}

// fp32 parity path of the gather wgrad: one thread per (pair, co, ci), loop over rows (small sizes)
__global__ void gconv_wgrad_f32_kernel(const stgcn_gconv_wgrad_desc a) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long total = (long)a.V * a.J * a.Cout * a.Cin;
  if (idx >= total) return;
  const int ci = (int)(idx % a.Cin);
  const int co = (int)((idx / a.Cin) % a.Cout);
  const int pair = (int)(idx / ((long)a.Cin * a.Cout));
  const int w = pair / a.J, j = pair % a.J;
  if (j >= a.deg[w]) {
    a.dweff[idx] = 0.f;
    return;
  }
  const int src = a.nbr[pair];
  const float* dy = reinterpret_cast<const float*>(a.dy);
  const float* x = reinterpret_cast<const float*>(a.x);
  float s = 0.f;
  for (int i = 0; i < a.NT; ++i)
    s += dy[((long)i * a.V + w) * a.dy_ld + co] * x[((long)i * a.V + src) * a.x_ld + ci];
  a.dweff[idx] = s;
}

// out[e] = sum_r part[r][e] in fixed order (per-joint row-sum partials of the joint-grouped kernel)
__global__ void rowpart_sum_kernel(const float* __restrict__ part, int R, long E, float* __restrict__ out) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  float s = 0.f;
  for (int r = 0; r < R; ++r) s += part[(long)r * E + e];
  out[e] = s;
}

// gslab_reduce (blocks [0, nb1)) and rowpart_sum (the rest) of one joint-grouped wgrad in one launch
__global__ void gslab_rowpart_kernel(const float* __restrict__ slab, int R, long E, long EC, const int* deg, int J,
                                     float* __restrict__ dweff, int nb1, const float* __restrict__ rpart, long ER,
                                     float* __restrict__ rowsum) {
  if ((int)blockIdx.x < nb1) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    const int pair = (int)(e / EC);
    float s = 0.f;
    if (pair % J < deg[pair / J])
      for (int r = 0; r < R; ++r) s += slab[(long)r * E + e];
    dweff[e] = s;
    return;
  }
  const long e = (long)(blockIdx.x - nb1) * blockDim.x + threadIdx.x;
  if (e >= ER) return;
  float s = 0.f;
  for (int r = 0; r < R; ++r) s += rpart[(long)r * ER + e];
  rowsum[e] = s;
}

// slab reduction (rows of the slab are whole [V*J][Cout][Cin] images): dweff[e] = sum_r slab[r][e]
__global__ void gslab_reduce_kernel(const float* __restrict__ slab, int R, long E, long EC, const int* deg, int J,
                                    float* __restrict__ out) {
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const int pair = (int)(e / EC);
  float s = 0.f;
  if (pair % J < deg[pair / J])  // slab slots of unused pairs are never written (nor read)
    for (int r = 0; r < R; ++r) s += slab[(long)r * E + e];
  out[e] = s;
}

// dW[p*Cout+co][ci] (+)= sum_{w, j<deg} A[p][nbr[w][j]][w] * dWeff[w][j][co][ci]
__global__ void gconv_dw_kernel(const float* __restrict__ dweff, const float* __restrict__ A, const int* nbr,
                                const int* deg, int P, int V, int J, int Cout, int Cin, float* dW) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long E = (long)Cout * Cin;
  if (idx >= (long)P * E) return;
  const int p = (int)(idx / E);
  const long e = idx % E;
  float s = 0.f;
  for (int w = 0; w < V; ++w)
    for (int j = 0; j < deg[w]; ++j) s += A[((long)p * V + nbr[w * J + j]) * V + w] * dweff[(long)(w * J + j) * E + e];
  dW[idx] += s;
}

// dA[p][nbr[w][j]][w] (+)= sum_{co,ci} W[p*Cout+co][ci] * dWeff[w][j][co][ci]; block per (pair, p)
__global__ void gconv_dA_kernel(const float* __restrict__ dweff, const float* __restrict__ W, const int* nbr,
                                const int* deg, int P, int V, int J, int Cout, int Cin, float* dA) {
  const int pair = blockIdx.x, p = blockIdx.y;
  const int w = pair / J, j = pair % J;
  if (j >= deg[w]) return;
  const long E = (long)Cout * Cin;
  const float* d = dweff + (long)pair * E;
  const float* wp = W + (long)p * E;
  float s = 0.f;
  for (long e = threadIdx.x; e < E; e += blockDim.x) s += wp[e] * d[e];
  s = wave_sum(s);
  __shared__ float part[4];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float t = part[0] + part[1] + part[2] + part[3];
    dA[((long)p * V + nbr[w * J + j]) * V + w] += t;
  }
}

constexpr int PMAX = 4;
// dW[p][e] += sum_{pairs} A[p][v][w] dWeff[pair][e] for all p in one pass (dWeff read once).
// Block = 256 e-columns (4 per lane) x 4 groups over the used (w, j) pairs (pair list and coefficients A[p][S(w)_j][w]
// staged in LDS first: the per-pair deg -> nbr -> A chain of dependent global loads was this kernel's
// cost); fixed-order LDS combine.
constexpr int DW_PAIRS = 32 * 8;  // V * J upper bound for the LDS tables
// one block's work (block index bb of ceil(E / 64)); ``acc_out``: dW += (else dW =, the caller's buffer
// needs no zero fill)
DEV void gconv_dw_all_body(const float* __restrict__ dweff, const float* __restrict__ A, const int* nbr,
                           const int* deg, int P, int V, int J, long E, float* dW, long bb, bool acc_out) {
  __shared__ int spair[DW_PAIRS];
  __shared__ float scoef[DW_PAIRS][PMAX];
  __shared__ int snp;
  if (threadIdx.x == 0) {  // compacted list of used pairs, in (w, j) order
    int n = 0;
    for (int w = 0; w < V; ++w)
      for (int j = 0; j < deg[w]; ++j) spair[n++] = w * J + j;
    snp = n;
  }
  __syncthreads();
  const int np = snp;
  for (int i = threadIdx.x; i < np * PMAX; i += 256) {
    const int k = i / PMAX, p = i % PMAX;
    const int pr = spair[k], w = pr / J;
    scoef[k][p] = p < P ? A[((long)p * V + nbr[pr]) * V + w] : 0.f;
  }
  __syncthreads();
  const int g = threadIdx.x >> 6;
  // 4 consecutive e per lane (16-B loads of dWeff): a block covers 256 columns of E (E % 4 == 0)
  const long e = (bb * 64 + (threadIdx.x & 63)) * 4;
  float4 acc[PMAX];
#pragma unroll
  for (int p = 0; p < PMAX; ++p) acc[p] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (e < E) {
#pragma unroll 4
    for (int k = g; k < np; k += 4) {
      const float4 d = *reinterpret_cast<const float4*>(dweff + (long)spair[k] * E + e);
#pragma unroll
      for (int p = 0; p < PMAX; ++p) {
        const float c = scoef[k][p];
        acc[p].x += c * d.x; acc[p].y += c * d.y; acc[p].z += c * d.z; acc[p].w += c * d.w;
      }
    }
  }
  __shared__ float4 part[4][PMAX][64];
#pragma unroll
  for (int p = 0; p < PMAX; ++p) part[g][p][threadIdx.x & 63] = acc[p];
  __syncthreads();
  if (threadIdx.x < 64 && e < E) {
    const int l = threadIdx.x;
#pragma unroll
    for (int p = 0; p < PMAX; ++p)
      if (p < P) {
        const float4 a0 = part[0][p][l], a1 = part[1][p][l], a2 = part[2][p][l], a3 = part[3][p][l];
        float4 t = make_float4(((a0.x + a1.x) + a2.x) + a3.x, ((a0.y + a1.y) + a2.y) + a3.y,
                               ((a0.z + a1.z) + a2.z) + a3.z, ((a0.w + a1.w) + a2.w) + a3.w);
        float4* o = reinterpret_cast<float4*>(dW + (long)p * E + e);
        if (acc_out) {
          const float4 q = *o;
          t.x += q.x; t.y += q.y; t.z += q.z; t.w += q.w;
        }
        *o = t;
      }
  }
}
__global__ __launch_bounds__(256) void gconv_dw_all_kernel(const float* __restrict__ dweff, const float* __restrict__ A,
                                                           const int* nbr, const int* deg, int P, int V, int J, long E,
                                                           float* dW) {
  gconv_dw_all_body(dweff, A, nbr, deg, P, V, J, E, dW, blockIdx.x, true);
}

// dA[p][v][w] += <W_p, dWeff[pair]> for all p, in two deterministic steps: block (pair, chunk) writes the
// P partial dots of its DA_CHUNK-element slice to part[pair][chunk][p]; gconv_dA_reduce sums the chunks in
// order.  (pair, chunk) grid keeps >= ~1000 blocks in flight even for C = 64.
constexpr int DA_CHUNK = 2048;
DEV void gconv_dA_part_body(const float* __restrict__ dweff, const float* __restrict__ W, const int* deg, int P, int J,
                           long E, float* part, int pair, int c, int nch) {
  if (pair % J >= deg[pair / J]) return;  // block-uniform, no barrier after it
  const float* d = dweff + (long)pair * E;
  float acc[PMAX] = {0.f, 0.f, 0.f, 0.f};
  const long e1 = min(E, (long)(c + 1) * DA_CHUNK);
  for (long e = (long)c * DA_CHUNK + threadIdx.x * 4; e < e1; e += 1024) {  // 16-B loads (E % 4 == 0)
    const float4 dv = *reinterpret_cast<const float4*>(d + e);
#pragma unroll
    for (int p = 0; p < PMAX; ++p)
      if (p < P) {
        const float4 w = *reinterpret_cast<const float4*>(W + (long)p * E + e);
        acc[p] += ((w.x * dv.x + w.y * dv.y) + w.z * dv.z) + w.w * dv.w;
      }
  }
  __shared__ float red[4][PMAX];
#pragma unroll
  for (int p = 0; p < PMAX; ++p) {
    const float t = wave_sum(acc[p]);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][p] = t;
  }
  __syncthreads();
  if (threadIdx.x < P)
    part[((long)pair * nch + c) * PMAX + threadIdx.x] =
        ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x];
}
__global__ __launch_bounds__(256) void gconv_dA_part_kernel(const float* __restrict__ dweff, const float* __restrict__ W,
                                                            const int* deg, int P, int J, long E, float* part) {
  gconv_dA_part_body(dweff, W, deg, P, J, E, part, blockIdx.x, blockIdx.y, gridDim.y);
}

// The finish of the graph-conv weight / adjacency gradient with the conv bias pushed through A folded in, two
// launches instead of four (stgcn_gconv_wgrad_finish_bias).  Launch 1: blocks [0, nb_dw) the dW pass
// (overwriting), the rest the dA partial dots of (pair, chunk) = (b' / nch, b' % nch).
__global__ __launch_bounds__(256) void gconv_finish1_kernel(const float* __restrict__ dweff, const float* __restrict__ A,
                                                            const float* __restrict__ W, const int* nbr, const int* deg,
                                                            int P, int V, int J, long E, float* dW, int nb_dw, int nch,
                                                            float* part) {
  const int b = blockIdx.x;
  if (b < nb_dw) {
    gconv_dw_all_body(dweff, A, nbr, deg, P, V, J, E, dW, b, false);
  } else {
    const int b2 = b - nb_dw;
    gconv_dA_part_body(dweff, W, deg, P, J, E, part, b2 / nch, b2 % nch, nch);
  }
}

// Launch 2: blocks [0, P*V): (p, w) — every dA[p][v][w] written once: the support entries' chunk sums
// (fixed order) plus the bias term sum_c b[p][c] S[w][c] (v-independent; gcn_bias_bwd's value and order);
// blocks [P*V, ...): db[p*C + c] = sum_w colsum_p(A)[w] S[w][c] (gcn_bias_bwd's).
constexpr int FV_MAX = 32;
__global__ __launch_bounds__(256) void gconv_finish2_kernel(const float* __restrict__ part, const float* __restrict__ A,
                                                            const float* __restrict__ b, const float* __restrict__ S,
                                                            const int* nbr, const int* deg, int P, int V, int J, int C,
                                                            int nch, float* dA, float* db) {
  const int bx = blockIdx.x;
  if (bx < P * V) {
    const int p = bx / V, w = bx % V;
    float t = 0.f;
    for (int c = threadIdx.x; c < C; c += 256) t += b[p * C + c] * S[w * C + c];
    t = wave_sum(t);
    __shared__ float red[4];
    __shared__ float sup[FV_MAX];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = t;
    if (threadIdx.x < V) sup[threadIdx.x] = 0.f;
    __syncthreads();
    const float tot = ((red[0] + red[1]) + red[2]) + red[3];
    if (threadIdx.x < deg[w]) {  // the support entries of column w: chunk sums in order
      const int j = threadIdx.x, pair = w * J + j;
      float s = 0.f;
      for (int c = 0; c < nch; ++c) s += part[((long)pair * nch + c) * PMAX + p];
      sup[nbr[pair]] = s;
    }
    __syncthreads();
    for (int v = threadIdx.x; v < V; v += 256) dA[(p * V + v) * V + w] = sup[v] + tot;
    return;
  }
  __shared__ float cs[PMAX * FV_MAX];
  for (int i = threadIdx.x; i < P * V; i += 256) {
    const int p = i / V, w = i % V;
    float t = 0.f;
    for (int v = 0; v < V; ++v) t += A[(p * V + v) * V + w];
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

__global__ void gconv_dA_reduce_kernel(const float* __restrict__ part, const int* nbr, const int* deg, int P, int V,
                                       int J, int nch, float* dA) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;  // (pair, p)
  if (i >= V * J * P) return;
  const int pair = i / P, p = i % P, w = pair / J, j = pair % J;
  if (j >= deg[w]) return;
  float s = 0.f;
  for (int c = 0; c < nch; ++c) s += part[((long)pair * nch + c) * PMAX + p];
  dA[((long)p * V + nbr[w * J + j]) * V + w] += s;
}

// joint-grouped plan (gconv_wgrad2_kernel): COB (output channels per block); 0 = not taken
int w2_cob(const stgcn_gconv_wgrad_desc& a) {
  if (a.J > J2 || a.Cin % 64 || a.Cout % 64) return 0;
  // COB = 64: 32-row tiles, 48 KB of LDS, three 4-wave blocks per CU.  Measured against COB = 128 (64-row
  // tiles, one 8-wave block per CU): C=128 78 vs 85 us, C=256 143 vs 153 us, equal at 64 -> 128; and
  // 56 vs 72 us (per-pair kernel) at C = 64.
  return 64;
}

// the DMA-ring kernel (gconv_wgrad3) for COB = 64, except 64 -> 128 channels, where the register-staged
// kernel measured 74 vs 82 us
bool w3_ok(const stgcn_gconv_wgrad_desc& a) { return !(a.Cin == 64 && a.Cout == 128); }

// DMA-ring block target once a joint has several channel groups: 512 at C = 128 (100 groups: R = 6, 67 + 12 us
// with the slab reduction, against 87 + 9 at R = 3), 256 from 200 groups up (128 -> 256: R = 2, 114 + 13 us vs
// 127 + 15 at R = 3; C = 256: R = 1).  A plan with R = 1 (one row range per block) writes dWeff and the row
// sums directly, with no slab and no reduction launch (C = 256: 114-123 us vs 117 + 25 us at R = 2)
// STGCN_W3_DEEP (A/B build flag): the direct plans with 160 KB of LDS, one block per CU and a deeper ring —
// measured slower in the step (8.09 vs 8.01 ms, 3 interleaved runs), off
#ifndef STGCN_W3_DEEP
#define STGCN_W3_DEEP 0
#endif
#ifndef STGCN_W3_WIDE_TARGET
#define STGCN_W3_WIDE_TARGET 256
#endif
WGG wplan2(const stgcn_gconv_wgrad_desc& a, int cob) {
  WGG g{};
  g.ntile = (a.NT + w2m(cob) - 1) / w2m(cob);
  g.nco = a.Cout / cob;
  g.nci = a.Cin / 64;
  const long groups = (long)a.V * g.nco * g.nci;
  const long target = cob == 64 ? 512 : 256;  // COB 64: 3 register-staged / 2 DMA-ring blocks fit a CU
  // DMA ring: block target by the group count, measured per layer (targets 512 / 1024 / 2048): C = 64
  // (25 groups) 49 / 40 / 56 us, C = 128 64 / 81 / 75 us, C = 256 108 / 113 / 130 us
#ifndef STGCN_W3_NARROW_TARGET
#define STGCN_W3_NARROW_TARGET 1024
#endif
  const long t3 = groups <= 32 ? STGCN_W3_NARROW_TARGET : groups < 200 ? 512 : STGCN_W3_WIDE_TARGET;
  long R = (cob == 64 && w3_ok(a)) ? (t3 + groups - 1) / groups : (target + groups - 1) / groups;
  if (R > g.ntile) R = g.ntile;
  if (R < 1) R = 1;
  g.tpb = (int)((g.ntile + R - 1) / R);
  g.R = (g.ntile + g.tpb - 1) / g.tpb;
  return g;
}

// taken where the machine fills with at most 2 row parts (C = 256: 100 groups; tools/bench_conv.py, us, wide vs the
// 64 x 64 plans: C = 256 98.7 vs 101.5; with more parts the last arriver's serial merge of R partials dominates:
// C = 128 (R = 8) 162 vs 73.5, 128 -> 256 (R = 4) 156 vs 126)
bool w3w_ok(const stgcn_gconv_wgrad_desc& a) {
  if (!STGCN_W3W || a.Cin % 128 || a.Cout % 128 || a.V > 64 || a.J > 2 * W3W_JE) return false;
  const long groups = (long)a.V * (a.Cout / 128) * (a.Cin / 128);
  return STGCN_W3W_TARGET / groups <= 2;
}
WGG wplan3w(const stgcn_gconv_wgrad_desc& a) {
  WGG g{};
  g.ntile = (a.NT + 31) / 32;
  g.nco = a.Cout / 128;
  g.nci = a.Cin / 128;
  const long groups = (long)a.V * g.nco * g.nci;
  long R = STGCN_W3W_TARGET / groups;
  if (R > g.ntile) R = g.ntile;
  if (R < 1) R = 1;
  g.tpb = (int)((g.ntile + R - 1) / R);
  g.R = (g.ntile + g.tpb - 1) / g.tpb;
  return g;
}
// wide plan workspace: part partials [2V entries][ngrp][R][3*16384 + 128] floats, then the arrival counters [2V*ngrp]
long w3w_part_floats(const stgcn_gconv_wgrad_desc& a, const WGG& g) {
  return g.R > 1 ? 2L * a.V * g.nco * g.nci * g.R * ((long)W3W_JE * W3W_PSZ_J + 128) : 0;
}
long w3w_cnt_bytes(const stgcn_gconv_wgrad_desc& a, const WGG& g) {
  return g.R > 1 ? ((2L * a.V * g.nco * g.nci * 4) + 15) / 16 * 16 : 0;
}

WGG wplan(const stgcn_gconv_wgrad_desc& a) {
  WGG g{};
  g.ntile = (a.NT + WKM - 1) / WKM;
  g.nco = (a.Cout + 63) / 64;
  g.nci = (a.Cin + 63) / 64;
  long used = 0;
  // blocks of unused pairs exit at once; size R by the used pairs (<= V*J)
  used = (long)a.V * a.J;
  const long groups = used * g.nco * g.nci;
  long R = (1024 + groups - 1) / groups;
  if (R > g.ntile) R = g.ntile;
  if (R < 1) R = 1;
  g.tpb = (int)((g.ntile + R - 1) / R);
  g.R = (g.ntile + g.tpb - 1) / g.tpb;
  return g;
}

}  // namespace

long gconv_row_blocks(int NT, int V) { return (long)((NT + 127) / 128) * V; }

int gconv_launch(const stgcn_gconv_desc& a, int dtype, hipStream_t s) {
  // column tile: 64 for Cout <= 64, else 128 (weights padded accordingly by stgcn_gconv_weights)
  const bool wide = a.Cout > 64;
  // bf16, Cout <= 64: 128-row tiles (TM = 1, TN = 2) — twice the blocks of the 256-row tile, measured
  // 46 vs 54 us (C=64 fwd), 42 vs 47 us (dgrad), 68 vs 72 us (128 -> 64 dgrad); wider outputs keep
  // 256 x 128 tiles (128-row variants measured 5-10 % slower there)
  // K chunk of 64 channels (one barrier per 64 instead of 32) once Cin >= 128, with 128-row tiles at the
  // wide outputs (tools/bench_conv.py gconv, us, 32-chunk -> 64-chunk: fwd C=128 63 -> 56.5, C=256 96.5 ->
  // 92; dgrad 128 -> 64 67 -> 55; at Cin = 64 the 32-chunk tiles stay ahead or even)
  if (dtype == 1) {
    // DMA K loop (two LDS stages, 64-channel chunks) whenever rows allow it: tools/bench_conv.py gconv, us,
    // register-staged -> DMA: C=64 fwd 44.7 -> 42.7, dgrad 40.7 -> 36.6; C=128 59.8 -> 56.0 / 51.8 -> 48.9;
    // 64->128 69.8 -> 67.2 / 58.2 -> 49.8; C=256 (256-row tiles) 95.7 -> 85.2 / 88.1 -> 75.2
    const bool dma = a.Cin % 64 == 0 && a.Cin == a.Cin_pad && a.in_ld % 8 == 0;
    if (dma) {
      if (!wide) return launch_gconv<bf16, 4, 1, 1, 2, 64, GCONV_NSTG_N>(a, s);
      return a.Cin >= 256 ? launch_gconv<bf16, 4, 2, GCONV_TM_W, 2, 64, GCONV_NSTG_W>(a, s)
                          : launch_gconv<bf16, 4, 2, GCONV_TM_M, 2, 64, GCONV_NSTG_M>(a, s);
    }
    const bool k64 = a.Cin >= 128 && a.Cin_pad % 64 == 0;
    if (wide) return k64 ? launch_gconv<bf16, 4, 2, 1, 2, 64>(a, s) : launch_gconv<bf16, 4, 2, 2, 2, 32>(a, s);
    return k64 ? launch_gconv<bf16, 4, 1, 1, 2, 64>(a, s) : launch_gconv<bf16, 4, 1, 1, 2, 32>(a, s);
  }
  return wide ? launch_gconv<float, 4, 2, 2, 2, 16>(a, s) : launch_gconv<float, 4, 1, 2, 2, 16>(a, s);
}

int gconv_weights_launch(const float* A, const float* W, const int* nbr, const int* deg, int P, int V, int J, int Cout,
                         int Cin, int trans, void* out, int R_pad, int C_pad, int dtype, hipStream_t s,
                         const float* bconv, float* bias2d) {
  if (C_pad % 8 || P > GW_PMAX || (bconv && P * V > GW_COLSUM_MAX)) return STGCN_EBADSHAPE;
  const long total = (long)V * R_pad * (C_pad / 8);
  const unsigned blocks = (unsigned)((total + 255) / 256);
  if (dtype == 1)
    hipLaunchKernelGGL(gconv_weights_kernel<bf16>, dim3(blocks), dim3(256), 0, s, A, W, nbr, deg, P, V, J, Cout, Cin,
                       trans, (bf16*)out, R_pad, C_pad, bconv, bias2d);
  else
    hipLaunchKernelGGL(gconv_weights_kernel<float>, dim3(blocks), dim3(256), 0, s, A, W, nbr, deg, P, V, J, Cout,
                       Cin, trans, (float*)out, R_pad, C_pad, bconv, bias2d);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

// the degree-balanced direct plan's workspace: half partials [V][ngrp][2][J*4096 + 64] floats, then the arrival
// counters [V*ngrp] (16-B padded)
long w3_split_part_floats(const stgcn_gconv_wgrad_desc& a, const WGG& g) {
  return (long)a.V * g.nco * g.nci * 2 * ((long)a.J * 4096 + 64);
}
long w3_split_cnt_bytes(const stgcn_gconv_wgrad_desc& a, const WGG& g) {
  return (((long)a.V * g.nco * g.nci * 4) + 15) / 16 * 16;
}

long gconv_wgrad_workspace(const stgcn_gconv_wgrad_desc& a, int dtype) {
  if (dtype != 1) return 0;
  const int cob = w2_cob(a);
  if (cob && w3w_ok(a)) {
    const WGG g = wplan3w(a);
    return w3w_part_floats(a, g) * (long)sizeof(float) + w3w_cnt_bytes(a, g);
  }
  const WGG g = cob ? wplan2(a, cob) : wplan(a);
  if (cob && w3_ok(a) && g.R == 1)  // direct
    return STGCN_W3_SPLIT ? w3_split_part_floats(a, g) * (long)sizeof(float) + w3_split_cnt_bytes(a, g) : 0;
  if (cob && a.rowsum)
    return ((long)g.R * a.V * a.J * a.Cout * a.Cin + (long)g.R * a.V * a.Cout) * (long)sizeof(float);
  return (long)g.R * a.V * a.J * a.Cout * a.Cin * (long)sizeof(float);
}

int gconv_wgrad_launch(const stgcn_gconv_wgrad_desc& a, int dtype, hipStream_t s) {
  const long E = (long)a.V * a.J * a.Cout * a.Cin;
  if (a.phase < 0 || a.phase > 2) return STGCN_EBADSHAPE;
  if (dtype != 1) {
    if (a.phase == 2) return STGCN_OK;  // one kernel, run in phase 1
    hipLaunchKernelGGL(gconv_wgrad_f32_kernel, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, s, a);
    return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
  }
  if (a.Cin % 8 || a.Cout % 8 || a.x_ld % 8 || a.dy_ld % 8) return STGCN_EBADSHAPE;
  const int cob = w2_cob(a);
  if (cob && w3w_ok(a)) {  // wide plan: direct, row parts merged in-kernel
    if (a.phase == 2) return STGCN_OK;
    WGG g = wplan3w(a);
    g.slab = a.dweff;
    g.rowpart = a.rowsum;
    g.zero_unused = 1;
    if (g.R > 1) {
      const long pf = w3w_part_floats(a, g), cb = w3w_cnt_bytes(a, g);
      if (!a.work || a.work_bytes < pf * (long)sizeof(float) + cb) return STGCN_EBADSHAPE;
      g.part = reinterpret_cast<float*>(a.work);
      g.cnt = reinterpret_cast<unsigned*>(g.part + pf);
      if (hipMemsetAsync(g.cnt, 0, (size_t)cb, s) != hipSuccess) return STGCN_EHIP;
    }
    if (stgcn_lds_attr((const void*)gconv_wgrad3w_kernel, W3W_LDS, s)) return STGCN_EHIP;
    const long blocks = 2L * a.V * g.nco * g.nci * g.R;
    hipLaunchKernelGGL(gconv_wgrad3w_kernel, dim3((unsigned)blocks), dim3(256), W3W_LDS, s, a, g);
    return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
  }
  if (cob) {
    WGG g = wplan2(a, cob);
    const bool ring = cob == 64 && w3_ok(a);
    const bool direct = ring && g.R == 1;  // the only row range: partials are the result
    const long need = (long)g.R * E + (a.rowsum ? (long)g.R * a.V * a.Cout : 0);
    if (direct) {
      g.slab = a.dweff;
      g.rowpart = a.rowsum;
      g.zero_unused = 1;
      if (STGCN_W3_SPLIT) {  // degree-balanced: half partials + counters in the workspace, counters zeroed per launch
        const long pf = w3_split_part_floats(a, g), cb = w3_split_cnt_bytes(a, g);
        if (!a.work || a.work_bytes < pf * (long)sizeof(float) + cb) return STGCN_EBADSHAPE;
        g.part = reinterpret_cast<float*>(a.work);
        g.cnt = reinterpret_cast<unsigned*>(g.part + pf);
        if (a.phase != 2 && hipMemsetAsync(g.cnt, 0, (size_t)cb, s) != hipSuccess) return STGCN_EHIP;
      }
    } else {
      if (!a.work || a.work_bytes < need * (long)sizeof(float)) return STGCN_EBADSHAPE;
      g.slab = reinterpret_cast<float*>(a.work);
      g.rowpart = a.rowsum ? g.slab + (long)g.R * E : nullptr;
    }
    const bool deep = (direct || STGCN_W3_DEEP > 1) && STGCN_W3_DEEP;  // one block per CU, deeper ring
    const size_t lds = ring ? (size_t)(deep ? 160 : 80) * 1024 : 2 * (size_t)(cob / 32 + 2 * J2) * w2m(cob) * WPR;
    auto* k = ring ? (deep ? gconv_wgrad3_kernel<160 * 1024> : gconv_wgrad3_kernel<80 * 1024>) : gconv_wgrad2_kernel<64>;
    if (stgcn_lds_attr((const void*)k, 160 * 1024, s)) return STGCN_EHIP;
    const long blocks = (long)a.V * g.nco * g.nci * g.R * (g.part ? 2 : 1);
    if (a.phase != 2) hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(ring ? 256 : cob / 16 * 64), lds, s, a, g);
    if (direct || a.phase == 1) return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
    if (a.rowsum) {  // slab reduction and row sums in one launch
      const long ER = (long)a.V * a.Cout;
      const int nb1 = (int)((E + 255) / 256);
      hipLaunchKernelGGL(gslab_rowpart_kernel, dim3((unsigned)(nb1 + (ER + 255) / 256)), dim3(256), 0, s,
                         (const float*)g.slab, g.R, E, (long)a.Cout * a.Cin, a.deg, a.J, a.dweff, nb1,
                         (const float*)g.rowpart, ER, a.rowsum);
    } else {
      hipLaunchKernelGGL(gslab_reduce_kernel, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, s, (const float*)g.slab,
                         g.R, E, (long)a.Cout * a.Cin, a.deg, a.J, a.dweff);
    }
    return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
  }
  if (a.rowsum) return STGCN_EBADSHAPE;  // row sums ride only on the joint-grouped kernel
  WGG g = wplan(a);
  if (!a.work || a.work_bytes < (long)g.R * E * (long)sizeof(float)) return STGCN_EBADSHAPE;
  g.slab = reinterpret_cast<float*>(a.work);
  if (stgcn_lds_attr((const void*)gconv_wgrad_kernel, 160 * 1024, s)) return STGCN_EHIP;
  const long blocks = (long)a.V * a.J * g.nco * g.nci * g.R;
  const size_t lds = 2 * 4 * WKM * WPR;  // >= the 48 KB cross-wave reduction buffer
  if (a.phase != 2) hipLaunchKernelGGL(gconv_wgrad_kernel, dim3((unsigned)blocks), dim3(256), lds, s, a, g);
  if (a.phase == 1) return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
  hipLaunchKernelGGL(gslab_reduce_kernel, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, s, (const float*)g.slab,
                     g.R, E, (long)a.Cout * a.Cin, a.deg, a.J, a.dweff);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

long gconv_wgrad_finish_workspace(int P, int V, int J, int Cout, int Cin) {
  const long E = (long)Cout * Cin;
  return P > PMAX ? 0 : (long)V * J * ((E + DA_CHUNK - 1) / DA_CHUNK) * PMAX * (long)sizeof(float);
}

bool gconv_finish_bias_ok(int P, int V, int J) { return P <= PMAX && V <= FV_MAX && V * J <= DW_PAIRS; }
// the one-pass dW and the chunked dA read dWeff / W as float4 (Cout * Cin % 4 == 0)

int gconv_wgrad_finish_bias_launch(const float* dweff, const float* A, const float* W, const int* nbr, const int* deg,
                                   int P, int V, int J, int Cout, int Cin, const float* bconv, const float* S, float* dW,
                                   float* dA, float* db, void* work, hipStream_t s) {
  if (!gconv_finish_bias_ok(P, V, J) || !work || ((long)Cout * Cin) % 4) return STGCN_EBADSHAPE;
  const long E = (long)Cout * Cin;
  const int nch = (int)((E + DA_CHUNK - 1) / DA_CHUNK);
  const int nb_dw = (int)((E + 255) / 256);  // 256 columns per dW block
  float* part = reinterpret_cast<float*>(work);
  hipLaunchKernelGGL(gconv_finish1_kernel, dim3((unsigned)(nb_dw + V * J * nch)), dim3(256), 0, s, dweff, A, W, nbr,
                     deg, P, V, J, E, dW, nb_dw, nch, part);
  hipLaunchKernelGGL(gconv_finish2_kernel, dim3((unsigned)(P * V + (P * Cout + 255) / 256)), dim3(256), 0, s,
                     (const float*)part, A, bconv, S, nbr, deg, P, V, J, Cout, nch, dA, db);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

int gconv_wgrad_finish_launch(const float* dweff, const float* A, const float* W, const int* nbr, const int* deg,
                              int P, int V, int J, int Cout, int Cin, float* dW, float* dA, void* work, hipStream_t s) {
  const long E = (long)Cout * Cin;
  if (P > PMAX || (dA && !work) || V * J > DW_PAIRS || E % 4) {  // generic per-partition path (dA per (pair,p) block)
    const long n = (long)P * E;
    if (dW)
      hipLaunchKernelGGL(gconv_dw_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, dweff, A, nbr, deg, P,
                         V, J, Cout, Cin, dW);
    if (dA)
      hipLaunchKernelGGL(gconv_dA_kernel, dim3((unsigned)(V * J), (unsigned)P), dim3(256), 0, s, dweff, W, nbr, deg,
                         P, V, J, Cout, Cin, dA);
  } else {  // one pass over dWeff per output, all partitions at once
    if (dW)
      hipLaunchKernelGGL(gconv_dw_all_kernel, dim3((unsigned)((E + 255) / 256)), dim3(256), 0, s, dweff, A, nbr, deg,
                         P, V, J, E, dW);
    if (dA) {
      const int nch = (int)((E + DA_CHUNK - 1) / DA_CHUNK);
      float* part = reinterpret_cast<float*>(work);
      hipLaunchKernelGGL(gconv_dA_part_kernel, dim3((unsigned)(V * J), (unsigned)nch), dim3(256), 0, s, dweff, W,
                         deg, P, J, E, part);
      hipLaunchKernelGGL(gconv_dA_reduce_kernel, dim3((unsigned)((V * J * P + 255) / 256)), dim3(256), 0, s, part,
                         nbr, deg, P, V, J, nch, dA);
    }
  }
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
