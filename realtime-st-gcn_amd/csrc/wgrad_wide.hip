// Weight gradient of the Kt = 9, stride-1 temporal convs with >= 128 output channels (bf16): the
// convolution_backward weight path of tcn.2 (stgcn.py:154-159, the reference's top CPU op) at the
// config-2 layer 4, 5, 7, 8 shapes.
//
//   dW[dt][co][ci] += sum_m dY[m][co] * pro(in[m + (dt - 4) V][ci])        (rows m of one sample)
//
// A GEMM with M = co, N = (dt, ci), K = output rows.  wgrad_tile.hip gives each block a 64-co x 32-ci
// output block, so every dY element is staged Cin/32 times and the input halo of 5+8 frames is
// staged for every 5-frame tile (2.6x).  Here:
//   * a block (8 waves, two per SIMD) owns a 128-co x 64-ci x 9-tap output block (wave (wc, wi):
//     32 co x 32 ci x 9 taps = 9 accumulators of 32 x 32) and walks a contiguous range of tiles of
//     F = floor(128 / V) frames (5 at V = 25): dY is staged Cin/64 times, the input Cout/128 times;
//   * the input lives in a frame RING of RS = 2F + 8 slots plus a MIRROR of its first F + 7 slots
//     (every frame written to slot f mod RS, and again to slot f mod RS + RS when that is < RS + F + 7):
//     a tile's window (frames f0-4 .. f0+F+3) is then always LDS-contiguous, the next tile's F new
//     frames land in slots the current tile does not read, and each input frame is staged (BatchNorm1
//     scale/shift + ReLU prologue applied, zero frames outside [0, T)) exactly once per block, with
//     one barrier per tile;
//   * both operands are read with the transposing ds_read_b64_tr_b16 from 32-channel panels of 64-B
//     rows (8 consecutive K rows per lane), the input fragment of tap dt at a uniform offset dt*V rows;
//     fragments are read two tap-steps ahead of their MFMAs;
//   * the next tile's dY rows and new frames are loaded into registers while the current tile computes;
//   * the fp32 block result goes to a slab [range][9][Cout][Cin], summed deterministically into dW by
//     slab_reduce (wgrad_tile.hip).
#include "common.h"
#include "../../include/stgcn_amd.h"
#include <stdlib.h>
#include <utility>

namespace {

constexpr int NT = 512;              // 8 waves
constexpr int KM = 128;              // K rows per tile (F*V <= 128, rest zero rows)
constexpr int PR = 64;               // bytes per panel row (32 bf16 channels)
constexpr int COB = 128, CIB = 64;   // output block
constexpr int DY_PANEL = KM * PR;    // 8 KB
constexpr int DY_BYTES = (COB / 32) * DY_PANEL;  // 32 KB per buffer
constexpr int DY_U = KM * (COB / 8) / NT;        // 16-B dY units per thread per tile (4)
constexpr int X_U = (KM * (CIB / 8) + NT - 1) / NT;  // input units per thread per batch of <= 128 rows (2)
constexpr int LDS_MAX = 160 * 1024;

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

template <int N, typename F>
DEV void static_for(F&& f) {
  [&]<int... I>(std::integer_sequence<int, I...>) { (f.template operator()<I>(), ...); }(
      std::make_integer_sequence<int, N>{});
}

DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// two ds_read_b64_tr_b16 (rows lo and lo + 4 of a 64-B-row panel) -> one MFMA fragment: lane
// (c = column, h) receives rows 8h .. 8h+7 of its column
DEV bf16x8 trpair(const char* lo) {
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)lo);
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(lo + 4 * PR));
  s16x8 v;
  v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
  v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
  return __builtin_bit_cast(bf16x8, v);
}

struct WWGeom {
  int F;         // output frames per tile
  int RS;        // ring slots (frames)
  int MS;        // ring + mirror slots
  int nco, nci;  // output blocks along co (128) and ci (64)
  int tiles_n;   // tiles per sample
  int tpb;       // tiles per block (contiguous range of the sample-major tile sequence)
  int R;         // row-range blocks per output block (slab count)
  int fold;      // 1: stride-2 conv folded into 5 taps over frame pairs (input channels 2*Cin, parity-major)
  int cin_f;     // input channels of the (folded) GEMM
  float* slab;   // [R][KTAP][Cout][cin_f]
};

template <int PRO, int KTAP>
__global__ __launch_bounds__(NT, 1) void wgrad_wide_kernel(const stgcn_wgrad_desc a, const WWGeom g) {
  constexpr int KT = KTAP, PADT = (KTAP - 1) / 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int V = a.V, F = g.F;
  const int XP = g.MS * V * PR;                 // bytes per input panel (ring + mirror)
  char* const sX = smem;                        // input panel p (ci 32p ..) at p * XP
  char* const sY = smem + 2 * XP;               // dY buffers [2][4 panels][KM rows]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wc = wave >> 1, wi = wave & 1;      // co tile (32), ci tile (32)
  {
    // Zero the whole LDS image first: the K-padding rows of a tap window and ring slots of frames never
    // staged are read as MFMA operands multiplied by zero dY rows, and LDS left by an earlier kernel
    // may hold NaN bit patterns (0 * NaN = NaN).
    uint4* z = reinterpret_cast<uint4*>(smem);
    const int nz = (2 * XP + 2 * DY_BYTES) / 16;
    for (int e = tid; e < nz; e += NT) z[e] = make_uint4(0, 0, 0, 0);
    __syncthreads();
  }
  const int ob = blockIdx.x % (g.nco * g.nci), rg = blockIdx.x / (g.nco * g.nci);
  const int co0 = (ob % g.nco) * COB, cf0 = (ob / g.nco) * CIB;  // cf0: folded input channel
  // fold: ring frame z holds input frame 2z + par of the source channels ci0 .. ci0+63
  const int par = g.fold ? cf0 / a.Cin : 0;
  const int ci0 = cf0 - par * a.Cin;
  const int fmul = g.fold ? 2 : 1;
  const int tiles_n = g.tiles_n;
  const int k_begin = rg * g.tpb, k_end = min(a.N * tiles_n, k_begin + g.tpb);

  const bf16* __restrict__ xin = reinterpret_cast<const bf16*>(a.in);
  const bf16* __restrict__ dy = reinterpret_cast<const bf16*>(a.dy);

  // ---- staging: dY unit (row tid/16 + 32 i, 8 co at 8*(tid%16)); input unit (row tid/8 + 64 i, 8 ci at 8*(tid%8))
  const int ycu = tid & 15, xcu = tid & 7;
  float sc[8], sh[8];
  if (PRO == 1) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = ci0 + xcu * 8 + j;
      sc[j] = c < a.Cin ? a.pro_a[c] : 0.f;
      sh[j] = c < a.Cin ? a.pro_b[c] : 0.f;
    }
  }
  // Two register sets: tile j's staged loads live in set j & 1, and tile j + 1's set goes to LDS at the end of
  // tile j.  5-tap (stride-2 folded) tiles have 40 k-steps, too few to cover one tile's load latency: there
  // tile j + 2's loads are issued at the start of tile j (AHEAD2).  The 9-tap tiles keep one tile ahead (a
  // second live set pushes them past 256 VGPRs).  Every load is unconditional (out-of-range rows clamp to an
  // in-bounds row and are zeroed at the LDS store), so the number of loads in flight is fixed and the vmcnt wait
  // before the store of set j+1 leaves tile j+2's loads pending.
  constexpr bool AHEAD2 = KT < 9;
  uint4 ry[2][DY_U], rx[2][X_U];
  const bool ycok = co0 + ycu * 8 < a.Cout, xcok = ci0 + xcu * 8 < a.Cin;
  const bf16* __restrict__ dyb = dy + co0 + (ycok ? ycu * 8 : 0);
  const bf16* __restrict__ xb = xin + ci0 + (xcok ? xcu * 8 : 0);
  auto load_dy = [&]<int S>(int n, int f0) {  // rows of output frames f0 .. f0+F-1 (f0 clamped into the sample)
    f0 = min(f0, a.T_out - 1);
    const int rows_valid = min(F, a.T_out - f0) * V;
    const bf16* base = dyb + ((long)n * a.T_out + f0) * V * a.dy_ld;
    static_for<DY_U>([&]<int i>() {
      const int r = (tid >> 4) + 32 * i;
      ry[S][i] = *reinterpret_cast<const uint4*>(base + (long)(r < rows_valid ? r : 0) * a.dy_ld);
    });
  };
  auto store_dy = [&]<int S>(int buf, int f0) {  // rows past T_out / F*V and channels past Cout: zero
    const int rows_valid = ycok ? min(F, a.T_out - f0) * V : 0;
    char* p = sY + buf * DY_BYTES + (ycu >> 2) * DY_PANEL + (ycu & 3) * 16;
    static_for<DY_U>([&]<int i>() {
      const int r = (tid >> 4) + 32 * i;
      *reinterpret_cast<uint4*>(p + r * PR) = r < rows_valid ? ry[S][i] : make_uint4(0, 0, 0, 0);
    });
  };
  // input frames [fa, fa + nf) of sample n (nf * V <= 128) -> register set S (source frames clamped into [0, T_in))
  auto load_x = [&]<int S>(int n, int fa, int nf) {
    static_for<X_U>([&]<int i>() {
      const int r = (tid >> 3) + 64 * i;
      const int rr = r < nf * V ? r : 0;
      const int fl = rr / V, v = rr - fl * V, f = fa + fl;
      const int fs = min(max(fmul * f + par, 0), a.T_in - 1);
      rx[S][i] = *reinterpret_cast<const uint4*>(xb + (((long)n * a.T_in + fs) * V + v) * a.in_ld);
    });
  };
  auto store_x = [&]<int S>(int fa, int nf) {  // slot f mod RS and its mirror; frames outside [0, T_in) zero
    static_for<X_U>([&]<int i>() {
      const int r = (tid >> 3) + 64 * i;
      if (r < nf * V) {
        const int fl = r / V, v = r - fl * V, f = fa + fl;
        const bool ok = xcok && f >= 0 && fmul * f + par < a.T_in;
        uint4 u = ok ? rx[S][i] : make_uint4(0, 0, 0, 0);
        if (PRO == 1 && ok) {
          float e[8];
          unpack16(u, e, (bf16*)nullptr);
#pragma unroll
          for (int j = 0; j < 8; ++j) e[j] = fmaxf(fmaf(e[j], sc[j], sh[j]), 0.f);
          u = pack16(e, (bf16*)nullptr);
        }
        int slot = f % g.RS;
        slot += slot < 0 ? g.RS : 0;
        char* p = sX + (xcu >> 2) * XP + (xcu & 3) * 16 + v * PR;
        *reinterpret_cast<uint4*>(p + slot * V * PR) = u;
        if (slot + g.RS < g.MS) *reinterpret_cast<uint4*>(p + (slot + g.RS) * V * PR) = u;
      }
    });
  };
  // the whole window of a range's / sample's first tile (F + 8 frames) in batches of F frames, through set S
  auto stage_window = [&]<int S>(int n, int f0) {
    for (int fb = f0 - PADT; fb < f0 + F + PADT; fb += F) {
      const int nf = min(F, f0 + F + PADT - fb);
      load_x.template operator()<S>(n, fb, nf);
      store_x.template operator()<S>(fb, nf);
    }
  };

  // ---- fragments: lane (i = lane&15, gq = lane>>4): row 8h + q (+4), column 16(gq&1) + 4p
  const int li = lane & 15, gq = lane >> 4;
  const int colb = (16 * (gq & 1) + 4 * (li & 3)) * 2;
  const int rlo = 8 * (gq >> 1) + (li >> 2);

  f32x16 acc[KT];
#pragma unroll
  for (int t = 0; t < KT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;

  // zero the input panels once: K padding rows of a tile read past the window (finite values needed)
  for (int o = tid * 16; o < 2 * XP; o += NT * 16) *reinterpret_cast<uint4*>(sX + o) = make_uint4(0, 0, 0, 0);
  __syncthreads();

  const int tapb = V * PR;  // bytes between taps
  const int nk = k_end - k_begin;
  auto tile = [&]<int S>(int j) {
    const int k = k_begin + j;
    const int n = k / tiles_n, tt = k - n * tiles_n, f0 = tt * F;
    const bool next1 = j + 1 < nk && tt + 1 < tiles_n;  // tile j+1: same sample (else it restages itself)
    if (tt == 0 || j == 0) {  // range/sample start: dY of this tile and the whole input window, then tile j+1's loads
      __syncthreads();
      load_dy.template operator()<S>(n, f0);
      store_dy.template operator()<S>(k & 1, f0);
      stage_window.template operator()<S>(n, f0);
      __syncthreads();
      if constexpr (AHEAD2) {
        load_dy.template operator()<S ^ 1>(n, f0 + F);
        load_x.template operator()<S ^ 1>(n, f0 + F + PADT, F);
      }
    }
    // loads of tile j+2 (two ahead) or j+1 (one ahead), always issued: past the sample / range they re-read
    // rows of this sample, unused
    if constexpr (AHEAD2) {
      load_dy.template operator()<S>(n, f0 + 2 * F);
      load_x.template operator()<S>(n, f0 + 2 * F + PADT, F);
    } else {
      load_dy.template operator()<S ^ 1>(n, f0 + F);
      load_x.template operator()<S ^ 1>(n, f0 + F + PADT, F);
    }
    // ---- compute tile j: NU tap-steps u = (ks, t), fragments read D steps ahead
    int s0 = (f0 - PADT) % g.RS;
    s0 += s0 < 0 ? g.RS : 0;
    const char* Y = sY + (k & 1) * DY_BYTES + wc * DY_PANEL + colb + rlo * PR;
    const char* X = sX + wi * XP + colb + (s0 * V + rlo) * PR;
    int tb = tapb;
    asm volatile("" : "+s"(tb));
    constexpr int NU = (KM / 16) * KT, D = 2;
    bf16x8 fx[D + 1], fy[2];
    auto rd = [&]<int u>() {
      constexpr int ks = u / KT, t = u % KT;
      if constexpr (t == 0) fy[ks & 1] = trpair(Y + 16 * ks * PR);
      fx[u % (D + 1)] = trpair(X + t * tb + 16 * ks * PR);
    };
    static_for<D>([&]<int u>() { rd.template operator()<u>(); });
    static_for<NU>([&]<int u>() {
      if constexpr (u + D < NU) rd.template operator()<u + D>();
      constexpr int ks = u / KT, t = u % KT;
      acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fy[ks & 1], fx[u % (D + 1)], acc[t], 0, 0, 0);
    });
    // ---- hand tile j+1's set to LDS (ring slots / dY buffer not read by tile j)
    if (next1) {
      store_dy.template operator()<S ^ 1>((k + 1) & 1, f0 + F);
      store_x.template operator()<S ^ 1>(f0 + F + PADT, F);
    }
    lds_barrier();
  };
  for (int j = 0; j < nk; j += 2) {
    tile.template operator()<0>(j);
    if (j + 1 < nk) tile.template operator()<1>(j + 1);
  }

  // ---- block partial -> slab [rg][t][co][ci]: lane holds ci = ci0 + 32 wi + (lane&31), co rows acc_row
  float* __restrict__ out = g.slab + (long)rg * KT * a.Cout * g.cin_f;
  const int ci = cf0 + 32 * wi + (lane & 31);
#pragma unroll
  for (int t = 0; t < KT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = co0 + 32 * wc + acc_row(r, lane);
      if (co < a.Cout && ci < g.cin_f) out[((long)t * a.Cout + co) * g.cin_f + ci] = acc[t][r];
    }
}

struct WPlan {
  bool ok;
  WWGeom g;
  int ktap;
  size_t lds;
  long slab_elems;
};

constexpr int RS_PART = 16;  // level-1 partials of slab_reduce

// level 2 of the folded reduction: dW[2t + par][co][ci] += sum_r part[r][t][co][par*Cin + ci]
// (mode 1: dw overwritten in the nn.Conv2d order [Cout][Cin][9])
__global__ void unfold_reduce2_kernel(const float* __restrict__ part, int RS, int Cout, int Cin, float* __restrict__ dw,
                                      int mode) {
  const long E4 = 5L * Cout * 2 * Cin / 4;
  const long e4 = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e4 >= E4) return;
  const long e = e4 * 4;
  const int cf = (int)(e % (2 * Cin));
  const long tc = e / (2 * Cin);
  const int co = (int)(tc % Cout), t = (int)(tc / Cout);
  const int par = cf / Cin, ci = cf - par * Cin, dt = 2 * t + par;
  if (dt > 8) return;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int r = 0; r < RS; ++r) {
    const float4 v = *reinterpret_cast<const float4*>(part + (long)r * 4 * E4 + e);
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  if (mode) {
    float* d = dw + ((long)co * Cin + ci) * 9 + dt;
    d[0] = acc.x;
    d[9] = acc.y;
    d[18] = acc.z;
    d[27] = acc.w;
    return;
  }
  float4* d = reinterpret_cast<float4*>(dw + ((long)dt * Cout + co) * Cin + ci);
  float4 o = *d;
  o.x += acc.x; o.y += acc.y; o.z += acc.z; o.w += acc.w;
  *d = o;
}

WPlan wplan(const stgcn_wgrad_desc& a) {
  WPlan p{};
  p.ok = false;
  if (a.Kt != 9 || a.pad != 4) return p;
  WWGeom& g = p.g;
  if (a.stride == 1 && a.T_in == a.T_out) {
    g.fold = 0;
    p.ktap = 9;
    g.cin_f = a.Cin;
  } else if (a.stride == 2 && a.T_out == (a.T_in - 1) / 2 + 1 && a.Cin % CIB == 0) {
    // dW[2t + par][co][ci] = sum_f dY[f][co] x[2(f + t - 2) + par][ci]: a 5-tap weight gradient over
    // frame pairs (input channels parity-major, 2*Cin), unfolded by the final reduction
    g.fold = 1;
    p.ktap = 5;
    g.cin_f = 2 * a.Cin;
  } else {
    return p;
  }
  if (a.pro != 0 && a.pro != 1) return p;
  if (a.Cout < COB || a.Cin < CIB || a.Cout % 8 || a.Cin % 8 || a.in_ld % 8 || a.dy_ld % 8 || a.V > 32) return p;
  const int padt = (p.ktap - 1) / 2;
  g.F = KM / a.V;
  g.RS = 2 * g.F + 2 * padt;
  g.MS = g.RS + g.F + 2 * padt - 1;  // a window starting at slot RS-1 ends at slot MS-1
  if (g.F < 1 || g.F * a.V > KM || g.F * a.V > 64 * X_U) return p;
  g.nco = (a.Cout + COB - 1) / COB;
  g.nci = (g.cin_f + CIB - 1) / CIB;
  const int nob = g.nco * g.nci;
  g.tiles_n = (a.T_out + g.F - 1) / g.F;
  const long total = (long)a.N * g.tiles_n;
  if (total > 0x7fffffffL) return p;
  // one block per CU (LDS): split the tile sequence so that nob * R ~ 256 blocks
  int R = 256 / nob;
  if (R < 1) R = 1;
  if (R > total) R = (int)total;
  g.tpb = (int)((total + R - 1) / R);
  g.R = (int)((total + g.tpb - 1) / g.tpb);
  // K padding rows of the window's last tap read up to KM - F*V rows past slot MS: keep them inside
  // the allocation (they land in the dY buffers; finite, multiplied by zero dY rows)
  p.lds = 2 * (size_t)g.MS * a.V * PR + 2 * (size_t)DY_BYTES;
  if (p.lds > LDS_MAX || (size_t)(KM - g.F * a.V) * PR > 2 * (size_t)DY_BYTES) return p;
  p.slab_elems = (long)(g.R + RS_PART) * p.ktap * a.Cout * g.cin_f;
  p.ok = true;
  return p;
}

}  // namespace

int slab_reduce_launch(const float* slab, int R, long E, float* part, float* dw, hipStream_t s, int mode, int Kt,
                       long CoCi);
int slab_reduce1_launch(const float* slab, int R, long E, float* part, hipStream_t s);

long wgrad_wide_workspace(const stgcn_wgrad_desc& a, int dtype) {
  if (dtype != 1) return 0;
  const WPlan p = wplan(a);
  return p.ok ? p.slab_elems * (long)sizeof(float) : 0;
}

// -1: not handled here
int wgrad_wide_launch(const stgcn_wgrad_desc& a, int dtype, hipStream_t s) {
  if (dtype != 1 || a.work == nullptr) return -1;
  WPlan p = wplan(a);
  if (!p.ok || a.work_bytes < p.slab_elems * (long)sizeof(float)) return -1;
  p.g.slab = reinterpret_cast<float*>(a.work);
  auto* k = p.ktap == 9 ? (a.pro == 1 ? wgrad_wide_kernel<1, 9> : wgrad_wide_kernel<0, 9>)
                        : (a.pro == 1 ? wgrad_wide_kernel<1, 5> : wgrad_wide_kernel<0, 5>);
  if (stgcn_lds_attr((const void*)k, LDS_MAX, s)) return STGCN_EHIP;
  const unsigned grid = (unsigned)(p.g.nco * p.g.nci * p.g.R);
  hipLaunchKernelGGL(k, dim3(grid), dim3(NT), p.lds, s, a, p.g);
  if (hipGetLastError() != hipSuccess) return STGCN_EHIP;
  const long E = (long)p.ktap * a.Cout * p.g.cin_f;
  float* part = p.g.slab + (long)p.g.R * E;
  if (!p.g.fold) return slab_reduce_launch(p.g.slab, p.g.R, E, part, a.dw, s, a.out_mode, 9, (long)a.Cout * a.Cin);
  const int RS = slab_reduce1_launch(p.g.slab, p.g.R, E, part, s);
  if (RS < 0) return -RS;
  hipLaunchKernelGGL(unfold_reduce2_kernel, dim3((unsigned)((E / 4 + 255) / 256)), dim3(256), 0, s, (const float*)part,
                     RS, a.Cout, a.Cin, a.dw, a.out_mode);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
