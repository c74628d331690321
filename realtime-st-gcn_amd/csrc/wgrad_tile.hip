// Frame-tiled weight gradient (v2, bf16) of the (Kt x 1) row convolutions — fast path of
// stgcn_conv_wgrad (conv_wgrad.hip keeps the fp32 parity path and the shapes not covered here).
//
//   dW[dt][co][ci] += sum_m dY[m, co] * pro(in[src(m, dt), ci])      (convolution_backward weight
//   path of stgcn.py:154-170, the reference's top CPU op)
//
// Per tap this is a GEMM with K = output rows.  A block owns one (64-co x 32*NB-ci) output block
// and a contiguous range of row tiles (F frames of one sample, or 128 flat rows for 1x1 convs).
// For each tile it stages
//   * dY rows [KM x 64 co] (rows past the tile's valid frames zeroed: they must not contribute),
//   * the input halo once for all taps (prologue BatchNorm/LayerNorm + ReLU applied while staging;
//     frames outside [0, T_in) = zero padding).  Stride 2 stores the halo split by frame parity so
//     that every tap reads a contiguous row range: tap dt -> parity dt%S, shift (dt/S)*V rows,
// as 32-channel panels of 64-B rows, which the gfx950 transposing read ds_read_b64_tr_b16 turns
// into MFMA fragments (8 consecutive rows per lane) bank-conflict free.  Each wave accumulates
// TW taps x NBW ci-tiles of 32x32 in registers across all of its block's tiles (the dY fragment
// is reused by every tap), so the only output traffic is one fp32 partial per block: written to a
// workspace slab with plain stores, then summed deterministically into dW by a second kernel.
#include "common.h"
#include <stdlib.h>
#include "../../include/stgcn_amd.h"

namespace {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int KM = 128;      // rows (K) per tile
constexpr int PR = 64;       // bytes per panel row (32 bf16 channels)

// MFMA operand fragment from a [rows][32] bf16 panel: lane (c = lane&31, h = lane>>5) gets
// panel[row0 + 8h + j][c], j = 0..7, via two ds_read_b64_tr_b16 (4 rows each).
DEV bf16x8 trfrag(const char* panel, int row0, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const int q = i >> 2, p = i & 3, h = g >> 1;
  const char* a0 = panel + (row0 + 8 * h + q) * PR + (16 * (g & 1) + 4 * p) * 2;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 4 * PR));
  s16x8 v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return __builtin_bit_cast(bf16x8, v);
}

struct WGeom {
  int F;          // frames per tile (0 = flat)
  int tiles_n;    // tiles per sample (framed) / total tiles (flat)
  int ntiles;     // total tiles
  int tpb;        // tiles per block
  int HRS;        // halo rows per parity block
  int nco, nci;   // output blocks along co (64) and ci (32*NB)
  int R;          // row-range blocks per output block
  float* slab;    // [R][nco*nci blocks] partials laid out as [R][Kt][Cout][Cin]
};

// TW taps per wave, NB ci panels per block, NBW ci tiles per wave
template <int KT, int S, int NB, int TW, int NBW, bool LN>
__global__ __launch_bounds__(256, LN ? 1 : 2) void wgrad_tile_kernel(const stgcn_wgrad_desc a, const WGeom g) {
  constexpr int HR_MAX = KM + ((KT - 1) / S) * 32;       // V <= 32
  constexpr int DY_UNITS = KM * 8;                        // 2 panels x 4 units per row
  constexpr int DY_PT = DY_UNITS / 256;
  constexpr int X_UPR = NB * 4;                           // units per halo row
  constexpr int SP = KT >= S ? S : 1;                     // parity blocks actually read
  constexpr int X_PT = (SP * HR_MAX * X_UPR + 255) / 256;
  static_assert(DY_UNITS % 256 == 0, "dy units");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int DY_BYTES = 2 * KM * PR;
  const int XP_BYTES = SP * g.HRS * PR;                   // one ci panel, all parities
  const int STAGE = DY_BYTES + NB * XP_BYTES;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int V = a.V;
  const int ob = blockIdx.x % (g.nco * g.nci), rr = blockIdx.x / (g.nco * g.nci);
  const int co0 = (ob % g.nco) * 64, ci0 = (ob / g.nco) * (32 * NB);
  const int t_begin = rr * g.tpb, t_end = min(g.ntiles, t_begin + g.tpb);

  // wave -> (co tile, taps [tw0, tw1), ci tiles [bw0, bw0 + NBW))
  const int wa = wave & 1;
  int tw0, tw1, bw0;
  if (KT > 1) {
    tw0 = (wave >> 1) * TW;
    tw1 = min(KT, tw0 + TW);
    bw0 = 0;
  } else {
    tw0 = 0;
    tw1 = 1;
    bw0 = (wave >> 1) * NBW;
  }

  const bf16* __restrict__ in = reinterpret_cast<const bf16*>(a.in);
  const bf16* __restrict__ dy = reinterpret_cast<const bf16*>(a.dy);

  // thread-fixed channel of its staging units (unit column = tid % units-per-row)
  const int dy_u = tid & 7;                  // dy: 8 units per row (co0 + 8*dy_u)
  const int x_u = tid % X_UPR;               // halo: X_UPR units per row
  const int x_ci = ci0 + x_u * 8;
  // BatchNorm prologue scale / shift of the block's 32*NB input channels in LDS after the two stages (read at
  // each halo store instead of held in 16 registers for the whole kernel)
  float* const sScSh = reinterpret_cast<float*>(smem + 2 * STAGE);  // [2][32 * NB]
  if (a.pro == 1 && tid < 32 * NB) {
    const int c = ci0 + tid;
    sScSh[tid] = c < a.Cin ? a.pro_a[c] : 0.f;
    sScSh[32 * NB + tid] = c < a.Cin ? a.pro_b[c] : 0.f;
  }
  // the first tile's halo store below reads the table from every wave: without this barrier the waves past
  // the writers read whatever the CU's previous workgroup left in that LDS (intermittent garbage gradients,
  // seen when two processes share the GPU: config-4 DDP test)
  __syncthreads();

  // tile-invariant part of each halo unit: frame offset from the tile's first halo frame (fo, -1 = unused unit)
  // and joint (v < 32), packed as fo * 32 + v (registers: two staged sets are live in the tile loop)
  int x_fv[X_PT];
#pragma unroll
  for (int i = 0; i < X_PT; ++i) {
    const int prow = (tid + i * 256) / X_UPR;
    const int par = prow / g.HRS, j = prow - par * g.HRS;
    if (prow >= SP * g.HRS) {
      x_fv[i] = -32;
    } else if (g.F) {
      const int fl = j / V;
      x_fv[i] = (S * fl + par) * 32 + (j - fl * V);
    } else {
      x_fv[i] = j * 32;  // flat: row within the tile
    }
  }
  auto x_fo = [&](int i) { return x_fv[i] >> 5; };
  auto x_v = [&](int i) { return x_fv[i] & 31; };

  // Two register sets of staged loads: tile j's in set j & 1, tile j + 1's set goes to LDS at the end of tile j;
  // with AHEAD2 (below) tile j + 2's loads are issued at the start of tile j.  Loads are unconditional (invalid units read an in-bounds row of
  // the same sample and are zeroed at the store through a per-set validity mask), so the count in flight is
  // fixed and the wait before storing set j+1 leaves tile j+2's loads pending.
  static_assert(DY_PT + X_PT <= 32, "validity mask");
  uint4 ry[2][DY_PT], rx[2][X_PT];
  int rxs[2][X_PT];  // input frame n*T_in + t of the halo unit (LN prologue), -1 = zero
  unsigned msk[2];
  const int coc = co0 + dy_u * 8 < a.Cout ? co0 + dy_u * 8 : 0;
  const int xcc = x_ci < a.Cin ? x_ci : 0;

  auto load = [&]<int SS>(int t) {
    t = min(t, t_end - 1);  // past the block's range: re-read its last tile (never stored)
    long orow0, irow0;
    int rows_valid, fi0 = 0, nT = 0;
    if (g.F) {
      const int n = t / g.tiles_n, f0 = (t % g.tiles_n) * g.F;
      orow0 = ((long)n * a.T_out + f0) * V;
      rows_valid = min(g.F, a.T_out - f0) * V;
      nT = n * a.T_in;
      irow0 = (long)nT * V;
      fi0 = f0 * S - a.pad;
    } else {
      orow0 = (long)t * KM;
      rows_valid = (int)min((long)KM, (long)a.N * a.T_out * V - orow0);
      irow0 = orow0;
    }
    unsigned m = 0;
#pragma unroll
    for (int i = 0; i < DY_PT; ++i) {
      const int id = tid + i * 256, row = id >> 3;
      const bool ok = row < rows_valid && co0 + dy_u * 8 < a.Cout;
      ry[SS][i] = *reinterpret_cast<const uint4*>(dy + (orow0 + (ok ? row : 0)) * a.dy_ld + coc);
      m |= (unsigned)ok << i;
    }
#pragma unroll
    for (int i = 0; i < X_PT; ++i) {
      long src = -1;
      int fr = -1;
      if (x_fo(i) >= 0) {
        if (g.F) {
          const int fi = fi0 + x_fo(i);
          if (fi >= 0 && fi < a.T_in) {
            src = irow0 + (long)fi * V + x_v(i);
            fr = nT + fi;
          }
        } else if (x_fo(i) < rows_valid) {
          src = irow0 + x_fo(i);
        }
      }
      const bool ok = src >= 0 && x_ci < a.Cin;
      rx[SS][i] = *reinterpret_cast<const uint4*>(in + (ok ? src : irow0) * a.in_ld + xcc);
      rxs[SS][i] = ok ? fr : -1;
      m |= (unsigned)ok << (DY_PT + i);
    }
    msk[SS] = m;
  };

  auto store = [&]<int SS>(int buf) {
    char* sdy = smem + buf * STAGE;
    char* sx = sdy + DY_BYTES;
    const unsigned m = msk[SS];
#pragma unroll
    for (int i = 0; i < DY_PT; ++i) {
      const int id = tid + i * 256, row = id >> 3;
      *reinterpret_cast<uint4*>(sdy + (dy_u >> 2) * (KM * PR) + row * PR + (dy_u & 3) * 16) =
          (m >> i) & 1u ? ry[SS][i] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < X_PT; ++i) {
      if constexpr (LN) __builtin_amdgcn_sched_barrier(0);  // keep the per-element gathers unit by unit
      const int id = tid + i * 256;
      const int prow = id / X_UPR;
      if (prow < SP * g.HRS) {
        const bool ok = (m >> (DY_PT + i)) & 1u;
        uint4 v = ok ? rx[SS][i] : make_uint4(0, 0, 0, 0);
        if (a.pro != 0 && ok && (!LN || rxs[SS][i] >= 0)) {
          float f[8];
          unpack16(v, f, (bf16*)nullptr);
          if constexpr (!LN) {
            const float4 s0 = *reinterpret_cast<const float4*>(sScSh + x_u * 8);
            const float4 s1 = *reinterpret_cast<const float4*>(sScSh + x_u * 8 + 4);
            const float4 h0 = *reinterpret_cast<const float4*>(sScSh + 32 * NB + x_u * 8);
            const float4 h1 = *reinterpret_cast<const float4*>(sScSh + 32 * NB + x_u * 8 + 4);
            const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
            const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], sc[j], sh[j]), 0.f);
          } else {
            const float2 st = reinterpret_cast<const float2*>(a.pro_stats)[rxs[SS][i]];
            const int av = x_v(i);  // LN prologue only in framed tiles (plan())
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const int gi = (x_ci + j) * V + av;
              f[j] = x_ci + j < a.Cin ? fmaxf((f[j] - st.x) * st.y * a.pro_a[gi] + a.pro_b[gi], 0.f) : 0.f;
            }
          }
          v = pack16(f, (bf16*)nullptr);
        }
        *reinterpret_cast<uint4*>(sx + (x_u >> 2) * XP_BYTES + prow * PR + (x_u & 3) * 16) = v;
      }
    }
  };

  f32x16 acc[TW][NBW];
#pragma unroll
  for (int i = 0; i < TW; ++i)
#pragma unroll
    for (int j = 0; j < NBW; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // two tiles ahead: measured equal or slower here (config-2 step 8.037 vs 8.027 ms with one tile ahead, 3
  // interleaved runs; the C = 64 wgrad's 2 blocks per CU already hide the loads), so off; the stride-2
  // instantiations could not take it anyway (a second live set spills).  -DSTGCN_WT_AHEAD2=1: A/B builds.
#ifndef STGCN_WT_AHEAD2
#define STGCN_WT_AHEAD2 0
#endif
  constexpr bool AHEAD2 = STGCN_WT_AHEAD2 && S == 1;
  const int nt = t_end - t_begin;
  if (nt > 0) {
    load.template operator()<0>(t_begin);
    store.template operator()<0>(0);
    if constexpr (AHEAD2) load.template operator()<1>(t_begin + 1);
  }
  __syncthreads();
  auto tile = [&]<int SET>(int j) {  // tile j from LDS buffer j & 1 (= SET); tile j+1's loads go to set SET^1
    if constexpr (AHEAD2) load.template operator()<SET>(t_begin + j + 2);
    else load.template operator()<SET ^ 1>(t_begin + j + 1);
    const char* sdy = smem + SET * STAGE;
    const char* sx = sdy + DY_BYTES;
#pragma unroll 1
    for (int ks = 0; ks < KM / 16; ++ks) {
      const bf16x8 fa = trfrag(sdy + wa * (KM * PR), ks * 16, lane);
#pragma unroll
      for (int i = 0; i < TW; ++i) {
        const int dt = tw0 + i;
        if (dt < tw1) {  // wave-uniform
          const int par = dt % S, e = dt / S;
#pragma unroll
          for (int jb = 0; jb < NBW; ++jb) {
            const char* panel = sx + (bw0 + jb) * XP_BYTES + par * g.HRS * PR;
            const bf16x8 fb = trfrag(panel, ks * 16 + e * V, lane);
            acc[i][jb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb, acc[i][jb], 0, 0, 0);
          }
        }
      }
    }
    if (j + 1 < nt) store.template operator()<SET ^ 1>(SET ^ 1);
    __syncthreads();
  };
  for (int j = 0; j < nt; j += 2) {
    tile.template operator()<0>(j);
    if (j + 1 < nt) tile.template operator()<1>(j + 1);
  }

  // ---- partial of this block -> slab [rr][dt][co][ci] (full Kt x Cout x Cin image per rr)
  float* slab = g.slab + (long)rr * KT * a.Cout * a.Cin;
#pragma unroll
  for (int j = 0; j < NBW; ++j) {
    const int ci = ci0 + (bw0 + j) * 32 + (lane & 31);
#pragma unroll
    for (int i = 0; i < TW; ++i) {
      const int dt = tw0 + i;
      if (dt < tw1 && ci < a.Cin) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int co = co0 + wa * 32 + acc_row(r, lane);
          if (co < a.Cout) slab[((long)dt * a.Cout + co) * a.Cin + ci] = acc[i][j][r];
        }
      }
    }
  }
}

constexpr int RS_MAX = 16;

// Deterministic two-level reduction of the per-block partials:
//   level 1: part[s][e] = sum_{r = s, s+RS, ...} slab[r][e]     grid (E/1024, RS)
//   level 2: dw[e]     += sum_s part[s][e]
__global__ void slab_reduce1_kernel(const float* __restrict__ slab, int R, int RS, long E, float* __restrict__ part) {
  const long e4 = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  const int sidx = blockIdx.y;
  if (e4 >= E) return;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  int r = sidx;
  // eight slabs' loads in flight before their (sequential, unchanged-order) adds: one load at a time per thread
  // left the pass latency-bound (37.7 MB in 12 us at C = 64)
  for (; r + 7 * RS < R; r += 8 * RS) {
    float4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = *reinterpret_cast<const float4*>(slab + (long)(r + k * RS) * E + e4);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      acc.x += v[k].x; acc.y += v[k].y; acc.z += v[k].z; acc.w += v[k].w;
    }
  }
  for (; r < R; r += RS) {
    const float4 v = *reinterpret_cast<const float4*>(slab + (long)r * E + e4);
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  *reinterpret_cast<float4*>(part + (long)sidx * E + e4) = acc;
}

// level 2: dw (+)= sum_r part[r]; mode 0: dw[e] += (layout [Kt][Cout][Cin] of e); mode 1: dw overwritten in the
// nn.Conv2d order [Cout][Cin][Kt] (CoCi = Cout * Cin, Kt taps)
__global__ void slab_reduce2_kernel(const float* __restrict__ part, int RS, long E, float* __restrict__ dw, int mode,
                                    int Kt, long CoCi) {
  const long e4 = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (e4 >= E) return;
  float4 s = mode ? make_float4(0.f, 0.f, 0.f, 0.f) : *reinterpret_cast<const float4*>(dw + e4);
  float4 v[RS_MAX];  // every partial's load in flight first (RS <= RS_MAX), then the adds in the fixed order
#pragma unroll
  for (int r = 0; r < RS_MAX; ++r)
    if (r < RS) v[r] = *reinterpret_cast<const float4*>(part + (long)r * E + e4);
#pragma unroll
  for (int r = 0; r < RS_MAX; ++r)
    if (r < RS) {
      s.x += v[r].x; s.y += v[r].y; s.z += v[r].z; s.w += v[r].w;
    }
  if (mode == 0 || Kt == 1) {
    *reinterpret_cast<float4*>(dw + e4) = s;
  } else {  // e = k * CoCi + (co * Cin + ci) -> (co * Cin + ci) * Kt + k; 4 consecutive ci never cross a co row
    const long k = e4 / CoCi, r = e4 - k * CoCi;
    float* d = dw + r * Kt + k;
    d[0] = s.x;
    d[Kt] = s.y;
    d[2 * Kt] = s.z;
    d[3 * Kt] = s.w;
  }
}

struct Plan {
  bool ok;
  WGeom g;
  int kind;       // 0: KT9 S1, 1: KT9 S2, 2: KT1 S1 flat, 3: KT1 S2
  size_t lds;
  long slab_elems;
};

Plan plan(const stgcn_wgrad_desc& a) {
  Plan p{};
  p.ok = false;
  const int S = a.stride;
  if (a.Cin % 8 || a.Cout % 8 || a.in_ld % 8 || a.dy_ld % 8) return p;
  if (a.Kt == 9 && a.pad == 4 && (S == 1 || S == 2)) {
    p.kind = S == 1 ? 0 : 1;
  } else if (a.Kt == 1 && a.pad == 0 && S == 1 && a.T_in == a.T_out && a.pro != 2) {
    p.kind = 2;
  } else if (a.Kt == 1 && a.pad == 0 && S == 2 && a.pro != 2) {
    p.kind = 3;
  } else {
    return p;
  }
  if (a.T_out != (a.T_in + 2 * a.pad - a.Kt) / S + 1) return p;
  const int NB = (p.kind == 2 || p.kind == 3) ? 4 : 1;
  WGeom& g = p.g;
  if (p.kind == 2) {
    const long M = (long)a.N * a.T_out * a.V;
    g.F = 0;
    g.tiles_n = (int)((M + KM - 1) / KM);
    g.ntiles = g.tiles_n;
    g.HRS = KM;
  } else {
    if (a.V > 32) return p;
    g.F = KM / a.V;
    g.tiles_n = (a.T_out + g.F - 1) / g.F;
    const long nt = (long)a.N * g.tiles_n;
    if (nt > 0x7fffffffL) return p;
    g.ntiles = (int)nt;
    g.HRS = KM + ((a.Kt - 1) / S) * a.V;
  }
  g.nco = (a.Cout + 63) / 64;
  g.nci = (a.Cin + 32 * NB - 1) / (32 * NB);
  const int groups = g.nco * g.nci;
  // block-count target (measured: 512 best for the Kt = 9 C = 64 case, 256 for the 1x1 residual convs)
  const int tgt = a.Kt == 1 ? 256 : 512;
  int R = (tgt + groups - 1) / groups;
  if (R > g.ntiles) R = g.ntiles;
  if (R < 1) R = 1;
  g.tpb = (g.ntiles + R - 1) / R;
  g.R = (g.ntiles + g.tpb - 1) / g.tpb;
  p.lds = 2 * (size_t)(2 * KM * PR + NB * (a.Kt >= S ? S : 1) * g.HRS * PR) + 2 * 32 * NB * sizeof(float);
  if (p.lds > 160 * 1024) return p;
  // slabs + level-1 partials; E % 4 == 0 holds since Cin % 8 == 0
  p.slab_elems = (long)(g.R + RS_MAX) * a.Kt * a.Cout * a.Cin;
  p.ok = true;
  return p;
}

template <int KT, int S, int NB, int TW, int NBW, bool LN>
int launch_w1(const stgcn_wgrad_desc& a, const Plan& p, hipStream_t s) {
  if (stgcn_lds_attr((const void*)wgrad_tile_kernel<KT, S, NB, TW, NBW, LN>, 160 * 1024, s)) return STGCN_EHIP;
  const unsigned grid = (unsigned)(p.g.R * p.g.nco * p.g.nci);
  hipLaunchKernelGGL((wgrad_tile_kernel<KT, S, NB, TW, NBW, LN>), dim3(grid), dim3(256), p.lds, s, a, p.g);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

template <int KT, int S, int NB, int TW, int NBW>
int launch_w(const stgcn_wgrad_desc& a, const Plan& p, hipStream_t s) {
  if (a.pro == 2) {
    if constexpr (KT > 1) return launch_w1<KT, S, NB, TW, NBW, true>(a, p, s);
    return -1;
  }
  return launch_w1<KT, S, NB, TW, NBW, false>(a, p, s);
}

}  // namespace

// level 1 of slab_reduce alone: part[RS][E] = fixed-order sums of the R slabs; returns RS (< 0 on error)
int slab_reduce1_launch(const float* slab, int R, long E, float* part, hipStream_t s) {
  const int RS = R < RS_MAX ? R : RS_MAX;
  const unsigned blocks = (unsigned)((E / 4 + 255) / 256);
  hipLaunchKernelGGL(slab_reduce1_kernel, dim3(blocks, RS), dim3(256), 0, s, slab, R, RS, E, part);
  return hipGetLastError() == hipSuccess ? RS : -STGCN_EHIP;
}

// deterministic two-level sum of R fp32 slabs [R][E] into dw (out mode as slab_reduce2); part holds RS_MAX * E floats
int slab_reduce_launch(const float* slab, int R, long E, float* part, float* dw, hipStream_t s, int mode, int Kt,
                       long CoCi) {
  const int RS = R < RS_MAX ? R : RS_MAX;
  const unsigned blocks = (unsigned)((E / 4 + 255) / 256);
  hipLaunchKernelGGL(slab_reduce1_kernel, dim3(blocks, RS), dim3(256), 0, s, slab, R, RS, E, part);
  // level 2 reads RS * E floats: 64-thread blocks, four times as many CUs as 256-thread ones at E = 36 864
  hipLaunchKernelGGL(slab_reduce2_kernel, dim3((unsigned)((E / 4 + 63) / 64)), dim3(64), 0, s, (const float*)part, RS, E,
                     dw, mode, Kt, CoCi);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

// bytes of workspace the tile path needs (0 = shape not covered: conv_wgrad.hip handles it)
long wgrad_tile_workspace(const stgcn_wgrad_desc& a, int dtype) {
  if (dtype != 1) return 0;
  const Plan p = plan(a);
  return p.ok ? p.slab_elems * (long)sizeof(float) : 0;
}

// -1: not handled here
int wgrad_tile_launch(const stgcn_wgrad_desc& a, int dtype, hipStream_t s) {
  if (dtype != 1 || a.work == nullptr) return -1;
  Plan p = plan(a);
  if (!p.ok || a.work_bytes < p.slab_elems * (long)sizeof(float)) return -1;
  p.g.slab = reinterpret_cast<float*>(a.work);
  int rc;
  switch (p.kind) {
    case 0: rc = launch_w<9, 1, 1, 5, 1>(a, p, s); break;
    case 1: rc = launch_w<9, 2, 1, 5, 1>(a, p, s); break;
    case 2: rc = launch_w<1, 1, 4, 1, 2>(a, p, s); break;
    default: rc = launch_w<1, 2, 4, 1, 2>(a, p, s); break;
  }
  if (rc < 0) return -1;
  if (rc != STGCN_OK) return rc;
  const long E = (long)a.Kt * a.Cout * a.Cin;
  const int RS = p.g.R < RS_MAX ? p.g.R : RS_MAX;
  float* part = p.g.slab + (long)p.g.R * E;
  const unsigned blocks = (unsigned)((E / 4 + 255) / 256);
  hipLaunchKernelGGL(slab_reduce1_kernel, dim3(blocks, RS), dim3(256), 0, s, (const float*)p.g.slab, p.g.R, RS, E,
                     part);
  hipLaunchKernelGGL(slab_reduce2_kernel, dim3((unsigned)((E / 4 + 63) / 64)), dim3(64), 0, s, (const float*)part, RS, E,
                     a.dw, a.out_mode, a.Kt, (long)a.Cout * a.Cin);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
