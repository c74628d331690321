// Graph convolution of ST-GCN (ConvTemporalGraphical, models/utils/tgcn.py:58-79) as ONE fused,
// persistent, warp-specialised kernel: the joint mix (A) is applied while staging, the 1x1 conv runs
// on MFMA, nothing intermediate touches HBM.
//
//   forward (trans_a = 0):  out[(i,w)][co] = sum_p sum_ci W'[co][p*Cin+ci] XA_p[(i,w)][ci]  (+ bias[w][co])
//                           XA_p[(i,w)][ci] = sum_v A[p][v][w] in[(i,v)][ci]
//   data grad (trans_a = 1): XA_p[(i,v)] = sum_w A[p][v][w] in[(i,w)] (in = dg), W'[ci][p*Cout+co] = W_p[co][ci]
//                           -> dx = sum_p A_p (dg W_p)                           (autograd of tgcn.py:71-79)
//
// The reference materialises conv1x1(x) (N, P*Cout, T, V) and multiplies it by A; gconv.hip expands
// the 1x1 weights into per-(joint, neighbour) matrices rebuilt every call and gathers neighbour rows per
// output joint.  Here (same skeleton as conv_wide.hip):
//   * a tile = F = floor(256 / V) WHOLE frames (all joints) x BN output channels; blocks are
//     persistent and walk (tile, 32-input-channel item) pairs;
//   * helper waves 4-7 each own a slice of the tile's frames: they load the item's input rows (one item
//     ahead), park them in a private LDS scratch (a frame's joints never leave the wave, so no barrier),
//     and write XA_p = sum_j a_j * row(u + off_j) for every partition p (neighbour tables built from A
//     in LDS at kernel start) into the item's LDS buffer [p][row][32 ch];
//   * MMA waves 0-3 read XA fragments like conv_wide reads halo taps ("tap" = partition) and stream the
//     W' fragments (stgcn_pack_weight_frag image, Kt = 1) from L2 through a register ring;
//   * tile end: the MMA waves dump the raw fp32 sums as a bf16 column-major image; the helpers add
//     bias[w][co], store 16-B rows and write the BatchNorm partials (count, mean, M2) of the stored
//     values per (tile, channel) from wave reductions.
#include "common.h"
#include "../../include/stgcn_amd.h"
#include <stdlib.h>
#include <utility>

namespace {

constexpr int KG = 32;               // input channels per item
constexpr int KS = KG / 16;          // k-steps per partition per item
constexpr int NT = 256;              // threads per role (4 waves)
constexpr int WM = 2, WN = 2, TM = 4;
constexpr int ROWS = 256;            // MFMA rows per tile
constexpr int RSA = KG * 2 + 16;     // padded XA / scratch row bytes (80)
constexpr int CSO = ROWS * 2 + 8;    // column bytes of the output image
constexpr int PMAX = 3, DMAX = 8, VMAX = 32;
constexpr int XU = 5;                // input units (16 B) per helper lane per item: ceil(3 frames*25*4/64)
constexpr int LDS_MAX = 160 * 1024;

template <int N, typename F>
DEV void static_for(F&& f) {
  [&]<int... I>(std::integer_sequence<int, I...>) { (f.template operator()<I>(), ...); }(
      std::make_integer_sequence<int, N>{});
}

DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

struct GWGeom {
  int F;         // frames per tile
  int ntiles;    // row tiles * ncol
  int ncol;      // column tiles (BN)
  int G;         // items per tile (Cin / 32, even)
  int abytes;    // bytes per item buffer
  int k16n;      // fragment image K blocks (Kw_pad / 16)
  int cin16;     // Cin / 16 (K blocks per partition)
  int dm[PMAX];  // neighbour-table width per partition
};

template <int BN, int P, int NBUF>
__global__ __launch_bounds__(2 * NT, 1) void gcn_wide_kernel(const stgcn_gcn_tile_desc a, const GWGeom g) {
  constexpr int SPI = P * KS;  // k-steps per item
  constexpr int TN = BN / 64;
  constexpr int LEAD = NBUF - 1;
  constexpr int PAIR = 2 * SPI;
  static_assert(PAIR % NBUF == 0, "B register ring must divide the pair");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int V = a.V;
  const int grid = gridDim.x;
  const int ntile_b = (g.ntiles - (int)blockIdx.x + grid - 1) / grid;
  if (ntile_b <= 0) return;
  const int nitems = ntile_b * g.G;
  char* const sA0 = smem;
  char* const sA1 = smem + g.abytes;
  char* const sS = smem + 2 * g.abytes;                       // helpers' input scratch [ROWS][RSA]
  int2* const tT = reinterpret_cast<int2*>(sS + ROWS * RSA);  // [P][VMAX][DMAX] (row offset * RSA, weight bits)

  // ---- neighbour tables from a copy of A in the scratch (all waves)
  {
    float* Ad = reinterpret_cast<float*>(sS);
    for (int e = tid; e < P * V * V; e += 2 * NT) Ad[e] = a.A[e];
    __syncthreads();
    for (int e = tid; e < P * V; e += 2 * NT) {
      const int p = e / V, u = e - p * V;
      int d = 0;
      for (int q = 0; q < V && d < DMAX; ++q) {
        const float c = a.trans_a ? Ad[(p * V + u) * V + q] : Ad[(p * V + q) * V + u];
        if (c != 0.f) {
          tT[(p * VMAX + u) * DMAX + d] = make_int2((q - u) * RSA, __float_as_int(c));
          ++d;
        }
      }
      for (; d < DMAX; ++d) tT[(p * VMAX + u) * DMAX + d] = make_int2(0, 0);
    }
    __syncthreads();
  }

  auto item_tile = [&](int w, int& gi) {  // items past the block's last one are clamped to it
    w = min(w, nitems - 1);
    const int tl = w / g.G;
    gi = w - tl * g.G;
    return (int)blockIdx.x + tl * grid;
  };
  auto tile_end = [&](int w) { return w < nitems && (w % g.G) == g.G - 1; };
  auto tile_rows = [&](int tile, long& row0) {
    const int rt = tile / g.ncol;
    row0 = (long)rt * g.F * V;
    return (int)min((long)g.F * V, (long)a.NT * V - row0);
  };

  if (wave >= 4) {
    // =============================== helper waves ===============================
    const int hw = wave - 4;
    // frames [fb, fe) of the tile belong to this wave
    const int fb = (g.F * hw) / 4, fe = (g.F * (hw + 1)) / 4;
    const int nrow = (fe - fb) * V;  // <= 3 * 25 = 75 rows, 4 units each
    const bf16* __restrict__ in = reinterpret_cast<const bf16*>(a.in);
    uint4 rx[XU];
    auto issue = [&](int w) {
      int gi;
      const int tile = item_tile(w, gi);
      long row0;
      const int rows = tile_rows(tile, row0);
      static_for<XU>([&]<int i>() {
        const int id = lane + 64 * i, r = fb * V + id / 4, cu = id & 3;
        rx[i] = make_uint4(0, 0, 0, 0);
        if (id < nrow * 4 && r < rows) rx[i] = *reinterpret_cast<const uint4*>(in + (row0 + r) * a.in_ld + gi * KG + cu * 8);
      });
    };
    // raw rows -> private scratch, then XA_p rows of this wave's frames -> item buffer.  Lane = (row
    // sub-index rsub, 16-B unit cu); rows rsub + 16 k (k < KR) of the wave's slice, joint u_k fixed per lane.
    constexpr int KR = (XU * 64 / 4 + 15) / 16;  // row blocks of 16 (5)
    const int cu = lane & 3, rsub = lane >> 2;
    int rofs[KR], tofs[KR];  // scratch byte offset of the row; table index of (p = 0, u_k)
#pragma unroll
    for (int k = 0; k < KR; ++k) {
      const int rl = rsub + 16 * k;
      const int r = fb * V + (rl < nrow ? rl : 0);
      rofs[k] = r * RSA + cu * 16;
      tofs[k] = (r % V) * DMAX;
    }
    auto stage = [&](char* buf) {
      static_for<XU>([&]<int i>() {
        const int id = lane + 64 * i;
        if (id < nrow * 4) *reinterpret_cast<uint4*>(sS + (fb * V + id / 4) * RSA + (id & 3) * 16) = rx[i];
      });
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's own writes, read back below
      static_for<P>([&]<int p>() {
        const int dmp = g.dm[p];
        static_for<KR>([&]<int k>() {
          if (rsub + 16 * k < nrow) {
            const int2* tb = tT + p * VMAX * DMAX + tofs[k];
            int2 e[DMAX];
            uint4 xv[DMAX];
#pragma unroll
            for (int j = 0; j < DMAX; ++j)
              if (j < dmp) e[j] = tb[j];
#pragma unroll
            for (int j = 0; j < DMAX; ++j)
              if (j < dmp) xv[j] = *reinterpret_cast<const uint4*>(sS + rofs[k] + e[j].x);
            float v8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int j = 0; j < DMAX; ++j)
              if (j < dmp) {
                float f[8];
                unpack16(xv[j], f, (bf16*)nullptr);
                const float c = __int_as_float(e[j].y);
#pragma unroll
                for (int q = 0; q < 8; ++q) v8[q] = fmaf(c, f[q], v8[q]);
              }
            *reinterpret_cast<uint4*>(buf + p * ROWS * RSA + rofs[k]) = pack16(v8, (bf16*)nullptr);
          }
        });
      });
    };
    // finished tile: image (raw sums, column-major) + bias -> rows; BN partials of the stored values
    auto drain = [&](int w, const char* img) {
      int gi;
      const int tile = item_tile(w, gi);
      long row0;
      const int rows = tile_rows(tile, row0);
      const int n0 = (tile % g.ncol) * BN;
      bf16* __restrict__ outb = reinterpret_cast<bf16*>(a.out) + row0 * a.out_ld;
      const int rq = lane;  // row quad
#pragma unroll
      for (int k = 0; k < BN / 32; ++k) {
        const int cu = hw * (BN / 32) + k;  // 8-channel unit
        const int c0 = n0 + cu * 8;
        const bool cok = c0 < a.Cout;
        uint2 col[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) col[c] = *reinterpret_cast<const uint2*>(img + (cu * 8 + c) * CSO + rq * 8);
        float s1[8], s2[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) s1[c] = s2[c] = 0.f;
        float cnt = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int rl = 4 * rq + e;
          const unsigned sel = (e & 1) ? 0x07060302u : 0x05040100u;
          uint4 u4;
          u4.x = __builtin_amdgcn_perm((e >> 1) ? col[1].y : col[1].x, (e >> 1) ? col[0].y : col[0].x, sel);
          u4.y = __builtin_amdgcn_perm((e >> 1) ? col[3].y : col[3].x, (e >> 1) ? col[2].y : col[2].x, sel);
          u4.z = __builtin_amdgcn_perm((e >> 1) ? col[5].y : col[5].x, (e >> 1) ? col[4].y : col[4].x, sel);
          u4.w = __builtin_amdgcn_perm((e >> 1) ? col[7].y : col[7].x, (e >> 1) ? col[6].y : col[6].x, sel);
          if (rl < rows && cok) {
            float f[8];
            unpack16(u4, f, (bf16*)nullptr);
            bf16* p = outb + (long)rl * a.out_ld + c0;
            if (a.bias) {
              const float* b = a.bias + (long)(rl % V) * a.Cout + c0;
              const float4 b0 = *reinterpret_cast<const float4*>(b), b1 = *reinterpret_cast<const float4*>(b + 4);
              f[0] += b0.x; f[1] += b0.y; f[2] += b0.z; f[3] += b0.w;
              f[4] += b1.x; f[5] += b1.y; f[6] += b1.z; f[7] += b1.w;
            }
            if (a.accumulate) {
              float o[8];
              unpack16(*reinterpret_cast<const uint4*>(p), o, (bf16*)nullptr);
#pragma unroll
              for (int c = 0; c < 8; ++c) f[c] += o[c];
            }
            const uint4 st = pack16(f, (bf16*)nullptr);
            *reinterpret_cast<uint4*>(p) = st;
            if (a.stats) {
              float q[8];
              unpack16(st, q, (bf16*)nullptr);  // statistics of the stored values
#pragma unroll
              for (int c = 0; c < 8; ++c) {
                s1[c] += q[c];
                s2[c] = fmaf(q[c], q[c], s2[c]);
              }
              cnt += 1.f;
            }
          }
        }
        if (a.stats) {
          const float n = wave_sum(cnt);
#pragma unroll
          for (int c = 0; c < 8; ++c) {
            const float t1 = wave_sum(s1[c]), t2 = wave_sum(s2[c]);
            if (lane == c && cok) {
              const float mean = n > 0.f ? t1 / n : 0.f;
              const float m2 = n > 0.f ? fmaxf(t2 - t1 * mean, 0.f) : 0.f;
              reinterpret_cast<float4*>(a.stats)[(long)(tile / g.ncol) * a.Cout_pad + c0 + c] =
                  make_float4(n, mean, m2, 0.f);
            }
          }
        }
      }
    };

    issue(0);
    stage(sA0);
    if (nitems > 1) issue(1);
    lds_barrier();  // P
    for (int w = 0; w < nitems; ++w) {
      char* const nb = (w & 1) ? sA0 : sA1;  // buffer of item w + 1
      if (w > 0 && tile_end(w - 1)) drain(w - 1, nb);
      if (w + 1 < nitems) stage(nb);
      if (w + 2 < nitems) issue(w + 2);
      lds_barrier();  // E_w
      if (tile_end(w)) lds_barrier();  // I_w
    }
    drain(nitems - 1, ((nitems - 1) & 1) ? sA1 : sA0);
    return;
  }

  // =============================== MMA waves ===============================
  const int wm = wave >> 1, wn = wave & 1;
  const int lr = lane & 31, lh = lane >> 5;
  const bf16* __restrict__ wp = reinterpret_cast<const bf16*>(a.w_frag);
  const int k16n = g.k16n;
  const int wnu = __builtin_amdgcn_readfirstlane(wn);
  const int wlane = lane * 8;
  // B fragment j at k-step (p, ks) of item (ct, gi): block [c32 = ct*BN/32 + wn*TN + j][k16 = p*Cin/16 + 2 gi + ks]
  auto item_woff = [&](int w) {
    int gi;
    const int tile = item_tile(w, gi);
    return ((tile % g.ncol) * (BN / 32) + wnu * TN) * k16n * 512 + gi * KS * 512;
  };
  bf16x8 fb[NBUF][TN];
  auto load_B = [&](bf16x8 (&dst)[TN], int hs, int woff, int wl, int pstr, int k16) {
    const int p = hs / KS, ks = hs % KS;
    const bf16* q = wp + (p * pstr + woff + ks * 512) + wl;
#pragma unroll
    for (int j = 0; j < TN; ++j)
      dst[j] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(q + j * k16 * 512));
  };
  int a_frag[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int r = (wm * TM + i) * 32 + lr;
    a_frag[i] = (r < g.F * V ? r : 0) * RSA + lh * 16;
  }
  const int pstr_b = g.cin16 * 512;  // B elements between partitions

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto dump = [&](char* img) {  // raw sums -> column-major bf16 image; acc reset
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int cl = (wn * TN + j) * 32 + lr;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int rb = (wm * TM + i) * 32;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          bf16x4 pk;
#pragma unroll
          for (int e = 0; e < 4; ++e) pk[e] = (bf16)acc[i][j][4 * q + e];
          *reinterpret_cast<bf16x4*>(img + cl * CSO + (rb + 4 * lh + 8 * q) * 2) = pk;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
      }
    }
  };

  {
    const int w0 = item_woff(0);
#pragma unroll
    for (int hs = 0; hs < LEAD; ++hs) load_B(fb[hs % NBUF], hs, w0, wlane, pstr_b, k16n);
  }
  lds_barrier();  // P

  for (int w = 0; w < nitems; w += 2) {
    const int woff0 = item_woff(w), woff1 = item_woff(w + 1), woff2 = item_woff(w + 2);
    int af[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      af[i] = a_frag[i];
      asm volatile("" : "+v"(af[i]));
    }
    int wl = wlane;
    asm volatile("" : "+v"(wl));
    int pstr = pstr_b, k16 = k16n;
    asm volatile("" : "+s"(pstr));
    asm volatile("" : "+s"(k16));
    bf16x8 fa[2][TM];
    auto step = [&]<int hs>() {
      constexpr int h = hs / SPI, s = hs % SPI, p = s / KS, ks = s % KS;
      char* const cur = h == 0 ? sA0 : sA1;
      {
        constexpr int hn = hs + LEAD;
        const int woff = hn < SPI ? woff0 : (hn < PAIR ? woff1 : woff2);
        load_B(fb[hn % NBUF], hn % SPI, woff, wl, pstr, k16);
      }
      if constexpr (s == 0) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
          fa[hs & 1][i] = __builtin_bit_cast(
              bf16x8, *reinterpret_cast<const uint4*>(cur + af[i] + p * ROWS * RSA + ks * 32));
      }
      if constexpr (s + 1 < SPI) {
        constexpr int p1 = (s + 1) / KS, ks1 = (s + 1) % KS;
#pragma unroll
        for (int i = 0; i < TM; ++i)
          fa[(hs + 1) & 1][i] = __builtin_bit_cast(
              bf16x8, *reinterpret_cast<const uint4*>(cur + af[i] + p1 * ROWS * RSA + ks1 * 32));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[hs & 1][i], fb[hs % NBUF][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (s == SPI - 1) lds_barrier();  // E_{w+h}
    };
    static_for<PAIR>(step);
    if (tile_end(w + 1)) {
      dump(sA1);
      lds_barrier();  // I_{w+1}
    }
  }
}

}  // namespace

long gcn_tile_row_blocks(int NT, int V) {
  const int F = V > 0 && V <= VMAX ? 256 / V : 1;
  return (NT + F - 1) / F;
}

int gcn_tile_launch(const stgcn_gcn_tile_desc& a, hipStream_t s) {
  if (a.V < 1 || a.V > VMAX || a.P < 1 || a.P > PMAX || a.NT < 1) return STGCN_EBADSHAPE;
  if (a.Cin % (2 * KG) || a.in_ld % 8 || a.Cout % 64 || a.Cout_pad < a.Cout || a.out_ld % 8) return STGCN_EBADSHAPE;
  if (a.Kw_pad < a.P * a.Cin || a.Kw_pad % 16) return STGCN_EBADSHAPE;
  GWGeom g;
  g.F = 256 / a.V;
  if (g.F * a.V > ROWS || (g.F + 3) / 4 * a.V * 4 > XU * 64) return STGCN_EBADSHAPE;
  for (int p = 0; p < PMAX; ++p) g.dm[p] = p < a.P ? a.dmax[p] : 0;
  for (int p = 0; p < a.P; ++p)
    if (g.dm[p] < 0 || g.dm[p] > DMAX) return STGCN_EBADSHAPE;
  const int BN = a.Cout % 128 == 0 ? 128 : 64;
  g.ncol = a.Cout / BN;
  g.G = a.Cin / KG;
  g.k16n = a.Kw_pad / 16;
  g.cin16 = a.Cin / 16;
  const long rt = (a.NT + g.F - 1) / g.F;
  const long nt = rt * g.ncol;
  if (nt > 0x7fffffffL) return STGCN_EBADSHAPE;
  g.ntiles = (int)nt;
  const int xa = a.P * ROWS * RSA, im = BN * CSO;
  g.abytes = xa > im ? xa : im;
  const size_t lds = 2 * (size_t)g.abytes + (size_t)ROWS * RSA + (size_t)PMAX * VMAX * DMAX * sizeof(int2);
  if (lds > (size_t)LDS_MAX || (size_t)a.P * a.V * a.V * 4 > (size_t)ROWS * RSA) return STGCN_EBADSHAPE;
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (ncu <= 0) ncu = 256;
  }
  const int tpb = (g.ntiles + ncu - 1) / ncu;
  const int grid = (g.ntiles + tpb - 1) / tpb;
  void (*k)(const stgcn_gcn_tile_desc, const GWGeom) = nullptr;
  if (BN == 128) k = a.P == 3 ? gcn_wide_kernel<128, 3, 6> : a.P == 2 ? gcn_wide_kernel<128, 2, 4> : gcn_wide_kernel<128, 1, 4>;
  else k = a.P == 3 ? gcn_wide_kernel<64, 3, 6> : a.P == 2 ? gcn_wide_kernel<64, 2, 4> : gcn_wide_kernel<64, 1, 4>;
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(2 * NT), lds, s, a, g);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
