// Persistent wide-channel temporal conv (bf16): the Kt = 9, stride-1 convs of the 128- and 256-channel
// layers (tcn.2 of stgcn.py:154-159 on relu(BN1(g)), forward, and its data gradient trans = 1) — the
// config-2 layers 4, 5, 7, 8 shapes (C = 128 at T = 150, C = 256 at T = 75).
//
// Why a third conv kernel: conv_tile.hip stages the weight tile of all 9 taps through LDS per
// 16-channel chunk, so at C >= 128 each block pays a barrier, an LDS-DMA burst and a register-staged
// halo store for every 36 MFMAs per wave (measured: ~4600 cycles per chunk against ~1600 of MFMA).
// Here:
//   * a block (4 waves, one per SIMD, 2 x 2) owns a tile of F = floor(256 / V) whole output frames of
//     one sample (250 rows at V = 25) x BN output channels (BN = 128 or 256); wave (wm, wn) holds the
//     128 x BN/2 accumulator block in registers (TM = 4 x TN = BN/64 MFMA tiles of 32 x 32);
//   * K is walked as items of 64 input channels: per item the input halo (F + 8 frames x V joints x
//     64 ch) sits in LDS (rows padded to 144 B: conflict-free ds_read_b128 for any tap offset) and all
//     9 taps read it at a uniform row offset q(dt) * V (q = dt forward, 8 - dt transposed);
//   * the weights never touch LDS: each wave streams its B fragments (16 B per lane, fragment-shaped)
//     from L2 straight into a ring of NBUF register sets, LEAD = NBUF - 1 k-steps ahead of use, so the
//     9-tap loop has no barrier at all; the two waves of a column half share each fragment through L1;
//   * the next item's halo (next 64 channels, or the next tile) is loaded into registers at the
//     item's first k-step and written (BN1 scale/shift + ReLU prologue applied, zero frames outside
//     [0, T)) into the other LDS halo buffer a few k-steps later, spread over several k-steps so the
//     VALU work runs beside the MFMAs: ONE barrier per 64-channel item;
//   * blocks are persistent (grid = CU count), walking tiles blockIdx.x, +grid, ...; items are
//     processed in pairs (the channel-group count G = Cin / 64 is even), which makes the halo buffer
//     and the B register set of every k-step compile-time;
//   * epilogue per tile: + bias, bf16 store, BatchNorm Welford partials per (tile, channel) (the
//     float4 (count, mean, M2) layout bn_finalize merges; row-tile index = n * tiles_n + tile).
#include "common.h"
#include "../../include/stgcn_amd.h"
#include <stdlib.h>
#include <utility>

namespace {

constexpr int KT = 9;
constexpr int KG = 64;               // input channels per item
constexpr int KS = KG / 16;          // MFMA k-steps per tap
constexpr int SPI = KT * KS;         // k-steps per item (36)
constexpr int NT = 256;              // 4 waves
constexpr int WM = 2, WN = 2, TM = 4;
constexpr int RSA = KG * 2 + 16;     // padded halo row bytes (144)
constexpr int HR_CAP = 456;          // max halo rows per item (V = 25: 18 frames x 25 = 450)
constexpr int NA = (HR_CAP * 8 + NT - 1) / NT;  // 16-B halo units per thread (15)
constexpr int RSO = 128 * 2 + 16;                 // epilogue tile image row bytes (BN = 128 bf16, padded)
constexpr int ABYTES_MIN = 256 * RSO;             // LDS halo buffer (>= NA*32 halo rows of RSA bytes) = tile image
constexpr int LDS_MAX = 160 * 1024;

// compile-time loop: f.template operator()<I>() for I = 0..N-1 (guaranteed unrolled; register arrays
// indexed by I never fall back to scratch)
template <int N, typename F>
DEV void static_for(F&& f) {
  [&]<int... I>(std::integer_sequence<int, I...>) { (f.template operator()<I>(), ...); }(
      std::make_integer_sequence<int, N>{});
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops (lgkmcnt) but NOT for its
// outstanding global loads — __syncthreads() would drain the B-fragment prefetch ring (vmcnt(0)) at
// every 64-channel item.  The "memory" clobber keeps the compiler from moving memory ops across it.
DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

struct WGeom {
  int F;        // output frames per tile
  int tiles_n;  // tiles per sample
  int ncol;     // column tiles (Cout_pad / BN)
  int ntiles;   // N * tiles_n * ncol
  int G;        // 64-channel items per tile (even)
  int HR;       // halo rows per item ((F + 8) * V)
  int abytes;   // bytes per LDS halo buffer
};

struct TileInfo {
  int n, f0, fe, ct;
};

DEV TileInfo tile_info(int tile, const WGeom& g, int T_out) {
  TileInfo ti;
  ti.ct = tile % g.ncol;
  const int rt = tile / g.ncol;
  ti.n = rt / g.tiles_n;
  ti.f0 = (rt - ti.n * g.tiles_n) * g.F;
  ti.fe = min(g.F, T_out - ti.f0);
  return ti;
}

// DBG (diagnostic instantiations, STGCN_WIDE_DBG=<bits>, results wrong): bit0 contiguous 1-KiB B fragments
// (layout probe), bit1 no halo LDS writes, bit2 no epilogue
template <int BN, int NBUF, int PRO, int DBG = 0>
__global__ __launch_bounds__(NT, 1) void conv_wide_kernel(const stgcn_conv_desc a, const WGeom g) {
  constexpr int TN = BN / 64;
  constexpr int LEAD = NBUF - 1;
  constexpr int PAIR = 2 * SPI;  // k-steps per item pair
  static_assert(PAIR % NBUF == 0, "B register ring must divide the pair");
  constexpr int SA = LEAD + 2;   // first k-step that writes the next halo (its loads issued at k-step 0)
  constexpr int NST = 5;         // k-steps the halo writes are spread over
  constexpr int UPS = (NA + NST - 1) / NST;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int lr = lane & 31, lh = lane >> 5;
  const int V = a.V;
  const int grid = gridDim.x;
  const int ntile_b = (g.ntiles - (int)blockIdx.x + grid - 1) / grid;
  if (ntile_b <= 0) return;
  const int nitems = ntile_b * g.G;

  const bf16* __restrict__ in = reinterpret_cast<const bf16*>(a.in);
  const bf16* __restrict__ wp = reinterpret_cast<const bf16*>(a.w);
  char* const sA0 = smem;
  char* const sA1 = smem + g.abytes;
  float4* const sRed = reinterpret_cast<float4*>(smem + 2 * g.abytes);  // [WM][BN]

  // Items past the block's last one are clamped to it: their loads are issued (keeps the unrolled
  // k-step body branch-free) and their halo writes land in a buffer nobody reads again.
  auto item_tile = [&](int w, int& gi) {
    w = min(w, nitems - 1);
    const int tl = w / g.G;
    gi = w - tl * g.G;
    return (int)blockIdx.x + tl * grid;
  };

  // ---- B fragment addressing: lane (lr, lh) of frag j at k-step (t, ks) of item (ct, gi) reads
  // w[t][ct*BN + (wn*TN + j)*32 + lr][gi*64 + ks*16 + lh*8 .. +8]
  const int kcc = a.Cout_pad * a.Cin_pad;
  const int wlane = (DBG & 1) ? lane * 8 + wn * 4096 : ((wn * TN) * 32 + lr) * a.Cin_pad + lh * 8;
  auto item_woff = [&](int w) {
    int gi;
    const int tile = item_tile(w, gi);
    return (tile % g.ncol) * BN * a.Cin_pad + gi * KG;
  };
  bf16x8 fb[NBUF][TN];
  auto load_B = [&](bf16x8 (&dst)[TN], int hs, int woff, int wl, int kc, int cinp) {
    const int t = hs / KS, ks = hs % KS;
    const bf16* p = wp + (t * kc + woff + ks * 16) + wl;
#pragma unroll
    for (int j = 0; j < TN; ++j)
      dst[j] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(p + j * 32 * cinp));
  };

  // ---- halo staging of the NEXT item: unit i of this thread = halo row tid/8 + 32 i, 16-B column tid%8.
  // Rows outside [lo, hi) (frames outside [0, T_in), rows past the halo) are written as zeros; their
  // load address is clamped into the valid range.
  const int ucol = tid & 7, row0u = tid >> 3;
  const bf16* a_base = in;  // element (row 0 of the halo, channel 0) of the staged item
  int a_lo = 0, a_hi = 0;
  uint4 ra[NA];
  float sc[8], sh[8];
  auto issue_A = [&](int w) {
    int gi;
    const int tile = item_tile(w, gi);
    const TileInfo ti = tile_info(tile, g, a.T_out);
    const int fi0 = ti.f0 - (KT - 1) / 2;
    a_lo = max(0, -fi0) * V;
    a_hi = min(g.HR, (a.T_in - fi0) * V);
    a_base = in + ((long)ti.n * a.T_in + fi0) * V * a.in_ld + gi * KG + ucol * 8;
    static_for<NA>([&]<int i>() {
      const int row = min(max(row0u + 32 * i, a_lo), a_hi - 1);
      ra[i] = *reinterpret_cast<const uint4*>(a_base + row * a.in_ld);
    });
    if (PRO == 1) {
      const int c = gi * KG + ucol * 8;
      const float4 s0 = *reinterpret_cast<const float4*>(a.pro_a + c);
      const float4 s1 = *reinterpret_cast<const float4*>(a.pro_a + c + 4);
      const float4 h0 = *reinterpret_cast<const float4*>(a.pro_b + c);
      const float4 h1 = *reinterpret_cast<const float4*>(a.pro_b + c + 4);
      sc[0] = s0.x; sc[1] = s0.y; sc[2] = s0.z; sc[3] = s0.w;
      sc[4] = s1.x; sc[5] = s1.y; sc[6] = s1.z; sc[7] = s1.w;
      sh[0] = h0.x; sh[1] = h0.y; sh[2] = h0.z; sh[3] = h0.w;
      sh[4] = h1.x; sh[5] = h1.y; sh[6] = h1.z; sh[7] = h1.w;
    }
  };
  auto store_A = [&]<int i0, int i1>(char* buf) {  // units [i0, i1) -> LDS halo buffer
    static_for<NA>([&]<int i>() {
      if constexpr (i < i0 || i >= i1) return;
      const int row = row0u + 32 * i;
      uint4 v = ra[i];
      if (PRO == 1) {
        float f[8];
        unpack16(v, f, (bf16*)nullptr);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], sc[j], sh[j]), 0.f);
        v = pack16(f, (bf16*)nullptr);
      }
      const bool ok = row >= a_lo && row < a_hi;
      v.x = ok ? v.x : 0u;
      v.y = ok ? v.y : 0u;
      v.z = ok ? v.z : 0u;
      v.w = ok ? v.w : 0u;
      *reinterpret_cast<uint4*>(buf + row * RSA + ucol * 16) = v;
    });
  };

  // ---- A fragment rows: MFMA row r = (wm*TM + i)*32 + lr reads halo row r + q(dt)*V (padding rows of
  // the 256-row MFMA tile past F*V read row 0: in range, never stored)
  int a_frag[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int r = (wm * TM + i) * 32 + lr;
    a_frag[i] = (r < g.F * V ? r : 0) * RSA + lh * 16;
  }
  const int tap_bytes = V * RSA;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // ---- epilogue of a finished tile (called after a barrier; the halo buffer sA1 is free): acc + bias
  // -> bf16 tile image in sA1 (rows of BN channels, padded) -> 16-B row stores; BatchNorm Welford
  // partials per (tile, channel) from the fp32 values (two passes over the registers).
  auto epilogue = [&](int tile) {
    const TileInfo ti = tile_info(tile, g, a.T_out);
    const int rows_valid = ti.fe * V;
    const int n0 = ti.ct * BN;
    Welford ws[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int cl = (wn * TN + j) * 32 + lr;  // column within the tile
      const bool cok = n0 + cl < a.Cout;
      const float b1 = (a.bias_mode == 1 && cok) ? a.bias[n0 + cl] : 0.f;
      float sum = 0.f, cnt = 0.f;
      int lim1 = cok ? rows_valid - 4 * lh : 0;
      asm volatile("" : "+v"(lim1));
#pragma unroll
      for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rl = (wm * TM + i) * 32 + 4 * lh + (r & 3) + 8 * (r >> 2);
          const float v = acc[i][j][r] + b1;
          acc[i][j][r] = v;
          const bool ok = (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2) < lim1;
          sum += ok ? v : 0.f;
          cnt += ok ? 1.f : 0.f;
          *reinterpret_cast<bf16*>(sA1 + rl * RSO + cl * 2) = (bf16)v;
        }
      }
      Welford w;
      w.n = cnt;
      w.mean = cnt > 0.f ? sum / cnt : 0.f;
      float m2 = 0.f;
      if (a.stats) {
        // row limit re-derived per lane (opaque to CSE: the 16 x TM row masks of the first pass
        // would otherwise be kept alive in SGPR pairs and spill)
        int lim = cok ? rows_valid - 4 * lh : 0;
        asm volatile("" : "+v"(lim));
#pragma unroll
        for (int i = 0; i < TM; ++i) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int rr = (wm * TM + i) * 32 + (r & 3) + 8 * (r >> 2);
            const float d = acc[i][j][r] - w.mean;
            m2 += rr < lim ? d * d : 0.f;
          }
        }
      }
      w.m2 = m2;
      ws[j] = w;
    }
    if (a.stats) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        Welford o;
        o.n = __shfl_xor(ws[j].n, 32);
        o.mean = __shfl_xor(ws[j].mean, 32);
        o.m2 = __shfl_xor(ws[j].m2, 32);
        const Welford w = welford_merge(ws[j], o);
        if (lh == 0) sRed[wm * BN + (wn * TN + j) * 32 + lr] = make_float4(w.n, w.mean, w.m2, 0.f);
      }
    }
    __syncthreads();
    if (a.stats) {
      const int rt = tile / g.ncol;
      for (int c = tid; c < BN; c += NT) {
        const float4 f0 = sRed[c], f1 = sRed[BN + c];
        const Welford w = welford_merge(Welford{f0.x, f0.y, f0.z}, Welford{f1.x, f1.y, f1.z});
        if (n0 + c < a.Cout_pad)
          reinterpret_cast<float4*>(a.stats)[(long)rt * a.Cout_pad + n0 + c] = make_float4(w.n, w.mean, w.m2, 0.f);
      }
    }
    // rows -> global: 16 threads per row (16 B each), 16 rows per pass
    bf16* __restrict__ outb = reinterpret_cast<bf16*>(a.out) + ((long)ti.n * a.T_out + ti.f0) * V * (long)a.out_ld;
    const int cu = tid & 15, r0 = tid >> 4;
    const bool cvalid = n0 + cu * 8 < a.Cout;
    for (int rl = r0; rl < rows_valid; rl += NT / 16) {
      uint4 v = *reinterpret_cast<const uint4*>(sA1 + rl * RSO + cu * 16);
      bf16* p = outb + (long)rl * a.out_ld + n0 + cu * 8;
      if (!cvalid) continue;
      if (a.accumulate) {
        float f[8], o[8];
        unpack16(v, f, (bf16*)nullptr);
        unpack16(*reinterpret_cast<const uint4*>(p), o, (bf16*)nullptr);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] += o[e];
        v = pack16(f, (bf16*)nullptr);
      }
      *reinterpret_cast<uint4*>(p) = v;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  };

  // ---- prologue: halo of item 0 staged synchronously; B of its first LEAD k-steps in flight
  issue_A(0);
  store_A.template operator()<0, NA>(sA0);
  {
    const int w0 = item_woff(0);
#pragma unroll
    for (int hs = 0; hs < LEAD; ++hs) load_B(fb[hs % NBUF], hs, w0, wlane, kcc, a.Cin_pad);
  }
  __syncthreads();

  const int qsign = a.trans ? -1 : 1;
  const int qbase = a.trans ? KT - 1 : 0;
  for (int w = 0; w < nitems; w += 2) {
    const int woff0 = item_woff(w), woff1 = item_woff(w + 1), woff2 = item_woff(w + 2);
    // per-lane/uniform address bases re-materialised each pair (opaque to LICM: otherwise the
    // compiler hoists the addresses of all 72 k-steps out of the loop and spills)
    int af[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      af[i] = a_frag[i];
      asm volatile("" : "+v"(af[i]));
    }
    int wl = wlane;
    asm volatile("" : "+v"(wl));
    int tbytes = tap_bytes, kcc_l = kcc, cinp_l = a.Cin_pad;
    asm volatile("" : "+s"(tbytes));
    asm volatile("" : "+s"(kcc_l));
    asm volatile("" : "+s"(cinp_l));
    bf16x8 fa[2][TM];
    // one k-step; hs is a template parameter so every ring index below is a compile-time constant
    auto step = [&]<int hs>() {
      constexpr int h = hs / SPI, s = hs % SPI, t = s / KS, ks = s % KS;
      char* const cur = h == 0 ? sA0 : sA1;
      char* const nxt = h == 0 ? sA1 : sA0;
      // 1. B fragments LEAD k-steps ahead (may belong to the next item or the next pair)
      {
        const int hn = hs + LEAD;
        const int woff = hn < SPI ? woff0 : (hn < PAIR ? woff1 : woff2);
        load_B(fb[hn % NBUF], hn % SPI, woff, wl, kcc_l, cinp_l);
      }
      // 2. next item's halo: loads at the item's first k-step, LDS writes spread over NST k-steps
      if constexpr (s == 0) issue_A(w + h + 1);
      if constexpr ((DBG & 2) == 0 && s >= SA && s < SA + NST) store_A.template operator()<(s - SA) * UPS, (s - SA + 1) * UPS>(nxt);
      // 3. A fragments (read one k-step ahead inside an item)
      if constexpr (s == 0) {
        const int tb = (qbase + qsign * t) * tbytes + ks * 32;
#pragma unroll
        for (int i = 0; i < TM; ++i)
          fa[hs & 1][i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(cur + af[i] + tb));
      }
      if constexpr (s + 1 < SPI) {
        const int t1 = (s + 1) / KS, ks1 = (s + 1) % KS;
        const int tb1 = (qbase + qsign * t1) * tbytes + ks1 * 32;
#pragma unroll
        for (int i = 0; i < TM; ++i)
          fa[(hs + 1) & 1][i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(cur + af[i] + tb1));
      }
      // 4. MFMAs
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[hs & 1][i], fb[hs % NBUF][j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (hs == SPI - 1) lds_barrier();
    };
    [&]<int... I>(std::integer_sequence<int, I...>) { (step.template operator()<I>(), ...); }(
        std::make_integer_sequence<int, PAIR>{});
    const int tl = w / g.G;
    if ((DBG & 4) != 0 && a.N < 0) epilogue(0);  // never runs: keeps the MFMAs alive
    if ((DBG & 4) == 0 && (w + 1) - tl * g.G == g.G - 1) {
      lds_barrier();  // every wave done reading sA1 (item w + 1's halo)
      epilogue((int)blockIdx.x + tl * grid);
    }
    lds_barrier();
  }
}

}  // namespace

long conv_rows_num_row_blocks(long M, int cout);

int conv_wide_launch(const stgcn_conv_desc& a, int dtype, hipStream_t s) {
  static const bool off = getenv("STGCN_NO_WIDE") != nullptr;  // A/B switch
  if (off || dtype != 1) return -1;
  if (a.Kt != KT || a.pad != (KT - 1) / 2 || a.stride != 1 || a.T_in != a.T_out) return -1;
  if (a.pro != 0 && a.pro != 1) return -1;
  if (a.bias_mode != 0 && a.bias_mode != 1) return -1;
  if (a.Cin != a.Cin_pad || a.Cin_pad % (2 * KG) || a.in_ld % 8 || a.V > 32) return -1;
  if (a.Cout % 8 || a.out_ld % 8) return -1;  // 16-B row stores of the epilogue
  const int BN = 128;  // BN = 256 (acc 256 + B ring) does not fit the register file without spills
  if (a.Cout_pad % BN) return -1;
  WGeom g;
  g.F = 256 / a.V;
  g.HR = (g.F + KT - 1) * a.V;
  if (g.HR > HR_CAP || g.F < 1) return -1;
  g.G = a.Cin_pad / KG;
  g.tiles_n = (a.T_out + g.F - 1) / g.F;
  g.ncol = a.Cout_pad / BN;
  const long nt = (long)a.N * g.tiles_n * g.ncol;
  if (nt <= 0 || nt > 0x7fffffffL) return -1;
  g.ntiles = (int)nt;
  if (a.stats && (long)a.N * g.tiles_n > conv_rows_num_row_blocks((long)a.N * a.T_out * a.V, a.Cout)) return -1;
  g.abytes = ABYTES_MIN;
  const size_t lds = 2 * (size_t)g.abytes + (size_t)WM * BN * 16;
  if (lds > (size_t)LDS_MAX) return -1;
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (ncu <= 0) ncu = 256;
  }
  const int tpb = (g.ntiles + ncu - 1) / ncu;
  const int grid = (g.ntiles + tpb - 1) / tpb;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv_wide_kernel<128, 6, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    (void)hipFuncSetAttribute((const void*)conv_wide_kernel<128, 6, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    attr = true;
  }
  const dim3 gd((unsigned)grid), bd(NT);
  static const int dbg = getenv("STGCN_WIDE_DBG") ? atoi(getenv("STGCN_WIDE_DBG")) : 0;
  if (dbg) {
    auto* k = dbg == 1 ? conv_wide_kernel<128, 6, 1, 1> : dbg == 2 ? conv_wide_kernel<128, 6, 1, 2>
            : dbg == 4 ? conv_wide_kernel<128, 6, 1, 4> : dbg == 6 ? conv_wide_kernel<128, 6, 1, 6>
                       : conv_wide_kernel<128, 6, 1, 7>;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
    hipLaunchKernelGGL(k, gd, bd, lds, s, a, g);
    return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
  }
  if (a.pro) hipLaunchKernelGGL((conv_wide_kernel<128, 6, 1>), gd, bd, lds, s, a, g);
  else hipLaunchKernelGGL((conv_wide_kernel<128, 6, 0>), gd, bd, lds, s, a, g);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
