// Weight gradient of the Kt = 9, stride-1 temporal convs (tcn.2, stgcn.py:154-159; the convolution_backward weight
// path, the reference's top CPU op) at 64 and 128 channels, bf16:
//
//   dW[dt][co][ci] = sum_q dY[q][co] * h[q + (dt - 4) V][ci],   h = relu(in * scale + shift) (BN1 + ReLU, pro 1) or in
//
// a GEMM with M = co, N = (dt, ci), K = the output rows of a sample (frames outside [0, T) of h are zeros).
//
// wgrad_tile.hip (C = 64) gives a block a 64-co x 32-ci output block and re-stages the 8-frame input halo of every
// 5-frame tile (2.6x, twice over the ci blocks) through registers; wgrad_wide.hip (C >= 128) stages each frame once
// but through registers, one tile ahead with a barrier per tile, and waits out its loads.  Here:
//   * a block (8 waves, one per CU) owns a COB-co x 64-ci x 9-tap output block for a run of frames of ONE sample and
//     streams the run's rows once: dY rows and input rows go global -> LDS by DMA (global_load_lds, 16 rows x 32
//     channels per instruction, no register staging) into rings of 64-row chunks, the input two chunks and dY two
//     steps ahead of their use;
//   * the BatchNorm1 + ReLU prologue is applied to every input row ONCE, in place in the ring, five steps before the
//     first MFMA reads it (the DMA cannot transform); rows outside the sample come from a zero page (the conv's zero
//     padding applies to h), so nothing is transformed there;
//   * a step = 64 output rows: per wave 4 k-steps x (its taps) 32x32x16 MFMAs, dY^T and tap-shifted input fragments
//     read with the transposing ds_read_b64_tr_b16 from 64-B-row panels; the tap window of a step spans 64 + 8V rows
//     of the 512-row input ring, so chunks in ring slots 0-3 also live in a 4-slot guard after slot 7 (written by the
//     transform pass) and every window is LDS-contiguous;
//   * one LDS barrier per step; every wave issues the same DMA count per step (zero-page dummies past the run), so
//     the wait before a step is an exact vmcnt;
//   * the fp32 block result goes to a slab [row range][9][Cout][Cin], summed in a fixed order by slab_reduce
//     (wgrad_tile.hip): deterministic.
#include "common.h"
#include "../../include/stgcn_amd.h"
#include <utility>

#ifndef WR_G64
#define WR_G64 2
#endif
#ifndef WR_D
#define WR_D 2
#endif

namespace {

constexpr int NW = 8, NT = NW * 64;
constexpr int KS = 64;                          // output rows per step (4 MFMA k-steps of 16)
constexpr int XGUARD = 4;                       // guard copy of input ring slots 0-3 after the last slot
constexpr int PR = 64;                          // panel row bytes: 32 bf16 channels
constexpr int CIB = 64;                         // input channels per block (two panels)
constexpr int KT = 9, PADT = 4;
constexpr int XFORM = 5;                        // input chunk s + 5 is transformed at step s (first read at s + 1)
// Ring schedule for G DMA groups in flight: at step s the DMA of input chunk s + 5 + G and dY chunk s + G is issued
// (into the slots of chunks s - 1), chunk s + 5 / dY s have landed (waited), compute reads input chunks s .. s + 4.
template <int G> struct Ring {
  static constexpr int LOOK_X = XFORM + G, LOOK_Y = G;
  static constexpr int XSLOT = LOOK_X + 1, YSLOT = LOOK_Y + 1;
  static constexpr int XPANEL = (XSLOT + XGUARD) * KS * PR;  // bytes per 32-channel input panel
  static constexpr int YPANEL = YSLOT * KS * PR;             // bytes per 32-channel dY panel
};
// groups in flight: 2 (64 co: 120 KB of LDS, 128 co: 144 KB; 4 groups at 64 co measured slower, 79 vs 74 us)
constexpr int ring_g(int cob) { return cob == 64 ? WR_G64 : 2; }
constexpr size_t ring_lds(int cob) {
  return ring_g(cob) == 4 ? 2 * (size_t)Ring<4>::XPANEL + (cob / 32) * (size_t)Ring<4>::YPANEL
                          : ring_g(cob) == 3 ? 2 * (size_t)Ring<3>::XPANEL + (cob / 32) * (size_t)Ring<3>::YPANEL
                                             : 2 * (size_t)Ring<2>::XPANEL + (cob / 32) * (size_t)Ring<2>::YPANEL;
}

__device__ uint4 g_wr_zero[64];

// -DWR_PROF=1 (tools builds only): per-wave cycle accounts (s_memtime) of the step loop into g_wr_prof
// [block < 256][wave][5] = vmcnt wait, barrier wait, DMA issue + transform, compute, total; read by stgcn_wr_prof
#ifndef WR_PROF
#define WR_PROF 0
#endif
__device__ long long g_wr_prof[WR_PROF ? 256 * 8 * 5 : 1];
DEV long long wr_time() {
  if constexpr (WR_PROF) return __builtin_amdgcn_s_memtime();
  return 0;
}  // DMA source of rows outside the sample / the run (zero-initialised code object data)

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

template <int N, typename F>
DEV void sfor(F&& f) {
  [&]<int... I>(std::integer_sequence<int, I...>) { (f.template operator()<I>(), ...); }(
      std::make_integer_sequence<int, N>{});
}

DEV unsigned lds_u32(const void* p) { return (unsigned)(size_t)(const __attribute__((address_space(3))) char*)p; }

// 16 B per lane, global -> LDS at M0 = lds_off (lane-linear); m0 saved / restored around the issue
DEV void glds16(const void* src, unsigned lds_off) {
  unsigned saved;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(saved) : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds_off)) : "memory");
}

// MFMA fragment from a [rows][32 ch] panel: lane (c, h) gets rows r0 + 8h .. r0 + 8h + 7 of column c, as two
// ds_read_b64_tr_b16 (rows +q and +q+4); p = panel + r0 * PR (uniform), loff = the lane's constant offset
DEV bf16x8 trfrag(const char* p, int loff) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p + loff));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p + loff + 4 * PR));
  s16x8 v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return __builtin_bit_cast(bf16x8, v);
}

struct WRGeom {
  int runs_n, run;  // runs per sample, frames per run
  int nco, nci;     // output blocks along co (COB) and ci (64)
  int R;            // row ranges (= N * runs_n): slab rows
  float* slab;      // [R][9][Cout][Cin]
};

// VT: the joint count as a compile-time constant (0: runtime V) — the tap offsets t * V rows then fold into the
// ds_read immediate offsets, leaving one address add per step instead of one per read (measured 6.3 VALU per MFMA
// with a runtime V, most of them the 48 per-read address adds of a 64-co step)
template <int COB, int PRO, int VT>
__global__ __launch_bounds__(NT, 1) void wgrad_ring_kernel(const stgcn_wgrad_desc a, const WRGeom g) {
  typedef Ring<ring_g(COB)> RG;
  constexpr int LOOK_X = RG::LOOK_X, LOOK_Y = RG::LOOK_Y, XSLOT = RG::XSLOT, YSLOT = RG::YSLOT;
  constexpr int XPANEL = RG::XPANEL, YPANEL = RG::YPANEL;
  constexpr int NYP = COB / 32;                 // dY panels
  constexpr int NI = 2 * 4 + NYP * 4;           // DMA instructions per step (16 rows x 32 channels each)
  constexpr int NDMA = NI / NW;                 // ... per wave: 2 (COB 64) or 3 (COB 128)
  static_assert(NI % NW == 0, "dma split");
  constexpr int TW = COB == 64 ? 5 : 9;         // taps per wave (COB 64: taps 0-4 / 5-8 by wave half)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const sX = smem;                        // [2 panels][XSLOT + 4 slots * 64 rows][64 B]
  char* const sY = smem + 2 * XPANEL;           // [NYP panels][YSLOT slots * 64 rows][64 B]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int V = VT ? VT : a.V, T = a.T_in;
  // block -> (row range rg, output block ob): the nob output blocks of a row range are ids b, b + 8, ... (one XCD
  // under the round-robin dealing: they stream the same rows through one L2; speed only)
  const int nob = g.nco * g.nci;
  const int xq = blockIdx.x & 7, jq = blockIdx.x >> 3;
  const int ob = jq % nob, rg = (jq / nob) * 8 + xq;
  if (rg >= g.R) return;  // block-uniform, before any barrier
  const int n = rg / g.runs_n, run = rg - n * g.runs_n;
  const int f0 = run * g.run, f1 = min(T, f0 + g.run);
  const int co0 = (ob % g.nco) * COB, ci0 = (ob / g.nco) * CIB;
  const int nrow = (f1 - f0) * V;                     // output rows of the run
  const int nsteps = (nrow + KS - 1) / KS;
  const int nxrow = (f1 - f0 + 2 * PADT) * V;         // input rows: frames f0 - 4 .. f1 + 3
  const int nxc = (nxrow + KS - 1) / KS;
  const long srow = (long)n * T * V;                  // first row of the sample
  const float invV = 1.f / (float)V;

  // ---- zero the LDS image: ring rows never written (dummy chunks' guards) are read as operands of zero dY rows
  {
    uint4* z = reinterpret_cast<uint4*>(smem);
    for (int e = tid; e < (2 * XPANEL + NYP * YPANEL) / 16; e += NT) z[e] = make_uint4(0, 0, 0, 0);
  }
  // prologue constants of this thread's transform unit (8 channels)
  // transform units: waves 4-7, two 16-B units (rows r and r + 32 of a chunk, 8 channels) per thread; their VALU
  // runs beside the MFMAs of waves 0-3 (the other wave of each SIMD), which hold the 5-tap half at 64 co
  const int tu_row = (tid & 255) >> 3, tu_pan = (tid >> 2) & 1, tu_col = tid & 3;
  float sc[8], sh[8];
  if constexpr (PRO == 1) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = ci0 + tu_pan * 32 + tu_col * 8 + j;
      sc[j] = a.pro_a[c];
      sh[j] = a.pro_b[c];
    }
  }
  // consume the constants here: the compiler's wait insertion does not see the DMA asm, and a first use inside the
  // step loop made it wait vmcnt(0) there on every step (draining the DMA look-ahead)
#pragma unroll
  for (int j = 0; j < 8; ++j) asm volatile("" ::"v"(sc[j]), "v"(sh[j]));
  __syncthreads();

  const unsigned xbase = lds_u32(sX), ybase = lds_u32(sY);
  const int lr = lane >> 2, lu = lane & 3;  // DMA lane: row of the 16-row group, 16-B unit
  // DMA instructions of a step: 8 input (panel i & 1, 16-row group i >> 1) + 4 NYP dY (panel j % NYP, group j / NYP);
  // wave w issues instruction w (input) and 8 + w + 8k (dY).  Per instruction: the lane's source row (relative to the
  // sample's first row; +64 per step), its valid row range, the sample-based source pointer, the LDS offset in a slot
  const int xhi = min(T, f1 + PADT) * V;                   // input rows [0, xhi) of the sample are read; others zero
  const int ylo = f0 * V, yhi = f1 * V;                    // dY rows of the run
  int xr = (f0 - PADT) * V + 16 * (wave >> 1) + lr;        // input row of the lane at step -LOOK_X (chunk 0)
  const bf16* xp = reinterpret_cast<const bf16*>(a.in) + (srow + xr) * a.in_ld + ci0 + 32 * (wave & 1) + 8 * lu;
  const unsigned xoff = xbase + (unsigned)((wave & 1) * XPANEL + 16 * (wave >> 1) * PR);
  const long xstep = (long)KS * a.in_ld;
  int yr[NDMA - 1];
  const bf16* yp[NDMA - 1];
  unsigned yoff[NDMA - 1];
#pragma unroll
  for (int k = 0; k + 1 < NDMA; ++k) {
    const int j = wave + NW * k, pan = j % NYP, grp = j / NYP;
    yr[k] = f0 * V + (LOOK_Y - LOOK_X) * KS + 16 * grp + lr;  // dY row at step -LOOK_X (chunk LOOK_Y - LOOK_X < 0)
    yp[k] = reinterpret_cast<const bf16*>(a.dy) + (srow + yr[k]) * a.dy_ld + co0 + 32 * pan + 8 * lu;
    yoff[k] = ybase + (unsigned)(pan * YPANEL + 16 * grp * PR);
  }
  const long ystep = (long)KS * a.dy_ld;
  const uint4* const zsrc = g_wr_zero + lane;
  // group of step s: input chunk s + LOOK_X, dY chunk s + LOOK_Y (dummies from the zero page past the run).  The
  // fill's dY chunks < 0 are never read and are skipped (withy false): issued back to back they would land in ring
  // slots that chunks 0 .. LOOK_Y - 1 are loading at the same time; the fill's last G - 1 groups are always full
  auto issue = [&](int s, bool withy) {
    const int xslot = (s + LOOK_X) % XSLOT;
    glds16(xr >= 0 && xr < xhi ? (const void*)xp : (const void*)zsrc, xoff + (unsigned)(xslot * KS * PR));
    xr += KS;
    xp += xstep;
    const int yslot = ((s + LOOK_Y) % YSLOT + YSLOT) % YSLOT;
#pragma unroll
    for (int k = 0; k + 1 < NDMA; ++k) {
      if (withy) glds16(yr[k] >= ylo && yr[k] < yhi ? (const void*)yp[k] : (const void*)zsrc, yoff[k] + (unsigned)(yslot * KS * PR));
      yr[k] += KS;
      yp[k] += ystep;
    }
  };
  // in-place prologue of an input chunk (rows of frames inside the sample) and its guard copy (ring slots 0-3), in
  // two halves so that the LDS read can be issued well before the VALU that consumes it: xload (read), xstore
  // (prologue + writes); rr = row in the chunk
  auto xptr = [&](int c, int rr) { return sX + tu_pan * XPANEL + ((c % XSLOT) * KS + rr) * PR + tu_col * 16; };
  auto xstore = [&](char* ptr, uint4 u, bool valid, bool guard) {
    if (PRO == 1 && valid) {
      float f[8];
      unpack16(u, f, (bf16*)nullptr);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], sc[j], sh[j]), 0.f);
      u = pack16(f, (bf16*)nullptr);
      *reinterpret_cast<uint4*>(ptr) = u;
    }
    if (guard) *reinterpret_cast<uint4*>(ptr + XSLOT * KS * PR) = u;
  };
  const int xrow0 = (f0 - PADT) * V;  // sample row of input chunk 0's first row
  // main loop: waves 4-7 transform chunk s + XFORM, rows tu_row and tu_row + 32 (their VALU beside the MFMAs of
  // waves 0-3, the 5-tap half at 64 co); read at the step's start, finished halfway through its MFMAs
  const bool txw = wave >= 4;
  uint4 tu[2];
  auto tload = [&](int s) {
    const int c = s + XFORM;
    if (!txw || c >= nxc || (PRO == 0 && c % XSLOT >= XGUARD)) return;  // wave-uniform
#pragma unroll
    for (int h = 0; h < 2; ++h) tu[h] = *reinterpret_cast<const uint4*>(xptr(c, tu_row + 32 * h));
  };
  auto tfinish = [&](int s) {
    const int c = s + XFORM;
    if (!txw || c >= nxc || (PRO == 0 && c % XSLOT >= XGUARD)) return;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = xrow0 + c * KS + tu_row + 32 * h;
      xstore(xptr(c, tu_row + 32 * h), tu[h], r >= 0 && r < xhi, c % XSLOT < XGUARD);
    }
  };

  // ---- wave roles: co tile wc, ci tile wi, taps [t0, t0 + ntap)
  int wc, wi, t0, ntap;
  if constexpr (COB == 64) {
    wc = wave & 1;
    wi = (wave >> 1) & 1;
    t0 = (wave >> 2) ? 5 : 0;
    ntap = (wave >> 2) ? 4 : 5;
  } else {
    wc = wave & 3;
    wi = wave >> 2;
    t0 = 0;
    ntap = 9;
  }
  // trfrag lane offset: rows 8h + q (+4 via the second read), columns 16 (g & 1) + 4 p
  const int li = lane & 15, gq = lane >> 4;
  const int loff = (8 * (gq >> 1) + (li >> 2)) * PR + (16 * (gq & 1) + 4 * (li & 3)) * 2;
  f32x16 acc[TW];
#pragma unroll
  for (int t = 0; t < TW; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  const int tapb = V * PR;

  // ring fill: every fill group's DMA back to back, then chunks 0 .. XFORM-1 transformed by all threads (one unit each)
  for (int s = -LOOK_X; s < 0; ++s) issue(s, s + LOOK_Y >= 0);
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NDMA * (LOOK_Y - 1)) : "memory");  // all but the last G - 1 groups
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  {
    const int rr = tid >> 3;
    uint4 u[XFORM];
    bool use[XFORM];
#pragma unroll
    for (int c = 0; c < XFORM; ++c) {
      use[c] = c < nxc && (PRO == 1 || c % XSLOT < XGUARD);
      if (use[c]) u[c] = *reinterpret_cast<const uint4*>(xptr(c, rr));
    }
#pragma unroll
    for (int c = 0; c < XFORM; ++c) {
      const int r = xrow0 + c * KS + rr;
      if (use[c]) xstore(xptr(c, rr), u[c], r >= 0 && r < xhi, c % XSLOT < XGUARD);
    }
  }
  long long pacc[5] = {0, 0, 0, 0, 0};
  const long long pst = wr_time();
  for (int s = 0; s < nsteps; ++s) {
    const long long p0 = wr_time();
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NDMA * (LOOK_Y - 1)) : "memory");  // group s - G landed (input s + 5, dY s)
    const long long p1 = wr_time();
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    const long long p2 = wr_time();
    issue(s, true);
    tload(s);
    const long long p3 = wr_time();
    if constexpr (WR_PROF) {
      pacc[0] += p1 - p0;
      pacc[1] += p2 - p1;
      pacc[2] += p3 - p2;
    }
    // compute step s (the transform of chunk s + 5 completes halfway: it touches ring slots the step does not read);
    // lane bases (one add each per step); reads at compile-time offsets from them when VT > 0
    const char* Yl = sY + wc * YPANEL + (s % YSLOT) * KS * PR + loff;
    const char* Xl = sX + wi * XPANEL + ((s % XSLOT) * KS + t0 * V) * PR + loff;
    int tb = tapb;
    if constexpr (VT == 0) asm volatile("" : "+s"(tb));
    constexpr int NU = 4 * TW, D = WR_D;  // fragments read D (ks, tap) steps ahead of their MFMA
    bf16x8 fx[D + 1], fy[2];
    auto rd = [&]<int u>() {
      constexpr int ks = u / TW, t = u % TW;
      if constexpr (t == 0) fy[ks & 1] = trfrag(Yl + 16 * ks * PR, 0);
      if (t < ntap) fx[u % (D + 1)] = trfrag(Xl + (VT ? t * VT * PR : t * tb) + 16 * ks * PR, 0);
    };
    sfor<D>([&]<int u>() { rd.template operator()<u>(); });
    sfor<NU>([&]<int u>() {
      if constexpr (u + D < NU) rd.template operator()<u + D>();
      constexpr int ks = u / TW, t = u % TW;
      if (t < ntap) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fy[ks & 1], fx[u % (D + 1)], acc[t], 0, 0, 0);
      if constexpr (u == NU / 2) tfinish(s);
    });
  }
  if constexpr (WR_PROF) {
    pacc[4] = wr_time() - pst;
    pacc[3] = pacc[4] - pacc[0] - pacc[1] - pacc[2];
    if (lane == 0 && blockIdx.x < 256)
      for (int j = 0; j < 5; ++j) g_wr_prof[((long)blockIdx.x * 8 + wave) * 5 + j] = pacc[j];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may land after the workgroup's LDS is released

  // ---- block partial -> slab [rg][dt][co][ci]: lane holds ci = ci0 + 32 wi + (lane & 31), co rows acc_row
  float* __restrict__ out = g.slab + (long)rg * KT * a.Cout * a.Cin;
  const int ci = ci0 + 32 * wi + (lane & 31);
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    if (t >= ntap) break;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = co0 + 32 * wc + acc_row(r, lane);
      out[((long)(t0 + t) * a.Cout + co) * a.Cin + ci] = acc[t][r];
    }
  }
}

struct RPlan {
  bool ok;
  int cob;
  WRGeom g;
  size_t lds;
  long slab_elems;
};

constexpr int RS_PART = 16;  // level-1 partials of slab_reduce
constexpr int R_MAX = 320;   // slab rows (config 2: 256 at 64 channels, 128 at 128; config-4 units: 260)

RPlan rplan(const stgcn_wgrad_desc& a) {
  RPlan p{};
  p.ok = false;
  if (a.Kt != KT || a.pad != PADT || a.stride != 1 || a.T_in != a.T_out || (a.pro != 0 && a.pro != 1)) return p;
  if (a.V < 1 || a.V > 32 || a.Cin % CIB || a.in_ld % 8 || a.dy_ld % 8) return p;
  if (a.Cout == 64) p.cob = 64;
  else if (a.Cout == 128) p.cob = 128;
  else return p;
  WRGeom& g = p.g;
  g.nco = a.Cout / p.cob;
  g.nci = a.Cin / CIB;
  const int nob = g.nco * g.nci;
  // one block per CU: runs per sample so that nob * N * runs ~ 256
  int runs = (int)((256L + (long)nob * a.N / 2) / ((long)nob * a.N));
  if (runs < 1) runs = 1;
  if (runs > a.T_in) runs = a.T_in;
  g.run = (a.T_in + runs - 1) / runs;
  g.runs_n = (a.T_in + g.run - 1) / g.run;
  g.R = a.N * g.runs_n;
  p.lds = ring_lds(p.cob);
  p.slab_elems = ((long)g.R + RS_PART) * KT * a.Cout * a.Cin;
  // one slab row per (sample, run): at least N rows, so the workspace grows with the batch.  Past R_MAX rows
  // (N > 320: > 190 MB at 128 channels) the call falls through to the bounded-workspace kernels (wgrad_tile)
  p.ok = p.lds <= 160 * 1024 && g.R <= R_MAX;
  return p;
}

}  // namespace

int slab_reduce_launch(const float* slab, int R, long E, float* part, float* dw, hipStream_t s, int mode, int Kt,
                       long CoCi);

// WR_PROF builds: copy the per-wave cycle accounts [256][8][5] (long long) to host memory; -1 in the shipped library
extern "C" int stgcn_wr_prof(void* dst, long n) {
  if (!WR_PROF) return -1;
  if (n > 256L * 8 * 5) n = 256L * 8 * 5;
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_wr_prof), n * sizeof(long long), 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}

long wgrad_ring_workspace(const stgcn_wgrad_desc& a, int dtype) {
  if (dtype != 1) return 0;
  const RPlan p = rplan(a);
  return p.ok ? p.slab_elems * (long)sizeof(float) : 0;
}

// -1: not handled here
int wgrad_ring_launch(const stgcn_wgrad_desc& a, int dtype, hipStream_t s) {
  if (dtype != 1 || a.work == nullptr) return -1;
  RPlan p = rplan(a);
  if (!p.ok || a.work_bytes < p.slab_elems * (long)sizeof(float)) return -1;
  p.g.slab = reinterpret_cast<float*>(a.work);
  typedef void (*KFn)(const stgcn_wgrad_desc, const WRGeom);
  static const KFn tab[2][2][2] = {{{wgrad_ring_kernel<64, 0, 0>, wgrad_ring_kernel<64, 0, 25>},
                                    {wgrad_ring_kernel<64, 1, 0>, wgrad_ring_kernel<64, 1, 25>}},
                                   {{wgrad_ring_kernel<128, 0, 0>, wgrad_ring_kernel<128, 0, 25>},
                                    {wgrad_ring_kernel<128, 1, 0>, wgrad_ring_kernel<128, 1, 25>}}};
  const KFn k = tab[p.cob == 128][a.pro == 1][a.V == 25];
  if (stgcn_lds_attr((const void*)k, 160 * 1024, s)) return STGCN_EHIP;
  const int nob = p.g.nco * p.g.nci;
  const unsigned grid = (unsigned)(8L * ((p.g.R + 7) / 8) * nob);
  hipLaunchKernelGGL(k, dim3(grid), dim3(NT), p.lds, s, a, p.g);
  if (hipGetLastError() != hipSuccess) return STGCN_EHIP;
  const long E = (long)KT * a.Cout * a.Cin;
  float* part = p.g.slab + (long)p.g.R * E;
  return slab_reduce_launch(p.g.slab, p.g.R, E, part, a.dw, s, a.out_mode, KT, (long)a.Cout * a.Cin);
}
