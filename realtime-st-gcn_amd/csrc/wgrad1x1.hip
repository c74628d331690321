// Weight gradient of the 1x1 convolutions (Kt = 1, stride 1): dW[co][ci] += sum_m dy[m][co] x[m][ci] over
// all M = N*T*V rows — the A-first graph conv's channel GEMM (tgcn.py:71-79 on A-mixed rows, AAGCN), the
// attention projections (aagcn.py:139-141) and the other row GEMMs.  K = M is huge and the output small,
// so this is a split-K reduction bound by reading x and dy once:
//   * a block owns a contiguous chunk of 32-row steps and a group of <= 2 x 12 (co, ci) 32x32 output tiles,
//     spread over its 4 waves (<= 6 accumulator tiles per wave);
//   * per step the group's dy and x row panels ([32 rows][32 ch] bf16) are DMA'd into LDS, a ring of 3-6
//     stages (~64 KB per block, sized to the group's panels) with all but one in flight (every wave issues a
//     fixed number of DMAs per step, so the waits are counted vmcnt waits);
//   * both MFMA operands are transposed reads of the panels (ds_read_tr16_b64: m = co / n = ci, k = rows);
//   * per-block fp32 partials go to a slab, summed over the chunks in a fixed order (deterministic).
// Served: bf16, M % 32 == 0, Cin and Cout multiples of 32, 16-B aligned rows; else the frame-tiled kernel.
#include "common.h"
#include "../../include/stgcn_amd.h"

namespace {

constexpr int NT1 = 256;
constexpr int PANEL = 32 * 64;  // [32 rows][32 ch] bf16
// co / ci blocks per group: GCO x gci with gci = all ci blocks up to 8, else 6 (a group of 14 panels took 84 KB
// of LDS at its 3-stage minimum: one block per CU; 8 panels make a 4-stage ring in 64 KB, two blocks per CU)
constexpr int GCO = 2, GCI_MAX = 8;
constexpr int TPW = GCO * GCI_MAX / 4;  // tiles per wave (<= 4)
constexpr int NSTAGE = 3;  // minimum ring depth
constexpr int TARGET_BLOCKS = 512;

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

DEV bf16x8 trfrag16(const char* panel, int row0, int lane) {
  const int i = lane & 15, gq = lane >> 4;
  const int q = i >> 2, p = i & 3, h = gq >> 1;
  const char* a0 = panel + (row0 + 8 * h + q) * 64 + (16 * (gq & 1) + 4 * p) * 2;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 4 * 64));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return __builtin_bit_cast(bf16x8, v);
}

// global -> LDS, lane-linear; asm so the compiler keeps no alias-driven vmcnt drains; m0 saved/restored
DEV void dma16(const void* src, unsigned lds_off) {
  unsigned saved;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(saved) : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds_off)) : "memory");
}
DEV unsigned lds_u32(const void* p) { return (unsigned)(size_t)(const __attribute__((address_space(3))) char*)p; }

// s_waitcnt vmcnt(n) for a wave-uniform run-time n (clamped to 63, the counter's range: waiting for fewer
// outstanding operations is always safe)
template <int N>
DEV void wait_vm_upto(int n) {
  if constexpr (N < 63) {
    if (n <= N) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
      return;
    }
    wait_vm_upto<N + 1>(n);
  } else {
    asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
  }
}
DEV void wait_vm(int n) { wait_vm_upto<0>(n < 0 ? 0 : n); }

struct W1Geom {
  long steps;    // M / 32
  int spb;       // steps per block (chunk)
  int nchunk;
  int ncog, ncig;  // groups along co / ci
  int ncob, ncib;  // 32-channel blocks
  int gci;         // ci blocks per group
  int pstage;      // panels per ring stage: the largest group's (LDS sized to it)
  int nstage;      // ring depth (3..6: ~64 KB of LDS per block)
};

__global__ __launch_bounds__(NT1) void wgrad1x1_kernel(const stgcn_wgrad_desc a, const W1Geom g, float* __restrict__ slab) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int chunk = blockIdx.x, grp = blockIdx.y;
  const int gco = grp / g.ncig, gci = grp - gco * g.ncig;
  const int cob0 = gco * GCO, cib0 = gci * g.gci;
  const int nco = min(GCO, g.ncob - cob0), nci = min(g.gci, g.ncib - cib0);
  const int npan = nco + nci;  // panels per step: the dy blocks first, then the x blocks
  const long s0 = (long)chunk * g.spb, s1 = min(g.steps, s0 + g.spb);
  if (s0 >= s1) return;  // block-uniform, before any barrier
  const bf16* __restrict__ dy = reinterpret_cast<const bf16*>(a.dy);
  const bf16* __restrict__ x = reinterpret_cast<const bf16*>(a.in);

  // DMA: panel p -> wave p % 4; two instructions (16 rows each) per panel
  const int lrow = lane >> 2, lunit = lane & 3;
  const int my_pan = (npan - wave + 3) / 4;  // panels of this wave
  const int ops = 2 * my_pan;                 // DMA instructions per step of this wave
  auto issue = [&](long st, int stage) {
    char* base = smem + stage * g.pstage * PANEL;
    for (int p = wave; p < npan; p += 4) {
      const bf16* src;
      int ld;
      if (p < nco) {
        src = dy + (cob0 + p) * 32;
        ld = a.dy_ld;
      } else {
        src = x + (cib0 + p - nco) * 32;
        ld = a.in_ld;
      }
      const bf16* r0 = src + (st * 32 + lrow) * (long)ld + lunit * 8;
      const unsigned dst = lds_u32(base + p * PANEL);
      dma16(r0, dst);
      dma16(r0 + 16L * ld, dst + 1024);
    }
  };

  // this wave's tiles: t = wave + 4k over the group's nco x nci tiles (co-major)
  const int ntile = nco * nci;
  f32x16 acc[TPW];
#pragma unroll
  for (int k = 0; k < TPW; ++k) acc[k] = f32x16{};

  const int nst = (int)(s1 - s0);
  const int ahead = g.nstage - 1;  // steps in flight
  for (int k = 0; k < ahead && k < nst; ++k) issue(s0 + k, k);
  int cur = 0, nxt = ahead;  // ring stages of step si and of step si + ahead (no run-time modulo)
  for (int si = 0; si < nst; ++si) {
    // this step's panels: own DMAs of the younger steps already issued may stay in flight
    const int left = nst - 1 - si;
    wait_vm((left < ahead - 1 ? left : ahead - 1) * ops);
    // LDS-only barrier (no vmcnt drain): every wave's DMAs of this step landed; the stage refilled below
    // was last read in the previous step
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (si + ahead < nst) issue(s0 + si + ahead, nxt);
    nxt = nxt + 1 == g.nstage ? 0 : nxt + 1;
    const char* base = smem + cur * g.pstage * PANEL;
    cur = cur + 1 == g.nstage ? 0 : cur + 1;
#pragma unroll
    for (int k = 0; k < TPW; ++k) {
      const int t = wave + 4 * k;
      if (t >= ntile) break;
      const int cb = t / nci, ib = t - cb * nci;
      const char* pdy = base + cb * PANEL;
      const char* px = base + (nco + ib) * PANEL;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16x8 fa = trfrag16(pdy, 16 * ks, lane);  // m = co, k = rows
        const bf16x8 fb = trfrag16(px, 16 * ks, lane);   // n = ci, k = rows
        acc[k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb, acc[k], 0, 0, 0);
      }
    }
  }
  // partials: D[m = co][n = ci]: lane n = ci = lane & 31, rows co = acc_row(r, lane)
  float* part = slab + (long)chunk * a.Cout * a.Cin;
#pragma unroll
  for (int k = 0; k < TPW; ++k) {
    const int t = wave + 4 * k;
    if (t >= ntile) break;
    const int cb = t / nci, ib = t - cb * nci;
    const int ci = (cib0 + ib) * 32 + (lane & 31);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = (cob0 + cb) * 32 + acc_row(r, lane);
      part[(long)co * a.Cin + ci] = acc[k][r];
    }
  }
}

// dw[e] (+)= sum over chunks of slab[c][e], fixed order: 64 entries x 16 chunk groups per block (overwrite: the
// desc's out_mode 1; Kt = 1, so both layouts agree)
__global__ __launch_bounds__(1024) void wgrad1x1_reduce_kernel(const float* __restrict__ slab, int nchunk, long E,
                                                               float* __restrict__ dw, int overwrite) {
  __shared__ float part[16][64];
  const int le = threadIdx.x & 63, q = threadIdx.x >> 6;
  const long e = (long)blockIdx.x * 64 + le;
  float s = 0.f;
  if (e < E)
    for (int c = q; c < nchunk; c += 16) s += slab[(long)c * E + e];
  part[q][le] = s;
  __syncthreads();
  if (q != 0 || e >= E) return;
  s = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) s += part[j][le];
  dw[e] = overwrite ? s : dw[e] + s;
}

bool w1_ok(const stgcn_wgrad_desc& a, int dtype) {
  const long M = (long)a.N * a.T_out * a.V;
  return dtype == 1 && a.Kt == 1 && a.stride == 1 && a.pad == 0 && a.pro == 0 && a.T_in == a.T_out && M % 32 == 0 &&
         M >= 32 && a.Cin % 32 == 0 && a.Cout % 32 == 0 && a.in_ld % 8 == 0 && a.dy_ld % 8 == 0 &&
         a.in_ld >= a.Cin && a.dy_ld >= a.Cout;
}

W1Geom w1_plan(const stgcn_wgrad_desc& a) {
  W1Geom g;
  g.steps = (long)a.N * a.T_out * a.V / 32;
  g.ncob = a.Cout / 32;
  g.ncib = a.Cin / 32;
  g.gci = g.ncib <= GCI_MAX ? g.ncib : 6;
  g.ncog = (g.ncob + GCO - 1) / GCO;
  g.ncig = (g.ncib + g.gci - 1) / g.gci;
  g.pstage = (g.ncob < GCO ? g.ncob : GCO) + g.gci;
  g.nstage = (64 * 1024) / (g.pstage * PANEL);
  g.nstage = g.nstage < NSTAGE ? NSTAGE : (g.nstage > 6 ? 6 : g.nstage);
  const int groups = g.ncog * g.ncig;
  long nch = TARGET_BLOCKS / groups;
  if (nch < 1) nch = 1;
  if (nch > g.steps) nch = g.steps;
  g.spb = (int)((g.steps + nch - 1) / nch);
  g.nchunk = (int)((g.steps + g.spb - 1) / g.spb);
  return g;
}

}  // namespace

long wgrad1x1_workspace(const stgcn_wgrad_desc& a, int dtype) {
  if (!w1_ok(a, dtype)) return 0;
  const W1Geom g = w1_plan(a);
  return (long)g.nchunk * a.Cout * a.Cin * (long)sizeof(float);
}

// -1: not handled here
int wgrad1x1_launch(const stgcn_wgrad_desc& a, int dtype, hipStream_t s) {
  if (!w1_ok(a, dtype) || !a.work) return -1;
  const W1Geom g = w1_plan(a);
  if (a.work_bytes < (long)g.nchunk * a.Cout * a.Cin * (long)sizeof(float)) return -1;
  float* slab = reinterpret_cast<float*>(a.work);
  // LDS of the actual group (the 14-panel maximum took 84 KB: one block per CU at the A-first graph conv's
  // 64 x 192 groups, whose 8 panels need 48 KB — three blocks, three times the DMAs in flight)
  const size_t lds = (size_t)g.nstage * g.pstage * PANEL;
  if (stgcn_lds_attr((const void*)wgrad1x1_kernel, (int)lds, s)) return STGCN_EHIP;
  hipLaunchKernelGGL(wgrad1x1_kernel, dim3((unsigned)g.nchunk, (unsigned)(g.ncog * g.ncig)), dim3(NT1), lds, s, a, g,
                     slab);
  if (hipGetLastError() != hipSuccess) return STGCN_EHIP;
  const long E = (long)a.Cout * a.Cin;
  hipLaunchKernelGGL(wgrad1x1_reduce_kernel, dim3((unsigned)((E + 63) / 64)), dim3(1024), 0, s, (const float*)slab,
                     g.nchunk, E, a.dw, a.out_mode);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
