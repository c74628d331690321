// Temporal convolution of the 64-channel ST-GCN layers (the tcn's Conv2d (Kt, 1), stride 1, stgcn.py:151-159)
// forward and data gradient as a frame-streaming MFMA kernel:
//
//   forward  (trans 0): out[t][v][co] = sum_dt sum_ci W[dt][co][ci] h[t + dt - 4][v][ci] + bias[co],
//                       h = relu(in * scale + shift) (BN1 + ReLU folded, pro 1) or in (pro 0); frames outside
//                       [0, T) are zeros AFTER the prologue (the conv's zero padding applies to h)
//   data grad (trans 1): out[t][v][ci] = sum_dt sum_co W'[dt][ci][co] in[t + 4 - dt][v][co]   (conv_rows' trans)
//
// Per output frame and 32-channel output quarter, out^T[c][v] = sum_{dt,k} W[dt][c][k] * in^T[k][v]: the 9 x 4
// A fragments (the weight's MFMA-fragment image, stgcn_pack_weight_frag) stay in registers for the whole kernel,
// the B fragments are the input frame's joint rows read from LDS, one 32x32x16 MFMA each (36 per frame).
// The accumulator is out^T (lane = joint, 4 consecutive channels per register group): bias, 8-B row stores,
// BatchNorm partial sums in registers over the block's frames.
//
// Block = (sample, run of frames), 4 waves = (32-channel quarter, frame parity): a step is two output frames,
// which read input frames t - 4 .. t + 5.  Input frames enter a ring of RS slots ([32 joint rows][64 ch] as two
// XOR-swizzled 32-channel panels) by global -> LDS DMA, L steps ahead; the prologue (BN1 + ReLU, or zeros for
// frames outside [0, T)) is applied to each frame ONCE, in place, by all threads in the step before its first
// use (the DMA cannot transform); one LDS-only barrier per step.  Every wave issues the same DMA count per step
// (dummy re-loads past the run), so the wait before a step is an exact vmcnt.
// Replaces conv_wide (forward) and conv_persist (data grad) at C = 64: there the halo of every 10-frame tile is
// staged through the helper waves' BN1 prologue 1.8 times and those waves bound the kernel.
#include "common.h"
#include "../../include/stgcn_amd.h"
#include <utility>

namespace {

constexpr int NW = 4;
constexpr int C = 64, KT = 9, HALO = 4;
constexpr int PAN = 32 * 64;   // [32 rows][32 ch] bf16
constexpr int FSL = 2 * PAN;   // one frame: two panels
constexpr int L = 2;           // DMA lookahead (steps)
constexpr int RS = 12 + 2 * L; // ring slots: 10 read + 2 being transformed + 2L in flight
constexpr int NDMA = 2;        // DMA instructions per wave per step (2 frames x 2 panels x 2 / 4 waves)
constexpr int NST = 4;         // 8-B stores per wave per output frame
constexpr int BLOCKS = 512;

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

DEV int swz(int row) { return (row >> 2) & 3; }
DEV int poff(int row, int unit) { return row * 64 + ((unit ^ swz(row)) << 4); }
DEV unsigned lds_u32(const void* p) { return (unsigned)(size_t)(const __attribute__((address_space(3))) char*)p; }

DEV void glds16(const void* src, unsigned lds_off) {
  unsigned saved;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(saved) : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds_off)) : "memory");
}

template <int N, typename F>
DEV void sfor(F&& f) {
  [&]<int... I>(std::integer_sequence<int, I...>) { (f.template operator()<I>(), ...); }(
      std::make_integer_sequence<int, N>{});
}
template <int MAXN>
DEV void wait_vm(int n) {
  sfor<MAXN + 1>([&]<int m>() {
    if (n == m) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(m) : "memory");
  });
}

struct TCF {
  int runs_n, run;  // runs per sample, output frames per run
};

template <int PRO, bool TRANS>
__global__ __launch_bounds__(NW * 64, 2) void tcf_kernel(const stgcn_conv_desc a, const TCF g) {
  constexpr int XMAX = (L - 1) * (NDMA + NST);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cq = wave & 1, fp = wave >> 1;
  const int l31 = lane & 31, lh = lane >> 5;
  const int V = a.V, T = a.T_in;
  const int n = blockIdx.x / g.runs_n;
  const int t0 = (blockIdx.x - n * g.runs_n) * g.run;
  const int t1 = min(T, t0 + g.run);
  if (n >= a.N || t0 >= T) return;  // block-uniform, before any barrier
  const int nsteps = (t1 - t0 + 1) / 2;
  const int nin = 2 * nsteps + 2 * HALO;  // input frames the run reads: j <-> frame t0 - 4 + j

  char* const ring = smem;                                        // [RS][FSL]
  float* const ssc = reinterpret_cast<float*>(smem + RS * FSL);   // [64] prologue scale
  float* const ssh = ssc + C;                                     // [64] prologue shift
  float* const red = reinterpret_cast<float*>(ring);              // epilogue scratch

  {
    uint4* z = reinterpret_cast<uint4*>(ring);
    for (int e = tid; e < RS * FSL / 16; e += NW * 64) z[e] = make_uint4(0, 0, 0, 0);
    if (PRO == 1 && tid < C) {
      ssc[tid] = a.pro_a[tid];
      ssh[tid] = a.pro_b[tid];
    }
  }
  // weight fragments of this wave's quarter: [dt][k-step] (A operand: row = output channel, k = input channel)
  bf16x8 wf[KT][4];
  {
    const uint4* src = reinterpret_cast<const uint4*>(a.w_frag);
    const int nq = a.Cout_pad / 32, k16n = a.Cin_pad / 16;
#pragma unroll
    for (int dt = 0; dt < KT; ++dt)
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
        wf[dt][kk] = __builtin_bit_cast(bf16x8, src[(((long)dt * nq + cq) * k16n + kk) * 64 + lane]);
  }
  float breg[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) breg[r] = a.bias ? a.bias[cq * 32 + acc_row(r, lane)] : 0.f;
  __syncthreads();

  const bf16* __restrict__ in = reinterpret_cast<const bf16*>(a.in);
  bf16* __restrict__ out = reinterpret_cast<bf16*>(a.out);
  const long sbase = (long)n * T;  // first frame row block of the sample
  const int prow = lane >> 2, pu = lane & 3;
  const unsigned ring0 = lds_u32(ring);
  // step k (k >= -5) DMAs input frames 2(k + L) + 10 and + 11; wave w: frame (w >> 1), panel (w & 1)
  auto issue = [&](int k) {
    const int j = 2 * (k + L) + 10 + (wave >> 1), pan = wave & 1;
    const int tt = min(max(t0 - HALO + j, 0), T - 1);  // frames outside [0, T) or past the run: dummy loads
    const bf16* base = in + (sbase + tt) * V * a.in_ld + 32 * pan;
    const unsigned dst = ring0 + (unsigned)((j % RS) * FSL + pan * PAN);
    glds16(base + (long)prow * a.in_ld + 8 * (pu ^ swz(prow)), dst);
    if (prow + 16 < V) glds16(base + (long)(prow + 16) * a.in_ld + 8 * (pu ^ swz(prow + 16)), dst + 1024);
  };
#pragma unroll
  for (int k = -5 - L; k < -5; ++k) issue(k);

  const f32x16 zero = {};
  float s1[16], s2[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    s1[r] = 0.f;
    s2[r] = 0.f;
  }
  const bool stats = a.stats != nullptr;
  const bool jok = l31 < V;

  for (int k = -5; k < nsteps; ++k) {
    {  // frames of step k landed: younger ops = (L - 1) DMA steps + the stores of this wave's output frames
      int nv = 0;
      for (int s = max(0, k - L + 1); s < k; ++s) nv += (t0 + 2 * s + fp < t1) ? 1 : 0;
      wait_vm<XMAX>((L - 1) * NDMA + NST * nv);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    // ---- prologue of input frames 2k + 10, 2k + 11 in place (2 x V rows x 8 units of 16 B)
    for (int u = tid; u < 2 * V * 8; u += NW * 64) {
      const int fi = u / (V * 8), rem = u - fi * V * 8, row = rem >> 3, pu8 = rem & 7;
      const int j = 2 * k + 10 + fi;
      if (j >= nin) continue;
      const int tt = t0 - HALO + j;
      uint4* p = reinterpret_cast<uint4*>(ring + (j % RS) * FSL + (pu8 >> 2) * PAN + row * 64 + (pu8 & 3) * 16);
      if (tt < 0 || tt >= T) {
        *p = make_uint4(0, 0, 0, 0);
      } else if (PRO == 1) {
        const int c0 = (pu8 >> 2) * 32 + (((pu8 & 3) ^ swz(row)) << 3);
        float f[8];
        unpack16(*p, f, (bf16*)nullptr);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = fmaxf(fmaf(f[e], ssc[c0 + e], ssh[c0 + e]), 0.f);
        *p = pack16(f, (bf16*)nullptr);
      }
    }
    const int t = t0 + 2 * k + fp;
    if (k >= 0 && t < t1) {
      f32x16 acc = zero;
#pragma unroll
      for (int dt = 0; dt < KT; ++dt) {
        const int j = 2 * k + fp + (TRANS ? KT - 1 - dt : dt);
        const char* slot = ring + (j % RS) * FSL;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const bf16x8 b = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(slot + (kk >> 1) * PAN +
                                                                                         poff(l31, 2 * (kk & 1) + lh)));
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[dt][kk], b, acc, 0, 0, 0);
        }
      }
      float v[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = acc[r] + breg[r];
      bf16* orow = out + ((sbase + t) * V + min(l31, V - 1)) * a.out_ld + cq * 32 + 4 * lh;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        bf16x4 st;
#pragma unroll
        for (int e = 0; e < 4; ++e) st[e] = (bf16)v[4 * q + e];
        if (jok) *reinterpret_cast<u32x2*>(orow + 8 * q) = __builtin_bit_cast(u32x2, st);
      }
      if (stats && jok) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          s1[r] += v[r];
          s2[r] = fmaf(v[r], v[r], s2[r]);
        }
      }
    }
    issue(k);  // frames 2(k + L) + 10, + 11 into the slots of frames 2k - 2, 2k - 1 (read in step k - 1 only)
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  if (!stats) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float x1 = s1[r], x2 = s2[r];
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) {
      x1 += __shfl_xor(x1, o);
      x2 += __shfl_xor(x2, o);
    }
    if (l31 == 0) {
      const int c = cq * 32 + acc_row(r, lane);
      red[(fp * 64 + c) * 2] = x1;
      red[(fp * 64 + c) * 2 + 1] = x2;
    }
  }
  __syncthreads();
  if (tid < 64) {
    const float x1 = red[tid * 2] + red[(64 + tid) * 2], x2 = red[tid * 2 + 1] + red[(64 + tid) * 2 + 1];
    const float cnt = (float)((t1 - t0) * V);
    const float mean = x1 / cnt;
    reinterpret_cast<float4*>(a.stats)[(long)blockIdx.x * a.Cout_pad + tid] =
        make_float4(cnt, mean, fmaxf(x2 - x1 * mean, 0.f), 0.f);
  }
}

// ------------------------------------------------------------------------------------------------------------
// Row-streaming form (the default; STGCN_TCF_ROWS=0 builds the frame form above for A/B): the block's output rows
// are walked in steps of 256 contiguous rows (8 row tiles of 32, not frame-aligned: no padded joint lanes), the
// input rows live in a ring of RR rows (128-B rows, XOR-swizzled: conflict-free ds_read_b128 from any row offset),
// all 8 waves (two per SIMD) run MFMAs: wave = (32-channel output half ct, row group rq), row tiles rq and rq + 4
// of every step, two independent accumulators that share each weight fragment.  Weight fragments: k-steps 0..15
// (taps 0..3) in registers, 16..35 in LDS (72 KB of fragments do not fit beside the ring) — 1.28 LDS reads of
// 1 KB per MFMA.  Staging: every thread loads 4 16-B units of the NEXT step's 256 new input rows at the start of
// a step, applies the prologue after the step's MFMAs and writes them to ring slots the step does not read;
// one LDS-only barrier per step.
// timing ablations (results wrong; tools only): bit 0 no MFMA k-loop, bit 1 no staging loads, bit 2 no output stores
#ifndef STGCN_TCR_DBG
#define STGCN_TCR_DBG 0
#endif
constexpr int TDBG = STGCN_TCR_DBG;
// bit 8: per-wave cycle accounts (s_memtime) written over the output's first rows (k-loop, barrier B1, epilogue
// writes, barrier B2, readback + stores, transform wait, total) as floats: tools/tcr_prof.py
constexpr bool TPROF = (TDBG & 256) != 0;
DEV long long tstamp() {
  if constexpr (TPROF) return __builtin_amdgcn_s_memtime();
  return 0;
}
constexpr int RW = 8;                    // waves
constexpr int RSTEP = 256;               // output rows per step
constexpr int KR = 20;                   // k-steps whose weight fragments stay in registers
constexpr int KSTEPS = KT * C / 16;      // 36

struct TCR {
  int runs_n, run;  // runs per sample, output rows per run (multiple of 32)
  int RR;           // ring rows
};

DEV int rswz(int q, int chunk) { return q * 128 + ((chunk ^ ((q >> 1) & 7)) << 4); }

template <int PRO, bool TRANS, bool STATS>
__global__ __launch_bounds__(RW * 64, 1) void tcr_kernel(const stgcn_conv_desc a, const TCR g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ct = wave & 1, rq = wave >> 1;
  const int lr = lane & 31, lh = lane >> 5;
  const int V = a.V, RS = a.T_in * a.V, RR = g.RR;
  const int n = blockIdx.x / g.runs_n;
  const int r0 = (blockIdx.x - n * g.runs_n) * g.run;
  if (n >= a.N || r0 >= RS) return;  // block-uniform, before any barrier
  const int r1 = min(RS, r0 + g.run);
  const int nsteps = (r1 - r0 + RSTEP - 1) / RSTEP;
  const int HV = HALO * V;

  char* const ring = smem;                                                  // [RR][128 B]
  char* const sw = smem + RR * 128;                                         // [16 k-steps][2 ct][1 KiB]
  float* const ssc = reinterpret_cast<float*>(sw + (KSTEPS - KR) * 2 * 1024);  // [64] prologue scale
  float* const ssh = ssc + C;                                               // [64] prologue shift
  float* const sbias = ssh + C;                                             // [64] bias
  float2* const red = reinterpret_cast<float2*>(sbias + C);                 // [4 rq][64] (sum, sum of squares)

  // ---- weight fragments: image [dt][co half][k16][64 lanes][8] (stgcn_pack_weight_frag); A operand (m = output
  // channel, k = input channel)
  const uint4* wsrc = reinterpret_cast<const uint4*>(a.w_frag);
  const int nq = a.Cout_pad / 32, k16n = a.Cin_pad / 16;
  auto wimg = [&](int k, int c) { return ((long)(k >> 2) * nq + c) * k16n + (k & 3); };
  bf16x8 wr[KR];
#pragma unroll
  for (int k = 0; k < KR; ++k) wr[k] = __builtin_bit_cast(bf16x8, wsrc[wimg(k, ct) * 64 + lane]);
  for (int e = tid; e < (KSTEPS - KR) * 2 * 64; e += RW * 64) {
    const int l = e & 63, c = (e >> 6) & 1, k = KR + (e >> 7);
    reinterpret_cast<uint4*>(sw)[e] = wsrc[wimg(k, c) * 64 + l];
  }
  if (tid < C) {
    ssc[tid] = PRO == 1 ? a.pro_a[tid] : 1.f;
    ssh[tid] = PRO == 1 ? a.pro_b[tid] : 0.f;
    sbias[tid] = a.bias ? a.bias[tid] : 0.f;
  }
  __syncthreads();

  const bf16* __restrict__ in = reinterpret_cast<const bf16*>(a.in) + (long)n * RS * a.in_ld;
  bf16* __restrict__ out = reinterpret_cast<bf16*>(a.out) + (long)n * RS * a.out_ld;
  // ---- staging by global -> LDS DMA in 8-row groups (one 1-KiB DMA per wave instruction: lane l -> row 8g + (l >> 3)
  // of the group, physical 16-B slot l & 7, i.e. logical chunk (l & 7) ^ swizzle).  Batch 0 = the first step's window
  // (q in [0, 256 + 8V)), batch b >= 1 = step b's new rows (q in [256b + 8V, 256b + 256 + 8V)), issued two steps ahead.
  // Rows outside the sample load row 0 and are zeroed by the transform.  A lane transforms (prologue / zero fill) in
  // place exactly the unit it DMA'd itself, after its own vmcnt wait: no barrier between landing and transform.
  const unsigned ring0 = lds_u32(ring);
  const int drow = lane >> 3, dslot = lane & 7;
  auto dma_group = [&](int q) {  // q: first ring-relative row of the group (wave-uniform, a multiple of 8)
    const int p = q % RR;        // RR % 8 == 0: a group never wraps
    const int ir = r0 - HV + q + drow;
    const int irc = (ir >= 0 && ir < RS) ? ir : 0;
    const int c = dslot ^ (((p + drow) >> 1) & 7);
    if (TDBG & 2) return;
    glds16(in + (long)irc * a.in_ld + c * 8, ring0 + (unsigned)(p * 128));
  };
  auto xform_group = [&](int q) {
    const int p = q % RR;
    const int ir = r0 - HV + q + drow;
    uint4* u = reinterpret_cast<uint4*>(ring + p * 128 + lane * 16);
    if (ir < 0 || ir >= RS) {
      *u = make_uint4(0, 0, 0, 0);
    } else if (PRO == 1) {
      const int c = dslot ^ (((p + drow) >> 1) & 7);
      float f[8];
      unpack16(*u, f, (bf16*)nullptr);
      const float4 a0 = *reinterpret_cast<const float4*>(ssc + 8 * c), a1 = *reinterpret_cast<const float4*>(ssc + 8 * c + 4);
      const float4 b0 = *reinterpret_cast<const float4*>(ssh + 8 * c), b1 = *reinterpret_cast<const float4*>(ssh + 8 * c + 4);
      const float sa[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
      const float sb[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = fmaxf(fmaf(f[e], sa[e], sb[e]), 0.f);
      *u = pack16(f, (bf16*)nullptr);
    }
  };
  const int win = RSTEP + 2 * HV;  // rows of batch 0
  auto batch_q = [&](int b, int j) { return RSTEP * b + 2 * HV + 8 * (wave + 8 * j); };  // b >= 1, j < 4
  // prologue: batches 0 and 1 landed and transformed
  for (int q = 8 * wave; q < win; q += 64) dma_group(q);
#pragma unroll
  for (int j = 0; j < 4; ++j) dma_group(batch_q(1, j));
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int q = 8 * wave; q < win; q += 64) xform_group(q);
#pragma unroll
  for (int j = 0; j < 4; ++j) xform_group(batch_q(1, j));
  __syncthreads();

  float s1[16], s2[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) s1[r] = s2[r] = 0.f;
  int cnt = 0;
  const f32x16 zero = {};
  int bs = 0;  // physical slot of q = 256 s
  f32x16 ap[2] = {zero, zero};  // the previous step's accumulators
  // one epilogue unit: tile i, channel groups q4 = 2 pr, 2 pr + 1 of output row r0 + 256 sp + 32 (rq + 4 i) + lr.
  // A lane holds 4 channels of each group (32 ct + 8 q4 + 4 lh ..); one v_permlane32_swap per dword gives lanes
  // 0-31 the 8 channels of group 2 pr and lanes 32-63 those of group 2 pr + 1: ONE 16-B store per lane instead of
  // two 8-B stores (the epilogue is store-issue bound)
  auto ep_unit = [&](int i, int pr, int sp) {
    const int o = r0 + RSTEP * sp + 32 * (rq + 4 * i) + lr;
    const bool ok = o < r1;
    if (pr == 0) cnt += ok ? 1 : 0;
    unsigned pk[2][2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int q4 = 2 * pr + h;
      const float4 b4 = *reinterpret_cast<const float4*>(sbias + 32 * ct + 8 * q4 + 4 * lh);
      const float bb[4] = {b4.x, b4.y, b4.z, b4.w};
      bf16x4 st;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float v = ap[i][4 * q4 + e];
        if (STATS && ok) {
          s1[4 * q4 + e] += v;
          s2[4 * q4 + e] = fmaf(v, v, s2[4 * q4 + e]);
        }
        st[e] = (bf16)(v + bb[e]);
      }
      const u32x2 w2 = __builtin_bit_cast(u32x2, st);
      pk[h][0] = w2.x;
      pk[h][1] = w2.y;
    }
#pragma unroll
    for (int d = 0; d < 2; ++d) {
      const auto r = __builtin_amdgcn_permlane32_swap(pk[0][d], pk[1][d], false, false);
      pk[0][d] = r[0];
      pk[1][d] = r[1];
    }
    if (ok && !(TDBG & 4))
      *reinterpret_cast<uint4*>(out + (long)o * a.out_ld + 32 * ct + 16 * pr + 8 * lh) =
          make_uint4(pk[0][0], pk[0][1], pk[1][0], pk[1][1]);
  };
  long long pa[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const long long pstart = tstamp();
  for (int s = 0; s < nsteps; ++s) {
    const long long p0 = tstamp();
    const bool ahead = s + 2 < nsteps;
    if (ahead) {
#pragma unroll
      for (int j = 0; j < 4; ++j) dma_group(batch_q(s + 2, j));
    }
    // ---- MFMAs: tiles t = rq, rq + 4 of the step; B fragment of tap e (input row offset e*V from the window start).
    // The previous step's epilogue (acc -> + bias -> bf16 8-B stores, BN partials) is spread over the first 8
    // k-steps, one (tile, 4-channel group) unit per k-step between the MFMAs, instead of a phase of its own in which
    // every wave of the block would leave the matrix cores idle at once.
    f32x16 acc[2] = {zero, zero};
    int ra[2], rx[2];  // row byte address and swizzle key of the current tap, per tile
    auto tap_addr = [&](int dt) {
      const int e = TRANS ? KT - 1 - dt : dt;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        int q = bs + 32 * (rq + 4 * i) + lr + e * V;
        q -= q >= RR ? RR : 0;
        ra[i] = q * 128;
        rx[i] = lh ^ ((q >> 1) & 7);
        asm volatile("" : "+v"(ra[i]), "+v"(rx[i]));
      }
    };
    auto hread = [&](int i, int ks) {
      return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(ring + ra[i] + (((2 * ks) ^ rx[i]) << 4)));
    };
    auto wread = [&](int k) {
      return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(sw + (((k - KR) * 2 + ct) * 64 + lane) * 16));
    };
    bf16x8 fb[3][2], fw[3];
    tap_addr(0);
    fb[0][0] = hread(0, 0);
    fb[0][1] = hread(1, 0);
    fb[1][0] = hread(0, 1);
    fb[1][1] = hread(1, 1);
    const bool prev = s >= 1;
    if (!(TDBG & 1)) sfor<KSTEPS>([&]<int k>() {
      constexpr int k2 = k + 2;
      if constexpr (k2 < KSTEPS) {
        if constexpr ((k2 & 3) == 0) tap_addr(k2 >> 2);
        fb[k2 % 3][0] = hread(0, k2 & 3);
        fb[k2 % 3][1] = hread(1, k2 & 3);
        if constexpr (k2 >= KR) fw[k2 % 3] = wread(k2);
      }
      bf16x8 w;
      if constexpr (k < KR) w = wr[k];
      else w = fw[k % 3];
      acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w, fb[k % 3][0], acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w, fb[k % 3][1], acc[1], 0, 0, 0);
      if constexpr (k < 4) {
        if (prev) ep_unit(k >> 1, k & 1, s - 1);
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the reads two k-steps ahead (the scheduler sinks them to their use)
    });
    ap[0] = acc[0];
    ap[1] = acc[1];
    const long long p1 = tstamp();
    pa[0] += p1 - p0;
    // ---- batch s + 1 (DMA'd in step s - 1; batch 1 in the prologue) landed: transform it (the vmcnt wait leaves the
    // batch s + 2 DMAs outstanding; the stores before them are a step old)
    if (s >= 1 && s + 1 < nsteps) {
      if (ahead) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int j = 0; j < 4; ++j) xform_group(batch_q(s + 1, j));
    }
    const long long p2 = tstamp();
    pa[5] += p2 - p1;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // window s read by all, batch s + 1 transformed
    pa[1] += tstamp() - p2;
    bs += RSTEP;
    bs -= bs >= RR ? RR : 0;
  }
  {
    const long long p3 = tstamp();
#pragma unroll
    for (int u = 0; u < 4; ++u) ep_unit(u >> 1, u & 1, nsteps - 1);
    pa[2] += tstamp() - p3;
  }
  if constexpr (TPROF) {
    pa[6] = tstamp() - pstart;
    pa[7] = nsteps;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane < 8) reinterpret_cast<float*>(a.out)[((long)blockIdx.x * RW + wave) * 8 + lane] = (float)pa[lane];
    return;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may land after the block's LDS is released
  if (!STATS) return;
  // ---- BN partials of the block: per (rq, channel) lane sums -> LDS, combined over rq in a fixed order; the sums
  // are of z - bias (the bias is the pivot: added back to the mean)
  int ctot = cnt;
#pragma unroll
  for (int o = 1; o < 32; o <<= 1) ctot += __shfl_xor(ctot, o);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float x1 = s1[r], x2 = s2[r];
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) {
      x1 += __shfl_xor(x1, o);
      x2 += __shfl_xor(x2, o);
    }
    if (lr == 0) red[rq * C + 32 * ct + acc_row(r, lane)] = make_float2(x1, x2);
  }
  __shared__ int scnt[4];
  if (lane == 0 && ct == 0) scnt[rq] = ctot;
  __syncthreads();
  if (tid < C) {
    float x1 = 0.f, x2 = 0.f;
    int c = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x1 += red[j * C + tid].x;
      x2 += red[j * C + tid].y;
      c += scnt[j];
    }
    const float fc = (float)c;
    const float mu = c ? x1 / fc : 0.f;
    reinterpret_cast<float4*>(a.stats)[(long)blockIdx.x * a.Cout_pad + tid] =
        c ? make_float4(fc, sbias[tid] + mu, fmaxf(x2 - x1 * mu, 0.f), 0.f) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

TCR rplan(int N, int T, int V) {
  TCR g{};
  const int RS = T * V;
  int runs = 256 / (N > 0 ? N : 1);
  if (runs < 1) runs = 1;
  int run = (RS + runs - 1) / runs;
  run = (run + 31) / 32 * 32;
  g.run = run;
  g.runs_n = (RS + run - 1) / run;
  g.RR = (3 * RSTEP + 2 * HALO * V + 15) / 16 * 16;  // window + two batches ahead
  return g;
}

#ifndef STGCN_TCF_ROWS
#define STGCN_TCF_ROWS 1
#endif

TCF plan(int N, int T) {
  TCF g{};
  int runs = BLOCKS / (N > 0 ? N : 1);
  if (runs < 1) runs = 1;
  g.run = (T + runs - 1) / runs;
  g.run += g.run & 1;  // even: steps of two frames
  g.runs_n = (T + g.run - 1) / g.run;
  return g;
}

}  // namespace

long tconv_frame_row_blocks(int N, int T) {
  if (N < 1 || T < 1) return 1;
  // sized for the largest run count of either form over 16 < V <= 32 (the row form runs V <= 25)
  long m = plan(N, T).runs_n;
  if (STGCN_TCF_ROWS)
    for (int V = 17; V <= 25; ++V) {
      const TCR r = rplan(N, T, V);
      m = r.runs_n > m ? r.runs_n : m;
    }
  return (long)N * m;
}

int tconv_frame_launch(const stgcn_conv_desc& a, hipStream_t s) {
  if (!a.in || !a.out || !a.w_frag || a.N < 1 || a.T_in < 1 || a.T_out != a.T_in || a.V <= 16 || a.V > 32)
    return STGCN_EBADSHAPE;
  if (a.Cin != C || a.Cout != C || a.Kt != KT || a.stride != 1 || a.pad != HALO || a.accumulate || a.in_ld % 8 ||
      a.out_ld % 4 || a.Cout_pad % 32 || a.Cin_pad % 16 || a.Cin_pad < C || a.Cout_pad < C)
    return STGCN_EBADSHAPE;
  if ((a.pro != 0 && a.pro != 1) || (a.pro == 1 && (!a.pro_a || !a.pro_b)) || (a.bias && a.bias_mode > 1))
    return STGCN_EBADSHAPE;
  if (STGCN_TCF_ROWS && a.V <= 25) {  // the ring + LDS weight fragments fit 160 KiB up to V = 25
    const TCR r = rplan(a.N, a.T_in, a.V);
    const long nblk = (long)a.N * r.runs_n;
    if (nblk > 0x7fffffffL || (long)a.T_in * a.V > 0x3fffffffL || a.out_ld % 8) return STGCN_EBADSHAPE;
    typedef void (*RFn)(const stgcn_conv_desc, const TCR);
    static const RFn tab[2][2][2] = {{{tcr_kernel<0, false, false>, tcr_kernel<0, false, true>},
                                      {tcr_kernel<0, true, false>, tcr_kernel<0, true, true>}},
                                     {{tcr_kernel<1, false, false>, tcr_kernel<1, false, true>},
                                      {tcr_kernel<1, true, false>, tcr_kernel<1, true, true>}}};
    const RFn k = tab[a.pro ? 1 : 0][a.trans ? 1 : 0][a.stats ? 1 : 0];
    const int lds = r.RR * 128 + (KSTEPS - KR) * 2 * 1024 + 3 * C * 4 + 4 * C * 8;
    if (lds > 160 * 1024 || stgcn_lds_attr((const void*)k, lds, s)) return STGCN_EHIP;
    hipLaunchKernelGGL(k, dim3((unsigned)nblk), dim3(RW * 64), lds, s, a, r);
    return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
  }
  const TCF g = plan(a.N, a.T_in);
  typedef void (*KFn)(const stgcn_conv_desc, const TCF);
  const KFn k = a.trans ? (a.pro ? tcf_kernel<1, true> : tcf_kernel<0, true>)
                        : (a.pro ? tcf_kernel<1, false> : tcf_kernel<0, false>);
  const int lds = RS * FSL + 2 * C * 4;
  if (stgcn_lds_attr((const void*)k, lds, s)) return STGCN_EHIP;
  hipLaunchKernelGGL(k, dim3((unsigned)(a.N * g.runs_n)), dim3(NW * 64), lds, s, a, g);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
