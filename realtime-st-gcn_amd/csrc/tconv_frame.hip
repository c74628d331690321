// Temporal convolution of the 64-channel ST-GCN layers (the tcn's Conv2d (Kt, 1), stride 1, stgcn.py:151-159)
// forward and data gradient as a row-streaming MFMA kernel:
//
//   forward  (trans 0): out[t][v][co] = sum_dt sum_ci W[dt][co][ci] h[t + dt - 4][v][ci] + bias[co],
//                       h = relu(in * scale + shift) (BN1 + ReLU folded, pro 1) or in (pro 0); frames outside
//                       [0, T) are zeros AFTER the prologue (the conv's zero padding applies to h)
//   data grad (trans 1): out[t][v][ci] = sum_dt sum_co W'[dt][ci][co] in[t + 4 - dt][v][co]   (conv_rows' trans)
//
// out^T[c][row] = sum_{dt,k} W[dt][c][k] * in^T[k][row + (dt - 4) V]: the A fragments come from the weight's
// MFMA-fragment image (stgcn_pack_weight_frag), the B fragments are input rows read from an LDS ring, one 32x32x16
// MFMA each (36 per 32-row tile).  The accumulator is out^T (lane = row, 4 consecutive channels per register
// group): bias, 16-B row stores, BatchNorm partial sums in registers over the block's rows.
// Shapes: 16 < V <= 25 (the ring and the LDS weight fragments fit 160 KiB; every reference skeleton has 6-25
// joints).  The data gradient of the 64-channel layers ships on this kernel; a frame-per-step form
// for 25 < V <= 32 was removed in round 6 (no skeleton needs it).
#include "common.h"
#include "../../include/stgcn_amd.h"
#include <utility>

namespace {

constexpr int C = 64, KT = 9, HALO = 4;

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

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

// ------------------------------------------------------------------------------------------------------------
// Row-streaming form: the block's output rows
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

}  // namespace

long tconv_frame_row_blocks(int N, int T) {
  if (N < 1 || T < 1) return 1;
  // sized for the largest run count over 16 < V <= 25
  long m = 1;
  for (int V = 17; V <= 25; ++V) {
    const TCR r = rplan(N, T, V);
    m = r.runs_n > m ? r.runs_n : m;
  }
  return (long)N * m;
}

int tconv_frame_launch(const stgcn_conv_desc& a, hipStream_t s) {
  // V <= 25: the ring + LDS weight fragments fit 160 KiB (every reference skeleton has 6-25 joints)
  if (!a.in || !a.out || !a.w_frag || a.N < 1 || a.T_in < 1 || a.T_out != a.T_in || a.V <= 16 || a.V > 25)
    return STGCN_EBADSHAPE;
  if (a.Cin != C || a.Cout != C || a.Kt != KT || a.stride != 1 || a.pad != HALO || a.accumulate || a.in_ld % 8 ||
      a.out_ld % 8 || a.Cout_pad % 32 || a.Cin_pad % 16 || a.Cin_pad < C || a.Cout_pad < C)
    return STGCN_EBADSHAPE;
  if ((a.pro != 0 && a.pro != 1) || (a.pro == 1 && (!a.pro_a || !a.pro_b)) || (a.bias && a.bias_mode > 1))
    return STGCN_EBADSHAPE;
  const TCR r = rplan(a.N, a.T_in, a.V);
  const long nblk = (long)a.N * r.runs_n;
  if (nblk > 0x7fffffffL || (long)a.T_in * a.V > 0x3fffffffL) return STGCN_EBADSHAPE;
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
