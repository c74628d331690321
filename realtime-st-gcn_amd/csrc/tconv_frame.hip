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
  const TCF g = plan(N, T);
  return (long)N * g.runs_n;
}

int tconv_frame_launch(const stgcn_conv_desc& a, hipStream_t s) {
  if (!a.in || !a.out || !a.w_frag || a.N < 1 || a.T_in < 1 || a.T_out != a.T_in || a.V <= 16 || a.V > 32)
    return STGCN_EBADSHAPE;
  if (a.Cin != C || a.Cout != C || a.Kt != KT || a.stride != 1 || a.pad != HALO || a.accumulate || a.in_ld % 8 ||
      a.out_ld % 4 || a.Cout_pad % 32 || a.Cin_pad % 16 || a.Cin_pad < C || a.Cout_pad < C)
    return STGCN_EBADSHAPE;
  if ((a.pro != 0 && a.pro != 1) || (a.pro == 1 && (!a.pro_a || !a.pro_b)) || (a.bias && a.bias_mode > 1))
    return STGCN_EBADSHAPE;
  const TCF g = plan(a.N, a.T_in);
  typedef void (*KFn)(const stgcn_conv_desc, const TCF);
  const KFn k = a.trans ? (a.pro ? tcf_kernel<1, true> : tcf_kernel<0, true>)
                        : (a.pro ? tcf_kernel<1, false> : tcf_kernel<0, false>);
  const int lds = RS * FSL + 2 * C * 4;
  if (stgcn_lds_attr((const void*)k, lds, s)) return STGCN_EHIP;
  hipLaunchKernelGGL(k, dim3((unsigned)(a.N * g.runs_n)), dim3(NW * 64), lds, s, a, g);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
