// Graph convolution (ConvTemporalGraphical, tgcn.py:58-79) forward and data gradient as a frame-streaming
// MFMA kernel: the tgcn's own order, the 1x1 conv first and the joint mix after, per frame, with nothing
// intermediate leaving the registers.
//
//   out[(i,a)][r] (+)= sum_p sum_b M_p[b][a] Y_p[(i,b)][r]  (+ bias[a][r]),   Y_p[(i,b)][r] = sum_c U_p[r][c] in[(i,b)][c]
//   forward:   in = x,  M_p = A_p (b = v, a = w),   U_p[co][ci] = W[p*Cout+co][ci]
//   data grad: in = dg, M_p[w][v] = A_p[v][w],      U_p[ci][co] = W[p*Cout+co][ci]    (autograd of tgcn.py:71-79)
//
// Per frame (V <= 32 joint rows, zero-padded to 32) and 32-channel output quarter:
//   Y_p  = in_i U_p^T        M = joint b, N = r, K = c: A operand = the frame's rows (LDS), B = U_p^T fragments (LDS)
//   out^T += Y_p^T M_p       M = r, N = joint a, K = b: the Y_p accumulators ARE the A operand (K = b in the
//                            accumulator's row order; M_p's fragments are built in that order)
// The accumulator holds out^T (lane = joint a, rows = 4 consecutive channels per register group): bias,
// optional read-modify-write (accumulate; the old rows come through the same DMA ring), 8-B row stores,
// BatchNorm partial sums in registers over the block's frames.
//
// Block = (64 output channels, run of frames), 4 waves = (32-channel quarter, frame parity): a step is 2 frames;
// the frames' input rows (and, accumulating, the old output rows) are DMA'd global -> LDS as [32 row][32 ch]
// panels with XOR-swizzled 16-B units into a ring of D steps, every wave issuing the same number of DMA
// instructions per step (dummy re-loads past the end), so the wait before step k is an exact vmcnt.  The
// block's U slice ([2 quarters][P * Cin / 16 k-steps] fragments, 1 KiB each) sits in LDS, copied from the Kt = P
// MFMA-fragment image of U (stgcn_pack_weight_frag of U viewed (P, rows, Cin)).
// Replaces the joint-gathered GEMM (gconv.hip) where Cin <= 128: that kernel's blocks are (128 frames, one
// joint, 64 channels) with a 3-step K loop, latency-bound (2.5 TB/s at C = 64).
#include "common.h"
#include "../../include/stgcn_amd.h"
#include <utility>

namespace {

constexpr int NW = 4;
constexpr int PAN = 32 * 64;  // [32 rows][32 ch] bf16
constexpr int BLOCKS = 512;   // 2 per CU
// timing ablations (results wrong; tools builds only, -DGCF_DBG=<mask>): 1 skip the LDS reads and MFMAs, 2 skip the
// output stores, 4 skip the DMA, 8 skip the per-step barrier
#ifndef GCF_DBG
#define GCF_DBG 0
#endif

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
DEV void wait_vm(int n) {  // s_waitcnt vmcnt(n), n a runtime value <= MAXN
  sfor<MAXN + 1>([&]<int m>() {
    if (n == m) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(m) : "memory");
  });
}

DEV bf16x8 cvt8(const f32x16& c, int base) {
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (bf16)c[base + j];
  return v;
}

// ring depth in steps: the U slice (2 * P * G * 2 KiB) plus D slots within 80 KiB (two blocks per CU), except
// the accumulating Cin = 128 form (one block per CU: 144 KiB)
constexpr int ring_depth(int G, bool acc) { return G == 2 ? (acc ? 3 : 6) : (acc ? 4 : 2); }

struct GCF {
  int ncol, R, FB;
};

// G = Cin / 32 input panels per frame; ACC: read-modify-write of the output
template <int P, int G, bool ACC>
__global__ __launch_bounds__(NW * 64, 2) void gcf_kernel(const stgcn_gcn_tile_desc a, const GCF g) {
  constexpr int K16 = P * G * 2;                 // k-steps of U per quarter
  constexpr int IN_P = 2 * G, OLD_P = ACC ? 4 : 0;  // panels per step (2 frames)
  constexpr int SLOT = (IN_P + OLD_P) * PAN;
  constexpr int D = ring_depth(G, ACC);          // ring depth (steps)
  constexpr int NDMA = (IN_P + OLD_P) * 2 / NW;  // DMA instructions per wave per step
  constexpr int NST = 4;                         // 8-B stores per wave per frame
  constexpr int XMAX = (D - 2) * (NDMA + NST);
  static_assert(((IN_P + OLD_P) * 2) % NW == 0 && XMAX <= 63, "dma");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int rq = wave & 1, fp = wave >> 1;
  const int l31 = lane & 31, lh = lane >> 5;
  const int V = a.V;

  int wg;
  {
    const int id = blockIdx.x, nb = gridDim.x, x = id & 7, q = nb >> 3, r = nb & 7;
    wg = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (id >> 3);
  }
  const int ct = wg % g.ncol, rb = wg / g.ncol;
  const int f0 = min(a.NT, rb * g.FB), f1 = min(a.NT, f0 + g.FB);
  const int nsteps = (f1 - f0 + 1) / 2;
  const int c0 = ct * 64;

  char* const sU = smem;                          // [2][K16][64 lanes] x 16 B
  char* const ring = smem + 2 * K16 * 1024;       // [D][SLOT]
  float* const red = reinterpret_cast<float*>(ring);  // epilogue scratch (after the loop)

  // ---- U slice -> LDS: the Kt = P fragment image of U (blocks [p][32-row quarter][16-column step]) -> [q][p*2G + c16];
  // ring zeroed (rows V..31 stay zero)
  {
    const uint4* src = reinterpret_cast<const uint4*>(a.w_frag);
    uint4* dst = reinterpret_cast<uint4*>(sU);
    const int nq = a.Cout_pad / 32, k16n = a.Kw_pad / 16;
    for (int e = tid; e < 2 * K16 * 64; e += NW * 64) {
      const int blk = e >> 6, q = blk / K16, k = blk - q * K16, p = k / (2 * G), c16 = k - p * 2 * G;
      dst[e] = src[(((long)p * nq + 2 * ct + q) * k16n + c16) * 64 + (e & 63)];
    }
    uint4* z = reinterpret_cast<uint4*>(ring);
    for (int e = tid; e < D * SLOT / 16; e += NW * 64) z[e] = make_uint4(0, 0, 0, 0);
  }
  // ---- M_p fragments (B operand of the mix: lane = joint a, k = b in the accumulator's row order),
  // bias of this lane's joint and rows
  bf16x8 mf[P][2];
  {
    const int av = min(l31, V - 1);
#pragma unroll
    for (int p = 0; p < P; ++p)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        float m[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int b = min(16 * s + 4 * lh + (j & 3) + 8 * (j >> 2), V - 1);
          // forward M_p[b][a] = A[p][b][a]; data grad M_p[b][a] = A[p][a][b]
          m[j] = a.trans_a ? a.A[((long)p * V + av) * V + b] : a.A[((long)p * V + b) * V + av];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int b = 16 * s + 4 * lh + (j & 3) + 8 * (j >> 2);
          mf[p][s][j] = (bf16)((b < V && l31 < V) ? m[j] : 0.f);
        }
      }
  }
  const bool jok = l31 < V;
  float breg[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int ch = c0 + rq * 32 + acc_row(r, lane);
    breg[r] = (a.bias && jok) ? a.bias[(long)l31 * a.Cout + ch] : 0.f;
  }
  __syncthreads();

  // ---- DMA plan: the step's panels, (frame parity, input panel) then (frame parity, old-output quarter);
  // panel e of the step -> wave e % NW's instructions (rows 0-15, rows 16-31 masked to V)
  const bf16* __restrict__ in = reinterpret_cast<const bf16*>(a.in);
  bf16* __restrict__ out = reinterpret_cast<bf16*>(a.out);
  const int prow = lane >> 2, pu = lane & 3;
  const unsigned ring0 = lds_u32(ring);
  auto issue = [&](int k) {
    const unsigned slot = ring0 + (unsigned)((k % D) * SLOT);
#pragma unroll
    for (int i = 0; i < NDMA / 2; ++i) {
      const int e = wave + NW * i;  // panel index within the step (wave-uniform)
      const bool old = e >= IN_P;
      const int pe = old ? e - IN_P : e;
      const int fpar = old ? pe >> 1 : pe / G, pan = old ? pe & 1 : pe % G;
      const int f = min(f0 + 2 * k + fpar, f1 - 1);  // dummy re-load of a valid frame past the end
      const bf16* base = old ? out + (long)f * V * a.out_ld + c0 + 32 * pan : in + (long)f * V * a.in_ld + 32 * pan;
      const long ld = old ? a.out_ld : a.in_ld;
      const unsigned dst = slot + (unsigned)(e * PAN);
      glds16(base + (long)prow * ld + 8 * (pu ^ swz(prow)), dst);
      if (prow + 16 < V) glds16(base + (long)(prow + 16) * ld + 8 * (pu ^ swz(prow + 16)), dst + 1024);
    }
  };
#pragma unroll
  for (int k = 0; k < D - 1; ++k)
    if constexpr (!(GCF_DBG & 4)) issue(k);

  const f32x16 zero = {};
  float s1[16], s2[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    s1[r] = 0.f;
    s2[r] = 0.f;
  }
  const bool stats = a.stats != nullptr;
  const bool has_out = a.out != nullptr;  // NULL: BatchNorm statistics only (pass 1 of the fused BN layer)

  for (int k = 0; k < nsteps; ++k) {
    // ops issued after step k's DMA: (D - 2) DMA steps + the stores of this wave's valid frames among the
    // last (D - 2) steps (frames are valid up to some step, then not)
    {
      const int j0 = max(0, k - D + 2);
      int nv = 0;
      for (int j = j0; j < k; ++j) nv += (f0 + 2 * j + fp < f1) ? 1 : 0;
      wait_vm<XMAX>((D - 2) * NDMA + (has_out ? NST : 0) * nv);
    }
    if constexpr (!(GCF_DBG & 8)) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    const int f = f0 + 2 * k + fp;
    if (f < f1) {
      const char* slot = ring + (k % D) * SLOT;
      const char* pin = slot + fp * G * PAN;
      f32x16 acc = zero;
#pragma unroll
      for (int p = 0; p < P; ++p) {
        if constexpr ((GCF_DBG & 1) != 0) break;
        f32x16 y = zero;
#pragma unroll
        for (int kk = 0; kk < 2 * G; ++kk) {
          const bf16x8 xa =
              __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(pin + (kk >> 1) * PAN + poff(l31, 2 * (kk & 1) + lh)));
          const bf16x8 ub = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(sU + ((rq * K16 + p * 2 * G + kk) * 64 + lane) * 16));
          y = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xa, ub, y, 0, 0, 0);
        }
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cvt8(y, 0), mf[p][0], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cvt8(y, 8), mf[p][1], acc, 0, 0, 0);
      }
      // out row (f, joint l31), channels c0 + 32 rq + 8q + 4h + e
      float v[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = acc[r] + breg[r];
      if constexpr (ACC) {
        const char* pold = slot + (IN_P + 2 * fp + rq) * PAN;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const bf16x4 o = __builtin_bit_cast(bf16x4, *reinterpret_cast<const u32x2*>(pold + poff(l31, q) + 8 * lh));
#pragma unroll
          for (int e = 0; e < 4; ++e) v[4 * q + e] += (float)o[e];
        }
      }
      bf16* orow = out + ((long)f * V + min(l31, V - 1)) * a.out_ld + c0 + rq * 32 + 4 * lh;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        bf16x4 st;
#pragma unroll
        for (int e = 0; e < 4; ++e) st[e] = (bf16)v[4 * q + e];
        // lanes past V store nothing; the wave's store instruction still issues (counted above)
        if (!(GCF_DBG & 2) && has_out && jok) *reinterpret_cast<u32x2*>(orow + 8 * q) = __builtin_bit_cast(u32x2, st);
      }
      if (stats && jok) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          s1[r] += v[r];
          s2[r] = fmaf(v[r], v[r], s2[r]);
        }
      }
    }
    if constexpr (!(GCF_DBG & 4)) issue(k + D - 1);  // into the slot read in step k - 1 (every wave is past this step's barrier)
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  if (!stats) return;
  // ---- BatchNorm partials of the block: sums over joints (lanes of a half) and the two frame parities
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float x1 = s1[r], x2 = s2[r];
#pragma unroll
    for (int o = 1; o < 32; o <<= 1) {
      x1 += __shfl_xor(x1, o);
      x2 += __shfl_xor(x2, o);
    }
    if (l31 == 0) {
      const int c = rq * 32 + acc_row(r, lane);
      red[(fp * 64 + c) * 2] = x1;
      red[(fp * 64 + c) * 2 + 1] = x2;
    }
  }
  __syncthreads();
  if (tid < 64) {
    const float t1 = red[tid * 2] + red[(64 + tid) * 2], t2 = red[tid * 2 + 1] + red[(64 + tid) * 2 + 1];
    const float n = (float)((f1 - f0) * V);
    const float mean = n > 0.f ? t1 / n : 0.f;
    reinterpret_cast<float4*>(a.stats)[(long)rb * a.Cout_pad + c0 + tid] =
        make_float4(n, mean, fmaxf(t2 - t1 * mean, 0.f), 0.f);
  }
}

GCF plan(int NT, int Cout) {
  GCF g{};
  g.ncol = Cout / 64;
  int R = BLOCKS / (g.ncol > 0 ? g.ncol : 1);
  if (R < 1) R = 1;
  if (R > NT) R = NT;
  g.FB = (NT + R - 1) / R;
  g.R = (NT + g.FB - 1) / g.FB;
  return g;
}

}  // namespace

long gcn_frame_row_blocks(int NT, int Cout) {
  if (NT < 1 || Cout < 64) return 1;
  return plan(NT, Cout).R;
}

int gcn_frame_launch(const stgcn_gcn_tile_desc& a, hipStream_t s) {
  if (a.V <= 16 || a.V > 32 || a.P < 1 || a.P > 3 || a.NT < 1 || !a.in || !a.w_frag || !a.A) return STGCN_EBADSHAPE;
  if (!a.out && (!a.stats || a.accumulate)) return STGCN_EBADSHAPE;  // statistics-only launches need stats
  if ((a.Cin != 64 && a.Cin != 128) || a.in_ld % 8 || a.Cout % 64 || a.Cout_pad < a.Cout || a.out_ld % 8)
    return STGCN_EBADSHAPE;
  if (a.Kw_pad < a.Cin || a.Kw_pad % 16 || a.Cout_pad % 32) return STGCN_EBADSHAPE;
  const GCF g = plan(a.NT, a.Cout);
  const int G = a.Cin / 32;
  const bool acc = a.accumulate != 0;
  const int slot = (2 * G + (acc ? 4 : 0)) * PAN;
  const size_t lds = (size_t)2 * a.P * G * 2 * 1024 + (size_t)ring_depth(G, acc) * slot;
  typedef void (*KFn)(const stgcn_gcn_tile_desc, const GCF);
#define GCF_ROW(P) {gcf_kernel<P, 2, false>, gcf_kernel<P, 4, false>, gcf_kernel<P, 2, true>, gcf_kernel<P, 4, true>}
  static const KFn tab[3][4] = {GCF_ROW(1), GCF_ROW(2), GCF_ROW(3)};
#undef GCF_ROW
  const KFn k = tab[a.P - 1][(G == 4 ? 1 : 0) + (acc ? 2 : 0)];
  if (stgcn_lds_attr((const void*)k, (int)lds, s)) return STGCN_EHIP;
  hipLaunchKernelGGL(k, dim3((unsigned)(g.R * g.ncol)), dim3(NW * 64), lds, s, a, g);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
