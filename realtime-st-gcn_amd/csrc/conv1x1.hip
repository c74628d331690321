// 1x1 convolutions of the layer (residual.0 stgcn.py:165-170 at stride 1 or 2, and their input grads)
// as a row GEMM: out[m][co] (+)= sum_ci W[co][ci] in[row(m)][ci] (+ bias[co]), with optional BatchNorm
// partial statistics of the output.
//   forward, stride S:  row(m) = input row of frame S*t for output frame t (the temporal subsampling of
//                       a 1x1 conv with stride (S, 1));
//   trans (input grad): output frame t takes input frame t/S when S divides t, else it is zero (the
//                       transposed strided 1x1 conv scatters into every S-th frame only).
// A tile is 128 output rows x BN output channels; the block stages its 128 input rows whole (all Cin
// channels, rows padded by 16 B: conflict-free ds_read_b128) and streams the Kt = 1 MFMA-fragment
// image of W (stgcn_pack_weight_frag) from L2 straight into registers; 4 waves = 2 row halves x 2
// column halves, 32x32x16 bf16 MFMA.  The epilogue adds the bias, computes per-channel Welford
// partials on the fp32 sums and writes 16-B rows through an LDS transpose of the tile.
// The frame-tiled conv_tile kernel staged (F-1)*S + 1 input frames per F output frames with the
// generic Kt halo logic: at stride 2 half of every halo was discarded; this kernel reads each needed
// input row once.
#include "common.h"
#include "../../include/stgcn_amd.h"
#include <stdlib.h>

namespace {

constexpr int BM = 128;  // output rows per tile
constexpr int NT = 256;

struct XGeom {
  long M;     // output rows
  int ncol;   // column tiles
  int nrow;   // row tiles
  int k16n;   // K blocks per column of the fragment image (Cin_pad / 16)
};

template <int KS, int BN, bool ROWB>
__global__ __launch_bounds__(NT, 2) void conv1x1_kernel(const stgcn_conv_desc a, const XGeom g) {
  constexpr int CIN = KS * 16;
  constexpr int RS = CIN * 2 + 16;           // padded LDS row (bytes)
  constexpr int TM = 2, TN = BN / 64;        // wave tile: 64 rows x BN/2 columns
  constexpr int UPR = CIN / 8;               // 16-B units per input row
  constexpr int AU = BM * UPR / NT;          // units per thread
  static_assert(BM * UPR % NT == 0, "A units");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int lr = lane & 31, lh = lane >> 5;
  // the column tiles of one row tile are consecutive rounds on ONE XCD (block ids are dealt round-robin over the
  // 8 XCDs): the staged input rows come from HBM once and from that XCD's L2 for the other column tiles
  // (with the row tile's ncol blocks spread over ncol XCDs the input was fetched ncol times)
  const int L = blockIdx.x, k = L >> 3;
  const int ct = k % g.ncol, rt = (k / g.ncol) * 8 + (L & 7);
  if (rt >= g.nrow) return;  // block-uniform, before any barrier
  const long m0 = (long)rt * BM;
  const int n0 = ct * BN;
  const int V = a.V, S = a.stride;

  // ---- stage the tile's input rows (zero rows: past M, or frames the transposed conv does not feed)
  const bf16* __restrict__ in = reinterpret_cast<const bf16*>(a.in);
  {
    uint4 ra[AU];
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      const int e = tid + u * NT, row = e / UPR, cu = e % UPR;
      const long m = m0 + row;
      ra[u] = make_uint4(0, 0, 0, 0);
      if (m < g.M) {
        const long fr = m / V;
        const int v = (int)(m - fr * V);
        const int t = (int)(fr % a.T_out);
        const long n = fr / a.T_out;
        int ti = -1;
        if (!a.trans) ti = t * S;
        else if (t % S == 0) ti = t / S;
        if (ti >= 0) ra[u] = *reinterpret_cast<const uint4*>(in + ((n * a.T_in + ti) * V + v) * a.in_ld + cu * 8);
      }
    }
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      const int e = tid + u * NT, row = e / UPR, cu = e % UPR;
      *reinterpret_cast<uint4*>(smem + row * RS + cu * 16) = ra[u];
    }
  }
  __syncthreads();

  // ---- K loop: A fragments from LDS, B fragments (fragment image blocks [c32][k16]) from L2
  const bf16* __restrict__ wf = reinterpret_cast<const bf16*>(a.w_frag);
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const char* arow[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) arow[i] = smem + ((wm * TM + i) * 32 + lr) * RS + lh * 16;
  const bf16* bcol[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) bcol[j] = wf + (long)((n0 >> 5) + wn * TN + j) * g.k16n * 512 + lane * 8;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    bf16x8 fb[TN], fa[TM];
#pragma unroll
    for (int j = 0; j < TN; ++j) fb[j] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(bcol[j] + ks * 512));
#pragma unroll
    for (int i = 0; i < TM; ++i) fa[i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(arow[i] + ks * 32));
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
  }

  // ---- epilogue: bias, BN partials (fp32 values of the valid rows), bf16 tile -> LDS -> 16-B rows
  const int rows_valid = (int)((g.M - m0) < BM ? (g.M - m0) : BM);
  __syncthreads();  // every wave is done reading the staged rows
  constexpr int OS = BN * 2 + 16;  // padded output row in LDS
  float4* red = reinterpret_cast<float4*>(smem + BM * OS);  // [2 row halves][BN]
  // ROWB: each row's bias row index, once per tile (a 64-bit division per accumulator element cost 3x the kernel)
  int* const sbi = reinterpret_cast<int*>(smem + BM * OS + 2 * BN * 16);
  if (ROWB) {
    for (int t = tid; t < BM; t += NT) {
      const long m = m0 + (t < rows_valid ? t : 0);
      const long fr = m / V;
      const int v = (int)(m - fr * V);
      sbi[t] = a.bias_mode == 2 ? v : (int)((fr / a.T_out) * V + v);
    }
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int cl = (wn * TN + j) * 32 + lr;  // column within the tile
    const int col = n0 + cl;
    const float b = (!ROWB && a.bias && a.bias_mode == 1) ? a.bias[col] : 0.f;
    // ROWB (bias_mode 2 / 3): the graph-conv bias pushed through A, per joint [V][Cout] / per (sample,
    // joint) [N][V][Cout] (tgcn.py:76 with the bias applied before the A-mix).  A template flag: the
    // per-row index math as a runtime branch cost the plain instantiations 2x (register pressure).
    float s = 0.f, cnt = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = (wm * TM + i) * 32 + acc_row(r, lane);
        float bb = b;
        if (ROWB) bb = a.bias[(long)sbi[row] * a.Cout + col];
        const float v = acc[i][j][r] + bb;
        acc[i][j][r] = v;
        *reinterpret_cast<bf16*>(smem + row * OS + cl * 2) = (bf16)v;
        if (row < rows_valid) {
          s += v;
          cnt += 1.f;
        }
      }
    if (a.stats) {
      Welford w;
      w.n = cnt;
      w.mean = cnt > 0.f ? s / cnt : 0.f;
      float m2 = 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = (wm * TM + i) * 32 + acc_row(r, lane);
          const float d = acc[i][j][r] - w.mean;
          if (row < rows_valid) m2 += d * d;
        }
      w.m2 = m2;
      Welford o;
      o.n = __shfl_xor(w.n, 32);
      o.mean = __shfl_xor(w.mean, 32);
      o.m2 = __shfl_xor(w.m2, 32);
      const Welford t = welford_merge(w, o);
      if (lh == 0) red[wm * BN + cl] = make_float4(t.n, t.mean, t.m2, 0.f);
    }
  }
  __syncthreads();
  if (a.stats && tid < BN) {
    const float4 p = red[tid], q = red[BN + tid];
    const Welford t = welford_merge(Welford{p.x, p.y, p.z}, Welford{q.x, q.y, q.z});
    reinterpret_cast<float4*>(a.stats)[(long)rt * a.Cout_pad + n0 + tid] = make_float4(t.n, t.mean, t.m2, 0.f);
  }
  bf16* __restrict__ out = reinterpret_cast<bf16*>(a.out);
  constexpr int OU = BN / 8;  // 16-B units per output row
#pragma unroll
  for (int u = 0; u < BM * OU / NT; ++u) {
    const int e = tid + u * NT, row = e / OU, cu = e % OU;
    if (row < rows_valid) {
      uint4 v = *reinterpret_cast<const uint4*>(smem + row * OS + cu * 16);
      uint4* p = reinterpret_cast<uint4*>(out + (m0 + row) * a.out_ld + n0 + cu * 8);
      if (a.accumulate) {
        float f[8], o[8];
        unpack16(v, f, (bf16*)nullptr);
        unpack16(*p, o, (bf16*)nullptr);
#pragma unroll
        for (int k = 0; k < 8; ++k) f[k] += o[k];
        v = pack16(f, (bf16*)nullptr);
      }
      *p = v;
    }
  }
}

// Narrow 1x1 convs (fcn_in 3 -> 64, stgcn.py:49, and its input grad 64 -> 3) are pure streaming: VALU
// dot products, weights ([Cout_pad][Cin_pad] packed image) staged once per block in LDS; blocks stride
// over the rows.
//   WIDE_OUT (Cin <= 16, Cout <= 64, Cout % 8 == 0): thread = (row, 8 output channels), the row's Cin
//     inputs as scalars (any ld), coalesced 16-B stores, weights k-major in LDS (conflict-free)
//   !WIDE_OUT (Cout <= 8, Cin % 8 == 0): thread = row, 16-B input loads, Cout scalar outputs (any ld),
//     weights read as broadcasts
template <bool WIDE_OUT>
__global__ __launch_bounds__(NT) void conv1x1_narrow_kernel(const stgcn_conv_desc a, long M) {
  __shared__ __attribute__((aligned(16))) float sw[4096];
  const int KP = a.Cin_pad;
  const bf16* __restrict__ w = reinterpret_cast<const bf16*>(a.w);
  for (int e = threadIdx.x; e < a.Cout_pad * KP; e += NT) sw[e] = (float)w[e];
  __syncthreads();
  const bf16* __restrict__ in = reinterpret_cast<const bf16*>(a.in);
  bf16* __restrict__ out = reinterpret_cast<bf16*>(a.out);
  const bool bias = a.bias && a.bias_mode == 1;
  if constexpr (WIDE_OUT) {
    // weights transposed in LDS (k-major): the 8 units of a row sit in 8 distinct banks
    const int CP = a.Cout_pad, CU = a.Cout / 8;
    __syncthreads();
    for (int e = threadIdx.x; e < CP * KP; e += NT) {
      const int co = e / KP, k = e - co * KP;
      sw[k * CP + co] = (float)w[e];
    }
    __syncthreads();
    // 32-bit index math (the launcher guarantees M * Cout / 8 < 2^31): a 64-bit division per unit
    // cost more than the unit's arithmetic
    const unsigned n = (unsigned)(M * CU);
    // rows of <= 8 input channels at a 16-B aligned stride (fcn_in: 3 channels padded to 8): one 16-B load
    // per row, and UNR units' loads issued before any of their math — the grid-stride loop was a chain
    // of dependent load -> math -> store iterations (latency-bound: 52 us for 61 MB of output)
    constexpr int UNR = 4;
    const bool vec_in = a.Cin <= 8 && (a.in_ld & 7) == 0 && (reinterpret_cast<size_t>(a.in) & 15) == 0;
    const unsigned gstride = gridDim.x * NT;
    for (unsigned i0 = blockIdx.x * NT + threadIdx.x; i0 < n; i0 += UNR * gstride) {
      uint4 xv[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const unsigned i = i0 + u * gstride;
        if (vec_in && i < n) xv[u] = *reinterpret_cast<const uint4*>(in + (long)(i / (unsigned)CU) * a.in_ld);
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
      const unsigned i = i0 + u * gstride;
      if (i >= n) break;
      const unsigned m = i / (unsigned)CU;
      const int c0 = (int)(i - m * (unsigned)CU) * 8;
      const bf16* xr = in + (long)m * a.in_ld;
      float xf[8];
      if (vec_in) unpack16(xv[u], xf, (bf16*)nullptr);
      float f[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) f[e] = bias ? a.bias[c0 + e] : 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (k < a.Cin) {
          const float xk = vec_in ? xf[k & 7] : (float)xr[k];
          const float4 w0 = *reinterpret_cast<const float4*>(&sw[k * CP + c0]);
          const float4 w1 = *reinterpret_cast<const float4*>(&sw[k * CP + c0 + 4]);
          f[0] = fmaf(w0.x, xk, f[0]); f[1] = fmaf(w0.y, xk, f[1]); f[2] = fmaf(w0.z, xk, f[2]); f[3] = fmaf(w0.w, xk, f[3]);
          f[4] = fmaf(w1.x, xk, f[4]); f[5] = fmaf(w1.y, xk, f[5]); f[6] = fmaf(w1.z, xk, f[6]); f[7] = fmaf(w1.w, xk, f[7]);
        }
      uint4* p = reinterpret_cast<uint4*>(out + (long)m * a.out_ld + c0);
      if (a.accumulate) {
        float o[8];
        unpack16(*p, o, (bf16*)nullptr);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] += o[e];
      }
      *p = pack16(f, (bf16*)nullptr);
      }
    }
    return;
  }
  for (long m = (long)blockIdx.x * NT + threadIdx.x; m < M; m += (long)gridDim.x * NT) {
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = (bias && e < a.Cout) ? a.bias[e] : 0.f;
    // the row's 16-B units (up to 64 channels) are all requested before the math (one round trip per row)
    uint4 xr[8];
#pragma unroll
    for (int c = 0; c < 8; ++c)
      if (c * 8 < a.Cin) xr[c] = *reinterpret_cast<const uint4*>(in + m * a.in_ld + c * 8);
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      if (c * 8 >= a.Cin) break;
      const int k0 = c * 8;
      float x[8];
      unpack16(xr[c], x, (bf16*)nullptr);
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (e < a.Cout) {
#pragma unroll
          for (int k = 0; k < 8; ++k) acc[e] = fmaf(sw[e * KP + k0 + k], x[k], acc[e]);
        }
    }
    for (int k0 = 64; k0 < a.Cin; k0 += 8) {
      float x[8];
      unpack16(*reinterpret_cast<const uint4*>(in + m * a.in_ld + k0), x, (bf16*)nullptr);
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (e < a.Cout) {
#pragma unroll
          for (int k = 0; k < 8; ++k) acc[e] = fmaf(sw[e * KP + k0 + k], x[k], acc[e]);
        }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e)
      if (e < a.Cout) {
        bf16* p = out + m * a.out_ld + e;
        *p = (bf16)(a.accumulate ? acc[e] + (float)*p : acc[e]);
      }
  }
}

template <int KS, int BN, bool ROWB = false>
int launch1(const stgcn_conv_desc& a, const XGeom& g, hipStream_t s) {
  constexpr int RS = KS * 16 * 2 + 16, OS = BN * 2 + 16;
  size_t lds = (size_t)BM * RS;
  const size_t lout = (size_t)BM * OS + 2 * BN * 16 + (ROWB ? BM * sizeof(int) : 0);
  if (lout > lds) lds = lout;
  constexpr bool RB = ROWB;
  if (stgcn_lds_attr((const void*)conv1x1_kernel<KS, BN, RB>, 160 * 1024, s)) return STGCN_EHIP;
  const long rounds = ((long)g.nrow + 7) / 8;  // row tiles in whole rounds of the 8 XCDs (kernel mapping)
  hipLaunchKernelGGL((conv1x1_kernel<KS, BN, RB>), dim3((unsigned)(rounds * 8 * g.ncol)), dim3(NT), lds, s, a, g);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

}  // namespace

long conv_rows_num_row_blocks(long M, int cout);

// returns -1 when the shape is not handled here
int conv1x1_launch(const stgcn_conv_desc& a, int dtype, hipStream_t s) {
  if (dtype != 1 || a.Kt != 1 || a.pad != 0 || a.pro != 0) return -1;
  if (a.stride == 1 && a.T_in == a.T_out && !a.stats && a.bias_mode >= 0 && a.bias_mode <= 1 &&
      (long)a.Cout_pad * a.Cin_pad <= 4096) {
    const long M = (long)a.N * a.T_out * a.V;
    long nb = (M + NT - 1) / NT;
    if (nb > 1024) nb = 1024;
    if (a.Cin <= 16 && a.Cout <= 64 && a.Cout % 8 == 0 && a.out_ld % 8 == 0 && M * (a.Cout / 8) < 0x7fffffffL) {
      hipLaunchKernelGGL(conv1x1_narrow_kernel<true>, dim3((unsigned)nb), dim3(NT), 0, s, a, M);
      return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
    }
    if (a.Cout <= 8 && a.Cin % 8 == 0 && a.in_ld % 8 == 0) {
      hipLaunchKernelGGL(conv1x1_narrow_kernel<false>, dim3((unsigned)nb), dim3(NT), 0, s, a, M);
      return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
    }
  }
  if (!a.w_frag) return -1;
  if (a.stride < 1 || a.bias_mode < 0 || a.bias_mode > 3) return -1;
  if (a.bias_mode >= 2 && (a.stride != 1 || a.trans)) return -1;
  if (a.trans ? a.T_in != (a.T_out - 1) / a.stride + 1 : a.T_out != (a.T_in - 1) / a.stride + 1) return -1;
  if (a.in_ld % 8 || a.out_ld % 8 || a.Cout % 64 || a.Cin_pad != a.Cin || a.Cout_pad < a.Cout) return -1;
  // K = Cin: also the A-first graph conv's P * Cin = 192 at C = 64 (83 vs 125 us against conv_tile); at
  // K = 384 the staged tile (100 KB of LDS, one block per CU) measured 2x slower than conv_tile
  if (a.Cin != 64 && a.Cin != 128 && a.Cin != 192 && a.Cin != 256) return -1;
  XGeom g;
  g.M = (long)a.N * a.T_out * a.V;
  // the per-row bias (bias_mode 2 / 3) only at 64-column tiles: at 128 its index math spills
  const bool rowb = a.bias && a.bias_mode >= 2;
  const int BN = a.Cout % 128 == 0 && !rowb ? 128 : 64;
  g.ncol = a.Cout / BN;
  const long nrow = (g.M + BM - 1) / BM;
  if ((nrow + 7) / 8 * 8 * g.ncol > 0x7fffffffL) return -1;
  g.nrow = (int)nrow;
  g.k16n = a.Cin_pad / 16;
  if (a.stats && nrow > conv_rows_num_row_blocks(g.M, a.Cout)) return -1;
  if (BN == 128) {
    if (a.Cin == 64) return launch1<4, 128>(a, g, s);
    if (a.Cin == 128) return launch1<8, 128>(a, g, s);
    if (a.Cin == 192) return launch1<12, 128>(a, g, s);
    return launch1<16, 128>(a, g, s);
  }
  if (rowb) {
    if (a.Cin == 64) return launch1<4, 64, true>(a, g, s);
    if (a.Cin == 128) return launch1<8, 64, true>(a, g, s);
    if (a.Cin == 192) return launch1<12, 64, true>(a, g, s);
    return launch1<16, 64, true>(a, g, s);
  }
  if (a.Cin == 64) return launch1<4, 64>(a, g, s);
  if (a.Cin == 128) return launch1<8, 64>(a, g, s);
  if (a.Cin == 192) return launch1<12, 64>(a, g, s);
  return launch1<16, 64>(a, g, s);
}
