// The 64-channel graph convolution of ST-GCN (ConvTemporalGraphical, models/utils/tgcn.py:58-79) in its A-first
// form, for a graph shared by the batch, fused into one persistent kernel: forward and data gradient.
//
//   forward   g[f,w,co]  = bias2d[w][co] + sum_{p,ci} W[p*64+co][ci] * XA[f,w,p,ci],
//             XA[f,w,p,ci] = sum_{j < deg[w]} A[p][S(w)_j][w] * x[f, S(w)_j, ci]          (S = support lists)
//   data grad dx[f,v,ci] = sum_{p,co} W[p*64+co][ci] * XA[f,v,p,co],
//             XA[f,v,p,co] = sum_{j < rdeg[v]} A[p][v][R(v)_j] * dg[f, R(v)_j, co]        (R = reverse lists)
//
// i.e. the joint mix first (as the reference's einsum, moved in front of the 1x1 conv: both are linear), then ONE
// GEMM whose weights (P*64 x 64, 24 KB bf16) are shared by every joint and frame — so each wave keeps its B
// fragments in registers for the whole launch, and x is read from HBM exactly once.  The joint-gathered GEMM
// (gconv.hip) instead streams per-joint effective weights (deg x 8 KB per joint and row tile) and runs short
// latency-bound K loops of deg 64-channel chunks per (row tile, joint) block.
//
// Block (persistent, 256 threads = 4 waves, two per CU so one block's DMA / store waits overlap the other's
// arithmetic): tiles of FT = 4 frames (4V rows, contiguous in HBM):
//   (0) the next tile's x rows go global -> LDS by DMA (double buffer) while this tile is processed;
//   (1) the mix (VALU, fp32) writes XA as bf16 rows [4V (+pad to 32)][P*64] into LDS (400-B padded rows);
//   (2) the GEMM: wave = (32-column tile ct, row tiles {rt, rt + 2}), A fragments from LDS, B in registers,
//       v_mfma_f32_32x32x16_bf16, K = P*64 (12 k-steps at P = 3);
//   (3) epilogue: + bias2d (forward), BN partial statistics (forward: per column shifted sums over every row the
//       block produced, one (count, mean, M2) row per block at the end), the tile staged through LDS as bf16 rows
//       and stored 16 B per lane, whole 128-B rows (data grad: + the masked identity residual, or accumulate).
// Rounding: XA is rounded to bf16 once (the reference under autocast rounds the conv output instead); fp32 GEMM
// accumulation.  bf16 only; Cin = Cout = 64, P <= 3, V <= 25, J <= 8.
#include "common.h"
#include "../../include/stgcn_amd.h"

namespace {

constexpr int AF_NT = 256;
constexpr int AF_FT = 4;      // frames per tile
constexpr int AF_C = 64;      // channels in and out
constexpr int AF_PMAX = 3;
constexpr int AF_VMAX = 25;
constexpr int AF_JMAX = 8;
constexpr int AF_ARS = 400;   // XA / staged-W row stride in LDS (384 B + 16)
constexpr int AF_SRS = 68;    // fp32 output staging row stride (floats)

DEV int af_rows(int V) { return AF_FT * V; }
DEV int af_rtiles(int V) { return (af_rows(V) + 31) / 32; }

// LDS carve (bytes): xb[2][4V][128] (dense rows: the DMA writes lane-linearly) | xa[4V][400] (also: W staged as
// bf16 [64][400 B] at setup, the fp32 output tile [4V][68] in the epilogue, the statistics merge at the end) |
// bias[V][64] f32 | coef[V][8] float4 (p0, p1, p2, 0) | lst[V][8] i32
constexpr int AF_XB = AF_FT * AF_VMAX * 128;
constexpr int AF_XA = AF_FT * AF_VMAX * AF_ARS;  // the last row tile's rows past 4V read row 4V-1 (discarded)
constexpr int af_lds_bytes_max() {
  return 2 * AF_XB + AF_XA + AF_VMAX * AF_C * 4 + AF_VMAX * AF_JMAX * 16 + AF_VMAX * AF_JMAX * 4;
}
static_assert(AF_C * AF_ARS <= AF_XA && AF_FT * AF_VMAX * AF_SRS * 4 <= AF_XA && AF_NT * 17 * 4 <= AF_XA, "xa reuse");

DEV unsigned lds_u32(const void* p) { return (unsigned)(size_t)(const __attribute__((address_space(3))) char*)p; }
// 16 B per lane, global -> LDS at M0 = lds_off (lane-linear), m0 saved and restored (gconv.hip's glds16m)
DEV void af_dma16(const void* src, unsigned lds_off) {
  unsigned saved;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(saved) : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds_off)) : "memory");
}

__global__ __launch_bounds__(AF_NT, 2) void gcn_af_kernel(const stgcn_gcn_af_desc a) {
  extern __shared__ __attribute__((aligned(16))) char sm[];
  const int V = a.V, P = a.P, J = a.J, K = P * AF_C, KS = K / 16;
  const int rows = af_rows(V), rtn = af_rtiles(V);
  char* xb = sm;                                                          // [2][rows][128]
  char* xa = xb + 2 * AF_XB;                                               // [rows][AF_ARS]
  float* bs = reinterpret_cast<float*>(xa + AF_XA);                        // [V][64]
  float4* coef = reinterpret_cast<float4*>(bs + AF_VMAX * AF_C);           // [V][8]
  int* lst = reinterpret_cast<int*>(coef + AF_VMAX * AF_JMAX);             // [V][8]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bf16* __restrict__ x = reinterpret_cast<const bf16*>(a.x);
  bf16* __restrict__ out = reinterpret_cast<bf16*>(a.out);
  const long nfr = a.NT;  // frames
  const int ntile = (int)((nfr + AF_FT - 1) / AF_FT);

  // DMA of one tile's x rows into xb[buf]: 8 16-B units per row; the waves split the 1-KB wave-instructions
  // (8 rows x 128 B: lane -> row lane >> 3, unit lane & 7); rows past the valid ones re-read the last valid row
  auto issue = [&](int t, int buf) {
    const long f0 = (long)t * AF_FT;
    const int rv = (int)min((long)rows, (nfr - f0) * V);
    const unsigned base = lds_u32(xb + buf * AF_XB);
    for (int r0 = wave * 8; r0 < rows; r0 += 8 * (AF_NT / 64)) {
      const int r = min(r0 + (lane >> 3), rv - 1);
      af_dma16(x + (f0 * V + r) * (long)a.x_ld + (lane & 7) * 8, base + (unsigned)(r0 * 128));
    }
  };
  if ((int)blockIdx.x < ntile) issue(blockIdx.x, 0);  // the first tile's rows travel while the tables are built

  // W -> LDS as bf16 in B-operand order, row n = output column of the GEMM, k = p*64 + m contiguous:
  //   forward   wl[n][p*64+m] = W[p*64+n][m];   data grad   wl[n][p*64+m] = W[p*64+m][n]
  // (coalesced float4 reads of W's [P*64][64] rows: element (R = p*64 + rr, cc))
  {
    const float4* w4 = reinterpret_cast<const float4*>(a.w);
    const int n4 = P * AF_C * AF_C / 4;
    for (int i0 = 0; i0 < AF_PMAX * AF_C * AF_C / 4; i0 += 4 * AF_NT) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + u * AF_NT + tid;
        v[u] = i < n4 ? w4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 + u * AF_NT + tid;
        if (i < n4) {
          const int R = (4 * i) / AF_C, cc0 = (4 * i) % AF_C, p = R / AF_C, rr = R % AF_C;
          const float f[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int n = a.trans ? cc0 + e : rr, m = a.trans ? rr : cc0 + e;
            *reinterpret_cast<bf16*>(xa + n * AF_ARS + (p * AF_C + m) * 2) = (bf16)f[e];
          }
        }
      }
    }
  }
  // bias rows (forward) and the mix tables: lst[o][j], coef[o][j] = (c_0, c_1, c_2, 0) with c_p = A[p][lst][o]
  // (forward) | A[p][o][lst] (data grad), times M if given; slots j >= deg: row 0 with coefficients 0
  if (a.bias)
    for (int i = tid; i < V * AF_C / 4; i += AF_NT)
      reinterpret_cast<float4*>(bs)[i] = reinterpret_cast<const float4*>(a.bias)[i];
  for (int i = tid; i < V * AF_JMAX; i += AF_NT) {
    const int o = i / AF_JMAX, j = i % AF_JMAX;
    const int d = min(a.deg[o], J);
    const int s = j < d ? a.nbr[o * J + j] : 0;
    float c[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int p = 0; p < AF_PMAX; ++p)
      if (j < d && p < P) {
        const long ia = a.trans ? ((long)p * V + o) * V + s : ((long)p * V + s) * V + o;
        c[p] = a.M ? __fmul_rn(a.A[ia], a.M[ia]) : a.A[ia];
      }
    lst[i] = s;
    coef[i] = make_float4(c[0], c[1], c[2], 0.f);
  }
  __syncthreads();

  // B fragments of this wave's column tile for every k-step (registers for the whole launch):
  // lane l: n = ct*32 + (l & 31), k = ks*16 + 8*(l >> 5) + e
  const int ct = wave & 1, rt0 = wave >> 1;  // row tiles rt0, rt0 + 2
  bf16x8 bfr[AF_PMAX * AF_C / 16];
  {
    const char* wrow = xa + (ct * 32 + (lane & 31)) * AF_ARS + 16 * (lane >> 5);
#pragma unroll
    for (int ks = 0; ks < AF_PMAX * AF_C / 16; ++ks) {
      const uint4 z = ks < KS ? *reinterpret_cast<const uint4*>(wrow + ks * 32) : make_uint4(0, 0, 0, 0);
      bfr[ks] = __builtin_bit_cast(bf16x8, z);
    }
  }
  // running BN statistics of this thread's 8 store-loop columns q*8 .. q*8+7 (q = tid & 7 for every unit it
  // stores: AF_NT % 8 == 0): shifted sums, shift = the first value of each column
  const int q = tid & 7;
  float st_n = 0.f, st_k[8], st_s1[8], st_s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) st_k[e] = st_s1[e] = st_s2[e] = 0.f;

  int buf = 0;
  for (int t = blockIdx.x; t < ntile; t += gridDim.x) {
    const long f0 = (long)t * AF_FT;
    const int rv = (int)min((long)rows, (nfr - f0) * V);  // valid rows of this tile
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      // this tile's DMA (and the last tile's stores)
    __syncthreads();                                       // every wave's DMA landed; the previous tile is done
    if (t + (int)gridDim.x < ntile) issue(t + gridDim.x, buf ^ 1);
    const char* xt = xb + buf * AF_XB;

    // (1) mix: unit = (row r, 8-channel chunk q): all 8 neighbour slots' 16-B pieces read at once, all P
    // partitions accumulated (unused slots: row 0 of the frame, coefficients 0)
    for (int u = tid; u < rv * 8; u += AF_NT) {
      const int r = u >> 3;
      const int f = r / V, o = r - f * V;
      const int4 l0 = reinterpret_cast<const int4*>(lst)[o * 2], l1 = reinterpret_cast<const int4*>(lst)[o * 2 + 1];
      const int ls[8] = {l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, l1.z, l1.w};
      const char* xf = xt + f * V * 128 + q * 16;
      uint4 xr[AF_JMAX];
#pragma unroll
      for (int j = 0; j < AF_JMAX; ++j) xr[j] = *reinterpret_cast<const uint4*>(xf + ls[j] * 128);
      float acc[AF_PMAX][8];
#pragma unroll
      for (int p = 0; p < AF_PMAX; ++p)
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[p][e] = 0.f;
#pragma unroll
      for (int j = 0; j < AF_JMAX; ++j) {
        const float4 c = coef[o * AF_JMAX + j];
        float xv[8];
        unpack16(xr[j], xv, (bf16*)nullptr);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          acc[0][e] = fmaf(c.x, xv[e], acc[0][e]);
          acc[1][e] = fmaf(c.y, xv[e], acc[1][e]);
          acc[2][e] = fmaf(c.z, xv[e], acc[2][e]);
        }
      }
#pragma unroll
      for (int p = 0; p < AF_PMAX; ++p)
        if (p < P) *reinterpret_cast<uint4*>(xa + r * AF_ARS + (p * AF_C + q * 8) * 2) = pack16(acc[p], (bf16*)nullptr);
    }
    __syncthreads();

    // (2) GEMM: this wave's row tiles rt0, rt0 + 2 (rows past the tile's valid ones read stale XA: discarded)
    f32x16 acc[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int rt = rt0 + 2 * i;
      if (rt < rtn) {
        const char* arow = xa + min(rt * 32 + (lane & 31), rows - 1) * AF_ARS + 16 * (lane >> 5);
#pragma unroll
        for (int ks = 0; ks < AF_PMAX * AF_C / 16; ++ks) {
          if (ks < KS) {
            const bf16x8 fa = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(arow + ks * 32));
            acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, bfr[ks], acc[i], 0, 0, 0);
          }
        }
      }
    }
    __syncthreads();  // every read of xa done: it becomes the fp32 output staging area

    float* stg = reinterpret_cast<float*>(xa);  // [rows][AF_SRS]
    const int col = ct * 32 + (lane & 31);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int rt = rt0 + 2 * i;
      if (rt >= rtn) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rt * 32 + acc_row(r, lane);
        if (row < rv) stg[row * AF_SRS + col] = acc[i][r];
      }
    }
    __syncthreads();

    // (3) epilogue per unit (row r, columns q*8 ..): + bias, statistics, + masked residual / accumulate, bf16,
    // one 16-B store (8 lanes = one whole 128-B row)
    for (int u = tid; u < rv * 8; u += AF_NT) {
      const int r = u >> 3;
      const long grow = f0 * V + r;
      const float4 g0 = *reinterpret_cast<const float4*>(stg + r * AF_SRS + q * 8);
      const float4 g1 = *reinterpret_cast<const float4*>(stg + r * AF_SRS + q * 8 + 4);
      float f[8] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
      if (a.bias) {
        const float* b = bs + (r % V) * AF_C + q * 8;
        const float4 b0 = *reinterpret_cast<const float4*>(b), b1 = *reinterpret_cast<const float4*>(b + 4);
        f[0] += b0.x; f[1] += b0.y; f[2] += b0.z; f[3] += b0.w;
        f[4] += b1.x; f[5] += b1.y; f[6] += b1.z; f[7] += b1.w;
      }
      if (a.stats) {
        if (st_n == 0.f) {
#pragma unroll
          for (int e = 0; e < 8; ++e) st_k[e] = f[e];
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float dv = f[e] - st_k[e];
          st_s1[e] += dv;
          st_s2[e] = fmaf(dv, dv, st_s2[e]);
        }
        st_n += 1.f;
      }
      bf16* dst = out + grow * (long)a.out_ld + q * 8;
      if (a.res) {
        float g[8];
        unpack16(*reinterpret_cast<const uint4*>(reinterpret_cast<const bf16*>(a.res) + grow * (long)a.res_ld + q * 8),
                 g, (bf16*)nullptr);
        const unsigned mb = reinterpret_cast<const unsigned char*>(a.res_bits)[grow * (AF_C / 8) + q];
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] += ((mb >> e) & 1u) ? g[e] : 0.f;  // fp32 sum, rounded once
      } else if (a.accumulate) {
        float g[8];
        unpack16(*reinterpret_cast<const uint4*>(dst), g, (bf16*)nullptr);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] += g[e];
      }
      *reinterpret_cast<uint4*>(dst) = pack16(f, (bf16*)nullptr);
    }
    buf ^= 1;
  }

  // the block's BN partial statistics: per thread (count, mean, M2) of its 8 columns; the 32 threads of one
  // column group q are merged in LDS (Chan, fixed order), one float4 (count, mean, M2, 0) per column
  if (a.stats) {
    __syncthreads();  // the last tile's staging reads are done: xa holds the merge
    float* red = reinterpret_cast<float*>(xa);  // [AF_NT][17]: count, then (mean, M2) x 8
    red[tid * 17] = st_n;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float mean = st_n > 0.f ? st_k[e] + st_s1[e] / st_n : 0.f;
      red[tid * 17 + 1 + 2 * e] = mean;
      red[tid * 17 + 2 + 2 * e] = st_n > 0.f ? fmaxf(st_s2[e] - st_s1[e] * st_s1[e] / st_n, 0.f) : 0.f;
    }
    __syncthreads();
    if (tid < AF_C) {
      const int c = tid, cq = c >> 3, e = c & 7;
      Welford w = {0.f, 0.f, 0.f};
      for (int k = 0; k < AF_NT / 8; ++k) {
        const float* h = red + (cq + 8 * k) * 17;
        w = welford_merge(w, Welford{h[0], h[1 + 2 * e], h[2 + 2 * e]});
      }
      reinterpret_cast<float4*>(a.stats)[(long)blockIdx.x * a.stats_ld + c] = make_float4(w.n, w.mean, w.m2, 0.f);
    }
  }
}

}  // namespace

long gcn_af_blocks(long NT, int V) {
  const long ntile = (NT + AF_FT - 1) / AF_FT;
  return ntile < 512 ? ntile : 512;  // two per CU
}

int gcn_af_launch(const stgcn_gcn_af_desc& a, hipStream_t s) {
  if (!a.x || !a.out || !a.A || !a.w || !a.nbr || !a.deg || a.NT <= 0) return STGCN_EBADSHAPE;
  if (a.V < 1 || a.V > AF_VMAX || a.P < 1 || a.P > AF_PMAX || a.J < 1 || a.J > AF_JMAX || a.trans < 0 || a.trans > 1)
    return STGCN_EBADSHAPE;
  if (a.x_ld % 8 || a.out_ld % 8 || a.x_ld < AF_C || a.out_ld < AF_C) return STGCN_EBADSHAPE;
  if ((a.res && (!a.res_bits || a.res_ld % 8 || a.accumulate)) || (a.stats && a.stats_ld < AF_C)) return STGCN_EBADSHAPE;
  const long nb = gcn_af_blocks(a.NT, a.V);
  constexpr int lds = af_lds_bytes_max();
  static_assert(2 * lds <= 160 * 1024, "two blocks per CU");
  if (stgcn_lds_attr((const void*)gcn_af_kernel, lds, s)) return STGCN_EHIP;
  hipLaunchKernelGGL(gcn_af_kernel, dim3((unsigned)nb), dim3(AF_NT), lds, s, a);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
