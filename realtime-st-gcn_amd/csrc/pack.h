// Per-thread bodies of the weight-preparation kernels (packed GEMM operands, MFMA-fragment images, the
// graph conv's per-joint effective weights), shared by their single-job launches (conv_rows.hip,
// conv_wide.hip, gconv.hip) and the batched launch that prepares every layer of a model at once (prep.hip).
#pragma once
#include "common.h"

// 8 consecutive elements of T as 16 (bf16) or 32 (fp32) bytes
template <typename T>
DEV void store8(T* p, const float* v) {
  if constexpr (sizeof(T) == 2) {
    *reinterpret_cast<uint4*>(p) = pack16(v, (T*)nullptr);
  } else {
    *reinterpret_cast<uint4*>(p) = pack16(v, (T*)nullptr);
    *reinterpret_cast<uint4*>(p + 4) = pack16(v + 4, (T*)nullptr);
  }
}

// dst[k][co][ci] = src[k*s0 + co*s1 + ci*s2] (0 in the padding), cast to T: any strided view of the
// fp32 parameter (permuted / transposed) packs in one pass.  Thread i of Kt * cp * kp / 8 handles 8
// consecutive ci (kp % 8 == 0): one 16/32-byte store into dst and one into the fragment image.
template <typename T>
DEV void pack_weight_elem(const float* __restrict__ src, long s0, long s1, long s2, int Co, int Ci, int cp, int kp,
                          long i, T* __restrict__ dst, T* __restrict__ dst_frag) {
  const int k8 = kp >> 3;
  const int ci0 = (int)(i % k8) * 8;
  const long r = i / k8;
  const int co = (int)(r % cp);
  const long k = r / cp;
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e)
    v[e] = (co < Co && ci0 + e < Ci) ? src[k * s0 + co * s1 + (long)(ci0 + e) * s2] : 0.f;
  store8(dst + ((k * cp + co) * (long)kp + ci0), v);
  if (dst_frag) {
    // MFMA-fragment image (conv_wide.hip): 1-KiB blocks [k][co/32][ci/16], lane l = (ci%16)/8*32 + co%32
    // holding 8 consecutive ci: a wave's B fragment is one contiguous 1-KiB load
    const long blk = ((long)k * (cp / 32) + co / 32) * (kp / 16) + ci0 / 16;
    const int l = ((ci0 & 15) >> 3) * 32 + (co & 31);
    store8(dst_frag + blk * 512 + l * 8, v);
  }
}

// Parity-folded fragment image of a stride-2 Kt = 9 weight [9][Co][Ci] (fp32, any strides): the 5-tap
// conv the wide kernel runs instead (see conv_wide_launch) —
//   forward   W'[t][co][par*Ci + ci] = W[2t + par][co][ci]
//   data grad W'[t][par*Co + co][ci] = W[8 - 2t + par][co][ci]      (taps outside 0..8 are zero)
// laid out like stgcn_pack_weight_frag (1-KiB blocks [t][co'/32][ci'/16]).  Thread idx of 5 * co_f * ci_f / 8
// handles 8 consecutive ci' (Ci % 8 == 0, so they share the parity).
DEV void pack_s2frag_elem(const float* __restrict__ src, long s0, long s1, long s2, int Co, int Ci, int trans,
                          int co_f, int ci_f, long idx, bf16* __restrict__ dst) {
  const int c8 = ci_f >> 3;
  const int cip = (int)(idx % c8) * 8;
  const int cop = (int)((idx / c8) % co_f);
  const int t = (int)(idx / ((long)co_f * c8));
  int co = cop, ci = cip, dt;
  if (trans) {
    const int par = cop >= Co;
    co = cop - par * Co;
    dt = 8 - 2 * t + par;
  } else {
    const int par = cip >= Ci;
    ci = cip - par * Ci;
    dt = 2 * t + par;
  }
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = (dt >= 0 && dt <= 8) ? src[dt * s0 + co * s1 + (long)(ci + e) * s2] : 0.f;
  const long blk = ((long)t * (co_f / 32) + cop / 32) * (ci_f / 16) + cip / 16;
  const int l = ((cip & 15) >> 3) * 32 + (cop & 31);
  store8(dst + blk * 512 + l * 8, v);
}

// Graph conv effective weights (gconv.hip):
// out[a][j][r][c] (dtype, padded to [R_pad][C_pad]):
//   trans 0: sum_p A[p][nbr[a][j]][a] * W[p*Cout + r][c]          (r = co < Cout, c = ci < Cin)
//   trans 1: sum_p A[p][a][nbr[a][j]] * W[p*Cout + c][r]          (r = ci < Cin,  c = co < Cout)
// One thread per (joint a, 8 consecutive c, r): it loads its P x 8 weights once and writes all deg[a]
// neighbour slots of joint a (a thread per slot re-read the same weights J times: ~100 MB of L2 reads per
// C = 256 launch).  Slots j >= deg[a] are never read by gconv and are skipped; padding rows / columns are
// written as zeros (they meet zero-filled operands).
constexpr int GW_PMAX = 4;
constexpr int GW_JMAX = 1;  // neighbour slots per joint whose loads are issued together (8 and 4 held 138 / 98
                            // VGPRs: 3 / 4 waves per SIMD for the batched prep launch, 93 / 61 us vs 51 us at 1)
// M (optional, the layer's edge importance [P][V][V]): coefficients are A * M, the same fp32 product the
// model forms for the layer (stgcn.py:89), so a model can prepare every layer before that product exists.
// Column sums of A * M for the bias through A, colsum[p * V + a] = sum_v (A * M)[p][v][a] (summed in v order),
// computed once per block into LDS by every thread of the block (call before any thread returns; the loads
// of a column are issued together) — per-thread sums were a chain of 75 dependent loads per output.
DEV void gconv_colsum_block(const float* __restrict__ A, const float* __restrict__ M, int P, int V, float* colsum) {
  for (int t = threadIdx.x; t < P * V; t += blockDim.x) {
    const int p = t / V, a = t - p * V;
    float cs = 0.f;
    if (V <= 32) {
      float c[32];
#pragma unroll
      for (int v = 0; v < 32; ++v) {
        const long ia = ((long)p * V + v) * V + a;
        c[v] = v < V ? (M ? __fmul_rn(A[ia], M[ia]) : A[ia]) : 0.f;  // rounded product, never fused into the sum
      }
#pragma unroll
      for (int v = 0; v < 32; ++v)
        if (v < V) cs += c[v];
    } else {
      for (int v = 0; v < V; ++v) {
        const long ia = ((long)p * V + v) * V + a;
        cs += M ? __fmul_rn(A[ia], M[ia]) : A[ia];
      }
    }
    colsum[t] = cs;
  }
  __syncthreads();
}
constexpr int GW_COLSUM_MAX = GW_PMAX * 64;  // LDS floats for the column sums (P <= 4, V <= 64)

// Thread idx of V * R_pad * (C_pad / 8); colsum: gconv_colsum_block's LDS table when bias2d != NULL.
template <typename T>
DEV void gconv_weights_elem(const float* __restrict__ A, const float* __restrict__ M, const float* __restrict__ W,
                            const int* nbr, const int* deg, int P, int V, int J, int Cout, int Cin, int trans, T* out,
                            int R_pad, int C_pad, const float* __restrict__ bconv, float* __restrict__ bias2d,
                            const float* colsum, long idx) {
  const int C8 = C_pad / 8;
  // forward: c (ci) fastest across lanes, so W rows are read as float4 runs; trans: r (ci) fastest, so
  // the 8 scalar reads of W[co][r] per thread are coalesced across lanes (c fastest for trans too, for
  // contiguous stores, measured 1.6x slower: its W reads are 8 rows per lane)
  int c0, r, a;
  if (!trans) {
    c0 = (int)(idx % C8) * 8;
    const long t1 = idx / C8;
    r = (int)(t1 % R_pad);
    a = (int)(t1 / R_pad);
  } else {
    r = (int)(idx % R_pad);
    const long t1 = idx / R_pad;
    c0 = (int)(t1 % C8) * 8;
    a = (int)(t1 / C8);
  }
  const int R = trans ? Cin : Cout, C = trans ? Cout : Cin;
  if (bias2d && !trans && c0 == 0 && r < Cout) {
    // the graph conv's bias pushed through A in the same launch (stgcn_gcn_bias, same summation order):
    // bias2d[a][co] = sum_p b[p*Cout + co] * colsum_p[a], colsum_p[a] = sum_v A[p][v][a] (gconv_colsum_block)
    float sb = 0.f;
    for (int p = 0; p < P; ++p) sb += bconv[p * Cout + r] * colsum[p * V + a];
    bias2d[(long)a * Cout + r] = sb;
  }
  float wv[GW_PMAX][8];
#pragma unroll
  for (int p = 0; p < GW_PMAX; ++p)
#pragma unroll
    for (int e = 0; e < 8; ++e) wv[p][e] = 0.f;
  if (r < R) {
#pragma unroll
    for (int p = 0; p < GW_PMAX; ++p) {
      if (p >= P) break;
      if (!trans) {
        const float* w = W + ((long)p * Cout + r) * Cin + c0;
        if (c0 + 8 <= C && (Cin & 3) == 0) {
          const float4 w0 = *reinterpret_cast<const float4*>(w), w1 = *reinterpret_cast<const float4*>(w + 4);
          wv[p][0] = w0.x; wv[p][1] = w0.y; wv[p][2] = w0.z; wv[p][3] = w0.w;
          wv[p][4] = w1.x; wv[p][5] = w1.y; wv[p][6] = w1.z; wv[p][7] = w1.w;
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (c0 + e < C) wv[p][e] = w[e];
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (c0 + e < C) wv[p][e] = W[((long)p * Cout + c0 + e) * Cin + r];
      }
    }
  }
  // the neighbour list and coefficients of up to GW_JMAX slots are requested together (independent loads),
  // not as a chain of dependent loads per slot: the small launches are latency-bound
  const int dtot = deg[a];
  for (int j0 = 0; j0 < dtot; j0 += GW_JMAX) {
    const int da = min(dtot - j0, GW_JMAX);
    int nb[GW_JMAX];
#pragma unroll
    for (int jj = 0; jj < GW_JMAX; ++jj) nb[jj] = jj < da ? nbr[a * J + j0 + jj] : a;
    float cf[GW_JMAX][GW_PMAX];
#pragma unroll
    for (int jj = 0; jj < GW_JMAX; ++jj)
#pragma unroll
      for (int p = 0; p < GW_PMAX; ++p)
        if (jj < da && p < P) {
          const long ia = trans ? ((long)p * V + a) * V + nb[jj] : ((long)p * V + nb[jj]) * V + a;
          cf[jj][p] = M ? __fmul_rn(A[ia], M[ia]) : A[ia];
        } else {
          cf[jj][p] = 0.f;
        }
#pragma unroll
    for (int jj = 0; jj < GW_JMAX; ++jj) {
      if (jj >= da) break;
      const int j = j0 + jj;
      float s[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) s[e] = 0.f;
#pragma unroll
      for (int p = 0; p < GW_PMAX; ++p) {
        if (p >= P) break;
#pragma unroll
        for (int e = 0; e < 8; ++e) s[e] += cf[jj][p] * wv[p][e];
      }
      T* o = out + (((long)a * J + j) * R_pad + r) * (long)C_pad + c0;
      if constexpr (sizeof(T) == 2) {
        *reinterpret_cast<uint4*>(o) = pack16(s, (T*)nullptr);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = s[e];
      }
    }
  }
}

