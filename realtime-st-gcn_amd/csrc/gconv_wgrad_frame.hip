// Weight, adjacency and bias gradients of the graph convolution (ConvTemporalGraphical, tgcn.py:58-79,
// autograd of its conv1x1 + einsum with A) in ONE pass over (x, dg) per layer, frame by frame on MFMA.
//
// Forward (shared A [P][V][V]):  g[(i,w)][co] = sum_p sum_v A_p[v][w] (sum_ci W_p[co][ci] x[(i,v)][ci] + b_p[co])
// Gradients, per frame i (V <= 32 joint rows, zero-padded to 32):
//   D_p   = A_p dg_i                      [v][co]   joint mix of dg (K = w)
//   dW_p += D_p^T x_i                     [co][ci]  (K = v)
//   Z_p^T = W_p^T dg_i^T                  [ci][w]   (K = co)
//   dA_p += x_i Z_p^T                     [v][w]    (K = ci)          = sum_i (x W_p^T)[v] . dg[w]
//   S    += dg_i                          [w][co]   (identity MFMA, K = w) -> the bias through A:
//   dA_p[v][w] += sum_co b_p[co] S[w][co],   db_p[co] = sum_w colsum_p(A)[w] S[w][co]
// The accumulators D_p and Z_p^T are used directly as the next product's MFMA operand (an accumulator
// C[m][n] is an operand with K = m: lane n&31 holds rows (r&3) + 8(r>>2) + 4h, so the other operand is
// read with that K order), so nothing intermediate leaves the registers.  This replaces the per-joint
// dWeff blocks (73 of Cout x Cin at V = 25, x re-read once per neighbour) and their four-launch finish:
// x and dg are read once per (64-co, 64-ci) tile, and dA comes out dense (the reference's dA, also off the
// graph's support).
//
// Block = (64-co x 64-ci tile, run of frames); 4 waves = (32-co quarter cq, 32-ci half ch) of the tile, all
// on the same frame: per frame 4 panels [32 joint rows][32 channels] bf16 (dg: co quarters 0/1, x: ci
// halves 0/1) DMA'd global -> LDS (one panel per wave, 16-B units XOR-swizzled by row so that row reads
// and transposing reads are conflict-free) into a ring of D frame slots; one LDS-only barrier per frame.
// Per-block fp32 partials (dW tile, dA, db) go to a workspace and a second launch sums them in a fixed
// order (deterministic, no atomics).
#include "common.h"
#include "../../include/stgcn_amd.h"
#include <utility>

namespace {

constexpr int NW = 4;                 // waves per block
constexpr int PAN = 32 * 64;          // one panel: 32 rows x 64 B
constexpr int SLOT = 4 * PAN;         // one frame: dg q0, dg q1, x h0, x h1
constexpr int DR = 8;                 // frame slots in the ring
constexpr int BLOCKS = 512;           // target blocks per launch (2 per CU)
// timing ablations (results wrong; tools builds only, -DGWF_DBG=<mask>): 1 skip the per-frame LDS reads and MFMAs,
// 2 skip the per-frame barrier, 4 skip the DMA
#ifndef GWF_DBG
#define GWF_DBG 0
#endif

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

template <int N, typename F>
DEV void sfor(F&& f) {
  [&]<int... I>(std::integer_sequence<int, I...>) { (f.template operator()<I>(), ...); }(
      std::make_integer_sequence<int, N>{});
}

DEV int swz(int row) { return (row >> 2) & 3; }  // 16-B unit swizzle of a 64-B panel row
DEV int poff(int row, int unit) { return row * 64 + ((unit ^ swz(row)) << 4); }

DEV unsigned lds_u32(const void* p) { return (unsigned)(size_t)(const __attribute__((address_space(3))) char*)p; }

// 16 B per lane, global -> LDS at M0 = lds_off (lane-linear); m0 saved/restored around the issue
DEV void glds16(const void* src, unsigned lds_off) {
  unsigned saved;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(saved) : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds_off)) : "memory");
}

// Transposing read of a swizzled panel: lane (m = lane & 31, h = lane >> 5) gets channel m of rows
// rlo + q (j = 0..3) and rhi + q (j = 4..7), where the row bases are given per h.
DEV bf16x8 trread(const char* panel, int rlo, int rhi, int lane) {
  const int i = lane & 15, gq = lane >> 4;
  const int q = i >> 2, p = i & 3;
  const int unit = 2 * (gq & 1) + (p >> 1), off = 8 * (p & 1);
  const int r0 = rlo + q, r1 = rhi + q;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(panel + poff(r0, unit) + off));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(panel + poff(r1, unit) + off));
  s16x8 v;
  v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
  v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
  return __builtin_bit_cast(bf16x8, v);
}

DEV bf16x8 cvt8(const f32x16& c, int base) {
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (bf16)c[base + j];
  return v;
}

struct GWF {
  int nco, nci, ntiles, R, FB;
  float* part_w;  // [R][P][Cout][Cin]
  float* part_a;  // [R][ntiles][P][32][32]
  float* part_b;  // [R][P][Cout]
};

template <int P>
__global__ __launch_bounds__(NW * 64, 2) void gwf_kernel(const stgcn_gconv_wgrad_frame_desc a, const GWF g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cq = wave & 1, ch = wave >> 1;
  const int l31 = lane & 31, lh = lane >> 5;
  const int V = a.V;

  // XCD-aware order: the tiles of one run of frames are consecutive ids of one XCD (shared panels in L2)
  int wg;
  {
    const int id = blockIdx.x, nb = gridDim.x, x = id & 7, q = nb >> 3, r = nb & 7;
    wg = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (id >> 3);
  }
  const int tile = wg % g.ntiles, rr = wg / g.ntiles;
  const int tco = tile / g.nci, tci = tile % g.nci;
  const int co0 = tco * 64, ci0 = tci * 64;
  const int f0 = min(a.NT, rr * g.FB), f1 = min(a.NT, f0 + g.FB);
  const bool bias_part = tci == 0;  // S (and the bias terms) from the first ci tile of each co tile

  char* const ring = smem;
  float* const colsum = reinterpret_cast<float*>(smem + DR * SLOT);  // [P][32]
  float* const beta = colsum + P * 32;                                // [2][P][32]
  char* const afr = reinterpret_cast<char*>(beta + 2 * P * 32);       // [P + 1][2][64] fragments

  // ---- ring zeroed (rows V..31 of every panel stay zero: the DMA never writes them); column sums of A
  {
    uint4* z = reinterpret_cast<uint4*>(ring);
    for (int e = tid; e < DR * SLOT / 16; e += NW * 64) z[e] = make_uint4(0, 0, 0, 0);
    if (tid < P * 32) {
      const int p = tid >> 5, w = tid & 31;
      float s = 0.f;
      if (w < V)
        for (int v = 0; v < V; ++v) s += a.A[((long)p * V + v) * V + w];
      colsum[tid] = s;
    }
  }
  // ---- operands: W_p^T fragments in registers (Z's A operand: row ci, k = co of this wave's quarter); the A_p
  // fragments (D's A operand: row v, k = w) and the identity (S's A operand) as a fragment image in LDS,
  // [P + 1][2 k-steps][64 lanes] x 16 B, read per frame (registers are the kernel's limit)
  bf16x8 wf[P][2];
  {
    const int ci = ci0 + ch * 32 + l31;
#pragma unroll
    for (int p = 0; p < P; ++p)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        float wv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) wv[j] = a.W[((long)p * a.Cout + co0 + cq * 32 + 16 * s + 8 * lh + j) * a.Cin + ci];
#pragma unroll
        for (int j = 0; j < 8; ++j) wf[p][s][j] = (bf16)wv[j];
      }
    for (int e = tid; e < (P + 1) * 2 * 64; e += NW * 64) {
      const int p = e >> 7, s = (e >> 6) & 1, ln = e & 63, v = ln & 31, h = ln >> 5;
      bf16x8 f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int w = 16 * s + 8 * h + j;
        f[j] = (bf16)(p == P ? (v == w ? 1.f : 0.f) : (v < V && w < V ? a.A[((long)p * V + v) * V + w] : 0.f));
      }
      *reinterpret_cast<bf16x8*>(afr + e * 16) = f;
    }
  }
  __syncthreads();

  // ---- DMA: wave s stages panel s of every frame (0/1: dg co quarters, 2/3: x ci halves); lane -> (row
  // lane / 4 (+16), 16-B unit lane % 4), the source unit swizzled so the LDS image is poff-ordered
  const bf16* __restrict__ dy = reinterpret_cast<const bf16*>(a.dy);
  const bf16* __restrict__ xs = reinterpret_cast<const bf16*>(a.x);
  const int prow = lane >> 2, pu = lane & 3;
  const bool is_dy = wave < 2;
  const long ld = is_dy ? a.dy_ld : a.x_ld;
  const bf16* base0 = (is_dy ? dy + co0 + 32 * wave : xs + ci0 + 32 * (wave - 2));
  const bf16* src_lo = base0 + (long)prow * ld + 8 * (pu ^ swz(prow));
  const bf16* src_hi = base0 + (long)(prow + 16) * ld + 8 * (pu ^ swz(prow + 16));
  const bool hi_ok = prow + 16 < V;
  const long fstep = (long)V * ld;
  const unsigned ring0 = lds_u32(ring) + (unsigned)(wave * PAN);
  auto issue = [&](int f) {
    const unsigned dst = ring0 + (unsigned)(((f - f0) % DR) * SLOT);
    glds16(src_lo + f * fstep, dst);
    if (hi_ok) glds16(src_hi + f * fstep, dst + 1024);
  };
#pragma unroll
  for (int k = 0; k < DR - 1; ++k)
    if (!(GWF_DBG & 4) && f0 + k < f1) issue(f0 + k);

  const f32x16 zero = {};
  f32x16 accW[P], accA[P], accS = zero;
#pragma unroll
  for (int p = 0; p < P; ++p) {
    accW[p] = zero;
    accA[p] = zero;
  }
  const bool do_s = bias_part && ch == 0;

  for (int f = f0; f < f1; ++f) {
    const int after = min(DR - 2, f1 - 1 - f);  // frames issued after f
    sfor<DR - 1>([&]<int m>() {
      if (after == m) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * m) : "memory");
    });
    if constexpr (!(GWF_DBG & 2)) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (!(GWF_DBG & 4) && f + DR - 1 < f1) issue(f + DR - 1);  // into the slot of frame f - 1, free after the barrier
    if constexpr ((GWF_DBG & 1) != 0) continue;
    const char* slot = ring + ((f - f0) % DR) * SLOT;
    const char* pdy = slot + cq * PAN;
    const char* px = slot + (2 + ch) * PAN;
    // dg row w = l31, channels 16s + 8h .. +7 of the quarter (Z's B operand, k = co)
    bf16x8 zb[2], dt[2], xa[2], xt[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      zb[s] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(pdy + poff(l31, 2 * s + lh)));
      // dg transposed: channel l31 of rows 16s + 8h + j (D's and S's B operand, k = w)
      dt[s] = trread(pdy, 16 * s + 8 * lh, 16 * s + 8 * lh + 4, lane);
      // x row v = l31, channels 16s + 4h + (j&3) + 8(j>>2) (dA's A operand, k = ci in Z's accumulator order)
      const uint2 u0 = *reinterpret_cast<const uint2*>(px + poff(l31, 2 * s) + 8 * lh);
      const uint2 u1 = *reinterpret_cast<const uint2*>(px + poff(l31, 2 * s + 1) + 8 * lh);
      xa[s] = __builtin_bit_cast(bf16x8, make_uint4(u0.x, u0.y, u1.x, u1.y));
      // x transposed: channel l31 of rows 16s + 4h + (j&3) + 8(j>>2) (dW's B operand, k = v in D's order)
      xt[s] = trread(px, 16 * s + 4 * lh, 16 * s + 8 + 4 * lh, lane);
    }
#pragma unroll
    for (int p = 0; p < P; ++p) {
      f32x16 z = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[p][0], zb[0], zero, 0, 0, 0);
      z = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[p][1], zb[1], z, 0, 0, 0);
      const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(afr + ((p * 2) * 64 + lane) * 16);
      const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(afr + ((p * 2 + 1) * 64 + lane) * 16);
      f32x16 d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, dt[0], zero, 0, 0, 0);
      d = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, dt[1], d, 0, 0, 0);
      accA[p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xa[0], cvt8(z, 0), accA[p], 0, 0, 0);
      accA[p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(xa[1], cvt8(z, 8), accA[p], 0, 0, 0);
      accW[p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cvt8(d, 0), xt[0], accW[p], 0, 0, 0);
      accW[p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cvt8(d, 8), xt[1], accW[p], 0, 0, 0);
    }
    if (do_s) {
      const bf16x8 i0 = *reinterpret_cast<const bf16x8*>(afr + ((P * 2) * 64 + lane) * 16);
      const bf16x8 i1 = *reinterpret_cast<const bf16x8*>(afr + ((P * 2 + 1) * 64 + lane) * 16);
      accS = __builtin_amdgcn_mfma_f32_32x32x16_bf16(i0, dt[0], accS, 0, 0, 0);
      accS = __builtin_amdgcn_mfma_f32_32x32x16_bf16(i1, dt[1], accS, 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");

  // ---- dW tile partial: lane = ci, rows = co
  {
    const int ci = ci0 + ch * 32 + l31;
#pragma unroll
    for (int p = 0; p < P; ++p) {
      float* dst = g.part_w + (((long)rr * P + p) * a.Cout + co0 + cq * 32) * a.Cin + ci;
#pragma unroll
      for (int r = 0; r < 16; ++r) dst[(long)acc_row(r, lane) * a.Cin] = accW[p][r];
    }
  }
  // ---- bias terms from S (lane = co, rows = w): beta_p[w] = sum_co b_p[co] S[w][co] (into LDS, per quarter),
  // db_p[co] = sum_w colsum_p[w] S[w][co] (partial of this run of frames)
  float* red = reinterpret_cast<float*>(ring);  // [NW][P][16][64]
  if (do_s) {
    const int co = co0 + cq * 32 + l31;
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const float bp = a.bconv ? a.bconv[(long)p * a.Cout + co] : 0.f;
      float dbs = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float t = accS[r] * bp;
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) t += __shfl_xor(t, o);
        if (l31 == 0) beta[(cq * P + p) * 32 + acc_row(r, lane)] = t;
        dbs = fmaf(colsum[p * 32 + acc_row(r, lane)], accS[r], dbs);
      }
      dbs += __shfl_xor(dbs, 32);
      if (lh == 0) g.part_b[((long)rr * P + p) * a.Cout + co] = dbs;
    }
  }
  // ---- dA: the four waves' partials summed in LDS (+ beta on every row v), one partial per block
#pragma unroll
  for (int p = 0; p < P; ++p)
#pragma unroll
    for (int r = 0; r < 16; ++r) red[((wave * P + p) * 16 + r) * 64 + lane] = accA[p][r];
  __syncthreads();
  float* pa = g.part_a + ((long)rr * g.ntiles + tile) * P * 1024;
  for (int e = tid; e < P * 1024; e += NW * 64) {
    const int p = e >> 10, rem = e & 1023, r = rem >> 6, ln = rem & 63;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) s += red[((w * P + p) * 16 + r) * 64 + ln];
    if (bias_part) s += beta[p * 32 + (ln & 31)] + beta[(P + p) * 32 + (ln & 31)];
    pa[p * 1024 + acc_row(r, ln) * 32 + (ln & 31)] = s;
  }
}

// dA[p][v][w] = sum_{r,tile} part_a; db[e] = sum_r part_b[r][e] in a fixed order (dW goes through the float4
// slab reduction).  Block = 64 consecutive outputs x 4 groups of partial rows, summed in LDS.
__global__ __launch_bounds__(256) void gwf_reduce_kernel(const GWF g, int P, int V, int Cout, int Cin, float* dW,
                                                         float* dA, float* db) {
  __shared__ float red[4][64];
  const int tid = threadIdx.x, el = tid & 63, grp = tid >> 6;
  const long Ew = (long)P * Cout * Cin, Ea = (long)P * V * V, Eb = (long)P * Cout;
  const long nbw = 0, nba = (Ea + 63) / 64;  // dW: slab_reduce_launch
  long b = blockIdx.x;
  float s = 0.f;
  float* out;
  long e;
  if (b < nbw) {
    e = b * 64 + el;
    if (e < Ew)
      for (int r = grp; r < g.R; r += 4) s += g.part_w[(long)r * Ew + e];
    out = dW;
  } else if (b < nbw + nba) {
    e = (b - nbw) * 64 + el;
    if (e < Ea) {
      const int p = (int)(e / (V * V)), vw = (int)(e % (V * V)), v = vw / V, w = vw % V;
      const long n = (long)g.R * g.ntiles;
      for (long r = grp; r < n; r += 4) s += g.part_a[(r * P + p) * 1024 + v * 32 + w];
    }
    out = dA;
  } else {
    e = (b - nbw - nba) * 64 + el;
    if (e < Eb)
      for (int r = grp; r < g.R; r += 4) s += g.part_b[(long)r * Eb + e];
    out = db;
  }
  red[grp][el] = s;
  __syncthreads();
  const long lim = b < nbw ? Ew : b < nbw + nba ? Ea : Eb;
  if (grp == 0 && e < lim) out[e] = (red[0][el] + red[1][el]) + (red[2][el] + red[3][el]);
}

GWF plan(const stgcn_gconv_wgrad_frame_desc& a) {
  GWF g{};
  g.nco = a.Cout / 64;
  g.nci = a.Cin / 64;
  g.ntiles = g.nco * g.nci;
  int R = BLOCKS / g.ntiles;
  if (R < 1) R = 1;
  if (R > a.NT) R = a.NT;
  g.FB = (a.NT + R - 1) / R;
  g.R = (a.NT + g.FB - 1) / g.FB;
  return g;
}

bool shape_ok(const stgcn_gconv_wgrad_frame_desc& a) {
  return a.NT >= 1 && a.V > 16 && a.V <= 32 && a.P >= 1 && a.P <= 3 && a.Cin >= 64 && a.Cin % 64 == 0 &&
         a.Cout >= 64 && a.Cout % 64 == 0 && a.x_ld % 8 == 0 && a.dy_ld % 8 == 0 && a.x_ld >= a.Cin &&
         a.dy_ld >= a.Cout;
}

}  // namespace

// deterministic two-level float4 sum of R fp32 slabs (wgrad_tile.hip); part holds 16 * E floats
int slab_reduce_launch(const float* slab, int R, long E, float* part, float* dw, hipStream_t s, int mode, int Kt,
                       long CoCi);

long gconv_wgrad_frame_workspace(const stgcn_gconv_wgrad_frame_desc& a) {
  if (!shape_ok(a)) return -1;
  const GWF g = plan(a);
  const long Ew = (long)a.P * a.Cout * a.Cin;
  return 4L * ((long)g.R * Ew + (long)g.R * g.ntiles * a.P * 1024 + (long)g.R * a.P * a.Cout + 16 * Ew);
}

int gconv_wgrad_frame_launch(const stgcn_gconv_wgrad_frame_desc& a, hipStream_t s) {
  if (!shape_ok(a) || !a.x || !a.dy || !a.A || !a.W || !a.dW || !a.dA || !a.db) return STGCN_EBADSHAPE;
  GWF g = plan(a);
  const long need = gconv_wgrad_frame_workspace(a);
  if (!a.work || a.work_bytes < need) return STGCN_EBADSHAPE;
  float* w = reinterpret_cast<float*>(a.work);
  g.part_w = w;
  g.part_a = g.part_w + (long)g.R * a.P * a.Cout * a.Cin;
  g.part_b = g.part_a + (long)g.R * g.ntiles * a.P * 1024;
  typedef void (*KFn)(const stgcn_gconv_wgrad_frame_desc, const GWF);
  static const KFn tab[3] = {gwf_kernel<1>, gwf_kernel<2>, gwf_kernel<3>};
  const KFn k = tab[a.P - 1];
  const int lds = DR * SLOT + 3 * a.P * 32 * 4 + (a.P + 1) * 2 * 64 * 16;
  if (stgcn_lds_attr((const void*)k, lds, s)) return STGCN_EHIP;
  hipLaunchKernelGGL(k, dim3((unsigned)(g.R * g.ntiles)), dim3(NW * 64), lds, s, a, g);
  if (hipGetLastError() != hipSuccess) return STGCN_EHIP;
  // dW: the float4 two-level slab reduction (16 row groups in parallel, then their fixed-order sum); dA, db here
  const long Ew = (long)a.P * a.Cout * a.Cin;
  float* part = g.part_b + (long)g.R * a.P * a.Cout;
  if (slab_reduce_launch(g.part_w, g.R, Ew, part, a.dW, s, 1, 1, Ew) != STGCN_OK) return STGCN_EHIP;
  const long nb = ((long)a.P * a.V * a.V + 63) / 64 + ((long)a.P * a.Cout + 63) / 64;
  hipLaunchKernelGGL(gwf_reduce_kernel, dim3((unsigned)nb), dim3(256), 0, s, g, a.P, a.V, a.Cout, a.Cin, a.dW, a.dA,
                     a.db);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
