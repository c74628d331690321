// Graph convolution of ST-GCN (ConvTemporalGraphical, models/utils/tgcn.py:58-79) as ONE fused kernel
// that runs both of its products on the matrix cores, frame by frame, with nothing intermediate in HBM.
//
//   forward (trans_a = 0):  out[(i,w)][co] = sum_p sum_ci W'[co][p*Cin+ci] XA_p[(i,w)][ci]  (+ bias[w][co])
//                           XA_p[(i,w)][ci] = sum_v A[p][v][w] in[(i,v)][ci]
//   data grad (trans_a = 1): XA_p[(i,v)] = sum_w A[p][v][w] in[(i,w)] (in = dg), W'[ci][p*Cout+co] = W_p[co][ci]
//                           -> dx = sum_p A_p (dg W_p)                           (autograd of tgcn.py:71-79)
//
// The reference materialises conv1x1(x) (N, P*Cout, T, V) and multiplies it by A.  Here, per frame i
// (its V <= 32 joint rows, zero-padded to 32) and 32-channel block b of the input:
//   stage 1 (joint mix):  XA_p^T[ci][w] = sum_v X^T[ci][v] A_p[v][w]      one 32x32x32 MFMA pair per p;
//                         X^T comes from the frame's LDS panel by transposing reads (ds_read_b64_tr_b16),
//                         A_p lives in registers for the whole kernel;
//   stage 2 (1x1 conv):   out^T[co][w] += sum_{p,ci} W'[co][p,ci] XA_p^T[ci][w]   the stage-1 accumulators,
//                         rounded to bf16, ARE the B operand (lane = joint w, rows = channels): no LDS
//                         round trip.  The K order inside each 16-channel step follows the accumulator
//                         rows (slot (h, j) = channel 8(j/4) + 4h + j%4), so the host packs W' with its
//                         columns permuted the same way (stgcn_gcn_tile weight image, include/stgcn_amd.h).
// Output tile = 64 channels x one frame (lane = joint): bias + 8-B row stores from the accumulators;
// BatchNorm partial sums stay in registers per (lane, channel) over the block's frames and are reduced
// once per block.  Blocks own (row block of frames, 64-channel column tile); their W' slice (P*Cin x 64)
// sits in LDS, each wave streams its own frames' input panels through a private 8-deep LDS ring filled
// by global->LDS DMA (no block barrier in the main loop).
#include "common.h"
#include "../../include/stgcn_amd.h"
#include <stdlib.h>
#include <utility>

namespace {

constexpr int BN = 64, TN = 2;          // output channels per block (two 32-channel MFMA tiles)
constexpr int NW = 4;                   // waves per block
constexpr int D = 8;                    // panels in flight per wave
constexpr int PANEL = 32 * 64;          // 32 joint rows x 32 channels bf16
constexpr int RING = D * PANEL;
constexpr int PMAX = 3;
constexpr int LDS_MAX = 160 * 1024;
constexpr int NCU = 256;                // blocks per launch target (MI355X CUs)
constexpr int ST = 4 * TN;              // output store instructions per frame

template <int N, typename F>
DEV void static_for(F&& f) {
  [&]<int... I>(std::integer_sequence<int, I...>) { (f.template operator()<I>(), ...); }(
      std::make_integer_sequence<int, N>{});
}

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// A operand of a 32x32x16 MFMA (m = channel, k = joint row) from a [row][32 ch] panel: lane (m, h) gets
// rows row0 + 8h + 0..7 of channel m
DEV bf16x8 trfrag(const char* panel, int row0, int lane) {
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

// 16 B per lane, global -> LDS (lane-linear at M0 = lds_off).  Issued from inline asm on purpose: the
// compiler would otherwise treat every later LDS read as aliasing the DMA and drain vmcnt to 0 before it,
// which serialises the panel ring.  Ordering is kept by the "memory" clobbers here and on the explicit
// vmcnt waits of the main loop.
// m0 is reserved, so it is saved in an SGPR the asm owns and restored after the issue (not clobbered).
DEV void glds16(const void* src, unsigned lds_off) {
  unsigned saved;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(saved) : "v"(src), "s"(lds_off) : "memory");
}
DEV unsigned lds_u32(const void* p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) char*)p;
}

struct GMGeom {
  int FB;    // frames per row block
  int R;     // row blocks
  int ncol;  // column tiles (Cout / 64)
  int k16n;  // K blocks per column of the weight image (Kw_pad / 16)
};

template <int P, int G, int DBG = 0>
__global__ __launch_bounds__(NW * 64, 1) void gcn_mfma_kernel(const stgcn_gcn_tile_desc a, const GMGeom g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 31, lh = lane >> 5;
  const int V = a.V;

  // XCD-aware order: consecutive ids (the column tiles of one row block) share the input panels in L2
  int wg;
  {
    const int id = blockIdx.x, nb = gridDim.x, x = id & 7, q = nb >> 3, r = nb & 7;
    wg = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (id >> 3);
  }
  const int ct = wg % g.ncol, rb = wg / g.ncol;
  const int f0 = rb * g.FB, f1 = min(a.NT, f0 + g.FB);
  if (f0 >= f1) return;  // block-uniform, before any barrier
  const int n0 = ct * BN;
  constexpr int K16 = P * G * 2;  // 16-wide K steps of the block's W' slice
  char* const sW = smem;        // [t][K16] 1-KiB fragment blocks
  char* const sRing = smem + TN * K16 * 1024 + wave * RING;

  // ---- W' slice -> LDS; rings zeroed (rows V..31 of every panel stay zero: the DMA never writes them)
  {
    const uint4* wsrc = reinterpret_cast<const uint4*>(a.w_frag);
    uint4* wdst = reinterpret_cast<uint4*>(sW);
    static_assert(TN * K16 % NW == 0, "W' copy");
    constexpr int NCP = TN * K16 / NW;  // 16-B units per thread
    uint4 wv[NCP];
#pragma unroll
    for (int i = 0; i < NCP; ++i) {
      const int e = tid + i * NW * 64, blk = e >> 6, l = e & 63, t = blk / K16, k = blk - t * K16;
      wv[i] = wsrc[((long)(2 * ct + t) * g.k16n + k) * 64 + l];
    }
#pragma unroll
    for (int i = 0; i < NCP; ++i) wdst[tid + i * NW * 64] = wv[i];
    uint4* z = reinterpret_cast<uint4*>(smem + TN * K16 * 1024);
    for (int e = tid; e < NW * RING / 16; e += NW * 64) z[e] = make_uint4(0, 0, 0, 0);
  }
  // ---- stage-1 B operands: B[k = input joint u][n = output joint o] = A[p][u][o] (fwd) / A[p][o][u] (dgrad)
  // (unguarded loads at clamped indices, masked afterwards: all in flight at once)
  bf16x8 ac[P][2];
  {
    const int o = min(lr, V - 1);
    const int sr = a.trans_a ? V : 1, sc = a.trans_a ? 1 : V;  // strides of o and u in A[p]
    float av[P][2][8];
#pragma unroll
    for (int p = 0; p < P; ++p)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int u = min(16 * ks + 8 * lh + j, V - 1);
          // fwd: A[p][u][o]; dgrad: A[p][o][u]
          av[p][ks][j] = a.A[(long)p * V * V + (long)u * sc + (long)o * sr];
        }
#pragma unroll
    for (int p = 0; p < P; ++p)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int u = 16 * ks + 8 * lh + j;
          ac[p][ks][j] = (bf16)((u < V && lr < V) ? av[p][ks][j] : 0.f);
        }
  }
  // ---- bias of this lane's (joint, channels)
  const bool jok = lr < V;
  float breg[TN][16];
  {
    const float* bp = a.bias ? a.bias + (long)min(lr, V - 1) * a.Cout + n0 + 4 * lh : nullptr;
#pragma unroll
    for (int t = 0; t < TN; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float4 b4 = make_float4(0.f, 0.f, 0.f, 0.f);
        if (bp) b4 = *reinterpret_cast<const float4*>(bp + 32 * t + 8 * q);
        breg[t][4 * q] = jok ? b4.x : 0.f;
        breg[t][4 * q + 1] = jok ? b4.y : 0.f;
        breg[t][4 * q + 2] = jok ? b4.z : 0.f;
        breg[t][4 * q + 3] = jok ? b4.w : 0.f;
      }
  }
  __syncthreads();

  // ---- this wave's frames f = f0 + wave + 4k; panel stream (frame, channel block) in order
  const int fw = f0 + wave;
  const int nfw = fw < f1 ? (f1 - fw + NW - 1) / NW : 0;
  const int NP = nfw * G;
  const bf16* __restrict__ in = reinterpret_cast<const bf16*>(a.in);
  const int lrow = lane >> 2, lunit = lane & 3;
  const unsigned ring0 = lds_u32(sRing);
  const bool row2 = lrow + 16 < V;
  const bf16* src0 = in + ((long)fw * V + lrow) * a.in_ld + lunit * 8;
  const long fstep = (long)NW * V * a.in_ld;  // elements between a wave's consecutive frames
  auto issue = [&](int k) {  // panel k of the wave's stream -> ring slot k % D
    const int f = k / G, b = k - f * G;
    const unsigned dst = ring0 + (unsigned)((k & (D - 1)) * PANEL);
    const bf16* src = src0 + f * fstep + b * 32;
    glds16(src, dst);  // rows 0..15 (all < V)
    if (row2) glds16(src + 16L * a.in_ld, dst + 1024);
  };
  const int npre = NP < D ? NP : D;
  if constexpr (!(DBG & 1))
    for (int k = 0; k < npre; ++k) issue(k);

  f32x16 acc[TN];
  float s1[TN][16], s2[TN][16];
#pragma unroll
  for (int t = 0; t < TN; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      s1[t][r] = 0.f;
      s2[t][r] = 0.f;
    }
  const f32x16 zero = {};
#pragma unroll
  for (int t = 0; t < TN; ++t) acc[t] = zero;
  bf16* __restrict__ out = reinterpret_cast<bf16*>(a.out);
  const bool has_out = out != nullptr;
  const bool stats = a.stats != nullptr, accum = a.accumulate != 0;
  const char* const wl = sW + lane * 16;
  float sink = 0.f;

  // Software pipeline over the wave's panel stream: panel q's X^T fragments are read two iterations
  // before its stage 2, its mix (stage 1) runs one iteration before, its W' fragments are read at the
  // end of the previous iteration.  Iteration q: [stage 1 of q+1] [DMA wait, X^T reads of q+2]
  // [stage 2 of q (+ frame epilogue)] [bf16 mix operands of q+1] [W' reads of q+1].
  bf16x8 fx0, fx1, xb[2][P][2], wf[2][P][2][TN];  // [panel parity]: written while the other is consumed
  f32x16 c1[P];
  auto read_x = [&](int q) {
    const char* pan = sRing + (q & (D - 1)) * PANEL;
    fx0 = trfrag(pan, 0, lane);
    fx1 = trfrag(pan, 16, lane);
  };
  auto stage1 = [&]() {
#pragma unroll
    for (int p = 0; p < P; ++p) {
      c1[p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fx0, ac[p][0], zero, 0, 0, 0);
      c1[p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fx1, ac[p][1], c1[p], 0, 0, 0);
    }
  };
  auto to_xb = [&]<int par>() {
#pragma unroll
    for (int p = 0; p < P; ++p)
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) xb[par][p][s][j] = (bf16)c1[p][8 * s + j];
  };
  auto read_w = [&]<int cb>() {
    constexpr int par = cb & 1;
#pragma unroll
    for (int p = 0; p < P; ++p)
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int t = 0; t < TN; ++t)
          wf[par][p][s][t] = __builtin_bit_cast(
              bf16x8, *reinterpret_cast<const uint4*>(wl + (t * K16 + (p * G + cb) * 2 + s) * 1024));
  };
  if (NP > 0) {
    if constexpr (!(DBG & 1)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    read_x(0);
    stage1();
    to_xb.template operator()<0>();
    read_x(1);  // past the stream's end: a stale slot, never used
    read_w.template operator()<0>();
  }
  for (int k = 0; k < nfw; ++k) {
    const int cf = fw + k * NW;
    static_for<G>([&]<int cb>() {
      const int pi = k * G + cb;
      constexpr int par = cb & 1;  // parity of panel pi (G is even)
      // Wait for panel pi + 2's DMA.  vmcnt counts loads, DMA and stores in issue order, so the wait
      // names every op issued after that DMA: the D - 2 later panels (2 ops each) and, once the wave is
      // CNT frames in, the ST output stores of each of the last CNT frames.  A smaller count only
      // over-waits; a larger one would read a half-written panel.  (Checked by enumeration of the issue
      // order for D = 8, G = 2, 4, 8.)
      if constexpr (!(DBG & 1)) {
        constexpr int c = cb + 3 - D;
        constexpr int CNT = 1 - (c <= 0 ? -((-c) / G) : (c + G - 1) / G);  // 1 - ceil(c / G)
        static_assert(2 * (D - 2) + ST * CNT <= 63, "vmcnt range");
        if (pi + D < NP) {
          issue(pi + D);
          if (k >= CNT && has_out)  // stats-only launches issue no stores: the DMA-only count below
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (D - 2) + ST * CNT) : "memory");
          else
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (D - 2)) : "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      }
      // one scheduling region: stage 1 of pi + 1, stage 2 of pi, and around them the LDS reads of
      // pi + 2 / pi + 1 and the bf16 conversion of the mix; interleaved below so that the loads and the
      // conversion ride in the MFMA gaps instead of stalling between the two stages
      stage1();                                            // panel pi + 1
      read_x(pi + 2);
      read_w.template operator()<(cb + 1) % G>();         // panel pi + 1
#pragma unroll
      for (int p = 0; p < P; ++p)
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int t = 0; t < TN; ++t)
            acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[par][p][s][t], xb[par][p][s], acc[t], 0, 0, 0);
      to_xb.template operator()<par ^ 1>();               // panel pi + 1
      __builtin_amdgcn_sched_group_barrier(0x008, 2 * P, 0);  // stage-1 MFMAs
      static_for<2 * P * TN>([&]<int i>() {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                               // a stage-2 MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, i < 8 ? 2 : 0, 0);                 // LDS reads
        __builtin_amdgcn_sched_group_barrier(0x002, i >= 2 ? (72 + 2 * P * TN - 3) / (2 * P * TN - 2) : 0, 0);  // VALU
      });
      if constexpr (cb == G - 1) {
        // ---- frame cf done: out[(cf, joint lr)][n0 + 32t + 8q + 4lh + e]
        if (jok) {  // out == NULL: statistics only (pass 1 of the fused layer, layer_fused.hip)
          bf16* orow = out ? out + ((long)cf * V + lr) * a.out_ld + n0 + 4 * lh : nullptr;
#pragma unroll
          for (int t = 0; t < TN; ++t)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              float v[4];
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = acc[t][4 * q + e] + breg[t][4 * q + e];
              uint2* po = reinterpret_cast<uint2*>(orow + 32 * t + 8 * q);
              if (accum && orow) {
                const bf16x4 o = __builtin_bit_cast(bf16x4, *po);
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] += (float)o[e];
              }
              bf16x4 st;
#pragma unroll
              for (int e = 0; e < 4; ++e) st[e] = (bf16)v[e];
              if constexpr (DBG & 2) {
                sink += (float)st[0] + (float)st[1] + (float)st[2] + (float)st[3];
              } else if (orow) {
                *po = __builtin_bit_cast(uint2, st);
              }
              if (stats) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                  s1[t][4 * q + e] += v[e];
                  s2[t][4 * q + e] = fmaf(v[e], v[e], s2[t][4 * q + e]);
                }
              }
            }
        }
#pragma unroll
        for (int t = 0; t < TN; ++t) acc[t] = zero;
      }
    });
  }

  if constexpr ((DBG & 2) != 0) {
    if (sink == 1234.5f) out[0] = (bf16)sink;  // keeps the compute of the store-free variant alive
  }
  if (!stats) return;
  // ---- BatchNorm partials of the block: sum over joints (lanes of a half) and waves
  __syncthreads();  // every wave is past its ring: reuse the rings as [wave][64 ch][2] scratch
  float* red = reinterpret_cast<float*>(smem + TN * K16 * 1024);
#pragma unroll
  for (int t = 0; t < TN; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      float x1 = s1[t][r], x2 = s2[t][r];
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) {
        x1 += __shfl_xor(x1, o);
        x2 += __shfl_xor(x2, o);
      }
      if (lr == 0) {
        const int c = 32 * t + 8 * (r >> 2) + 4 * lh + (r & 3);
        red[(wave * BN + c) * 2] = x1;
        red[(wave * BN + c) * 2 + 1] = x2;
      }
    }
  __syncthreads();
  if (tid < BN) {
    float t1 = 0.f, t2 = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      t1 += red[(w * BN + tid) * 2];
      t2 += red[(w * BN + tid) * 2 + 1];
    }
    const float n = (float)((f1 - f0) * V);
    const float mean = t1 / n;
    reinterpret_cast<float4*>(a.stats)[(long)rb * a.Cout_pad + n0 + tid] =
        make_float4(n, mean, fmaxf(t2 - t1 * mean, 0.f), 0.f);
  }
}

GMGeom plan(int NT, int Cout) {
  GMGeom g{};
  g.ncol = Cout / BN;
  int R = NCU / (g.ncol > 0 ? g.ncol : 1);
  if (R < 1) R = 1;
  if (R > NT) R = NT;
  g.FB = (NT + R - 1) / R;
  g.R = (NT + g.FB - 1) / g.FB;
  return g;
}

}  // namespace

long gcn_tile_row_blocks(int NT, int V, int Cout) {
  (void)V;
  if (NT < 1 || Cout < BN) return 1;
  return plan(NT, Cout).R;
}

int gcn_tile_launch(const stgcn_gcn_tile_desc& a, hipStream_t s) {
  if (a.V <= 16 || a.V > 32 || a.P < 1 || a.P > PMAX || a.NT < 1) return STGCN_EBADSHAPE;
  if (a.Cin % 32 || a.in_ld % 8 || a.Cout % BN || a.Cout_pad < a.Cout || a.out_ld % 4) return STGCN_EBADSHAPE;
  if (a.Kw_pad < a.P * a.Cin || a.Kw_pad % 16) return STGCN_EBADSHAPE;
  GMGeom g = plan(a.NT, a.Cout);
  const int G = a.Cin / 32;
  g.k16n = a.Kw_pad / 16;
  const size_t lds = (size_t)TN * a.P * G * 2 * 1024 + (size_t)NW * RING;
  if (lds > (size_t)LDS_MAX) return STGCN_EBADSHAPE;
  typedef void (*KFn)(const stgcn_gcn_tile_desc, const GMGeom);
  static const KFn tab[3][3] = {{gcn_mfma_kernel<1, 2>, gcn_mfma_kernel<1, 4>, gcn_mfma_kernel<1, 8>},
                                {gcn_mfma_kernel<2, 2>, gcn_mfma_kernel<2, 4>, gcn_mfma_kernel<2, 8>},
                                {gcn_mfma_kernel<3, 2>, gcn_mfma_kernel<3, 4>, gcn_mfma_kernel<3, 8>}};
  const int gi = G == 2 ? 0 : G == 4 ? 1 : G == 8 ? 2 : -1;
  if (gi < 0) return STGCN_EBADSHAPE;
  KFn k = tab[a.P - 1][gi];
  if (stgcn_lds_attr((const void*)k, LDS_MAX, s)) return STGCN_EHIP;
  hipLaunchKernelGGL(k, dim3((unsigned)(g.R * g.ncol)), dim3(NW * 64), lds, s, a, g);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
