// The fused ST-GCN layer (BASELINE north_star) for LayerNorm layers: ConvTemporalGraphical (tgcn.py:58-79) ->
// LN1 -> ReLU -> temporal Conv2d (Kt = 9) + bias (stgcn.py:151-159) -> LN2 -> + residual -> ReLU (stgcn.py:181-193)
// as ONE kernel: the graph-conv output g and h = relu(LN1(g)) live only in LDS, and no statistics leave the chip,
// because both LayerNorm([64,1,V]) norms are per frame over C x V (layernorm.py:22-28, unbiased variance).
// (BatchNorm layers cannot be one kernel: BN1's batch statistics need all of g before any h is consumed.  The
// two-pass BatchNorm form of this kernel lost to the unfused forward on every box and was removed in round 6;
// DESIGN 4.6 keeps its numbers.)
//
// Shapes: bf16, Cin = Cout = 64, stride 1, Kt = 9 (pad 4), P <= 3 partitions, 16 < V <= 25 — the north_star
// layer (N = 64, C = 64, T = 300, V = 25) and the 64 -> 64 layers of the ln/ configs.
//
// Block = 8 waves, one contiguous run of output frames of one sample (a quarter of a sample at N = 64:
// 256 blocks), walked in steps of CF = 8 frames.  Two roles run concurrently, one wave of each per SIMD,
// so one role's MFMAs fill the other's latency gaps:
//   GCN waves 4-7 (producers): per step, the 8 h frames the NEXT step needs.  A frame's x rows arrive as
//     two 32-channel panels [32 joint rows][32 ch] by global->LDS DMA (issued one step ahead); stage 1
//     mixes the joints (X^T A_p on MFMA, X^T by transposing LDS reads, A_p in registers), stage 2 runs the
//     1x1 conv from the stage-1 accumulators (W' in LDS).  A frame's 64 x V graph-conv values are one wave's
//     accumulators (initialised with the bias through A) -> the frame's mean and variance by two DPP wave
//     reductions -> h = relu(LN1(g)) -> bf16 -> the h ring.  Frames outside [0, T) are written as zeros (the
//     temporal conv's zero padding applies to h).
//   TCN waves 0-3 (consumers): out^T[co][row] = sum_{dt,ci} W[dt][co][ci] h[frame + dt - 4][row's joint][ci],
//     32x32x16 MFMAs with the weight fragments streamed from L2 (conv_wide.hip's fragment image) through a
//     register ring and the h fragments read from LDS.  Wave = (32 output channels, 4 frame-aligned row
//     tiles); each frame's LN2 (sum, sum of squares) is one DPP wave reduction plus ONE exchange with the
//     partner wave (the other 32 channels) through LDS, combined in a fixed order (deterministic); then
//     y = relu(LN2(z) + x) (identity residual of the 64 -> 64 stride-1 layer, x rows re-read from L2,
//     gamma2/beta2 staged in LDS) with 16-B stores.
// The h ring holds RF = 24 frames (a frame at slot a % RF): 16 being read for step s (frames 8s-4 ..
// 8s+11 of the run) and 8 being written for step s+1; one block barrier per step hands them over.
// Training forward: the kernel also writes g, u = z (pre-LN2), h and both LN statistics for the backward.
#include "common.h"
#include "../../include/stgcn_amd.h"
#include <stdlib.h>
#include <utility>

namespace {

// Timing ablations (results wrong): build with -DSTGCN_FUSED_DBG=<mask> (tools only, never the shipped library):
// bit 0 skip the GCN math, bit 1 the TCN math, bit 2 (LN) the residual loads, bit 3 (LN) the LN2 statistics,
// bit 4 the TCN z / BN2-partial stores, bit 5 the TCN weight-fragment loads, bit 6 the TCN h-fragment LDS reads,
// bit 7 three of the four z stores per row tile, bit 8 the BN2-partial stores
#ifndef STGCN_FUSED_DBG
#define STGCN_FUSED_DBG 0
#endif
constexpr int DBG = STGCN_FUSED_DBG;
// bit 10: per-wave cycle accounts (s_memtime) into g_fused_prof, read back with stgcn_fused_prof (tools only)
constexpr bool PROF = (DBG & 1024) != 0;
constexpr int PROF_BLOCKS = 4096;
__device__ long long g_fused_prof[PROF ? PROF_BLOCKS * 8 * 6 : 1];
DEV long long ptime() {
  if constexpr (PROF) return __builtin_amdgcn_s_memtime();
  return 0;
}

constexpr int NWT = 4, NWG = 4, NW = NWT + NWG;
constexpr int C = 64, G = C / 32;      // channels (in = out), 32-channel blocks
constexpr int HALO = 4, KT = 9;
constexpr int CF = 8;                  // output frames per step
constexpr int RF = 24;                 // h ring frames (16 read + 8 written per step)
constexpr int FPW = CF / NWG;          // h frames per GCN wave per step (2)
constexpr int PRO = 2 * HALO + CF;     // h frames before the first step (16)
constexpr int RSH = 2 * C + 16;        // h row bytes (144: conflict-free ds_read_b128 for any row offset)
// per-joint LDS tables read by 32 lanes of 32 different joints at once: row strides padded off the 256-B
// bank period (16 B further per joint), or every lane of a ds_read_b128 group hits the same four banks
constexpr int CGP = C + 4;             // gamma2 / beta2 row, floats (two planes)
constexpr int PANEL = 32 * 64;         // [32 joint rows][32 ch] bf16
constexpr int SLOTS = FPW * G;         // panel slots per GCN wave (one step's panels)
constexpr int RT = 4;                  // 32-row output tiles per TCN wave (8 frames x 25 joints = 7 tiles)
constexpr int NB = 9;                  // temporal-conv weight fragment ring depth (divides KSTEPS)
constexpr int KSTEPS = KT * C / 16;    // 36 k-steps of the temporal conv
constexpr int VMAX = 25;
constexpr int TARGET_BLOCKS = 256;     // MI355X CUs: runs per sample = 256 / N
constexpr int LDS_MAX = 160 * 1024;
static_assert(CF * VMAX <= 2 * RT * 32, "row tiles");

template <int N, typename F>
DEV void static_for(F&& f) {
  [&]<int... I>(std::integer_sequence<int, I...>) { (f.template operator()<I>(), ...); }(
      std::make_integer_sequence<int, N>{});
}

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x2n __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// A operand of a 32x32x16 MFMA (m = channel, k = joint row) from a [row][32 ch] panel (gcn_tile.hip)
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

// 16 B per lane, global -> LDS (lane-linear at M0 = lds_off), issued from asm so the compiler does not
// drain vmcnt before every later LDS read; m0 is saved and restored inside the asm (never clobbered).
DEV void glds16(const void* src, unsigned lds_off) {
  unsigned saved;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(saved) : "v"(src), "s"(lds_off) : "memory");
}
// Block barrier for the LDS hand-offs only: waits for this wave's LDS ops, NOT its outstanding global
// loads, DMA and stores (__syncthreads() would drain vmcnt: the weight-fragment ring, the next batch's
// x DMA and the z stores would all be waited for at every step).
DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Sum over the 32 lanes of each wave half (lanes 0-31, 32-63) with DPP (VALU only, no LDS crossbar): the
// totals land in lanes 31 and 63.
template <int CTRL, int ROWS>
DEV float dpp(float old, float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old), __builtin_bit_cast(int, v),
                                                                 CTRL, ROWS, 0xf, false));
}
DEV float half_sum(float v) {
  v += dpp<0xB1, 0xf>(0.f, v);   // quad_perm [1,0,3,2]
  v += dpp<0x4E, 0xf>(0.f, v);   // quad_perm [2,3,0,1]
  v += dpp<0x141, 0xf>(0.f, v);  // row_half_mirror: 8-lane sums
  v += dpp<0x140, 0xf>(0.f, v);  // row_mirror: 16-lane (row) sums
  v += dpp<0x142, 0xa>(0.f, v);  // row_bcast15 into rows 1 and 3: lanes 16-31 / 48-63 hold the half sums
  return v;
}

// total over all 64 lanes (both halves)
DEV float wave_total(float v) {
  v = half_sum(v);
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 31)) +
         __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}

DEV unsigned lds_u32(const void* p) { return (unsigned)(size_t)(const __attribute__((address_space(3))) char*)p; }

struct FGeom {
  int runs_n;  // runs per sample
  int run;     // frames per run (multiple of CF)
  int nsm;     // steps per run (run / CF)
  int off_tab, off_ring, off_h, off_red;  // LDS offsets
};

template <int P>
__global__ __launch_bounds__(NW * 64, 1) void layer_fused_kernel(const stgcn_layer_fused_desc a, const FGeom g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int K16 = P * G * 2;  // 16-wide K steps of W' (P*64 / 16)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 31, lh = lane >> 5;
  const int V = a.V, T = a.T;
  const int n = blockIdx.x / g.runs_n;
  const int R0 = (blockIdx.x - n * g.runs_n) * g.run;
  if (n >= a.N || R0 >= T) return;  // block-uniform, before any barrier
  const int R1 = min(T, R0 + g.run);
  const int nsteps = (R1 - R0 + CF - 1) / CF;
  const int nfr = (R1 - R0) + 2 * HALO;  // h frames the run needs: a in [0, nfr) <-> frame R0 - 4 + a

  char* const sW = smem;                                          // [2][K16] 1-KiB W' fragment blocks
  char* const sH = smem + g.off_h;                                // [RF * V][RSH]
  float* const sGam = reinterpret_cast<float*>(smem + g.off_tab);  // LN: [V][CGP] gamma2, then [V][CGP] beta2
  float* const sBet = sGam + V * CGP;
  float2* const sPart = reinterpret_cast<float2*>(smem + g.off_red);  // LN: [TCN wave][4 frames] (sum, sum of squares)
  unsigned* const sCnt = reinterpret_cast<unsigned*>(smem + g.off_red + NWT * 4 * 8);  // LN: per TCN wave, last step posted
  const int vrs = V * RSH;  // bytes per h frame
  float* const sTb = reinterpret_cast<float*>(smem + g.off_tab + 2 * V * CGP * 4);  // [64] tcn bias

  // ---- per block: W' slice, LN2 tables, zeroed panel rings (rows V..31 stay zero)
  {
    const uint4* wsrc = reinterpret_cast<const uint4*>(a.wg_frag);
    uint4* wdst = reinterpret_cast<uint4*>(sW);
    for (int e = tid; e < 2 * K16 * 64; e += NW * 64) wdst[e] = wsrc[e];
    for (int e = tid; e < V * C; e += NW * 64) {
      sGam[(e / C) * CGP + e % C] = a.ln2_g[e];
      sBet[(e / C) * CGP + e % C] = a.ln2_b[e];
    }
    if (tid < NWT) sCnt[tid] = 0u;
    for (int c = tid; c < C; c += NW * 64) sTb[c] = a.tbias ? a.tbias[c] : 0.f;
    uint4* z = reinterpret_cast<uint4*>(smem + g.off_ring);
    for (int e = tid; e < NWG * SLOTS * PANEL / 16; e += NW * 64) z[e] = make_uint4(0, 0, 0, 0);
  }
  __syncthreads();

  long long pa[6] = {0, 0, 0, 0, 0, 0};  // PROF: cycle accounts of this wave
  const long long pstart = ptime();
  auto prof_out = [&]() {
    pa[3] = ptime() - pstart;
    if (lane == 0 && blockIdx.x < PROF_BLOCKS)
      for (int j = 0; j < 6; ++j) g_fused_prof[((long)blockIdx.x * 8 + wave) * 6 + j] = pa[j];
  };
  if (wave >= NWT) {
    // =============================== GCN waves: h frames ===============================
    const int gw = wave - NWT;
    bf16x8 ac[P][2];  // stage-1 B operands: B[k = input joint u][n = output joint o] = A[p][u][o]
    {
      const int o = min(lr, V - 1);
      float av[P][2][8];
#pragma unroll
      for (int p = 0; p < P; ++p)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int u = min(16 * ks + 8 * lh + j, V - 1);
            av[p][ks][j] = a.A[(long)p * V * V + (long)u * V + o];
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
    const bf16* __restrict__ xg = reinterpret_cast<const bf16*>(a.x);
    const int lrow = lane >> 2, lunit = lane & 3;
    const bool row2 = lrow + 16 < V;
    const unsigned ring0 = lds_u32(smem + g.off_ring + gw * SLOTS * PANEL);
    const char* const ringp = smem + g.off_ring + gw * SLOTS * PANEL;
    const char* const wl = sW + lane * 16;
    const bf16* xs = xg + (long)n * T * V * a.x_ld + (long)lrow * a.x_ld + lunit * 8;
    const f32x16 zero = {};

    // the h frames of a "batch" b (b = 0: the prologue's first half, ...): frame a = base + gw + NWG*i
    auto frame_ok = [&](int fa) { return fa < nfr && R0 - HALO + fa >= 0 && R0 - HALO + fa < T; };
    auto issue = [&](int fa0) {  // DMA the panels of this wave's FPW frames fa0 + NWG*i (valid ones)
#pragma unroll
      for (int i = 0; i < FPW; ++i) {
        const int fa = fa0 + NWG * i;
        if (!frame_ok(fa)) continue;
        const bf16* src = xs + (long)(R0 - HALO + fa) * V * a.x_ld;
#pragma unroll
        for (int cb = 0; cb < G; ++cb) {
          const unsigned dst = ring0 + (unsigned)((i * G + cb) * PANEL);
          glds16(src + cb * 32, dst);
          if (row2) glds16(src + cb * 32 + 16L * a.x_ld, dst + 1024);
        }
      }
    };
    // compute the FPW frames whose panels sit in the ring; `next` >= 0: DMA that batch once the panels are read
    auto compute = [&](int fa0, int next) {
      const long long pt0 = ptime();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const long long pt1 = ptime();
      pa[0] += pt1 - pt0;
      bf16x8 fx[FPW][G][2];
#pragma unroll
      for (int i = 0; i < FPW; ++i)
#pragma unroll
        for (int cb = 0; cb < G; ++cb) {
          const char* pan = ringp + (i * G + cb) * PANEL;
          fx[i][cb][0] = trfrag(pan, 0, lane);
          fx[i][cb][1] = trfrag(pan, 16, lane);
        }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // ring read: refill it with the next batch
      // the DMA goes out after the epilogue, whose parameter loads (global) would otherwise wait behind it on the
      // in-order vmcnt
      // the FPW frames' chains interleaved per (channel block, partition): mix (stage 1) of every frame, then
      // bf16 + 1x1 conv (stage 2) of every frame, so one frame's MFMA latency hides under the other's MFMAs
      // (padding frames are computed too and replaced by zeros below)
      f32x16 accf[FPW][2];
#pragma unroll
      for (int i = 0; i < FPW; ++i) accf[i][0] = accf[i][1] = zero;
{
        // LN: the graph-conv bias enters as the accumulators' initial value (acc layout: lane = joint lr,
        // register r of tile t = channel 32t + 8(r>>2) + 4lh + (r&3)), loaded before the MFMAs run
        if (a.gbias) {
          const int lc = min(lr, V - 1);
#pragma unroll
          for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) {
              const float4 b4 = *reinterpret_cast<const float4*>(a.gbias + lc * C + 32 * t + 8 * q4 + 4 * lh);
#pragma unroll
              for (int i = 0; i < FPW; ++i) {
                accf[i][t][4 * q4 + 0] = b4.x;
                accf[i][t][4 * q4 + 1] = b4.y;
                accf[i][t][4 * q4 + 2] = b4.z;
                accf[i][t][4 * q4 + 3] = b4.w;
              }
            }
        }
      }
      if (fa0 < nfr) {
#pragma unroll
        for (int cb = 0; cb < G; ++cb)
#pragma unroll
          for (int p = 0; p < P; ++p) {
            f32x16 c1[FPW];
#pragma unroll
            for (int i = 0; i < FPW; ++i) {
              c1[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fx[i][cb][0], ac[p][0], zero, 0, 0, 0);
              c1[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fx[i][cb][1], ac[p][1], c1[i], 0, 0, 0);
            }
            bf16x8 wf[2][2];
#pragma unroll
            for (int s = 0; s < 2; ++s)
#pragma unroll
              for (int t = 0; t < 2; ++t)
                wf[s][t] = __builtin_bit_cast(
                    bf16x8, *reinterpret_cast<const uint4*>(wl + (t * K16 + (p * G + cb) * 2 + s) * 1024));
#pragma unroll
            for (int i = 0; i < FPW; ++i)
#pragma unroll
              for (int s = 0; s < 2; ++s) {
                bf16x8 xb;
#pragma unroll
                for (int j = 0; j < 8; ++j) xb[j] = (bf16)c1[i][8 * s + j];
#pragma unroll
                for (int t = 0; t < 2; ++t)
                  accf[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[s][t], xb, accf[i][t], 0, 0, 0);
              }
          }
      }
{
        // the frames' LayerNorm statistics over their 64 x V values (lanes lr < V), both frames' wave reductions
        // interleaved; gamma1 / beta1 of this lane's joint and channels loaded once for both frames
        const int lc = min(lr, V - 1);
        const bool jv = lr < V;
        float4 g4[2][4], b4[2][4];
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int q4 = 0; q4 < 4; ++q4) {
            const int co = 32 * t + 8 * q4 + 4 * lh;
            g4[t][q4] = *reinterpret_cast<const float4*>(a.ln1_g + lc * C + co);
            b4[t][q4] = *reinterpret_cast<const float4*>(a.ln1_b + lc * C + co);
          }
        const float cnt = (float)(V * C);
        float mean[FPW], rstd[FPW];
        {  // two-pass statistics on channel pairs (packed adds / FMAs)
          float sum[FPW];
#pragma unroll
          for (int i = 0; i < FPW; ++i) {
            f32x2 s2 = {0.f, 0.f};
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
              for (int r = 0; r < 16; r += 2) s2 += f32x2{accf[i][t][r], accf[i][t][r + 1]};
            sum[i] = jv ? s2.x + s2.y : 0.f;
          }
#pragma unroll
          for (int i = 0; i < FPW; ++i) mean[i] = wave_total(sum[i]) / cnt;
          float sq[FPW];
#pragma unroll
          for (int i = 0; i < FPW; ++i) {
            const f32x2 m2 = {mean[i], mean[i]};
            f32x2 q2 = {0.f, 0.f};
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
              for (int r = 0; r < 16; r += 2) {
                const f32x2 d = f32x2{accf[i][t][r], accf[i][t][r + 1]} - m2;
                q2 = __builtin_elementwise_fma(d, d, q2);
              }
            sq[i] = jv ? q2.x + q2.y : 0.f;
          }
#pragma unroll
          for (int i = 0; i < FPW; ++i) rstd[i] = 1.f / sqrtf(wave_total(sq[i]) / (cnt - 1.f) + 1e-5f);
        }
#pragma unroll
        for (int i = 0; i < FPW; ++i) {
          const int fa = fa0 + NWG * i;
          if (fa >= nfr) continue;
          char* hrow = sH + (fa % RF) * vrs;
          if (!frame_ok(fa)) {  // padding frame: h = 0
            for (int e = lane; e < V * 8; e += 64)
              *reinterpret_cast<uint4*>(hrow + (e >> 3) * RSH + (e & 7) * 16) = make_uint4(0, 0, 0, 0);
            continue;
          }
          if (a.g_out && fa >= HALO && fa < HALO + (R1 - R0)) {
            // training forward: this run's own frames (the halo frames are some other block's) — g rows
            // (pre-LN1, bias included) and the frame's LN1 statistics, for the unfused backward
            const long frow = (long)n * T + (R0 - HALO + fa);
            if (lane == 0) reinterpret_cast<float2*>(a.st1_out)[frow] = make_float2(mean[i], rstd[i]);
            if (jv) {
              bf16* gr = reinterpret_cast<bf16*>(a.g_out) + (frow * V + lr) * a.g_ld + 4 * lh;
#pragma unroll
              for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int q4 = 0; q4 < 4; ++q4) {
                  bf16x4 gv;
#pragma unroll
                  for (int e = 0; e < 4; ++e) gv[e] = (bf16)accf[i][t][4 * q4 + e];
                  *reinterpret_cast<bf16x4*>(gr + 32 * t + 8 * q4) = gv;
                }
            }
          }
          // training forward with h_out: this run's own frames of h also go to HBM (the backward's weight gradient)
          bf16* const hg = (a.h_out && fa >= HALO && fa < HALO + (R1 - R0))
                               ? reinterpret_cast<bf16*>(a.h_out) + (((long)n * T + (R0 - HALO + fa)) * V + lr) * a.h_ld + 4 * lh
                               : nullptr;
          if (jv) {
            // h = relu(fma(fma(g, A, B), gamma, beta)), A = rstd, B = -mean * rstd, on channel pairs
            char* hr = hrow + lr * RSH;
            const f32x2 A2 = {rstd[i], rstd[i]}, B2 = {-mean[i] * rstd[i], -mean[i] * rstd[i]};
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
              for (int q4 = 0; q4 < 4; ++q4) {
                const float4 gg = g4[t][q4], bb = b4[t][q4];
                const f32x2 v01 = {accf[i][t][4 * q4], accf[i][t][4 * q4 + 1]};
                const f32x2 v23 = {accf[i][t][4 * q4 + 2], accf[i][t][4 * q4 + 3]};
                const f32x2 h01 = __builtin_elementwise_fma(__builtin_elementwise_fma(v01, A2, B2), f32x2{gg.x, gg.y},
                                                            f32x2{bb.x, bb.y});
                const f32x2 h23 = __builtin_elementwise_fma(__builtin_elementwise_fma(v23, A2, B2), f32x2{gg.z, gg.w},
                                                            f32x2{bb.z, bb.w});
                bf16x4 hv;
                hv[0] = (bf16)fmaxf(h01.x, 0.f);
                hv[1] = (bf16)fmaxf(h01.y, 0.f);
                hv[2] = (bf16)fmaxf(h23.x, 0.f);
                hv[3] = (bf16)fmaxf(h23.y, 0.f);
                *reinterpret_cast<bf16x4*>(hr + (32 * t + 8 * q4 + 4 * lh) * 2) = hv;
                if (hg) *reinterpret_cast<bf16x4*>(hg + 32 * t + 8 * q4) = hv;
              }
          }
        }
      }
      if (next >= 0) issue(next);
      pa[1] += ptime() - pt1;
    };
    // prologue: frames 0..15 in two batches of 8 (base 0 and 8); then step s produces base 8s + 8
    issue(gw);
    compute(gw, CF + gw);
    compute(CF + gw, nsteps > 1 ? 2 * CF + gw : -1);
    lds_barrier();  // S_0: frames 0..15 ready
    for (int s = 1; s <= nsteps; ++s) {
      // step s: the TCN waves read frames [8s-8, 8s+8); this wave writes frames base = 8s + 8 ..
      if (s < nsteps && !(DBG & 1)) compute(CF * (s + 1) + gw, s + 1 < nsteps ? CF * (s + 2) + gw : -1);
      const long long pb = ptime();
      lds_barrier();  // S_s
      pa[2] += ptime() - pb;
    }
    if constexpr (PROF) prof_out();
    return;
  }

  // =============================== TCN waves: temporal conv ===============================
  const bf16* __restrict__ wt = reinterpret_cast<const bf16*>(a.wt_frag);
  bf16* __restrict__ zg = reinterpret_cast<bf16*>(a.z);
{
    // LayerNorm: frame-aligned row tiles.  TCN wave w = (channel half ct = w & 1, frame group fg = w >> 1) owns
    // row tile i = frame 4fg + i of every step (lane = joint, lanes >= V pad) for its 32 output channels, so a
    // frame's LN2 statistics are one wave reduction per (frame, channel half) plus ONE exchange with the partner
    // wave w ^ 1 (same frames, other channels) through LDS: no 4-wave hand-off and no partials of frames cut by
    // 32-row tiles (the BatchNorm layout's tiles straddle frames: its LN form needed per-tile partials of <= 3
    // frames, a 4-wave arrival counter and a combine, ~40 % of the role's cycles).  256 MFMA rows per 200 output
    // rows instead of 224; one weight fragment per k-step as in the BatchNorm layout (both channel halves per
    // wave doubled the per-CU vector-memory traffic of the weight stream and measured slower).
    const int ct = wave & 1, fg = wave >> 1;
    const int jw = min(lr, V - 1);
    const bool jv = lr < V;
    const int hw = jw * RSH + lh * 16;
    const int wl = ct * 4 * 512 + lane * 8;  // 1-KiB block [dt][ct][ks] of the [9][2][4] image
    int wcur = wl;
    auto load_w = [&](int k) {
      const int dt = k >> 2, ks = k & 3;
      int o = wcur + dt * 8 * 512;
      asm volatile("" : "+v"(o));
      return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(wt + o + ks * 512));
    };
    static_assert(KSTEPS % NB == 0, "the weight ring runs on across steps");
    bf16x8 fw[NB];
#pragma unroll
    for (int k = 0; k < (DBG & 32 ? NB : NB - 1); ++k) fw[k] = load_w(k);
    const f32x16 zero = {};
    // statistics shifted by the pivot mean_c(bias) (the same constant in every wave), so a large common bias
    // does not cancel catastrophically in sum(z^2) - sum(z) * mean
    const float piv = wave_total(sTb[lane]) * (1.f / C);
    const float cnt = (float)(V * C);
    float2* const myPart = sPart + wave * 4;
    const float2* const pePart = sPart + (wave ^ 1) * 4;
    lds_barrier();  // S_0
    for (int s = 1; s <= nsteps; ++s) {
      wcur = wl;
      asm volatile("" : "+v"(wcur));
      const int f0 = R0 + CF * (s - 1);      // first output frame of the step
      const int base = (CF * (s - 1)) % RF;  // ring slot of run frame 8(s-1) (= output frame f0 - 4)
      int q_[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) q_[i] = base + 4 * fg + i;
      auto hoff = [&](int i, int dt) {
        const int sl = q_[i] + dt;
        return (sl >= RF ? sl - RF : sl) * vrs + hw;
      };
      f32x16 acc[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = zero;
      bf16x8 fb[3][4];
      int ad[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        ad[i] = hoff(i, 0);
        asm volatile("" : "+v"(ad[i]));
        fb[0][i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(sH + ad[i]));
        fb[1][i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(sH + ad[i] + 32));
        if (DBG & 64) fb[2][i] = fb[0][i];
      }
      const long long pk0 = ptime();
      static_for<KSTEPS>([&]<int k>() {
        if constexpr (!(DBG & 32)) fw[(k + NB - 1) % NB] = load_w((k + NB - 1) % KSTEPS);  // runs into the next step
        if constexpr (k + 2 < KSTEPS && !(DBG & 64)) {
          constexpr int dt2 = (k + 2) >> 2, ks2 = (k + 2) & 3;
          if constexpr (ks2 == 0) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              ad[i] = hoff(i, dt2);
              asm volatile("" : "+v"(ad[i]));
            }
          }
#pragma unroll
          for (int i = 0; i < 4; ++i)
            fb[(k + 2) % 3][i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(sH + ad[i] + ks2 * 32));
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw[k % NB], fb[k % 3][i], acc[i], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      });
      const long long pk1 = ptime();
      pa[0] += pk1 - pk0;
      // epilogue: acc[i][q] = out^T[co = 32ct + 8(q>>2) + 4lh + (q&3)][frame 4fg+i, joint lr]
      const int nfv = min(CF, R1 - f0);  // frames of the step inside the run
      bf16* zt = zg + ((long)n * T + f0) * V * a.z_ld;
      // the residual rows first: their L2 latency runs under the statistics
      const bf16* xres = reinterpret_cast<const bf16*>(a.x) + ((long)n * T + f0) * V * a.x_ld;
      bf16x4 rv[4][4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int fo = 4 * fg + i;
        const bool ok = jv && fo < nfv && a.residual && !(DBG & 4);
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
          const bf16x4 zr = {};
          rv[i][q4] = ok ? *reinterpret_cast<const bf16x4*>(xres + (long)(fo * V + lr) * a.x_ld + 32 * ct + 8 * q4 + 4 * lh)
                         : zr;
        }
      }
      // d = z - piv (bias added); each frame's (sum, sum of squares) of d over this wave's 32 x V values
      float tb[16];
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) {
        const float4 b4 = *reinterpret_cast<const float4*>(sTb + 32 * ct + 8 * q4 + 4 * lh);
        tb[4 * q4] = b4.x - piv;
        tb[4 * q4 + 1] = b4.y - piv;
        tb[4 * q4 + 2] = b4.z - piv;
        tb[4 * q4 + 3] = b4.w - piv;
      }
      // (vector forms: the fp32 adds / FMAs issue as packed 2-wide VALU ops)
      f32x16 tbv;
#pragma unroll
      for (int q = 0; q < 16; ++q) tbv[q] = tb[q];
      float ts[4], tq[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        acc[i] += tbv;
        f32x2 su = {0.f, 0.f}, sq = {0.f, 0.f};
#pragma unroll
        for (int q = 0; q < 16; q += 2) {
          const f32x2 d = {acc[i][q], acc[i][q + 1]};
          su += d;
          sq = __builtin_elementwise_fma(d, d, sq);
        }
        const bool ok = jv && 4 * fg + i < nfv;
        ts[i] = ok ? su.x + su.y : 0.f;
        tq[i] = ok ? sq.x + sq.y : 0.f;
      }
      if (!(DBG & 8)) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          ts[i] = wave_total(ts[i]);
          tq[i] = wave_total(tq[i]);
        }
      }
      // exchange with the partner wave (same frames, other 32 channels): post, then wait for its post of this
      // step.  The partner's slot is rewritten only after the step's closing barrier, which follows this read.
      if (lane == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) myPart[i] = make_float2(ts[i], tq[i]);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const long long pl0 = ptime();
      pa[1] += pl0 - pk1;
      if (lane == 0) __hip_atomic_store(sCnt + wave, (unsigned)s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      while (__hip_atomic_load(sCnt + (wave ^ 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < (unsigned)s)
        __builtin_amdgcn_s_sleep(1);
      const long long pl1 = ptime();
      pa[5] += pl1 - pl0;
      float dmean[4], rstd[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float2 p = pePart[i];
        const float su = ts[i] + p.x, sq = tq[i] + p.y;  // a + b == b + a: both waves get identical totals
        dmean[i] = su / cnt;
        rstd[i] = 1.f / sqrtf(fmaxf(sq - su * dmean[i], 0.f) / (cnt - 1.f) + 1e-5f);
      }
      // 16-B stores: a lane holds 4 channels of each 8-channel group; one v_permlane32_swap per dword gives lanes
      // 0-31 group 2p and lanes 32-63 group 2p + 1 whole (jv is the same for lanes lr and lr + 32)
      auto store_swapped = [&](bf16* row, unsigned (&pk)[4][2]) {
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
          for (int d = 0; d < 2; ++d) {
            const auto sw = __builtin_amdgcn_permlane32_swap(pk[2 * p][d], pk[2 * p + 1][d], false, false);
            pk[2 * p][d] = sw[0];
            pk[2 * p + 1][d] = sw[1];
          }
        if (jv) {
#pragma unroll
          for (int p = 0; p < 2; ++p)
            *reinterpret_cast<uint4*>(row + 32 * ct + 16 * p + 8 * lh) =
                make_uint4(pk[2 * p][0], pk[2 * p][1], pk[2 * p + 1][0], pk[2 * p + 1][1]);
        }
      };
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int fo = 4 * fg + i;
        if (fo >= nfv) continue;
        const int r = fo * V + min(lr, V - 1);
        if (a.u_out) {  // training forward: u = z (pre-LN2, bias included) rows and the frame's LN2 statistics
          bf16* ur = reinterpret_cast<bf16*>(a.u_out) + (((long)n * T + f0) * V + r) * a.u_ld;
          unsigned pk[4][2];
#pragma unroll
          for (int q4 = 0; q4 < 4; ++q4) {
            bf16x4 uv;
#pragma unroll
            for (int e = 0; e < 4; ++e) uv[e] = (bf16)(acc[i][4 * q4 + e] + piv);
            const u32x2n w2 = __builtin_bit_cast(u32x2n, uv);
            pk[q4][0] = w2.x;
            pk[q4][1] = w2.y;
          }
          store_swapped(ur, pk);
          if (ct == 0 && lane == 0)
            reinterpret_cast<float2*>(a.st2_out)[(long)n * T + f0 + fo] = make_float2(piv + dmean[i], rstd[i]);
        }
        // y = relu(((d - dmean) * rstd) * gamma + beta + x) as relu(fma(fma(d, A, B), gamma, beta) + x), A = rstd,
        // B = -dmean * rstd, on pairs of channels (packed FMAs)
        const f32x2 A2 = {rstd[i], rstd[i]}, B2 = {-dmean[i] * rstd[i], -dmean[i] * rstd[i]};
        unsigned pk[4][2];
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
          const int co = 32 * ct + 8 * q4 + 4 * lh;
          const float4 g4 = *reinterpret_cast<const float4*>(sGam + jw * CGP + co);
          const float4 b4 = *reinterpret_cast<const float4*>(sBet + jw * CGP + co);
          const f32x2 g01 = {g4.x, g4.y}, g23 = {g4.z, g4.w}, b01 = {b4.x, b4.y}, b23 = {b4.z, b4.w};
          const f32x2 r01 = {(float)rv[i][q4][0], (float)rv[i][q4][1]}, r23 = {(float)rv[i][q4][2], (float)rv[i][q4][3]};
          const f32x2 d01 = {acc[i][4 * q4], acc[i][4 * q4 + 1]}, d23 = {acc[i][4 * q4 + 2], acc[i][4 * q4 + 3]};
          f32x2 t01 = __builtin_elementwise_fma(__builtin_elementwise_fma(d01, A2, B2), g01, b01) + r01;
          f32x2 t23 = __builtin_elementwise_fma(__builtin_elementwise_fma(d23, A2, B2), g23, b23) + r23;
          bf16x4 o;
          o[0] = (bf16)fmaxf(t01.x, 0.f);
          o[1] = (bf16)fmaxf(t01.y, 0.f);
          o[2] = (bf16)fmaxf(t23.x, 0.f);
          o[3] = (bf16)fmaxf(t23.y, 0.f);
          const u32x2n w2 = __builtin_bit_cast(u32x2n, o);
          pk[q4][0] = w2.x;
          pk[q4][1] = w2.y;
        }
        store_swapped(zt + (long)r * a.z_ld, pk);
      }
      const long long pl2 = ptime();
      pa[4] += pl2 - pl1;
      lds_barrier();  // S_s: the GCN waves may overwrite the frames this step read
      pa[2] += ptime() - pl2;
    }
    if constexpr (PROF) prof_out();
    return;
  }
}

FGeom plan(int N, int T) {
  FGeom g{};
  int per = TARGET_BLOCKS / (N > 0 ? N : 1);
  if (per < 1) per = 1;
  const int span = (T + per - 1) / per;
  g.run = (span + CF - 1) / CF * CF;
  g.runs_n = (T + g.run - 1) / g.run;
  g.nsm = g.run / CF;
  return g;
}

}  // namespace

// PROF builds: copy the per-wave cycle accounts [block][8 waves][6] (long long; GCN: DMA wait, compute, barrier,
// total; TCN: k-loop, LN2 statistics, barrier, total, normalise + stores, partner hand-off) to host memory; -1 in the
// shipped library
extern "C" int stgcn_fused_prof(void* dst, long n) {
  if (!PROF) return -1;
  if (n > (long)PROF_BLOCKS * 8 * 6) n = (long)PROF_BLOCKS * 8 * 6;
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_fused_prof), n * sizeof(long long), 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}

int layer_fused_launch(const stgcn_layer_fused_desc& a, hipStream_t s) {
  if (!a.z || !a.wt_frag || !a.x || !a.wg_frag || !a.A || !a.ln1_g || !a.ln1_b || !a.ln2_g || !a.ln2_b)
    return STGCN_EBADSHAPE;
  const int ntrain = !!a.g_out + !!a.u_out + !!a.st1_out + !!a.st2_out;
  if (ntrain != 0 && (ntrain != 4 || a.g_ld < C || a.g_ld % 4 || a.u_ld < C || a.u_ld % 8)) return STGCN_EBADSHAPE;
  if (a.h_out && (ntrain != 4 || a.h_ld < C || a.h_ld % 4)) return STGCN_EBADSHAPE;
  if (a.N < 1 || a.T < 1 || a.V <= 16 || a.V > VMAX || a.P < 1 || a.P > 3) return STGCN_EBADSHAPE;
  if (a.x_ld < C || a.x_ld % 8 || a.z_ld < C || a.z_ld % 8) return STGCN_EBADSHAPE;
  FGeom g = plan(a.N, a.T);
  const long nblk = (long)a.N * g.runs_n;
  if (nblk > 0x7fffffffL) return STGCN_EBADSHAPE;
  const int K16 = a.P * G * 2;
  g.off_tab = 2 * K16 * 1024;
  g.off_ring = g.off_tab + (2 * a.V * CGP * 4 + C * 4 + 255) / 256 * 256;
  g.off_h = g.off_ring + NWG * SLOTS * PANEL;
  g.off_red = g.off_h + (RF * a.V * RSH + 255) / 256 * 256;
  const size_t lds = (size_t)g.off_red + NWT * 4 * 8 + NWT * 4;
  if (lds > (size_t)LDS_MAX) return STGCN_EBADSHAPE;
  typedef void (*KFn)(const stgcn_layer_fused_desc, const FGeom);
  static const KFn tab[3] = {layer_fused_kernel<1>, layer_fused_kernel<2>, layer_fused_kernel<3>};
  const KFn k = tab[a.P - 1];
  if (stgcn_lds_attr((const void*)k, LDS_MAX, s)) return STGCN_EHIP;
  hipLaunchKernelGGL(k, dim3((unsigned)nblk), dim3(NW * 64), lds, s, a, g);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
