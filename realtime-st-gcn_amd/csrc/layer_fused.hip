// The fused ST-GCN layer forward (BASELINE north_star): ConvTemporalGraphical (tgcn.py:58-79) -> BN1 ->
// ReLU -> temporal Conv2d (Kt = 9) + bias (stgcn.py:151-159) in ONE kernel, with the graph-conv output
// g and its normalised form h = relu(BN1(g)) living only in LDS.  The second BatchNorm's batch
// statistics are emitted as per-tile partials (the consumer folds BN2 + residual + ReLU, stgcn.py:160,193).
//
// BatchNorm needs global statistics of g before the temporal conv can consume h, so the layer is the
// two-pass form of SURVEY §7: pass 1 = the fused graph conv with statistics only (gcn_tile.hip, no output
// stores), bn_finalize -> BN1 scale/shift; pass 2 = this kernel, which RECOMPUTES the graph conv of its
// tile (plus the temporal halo) on the matrix cores instead of reading g back from HBM.
//
// Shapes: bf16, Cin = Cout = 64, stride 1, Kt = 9 (pad 4), P <= 3 partitions, 16 < V <= 25 — the
// north_star layer (N = 64, C = 64, T = 300, V = 25) and config 2's layers 0-2.
//
// Block = 4 waves, persistent over contiguous runs of tiles; tile = CF = 16 output frames of one sample.
//   phase 1 (graph conv, per frame; gcn_tile.hip's two chained MFMA products): the HF = 24 frames
//     [f0 - 4, f0 + 20) are split over the waves (6 each).  A frame's x rows arrive as two 32-channel
//     panels [32 joint rows][32 ch] by global->LDS DMA into a per-wave ring (DP panels in flight); stage 1
//     mixes the joints (X^T A_p on MFMA, X^T by transposing LDS reads, A_p in registers), stage 2 runs the
//     1x1 conv from the stage-1 accumulators (W' in LDS).  Epilogue: h = relu(g * s1 + (bias2d * s1 + b1))
//     (BN1 folded; s1/b1 from pass 1) -> bf16 -> LDS rows [frame][joint][64 ch] (144-B rows).  Frames
//     outside [0, T) are written as zeros: the temporal conv's zero padding applies to h.
//   phase 2 (temporal conv): out^T[co][row] = sum_{dt,ci} W[dt][co][ci] h[row + dt*V][ci] over the tile's
//     CF*V rows (flattened (frame, joint) rows: tap dt is a row offset of dt*V), 32x32x16 MFMAs with the
//     weight fragments streamed from L2 (conv_wide.hip's fragment image) through a register ring and the
//     h fragments read from LDS.  Wave = (32-channel half, row half: 7 row tiles of 32).  Epilogue: + bias,
//     8-B stores of 4 consecutive channels per lane, BN2 (count, mean, M2) partials per (tile, channel).
#include "common.h"
#include "../../include/stgcn_amd.h"
#include <utility>

namespace {

constexpr int NW = 4;
constexpr int C = 64, G = C / 32;      // channels (in = out), 32-channel blocks
constexpr int HALO = 4, KT = 9;
constexpr int CF = 16, HF = CF + 2 * HALO;
constexpr int KF = HF / NW;            // h frames per wave in phase 1
constexpr int RSH = 2 * C + 16;        // h row bytes (144: conflict-free ds_read_b128 for any row offset)
constexpr int PANEL = 32 * 64;         // [32 joint rows][32 ch] bf16
constexpr int DP = 4;                  // panels in flight per wave
constexpr int RT_MAX = 7;              // 32-row output tiles per wave (two row halves: 13 tiles at V = 25)
constexpr int NB = 6;                  // temporal-conv weight fragment ring depth
constexpr int KSTEPS = KT * C / 16;    // 36 k-steps of the temporal conv
constexpr int VMAX = 25;
constexpr int LDS_MAX = 160 * 1024;
static_assert(HF % NW == 0, "frames per wave");

template <int N, typename F>
DEV void static_for(F&& f) {
  [&]<int... I>(std::integer_sequence<int, I...>) { (f.template operator()<I>(), ...); }(
      std::make_integer_sequence<int, N>{});
}

typedef short s16x4 __attribute__((ext_vector_type(4)));
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
DEV unsigned lds_u32(const void* p) { return (unsigned)(size_t)(const __attribute__((address_space(3))) char*)p; }

// wait until at most n of this wave's vector-memory ops are outstanding (n wave-uniform; rounded down)
DEV void vm_wait(int n) {
  if (n >= 6)
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if (n >= 4)
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (n >= 2)
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

struct FGeom {
  int tiles_n;  // tiles per sample
  int ntiles;   // N * tiles_n
  int tpb;      // contiguous tiles per block
  int nrt;      // 32-row output tiles per tile (ceil(CF * V / 32))
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
  const int t_first = blockIdx.x * g.tpb;
  const int t_last = min(g.ntiles, t_first + g.tpb);
  if (t_first >= t_last) return;  // block-uniform, before any barrier

  char* const sW = smem;                                        // [2][K16] 1-KiB W' fragment blocks
  float* const sSc = reinterpret_cast<float*>(smem + g.off_tab);  // [64] BN1 scale
  float* const sBp = sSc + C;                                   // [V][64] bias2d * scale + shift
  char* const sRing = smem + g.off_ring + wave * DP * PANEL;
  char* const sH = smem + g.off_h;                              // [HF * V][RSH]
  float2* const sRed = reinterpret_cast<float2*>(smem + g.off_red);  // [2][64] (sum, sum of squares)

  // ---- per block: W' slice, BN1 tables, zeroed panel rings (rows V..31 stay zero), stage-1 A operands
  {
    const uint4* wsrc = reinterpret_cast<const uint4*>(a.wg_frag);
    uint4* wdst = reinterpret_cast<uint4*>(sW);
    for (int e = tid; e < 2 * K16 * 64; e += NW * 64) wdst[e] = wsrc[e];
    for (int c = tid; c < C; c += NW * 64) sSc[c] = a.n1_scale[c];
    for (int e = tid; e < V * C; e += NW * 64) {
      const int c = e % C;
      const float b = a.gbias ? a.gbias[e] : 0.f;
      sBp[e] = fmaf(b, a.n1_scale[c], a.n1_shift[c]);
    }
    uint4* z = reinterpret_cast<uint4*>(smem + g.off_ring);
    for (int e = tid; e < NW * DP * PANEL / 16; e += NW * 64) z[e] = make_uint4(0, 0, 0, 0);
  }
  // B[k = input joint u][n = output joint o] = A[p][u][o]
  bf16x8 ac[P][2];
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
  __syncthreads();

  const bf16* __restrict__ xg = reinterpret_cast<const bf16*>(a.x);
  const bf16* __restrict__ wt = reinterpret_cast<const bf16*>(a.wt_frag);
  bf16* __restrict__ zg = reinterpret_cast<bf16*>(a.z);
  const int lrow = lane >> 2, lunit = lane & 3;
  const bool row2 = lrow + 16 < V;
  const unsigned ring0 = lds_u32(sRing);
  const f32x16 zero = {};
  const char* const wl = sW + lane * 16;
  const int vrs = V * RSH;  // bytes per h frame

  for (int tile = t_first; tile < t_last; ++tile) {
    const int n = tile / g.tiles_n;
    const int f0 = (tile - n * g.tiles_n) * CF;
    const int cfv = min(CF, T - f0);

    // ================= phase 1: h = relu(BN1(graph conv)) for frames f0 - 4 .. f0 + 19 =================
    // this wave's frames fl = wave + NW*k (k < KF); valid (inside [0, T)) for k in [k0, k1)
    const int lo = max(0, HALO - f0), hi = min(HF, T - f0 + HALO);
    const int k0 = lo > wave ? (lo - wave + NW - 1) / NW : 0;
    const int k1 = min(KF, hi > wave ? (hi - wave + NW - 1) / NW : 0);
    for (int k = 0; k < KF; ++k) {  // zero rows of the padding frames
      if (k >= k0 && k < k1) continue;
      char* fr = sH + (wave + NW * k) * vrs;
      for (int e = lane; e < V * 8; e += 64)
        *reinterpret_cast<uint4*>(fr + (e >> 3) * RSH + (e & 7) * 16) = make_uint4(0, 0, 0, 0);
    }
    const int npv = 2 * max(0, k1 - k0);
    const bf16* src0 = xg + ((long)n * T + (f0 - HALO + wave + NW * k0)) * V * a.x_ld + (long)lrow * a.x_ld + lunit * 8;
    const long fstep = (long)NW * V * a.x_ld;
    auto issue = [&](int q) {  // panel q = (valid frame q/2, channel block q%2) -> ring slot q % DP
      const bf16* src = src0 + (q >> 1) * fstep + (q & 1) * 32;
      const unsigned dst = ring0 + (unsigned)((q % DP) * PANEL);
      glds16(src, dst);
      if (row2) glds16(src + 16L * a.x_ld, dst + 1024);
    };
    for (int q = 0; q < min(DP, npv); ++q) issue(q);
    for (int vk = 0; vk < k1 - k0; ++vk) {
      f32x16 acc[2];
      acc[0] = zero;
      acc[1] = zero;
#pragma unroll
      for (int cb = 0; cb < G; ++cb) {
        const int q = 2 * vk + cb;
        vm_wait(2 * min(DP - 1, npv - 1 - q));  // panel q landed (later panels may still be in flight)
        const char* pan = sRing + (q % DP) * PANEL;
        const bf16x8 fx0 = trfrag(pan, 0, lane);
        const bf16x8 fx1 = trfrag(pan, 16, lane);
        f32x16 c1[P];
#pragma unroll
        for (int p = 0; p < P; ++p) {
          c1[p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fx0, ac[p][0], zero, 0, 0, 0);
          c1[p] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fx1, ac[p][1], c1[p], 0, 0, 0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slot's reads retired: refill it
        if (q + DP < npv) issue(q + DP);
        bf16x8 wf[P][2][2];
#pragma unroll
        for (int p = 0; p < P; ++p)
#pragma unroll
          for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int t = 0; t < 2; ++t)
              wf[p][s][t] = __builtin_bit_cast(
                  bf16x8, *reinterpret_cast<const uint4*>(wl + (t * K16 + (p * G + cb) * 2 + s) * 1024));
#pragma unroll
        for (int p = 0; p < P; ++p)
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            bf16x8 xb;
#pragma unroll
            for (int j = 0; j < 8; ++j) xb[j] = (bf16)c1[p][8 * s + j];
#pragma unroll
            for (int t = 0; t < 2; ++t)
              acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[p][s][t], xb, acc[t], 0, 0, 0);
          }
      }
      // epilogue: lane = joint lr, acc[t][r] = g^T[co = 32t + 8(r>>2) + 4lh + (r&3)][lr]
      if (lr < V) {
        const int fl = wave + NW * (k0 + vk);
        char* hrow = sH + (fl * V + lr) * RSH;
        const float* bp = sBp + lr * C;
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int q4 = 0; q4 < 4; ++q4) {
            const int co = 32 * t + 8 * q4 + 4 * lh;
            const float4 s4 = *reinterpret_cast<const float4*>(sSc + co);
            const float4 b4 = *reinterpret_cast<const float4*>(bp + co);
            bf16x4 hv;
            hv[0] = (bf16)fmaxf(fmaf(acc[t][4 * q4 + 0], s4.x, b4.x), 0.f);
            hv[1] = (bf16)fmaxf(fmaf(acc[t][4 * q4 + 1], s4.y, b4.y), 0.f);
            hv[2] = (bf16)fmaxf(fmaf(acc[t][4 * q4 + 2], s4.z, b4.z), 0.f);
            hv[3] = (bf16)fmaxf(fmaf(acc[t][4 * q4 + 3], s4.w, b4.w), 0.f);
            *reinterpret_cast<bf16x4*>(hrow + co * 2) = hv;
          }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    // ================= phase 2: temporal conv over the tile's CF*V rows =================
    const int ct = wave & 1, rh = wave >> 1;
    const int rows = CF * V;  // rows of a full tile (a short last tile reads zero h frames, never stored)
    int hoff[RT_MAX];
#pragma unroll
    for (int i = 0; i < RT_MAX; ++i) {
      const int r = (rh * RT_MAX + i) * 32 + lr;
      hoff[i] = (r < rows ? r : 0) * RSH + lh * 16;
    }
    f32x16 acc2[RT_MAX];
#pragma unroll
    for (int i = 0; i < RT_MAX; ++i) acc2[i] = zero;
    // A fragment (weights) of k-step s = (dt, ks): 1-KiB block [dt][ct][ks] of the [9][2][4] image
    const bf16* wlane = wt + ct * 4 * 512 + lane * 8;
    bf16x8 fw[NB];
    auto load_w = [&](int s) {
      const int dt = s >> 2, ks = s & 3;
      return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(wlane + (dt * 8 + ks) * 512));
    };
#pragma unroll
    for (int s = 0; s < NB - 1; ++s) fw[s] = load_w(s);
    bf16x8 fb[2][RT_MAX];
#pragma unroll
    for (int i = 0; i < RT_MAX; ++i) fb[0][i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(sH + hoff[i]));
    static_for<KSTEPS>([&]<int s>() {
      constexpr int dt = s >> 2, ks = s & 3;
      if constexpr (s + NB - 1 < KSTEPS) fw[(s + NB - 1) % NB] = load_w(s + NB - 1);
      if constexpr (s + 1 < KSTEPS) {
        constexpr int dt1 = (s + 1) >> 2, ks1 = (s + 1) & 3;
        const int off = dt1 * vrs + ks1 * 32;
#pragma unroll
        for (int i = 0; i < RT_MAX; ++i)
          fb[(s + 1) & 1][i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(sH + hoff[i] + off));
      }
      (void)dt;
      (void)ks;
#pragma unroll
      for (int i = 0; i < RT_MAX; ++i)
        acc2[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fw[s % NB], fb[s & 1][i], acc2[i], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    });
    // epilogue: acc2[i][r] = out^T[co = 32ct + 8(r>>2) + 4lh + (r&3)][row (rh*7 + i)*32 + lr]
    float s1[16], s2[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) s1[r] = s2[r] = 0.f;
    float tb[16];
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      const int co = 32 * ct + 8 * q4 + 4 * lh;
      const float4 b4 = a.tbias ? *reinterpret_cast<const float4*>(a.tbias + co) : make_float4(0.f, 0.f, 0.f, 0.f);
      tb[4 * q4] = b4.x;
      tb[4 * q4 + 1] = b4.y;
      tb[4 * q4 + 2] = b4.z;
      tb[4 * q4 + 3] = b4.w;
    }
    const int vrows = cfv * V;
    bf16* zt = zg + ((long)n * T + f0) * V * a.z_ld;
#pragma unroll
    for (int i = 0; i < RT_MAX; ++i) {
      const int r = (rh * RT_MAX + i) * 32 + lr;
      if (r < vrows) {
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
          bf16x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float v = acc2[i][4 * q4 + e];
            s1[4 * q4 + e] += v;
            s2[4 * q4 + e] = fmaf(v, v, s2[4 * q4 + e]);
            o[e] = (bf16)(v + tb[4 * q4 + e]);
          }
          *reinterpret_cast<bf16x4*>(zt + (long)r * a.z_ld + 32 * ct + 8 * q4 + 4 * lh) = o;
        }
      }
    }
    if (a.stats) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
#pragma unroll
        for (int o = 1; o < 32; o <<= 1) {
          s1[r] += __shfl_xor(s1[r], o);
          s2[r] += __shfl_xor(s2[r], o);
        }
      }
      if (lr == 0) {
#pragma unroll
        for (int r = 0; r < 16; ++r) sRed[rh * C + 32 * ct + 8 * (r >> 2) + 4 * lh + (r & 3)] = make_float2(s1[r], s2[r]);
      }
      __syncthreads();
      if (tid < C) {
        const float2 u0 = sRed[tid], u1 = sRed[C + tid];
        const float t1 = u0.x + u1.x, t2 = u0.y + u1.y;
        const float cnt = (float)vrows;
        const float mu = t1 / cnt;
        const float b = a.tbias ? a.tbias[tid] : 0.f;
        reinterpret_cast<float4*>(a.stats)[(long)tile * C + tid] = make_float4(cnt, b + mu, fmaxf(t2 - t1 * mu, 0.f), 0.f);
      }
    }
    __syncthreads();  // sH / sRed are rewritten by the next tile
  }
}

}  // namespace

long layer_fused_row_blocks(int N, int T) { return (long)N * ((T + CF - 1) / CF); }

int layer_fused_launch(const stgcn_layer_fused_desc& a, hipStream_t s) {
  if (!a.x || !a.z || !a.wg_frag || !a.A || !a.n1_scale || !a.n1_shift || !a.wt_frag) return STGCN_EBADSHAPE;
  if (a.N < 1 || a.T < 1 || a.V <= 16 || a.V > VMAX || a.P < 1 || a.P > 3) return STGCN_EBADSHAPE;
  if (a.x_ld < C || a.x_ld % 8 || a.z_ld < C || a.z_ld % 4) return STGCN_EBADSHAPE;
  FGeom g{};
  g.tiles_n = (a.T + CF - 1) / CF;
  const long nt = (long)a.N * g.tiles_n;
  if (nt > 0x7fffffffL) return STGCN_EBADSHAPE;
  g.ntiles = (int)nt;
  g.nrt = (CF * a.V + 31) / 32;
  if (g.nrt > 2 * RT_MAX) return STGCN_EBADSHAPE;
  const int K16 = a.P * G * 2;
  g.off_tab = 2 * K16 * 1024;
  g.off_ring = g.off_tab + ((C + a.V * C) * 4 + 255) / 256 * 256;
  g.off_h = g.off_ring + NW * DP * PANEL;
  g.off_red = g.off_h + (HF * a.V * RSH + 255) / 256 * 256;
  const size_t lds = (size_t)g.off_red + 2 * C * 8;
  if (lds > (size_t)LDS_MAX) return STGCN_EBADSHAPE;
  const int ncu = stgcn_cu_count(s);
  g.tpb = (g.ntiles + ncu - 1) / ncu;
  const int grid = (g.ntiles + g.tpb - 1) / g.tpb;
  typedef void (*KFn)(const stgcn_layer_fused_desc, const FGeom);
  static const KFn tab[3] = {layer_fused_kernel<1>, layer_fused_kernel<2>, layer_fused_kernel<3>};
  const KFn k = tab[a.P - 1];
  if (stgcn_lds_attr((const void*)k, LDS_MAX, s)) return STGCN_EHIP;
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(NW * 64), lds, s, a, g);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
