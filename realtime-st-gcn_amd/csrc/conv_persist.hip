// Persistent, weight-resident temporal conv for the 64-channel layers (bf16) — the config-2
// layers 1-3 shape (tcn.2 of stgcn.py:154-159: Conv2d(64, 64, (9,1), pad (4,0)) on relu(BN1(g)),
// and its data gradient).
//
// Why: at C = 64 the K axis is only Kt*64 = 576 deep, so the frame-tiled kernel (conv_tile.hip)
// spends more time fetching the 74 KB weight tile into every block and waiting on each short
// K-chunk than in MFMA, and its VALU work (prologue, epilogue) runs in lock-step with the MFMAs
// of the same waves.  Here one block per CU
//   * loads the whole packed weight [9][64 co][64 ci] into LDS once (LDS-DMA, XOR-swizzled 128-B
//     rows, conflict-free ds_read_b128),
//   * walks a contiguous range of F-frame tiles (F = floor(128/V): 5 frames at V = 25) through a
//     ring of RS = 2F+8 frame slots in LDS (rows padded to 144 B): a tile reads frames
//     f0-4 .. f0+F+3 and only the F newest are not in the ring already — each frame is fetched and
//     transformed (BN1+ReLU prologue; zero padding outside [0,T)) once per block,
//   * splits its 8 waves into two groups of 4 that alternate roles every phase: group (k & 1)
//     computes tile k (4 waves x 64 rows x 32 cols, 72 MFMAs each) while the other group runs the
//     epilogue of tile k-1 (bias, bf16 store, BatchNorm Welford partials), writes tile k+1's new
//     frames into the ring from registers and issues the global loads for tile k+3.  Waves w and
//     w+4 share a SIMD, so every SIMD always has one MFMA wave and one VALU/memory wave,
//   * tap dt reads frame slot (f0 + fl + q(dt)) mod RS, q = dt (fwd) or 8 - dt (transposed = data
//     gradient); a tile that starts a new sample is staged in an extra synchronous phase.
#include "common.h"
#include "../../include/stgcn_amd.h"
#include <stdlib.h>

namespace {

constexpr int KT = 9;
constexpr int PADT = (KT - 1) / 2;
constexpr int C = 64;                  // Cin_pad = Cout_pad = 64
constexpr int RB = C * 2;              // bytes per weight row (bf16)
constexpr int RS_A = RB + 16;          // bytes per activation row in the ring (padded)
constexpr int NWAVE = 8, NT = NWAVE * 64, GT = NT / 2;  // two groups of 4 waves
constexpr int ROWS = 128;              // MFMA rows per tile (2 row groups x 64)
constexpr int TM = 2;                  // 32-row MFMA tiles per wave
constexpr int B_BYTES = KT * C * RB;   // 73 728
constexpr int LDS_MAX = 160 * 1024;
constexpr int RA = ROWS * 8 / GT;      // steady-state units per thread of a group: F*V <= 128 rows -> 4

DEV int swz(int row) { return (row >> 1) & 7; }  // weight rows: 2 rows per 256-B bank row

DEV void glds16(const void* src, char* lds_base) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
#endif
}

struct PGeom {
  int F;        // frames per tile
  int RSL;      // ring slots (frames)
  int tiles_n;  // tiles per sample
  int ntiles;   // total tiles
  int tpb;      // tiles per block
};

__global__ __launch_bounds__(NT, 1) void conv_persist_kernel(const stgcn_conv_desc a, const PGeom g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sB = smem;
  char* sR = smem + B_BYTES;  // ring: slot s, joint v at (s*V + v) * RS_A

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int grp = wave >> 2, gw = wave & 3, gtid = tid & (GT - 1);
  const int wr = gw & 1, wc = gw >> 1;  // rows [64 wr, +64) x cols [32 wc, +32)
  const int lr = lane & 31, lh = lane >> 5;
  const int V = a.V;
  const int t_begin = blockIdx.x * g.tpb;
  const int K = min(g.ntiles, t_begin + g.tpb) - t_begin;
  if (K <= 0) return;

  const bf16* __restrict__ in = reinterpret_cast<const bf16*>(a.in);
  const bf16* __restrict__ wp = reinterpret_cast<const bf16*>(a.w);

  // ---- all weights -> LDS once (72 LDS-DMA pieces, 9 per wave), XOR swizzle on the source
  for (int piece = wave; piece < B_BYTES / 1024; piece += NWAVE) {
    const int byte = piece * 1024 + lane * 16;
    const int br = byte / RB, pu = (byte % RB) >> 4;  // br = dt*64 + co
    const int dt = br >> 6, co = br & 63;
    glds16(wp + ((long)dt * a.Cout_pad + co) * a.Cin_pad + (pu ^ swz(br)) * 8, sB + piece * 1024);
  }
  float* s_aff = reinterpret_cast<float*>(sR + g.RSL * V * RS_A);  // [2][64] BN1 scale / shift
  if (tid < 2 * C) s_aff[tid] = a.pro == 1 ? (tid < C ? a.pro_a[tid] : a.pro_b[tid - C]) : (tid < C ? 1.f : 0.f);

  // ---- staging helpers; a unit = 16 B (8 channels) of one joint row of one frame
  const int ucol = tid & 7;
  auto transform = [&](uint4 v) -> uint4 {
    if (a.pro != 1) return v;
    const float4* sa = reinterpret_cast<const float4*>(s_aff + ucol * 8);
    const float4* sb = reinterpret_cast<const float4*>(s_aff + C + ucol * 8);
    const float4 a0 = sa[0], a1 = sa[1], b0 = sb[0], b1 = sb[1];
    const float sc[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
    const float sh[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
    float f[8];
    unpack16(v, f, (bf16*)nullptr);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], sc[j], sh[j]), 0.f);
    return pack16(f, (bf16*)nullptr);
  };
  auto put = [&](uint4 v, int f, int vj) {  // frame f -> ring slot (f + PADT) mod RS
    const int slot = (f + PADT) % g.RSL;
    *reinterpret_cast<uint4*>(sR + (slot * V + vj) * RS_A + ucol * 16) = v;
  };
  auto fetch = [&](long base, int f, int vj) -> uint4 {
    if (f < 0 || f >= a.T_in) return make_uint4(0, 0, 0, 0);
    return *reinterpret_cast<const uint4*>(in + ((base + f) * V + vj) * a.in_ld + ucol * 8);
  };
  auto tile_nf = [&](int k, int& n, int& f0) {
    const int t = t_begin + k;
    n = t / g.tiles_n;
    f0 = (t - n * g.tiles_n) * g.F;
  };
  // fresh halo of tile k (frames f0-4 .. f0+F+3), all 512 threads, synchronous
  auto stage_fresh = [&](int k) {
    int n, f0;
    tile_nf(k, n, f0);
    const long base = (long)n * a.T_in;
    const int rows = (g.F + KT - 1) * V;
    for (int r = tid >> 3; r < rows; r += NT / 8) {
      const int j = r / V, vj = r - j * V;
      const int f = f0 - PADT + j;
      const uint4 v = fetch(base, f, vj);
      put((f < 0 || f >= a.T_in) ? v : transform(v), f, vj);
    }
  };
  // steady state: tile k's F new frames f0+4 .. f0+F+3, by one group (256 threads, <= 4 units each).
  // The (frame j, joint v) of each unit and its ring-row offset are tile-invariant: precomputed.
  uint4 ra[RA];
  int u_j[RA], u_r[RA], u_row[RA];  // frame in the new range (>= F: unused); row in it; LDS offset in a slot
#pragma unroll
  for (int i = 0; i < RA; ++i) {
    u_r[i] = (gtid >> 3) + i * (GT / 8);
    u_j[i] = u_r[i] / V;
    u_row[i] = (u_r[i] - u_j[i] * V) * RS_A + ucol * 16;
  }
  auto prefetch = [&](int k) {
    int n, f0;
    tile_nf(k, n, f0);
    const bf16* src = in + ((long)n * a.T_in + f0 + PADT) * V * a.in_ld + ucol * 8;
#pragma unroll
    for (int i = 0; i < RA; ++i) {
      const int f = f0 + PADT + u_j[i];
      ra[i] = (u_j[i] < g.F && f < a.T_in) ? *reinterpret_cast<const uint4*>(src + (long)u_r[i] * a.in_ld)
                                            : make_uint4(0, 0, 0, 0);
    }
  };
  auto commit = [&](int k) {
    int n, f0;
    tile_nf(k, n, f0);
    const int s0 = (f0 + 2 * PADT) % g.RSL;  // slot of frame f0 + PADT (block-uniform)
#pragma unroll
    for (int i = 0; i < RA; ++i) {
      if (u_j[i] < g.F) {
        const int f = f0 + PADT + u_j[i];
        int slot = s0 + u_j[i];
        slot = slot >= g.RSL ? slot - g.RSL : slot;
        *reinterpret_cast<uint4*>(sR + slot * (V * RS_A) + u_row[i]) = f < a.T_in ? transform(ra[i]) : ra[i];
      }
    }
  };
  auto fresh = [&](int k) {  // tile k starts a sample (or the block's range)
    int n, f0;
    tile_nf(k, n, f0);
    return k == 0 || f0 == 0;
  };

  // ---- MFMA fragment addressing (two 32-row tiles per wave)
  int fl[TM], a_lane[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int r_l = wr * 64 + i * 32 + lr;
    const int rr = r_l < g.F * V ? r_l : 0;  // padding rows of the tile read anything in range
    fl[i] = rr / V;
    a_lane[i] = (rr - fl[i] * V) * RS_A + lh * 16;  // + slot * V * RS_A + ks * 32
  }
  const int slot_stride = V * RS_A;
  int boff[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) boff[ks] = (wc * 32 + lr) * RB + (((2 * ks + lh) ^ swz(lr)) << 4);
  const bool rev = a.trans != 0;

  const int col = wc * 32 + lr;
  const bool cok = col < a.Cout;
  const float bias_c = (a.bias_mode == 1 && cok) ? a.bias[col] : 0.f;
  bf16* __restrict__ out = reinterpret_cast<bf16*>(a.out);
  const long ld = a.out_ld;
  Welford run = {0.f, 0.f, 0.f};
  f32x16 acc[TM];

  auto compute = [&](int k) {
    int n, f0;
    tile_nf(k, n, f0);
    const int f0m = f0 % g.RSL;  // the lane's frame at tap offset q: slot (f0 + fl + q) mod RS
    int sb[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      sb[i] = f0m + fl[i];
      sb[i] = sb[i] >= g.RSL ? sb[i] - g.RSL : sb[i];
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
    bf16x8 fa[3][TM], fb[3];
    int base[TM];
    auto rd = [&](int st, int b) {
      const int dt = st >> 2, ks = st & 3;
      if (ks == 0) {
        const int q = rev ? KT - 1 - dt : dt;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          int s = sb[i] + q;
          s = s >= g.RSL ? s - g.RSL : s;
          base[i] = s * slot_stride + a_lane[i];
        }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fa[b][i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(sR + base[i] + ks * 32));
      fb[b] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(sB + dt * C * RB + boff[ks]));
    };
    rd(0, 0);
    rd(1, 1);
#pragma unroll
    for (int st = 0; st < KT * 4; ++st) {
      if (st + 2 < KT * 4) rd(st + 2, (st + 2) % 3);
#pragma unroll
      for (int i = 0; i < TM; ++i)
        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[st % 3][i], fb[st % 3], acc[i], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // Epilogue: bias, BatchNorm partials from the fp32 accumulators (lane = column: in-lane Welford),
  // then the bf16 tile goes through a per-wave LDS scratch [64 rows][32 cols] so that the global
  // stores are 16 B per lane (4 per wave) instead of 32 scattered 2-byte stores.
  char* scratch = sR + g.RSL * V * RS_A + 2 * C * sizeof(float) + gw * (64 * 64);
  auto epilogue = [&](int k) {
    int n, f0;
    tile_nf(k, n, f0);
    const int fe = min(g.F, a.T_out - f0);
    const int rows_valid = fe * V;
    const long row0 = ((long)n * a.T_out + f0) * V;
    float s = 0.f, cnt = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int lb = wr * 64 + i * 32 + 4 * lh;
      const bool full = cok && wr * 64 + i * 32 + 32 <= rows_valid;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ro = (r & 3) + 8 * (r >> 2);
        const float v = acc[i][r] + bias_c;
        acc[i][r] = v;
        *reinterpret_cast<bf16*>(scratch + (i * 32 + 4 * lh + ro) * 64 + lr * 2) = (bf16)v;
        if (full || (cok && lb + ro < rows_valid)) {
          s += v;
          cnt += 1.f;
        }
      }
    }
    // rows of this wave: wr*64 + lrow, 16 B units u = 0..3 of its 32 columns
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int lrow = q * 16 + (lane >> 2), u = lane & 3;
      uint4 v = *reinterpret_cast<const uint4*>(scratch + lrow * 64 + u * 16);
      const int trow = wr * 64 + lrow;
      if (trow < rows_valid) {
        bf16* p = out + (row0 + trow) * ld + wc * 32 + u * 8;
        if (a.accumulate) {
          float f[8], o[8];
          unpack16(v, f, (bf16*)nullptr);
          unpack16(*reinterpret_cast<const uint4*>(p), o, (bf16*)nullptr);
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] += o[e];
          v = pack16(f, (bf16*)nullptr);
        }
        if (wc * 32 + u * 8 < a.Cout) *reinterpret_cast<uint4*>(p) = v;
      }
    }
    if (a.stats && cnt > 0.f) {
      const float mean = s / cnt;
      float m2 = 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int lb = wr * 64 + i * 32 + 4 * lh;
        const bool full = cok && wr * 64 + i * 32 + 32 <= rows_valid;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float d = acc[i][r] - mean;
          if (full || (cok && lb + (r & 3) + 8 * (r >> 2) < rows_valid)) m2 += d * d;
        }
      }
      run = welford_merge(run, Welford{cnt, mean, m2});
    }
  };

  // Phase barrier: LDS traffic retired (lgkmcnt) + s_barrier, WITHOUT draining vmcnt — the
  // prefetched global loads and the epilogue's global stores stay in flight across phases
  // (__syncthreads() would wait for all of them every phase).
  auto bar = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // ---- prologue: weights + BN table, tile 0 staged by everyone, groups prefetch tiles 1 / 2
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  stage_fresh(0);
  if (grp == 1 && K > 1 && !fresh(1)) prefetch(1);
  if (grp == 0 && K > 2 && !fresh(2)) prefetch(2);
  __syncthreads();

  // ---- phases: group (p & 1) computes tile p; the other group finishes tile p-1, commits tile
  // p+1's frames (its own next tile) and prefetches tile p+3 (its tile after that)
  for (int p = 0; p <= K; ++p) {
    if (grp == (p & 1)) {
      if (p < K) compute(p);
    } else {
      if (p >= 1) epilogue(p - 1);
      if (p + 1 < K && !fresh(p + 1)) commit(p + 1);
      if (p + 3 < K && !fresh(p + 3)) prefetch(p + 3);
    }
    bar();
    if (p + 1 < K && fresh(p + 1)) {  // a new sample: its halo overwrites slots of tile p
      stage_fresh(p + 1);
      bar();
    }
  }

  if (a.stats) {
    // merge lane halves (same column), then the 2 row groups x 2 wave groups per column via LDS
    Welford o;
    o.n = __shfl_xor(run.n, 32);
    o.mean = __shfl_xor(run.mean, 32);
    o.m2 = __shfl_xor(run.m2, 32);
    run = welford_merge(run, o);
    float4* red = reinterpret_cast<float4*>(smem);  // [4][64]; LDS is free now
    if (lh == 0) red[(grp * 2 + wr) * C + col] = make_float4(run.n, run.mean, run.m2, 0.f);
    __syncthreads();
    if (tid < C) {
      float4 f = red[tid];
      Welford w = {f.x, f.y, f.z};
      for (int kk = 1; kk < 4; ++kk) {
        const float4 h = red[kk * C + tid];
        w = welford_merge(w, Welford{h.x, h.y, h.z});
      }
      reinterpret_cast<float4*>(a.stats)[(long)blockIdx.x * a.Cout_pad + tid] = make_float4(w.n, w.mean, w.m2, 0.f);
    }
  }
}

}  // namespace

long conv_rows_num_row_blocks(long M, int cout);

// -1: shape not handled (caller tries the next kernel)
int conv_persist_launch(const stgcn_conv_desc& a, int dtype, hipStream_t s) {
  if (dtype != 1 || a.Kt != KT || a.stride != 1 || a.pad != PADT || a.T_in != a.T_out) return -1;
  if (a.Cin_pad != C || a.Cout_pad != C || a.Cin != C || a.in_ld % 8 || a.pro > 1) return -1;
  if (a.bias_mode > 1 || a.V > 32 || a.out_ld % 8 || a.Cout % 8) return -1;
  PGeom g;
  g.F = ROWS / a.V;
  if (g.F < 1) return -1;
  g.RSL = 2 * g.F + KT - 1;
  const size_t lds = B_BYTES + (size_t)g.RSL * a.V * RS_A + 2 * C * sizeof(float) + 4 * 64 * 64;
  if (lds > (size_t)LDS_MAX) return -1;
  g.tiles_n = (a.T_out + g.F - 1) / g.F;
  const long nt = (long)a.N * g.tiles_n;
  if (nt > 0x7fffffffL) return -1;
  g.ntiles = (int)nt;
  const int ncu = stgcn_cu_count(s);
  g.tpb = (g.ntiles + ncu - 1) / ncu;
  const int grid = (g.ntiles + g.tpb - 1) / g.tpb;
  if (a.stats && grid > conv_rows_num_row_blocks((long)a.N * a.T_out * a.V, a.Cout)) return -1;
  if (stgcn_lds_attr((const void*)conv_persist_kernel, LDS_MAX, s)) return STGCN_EHIP;
  hipLaunchKernelGGL(conv_persist_kernel, dim3(grid), dim3(NT), lds, s, a, g);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
