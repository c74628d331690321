// Persistent, weight-resident temporal conv for the 64-channel layers (bf16) — the config-2
// layers 1-3 shape (tcn.2 of stgcn.py:154-159: Conv2d(64, 64, (9,1), pad (4,0)) on relu(BN1(g)),
// and its data gradient).
//
// Why: at C = 64 the K axis is only Kt*64 = 576 deep, so the frame-tiled kernel (conv_tile.hip)
// spends more time fetching the 74 KB weight tile (all 9 taps) into every block and waiting on
// each short K-chunk than it spends in MFMA (measured ~10 % of peak).  Here one block per CU
//   * loads the whole packed weight [9][64 co][64 ci] into LDS ONCE (LDS-DMA, XOR-swizzled 128-B
//     rows, conflict-free ds_read_b128),
//   * walks a contiguous range of F-frame tiles of the same samples (F = floor(128/V): 5 frames at
//     V = 25), staging each tile's halo of F+8 frames x 64 channels (BN1+ReLU prologue applied once
//     per element; frames outside [0,T) zero) into a double-buffered, XOR-swizzled LDS ring while
//     the previous tile computes,
//   * runs 8 waves = 4 row groups (32 rows) x 2 column tiles (32 cols): per k-step one A and one B
//     fragment per MFMA, tap dt reading halo rows r + q(dt)*V (q = dt fwd, 8-dt transposed),
//   * accumulates the BatchNorm partial statistics (Welford) of all its tiles in registers and
//     writes one partial row per block.
#include "common.h"
#include "../../include/stgcn_amd.h"

namespace {

constexpr int KT = 9;
constexpr int C = 64;            // Cin_pad = Cout_pad = 64
constexpr int RB = C * 2;        // bytes per row (bf16)
constexpr int NWAVE = 8, NT = NWAVE * 64;
constexpr int ROWS = 128;        // MFMA rows per tile (4 row groups x 32)
constexpr int B_BYTES = KT * C * RB;   // 73 728
constexpr int HR_MAX = 352;      // halo rows per stage: (F + 8) * V <= 352
constexpr int A_BYTES = HR_MAX * RB;   // 45 056
constexpr int A_MAX = (HR_MAX * 8 + NT - 1) / NT;  // 16-B units per thread per tile (6)

DEV int swz(int row) { return (row >> 1) & 7; }  // 128-B rows: 2 rows per 256-B bank row

DEV void glds16(const void* src, char* lds_base) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
#endif
}

struct PGeom {
  int F;         // frames per tile
  int tiles_n;   // tiles per sample
  int ntiles;    // total tiles
  int tpb;       // tiles per block
  int HR;        // halo rows
};

__global__ __launch_bounds__(NT, 1) void conv_persist_kernel(const stgcn_conv_desc a, const PGeom g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sB = smem;
  char* sA0 = smem + B_BYTES;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave & 3, wc = wave >> 2;
  const int lr = lane & 31, lh = lane >> 5;
  const int V = a.V;
  const int t_begin = blockIdx.x * g.tpb;
  const int t_end = min(g.ntiles, t_begin + g.tpb);
  if (t_begin >= t_end) {
    // no tiles: still publish an empty statistics row (the caller zero-fills, nothing to do)
    return;
  }

  const bf16* __restrict__ in = reinterpret_cast<const bf16*>(a.in);
  const bf16* __restrict__ wp = reinterpret_cast<const bf16*>(a.w);

  // ---- all weights -> LDS once (72 LDS-DMA pieces, 9 per wave), XOR swizzle on the source
  for (int piece = wave; piece < B_BYTES / 1024; piece += NWAVE) {
    const int byte = piece * 1024 + lane * 16;
    const int br = byte / RB, pu = (byte % RB) >> 4;  // br = dt*64 + co
    const int dt = br >> 6, co = br & 63;
    glds16(wp + ((long)dt * a.Cout_pad + co) * a.Cin_pad + (pu ^ swz(br)) * 8, sB + piece * 1024);
  }

  // ---- per-thread staging units: unit id = tid + i*NT -> (halo row, 16-B column)
  const int ucol = tid & 7;
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int ci = ucol * 8 + j;
    sc[j] = (a.pro == 1 && ci < a.Cin) ? a.pro_a[ci] : 1.f;
    sh[j] = (a.pro == 1 && ci < a.Cin) ? a.pro_b[ci] : 0.f;
  }
  int u_fl[A_MAX], u_v[A_MAX], u_lds[A_MAX];
#pragma unroll
  for (int i = 0; i < A_MAX; ++i) {
    const int row = (tid + i * NT) >> 3;
    u_fl[i] = row / V;
    u_v[i] = row - u_fl[i] * V;
    u_lds[i] = row < g.HR ? row * RB + ((ucol ^ swz(row)) << 4) : -1;
  }
  const int pad = (KT - 1) / 2;
  uint4 ra[A_MAX];
  unsigned zm = 0;  // bit i: unit i of the staged tile is a zero-padding row (frame outside [0, T))

  auto load = [&](int t) {
    const int n = t / g.tiles_n, f0 = (t - n * g.tiles_n) * g.F;
    const long base = (long)n * a.T_in;
    zm = 0;
#pragma unroll
    for (int i = 0; i < A_MAX; ++i) {
      ra[i] = make_uint4(0, 0, 0, 0);
      const int fi = f0 - pad + u_fl[i];
      if (u_lds[i] >= 0 && fi >= 0 && fi < a.T_in)
        ra[i] = *reinterpret_cast<const uint4*>(in + ((base + fi) * V + u_v[i]) * a.in_ld + ucol * 8);
      else
        zm |= 1u << i;
    }
  };
  auto store = [&](int buf) {
    char* A_ = sA0 + buf * A_BYTES;
#pragma unroll
    for (int i = 0; i < A_MAX; ++i) {
      if (u_lds[i] < 0) continue;
      const bool zero = (zm >> i) & 1u;
      uint4 v = ra[i];
      if (zero) {
        v = make_uint4(0, 0, 0, 0);
      } else if (a.pro == 1) {
        float f[8];
        unpack16(v, f, (bf16*)nullptr);
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], sc[j], sh[j]), 0.f);
        v = pack16(f, (bf16*)nullptr);
      }
      *reinterpret_cast<uint4*>(A_ + u_lds[i]) = v;
    }
  };

  // ---- fragment addressing
  int a_base;  // halo row of this lane's MFMA row at tap offset 0
  {
    const int r = wr * 32 + lr;
    const int rr = r < g.F * V ? r : 0;  // padding rows of the tile read anything in range
    const int fl = rr / V;
    a_base = fl * V + (rr - fl * V);
  }
  const int b_lane = (wc * 32 + lr) * RB;  // + dt*64*RB ; unit (2ks+lh) ^ swz(lr)
  const int b_sw = swz(lr);
  const bool rev = a.trans != 0;

  const float bias_c = (a.bias_mode == 1 && wc * 32 + lr < a.Cout) ? a.bias[wc * 32 + lr] : 0.f;
  const int col = wc * 32 + lr;
  const bool cok = col < a.Cout;
  bf16* __restrict__ out = reinterpret_cast<bf16*>(a.out);
  const long ld = a.out_ld;
  Welford run = {0.f, 0.f, 0.f};

  __builtin_amdgcn_s_waitcnt(0);  // weights landed (vmcnt) before the first barrier
  load(t_begin);
  store(0);
  __syncthreads();
  int cur = 0;
  for (int t = t_begin; t < t_end; ++t) {
    const bool more = t + 1 < t_end;
    if (more) load(t + 1);
    const char* A_ = sA0 + cur * A_BYTES;
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    bf16x8 fa[2], fb[2];
    auto rd = [&](int st, int b) {
      const int dt = st >> 2, ks = st & 3;
      const int q = rev ? KT - 1 - dt : dt;
      const int row = a_base + q * V;
      fa[b] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(
                                             A_ + row * RB + (((2 * ks + lh) ^ swz(row)) << 4)));
      fb[b] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(
                                             sB + dt * C * RB + b_lane + (((2 * ks + lh) ^ b_sw) << 4)));
    };
    rd(0, 0);
#pragma unroll
    for (int st = 0; st < KT * 4; ++st) {
      if (st + 1 < KT * 4) rd(st + 1, (st + 1) & 1);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[st & 1], fb[st & 1], acc, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }

    // ---- epilogue of tile t: rows r = wr*32 + acc_row(i) of the tile
    const int n = t / g.tiles_n, f0 = (t - n * g.tiles_n) * g.F;
    const int fe = min(g.F, a.T_out - f0);
    const int rows_valid = fe * V;
    const long row0 = ((long)n * a.T_out + f0) * V;
    const int lb = wr * 32 + 4 * lh;
    bf16* pb = out + (row0 + lb) * ld + col;
    float s = 0.f, cnt = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ro = (r & 3) + 8 * (r >> 2);
      const bool ok = cok && lb + ro < rows_valid;
      float v = acc[r] + bias_c;
      if (ok) {
        bf16* p = pb + ro * ld;
        if (a.accumulate) v += (float)*p;
        *p = (bf16)v;
        s += v;
        cnt += 1.f;
      }
      acc[r] = v;
    }
    if (a.stats && cnt > 0.f) {
      const float mean = s / cnt;
      float m2 = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float d = acc[r] - mean;
        if (cok && lb + (r & 3) + 8 * (r >> 2) < rows_valid) m2 += d * d;
      }
      run = welford_merge(run, Welford{cnt, mean, m2});
    }

    if (more) store(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  if (a.stats) {
    // merge lane halves (same column), then the 4 row-group waves of each column tile via LDS
    Welford o;
    o.n = __shfl_xor(run.n, 32);
    o.mean = __shfl_xor(run.mean, 32);
    o.m2 = __shfl_xor(run.m2, 32);
    run = welford_merge(run, o);
    float4* red = reinterpret_cast<float4*>(smem);  // [4 row groups][64 cols]; LDS is free now
    if (lh == 0) red[wr * C + col] = make_float4(run.n, run.mean, run.m2, 0.f);
    __syncthreads();
    if (tid < C) {
      float4 f = red[tid];
      Welford w = {f.x, f.y, f.z};
      for (int k = 1; k < 4; ++k) {
        const float4 h = red[k * C + tid];
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
  if (dtype != 1 || a.Kt != KT || a.stride != 1 || a.pad != 4 || a.T_in != a.T_out) return -1;
  if (a.Cin_pad != C || a.Cout_pad != C || a.Cin != C || a.in_ld % 8 || a.pro > 1) return -1;
  if (a.bias_mode > 1 || a.V > 32) return -1;
  PGeom g;
  g.F = ROWS / a.V;
  g.HR = (g.F + KT - 1) * a.V;
  if (g.HR > HR_MAX || g.F < 1) return -1;
  g.tiles_n = (a.T_out + g.F - 1) / g.F;
  const long nt = (long)a.N * g.tiles_n;
  if (nt > 0x7fffffffL) return -1;
  g.ntiles = (int)nt;
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (ncu <= 0) ncu = 256;
  }
  int grid = ncu;
  g.tpb = (g.ntiles + grid - 1) / grid;
  grid = (g.ntiles + g.tpb - 1) / g.tpb;
  if (a.stats && grid > conv_rows_num_row_blocks((long)a.N * a.T_out * a.V, a.Cout)) return -1;
  const size_t lds = B_BYTES + 2 * (size_t)A_BYTES;  // 163 840
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv_persist_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL(conv_persist_kernel, dim3(grid), dim3(NT), lds, s, a, g);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
