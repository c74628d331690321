// Frame-tiled implicit-GEMM row convolution (v2) — the fast path of stgcn_conv_rows.
//
// Same contract as conv_rows.hip (stgcn_conv_desc; see that file for the math).  Handles
//   * stride-1 Kt x 1 convs, forward and transposed (temporal conv fwd + data grad, stgcn.py:154-159)
//   * stride-2 Kt x 1 convs, forward (the strided temporal conv / residual conv of layers 4 and 7)
//   * flat 1x1 convs (gcn.conv on the A-mixed rows, fcn_in/out, 1x1 data grads)
// and returns -1 for anything else (the caller falls back to conv_rows.hip).
//
// Why a second kernel: conv_rows.hip re-gathers a BM-row tile for every tap, re-applying the
// BatchNorm+ReLU prologue Kt times per element and doing 64-bit address math and a validity test
// per 16-B unit and tap (~48 VALU per MFMA measured, profiles/).  Here a block owns F whole frames
// of ONE sample (F = floor(BM / V)), so
//   * the block stages ONE halo of S*(F-1)+Kt frames per K-chunk (prologue applied once per element;
//     frames outside [0, T_in) are written as zeros = the conv's zero padding AFTER the prologue),
//   * tap dt of MFMA row r reads LDS row base(r) + q(dt)*V with q(dt) = dt (fwd) or Kt-1-dt
//     (trans): no per-fragment masking, only a uniform offset per tap,
//   * rows of the last, partial tile are simply not stored.
// Flat mode (Kt = 1, stride 1) tiles BM consecutive rows across samples instead.
//
// Block: WM x WN waves, wave (wm, wn) owns TM x TN 32x32 MFMA tiles.  K is walked in chunks of
// KC input channels; per chunk the A halo (register-staged: global -> regs -> prologue -> LDS,
// padded rows of KC*sizeof(T)+16 B, conflict-free ds_read_b128) and the B tile of all Kt taps
// (LDS-DMA global_load_lds_dwordx4, lane-linear image with the XOR swizzle applied on the source
// address) are double-buffered: chunk c+1 is issued before chunk c's Kt*KC/16*TM*TN MFMAs and
// written after them, one barrier per chunk.  blockIdx is remapped so consecutive tiles (which
// share halo frames and, for several column tiles, the whole A halo) land on the same XCD.
#include "common.h"
#include "../../include/stgcn_amd.h"
#include <stdlib.h>

namespace {

template <typename T, int KC>
struct TL {
  static constexpr int RB = KC * (int)sizeof(T);        // B row bytes (swizzled LDS-DMA image)
  static constexpr int UPR = RB / 16;                    // 16-B units per row
  static constexpr int RPB = RB >= 256 ? 1 : 256 / RB;   // rows per 256-B bank row
  static constexpr int RS = RB + 16;                     // A row stride (padded)
  static DEV int swz(int row) { return (row / RPB) & (UPR - 1); }
};

// 16-byte LDS-DMA: lane l writes lds_base + 16*l (device-only builtin)
DEV void glds16(const void* src, char* lds_base) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
#endif
}

template <typename T>
DEV typename Tr<T>::frag frag2(const char* p0, const char* p1) {
  if constexpr (sizeof(T) == 2) {
    (void)p1;
    return __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(p0));
  } else {
    const f32x4 a = __builtin_bit_cast(f32x4, *reinterpret_cast<const uint4*>(p0));
    const f32x4 b = __builtin_bit_cast(f32x4, *reinterpret_cast<const uint4*>(p1));
    f32x8 f;
    f[0] = a[0]; f[1] = a[1]; f[2] = a[2]; f[3] = a[3];
    f[4] = b[0]; f[5] = b[1]; f[6] = b[2]; f[7] = b[3];
    return f;
  }
}

struct TileGeom {
  int F;           // output frames per tile (framed) ; 0 = flat mode
  int tiles_n;     // tiles per sample (framed) or total row tiles (flat)
  int HR;          // staged A rows per chunk (max over tiles)
  int ncol;        // column tiles
  int nblk;        // total blocks
  int parity;      // 1: stride-2 transposed conv, tiles hold output frames of one parity
  int tiles_half;  // parity mode: tiles per (sample, parity)
  float inv_v;     // 1 / V
};

// s_waitcnt vmcnt(n) lgkmcnt(0) (gfx9 encoding: vmcnt[3:0] | expcnt[6:4]=7 | lgkmcnt[11:8] | vmcnt[5:4]<<14)
template <int N>
DEV void wait_vm_lgkm0() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | ((N >> 4) << 14));
}

// NBS: B-tile LDS stages.  2: chunk c+1 is prefetched while chunk c computes (one __syncthreads per
// chunk).  3: chunk c+2 is prefetched (A halo into a second register set, B by LDS-DMA into the third
// stage) and the chunk barrier waits only for chunk c+1's loads (explicit vmcnt), so ~2 chunks of MFMA
// time cover the global-load latency instead of one.
template <typename T, int WM, int WN, int TM, int TN, int KC, int KT, int S, int MINW, bool PAR, int NBS>
__global__ __launch_bounds__(WM * WN * 64, MINW) void conv_tile_kernel(const stgcn_conv_desc a, const TileGeom g) {
  typedef TL<T, KC> L;
  constexpr int NW = WM * WN, NT = NW * 64;
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  constexpr int VEC = 16 / (int)sizeof(T);
  constexpr int KS = KC / 16;
  constexpr int HR_MAX = S * BM + (KT - S > 0 ? (KT - S) * 32 : 0);  // V <= 32 (checked at launch)
  constexpr int A_MAX = (HR_MAX * L::UPR + NT - 1) / NT;
  constexpr int B_BYTES = KT * BN * L::RB;
  constexpr int B_PIECES = B_BYTES / 1024;
  static_assert(B_BYTES % 1024 == 0, "B tile must be whole 1-KiB LDS-DMA pieces");
  static_assert(NT % L::UPR == 0, "unit column must be fixed per thread");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int A_BYTES = (g.HR * L::RS + 1023) & ~1023;
  char* const Abase = smem;                    // A halo stages [2]
  char* const Bbase = smem + 2 * A_BYTES;      // B stages [NBS]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int lr = lane & 31, lh = lane >> 5;
  const int V = a.V;

  // ---- XCD-aware tile order (bijective): blocks b, b+8, b+16, ... share an XCD -> give them
  // consecutive tiles (same sample, neighbouring frames, all column tiles of a row tile).
  int wg;
  {
    const int id = blockIdx.x, x = id & 7, q = g.nblk >> 3, r = g.nblk & 7;
    wg = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (id >> 3);
  }
  const int ct = wg % g.ncol, rt = wg / g.ncol;
  const int n0 = ct * BN;

  // ---- tile geometry.  Taps run as u = 0..nv-1 with weight tap dt(u) = da + db*u reading halo
  // frame offset q(u) = qa + qb*u (frames relative to the tile's halo start fi0).
  long row0;       // output row of the tile's local row 0
  int rows_valid;  // output rows of this tile
  long src0;       // flat: first input row ; framed: first input row of sample n
  int fi0 = 0;     // framed: first halo input frame
  int nv = KT, qa = 0, qb = 1, da = 0, db = 1;
  int rstep = S;   // halo frames per output frame (row base of MFMA row r)
  if (PAR) {
    // out frame f = 2i + par receives dy frame j = i + (par + pad - dt)/2 for taps with
    // (par + pad - dt) even (the stride-2 transposed conv split into two stride-1 convs)
    const int n = rt / g.tiles_n, tt = rt % g.tiles_n;
    const int par = tt / g.tiles_half, i0 = (tt % g.tiles_half) * g.F;
    const int Tp = (a.T_out - par + 1) / 2;
    const int fe = max(0, min(g.F, Tp - i0));
    const int dlo = (par + a.pad) & 1;
    nv = dlo < KT ? (KT - 1 - dlo) / 2 + 1 : 0;
    const int dhi = dlo + 2 * (nv - 1);
    const int smax = (par + a.pad - dlo) / 2, smin = (par + a.pad - dhi) / 2;
    row0 = ((long)n * a.T_out + 2 * i0 + par) * V;
    rows_valid = fe * V;
    src0 = (long)n * a.T_in * V;
    fi0 = i0 + smin;
    qa = smax - smin;
    qb = -1;
    da = dlo;
    db = 2;
    rstep = 1;
  } else if (g.F) {
    const int n = rt / g.tiles_n, f0 = (rt % g.tiles_n) * g.F;
    const int fe = min(g.F, a.T_out - f0);
    row0 = ((long)n * a.T_out + f0) * V;
    rows_valid = fe * V;
    src0 = (long)n * a.T_in * V;
    fi0 = f0 * S - ((KT - 1) / 2) * (KT > 1);
    if (KT > 1 && a.trans) {  // stride-1 transposed: frame t + pad - dt
      qa = KT - 1;
      qb = -1;
    }
  } else {
    row0 = (long)rt * BM;
    const long M = (long)a.N * a.T_out * V;
    rows_valid = (int)min((long)BM, M - row0);
    src0 = row0;
  }

  const T* __restrict__ in = reinterpret_cast<const T*>(a.in);
  const T* __restrict__ wp = reinterpret_cast<const T*>(a.w);

  // ---- per-thread A staging units (row, unit column fixed per thread)
  const int ucol = tid % L::UPR;
  const int a_units = g.HR * L::UPR;
  const T* a_ptr[A_MAX];  // chunk-0 source of each unit (nullptr = zero row)
  int a_lds[A_MAX];       // LDS byte offset within the A stage
  int a_src[A_MAX];       // source row index relative to src0 (LN prologue), -1 = zero
#pragma unroll
  for (int i = 0; i < A_MAX; ++i) {
    const int id = tid + i * NT;
    const int row = id / L::UPR;
    a_ptr[i] = nullptr;
    a_src[i] = -1;
    a_lds[i] = row * L::RS + ucol * 16;
    if (id < a_units) {
      int sr;
      bool ok;
      if (g.F) {
        const int fl = row / V, v = row - fl * V, fi = fi0 + fl;
        ok = fi >= 0 && fi < a.T_in;
        sr = fi * V + v;
      } else {
        sr = row;
        ok = row < rows_valid;
      }
      if (ok) {
        a_src[i] = sr;
        a_ptr[i] = in + (src0 + sr) * a.in_ld + ucol * VEC;
      }
    } else {
      a_lds[i] = -1;
    }
  }
  const bool fast_ld = (a.in_ld % VEC) == 0 && (a.Cin % KC) == 0;

  // ---- per-lane fragment offsets
  int a_off[TM];  // byte offset of this lane's row (tap 0) within the A stage
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int r = (wm * TM + i) * 32 + lr;
    int br;
    if (g.F) {
      if (r < g.F * V) {
        const int fl = r / V;
        br = (rstep * fl) * V + (r - fl * V);
      } else {
        br = 0;  // padding rows of the MFMA tile: read anything in range, never stored
      }
    } else {
      br = r;
    }
    a_off[i] = br * L::RS + lh * 16 * (int)(sizeof(T) / 2);
  }
  int b_off[KS][2];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int f = L::swz(lr);  // rows dt*BN + j*32 + lr share lr's swizzle (BN, 32 multiples of RPB*UPR)
    if constexpr (sizeof(T) == 2) {
      b_off[ks][0] = lr * L::RB + (((2 * ks + lh) ^ f) << 4);
      b_off[ks][1] = b_off[ks][0];
    } else {
      b_off[ks][0] = lr * L::RB + (((4 * ks + 2 * lh) ^ f) << 4);
      b_off[ks][1] = lr * L::RB + (((4 * ks + 2 * lh + 1) ^ f) << 4);
    }
  }

  const int nchunks = a.Cin_pad / KC;
  // BatchNorm prologue (pro 1) scale/shift for all input channels staged once in LDS
  const bool pro_lds = a.pro == 1 && fast_ld;
  float* const sPro = reinterpret_cast<float*>(Bbase + NBS * B_BYTES);  // [2][Cin_pad]
  if (pro_lds) {
    for (int i = tid; i < a.Cin_pad; i += NT) {
      sPro[i] = i < a.Cin ? a.pro_a[i] : 0.f;
      sPro[a.Cin_pad + i] = i < a.Cin ? a.pro_b[i] : 0.f;
    }
    __syncthreads();  // the first halo store reads the table from every wave (block-uniform condition)
  }
  uint4 ra[2][A_MAX];
  float sc[VEC], sh[VEC];  // pro 1 without pro_lds (ragged channels)

  // A halo units of chunk c -> registers (fast path: unconditional 16-B loads, zero rows masked at store)
  auto issue_A = [&](int c, uint4(&r)[A_MAX]) {
    const int cb = c * KC;
#pragma unroll
    for (int i = 0; i < A_MAX; ++i) {
      if (fast_ld) {
        r[i] = *reinterpret_cast<const uint4*>((a_ptr[i] != nullptr ? a_ptr[i] : in) + cb);
      } else {
        r[i] = make_uint4(0, 0, 0, 0);
        const int ci = cb + ucol * VEC;
        if (a_ptr[i] != nullptr && ci < a.Cin) {
          const T* p = a_ptr[i] + cb;
          float f[VEC];
#pragma unroll
          for (int j = 0; j < VEC; ++j) f[j] = ci + j < a.Cin ? Tr<T>::to_f(p[j]) : 0.f;
          r[i] = pack16(f, (T*)nullptr);
        }
      }
    }
    if (a.pro == 1 && !pro_lds) {
      const int ci = cb + ucol * VEC;
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        sc[j] = ci + j < a.Cin ? a.pro_a[ci + j] : 0.f;
        sh[j] = ci + j < a.Cin ? a.pro_b[ci + j] : 0.f;
      }
    }
  };

  // B tile of chunk c (all KT taps x BN columns x KC channels) -> LDS stage bb by LDS-DMA; whole rounds of
  // NW pieces first, then the wave-uniform tail (vmcnt bookkeeping counts B_PIECES / NW per wave)
  constexpr int B_FULL = B_PIECES / NW, B_TAIL = B_PIECES % NW;
  auto issue_B = [&](int c, int bb) {
    const int cb = c * KC;
    char* B_ = Bbase + bb * B_BYTES;
    auto piece_load = [&](int piece) {
      const int byte = piece * 1024 + lane * 16;
      const int br = byte / L::RB, pu = (byte % L::RB) >> 4;
      const int u = pu ^ L::swz(br);
      const int dt = br / BN, col = br % BN;
      glds16(wp + ((long)dt * a.Cout_pad + n0 + col) * a.Cin_pad + cb + u * VEC, B_ + piece * 1024);
    };
#pragma unroll
    for (int k = 0; k < B_FULL; ++k) piece_load(wave + k * NW);
    if (B_TAIL && wave < B_TAIL) piece_load(B_FULL * NW + wave);
  };

  auto store = [&](int c, int ab, const uint4(&r)[A_MAX]) {
    char* A_ = Abase + ab * A_BYTES;
    if (pro_lds) {
      const int ci = c * KC + ucol * VEC;
#pragma unroll
      for (int j = 0; j < VEC; j += 4) {
        const float4 s4 = *reinterpret_cast<const float4*>(sPro + ci + j);
        const float4 h4 = *reinterpret_cast<const float4*>(sPro + a.Cin_pad + ci + j);
        sc[j] = s4.x; sc[j + 1] = s4.y; sc[j + 2] = s4.z; sc[j + 3] = s4.w;
        sh[j] = h4.x; sh[j + 1] = h4.y; sh[j + 2] = h4.z; sh[j + 3] = h4.w;
      }
    }
#pragma unroll
    for (int i = 0; i < A_MAX; ++i) {
      if (a_lds[i] >= 0) {
        uint4 v = a_src[i] >= 0 ? r[i] : make_uint4(0, 0, 0, 0);
        if (a.pro != 0 && a_src[i] >= 0) {
          float f[VEC];
          unpack16(v, f, (T*)nullptr);
          if (a.pro == 1) {
#pragma unroll
            for (int j = 0; j < VEC; ++j) f[j] = fmaxf(fmaf(f[j], sc[j], sh[j]), 0.f);
          } else {
            const long srow = src0 + a_src[i];
            const float2 st = reinterpret_cast<const float2*>(a.pro_stats)[srow / V];
            const int av = (int)(srow % V);
            const int ci = c * KC + ucol * VEC;
#pragma unroll
            for (int j = 0; j < VEC; ++j) {
              const int gi = (ci + j) * V + av;
              f[j] = ci + j < a.Cin ? fmaxf((f[j] - st.x) * st.y * a.pro_a[gi] + a.pro_b[gi], 0.f) : 0.f;
            }
          }
          v = pack16(f, (T*)nullptr);
        }
        *reinterpret_cast<uint4*>(A_ + a_lds[i]) = v;
      }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  // per-row bias (bias_mode 2 / 3: the graph-conv bias through A, per joint / per sample and joint) as the
  // accumulators' initial value: its loads complete under the K loop instead of stalling the epilogue (+55 us
  // per launch at K = 384 / 768 when added there)
  if (!PAR && a.bias_mode >= 2) {
    // the tile's bias row of every local row, once per block (one division per row, not per element)
    int* const sRb = reinterpret_cast<int*>(sPro + (a.pro == 1 ? 2 * a.Cin_pad : 0));  // [BM]
    for (int t = tid; t < BM; t += NT) {
      const long m = row0 + (t < rows_valid ? t : 0), fr = m / V;
      const int v = (int)(m - fr * V);
      sRb[t] = a.bias_mode == 2 ? v : (int)((fr / a.T_out) * V + v);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + (wn * TN + j) * 32 + lr;
      if (col >= a.Cout) continue;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int lb = (wm * TM + i) * 32 + 4 * lh;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int ro = (r & 3) + 8 * (r >> 2);
          if (lb + ro < rows_valid) acc[i][j][r] = a.bias[(long)sRb[lb + ro] * a.Cout + col];
        }
      }
    }
  }

  const int tap_stride = V * L::RS;
  constexpr int NSTEP = KT * KS;  // k-steps of 16 per chunk
  typedef typename Tr<T>::frag Frag;
  auto compute = [&](int ab, int bb) {
    const char* A_ = Abase + ab * A_BYTES;
    const char* B_ = Bbase + bb * B_BYTES;
    // fragments of k-step st+1 are read while the MFMAs of k-step st run (explicit double buffer;
    // sched_barrier keeps the compiler from hoisting every tap's reads and blowing the VGPR budget)
    Frag fa[2][TM], fb[2][TN];
    auto rd = [&](int st, int b) {
      const int u = st / KS, ks = st % KS;
      const int q = qa + qb * u, dt = PAR ? da + db * u : u;
      const char* At = A_ + q * tap_stride + ks * 16 * (int)sizeof(T);
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[b][i] = frag2<T>(At + a_off[i], At + a_off[i] + 16);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const char* p = B_ + (dt * BN + (wn * TN + j) * 32) * L::RB;
        fb[b][j] = frag2<T>(p + b_off[ks][0], p + b_off[ks][1]);
      }
    };
    if (!PAR || nv > 0) rd(0, 0);
#pragma unroll
    for (int st = 0; st < NSTEP; ++st) {
      if (!PAR || st / KS < nv) {  // wave-uniform (parity mode runs fewer taps)
        if (st + 1 < NSTEP && (!PAR || (st + 1) / KS < nv)) rd(st + 1, (st + 1) & 1);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) Tr<T>::mma(acc[i][j], fa[st & 1][i], fb[st & 1][j]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };


  if constexpr (NBS == 2) {
    issue_A(0, ra[0]);
    issue_B(0, 0);
    store(0, 0, ra[0]);
    __syncthreads();
    for (int c = 0; c < nchunks; ++c) {
      const bool more = c + 1 < nchunks;
      if (more) {
        issue_A(c + 1, ra[0]);
        issue_B(c + 1, (c + 1) & 1);
      }
      compute(c & 1, c & 1);
      if (more) store(c + 1, (c + 1) & 1, ra[0]);
      __syncthreads();
    }
  } else {
    // VMEM instructions a wave issues for one chunk (fast path: A_MAX loads + the whole B rounds)
    constexpr int VM_CHUNK = A_MAX + B_FULL;
    issue_B(0, 0);
    issue_A(0, ra[0]);
    if (nchunks > 1) {
      issue_B(1, 1);
      issue_A(1, ra[1]);
    }
    store(0, 0, ra[0]);
    if (nchunks > 1) wait_vm_lgkm0<VM_CHUNK>(); else wait_vm_lgkm0<0>();
    __builtin_amdgcn_s_barrier();
    int b0 = 0;  // B stage of chunk c
    for (int c = 0; c < nchunks; c += 2) {
      // even chunk c: A regs set 0 is free (chunk c was stored last step), B stage (c+2)%3 too
      const int b2 = b0 == 0 ? 2 : b0 - 1;  // (c+2) % 3
      if (c + 2 < nchunks) {
        issue_B(c + 2, b2);
        issue_A(c + 2, ra[0]);
      }
      compute(0, b0);
      if (c + 1 < nchunks) store(c + 1, 1, ra[1]);
      if (c + 2 < nchunks) wait_vm_lgkm0<VM_CHUNK>(); else wait_vm_lgkm0<0>();
      __builtin_amdgcn_s_barrier();
      if (c + 1 >= nchunks) break;
      // odd chunk c+1
      const int b1 = b0 == 2 ? 0 : b0 + 1;  // (c+1) % 3
      if (c + 3 < nchunks) {
        issue_B(c + 3, b0);  // (c+3) % 3 == c % 3
        issue_A(c + 3, ra[1]);
      }
      compute(1, b1);
      if (c + 2 < nchunks) store(c + 2, 0, ra[0]);
      if (c + 3 < nchunks) wait_vm_lgkm0<VM_CHUNK>(); else wait_vm_lgkm0<0>();
      __builtin_amdgcn_s_barrier();
      b0 = b2;  // (c+2) % 3
    }
  }

  // ---------------------------------------------------------------- epilogue
  // lane holds column col of rows lb(i) + (r&3) + 8*(r>>2) (32x32 C/D map); row offsets are
  // compile-time multiples of the uniform out_ld.
  T* __restrict__ out = reinterpret_cast<T*>(a.out);
  const long ld = a.out_ld;
  Welford ws[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + (wn * TN + j) * 32 + lr;
    const bool cok = col < a.Cout;
    const float b1 = (a.bias_mode == 1 && cok) ? a.bias[col] : 0.f;
    float s = 0.f, cnt = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int lb = (wm * TM + i) * 32 + 4 * lh;
      T* pb = out + (row0 + lb) * ld + col;
      // per-row bias of the parity tiles (bias_mode 2 / 3; the other tiles start from it in the accumulators):
      // joint and sample of the lane's first row once, rows lb + ro advance by < 2V
      int vb = 0, tb = 0;
      long nb = 0;
      if (PAR && a.bias_mode >= 2) {
        const long mb = row0 + lb, ntb = mb / V;
        vb = (int)(mb - ntb * V);
        nb = a.bias_mode == 3 ? ntb / a.T_out : 0;
        tb = (int)(ntb - nb * a.T_out);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ro = (r & 3) + 8 * (r >> 2);
        const bool ok = cok && lb + ro < rows_valid;
        float v = acc[i][j][r] + b1;
        if (PAR && a.bias_mode >= 2 && ok) {
          int vv = vb + ro, dt = 0;
          while (vv >= V) {
            vv -= V;
            ++dt;
          }
          long bi = vv;
          if (a.bias_mode == 3) bi += (nb + (tb + dt) / a.T_out) * V;
          v += a.bias[bi * a.Cout + col];
        }
        if (ok) {
          T* p = pb + ro * ld;
          if (PAR) {  // parity tiles: local frame fl sits at output frame 2*(i0+fl)+par
            const int lrow = lb + ro, fl = (int)((lrow + 0.5f) * g.inv_v);
            p = out + (row0 + lrow + (long)fl * V) * ld + col;
          }
          if (a.accumulate) v += Tr<T>::to_f(*p);
          *p = Tr<T>::from_f(v);
          s += v;
          cnt += 1.f;
        }
        acc[i][j][r] = v;
      }
    }
    Welford w;
    w.n = cnt;
    w.mean = cnt > 0.f ? s / cnt : 0.f;
    float m2 = 0.f;
    if (a.stats) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int lb = (wm * TM + i) * 32 + 4 * lh;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float d = acc[i][j][r] - w.mean;
          if (cok && lb + (r & 3) + 8 * (r >> 2) < rows_valid) m2 += d * d;
        }
      }
    }
    w.m2 = m2;
    ws[j] = w;
  }
  if (a.stats) {
    __syncthreads();
    float4* red = reinterpret_cast<float4*>(smem);  // [WM][BN]
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      Welford o;
      o.n = __shfl_xor(ws[j].n, 32);
      o.mean = __shfl_xor(ws[j].mean, 32);
      o.m2 = __shfl_xor(ws[j].m2, 32);
      const Welford w = welford_merge(ws[j], o);
      if (lh == 0) red[wm * BN + (wn * TN + j) * 32 + lr] = make_float4(w.n, w.mean, w.m2, 0.f);
    }
    __syncthreads();
    for (int c = tid; c < BN; c += NT) {
      const float4 f = red[c];
      Welford w = {f.x, f.y, f.z};
      for (int k = 1; k < WM; ++k) {
        const float4 h = red[k * BN + c];
        w = welford_merge(w, Welford{h.x, h.y, h.z});
      }
      if (n0 + c < a.Cout_pad)
        reinterpret_cast<float4*>(a.stats)[(long)rt * a.Cout_pad + n0 + c] = make_float4(w.n, w.mean, w.m2, 0.f);
    }
  }
}


template <typename T, int WM, int WN, int TM, int TN, int KC, int KT, int S, int MINW = 2>
int launch_tile(const stgcn_conv_desc& a, long max_row_blocks, hipStream_t s) {
  typedef TL<T, KC> L;
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  constexpr int HR_MAX = S * BM + (KT - S > 0 ? (KT - S) * 32 : 0);
  if (a.Cout_pad % BN || a.Cin_pad % KC) return -1;
  TileGeom g;
  const bool flat = KT == 1 && S == 1;
  g.parity = (S == 2 && a.trans) ? 1 : 0;
  g.inv_v = 1.f / (float)a.V;
  g.tiles_half = 0;
  if (flat) {
    const long M = (long)a.N * a.T_out * a.V;
    g.F = 0;
    g.tiles_n = (int)((M + BM - 1) / BM);
    g.HR = BM;
  } else {
    if (a.V > 32 || a.V > BM) return -1;
    g.F = BM / a.V;
    if (g.parity) {
      // halo frames per parity: F + (smax - smin); smax - smin = 2*(nv-1)/2 = nv - 1
      int hf = g.F;
      for (int par = 0; par < 2; ++par) {
        const int dlo = (par + a.pad) & 1;
        const int nv = dlo < KT ? (KT - 1 - dlo) / 2 + 1 : 0;
        hf = nv > 0 && g.F + nv - 1 > hf ? g.F + nv - 1 : hf;
      }
      g.tiles_half = ((a.T_out + 1) / 2 + g.F - 1) / g.F;
      g.tiles_n = 2 * g.tiles_half;
      g.HR = hf * a.V;
    } else {
      g.tiles_n = (a.T_out + g.F - 1) / g.F;
      g.HR = (S * (g.F - 1) + KT) * a.V;
    }
    if (g.HR > HR_MAX) return -1;
  }
  g.ncol = a.Cout_pad / BN;
  const long rows_tiles = flat ? (long)g.tiles_n : (long)a.N * g.tiles_n;
  if (a.stats && rows_tiles > max_row_blocks) return -1;
  const long nblk = rows_tiles * g.ncol;
  if (nblk <= 0 || nblk > 0x7fffffffL) return -1;
  g.nblk = (int)nblk;
  const int A_BYTES = (g.HR * L::RS + 1023) & ~1023;
  const size_t B_BYTES = (size_t)KT * BN * L::RB;
  const size_t pro_bytes = a.pro == 1 ? 2 * sizeof(float) * (size_t)a.Cin_pad : 0;
  const size_t red = a.stats ? (size_t)WM * BN * 16 : 0;
  // two B stages: a 3-stage pipeline (prefetch distance 2) measured no gain on the config-2 shapes (the
  // chunk barriers, not load latency, bound this kernel) and was removed
  const size_t rb_bytes = a.bias_mode >= 2 ? (size_t)BM * sizeof(int) : 0;  // per-row bias indices
  size_t lds = 2 * ((size_t)A_BYTES + B_BYTES) + pro_bytes + rb_bytes;
  if (red > lds) lds = red;
  if (lds > 160 * 1024) return -1;
  if (stgcn_lds_attr((const void*)conv_tile_kernel<T, WM, WN, TM, TN, KC, KT, S, MINW, false, 2>, 160 * 1024, s) ||
      (S == 2 &&
       stgcn_lds_attr((const void*)conv_tile_kernel<T, WM, WN, TM, TN, KC, KT, S, MINW, S == 2, 2>, 160 * 1024, s)))
    return STGCN_EHIP;
  if (g.parity)
    hipLaunchKernelGGL((conv_tile_kernel<T, WM, WN, TM, TN, KC, KT, S, MINW, S == 2, 2>), dim3((unsigned)nblk),
                       dim3(WM * WN * 64), lds, s, a, g);
  else
    hipLaunchKernelGGL((conv_tile_kernel<T, WM, WN, TM, TN, KC, KT, S, MINW, false, 2>), dim3((unsigned)nblk),
                       dim3(WM * WN * 64), lds, s, a, g);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

template <typename T, int KT, int S>
int tile_dispatch(const stgcn_conv_desc& a, long mrb, hipStream_t s) {
  // column tile follows conv_rows_bn_tile: 64 for Cout <= 64, else 128
  const bool wide = a.Cout > 64;
  if constexpr (sizeof(T) == 2) {
    constexpr int KCB = (KT == 1 && S == 1) ? 32 : 16;  // flat GEMM: deeper chunks
    if (!wide) return launch_tile<T, 4, 1, 2, 2, KCB, KT, S>(a, mrb, s);
    return launch_tile<T, 4, 2, 2, 2, KCB, KT, S>(a, mrb, s);
  } else {
    return wide ? launch_tile<T, 4, 2, 2, 2, 16, KT, S, 1>(a, mrb, s) : launch_tile<T, 4, 1, 2, 2, 16, KT, S, 1>(a, mrb, s);
  }
}

}  // namespace

long conv_rows_num_row_blocks(long M, int cout);

// returns -1 when the shape is not handled here (caller falls back to conv_rows.hip)
int conv_persist_launch(const stgcn_conv_desc& a, int dtype, hipStream_t s);

int conv_wide_launch(const stgcn_conv_desc& a, int dtype, hipStream_t s);

int conv1x1_launch(const stgcn_conv_desc& a, int dtype, hipStream_t s);

int conv_tile_launch(const stgcn_conv_desc& a, int dtype, hipStream_t s) {
  if (a.Kt == 1) {  // 1x1 convs (residual, stride 1 or 2, and their input grads): row GEMM (conv1x1.hip)
    const int r = conv1x1_launch(a, dtype, s);
    if (r >= 0) return r;
  }
  // 64-channel stride-1 forward: the wide kernel's 32-channel items beat the weight-resident kernel
  // (70 vs 74 us on the config-2 shape); the transposed (data-grad) pass stays on conv_persist (61 vs 64 us)
  if (a.stride == 1 && !a.trans && a.Cin == 64) {
    const int r = conv_wide_launch(a, dtype, s);
    if (r >= 0) return r;
  }
  {  // weight-resident persistent kernel for the 64-channel Kt=9 convs
    const int r = conv_persist_launch(a, dtype, s);
    if (r >= 0) return r;
  }
  {  // persistent register-tiled kernel for the >= 128-channel Kt=9 stride-1 convs (conv_wide.hip)
    const int r = conv_wide_launch(a, dtype, s);
    if (r >= 0) return r;
  }
  const long mrb = conv_rows_num_row_blocks((long)a.N * a.T_out * a.V, a.Cout);
  const int S = a.stride;
  if (a.Kt == 1) {
    if (a.pad != 0) return -1;
    if (S == 1) {
      if (a.T_in != a.T_out) return -1;
      return dtype ? tile_dispatch<bf16, 1, 1>(a, mrb, s) : tile_dispatch<float, 1, 1>(a, mrb, s);
    }
    const bool ok = S == 2 && (a.trans ? a.T_in == (a.T_out - 1) / 2 + 1 : a.T_out == (a.T_in - 1) / 2 + 1);
    if (ok) return dtype ? tile_dispatch<bf16, 1, 2>(a, mrb, s) : tile_dispatch<float, 1, 2>(a, mrb, s);
    return -1;
  }
  if (a.Kt != 9 || a.pad != 4) return -1;
  if (S == 1 && a.T_out == a.T_in)
    return dtype ? tile_dispatch<bf16, 9, 1>(a, mrb, s) : tile_dispatch<float, 9, 1>(a, mrb, s);
  if (S == 2 && (a.trans ? a.T_in == (a.T_out + 2 * 4 - 9) / 2 + 1 : a.T_out == (a.T_in + 2 * 4 - 9) / 2 + 1))
    return dtype ? tile_dispatch<bf16, 9, 2>(a, mrb, s) : tile_dispatch<float, 9, 2>(a, mrb, s);
  return -1;
}
