// Persistent wide-channel temporal conv (bf16): the Kt = 9, stride-1 convs of the 128- and 256-channel
// layers (tcn.2 of stgcn.py:154-159 on relu(BN1(g)), forward, and its data gradient trans = 1) — the
// config-2 layers 4, 5, 7, 8 shapes (C = 128 at T = 150, C = 256 at T = 75).
//
// Why a third conv kernel: conv_tile.hip stages the weight tile of all 9 taps through LDS per
// 16-channel chunk, so at C >= 128 each block pays a barrier, an LDS-DMA burst and a register-staged
// halo store for every 36 MFMAs per wave (measured: ~4600 cycles per chunk against ~1600 of MFMA).
// Here:
//   * a block (4 waves, one per SIMD, 2 x 2) owns a tile of F = floor(256 / V) whole output frames of
//     one sample (250 rows at V = 25) x BN output channels (BN = 128 or 256); wave (wm, wn) holds the
//     128 x BN/2 accumulator block in registers (TM = 4 x TN = BN/64 MFMA tiles of 32 x 32);
//   * K is walked as items of 64 input channels: per item the input halo (F + 8 frames x V joints x
//     64 ch) sits in LDS (rows padded to 144 B: conflict-free ds_read_b128 for any tap offset) and all
//     9 taps read it at a uniform row offset q(dt) * V (q = dt forward, 8 - dt transposed);
//   * the weights never touch LDS: each wave streams its B fragments (16 B per lane, fragment-shaped)
//     from L2 straight into a ring of NBUF register sets, LEAD = NBUF - 1 k-steps ahead of use, so the
//     9-tap loop has no barrier at all; the two waves of a column half share each fragment through L1;
//   * the next item's halo (next 64 channels, or the next tile) is loaded into registers at the
//     item's first k-step and written (BN1 scale/shift + ReLU prologue applied, zero frames outside
//     [0, T)) into the other LDS halo buffer a few k-steps later, spread over several k-steps so the
//     VALU work runs beside the MFMAs: ONE barrier per 64-channel item;
//   * blocks are persistent (grid = CU count), each walking a contiguous run of tiles; items are
//     processed in pairs (the channel-group count G = Cin / 64 is even), which makes the halo buffer
//     and the B register set of every k-step compile-time;
//   * C = 64 (two 32-channel items per tile): 8 helper waves and a separate tile-image buffer (the helpers
//     bound that instantiation);
//   * epilogue per tile: + bias, bf16 store, BatchNorm Welford partials per (tile, channel) (the
//     float4 (count, mean, M2) layout bn_finalize merges; row-tile index = n * tiles_n + tile).
#include "common.h"
#include "pack.h"
#include "../../include/stgcn_amd.h"
#include <stdlib.h>
#include <utility>

namespace {

constexpr int KG = 64;               // input channels per item
constexpr int KS = KG / 16;          // MFMA k-steps per tap
constexpr int NT = 256;              // 4 waves
constexpr int WM_MAX = 4;  // MMA wave rows (sRed is sized for the largest layout)
constexpr int RSA = KG * 2 + 16;     // padded halo row bytes (144)
constexpr int HR_CAP = 456;          // max halo rows per item (V = 25: 18 frames x 25 = 450)
constexpr int NA = (HR_CAP * 8 + NT - 1) / NT;  // 16-B halo units per thread (15)
constexpr int CSO = 256 * 2 + 8;                  // column bytes of the column-major output tile image (256 rows)
constexpr int ABYTES_MIN = (128 * CSO > NA * 32 * RSA ? 128 * CSO : NA * 32 * RSA);  // halo buffer / tile image
// halo buffer bytes for item width kg (>= every staged unit row of a helper thread, and the tile image)
constexpr int abytes_for(int kg) {
  const int upr = kg / 8, rstep = 256 / upr, na = (HR_CAP * upr + 255) / 256, halo = na * rstep * (2 * kg + 16);
  return halo > 128 * CSO ? halo : 128 * CSO;
}
constexpr int LDS_MAX = 160 * 1024;

// compile-time loop: f.template operator()<I>() for I = 0..N-1 (guaranteed unrolled; register arrays
// indexed by I never fall back to scratch)
template <int N, typename F>
DEV void static_for(F&& f) {
  [&]<int... I>(std::integer_sequence<int, I...>) { (f.template operator()<I>(), ...); }(
      std::make_integer_sequence<int, N>{});
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops (lgkmcnt) but NOT for its
// outstanding global loads — __syncthreads() would drain the B-fragment prefetch ring (vmcnt(0)) at
// every 64-channel item.  The "memory" clobber keeps the compiler from moving memory ops across it.
DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

struct WGeom {
  int F;        // output frames per tile
  int tiles_n;  // tiles per sample
  int ncol;     // column tiles (Cout_pad / BN)
  int ntiles;   // N * tiles_n * ncol
  int G;        // 64-channel items per tile (even)
  int HR;       // halo rows per item ((F + KTAP - 1) * V)
  int abytes;   // bytes per LDS halo buffer
  int T_tile;   // frames the tiles walk (output frames; fold 2: dY frames)
  int fold;     // stride-2 folding: 0 none, 1 input parity (forward), 2 output parity (data grad)
  int cpar;     // fold 1: 64-channel items per input parity; fold 2: output channels per parity
  int wc32, wk16;  // fragment image dims: (output channels / 32, input channels / 16)
  int pair;        // ncol == 2: blocks b and b + 8 (one XCD) take the two column tiles of the same row-tile run
  int red_off;     // LDS byte offset of the Welford partials (after the halo buffers and, SEP, the tile image)
};

struct TileInfo {
  int n, f0, fe, ct;
};

DEV TileInfo tile_info(int tile, const WGeom& g) {
  TileInfo ti;
  ti.ct = tile % g.ncol;
  const int rt = tile / g.ncol;
  ti.n = rt / g.tiles_n;
  ti.f0 = (rt - ti.n * g.tiles_n) * g.F;
  ti.fe = min(g.F, g.T_tile - ti.f0);
  return ti;
}

// Block = 8 waves in two roles (wave-uniform branch; both roles execute the same barrier sequence):
//   MMA waves 0-3 (wm = w>>1, wn = w&1): B-fragment ring + LDS A fragments + MFMAs only, so their
//     vmcnt never waits on anything but L2-resident weights;
//   helper waves 4-7: stage the NEXT item's halo (global loads -> prologue -> LDS) and drain finished
//     output tiles (LDS image -> 16-B row stores, BN partials -> global), i.e. all HBM traffic.
// Per item k (buffer b = k & 1): MMA computes item k from buf b while the helpers fill buf b^1 with
// item k+1; barrier E_k.  At a tile end the MMA waves dump acc (+ bias) as a column-major bf16 image
// into buf b (8-B ds_write_b64 per 4 rows) and their Welford partials into sRed; barrier I_k; the
// helpers drain that image during item k+1 before they overwrite buf b with item k+2's halo.
// DBG (compile-time A/B instantiations only): bit1 no helper work, bit2 no MFMAs (timing; results wrong)
// WMT: MMA-wave layout, WMT x (4 / WMT) waves over (256 rows x BN columns).  WMT = 4 at BN = 64: each wave
// holds 64 rows x 64 columns, so every A fragment read from LDS feeds two MFMAs (the 2 x 2 layout reads
// each A fragment in both column-half waves: LDS reads = MFMAs at C = 64)
// NHW: helper waves (4, or 8 where staging + drain bound the kernel: C = 64)
// SEPT (two-item tiles only, C = 64): the finished tile image gets its own LDS buffer, so the helpers drain it
// in halves over both windows of the next tile instead of all of it before the next halo store
template <int BN, int KTAP, int NBUF, int PRO, int DBG = 0, int KGT = 64, int WMT = 2, int APD = 1, int NHW = 4,
          bool SEPT = false>
__global__ __launch_bounds__((4 + NHW) * 64, 1) void conv_wide_kernel(const stgcn_conv_desc a, const WGeom g) {
  constexpr int WM = WMT, WN = 4 / WMT, TM = 8 / WMT;
  // item width: 64 input channels (>= 128-channel layers) or 32 (64-channel layers: two items per tile)
  constexpr int KG = KGT, KS = KG / 16, RSA = 2 * KG + 16;
  constexpr int NTH = NHW * 64;                            // helper threads
  constexpr int UPR = KG / 8, RSTEP = NTH / UPR;           // 16-B units per halo row, rows per staging pass
  constexpr int NA = (HR_CAP * UPR + NTH - 1) / NTH;       // halo units per helper thread
  constexpr int SPI = KTAP * KS;  // k-steps per item
  constexpr int TN = BN / 32 / WN;
  static_assert(TN >= 1 && WM * WN == 4, "wave layout");
  constexpr int LEAD = NBUF - 1;
  constexpr int PAIR = 2 * SPI;  // k-steps per item pair
  static_assert(PAIR % NBUF == 0, "B register ring must divide the pair");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool mma = wave < 4;
  const int V = a.V;
  const int grid = gridDim.x;
  const int tpb = (g.ntiles + grid - 1) / grid;  // contiguous tile runs: neighbour halos stay in L2
  int tile0 = (int)blockIdx.x * tpb;
  int tstep = 1;
  int ntile_b = min(tpb, g.ntiles - tile0);
  if (g.pair) {
    // workgroups are dealt round-robin to the 8 XCDs: blocks b = x + 8 s share XCD x; the pair (s = 2q, 2q+1)
    // walks the same run of row tiles, one column tile each, at the same pace, so every halo item one of
    // them stages from HBM the other finds in the XCD's L2 (a block walking both column tiles of a row tile
    // in turn re-fetched the halo: 32 CUs' halos overrun the 4 MB L2)
    const int b = blockIdx.x, sx = b >> 3;
    const int nrt = g.ntiles >> 1, npair = grid >> 1;
    const int rpp = (nrt + npair - 1) / npair;
    const int rt0 = ((b & 7) * (grid >> 4) + (sx >> 1)) * rpp;
    tile0 = 2 * rt0 + (sx & 1);
    tstep = 2;
    ntile_b = min(rpp, nrt - rt0);
  }
  if (ntile_b <= 0) return;
  const int nitems = ntile_b * g.G;

  const bf16* __restrict__ in = reinterpret_cast<const bf16*>(a.in);
  const bf16* __restrict__ wp = reinterpret_cast<const bf16*>(a.w_frag);
  char* const sA0 = smem;
  char* const sA1 = smem + g.abytes;
  constexpr bool SEP = SEPT && KG == 32;
  char* const sImg = SEP ? smem + 2 * g.abytes : nullptr;  // [BN][CSO] tile image (SEP)
  float4* const sRed = reinterpret_cast<float4*>(smem + g.red_off);  // [WM][BN]
  // drain counter: each helper wave adds 1 when its reads of a tile image are done; the halo writes into
  // that buffer wait until all four have (the image and the next halo share the buffer)
  unsigned* const sCnt = reinterpret_cast<unsigned*>(smem + g.red_off + WM_MAX * BN * 16);

  auto item_tile = [&](int w, int& gi) {  // items past the block's last one are clamped to it
    w = min(w, nitems - 1);
    const int tl = w / g.G;
    gi = w - tl * g.G;
    return tile0 + tl * tstep;
  };
  auto tile_end = [&](int w) { return w < nitems && (w % g.G) == g.G - 1; };

  if (!mma) {
    // =============================== helper waves ===============================
    const int htid = tid - NT;
    const int ucol = htid % UPR, row0u = htid / UPR;
    // NSET register sets: item w + 1 + NSET's halo is requested in window w.  Two sets for the 32-channel
    // items (short MMA time per item: the loads need two items of cover), one for 64-channel items
    constexpr int NSET = KG == 32 ? 2 : 1;
    int a_lo[NSET], a_hi[NSET];
    uint4 ra[NSET][NA];
    float sc[NSET][8], sh[NSET][8];
    auto issue_A = [&]<int SET>(int w) {  // item w's halo units -> register set SET
      int gi;
      const int tile = item_tile(w, gi);
      const TileInfo ti = tile_info(tile, g);
      const int fi0 = ti.f0 - (KTAP - 1) / 2;
      int cg = gi;  // 64-channel group of the source tensor
      if (g.fold == 1) {
        // halo frame z = fi0 + fl is the pair (x[2z], x[2z+1]); this item reads parity gi / cpar
        const int par = gi / g.cpar;
        cg = gi - par * g.cpar;
        a_lo[SET] = max(0, -fi0) * V;
        a_hi[SET] = min(g.HR, ((a.T_in - par + 1) / 2 - fi0) * V);
        const bf16* base = in + (long)ti.n * a.T_in * V * a.in_ld + cg * KG + ucol * 8;
        static_for<NA>([&]<int i>() {
          const int row = min(max(row0u + RSTEP * i, a_lo[SET]), a_hi[SET] - 1);
          const int fl = row / V, v = row - fl * V;
          ra[SET][i] = *reinterpret_cast<const uint4*>(base + ((2 * (fi0 + fl) + par) * V + v) * (long)a.in_ld);
        });
      } else {
        a_lo[SET] = max(0, -fi0) * V;
        a_hi[SET] = min(g.HR, (a.T_in - fi0) * V);
        const bf16* base = in + ((long)ti.n * a.T_in + fi0) * V * a.in_ld + gi * KG + ucol * 8;
        static_for<NA>([&]<int i>() {
          const int row = min(max(row0u + RSTEP * i, a_lo[SET]), a_hi[SET] - 1);
          ra[SET][i] = *reinterpret_cast<const uint4*>(base + row * a.in_ld);
        });
      }
      if (PRO == 1) {
        const int c = cg * KG + ucol * 8;
        const float4 s0 = *reinterpret_cast<const float4*>(a.pro_a + c);
        const float4 s1 = *reinterpret_cast<const float4*>(a.pro_a + c + 4);
        const float4 h0 = *reinterpret_cast<const float4*>(a.pro_b + c);
        const float4 h1 = *reinterpret_cast<const float4*>(a.pro_b + c + 4);
        sc[SET][0] = s0.x; sc[SET][1] = s0.y; sc[SET][2] = s0.z; sc[SET][3] = s0.w;
        sc[SET][4] = s1.x; sc[SET][5] = s1.y; sc[SET][6] = s1.z; sc[SET][7] = s1.w;
        sh[SET][0] = h0.x; sh[SET][1] = h0.y; sh[SET][2] = h0.z; sh[SET][3] = h0.w;
        sh[SET][4] = h1.x; sh[SET][5] = h1.y; sh[SET][6] = h1.z; sh[SET][7] = h1.w;
      }
    };
    auto store_A = [&]<int SET>(char* buf) {  // prologue (BN1 scale/shift + ReLU) + zero rows -> LDS halo buffer
      static_for<NA>([&]<int i>() {
        const int row = row0u + RSTEP * i;
        uint4 v = ra[SET][i];
        if (PRO == 1) {
          float f[8];
          unpack16(v, f, (bf16*)nullptr);
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = fmaxf(fmaf(f[j], sc[SET][j], sh[SET][j]), 0.f);
          v = pack16(f, (bf16*)nullptr);
        }
        const bool ok = row >= a_lo[SET] && row < a_hi[SET];
        v.x = ok ? v.x : 0u;
        v.y = ok ? v.y : 0u;
        v.z = ok ? v.z : 0u;
        v.w = ok ? v.w : 0u;
        *reinterpret_cast<uint4*>(buf + row * RSA + ucol * 16) = v;
      });
    };
    // finished tile image (column-major [BN][CSO bytes]) -> global rows; BN partials -> global
    auto drain = [&](int w, const char* img, int part = 0, int nparts = 1) {
      int gi;
      const int tile = item_tile(w, gi);
      const TileInfo ti = tile_info(tile, g);
      const int rows_valid = ti.fe * V;
      const int n0 = ti.ct * BN;
      if (a.stats && part == 0) {
        const int rt = tile / g.ncol;
        for (int c = htid; c < BN; c += NTH) {
          const float4 f0 = sRed[c];
          Welford wv{f0.x, f0.y, f0.z};
#pragma unroll
          for (int k = 1; k < WM; ++k) {
            const float4 f1 = sRed[k * BN + c];
            wv = welford_merge(wv, Welford{f1.x, f1.y, f1.z});
          }
          if (n0 + c < a.Cout_pad)
            reinterpret_cast<float4*>(a.stats)[(long)rt * a.Cout_pad + n0 + c] = make_float4(wv.n, wv.mean, wv.m2, 0.f);
        }
      }
      // thread = (row quad rq, 8-channel unit cu): a lane reads its unit's 8 columns x 4 rows (ds_read_b64
      // each) and transposes them in registers into 4 row units of 16 B; in every store instruction
      // groups of 8 consecutive lanes write 8 consecutive units of one row, i.e. whole 128-B lines (16-B
      // pieces of a line stored by different instructions measured ~1.9x the output bytes in HBM writes)
      // fold 2: column tile n0 of the folded [dx_even | dx_odd] space -> parity par, channel base cb
      const int par = g.fold == 2 ? n0 / g.cpar : 0;
      const int cb = n0 - par * (g.fold == 2 ? g.cpar : 0);
      bf16* __restrict__ outs = reinterpret_cast<bf16*>(a.out) + (long)ti.n * a.T_out * V * a.out_ld;
      bf16* __restrict__ outb = outs + (long)ti.f0 * V * a.out_ld;
      // 64 lanes = 8 row quads x 8 units (a 128-B line per row and store instruction); with the 520-B
      // column stride the 8 units x 8 quads of one ds_read_b64 land on 32 distinct bank pairs (2-way)
      constexpr int UG = BN / 64;  // groups of 8 units per row
      const int nq = (rows_valid + 3) >> 2, nq8 = (nq + 7) >> 3;
      for (int idx = htid + part * NTH; idx < UG * nq8 * 64; idx += nparts * NTH) {
        const int cl = idx & 7, ql = (idx >> 3) & 7, rest = idx >> 6;
        const int ug = rest / nq8, qh = rest - ug * nq8;
        const int rq = qh * 8 + ql, cu = ug * 8 + cl;
        if (rq >= nq) continue;
        if (cb + cu * 8 >= a.Cout) continue;
        uint2 col[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) col[c] = *reinterpret_cast<const uint2*>(img + (cu * 8 + c) * CSO + rq * 8);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int rl = 4 * rq + e;
          if (rl >= rows_valid) break;
          // row e of the quad: low/high halves of dword e>>1 of each column
          const unsigned sel = (e & 1) ? 0x07060302u : 0x05040100u;
          uint4 u;
          u.x = __builtin_amdgcn_perm((e >> 1) ? col[1].y : col[1].x, (e >> 1) ? col[0].y : col[0].x, sel);
          u.y = __builtin_amdgcn_perm((e >> 1) ? col[3].y : col[3].x, (e >> 1) ? col[2].y : col[2].x, sel);
          u.z = __builtin_amdgcn_perm((e >> 1) ? col[5].y : col[5].x, (e >> 1) ? col[4].y : col[4].x, sel);
          u.w = __builtin_amdgcn_perm((e >> 1) ? col[7].y : col[7].x, (e >> 1) ? col[6].y : col[6].x, sel);
          bf16* p = outb + (long)rl * a.out_ld + cb + cu * 8;
          if (g.fold == 2) {  // tile frame u -> output frame 2u + par
            const int fl = rl / V, v = rl - fl * V, fr = 2 * (ti.f0 + fl) + par;
            if (fr >= a.T_out) continue;
            p = outs + ((long)fr * V + v) * a.out_ld + cb + cu * 8;
          }
          if (a.accumulate) {
            float f[8], o[8];
            unpack16(u, f, (bf16*)nullptr);
            unpack16(*reinterpret_cast<const uint4*>(p), o, (bf16*)nullptr);
#pragma unroll
            for (int q = 0; q < 8; ++q) f[q] += o[q];
            u = pack16(f, (bf16*)nullptr);
          }
          *reinterpret_cast<uint4*>(p) = u;
        }
      }
    };

    // Helper waves are not synchronised with each other inside a window, so a wave that finished its share
    // of a drain must not overwrite the buffer with the next halo while another still reads the image:
    // count finished drains per wave in LDS and wait for all four before the first halo write.
    unsigned ndrain = 0;
    auto drain_sync = [&]() {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_fetch_add(sCnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      ndrain += NHW;
      while (__hip_atomic_load(sCnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < ndrain)
        __builtin_amdgcn_s_sleep(1);
    };
    if (htid == 0) *sCnt = 0u;  // visible to all helpers after barrier P
    // item w lives in register set w % NSET and LDS buffer w & 1; nitems is even (G even)
    issue_A.template operator()<0>(0);
    store_A.template operator()<0>(sA0);
    if (nitems > 1) issue_A.template operator()<1 % NSET>(1);
    if (NSET == 2 && nitems > 2) issue_A.template operator()<0>(2);
    lds_barrier();  // P
    for (int w = 0; w < nitems && SEP; w += 2) {
      // SEP (G = 2: the pair (w, w+1) is one tile): drain the previous tile's image in two halves, one per
      // window, beside the two halo stores; the next dump comes after E_{w+1}
      if (w > 0) drain(w - 1, sImg, 0, 2);
      store_A.template operator()<1 % NSET>(sA1);
      if (w + 1 + NSET < nitems) issue_A.template operator()<(1 + NSET) % NSET>(w + 1 + NSET);
      lds_barrier();  // E_w
      if (w > 0) drain(w - 1, sImg, 1, 2);
      if (w + 2 < nitems) store_A.template operator()<2 % NSET>(sA0);
      if (w + 2 + NSET < nitems) issue_A.template operator()<(2 + NSET) % NSET>(w + 2 + NSET);
      lds_barrier();  // E_{w+1}
      lds_barrier();  // I_{w+1}
    }
    if (SEP) {
      drain(nitems - 1, sImg);
      return;
    }
    for (int w = 0; w < nitems; w += 2) {
      // window w: item w+1 -> sA1, request item w+1+NSET
      if ((DBG & 2) == 0) {
        if (w > 0 && tile_end(w - 1)) {
          drain(w - 1, sA1);
          if (w + 1 < nitems) drain_sync();
        }
        if (w + 1 < nitems) store_A.template operator()<1 % NSET>(sA1);
        if (w + 1 + NSET < nitems) issue_A.template operator()<(1 + NSET) % NSET>(w + 1 + NSET);
      }
      lds_barrier();  // E_w
      if (tile_end(w)) lds_barrier();  // I_w
      // window w+1: item w+2 -> sA0, request item w+2+NSET
      if ((DBG & 2) == 0) {
        if (tile_end(w)) {
          drain(w, sA0);
          if (w + 2 < nitems) drain_sync();
        }
        if (w + 2 < nitems) store_A.template operator()<2 % NSET>(sA0);
        if (w + 2 + NSET < nitems) issue_A.template operator()<(2 + NSET) % NSET>(w + 2 + NSET);
      }
      lds_barrier();  // E_{w+1}
      if (tile_end(w + 1)) lds_barrier();  // I_{w+1}
    }
    if ((DBG & 2) == 0) drain(nitems - 1, ((nitems - 1) & 1) ? sA1 : sA0);
    return;
  }

  // =============================== MMA waves ===============================
  const int wm = wave / WN, wn = wave % WN;
  const int lr = lane & 31, lh = lane >> 5;
  // B fragment j at k-step (t, ks) of item (ct, gi): the contiguous 1-KiB block
  // [t][c32 = ct*BN/32 + wn*TN + j][k16 = gi*4 + ks] of the fragment image (stgcn_pack_weight_frag)
  const int c32n = g.wc32, k16n = g.wk16;
  const int kcc = c32n * k16n * 512;  // elements per tap
  const int wnu = __builtin_amdgcn_readfirstlane(wn);
  const int wlane = lane * 8;
  auto item_woff = [&](int w) {
    int gi;
    const int tile = item_tile(w, gi);
    return ((tile % g.ncol) * (BN / 32) + wnu * TN) * k16n * 512 + gi * KS * 512;
  };
  bf16x8 fb[NBUF][TN];
  auto load_B = [&](bf16x8 (&dst)[TN], int hs, int woff, int wl, int kc, int k16) {
    const int t = hs / KS, ks = hs % KS;
    const bf16* p = wp + (t * kc + woff + ks * 512) + wl;
#pragma unroll
    for (int j = 0; j < TN; ++j)
      dst[j] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(p + j * k16 * 512));
  };
  // A fragment rows: MFMA row r = (wm*TM + i)*32 + lr reads halo row r + q(dt)*V (padding rows of the
  // 256-row MFMA tile past F*V read row 0: in range, never stored)
  int a_frag[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int r = (wm * TM + i) * 32 + lr;
    a_frag[i] = (r < g.F * V ? r : 0) * RSA + lh * 16;
  }
  const int tap_bytes = V * RSA;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // tile end: acc + bias -> column-major bf16 image (4 consecutive rows of one column per ds_write_b64)
  // and per-column Welford partials of the fp32 values -> sRed; acc reset
  // bias of the current tile's columns, loaded at its first pair (a load issued in the dump itself
  // would wait behind the whole in-flight B ring: loads retire in order)
  float bias_r[TN];
  auto load_bias = [&](int w) {
    int gi;
    const int n0 = (item_tile(w, gi) % g.ncol) * BN;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + (wn * TN + j) * 32 + lr;
      bias_r[j] = (a.bias_mode == 1 && col < a.Cout) ? a.bias[col] : 0.f;
    }
  };
  auto dump = [&](int w, char* img) {
    int gi;
    const int tile = item_tile(w, gi);
    const TileInfo ti = tile_info(tile, g);
    const int rows_valid = ti.fe * V;
    const int n0 = ti.ct * BN;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int cl = (wn * TN + j) * 32 + lr;
      const bool cok = n0 + cl < a.Cout;
      const float b1 = bias_r[j];
      // single pass: statistics of v = acc + b1 shifted by b1 (s1 = sum acc, s2 = sum acc^2 over valid
      // rows); row masks only in the 32-row blocks that cross rows_valid (wave-uniform test)
      float s1 = 0.f, s2 = 0.f, cnt = 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int rb = (wm * TM + i) * 32;
        if (rb + 32 <= rows_valid) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            s1 += acc[i][j][r];
            s2 = fmaf(acc[i][j][r], acc[i][j][r], s2);
          }
          cnt += 16.f;
        } else if (rb < rows_valid) {
          const int lim = rows_valid - rb - 4 * lh;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const bool ok = (r & 3) + 8 * (r >> 2) < lim;
            const float d = ok ? acc[i][j][r] : 0.f;
            s1 += d;
            s2 = fmaf(d, d, s2);
            cnt += ok ? 1.f : 0.f;
          }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          bf16x4 pk;
#pragma unroll
          for (int e = 0; e < 4; ++e) pk[e] = (bf16)(acc[i][j][4 * q + e] + b1);
          *reinterpret_cast<bf16x4*>(img + cl * CSO + (rb + 4 * lh + 8 * q) * 2) = pk;
        }
      }
      if (a.stats) {
        Welford wv;
        wv.n = cok ? cnt : 0.f;
        const float mu = wv.n > 0.f ? s1 / wv.n : 0.f;
        wv.mean = b1 + mu;
        wv.m2 = wv.n > 0.f ? fmaxf(s2 - s1 * mu, 0.f) : 0.f;
        Welford o;
        o.n = __shfl_xor(wv.n, 32);
        o.mean = __shfl_xor(wv.mean, 32);
        o.m2 = __shfl_xor(wv.m2, 32);
        const Welford m = welford_merge(wv, o);
        if (lh == 0) sRed[wm * BN + cl] = make_float4(m.n, m.mean, m.m2, 0.f);
      }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  };

  {
    const int w0 = item_woff(0);
#pragma unroll
    for (int hs = 0; hs < LEAD; ++hs) load_B(fb[hs % NBUF], hs, w0, wlane, kcc, k16n);
  }
  lds_barrier();  // P

  const bool rev = a.trans && g.fold == 0;  // stride-1 data grad: taps reversed
  const int qsign = rev ? -1 : 1;
  const int qbase = rev ? KTAP - 1 : 0;
  for (int w = 0; w < nitems; w += 2) {
    const int woff0 = item_woff(w), woff1 = item_woff(w + 1), woff2 = item_woff(w + 2);
    // per-lane/uniform address bases re-materialised each pair (opaque to LICM: otherwise the
    // compiler hoists the addresses of all 72 k-steps out of the loop and spills)
    int af[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      af[i] = a_frag[i];
      asm volatile("" : "+v"(af[i]));
    }
    int wl = wlane;
    asm volatile("" : "+v"(wl));
    int tbytes = tap_bytes, kcc_l = kcc, cinp_l = k16n;
    asm volatile("" : "+s"(tbytes));
    asm volatile("" : "+s"(kcc_l));
    asm volatile("" : "+s"(cinp_l));
    constexpr int AR = APD + 1;  // A fragment ring: reads APD k-steps ahead inside an item
    bf16x8 fa[AR][TM];
    // one k-step; hs is a template parameter so every ring index below is a compile-time constant
    auto step = [&]<int hs>() {
      constexpr int h = hs / SPI, s = hs % SPI, t = s / KS, ks = s % KS;
      char* const cur = h == 0 ? sA0 : sA1;
      {  // B fragments LEAD k-steps ahead (may belong to the next item or the next pair)
        constexpr int hn = hs + LEAD;
        const int woff = hn < SPI ? woff0 : (hn < PAIR ? woff1 : woff2);
        load_B(fb[hn % NBUF], hn % SPI, woff, wl, kcc_l, cinp_l);
      }
      auto read_a = [&]<int sd>() {  // A fragments of k-step sd of this item -> ring slot
        constexpr int td = sd / KS, ksd = sd % KS;
        const int tb = (qbase + qsign * td) * tbytes + ksd * 32;
#pragma unroll
        for (int i = 0; i < TM; ++i)
          fa[(h * SPI + sd) % AR][i] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(cur + af[i] + tb));
      };
      if constexpr (s == 0) {
        static_for<APD>([&]<int d>() { read_a.template operator()<d>(); });
      }
      if constexpr (s + APD < SPI) read_a.template operator()<s + APD>();
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr ((DBG & 4) != 0)  // timing only: operands consumed without MFMA work
            acc[i][j][0] += (float)fa[hs % AR][i][0] + (float)fb[hs % NBUF][j][0];
          else
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[hs % AR][i], fb[hs % NBUF][j], acc[i][j], 0, 0, 0);
        }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (s == SPI - 1) {
        lds_barrier();  // E_{w+h}
      }
    };
    if (w % g.G == 0) load_bias(w);
    static_for<PAIR>(step);
    if (tile_end(w + 1)) {
      dump(w + 1, SEP ? sImg : sA1);
      lds_barrier();  // I_{w+1}
    }
  }
}

__global__ void pack_s2frag_kernel(const float* __restrict__ src, long s0, long s1, long s2, int Co, int Ci, int trans,
                                   int co_f, int ci_f, bf16* __restrict__ dst) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx < 5L * co_f * ci_f / 8) pack_s2frag_elem(src, s0, s1, s2, Co, Ci, trans, co_f, ci_f, idx, dst);
}

}  // namespace

int pack_s2frag_launch(const float* src, long s0, long s1, long s2, int Co, int Ci, void* dst, int trans,
                       hipStream_t s) {
  const int co_f = trans ? 2 * Co : Co, ci_f = trans ? Ci : 2 * Ci;
  if (co_f % 32 || ci_f % 16) return STGCN_EBADSHAPE;
  if (Ci % 8 || Co % 8) return STGCN_EBADSHAPE;
  const long total = 5L * co_f * ci_f / 8;  // threads: 8 consecutive folded input channels each
  hipLaunchKernelGGL(pack_s2frag_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, src, s0, s1, s2, Co,
                     Ci, trans, co_f, ci_f, (bf16*)dst);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}


long conv_rows_num_row_blocks(long M, int cout);

int conv_wide_launch(const stgcn_conv_desc& a, int dtype, hipStream_t s) {
  if (dtype != 1 || !a.w_frag) return -1;
  if (a.Kt != 9 || a.pad != 4) return -1;
  if (a.pro != 0 && a.pro != 1) return -1;
  if (a.bias_mode != 0 && a.bias_mode != 1) return -1;
  if (a.in_ld % 8 || a.V > 32 || a.Cin % 8 || a.Cout % 8 || a.out_ld % 8) return -1;
  WGeom g;
  int ktap, cin_f, cout_f;  // folded conv: taps, input / output channels
  if (a.stride == 1) {
    if (a.T_in != a.T_out) return -1;
    g.fold = 0;
    ktap = 9;
    cin_f = a.Cin;
    cout_f = a.Cout;
    g.T_tile = a.T_out;
  } else if (a.stride == 2 && !a.trans) {
    // y[f] = sum_{j=-2..2} [W(2j+4) | W(2j+5)] (x[2(f+j)], x[2(f+j)+1]): a 5-tap conv over frame pairs
    if (a.T_out != (a.T_in - 1) / 2 + 1) return -1;
    g.fold = 1;
    ktap = 5;
    cin_f = 2 * a.Cin;
    cout_f = a.Cout;
    g.T_tile = a.T_out;
    g.cpar = a.Cin / KG;
    if (a.Cin % KG) return -1;
  } else if (a.stride == 2 && a.trans) {
    // [dx(2u) | dx(2u+1)] = sum_{j=-2..2} [Wd(4-2j) ; Wd(5-2j)] dy(u+j): a 5-tap conv with 2*Cout outputs
    if (a.T_in != (a.T_out - 1) / 2 + 1 || a.bias_mode != 0 || a.stats || a.pro != 0) return -1;
    g.fold = 2;
    ktap = 5;
    cin_f = a.Cin;
    cout_f = 2 * a.Cout;
    g.T_tile = a.T_in;
    g.cpar = a.Cout;
    if (a.Cout % 128) return -1;
  } else {
    return -1;
  }
  // item width: 64 input channels, or 32 for the 64-channel stride-1 convs (two items per tile)
  const int kg = (g.fold == 0 && cin_f == 64) ? 32 : KG;
  if (cin_f % (2 * kg) || cout_f % 64) return -1;  // unpadded folded channels: the image is exact
  // BN = 256 (acc 256 + B ring) does not fit the register file without spills
  const int BN = cout_f % 128 == 0 ? 128 : 64;
  if (BN == 64 && kg != 32) return -1;
  g.wc32 = cout_f / 32;
  g.wk16 = cin_f / 16;
  g.F = 256 / a.V;
  g.HR = (g.F + ktap - 1) * a.V;
  if (g.HR > HR_CAP || g.F < 1) return -1;
  g.G = cin_f / kg;
  g.tiles_n = (g.T_tile + g.F - 1) / g.F;
  g.ncol = cout_f / BN;
  const long nt = (long)a.N * g.tiles_n * g.ncol;
  if (nt <= 0 || nt > 0x7fffffffL) return -1;
  g.ntiles = (int)nt;
  if (a.stats && (long)a.N * g.tiles_n > conv_rows_num_row_blocks((long)a.N * a.T_out * a.V, a.Cout)) return -1;
  // C = 64 (two 32-channel items per tile): its own tile-image buffer (SEPT) and 8 helper waves (NHW)
  const bool sep = kg == 32;
  if (sep && BN != 64) return -1;
  if (sep) {  // halo buffers sized for the halo alone; the tile image separate
    const int upr = kg / 8, nth = 8 * 64, rstep = nth / upr, na = (HR_CAP * upr + nth - 1) / nth;
    g.abytes = na * rstep * (2 * kg + 16);
    g.red_off = 2 * g.abytes + BN * CSO;
  } else {
    g.abytes = abytes_for(kg);
    g.red_off = 2 * g.abytes;
  }
  const size_t lds = (size_t)g.red_off + (size_t)WM_MAX * BN * 16 + 16;
  if (lds > (size_t)LDS_MAX) return -1;
  const int ncu = stgcn_cu_count(s);
  const int tpb = (g.ntiles + ncu - 1) / ncu;
  int grid = (g.ntiles + tpb - 1) / tpb;
  g.pair = g.ncol == 2 && ncu >= 16;
  if (g.pair) grid = ncu & ~15;
  const dim3 gd((unsigned)grid);
  auto kern = [&]() -> void (*)(const stgcn_conv_desc, const WGeom) {
    if (kg == 32)  // C = 64: 8 helper waves, separate tile image (64.6 vs 70.5 us, tools/bench_conv.py tcn_fwd_c64)
      return a.pro ? conv_wide_kernel<64, 9, 9, 1, 0, 32, 2, 1, 8, true> : conv_wide_kernel<64, 9, 9, 0, 0, 32, 2, 1, 8, true>;
    // B ring depth 8 (7 k-steps of L2 latency cover): measured 2-3 % faster than 4, 6 or 9 at C = 128/256
    if (ktap == 9) return a.pro ? conv_wide_kernel<128, 9, 8, 1> : conv_wide_kernel<128, 9, 8, 0>;
    // stride-2 folded 5-tap form: ring depth must divide 40 k-steps per item pair.  Depth 8 measured equal
    // to 5 in the full step (9.40 vs 9.39 ms, 3 interleaved runs); 10 spills (35 VGPRs).
    return a.pro ? conv_wide_kernel<128, 5, 5, 1> : conv_wide_kernel<128, 5, 5, 0>;
  };
  auto* k = kern();
  const int nhw = sep ? 8 : 4;
  const dim3 bd((unsigned)((4 + nhw) * 64));
  if (stgcn_lds_attr((const void*)k, LDS_MAX, s)) return STGCN_EHIP;
  hipLaunchKernelGGL(k, gd, bd, lds, s, a, g);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
