// Dense joint mixing on the matrix cores: the per-sample (AAGCN) graph-conv mixes and the attention
// backward mixes, frame by frame.
//
//   mode 0 (expand, amix fwd,  tgcn.py:76):    out[(i,a)][p*C + c]  = sum_b M[p][b][a] in[(i,b)][c]
//   mode 1 (reduce, amix trans, its autograd):  out[(i,a)][c]       (+)= sum_p sum_b M[p][a][b] in[(i,b)][p*C + c]
//   mode 2 (grouped, attention bwd, aagcn.py:142-145 autograd):
//                                               out[(i,a)][p*C + c]  = sum_b Mg[p][a][b] in[(i,b)][p*C + c]
//                                               Mg = M (bt = 1) or M^T (bt = 0)
// with M [P][V][V] fp32 shared or per sample n (i = n*T + t).  These mixes are dense for AAGCN (A + B + C
// with C a softmax), 25 coefficients per output element: the earlier gather kernels issued 25-75 loads
// per output unit and ran at 5-15 % of HBM bandwidth.  Here a frame's 32-channel input block (V <= 32
// joint rows) is DMA'd into an LDS panel and mixed as Y^T = X^T M (32 x 32, K = joints) on MFMA:
//   bf16: 32x32x16 MFMAs, X^T fragments by transposing LDS reads (ds_read_tr16_b64), the coefficients in
//         registers as a hi + lo bf16 pair (two MFMAs: ~fp32 coefficient precision; rounding them to bf16
//         alone would add 2^-9 relative error per coefficient);
//   fp32: 32x32x2 fp32 MFMAs (exact fp32 products), one LDS read per fragment.
// Work item = (frame, 32-channel output block); a wave walks a contiguous run of items (the coefficients
// are reloaded only when the sample changes), through a ring of 2-5 item slots: the next items' panels (and,
// accumulating, the old output block, DMA'd like an input panel) are in flight while the current one is mixed,
// and the counted vmcnt wait before an item never waits for the stores of the last slots' items (vmcnt
// completes in order: waiting behind a store's write latency per item had serialised the waves).
// Output: lane = output joint, 4 consecutive channels per store.
#include "common.h"
#include <type_traits>

namespace {

constexpr int NWJ = 4;             // waves per block
// item slots per wave: 2..5, as many as keep a block's ring within 80 KB of LDS (two blocks per CU)
constexpr int jmix_nbuf(int panel, int ns) {
  const int n = (80 * 1024) / (NWJ * ns * panel);
  return n < 2 ? 2 : (n > 5 ? 5 : n);
}
constexpr int PMAXJ = 3;
constexpr int ITEMS_PER_WAVE = 16;  // target work items per wave (sizes the grid)

template <typename T> struct JT;
template <> struct JT<bf16> {
  static constexpr int KS = 2;       // k-steps of 16 joints
  static constexpr int PANEL = 32 * 64;  // [32 rows][32 ch] bf16
};
template <> struct JT<float> {
  static constexpr int KS = 16;      // k-steps of 2 joints
  static constexpr int PANEL = 32 * 128;
};

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// A operand (m = channel, k = 16 joints from row0) of a 32x32x16 MFMA from a [row][32 ch] bf16 panel
DEV bf16x8 trfrag16(const char* panel, int row0, int lane) {
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

// 16 B per lane, global -> LDS (lane-linear from lds_off).  Issued from asm so the compiler does not treat
// later LDS reads as aliasing the copy and drain vmcnt before each of them (the ring would serialise);
// ordering is by the explicit vmcnt waits.  m0 is saved and restored inside the asm (never clobbered).
DEV void dma16(const void* src, unsigned lds_off) {
  unsigned saved;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(saved) : "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds_off)) : "memory");
}
DEV unsigned lds_u32(const void* p) { return (unsigned)(size_t)(const __attribute__((address_space(3))) char*)p; }

// s_waitcnt vmcnt(n) for a wave-uniform run-time n (clamped to 63; waiting for fewer is always safe)
template <int N>
DEV void wait_vm_upto(int n) {
  if constexpr (N < 63) {
    if (n <= N) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
      return;
    }
    wait_vm_upto<N + 1>(n);
  } else {
    asm volatile("s_waitcnt vmcnt(63)" ::: "memory");
  }
}
DEV void wait_vm(int n) { wait_vm_upto<0>(n < 0 ? 0 : n); }

struct JmixArgs {
  const void* in;
  void* out;
  const float* M;
  int N, T, V, P, C;
  int in_ld, out_ld;
  int mode, bt, per_sample, accumulate;
  int nob;      // 32-channel output blocks per frame
  int npan;     // input panels per item (mode 1: P, else 1)
  long items;   // N*T*nob
  long ipw;     // items per wave
  int cout;     // output channels per row (mode 0/2: P*C, mode 1: C)
  int cin;      // input channels per row (mode 0: C, else P*C)
};

template <typename T, int NP, bool ACC>
__global__ __launch_bounds__(NWJ * 64) void jmix_kernel(const JmixArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int PANEL = JT<T>::PANEL, KS = JT<T>::KS;
  constexpr int ELT = (int)sizeof(T);
  constexpr int UPR = 32 * ELT / 16;  // 16-B units per panel row
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lr = lane & 31, lh = lane >> 5;
  const int V = a.V;
  constexpr int NS = NP + (ACC ? 1 : 0);  // panels per slot: the inputs, then (accumulating) the old output block
  constexpr int NBUF = jmix_nbuf(PANEL, NS);  // item slots per wave: the current item and the ones in flight
  char* const buf = smem + wave * NBUF * NS * PANEL;  // [NBUF][NS] panels
  // rows V..31 stay zero (the DMA never writes them)
  for (int e = lane; e < NBUF * NS * PANEL / 16; e += 64) reinterpret_cast<uint4*>(buf)[e] = make_uint4(0, 0, 0, 0);
  __builtin_amdgcn_s_waitcnt(0);

  const long gw = (long)blockIdx.x * NWJ + wave;
  const long it0 = gw * a.ipw, it1 = min(a.items, it0 + a.ipw);
  if (it0 >= it1) return;  // wave-uniform; no block barriers below
  const T* __restrict__ in = reinterpret_cast<const T*>(a.in);
  T* __restrict__ out = reinterpret_cast<T*>(a.out);

  // item -> (frame i, output block ob, panel column bases)
  auto panel_col = [&](int ob, int k) {  // input channel base of panel k of block ob
    if (a.mode == 0) return (32 * ob) % a.C;
    if (a.mode == 1) return k * a.C + 32 * ob;
    return 32 * ob;
  };
  const int lrow = lane / UPR, lunit = lane % UPR;
  constexpr int RPI = 64 / UPR;  // panel rows per DMA instruction
  // Every lane issues every DMA instruction (a fixed count per item, DOPS, for the counted waits below):
  // lanes past the frame's V rows or past a partial last channel block (mode 2) copy the frame's first
  // unit instead — finite data, multiplied by zero coefficients (rows >= V) or masked (channels).
  auto issue_io = [&](long i, int ob, int slot) {
    const T* src0 = in + i * V * (long)a.in_ld;
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const unsigned pan = lds_u32(buf + (slot * NS + k) * PANEL);
      const int cb = panel_col(ob, k);
      const bool uok = cb + lunit * (16 / ELT) < a.cin;
#pragma unroll
      for (int rr = 0; rr < 32; rr += RPI) {
        const int row = rr + lrow;
        const bool ok = row < V && uok;
        dma16(ok ? src0 + (long)row * a.in_ld + cb + lunit * (16 / ELT) : src0, pan + rr * 32 * ELT);
      }
    }
    if constexpr (ACC) {  // the old output block [V rows][32 channels], read back in the flush from LDS
      const T* o0 = out + i * V * (long)a.out_ld + 32 * ob;
      const unsigned pan = lds_u32(buf + (slot * NS + NP) * PANEL);
      const bool uok = 32 * ob + lunit * (16 / ELT) < a.cout;
#pragma unroll
      for (int rr = 0; rr < 32; rr += RPI) {
        const int row = rr + lrow;
        const bool ok = row < V && uok;
        dma16(ok ? o0 + (long)row * a.out_ld + lunit * (16 / ELT) : o0, pan + rr * 32 * ELT);
      }
    }
  };
  // coefficients of one sample as B operands: B[k = in joint b][n = out joint a] = coef(a, b, p)
  //   mode 0: M[p][b][a]; mode 1: M[p][a][b]; mode 2: bt ? M[p][a][b] : M[p][b][a]
  const bool ab = a.mode == 1 || (a.mode == 2 && a.bt);
  auto coef = [&](const float* Mn, int p, int b) {
    const int o = lr;
    if (o >= V || b >= V) return 0.f;
    return ab ? Mn[(p * V + o) * V + b] : Mn[(p * V + b) * V + o];
  };
  typedef std::conditional_t<sizeof(T) == 2, bf16x8, float> Frag;
  Frag bh[PMAXJ][KS], bl[PMAXJ][KS];
  long cur_n = -1;
  auto load_coef = [&](long n) {
    const float* Mn = a.M + (a.per_sample ? n * a.P * V * V : 0);
#pragma unroll
    for (int p = 0; p < PMAXJ; ++p) {
      if (p >= a.P) break;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        if constexpr (sizeof(T) == 2) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float c = coef(Mn, p, 16 * ks + 8 * lh + j);
            const bf16 h = (bf16)c;
            bh[p][ks][j] = h;
            bl[p][ks][j] = (bf16)(c - (float)h);
          }
        } else {
          bh[p][ks] = coef(Mn, p, 2 * ks + lh);
        }
      }
    }
  };

  typedef std::conditional_t<sizeof(T) == 2, bf16x4, float4> OVec;
  const f32x16 zero = {};
  f32x16 pend = zero;  // the item's results
  long pend_i = -1;
  int pend_ob = 0, pend_slot = 0;
  auto out_ptr = [&](long i, int ob, int q4) {
    return out + (i * V + lr) * (long)a.out_ld + 32 * ob + 8 * q4 + 4 * lh;
  };
  auto ch_ok = [&](int ob, int q4) { return lr < V && 32 * ob + 8 * q4 + 4 * lh < a.cout; };
  auto flush = [&]() {
    if (pend_i < 0) return;
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) {
      if (!ch_ok(pend_ob, q4)) continue;
      float v[4] = {pend[4 * q4], pend[4 * q4 + 1], pend[4 * q4 + 2], pend[4 * q4 + 3]};
      if constexpr (ACC) {  // old output: row lr, channels 8*q4 + 4*lh .. +3 of the slot's output panel
        const OVec o = *reinterpret_cast<const OVec*>(buf + (pend_slot * NS + NP) * PANEL + lr * 32 * ELT +
                                                      (8 * q4 + 4 * lh) * ELT);
        if constexpr (sizeof(T) == 2) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += (float)o[e];
        } else {
          v[0] += o.x; v[1] += o.y; v[2] += o.z; v[3] += o.w;
        }
      }
      if constexpr (sizeof(T) == 2) {
        bf16x4 r;
#pragma unroll
        for (int e = 0; e < 4; ++e) r[e] = (bf16)v[e];
        *reinterpret_cast<bf16x4*>(out_ptr(pend_i, pend_ob, q4)) = r;
      } else {
        *reinterpret_cast<float4*>(out_ptr(pend_i, pend_ob, q4)) = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
  };

  // store instructions of an item: the 8-channel quarters with any channel below cout (an instruction whose
  // lanes are all masked is branched over and does not count on vmcnt)
  auto nstores = [&](int ob) {
    int n = 0;
#pragma unroll
    for (int q4 = 0; q4 < 4; ++q4) n += 32 * ob + 8 * q4 < a.cout ? 1 : 0;
    return n;
  };
  {
    // Order per item j: [wait: panels(j)] [mix(j)] [DMA(j+AH)] [stores(j)], AH = NBUF - 1 items in flight.
    // vmcnt completes in order, so the wait before item j counts exactly the ops issued after DMA(j): the DMAs
    // of the next items already issued and the stores of the last AH items — a store is waited for only AH
    // items after it (waiting for the previous item's stores had serialised the items behind the write
    // latency).  Item -> (frame, block) and the sample advance by counters: no 64-bit division per item.
    constexpr int AH = NBUF - 1;
    constexpr int DOPS = NS * (32 / RPI);
    long ci = it0 / a.nob;  // item j's frame and block
    int cob = (int)(it0 - ci * a.nob);
    long ii = ci;  // next item to issue
    int iob = cob;
    auto adv = [&](long& f, int& o) {
      if (++o == a.nob) {
        o = 0;
        ++f;
      }
    };
    long oi = ci;  // item j - AH (its stores leave the wait count once j passes it)
    int oob = cob;
    for (int k = 0; k < AH && it0 + k < it1; ++k) {
      issue_io(ii, iob, k);
      adv(ii, iob);
    }
    int nsum = 0;  // store instructions of items max(it0, j-AH) .. j-1
    int slot = 0, islot = AH;
    long nt = ci / a.T, tt = ci - nt * a.T;  // sample and frame-in-sample of item j's frame
    for (long it = it0; it < it1; ++it) {
      const long i = ci;
      const int ob = cob;
      const long ndma = it1 - 1 - it < AH - 1 ? it1 - 1 - it : AH - 1;
      wait_vm((int)ndma * DOPS + nsum);
      const long n = nt;
      if (n != cur_n) {
        load_coef(n);
        cur_n = n;
      }
    f32x16 acc = zero;
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const char* pan = buf + (slot * NS + k) * PANEL;
      // partitions feeding this (block, panel) and the channel rows each one owns (mode 2: groups of C)
      int p0, p1;
      if (a.mode == 0) p0 = p1 = (32 * ob) / a.C;
      else if (a.mode == 1) p0 = p1 = k;
      else {
        p0 = (32 * ob) / a.C;
        p1 = min(a.P - 1, (32 * ob + 31) / a.C);
      }
#pragma unroll
      for (int p = 0; p < PMAXJ; ++p) {  // compile-time p: the coefficient registers are never indexed at run time
        if (p < p0 || p > p1) continue;
        bool mok = true;  // this lane's A row (channel m = lr) belongs to partition p
        if (a.mode == 2) {
          const int ch = 32 * ob + lr;
          mok = ch >= p * a.C && ch < (p + 1) * a.C;
        }
        if constexpr (sizeof(T) == 2) {
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) {
            bf16x8 af = trfrag16(pan, 16 * ks, lane);
            if (!mok) af = bf16x8{};
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bh[p][ks], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bl[p][ks], acc, 0, 0, 0);
          }
        } else {
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) {
            if (2 * ks >= V) break;
            float av = *reinterpret_cast<const float*>(pan + ((2 * ks + lh) * 32 + lr) * 4);
            av = mok ? av : 0.f;
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bh[p][ks], acc, 0, 0, 0);
          }
        }
      }
    }
    // D: lane = output joint lr, acc[r] = channel 32*ob + 8*(r>>2) + 4*lh + (r&3); stored next item
    pend = acc;
    pend_i = i;
    pend_ob = ob;
    pend_slot = slot;
      if (it + AH < it1) {
        issue_io(ii, iob, islot);
        adv(ii, iob);
        islot = islot + 1 == NBUF ? 0 : islot + 1;
      }
      flush();
      nsum += nstores(ob);
      if (it - it0 >= AH) {  // item j-AH leaves the window of item j+1
        nsum -= nstores(oob);
        adv(oi, oob);
      }
      slot = slot + 1 == NBUF ? 0 : slot + 1;
      adv(ci, cob);
      if (cob == 0 && ++tt == a.T) {
        tt = 0;
        ++nt;
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return;
  }
}

}  // namespace

// Shapes served (else the caller keeps its gather kernel): V <= 32, P <= 4; mode 0/1: C % 32 == 0;
// mode 2: C % 4 == 0 and P*C a multiple of 4; rows 16-B aligned.  Returns -1 when not served.
int jmix_launch(const void* in, int in_ld, void* out, int out_ld, const float* M, int N, int T, int V, int P, int C,
                int mode, int bt, int per_sample, int accumulate, int dtype, hipStream_t s) {
  const int elt = dtype ? 2 : 4;
  const int cin = mode == 1 ? P * C : (mode == 0 ? C : P * C);
  const int cout = mode == 1 ? C : P * C;
  if (V < 1 || V > 32 || P < 1 || P > PMAXJ) return -1;
  if (mode == 1 && P > 3) return -1;
  if ((mode == 0 || mode == 1) && C % 32) return -1;
  if (mode == 2 && (C % 4 || cout % 4)) return -1;
  if ((in_ld * elt) % 16 || (out_ld * elt) % 16 || in_ld < cin || out_ld < cout) return -1;
  const int nob = (cout + 31) / 32;
  JmixArgs a;
  a.in = in; a.out = out; a.M = M;
  a.N = N; a.T = T; a.V = V; a.P = P; a.C = C;
  a.in_ld = in_ld; a.out_ld = out_ld;
  a.mode = mode; a.bt = bt; a.per_sample = per_sample; a.accumulate = accumulate;
  a.nob = nob;
  a.npan = mode == 1 ? P : 1;
  a.cout = cout;
  a.cin = cin;
  a.items = (long)N * T * nob;
  const int ncu = stgcn_cu_count(s);
  long waves = a.items / ITEMS_PER_WAVE;
  // one round of resident waves (2 per SIMD at the kernel's ~210 VGPRs): more waves only queue behind them
  const long wmax = (long)(ncu > 0 ? ncu : 256) * 2 * NWJ;
  if (waves > wmax) waves = wmax;
  if (waves < 1) waves = 1;
  a.ipw = (a.items + waves - 1) / waves;
  const long blocks = (a.items + a.ipw * NWJ - 1) / (a.ipw * NWJ);
  const int panel = dtype ? JT<bf16>::PANEL : JT<float>::PANEL;
  const int ns = a.npan + (accumulate ? 1 : 0);
  const size_t lds = (size_t)NWJ * jmix_nbuf(panel, ns) * ns * panel;
#define JM_LAUNCH1(TT, NPV, AC)                                                                               \
  do {                                                                                                       \
    if (stgcn_lds_attr((const void*)jmix_kernel<TT, NPV, AC>, (int)lds, s)) return STGCN_EHIP;                \
    hipLaunchKernelGGL((jmix_kernel<TT, NPV, AC>), dim3((unsigned)blocks), dim3(NWJ * 64), lds, s, a);        \
  } while (0)
#define JM_LAUNCH(TT, NPV)                   \
  do {                                       \
    if (accumulate) JM_LAUNCH1(TT, NPV, true); \
    else JM_LAUNCH1(TT, NPV, false);         \
  } while (0)
  if (dtype) {
    if (a.npan == 1) JM_LAUNCH(bf16, 1);
    else if (a.npan == 2) JM_LAUNCH(bf16, 2);
    else JM_LAUNCH(bf16, 3);
  } else {
    if (a.npan == 1) JM_LAUNCH(float, 1);
    else if (a.npan == 2) JM_LAUNCH(float, 2);
    else JM_LAUNCH(float, 3);
  }
#undef JM_LAUNCH
#undef JM_LAUNCH1
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
