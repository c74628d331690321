// Weight gradient of the (Kt x 1) row convolutions (conv_rows.hip, trans = 0):
//
//   dW[dt][co][ci] += sum_m dY[m, co] * pro(in[src(m, dt), ci])     (fp32 atomics)
//
// i.e. the convolution_backward weight path that dominates the reference's CPU profile
// (convolution_backward 40%).  The reduction over m (N*T*V rows, 480 000 at
// config 2) is a GEMM with K = m:  C[co][ci] = dY^T[co][m] * X_dt[m][ci].  Both operands are
// m-major in memory, so tiles are staged row-major in LDS as 32-column panels and the MFMA
// fragments (8 consecutive m per lane) are read with ds_read_b64_tr_b16 (bf16) — the gfx950
// transposing LDS read — or 8 scalar reads (fp32 parity path).
//
// Grid: x = m-range, y = tap dt, z = (co tile, ci tile); block tile 64(co) x 64(ci), 4 waves
// each owning a 32x32 quadrant; K walked in 32-row steps, double-buffered.
#include "common.h"

#include "../../include/stgcn_amd.h"
typedef stgcn_wgrad_desc WgradArgs;

namespace {

constexpr int MK = 32;   // rows per K step
constexpr int TC = 64;   // output tile (co and ci)

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

template <typename T>
DEV typename Tr<T>::frag tr_frag(const char* panel, int ks, int lane) {
  // element j of lane (col = lane&31, h = lane>>5) = panel[ks*16 + 8h + j][lane&31]
  if constexpr (sizeof(T) == 2) {
    const int i = lane & 15, g = lane >> 4;
    const int q = i >> 2, p = i & 3, h = g >> 1;
    const int row = ks * 16 + 8 * h + q;
    const int col = 16 * (g & 1) + 4 * p;
    const char* a0 = panel + row * 64 + col * 2;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 4 * 64));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    s16x8 v;
    v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3];
    v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
    return __builtin_bit_cast(bf16x8, v);
  } else {
    const float* pf = reinterpret_cast<const float*>(panel);
    const int c = lane & 31, h = lane >> 5;
    f32x8 f;
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = pf[(ks * 16 + 8 * h + j) * 32 + c];
    return f;
  }
}

// 16-byte unit of up to VEC elements: vector load when aligned and complete, else element loads
template <typename T>
DEV uint4 load_unit(const T* p, int avail, bool vec) {
  constexpr int VEC = 16 / sizeof(T);
  if (vec && avail >= VEC) return *reinterpret_cast<const uint4*>(p);
  T tmp[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) tmp[j] = j < avail ? p[j] : Tr<T>::from_f(0.f);
  return *reinterpret_cast<const uint4*>(tmp);
}

template <typename T>
__global__ __launch_bounds__(256) void wgrad_kernel(const WgradArgs a) {
  constexpr int VEC = 16 / sizeof(T);
  constexpr int UPR = TC / VEC;                       // units per tile row
  constexpr int UNITS = (MK * UPR + 255) / 256;        // per thread per tile
  constexpr int PANEL = MK * 32 * sizeof(T);           // bytes per 32-column panel
  constexpr int TILE = 2 * PANEL;
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILE];  // [buf][Y|X]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int dt = blockIdx.y;
  const int nct = (a.Cout + TC - 1) / TC;
  const int co0 = (blockIdx.z % nct) * TC;
  const int ci0 = (blockIdx.z / nct) * TC;
  const long M = (long)a.N * a.T_out * a.V;
  const long mb = (long)blockIdx.x * a.rows_per_block;
  const long me = mb + a.rows_per_block < M ? mb + a.rows_per_block : M;
  const int wco = wave >> 1, wci = wave & 1;

  const T* __restrict__ in = reinterpret_cast<const T*>(a.in);
  const T* __restrict__ dy = reinterpret_cast<const T*>(a.dy);

  const bool vec_y = (a.dy_ld % VEC) == 0, vec_x = (a.in_ld % VEC) == 0;
  uint4 ry[UNITS], rx[UNITS];
  int rt[UNITS];
  long rn[UNITS];
  int rv[UNITS];

  auto load = [&](long m0) {
#pragma unroll
    for (int i = 0; i < UNITS; ++i) {
      const int id = tid + i * 256;
      ry[i] = make_uint4(0, 0, 0, 0);
      rx[i] = make_uint4(0, 0, 0, 0);
      rt[i] = -1;
      if (id < MK * UPR) {
        const int r = id / UPR, cu = id % UPR;
        const long m = m0 + r;
        if (m < me) {
          const int co = co0 + cu * VEC;
          if (co < a.Cout) ry[i] = load_unit(dy + m * a.dy_ld + co, a.Cout - co, vec_y);
          const int v = (int)(m % a.V);
          const long nt = m / a.V;
          const int t = (int)(nt % a.T_out);
          const long n = nt / a.T_out;
          const int t_in = t * a.stride + dt - a.pad;
          const int ci = ci0 + cu * VEC;
          if (t_in >= 0 && t_in < a.T_in && ci < a.Cin) {
            rx[i] = load_unit(in + ((n * a.T_in + t_in) * a.V + v) * a.in_ld + ci, a.Cin - ci, vec_x);
            rt[i] = t_in;
            rn[i] = n;
            rv[i] = v;
          }
        }
      }
    }
  };
  auto store = [&](int buf) {
    char* sy = smem + buf * 2 * TILE;
    char* sx = sy + TILE;
#pragma unroll
    for (int i = 0; i < UNITS; ++i) {
      const int id = tid + i * 256;
      if (id < MK * UPR) {
        const int r = id / UPR, cu = id % UPR;
        const int col = cu * VEC;
        uint4 vx = rx[i];
        if (a.pro != 0 && rt[i] >= 0) {
          float f[VEC];
          unpack16(vx, f, (T*)nullptr);
          const int ci = ci0 + col;
          if (a.pro == 1) {
#pragma unroll
            for (int j = 0; j < VEC; ++j) f[j] = fmaxf(f[j] * a.pro_a[ci + j] + a.pro_b[ci + j], 0.f);
          } else {
            const float2 st = reinterpret_cast<const float2*>(a.pro_stats)[rn[i] * a.T_in + rt[i]];
#pragma unroll
            for (int j = 0; j < VEC; ++j) {
              const int g = (ci + j) * a.V + rv[i];
              f[j] = fmaxf((f[j] - st.x) * st.y * a.pro_a[g] + a.pro_b[g], 0.f);
            }
          }
          vx = pack16(f, (T*)nullptr);
        }
        const int off = (col / 32) * PANEL + r * 32 * (int)sizeof(T) + (col % 32) * (int)sizeof(T);
        *reinterpret_cast<uint4*>(sy + off) = ry[i];
        *reinterpret_cast<uint4*>(sx + off) = vx;
      }
    }
  };

  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;

  if (mb < me) {
    load(mb);
    store(0);
  }
  __syncthreads();
  int cur = 0;
  for (long m0 = mb; m0 < me; m0 += MK) {
    const bool more = m0 + MK < me;
    if (more) load(m0 + MK);
    const char* sy = smem + cur * 2 * TILE;
    const char* sx = sy + TILE;
#pragma unroll
    for (int ks = 0; ks < MK / 16; ++ks) {
      typename Tr<T>::frag fa = tr_frag<T>(sy + wco * PANEL, ks, lane);
      typename Tr<T>::frag fb = tr_frag<T>(sx + wci * PANEL, ks, lane);
      Tr<T>::mma(acc, fa, fb);
    }
    if (more) store(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  const int ci = ci0 + wci * 32 + (lane & 31);
  if (ci < a.Cin) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = co0 + wco * 32 + acc_row(r, lane);
      if (co < a.Cout) atomicAdd(a.dw + ((long)dt * a.Cout + co) * a.Cin + ci, acc[r]);
    }
  }
}

}  // namespace

int conv_wgrad_launch(WgradArgs a, int dtype, hipStream_t s) {
  const long M = (long)a.N * a.T_out * a.V;
  const int tiles = ((a.Cout + TC - 1) / TC) * ((a.Cin + TC - 1) / TC);
  // aim for ~2048 blocks in total, at least 512 rows per block
  long target = 2048 / ((long)tiles * a.Kt);
  if (target < 1) target = 1;
  long rpb = (M + target - 1) / target;
  if (rpb < 512) rpb = 512;
  rpb = (rpb + MK - 1) / MK * MK;
  a.rows_per_block = rpb;
  dim3 grid((unsigned)((M + rpb - 1) / rpb), (unsigned)a.Kt, (unsigned)tiles);
  if (dtype == 1)
    hipLaunchKernelGGL(wgrad_kernel<bf16>, grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(wgrad_kernel<float>, grid, dim3(256), 0, s, a);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
