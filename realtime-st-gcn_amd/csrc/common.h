// Shared device helpers for the MI355X (gfx950, CDNA4) ST-GCN kernels.
//
// Layout convention: every activation tensor is the reference's logical
// (N, C, T, V) tensor stored CHANNELS-LAST, i.e. physically [N][T][V][C] ("rows" of C
// contiguous channels, row index m = (n*T + t)*V + v).  Element types: fp32 (parity path)
// and bf16 (perf path); accumulation is always fp32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x8 __attribute__((ext_vector_type(8)));

#define DEV __device__ __forceinline__

// ------------------------------------------------------------------------------------------
// Element traits.  A "fragment" is the 8 consecutive-k values one lane contributes to one
// 32x32 MFMA k-step of 16 (lane l: row/col l&31, k = 8*(l>>5) + j, j = 0..7).
//   bf16: one v_mfma_f32_32x32x16_bf16.
//   fp32: eight v_mfma_f32_32x32x2_f32, instruction j consuming element j of both operands
//         (a relabelling of the k axis that keeps the bf16 lane map: exact fp32 products).
// ------------------------------------------------------------------------------------------
template <typename T> struct Tr;

template <> struct Tr<float> {
  typedef f32x8 frag;
  static constexpr int VEC = 4;  // elements per 16-byte unit
  static DEV float to_f(float v) { return v; }
  static DEV float from_f(float v) { return v; }
  static DEV void mma(f32x16& acc, const frag& a, const frag& b) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[j], b[j], acc, 0, 0, 0);
  }
};

template <> struct Tr<bf16> {
  typedef bf16x8 frag;
  static constexpr int VEC = 8;
  static DEV float to_f(bf16 v) { return (float)v; }
  static DEV bf16 from_f(float v) { return (bf16)v; }
  static DEV void mma(f32x16& acc, const frag& a, const frag& b) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
  }
};

// 16-byte unit <-> 8 floats (bf16) or 4 floats (fp32)
// Channel of block b in a one-block-per-channel reduction over [nb][C] partial rows (grid = C): workgroups
// are dealt round-robin to the 8 XCDs, so with c = b every 128-B line of partials (8 float4 channels) was
// fetched into all eight L2s; this mapping gives each XCD a contiguous channel range (C % 64 == 0), so each
// line goes to one L2.
DEV int xcd_channel(int b, int C) { return (C & 63) ? b : (b & 7) * (C >> 3) + (b >> 3); }

DEV void unpack16(const uint4& u, float* f, bf16*) {
  const bf16x8 v = __builtin_bit_cast(bf16x8, u);
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (float)v[j];
}
DEV void unpack16(const uint4& u, float* f, float*) {
  const f32x4 v = __builtin_bit_cast(f32x4, u);
#pragma unroll
  for (int j = 0; j < 4; ++j) f[j] = v[j];
}
DEV uint4 pack16(const float* f, bf16*) {
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (bf16)f[j];
  return __builtin_bit_cast(uint4, v);
}
DEV uint4 pack16(const float* f, float*) {
  f32x4 v;
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = f[j];
  return __builtin_bit_cast(uint4, v);
}

// C/D map of the 32x32 MFMAs (dtype independent on gfx950): col = lane&31,
// row = (r&3) + 8*(r>>2) + 4*(lane>>5), r = accumulator register 0..15.
DEV int acc_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// Chan's parallel combination of (count, mean, M2) triples (numerically robust variance).
struct Welford {
  float n, mean, m2;
};
DEV Welford welford_merge(Welford a, Welford b) {
  const float n = a.n + b.n;
  if (n == 0.f) return a;
  const float d = b.mean - a.mean;
  const float fb = b.n / n;
  Welford r;
  r.n = n;
  r.mean = a.mean + d * fb;
  r.m2 = a.m2 + b.m2 + d * d * a.n * fb;
  return r;
}

DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// status codes of the C-ABI (include/stgcn_amd.h)
#define STGCN_OK 0
#define STGCN_EBADSHAPE 1
#define STGCN_EDTYPE 2
#define STGCN_EHIP 3

// Per-device launcher state (runtime.cpp): the CU count of the stream's device, and a one-time (per kernel
// and device) raise of a kernel's dynamic LDS limit.  Thread-safe; no other mutable state in the launchers.
int stgcn_cu_count(hipStream_t s);
int stgcn_lds_attr(const void* kernel, int bytes, hipStream_t s);
