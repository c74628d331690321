// Micro-benchmark: how long a wave waits for a load issued right after a burst of global stores (gfx9 keeps
// one in-order vmcnt for loads and stores, so the load's wait includes the stores' completion).
// Each wave loops: [S stores of the fused layer's z shape (lane = row, 8 B, rows 128 B apart) or none]
// -> one 16-B load from a small L2-resident buffer -> s_waitcnt vmcnt(0); cycles of the wait are summed.
//   hipcc --offload-arch=gfx950 -O3 -o tools/store_lat tools/store_lat.hip && ./tools/store_lat
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void lat_kernel(u16x4* out, const uint4* w, long long* res, int mode, int iters,
                                                  int stores, long rows_per_wave) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long gw = (long)blockIdx.x * 4 + wave;
  const int lr = lane & 31, lh = lane >> 5;
  u16x4* base = out + gw * rows_per_wave * 16;  // 16 u16x4 (128 B) per row
  uint4 acc = make_uint4(0, 0, 0, 0);
  long long tw = 0;
  for (int it = 0; it < iters; ++it) {
    if (mode & 1) {
      u16x4 v = {(unsigned short)it, (unsigned short)lane, 0, 0};
      for (int q = 0; q < stores; ++q) {
        const long row = ((long)it * 32 + lr) % rows_per_wave;
        if (mode & 2)  // 16 B per lane, 8 lanes per 128-B row (whole lines)
          reinterpret_cast<uint4*>(base + row * 16)[0] = make_uint4(it, lane, q, 0);
        else
          base[row * 16 + (q & 3) * 2 + lh + (q >> 2) * 8] = v;
      }
    }
    const long long t0 = __builtin_amdgcn_s_memtime();
    const uint4 x = w[(it * 64 + lane) & 4095];
    acc.x ^= x.x;
    acc.y += x.y;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const long long t1 = __builtin_amdgcn_s_memtime();
    tw += t1 - t0;
    // some compute between iterations (like a k-loop)
    for (int d = 0; d < 64; ++d) acc.z = acc.z * 1664525u + 1013904223u;
  }
  if (lane == 0) res[gw] = tw;
  if (acc.x == 0xdeadbeef && acc.z == 7) out[0] = u16x4{1, 2, 3, 4};
}

int main() {
  const int blocks = 256, iters = 200;
  const long rows_per_wave = 32 * iters;
  u16x4* out;
  uint4* w;
  long long* res;
  hipMalloc(&out, (size_t)blocks * 4 * rows_per_wave * 128);
  hipMalloc(&w, 4096 * 16);
  hipMemset(w, 0, 4096 * 16);
  hipMalloc(&res, blocks * 4 * sizeof(long long));
  long long* h = (long long*)malloc(blocks * 4 * sizeof(long long));
  const int modes[][2] = {{0, 0}, {1, 1}, {1, 4}, {1, 16}, {3, 4}, {3, 16}};
  for (auto& m : modes) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      hipEventRecord(e0);
      hipLaunchKernelGGL(lat_kernel, dim3(blocks), dim3(256), 0, 0, out, w, res, m[0], iters, m[1], rows_per_wave);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      hipMemcpy(h, res, blocks * 4 * sizeof(long long), hipMemcpyDeviceToHost);
      double s = 0;
      for (int i = 0; i < blocks * 4; ++i) s += h[i];
      if (rep == 1)
        printf("mode %d stores %2d: load wait %8.0f cycles/iter (s_memtime), kernel %.3f ms\n", m[0], m[1],
               s / (blocks * 4) / iters, ms);
    }
  }
  return 0;
}
