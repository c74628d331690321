// Micro-benchmark for the LN one-kernel layer's WRITE_SIZE question (round-5 verdict: 114 MB counted for a 61.4 MB
// output): the same 61.44 MB of bf16 rows [M][64] (128-B rows) written by three store shapes, each a 16-B store
// per lane:
//   mode 0: the layer's epilogue shape — one instruction covers 32 rows x 32 B (lanes 2r, 2r+1 -> row r, 16 B each),
//           a row's four 32-B sectors come from four instructions;
//   mode 1: 16 rows x 64 B per instruction (4 lanes per row);
//   mode 2: 8 rows x 128 B per instruction (8 lanes per row: whole lines, the streaming shape).
// Run under rocprofv3 --pmc WRITE_SIZE (and TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum) and with its own HIP-event timing:
//   hipcc --offload-arch=gfx950 -O3 -o tools/store_pattern tools/store_pattern.hip && ./tools/store_pattern
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ __launch_bounds__(256) void store_kernel(uint4* out, long rows, int mode) {
  const int lane = threadIdx.x & 63;
  const long wave = ((long)blockIdx.x * 256 + threadIdx.x) >> 6;
  const long nwaves = ((long)gridDim.x * 256) >> 6;
  // every wave writes 32 rows x 128 B per "unit": mode 0: 4 instructions of 32 rows x 32 B;
  // mode 1: 4 instructions of 16 rows x 64 B (rows 0-15 then 16-31, two column halves); mode 2: 4 x 8 rows x 128 B
  for (long u = wave; u * 32 < rows; u += nwaves) {
    const long r0 = u * 32;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      long row;
      int unit;  // 16-B unit of the row (0..7)
      if (mode == 0) {
        row = r0 + (lane >> 1);
        unit = 2 * q + (lane & 1);
      } else if (mode == 1) {
        row = r0 + 16 * (q >> 1) + (lane >> 2);
        unit = 4 * (q & 1) + (lane & 3);
      } else {
        row = r0 + 8 * q + (lane >> 3);
        unit = lane & 7;
      }
      if (row < rows) out[row * 8 + unit] = make_uint4((unsigned)row, (unsigned)unit, (unsigned)q, 0u);
    }
  }
}

int main() {
  const long rows = 64L * 300 * 25;  // N*T*V of the north_star layer: 61.44 MB of bf16 [rows][64]
  uint4* out;
  if (hipMalloc(&out, rows * 128) != hipSuccess) return 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[3] = {"32 rows x 32 B / instr (layer epilogue)", "16 rows x 64 B / instr", "8 rows x 128 B / instr"};
  for (int mode = 0; mode < 3; ++mode) {
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(store_kernel, dim3(2048), dim3(256), 0, 0, out, rows, mode);
    hipEventRecord(e0);
    const int reps = 20;
    for (int w = 0; w < reps; ++w) hipLaunchKernelGGL(store_kernel, dim3(2048), dim3(256), 0, 0, out, rows, mode);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    ms /= reps;
    printf("mode %d %-40s %8.1f us  %7.1f GB/s (61.44 MB)\n", mode, names[mode], ms * 1e3, rows * 128 / (ms * 1e-3) / 1e9);
  }
  hipFree(out);
  return 0;
}
