// Batched weight preparation: every packed operand of a model's training step in one launch (include/
// stgcn_amd.h, stgcn_prep_*).  The jobs are the single-job pack / fragment-image / effective-weight kernels
// (pack.h bodies, identical per-element arithmetic); each 256-thread block finds its job by a binary search
// over block_start and runs that job's body for its thread index.  Bound: launch latency — ~50 small kernels
// (4-18 us each in the config-2 step, tens of MB in total) become one grid that streams the same bytes.
#include "common.h"
#include "pack.h"
#include "../../include/stgcn_amd.h"

namespace {

constexpr int PREP_LDS_STARTS = 512;  // job starts searched in LDS (larger tables: the search reads global memory)

__global__ __launch_bounds__(256) void prep_kernel(const stgcn_prep_job* __restrict__ jobs,
                                                   const long* __restrict__ start, int njobs) {
  // Every block pays this prologue before its job's own loads: the starts are fetched by one load per thread
  // into LDS and searched there (a binary search over global memory was ~6 dependent load latencies per
  // block, with ~8 k blocks in the config-2 step's launch), and the job index is made wave-uniform so the
  // job's fields come through scalar loads.
  const long b = blockIdx.x;
  __shared__ long sst[PREP_LDS_STARTS];
  const bool lds = njobs <= PREP_LDS_STARTS;
  if (lds) {
    for (int t = threadIdx.x; t < njobs; t += blockDim.x) sst[t] = start[t];
    __syncthreads();
  }
  int lo = 0, hi = njobs - 1;  // last job with start[j] <= b
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if ((lds ? sst[mid] : start[mid]) <= b) lo = mid;
    else hi = mid - 1;
  }
  lo = __builtin_amdgcn_readfirstlane(lo);
  const stgcn_prep_job& j = jobs[lo];
  const long j0 = lds ? sst[lo] : start[lo];
  __shared__ float colsum[GW_COLSUM_MAX];
  if ((j.kind == 2 && j.bias2d) || j.kind == 3) gconv_colsum_block(j.A, j.M, j.P, j.V, colsum);  // block-uniform
  const long i = (b - j0) * 256 + threadIdx.x;
  if (i >= j.threads) return;
  if (j.kind == 0) {
    if (j.dtype == 1)
      pack_weight_elem<bf16>(j.src, j.s0, j.s1, j.s2, j.Co, j.Ci, j.cp, j.kp, i, (bf16*)j.dst, (bf16*)j.dst_frag);
    else
      pack_weight_elem<float>(j.src, j.s0, j.s1, j.s2, j.Co, j.Ci, j.cp, j.kp, i, (float*)j.dst, (float*)j.dst_frag);
  } else if (j.kind == 1) {
    const int co_f = j.trans ? 2 * j.Co : j.Co, ci_f = j.trans ? j.Ci : 2 * j.Ci;
    pack_s2frag_elem(j.src, j.s0, j.s1, j.s2, j.Co, j.Ci, j.trans, co_f, ci_f, i, (bf16*)j.dst);
  } else if (j.kind == 3) {
    // the graph-conv bias pushed through A alone (frame-kernel route, gcn_frame.hip): thread = (joint, channel)
    const int a = (int)(i / j.Co), r = (int)(i - (long)a * j.Co);
    float sb = 0.f;
    for (int p = 0; p < j.P; ++p) sb += j.bconv[p * j.Co + r] * colsum[p * j.V + a];
    j.bias2d[(long)a * j.Co + r] = sb;
  } else {
    if (j.dtype == 1)
      gconv_weights_elem<bf16>(j.A, j.M, j.src, j.nbr, j.deg, j.P, j.V, j.J, j.Co, j.Ci, j.trans, (bf16*)j.dst,
                               j.R_pad, j.C_pad, j.bconv, j.bias2d, colsum, i);
    else
      gconv_weights_elem<float>(j.A, j.M, j.src, j.nbr, j.deg, j.P, j.V, j.J, j.Co, j.Ci, j.trans, (float*)j.dst,
                                j.R_pad, j.C_pad, j.bconv, j.bias2d, colsum, i);
  }
}

}  // namespace

extern "C" int stgcn_prep_check(stgcn_prep_job* jobs, int njobs) {
  if (!jobs || njobs <= 0) return STGCN_EBADSHAPE;
  for (int k = 0; k < njobs; ++k) {
    stgcn_prep_job& j = jobs[k];
    if (j.dtype != 0 && j.dtype != 1) return STGCN_EDTYPE;
    if (!j.src || !j.dst || j.Co <= 0 || j.Ci <= 0) return STGCN_EBADSHAPE;
    if (j.kind == 0) {
      if (j.Kt <= 0 || j.cp < j.Co || j.kp < j.Ci) return STGCN_EBADSHAPE;
      if (j.kp % 8 || (j.dst_frag && (j.cp % 32 || j.kp % 16))) return STGCN_EBADSHAPE;
      j.threads = (long)j.Kt * j.cp * j.kp / 8;
    } else if (j.kind == 1) {
      if (j.dtype != 1) return STGCN_EDTYPE;
      const int co_f = j.trans ? 2 * j.Co : j.Co, ci_f = j.trans ? j.Ci : 2 * j.Ci;
      if (co_f % 32 || ci_f % 16 || j.Ci % 8 || j.Co % 8) return STGCN_EBADSHAPE;
      j.threads = 5L * co_f * ci_f / 8;
    } else if (j.kind == 2) {
      if (!j.A || !j.nbr || !j.deg || j.P <= 0 || j.P > GW_PMAX || j.V <= 0 || j.J <= 0 || j.C_pad % 8 ||
          j.R_pad < (j.trans ? j.Ci : j.Co) || j.C_pad < (j.trans ? j.Co : j.Ci) ||
          (j.bias2d && (j.trans || !j.bconv || j.P * j.V > GW_COLSUM_MAX)))
        return STGCN_EBADSHAPE;
      j.threads = (long)j.V * j.R_pad * (j.C_pad / 8);
    } else if (j.kind == 3) {
      if (!j.A || !j.bconv || !j.bias2d || j.P <= 0 || j.P > GW_PMAX || j.V <= 0 || j.P * j.V > GW_COLSUM_MAX)
        return STGCN_EBADSHAPE;
      j.threads = (long)j.V * j.Co;
    } else {
      return STGCN_EBADSHAPE;
    }
  }
  return STGCN_OK;
}

extern "C" int stgcn_prep_run(const stgcn_prep_job* jobs_dev, const long* block_start_dev, int njobs, long nblocks,
                              void* stream) {
  if (!jobs_dev || !block_start_dev || njobs <= 0 || nblocks <= 0 || nblocks > 0x7fffffffL) return STGCN_EBADSHAPE;
  hipLaunchKernelGGL(prep_kernel, dim3((unsigned)nblocks), dim3(256), 0, (hipStream_t)stream, jobs_dev,
                     block_start_dev, njobs);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
