// Segment metrics of one trial on the GPU (evaluation): segmental F1@k (Lea et al.,
// utils/metrics/f1.py:14-67), segmental edit score (Levenshtein over segment labels, utils/metrics/edit.py:
// 10-38) and the framewise confusion matrix (utils/metrics/confusion.py:10-29), with the segment edges of
// utils/metrics/metric.py:14-28 (a segment starts where the label changes).  The reference runs these as
// Python loops over segments (O(m*n) interpreter steps per trial); here ONE wave does a trial:
//   * segment extraction: ballot + popcount compaction of the change points, 64 frames per step;
//   * F1: for each predicted segment i in order, the IoU with every ground-truth segment (lanes), a wave
//     argmax (first maximum, as torch.argmax), then the hit / false-positive bookkeeping with the "ground
//     truth already matched" flags as an LDS bitmask (sequential in i, exactly as the reference);
//   * edit: the (m+1) x (n+1) DP on anti-diagonals, three diagonals in LDS, the shorter sequence as rows;
//   * confusion: cm[pred][label] += 1 (64-bit atomics; integer, so order-independent).
// Arithmetic follows the reference's dtypes: IoU = float(inter) / float(union) * (class match), precision
// and recall float32 ratios of integer counts, F1 = 2 * P * R / (P + R) (NaN when the trial has no hit),
// edit = 1 - D[m][n] / max(m, n).  Integer work is exact; the float results are bit-identical.
#include "common.h"

namespace {

constexpr int KMAX = 8;        // IoU thresholds
constexpr int RMAX = 8192;     // rows of the edit DP (the shorter segment sequence)

__global__ __launch_bounds__(64) void seg_metrics_kernel(const long* __restrict__ lab, const long* __restrict__ pred,
                                                         int L, int C, const float* __restrict__ ov, int K,
                                                         int* __restrict__ ws, unsigned long long* cm,
                                                         float* __restrict__ out, int* __restrict__ status) {
  extern __shared__ __attribute__((aligned(16))) int lds[];
  const int lane = threadIdx.x;
  int* ls = ws;              // label segment starts [L + 1]
  int* lc = ls + (L + 1);    // label segment classes [L]
  int* ps = lc + L;          // predicted segment starts [L + 1]
  int* pc = ps + (L + 1);    // predicted segment classes [L]

  auto extract = [&](const long* x, int* st, int* cl) {
    int cnt = 0;
    for (int base = 0; base < L; base += 64) {
      const int t = base + lane;
      const bool f = t < L && (t == 0 || x[t] != x[t - 1]);
      const unsigned long long b = __ballot(f);
      const int pos = cnt + __popcll(b & ((1ull << lane) - 1ull));
      if (f) {
        st[pos] = t;
        cl[pos] = (int)x[t];
      }
      cnt += __popcll(b);
    }
    if (lane == 0) st[cnt] = L;
    return cnt;
  };
  const int n = extract(lab, ls, lc);   // ground-truth segments
  const int m = extract(pred, ps, pc);  // predicted segments
  __threadfence_block();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the wave's segment stores are visible to its loads

  if (cm)
    for (int t = lane; t < L; t += 64) {
      const long p = pred[t], l = lab[t];
      if (p >= 0 && p < C && l >= 0 && l < C) atomicAdd(cm + p * C + l, 1ull);
    }

  // ---- F1@k
  unsigned* used = reinterpret_cast<unsigned*>(lds);  // bit (j*K + k): ground-truth segment j matched at k
  const int uw = (n * K + 31) / 32;
  for (int w = lane; w < uw; w += 64) used[w] = 0u;
  int tp[KMAX], fp[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) tp[k] = fp[k] = 0;
  for (int i = 0; i < m; ++i) {
    const int s = ps[i], e = ps[i + 1], c = pc[i];
    float best = -INFINITY;
    int bj = 0x7fffffff;
    for (int j = lane; j < n; j += 64) {
      const int s2 = ls[j], e2 = ls[j + 1];
      const float inter = (float)(min(e, e2) - max(s, s2));
      const float uni = (float)(max(e, e2) - min(s, s2));
      const float iou = (inter / uni) * (c == lc[j] ? 1.f : 0.f);
      if (iou > best) {  // j increases within a lane: the first maximum stays
        best = iou;
        bj = j;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ob = __shfl_xor(best, o);
      const int oj = __shfl_xor(bj, o);
      if (ob > best || (ob == best && oj < bj)) {
        best = ob;
        bj = oj;
      }
    }
    if (bj >= n) continue;  // n == 0 cannot happen (L >= 1)
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      if (k >= K) break;
      const int bit = bj * K + k;
      const bool hit = best > ov[k] && !((used[bit >> 5] >> (bit & 31)) & 1u);
      tp[k] += hit ? 1 : 0;
      fp[k] += hit ? 0 : 1;
      if (hit && lane == 0) used[bit >> 5] |= 1u << (bit & 31);
    }
    __builtin_amdgcn_s_waitcnt(0);  // the flag update is visible to the next segment's reads
  }
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      if (k >= K) break;
      const float TP = (float)tp[k], FP = (float)fp[k], FN = (float)(n - tp[k]);  // matched GT = hits
      const float P = TP / (TP + FP), R = TP / (TP + FN);
      out[k] = 2.f * P * R / (P + R);
    }
  }

  // ---- edit score: rows = the shorter sequence (the distance is symmetric)
  const bool swap = m > n;
  const int R = swap ? n : m, Ccols = swap ? m : n;
  const int* rc = swap ? lc : pc;
  const int* cc = swap ? pc : lc;
  if (R > RMAX) {
    if (lane == 0) *status = 1;
    return;
  }
  int* d0 = lds + uw;      // diagonal d-2
  int* d1 = d0 + RMAX + 1;  // diagonal d-1
  int* d2 = d1 + RMAX + 1;  // diagonal d
  for (int d = 0; d <= R + Ccols; ++d) {
    const int i0 = max(0, d - Ccols), i1 = min(R, d);
    for (int i = i0 + lane; i <= i1; i += 64) {
      const int j = d - i;
      int v;
      if (i == 0)
        v = j;
      else if (j == 0)
        v = i;
      else if (rc[i - 1] == cc[j - 1])
        v = d0[i - 1];
      else
        v = 1 + min(min(d1[i - 1], d1[i]), d0[i - 1]);
      d2[i] = v;
    }
    __builtin_amdgcn_s_waitcnt(0);  // the wave's LDS writes land before the next diagonal reads them
    int* tmp = d0;
    d0 = d1;
    d1 = d2;
    d2 = tmp;
  }
  if (lane == 0) {
    const float D = (float)d1[R];
    out[K] = 1.f - D / (float)max(m, n);
    *status = 0;
  }
}

}  // namespace

long seg_metrics_workspace_launch(int L) { return 4L * (2L * (L + 1) + 2L * L); }

int seg_metrics_launch(const long* lab, const long* pred, int L, int C, const float* ov, int K, int* ws,
                       unsigned long long* cm, float* out, int* status, hipStream_t s) {
  if (L < 1 || C < 1 || K < 1 || K > KMAX || !lab || !pred || !ov || !ws || !out || !status) return STGCN_EBADSHAPE;
  const size_t lds = (size_t)((L * (long)K + 31) / 32) * 4 + 3 * (size_t)(RMAX + 1) * 4;
  if (lds > 160 * 1024) return STGCN_EBADSHAPE;
  if (stgcn_lds_attr((const void*)seg_metrics_kernel, 160 * 1024, s)) return STGCN_EHIP;
  hipLaunchKernelGGL(seg_metrics_kernel, dim3(1), dim3(64), lds, s, lab, pred, L, C, ov, K, ws, cm, out, status);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
