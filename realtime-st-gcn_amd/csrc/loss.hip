// Segmentation loss + top-k statistics of one trial (or one rank's shard of it), forward and the
// gradient w.r.t. the predictions in the same pass.
//
// Reference: utils/loss.py:25-41 (Loss.__call__) and utils/statistics.py:5-16 (Statistics.__call__),
// applied to the (1, C, L) prediction series that segment_generator.mask_segment builds.  With
// p[w][c] the prediction of window/frame w (w < L) and class c:
//     z  = foo(p)            logits: p | logsoftmax: p | softmax: log p            (loss.py:10-18)
//     q  = bar(p)            logits: log_softmax(p) | logsoftmax: exp p | softmax: p
//     ce = sum_{w >= first} wt[y_w] * (-log_softmax(z_w)[y_w]) / D,   D = sum_{w >= first} wt[y_w]
//     mse = 0.15 * sum_{w >= 1} sum_c clamp((q_w[c] - q_{w-1}[c])^2, 0, 16) / (C * pairs)
// (nn.CrossEntropyLoss(weight, reduction='mean'); the MSE's left operand is detached, so its gradient
// reaches only q_w).  `first` = 1 drops the frame a subsegment shares with the previous one from the CE
// and the statistics (loss.py:27-28, statistics.py:8).  top-1/top-5 hits rank p itself.
//
// Data-parallel shards (parallel.py): a shard passes the predictions of the frame before its first one
// (`prev`, or NULL for the first shard) and the GLOBAL D and pair count, so the per-shard values sum to
// the loss of the whole trial and the gradients equal the single-process ones.
//
// Layout: p [L][ldp] fp32 rows, labels int64 [L - first] (frames first..L-1), wt fp32 [C].  One wave per window: lane l holds classes
// l, l+64, l+128, l+192 (C <= 256).  Sums are fixed-order (wave butterfly, then waves, then blocks):
// bit-reproducible.
#include "common.h"

namespace {

constexpr int kMaxC = 256;
constexpr int kPer = kMaxC / 64;
constexpr float kMseWeight = 0.15f;  // loss.py:34
constexpr float kMseClamp = 16.f;    // loss.py:41
constexpr int kWaves = 16;           // waves per block
constexpr int kPartials = 8;         // per block: ce, mse, top1, top5, D, pad

DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

struct RowQ {
  float p[kPer], z[kPer], ls[kPer], sm[kPer], q[kPer];
};

// predictions of one frame -> CE operand z, its log-softmax / softmax, and the MSE operand q
DEV void load_row(const float* __restrict__ row, int C, int mode, int lane, RowQ& r) {
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int c = lane + 64 * k;
    const float v = c < C ? row[c] : 0.f;
    r.p[k] = v;
    r.z[k] = c < C ? (mode == 2 ? logf(v) : v) : -INFINITY;
    m = fmaxf(m, r.z[k]);
  }
  m = wave_max(m);
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < kPer; ++k) s += (lane + 64 * k < C) ? expf(r.z[k] - m) : 0.f;
  const float lse = m + logf(wave_sum(s));
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const bool on = lane + 64 * k < C;
    r.ls[k] = on ? r.z[k] - lse : 0.f;
    r.sm[k] = on ? expf(r.ls[k]) : 0.f;
    r.q[k] = on ? (mode == 0 ? r.ls[k] : (mode == 1 ? expf(r.p[k]) : r.p[k])) : 0.f;
  }
}

DEV float lane_pick(const float* v, int c, int lane) {  // value of class c (all lanes get it)
  float mine = 0.f;
#pragma unroll
  for (int k = 0; k < kPer; ++k)
    if (c == lane + 64 * k) mine = v[k];
  return wave_sum(mine);  // exactly one lane contributes
}

struct LossArgs {
  const float* p;
  int ldp;
  const long* labels;
  const float* wt;
  const float* prev;  // predictions of the frame before this shard (MSE pair), or NULL
  int L, C, first, mode;
  const float* den;   // global D (device scalar) or NULL: this launch's own sum
  float pairs;        // global MSE pair count (> 0) or <= 0: this launch's own
  float* dce;         // [L][C] d ce / d p, or NULL
  float* dmse;        // [L][C] d mse / d p, or NULL
  int* top5;          // [L][5] class indices (descending), or NULL
  float* partial;     // [gridDim.x][kPartials] (multi-block) or the final [kPartials]
};

__global__ __launch_bounds__(1024) void seg_loss_kernel(LossArgs a) {
  __shared__ float red[kWaves][kPartials];
  __shared__ float sden;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int C = a.C;

  // D: every block sums the label weights itself (L loads; no cross-block dependency)
  float den = a.den ? *a.den : 0.f;
  if (!a.den) {
    // eight labels, then their eight weights, requested together per batch (same per-thread order as one
    // window at a time, which was a chain of ~19 dependent label -> weight loads ahead of everything: the
    // 36 us of this launch in the config-2 step)
    float d = 0.f;
    for (int w0 = a.first + threadIdx.x; w0 < a.L; w0 += 8 * blockDim.x) {
      long y[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int w = w0 + u * blockDim.x;
        y[u] = w < a.L ? a.labels[w - a.first] : -1;
      }
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = (y[u] >= 0 && y[u] < C) ? a.wt[y[u]] : 0.f;  // out-of-range: weight 0
#pragma unroll
      for (int u = 0; u < 8; ++u) d += v[u];
    }
    d = wave_sum(d);
    if (lane == 0) red[wave][0] = d;
    __syncthreads();
    if (threadIdx.x == 0) {
      float t = 0.f;
      for (int i = 0; i < kWaves; ++i) t += red[i][0];
      sden = t;
    }
    __syncthreads();
    den = sden;
    __syncthreads();
  }
  float pairs = a.pairs;
  if (!(pairs > 0.f)) pairs = (float)(a.L - 1 + (a.prev ? 1 : 0));
  const float mse_coef = kMseWeight / ((float)C * pairs);

  float ce_acc = 0.f, mse_acc = 0.f, top1 = 0.f, top5 = 0.f, dsum = 0.f;
  const int wpb = (a.L + gridDim.x - 1) / gridDim.x;  // contiguous windows per block
  const int w0 = blockIdx.x * wpb, w1 = min(a.L, w0 + wpb);
  for (int w = w0 + wave; w < w1; w += kWaves) {
    RowQ cur;
    load_row(a.p + (long)w * a.ldp, C, a.mode, lane, cur);
    float gce[kPer], gm[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) gce[k] = gm[k] = 0.f;

    if (w >= a.first) {  // CE + statistics
      const long yl = a.labels[w - a.first];
      const int y = (yl >= 0 && yl < C) ? (int)yl : -1;
      const float wy = y >= 0 ? a.wt[y] : 0.f;
      ce_acc += -wy * lane_pick(cur.ls, y, lane);
      dsum += wy;
      const float sc = wy / den;
#pragma unroll
      for (int k = 0; k < kPer; ++k) {
        const int c = lane + 64 * k;
        if (c < C) {
          const float dz = sc * (cur.sm[k] - (c == y ? 1.f : 0.f));
          gce[k] = a.mode == 2 ? dz / cur.p[k] : dz;  // z = log p
        }
      }
      // top-1 / top-5 from five rounds of argmax (torch.topk order: NaN ranks above every number, equal
      // values by lowest class index), so the hit counts always agree with the returned top-5 classes
      float v[kPer];
#pragma unroll
      for (int k = 0; k < kPer; ++k) {
        const float pv = cur.p[k];
        v[k] = lane + 64 * k < C ? (pv != pv ? INFINITY : pv) : -INFINITY;
      }
      bool hit = false;
      for (int r = 0; r < 5 && r < C; ++r) {
        float bv = -INFINITY;
        int bc = 1 << 30;
#pragma unroll
        for (int k = 0; k < kPer; ++k)
          if (v[k] > bv || (v[k] == bv && lane + 64 * k < bc && lane + 64 * k < C)) bv = v[k], bc = lane + 64 * k;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          const float ov = __shfl_xor(bv, o);
          const int oc = __shfl_xor(bc, o);
          if (ov > bv || (ov == bv && oc < bc)) bv = ov, bc = oc;
        }
        if (a.top5 && lane == 0) a.top5[(long)w * 5 + r] = bc;
        if (bc == y) {
          hit = true;
          if (r == 0) top1 += 1.f;
        }
#pragma unroll
        for (int k = 0; k < kPer; ++k)
          if (lane + 64 * k == bc) v[k] = -INFINITY;
      }
      top5 += hit ? 1.f : 0.f;
    }

    const float* prow = w > 0 ? a.p + (long)(w - 1) * a.ldp : a.prev;
    if (prow) {  // MSE pair (w-1, w); gradient only through q_w
      RowQ pr;
      load_row(prow, C, a.mode, lane, pr);
      float gq[kPer], s = 0.f;
#pragma unroll
      for (int k = 0; k < kPer; ++k) {
        const float d = cur.q[k] - pr.q[k];
        const float d2 = d * d;
        const bool on = lane + 64 * k < C;
        mse_acc += on ? fminf(d2, kMseClamp) : 0.f;
        gq[k] = on && d2 <= kMseClamp ? mse_coef * 2.f * d : 0.f;
        s += gq[k];
      }
      if (a.mode == 0) s = wave_sum(s);
#pragma unroll
      for (int k = 0; k < kPer; ++k)
        gm[k] = a.mode == 0 ? gq[k] - cur.sm[k] * s : (a.mode == 1 ? gq[k] * cur.q[k] : gq[k]);
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int c = lane + 64 * k;
      if (c < C) {
        if (a.dce) a.dce[(long)w * C + c] = gce[k];
        if (a.dmse) a.dmse[(long)w * C + c] = gm[k];
      }
    }
  }
  mse_acc = wave_sum(mse_acc);
  if (lane == 0) {
    red[wave][0] = ce_acc;
    red[wave][1] = mse_acc;
    red[wave][2] = top1;
    red[wave][3] = top5;
    red[wave][4] = dsum;
  }
  __syncthreads();
  if (threadIdx.x < kPartials) {
    float t = 0.f;
    if (threadIdx.x < 5)
      for (int i = 0; i < kWaves; ++i) t += red[i][threadIdx.x];
    if (threadIdx.x == 0) t /= den;
    if (threadIdx.x == 1) t *= kMseWeight / ((float)C * pairs);
    a.partial[blockIdx.x * kPartials + threadIdx.x] = t;
  }
}

// multi-block: fixed-order sum of the block partials
__global__ __launch_bounds__(64) void seg_loss_finish_kernel(const float* __restrict__ partial, int nblk, float* out) {
  // lane = (block group g, partial k): eight independent strided sums per partial, then two shuffle steps
  // (one lane walking every block's partial was a chain of nblk dependent load-adds)
  const int k = threadIdx.x & (kPartials - 1), g = threadIdx.x / kPartials;
  float t = 0.f;
  for (int b = g; b < nblk; b += 64 / kPartials) t += partial[b * kPartials + k];
#pragma unroll
  for (int o = kPartials; o < 64; o <<= 1) t += __shfl_xor(t, o);
  if (threadIdx.x < kPartials) out[k] = t;
}

// d loss / d p = g_ce * dce + g_mse * dmse, the upstream scalars read on the device (no host sync)
__global__ __launch_bounds__(256) void seg_loss_bwd_kernel(const float* __restrict__ dce, const float* __restrict__ dmse,
                                                          const float* __restrict__ gce, const float* __restrict__ gmse,
                                                          long n, float* __restrict__ dp) {
  const float a = gce ? *gce : 0.f, b = gmse ? *gmse : 0.f;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    dp[i] = a * dce[i] + b * dmse[i];
}

int seg_loss_blocks(int L) {
  // a window per wave: the per-window work is a chain of ~30 dependent wave reductions (softmax, 5 argmax
  // rounds, MSE), so one 16-wave block walking the config-2 step's 64 windows 4 per wave took 36 us on one
  // CU; up to 256 blocks
  int nb = (L + kWaves - 1) / kWaves;
  return nb < 1 ? 1 : (nb > 256 ? 256 : nb);
}

}  // namespace

long seg_loss_workspace_launch(int L) { return (long)seg_loss_blocks(L) * kPartials * sizeof(float); }

int seg_loss_launch(const float* p, int ldp, const long* labels, const float* wt, const float* prev, int L, int C,
                    int first, int mode, const float* den, float pairs, float* dce, float* dmse, int* top5,
                    float* work, float* out, hipStream_t s) {
  if (L < 1 || C < 1 || C > kMaxC || ldp < C || first < 0 || first > 1 || mode < 0 || mode > 2 || !p || !labels ||
      !wt || !out)
    return STGCN_EBADSHAPE;
  const int nb = seg_loss_blocks(L);
  if (nb > 1 && !work) return STGCN_EBADSHAPE;
  LossArgs a{p, ldp, labels, wt, prev, L, C, first, mode, den, pairs, dce, dmse, top5, nb > 1 ? work : out};
  hipLaunchKernelGGL(seg_loss_kernel, dim3(nb), dim3(64 * kWaves), 0, s, a);
  if (nb > 1) hipLaunchKernelGGL(seg_loss_finish_kernel, dim3(1), dim3(64), 0, s, work, nb, out);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}

int seg_loss_bwd_launch(const float* dce, const float* dmse, const float* gce, const float* gmse, long n, float* dp,
                        hipStream_t s) {
  if (n < 0 || !dce || !dmse || !dp) return STGCN_EBADSHAPE;
  long g = (n + 255) / 256;
  g = g < 1 ? 1 : (g > 1024 ? 1024 : g);
  hipLaunchKernelGGL(seg_loss_bwd_kernel, dim3((unsigned)g), dim3(256), 0, s, dce, dmse, gce, gmse, n, dp);
  return hipGetLastError() == hipSuccess ? STGCN_OK : STGCN_EHIP;
}
