// extern "C" entry points of libstgcn_amd.so (declared and documented in include/stgcn_amd.h).
// Thin validation + dispatch to the kernel launchers; no global mutable state.
#include <hip/hip_runtime.h>

#include "../../include/stgcn_amd.h"

typedef stgcn_conv_desc ConvArgs;
typedef stgcn_wgrad_desc WgradArgs;
typedef stgcn_amix_desc AmixArgs;

#define STGCN_OK 0
#define STGCN_EBADSHAPE 1
#define STGCN_EDTYPE 2

// launchers (defined in the .hip translation units)
int conv_rows_launch(const ConvArgs& a, int dtype, hipStream_t s);
int conv_rows_bn_tile(int cout);
int pack_weight_launch(const float* src, long s0, long s1, long s2, int Kt, int Co, int Ci, void* dst, int cp, int kp,
                       int dtype, hipStream_t s, void* dst_frag);
long conv_rows_num_row_blocks(long M, int cout);
int conv_wgrad_launch(WgradArgs a, int dtype, hipStream_t s);
int pack_s2frag_launch(const float* src, long s0, long s1, long s2, int Co, int Ci, void* dst, int trans,
                       hipStream_t s);
long wgrad_tile_workspace(const WgradArgs& a, int dtype);
long wgrad_wide_workspace(const WgradArgs& a, int dtype);
long wgrad_ring_workspace(const WgradArgs& a, int dtype);
int wgrad_ring_launch(const WgradArgs& a, int dtype, hipStream_t s);
int wgrad_wide_launch(const WgradArgs& a, int dtype, hipStream_t s);
int wgrad_tile_launch(const WgradArgs& a, int dtype, hipStream_t s);
long wgrad1x1_workspace(const WgradArgs& a, int dtype);
int wgrad1x1_launch(const WgradArgs& a, int dtype, hipStream_t s);
int amix_fwd_launch(const AmixArgs& a, int dtype, hipStream_t s);
long gconv_row_blocks(int NT, int V);
long bn_bwd_fused_work_floats(long M, int C, int dtype);
int bn_bwd_fused_reduce_launch(const stgcn_bn_bwd_desc& a, int dtype, hipStream_t s);
int bn_bwd_fused_apply_launch(const stgcn_bn_bwd_desc& a, int dtype, hipStream_t s);
int gconv_launch(const stgcn_gconv_desc& a, int dtype, hipStream_t s);
int gconv_weights_launch(const float* A, const float* W, const int* nbr, const int* deg, int P, int V, int J, int Cout,
                         int Cin, int trans, void* out, int R_pad, int C_pad, int dtype, hipStream_t s,
                         const float* bconv = nullptr, float* bias2d = nullptr);
long gconv_wgrad_workspace(const stgcn_gconv_wgrad_desc& a, int dtype);
int gconv_wgrad_launch(const stgcn_gconv_wgrad_desc& a, int dtype, hipStream_t s);
int gconv_wgrad_finish_launch(const float* dweff, const float* A, const float* W, const int* nbr, const int* deg,
                              int P, int V, int J, int Cout, int Cin, float* dW, float* dA, void* work, hipStream_t s);
long gconv_wgrad_finish_workspace(int P, int V, int J, int Cout, int Cin);
int gconv_wgrad_finish_bias_launch(const float* dweff, const float* A, const float* W, const int* nbr, const int* deg,
                                   int P, int V, int J, int Cout, int Cin, const float* bconv, const float* S, float* dW,
                                   float* dA, float* db, void* work, hipStream_t s);
int amix_trans_launch(const AmixArgs& a, int dtype, hipStream_t s);
int tconv_frame_launch(const stgcn_conv_desc& a, hipStream_t s);
long tconv_frame_row_blocks(int N, int T);
int amix_dA_launch(const AmixArgs& a, const void* dw, float* dA, void* work, int dtype, hipStream_t s);
long amix_dA_workspace(const AmixArgs& a);
int gcn_bias_bwd_launch(const float* A, const float* b, const float* S, int P, int V, int C, float* dA, float* db,
                        hipStream_t s);
int gcn_bias_launch(const float* A, const float* b, float* out, int N, int P, int V, int C, int per_sample,
                    hipStream_t s);
long norm_stats_num_blocks(long M);
int bn_stats_partial_launch(const void* x, int ld, long M, int C, float4* part, int dtype, hipStream_t s);
int bn_finalize_launch(const float4* part, int nb, int ldp, int C, const float* gamma, const float* beta, float eps,
                       float2* mean_rstd, float* scale, float* shift, hipStream_t s);
int bn_merge_launch(const float4* part, int nb, int ldp, int C, float4* merged, hipStream_t s);
int bn_apply_launch(const void* u, int ldu, const float* sc, const float* sh, int res_mode, const void* r, int ldr,
                    const float* rsc, const float* rsh, int relu, void* y, int ldy, long M, int C, int dtype,
                    hipStream_t s,
                    unsigned char* bits = nullptr);
int bn_bwd_reduce_launch(const void* dy, int lddy, int mask, const void* mref, int ldm, const float* msc,
                         const float* msh, const void* x, int ldx, const float2* mean_rstd, long M, int C,
                         float2* part, float2* out, int dtype, hipStream_t s);
int bn_bwd_apply_launch(const void* dy, int lddy, int mask, const void* mref, int ldm, const float* msc,
                        const float* msh, const void* x, int ldx, const float2* mean_rstd, const float* gamma,
                        const float2* sums, long M, int C, void* dx, int lddx, int accumulate, int dtype,
                        hipStream_t s);
int rowgroup_sum_launch(const void* x, int ld, long M, int C, int G, long period, float* S, float* work, int dtype,
                        hipStream_t s);
long rowgroup_sum_workspace(long M, int C, int G, long period);
int ln_stats_launch(const void* x, int ld, long F, int V, int C, float eps, float2* stats, int dtype, hipStream_t s);
int ln_apply_launch(const void* u, int ldu, const float2* st, const float* g, const float* b, int res_mode,
                    const void* r, int ldr, const float2* rst, const float* rg, const float* rb, int relu, void* y,
                    int ldy, long M, int V, int C, int dtype, hipStream_t s);
long ln_bwd_workspace(long F, int V, int C, int dtype);
long cast_colsum_workspace(long M, int C);
int cast_colsum_launch(const float* x, int ldx, long M, int C, void* out16, int ldo, float* colsum, float* work,
                       hipStream_t s);
int ln_bwd_launch(const void* dy, int lddy, int mask, const void* mref, int ldm, const void* x, int ldx,
                  const float2* st, const float* g, const float* b, long F, int V, int C, void* dx, int lddx,
                  int accumulate, float* dgb, void* work, long work_bytes, int dtype, hipStream_t s);
int pool_rows_launch(const void* x, int ld, int N, int R, int C, void* out, int ldo, int dtype, hipStream_t s);
int unpool_rows_launch(const void* dp, int ldp, int R, int C, long M, void* dx, int ldx, int dtype, hipStream_t s);
int box_sum_launch(const void* x, int ldx, void* y, int ldy, int N, int T_, int V, int C, int K, int S, int trans,
                   int accumulate, int dtype, hipStream_t s);
int rt_online_launch(const float* z, float* fifo, float* acc, int* idx, int C, int V, int fifo_size, int S,
                     float* out, hipStream_t s);

int attn_scores_launch(const void* th, const void* ph, int ld, int N, int T_, int V, int P, int ce, float* S,
                       void* work, int dtype, hipStream_t s);
long attn_scores_workspace(int N, int T_, int V, int P);
int attn_proj_launch(const void* x, int ldx, long M, int Cin, const float* W, const float* bias, int Nout, float* out,
                     int ldo, hipStream_t s);
int attn_bwd_launch(const void* th, const void* ph, int ld, int N, int T_, int V, int P, int ce, const float* C,
                    const float* dC, float* dS, void* dth, void* dph, int dtype, hipStream_t s);
int layer_fused_launch(const stgcn_layer_fused_desc& a, hipStream_t s);
int rt_in_launch(const float* x, int V, const float* g, const float* b, const float* W, const float* bias, int C0,
                 float* out, hipStream_t s);
int rt_gcn_launch(const float* x, int V, int Cin, int Cout, int P, const float* A, const float* W, const float* bias2d,
                  float* fifo, float* acc, const int* idx, const float* Wr, float* a_out, float* r_out,
                  hipStream_t s);
int rt_norm_launch(const float* a, const float* g, const float* b, int res_mode, const float* res, const float* gr,
                   const float* br, int V, int C, int* idx, int fifo_size, int S, float* y, hipStream_t s);
int rt_out_launch(const float* x, int V, int C, const float* W, const float* bias, int K, float* out, hipStream_t s);
int rt_frame_launch(const stgcn_rt_frame_desc& d, hipStream_t s);
int window_stat_blocks_launch(int nw, int W);
int window_stats_launch(const float* x, int Cin, int Lp, int V, int W, int n0, int nw, int mode, float eps, float* out,
                        hipStream_t s);
int window_expand_launch(const float* x, int Cin, int Lp, int V, int W, int n0, int nw, int mode, const float* g,
                         const float* b, const float* fst, const float* w, const float* bias, int Cout, void* out,
                         int ldo, int dtype, hipStream_t s);
long window_grad_workspace_launch(int nw, int W, int V, int Cin, int Cout);
int window_grad_launch(const void* dy, int ldd, int dtype, const float* x, int Cin, int Lp, int V, int W, int n0, int nw,
                       int mode, const float* st, const float* g, const float* b, const float* w, int Cout, float* work,
                       float* dg, float* dbeta, float* dw, float* db, hipStream_t s);
long seg_metrics_workspace_launch(int L);
int seg_metrics_launch(const long* lab, const long* pred, int L, int C, const float* ov, int K, int* ws,
                       unsigned long long* cm, float* out, int* status, hipStream_t s);
long seg_loss_workspace_launch(int L);
int seg_loss_launch(const float* p, int ldp, const long* labels, const float* wt, const float* prev, int L, int C,
                    int first, int mode, const float* den, float pairs, float* dce, float* dmse, int* top5, float* work,
                    float* out, hipStream_t s);
int seg_loss_bwd_launch(const float* dce, const float* dmse, const float* gce, const float* gmse, long n, float* dp,
                        hipStream_t s);

#define CHECK_DTYPE(dt) \
  if ((dt) != 0 && (dt) != 1) return STGCN_EDTYPE
#define STREAM(s) reinterpret_cast<hipStream_t>(s)

extern "C" {

int stgcn_abi_version(void) { return STGCN_ABI_VERSION; }

int stgcn_conv_rows(const stgcn_conv_desc* d, int dtype, void* stream) {
  CHECK_DTYPE(dtype);
  if (!d || !d->in || !d->out || !d->w || d->N <= 0 || d->V <= 0 || d->T_in <= 0 || d->T_out <= 0 || d->Kt <= 0 ||
      d->stride <= 0 || d->Cin <= 0 || d->Cout <= 0 || d->in_ld < d->Cin || d->out_ld < d->Cout ||
      d->Cin_pad < d->Cin || d->Cout_pad < d->Cout)
    return STGCN_EBADSHAPE;
  if ((d->pro == 1 && (!d->pro_a || !d->pro_b)) || (d->pro == 2 && (!d->pro_a || !d->pro_b || !d->pro_stats)))
    return STGCN_EBADSHAPE;
  if (d->bias_mode && !d->bias) return STGCN_EBADSHAPE;
  return conv_rows_launch(*d, dtype, STREAM(stream));
}

int stgcn_conv_rows_col_tile(int cout) { return conv_rows_bn_tile(cout); }
int stgcn_pack_weight(const float* src, long s0, long s1, long s2, int Kt, int Co, int Ci, void* dst, int Cout_pad,
                      int Cin_pad, int dtype, void* stream) {
  CHECK_DTYPE(dtype);
  if (!src || !dst || Kt <= 0 || Co <= 0 || Ci <= 0 || Cout_pad < Co || Cin_pad < Ci) return STGCN_EBADSHAPE;
  return pack_weight_launch(src, s0, s1, s2, Kt, Co, Ci, dst, Cout_pad, Cin_pad, dtype, STREAM(stream), nullptr);
}
int stgcn_pack_weight_s2frag(const float* src, long s0, long s1, long s2, int Co, int Ci, void* dst_frag, int trans,
                             int dtype, void* stream) {
  if (dtype != 1) return STGCN_EDTYPE;
  if (!src || !dst_frag || Co <= 0 || Ci <= 0) return STGCN_EBADSHAPE;
  return pack_s2frag_launch(src, s0, s1, s2, Co, Ci, dst_frag, trans ? 1 : 0, STREAM(stream));
}
int stgcn_pack_weight_frag(const float* src, long s0, long s1, long s2, int Kt, int Co, int Ci, void* dst,
                           void* dst_frag, int Cout_pad, int Cin_pad, int dtype, void* stream) {
  CHECK_DTYPE(dtype);
  if (!src || !dst || !dst_frag || Kt <= 0 || Co <= 0 || Ci <= 0 || Cout_pad < Co || Cin_pad < Ci) return STGCN_EBADSHAPE;
  return pack_weight_launch(src, s0, s1, s2, Kt, Co, Ci, dst, Cout_pad, Cin_pad, dtype, STREAM(stream), dst_frag);
}
long stgcn_conv_rows_row_blocks(long M, int cout) { return conv_rows_num_row_blocks(M, cout); }

long stgcn_conv_wgrad_workspace(const stgcn_wgrad_desc* d, int dtype) {
  if (!d || (dtype != 0 && dtype != 1)) return 0;
  const long wr = wgrad_ring_workspace(*d, dtype);  // 64 / 128-channel Kt=9 stride-1 DMA-ring path first
  if (wr > 0) return wr;
  const long w = wgrad_wide_workspace(*d, dtype);  // >= 128-channel Kt=9 stride-1 path
  if (w > 0) return w;
  const long w1 = wgrad1x1_workspace(*d, dtype);   // 1x1 split-K path
  return w1 > 0 ? w1 : wgrad_tile_workspace(*d, dtype);
}

int stgcn_conv_wgrad(const stgcn_wgrad_desc* d, int dtype, void* stream) {
  CHECK_DTYPE(dtype);
  if (!d || !d->in || !d->dy || !d->dw || d->N <= 0 || d->Kt <= 0 || d->stride <= 0) return STGCN_EBADSHAPE;
  if (d->pro && (!d->pro_a || !d->pro_b || (d->pro == 2 && !d->pro_stats))) return STGCN_EBADSHAPE;
  if (d->out_mode != 0 && d->out_mode != 1) return STGCN_EBADSHAPE;
  const int rr = wgrad_ring_launch(*d, dtype, STREAM(stream));  // bf16 64 / 128-channel DMA-ring path (needs work)
  if (rr >= 0) return rr;
  const int rw = wgrad_wide_launch(*d, dtype, STREAM(stream));  // bf16 >= 128-channel ring path (needs work)
  if (rw >= 0) return rw;
  const int r1 = wgrad1x1_launch(*d, dtype, STREAM(stream));  // bf16 1x1 split-K row reduction (needs work)
  if (r1 >= 0) return r1;
  const int r = wgrad_tile_launch(*d, dtype, STREAM(stream));  // bf16 frame-tiled path (needs work)
  if (r >= 0) return r;
  if (d->out_mode) return STGCN_EBADSHAPE;  // the accumulating paths below: += [Kt][Cout][Cin] only
  return conv_wgrad_launch(*d, dtype, STREAM(stream));
}

long stgcn_bn_bwd_fused_workspace(long M, int C, int dtype) {
  if (M <= 0 || C <= 0 || (dtype != 0 && dtype != 1)) return 0;
  return bn_bwd_fused_work_floats(M, C, dtype);
}
int stgcn_bn_bwd_fused_reduce(const stgcn_bn_bwd_desc* d, int dtype, void* stream) {
  CHECK_DTYPE(dtype);
  if (!d || !d->dy || d->M <= 0 || d->C <= 0 || (d->mask && !d->mref) || (d->mask == 2 && (!d->msc || !d->msh)) ||
      (d->x1 && !d->mean_rstd1) || (d->x2 && !d->mean_rstd2) || (d->mask == 3 && (dtype != 1 || d->C % 8 || d->ldm < d->C / 8)))
    return STGCN_EBADSHAPE;
  return bn_bwd_fused_reduce_launch(*d, dtype, STREAM(stream));
}
int stgcn_bn_bwd_fused_apply(const stgcn_bn_bwd_desc* d, int dtype, void* stream) {
  CHECK_DTYPE(dtype);
  if (!d || !d->dy || d->M <= 0 || d->C <= 0 || (d->mask && !d->mref) || (d->mask == 2 && (!d->msc || !d->msh)) ||
      (d->x1 && !d->mean_rstd1) || (d->x2 && !d->mean_rstd2) || (d->mask == 3 && (dtype != 1 || d->C % 8 || d->ldm < d->C / 8)))
    return STGCN_EBADSHAPE;
  return bn_bwd_fused_apply_launch(*d, dtype, STREAM(stream));
}

int stgcn_gconv(const stgcn_gconv_desc* d, int dtype, void* stream) {
  CHECK_DTYPE(dtype);
  if (!d || !d->in || !d->out || !d->w || !d->nbr || !d->deg || d->NT <= 0 || d->V <= 0 || d->J <= 0 ||
      d->Cin <= 0 || d->Cout <= 0 || d->Cin_pad < d->Cin || d->Cout_pad < d->Cout || d->in_ld < d->Cin ||
      d->out_ld < d->Cout)
    return STGCN_EBADSHAPE;
  return gconv_launch(*d, dtype, STREAM(stream));
}
long stgcn_gconv_row_blocks(int NT, int V) { return gconv_row_blocks(NT, V); }
int stgcn_gconv_weights(const float* A, const float* W, const int* nbr, const int* deg, int P, int V, int J, int Cout,
                        int Cin, int trans, void* out, int rows_pad, int cols_pad, int dtype, void* stream) {
  CHECK_DTYPE(dtype);
  if (!A || !W || !nbr || !deg || !out || P <= 0 || V <= 0 || J <= 0 || Cout <= 0 || Cin <= 0 ||
      rows_pad < (trans ? Cin : Cout) || cols_pad < (trans ? Cout : Cin))
    return STGCN_EBADSHAPE;
  return gconv_weights_launch(A, W, nbr, deg, P, V, J, Cout, Cin, trans, out, rows_pad, cols_pad, dtype,
                              STREAM(stream));
}
int stgcn_gconv_weights_bias(const float* A, const float* W, const float* b, const int* nbr, const int* deg, int P,
                             int V, int J, int Cout, int Cin, void* out, int rows_pad, int cols_pad, float* bias2d,
                             int dtype, void* stream) {
  CHECK_DTYPE(dtype);
  if (!A || !W || !b || !nbr || !deg || !out || !bias2d || P <= 0 || V <= 0 || J <= 0 || Cout <= 0 || Cin <= 0 ||
      rows_pad < Cout || cols_pad < Cin || (cols_pad % 8) != 0)
    return STGCN_EBADSHAPE;
  return gconv_weights_launch(A, W, nbr, deg, P, V, J, Cout, Cin, 0, out, rows_pad, cols_pad, dtype, STREAM(stream),
                              b, bias2d);
}
long stgcn_gconv_wgrad_workspace(const stgcn_gconv_wgrad_desc* d, int dtype) {
  if (!d || (dtype != 0 && dtype != 1)) return 0;
  return gconv_wgrad_workspace(*d, dtype);
}
int stgcn_gconv_wgrad(const stgcn_gconv_wgrad_desc* d, int dtype, void* stream) {
  CHECK_DTYPE(dtype);
  if (!d || !d->x || !d->dy || !d->nbr || !d->deg || !d->dweff || d->NT <= 0 || d->V <= 0 || d->J <= 0 ||
      d->Cin <= 0 || d->Cout <= 0)
    return STGCN_EBADSHAPE;
  return gconv_wgrad_launch(*d, dtype, STREAM(stream));
}
int stgcn_gconv_wgrad_finish_bias(const float* dweff, const float* A, const float* W, const int* nbr, const int* deg,
                                  int P, int V, int J, int Cout, int Cin, const float* bconv, const float* S, float* dW,
                                  float* dA, float* db, void* work, void* stream) {
  if (!dweff || !A || !W || !nbr || !deg || !bconv || !S || !dW || !dA || !db || !work || P <= 0 || V <= 0 || J <= 0 ||
      Cout <= 0 || Cin <= 0)
    return STGCN_EBADSHAPE;
  return gconv_wgrad_finish_bias_launch(dweff, A, W, nbr, deg, P, V, J, Cout, Cin, bconv, S, dW, dA, db, work,
                                        STREAM(stream));
}
long stgcn_gconv_wgrad_finish_workspace(int P, int V, int J, int Cout, int Cin) {
  return gconv_wgrad_finish_workspace(P, V, J, Cout, Cin);
}
int stgcn_gconv_wgrad_finish(const float* dweff, const float* A, const float* W, const int* nbr, const int* deg, int P,
                             int V, int J, int Cout, int Cin, float* dW, float* dA, void* work, void* stream) {
  if (!dweff || !A || !W || !nbr || !deg || P <= 0 || V <= 0 || J <= 0 || Cout <= 0 || Cin <= 0)
    return STGCN_EBADSHAPE;
  return gconv_wgrad_finish_launch(dweff, A, W, nbr, deg, P, V, J, Cout, Cin, dW, dA, work, STREAM(stream));
}
int stgcn_tconv_frame(const stgcn_conv_desc* d, void* stream) {
  if (!d) return STGCN_EBADSHAPE;
  return tconv_frame_launch(*d, STREAM(stream));
}
long stgcn_tconv_frame_row_blocks(int N, int T) { return tconv_frame_row_blocks(N, T); }

int stgcn_amix_fwd(const stgcn_amix_desc* d, int dtype, void* stream) {
  CHECK_DTYPE(dtype);
  if (!d || !d->x || !d->out || !d->A) return STGCN_EBADSHAPE;
  return amix_fwd_launch(*d, dtype, STREAM(stream));
}
int stgcn_amix_trans(const stgcn_amix_desc* d, int dtype, void* stream) {
  CHECK_DTYPE(dtype);
  if (!d || !d->x || !d->out || !d->A) return STGCN_EBADSHAPE;
  return amix_trans_launch(*d, dtype, STREAM(stream));
}
long stgcn_amix_dA_workspace(const stgcn_amix_desc* d) { return d ? amix_dA_workspace(*d) : 0; }
int stgcn_amix_dA(const stgcn_amix_desc* d, const void* dw, float* dA, void* work, int dtype, void* stream) {
  CHECK_DTYPE(dtype);
  if (!d || !d->x || !dw || !dA) return STGCN_EBADSHAPE;
  return amix_dA_launch(*d, dw, dA, work, dtype, STREAM(stream));
}
int stgcn_gcn_bias_bwd(const float* A, const float* b, const float* S, int P, int V, int C, float* dA, float* db,
                       void* stream) {
  if (!A || !b || !S || !dA || !db || P <= 0 || V <= 0 || C <= 0) return STGCN_EBADSHAPE;
  return gcn_bias_bwd_launch(A, b, S, P, V, C, dA, db, STREAM(stream));
}
int stgcn_gcn_bias(const float* A, const float* b, float* out, int N, int P, int V, int C, int per_sample,
                   void* stream) {
  if (!A || !b || !out) return STGCN_EBADSHAPE;
  return gcn_bias_launch(A, b, out, N, P, V, C, per_sample, STREAM(stream));
}

long stgcn_bn_stat_blocks(long M) { return norm_stats_num_blocks(M); }
int stgcn_bn_stats_partial(const void* x, int ld, long M, int C, void* part, int dtype, void* stream) {
  CHECK_DTYPE(dtype);
  return bn_stats_partial_launch(x, ld, M, C, (float4*)part, dtype, STREAM(stream));
}
int stgcn_bn_finalize(const void* part, int nb, int ldp, int C, const float* gamma, const float* beta, float eps,
                      void* mean_rstd, float* scale, float* shift, void* stream) {
  return bn_finalize_launch((const float4*)part, nb, ldp, C, gamma, beta, eps, (float2*)mean_rstd, scale, shift,
                            STREAM(stream));
}
int stgcn_bn_merge(const void* part, int nb, int ldp, int C, void* merged, void* stream) {
  return bn_merge_launch((const float4*)part, nb, ldp, C, (float4*)merged, STREAM(stream));
}
int stgcn_bn_apply(const void* u, int ldu, const float* sc, const float* sh, int res_mode, const void* r, int ldr,
                   const float* rsc, const float* rsh, int relu, void* y, int ldy, long M, int C, int dtype,
                   void* stream) {
  CHECK_DTYPE(dtype);
  if (res_mode && !r) return STGCN_EBADSHAPE;
  return bn_apply_launch(u, ldu, sc, sh, res_mode, r, ldr, rsc, rsh, relu, y, ldy, M, C, dtype, STREAM(stream));
}
int stgcn_bn_apply_bits(const void* u, int ldu, const float* sc, const float* sh, int res_mode, const void* r, int ldr,
                        const float* rsc, const float* rsh, int relu, void* y, int ldy, long M, int C, void* bits,
                        void* stream) {
  if ((res_mode && !r) || !bits || C % 8) return STGCN_EBADSHAPE;
  return bn_apply_launch(u, ldu, sc, sh, res_mode, r, ldr, rsc, rsh, relu, y, ldy, M, C, 1, STREAM(stream),
                         static_cast<unsigned char*>(bits));
}
int stgcn_bn_bwd_reduce(const void* dy, int lddy, int mask, const void* mref, int ldm, const float* msc,
                        const float* msh, const void* x, int ldx, const void* mean_rstd, long M, int C, void* part,
                        void* sums, int dtype, void* stream) {
  CHECK_DTYPE(dtype);
  return bn_bwd_reduce_launch(dy, lddy, mask, mref, ldm, msc, msh, x, ldx, (const float2*)mean_rstd, M, C,
                              (float2*)part, (float2*)sums, dtype, STREAM(stream));
}
int stgcn_bn_bwd_apply(const void* dy, int lddy, int mask, const void* mref, int ldm, const float* msc,
                       const float* msh, const void* x, int ldx, const void* mean_rstd, const float* gamma,
                       const void* sums, long M, int C, void* dx, int lddx, int accumulate, int dtype,
                       void* stream) {
  CHECK_DTYPE(dtype);
  return bn_bwd_apply_launch(dy, lddy, mask, mref, ldm, msc, msh, x, ldx, (const float2*)mean_rstd, gamma,
                             (const float2*)sums, M, C, dx, lddx, accumulate, dtype, STREAM(stream));
}
long stgcn_rowgroup_sum_workspace(long M, int C, int G, long period) {
  return rowgroup_sum_workspace(M, C, G, period);
}
int stgcn_rowgroup_sum(const void* x, int ld, long M, int C, int G, long period, float* S, float* work, int dtype,
                       void* stream) {
  CHECK_DTYPE(dtype);
  if (!x || !S || !work || G <= 0) return STGCN_EBADSHAPE;
  return rowgroup_sum_launch(x, ld, M, C, G, period, S, work, dtype, STREAM(stream));
}
int stgcn_ln_stats(const void* x, int ld, long frames, int V, int C, float eps, void* st, int dtype, void* stream) {
  CHECK_DTYPE(dtype);
  return ln_stats_launch(x, ld, frames, V, C, eps, (float2*)st, dtype, STREAM(stream));
}
int stgcn_ln_apply(const void* u, int ldu, const void* st, const float* g, const float* b, int res_mode,
                   const void* r, int ldr, const void* rst, const float* rg, const float* rb, int relu, void* y,
                   int ldy, long M, int V, int C, int dtype, void* stream) {
  CHECK_DTYPE(dtype);
  return ln_apply_launch(u, ldu, (const float2*)st, g, b, res_mode, r, ldr, (const float2*)rst, rg, rb, relu, y, ldy,
                         M, V, C, dtype, STREAM(stream));
}
int stgcn_ln_bwd(const void* dy, int lddy, int mask, const void* mref, int ldm, const void* x, int ldx,
                 const void* st, const float* g, const float* b, long frames, int V, int C, void* dx, int lddx,
                 int accumulate, float* dgb, void* work, long work_bytes, int dtype, void* stream) {
  CHECK_DTYPE(dtype);
  return ln_bwd_launch(dy, lddy, mask, mref, ldm, x, ldx, (const float2*)st, g, b, frames, V, C, dx, lddx,
                       accumulate, dgb, work, work_bytes, dtype, STREAM(stream));
}
long stgcn_ln_bwd_workspace(long frames, int V, int C, int dtype) { return ln_bwd_workspace(frames, V, C, dtype); }
int stgcn_cast_colsum(const float* x, int ldx, long M, int C, void* out_bf16, int ldo, float* colsum, float* work,
                      void* stream) {
  if (!x || !out_bf16 || !colsum || (!work && M > 0)) return STGCN_EBADSHAPE;
  return cast_colsum_launch(x, ldx, M, C, out_bf16, ldo, colsum, work, STREAM(stream));
}
long stgcn_cast_colsum_workspace(long M, int C) { return cast_colsum_workspace(M, C); }
int stgcn_pool_rows(const void* x, int ld, int N, int R, int C, void* out, int ldo, int dtype, void* stream) {
  CHECK_DTYPE(dtype);
  return pool_rows_launch(x, ld, N, R, C, out, ldo, dtype, STREAM(stream));
}
int stgcn_unpool_rows(const void* dp, int ldp, int R, int C, long M, void* dx, int ldx, int dtype, void* stream) {
  CHECK_DTYPE(dtype);
  return unpool_rows_launch(dp, ldp, R, C, M, dx, ldx, dtype, STREAM(stream));
}
int stgcn_box_sum(const void* x, int ldx, void* y, int ldy, int N, int T, int V, int C, int K, int S, int trans,
                  int accumulate, int dtype, void* stream) {
  CHECK_DTYPE(dtype);
  return box_sum_launch(x, ldx, y, ldy, N, T, V, C, K, S, trans, accumulate, dtype, STREAM(stream));
}
int stgcn_rt_online_step(const void* z, float* fifo, float* acc, int* idx, int C, int V, int fifo_size, int S,
                         float* out, void* stream) {
  if (!z || !fifo || !acc || !idx || !out) return STGCN_EBADSHAPE;
  return rt_online_launch((const float*)z, fifo, acc, idx, C, V, fifo_size, S, out, STREAM(stream));
}

long stgcn_attn_scores_workspace(int N, int T, int V, int P) { return attn_scores_workspace(N, T, V, P); }
int stgcn_attn_proj(const void* x, int ldx, long M, int Cin, const float* w, const float* bias, int Nout, float* out,
                    int ldo, void* stream) {
  return attn_proj_launch(x, ldx, M, Cin, w, bias, Nout, out, ldo, STREAM(stream));
}
int stgcn_attn_scores(const void* th, const void* ph, int ld, int N, int T, int V, int P, int ce, float* C, void* work,
                      int dtype, void* stream) {
  CHECK_DTYPE(dtype);
  if (!th || !ph || !C || ld < P * ce) return STGCN_EBADSHAPE;
  return attn_scores_launch(th, ph, ld, N, T, V, P, ce, C, work, dtype, STREAM(stream));
}
int stgcn_attn_bwd(const void* th, const void* ph, int ld, int N, int T, int V, int P, int ce, const float* C,
                   const float* dC, float* dS, void* dth, void* dph, int dtype, void* stream) {
  CHECK_DTYPE(dtype);
  if (!th || !ph || !C || !dC || !dS || !dth || !dph || ld < P * ce) return STGCN_EBADSHAPE;
  return attn_bwd_launch(th, ph, ld, N, T, V, P, ce, C, dC, dS, dth, dph, dtype, STREAM(stream));
}

int stgcn_layer_fused_fwd(const stgcn_layer_fused_desc* d, void* stream) {
  if (!d) return STGCN_EBADSHAPE;
  return layer_fused_launch(*d, STREAM(stream));
}

int stgcn_rt_frame_in(const float* x, int V, const float* ln_w, const float* ln_b, const float* w, const float* b, int C0,
                      float* out, void* stream) {
  return rt_in_launch(x, V, ln_w, ln_b, w, b, C0, out, STREAM(stream));
}
int stgcn_rt_frame_gcn(const float* x, int V, int Cin, int Cout, int P, const float* A, const float* w, const float* bias2d,
                       float* fifo, float* acc, const int* idx, const float* wr, float* a_out, float* r_out,
                       void* stream) {
  return rt_gcn_launch(x, V, Cin, Cout, P, A, w, bias2d, fifo, acc, idx, wr, a_out, r_out, STREAM(stream));
}
int stgcn_rt_frame_norm(const float* a, const float* ln_w, const float* ln_b, int res_mode, const float* res,
                        const float* lnr_w, const float* lnr_b, int V, int C, int* idx, int fifo_size, int S, float* y,
                        void* stream) {
  return rt_norm_launch(a, ln_w, ln_b, res_mode, res, lnr_w, lnr_b, V, C, idx, fifo_size, S, y, STREAM(stream));
}
int stgcn_rt_frame_out(const float* x, int V, int C, const float* w, const float* b, int K, float* out, void* stream) {
  return rt_out_launch(x, V, C, w, b, K, out, STREAM(stream));
}
int stgcn_rt_frame(const stgcn_rt_frame_desc* d, void* stream) {
  return d ? rt_frame_launch(*d, STREAM(stream)) : STGCN_EBADSHAPE;
}

int stgcn_window_stat_blocks(int nw, int W) { return window_stat_blocks_launch(nw, W); }
int stgcn_window_stats(const float* x, int Cin, int Lp, int V, int W, int n0, int nw, int mode, float eps, float* out,
                       void* stream) {
  return window_stats_launch(x, Cin, Lp, V, W, n0, nw, mode, eps, out, STREAM(stream));
}
int stgcn_window_expand(const float* x, int Cin, int Lp, int V, int W, int n0, int nw, int mode, const float* g,
                        const float* b, const float* fst, const float* w, const float* bias, int Cout, void* out,
                        int ldo, int dtype, void* stream) {
  return window_expand_launch(x, Cin, Lp, V, W, n0, nw, mode, g, b, fst, w, bias, Cout, out, ldo, dtype,
                              STREAM(stream));
}
long stgcn_window_grad_workspace(int nw, int W, int V, int Cin, int Cout) {
  return window_grad_workspace_launch(nw, W, V, Cin, Cout);
}
int stgcn_window_grad(const void* dy, int ldd, int dtype, const float* x, int Cin, int Lp, int V, int W, int n0, int nw,
                      int mode, const float* st, const float* gamma, const float* beta, const float* w, int Cout,
                      void* work, float* dgamma, float* dbeta, float* dw, float* db, void* stream) {
  return window_grad_launch(dy, ldd, dtype, x, Cin, Lp, V, W, n0, nw, mode, st, gamma, beta, w, Cout, (float*)work,
                            dgamma, dbeta, dw, db, STREAM(stream));
}

long stgcn_segment_metrics_workspace(int L) { return seg_metrics_workspace_launch(L); }
int stgcn_segment_metrics(const long* labels, const long* pred, int L, int C, const float* overlap, int K, void* work,
                          long long* confusion, float* out, int* status, void* stream) {
  return seg_metrics_launch(labels, pred, L, C, overlap, K, (int*)work, (unsigned long long*)confusion, out, status,
                            STREAM(stream));
}

long stgcn_seg_loss_workspace(int L) { return seg_loss_workspace_launch(L); }
int stgcn_seg_loss(const float* p, int ldp, const long* labels, const float* wt, const float* prev, int L, int C,
                   int first, int mode, const float* den, float pairs, float* dce, float* dmse, int* top5, float* work,
                   float* out, void* stream) {
  return seg_loss_launch(p, ldp, labels, wt, prev, L, C, first, mode, den, pairs, dce, dmse, top5, work, out,
                         STREAM(stream));
}
int stgcn_seg_loss_bwd(const float* dce, const float* dmse, const float* gce, const float* gmse, long n, float* dp,
                       void* stream) {
  return seg_loss_bwd_launch(dce, dmse, gce, gmse, n, dp, STREAM(stream));
}

}  // extern "C"

