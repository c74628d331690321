/*
 * stgcn_amd.h — C-ABI of the MI355X-native ST-GCN hot path (libstgcn_amd.so).
 *
 * The reference (maximyudayev/Realtime-ST-GCN) has no native code and no FFI: its hot path is
 * a stack of PyTorch aten ops inside nn.Modules.  Each entry point below replaces one or more of
 * those aten calls; the reference call site it replaces is cited (file:line, relative to the
 * reference root).  The Python package realtime-st-gcn_amd/ binds these with ctypes underneath
 * modules that keep the reference's nn.Module API and state_dict names.
 *
 * Conventions
 *   - Plain pointers and sizes only; device pointers unless noted; no framework types.
 *   - Activations are the reference's logical (N, C, T, V) tensors stored channels-last:
 *     element (n, c, t, v) at ((n*T + t)*V + v)*ld + c  ("rows" of ld >= C elements).
 *   - dtype: 0 = fp32 (parity path), 1 = bf16 (perf path).  Accumulation is fp32.
 *   - stream: a hipStream_t (NULL = default stream).  Every call is asynchronous.
 *   - Return: 0 ok, 1 bad shape/arguments, 2 unsupported dtype, 3 HIP launch error.
 *   - Thread-safety: no global mutable state; calls on different streams/devices are independent
 *     (the reference runs replicas from nn.DataParallel threads, processor.py:32-33).
 */
#ifndef STGCN_AMD_H
#define STGCN_AMD_H

#ifdef __cplusplus
extern "C" {
#endif

/* Bumped on every change of a descriptor's layout or of an entry point's signature; realtime-st-gcn_amd/_lib.py
 * refuses a library whose stgcn_abi_version() differs from the version it was written against.
 *   1: rounds 1-4;  2: round 5 (stgcn_gconv_desc gained res / res_bits / res_ld);
 *   3: round 6 (stgcn_gcn_tile removed; stgcn_layer_fused_desc is the LayerNorm layer only: the BatchNorm
 *      fields n1_scale / n1_shift / stats / ln / g_in / g_in_ld and stgcn_layer_fused_row_blocks removed);
 *   4: round 6 (stgcn_rt_frame + stgcn_rt_layer / stgcn_rt_frame_desc: the RT per-frame step in one launch;
 *      stgcn_gconv_wgrad_desc gained phase);
 *   5: round 6 (stgcn_bn_merge: one (count, mean, M2) entry per channel, the SyncBatchNorm exchange unit). */
#define STGCN_ABI_VERSION 5

/* Implicit-GEMM (Kt x 1) row convolution; see conv_rows.hip for the exact contract.
 * Replaces: nn.Conv2d tcn.2 (models/stgcn/stgcn.py:154-159), residual.0 (stgcn.py:165-170),
 * gcn.conv (models/utils/tgcn.py:48-55,71), fcn_in/fcn_out (stgcn.py:49,74,85,95), OfflineLayer
 * conv/residual (models/rtstgcn/rtstgcn.py:316,330) and their input-gradients (trans = 1). */
typedef struct {
  const void* in;
  void* out;
  const void* w;          /* packed [Kt][Cout_pad][Cin_pad], element type = dtype */
  const float* bias;      /* [Cout] (bias_mode 1) | [V][Cout] (2) | [N][V][Cout] (3) | NULL */
  const float* pro_a;     /* prologue scale [Cin] (pro 1) | LN gamma [Cin][V] (pro 2) */
  const float* pro_b;     /* prologue shift [Cin] | LN beta [Cin][V] */
  const float* pro_stats; /* pro 2: float2 (mean, rstd) per input frame [N*T_in] */
  float* stats;           /* optional BN partials: float4 (count, mean, M2, 0) [row_blocks][Cout_pad] */
  int N, T_in, T_out, V, Cin, Cout, Cin_pad, Cout_pad;
  int Kt, stride, pad, trans, pro, bias_mode, accumulate;
  int in_ld, out_ld;
  const void* w_frag;     /* optional MFMA-fragment image of the weights for the wide-channel Kt = 9 kernel
                           * (NULL: other kernels): stride 1 -> stgcn_pack_weight_frag's image of w;
                           * stride 2 -> stgcn_pack_weight_s2frag's parity-folded image (trans to match) */
} stgcn_conv_desc;

int stgcn_conv_rows(const stgcn_conv_desc* d, int dtype, void* stream);
/* The 64-channel Kt = 9 stride-1 temporal conv (stgcn.py:151-159) forward (trans 0, pro 0 or 1: BN1 scale /
 * shift + ReLU on the input, bias_mode 0/1, optional BN partial statistics [stgcn_tconv_frame_row_blocks(N, T)]
 * [Cout_pad]) and data gradient (trans 1, pro 0), bf16, on the row-streaming kernel (tconv_frame.hip): the same
 * arithmetic as stgcn_conv_rows for these shapes; w_frag = the MFMA-fragment image of the packed weight
 * (stgcn_pack_weight_frag, Kt = 9), Cin = Cout = 64, pad = 4, 16 < V <= 25, in_ld % 8 == 0, out_ld % 8 == 0 (16-B
 * row stores), no accumulate; other shapes return STGCN_EBADSHAPE (use stgcn_conv_rows). */
int stgcn_tconv_frame(const stgcn_conv_desc* d, void* stream);
long stgcn_tconv_frame_row_blocks(int N, int T);
/* Pack an fp32 weight given as any strided [Kt][Cout][Cin] view (element (k,co,ci) at src[k*s0+co*s1+ci*s2])
 * into the zero-padded contiguous [Kt][Cout_pad][Cin_pad] dtype image stgcn_conv_rows reads. */
int stgcn_pack_weight(const float* src, long s0, long s1, long s2, int Kt, int Cout, int Cin, void* dst, int Cout_pad,
                      int Cin_pad, int dtype, void* stream);
/* stgcn_pack_weight plus the MFMA-fragment image dst_frag (same element count; Cout_pad % 32 == 0,
 * Cin_pad % 16 == 0): 1-KiB blocks [k][co/32][ci/16], lane (ci%16)/8*32 + co%32 holding 8 consecutive ci,
 * so one 32x32x16 B fragment is one contiguous wave load (conv_wide.hip). */
int stgcn_pack_weight_frag(const float* src, long s0, long s1, long s2, int Kt, int Cout, int Cin, void* dst,
                           void* dst_frag, int Cout_pad, int Cin_pad, int dtype, void* stream);
/* Parity-folded MFMA-fragment image of a stride-2 Kt = 9 weight src [9][Cout][Cin] (fp32, element
 * (k,co,ci) at src[k*s0+co*s1+ci*s2]) — the w_frag a stride-2 stgcn_conv_rows call takes: the 5-tap
 * conv over frame pairs (forward: W'[t][co][par*Cin+ci] = W[2t+par][co][ci]; trans = 1, the data grad:
 * W'[t][par*Cout+co][ci] = W[8-2t+par][co][ci]), dst_frag holding 5 * 2 * Cout * Cin bf16.
 * Replaces: the strided tcn.2 of layers with stride 2 (models/stgcn/stgcn.py:154-159) and its input grad. */
int stgcn_pack_weight_s2frag(const float* src, long s0, long s1, long s2, int Cout, int Cin, void* dst_frag, int trans,
                             int dtype, void* stream);
/* column tile the packed weights must be padded to (Cout_pad % tile == 0) */
int stgcn_conv_rows_col_tile(int cout);
/* upper bound on row blocks (first dim of the BN partial-stat buffer, which the caller zero-fills) */
long stgcn_conv_rows_row_blocks(long M, int cout);

/* Weight gradient of stgcn_conv_rows (trans = 0): dw[Kt][Cout][Cin] += ... (fp32, zeroed by caller).
 * Replaces: convolution_backward weight path of the convs above (autograd of stgcn.py:154-170). */
typedef struct {
  const void* in;
  const void* dy;
  float* dw;
  const float* pro_a;
  const float* pro_b;
  const float* pro_stats;
  int N, T_in, T_out, V, Cin, Cout, Kt, stride, pad, pro;
  int in_ld, dy_ld;
  long rows_per_block; /* filled by the library */
  void* work;          /* optional workspace (bf16 frame-tiled path: per-block fp32 partials) */
  long work_bytes;     /* its size; stgcn_conv_wgrad_workspace() tells how much the fast path needs */
  int out_mode;        /* 0: dw[Kt][Cout][Cin] += gradient; 1: dw OVERWRITTEN in nn.Conv2d weight order
                        * [Cout][Cin][Kt] (no zero fill, no permute copy) — the workspace paths only
                        * (stgcn_conv_wgrad_workspace() > 0), else STGCN_EBADSHAPE */
  int pad_;
} stgcn_wgrad_desc;

int stgcn_conv_wgrad(const stgcn_wgrad_desc* d, int dtype, void* stream);
/* workspace bytes for the deterministic frame-tiled path (0: shape/dtype served without one) */
long stgcn_conv_wgrad_workspace(const stgcn_wgrad_desc* d, int dtype);

/* Graph (joint-axis) mixing of ConvTemporalGraphical (models/utils/tgcn.py:58-79), A applied first.
 *   fwd  : XA[(n,t,w)][p*Cin+ci] = sum_v A[(n),p,v,w] x[(n,t,v)][ci]             (tgcn.py:76)
 *   trans: dx[(n,t,v)][ci] (+)= sum_{p,w} A[(n),p,v,w] DW[(n,t,w)][p*Cin+ci]       (autograd of :76)
 *   dA   : dA[(n),p,v,w] += sum_{t,ci} x[(n,t,v)][ci] DW[(n,t,w)][p*Cin+ci]          (grad of A)
 *   bias : bias2d[(n),w,c] = sum_p b[p*C+c] sum_v A[(n),p,v,w]   (the conv bias pushed through A)
 * A is fp32 [P][V][V] (shared) or [N][P][V][V] (per_sample, AAGCN models/aagcn/aagcn.py:148). */
typedef struct {
  const void* x;
  void* out;
  const float* A;
  int N, T, V, P, Cin, per_sample, accumulate;
  int x_ld, out_ld;
} stgcn_amix_desc;

int stgcn_amix_fwd(const stgcn_amix_desc* d, int dtype, void* stream);
int stgcn_amix_trans(const stgcn_amix_desc* d, int dtype, void* stream);
/* dA (+)= sum over frames of x (x) DW.  work: stgcn_amix_dA_workspace() bytes -> per-block partials summed
   in a fixed order (bit-reproducible); NULL -> fp32 atomics (run-to-run order noise). */
long stgcn_amix_dA_workspace(const stgcn_amix_desc* d);
int stgcn_amix_dA(const stgcn_amix_desc* d, const void* dw, float* dA, void* work, int dtype, void* stream);
/* Shared-A gradients of the graph-conv bias (autograd of tgcn.py:71-79 through the bias), from
 * S[w][c] = sum of dg over the rows of joint w (stgcn_rowgroup_sum):
 *   dA[p][v][w] += sum_c b[p*C+c] S[w][c];   db[p*C+c] = sum_w (sum_v A[p][v][w]) S[w][c] */
int stgcn_gcn_bias_bwd(const float* A, const float* b, const float* S, int P, int V, int C, float* dA, float* db,
                       void* stream);
int stgcn_gcn_bias(const float* A, const float* b, float* out, int N, int P, int V, int C, int per_sample,
                   void* stream);

/* Graph convolution as a joint-gathered GEMM for a batch-shared A (ConvTemporalGraphical,
 * models/utils/tgcn.py:58-79; replaces the conv1x1 + einsum pair):
 *   out[(i,a)][r] (+)= sum_{j<deg[a]} sum_c in[(i, nbr[a*J+j])][c] * w[a][j][r][c]  (+ bias[a][r]),
 * i = n*T + t in [0, NT).  w = effective weights from stgcn_gconv_weights ([V][J][Cout_pad][Cin_pad]):
 *   trans 0 (forward):   w[w][j][co][ci] = sum_p A[p][S(w)_j][w] * W[p*Cout+co][ci]
 *   trans 1 (data grad): w[v][j][ci][co] = sum_p A[p][v][R(v)_j] * W[p*Cout+co][ci]
 * with nbr = the support lists S (forward) or the reverse lists R (data grad).  Optional BN partial
 * statistics per (row block, channel) as stgcn_conv_rows, row blocks <= stgcn_gconv_row_blocks. */
typedef struct {
  const void* in;
  void* out;
  const void* w;
  const int* nbr;   /* [V][J] */
  const int* deg;   /* [V] */
  const float* bias; /* [V][Cout] or NULL */
  float* stats;
  int NT, V, J, Cin, Cout, Cin_pad, Cout_pad, in_ld, out_ld, accumulate;
  /* optional masked residual (bf16, accumulate = 0, 16-B aligned rows): out = result + res * mask with mask bit
   * c % 8 of byte res_bits[row * (Cout / 8) + c / 8] (stgcn_bn_apply_bits' layout) — the identity residual's
   * gradient dz = dy * [y > 0] of stgcn.py:191-193 added in the data gradient's epilogue instead of being
   * written by the BatchNorm backward and read back here.  res rows: ld res_ld, rows as out. */
  const void* res;
  const void* res_bits;
  int res_ld;
} stgcn_gconv_desc;

int stgcn_gconv(const stgcn_gconv_desc* d, int dtype, void* stream);

long stgcn_gconv_row_blocks(int NT, int V);
int stgcn_gconv_weights(const float* A, const float* W, const int* nbr, const int* deg, int P, int V, int J, int Cout,
                        int Cin, int trans, void* out, int rows_pad, int cols_pad, int dtype, void* stream);
/* stgcn_gconv_weights (forward form, trans = 0) and stgcn_gcn_bias for a shared A in ONE launch:
 * bias2d[w][co] = sum_p b[p*Cout + co] * sum_v A[p][v][w]  (fp32 [V][Cout]; replaces the separate
 * bias-through-A launch of ConvTemporalGraphical.forward, tgcn.py:71-79, conv bias then einsum with A) */
int stgcn_gconv_weights_bias(const float* A, const float* W, const float* b, const int* nbr, const int* deg, int P,
                             int V, int J, int Cout, int Cin, void* out, int rows_pad, int cols_pad, float* bias2d,
                             int dtype, void* stream);
/* dweff[w][j][co][ci] = sum_i dy[(i,w)][co] * x[(i, nbr[w][j])][ci]   (fp32 [V][J][Cout][Cin], written
 * whole: 0 for the unused slots j >= deg[w]) */
typedef struct {
  const void* x;
  const void* dy;
  const int* nbr;
  const int* deg;
  float* dweff;
  int NT, V, J, Cin, Cout, x_ld, dy_ld;
  void* work;
  long work_bytes;
  float* rowsum; /* optional [V][Cout]: rowsum[w][co] = sum_i dy[(i,w)][co] (bias through A), or NULL */
  int phase;     /* 0: the whole gradient; 1: the accumulation kernel only (row-range partials left in work);
                  * 2: the slab reduction only (work holds phase 1's partials of the same desc) — so a caller can
                  * time the accumulation kernel alone; plans without a slab do everything in phase 1 */
  int pad_;
} stgcn_gconv_wgrad_desc;

int stgcn_gconv_wgrad(const stgcn_gconv_wgrad_desc* d, int dtype, void* stream);
long stgcn_gconv_wgrad_workspace(const stgcn_gconv_wgrad_desc* d, int dtype);
/* dW[p*Cout+co][ci] += sum_{w,j} A[p][S(w)_j][w] dweff[w][j][co][ci]  (dW may be NULL);
 * dA[p][S(w)_j][w] += sum_{co,ci} W[p*Cout+co][ci] dweff[w][j][co][ci]  (dA may be NULL)
 * work: stgcn_gconv_wgrad_finish_workspace() bytes (chunked dA partials, fixed-order reduce) or NULL
 * (slower per-partition path).  Deterministic either way. */
long stgcn_gconv_wgrad_finish_workspace(int P, int V, int J, int Cout, int Cin);
/* The same finish with the conv bias pushed through A folded in (stgcn_gcn_bias_bwd), in two launches, every
 * output OVERWRITTEN (no zero fill needed):
 *   dW[p*Cout+co][ci] = sum_{w,j} A[p][S(w)_j][w] dweff[w][j][co][ci]
 *   dA[p][v][w]       = [v in S(w)] sum_{co,ci} W[p*Cout+co][ci] dweff[pair(v,w)][co][ci] + sum_c bconv[p*Cout+c] S[w][c]
 *   db[p*Cout+c]      = sum_w colsum_p(A)[w] S[w][c]
 * S = the per-joint row sums of dy [V][Cout] (stgcn_gconv_wgrad's rowsum); work as above (required);
 * P <= 4, V <= 32.  Bit-identical to stgcn_gconv_wgrad_finish into zeros followed by stgcn_gcn_bias_bwd. */
int stgcn_gconv_wgrad_finish_bias(const float* dweff, const float* A, const float* W, const int* nbr, const int* deg,
                                  int P, int V, int J, int Cout, int Cin, const float* bconv, const float* S, float* dW,
                                  float* dA, float* db, void* work, void* stream);
int stgcn_gconv_wgrad_finish(const float* dweff, const float* A, const float* W, const int* nbr, const int* deg, int P,
                             int V, int J, int Cout, int Cin, float* dW, float* dA, void* work, void* stream);

/* BatchNorm with batch statistics (nn.BatchNorm2d(track_running_stats=False), stgcn.py:152,160,171;
 * BatchNorm1d input norm, models/utils/batchnorm.py:13-23 viewed as [N*T][V*C]).
 * Partials are float4 (count, mean, M2, 0) per (row block, channel); finalize merges them (fp64). */
long stgcn_bn_stat_blocks(long M);
int stgcn_bn_stats_partial(const void* x, int ld, long M, int C, void* part_f4, int dtype, void* stream);
int stgcn_bn_finalize(const void* part_f4, int nblocks, int ld_part, int C, const float* gamma, const float* beta,
                      float eps, void* mean_rstd_f2, float* scale, float* shift, void* stream);
/* merged_f4[c] = the nblocks partials of channel c merged (fp64) into ONE (count, mean, M2, 0) entry: a rank's
 * contribution to SyncBatchNorm (torch.nn.SyncBatchNorm's batch_norm_gather_stats_with_counts role, the
 * north_star's optional SyncBN); the gathered [ranks][C] entries go back through stgcn_bn_finalize
 * (nblocks = ranks, ld_part = C).  No reference counterpart: the reference's DataParallel keeps per-replica
 * statistics (processor.py:32-33). */
int stgcn_bn_merge(const void* part_f4, int nblocks, int ld_part, int C, void* merged_f4, void* stream);
/* Fused BatchNorm backward (two row passes), see bn_fused.hip:
 *   reduce: dz = dy*mask; sums[c] = (sum dz, sum dz*xhat1, sum dz*xhat2, 0)
 *   apply : out1 = g1*rstd1*(dz - S0/M - xhat1*S1/M) (or dz when x1 == NULL);
 *           out2 (+)= g2*rstd2*(dz - S0/M - xhat2*S2/M) (or dz when x2 == NULL);  osum[c] = (sum out1,
 *           sum out2) — the conv-bias gradients.  mask: 0 none | 1 mref > 0 | 2 mref*msc + msh > 0 |
 *           3 (bf16, C % 8 == 0) mref = the bit mask stgcn_bn_apply_bits wrote: byte [m * ldm + c / 8], bit c % 8
 *           set where the stored output was > 0 (ldm = bytes per row, >= C / 8) — 1/16 of the bytes of mask 1.
 * Replaces: autograd of stgcn.py:160,171,191-193 (BN2 / residual BN / ReLU / add) and :152-153. */
typedef struct {
  const void* dy;
  const void* mref;
  const void* x1;
  const void* x2;
  const float* msc;
  const float* msh;
  const float* mean_rstd1; /* float2 [C] */
  const float* mean_rstd2;
  const float* gamma1;
  const float* gamma2;
  float* sums;  /* float4 [C], then the same planar: float [3][C] (7*C floats) */
  void* out1;
  void* out2;
  float* osum;  /* optional, layout as sums */
  float* work;  /* float4 [blocks][C], stgcn_bn_bwd_fused_workspace() floats */
  long M;
  int C, mask, lddy, ldm, ldx1, ldx2, ldo1, ldo2, acc2;
} stgcn_bn_bwd_desc;

long stgcn_bn_bwd_fused_workspace(long M, int C, int dtype);
int stgcn_bn_bwd_fused_reduce(const stgcn_bn_bwd_desc* d, int dtype, void* stream);
int stgcn_bn_bwd_fused_apply(const stgcn_bn_bwd_desc* d, int dtype, void* stream);
/* y = act(u*sc + sh + res), res_mode 0 none | 1 r | 2 r*rsc + rsh  (stgcn.py:191-193, rtstgcn.py:386-389);
 * relu bit 0: ReLU after the residual add; bit 1: ReLU on the normalised branch before the add. */
int stgcn_bn_apply(const void* u, int ldu, const float* sc, const float* sh, int res_mode, const void* r, int ldr,
                   const float* rsc, const float* rsh, int relu, void* y, int ldy, long M, int C, int dtype,
                   void* stream);
/* stgcn_bn_apply (bf16, C % 8 == 0) that also writes the output's sign bits for the backward's ReLU mask:
 * bits[m * (C / 8) + c / 8] bit c % 8 = (stored y[m][c] > 0) — what the fused backward reads as mask 3
 * instead of re-reading y (1/16 of the bytes). */
int stgcn_bn_apply_bits(const void* u, int ldu, const float* sc, const float* sh, int res_mode, const void* r, int ldr,
                        const float* rsc, const float* rsh, int relu, void* y, int ldy, long M, int C, void* bits,
                        void* stream);
/* sums_f2[c] = (sum dz, sum dz*xhat) with dz = dy * mask (mask 0 none | 1 mref>0 | 2 mref*msc+msh>0);
 * x may be NULL (then only sum dz).  part_f2 scratch: [stgcn_bn_stat_blocks(M)][C] float2. */
int stgcn_bn_bwd_reduce(const void* dy, int lddy, int mask, const void* mref, int ldm, const float* msc,
                        const float* msh, const void* x, int ldx, const void* mean_rstd_f2, long M, int C,
                        void* part_f2, void* sums_f2, int dtype, void* stream);
/* dx (+)= gamma*rstd*(dz - S1/M - xhat*S2/M); x == NULL: dx (+)= dz */
int stgcn_bn_bwd_apply(const void* dy, int lddy, int mask, const void* mref, int ldm, const float* msc,
                       const float* msh, const void* x, int ldx, const void* mean_rstd_f2, const float* gamma,
                       const void* sums_f2, long M, int C, void* dx, int lddx, int accumulate, int dtype,
                       void* stream);
/* S[g][c] += sum_{m % G == g} x[m][c]  (per-joint column sums: GCN bias gradient);
 * period > 0: per-sample S[n][g][c] over rows [n*period, (n+1)*period) (per-sample A, AAGCN). */
int stgcn_rowgroup_sum(const void* x, int ld, long M, int C, int G, long period, float* S, float* work, int dtype,
                       void* stream);
/* floats of scratch `work` stgcn_rowgroup_sum needs (per-block partial slabs, reduced deterministically) */
long stgcn_rowgroup_sum_workspace(long M, int C, int G, long period);

/* Custom LayerNorm([C,1,V]) (models/utils/layernorm.py:4-28): per (n,t) frame over (C,V),
 * unbiased variance, per-(c,v) affine. */
int stgcn_ln_stats(const void* x, int ld, long frames, int V, int C, float eps, void* stats_f2, int dtype,
                   void* stream);
int stgcn_ln_apply(const void* u, int ldu, const void* st_f2, const float* g, const float* b, int res_mode,
                   const void* r, int ldr, const void* rst_f2, const float* rg, const float* rb, int relu, void* y,
                   int ldy, long M, int V, int C, int dtype, void* stream);
/* dx (+)= rstd*(gz - mean(gz) - xhat*sum(gz*xhat)/(E-1)), gz = dz*g, dz = dy*mask (0 none | 1 mref > 0 |
 * 2 relu(LN(x)) > 0); dgb (optional, [2][C*V]) += (sum dz*xhat, sum dz) over all frames, reduced in a fixed
 * order through `work` (stgcn_ln_bwd_workspace bytes; unused when dgb is NULL). */
int stgcn_ln_bwd(const void* dy, int lddy, int mask, const void* mref, int ldm, const void* x, int ldx,
                 const void* st_f2, const float* g, const float* b, long frames, int V, int C, void* dx, int lddx,
                 int accumulate, float* dgb, void* work, long work_bytes, int dtype, void* stream);
long stgcn_ln_bwd_workspace(long frames, int V, int C, int dtype);

/* out_bf16[m][c] = bf16(x[m][c]) and colsum[c] = sum_m x[m][c] (fp32, fixed order) from one read of the fp32
 * rows: the attention projections' backward (models/aagcn/aagcn.py:139-141 autograd; the bf16 GEMM operand
 * and the bias gradients).  C % 4 == 0, C <= 1024; work: stgcn_cast_colsum_workspace floats. */
int stgcn_cast_colsum(const float* x, int ldx, long M, int C, void* out_bf16, int ldo, float* colsum, float* work,
                      void* stream);
long stgcn_cast_colsum_workspace(long M, int C);

/* Head: F.avg_pool2d over (T,V) (stgcn.py:92) and its gradient. */
int stgcn_pool_rows(const void* x, int ld, int N, int R, int C, void* out, int ldo, int dtype, void* stream);
int stgcn_unpool_rows(const void* dp, int ldp, int R, int C, long M, void* dx, int ldx, int dtype, void* stream);

/* RT-ST-GCN temporal aggregation (models/rtstgcn/rtstgcn.py):
 *   box_sum : y[...,t] = sum_{i < K/S} x[..., t - i*S]  on rows (Toeplitz matmul rtstgcn.py:366-379),
 *             trans = 1 gives its adjoint (gradient).
 *   online  : one frame of AggregateStgcn.forward (rtstgcn.py:591-627) with device-resident FIFO. */
int stgcn_box_sum(const void* x, int ldx, void* y, int ldy, int N, int T, int V, int C, int K, int S, int trans,
                  int accumulate, int dtype, void* stream);
int stgcn_rt_online_step(const void* z_f32, float* fifo, float* acc, int* idx, int C, int V, int fifo_size, int S,
                         float* out, void* stream);

/* AAGCN attention adjacency (models/aagcn/aagcn.py:142-145): C[n,p] = softmax_w(theta_p^T phi_p) over
 * K = T*ce, theta/phi rows [N][T][V][ld] (channel p*ce+c).  C: fp32 [N][P][V][V].  Backward writes
 * dS (scratch, fp32 like C) and dtheta/dphi (rows like theta/phi). */
/* AgcnLayer's theta / phi projections for a bf16 model (aagcn.py:139-141): out[r][o] = bias[o] +
 * sum_c w[o][c] x[r][c], x bf16 rows [M][ldx] (Cin % 16 == 0, <= 256), w fp32 [Nout][Cin] (theta and phi
 * stacked), out fp32 rows [M][ldo]: fp32-accurate outputs (w split into two bf16 parts on the matrix cores)
 * without converting x; the attention logits need fp32 theta/phi. */
int stgcn_attn_proj(const void* x, int ldx, long M, int Cin, const float* w, const float* bias, int Nout, float* out,
                    int ldo, void* stream);
/* work: stgcn_attn_scores_workspace() bytes (deterministic T-chunk reduction) or NULL (atomics). */
long stgcn_attn_scores_workspace(int N, int T, int V, int P);
int stgcn_attn_scores(const void* theta, const void* phi, int ld, int N, int T, int V, int P, int ce, float* C,
                      void* work, int dtype, void* stream);
int stgcn_attn_bwd(const void* theta, const void* phi, int ld, int N, int T, int V, int P, int ce, const float* C,
                   const float* dC, float* dS, void* dtheta, void* dphi, int dtype, void* stream);

int stgcn_abi_version(void);

/* Segmentation loss + statistics of a prediction series (replaces utils/loss.py:25-41 Loss.__call__ and
 * utils/statistics.py:5-16 Statistics.__call__ on the (1, C, L) output of segment_generator.mask_segment).
 *   p: fp32 [L][ldp] predictions (frame w, class c); labels: int64 [L - first]; wt: fp32 [C] class weights
 *   (1 - class_dist / sum, loss.py:20); mode: 0 'logits', 1 'logsoftmax', 2 'softmax' output_type;
 *   first: 1 drops frame 0 from the CE and statistics (subsegment i > 0).
 *   Data-parallel shards: prev = predictions of the frame before this shard (its MSE pair) or NULL,
 *   den = the global CE weight sum (device fp32 scalar; NULL: this call's own), pairs = the global MSE
 *   pair count (<= 0: this call's own).
 *   Outputs: out[0] ce, out[1] mse (this call's share of the trial's loss), out[2] top-1 hits,
 *   out[3] top-5 hits, out[4] this call's CE weight sum (out: fp32 [8]); dce / dmse [L][C] the gradients
 *   of ce and mse w.r.t. p (NULL: skipped); top5 int32 [L][5] class indices (NULL: skipped).
 *   work: stgcn_seg_loss_workspace(L) bytes.  Deterministic (fixed-order sums). */
long stgcn_seg_loss_workspace(int L);
int stgcn_seg_loss(const float* p, int ldp, const long* labels, const float* wt, const float* prev, int L, int C,
                   int first, int mode, const float* den, float pairs, float* dce, float* dmse, int* top5, float* work,
                   float* out, void* stream);
/* dp[i] = (*gce) * dce[i] + (*gmse) * dmse[i]  (gce/gmse: device fp32 scalars, NULL = 0) — the backward of
 * the two loss terms given the upstream gradients, without a host round trip. */
int stgcn_seg_loss_bwd(const float* dce, const float* dmse, const float* gce, const float* gmse, long n, float* dp,
                       void* stream);

/* The fused ST-GCN layer (layer_fused.hip; BASELINE north_star) of a LayerNorm StgcnLayer, 64 -> 64 channels,
 * stride 1, Kt = 9, identity or no residual, as ONE kernel:
 *   g = ConvTemporalGraphical(x) (tgcn.py:58-79; graph conv recomputed per frame on the matrix cores, never stored),
 *   h = relu(LN1(g)), u = tcn(h) + tbias (stgcn.py:151-159), y = relu(LN2(u) + residual * x) (stgcn.py:181-193),
 * with LayerNorm([64,1,V]) per frame over C x V, unbiased variance (layernorm.py:22-28); y is written to z.
 * bf16; P <= 3; 16 < V <= 25.  wg_frag: the Kt = 1 MFMA-fragment image of W'[co][p*64+ci] = W[p*64+co][ci] with
 * the columns of every 16-wide group permuted (realtime-st-gcn_amd/native.py pack_gcn_weight):
 * W''[c][16m + 8h + j] = W'[c][16m + 8(j/4) + 4h + j%4] (h < 2, j < 8); wt_frag: the stgcn_pack_weight_frag image
 * of the temporal weight [9][64][64]; gbias: the conv bias through A [V][64] (or NULL); ln*_g / ln*_b: the
 * LayerNorm([64,1,V]) parameters TRANSPOSED to [V][64] fp32.
 * Replaces: StgcnLayer.forward (models/stgcn/stgcn.py:181-193) of a LayerNorm layer. */
typedef struct {
  const void* x;         /* bf16 rows [N][T][V][x_ld], 64 channels */
  void* z;               /* bf16 rows [N][T][V][z_ld]: the layer output y */
  const void* wg_frag;
  const float* A;        /* [P][V][V] fp32 (A * edge importance) */
  const float* gbias;    /* [V][64] or NULL */
  const void* wt_frag;
  const float* tbias;    /* [64] or NULL */
  int N, T, V, P, x_ld, z_ld;
  const float* ln1_g;
  const float* ln1_b;
  const float* ln2_g;
  const float* ln2_b;
  int residual, pad_;
  /* training forward (all four set, or all NULL for inference): what the layer's backward (StgcnLayerFunction's
   * unfused LN backward) reads besides y — g_out: the graph-conv output incl. its bias (pre-LN1) rows
   * [N][T][V][g_ld]; u_out: the temporal-conv output incl. its bias (pre-LN2) rows, u_ld; st1_out / st2_out:
   * per-frame LayerNorm statistics (mean, 1/sqrt(unbiased var + 1e-5)) of g and u, float2 [N*T] —
   * stgcn_ln_stats's layout, computed here from the fp32 values before their bf16 rounding. */
  void* g_out;
  void* u_out;
  float* st1_out;
  float* st2_out;
  int g_ld, u_ld;
  /* optional with the training outputs (NULL otherwise): h = relu(LN1(g)) rows, h_ld — the temporal conv's input,
   * which the layer's weight gradient reads (saves recomputing it in the backward) */
  void* h_out;
  int h_ld, pad2_;
} stgcn_layer_fused_desc;

int stgcn_layer_fused_fwd(const stgcn_layer_fused_desc* d, void* stream);

/* Segment metrics of one trial (evaluation): labels / pred int64 [L] framewise classes (device).
 * out fp32 [K + 1]: F1@overlap[k] (utils/metrics/f1.py:14-52; NaN when the trial has no hit, as the
 * reference) and the segmental edit score out[K] (utils/metrics/edit.py:10-33); confusion (int64 [C][C],
 * [predicted][label], or NULL) += the framewise counts (utils/metrics/confusion.py:10-29).  overlap: fp32
 * [K] device, K <= 8; work: stgcn_segment_metrics_workspace(L) bytes; status (device int): 0 ok, 1 more than
 * 8192 segments in both sequences (edit score not computed).  One wave; bit-identical to the reference. */
long stgcn_segment_metrics_workspace(int L);
int stgcn_segment_metrics(const long* labels, const long* pred, int L, int C, const float* overlap, int K, void* work,
                          long long* confusion, float* out, int* status, void* stream);

/* RT-ST-GCN per-frame inference (config 3; rt_fused.hip), fp32, batch 1, rows [V][C] of one frame:
 *   stgcn_rt_frame_in  : x (1,3,1,V) -> LayerNorm([3,1,V]) (ln_w/ln_b [3*V], element c*V+v) -> fcn_in
 *                        (w [C0][3], b [C0]) -> out [V][C0]                        (rtstgcn.py:103,140-143)
 *   stgcn_rt_frame_gcn : OnlineLayer's conv1x1 + A-mix (A [P][V][V] = graph * importance, w [P*Cout][Cin],
 *                        bias2d [V][Cout] = the conv bias through A) and AggregateStgcn's FIFO step
 *                        (fifo [S*(K-1)+1][V][Cout], acc [S][V][Cout], idx int[2] = (fifo, acc) indices,
 *                        read only) -> a_out [V][Cout]; wr [Cout][Cin] (or NULL): the residual 1x1 conv
 *                        (no bias) -> r_out                                    (rtstgcn.py:528-537,591-627)
 *   stgcn_rt_frame_norm: y = relu(relu(LN(a)) + res) (res_mode 1: res = x, 2: res = LN_r(r)) or relu(LN(a))
 *                        (res_mode 0); LN per frame over C*V, unbiased; advances idx   (rtstgcn.py:538-553)
 *   stgcn_rt_frame_out : mean over V -> fcn_out (w [K][C], b [K]) -> out [K]          (rtstgcn.py:149-153) */
int stgcn_rt_frame_in(const float* x, int V, const float* ln_w, const float* ln_b, const float* w, const float* b, int C0,
                      float* out, void* stream);
int stgcn_rt_frame_gcn(const float* x, int V, int Cin, int Cout, int P, const float* A, const float* w, const float* bias2d,
                       float* fifo, float* acc, const int* idx, const float* wr, float* a_out, float* r_out,
                       void* stream);
int stgcn_rt_frame_norm(const float* a, const float* ln_w, const float* ln_b, int res_mode, const float* res,
                        const float* lnr_w, const float* lnr_b, int V, int C, int* idx, int fifo_size, int S, float* y,
                        void* stream);
int stgcn_rt_frame_out(const float* x, int V, int C, const float* w, const float* b, int K, float* out, void* stream);

/* The whole per-frame step of a LayerNorm RT-ST-GCN (Model.forward after prepare_benchmark, rtstgcn.py:130-153
 * with every OnlineLayer, rtstgcn.py:528-553 + 591-627) as ONE persistent launch (rt_fused.hip): stgcn_rt_frame_in,
 * then per layer stgcn_rt_frame_gcn's arithmetic spread over `blocks` workgroups (channel pairs), an in-launch grid
 * barrier (agent-scope release / acquire on a counter), stgcn_rt_frame_norm's arithmetic redundantly in every
 * workgroup (the next layer's input stays in LDS), the FIFO indices advanced, and stgcn_rt_frame_out.  Same math as
 * the four entry points above (LN sums in another fixed order).  Per layer: a_buf / r_buf [V][Cout] device scratch
 * (r_buf only when res_mode == 2), wr NULL unless res_mode == 2; lnr_w / lnr_b only for res_mode 2.
 * sync: 16 device bytes, zeroed by this call (a memset on the stream ahead of the launch) — the barrier counter;
 * status: a device int the kernel sets to 1 if a barrier wait gave up (bounded spin; never reset here).
 * Workgroups of 1024 threads; the hand-off of a / r between workgroups is write-through (sc1) stores and loads.
 * V <= 32, 4 <= C <= 256 (C % 4 == 0), V * C <= 7680, P <= 3, L <= STGCN_RT_MAX_LAYERS, blocks in [1, 256] (0 = 64). */
#define STGCN_RT_MAX_LAYERS 12
typedef struct {
  int Cin, Cout, P, fifo_size, S, res_mode;
  const float* A;       /* [P][V][V] graph * importance */
  const float* w;       /* [P*Cout][Cin] */
  const float* bias2d;  /* [V][Cout] or NULL */
  const float* wr;      /* [Cout][Cin] residual conv (res_mode 2) or NULL */
  const float* ln_w;    /* [V][Cout]: the LayerNorm([Cout,1,V]) affine in the rows' layout (transposed) */
  const float* ln_b;
  const float* lnr_w;   /* residual LN (res_mode 2), [V][Cout] */
  const float* lnr_b;
  float* fifo;          /* [fifo_size][V][Cout] */
  float* acc;           /* [S][V][Cout] */
  int* idx;             /* int[2] (fifo, acc) */
  float* a_buf;         /* [V][Cout] hand-off scratch */
  float* r_buf;         /* [V][Cout] (res_mode 2) */
} stgcn_rt_layer;
typedef struct {
  int V, L, C0, K, blocks;
  const float* x;       /* (1,3,1,V) frame, element c*V+v */
  const float* ln_w;    /* [3*V] */
  const float* ln_b;
  const float* w_in;    /* [C0][3] */
  const float* b_in;    /* [C0] */
  const float* w_out;   /* [K][C_last] */
  const float* b_out;   /* [K] or NULL */
  float* out;           /* [K] */
  unsigned* sync;       /* 16 B, zeroed per call */
  int* status;
  stgcn_rt_layer layers[STGCN_RT_MAX_LAYERS];
} stgcn_rt_frame_desc;
int stgcn_rt_frame(const stgcn_rt_frame_desc* d, void* stream);

/* Window staging (window.hip): the first activation of a batch of sliding windows
 * (WindowSegment, utils/segment_generator.py:132-145) computed from the padded capture without forming the
 * windows.  x: fp32 [Cin][Lp][V] (the reference's padded (1, Cin, Lp, V) capture, processor.py:372-374),
 * Cin in {1,2,3,4,6,8}; windows n in [n0, n0+nw) hold frames [n, n+W) (n0 + nw + W - 1 <= Lp).
 *   stgcn_window_stats : norm_in statistics of the windowed batch.  mode 0, BatchNorm1d(V*Cin) (batchnorm.py:
 *       13-23): out = float4 (count, mean, M2, 0) partials [stgcn_window_stat_blocks(nw, W)][V*Cin], each
 *       frame weighted by the number of windows holding it -> stgcn_bn_finalize(nb, ld = C = V*Cin);
 *       mode 1, LayerNorm([Cin,1,V]) (layernorm.py:22-28): out = float2 (mean, rstd) per frame [nw+W-1],
 *       unbiased variance.
 *   stgcn_window_expand: out rows (n, t, v) [nw][W][V], ld ldo, dtype: fcn_in(norm_in(x[:, n+t, v]))
 *       (stgcn.py:82-85) with w [Cout][Cin], bias [Cout] (or NULL).  mode 0: g/b = the folded affine
 *       (scale, shift) [V*Cin] of stgcn_bn_finalize, fst NULL; mode 1: g/b = gamma/beta [Cin*V] (element
 *       c*V+v), fst = the frame statistics.  Cout % (16 / element size) == 0.
 *   stgcn_window_grad  : from dy rows (the gradient of expand's output, ld ldd): dw [Cout][Cin], db [Cout],
 *       dgamma / dbeta (mode 0 [V*Cin] v*Cin+c with st = (mean, rstd) [V*Cin] of stgcn_bn_finalize; mode 1
 *       [Cin*V] with st = the frame statistics); any output may be NULL.  One pass over dy (windows folded
 *       onto frames); work: stgcn_window_grad_workspace bytes, no initialisation needed. */
int stgcn_window_stat_blocks(int nw, int W);
int stgcn_window_stats(const float* x, int Cin, int Lp, int V, int W, int n0, int nw, int mode, float eps, float* out,
                       void* stream);
int stgcn_window_expand(const float* x, int Cin, int Lp, int V, int W, int n0, int nw, int mode, const float* g,
                        const float* b, const float* fst, const float* w, const float* bias, int Cout, void* out,
                        int ldo, int dtype, void* stream);
long stgcn_window_grad_workspace(int nw, int W, int V, int Cin, int Cout);
int stgcn_window_grad(const void* dy, int ldd, int dtype, const float* x, int Cin, int Lp, int V, int W, int n0, int nw,
                      int mode, const float* st, const float* gamma, const float* beta, const float* w, int Cout,
                      void* work, float* dgamma, float* dbeta, float* dw, float* db, void* stream);

/* Batched weight preparation (prep.hip): every packed operand a model's layers read in one training step —
 * the GEMM packs and MFMA-fragment images of the temporal / residual / head 1x1 convs (stgcn_pack_weight,
 * _frag, _s2frag) and the graph conv's per-joint effective weights with the bias pushed through A
 * (stgcn_gconv_weights_bias), for the forward and the data gradient — in ONE launch instead of ~50
 * (stgcn.py:80-97 as a whole; replaces the per-layer packing of the reference's nn.Conv2d weights, which
 * PyTorch's own kernels read in place).  A job is one of those single-job entry points with the same
 * argument meaning:
 *   kind 0 (pack): src + strides (s0, s1, s2), Kt, Co, Ci -> dst [Kt][cp][kp] (dtype), and the fragment
 *                  image into dst_frag when non-NULL (cp % 32 == 0, kp % 16 == 0);
 *   kind 1 (stride-2 fold, bf16): src + strides, Co, Ci, trans -> dst (stgcn_pack_weight_s2frag);
 *   kind 2 (graph conv): A [P][V][V] (times the edge importance M [P][V][V] when non-NULL: the product the
 *                  model feeds the layer, formed here exactly as a rounded fp32 product), W = src
 *                  [P*Cout][Cin] (Co = Cout, Ci = Cin), nbr / deg support lists, trans, dst [V][J][R_pad]
 *                  [C_pad] (dtype), and for trans 0 with bconv non-NULL bias2d [V][Cout];
 *   kind 3 (graph-conv bias through A alone, the frame-kernel route): A (times M when non-NULL), bconv
 *                  [P*Cout] (Co = Cout) -> bias2d [V][Cout] = sum_p bconv[p*Cout+c] sum_v (A*M)[p][v][w]
 *                  (src = bconv, dst = bias2d, Ci = 1).
 * stgcn_prep_check validates a host-side job array and fills each job's thread count (threads);
 * stgcn_prep_run launches the jobs from a DEVICE copy of that array with block_start [njobs + 1] (device,
 * block_start[j] = first 256-thread block of job j, block_start[njobs] = nblocks). */
typedef struct {
  int kind, dtype, trans, Kt, Co, Ci, cp, kp;
  long s0, s1, s2, threads;
  const float* src;
  void* dst;
  void* dst_frag;
  const float* A;
  const float* M;
  const int* nbr;
  const int* deg;
  int P, V, J, R_pad, C_pad, pad_;
  const float* bconv;
  float* bias2d;
} stgcn_prep_job;
int stgcn_prep_check(stgcn_prep_job* jobs, int njobs);
int stgcn_prep_run(const stgcn_prep_job* jobs_dev, const long* block_start_dev, int njobs, long nblocks,
                   void* stream);

/* Adam over every parameter tensor of a model in one launch (adam.hip).
 * Replaces: the reference's optimizer step, torch.optim.Adam (processor.py:561, built at processor.py:579; optimizer
 * config learning_rate 5e-4, default betas / eps), with torch's update rule:
 *   g' = g + weight_decay * p;  m = lerp(m, g', 1 - b1);  v = b2 v + (1 - b2) g'^2;
 *   p += (-lr / (1 - b1^t)) * (m / (sqrt(v) / sqrt(1 - b2^t) + eps)),   t = the tensor's step count
 * (the default foreach implementation's operation order; hyper-parameters in double, as Python floats).
 * table_dev: device array of stgcn_adam_entry (p: the fp32 parameter, m / v: its moment slices, n elements,
 * b0 = first block of the tensor, b0 increasing, block counts from stgcn_adam_blocks(n); vec = 1 when p, m
 * and v are 16-B aligned).  grads: HOST array of ntensors device gradient pointers (NULL = no gradient:
 * the tensor is skipped, its step count unchanged).  steps: device float [nblocks], every block's copy of
 * its tensor's step count (zero-initialised; the caller reads a tensor's count at its first block). */
#define STGCN_ADAM_MAXT 256
typedef struct {
  float* p;
  float* m;
  float* v;
  long n, b0;
  int vec, pad_;
} stgcn_adam_entry;
long stgcn_adam_blocks(long n);
int stgcn_adam_step(const stgcn_adam_entry* table_dev, int ntensors, long nblocks, const float* const* grads,
                    float* steps, double lr, double beta1, double beta2, double eps, double weight_decay,
                    void* stream);

#ifdef __cplusplus
}
#endif
#endif /* STGCN_AMD_H */
