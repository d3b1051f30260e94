/*
 * stfunet.h -- C ABI of the MI355X (gfx950) STF-Unet training hot path.
 *
 * The reference (XiangFeng-Wen/STF-Unet) has no FFI: its hot path is the
 * PyTorch nn.Module surface of src/unet.py and src/stf_lstm_unet.py plus the
 * engine functions of train_utils/.  Every entry point below replaces the
 * PyTorch/MIOpen kernels behind one op *call site* of that path (cited per
 * function).  The Python host mirror (stf-unet_amd/stfunet) binds them with
 * ctypes; see INTEGRATION.md.
 *
 * Conventions
 *  - Activations: NHWC bf16.  A tensor argument is (pointer to its first used
 *    channel, channel stride in elements) so producers can write straight into
 *    a channel slice of a concat buffer ("virtual concat").
 *  - Weights: bf16, K-contiguous GEMM rows [Nout][R][S][Cs].
 *  - Statistics, master weights, gradients, optimizer state: fp32.
 *  - Every function is stream-ordered on `stream` (a hipStream_t), allocates
 *    nothing, keeps no pointer after it returns and has no mutable global state.
 *  - Return value: 0 on success, a hipError_t code on launch failure, or
 *    STF_EINVAL (100001) when the arguments violate a documented constraint.
 */
#ifndef STFUNET_H
#define STFUNET_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* stf_stream_t; /* hipStream_t */

/* Geometry of one implicit-GEMM pass.  GEMM rows m = (n, yd, xd) walk the
 * destination grid [N][Hd][Wd]; the reduction k = (r, s, c) gathers the source
 * tensor [N][Hs][Ws][Cs]:
 *   transposed == 0 : ys = yd*stride - pad + r        (Conv2d forward, ConvT dgrad)
 *   transposed == 1 : ys = (yd + pad - r) / stride    (Conv2d dgrad, ConvTranspose2d
 *                     forward); taps with a non-zero remainder contribute 0.
 */
typedef struct stf_conv_geom {
  int N;
  int Hs, Ws, Cs;      /* source spatial dims and reduction channels            */
  int src_cstride;     /* elements between consecutive source pixels (>= Cs)   */
  int Hd, Wd;          /* destination (GEMM row) spatial dims                   */
  int R, S;            /* taps                                                  */
  int stride, pad;     /* transposed==1 requires stride in {1, 2}               */
  int transposed;
} stf_conv_geom;

/* LSTM cell fused into the GEMM epilogue: the GEMM computes the gate
 * pre-activations [x_t | h_{t-1}] . [W_ih | W_hh]^T with gate-interleaved
 * columns (column 4c+q = gate q in torch order i, f, g, o, of hidden channel c),
 * the epilogue adds the bias and applies c_t = f*c_{t-1} + i*g, h_t = o*tanh(c_t)
 * (nn.LSTM, src/stf_lstm_unet.py:124-127,219-235). */
typedef struct stf_lstm_epi {
  const float* c_prev; /* [M][Ch] c_{t-1}, or NULL (zero initial state)           */
  float* c_out;        /* forward: c_t out [M][Ch]; backward: c_t in (read only)  */
  void* h_out;         /* bf16, h_t written with stride h_cstride (may be the next */
  int h_cstride;       /* step's [x | h] buffer or the decoder's concat slice)     */
  float* gates;        /* forward: [M][4Ch] activated gates (i, f, g, o), or NULL  */
                       /* when the backward recomputes them (backward = 1)        */
  /* backward = 1: the GEMM recomputes step t's gate pre-activations from the same
   * [x_t | h_{t-1}] rows and weights (same kernel, so bitwise the forward's gates)
   * and the epilogue runs the cell backward (h_out / gates unused):
   *   tc = tanh c_t; dc = dh*o*(1-tc^2) + dc_next; dc_prev = dc*f;
   *   dgates = (dc*g*i(1-i), dc*c_{t-1}*f(1-f), dc*i*(1-g^2), dh*tc*o(1-o)) */
  int backward;
  const void* dh;      /* bf16 dL/dh_t, stride dh_cstride                          */
  int dh_cstride;
  const float* dc_next;/* [M][Ch] dL/dc_t from step t+1, or NULL (t = T-1)          */
  float* dc_prev;      /* [M][Ch] out, dL/dc_{t-1} (may alias dc_next)              */
  void* dgates;        /* bf16 [M][4Ch] pre-activation gate gradients, interleaved */
} stf_lstm_epi;

/* BatchNorm-backward reduction fused into a dgrad: dst receives dz, the gradient
 * w.r.t. act(BN(y)); the epilogue also produces the partial sums of
 * stf_bn_bwd_reduce (g = relu ? dz * [y*scale+shift > 0] : dz; sum g, sum g*xhat)
 * without a separate pass over dz and y.  Affine arrays are [groups][C]. */
typedef struct stf_bnr_epi {
  const void* y;       /* bf16 pre-BN activation [M][y_cstride], first channel      */
  int y_cstride;
  const float* scale; const float* shift; const float* mean; const float* invstd;
  int relu;
  float* partial;      /* [groups][stf_igemm_bnr_tiles][2][C] for stf_bn_bwd_finalize */
} stf_bnr_epi;

typedef struct stf_igemm_args {
  stf_conv_geom g;
  const void* src;     /* bf16, first used channel                              */
  const void* wgt;     /* bf16 [Nout][R*S*Cs]                                   */
  int Nout;            /* GEMM columns; multiple of 8                           */
  void* dst;           /* bf16, first channel of the destination slice          */
  int dst_cstride;
  const float* bias;   /* [Nout] (scatter2x2: [Nout/4]) or NULL                 */
  float* stats;        /* [tiles][2][Nout] per-tile (sum, sum of squares) of    */
                       /* the stored bf16 outputs, or NULL (tiles: see          */
                       /* stf_igemm_stat_tiles)                                 */
  int scatter2x2;      /* 1: ConvTranspose2d(k=2,s=2) epilogue: column          */
                       /* n = (dy*2+dx)*Cout + co lands on pixel (2yd+dy,2xd+dx)*/
                       /* of a [N][2Hd][2Wd] destination                        */
  int group_rows;      /* >0: tiles aligned to groups of this many rows (whole  */
                       /* images) and stats laid out [M/group_rows][tiles][2][Nout] */
                       /* (per-time-step BatchNorm of the batched STF encoder)  */
  int accumulate;      /* 1: dst += result (bf16 read-modify-write)             */
  const stf_lstm_epi* lstm; /* non-NULL: LSTM cell epilogue, dst unused          */
  const stf_bnr_epi* bnr;   /* non-NULL: fused BN-backward reduction (no stats,  */
                            /* no scatter/LSTM); group_rows = the BN's groups    */
  float* ws;           /* split-K fp32 workspace of stf_igemm_ws_bytes(a) bytes */
                       /* (16-B aligned), or NULL when that is 0 (ABI v4)      */
} stf_igemm_args;

/* Workspace bytes stf_igemm needs for these args: > 0 when the GEMM is split over
 * K (small-M layers that would under-fill the chip; the partials are folded by a
 * second launch that also writes the statistics). */
size_t stf_igemm_ws_bytes(const stf_igemm_args* a);

/* Partial-statistics rows per group for these args (the tiling depends on the
 * kernel chosen): size `stats` as groups * stf_igemm_stat_tiles(a) * 2 * Nout. */
int stf_igemm_stat_tiles(const stf_igemm_args* a);
/* Partial rows per group stf_igemm writes into bnr->partial for these args. */
int stf_igemm_bnr_tiles(const stf_igemm_args* a);
/* Device kernel (template instance, as rocprofv3 names it) these args will run;
 * static thread-local string, for per-kernel timers and profile cross-checks. */
const char* stf_igemm_kernel_name(const stf_igemm_args* a);
/* Conv2d 3x3/1x1/strided forward with fused bias + BatchNorm partial statistics
 *   replaces nn.Conv2d in conv_block  (src/unet.py:12,15), ResidualConvBlock
 *   (src/stf_lstm_unet.py:13,16,23), ResNet-34 convs (src/stf_lstm_unet.py:108-114),
 *   out_conv/fusion/pk_fusion 1x1 (src/unet.py:37, src/stf_lstm_unet.py:46,118-121);
 * Conv2d input gradient (transposed gather) for the same layers;
 * ConvTranspose2d(k=2,s=2) forward with scatter epilogue straight into the
 *   concat buffer  (src/unet.py:28-34,47-54) and its input gradient (stride-2 2x2 gather);
 * ConvTranspose2d(k=3,s=2,p=1,op=1) forward (src/stf_lstm_unet.py:43,135). */
int stf_igemm(const stf_igemm_args* a, stf_stream_t stream);

typedef struct stf_wgrad_args {
  stf_conv_geom g;     /* forward geometry; transposed must be 0                */
  const void* dy;      /* bf16 [N*Hd*Wd][dy_cstride], first used channel        */
  int dy_cstride;
  int Nout;            /* columns of dy used; multiple of 8                     */
  const void* x;       /* bf16 source (gathered as in stf_conv_geom)            */
  float* ws;           /* workspace [splits][Nout][R*S*Cs] fp32                 */
  int splits;          /* pixel splits (from stf_wgrad_plan)                    */
  int grid_blocks;     /* workgroups the pixel split aims at (0: two per CU).   */
                       /* A weight gradient running on a side stream beside the */
                       /* dgrad / BatchNorm chain asks for one per CU, so the   */
                       /* chain's kernels still find registers on every CU (ABI v7) */
} stf_wgrad_args;

/* Choose splits and report workspace bytes for a weight-gradient pass. */
int stf_wgrad_plan(const stf_wgrad_args* a, int* splits, size_t* ws_bytes);
/* dW[n][r][s][c] partials = sum over pixels dy[m][n] * x[gather(m,r,s)][c]
 *   replaces the weight gradient of every Conv2d/ConvTranspose2d above. */
int stf_wgrad(const stf_wgrad_args* a, stf_stream_t stream);
/* Device kernel stf_wgrad runs for these args (see stf_igemm_kernel_name). */
const char* stf_wgrad_kernel_name(const stf_wgrad_args* a);
/* Sum `splits` slabs into out[Nout][Cs][R][S] (PyTorch Conv2d weight layout;
 * for ConvTranspose2d pass Nout=Cin, Cs=Cout and get [Cin][Cout][R][S]).
 * Partial-slab arguments of this and the *_finalize / channel-sum functions are
 * scratch: they are reduced in place (fixed order) and left clobbered. */
int stf_wgrad_reduce(float* ws, int splits, int Nout, int R, int S, int Cs,
                     float* out, stf_stream_t stream);

/* Per-channel column sums of a bf16 NHWC tensor (bias gradients of ConvT /
 * 1x1 convs, src/unet.py:28-37).  partial: [ceil(M/256)][C] scratch. */
int stf_channel_sum(const void* x, int x_cstride, int M, int C, float* partial,
                    float* out, stf_stream_t stream);
/* The same column sums taken from the BatchNorm statistics rows [tiles][2][Nout] that an
 * stf_igemm with `stats` produced (the per-tile sums of its stored outputs): out[c] = sum over
 * tiles of the sum half's column c0 + c, c < C.  The UNet's ConvT bias gradients come from the
 * statistics of the dgrad that writes the concat gradient, instead of another pass over it
 * (ABI v17). */
int stf_stat_sums(const float* stats, int tiles, int Nout, int c0, int C, float* out, stf_stream_t stream);

/* ---------------------------------------------------------------- BatchNorm2d
 * Training-mode BatchNorm2d (+ReLU) (src/unet.py:13-17; src/stf_lstm_unet.py:14-17,
 * ResNet bn1/bn2/downsample.1): batch mean, biased variance for normalisation,
 * unbiased variance into running_var, momentum 0.1, eps 1e-5 (torch defaults).
 * `groups` splits the N images into equal statistic groups (per-time-step BN of
 * the batched STF encoder, src/stf_lstm_unet.py:168-186): every group gets its
 * own mean/invstd/scale/shift ([groups][C]) and running stats advance once per
 * group, in order.  UNet passes groups = 1.  Partial-slab inputs are consumed. */
/* stats: [groups][tiles][2][C] from stf_igemm (tiles = per group), or NULL for
 * eval mode (normalise with running_mean/var, no update). */
int stf_bn_finalize(float* stats, int tiles, int groups, int C, int64_t M,
                    const float* gamma, const float* beta, float momentum, float eps,
                    float* running_mean, float* running_var, float* mean, float* invstd,
                    float* scale, float* shift, stf_stream_t stream);
/* Deferred running-statistics update of grouped BatchNorms (groups > 1): a
 * stf_bn_finalize call with running_mean = running_var = NULL leaves every
 * group's (mean, biased var) parked in row 0 of that group's stats slab; one
 * stf_bn_running_batch launch then advances each BatchNorm's running stats
 * group by group, in order (same arithmetic as the in-call update).  descs is a
 * HOST array; the stats slabs must stay alive until the launch has run. */
typedef struct stf_bn_run_desc {
  const float* stats;          /* [groups][tiles][2][C], parked by stf_bn_finalize */
  float* running_mean;
  float* running_var;
  int64_t Mg;                  /* rows per group */
  int tiles, groups, C;
  float momentum;
} stf_bn_run_desc;
int stf_bn_running_batch(const stf_bn_run_desc* descs, int count, stf_stream_t stream);
/* out = act(y*scale + shift [+ res | + res*res_scale + res_shift]) into a
 * channel slice.  Residual: identity shortcut (res_scale NULL) or a BN'd
 * downsample branch (ResNet BasicBlock src/stf_lstm_unet.py:108-114,
 * ResidualConvBlock :29-35).  Optional fused 2x2 max pool (MaxPool2d(2),
 * src/unet.py:25,41-45) into `pooled` [N][H/2][W/2][C] (no residual). */
int stf_bn_act(const void* y, int y_cstride, int N, int H, int W, int C, int groups,
               const float* scale, const float* shift, int relu, const void* res,
               int res_cstride, const float* res_scale, const float* res_shift, void* out,
               int out_cstride, void* pooled, stf_stream_t stream);
/* Backward of BN(+ReLU)(+2x2 max pool):  da = dz + maxpool_bwd(dpool) (either
 * may be NULL), g = da masked by mask_mode (0 none, 1 ReLU recomputed from
 * y*scale+shift, 2 mask_src > 0: ReLU after a residual add), written to g_out
 * [M][C]; partial [groups][tiles][2][C] = (sum g, sum g*xhat), tiles from
 * stf_bn_bwd_tiles. */
int stf_bn_bwd_tiles(int N, int H, int W, int C, int groups, int pooled);
int stf_bn_bwd_reduce(const void* dz, int dz_cstride, const void* dpool, const void* y,
                      int y_cstride, int N, int H, int W, int C, int groups,
                      const float* scale, const float* shift, const float* mean,
                      const float* invstd, int mask_mode, const void* mask_src,
                      int mask_cstride, void* g_out, float* partial, stf_stream_t stream);
/* (g_out may be NULL without dpool: the masked gradient is then not stored and
 * stf_bn_bwd_apply recomputes the mask.) */
/* dgamma, dbeta (summed over groups) and coef [groups][3][C] of dy = A*g + B*y + C. */
int stf_bn_bwd_finalize(float* partial, int tiles, int groups, int C, int64_t M,
                        const float* gamma, const float* mean, const float* invstd,
                        float* dgamma, float* dbeta, float* coef, stf_stream_t stream);
/* Deferred dgamma/dbeta of grouped BatchNorm backwards: stf_bn_bwd_finalize with
 * dgamma = dbeta = NULL and groups > 1 leaves each group's (sum g, sum g*xhat)
 * parked in row 0 of that group's partial slab; stf_bn_groupsum_batch sums them
 * over the groups for many BatchNorms in one launch (descs: HOST array). */
typedef struct stf_bn_gsum_desc {
  const float* partial;        /* [groups][tiles][2][C] */
  float* dgamma;
  float* dbeta;
  int tiles, groups, C;
} stf_bn_gsum_desc;
int stf_bn_groupsum_batch(const stf_bn_gsum_desc* descs, int count, stf_stream_t stream);
/* dy = A*g' + B*y + C (bf16, dy_cstride; may alias g when dense).  g' = g, or
 * with mask_scale/mask_shift ([groups][C], the forward BN affine) the ReLU mask
 * recomputed from y: g' = g where y*scale+shift > 0 else 0 -- then g is the raw
 * incoming gradient (any channel stride) and stf_bn_bwd_reduce ran with
 * g_out = NULL.  Optional per-tile column sums of dy for the bias of the
 * producing conv (bias_partial [stf_bn_bwd_apply_tiles][C]) reduced into dbias. */
int stf_bn_bwd_apply_tiles(int64_t M, int C);
int stf_bn_bwd_apply(const void* g, int g_cstride, const void* y, int y_cstride, int64_t M,
                     int C, int groups, const float* mask_scale, const float* mask_shift,
                     const float* coef, void* dy, int dy_cstride, float* bias_partial,
                     float* dbias, stf_stream_t stream);

/* ---------------------------------------------------------------- head + loss
 * UNet OutConv fused with the last BN+ReLU (src/unet.py:16-17,37,56):
 * logits[b][k][h][w] (fp32 NCHW, the {"out": ...} tensor) =
 * bias[k] + sum_c relu(y*scale+shift)[c] * W[k][c]. */
int stf_head_fwd(const void* y, int N, int H, int W, int C, const float* scale,
                 const float* shift, const float* w, const float* bias, int classes,
                 float* logits, stf_stream_t stream);
/* Backward of the head and the BN+ReLU it absorbed: g = (dlogits . W) * relu',
 * partial (sum g, sum g*xhat) as stf_bn_bwd_reduce, head dW/db partials in
 * head_partial [(tiles+1)][classes*(C+1)] (last row = the reduction) copied
 * into dw (classes*C) and db (classes).  tiles = stf_head_tiles(N, H, W, C). */
int stf_head_bwd(const float* dlogits, const void* y, int N, int H, int W, int C,
                 const float* scale, const float* shift, const float* mean,
                 const float* invstd, const float* w, int classes, void* g_out,
                 float* bn_partial, float* head_partial, float* dw, float* db,
                 stf_stream_t stream);
int stf_head_tiles(int N, int H, int W, int C);

/* criterion (train_utils/train_and_eval.py:299-313) = cross_entropy +
 * multiclass Dice loss on softmax (train_utils/dice_coefficient_loss.py:5-55),
 * branch-free empty-set rule.  terms: stf_loss_scratch_floats() floats; its
 * first N*classes*3 + 1 hold (sum p*t, sum p, sum t) per (image, class) and the
 * CE sum after stf_loss_fwd; loss: device scalar. */
int stf_loss_scratch_floats(int N, int classes);
int stf_loss_fwd(const float* logits, const int64_t* target, int N, int H, int W,
                 int classes, float* terms, float* loss, stf_stream_t stream);
int stf_loss_bwd(const float* logits, const int64_t* target, int N, int H, int W,
                 int classes, const float* terms, const float* grad_out, float* dlogits,
                 stf_stream_t stream);

/* ---------------------------------------------------------------- optimizer
 * torch.optim.AdamW(lr, betas, eps, weight_decay) (train.py:230-237) over one
 * flat fp32 parameter buffer. */
int stf_adamw(float* p, const float* g, float* m, float* v, int64_t n, float lr,
              float beta1, float beta2, float eps, float weight_decay, float bc1,
              float bc2, stf_stream_t stream);
/* Graph-capturable AdamW: hyper = DEVICE {lr, step} (step = this update's count,
 * already incremented); bias corrections computed on the device exactly as the host
 * computes them for stf_adamw. */
int stf_adamw_dev(float* p, const float* g, float* m, float* v, int64_t n, const float* hyper,
                  float beta1, float beta2, float eps, float weight_decay, stf_stream_t stream);
/* AdamW under torch.amp.GradScaler without a host sync (the optimizer advertises
 * _step_supports_amp_scaling, as torch's fused AdamW does, which the reference builds with
 * fused=True, train.py:230-237): grad_scale = DEVICE scale the gradients carry (NULL:
 * already unscaled; multiplied by 1/scale in fp32 = GradScaler.unscale_'s arithmetic),
 * found_inf = DEVICE flag, != 0 skips the update and leaves hyper[1] (the step count)
 * unchanged; otherwise hyper[1] += 1 and the update is stf_adamw_dev's. */
int stf_adamw_amp(float* p, const float* g, float* m, float* v, int64_t n, float* hyper,
                  const float* grad_scale, const float* found_inf, float beta1, float beta2, float eps,
                  float weight_decay, stf_stream_t stream);

/* ---------------------------------------------------------------- layout
 * x [N][C][H][W] fp32 -> NHWC bf16 with Cpad (>= C, multiple of 8) channels,
 * zero-filled (preprocess_input output, train_and_eval.py:9-22). */
int stf_pack_input(const float* x, int N, int C, int H, int W, int Cpad, void* out,
                   stf_stream_t stream);
/* fp32 weights -> bf16 GEMM rows.
 *  mode 0: Conv2d w[Co][Ci][R][S]       -> [Co][R][S][Cipad]   (forward)
 *  mode 1: Conv2d w[Co][Ci][R][S]       -> [Ci][R'][S'][Co]    (dgrad, no flip:
 *          the transposed gather indexes taps directly)
 *  mode 2: ConvT  w[Ci][Co][R][S]       -> [(r*S+s)*Co+co][Ci] (scatter2x2 fwd)
 *  mode 3: ConvT  w[Ci][Co][R][S]       -> [Ci][R][S][Co]      (ConvT dgrad)
 *  mode 4: ConvT  w[Ci][Co][R][S]       -> [Co][R][S][Ci]      (ConvT fwd gather)
 *  mode 5: Conv2d w[Co][Ci][R][S]       -> [Ci][R-1-r][S-1-s][Co] (stride-1 dgrad as a
 *          forward gather with pad' = R-1-pad) */
int stf_pack_weight(const float* w, int d0, int d1, int R, int S, int mode, int cpad,
                    void* out, stf_stream_t stream);
/* Many stf_pack_weight jobs in one launch.  descs: DEVICE array of count
 * descriptors (same fields and modes as stf_pack_weight); max_elems = the
 * largest packed element count among them (sizes the grid). */
typedef struct stf_pack_desc {
  const float* w;
  void* out;
  int d0, d1, R, S, mode, cpad;
} stf_pack_desc;
int stf_pack_weights(const stf_pack_desc* descs, int count, int64_t max_elems, stf_stream_t stream);
/* Same job through LDS-tiled transposes (whole source rows read, 16-B output
 * chunks written).  stf_pack_tiles(d0,d1,R,S,mode,cpad) = the tile count of one
 * descriptor, or -1 when the tiled kernel cannot take it (R*S > 9, or output rows
 * not a multiple of 8 elements); max_tiles = the largest count in the list (every
 * descriptor must have one >= 0).  ABI v5. */
int stf_pack_tiles(int d0, int d1, int R, int S, int mode, int cpad);
int stf_pack_weights_tiled(const stf_pack_desc* descs, int count, int max_tiles, stf_stream_t stream);

/* ---------------------------------------------------------------- STF-LSTM-UNet
 * x [B][Ttot][C][H][W] fp32 -> t-major NHWC bf16 [T*B][H][W][Cpad]: frame t of
 * sample b is image t*B+b; channels [0,C) the frame, [C,C+P) the P PK maps
 * x[b][T+p][0] (src/stf_lstm_unet.py:146-156,172-174), rest zero. */
int stf_pack_sequence(const float* x, int B, int Ttot, int C, int H, int W, int T, int P,
                      int Cpad, void* out, stf_stream_t stream);

/* Stem im2col (replaces the padded-channel input of the 7x7/s2 stem, reference
 * src/stf_lstm_unet.py:108,177): x as for stf_pack_sequence -> bf16
 * [T*B][Ho][Wo][Kpad], column k = ci*KS*KS + r*KS + s (PyTorch weight order),
 * zero padded; the stem conv is then a 1x1 GEMM over Kpad >= (C+P)*KS*KS columns. */
int stf_stem_im2col(const float* x, int B, int Ttot, int C, int H, int W, int T, int P, int KS,
                    int stride, int pad, int Kpad, void* out, stf_stream_t stream);
/* The same stem conv without the im2col tensor (ABI v15): x [B][Ttot][1][H][W] fp32 (frames 0..T-1,
 * no PK maps) -> y NHWC bf16 [T*B][Ho][Wo][64] (Ho = (H-1)/2+1), w = the 64 x 64 bf16 rows the GEMM
 * path packs (column k = r*7 + s, zero for k >= 49).  Bit-identical outputs to the im2col + 1x1 GEMM.
 * stats (NULL: none): BatchNorm partial rows [T][grid][2][64] (sum, sum of squares of the stored
 * bf16 values; grid = stf_stem_conv7_grid(B, T, H, W) rows per time step) for stf_bn_finalize. */
int stf_stem_conv7_grid(int B, int T, int H, int W);
int stf_stem_conv7(const float* x, int B, int Ttot, int H, int W, int T, const void* w, void* y, float* stats,
                   stf_stream_t stream);
/* Its weight gradient without the im2col tensor: dy NHWC bf16 [T*B][Ho][Wo][64] (the stem output's
 * gradient) -> fp32 partial slabs ws [grid][64][64] (dy channel x column k = r*7 + s; columns >= 49
 * zero; grid = stf_stem_conv7_grid(...)), folded with stf_wgrad_reduce(ws, grid, 64, 1, 1, 64, ..). */
int stf_stem_wgrad7(const float* x, int B, int Ttot, int H, int W, int T, const void* dy, float* ws,
                    stf_stream_t stream);
/* Input gradient of that stem conv (7x7/s2/p3, Cf input channels; what autograd returns for the
 * input sequence, src/stf_lstm_unet.py:139-256): dy [T*B][Ho][Wo][64] 16-bit (frame t*B + b), w the
 * fp32 conv1 weight [64][Cf][7][7] -> dx fp32 in the input's layout [B][Ttot][Cf][H][W], frames
 * t < T written (t >= T, the PK maps, untouched).  ABI v16. */
int stf_stem_dgrad7(const void* dy, const float* w, int B, int Ttot, int Cf, int H, int W, int T, float* dx,
                    stf_stream_t stream);
/* MaxPool2d(3, 2, 1) of the ResNet stem (src/stf_lstm_unet.py:110,180), NHWC bf16.
 * argmax (uint8 [N][Ho][Wo][C], NULL in eval) records each window's first maximum
 * (index dy*3+dx, torch's tie rule); backward gathers dout over the <= 4 windows
 * whose recorded maximum is the pixel. */
int stf_maxpool3s2_fwd(const void* x, int N, int H, int W, int C, void* out, void* argmax,
                       stf_stream_t stream);
int stf_maxpool3s2_bwd(const void* argmax, const void* dout, int N, int H, int W, int C, void* dx,
                       stf_stream_t stream);
/* The stem's BatchNorm + ReLU and that max pool in one pass (src/stf_lstm_unet.py:178-180):
 * pooled out and argmax exactly as stf_bn_act (scale / shift of group n / (N / groups), ReLU,
 * 16-bit rounding) followed by stf_maxpool3s2_fwd, without writing the activation.  ABI v11. */
int stf_bn_act_maxpool3s2(const void* y, int N, int H, int W, int C, int groups, const float* scale,
                          const float* shift, void* out, void* argmax, stf_stream_t stream);
/* The stem BatchNorm's backward through that max pool: the gradient of each pixel is gathered
 * from the pooled gradient dout [N][Ho][Wo][C] over the <= 4 windows whose recorded argmax it
 * is (rounded to 16 bits, as stf_maxpool3s2_bwd stores it), masked by the ReLU recomputed from
 * y; reduce -> partials as stf_bn_bwd_reduce (then stf_bn_bwd_finalize), apply -> dy, without
 * the full-size d(activation) tensor.  Same values as stf_maxpool3s2_bwd + stf_bn_bwd_reduce
 * (mask_mode 1) + stf_bn_bwd_apply.  ABI v11. */
int stf_bn_bwd_reduce_pool3(const void* argmax, const void* dout, const void* y, int N, int H, int W, int C,
                            int groups, const float* scale, const float* shift, const float* mean,
                            const float* invstd, float* partial, stf_stream_t stream);
int stf_bn_bwd_apply_pool3(const void* argmax, const void* dout, const void* y, int N, int H, int W, int C,
                           int groups, const float* scale, const float* shift, const float* coef, void* dy,
                           stf_stream_t stream);
/* nn.LSTM(C, C) weights -> gate-interleaved GEMM operands: wcat [4C][2C] (row
 * 4c+q = torch row q*C+c of [W_ih | W_hh]), wcat_t [2C][4C], bias = b_ih + b_hh
 * interleaved (src/stf_lstm_unet.py:124-127).  C in {16, 32, ..., 512} (STF_EINVAL otherwise). */
int stf_lstm_pack(const float* w_ih, const float* w_hh, const float* b_ih, const float* b_hh,
                  int C, void* wcat, void* wcat_t, float* bias, stf_stream_t stream);
/* The whole forward sequence of nn.LSTM(C, C) in one launch (src/stf_lstm_unet.py:214-242):
 * lbuf = [T][P][2C] 16-bit rows of step t = [x_t | h_{t-1}] (x_t given, the h slots of
 * steps 1..T-1 are written here, step 0's is ignored: h_{-1} = 0), wcat / bias from
 * stf_lstm_pack, c_out = [T][P][C] fp32 cell states, h_{T-1} -> h_last (stride h_cstride).
 * Same values as T launches of stf_igemm with the LSTM cell epilogue.  C = 64 only
 * (stf_lstm_seq_supported); 16-B aligned wcat / lbuf. */
int stf_lstm_seq_fwd(const void* wcat, const float* bias, void* lbuf, int P, int T, int C, float* c_out,
                     void* h_last, int h_cstride, stf_stream_t stream);
int stf_lstm_seq_supported(int C);
/* The whole backward (BPTT) of that sequence in one launch: recomputes every step's gates
 * from lbuf (as the forward computed them), runs the cell backward and the input-gradient
 * GEMM; dgates = [T][P][4C] 16-bit pre-activation gate gradients (for the weight gradient
 * afterwards), dx = rows [T][P] of stride dx_cstride receiving dL/dx_t in channels [0, C);
 * dh_last = dL/dh_{T-1} (stride dh_cstride).  Same values as the per-step path (stf_igemm
 * with the LSTM backward epilogue + the dgates x W GEMM).  C = 64 only; 16-B alignment. */
int stf_lstm_seq_bwd(const void* wcat, const void* wcat_t, const float* bias, const void* lbuf, int P, int T,
                     int C, const float* c_all, const void* dh_last, int dh_cstride, void* dgates, void* dx,
                     int dx_cstride, stf_stream_t stream);
/* Whole-sequence forward for C = 128 / 256 / 512 (stf_lstm_coop_supported) in ONE persistent
 * launch: the 4C gate rows are cut into C/32 slices of 128; the C/32 workgroups of a 64-pixel
 * block keep their weight slice in registers and hand h_t to each other through lbuf inside
 * the launch (agent-scope counters, write-through stores, an acquire per step).  Same
 * arguments, layout and values (bit for bit) as stf_lstm_seq_fwd / the per-step path, plus
 * `sync`: a caller-owned device buffer of stf_lstm_coop_sync_bytes(P, T) bytes (16-B aligned;
 * zeroed on the stream by the call itself; its last word is an error flag: nonzero = a step's
 * hand-off timed out, after which the launch drains at once with wrong values).  spin_limit: polls
 * before a hand-off gives up (0 = the default, ~4 s; 0xFFFFFFFF = every hand-off reports a timeout
 * at once: the error path, for tests).  ABI v12. */
size_t stf_lstm_coop_sync_bytes(int P, int T);
int stf_lstm_coop_supported(int C);
int stf_lstm_coop_fwd(const void* wcat, const float* bias, void* lbuf, int P, int T, int C, float* c_out,
                      void* h_last, int h_cstride, float* gates, unsigned* sync, int max_wg, unsigned spin_limit,
                      stf_stream_t stream);
/* gates (or NULL): [T][P][4C] fp32 activated gates (i, f, g, o interleaved per channel), kept
 * for stf_lstm_coop_bwd: the BPTT of the same sequence in one persistent launch (same
 * workgroup grid; per step the C/32 workgroups of a pixel block exchange the dgates rows and
 * then [dx_t | dh_{t-1}] in-launch).  Outputs as stf_lstm_seq_bwd: dgates [T][P][4C] 16-bit,
 * dx rows [T][P] of stride dx_cstride (>= 2C) receiving [dx_t | dh_{t-1}]; dh_last = dL/dh_{T-1}.
 * Same values as the per-step path (bit for bit where its dgates x W GEMM is not split over
 * K).  `sync` as for the forward (re-zeroed by the call).  max_wg (both directions): at most this
 * many workgroups (one per CU; 0 = one per CU of the device) -- a launch on a side stream beside
 * other work leaves the rest of the chip to it (a group of C/32 must fit). */
int stf_lstm_coop_bwd(const void* wcat_t, const float* gates, const float* c_all, int P, int T, int C,
                      const void* dh_last, int dh_cstride, void* dgates, void* dx, int dx_cstride,
                      unsigned* sync, int max_wg, unsigned spin_limit, stf_stream_t stream);
/* sticky |= the error word of the launch that used `sync` (stream-ordered, no host sync): a program
 * keeps one sticky device word across steps and reads it back at a step boundary. */
int stf_lstm_coop_error(const unsigned* sync, int P, int T, unsigned* sticky, stf_stream_t stream);
/* The DecoderBlock's size fallback (src/stf_lstm_unet.py:56-57): F.interpolate(mode="bilinear",
 * align_corners=True) of x [N][H][W] (C channels, stride x_cstride, 16-bit NHWC) to y [N][h][w]
 * (stride y_cstride; e.g. the concat slice), PyTorch's coordinate arithmetic; and its backward,
 * dx [N][H][W] = the gather of dy [N][h][w] (no atomics: each input pixel sums the output pixels
 * that read it, in a fixed order).  C % 8 == 0, strides % 8 == 0, 16-B aligned.  ABI v12. */
int stf_bilinear_ac_fwd(const void* x, int N, int H, int W, int C, int x_cstride, void* y, int h, int w,
                        int y_cstride, stf_stream_t stream);
int stf_bilinear_ac_bwd(const void* dy, int N, int h, int w, int C, int dy_cstride, void* dx, int H, int W,
                        int dx_cstride, stf_stream_t stream);
/* The PK maps' share of the input gradient (ABI v17): dy = T frames of B images [T*B][h][w] (t-major,
 * channels [0, 8) of stride dy_cstride, 16-bit NHWC), summed over the frames in fp32 at (h, w) and taken
 * back through the same resize; channels [0, P) (P <= 8) are ADDED to the fp32 out[b*out_bstride +
 * c*out_cstride + y*W + x] (x [B][T+P][1][H][W]: out = &x[0][T], strides (T+P)*H*W and H*W). */
int stf_bilinear_ac_bwd_tsum(const void* dy, int T, int B, int h, int w, int dy_cstride, int P, float* out,
                             int64_t out_bstride, int64_t out_cstride, int H, int W, stf_stream_t stream);
/* dwcat [4C][2C] / dbias [4C] (interleaved) -> torch-layout dW_ih, dW_hh, db_ih, db_hh. */
int stf_lstm_unpack_grad(const float* dwcat, const float* dbias, int C, float* dw_ih,
                         float* dw_hh, float* db_ih, float* db_hh, stf_stream_t stream);
/* One BPTT step of the LSTM cell: from activated gates [M][4C], c_t, c_{t-1}
 * (NULL = 0), dh_t (bf16, stride) and dc from step t+1 (NULL = 0) -> dgates
 * (pre-activation, bf16 [M][4C] interleaved) and dc for step t-1 (may alias dc_in). */
int stf_lstm_cell_bwd(const float* gates, const float* c_t, const float* c_prev, const void* dh,
                      int dh_cstride, const float* dc_in, float* dc_out, void* dgates, int64_t M,
                      int C, stf_stream_t stream);
/* F.interpolate(pk, (h, w), bilinear, align_corners=True) of the PK maps of x,
 * written for every time step into channels [coff, coff+P) of dst
 * [T*B][h][w][dst_cstride] (PK fusion concat, src/stf_lstm_unet.py:189-200). */
int stf_pk_resize(const float* x, int B, int Ttot, int T, int P, int H, int W, int h, int w,
                  void* dst, int dst_cstride, int coff, stf_stream_t stream);

/* ---------------------------------------------------------------- evaluation
 * One pass over a batch's logits [B][K][HW] (fp32, NCHW) and int64 targets [B][HW]
 * (train_utils/train_and_eval.py:30-39, 80-118, 316-336): pred = first argmax over K;
 * confmat [K][K] += (target t in [0,K)) at [t][pred]; dice_counts [K][3] += per-class
 * (|P&T|, |P|, |T|) after multiplying pred and target by (target != ignore_index)
 * when ignore_index >= 0 (the reference's DiceCoefficient masking).  Both outputs are
 * int64 device arrays that ACCUMULATE (zero them first).  K <= 16. */
int stf_eval_counts(const float* logits, const int64_t* target, int B, int K, int64_t HW,
                    int64_t ignore_index, int64_t* confmat, int64_t* dice_counts, stf_stream_t stream);
/* The same pass with the Dice prediction taken from probs (same layout): the first argmax
 * of torch.softmax(logits, 1), which is what DiceCoefficient.update argmaxes
 * (train_and_eval.py:84-85) -- fp32 softmax can round logits that differ by less than an
 * ulp of exp() into a tie that argmax(logits) would not see.  The confusion matrix keeps
 * the logits' argmax (evaluate(), :331).  ABI v9. */
int stf_eval_counts_sm(const float* logits, const float* probs, const int64_t* target, int B, int K,
                       int64_t HW, int64_t ignore_index, int64_t* confmat, int64_t* dice_counts,
                       stf_stream_t stream);

/* ---------------------------------------------------------------- PK maps (extended Tofts)
 * pk_fitting.py ToftsModelFitter, all fp32.  The host builds
 * the reference's constant tables exactly as the reference does (pk_fitting.py:
 * 193-203): time_points t[T], cp_t = Cp(t), the convolution grid tau = arange(0,
 * t[T-1], dt) and cp_tau = Cp(tau) (n_conv entries), and n_valid[i] = #{tau_j < t_i}
 * (device int array).  T <= 32, n_conv <= 8192. */
/* C[P][T] = extended_tofts_model_batch(t, ktrans, ve, vp) (pk_fitting.py:193-231). */
int stf_tofts_forward(const float* ktrans, const float* ve, const float* vp, int P, int T,
                      const float* time_points, const float* cp_t, const float* tau,
                      const float* cp_tau, const int* n_valid, int n_conv, float dt, float* out,
                      stf_stream_t stream);
/* The fit loop of fit_volume_gpu (pk_fitting.py:280-365) for P tissue curves [P][T]
 * (row-major pixel order): batches of `batch` pixels, `epochs` passes, torch Adam
 * over the whole parameter vectors after every batch (pixels outside the batch take
 * a zero-gradient step), clamps after each step.  params [3][P] (Ktrans, ve, vp):
 * initial values in, fitted values out.  adam_sched: DEVICE [epochs*nbatches][2] =
 * (lr / (1 - beta1^s), sqrt(1 - beta2^s)) for s = 1.. (double-precision bias
 * corrections rounded to fp32, as torch applies them).  bounds: HOST [3][2] clamp
 * ranges. */
int stf_tofts_fit(const float* curves, int P, int T, const float* time_points, const float* cp_t,
                  const float* tau, const float* cp_tau, const int* n_valid, int n_conv, float dt,
                  int batch, int epochs, const float* adam_sched, float beta1, float beta2, float eps,
                  const float* bounds, float* params, stf_stream_t stream);

/* ---------------------------------------------------------------- training augmentation
 * Replaces the per-sample CPU transforms of the reference's DataLoader workers
 * (transforms.py:18-157 as composed by train.py:51-73 get_transform; my_dataset.py:
 * 200-239 applies them per frame): RandomResize (Pillow bilinear / nearest) ->
 * RandomHorizontalFlip -> RandomVerticalFlip -> RandomRotation (Pillow bilinear /
 * nearest, expand=False) -> RandomCrop (zero pad) -> ToTensor + Normalize, bit-exact
 * to Pillow 12's integer / double arithmetic.  The host draws the random parameters
 * (Python `random`, the reference's draw order), builds Pillow's coefficient tables
 * and fills one descriptor per frame / mask; sources of any sizes sit in one uint8
 * arena (src offsets in bytes).
 *
 * frames: coefficient rows at coef[cx + j*(kx+2)] = {xmin, n, k_0..k_{kx-1}} for
 * output column j (likewise cy/ky for rows; 22-bit fixed point, Pillow
 * ImagingResample); the resized H2 x W2 image goes to scratch[rs]; the output
 * window oh x ow (crop origin h0, w0 in the zero-padded rotated image) is written
 * as fp32 (v/255 - mean)/std at out[out + y*ow + x].  m = Image.rotate's inverse
 * affine (double), used when flags & STF_AUG_ROTATE.
 * masks: cx / cy index int tables of W2 / H2 source columns / rows (-1 = outside,
 * Pillow ImagingScaleAffine), fx = {a0, a1, a3, a4, xo, yo} 16.16 fixed-point
 * rotation; output int64.
 * max_resized_px / max_out_px = largest H2*W2 / oh*ow in the list (grid size). */
#define STF_AUG_HFLIP 1
#define STF_AUG_VFLIP 2
#define STF_AUG_ROTATE 4
typedef struct stf_aug_frame {
  int64_t src, rs, out;
  int H, W, H2, W2;
  int cx, cy, kx, ky;
  int oh, ow, h0, w0;
  int flags;
  int fx[6];
  int pad_;
  double m[6];
} stf_aug_frame;
int stf_augment_frames(const uint8_t* src, const stf_aug_frame* frames, int n, const int* coef,
                       uint8_t* scratch, int max_resized_px, int max_out_px, float mean, float stdv,
                       float* out, stf_stream_t stream);
int stf_augment_masks(const uint8_t* src, const stf_aug_frame* masks, int n, const int* tabs,
                      int max_out_px, int64_t* out, stf_stream_t stream);

/* ---------------------------------------------------------------- launch plans
 * The native step runtime behind the models' forward / backward (stfunet/plan.py).
 * The reference's step is Python issuing one PyTorch op per layer and per LSTM time
 * step (src/stf_lstm_unet.py:168-254 forward, its autograd backward;
 * train_utils/train_and_eval.py:384-404); here the first steps of a shape run the
 * programs' schedule from Python and one of them RECORDS it: while a plan records on
 * the calling thread, every launch, async memset / device copy and stream wait of
 * this library executes as usual and is appended to the plan with its final
 * arguments (tile choices, split plans, workspace pointers resolved).  Later steps
 * replay ranges of it with stf_plan_replay: the same kernels, streams and events,
 * bit for bit the recorded step's results, no per-launch host logic.  The caller
 * keeps every buffer the recorded step touched alive at its address.
 * These are the only entry points that keep state: a plan owns its ops and events
 * (stf_plan_destroy frees them); the recording flag is per host thread.
 *
 * stf_plan_tag(name, flops) / stf_plan_tag_end(): while recording, mark the ops of
 * the following C-ABI call (a kernel family and its algorithmic FLOPs: bench.py's
 * roofline); stf_plan_replay(.., timed_tag) brackets every range with that name by
 * HIP events on its stream, stf_plan_timing sums them (and synchronizes).
 * stf_stream_wait: `waiter` waits for the work enqueued on `waitee` so far (an
 * event record + stream wait; recorded like a launch).
 * stf_memset / stf_copy_rows (dst[r][0:cols] = src[r][0:cols], fp32, row strides in
 * elements) / stf_i64_add_batch (*ptrs[i] += inc: BatchNorm num_batches_tracked):
 * the step's remaining tensor ops as plan-recordable launches. */
typedef struct stf_plan stf_plan;
stf_plan* stf_plan_create(void);
void stf_plan_destroy(stf_plan* plan);
int stf_plan_record(stf_plan* plan);
int stf_plan_stop(void);
int stf_plan_size(const stf_plan* plan);
int stf_plan_tag(const char* name, double flops);
int stf_plan_tag_end(void);
int stf_plan_replay(stf_plan* plan, int first, int last, const char* timed_tag);
int stf_plan_timing(stf_plan* plan, int* launches, double* ms, double* flops);
int stf_stream_wait(stf_stream_t waiter, stf_stream_t waitee);
int stf_memset(void* p, int value, size_t bytes, stf_stream_t stream);
int stf_copy_rows(const float* src, int64_t src_ld, float* dst, int64_t dst_ld, int rows, int cols,
                  stf_stream_t stream);
int stf_i64_add_batch(int64_t* const* ptrs, int count, int64_t inc, stf_stream_t stream);

const char* stf_error_string(int code);
int stf_abi_version(void);

/* 16-bit activation storage this library was built for: every entry point above
 * reads and writes its 16-bit tensors (activations, packed weights, gradients w.r.t.
 * activations) in this type.  libstfunet_hip.so = bf16, libstfunet_hip_f16.so = fp16
 * (the reference's autocast(float16) + GradScaler path, train_and_eval.py:389,
 * train.py:240); same entry points, layouts and constraints otherwise. */
#define STF_STORAGE_BF16 0
#define STF_STORAGE_FP16 1
int stf_storage_type(void);

#ifdef __cplusplus
}
#endif
#endif /* STFUNET_H */
