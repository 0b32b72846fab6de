/*
 * ugpg.h -- C-ABI of libugpg.so, the MI355X (gfx950) hot path of the
 * Uncertainty-Guided Progressive U-Net (reference: tridang04022004/UG-PG-UNet).
 *
 * The reference has no FFI: all of its hot-path arithmetic is PyTorch ATen
 * calls made from Python.  Each entry point below
 * replaces one family of those calls; the reference call site it replaces is
 * cited next to it.  The Python host layer (ug-pg-unet_amd/ugpg/_C.py) binds
 * these with ctypes and keeps the reference's module/trainer API on top.
 *
 * Conventions
 *  - Plain pointers + sizes only; no torch types cross this boundary.
 *  - Activations are NHWC fp32 ([B][H][W][C], C fastest) unless an entry says NCHW.
 *  - Every entry returns 0 on success or a negative UGPG_ERR_* code; the message is
 *    in ugpg_last_error() (thread-local).  No C++ exception crosses the ABI.
 *  - `stream` is a hipStream_t (torch.cuda.current_stream().cuda_stream).  All work
 *    is stream-ordered; nothing allocates, frees or synchronises (graph-capturable).
 *  - The caller owns every buffer, including workspaces sized by *_workspace().
 */
#ifndef UGPG_H_
#define UGPG_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define UGPG_OK 0
#define UGPG_ERR_INVALID (-1)     /* bad argument / unsupported shape */
#define UGPG_ERR_LAUNCH (-2)      /* hipGetLastError after a launch */
#define UGPG_ERR_WORKSPACE (-3)   /* workspace too small */
#define UGPG_ERR_COMM (-4)        /* RCCL / device error in a ugpg_comm_* call */

const char* ugpg_version(void);
/* Content hash of the sources and flags this library was built from (build.py
 * source_id()); the Python layer refuses a library whose id differs from its tree. */
const char* ugpg_build_id(void);
const char* ugpg_last_error(void);

/* A lazily-activated NHWC operand: value = relu(scale[c]*x + shift[c]) when
 * scale != NULL (train/eval BatchNorm + ReLU folded into the consumer's load,
 * UG_unet_parts.py:11-12,14-15), else x.  `C` is the channel count (stride). */
typedef struct {
    const float* data;
    const float* scale;
    const float* shift;
    int C;
    /* the same activation stored in bf16 (round to nearest even): with data == NULL the
     * only storage (the bf16 arithmetic's activation storage, read by the single-piece
     * persistent conv forms, their weight gradient, max-pool, bilinear x2, the heads,
     * avgpool and BatchNorm backward); with data != NULL an optional copy the
     * single-piece persistent conv forms read instead; NULL: none */
    const void* data_bf16;
} ugpg_src_t;

/* ---- 3x3 convolution, padding 1, stride 1 (UG_unet_parts.py:10,13) ---------
 * Implicit GEMM with LDS-staged halo tiles, in one of two fp32-accurate
 * arithmetic forms selected by the weight pack format `wfmt`:
 *   UGPG_WFMT_F32: v_mfma_f32_32x32x2_f32 (exact fp32 FMA chains);
 *   UGPG_WFMT_X6:  split-bf16 -- every operand split exactly into 3 bf16 pieces,
 *                  6 v_mfma_f32_32x32x16_bf16 products per k-step with fp32
 *                  accumulation (product error < 2^-25 relative, below one fp32
 *                  rounding); needs K channels % 16 == 0 and N % 64 == 0.
 *   UGPG_WFMT_BF16: bf16 arithmetic (BASELINE.json configs[2]) -- operands rounded
 *                  to bf16 (round to nearest even), one v_mfma_f32_32x32x16_bf16
 *                  product per k-step, fp32 accumulation; the output is stored in
 *                  bf16 when out_bf16 is set (out[0] == NULL: 2 bytes per value,
 *                  BatchNorm partials of the rounded values -- what
 *                  torch.autocast(bfloat16) does to a conv output), else in fp32
 *                  (the data gradients); same shape rules.
 * Input = channel-concat of src[0] and src[1] (src[1].data may be NULL):
 * this is the concat-free `torch.cat([x2, x1], dim=1)` of Up (UG_unet_parts.py:80).
 * Cin = src[0].C + src[1].C must be a multiple of 8 (pad the image to 8 channels).
 * Output channels [0, out_split) go to out[0] (channel stride out_split) and
 * [out_split, Cout) to out[1] (stride Cout - out_split); out_split == Cout for one
 * output.  accumulate[i] != 0 adds into out[i].  When `stats` != NULL the kernel
 * also writes per-tile BatchNorm partials [3][Cout][n] = (count, sum, M2) for
 * ugpg_bn_finalize, n = ugpg_conv3x3_fwd_ntiles(B, H, W, Cin, Cout, wfmt);
 * `stats_slots` is the buffer's capacity in slots (it holds 3*Cout*stats_slots
 * floats): a call whose n exceeds it fails with UGPG_ERR_WORKSPACE and writes nothing.
 * The kernel form, its tiling and hence n depend only on the shape and wfmt (there are
 * no runtime tuning knobs). */
typedef struct {
    int B, H, W;
    ugpg_src_t src[2];
    const void* wpk;       /* packed by ugpg_pack_conv3x3 in format wfmt */
    const float* bias;     /* [Cout] or NULL */
    int Cout;
    float* out[2];
    int out_split;
    int accumulate[2];
    float* stats;
    int stats_slots;       /* capacity of stats in slots (see above) */
    int wfmt;              /* UGPG_WFMT_F32, UGPG_WFMT_X6 or UGPG_WFMT_BF16 */
    /* Optional BatchNorm-backward partials of the output, for a data gradient whose
     * output da = dL/d(relu(bn(y))) feeds ugpg_bn_relu_bwd_partials (the reduction half
     * of ugpg_bn_relu_bwd, done while the output tile is in registers): when bnb_part
     * != NULL (one output, no accumulate, Cout % 4 == 0) the call also writes
     * bnb_part[3][Cout][slots] = per-slot (sum g, sum g*xhat, sum xhat) with
     * g = da*[scale*y+shift > 0], xhat = (y-mean)*invstd, y = bnb_y (NHWC, Cout
     * channels), slots = ugpg_conv3x3_fwd_ntiles(...), which must not exceed bnb_slots
     * (the capacity of bnb_part in slots; else UGPG_ERR_WORKSPACE).  Forms whose
     * epilogue does not fuse it run the reduction as a separate pass, same layout. */
    const float* bnb_y;
    const void* bnb_y_bf16;  /* the BN input stored in bf16 instead (bnb_y == NULL) */
    const float* bnb_mean;
    const float* bnb_invstd;
    const float* bnb_scale;
    const float* bnb_shift;
    float* bnb_part;
    int bnb_slots;         /* capacity of bnb_part in slots */
    /* bf16 output (one output, no accumulate): with out[0] != NULL a copy written beside
     * it; with out[0] == NULL the only storage of the output (the bf16 arithmetic's
     * activation storage: the BatchNorm partials then describe the rounded values; with
     * bnb_part, the bf16 arithmetic's data gradient, whose BatchNorm-backward partials
     * then describe the rounded da and need bnb_y_bf16) -- supported by the persistent
     * single-piece form (images >= 32 wide) and the image-layer kernel */
    void* out_bf16;
} ugpg_conv_t;

#define UGPG_WFMT_F32 0
#define UGPG_WFMT_X6 1
#define UGPG_WFMT_BF16 2

/* Replaces aten::convolution forward (cuDNN/oneDNN) for DoubleConv's 3x3 convs. */
int ugpg_conv3x3_fwd(const ugpg_conv_t* p, void* stream);
/* number of BatchNorm partial slots the forward writes (size stats as 3*Cout*ntiles);
 * a function of the shape and the weight format only */
int ugpg_conv3x3_fwd_ntiles(int B, int H, int W, int Cin, int Cout, int wfmt);

/* Weight repack from OIHW fp32 [Cout][Cin][3][3].
 *  mode 0 (forward):  N = Cout, K = Cin_pad, wpk = W[co][ci][t]
 *  mode 1 (dgrad):    N = Cin_pad, K = Cout,  wpk = W[co][ci][8-t]
 *    (the data-gradient of a 3x3/p1 conv is the forward conv of dY with the
 *     180-degree-rotated, channel-transposed kernel; replaces aten
 *     convolution_backward's grad_input)
 *  wfmt F32: fp32 [K/8][9][N][8];  wfmt X6: bf16 [N/64][K/16][3 pieces][2][9][64][8]
 *  ugpg_pack_conv3x3_bytes gives the size of wpk. */
size_t ugpg_pack_conv3x3_bytes(int Cout, int Cin_pad, int wfmt);
int ugpg_pack_conv3x3(const float* w_oihw, void* wpk, int Cout, int Cin, int Cin_pad,
                      int mode, int wfmt, void* stream);
/* Many ugpg_pack_conv3x3 calls of one split-bf16 format (UGPG_WFMT_X6 / _BF16) in
 * one launch (a step's forward and data-gradient packs): same bytes per item. */
typedef struct {
    const float* w;        /* OIHW fp32 [Cout][Cin][3][3] */
    void* wpk;             /* ugpg_pack_conv3x3_bytes(Cout, Cin_pad, wfmt) bytes */
    int Cout, Cin, Cin_pad, mode;
} ugpg_pack_item_t;
int ugpg_pack_conv3x3_batch(const ugpg_pack_item_t* items, int n, int wfmt, void* stream);

/* Weight gradient (aten convolution_backward grad_weight/grad_bias, K3):
 *   dw[co][ci][ky][kx] (+)= sum_p dy[p][co] * act(x)[p + (ky-1,kx-1)][ci]
 *   db[co] (+)= sum_p dy[p][co]
 * Deterministic split-K over pixel tiles (no float atomics). dw is OIHW with
 * Cin_real input channels (<= the padded Cin of src). */
typedef struct {
    int B, H, W;
    ugpg_src_t src[2];
    const float* dy;       /* NHWC [B][H][W][Cout] ... */
    const void* dy_bf16;   /* ... or stored in bf16 (dy == NULL: math UGPG_WFMT_BF16 with
                              64-channel sources and no db; what the bf16 arithmetic reads) */
    int Cout;
    float* dw;
    int Cin_real;
    float* db;             /* [Cout] or NULL */
    int accumulate;
    int math;              /* UGPG_WFMT_X6 (split-bf16) or UGPG_WFMT_BF16 (bf16) MFMA
                              where the shape allows (db == NULL, 64-channel
                              sources); else fp32 MFMA */
    /* Optional: dy formed while loading from the BatchNorm(+ReLU) backward of the layer
     * that follows (dy == dy_bf16 == NULL): dy = ugpg_bn_relu_bwd's apply of (da, y) with
     * the coefficients ugpg_bn_relu_bwd_partials left in its workspace when called with
     * dy == dy_bf16 == NULL, bit-identical to it; dy_out (nullable) receives that dy, the
     * operand of the data gradient, written once per pixel -- the BatchNorm-backward apply
     * pass folded into the weight gradient.  UGPG_WFMT_X6 math, fp32 sources, da, y and
     * dy_out, Cout % 64 == 0, 64-channel sources, db == NULL; or the image layer's form
     * (one 8-channel source without activation, Cout == 64, Cin_real <= 3, dy_out == NULL:
     * its dy has no other reader; any math; y fp32 or stored in bf16, y_bf16).  With route_src / route_argmax (the split-bf16 form):
     * da = the MaxPool2d backward of route_src routed by route_argmax (as
     * ugpg_bn_relu_bwd_partials_routed's UGPG_ROUTE_MAXPOOL2) plus `da` when da != NULL.
     * NULL: off. */
    const struct ugpg_bn_lazy* dy_bn;
} ugpg_wgrad_t;
typedef struct ugpg_bn_lazy {
    const float* da;       /* NHWC [B][H][W][Cout]: dL/d(relu(bn(y))) */
    const float* y;        /* NHWC [B][H][W][Cout]: the BatchNorm input */
    const float* mean;
    const float* invstd;
    const float* scale;
    const float* shift;
    const float* coef;     /* [2][Cout]: the first 2*Cout floats of that workspace */
    float* dy_out;         /* NHWC [B][H][W][Cout] or NULL; must not alias da or y */
    const float* route_src;       /* NHWC [B][H/2][W/2][Cout] pooled-output gradient or NULL */
    const uint8_t* route_argmax;  /* its window argmax (ugpg_maxpool2_fwd), or NULL */
    const void* y_bf16;    /* y stored in bf16 (y == NULL): the image layer's weight gradient only */
} ugpg_bn_lazy_t;
size_t ugpg_conv3x3_wgrad_workspace(const ugpg_wgrad_t* p);
int ugpg_conv3x3_wgrad(const ugpg_wgrad_t* p, void* ws, size_t ws_bytes, void* stream);

/* ---- BatchNorm2d (eps, momentum) -------------------------------------------
 * Train: combine the conv's tile partials (Chan merge in fp64), produce
 * mean/invstd and the folded (scale, shift) = (g*invstd, b - mean*g*invstd),
 * update running stats with the unbiased variance, num_batches_tracked += 1.
 * Replaces aten::native_batch_norm (train) at UG_unet_parts.py:11,14 (K4). */
int ugpg_bn_finalize(const float* stats, int ntiles, int C, const float* gamma,
                     const float* beta, float* running_mean, float* running_var,
                     int64_t* num_batches_tracked, float momentum, float eps,
                     float* mean, float* invstd, float* scale, float* shift, void* stream);
/* Synchronised BatchNorm across data-parallel ranks (SURVEY.md §8e's optional policy: the
 * reference's train-mode BN normalises over the whole batch, UG_unet_parts.py:11,14, which
 * a sharded batch only reproduces with a cross-rank exchange).  Forward:
 * ugpg_bn_stats_pack merges this rank's tile partials into fp64 (N, mean, M2) per channel,
 * out[3][C] (the caller places it in its rank's row of a zeroed [nranks][3][C] buffer and
 * SUM-all-reduces it); ugpg_bn_finalize_merged merges the rows in rank order (Chan) and
 * finalizes from the global statistics exactly as ugpg_bn_finalize does from tiles. */
int ugpg_bn_stats_pack(const float* stats, int ntiles, int C, double* out, void* stream);
int ugpg_bn_finalize_merged(const double* merged, int nranks, int C, const float* gamma,
                            const float* beta, float* running_mean, float* running_var,
                            int64_t* num_batches_tracked, float momentum, float eps,
                            float* mean, float* invstd, float* scale, float* shift,
                            void* stream);
/* Eval: (scale, shift) from running stats (K5). */
int ugpg_bn_eval_params(const float* gamma, const float* beta, const float* running_mean,
                        const float* running_var, float eps, int C, float* scale,
                        float* shift, void* stream);
/* Backward of relu(bn(y)) given da = dL/d(relu output) (K6+K7):
 *   g = da * [scale*y+shift > 0];  dgamma = sum g*xhat;  dbeta = sum g
 *   dy = scale * (g - mean(g) - xhat*mean(g*xhat))
 * dy may alias da.  dgamma/dbeta written (or accumulated).  dconv_bias (nullable)
 * receives sum_p dy = -scale*mean(g*xhat)*sum(xhat), evaluated in fp64: the bias
 * gradient of the conv that produced y (the reference's aten value is the same
 * sum in fp32; both are ~0 because train-mode BN cancels a preceding bias). */
size_t ugpg_bn_relu_bwd_workspace(int64_t npix, int C);
/* The same from partials a data gradient wrote (ugpg_conv_t.bnb_part, nslots slots):
 * finalize + apply only; workspace ugpg_bn_relu_bwd_partials_workspace(C).  With
 * dy == dy_bf16 == NULL the finalize only (dgamma, dbeta, dconv_bias, and the apply's
 * coefficients in the first 2*C floats of ws, for ugpg_wgrad_t.dy_bn). */
size_t ugpg_bn_relu_bwd_partials_workspace(int C);
/* Backward partials as a pass (when no producer wrote them): part [3][C][nslots]. */
int ugpg_bn_relu_bwd_reduce(const float* da, const float* y_f32, const void* y_bf16,
                            int64_t npix, int C, const float* mean, const float* invstd,
                            const float* scale, const float* shift, float* part, int nslots,
                            void* stream);
/* Synchronised BatchNorm backward: ugpg_bn_bwd_partials_pack sums the slots per channel
 * in fp64, out[3][C] = (sum g, sum g*xhat, sum xhat), and out[3C] = npix (this rank's
 * pixel count); after a SUM all-reduce of the 3C+1 values, ugpg_bn_bwd_partials_unpack
 * writes sums * npix / N_global (N_global = the all-reduced out[3C]) into slot 0 and zeroes
 * the others, so the finalize above (which divides by the local npix) sees the global means
 * (torch SyncBatchNorm's backward) for any shard sizes, and dgamma / dbeta / dconv_bias
 * average over ranks to the global-batch gradient. */
int ugpg_bn_bwd_partials_pack(const float* part, int nslots, int C, int64_t npix, double* out,
                              void* stream);
int ugpg_bn_bwd_partials_unpack(const double* sums, int64_t npix, float* part, int nslots,
                                int C, void* stream);
/* BatchNorm-backward partials folded into the kernel that last writes da (the pooling,
 * upsampling and head backward entries *_bnb): same partial layout, nslots from
 * ugpg_bnb_slots(npix, C) (0 for unsupported shapes). */
typedef struct {
    const float* y;        /* NHWC [npix][C]: the BN input (fp32) ... */
    const void* y_bf16;    /* ... or stored in bf16 (y == NULL; the bf16 arithmetic) */
    const float* mean;
    const float* invstd;
    const float* scale;
    const float* shift;
    float* part;           /* [3][C][nslots] */
    int nslots;
} ugpg_bnb_t;
int ugpg_bnb_slots(int64_t npix, int C);
/* (y: the BN input in fp32, or y == NULL and y_bf16 its bf16 storage) */
/* dy: fp32, or dy == NULL and dy_bf16 receives it rounded to bf16 (nearest even) -- under
 * the bf16 arithmetic exactly the operand its data and weight gradients read (one of the
 * two, never both).  da: fp32, or da == NULL and da_bf16 its bf16 storage (the bf16
 * arithmetic's data gradient written by ugpg_conv3x3_fwd with out_bf16 and bnb_part; y and
 * dy then in bf16 too). */
int ugpg_bn_relu_bwd_partials(const float* part, int nslots, const float* da,
                              const void* da_bf16, const float* y,
                              const void* y_bf16, int64_t npix, int C, const float* mean,
                              const float* invstd, const float* scale, const float* shift,
                              float* dy, void* dy_bf16, float* dgamma, float* dbeta,
                              float* dconv_bias, int accumulate_params, void* ws, size_t ws_bytes,
                              void* stream);
/* The same with the last producer of da folded in (its gradient is never stored):
 * da_eff = da (nullable: no base gradient) + the gradient the route recomputes per pixel,
 * summed in the order that producer's own entry sums it, so the result is bit-identical
 * to the producer writing da followed by ugpg_bn_relu_bwd_partials:
 *   UGPG_ROUTE_MAXPOOL2: MaxPool2d(2)'s backward routes src (NHWC [B][H/2][W/2][C]) to each
 *     window's argmax pixel (B*H*W == npix); part from ugpg_maxpool2_bwd_partials.
 *     Replaces max_pool2d_with_indices_backward behind Down (UG_unet_parts.py:44-55).
 *   UGPG_ROUTE_HEAD: the 1x1 head's input gradient sum_k src[p][k] * w[k][c] (src = dh,
 *     [npix][nc]; w [nc][C]); part from ugpg_head_bwd_bnb with accumulate_da bit 2
 *     (UGPG_HEAD_DA_DEFERRED).  Replaces OutConv's input gradient (UG_unet_parts.py:84-90). */
#define UGPG_ROUTE_MAXPOOL2 1
#define UGPG_ROUTE_HEAD 2
typedef struct {
    int kind;               /* UGPG_ROUTE_* */
    const float* src;       /* the pooled output's gradient, or the head's dh (fp32) */
    const uint8_t* argmax;  /* MAXPOOL2: ugpg_maxpool2_fwd's window argmax, src's shape */
    const float* w;         /* HEAD: the head weight [nc][C] */
    int nc;                 /* HEAD: classes (1..4) */
    int B, H, W;            /* MAXPOOL2: the pooled input's (= the BatchNorm's) shape */
} ugpg_bwd_route_t;
int ugpg_bn_relu_bwd_partials_routed(const ugpg_bwd_route_t* route, const float* part,
                                     int nslots, const float* da, const float* y,
                                     const void* y_bf16, int64_t npix, int C, const float* mean,
                                     const float* invstd, const float* scale, const float* shift,
                                     float* dy, void* dy_bf16, float* dgamma, float* dbeta,
                                     float* dconv_bias, int accumulate_params, void* ws,
                                     size_t ws_bytes, void* stream);
int ugpg_bn_relu_bwd(const float* da, const float* y, const void* y_bf16, int64_t npix, int C,
                     const float* mean, const float* invstd, const float* scale,
                     const float* shift, float* dy, void* dy_bf16, float* dgamma, float* dbeta,
                     float* dconv_bias, int accumulate_params, void* ws, size_t ws_bytes,
                     void* stream);
/* Materialise relu(scale*y+shift) (used only for the standalone block API). */
int ugpg_bn_relu_apply(ugpg_src_t src, int64_t npix, float* out, void* stream);

/* ---- MaxPool2d(2) (UG_unet_parts.py:49, K8) on an activated source -------- */
/* out: fp32, or out == NULL and out_bf16 receives it rounded to bf16 (nearest even): the
 * next conv's bf16 operand exactly (the bf16 arithmetic's storage) */
int ugpg_maxpool2_fwd(ugpg_src_t src, int B, int H, int W, float* out, void* out_bf16,
                      uint8_t* argmax, void* stream);
int ugpg_maxpool2_bwd(const float* dout, const uint8_t* argmax, int B, int H, int W, int C,
                      float* din, int accumulate, void* stream);
/* The same, also writing the BatchNorm-backward partials of din (see ugpg_bnb_t). */
int ugpg_maxpool2_bwd_bnb(const float* dout, const uint8_t* argmax, int B, int H, int W, int C,
                          float* din, int accumulate, const ugpg_bnb_t* bnb, void* stream);
/* Only the BatchNorm-backward partials of din_base (nullable: zero) + the routed gradient;
 * nothing is written but bnb->part.  The apply recomputes the routing
 * (ugpg_bn_relu_bwd_partials_routed), so the pool's full-resolution gradient never goes
 * to HBM. */
int ugpg_maxpool2_bwd_partials(const float* dout, const uint8_t* argmax, int B, int H, int W,
                               int C, const float* din_base, const ugpg_bnb_t* bnb, void* stream);

/* ---- align_corners=True bilinear resize, NHWC (UG_unet_parts.py:78, K9) ---- */
/* out == NULL: the result is stored in bf16 at out_bf16 (the bf16 arithmetic's storage of
 * an Up conv's upsampled input -- which that conv and its weight gradient round to bf16
 * anyway); else out_bf16 is ignored */
int ugpg_bilinear_nhwc_fwd(ugpg_src_t src, int B, int Hi, int Wi, float* out, int Ho, int Wo,
                           void* out_bf16, void* stream);
int ugpg_bilinear_nhwc_bwd(const float* dout, int B, int Ho, int Wo, int C, float* din, int Hi,
                           int Wi, int accumulate, void* stream);
/* The same, also writing the BatchNorm-backward partials of din (see ugpg_bnb_t), one
 * slot per input row: nslots = B * Hi (C/4 must divide 256). */
int ugpg_bilinear_nhwc_bwd_bnb(const float* dout, int B, int Ho, int Wo, int C, float* din,
                               int Hi, int Wi, int accumulate, const ugpg_bnb_t* bnb,
                               void* stream);

/* fp32 <-> bf16 (round to nearest even) casts of n elements: the bf16 gradient exchange
 * of BASELINE configs[2] (gradient buckets all-reduced in bf16). */
int ugpg_cast_f32_bf16(const float* in, uint16_t* out, int64_t n, void* stream);
int ugpg_cast_bf16_f32(const uint16_t* in, float* out, int64_t n, void* stream);

/* ---- NCHW resize (F.interpolate at uncertainty_guided_trainer.py:208-209,
 * UG_unet.py:36-53, 419-424; K12/K13)
 *  mode 0: bilinear align_corners;  mode 1: nearest;
 *  mode 2: U = 1 - 2|bilinear(sigmoid(in)) - 0.5|  (uncertainty map, UG_unet.py:45-57) */
int ugpg_resize_nchw(const float* in, int B, int C, int Hi, int Wi, float* out, int Ho, int Wo,
                     int mode, void* stream);
/* gradient of ugpg_resize_nchw mode 0 w.r.t. its input (autograd of F.interpolate(bilinear,
 * align_corners=True), ProgressiveUNet.forward UG_unet.py:418-424): din (B,C,Hi,Wi) from
 * dout (B,C,Ho,Wo), gather form, deterministic */
int ugpg_resize_nchw_bwd(const float* dout, int B, int C, int Ho, int Wo, float* din, int Hi,
                         int Wi, void* stream);
/* NCHW <-> NHWC (with zero channel padding to Cpad) */
int ugpg_nchw_to_nhwc(const float* in, int B, int C, int H, int W, float* out, int Cpad,
                      void* stream);
int ugpg_nhwc_to_nchw(const float* in, int B, int C, int H, int W, int Cstride, float* out,
                      int accumulate, void* stream);

/* ---- deep-supervision heads: 1x1 OutConv + align_corners upsample + sum
 * (UG_unet_parts.py:84-91, UG_unet.py:294-303; K11) */
int ugpg_head_fwd(ugpg_src_t src, int64_t npix, const float* w, const float* b, int nc,
                  float* h, void* stream);
/* logits[b][k][y][x] (NCHW, HxW) = sum_i up_i(h_i) in order i = 0..n-1; h_i NHWC at
 * (hres[i] x hres[i]) with nc channels; resolution HxW == finest. */
int ugpg_heads_combine(const float* const* h, const int* hres, int n, int B, int H, int W,
                       int nc, float* logits, void* stream);
/* dh_i = upsample_i^T(dlogits) for every head (NHWC nc channels; n <= 4, one launch). */
int ugpg_heads_split_bwd(const float* dlogits, int B, int H, int W, int nc, float* const* dh,
                         const int* hres, int n, void* stream);
size_t ugpg_head_bwd_workspace(int64_t npix, int C, int nc);
int ugpg_head_bwd(ugpg_src_t src, int64_t npix, const float* w, int nc, const float* dh,
                  float* dw, float* db, float* da, int accumulate_da, void* ws, size_t ws_bytes,
                  void* stream);
/* The same, also writing the BatchNorm-backward partials of da (ugpg_bnb_t; bnb->y must
 * be src.data, the BN input the head reads lazily): nslots = ugpg_head_bwd_bnb_slots.
 * accumulate_da | UGPG_HEAD_DA_DEFERRED: da is not written (read as the base gradient when
 * accumulate_da & 1; may be NULL otherwise) -- the partials are those of base + dh @ w,
 * which ugpg_bn_relu_bwd_partials_routed(UGPG_ROUTE_HEAD) recomputes. */
#define UGPG_HEAD_DA_DEFERRED 2
int ugpg_head_bwd_bnb_slots(int64_t npix);
int ugpg_head_bwd_bnb(ugpg_src_t src, int64_t npix, const float* w, int nc, const float* dh,
                      float* dw, float* db, float* da, int accumulate_da, void* ws,
                      size_t ws_bytes, const ugpg_bnb_t* bnb, void* stream);

/* ---- uncertainty-weighted BCE-with-logits (UG_unet.py:61-94, K13) ---------
 * pixel = (1-t)x + (1+(pw-1)t)*softplus(-x);  final = mean(pixel*(1+alpha*U))
 * (U == NULL: final = mean(pixel));  out[0]=final, out[1]=mean(pixel).
 * U is NCHW with Cu channels (1 or C; broadcast over C when Cu == 1). */
size_t ugpg_ug_loss_workspace(int64_t n);
int ugpg_ug_loss_fwd(const float* logits, const float* target, const float* umap, int B, int C,
                     int HW, int Cu, const float* pos_weight, float alpha, float* out,
                     void* ws, size_t ws_bytes, void* stream);
/* dlogits = gout[0] * (1+alpha*U) * ((1-t) - (1+(pw-1)t)*sigmoid(-x)) / N */
int ugpg_ug_loss_bwd(const float* logits, const float* target, const float* umap, int B, int C,
                     int HW, int Cu, const float* pos_weight, float alpha, const float* gout,
                     float* dlogits, void* stream);
/* weighted mean of an arbitrary per-pixel loss (non-BCE criteria) */
int ugpg_weighted_mean_fwd(const float* pixel_loss, const float* umap, int B, int C, int HW,
                           int Cu, float alpha, float* out, void* ws, size_t ws_bytes,
                           void* stream);
int ugpg_weighted_mean_bwd(const float* umap, int B, int C, int HW, int Cu, float alpha,
                           const float* gout, float* dpixel, void* stream);

/* ---- trainer metrics (uncertainty_guided_trainer.py:90-123, K14) ----------
 * pred = sigmoid(x) > 0.5 ; per-sample Dice (2I+1)/(P+T+1) averaged over B;
 * accuracy = 1 - #(pred != trunc(t)) / (B*HW).  out = [dice, acc, wrong_count]. */
size_t ugpg_seg_metrics_workspace(int B);
int ugpg_seg_metrics(const float* logits, const float* target, int B, int HW, float* out,
                     void* ws, size_t ws_bytes, void* stream);
/* ---- inference / evaluation (MoNuSegImprove/test_monuseg.py:164-297) ----------
 * Replaces MoNuSegTester.calculate_metrics (:264-297, numpy on float32 arrays) and the
 * sigmoid / threshold / mean of predict_image (:188-199) for a batch of logits
 * (B,1,H,W) against ground-truth masks (B,1,H,W): pred = sigmoid(x) > 0.5;
 * out[8*b + 0..7] = iou, dice, accuracy, precision, recall, specificity (float32,
 * eps 1e-8, the reference's operation order), confidence = mean sigmoid, tp count. */
size_t ugpg_seg_eval_workspace(int B, int HW);
int ugpg_seg_eval(const float* logits, const float* gt, int B, int HW, float* out, void* ws,
                  size_t ws_bytes, void* stream);
/* mask (B,1,Ho,Wo) = F.interpolate((sigmoid(x) > 0.5).float(), (Ho,Wo), mode='nearest')
 * (test_monuseg.py:190-195) */
int ugpg_predict_mask(const float* logits, int B, int H, int W, float* mask, int Ho, int Wo,
                      void* stream);
/* mean and unbiased std of n floats: out = [mean, std] (torch.mean/torch.std) */
size_t ugpg_mean_std_workspace(int64_t n);
int ugpg_mean_std(const float* x, int64_t n, float* out, void* ws, size_t ws_bytes,
                  void* stream);

/* ---- RCCL communicator (the reference has no collectives -- this is the
 * data-parallel exchange the build adds: gradient all-reduce, replica broadcast).
 * Rendezvous: rank 0 calls ugpg_comm_unique_id and passes the ugpg_comm_id_bytes() bytes
 * to every rank out of band; each rank calls ugpg_comm_init with its own device.  The
 * collectives are stream-ordered on `stream` (hipStream_t), in place when send == recv,
 * never synchronise the host and allocate nothing.  The handle is the only global state
 * of the library; destroy it on every rank. */
typedef struct ugpg_comm* ugpg_comm_t;
#define UGPG_DT_F32 0
#define UGPG_DT_BF16 1
#define UGPG_DT_F64 2
#define UGPG_DT_I64 3
#define UGPG_OP_SUM 0
#define UGPG_OP_AVG 1
#define UGPG_OP_MAX 2
size_t ugpg_comm_id_bytes(void);
int ugpg_comm_unique_id(unsigned char* out, size_t n);
int ugpg_comm_init(ugpg_comm_t* comm, int nranks, int rank, const unsigned char* id,
                   size_t id_bytes, int device);
int ugpg_comm_allreduce(ugpg_comm_t comm, const void* send, void* recv, size_t count, int dtype,
                        int op, void* stream);
int ugpg_comm_broadcast(ugpg_comm_t comm, const void* send, void* recv, size_t count, int dtype,
                        int root, void* stream);
int ugpg_comm_destroy(ugpg_comm_t comm);

/* ---- data-parallel metrics exchange (metrics all-reduced under DP; the
 * reference is single-process, its per-batch metrics are uncertainty_guided_trainer.py:
 * 171-182, 221-234 and Herlev/train_herlev.py:288-294, 328-337).
 * m[0..n) (n <= 32): entries with bit i of avg_mask are per-rank means (averaged over
 * ranks), other entries are sums; [ip, ip+1) is a (mean, unbiased std) pair over n_stat
 * values per rank (ip = -1: none).  pack writes double sums[n+2] for a SUM all-reduce;
 * unpack turns the reduced sums back into global metrics (Chan-style pooled std). */
int ugpg_metrics_pack(const float* m, int n, int ip, double n_stat, double* sums, void* stream);
int ugpg_metrics_unpack(const double* sums, int n, int ip, unsigned avg_mask, float* m,
                        void* stream);

/* ---- RMSprop (torch.optim.RMSprop rule, uncertainty_guided_trainer.py:84-88, K15)
 * g = grad*grad_scale + wd*p;  v = alpha*v + (1-alpha)*g^2;  p -= lr*g/(sqrt(v)+eps) */
int ugpg_rmsprop_step(float* param, const float* grad, float* square_avg, int64_t n, float lr,
                      float alpha, float eps, float weight_decay, float grad_scale,
                      void* stream);

/* ---- Herlev classifier head (Herlev/train_herlev.py:66-77, K16) ----------- */
/* global average pool of an activated NHWC source -> [B][C] */
int ugpg_avgpool_fwd(ugpg_src_t src, int B, int HW, float* out, void* stream);
int ugpg_avgpool_bwd(const float* dout, int B, int HW, int C, float* da, int accumulate,
                     void* stream);
/* y[m][n] = act(sum_k x[m][k]*w[n][k] + b[n]) (act: 0 none, 1 relu); x row-major [M][K] */
int ugpg_linear_fwd(const float* x, const float* w, const float* b, int M, int N, int K,
                    int relu, float* y, void* stream);
/* given dy (already masked by relu if any): dx = dy*w, dw = dy^T x, db = sum dy */
int ugpg_linear_bwd(const float* x, const float* w, const float* dy, int M, int N, int K,
                    float* dx, float* dw, float* db, void* stream);
/* nn.Dropout mask: mask[i] = (u_i >= p) / (1-p), u_i = counter hash of (seed, i) */
int ugpg_dropout_mask(float* mask, int64_t n, float p, uint64_t seed, void* stream);
/* Herlev uncertainty-guided CE (train_herlev.py:253-296), K > 2 classes:
 *   base = CE(x, y; class_weights) (weighted mean), u_b = H(softmax(prev_b))/log K,
 *   final = mean_b(CE_b * (1 + alpha*u_b))  (prev == NULL: final = base)
 * out = [final, base, mean(1+alpha*u), std(1+alpha*u), #(argmax == y)];
 * weights[b] = 1+alpha*u_b. */
int ugpg_ce_ug_fwd(const float* x, const int64_t* y, const float* prev,
                   const float* class_weights, int B, int K, float alpha, float* out,
                   float* weights, void* stream);
/* d final / d x (weights == NULL: gradient of the class-weighted base CE) */
int ugpg_ce_ug_bwd(const float* x, const int64_t* y, const float* weights,
                   const float* class_weights, int B, int K, const float* gout, float* dx,
                   void* stream);
/* torch.optim.Adam rule (no amsgrad): g += wd*p; m = lerp(m, g, 1-b1);
 * v = b2*v + (1-b2)*g^2; p -= lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps) */
int ugpg_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                   int64_t n, float lr, float beta1, float beta2, float eps, float weight_decay,
                   int64_t step, float grad_scale, void* stream);
/* relu backward: dx = dy * (y > 0)  (dx may alias dy) */
int ugpg_relu_bwd(const float* y, const float* dy, float* dx, int64_t n, void* stream);
/* elementwise y = x * mask (dropout with a precomputed scaled mask) */
int ugpg_mul(const float* x, const float* m, float* y, int64_t n, void* stream);

/* ---- MoNuSeg augmentation (aug_monuseg_dataset.py:113-148,
 * monuseg_dataset.py:137-190): PIL's 8-bit arithmetic reproduced on the GPU. -------- */
/* One separable pass of PIL's antialiasing resampler (Image.resize BILINEAR): `outer`
 * rows, resampled axis n_in -> n_out, `inner_after` contiguous bytes per axis position
 * (C for the horizontal pass over HWC rows, OW*C for the vertical pass);
 * bounds[2*o] = first tap, bounds[2*o+1] = tap count, kk[o*ksize + t] = PIL's 22-bit
 * fixed-point coefficients (host-computed, ugpg/augment.py:resample_coeffs). */
int ugpg_resample_aa_u8(const uint8_t* in, int64_t outer, int n_in, int n_out,
                        int inner_after, const int* bounds, const int* kk, int ksize,
                        uint8_t* out, void* stream);
/* nearest resize (Image.resize NEAREST) of B HWC images with host-tabulated source
 * rows / columns (PIL's accumulated coordinates) */
int ugpg_resize_nearest_u8(const uint8_t* in, int64_t B, int H, int W, int C, const int* ytab,
                           const int* xtab, uint8_t* out, int OH, int OW, void* stream);
/* sizes of the per-sample parameter records (host layout check) */
int ugpg_augment_param_sizes(int* geom_bytes, int* color_bytes);
/* hflip, vflip, Image.rotate (image BILINEAR: double-precision affine map, truncating
 * bilinear filter; mask NEAREST: 16.16 fixed point), adjust_brightness; B samples of
 * S x S (RGB HWC uint8 + mask uint8); lsum[B] receives each result's L sum */
int ugpg_augment_geom(const uint8_t* img, const uint8_t* mask, int S, int64_t B,
                      const void* params, uint8_t* out_img, uint8_t* out_mask, unsigned* lsum,
                      void* stream);
/* adjust_contrast (grey level int(mean L + .5)), adjust_saturation, adjust_hue (PIL HSV
 * round trip, uint8 hue shift), ToTensor (u8_to_f32[256] = torch's v/255) -> out
 * (B,3,S,S) float; mask -> out_mask (B,1,S,S) float */
int ugpg_augment_color(const uint8_t* img, const uint8_t* mask, int S, int64_t B,
                       const void* params, const unsigned* lsum, const float* u8_to_f32,
                       float* out, float* out_mask, void* stream);
/* XML annotation polygons -> mask: replaces the reference's per-region
 * `ImageDraw.Draw(mask).polygon(points, fill=1)` loop (MoNuSegImprove/
 * monuseg_dataset.py:117-132, aug_monuseg_dataset.py:89-111) with Pillow 12's scan
 * converter reproduced bit for bit (oracle/polygon_ref.py lists its rules).  npoly
 * polygons; polygon p = vertices [off[p], off[p+1]) of xy (x, y pairs of doubles: the
 * XML's float values; >= 2 vertices each, as PIL requires); each is filled with `ink`
 * into mask (H x W uint8, row-major), which is not cleared first (the reference draws
 * every region into one mask).  ws: device workspace of at least
 * ugpg_rasterize_polygons_ws_size(nverts, npoly) bytes (nverts = off[npoly]), else
 * UGPG_ERR_WORKSPACE. */
size_t ugpg_rasterize_polygons_ws_size(int64_t nverts, int64_t npoly);
int ugpg_rasterize_polygons(const double* xy, const int64_t* off, int64_t npoly, int64_t nverts,
                            uint8_t* mask, int H, int W, int ink, void* ws, size_t ws_bytes,
                            void* stream);

#ifdef __cplusplus
}
#endif
#endif /* UGPG_H_ */
