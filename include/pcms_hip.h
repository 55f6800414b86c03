/*
 * pcms_hip.h — C ABI of libpcms_hip.so, the MI355X (gfx950) kernels behind the drop-in
 * UNet3D / DiceLoss / BCEDiceLoss / Trainer.step of
 * qwertyhgb/Prostate-Cancer-Multimodal-Segmentation.
 *
 * The reference has no FFI: its hot path is PyTorch aten called from Python.  Each entry
 * point below replaces the aten op(s) named in its comment (paths relative to the
 * reference repo root).  The Python host layer (pcms_amd) binds these through ctypes.
 *
 * Conventions
 *   - dtype: 0 = fp32 storage (parity build), 1 = bf16 storage (performance build).
 *     Accumulation is always fp32; statistics are combined in fp64.
 *   - Activations are NDHWC, contiguous, channel pitch = channel count.
 *   - Pointers are device pointers; the caller owns every buffer (no allocation inside,
 *     except workspace passed in).  `s` is a hipStream_t; every call is stream-ordered and
 *     returns 0 on success, a hipError_t code, or a negative code for a bad argument.
 */
#ifndef PCMS_HIP_H
#define PCMS_HIP_H
#include <hip/hip_runtime.h>

#ifdef __cplusplus
extern "C" {
#endif

/* conv epilogue flags (pcms_conv3_fwd, pcms_split_epilogue, pcms_stem_fwd): ACCUMULATE
 * adds into y; RELU stores relu(conv + bias) -- eval mode with the BatchNorm folded into the
 * weights and bias (pcms_bn_fold), no statistics                                          */
#define PCMS_CONV_ACCUMULATE 1
#define PCMS_CONV_RELU 2
/* gradient writer flags (pcms_conv3_wgrad): STORE writes dw instead of adding into it -- the
 * first writer after zero_grad(set_to_none=True), so the gradient needs no zero fill       */
#define PCMS_GRAD_STORE 1
/* pcms_stem_fwd flag: the K-dense kernel (9 tap rows x 16 instead of 14 tap pairs x 16; the
 * pack's second form, valid for weights with cin_w <= 5)                                   */
#define PCMS_STEM_DENSE 16

/* ---- layout ---------------------------------------------------------------------- */
/* batch['image'] (N, Cin, D, H, W) fp32 NCDHW -> NDHWC, channels zero-padded to Cp.
 * Replaces the implicit layout of images.to(device) (utils/trainer.py:179).          */
int pcms_pack_input(int dtype, const float* in, void* out, int N, int Cin, long V, int Cp, hipStream_t s);

/* ---- Conv3d(k=3, padding=1): models/unet3d.py:29,35 ------------------------------- */
/* The conv3 entry points also take dtype 2 (PCMS_F32X3): fp32 data, bf16x3 arithmetic
 * (hi*hi + lo*hi + hi*lo, ~10x fp32 rounding error); dtype 0 there computes with bf16x6
 * (three bf16 parts per operand, fp32-grade: the parity build).                        */
int pcms_conv3_chunk(int dtype);                  /* input channels per K-chunk        */
/* elements (activation dtype) of one weight pack, J rows x Kdim input channels          */
int pcms_conv3_pack_elems(int dtype, int J, int Kdim);
int pcms_conv3_mblocks(int N, int D, int H, int W);/* general-kernel M blocks (an upper
                                                      bound on the BN partial rows)      */
/* BN partial rows an unsplit pcms_conv3_fwd over sources (c0, c1) writes: the persistent
 * big-box bf16 kernel (8x8x16 boxes, 16-channel chunks, >= pcms_conv3_big_min_boxes boxes)
 * writes one row per box slot (min(boxes, workgroups / (Cout / 64))), the general kernel
 * pcms_conv3_mblocks rows                                                               */
int pcms_conv3_fwd_rows(int dtype, int N, int D, int H, int W, int c0, int c1, int Cout);
int pcms_conv3_big_min_boxes(int v);               /* set (v > 0) / query; returns old */
int pcms_conv3_big_max_wgs(int v);                 /* persistent grid cap: set (v >= 0,
                                                      0 = one per CU) / query; old      */
/* general-kernel boxes of <= 256 voxels (level 4) on four waves of 2 M-tiles (1, default)
 * or two waves of 4 (0); v < 0 queries; returns the previous setting                   */
int pcms_conv3_small_box_mtw2(int v);
/* A/B switch: general forward / dgrad box volume, 512 or 256 voxels (v <= 0 queries) */
int pcms_conv3_fwd_box_vol(int v);
/* master W [Cout][Cin][3][3][3] fp32 -> kernel pack; flip=1 builds the dgrad pack      */
int pcms_conv3_pack(int dtype, const float* w, void* out, int Cout, int Cin, int flip, hipStream_t s);
// Both packs of one conv (forward and dgrad, as pcms_conv3_pack flip 0 / 1) from one read of w.
int pcms_conv3_pack2(int dtype, const float* w, void* fwd, void* dgrad, int Cout, int Cin, hipStream_t s);
/* Y = conv(X) + bias, X = channel-concat(x0[:, :c0], x1[:, :c1]) (Up3D cat, :156),
 * output channels [0, cy0) -> y0, [cy0, Cout) -> y1 (dgrad concat split).
 * stats: BN partials or NULL: [mblocks][Cout][2] fp32 (sum, M2 = sum of squared
 * deviations from the row's own mean) followed by [mblocks] fp32 row voxel counts
 * (numerically stable moments; consumed by pcms_bn_finalize).  splits > 1 (split-K over
 * input channels): every split stores its fp32 partial sums into its own slab of
 * yacc [pcms_conv3_splits(...)][Nvox][Cout] (plain stores, no zeroing, no atomics);
 * finish with pcms_split_epilogue, which adds the slabs in split order (deterministic).
 * Also used for dgrad with the flip pack.                                              */
int pcms_conv3_splits(int dtype, int Cin, int splits);  /* slabs a split-K launch uses   */
int pcms_conv3_fwd(int dtype, const void* x0, int c0, const void* x1, int c1,
                   const void* wpack, const float* bias, void* y0, void* y1, int cy0,
                   float* yacc, float* stats, int flags,
                   int N, int D, int H, int W, int Cout, int splits, hipStream_t s);
/* The conv of relu(x * isc + ish) (per input channel): the BatchNorm + ReLU of the layer
 * below (models/unet3d.py:31-35, bn -> relu -> conv) applied to the staged halo in LDS
 * instead of a separate HBM pass.  bf16, one source of <= 128 channels, the big-box shapes
 * (-5 otherwise); no split, no flags.  Measured against pcms_bn_relu + pcms_conv3_fwd in
 * DESIGN.md §0b (tests/tools/bnin_ab.py).                                                 */
int pcms_conv3_fwd_bnin(int dtype, const void* x, int cin, const float* isc, const float* ish, const void* wpack,
                        const float* bias, void* y, float* stats, int N, int D, int H, int W, int Cout,
                        hipStream_t s);
/* The weight gradient of that conv: x is the pre-BatchNorm input, relu(x * isc + ish) is
 * applied to the staged halo in LDS (bf16, one source, the LDS-DMA shapes; -5 otherwise).
 * pcms_conv3_bnin_ok: 1 when both pcms_conv3_fwd_bnin and this run the layer.              */
int pcms_conv3_wgrad_bnin(int dtype, const void* x, int cin, const float* isc, const float* ish, const void* dy,
                          float* dw, float* dwt, int N, int D, int H, int W, int Cout, int cin_w, int target_wgs,
                          int flags, hipStream_t s);
int pcms_conv3_bnin_ok(int N, int D, int H, int W, int cin, int Cout, int target_wgs);
/* dw [Cout][cin_w][27] fp32 += sum_v dy[v, co] * x[v + tap, ci] (ci < cin_w <= c0 + c1;
 * flags PCMS_GRAD_STORE: dw = ...);
 * dwt: pcms_conv3_wgrad_ws_floats(...) fp32 workspace (one partial row per voxel split,
 * summed in a fixed order: deterministic)                                               */
int pcms_conv3_wgrad_ws_floats(int dtype, int N, int D, int H, int W, int c0, int c1, int Cout, int target_wgs);
/* bf16 grids of at most v boxes split the taps over two workgroups (no partial rows) before
 * splitting the voxels; 0 never, v < 0 queries; returns the previous value              */
int pcms_conv3_wgrad_tg_maxbox(int v);
/* compile-time-box bf16 weight gradients (the LDS-DMA kernels of levels 0-4) on
 * v_mfma_f32_16x16x32_bf16 (1) or v_mfma_f32_32x32x16_bf16 (0, default); v < 0 queries;
 * returns the previous setting (A/B switch) */
int pcms_conv3_wgrad_k16(int v);
/* fp32 (bf16x6) weight gradient: boxes streamed by LDS-DMA into an fp32 staging buffer beside
 * the previous box's MFMAs (1) or staged synchronously through registers (0, default: measured
 * as fast); v < 0 queries; returns the previous setting (A/B switch) */
int pcms_conv3_wgrad_x6_dma(int v);
/* the weight gradient's per-split partial rows summed in one launch (1, default) or by the
 * group-sum + reduce pair (0); the sums are bit-identical; v < 0 queries; returns the previous
 * setting (A/B switch) */
int pcms_conv3_wgrad_reduce_fused(int v);
int pcms_conv3_wgrad(int dtype, const void* x0, int c0, const void* x1, int c1, const void* dy,
                     float* dw, float* dwt, int N, int D, int H, int W, int Cout, int cin_w,
                     int target_wgs, int flags, hipStream_t s);
/* The big-box convs on v_mfma_f32_16x16x32_bf16 (round 5): K = a pair of taps x 16 channels,
 * 8 M-tiles x 4 N-tiles per wave, one wave per box d-plane; boxes of 8 d-planes (levels 0-1,
 * the shapes of the 32x32x16 big-box path of pcms_conv3_fwd) or, where those leave CUs idle
 * and 4-deep boxes x 64-channel blocks fill them (level 2), of 4.  BN partial rows:
 * pcms_conv3_fwd16_rows (0: not a fwd16 shape).  Weights in the
 * pack16 layout: pcms_conv3_pack16 writes both directions of the convs of a table (int64 rows
 * {fp32 weight ptr, Cout, Cin, fwd16 ptr or 0, dgrad16 ptr or 0, first tile, 0, 0}, one tile
 * per 32 x 32 channels; fwd16 = rows Cout, k Cin; dgrad16 = rows Cin, k Cout, taps mirrored).
 * pcms_conv3_fwd16 takes isc / ish (the input's BatchNorm + ReLU, as pcms_conv3_fwd_bnin) or
 * NULL; flags 0 or PCMS_CONV_RELU; -5 where pcms_conv3_big16_ok is 0.                      */
int pcms_conv3_big16_ok(int N, int D, int H, int W, int c0, int c1, int Cout);
int pcms_conv3_fwd16_rows(int N, int D, int H, int W, int c0, int c1, int Cout);
/* 128-channel blocks (4-deep boxes, 8 N-tiles per wave: one staged halo feeds 128 output
 * channels) where Cout % 128 == 0 and they fill the CUs: 1 or 0 (default); v < 0 queries;
 * returns the previous setting (set before any workspace query)                          */
int pcms_conv3_b16_nt8(int v);
/* Level 3 (rows of 8 w): the same kernel on 4 d x 16 h x 8 w boxes, split over K into fp32
 * partial rows yacc[split][vox][Cout] (no bias / statistics; pcms_split_epilogue sums them in
 * split order).  _split_ok: the split count it uses for this conv, 0 where it does not apply. */
int pcms_conv3_fwd16_split_ok(int N, int D, int H, int W, int c0, int c1, int Cout);
int pcms_conv3_fwd16_split(const void* x0, int c0, const void* x1, int c1, const void* wpack16, float* yacc,
                           int N, int D, int H, int W, int Cout, int splits, hipStream_t s);
int pcms_conv3_pack16_elems(int J, int Kdim);
int pcms_conv3_pack16(const long long* table, int ntab, int ntiles, hipStream_t s);
int pcms_conv3_fwd16(const void* x0, int c0, const void* x1, int c1, const float* isc, const float* ish,
                     const void* wpack16, const float* bias, void* y0, void* y1, int cy0, float* stats, int flags,
                     int N, int D, int H, int W, int Cout, hipStream_t s);
/* Stem (inc.conv.0, bf16 build): input stored with 8 channels (n_modalities <= 8).
 * K packs two taps per MFMA k-step (14 x 16 = 224 instead of 27 x 32), or, with
 * PCMS_STEM_DENSE (cin_w <= 5), one (kd, kh) tap row of 3 kw x 5 channels per k-step (9 x 16);
 * pcms_stem_pack writes both forms.
 * pcms_stem_supported: bit 0 = pcms_stem_fwd runs this shape, bit 1 = pcms_stem_wgrad
 * does (other shapes: the general pcms_conv3_fwd / pcms_conv3_wgrad).                   */
int pcms_stem_supported(int N, int D, int H, int W);
int pcms_stem_pack_elems(void);
/* the stem weight gradient's MFMA columns: 0 (default) taps x 8 channels, 1 dense tap rows
 * x 16 for cin_w <= 5; v < 0 queries; returns the previous setting                        */
int pcms_stem_wgrad_dense(int v);
int pcms_stem_pack(const float* w, void* out, int cin_w, hipStream_t s);
/* y = stem conv(x) + bias; BatchNorm partial moments into stats, laid out as pcms_conv3_fwd
 * with rows = pcms_stem_fwd_rows(N, D, H, W) (one row per workgroup on the hot shapes)   */
int pcms_stem_fwd_rows(int N, int D, int H, int W);
int pcms_stem_fwd(const void* x, const void* wpack, const float* bias, void* y, float* stats,
                  int N, int D, int H, int W, int flags, hipStream_t s);
/* dw [64][cin_w][27] += stem weight gradient (streaming kernel: one partial row per
 * workgroup in ws, then a fixed-order sum), ws = pcms_stem_wgrad_ws_floats(...) floats.   */
int pcms_stem_wgrad_ws_floats(int N, int D, int H, int W, int cin_w);
int pcms_stem_wgrad(const void* x, const void* dy, float* dw, float* ws, int cin_w, int N, int D, int H,
                    int W, hipStream_t s);
/* Block fusion of the stem's BatchNorm + ReLU backward (models/unet3d.py:29-33) into its
 * weight gradient: da = gradient of the block's first ReLU output, y = the stem's pre-BN
 * output, scale / shift / mean / invstd = the forward's BN coefficients, coef = the apply
 * coefficients pcms_bn_relu_bwd(..., dy = NULL, ...) left; the stem's dy is formed in LDS
 * per box and never stored (the stem input needs no gradient).                          */
int pcms_stem_wgrad_bn(const void* x, const void* da, const void* y, const float* scale, const float* shift,
                       const float* mean, const float* invstd, const float* coef, float* dw, float* ws, int cin_w,
                       int N, int D, int H, int W, hipStream_t s);
/* y = sum of the `splits` slabs of acc (in split order) + bias -> storage type; stats
 * layout as pcms_conv3_fwd with rows = pcms_split_epilogue_rows(nvox)                    */
int pcms_split_epilogue_rows(long nvox);
int pcms_split_epilogue(int dtype, const float* acc, int splits, const float* bias, void* y0, void* y1,
                        int cy0, float* stats, int C, long nvox, int flags, hipStream_t s);

/* ---- BatchNorm3d (train / eval) + ReLU(inplace): models/unet3d.py:31-39 ----------- */
/* part: the [rows][C][2] (sum, M2) partials + [rows] counts written by the conv / stem /
 * split-epilogue kernels; ws: pcms_bn_ws_doubles(C) fp64 workspace (two-stage fp64
 * column reduction, rows merged with Chan's parallel-variance formula)                  */
int pcms_bn_ws_doubles(int C);
int pcms_bn_finalize(const float* part, int rows, int C, double count, const float* gamma,
                     const float* beta, float* rmean, float* rvar, long long* nbt, float momentum,
                     float eps, float* scale, float* shift, float* mean, float* invstd, double* ws,
                     hipStream_t s);
/* Eval-mode BatchNorm folded into the conv before it (UNet3D.predict / .inference,
 * models/unet3d.py:298-344): wo = w * sc[co], bo = b * sc + sh (sc = gamma / sqrt(rvar +
 * eps), sh = beta - rmean * sc, in fp64); w [Cout][K] fp32 (K = Cin * 27), b may be NULL.
 * The folded conv with PCMS_CONV_RELU is conv -> BN -> ReLU in one pass.                  */
int pcms_bn_fold(const float* w, const float* b, const float* gamma, const float* beta, const float* rmean,
                 const float* rvar, float eps, int Cout, long K, float* wo, float* bo, hipStream_t s);
int pcms_bn_eval_coeffs(const float* gamma, const float* beta, const float* rmean, const float* rvar,
                        float eps, int C, float* scale, float* shift, hipStream_t s);
int pcms_bn_relu(int dtype, const void* y, void* a, const float* scale, const float* shift, int C,
                 long nvox, hipStream_t s);
/* A/B switch: block cap of the BN-backward reduce passes (their partial rows): 512 (default,
 * the one-launch finalize) or more (2048: the two-stage finalize); v <= 0 queries; returns the
 * previous value; set before the workspace queries */
int pcms_bn_bwd_rows_cap(int v);
int pcms_bn_bwd_rows(int dtype, int C, long nvox);
/* dy = BN+ReLU backward(da); dgamma/dbeta += ; part: rows*C*2 fp32; coef: 3*C fp32 (the
 * apply coefficients k1, k2, k3 per channel: dy = k1 g + k2 xhat + k3).  dy == NULL: no
 * apply pass (a fused consumer applies from coef: pcms_stem_wgrad_bn)                    */
int pcms_bn_relu_bwd(int dtype, const void* da, const void* y, const float* scale, const float* shift,
                     const float* mean, const float* invstd, const float* gamma, float* part, float* coef,
                     float* dgamma, float* dbeta, void* dy, int C, long nvox, double* ws, hipStream_t s);
/* the same without the reduction pass: ``part`` holds ``rows`` partial rows [rows][C][2] of
 * (sum g, sum g xhat) written by a fused producer (pcms_maxpool_bwd_bn)                  */
int pcms_bn_relu_bwd_finish(int dtype, const void* da, const void* y, const float* scale, const float* shift,
                            const float* mean, const float* invstd, const float* gamma, const float* part,
                            int rows, float* coef, float* dgamma, float* dbeta, void* dy, int C, long nvox,
                            double* ws, hipStream_t s);

/* ---- MaxPool3d(2): models/unet3d.py:80 ------------------------------------------- */
int pcms_maxpool_fwd(int dtype, const void* a, void* p, int N, int D, int H, int W, int C, hipStream_t s);
/* da[argmax] += dp (first max in d,h,w scan order wins, as PyTorch)                  */
int pcms_maxpool_bwd(int dtype, const void* a, const void* dp, void* da, int N, int D, int H, int W,
                     int C, hipStream_t s);
/* Block fusion at the encoder's Down3D boundary (a DoubleConv's second BatchNorm3d + ReLU,
 * models/unet3d.py:37-39, and the next MaxPool3d, :80).  Forward: a = relu(y scale + shift)
 * is stored (the block output, also the skip input) and pooled into p in the same pass.
 * Backward: da (the block output's gradient, holding the skip part) += dp at the argmax of a,
 * which is recomputed from y; the pass also writes the BatchNorm-backward partial rows
 * [rows][C][2] for pcms_bn_relu_bwd_finish (rows = pcms_maxpool_bwd_bn_rows(...)).       */
int pcms_bn_relu_pool(int dtype, const void* y, void* a, void* p, const float* scale, const float* shift,
                      int N, int D, int H, int W, int C, hipStream_t s);
int pcms_maxpool_bwd_bn_rows(int dtype, int N, int D, int H, int W, int C);
int pcms_maxpool_bwd_bn(int dtype, const void* y, const float* scale, const float* shift, const float* mean,
                        const float* invstd, const void* dp, void* da, float* part, int N, int D, int H, int W,
                        int C, hipStream_t s);
/* The same pair with da never written: pcms_maxpool_bwd_bn_sums writes only the partial rows
 * (da, holding the skip part, is read); after pcms_bn_relu_bwd_finish(..., dy = NULL) has
 * formed coef, pcms_maxpool_bn_apply forms da = da_skip + dp at the argmax again per 2x2x2 cell
 * (rounded as pcms_maxpool_bwd_bn stores it) and writes dy = k1 g + k2 xhat + k3 -- the same
 * dy bits as pcms_maxpool_bwd_bn + pcms_bn_relu_bwd_finish(dy), one tensor write and read
 * fewer (engine.pool_bn_apply_fused; measured +0.19 % per step, so the engine keeps the pair
 * above by default).                                                                      */
int pcms_maxpool_bwd_bn_sums(int dtype, const void* y, const float* scale, const float* shift, const float* mean,
                             const float* invstd, const void* dp, const void* da, float* part, int N, int D, int H,
                             int W, int C, hipStream_t s);
int pcms_maxpool_bn_apply(int dtype, const void* y, const float* scale, const float* shift, const float* mean,
                          const float* invstd, const float* coef, const void* dp, const void* da, void* dy, int N,
                          int D, int H, int W, int C, hipStream_t s);

/* ---- ConvTranspose3d(k=2, s=2) + F.pad: models/unet3d.py:120,139-151 --------------- */
/* the persistent bf16 forward used at Cin 128 / Cout 64 (level-0 Up3D): on (1) / off (0),
 * v < 0 queries; returns the previous setting (A/B and tests)                          */
int pcms_convt_fwd_stream(int v);
/* elements (activation dtype) of one pack: bf16 8 Cin Cout; fp32 (bf16x6 fragments) 3x that */
int pcms_convt_pack_elems(int dtype, int Cin, int Cout);
int pcms_convt_pack(int dtype, const float* w, void* out, int Cin, int Cout, int dgrad, hipStream_t s);
int pcms_convt_fwd(int dtype, const void* x, const void* wpack, const float* bias, void* out,
                   int N, int Din, int Hin, int Win, int Cin, int Cout, int Do, int Ho, int Wo, hipStream_t s);
/* the same with a K-split workspace for small grids (bf16; fp32 partials summed in a fixed
   order with the bias): ws = pcms_convt_fwd_ws_floats(...) floats (0: no split, ws may be NULL) */
int pcms_convt_fwd_ws_floats(int N, int Din, int Hin, int Win, int Cin, int Cout);
int pcms_convt_fwd_ws(int dtype, const void* x, const void* wpack, const float* bias, void* out, float* ws,
                      int N, int Din, int Hin, int Win, int Cin, int Cout, int Do, int Ho, int Wo, hipStream_t s);
int pcms_convt_dgrad(int dtype, const void* dout, const void* wpack_d, void* dx,
                     int N, int Din, int Hin, int Win, int Cin, int Cout, int Do, int Ho, int Wo, hipStream_t s);
/* the same with an fp32 workspace of pcms_convt_dgrad_ws_floats(...) floats (0: none needed):
 * small grids (the deepest levels) split the 8 Cout reduction into K slabs summed in a fixed
 * order; ws may be NULL (no split)                                                        */
int pcms_convt_dgrad_ws_floats(int N, int Din, int Hin, int Win, int Cin, int Cout);
int pcms_convt_dgrad_ws(int dtype, const void* dout, const void* wpack_d, void* dx, float* ws,
                        int N, int Din, int Hin, int Win, int Cin, int Cout, int Do, int Ho, int Wo, hipStream_t s);
/* dw += ConvTranspose3d weight gradient; ws: pcms_convt_wgrad_ws_floats(...) fp32 (one
 * [Cin][8][Cout] partial row per voxel split, summed in a fixed order)                   */
int pcms_convt_wgrad_ws_floats(int N, int Din, int Hin, int Win, int Cin, int Cout, int target_wgs);
/* A/B switch: taps per workgroup of the bf16 Cin % 128 == 0 weight gradient (8, 4 or 2; 0 =
   chosen by shape); returns the previous setting.  Process-wide. */
/* the ConvTranspose weight gradient's split rows and (bf16 128-channel path) bias rows summed
 * by one launch (1, default) or by the group-sum / reduce / bias-reduce launches (0); the sums
 * are bit-identical; v < 0 queries; returns the previous setting (A/B switch) */
int pcms_convt_reduce_fused(int v);
int pcms_convt_wgrad_taps(int tt);
int pcms_convt_wgrad(int dtype, const void* x, const void* dout, float* dw, float* ws,
                     int N, int Din, int Hin, int Win, int Cin, int Cout, int Do, int Ho, int Wo,
                     int target_wgs, hipStream_t s);
/* pcms_convt_wgrad + the bias gradient db[co] += sum of dout over the ConvT output box
 * (F.pad front offsets floor((Do - 2 Din) / 2), ...), taken from the weight gradient's own
 * read of dout where the kernel allows it (bf16, Cin % 128 == 0), else by
 * pcms_box_channel_sum after it (models/unet3d.py:118-122 ConvTranspose3d bias, autograd);
 * bws: pcms_convt_wgrad_bias_ws_floats(...) fp32                                         */
int pcms_convt_wgrad_bias_ws_floats(int dtype, int N, int Din, int Hin, int Win, int Cin, int Cout, int target_wgs);
int pcms_convt_wgrad_bias(int dtype, const void* x, const void* dout, float* dw, float* db, float* ws, float* bws,
                          int N, int Din, int Hin, int Win, int Cin, int Cout, int Do, int Ho, int Wo,
                          int target_wgs, hipStream_t s);
/* out[c] += sum over the sub-box of x (ConvTranspose3d bias gradient); ws:
 * pcms_box_channel_sum_ws_floats(...) fp32 (per-block partial rows, fixed-order sum)     */
int pcms_box_channel_sum_ws_floats(int dtype, int N, int C, int bd, int bh, int bw);
int pcms_box_channel_sum(int dtype, const void* x, float* out, float* ws, int N, int D, int H, int W, int C,
                         int z0, int y0, int x0, int bd, int bh, int bw, hipStream_t s);

/* ---- outc Conv3d(64, ncls, 1): models/unet3d.py:222,295 ---------------------------- */
/* act 0: logits; 1: sigmoid (UNet3D.predict, :298-318); 2: sigmoid > thr as 0 / 1 floats
 * (UNet3D.inference, :320-344)                                                           */
int pcms_head_fwd(int dtype, const void* a, const float* w, const float* b, float* out,
                  long nvox_per_n, int N, int ncls, int act, float thr, hipStream_t s);
/* da = dlogits . w (written); dw / db += (per-block partial rows in ws, fixed-order sum);
 * ws: pcms_head_bwd_ws_floats(...) fp32                                                  */
int pcms_head_bwd_ws_floats(long nvox_per_n, int N, int ncls);
int pcms_head_bwd(int dtype, const void* a, const float* dlogits, const float* w, void* da, float* dw,
                  float* db, float* ws, long nvox_per_n, int N, int ncls, hipStream_t s);
/* Block fusion of the decoder's last BatchNorm3d + ReLU (models/unet3d.py:37-39, up4's
 * DoubleConv) with the head (:222, :295).  Forward: the head reads that block's pre-BN conv
 * output y and applies BN + ReLU itself (scale / shift from pcms_bn_finalize or
 * pcms_bn_eval_coeffs); the ReLU output is never stored.  Backward: dw / db += the head's
 * gradients, dgamma / dbeta += the BatchNorm's, and dy = the gradient of y -- the head's input
 * gradient is recomputed per voxel from dlogits instead of being stored and read twice.
 * ws: pcms_head_bwd_ws_floats; bnpart: pcms_head_bn_bwd_rows(...) * 64 * 2 fp32; coef: 3*64
 * fp32; bnws: pcms_bn_ws_doubles(64) fp64.  C = 64 input channels.                      */
int pcms_head_bn_fwd(int dtype, const void* y, const float* scale, const float* shift, const float* w,
                     const float* b, float* out, long nvox_per_n, int N, int ncls, int act, float thr,
                     hipStream_t s);
int pcms_head_bn_bwd_rows(long nvox_per_n, int N);
int pcms_head_bn_bwd(int dtype, const void* y, const float* scale, const float* shift, const float* mean,
                     const float* invstd, const float* gamma, const float* dlogits, const float* w, float* dw,
                     float* db, float* ws, float* bnpart, float* coef, float* dgamma, float* dbeta, void* dy,
                     long nvox_per_n, int N, int ncls, double* bnws, hipStream_t s);

/* ---- DiceLoss / BCEDiceLoss: utils/losses.py:44-92, 124-152 ------------------------ */
int pcms_loss_rows(long M);
int pcms_loss_fwd(const float* x, const float* t, long M, float smooth, float wb, float wd, float* part,
                  double* sums, float* loss, hipStream_t s);
int pcms_loss_bwd(const float* x, const float* t, long M, const double* sums, float smooth, float wb,
                  float wd, const float* gout, float* dx, hipStream_t s);

/* ---- torch.optim.Adam(lr, weight_decay=1e-5): utils/trainer.py:113-117 ------------- */
/* g_eff = s * g + wd * p, s = gscale * (*gmul if gmul != NULL): gscale = 1/world (the
 * data-parallel mean of summed gradients), *gmul = a device-side multiplier (gradient-clip
 * coefficient x AMP unscale, from pcms_grad_clip).  When s != 1, s * g is written back to g. */
int pcms_adam(float* p, float* g, float* m, float* v, long n, float step_size, float b1, float b2,
              float eps, float wd, float bc2_sqrt, float gscale, const float* gmul, hipStream_t s);
/* The same update split three ways so the weight packs come out of the same pass (bf16
 * build): conv weights by table rows int64[8] = {flat offset, Cout, Cin, fwd pack, dgrad
 * pack, first tile, fwd16 pack, dgrad16 pack} (one 32 x 32 tile per block, Cout % 32 ==
 * Cin % 32 == 0) writing each non-NULL pack: the pcms_conv3_pack2 pair and the
 * pcms_conv3_pack16 pair; ConvTranspose3d weights by rows {offset, Cin, Cout, fwd pack,
 * dgrad pack, first tile, 0, 0} writing both pcms_convt_pack packs; every other parameter
 * through [begin, end) element ranges (int64 pairs).  Identical per-element arithmetic.   */
int pcms_adam_pack_conv3(float* p, float* g, float* m, float* v, const long long* table, int ntab, int ntiles,
                         float step_size, float b1, float b2, float eps, float wd, float bc2_sqrt, float gscale,
                         const float* gmul, hipStream_t s);
int pcms_adam_pack_convt(float* p, float* g, float* m, float* v, const long long* table, int ntab, int ntiles,
                         float step_size, float b1, float b2, float eps, float wd, float bc2_sqrt, float gscale,
                         const float* gmul, hipStream_t s);
/* fp32 build: the same with the bf16x6 packs (pcms_conv3_pack / pcms_convt_pack dtype 0
 * layouts); conv tiles are 32 co x 16 ci (ntiles = sum Cout / 32 x Cin / 16), ConvT tiles
 * 32 x 32 as above.  Replaces the per-step repack of the fp32 build's weights.             */
int pcms_adam_pack_conv3_x6(float* p, float* g, float* m, float* v, const long long* table, int ntab, int ntiles,
                            float step_size, float b1, float b2, float eps, float wd, float bc2_sqrt, float gscale,
                            const float* gmul, hipStream_t s);
int pcms_adam_pack_convt_x6(float* p, float* g, float* m, float* v, const long long* table, int ntab, int ntiles,
                            float step_size, float b1, float b2, float eps, float wd, float bc2_sqrt, float gscale,
                            const float* gmul, hipStream_t s);
int pcms_adam_ranges(float* p, float* g, float* m, float* v, const long long* ranges, int nranges, long max_len,
                     float step_size, float b1, float b2, float eps, float wd, float bc2_sqrt, float gscale,
                     const float* gmul, hipStream_t s);

/* ---- torch.nn.utils.clip_grad_norm_(params, max_norm): train_bph.py:166,
 * train_bph_cv.py:311 ------------------------------------------------------------------
 * norm = gscale * ||g||_2 over the flat gradient (fp64 block partials, fixed-order sum);
 * mul = gscale * min(1, max_norm / (norm + 1e-6)) (max_norm <= 0: gscale) -> device floats;
 * apply != 0: g *= mul in place (else pass mul to pcms_adam as gmul).  A non-finite norm
 * flags inf/NaN gradients (GradScaler's found_inf).  ws: pcms_grad_clip_ws_doubles().      */
int pcms_grad_clip_ws_doubles(void);
/* p[b, e) = v for each int64 [b, e) pair of ranges (the gradient ranges no STORE writer
 * covers, zeroed before a backward into a fresh gradient)                                 */
int pcms_fill_ranges(float* p, const long long* ranges, int nranges, long max_len, float v, hipStream_t s);
int pcms_grad_clip(float* g, long n, float gscale, float max_norm, int apply, double* ws, float* norm_out,
                   float* mul_out, hipStream_t s);

/* ---- misc -------------------------------------------------------------------------- */
int pcms_add(int dtype, void* dst, const void* src, long n, hipStream_t s);
/* NDHWC (Cs stored channels) -> NCDHW fp32 (first C channels): the sub-module outputs
 * (DoubleConv3D / Down3D / Up3D called on their own, models/unet3d.py:42-158)          */
int pcms_unpack_output(int dtype, const void* in, float* out, int N, int C, int Cs, long V, hipStream_t s);

/* ---- measurement (bench.py, not a training path) ----------------------------------- */
/* One launch of nblocks single-wave workgroups; block b writes {s_memtime, s_memrealtime,
 * XCC id} to out[3b .. 3b+2] (uint64).  Two probes around a stretch of work give each XCD's
 * average shader clock over it: d(memtime) / d(memrealtime) x 100 MHz.                    */
int pcms_clock_probe(void* out, int nblocks, hipStream_t s);
/* check of the probe: every block spins `cycles` shader cycles and writes its own {t0, r0,
 * t1, r1, XCC id} to out[5b ..] (tests/tools/clock_check.py)                              */
int pcms_clock_spin(void* out, int nblocks, long cycles, hipStream_t s);

#ifdef __cplusplus
}
#endif
#endif /* PCMS_HIP_H */
