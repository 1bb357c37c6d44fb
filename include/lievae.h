/*
 * lievae.h — C ABI of liblievae_hip.so, the MI355X (gfx950) kernels behind the
 * drop-in `lie_vae` Python API (SO(3) latent hot path of pimdh/lie-vae).
 *
 * The reference has no FFI: its "operator API" is the Python functions of
 * lie_vae/lie_tools.py, the modules of lie_vae/reparameterize.py and
 * lie_vae/decoders.py.  Each entry point below names the reference symbol
 * (file:line under the reference root) it replaces.  The ctypes binding that
 * calls them is lie-vae_amd/lie_vae/_lib.py.
 *
 * Conventions
 *  - All tensor arguments are device pointers to contiguous row-major arrays,
 *    allocated and owned by the caller.  The library never allocates device
 *    memory; backward passes that need scratch take a caller workspace sized
 *    by the matching *_workspace() query.
 *  - `stream` is a hipStream_t passed as void* (NULL = default stream).  Calls
 *    are asynchronous on that stream and never synchronise the host, so they
 *    are safe to capture in a hipGraph.
 *  - Return 0 (LV_OK) or a negative LV_ERR_* code; lv_last_error() returns a
 *    thread-local message for the last failing call on this thread.
 *  - n == 0 is a valid no-op.
 *  - Rotation matrices are (n,3,3); quaternions are scalar-LAST (x,y,z,w) as in
 *    the reference; Euler angles are ZYZ (alpha, beta, gamma).
 */
#ifndef LIEVAE_H_
#define LIEVAE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LV_OK 0
#define LV_ERR_ARG (-1)         /* bad shape / pointer / unsupported size */
#define LV_ERR_HIP (-2)         /* HIP runtime error (launch failure)      */
#define LV_ERR_WORKSPACE (-3)   /* workspace too small                    */

#define LV_DTYPE_F32 0
#define LV_DTYPE_BF16 1

#define LV_MAX_DEGREE 20        /* largest l_max compiled in              */
#define LV_MAX_CHANNELS 64      /* largest rep_copies C per call          */

int lv_abi_version(void);
const char* lv_last_error(void);
int lv_max_degree(void);

/* ---- so(3) exponential: lie_tools.py:56-64 `rodrigues` (a1+a2) --------------
 * v (n,3) -> R (n,3,3).  No small-angle branch: |v| == 0 gives NaN like the
 * reference. */
int lv_so3_exp_fwd(const float* v, float* R, int64_t n, void* stream);
int lv_so3_exp_bwd(const float* v, const float* gR, float* gv, int64_t n, void* stream);

/* ---- SO3reparameterize.nsample: reparameterize.py:269-273 --------------------
 * z[s,b] = mu[b] @ rodrigues(v[s,b]);  v (ns,B,3), mu (B,3,3), z (ns,B,3,3).
 * Backward sums gmu over the ns samples in a fixed order (deterministic). */
int lv_so3_sample_fwd(const float* mu, const float* v, float* z, int64_t ns, int64_t B,
                      void* stream);
int lv_so3_sample_bwd(const float* mu, const float* v, const float* gz, float* gmu, float* gv,
                      int64_t ns, int64_t B, void* stream);

/* ---- backward of z = mu @ exp(v) -> group_matrix_to_eazyz(z) in one pass ----
 * reparameterize.py:269-273 -> vae.py:182 (the fused path's prologue).  mu may be NULL
 * (z = exp(v)); then gmu is not written.  gang (n,3) -> gv (n,3), gmu (n,3,3).
 * Bitwise the same as lv_so3_exp_fwd / lv_mat_to_eazyz_bwd / lv_so3_exp_bwd in turn. */
int lv_exp_eazyz_vjp(const float* mu, const float* v, const float* gang, float* gmu, float* gv,
                     int64_t n, void* stream);

/* ---- quaternions_to_group_matrix: lie_tools.py:183-192 (a3) ---------------- */
int lv_quat_to_mat_fwd(const float* q, float* R, int64_t n, void* stream);
int lv_quat_to_mat_bwd(const float* q, const float* gR, float* gq, int64_t n, void* stream);

/* ---- group_matrix_to_quaternions: lie_tools.py:112-157 (a4) -----------------
 * Mirrors the 1e-6 epsilon and the argmax case choice (gradient flows through
 * the chosen case only). */
int lv_mat_to_quat_fwd(const float* R, float* q, int64_t n, void* stream);
int lv_mat_to_quat_bwd(const float* R, const float* gq, float* gR, int64_t n, void* stream);

/* ---- quaternions_to_eazyz: lie_tools.py:160-175 (a5) ----------------------- */
int lv_quat_to_eazyz_fwd(const float* q, float* ang, int64_t n, void* stream);
int lv_quat_to_eazyz_bwd(const float* q, const float* gang, float* gq, int64_t n, void* stream);

/* ---- group_matrix_to_eazyz: lie_tools.py:178-180 (a6 = a4 then a5) --------- */
int lv_mat_to_eazyz_fwd(const float* R, float* ang, int64_t n, void* stream);
int lv_mat_to_eazyz_bwd(const float* R, const float* gang, float* gR, int64_t n, void* stream);

/* ---- s2s1rodrigues: lie_tools.py:67-78 (S2S1Mean, reparameterize.py:167-181) */
int lv_s2s1_fwd(const float* axis, const float* cs, float* R, int64_t n, void* stream);
int lv_s2s1_bwd(const float* axis, const float* cs, const float* gR, float* gaxis, float* gcs,
                int64_t n, void* stream);

/* ---- fp64 twins of the per-sample maps ---------------------------------------
 * The reference's maps follow their input dtype (lie_tools.py:28-38,61: v.new_tensor,
 * eye(dtype=v.dtype)) and its self-tests run them in fp64 (lie_tools.py:271-291).
 * Same contracts as the fp32 entry points above, double pointers. */
int lv_so3_exp_fwd_f64(const double* v, double* R, int64_t n, void* stream);
int lv_so3_exp_bwd_f64(const double* v, const double* gR, double* gv, int64_t n, void* stream);
int lv_so3_sample_fwd_f64(const double* mu, const double* v, double* z, int64_t ns, int64_t B,
                          void* stream);
int lv_so3_sample_bwd_f64(const double* mu, const double* v, const double* gz, double* gmu,
                          double* gv, int64_t ns, int64_t B, void* stream);
int lv_exp_eazyz_vjp_f64(const double* mu, const double* v, const double* gang, double* gmu,
                         double* gv, int64_t n, void* stream);
int lv_quat_to_mat_fwd_f64(const double* q, double* R, int64_t n, void* stream);
int lv_quat_to_mat_bwd_f64(const double* q, const double* gR, double* gq, int64_t n, void* stream);
int lv_mat_to_quat_fwd_f64(const double* R, double* q, int64_t n, void* stream);
int lv_mat_to_quat_bwd_f64(const double* R, const double* gq, double* gR, int64_t n, void* stream);
int lv_quat_to_eazyz_fwd_f64(const double* q, double* ang, int64_t n, void* stream);
int lv_quat_to_eazyz_bwd_f64(const double* q, const double* gang, double* gq, int64_t n,
                             void* stream);
int lv_mat_to_eazyz_fwd_f64(const double* R, double* ang, int64_t n, void* stream);
int lv_mat_to_eazyz_bwd_f64(const double* R, const double* gang, double* gR, int64_t n,
                            void* stream);
int lv_s2s1_fwd_f64(const double* axis, const double* cs, double* R, int64_t n, void* stream);
int lv_s2s1_bwd_f64(const double* axis, const double* cs, const double* gR, double* gaxis,
                    double* gcs, int64_t n, void* stream);

/* ---- s2s2_gram_schmidt, fp64: lie_tools.py:81-89 (S2S2Mean, reparameterize.py:184-197)
 * Crosses along the last axis (the reference's torch.cross without dim is
 * wrong at batch 3; documented deviation). */
int lv_s2s2_fwd_f64(const double* v1, const double* v2, double* R, int64_t n, void* stream);
int lv_s2s2_bwd_f64(const double* v1, const double* v2, const double* gR, double* gv1,
                    double* gv2, int64_t n, void* stream);

/* ---- wigner_d_matrix for l = 0..L, packed: lie_tools.py:211-223 (a9) -------
 * ang (n,3) -> D (n, sum_l (2l+1)^2), block l row-major at offset
 * sum_{k<l}(2k+1)^2.  Parity/debug entry point; the hot path never materialises D. */
int lv_wigner_d_fwd(const float* ang, float* D, int64_t n, int L, void* stream);

/* ---- block_wigner_matrix_multiply: lie_tools.py:226-253 (a10) --------------
 * out[s, l^2 + i, c] = sum_j D_l(ang[s])[i,j] (or D^T if transpose) F[s, l^2 + j, c]
 * F is (M, C) shared when F_batch_stride == 0 (ActionNet's expand, decoders.py:53)
 * or (n, M, C) with F_batch_stride == M*C.  M = (L+1)^2, 1 <= C <= 64.
 * out (n, M, C) in out_dtype (LV_DTYPE_F32 | LV_DTYPE_BF16); arithmetic is fp32. */
int lv_group_action_fwd(const float* ang, const float* F, int64_t F_batch_stride, void* out,
                        int out_dtype, int64_t n, int L, int C, int transpose, void* stream);

/* Backward of lv_group_action_fwd (fp32 gout).  gang (n,3).  gF is (M,C) summed
 * over the batch (deterministic two-stage reduction through the workspace) when
 * F_batch_stride == 0, else (n,M,C).  Workspace bytes from the query below.
 * ABI note (version 2 of the workspace contract, round 5): with a shared spectrum the
 * workspace holds the dF slabs AND a 12-byte-per-sample angle-gradient region that only
 * lv_fused_exp_action_bwd writes; both entry points take the same query, so a caller that
 * cached an older (slabs-only) size gets LV_ERR_WORKSPACE -- re-query per (n, L, C).
 * The slab count follows the device's CU count (lv_compute_units), so query on the device
 * the call runs on. */
size_t lv_group_action_bwd_workspace(int64_t n, int L, int C, int shared_F);

/* Compute units of the current HIP device (hipDeviceAttributeMultiprocessorCount, cached
 * per device; 256, the MI355X count, when no device is visible): the persistent
 * backward's grid is 3 blocks per CU, so its plan, workspace and dF summation order
 * follow the part (a CPX partition has fewer CUs). */
int lv_compute_units(void);

/* Launch plans (host only, no kernel launch; for tests and capacity planning; both read the
 * device's CU count as lv_compute_units does: the forward's waves per block and the
 * backward's persistent grid follow it).  plan[] gets
 * LV_PLAN_LEN values: [0] forward: tile kernel (1) or grid-stride kernel (0); backward:
 * spectrum mode (0 per-sample, 1 shared in LDS, 2 shared from global memory with the dF
 * slab in the workspace -- the large-tile fallback, 3 the persistent kernel: C = 10,
 * 3 <= l <= 10, shared spectrum, from CUs + 1 six-sample groups (257 on MI355X), a grid
 * of min(groups, 3 * CUs) blocks, one dF slab per block), [1] grid blocks,
 * [2] degree segments, [3] threads per block, [4] dynamic LDS bytes per block,
 * [5] samples per block group, [6] forward: write-through stores / backward: workspace
 * bytes, [7..23] segment boundaries seg_lo[0..segments] (then -1), [24..39] the degree
 * set of wave k (bit l = degree l; 0 past the last wave): the kernels run these sets --
 * contiguous ranges seg_lo where a kernel stages per-wave spectrum rows, cost-balanced
 * sets otherwise.  n > 0. */
#define LV_PLAN_LEN 40
int lv_action_fwd_plan(int fused, int64_t F_batch_stride, int out_dtype, int64_t n, int L, int C,
                       int64_t* plan);
int lv_group_action_bwd_plan(int64_t n, int L, int C, int shared_F, int64_t* plan);
int lv_group_action_bwd(const float* ang, const float* F, int64_t F_batch_stride,
                        const float* gout, float* gang, float* gF, int64_t n, int L, int C,
                        int transpose, void* workspace, size_t ws_bytes, void* stream);

/* ---- fused metric kernel: z = mu @ rodrigues(v) -> ZYZ -> block D(z)·F ------
 * reparameterize.py:269-273 + vae.py:182 + decoders.py:47-56 in one pass.
 * mu (n,3,3) or NULL (identity); v (n,3); optional ang_out (n,3) receives the
 * Euler angles (for the backward).  Other arguments as lv_group_action_fwd. */
int lv_fused_exp_action_fwd(const float* mu, const float* v, const float* F,
                            int64_t F_batch_stride, void* out, int out_dtype, float* ang_out,
                            int64_t n, int L, int C, int transpose, void* stream);
/* Its backward in two launches (shared spectrum): the group-action backward writes the
 * angle gradient to the workspace, and the exp -> ZYZ VJP runs per sample in the dF
 * reduce's launch, beside the reduce;
 * gmu (n,3,3, when mu is given), gv (n,3), gF (M,C).  Bitwise equal to
 * lv_group_action_bwd + lv_exp_eazyz_vjp.  ang = the forward's ang_out; workspace as
 * lv_group_action_bwd_workspace(n, L, C, 1). */
int lv_fused_exp_action_bwd(const float* mu, const float* v, const float* ang, const float* F,
                            const float* gout, float* gmu, float* gv, float* gF, int64_t n, int L,
                            int C, int transpose, void* workspace, size_t ws_bytes, void* stream);

/* ---- N0reparameterize: reparameterize.py:100-145 (a12) ---------------------
 * sigma = softplus(h) (beta 1, threshold 20), h/sigma (B,3). */
int lv_softplus_fwd(const float* h, float* sigma, int64_t n, void* stream);
int lv_softplus_bwd(const float* h, const float* gsigma, float* gh, int64_t n, void* stream);
/* v[s,b,:] = eps[s,b,:] * sigma[b,:]; backward sums gsigma over s (deterministic). */
int lv_n0_sample_fwd(const float* sigma, const float* eps, float* v, int64_t ns, int64_t B,
                     void* stream);
int lv_n0_sample_bwd(const float* eps, const float* gv, float* gsigma, int64_t ns, int64_t B,
                     void* stream);

/* ---- SO3reparameterize.log_posterior: reparameterize.py:233-263 (a13+a15) ---
 * v (ns,B,3), sigma (B,3) -> out (ns,B): logsumexp over the 2k+1 wrapped terms. */
int lv_so3_log_posterior_fwd(const float* v, const float* sigma, float* out, int64_t ns,
                             int64_t B, int k, void* stream);
int lv_so3_log_posterior_bwd(const float* v, const float* sigma, const float* gout, float* gv,
                             float* gsigma, int64_t ns, int64_t B, int k, void* stream);

/* ---- timing helper for bench.py: K back-to-back launches of the fused kernel
 * from C, so the host-side launch cost is not Python's.  Same arguments as
 * lv_fused_exp_action_fwd plus the repeat count. */
int lv_fused_exp_action_fwd_repeat(const float* mu, const float* v, const float* F,
                                   int64_t F_batch_stride, void* out, int out_dtype,
                                   float* ang_out, int64_t n, int L, int C, int transpose,
                                   int repeats, void* stream);

/* ---- decoder ConvTranspose2d(Cin, Cout, 4, stride 2, padding 1) on MFMA (§8 f1) -----
 * Replaces the MIOpen transposed convolution behind nn.ConvTranspose2d.forward for the
 * DeconvNet upsampling layers (reference experiments/nets.py:60-75), bf16 NHWC in/out,
 * fp32 accumulate.  Cin % 8 == 0, Cout % 4 == 0, Cout <= 208.  The weight (Cin, Cout, 4, 4)
 * bf16 is first repacked into lv_deconv4s2_packed_weight_elems(Cin) bf16 elements (four
 * output phases x 208 channels x 4*Cin taps, + 64 zero bytes); bias (Cout) fp32 or NULL.
 * The same call computes the input gradient of Conv2d(Cout, Cin, 4, 2, 1) (the encoder's
 * strided convolutions, nets.py:33-57): gx = conv_transpose2d(gy, W) with the Conv2d
 * weight W (Cin_conv_out, Cout_conv_in, 4, 4) read as this layer's (Cin, Cout, 4, 4). */
size_t lv_deconv4s2_packed_weight_elems(int Cin);
int lv_deconv4s2_pack_weight_bf16(const void* w, void* wt, int Cin, int Cout, void* stream);
int lv_deconv4s2_fwd_bf16(const void* x, const void* wt, const float* bias, void* y, int64_t N,
                          int H, int W, int Cin, int Cout, void* stream);
/* The same layer with Cout <= 4 (the decoder's RGB output layer, nets.py:74): one GEMM row
 * per output quad over the 3x3 input neighbourhood, all four phases x Cout in one 16-wide
 * MFMA tile.  Weight repacked into lv_deconv4s2_small_packed_weight_elems(Cin) bf16. */
size_t lv_deconv4s2_small_packed_weight_elems(int Cin);
int lv_deconv4s2_small_pack_weight_bf16(const void* w, void* wq, int Cin, int Cout, void* stream);
int lv_deconv4s2_small_fwd_bf16(const void* x, const void* wq, const float* bias, void* y,
                                int64_t N, int H, int W, int Cin, int Cout, void* stream);
/* Backward of the small-Cout layer: gx (dgrad; needs the weight repacked by
 * lv_deconv4s2_small_pack_dgrad_weight_bf16 into lv_deconv4s2_small_dgrad_weight_elems(Cin)
 * bf16), gw (bf16, the weight's (Cin, Cout, 4, 4) layout) and gb (fp32, optional, only with
 * gw) from x and gy (bf16 channels-last).  gx or gw may be null to skip that product; gw
 * needs ws of lv_deconv4s2_small_bwd_workspace_elems(...) floats.  Cin + 1 <= 256. */
size_t lv_deconv4s2_small_dgrad_weight_elems(int Cin);
int lv_deconv4s2_small_pack_dgrad_weight_bf16(const void* w, void* wd, int Cin, int Cout, void* stream);
size_t lv_deconv4s2_small_bwd_workspace_elems(int64_t N, int H, int W, int Cin, int Cout);
int lv_deconv4s2_small_bwd_bf16(const void* x, const void* gy, const void* wd, void* gx, void* gw, float* gb,
                                float* ws, int64_t N, int H, int W, int Cin, int Cout, void* stream);
/* out[c] = sum_p g[p, c] for a channels-last (P, C) bf16 tensor (the bias gradient of a
 * convolution), C % 8 == 0; fixed-order (deterministic) two-pass sum, ws of
 * lv_channel_sum_workspace_elems(P, C) floats. */
size_t lv_channel_sum_workspace_elems(int64_t P, int C);
int lv_channel_sum_bf16(const void* g, float* out, float* ws, int64_t P, int C, void* stream);
/* ---- encoder BatchNorm2d + LeakyReLU (csrc/bn.hip; reference nets.py:33-57) ------------
 * x: channels-last (P, C) bf16, P = N·H·W.  Supported when lv_bn_supported(P, C): C >= 8,
 * C / gcd(C, 8) <= 256 and P a multiple of 8 / gcd(C, 8).  training = 1: batch statistics
 * (biased variance), save_mean / save_invstd written, running stats (may be null) updated
 * with `momentum` (unbiased variance), as torch.nn.BatchNorm2d; training = 0: the running
 * statistics normalise.  y = z > 0 ? z : slope·z, z = gamma·(x - mean)·invstd + beta
 * (gamma / beta null = 1 / 0).  ws: lv_bn_workspace_elems(P, C) floats.  Deterministic. */
int lv_bn_supported(int64_t P, int C);
size_t lv_bn_workspace_elems(int64_t P, int C);
int lv_bn_lrelu_fwd_bf16(const void* x, const float* gamma, const float* beta, float* running_mean,
                         float* running_var, int training, float momentum, float eps, float slope, void* y,
                         float* save_mean, float* save_invstd, float* ws, int64_t P, int C, void* stream);
/* Backward of the training-mode forward: gx (bf16), ggamma / gbeta (fp32, may be null). */
int lv_bn_lrelu_bwd_bf16(const void* g, const void* x, const float* gamma, const float* beta,
                         const float* save_mean, const float* save_invstd, float slope, void* gx,
                         float* ggamma, float* gbeta, float* ws, int64_t P, int C, void* stream);
/* acc[i] += (float)g[i], i < n: a bf16 parameter gradient (the autocast copy's) added in
 * place into its fp32 master gradient, one pass (replaces the cast + AccumulateGrad add pair
 * of torch.autocast's weight casts in the bf16 training step; deterministic). */
int lv_accumulate_bf16_f32(const void* g, float* acc, int64_t n, void* stream);
/* Fused ReLU around the decoder layers (DeconvNet's nn.ReLU, nets.py:62-72), flags:
 *   LV_DECONV_RELU_OUT  y = max(conv_transpose(x) + b, 0) (the ReLU after the layer);
 *   LV_DECONV_MASK_GX   (backward, small-Cout layer) gx masked by x > 0 only: x is already a
 *                       ReLU output (e.g. written with LV_DECONV_RELU_OUT), so forward and
 *                       wgrad need no max and gx is the gradient w.r.t. the ReLU's input. */
#define LV_DECONV_RELU_OUT 1
#define LV_DECONV_MASK_GX 4
int lv_deconv4s2_fwd_bf16_ex(const void* x, const void* wt, const float* bias, void* y, int64_t N,
                             int H, int W, int Cin, int Cout, int flags, void* stream);
int lv_deconv4s2_small_bwd_bf16_ex(const void* x, const void* gy, const void* wd, void* gx, void* gw,
                                   float* gb, float* ws, int64_t N, int H, int W, int Cin, int Cout,
                                   int flags, void* stream);
/* The same layer in fp32 (the reference trains in fp32: unsupervised.py:108-117), on fp32
 * MFMA (v_mfma_f32_16x16x4_f32: exact fp32 products, fp32 accumulate).  x channels-last
 * (N, H, W, Cin) fp32, y NCHW (N, Cout, 2H, 2W) fp32; Cin % 4 == 0, 1 <= Cout <= 208.  The
 * weight (Cin, Cout, 4, 4) fp32 repacked into lv_deconv4s2_packed_weight_elems_f32(Cin)
 * floats; bias (Cout) or NULL; flags 0 or LV_DECONV_RELU_OUT.  y_cl (or NULL, Cout % 4 == 0):
 * the same output also channels-last (N, 2H, 2W, Cout), e.g. the next such layer's x. */
size_t lv_deconv4s2_packed_weight_elems_f32(int Cin);
int lv_deconv4s2_pack_weight_f32(const float* w, float* wt, int Cin, int Cout, void* stream);
int lv_deconv4s2_fwd_f32(const float* x, const float* wt, const float* bias, float* y, float* y_cl,
                         int64_t N, int H, int W, int Cin, int Cout, int flags, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* LIEVAE_H_ */
