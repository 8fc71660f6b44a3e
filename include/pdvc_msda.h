/*
 * pdvc_msda.h -- C ABI of the MI355X-native PDVC hot path (libpdvc_hip.so, gfx950).
 *
 * Plain pointers and sizes only: every tensor argument is a DEVICE pointer to a contiguous row-major
 * array, every `stream` is a hipStream_t passed as void*, and every host-side array argument is marked
 * "host".  Calls are asynchronous on `stream`, never synchronise, never allocate, and are safe to
 * capture into a hipGraph.  Outputs are fully written (callers need not zero them) unless a parameter
 * says "accumulated".  Every entry returns PDVC_OK (0) or a negative PDVC_ERR_*; pdvc_last_error()
 * returns a thread-local message for the last failure (argument checks mirror the reference's
 * AT_ASSERTM checks, and kernel launch failures are REPORTED here, where the reference only printf'd
 * them: pdvc/ops/src/cuda/ms_deform_im2col_cuda.cuh:949-953, 1322-1326).
 *
 * Reference interfaces replaced (paths relative to the reference repository):
 *   pdvc_ms_deform_attn_forward_*   <- MultiScaleDeformableAttention.ms_deform_attn_forward
 *                                      (pdvc/ops/src/vision.cpp:14, ms_deform_attn.h:20-41,
 *                                       cuda/ms_deform_attn_cuda.cu:20-80)
 *   pdvc_ms_deform_attn_backward_*  <- MultiScaleDeformableAttention.ms_deform_attn_backward
 *                                      (vision.cpp:15, ms_deform_attn.h:43-61, ms_deform_attn_cuda.cu:83-153)
 *   pdvc_ms_deform_sample_*         <- ms_deform_attn_core_pytorch(..., return_value=True)
 *                                      (pdvc/ops/functions/ms_deform_attn_func.py:41-68), both paddings
 *   pdvc_msda1d_*                   <- the body of MSDeformAttn.forward between its projections
 *                                      (pdvc/ops/modules/ms_deform_attn.py:167-192): softmax, sampling
 *                                      locations, 1-D lift and the op, fused; backward likewise
 *   pdvc_cap_gather_*               <- the body of MSDeformAttnCap.forward after value_proj
 *                                      (pdvc/ops/modules/ms_deform_attn_for_caption.py:92-121): sampling
 *                                      locations + border-padded raw samples
 *   pdvc_mha_*                      <- nn.MultiheadAttention's core (softmax(QK^T/sqrt(d)) V) used by
 *                                      DeformableTransformerDecoderLayer.self_attn
 *                                      (pdvc/deformable_transformer.py:231,256-258)
 *   pdvc_lstm_cell_*                <- the pointwise part of nn.LSTM (1 layer, 1 step, no bias) in
 *                                      ShowAttendTellCore.forward (pdvc/CaptioningHead/LSTM_DSA.py:206-207,261)
 *   pdvc_softattn_*                 <- ShowAttendTellCore's soft attention over the 16 samples
 *                                      (LSTM_DSA.py:245-258: tanh, alpha_net, softmax, weighted sum)
 *   pdvc_add_dropout_layernorm_*    <- the residual epilogue norm(x + dropout(s)) of every transformer sub-layer
 *                                      (deformable_transformer.py:150-156, 253-271)
 *   pdvc_layernorm_residual_* /
 *   pdvc_layernorm_backward_f32     <- NewModel front-end's ln(h) + residual (NewModel.py:41-65)
 *   pdvc_lsap_f32                   <- HungarianMatcher's scipy.optimize.linear_sum_assignment per video
 *                                      (pdvc/matcher.py:119-121), same algorithm and tie rule, on the GPU
 *   pdvc_match_cost_f32             <- HungarianMatcher's cost matrix (pdvc/matcher.py:87-117), torch's op order
 *   pdvc_graph_replace_memsets      <- (no reference counterpart) the captured training-step graph's memset nodes
 *                                      rewritten as kernel nodes before instantiation (csrc/graphfix.hip)
 *   pdvc_event_* / pdvc_stream_wait_event <- (no reference counterpart) the captured step's per-bucket events the
 *                                      data-parallel all-reduces wait on (csrc/graphfix.hip)
 *   pdvc_box_refine_*               <- iterative box refinement sigmoid(tmp + inverse_sigmoid(ref)) of the
 *                                      decoder (deformable_transformer.py:303-313) and PDVC's box heads
 *                                      (pdvc/pdvc.py:245-253, misc/detr_utils/misc.py:540-544)
 *   pdvc_set_losses_*               <- SetCriterion's loss terms of every (layer, video) problem and their
 *                                      gradients (pdvc/criterion.py:46-123 loss_labels / loss_boxes,
 *                                      :200-248 cross_entropy_with_gaussian_mask / sigmoid_focal_loss)
 *   pdvc_groupnorm_rows_*           <- nn.GroupNorm(32, d) of the base encoder's pyramid levels
 *                                      (pdvc/base_encoder.py:32-41), on channels-last rows
 *   pdvc_colsum_f32                 <- the bias gradients (sum over rows of dY) of those nn.Linear layers
 *   pdvc_cap_value_grad_f32         <- the value-gradient half of the caption sampling's backward
 *                                      (grid_sample backward in ms_deform_attn_core_pytorch), all steps at once
 *   pdvc_level_pos_rows_*           <- the encoder's positional input: PositionEmbeddingSine per level
 *                                      (position_encoding.py:20-75) + level_embed + the concatenation over levels
 *                                      (deformable_transformer.py:100-112)
 *   pdvc_relu_dropout_*             <- dropout(relu(.)) between the two FFN linears of every transformer layer
 *                                      (deformable_transformer.py:140-145 encoder, :233-237 decoder)
 *   pdvc_logprob_pick_*             <- log_softmax of the caption logits (LSTM_DSA.py:112-116) fused with the
 *                                      caption loss's target gather (LSTM_DSA.py:48-52), and its backward
 *   pdvc_seq_attention_*            <- the attention core of NewModel's two nn.MultiheadAttention front-end
 *                                      blocks over T clips (NewModel.py:41-65, cfgs/yc2_newModel_sound.yml)
 *   pdvc_gemm_f32                   <- the dense projections (nn.Linear forward/backward) of the layers
 *                                      above: MSDeformAttn value/offset/output projections
 *                                      (ms_deform_attn.py:79-126), the FFNs (deformable_transformer.py:150-156,
 *                                      240-243), fp32 on the f32-input matrix cores (round 1; an A/B form now)
 *   pdvc_gemm3_f32 / pdvc_gemm3p_f32 <- the same nn.Linear products (ms_deform_attn.py:55-58,
 *   / pdvc_split3_planes_f32           deformable_transformer.py:162-189, the caption head's gates and logits,
 *                                      LSTM_DSA.py:112-116, 206-207): fp32 GEMM by exact three-term bf16 splitting
 *                                      on the bf16 matrix cores, the default for encoder-scale products
 */
#ifndef PDVC_MSDA_H
#define PDVC_MSDA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PDVC_ABI_VERSION 1
#define PDVC_MAX_LEVELS 8

#define PDVC_OK 0
#define PDVC_ERR_INVALID_ARG (-1)
#define PDVC_ERR_LAUNCH (-2)
#define PDVC_ERR_UNSUPPORTED (-3)

#define PDVC_PAD_ZEROS 0  /* reference CUDA op semantics (ms_deform_im2col_cuda.cuh:286-291) */
#define PDVC_PAD_BORDER 1 /* grid_sample(padding_mode='border', align_corners=False) semantics */

int pdvc_abi_version(void);
const char* pdvc_last_error(void);

/* ---- drop-in operator: general 2-D multi-scale deformable attention, zero padding -------------------
 * value (N,S,M,D); spatial_shapes (L,2) int64 (H,W) DEVICE; level_start_index (L,) int64 DEVICE;
 * sampling_loc (N,Lq,M,L,P,2) [x,y]; attn_weight (N,Lq,M,L,P); output (N,Lq,M*D).
 * im2col_step is validated like the reference (N % min(N, im2col_step) == 0) but every batch element
 * is processed in one launch. */
int pdvc_ms_deform_attn_forward_f32(const float* value, const int64_t* spatial_shapes,
                                    const int64_t* level_start_index, const float* sampling_loc,
                                    const float* attn_weight, int batch, int spatial_size, int num_heads,
                                    int channels, int num_levels, int num_query, int num_point,
                                    int im2col_step, float* output, void* stream);
int pdvc_ms_deform_attn_forward_f64(const double* value, const int64_t* spatial_shapes,
                                    const int64_t* level_start_index, const double* sampling_loc,
                                    const double* attn_weight, int batch, int spatial_size, int num_heads,
                                    int channels, int num_levels, int num_query, int num_point,
                                    int im2col_step, double* output, void* stream);
/* grad_value (N,S,M,D), grad_sampling_loc (N,Lq,M,L,P,2), grad_attn_weight (N,Lq,M,L,P). */
int pdvc_ms_deform_attn_backward_f32(const float* value, const int64_t* spatial_shapes,
                                     const int64_t* level_start_index, const float* sampling_loc,
                                     const float* attn_weight, const float* grad_output, int batch,
                                     int spatial_size, int num_heads, int channels, int num_levels,
                                     int num_query, int num_point, int im2col_step, float* grad_value,
                                     float* grad_sampling_loc, float* grad_attn_weight, void* stream);
int pdvc_ms_deform_attn_backward_f64(const double* value, const int64_t* spatial_shapes,
                                     const int64_t* level_start_index, const double* sampling_loc,
                                     const double* attn_weight, const double* grad_output, int batch,
                                     int spatial_size, int num_heads, int channels, int num_levels,
                                     int num_query, int num_point, int im2col_step, double* grad_value,
                                     double* grad_sampling_loc, double* grad_attn_weight, void* stream);

/* The f32 entry points take a 1-D fast path when the level table (read on the device, never by the host) is
 * PDVC's lifted pyramid -- 4 levels, every H == 1, starts the prefix sums of W, sum W == S -- with D == 64 and
 * P == 4 (pdvc/ops/modules/ms_deform_attn.py:114-117 calls the op exactly so): the fused 1-D gather kernels,
 * and a value gradient without float atomics.  Any other table takes the general 2-D kernels.  The backward's
 * fast path needs a workspace of pdvc_ms_deform_attn_workspace_floats(...) floats (16-byte aligned): the
 * ws entry point below; pdvc_ms_deform_attn_backward_f32 (no workspace) is the general path.
 * PDVC_DROPIN_1D=0 in the environment disables the fast path (A/B). */
size_t pdvc_ms_deform_attn_workspace_floats(int batch, int num_heads, int num_levels, int num_query, int num_point);
int pdvc_ms_deform_attn_backward_ws_f32(const float* value, const int64_t* spatial_shapes,
                                        const int64_t* level_start_index, const float* sampling_loc,
                                        const float* attn_weight, const float* grad_output, int batch,
                                        int spatial_size, int num_heads, int channels, int num_levels, int num_query,
                                        int num_point, int im2col_step, float* grad_value, float* grad_sampling_loc,
                                        float* grad_attn_weight, float* workspace, size_t workspace_floats,
                                        void* stream);

/* ---- raw samples (return_value=True), general 2-D, padding PDVC_PAD_* --------------------------------
 * samples (N*M, D, Lq, L, P) exactly as the reference core returns them. */
int pdvc_ms_deform_sample_f32(const float* value, const int64_t* spatial_shapes,
                              const int64_t* level_start_index, const float* sampling_loc, int batch,
                              int spatial_size, int num_heads, int channels, int num_levels, int num_query,
                              int num_point, int padding, float* samples, void* stream);
int pdvc_ms_deform_sample_backward_f32(const float* value, const int64_t* spatial_shapes,
                                       const int64_t* level_start_index, const float* sampling_loc,
                                       const float* grad_samples, int batch, int spatial_size,
                                       int num_heads, int channels, int num_levels, int num_query,
                                       int num_point, int padding, float* grad_value,
                                       float* grad_sampling_loc, void* stream);

/* ---- fused 1-D PDVC deformable attention (zero padding = the reference GPU semantics) ----------------
 * value (N,S,M,D) = value_proj(input_flatten); value_pad_mask (N,S) uint8, 1 = padded (masked_fill 0),
 * may be NULL; proj (N,Lq,proj_stride) holds the sampling_offsets logits at [off_base + m*L*P + l*P + p]
 * and the attention_weights logits at [logit_base + ...]; ref (N,Lq,L,ref_dim), ref_dim 1 (centre) or
 * 2 (centre, length) -- ms_deform_attn.py:171-177; level_T host (L,) temporal lengths, S = sum(level_T).
 * output (N,Lq,M*D).  save_attn / save_loc (N,M,L,Lq,P), level-major: softmaxed weights and sampling
 * locations for the backward (may be NULL in inference).  Supported: L*P == 16, D in {16,32,64,128}. */
int pdvc_msda1d_forward_f32(const float* value, const uint8_t* value_pad_mask, const float* proj,
                            int proj_stride, int off_base, int logit_base, const float* ref, int ref_dim,
                            const int32_t* level_T, int num_levels, int batch, int num_query,
                            int num_heads, int head_dim, int num_point, float* output, float* save_attn,
                            float* save_loc, void* stream);
/* grad_value (N,S,M,D) (zero on padded rows); grad_proj (N,Lq,proj_stride): only the offset and logit
 * slots are written; grad_ref (N,Lq,L,ref_dim) or NULL.  `output` is the forward's output or NULL: the softmax
 * backward's row term sum_j a_j dL/da_j is computed as <grad_output, output> when it is given, else summed over
 * the sampled values themselves (no second read of a (N,Lq,M*D) tensor; the default). */
int pdvc_msda1d_backward_f32(const float* value, const uint8_t* value_pad_mask, const float* ref,
                             int ref_dim, const float* proj, int proj_stride, int off_base, int logit_base,
                             const int32_t* level_T, int num_levels, int batch, int num_query, int num_heads,
                             int head_dim, int num_point, const float* grad_output, const float* output,
                             const float* save_attn, const float* save_loc, float* grad_value, float* grad_proj,
                             float* grad_ref, void* stream);
/* The same, plus grad_value_level_sums (N, L, M*D) (NULL for none; M*D % 4 == 0, 16-byte aligned):
 * sums[(n*L + l)*M*D + c] = sum over the rows s of level l of grad_value[n, s, c] -- the value projection's bias
 * gradient is their sum over n and l.  At D = 64 the value-gradient kernel forms them from the rows it writes;
 * the other forms read grad_value once more. */
int pdvc_msda1d_backward_ex_f32(const float* value, const uint8_t* value_pad_mask, const float* ref,
                                int ref_dim, const float* proj, int proj_stride, int off_base, int logit_base,
                                const int32_t* level_T, int num_levels, int batch, int num_query, int num_heads,
                                int head_dim, int num_point, const float* grad_output, const float* output,
                                const float* save_attn, const float* save_loc, float* grad_value, float* grad_proj,
                                float* grad_ref, float* grad_value_level_sums, void* stream);
/* bf16 mode (pdvc/precision.py): the same passes, also writing the bf16 roundings (torch's RNE cast) of output /
 * grad_value / grad_proj, the operands of the projections' GEMMs -- output16 and grad_proj16 only on the encoder's
 * pyramid path (Lq = S, head_dim 64, level 0 <= 512 positions; grad_proj16 also needs proj_stride = 2 * num_heads *
 * 16); grad_value16 alone (grad_proj16 NULL: the decoder's cross-attention) wherever head_dim is 64 and the levels
 * are shorter than 65 535 positions.  Any other call returns PDVC_ERR_UNSUPPORTED before launching anything. */
int pdvc_msda1d_forward_f32_bf16out(const float* value, const uint8_t* value_pad_mask, const float* proj,
                                    int proj_stride, int off_base, int logit_base, const float* ref, int ref_dim,
                                    const int32_t* level_T, int num_levels, int batch, int num_query, int num_heads,
                                    int head_dim, int num_point, float* output, float* save_attn, float* save_loc,
                                    uint16_t* output16, void* stream);
int pdvc_msda1d_backward_ex_f32_bf16out(const float* value, const uint8_t* value_pad_mask, const float* ref,
                                        int ref_dim, const float* proj, int proj_stride, int off_base, int logit_base,
                                        const int32_t* level_T, int num_levels, int batch, int num_query,
                                        int num_heads, int head_dim, int num_point, const float* grad_output,
                                        const float* output, const float* save_attn, const float* save_loc,
                                        float* grad_value, float* grad_proj, float* grad_ref,
                                        float* grad_value_level_sums, uint16_t* grad_value16,
                                        uint16_t* grad_proj16, void* stream);

/* ---- caption-head border gather (MSDeformAttnCap) ----------------------------------------------------
 * value (N,S,M,D); value_pad_mask (N,S) or NULL; row_video (R,) int32 DEVICE: video of each query row;
 * offsets (R, off_stride) with the M*L*P sampling offsets at column off_col0, plus off_add (R, M*L*P) when
 * not NULL (the caption decoder passes the h-part and the event-part of its offset projection separately);
 * ref (R,L,ref_dim).  With ref_dim 2, rows r < rd1_rows use the centre-only formula of a 1-d reference
 * (loc = c + off / T_l; the caption heads of decoder layer 0 see the 1-d initial reference, later layers the
 * refined (c, len) boxes -- pdvc/pdvc.py:249,296), so one launch serves every decoder layer's rows.
 * samples (R, M, L*P, D) [the layout ShowAttendTellCore consumes after its permute, LSTM_DSA.py:241-242];
 * save_loc (R, M, L*P) (may be NULL). */
int pdvc_cap_gather_forward_f32(const float* value, const uint8_t* value_pad_mask, const int32_t* row_video,
                                const float* offsets, int off_stride, int off_col0, const float* off_add,
                                const float* ref, int ref_dim, int rd1_rows, const int32_t* level_T, int num_levels,
                                int batch, int rows, int num_heads, int head_dim, int num_point, float* samples,
                                float* save_loc, void* stream);
/* One caption step's sampling of the value rows (with value_pad_mask) and of the projected ctx2att rows U (same
 * shape, no mask) plus the soft attention over the 16 samples (pdvc_softattn_forward_f32 with att_h, alpha_w, alpha_b):
 * pdvc_cap_gather_forward_f32 twice and pdvc_softattn_forward_f32 in one launch, for head_dim = the attention width
 * = 512 (cap_nheads 1, every cfg).  value, U, att_h, alpha_w, samples, att and res 16-B aligned, ld_att_h % 4 == 0
 * (else PDVC_ERR_UNSUPPORTED).  Outputs as theirs: samples (R,M,16,512), save_loc (R,M,16), att (R*M*16, 512),
 * probs (R,M,16), res (R, M*512); samples and att may both be NULL (pdvc_cap_softattn_backward_f32 re-forms them). */
int pdvc_cap_softattn_forward_f32(const float* value, const uint8_t* value_pad_mask, const float* U,
                                  const int32_t* row_video, const float* offsets, int off_stride, int off_col0,
                                  const float* off_add, const float* ref, int ref_dim, int rd1_rows,
                                  const int32_t* level_T, int num_levels, int batch, int rows, int num_heads,
                                  int head_dim, int num_point, const float* att_h, int ld_att_h, const float* alpha_w,
                                  const float* alpha_b, float* samples, float* save_loc, float* att, float* probs,
                                  float* res, void* stream);
/* The backward of pdvc_cap_softattn_forward_f32 in the caption decoder's U-gradient form (the value and U gradients
 * come from pdvc_cap_value_grad_ranged_f32 after the loop): pdvc_softattn_backward_f32 and
 * pdvc_cap_gather_backward2_f32 (value2 = U) in one launch, re-forming the samples and att from their corner rows.
 * Writes grad_att (R*M*16, 512), grad_samples (R,M,16,512; may be NULL: they are probs * grad_res, rank 1, which
 * pdvc_cap_value_grad_rank1_f32 forms itself), grad_alpha_w_part (R*M, 512), grad_alpha_b_part (R*M),
 * grad_att_h (written at M == 1, accumulated otherwise) and the offset columns of grad_offsets (row stride off_stride);
 * grad_ref (may be NULL) is ACCUMULATED.  Alignment as pdvc_cap_softattn_forward_f32. */
int pdvc_cap_softattn_backward_f32(const float* value, const uint8_t* value_pad_mask, const float* U,
                                   const int32_t* row_video, const float* offsets, int off_stride, int off_col0,
                                   const float* off_add, const float* ref, int ref_dim, int rd1_rows,
                                   const int32_t* level_T, int num_levels, int batch, int rows, int num_heads,
                                   int head_dim, int num_point, const float* save_loc, const float* probs,
                                   const float* grad_res, const float* att_h, int ld_att_h, const float* alpha_w,
                                   float* grad_att, float* grad_att_h, int ld_grad_att_h, float* grad_samples,
                                   float* grad_alpha_w_part, float* grad_alpha_b_part, float* grad_offsets,
                                   float* grad_ref, void* stream);
/* grad_value and grad_ref (R,L,ref_dim, may be NULL) are ACCUMULATED (atomic adds; zero them before the first
 * call -- the caption decoder accumulates every step into one buffer); grad_offsets (R, off_stride): only the
 * offset columns are written (it is also the gradient of off_add). */
int pdvc_cap_gather_backward_f32(const float* value, const uint8_t* value_pad_mask, const int32_t* row_video,
                                 const float* offsets, int off_stride, int off_col0, const float* off_add,
                                 const float* ref, int ref_dim, int rd1_rows, const int32_t* level_T, int num_levels,
                                 int batch, int rows, int num_heads, int head_dim, int num_point,
                                 const float* save_loc, const float* grad_samples, float* grad_value,
                                 float* grad_offsets, float* grad_ref, void* stream);
/* The same with a second tensor sampled at the same locations (value2, same shape as value, no padding mask;
 * grad_samples2 its sample gradients, same shape as grad_samples): its location gradient is added to the offset and
 * reference gradients -- the caption head's ctx2att rows projected once (pdvc/ops/functions/caption_decode.py). */
int pdvc_cap_gather_backward2_f32(const float* value, const uint8_t* value_pad_mask, const int32_t* row_video,
                                  const float* offsets, int off_stride, int off_col0, const float* off_add,
                                  const float* ref, int ref_dim, int rd1_rows, const int32_t* level_T, int num_levels,
                                  int batch, int rows, int num_heads, int head_dim, int num_point,
                                  const float* save_loc, const float* grad_samples, float* grad_value,
                                  float* grad_offsets, float* grad_ref, const float* value2,
                                  const float* grad_samples2, void* stream);

/* ---- decoder query self-attention core (nn.MultiheadAttention, batch-first) -------------------------
 * qk (N,Q,2E) = [q | k] in-projections (E = num_heads*head_dim), v (N,Q,E); key_padding_mask (N,Q) uint8,
 * 1 = ignored key, may be NULL.  out (N,Q,E) = softmax(q*sqrt(1/D) k^T + mask) [dropout] v per head;
 * lse (N,M,Q) log-sum-exp of each score row (saved for the backward).  Dropout keeps a deterministic
 * counter-hash mask of (seed, video, head, query, key), regenerated by the backward.  head_dim <= 64,
 * Q <= 300. */
int pdvc_mha_forward_f32(const float* qk, const float* v, const uint8_t* key_padding_mask, int batch, int num_query,
                         int num_heads, int head_dim, float dropout_p, uint64_t seed, const uint64_t* seed_dev,
                         float* out, float* lse, void* stream);
/* workspace: pdvc_mha_workspace_floats(N, Q, M, D) floats; grad_qk (N,Q,2E) and grad_v (N,Q,E) fully
 * written.  seed_dev (device, may be NULL) overrides seed -- pass the forward's.  Q > 128 with head_dim in
 * {16,24,32,48,64} runs the flash-style MFMA kernels of pdvc_seq_attention_* (same dropout mask). */
int pdvc_mha_backward_f32(const float* qk, const float* v, const uint8_t* key_padding_mask, const float* out,
                          const float* grad_out, const float* lse, int batch, int num_query, int num_heads,
                          int head_dim, float dropout_p, uint64_t seed, const uint64_t* seed_dev, float* workspace,
                          float* grad_qk, float* grad_v, void* stream);
/* ---- caption detokenisation (host code; no GPU) ------------------------------------------------------
 * Replaces Translator.rtranslate (data/video_dataset.py:172-180) over a batch of rows for PostProcess
 * (pdvc/pdvc.py:493-546): seqs (rows, len) int64 host array; words = the concatenated vocabulary bytes,
 * word w at [word_off[w], word_off[w+1]) for 1 <= w < num_words (word_off has num_words + 1 entries).
 * Row r: ids up to the first 0, joined by ' ' plus '.', or empty when the row starts with 0; written to out
 * (out_cap bytes) back to back, row r ending at row_end[r].  Ids outside [1, num_words) are an error. */
int pdvc_detokenize(const int64_t* seqs, int rows, int len, const char* words, const int64_t* word_off,
                    int num_words, char* out, int64_t out_cap, int64_t* row_end);

/* floats of workspace pdvc_mha_backward_f32 needs: 2*N*M*Q*Q (P_d and dS tiles), or N*M*Q on the flash route */
long pdvc_mha_workspace_floats(int batch, int num_query, int num_heads, int head_dim);

/* ---- caption decoder step pieces (ShowAttendTellCore) ------------------------------------------------
 * softattn: att (R,M,16,A) = ctx2att(samples); att_h (R, ld_att_h) = h2att(h) (A values per row);
 * alpha_w (A), alpha_b (1) = alpha_net; clip (R,M,16,D) the samples.  att_res (R, M*D) = sum_j p_j clip_j with
 * p = softmax_j(alpha_net(tanh(att_j + att_h))); probs (R,M,16) saved.  Any 0 < A, D <= 512. */
int pdvc_softattn_forward_f32(const float* att, const float* att_h, int ld_att_h, const float* alpha_w,
                              const float* alpha_b, const float* clip, int rows, int num_heads, int att_hid,
                              int head_dim, float* att_res, float* probs, void* stream);
/* grad_att (R,M,16,A); grad_att_h (R, ld) (summed over heads); grad_clip (R,M,16,D) = p_j * grad_res (the
 * caller adds grad_att @ W_ctx2att); per-(row, head) partials of the alpha_net weight (R*M, A) and bias (R*M). */
int pdvc_softattn_backward_f32(const float* att, const float* att_h, int ld_att_h, const float* alpha_w,
                               const float* clip, const float* probs, const float* grad_res, int rows,
                               int num_heads, int att_hid, int head_dim, float* grad_att, float* grad_att_h,
                               int ld_grad_att_h, float* grad_clip, float* grad_alpha_w_part,
                               float* grad_alpha_b_part, void* stream);
/* lstm cell: gates = gates_a + gates_b + gates_c + gates_d (rows x 4*hidden, each with its own row stride;
 * b/c/d may be NULL), order (i,f,g,o); c_out = f*c_prev + i*g; h_out = o*tanh(c_out) (row stride ld_h_out);
 * acts (R,4H). */
int pdvc_lstm_cell_forward_f32(const float* gates_a, int lda, const float* gates_b, int ldb, const float* gates_c,
                               int ldc, const float* gates_d, int ldd, const float* c_prev, int rows, int hidden, float* h_out, int ld_h_out,
                               float* c_out, float* acts, void* stream);
/* The same with gates_a read through a row index -- row r adds gates_a[a_rows[r]] (a vocabulary table's rows: the
 * greedy decode's word gates, LSTM_DSA.py:229-231 embed then W_ih, without a gathered copy) -- and acts optional
 * (NULL: not written; greedy decoding has no backward). */
int pdvc_lstm_cell_forward_gather_f32(const float* gates_a, int lda, const int64_t* a_rows, const float* gates_b,
                                      int ldb, const float* gates_c, int ldc, const float* gates_d, int ldd,
                                      const float* c_prev, int rows, int hidden, float* h_out, int ld_h_out,
                                      float* c_out, float* acts, void* stream);
/* grad_gates (R, ld_grad_gates >= 4H; the first 4H columns written), grad_c_prev (R,H) from grad_h (+ grad_h2
 * if not NULL) and grad_c_next (or NULL). */
int pdvc_lstm_cell_backward_f32(const float* grad_h, int ld_grad_h, const float* grad_h2, int ld_grad_h2,
                                const float* grad_c_next, const float* acts, const float* c_prev, const float* c,
                                int rows, int hidden, float* grad_gates, int ld_grad_gates, float* grad_c_prev,
                                void* stream);

/* ---- fused residual epilogue: y = LayerNorm(x + dropout(s)) -----------------------------------------
 * x, s, y (rows, d) contiguous, d % 4 == 0, d <= 768; gamma, beta (d); mean, rstd (rows) saved for the backward.
 * Dropout keeps each element with probability 1-p from a counter hash of (seed, row, column), scaled by
 * 1/(1-p); seed_dev (device, may be NULL) overrides seed.  The backward regenerates the mask:
 * dx = dL/dx, ds = dL/ds, dgamma/dbeta fully written; ds_colsum (may be NULL) = column sums of ds (the bias
 * gradient of the linear that produced s) from the same pass; workspace 3*1024*d floats. */
int pdvc_add_dropout_layernorm_forward_f32(const float* x, const float* s, const float* gamma, const float* beta,
                                           int rows, int d, float p, uint64_t seed, const uint64_t* seed_dev,
                                           float eps, float* y, float* mean, float* rstd, void* stream);
int pdvc_add_dropout_layernorm_backward_f32(const float* x, const float* s, const float* gamma, const float* mean,
                                            const float* rstd, const float* dy, int rows, int d, float p,
                                            uint64_t seed, const uint64_t* seed_dev, float* dx, float* ds,
                                            float* dgamma, float* dbeta, float* ds_colsum, float* workspace,
                                            void* stream);
/* The bf16 mode's forms (pdvc/precision.py): the same passes, also writing y16 (forward) / ds16 (backward) =
 * the bf16 rounding (round to nearest even, NaN -> 0x7FC0: torch's cast) of y / ds, the operand of the GEMM
 * that reads it; y16 / ds16 rows x d uint16 (bf16 bits), 8-byte aligned. */
int pdvc_add_dropout_layernorm_forward_f32_bf16out(const float* x, const float* s, const float* gamma,
                                                   const float* beta, int rows, int d, float p, uint64_t seed,
                                                   const uint64_t* seed_dev, float eps, float* y, float* mean,
                                                   float* rstd, uint16_t* y16, void* stream);
int pdvc_add_dropout_layernorm_backward_f32_bf16out(const float* x, const float* s, const float* gamma,
                                                    const float* mean, const float* rstd, const float* dy, int rows,
                                                    int d, float p, uint64_t seed, const uint64_t* seed_dev, float* dx,
                                                    float* ds, float* dgamma, float* dbeta, float* ds_colsum,
                                                    float* workspace, uint16_t* ds16, void* stream);
/* NewModel's front-end epilogue (NewModel.py:41-65, `ln(h) + residual`): y = LayerNorm(x) * gamma + beta + r.
 * Same layout and limits; the backward writes dx and dgamma/dbeta (the residual's gradient is dy itself);
 * workspace 2*1024*d floats. */
int pdvc_layernorm_residual_forward_f32(const float* x, const float* r, const float* gamma, const float* beta, int rows,
                                        int d, float eps, float* y, float* mean, float* rstd, void* stream);
int pdvc_layernorm_backward_f32(const float* x, const float* gamma, const float* mean, const float* rstd,
                                const float* dy, int rows, int d, float* dx, float* dgamma, float* dbeta,
                                float* workspace, void* stream);

/* ---- linear sum assignment (the set matcher) --------------------------------------------------------
 * costs (P, Q, max_targets) float32: problem p matches its first sizes[p] targets (rows of scipy's transposed
 * problem) to the Q queries; sizes given on the host (validated) and on the device.  Outputs (P, max_targets)
 * int64: the matched queries of problem p in ascending order and the target of each -- scipy's
 * (row_ind, col_ind) of the (Q, sizes[p]) matrix; entries past sizes[p] are not written. */
int pdvc_lsap_f32(const float* costs, int num_problems, int num_query, int max_targets, const int32_t* sizes_host,
                  const int32_t* sizes_dev, int64_t* query_out, int64_t* target_out, void* stream);

/* ---- set criterion: matching cost and loss terms (pdvc/matcher.py:87-117, pdvc/criterion.py:46-123,200-248) ----
 * P problems (decoder layer x video) of Q queries, C classes, E target slots.  cost (P, Q, E) =
 * w_bbox * L1 + w_class * (focal pos - neg at the target's label) + w_giou * (-GIoU), every operation rounded to
 * fp32 in the order torch evaluates HungarianMatcher.cost_padded (alpha and 1 - alpha passed as the host rounds
 * them); exp / log / division as the device library rounds them. */
int pdvc_match_cost_f32(const float* logits, const float* boxes, const int64_t* labels, const float* tboxes, int P,
                        int Q, int C, int E, float alpha, float one_minus_alpha, float gamma, float w_bbox,
                        float w_class, float w_giou, float* cost, void* stream);
/* losses (P, 6) = focal ce / num_boxes, counter BCE (Gaussian-masked), L1 / num_boxes, (1 - GIoU) / num_boxes,
 * self-IoU of the matched predictions, cardinality error; logits (P, Q, C), boxes (P, Q, 2) (centre, length),
 * count (P, K1); labels (P, E) int64, tboxes (P, E, 2); nmatch (P) int64 = the true target count (ranks used);
 * num_boxes (P) float; match_query / match_target (P, E) int64 from pdvc_lsap_f32; query_mask (P, Q) u8 or NULL;
 * counter_rate (K1).  Local gradients written: dlogit (P, Q, C), dcount (P, K1), dbox (3, P, Q, 2) (L1, GIoU,
 * self-IoU planes).  E <= 64. */
int pdvc_set_losses_f32(const float* logits, const float* boxes, const float* count, const int64_t* labels,
                        const float* tboxes, const int64_t* nmatch, const float* num_boxes, const int64_t* match_query,
                        const int64_t* match_target, const uint8_t* query_mask, const float* counter_rate, int P,
                        int Q, int C, int E, int K1, float focal_alpha, float focal_gamma, int gau_mask, float beta,
                        float* losses, float* dlogit, float* dcount, float* dbox, void* stream);
/* grad_logits = g[:, 0] dlogit, grad_count = g[:, 1] dcount, grad_boxes = g[:, 2..4] . dbox planes; g (P, 6). */
int pdvc_set_losses_backward_f32(const float* grad_losses, const float* dlogit, const float* dcount, const float* dbox,
                                 int P, int Q, int C, int K1, float* grad_logits, float* grad_count, float* grad_boxes,
                                 void* stream);

/* ---- captured graphs: memset nodes as kernel nodes (csrc/graphfix.hip) -----------------------------------------
 * graph: a hipGraph_t not yet instantiated (torch.cuda.CUDAGraph(keep_graph=True).raw_cuda_graph()).  Every 1-D
 * memset node (element size 1, 2 or 4) is replaced by a kernel node writing the same value over the same elements,
 * with the same dependencies; *replaced receives the count.  Small memset nodes did not re-apply on replays on this
 * ROCm stack. */
int pdvc_graph_replace_memsets(void* graph, int* replaced);

/* Events a captured graph records for streams outside it (the data-parallel all-reduce overlap, pdvc/distributed.py;
 * no reference counterpart: the reference trains on one device).  pdvc_event_record_external on a capturing stream
 * adds an event-record node after the stream's current dependencies (every replay executes it, and the stream's later
 * captured work follows it); on any other stream it is a plain record.  pdvc_stream_wait_event makes `stream` wait
 * for the event's latest record. */
int pdvc_event_create(void** event);
int pdvc_event_destroy(void* event);
int pdvc_event_record_external(void* event, void* stream);
int pdvc_stream_wait_event(void* stream, void* event);
/* The same record, but an error unless `stream` is capturing (PDVC_ERR_INVALID_ARG): the reducer's bucket hooks use it, so a
 * hook that runs on a stream outside the capture fails the capture instead of recording a plain (already satisfied)
 * event that every replay's all-reduce would race past. */
int pdvc_event_record_captured(void* event, void* stream);

/* The overlap probe's gate (pdvc/step_graph.py dp_overlap_supported): a fine-grained host flag (coherent pinned
 * memory; *host and *dev address the same int) and a one-thread kernel that holds `stream` until the flag reads
 * `value` or timeout_ms elapses.  Captured before the probe's event record, it keeps the record from firing while
 * the host checks that a stream waiting on the event has not run -- the probe is then deterministic. */
int pdvc_host_flag_alloc(void** host, void** dev);
int pdvc_host_flag_free(void* host);
int pdvc_spin_until_flag(const int* dev_flag, int value, int timeout_ms, void* stream);

/* ---- box refinement: out = sigmoid(tmp + inverse_sigmoid(ref)) (deformable_transformer.py:303-313) ----------
 * tmp, out (rows, 2) (centre, length); ref (rows, rd), rd = 2, or 1 (only the centre refined); inverse_sigmoid clamps
 * to [0, 1] then log(max(x, eps) / max(1 - x, eps)).  Backward: grad_tmp = g s (1 - s), grad_ref (optional, NULL to
 * skip) through inverse_sigmoid with torch's clamp convention. */
int pdvc_box_refine_forward_f32(const float* tmp, const float* ref, long rows, int rd, float eps, float* out,
                                void* stream);
int pdvc_box_refine_backward_f32(const float* grad_out, const float* out, const float* ref, long rows, int rd,
                                 float eps, float* grad_tmp, float* grad_ref, void* stream);

/* ---- GroupNorm on channels-last rows (the base encoder's nn.GroupNorm(G, C) after each Conv1d) -------------
 * x, y, dy, dx (N, T, C) row-major; group g = channels [g*C/G, (g+1)*C/G) of every row of a video; mean, rstd
 * (N, G) saved by the forward (biased variance, as torch).  C/G = 4 x a power of two, C/4 divides 256.
 * chunks = ceil(T / 64).  Workspaces (floats): forward N*chunks*G*3; backward group_ws N*chunks*G*2 + N*G*2 and
 * col_partials N*chunks*2*C, whose column sums (pdvc_colsum_f32 over N*chunks rows of 2*C) are
 * [dgamma | dbeta]. */
int pdvc_groupnorm_rows_forward_f32(const float* x, int N, int T, int C, int G, float eps, const float* gamma,
                                    const float* beta, float* workspace, float* y, float* mean, float* rstd,
                                    void* stream);
int pdvc_groupnorm_rows_backward_f32(const float* x, const float* dy, const float* mean, const float* rstd,
                                     const float* gamma, int N, int T, int C, int G, float* group_ws,
                                     float* col_partials, float* dx, void* stream);
/* The pyramid-flattening forms (replace the torch.cat of the levels in deformable_transformer.py:84-106):
 * y is level l's slice of the flattened (N, S, C) encoder input, y_video_stride = S*C elements between videos
 * (>= T*C, a multiple of 4); y_copy (NULL for none) also receives the contiguous (N, T, C) result for the next
 * level's convolution.  The backward reads dy with the same video stride and adds dy_add (contiguous (N, T, C),
 * NULL for none) -- the gradient from the next level's convolution -- to it. */
int pdvc_groupnorm_rows_forward_out_f32(const float* x, int N, int T, int C, int G, float eps, const float* gamma,
                                        const float* beta, float* workspace, float* y, long y_video_stride,
                                        float* y_copy, float* mean, float* rstd, void* stream);
int pdvc_groupnorm_rows_backward_strided_f32(const float* x, const float* dy, long dy_video_stride,
                                             const float* dy_add, const float* mean, const float* rstd,
                                             const float* gamma, int N, int T, int C, int G, float* group_ws,
                                             float* col_partials, float* dx, void* stream);
/* Single-pass forms: one workgroup per (video, 64-channel block) holds the block in registers, so x (and dy) are
 * read once -- the forms above read them twice (statistics / group sums, then apply / dx).  T <= 512, C a multiple
 * of 64, C/G <= 64; any other shape returns PDVC_ERR_UNSUPPORTED before launching anything (use the forms above).
 * No workspaces; the backward's col_partials are (N, 2, C): one row of [dgamma | dbeta] partials per video.  y16
 * (NULL for none, 8-byte aligned): the forward also writes y's bf16 rounding (torch's RNE cast) at y's offsets. */
int pdvc_groupnorm_rows_forward_fused_f32(const float* x, int N, int T, int C, int G, float eps, const float* gamma,
                                          const float* beta, float* y, long y_video_stride, float* y_copy,
                                          float* mean, float* rstd, uint16_t* y16, void* stream);
int pdvc_groupnorm_rows_backward_fused_f32(const float* x, const float* dy, long dy_video_stride,
                                           const float* dy_add, const float* mean, const float* rstd,
                                           const float* gamma, int N, int T, int C, int G, float* col_partials,
                                           float* dx, void* stream);

/* ---- column sums (bias gradients) ---------------------------------------------------------------------
 * out[c] = sum_r x[r*cols + c] for a row-major (rows, cols) fp32 matrix, cols % 4 == 0, 16-byte aligned;
 * workspace: parts*cols floats (partial sums of `parts` row slabs, 1 <= parts); out 16-byte aligned.
 * Deterministic. */
int pdvc_colsum_f32(const float* x, int rows, int cols, int parts, float* workspace, float* out, void* stream);

/* ---- caption value gradient over all decoder steps -----------------------------------------------------
 * grad_value (batch, S, num_heads, head_dim), fully written (accumulation-free, no atomics): the value gradient
 * of pdvc_cap_gather_* for `steps` teacher-forced steps at once, from save_loc (steps, rows, num_heads, 16) and
 * grad_samples (steps, rows, num_heads, 16, head_dim) -- pdvc_cap_gather_backward_f32 called with
 * grad_value == NULL leaves this part out.  video_row_start (batch + 1) / video_rows (rows): DEVICE int32 CSR
 * of the caption rows of each video; max_rows_per_video bounds its row counts (host). */
int pdvc_cap_value_grad_f32(const uint8_t* value_pad_mask, const int32_t* level_T, int num_levels, int batch,
                            int num_heads, int head_dim, int num_point, int rows, int steps, int max_rows_per_video,
                            const int32_t* video_row_start, const int32_t* video_rows, const float* save_loc,
                            const float* grad_samples, float* grad_value, void* stream);
/* The same, plus grad_value_level_sums (N, L, M*D) or NULL: per-(video, level) column sums of grad_value, formed
 * from the rows the kernel writes (the caption value projection's bias gradient is their sum over n and l). */
int pdvc_cap_value_grad_ex_f32(const uint8_t* value_pad_mask, const int32_t* level_T, int num_levels, int batch,
                               int num_heads, int head_dim, int num_point, int rows, int steps, int max_rows_per_video,
                               const int32_t* video_row_start, const int32_t* video_rows, const float* save_loc,
                               const float* grad_samples, float* grad_value, float* grad_value_level_sums,
                               void* stream);
/* The same with step_rows (steps, 2) DEVICE int32 or NULL: step t of the recurrence computed only the rows
 * [step_rows[2t], step_rows[2t] + step_rows[2t + 1]) (each video's rows stop at its own last step,
 * LSTM_DSA.py:103-104); the samples of the other (step, row) pairs are skipped -- their save_loc / grad_samples
 * entries are never read. */
int pdvc_cap_value_grad_ranged_f32(const uint8_t* value_pad_mask, const int32_t* level_T, int num_levels, int batch,
                                   int num_heads, int head_dim, int num_point, int rows, int steps,
                                   int max_rows_per_video, const int32_t* video_row_start, const int32_t* video_rows,
                                   const int32_t* step_rows, const float* save_loc, const float* grad_samples,
                                   float* grad_value, float* grad_value_level_sums, void* stream);
/* bf16 mode (pdvc/precision.py): pdvc_cap_value_grad_ranged_f32 also writing grad_value's bf16 rounding (torch's RNE
 * cast) into grad_value16 (same layout, 4-byte aligned; num_heads * head_dim even). */
int pdvc_cap_value_grad_ranged_f32_bf16out(const uint8_t* value_pad_mask, const int32_t* level_T, int num_levels,
                                           int batch, int num_heads, int head_dim, int num_point, int rows, int steps,
                                           int max_rows_per_video, const int32_t* video_row_start,
                                           const int32_t* video_rows, const int32_t* step_rows, const float* save_loc,
                                           const float* grad_samples, float* grad_value, float* grad_value_level_sums,
                                           uint16_t* grad_value16, void* stream);
/* pdvc_cap_value_grad_ranged_f32 with rank-1 sample gradients: sample (step, row, head, k) has gradient
 * grad_scale[step, row, head, k] * grad_rows[step, row, head, :] -- grad_rows (steps, rows, heads, head_dim),
 * grad_scale (steps, rows, heads, 16) (the caption step's probabilities times its attended-row gradient). */
int pdvc_cap_value_grad_rank1_f32(const uint8_t* value_pad_mask, const int32_t* level_T, int num_levels, int batch,
                                  int num_heads, int head_dim, int num_point, int rows, int steps,
                                  int max_rows_per_video, const int32_t* video_row_start, const int32_t* video_rows,
                                  const int32_t* step_rows, const float* save_loc, const float* grad_rows,
                                  const float* grad_scale, float* grad_value, float* grad_value_level_sums,
                                  void* stream);

/* ---- encoder positional input ------------------------------------------------------------------------
 * pos[n, s, c] = (c < F ? (c even ? sin : cos)(xe[n*S + s] / dim_t[c]) : dur[n*Dd + c - F])
 *                + level_embed[l(s)*(F + Dd) + c],   l(s) the level of flattened row s (level_T: host array of
 * num_levels <= 8 lengths summing to S); F % 4 == Dd % 4 == 0; pos, level_embed, dur 16-byte aligned.
 * backward: partials[(n*num_levels + l)*C + c] = sum over the rows s of level l of dpos[n, s, c]. */
int pdvc_level_pos_rows_forward_f32(const float* xe, const float* dim_t, const float* dur, const float* level_embed,
                                    const int32_t* level_T, int num_levels, int N, int S, int F, int Dd, float* pos,
                                    void* stream);
int pdvc_level_pos_rows_backward_f32(const float* dpos, const int32_t* level_T, int num_levels, int N, int S, int C,
                                     float* partials, void* stream);
/* out = add + pos (add: (N, S, F + Dd), NULL for none, 16-byte aligned): the encoder's query input
 * src + lvl_pos (deformable_transformer.py:146) with the position rows generated in registers, never stored. */
int pdvc_level_pos_rows_add_f32(const float* xe, const float* dim_t, const float* dur, const float* level_embed,
                                const int32_t* level_T, int num_levels, int N, int S, int F, int Dd, const float* add,
                                float* out, void* stream);
/* bf16 mode (pdvc/precision.py): the same, also writing out16 = out rounded to bf16 (torch's RNE cast). */
int pdvc_level_pos_rows_add_f32_bf16out(const float* xe, const float* dim_t, const float* dur,
                                        const float* level_embed, const int32_t* level_T, int num_levels, int N, int S,
                                        int F, int Dd, const float* add, float* out, uint16_t* out16, void* stream);

/* ---- FFN relu + dropout --------------------------------------------------------------------------------
 * forward, in place on h (rows x cols, cols % 4 == 0, 16-byte aligned): h = relu(h) * keep / (1 - p), keep a
 * counter hash of (seed | *seed_dev, row, col) with P(keep) = 1 - p.
 * backward, in place on grad: grad = (hd > 0) ? grad / (1 - p) : 0 where hd is the forward's output; when
 * dbias != NULL also dbias[c] = sum_r grad[r, c] (workspace: parts * cols floats, parts >= 1). */
int pdvc_relu_dropout_forward_f32(float* h, long rows, int cols, float p, uint64_t seed, const uint64_t* seed_dev,
                                  void* stream);
int pdvc_relu_dropout_backward_f32(const float* hd, float* grad, int rows, int cols, float p, int parts,
                                   float* workspace, float* dbias, void* stream);
/* bf16 mode: the same passes, also writing the bf16 rounding of h / grad into h16 / g16 (rows x cols uint16). */
int pdvc_relu_dropout_forward_f32_bf16out(float* h, long rows, int cols, float p, uint64_t seed,
                                          const uint64_t* seed_dev, uint16_t* h16, void* stream);
int pdvc_relu_dropout_backward_f32_bf16out(const float* hd, float* grad, int rows, int cols, float p, int parts,
                                           float* workspace, float* dbias, uint16_t* g16, void* stream);

/* ---- caption word log-probabilities + target pick ----------------------------------------------------
 * Replaces log_softmax(logit(.)) (LSTM_DSA.py:112-116) and the target gather of the caption loss
 * (LSTM_DSA.py:48-52) for rows = caption rows x steps, V = vocabulary + 1 (row-major, row stride V).
 * forward: logp[r, :] = (x[r, :] - max) - log(sum exp(x[r, :] - max)); picked[r] = logp[r, target[r]]
 *          (NaN when target[r] is outside [0, V)).
 * backward (the loss depends on the logits only through picked): grad_logits[r, j] =
 *          grad_picked[r] * ([j == target[r]] - exp(logp[r, j])).  target: int64, one per row. */
int pdvc_logprob_pick_forward_f32(const float* logits, const int64_t* target, int rows, int V, float* logp,
                                  float* picked, void* stream);
int pdvc_logprob_pick_backward_f32(const float* logp, const int64_t* target, const float* grad_picked, int rows,
                                   int V, float* grad_logits, void* stream);
/* The same with grad_logits rows of stride ld >= V, columns [V, ld) written as zeros (a K-padded GEMM operand). */
int pdvc_logprob_pick_backward_ld_f32(const float* logp, const int64_t* target, const float* grad_picked, int rows,
                                      int V, int ld, float* grad_logits, void* stream);
/* bf16 mode (pdvc/precision.py): the same, also writing grad16 = grad_logits rounded to bf16 (torch's RNE cast) --
 * only in the register-resident row form (V % 4 == 0, V <= 8192, 16-byte aligned rows; else PDVC_ERR_UNSUPPORTED
 * and nothing is launched). */
int pdvc_logprob_pick_backward_f32_bf16out(const float* logp, const int64_t* target, const float* grad_picked,
                                           int rows, int V, float* grad_logits, uint16_t* grad16, void* stream);
/* greedy decoding's word choice (LSTM_DSA.py:149-151, torch.max over log_softmax(logits)): index[r] = the first index
 * of the largest logit of row r, logp_max[r] = its log-probability (x_max - max) - log(sum exp(x - max)); one read
 * of the logits, the (rows, V) log-probabilities are not written. */
int pdvc_logprob_argmax_f32(const float* logits, int rows, int V, int64_t* index, float* logp_max, void* stream);

/* ---- long-sequence attention core (dual-modality front-end, cfgs/yc2_newModel_sound) --------------------
 * Replaces the core of the two nn.MultiheadAttention(768, 32, batch_first=True) calls of NewModel
 * (NewModel.py:41-65): out = softmax(q k^T / sqrt(head_dim)) v per (video, head), no mask, no dropout.
 * q (N,Tq,*) row stride ldq, k / v (N,Tk,*) row strides ldk / ldv, head h at columns [h*head_dim, +head_dim);
 * out (N,Tq,num_heads*head_dim) contiguous; lse (N,num_heads,Tq) saved for the backward.  head_dim in
 * {16,24,32,48,64}; any Tq, Tk (keys streamed through LDS in tiles of 128).
 * backward: workspace N*num_heads*Tq floats; grad_q / grad_k / grad_v fully written with their row strides. */
int pdvc_seq_attention_forward_f32(const float* q, long ldq, const float* k, long ldk, const float* v, long ldv,
                                   int batch, int num_query, int num_key, int num_heads, int head_dim, float* out,
                                   float* lse, void* stream);
int pdvc_seq_attention_backward_f32(const float* q, long ldq, const float* k, long ldk, const float* v, long ldv,
                                    const float* out, const float* grad_out, const float* lse, int batch,
                                    int num_query, int num_key, int num_heads, int head_dim, float* workspace,
                                    float* grad_q, long ld_grad_q, float* grad_k, long ld_grad_k, float* grad_v,
                                    long ld_grad_v, void* stream);

/* ---- fp32 GEMM on the matrix cores ----------------------------------------------------------------
 * C[M,N] = op(A)[M,K] op(B)[K,N] (+ bias[N]) (ReLU).  op(A): trans_a 0 -> A[m*lda + k], 1 -> A[k*lda + m];
 * op(B): trans_b 0 -> B[k*ldb + n], 1 -> B[n*ldb + k].  epilogue 0 store, 1 + bias, 2 + bias then ReLU,
 * 3 atomic accumulate into C (the only epilogue allowed with split_k > 1; C is ACCUMULATED, zero it first).
 * Exact f32 products (v_mfma_f32_32x32x2_f32); summation order differs from a sequential loop. */
int pdvc_gemm_f32(int M, int N, int K, const float* A, int lda, int trans_a, const float* B, int ldb, int trans_b,
                  float* C, int ldc, const float* bias, int epilogue, int split_k, void* stream);

/* ---- fp32 GEMM on the bf16 matrix cores (three-term split) ----------------------------------------
 * Replaces the nn.Linear products of the reference's projections (pdvc/ops/modules/ms_deform_attn.py:55-58,
 * deformable_transformer.py:162-189 and their autograd backward; torch.addmm / mm in the reference).
 * C[M,N] (=|+=) sum_k opA[m,k] opB[n,k] (+ bias[n]) (ReLU), fp32 in and out.  a_kc 1 -> A[m*lda + k], 0 ->
 * A[k*lda + m]; b_kc 1 -> B[n*ldb + k], 0 -> B[k*ldb + n].  Each operand is split exactly into three bf16 terms
 * (x = x0 + x1 + x2) and the six products of order >= 2^-16 run on v_mfma_f32_32x32x16_bf16 with fp32
 * accumulation: the dropped terms are <= 2^-23 |a||b| per product (one fp32 product rounding is 2^-24).
 * epilogue 0 store, 1 + bias, 2 + bias then ReLU, 3 accumulate into C.  splits > 1 splits K over workgroups
 * into `workspace` (splits * M * N floats, epilogues 0/3 only) and sums the slabs deterministically.
 * K a multiple of 32; operands 16-byte aligned, leading dimensions divisible by 4, an mn-contiguous operand's
 * extent (M or N) divisible by 4. */
int pdvc_gemm3_f32(int M, int N, int K, const float* A, long lda, int a_kc, const float* B, long ldb, int b_kc,
                   float* C, long ldc, const float* bias, int epilogue, int splits, float* workspace, void* stream);

/* The weight gradient and the bias gradient of one nn.Linear from one pass over dy (the reference's autograd
 * backward of nn.Linear: grad_weight = dy^T x, grad_bias = dy.sum(0)): pdvc_gemm3_f32 with a_kc = b_kc = 0 and
 * epilogue 0 (C[M,N] = sum_k A[k*lda + m] B[k*ldb + n]), plus db[m] = sum_k A[k*lda + m], taken from the A rows the
 * GEMM loads (deterministic order).  M, N multiples of 4; db 16-byte aligned; splits > 1: workspace of
 * splits * M * N floats, db_ws of splits * M floats (16-byte aligned) and a dense C (ldc == N). */
int pdvc_gemm3_wgrad_bias_f32(int M, int N, int K, const float* A, long lda, const float* B, long ldb, float* C,
                              long ldc, int epilogue, int splits, float* workspace, float* db, float* db_ws,
                              void* stream);

/* Destination-sorted row sums (csrc/rowsum.hip): dst[v][c] = sum of src[order[j]][c] over the run of j with
 * sorted_keys[j] == v, for v < n_dst and c < cols (deterministic: a reduce-by-key over fixed chunks of the sorted
 * positions, the pieces of a run that crosses chunks added in chunk order; no atomics; an empty run writes zeros;
 * keys outside [0, n_dst) are ignored).  sorted_keys ascending (n entries), order the positions in that order (a
 * stable sort's permutation).  workspace: pdvc_sorted_row_sums_workspace(n, cols) floats, 16-byte aligned.
 * Replaces the scatter-add (index_add_) of the backward of a row gather -- the caption head's per-batch word-gate
 * table, LSTM_DSA.py:229-231 (embed then W_ih) in the reference.  cols a multiple of 4, src / dst 16-byte aligned,
 * ld / ldd multiples of 4. */
long pdvc_sorted_row_sums_workspace(long n, int cols);
int pdvc_sorted_row_sums_f32(const float* src, long ld, int cols, const int64_t* sorted_keys, const int64_t* order,
                             long n, int n_dst, float* dst, long ldd, float* workspace, void* stream);

/* The weight operand split once per call: planes[p][n][k] (bf16 bits, p = 0..2) of opB[n][k] (b_kc 1: B[n*ldb + k],
 * 0: B[k*ldb + n]); K a multiple of 32.  pdvc_gemm3p_f32 then computes C[M,N] (=|+=) sum_k A[m*lda + k] opB[n,k]
 * (+ bias) (ReLU) -- epilogues as pdvc_gemm3_f32 -- with the planes streamed into LDS by LDS-DMA, so that only A is
 * split inside the kernel (the forward x W^T and the data gradient dy W of nn.Linear). */
int pdvc_split3_planes_f32(const float* B, long ldb, int b_kc, int N, int K, uint16_t* planes, void* stream);
int pdvc_gemm3p_f32(int M, int N, int K, const float* A, long lda, const uint16_t* planes, float* C, long ldc,
                    const float* bias, int epilogue, void* stream);
/* linear1 of the transformer feed-forward block with its relu -> dropout in the epilogue (DeformableTransformer
 * EncoderLayer.forward_ffn, deformable_transformer.py:162-165: dropout(relu(linear1(x)))): C = keep(row, col) ?
 * relu(A opB^T + bias) / (1 - p) : 0, the keep mask of pdvc_relu_dropout_forward_f32 for the same device seed, bit for
 * bit (0 < p < 1; p = 0 is pdvc_gemm3p_f32's bias + ReLU epilogue). */
int pdvc_gemm3p_relu_dropout_f32(int M, int N, int K, const float* A, long lda, const uint16_t* planes, float* C,
                                 long ldc, const float* bias, float p, const uint64_t* seed_dev, void* stream);
/* Its backward in the data gradient of linear2's input: C = hd[m, n] > 0 ? (A opB^T)[m, n] / (1 - p) : 0, hd the
 * forward's output (C's shape and ldc) -- pdvc_relu_dropout_backward_f32's arithmetic on the GEMM result (the bias
 * gradient, its column sums, is the caller's). */
int pdvc_gemm3p_dmask_f32(int M, int N, int K, const float* A, long lda, const uint16_t* planes, float* C, long ldc,
                          const float* hd, float p, void* stream);
/* The residual sub-layer's sum before its LayerNorm, t = R + dropout(A opB^T + bias) (deformable_transformer.py:
 * 150-156 / :253-271: norm(src + dropout(src2)), src2 = a Linear): the keep mask of
 * pdvc_add_dropout_layernorm_forward_f32 for element (row, col) and the same device seed (p = 0: no dropout, seed_dev
 * may be NULL); R has C's shape and ldc.  The add-norm pass then takes t as x with s = NULL, forward and backward:
 * bit-identical to the unfused pair, one (rows x d) tensor fewer read each way. */
int pdvc_gemm3p_resid_dropout_f32(int M, int N, int K, const float* A, long lda, const uint16_t* planes, float* C,
                                  long ldc, const float* bias, const float* R, float p, const uint64_t* seed_dev,
                                  void* stream);

/* The bf16 mode's product (BASELINE configs[1]; pdvc/precision.py), the same call shape with one plane:
 * pdvc_round_plane_f32 writes plane[n][k] = bf16(opB[n][k]) (round to nearest even, torch's .to(bfloat16)) and
 * pdvc_gemm1p_f32 computes C (=|+=) sum_k bf16(A[m,k]) plane[n,k] (+ bias) (ReLU) with fp32 accumulation: A is
 * rounded inside the kernel, so an fp32 activation needs no separate cast pass (replaces the cast + hipBLASLt bf16
 * GEMM the mode issues for torch.addmm / mm). */
int pdvc_round_plane_f32(const float* B, long ldb, int b_kc, int N, int K, uint16_t* plane, void* stream);
int pdvc_gemm1p_f32(int M, int N, int K, const float* A, long lda, const uint16_t* plane, float* C, long ldc,
                    const float* bias, int epilogue, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PDVC_MSDA_H */
