/* ddmi — MI355X-native DiffusionDrive planner hot path: C ABI.
 *
 * The boundary the reference's agent API would bind for its inference forward. Every entry
 * point takes plain pointers and sizes (device pointers for tensors, hipStream_t passed as
 * void*), returns 0 on success or a negative code, and records a message for dd_last_error().
 * No torch types cross this boundary. Reference interfaces each entry replaces:
 *
 *   dd_create   <- TransfuserAgent.__init__ + initialize()        transfuser_agent.py:38-57,94-106
 *                  (V2TransfuserModel construction, strict state_dict load with the
 *                  `agent.` / `_transfuser_model.` prefixes already stripped by the caller)
 *   dd_forward  <- TransfuserAgent.forward -> V2TransfuserModel.forward (eval)
 *                                                                  transfuser_agent.py:120-125,
 *                                                                  transfuser_model_v2.py:98-162,578-641
 *   dd_forward_ex  same, with the full output dict (bev_semantic_map, agent_states, agent_labels,
 *                  all-mode poses) of transfuser_model_v2.py:144-162,165-205
 *   dd_destroy  <- agent teardown (no reference counterpart; frees device memory)
 *
 * Threading: a handle is bound to one device and is not re-entrant; concurrent calls on one
 * handle must be serialised by the caller (the reference runs one agent per worker process,
 * run_pdm_score.py:56-57). Different handles are independent.
 */
#ifndef DDMI_H_
#define DDMI_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DD_ABI_VERSION 1

#define DD_OK 0
#define DD_ERR_INVALID -1   /* bad argument / shape / missing or mis-shaped weight */
#define DD_ERR_RUNTIME -2   /* HIP runtime failure */

typedef struct dd_handle dd_handle;

/* Mirrors the TransfuserConfig fields the hot path reads (transfuser_config.py:10-149). */
typedef struct dd_config {
  int abi_version;     /* DD_ABI_VERSION */
  int image_arch;      /* 34 = resnet34 (default), 50 = resnet50 (nuScenes-style config C4) */
  int lidar_arch;      /* 34 */
  int cam_h, cam_w;    /* 256, 1024 */
  int lidar_h, lidar_w;/* 256, 256 */
  int lidar_channels;  /* 1 (use_ground_plane = False) */
  int num_modes;       /* 20 anchors */
  int num_poses;       /* 8 */
  int trunc_timestep;  /* 8  (transfuser_model_v2.py:594) */
  int step_span;       /* 20 (transfuser_model_v2.py:585) */
} dd_config;

/* Optional outputs of dd_forward_ex (device pointers; NULL = not requested). */
typedef struct dd_outputs {
  float* trajectory;       /* B x P x 3  [x, y, heading]  (required) */
  float* poses_reg;        /* B x Q x P x 3, last step / last layer */
  float* poses_cls;        /* B x Q */
  float* bev_semantic_map; /* B x 7 x (lidar_h/2) x lidar_w, NCHW */
  float* agent_states;     /* B x 30 x 5 */
  float* agent_labels;     /* B x 30 */
} dd_outputs;

/* Outputs of dd_forward_train (device pointers; NULL = not requested). */
typedef struct dd_train_outputs {
  float* trajectory;       /* B x P x 3: the last layer's argmax mode (required) */
  float* poses_reg[2];     /* per decoder layer: B x Q x P x 3 */
  float* poses_cls[2];     /* per decoder layer: B x Q */
  float* loss;             /* 3 floats: trajectory_loss_0, trajectory_loss_1, trajectory_loss (needs targets) */
  float* bev_semantic_map; /* B x 7 x (lidar_h/2) x lidar_w, NCHW */
  float* agent_states;     /* B x 30 x 5 */
  float* agent_labels;     /* B x 30 */
} dd_train_outputs;

/* Fill *cfg with the reference defaults. */
void dd_default_config(dd_config* cfg);

/* Parse a DDW1 weight blob (diffusiondrive_amd/weights.py:pack_blob; reference state_dict key
 * schema without the `_transfuser_model.` prefix), fold BatchNorm, re-layout for the kernels and
 * upload to `device`. Missing or mis-shaped keys are an error (strict load). */
int dd_create(const dd_config* cfg, const void* weights_blob, size_t blob_bytes, int device, dd_handle** out);

/* One eval forward of B scenes. Inputs are device pointers in the reference layouts:
 * camera (B,3,cam_h,cam_w), lidar (B,C,lidar_h,lidar_w), status (B,8), noise (B,Q,P,2)
 * (the DDIM start noise the reference draws with torch.randn, transfuser_model_v2.py:593).
 * noise may be NULL: the handle then draws it on the device (Philox4x32-10 keyed by dd_set_seed's seed,
 * Box-Muller; scene s of the handle's stream since the last dd_set_seed takes draws [s*Q*P*2, (s+1)*Q*P*2)).
 * That draw is N(0,1) but NOT bit-equal to torch.randn's CPU stream: pass the noise explicitly to reproduce
 * a reference run. Any B >= 1 (more than 128 scenes run as equal chunks of at most 128, same results).
 * steps = number of truncated DDIM steps (2 in the reference). out_modes / out_cls may be NULL. */
int dd_forward(dd_handle* h, const float* camera, const float* lidar, const float* status, const float* noise,
               int B, int steps, float* out_traj, float* out_modes, float* out_cls, void* stream);

int dd_forward_ex(dd_handle* h, const float* camera, const float* lidar, const float* status, const float* noise,
                  int B, int steps, const dd_outputs* outs, void* stream);

/* The training-mode trajectory head over the eval-mode network, as a loss evaluator: replaces
 * V2TransfuserModel.forward(features, targets) with TrajectoryHead.forward_train (transfuser_model_v2.py:520-576) and
 * LossComputer (modules/multimodal_loss.py:119-168). forward_train's two random draws are inputs: timesteps (B
 * int32 in [0, 1000); the reference draws torch.randint(0, 50)) and noise (B,Q,P,2, torch.randn). The head noises the
 * normalised plan anchors per scene (diffusers add_noise), clamps, runs ONE pass of both decoder layers with each
 * scene's own time embedding, and returns every layer's poses; with target_traj (B,P,3) it also returns the
 * layers' losses cls_weight * focal + reg_weight * L1 (the reference's trajectory_cls_weight 10 / reg_weight 8) and
 * their sum. Every submodule is in eval mode (dropout off, BatchNorm running statistics). Any B >= 1 (chunks of at
 * most 128; the loss is reduced over the whole batch). */
int dd_forward_train(dd_handle* h, const float* camera, const float* lidar, const float* status, const float* noise,
                     const int* timesteps, const float* target_traj, int B, float cls_weight, float reg_weight,
                     const dd_train_outputs* outs, void* stream);
/* The BEV-semantic term of the training loss, transfuser_loss.py:28-29 (F.cross_entropy(bev_semantic_map,
 * target.long()), mean over every pixel): logits (B,C,H,W) NCHW and target (B,H,W) uint8 class ids in device memory,
 * work = dd_bev_semantic_loss_work(B, H, W) floats of device scratch, loss = one device float. Deterministic (fixed
 * reduction order). */
int dd_bev_semantic_loss(const float* logits, const unsigned char* target, int B, int C, int H, int W, float* work,
                         float* loss, void* stream);
size_t dd_bev_semantic_loss_work(int B, int H, int W);

int dd_destroy(dd_handle* h);

/* Seed of the device noise draw (noise == NULL in dd_forward) and restart of its stream at scene 0. Default
 * seed 0. No reference counterpart (the reference draws on the CPU, transfuser_model_v2.py:593). */
int dd_set_seed(dd_handle* h, unsigned long long seed);
/* The same, with the stream positioned at global scene index first_scene: rank r of a scene-sharded job that
 * passes first_scene = r * (scenes per rank) draws exactly the noise of those scenes in an unsharded run. */
int dd_set_seed_at(dd_handle* h, unsigned long long seed, unsigned long long first_scene);

/* Last error message of the calling thread ("" if none). */
const char* dd_last_error(void);

/* ---- instrumentation (bench / tests) ---------------------------------------------------- */
/* Enable per-kernel HIP-event timing (disables graph replay while on). */
int dd_set_profiling(dd_handle* h, int enable);
int dd_reset_stats(dd_handle* h);
/* Accumulated stats of one kernel class ("conv_gemm", "layernorm", ...): total device ms,
 * launches and algorithmic FLOPs (conv_gemm) since the last reset. Synchronises pending events. */
int dd_kernel_stats(dd_handle* h, const char* kernel, double* total_ms, long long* launches, double* flops);
/* Algorithmic HBM bytes of the same launches (conv / GEMM classes: input map, output, residual and weight
 * image each counted once; 0 for the other classes). */
int dd_kernel_bytes(dd_handle* h, const char* kernel, double* bytes);
/* Enable / disable hipGraph capture + replay of the forward (default on). */
int dd_set_graph(dd_handle* h, int enable);
/* Streams of the captured forward: 2 (default; $DDMI_STREAMS=0 at dd_create gives 1) = the LiDAR trunk, the tf
 * decoder and the optional heads on the handle's second stream beside the rest. The forward is captured as a program
 * of SINGLE-stream graph segments (one per run of launches between fork / join points) replayed on the two streams
 * with event records / waits between the segment launches: no graph exec has internal branch streams (the HIP runtime
 * of ROCm 7.2 faults launching a multi-stream graph whose branch streams share the launch stream's hardware queue:
 * DESIGN.md section 4, Handle lifetime). 1 = everything in order on one stream, and a forward called on a non-default
 * stream runs on that stream itself (no hand-off through the handle's own stream): the batches-in-flight mode, N such
 * handles driven from N caller streams keep N forwards in flight on one device, one hardware queue each
 * (diffusiondrive_amd/model.py InFlightPlanner); such a handle runs the decoder's value_proj without its K split (less
 * work on a shared device; $DDMI_VPROJ_SPLITS overrides). No reference counterpart (the reference runs one eager
 * forward at a time). */
int dd_set_streams(dd_handle* h, int n);
/* The handle's current stream count (1 or 2, as dd_set_streams sets it): lets a caller that switches a handle to
 * single-stream for batches in flight restore what it found (diffusiondrive_amd/runner.py). */
int dd_get_streams(dd_handle* h, int* n);
/* The captured forwards the handle holds: programs (one per shape / mode), their single-stream graph segments in all,
 * and segments whose graph has parallel branches (more than one root node: a multi-stream exec; 0 by construction). */
int dd_graph_info(dd_handle* h, int* programs, int* segments, int* multi_stream_execs);
/* Node types of those captured segments: kernel nodes, and every other node (memset / memcpy / event nodes). The
 * forward captures kernel nodes only - input staging copies run on the stream ahead of the replay, outside any graph
 * - so other_nodes is 0 (tfdec_mk4: a memset node zeroing a megakernel's counters was not seen by the
 * kernel's memory-side atomics in graph replays). */
int dd_graph_nodes(dd_handle* h, int* kernel_nodes, int* other_nodes);
/* GEMM arithmetic of every conv / linear of the path:
 *   DD_GEMM_FP32   fp32-input MFMA (v_mfma_f32_32x32x2_f32), an exact fp32 fma chain;
 *   DD_GEMM_F16X3  3-product fp16 split on f16 MFMA (conv_x3.hip): each fp32 operand becomes
 *                  hi + lo fp16, products ah*bh + ah*bl + al*bh accumulate in fp32 - fp32-class
 *                  accuracy (<= ~3*2^-22 relative per product) at 5.3x the fp32 MFMA rate.
 *   DD_GEMM_BF16   one bf16 product per MAC (operands rounded to bf16, fp32 accumulation) in the
 *                  backbone (trunks + GPT fusion), f16x3 after it (FPN, BEV tokens, decoders, heads):
 *                  the REDUCED-precision mode of the bf16 configs (BASELINE configs C2-bf16 / C4),
 *                  held to no worse than the reference's own bf16 autocast (0.06-0.08 m).
 * Default DD_GEMM_FP32, or $DDMI_GEMM=fp32|f16x3|bf16 at dd_create. Attention scores: fp32 MFMA in DD_GEMM_FP32;
 * in DD_GEMM_F16X3 the GPT attention takes f16x3's three products and the tf-decoder megakernel a three-way fp16
 * split with six products (down to 2^-22); DD_GEMM_BF16 keeps the six-product scores in the GPT attention too
 * (DESIGN.md section 5). */
#define DD_GEMM_FP32 0
#define DD_GEMM_F16X3 1
#define DD_GEMM_BF16 2
int dd_set_gemm_mode(dd_handle* h, int mode);
int dd_get_gemm_mode(dd_handle* h, int* mode);
/* Denoising schedule of the trajectory head:
 *   DD_SCHED_TRUNCATED  the reference (transfuser_model_v2.py:578-641): anchors noised to t = 8,
 *                       steps over round(arange(steps) * 20 / steps)[::-1], DDIM prev = t - 1;
 *   DD_SCHED_VANILLA    ablation C5 (no reference counterpart): x_T = noise, diffusers "leading"
 *                       set_timesteps(steps) over 1000 train steps, prev = t - 1000 / steps. */
#define DD_SCHED_TRUNCATED 0
#define DD_SCHED_VANILLA 1
int dd_set_schedule(dd_handle* h, int schedule);
/* Numerics flags raised by kernels since the last clear (synchronises the handle's stream):
 * bit 0 (DD_NUM_F16_OVERFLOW_BIT) = an activation reached |x| >= 65504 under DD_GEMM_F16X3, so that
 * forward's result is not trustworthy (re-run it in DD_GEMM_FP32); bit 1 (DD_NUM_SYNC_TIMEOUT_BIT) = the
 * tf-decoder megakernel's inter-workgroup wait gave up (never on a healthy device; same remedy); bit 2
 * (DD_NUM_SYNC_STATE_BIT) = a megakernel's inter-workgroup counter (tf decoder groups, decoder query groups) held a
 * value no healthy launch leaves there, so the waits it guards passed or failed wrongly (same remedy).
 * clear != 0 resets them, and after bit 1 or 2 also re-zeroes the inter-workgroup counters. */
#define DD_NUM_F16_OVERFLOW_BIT 1u
#define DD_NUM_SYNC_TIMEOUT_BIT 2u
#define DD_NUM_SYNC_STATE_BIT 4u
int dd_numerics_flags(dd_handle* h, unsigned* flags, int clear);
/* Copy a named internal buffer (e.g. "p3", "keyval", "cross_bev", "reg_s0l1") of the last
 * forward into dst (device pointer), at most `count` floats; *actual = buffer length. */
int dd_tap(dd_handle* h, const char* name, float* dst, size_t count, size_t* actual, void* stream);

/* ---- input feature builder (TransfuserFeatureBuilder.compute_features on the GPU) ---------- */
/* Camera feature (transfuser_features.py:57-77): crop + stitch + cv2 INTER_LINEAR resize +
 * ToTensor. cams: device uint8, B scenes x 3 images (cam_l0, cam_f0, cam_r0) x src_h x src_w x 3
 * (HWC, as NAVSIM loads them); out: device float (B, 3, out_h, out_w). The stitched image must
 * down-scale by one even integer factor (NAVSIM: 1080x1920 cameras -> 4096x1024 -> 1024x256). */
int dd_build_camera(const uint8_t* cams, int B, int src_h, int src_w, float* out, int out_h, int out_w,
                    void* stream);
/* LiDAR feature (transfuser_features.py:79-138): np.histogramdd splat of the points with
 * z < max_height (split at split_height; channels = 2 for use_ground_plane: [below, above], 1:
 * [above]) over resolution^2 bins of [range_lo, range_hi] m, clip at hist_max, / hist_max.
 * xyz: device float, per scene b the planar rows x, y, z of its N_b points (= NAVSIM
 * lidar_pc[:3], contiguous) starting at element 3 * offsets[b]; offsets: device int64 [B + 1]
 * (offsets[0] = 0); max_points = max_b N_b (launch sizing); out: device float (B, channels, res, res). */
int dd_build_lidar(const float* xyz, const int64_t* offsets, int B, int channels, float* out, int resolution,
                   float range_lo, float range_hi, int pixels_per_meter, float max_height, float split_height,
                   int hist_max, long long max_points, void* stream);

/* ---- single-op entry points (parity tests of individual kernels) ---------------------------- */
/* Last error message of a dd_op_* call on the calling thread. */
const char* dd_op_last_error(void);
/* Kernel and tile configuration of the calling thread's last conv / GEMM launch (dd_op_* or forward), e.g.
 * "conv_x6<8,32,128,4,2>": lets tests prove which route a shape took. */
const char* dd_op_last_kernel(void);
/* The decoder megakernel's GEMM core (decoder_mk.hip): out[32][N] = A[32][K] W^T + bias, A and W fp32 (W
 * [N][K] packed on the host into the MFMA-fragment f16x3 image), K % 256 == 0, N % 32 == 0; synchronous. */
int dd_op_mk_linear(const float* A, int K, const float* wgt, const float* bias, float* out, int N, void* stream);
/* Fused bev_proj (transfuser_model_v2.py:123-140 concat_cross_bev + bev_proj): out[B*H*W][256] =
 * LayerNorm(ReLU(bilinear(kvp [B][Hk][Wk][256]) + p3 wgt^T + bias)) with p3 rows of 64 channels at stride
 * p3_ld floats and wgt [256][64] = bev_proj.0's p3 columns; kvp = bev_proj.0's keyval columns applied to
 * the Hk x Wk keyval tokens. Synchronises the stream. */
int dd_op_bevproj(const float* p3, int64_t p3_ld, const float* kvp, const float* wgt, const float* bias,
                  const float* ln_g, const float* ln_b, float* out, int B, int H, int W, int Hk, int Wk, void* stream);
/* NHWC conv: in (B,H,W,Cin), wgt (Cout,KH,KW,Cin), optional bias (Cout), res (B,Ho,Wo,Cout). */
int dd_op_conv2d(const float* in, int B, int H, int W, int Cin, const float* wgt, const float* bias,
                 const float* res, float* out, int Cout, int KH, int KW, int stride, int pad, int relu, void* stream);
/* Same conv on the split-precision kernel (conv_x3.hip; weights prepared on the host as dd_create
 * does; synchronous): prec 0 = f16x3, 1 = bf16. flags (device unsigned, nullable) receives
 * DD_NUM_F16_OVERFLOW_BIT. */
int dd_op_conv2d_x3(const float* in, int B, int H, int W, int Cin, const float* wgt, const float* bias,
                    const float* res, float* out, int Cout, int KH, int KW, int stride, int pad, int relu, int prec,
                    unsigned* flags, void* stream);
/* Fused stem (replaces timm conv1 / bn1 / act1 / maxpool, transfuser_backbone.py:23-33,175-192): in (B,H,W,4)
 * NHWC, wgt (64,7,7,4) OHWI with BN folded, bias (64) -> out (B,Hp,Wp,64) = maxpool3x3/2(relu(conv7x7/2(in) +
 * bias)) on the f16x3 kernel (synchronous; weights split on the host as dd_create does). */
int dd_op_stem_pool_x3(const float* in, int B, int H, int W, const float* wgt, const float* bias, float* out,
                       unsigned* flags, void* stream);
/* The same with the arithmetic chosen: prec 0 = f16x3, 1 = bf16 (one bf16 product per MAC). */
int dd_op_stem_pool(const float* in, int B, int H, int W, const float* wgt, const float* bias, float* out, int prec,
                    unsigned* flags, void* stream);
/* The same on the reference's NCHW feature tensor of C = 1..3 channels read in place (wgt still (64,7,7,4), the
 * missing channels' taps unused) - the path dd_forward takes for the camera (C = 3) and the LiDAR histogram (C = 1,
 * which runs a one-channel kernel form: 4 k16 steps instead of 14). */
int dd_op_stem_pool_nchw(const float* in, int B, int C, int H, int W, const float* wgt, const float* bias, float* out,
                         int prec, unsigned* flags, void* stream);
/* C (M,N) = A (M,K) . W(N,K)^T [+ bias] [+ res (M,N)] [relu] */
int dd_op_gemm(const float* A, int M, int K, const float* W, const float* bias, const float* res, float* C, int N,
               int relu, void* stream);
/* Batched C_z (M,N) = A_z (M,K) . B_z, B_z (K,N) row-major (kn = 1) or (N,K) (kn = 0). */
int dd_op_gemm_batched(const float* A, const float* Bm, float* C, int batch, int M, int N, int K, int kn,
                       void* stream);
int dd_op_layernorm(const float* x, const float* res, int res_div, const float* g, const float* b,
                    const float* film_scale, const float* film_shift, float* y, int rows, int C, void* stream);
int dd_op_softmax_rows(float* x, int rows, int L, float scale, void* stream);
int dd_op_bilinear(const float* in, int B, int Hi, int Wi, int C, float* out, int Ho, int Wo, void* stream);
/* out += bilinear(in) (NHWC): the GPT-fusion upsample-add back into the trunks (transfuser_backbone.py:241-276,
 * F.interpolate(..., mode="bilinear", align_corners=False) then `+`) */
int dd_op_bilinear_add(const float* in, int B, int Hi, int Wi, int C, float* out, int Ho, int Wo, void* stream);
int dd_op_maxpool3x3s2(const float* in, int B, int H, int W, int C, float* out, void* stream);
int dd_op_avgpool(const float* in, int B, int H, int W, int C, int oh, int ow, float* out, void* stream);
int dd_op_bev_sample_attn(const float* logits, const float* pts, const float* value, float* out, int B, int Q,
                          int P, int Hv, int Wv, int C, void* stream);
int dd_op_mha_small(const float* q, const float* k, const float* v, float* out, int B, int Lq, int Lk, int nh,
                    int hd, void* stream);
/* Fused GPT self-attention core (replaces transfuser_backbone.py:386-410, SelfAttention.forward between
 * the qkv projections and `proj`): qkv (B,T,3C) packed q | k | v, y (B,T,C) =
 * softmax(q_h k_h^T / sqrt(C/heads)) v_h per (scene, head). prec 0: fp32 MFMA, T % 64 == 0 and
 * (T/4) % 8 == 0 (T <= 512), C/heads in {16, 32, 64, 128, 256, 512}; prec 1: f16x3 MFMA (the f16x3 mode:
 * scores on two-way fp16 splits, three products), prec 2: the same with three-way score splits and six products
 * (the bf16 mode's choice); both T % 32 == 0, T <= 1024, C/heads in {16, 32, 64, 128}. */
int dd_op_gpt_attention(const float* qkv, float* y, int B, int T, int C, int heads, int prec, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DDMI_H_ */
