// Decoder-layer megakernel (decoder_mk.hip): parameters of one launch.
//
// One launch runs one CustomTransformerDecoderLayer (transfuser_model_v2.py:297-382) of one denoise
// step for every scene, one 512-thread workgroup per scene, the scene's 20 trajectory queries held
// in LDS from the first Linear to the last: BEV grid-sample attention, agent cross-attention, the
// hoisted ego attention, FFN, FiLM, the cls / reg heads and the cascade's point update; plus, for
// layer 0, the step's trajectory embedding and anchor encoder (:459-462, :607-617), and for layer 1
// the DDIM step / mode selection (:630-641). It also deduplicates the BEV taps of the NEXT
// (step, layer) so the gathered value_proj conv (conv_x3) can run between two launches.
#pragma once
#include <vector>

#include "common.h"

namespace ddmi {

// One f16x3 Linear (N = 256 outputs per launch unit) in MFMA-fragment order: block (nt, ks) = the
// 32 x 16 B operand fragment of output columns nt*32.. and k = ks*16.., 64 lanes x (16 B hi, 16 B lo)
// = 2 KB contiguous; lane = col % 32 + 32 * ((k % 16) / 8). `s` = per-column inverse power-of-two
// scale of the split, `b` = bias.
struct MkLin {
  const uint4* w = nullptr;
  const float* s = nullptr;
  const float* b = nullptr;
  int nks = 0;  // k16 steps of the full K
};

struct MkLayer {
  MkLin outp, ag_q, ag_out, ffn0, ffn2, c0, c3, r0, r2;
  const float *attw_w = nullptr, *attw_b = nullptr;  // [P][256] fp32
  const float *c6_w = nullptr, *c6_b = nullptr;      // [1][256]
  const float *r4_w = nullptr, *r4_b = nullptr;      // [P*3][256]
  const float *n1g, *n1b, *n2g, *n2b, *n3g, *n3b, *c2g, *c2b, *c5g, *c5b;
};

struct MkAnchor {
  MkLin pa0, pa3;  // plan_anchor_encoder Linear 512 -> 256, Linear 256 -> 256
  const float *pa2g = nullptr, *pa2b = nullptr;
};

struct MkArgs {
  MkLayer L;
  MkAnchor A;
  int layer = 0;        // 0: embed + anchor encoder first; 1: DDIM step / mode selection last
  int B = 0;
  // layer 0: DDIM sample in, this step's points / traj_feature out; layer 1: traj_feature and the
  // layer-0 points in
  float* imgx = nullptr;          // [B][Q][P][2]
  float* tfe = nullptr;           // [B*Q][256] traj_feature (written by layer 0, read by layer 1)
  float* pts = nullptr;           // [B*Q*P][2] points of this layer (layer 0 writes them)
  float* pts_next = nullptr;      // [B*Q*P][2] layer 0: its reg xy (layer 1's points)
  const float* vrows = nullptr;   // gathered value rows of this (step, layer)
  const int* slots = nullptr;     // [B][Q*P*4] compact row of each tap, -1 = zero padding
  const float* akv = nullptr;     // [B][30][512] agent K | V
  const float* ego = nullptr;     // [B][256] hoisted ego attention output
  const float* film = nullptr;    // [512] FiLM scale | shift of this (step, layer), or [B][512] (film_stride 512)
  int film_stride = 0;            // floats between scenes' FiLM vectors (0: one for the batch)
  float* gs_out = nullptr;        // [B*Q][256] BEV attention aggregate (tap)
  float* reg_out = nullptr;       // [B*Q][P][3]
  float* cls_out = nullptr;       // [B*Q]
  int* next_rows = nullptr;       // dedup tables of the next (step, layer), nullptr = none
  int* next_slots = nullptr;
  int* next_counts = nullptr;     // [B] distinct tap pixels per scene of the next (step, layer), or nullptr
  int ddim = 0;                   // layer 1: apply the DDIM step to imgx (not the last step)
  float sa_t = 0, sb_t = 0, sa_p = 0, sdir = 0;
  float* traj = nullptr;          // layer 1 of the last step: selected trajectory [B][P][3]
  int* mode_idx = nullptr;
  unsigned* flags = nullptr;
  const float* dim_t = nullptr;   // [16] gen_sineembed_for_position's 10000^(j/16), correctly rounded
  unsigned long long* stamps = nullptr;  // diagnostics: [B][32] shader-clock stamps per phase, or nullptr
  // query groups per scene (1, 2, 4): G workgroups of 20 / G queries each; the scene's last arriving group runs the
  // mode selection and the next taps' dedup (scene_cnt [B] zero between launches; next_pts [B][Q*P][2] carries the
  // DDIM-updated next points of a step's layer 1; cls_x [B][32] the scene's cls logits on 128-B lines of its own)
  int groups = 1;
  unsigned* scene_cnt = nullptr;
  float* next_pts = nullptr;
  float* cls_x = nullptr;
};

struct MkInitArgs {
  const float* anchor = nullptr;  // [Q][P][2]
  const float* noise = nullptr;   // [B][Q][P][2]
  float* imgx = nullptr;
  int* rows = nullptr;
  int* slots = nullptr;
  int* counts = nullptr;  // [B] distinct tap pixels per scene, or nullptr
  float sa = 0, s1a = 0;
  const float* sa_b = nullptr;   // per-scene add_noise coefficients (training head, forward_train), or nullptr
  const float* s1a_b = nullptr;
  int B = 0;
};

// Returns false (nothing launched) unless Q = 20 queries, P = 8 points, d = 256, 8 heads, 30 agents, a
// 64 x 64 BEV value map and ffn 1024 - the reference configuration this kernel is specialised for.
bool decoder_mk_supported(int Q, int P, int d, int nagents, int Hv, int Wv, int ffn);
// host: W [nout][nin] fp32 -> the MkLin fragment-order f16x3 image (nout % 32 == 0, nin % 16 == 0) and the
// per-output inverse scales (prep_split's power-of-two scaling)
void pack_mk_weights(const float* w, int nout, int nin, std::vector<_Float16>& packed, std::vector<float>& sinv);
// test entry: out[32][N] = A[32][K] W^T + bias through the megakernel's LDS split + MFMA GEMM core
void launch_mk_linear_test(const float* A, int K, const MkLin& W, int N, float* out, hipStream_t st);
void launch_decoder_mk(const MkArgs& a, hipStream_t st);
void launch_decoder_mk_init(const MkInitArgs& a, hipStream_t st);
// read [p, p + bytes) once so the decoder weights are cache-resident (MALL) when the first launch streams them
void launch_mk_prefetch(const void* p, size_t bytes, hipStream_t st);

// Transformer-decoder megakernel (tfdec_mk.hip): V2TransfuserModel._tf_decoder (3 post-norm
// nn.TransformerDecoderLayer, d 256, 8 heads, ffn 1024, ReLU; transfuser_model_v2.py:141-142) over the 31
// queries of one scene per workgroup, then the trajectory head's step-invariant hoists of those queries: the
// agent K / V projections and the ego attention (out_proj(v_proj(ego))) of both diffusion layers.
struct TfMkLayer {
  MkLin sa_in, sa_out, ca_q, ca_out, l1, l2;  // sa_in: 768 outputs (q | k | v); l1: 1024; l2: K = 1024
  const float *n1g = nullptr, *n1b = nullptr, *n2g = nullptr, *n2b = nullptr, *n3g = nullptr, *n3b = nullptr;
};
struct TfMkArgs {
  const TfMkLayer* layers = nullptr;  // [3] in device memory (read field by field; a by-value array in the
                                      // kernel arguments ended up copied to registers / scratch)
  const float* qemb = nullptr;  // [31][256] query embedding (the same for every scene)
  const float* kvx = nullptr;   // [B][65][1536]: layer l's cross-attention K | V of the memory at columns l * 512
  float* query_out = nullptr;   // [B][31][256]
  MkLin ag_kv[2], eg_v[2], eg_out[2];
  float* akv[2] = {nullptr, nullptr};  // [B][30][512]
  float* ego[2] = {nullptr, nullptr};  // [B][256]
  int B = 0;
  // groups = 4: four workgroups per scene (heads / hidden chunks split over them, exchanges through xbuf):
  // xbuf [B][9][4][32][256] floats (one buffer per exchange; tfdec_mk_xbuf_floats(B)), sync_cnt [2B] (arrivals,
  // finishes) zeroed at allocation; both capacities are checked at launch
  int groups = 1;
  float* xbuf = nullptr;
  size_t xbuf_floats = 0;
  unsigned* sync_cnt = nullptr;
  size_t sync_cnt_n = 0;
  int no_reset = 0;  // tests only (DDMI_TF_NORESET): the counters are left as they are
  unsigned spin_limit = 1u << 22;  // polls before a wait gives up (DD_NUM_SYNC_TIMEOUT); DDMI_TF_SPIN in tests
  unsigned* flags = nullptr;
  unsigned long long* stamps = nullptr;  // diagnostics (stamps build): [B][40] shader-clock stamps per phase
};
bool tfdec_mk_supported(int nq, int nmem, int d, int heads, int ffn, int layers);
size_t tfdec_mk_xbuf_floats(int B);  // exchange buffer of the four-workgroup form
bool tfdec_mk_layer_ok(const TfMkLayer& L);  // weight-image shapes of one layer (host check)
void launch_tfdec_mk(const TfMkArgs& a, hipStream_t st);

// Fused bev_proj (bevproj.hip): out = LN(ReLU(bilinear(kvp) + W_p3 p3 + b)) per BEV pixel, W_p3 = the
// p3 columns (256..319) of bev_proj.0 as an MkLin image (nks = 4)
struct BevProjArgs {
  const float* p3 = nullptr;  // [B*H*W] pixel rows of 64 channels at stride p3_ld floats
  int64_t p3_ld = 0;
  const float* kvp = nullptr;  // [B][Hk][Wk][256] = W[:, :256] keyval, no bias
  const uint4* w = nullptr;
  const float* s = nullptr;
  const float* bias = nullptr;
  const float* g = nullptr;  // LayerNorm
  const float* beta = nullptr;
  float* out = nullptr;  // [B*H*W][256]
  int B = 0, H = 0, W = 0, Hk = 0, Wk = 0;
  unsigned* flags = nullptr;
};
bool bevproj_supported(int C, int cin, int H, int W, int Hk, int Wk);
void launch_bevproj(const BevProjArgs& a, hipStream_t st);

}  // namespace ddmi
