// ddmi runtime: model construction from the reference state dict and the eval forward of
// V2TransfuserModel (transfuser_model_v2.py:98-162) as a sequence of MI355X kernels on one HIP
// stream, optionally captured once into a hipGraph and replayed.
//
// Exact algebraic hoists relative to the reference (same math, fewer launches):
//  * value_proj (3x3 conv + ReLU on the fixed cross-BEV map, blocks.py:68-76,114) runs once per
//    decoder layer instead of once per (step, layer): its input does not change across steps.
//  * cross_ego_attention (transfuser_model_v2.py:363-364) attends over ONE key, so softmax = 1
//    and its output is out_proj(v_proj(ego_query)) for every query and step.
//  * agent K/V projections of cross_agent_attention depend only on agents_query: once per layer.
//  * the time embedding and the FiLM scale/shift (ModulationLayer, :259-294) depend only on the
//    weights and the fixed denoise timesteps: computed once per (steps, schedule, arithmetic mode)
//    per handle and reused by every forward (ensure_film).
//  * the final DDIM step's output is never read (the trajectory comes from poses_reg, :637-641),
//    so it is skipped.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <vector>

#ifdef DDMI_SEGV_TRACE
#define DD_TRACE(...) (fprintf(stderr, "[ddmi-trace] " __VA_ARGS__), fputc('\n', stderr), fflush(stderr))
#else
#define DD_TRACE(...) ((void)0)
#endif
#include "../../include/ddmi.h"
#include "common.h"
#include "decoder_mk.h"
#include "weights.h"

namespace ddmi {

struct Block {
  bool bottleneck = false;
  Conv c1, c2, c3, ds;
  bool has_ds = false;
};
struct TrunkW {
  Conv stem;
  std::vector<std::vector<Block>> stages;
  int ch[5];
};
struct GptBlockW {
  LNp ln1, ln2;
  Lin qkv, proj, mlp0, mlp2;
};
struct GptW {
  size_t pos = kNone;
  std::vector<GptBlockW> blocks;
  LNp lnf;
  int C = 0;
};
struct TfLayerW {
  Lin sa_in, sa_out, ca_q, ca_kv, ca_out, l1, l2;
  LNp n1, n2, n3;
};
// a Linear packed for the decoder megakernel (decoder_mk.h MkLin): arena offsets
struct MkLinOff {
  size_t w = kNone, s = kNone, b = kNone;
  int nks = 0;
};
struct DiffLayerW {
  Lin attw, outp;
  Conv vproj;
  Lin ag_q, ag_kv, ag_out, eg_v, eg_out, ffn0, ffn2, film;
  LNp n1, n2, n3;
  Lin c0, c3, c6, r0, r2, r4;
  LNp c2, c5;
  MkLinOff m_outp, m_ag_q, m_ag_out, m_ffn0, m_ffn2, m_c0, m_c3, m_r0, m_r2;  // megakernel images
};

struct KStat {
  double ms = 0, flops = 0, bytes = 0;
  long long n = 0;
};

struct PendingEv {
  std::string name;
  double flops, bytes;
  hipEvent_t a, b;
  std::string detail;  // launch shape (profiling only; written to $DDMI_LAUNCH_LOG)
};

// Algorithmic HBM bytes of one conv / GEMM launch: every operand touched once - the input map (or, for
// gathered rows, the live rows' 3x3 neighbourhoods counted as one row each), the output, the residual,
// and the weight image of the arithmetic (f16x3: hi + lo fp16 = 4 B, bf16: 2 B, fp32: 4 B per weight).
static double conv_algo_bytes(const ConvArgs& c) {
  const double K = (double)c.KH * c.KW * c.Cin;
  const double rows_out = (double)c.Nimg * c.Ho * c.Wo * c.batch;
  const double in = c.rowmap ? rows_out * c.Cin : (double)c.Nimg * c.H * c.W * c.Cin * c.batch;
  const double out = rows_out * c.Cout;
  const double res = c.res ? out : 0.0;
  const double wb = (c.wh && c.prec == 1) ? 2.0 : 4.0;
  return 4.0 * (in + out + res) + wb * (double)c.Cout * K;
}

static void trunk_channels(int arch, int ch[5], bool& bottleneck) {
  if (arch == 34) {
    int c[5] = {64, 64, 128, 256, 512};
    std::memcpy(ch, c, sizeof(c));
    bottleneck = false;
  } else if (arch == 50) {
    int c[5] = {64, 256, 512, 1024, 2048};
    std::memcpy(ch, c, sizeof(c));
    bottleneck = true;
  } else {
    throw std::invalid_argument("unsupported trunk arch " + std::to_string(arch));
  }
}

// Process-wide pool of the handles' own streams: a destroyed handle returns its streams instead of destroying them,
// and a new handle takes them back. Creating and destroying many streams in one process (handles of the parity
// tests, batches-in-flight lanes and their clones) was followed by a host segfault inside hipGraphLaunch of a later
// handle's two-stream graph (ROCm 7.2; reproduced by tests/test_runner.py + test_inflight_gpu.py + test_agent.py in
// that order, the fault inside libamdhip64 under hipGraphLaunch).
static std::mutex g_stream_pool_mu;
static std::map<std::pair<int, int>, std::vector<hipStream_t>> g_stream_pool;  // (device, priority)

static bool stream_pool_on() {
  static const bool on = [] {
    const char* e = getenv("DDMI_STREAM_POOL");  // 0: create / destroy per handle (the reproducer's A/B)
    return !(e && atoi(e) == 0);
  }();
  return on;
}

static hipStream_t pooled_stream(int device, int priority = 0) {
  if (stream_pool_on()) {
    std::lock_guard<std::mutex> lk(g_stream_pool_mu);
    auto& v = g_stream_pool[{device, priority}];
    if (!v.empty()) {
      hipStream_t s = v.back();
      v.pop_back();
      return s;
    }
  }
  hipStream_t s = nullptr;
  DD_HIP_CHECK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority));
  return s;
}

static void release_stream(int device, hipStream_t s, int priority = 0) {
  (void)hipStreamSynchronize(s);
  if (!stream_pool_on()) {
    (void)hipStreamDestroy(s);
    return;
  }
  std::lock_guard<std::mutex> lk(g_stream_pool_mu);
  g_stream_pool[{device, priority}].push_back(s);
}

class Model {
 public:
  dd_config cfg;
  int device = 0;
  Arena ar;
  TrunkW img, lid;
  GptW gpt[4];
  Conv l2i[4], i2l[4];
  Conv c5, up5, up4;
  size_t kv_emb = kNone, q_emb = kNone, anchor = kNone;
  Conv bev_down;
  Lin status;
  Conv sem0, sem2;
  std::vector<TfLayerW> tf;
  Lin ag0, ag2, agl;
  Lin pa0, pa3, tm1, tm3, bevproj;
  LNp pa2, bevproj_ln;
  std::vector<DiffLayerW> dl;
  float ac[1000];  // diffusers alphas_cumprod (float32 arithmetic)

  // runtime state
  std::map<std::string, std::pair<float*, size_t>> bufs;
  bool profiling = false;
  bool use_graph = true;
  int gemm_mode = DD_GEMM_FP32;       // DD_GEMM_FP32 | DD_GEMM_F16X3 | DD_GEMM_BF16 (dd_set_gemm_mode)
  int schedule = DD_SCHED_TRUNCATED;  // DD_SCHED_TRUNCATED (reference) | DD_SCHED_VANILLA (C5 ablation)
  unsigned* num_flags = nullptr;      // device word: DD_NUM_* bits raised by kernels
  std::vector<PendingEv> pending;
  std::vector<hipEvent_t> ev_pool;
  std::map<std::string, KStat> stats;
  hipStream_t st = nullptr;   // the stream launches go to (the handle's main stream, or a side stream)
  hipStream_t st_main = nullptr, st_side = nullptr;  // the handle's own non-blocking streams (capturable)
  hipStream_t st_own = nullptr;                       // st_main as created (OnStream swaps st_main for a forward)
  hipEvent_t ev_in = nullptr, ev_out = nullptr;
  // fork / join events of one forward (reused across forwards: every record precedes its wait)
  std::vector<hipEvent_t> fj_ev;
  size_t fj_next = 0;
  // Two streams by default (dd_set_streams(h, 1) or DDMI_STREAMS=0 at dd_create: one). A two-stream forward is
  // captured as a Program of single-stream graph segments joined by event records / waits between their launches
  // (below): no graph exec has branch streams, so the HIP runtime's multi-stream graph launch - which read past its
  // candidate-stream list when a branch stream shared the launch stream's hardware queue (ROCm 7.2, DESIGN.md
  // section 4, Handle lifetime) - is never used. Batches-in-flight lanes are single-stream on their callers' streams.
  bool use_side = true;
  bool value_splitk = true;  // DDMI_VALUE_SPLITK=0: the gathered value_proj on conv_x3 (one launch, K whole)
  // DDMI_VPROJ_UNION: 1 (default) = value_proj stages each row tile's 3 x 3-neighbourhood union once per channel
  // group (value_proj.hip vproj_union_kernel); 0 = every (row, tap) gathered per K chunk
  bool vproj_union = true;
  bool ln_fold = true;  // DDMI_LN_FOLD=0: every GPT LayerNorm as its own launch (gemm_ln)
  int gpt_tail_env = -1;  // DDMI_GPT_TAIL=0 / 1: force the C <= 128 GPT block tail off / on (default: B <= 16)
  int vproj_umax = 1 << 30;  // DDMI_VPROJ_UMAX (tests): tiles with a larger union take the gathered fallback
  int vproj_usplit_env = 0;  // DDMI_VPROJ_USPLIT (1, 2, 4, 8): the union form's K split, else chosen from B
  bool stem_nchw = true;             // see use_nchw_stem
  const float** in_tab = nullptr;    // device input table: [0] camera, [1] LiDAR of the current forward
  const char* force_class = nullptr;  // profiling class of the next launch (else the chosen kernel)
  // bev_proj (DDMI_BEVPROJ): 2 "fused" = one bevproj.hip pass (f16x3 / bf16 modes; fp32 mode uses 1),
  // 1 "lowres" = keyval half at 8 x 8, upsample, K = 64 GEMM, LayerNorm; 0 "concat" = concat at 64 x 64
  int bevproj_mode = 2;
  MkLinOff m_bevp3;  // bev_proj.0's p3 columns as a fragment-order f16x3 image (bevproj.hip)
  // f16x3 + gathered value rows: the trajectory head as one megakernel launch per (step, layer)
  // (decoder_mk.hip; DDMI_DECODER_MK=0: the unfused per-op chain)
  bool decoder_mk = true;
  bool mk_ready = false;
  bool mk_stamps = false;  // diagnostics: per-phase clock stamps of the megakernel (tap "mk_stamps_s*l*")
  int mk_groups_env = 0;   // DDMI_MK_GROUPS (1, 2, 4): decoder_mk workgroups per scene, else chosen from B
  MkLinOff m_pa0, m_pa3;
  // f16x3: the tf decoder + the trajectory head's agent / ego hoists as one megakernel launch (tfdec_mk.hip;
  // DDMI_TFDEC_MK=0: the unfused per-op chain)
  bool tfdec_mk = true;
  int tf_groups_env = 0;  // DDMI_TF_GROUPS=1 / 4: force the one- / four-workgroup-per-scene tf-decoder kernel
  bool gpt_attn_x3 = true;  // f16x3 GPT attention in the f16x3 / bf16 modes (DDMI_GPT_ATTN_X3=0: the fp32-MFMA kernel)
  bool fuse_pool = true;    // GPT token pooling in the stage-final conv_x6 epilogue (DDMI_FUSE_POOL=0: avgpool launches)
  bool tf_mk_ready = false;
  struct TfMkW {
    MkLinOff sa_in, sa_out, ca_q, ca_out, l1, l2;
  } m_tf[3];
  MkLinOff m_agkv[2], m_egv[2], m_egout[2];
  Lin tf_cakv;  // the 3 layers' cross-attention K | V projections as one [1536][256] Linear
  TfMkLayer* tf_mk_layers = nullptr;  // device copy of the 3 layers' megakernel parameters
  size_t dim_t_off = kNone;
  size_t mk_w_begin = 0, mk_w_end = 0;  // arena float range of the megakernel images (prefetched per forward)
  // A captured forward: single-stream graph segments and the event operations between them, replayed in order.
  // A single-stream forward is one segment. A two-stream forward has one segment per maximal run of launches on one
  // logical stream between fork / join points (stems, the 4 trunk stages, tf decoder, heads, trajectory head: ~20);
  // each fork / join is an event record on one logical stream and a wait on the other, issued between the segment
  // launches exactly where the eager forward issues them.
  struct SegOp {
    int kind;               // 0: launch ex on stream s; 1: record fj_ev[ev] on s; 2: stream s waits fj_ev[ev]
    int s;                  // logical stream: 0 main, 1 side
    hipGraphExec_t ex;
    int ev;
  };
  struct Program {
    std::vector<SegOp> ops;
    int segments = 0;
    int branched = 0;  // segments whose graph has more than one root (parallel branches): 0 by construction
    int kernel_nodes = 0, other_nodes = 0;  // node types of the captured segments (memset / copy nodes: none)
  };
  // program cache keyed by the forward's shape signature; every entry belongs to the current buffer
  // generation (the cache is emptied when a workspace buffer is (re)allocated: graphs hold its pointers)
  std::map<std::string, Program> programs;
  static void destroy_program(Program& p) {
    for (auto& op : p.ops)
      if (op.kind == 0 && op.ex) (void)hipGraphExecDestroy(op.ex);
    p.ops.clear();
  }
  void drop_graphs() {
    for (auto& g : programs) destroy_program(g.second);
    programs.clear();
  }
  uint64_t graph_gen = 0;
  uint64_t generation = 0;  // bumped whenever a workspace buffer is (re)allocated
  std::set<std::string> known_shapes;
  // a forward of more than max_chunk scenes runs as equal chunks of at most max_chunk (every kernel's 32-bit
  // buffer offsets stay below 2 GiB up to 256 scenes; DDMI_MAX_CHUNK overrides, read at dd_create)
  int max_chunk = 128;
  // noise == NULL: the DDIM start noise is drawn on the device (Philox4x32-10 + Box-Muller, keyed by
  // rng_seed; scene s of the stream since dd_set_seed takes draws [s Q P 2, (s + 1) Q P 2))
  uint64_t rng_seed = 0, rng_next = 0;
  // dd_forward_train (the training-mode trajectory head as a loss evaluator, TrajectoryHead.forward_train
  // transfuser_model_v2.py:520-576): set for the duration of one such call. The head then runs ONE pass of the two
  // layers from per-scene noised anchors (timesteps staged in "in_tsteps"), with per-scene time embeddings / FiLM,
  // and - given targets ("in_target") - LossComputer's per-scene partials per layer (train_loss.hip).
  bool train = false;
  const int* train_t = nullptr;        // caller's timesteps of the current chunk (device int32)
  const float* train_target = nullptr;  // caller's target trajectories of the current chunk (device, or nullptr)
  float* ac_dev = nullptr;              // alphas_cumprod on the device (per-scene add_noise coefficients)
  float* train_part = nullptr;          // [2 layers][B][2] LossComputer partials of the whole call
  size_t train_part_n = 0;
  float* train_loss_dev = nullptr;      // [3] trajectory_loss_0, _1, sum

  Model(const dd_config& c, const void* blob, size_t bytes, int dev) : cfg(c), device(dev) {
    DD_HIP_CHECK(hipSetDevice(device));
    BlobIndex bx(blob, bytes);
    build(bx);
    ar.upload();
    decoder_init_constants();
    if (tf_mk_ready) {
      TfMkLayer h[3];
      for (int i = 0; i < 3; ++i) {
        h[i].sa_in = mk(m_tf[i].sa_in);
        h[i].sa_out = mk(m_tf[i].sa_out);
        h[i].ca_q = mk(m_tf[i].ca_q);
        h[i].ca_out = mk(m_tf[i].ca_out);
        h[i].l1 = mk(m_tf[i].l1);
        h[i].l2 = mk(m_tf[i].l2);
        h[i].n1g = W(tf[i].n1.g);
        h[i].n1b = W(tf[i].n1.b);
        h[i].n2g = W(tf[i].n2.g);
        h[i].n2b = W(tf[i].n2.b);
        h[i].n3g = W(tf[i].n3.g);
        h[i].n3b = W(tf[i].n3.b);
        if (!tfdec_mk_layer_ok(h[i])) throw std::runtime_error("tfdec_mk: weight image shapes");
      }
      DD_HIP_CHECK(hipMalloc(&tf_mk_layers, sizeof(h)));
      DD_HIP_CHECK(hipMemcpy(tf_mk_layers, h, sizeof(h), hipMemcpyHostToDevice));
    }
    // both streams at default priority (one at the device's greatest priority measured 3-3.5 % slower in the B = 64
    // bench graph, both at the least priority 33 % slower)
    if (const char* e = getenv("DDMI_STREAMS")) use_side = atoi(e) != 0;
    st_main = pooled_stream(device, 0);
    st_side = pooled_stream(device);
    st = st_own = st_main;
    DD_TRACE("create model %p st_main=%p st_side=%p", (void*)this, (void*)st_main, (void*)st_side);
    if (const char* e = getenv("DDMI_VALUE_SPLITK")) value_splitk = atoi(e) != 0;
    if (const char* e = getenv("DDMI_STEM_NCHW")) stem_nchw = atoi(e) != 0;
    if (const char* e = getenv("DDMI_VPROJ_UNION")) vproj_union = atoi(e) != 0;
    if (const char* e = getenv("DDMI_LN_FOLD")) ln_fold = atoi(e) != 0;
    if (const char* e = getenv("DDMI_GPT_TAIL")) gpt_tail_env = atoi(e) != 0;
    if (const char* e = getenv("DDMI_VPROJ_UMAX")) vproj_umax = std::max(0, atoi(e));
    if (const char* e = getenv("DDMI_VPROJ_USPLIT")) {
      vproj_usplit_env = atoi(e);
      if (vproj_usplit_env < 1 || vproj_usplit_env > 8 || (vproj_usplit_env & (vproj_usplit_env - 1)))
        throw std::invalid_argument("DDMI_VPROJ_USPLIT must be 1, 2, 4 or 8");
    }
    DD_HIP_CHECK(hipMalloc(&in_tab, 4 * sizeof(float*)));
    // zeroed on the handle's own stream and waited for: ordered before any forward, on whichever stream it runs
    DD_HIP_CHECK(hipMemsetAsync(in_tab, 0, 4 * sizeof(float*), st_own));
    if (const char* e = getenv("DDMI_BEVPROJ")) {
      if (!strcmp(e, "fused")) bevproj_mode = 2;
      else if (!strcmp(e, "lowres")) bevproj_mode = 1;
      else if (!strcmp(e, "concat")) bevproj_mode = 0;
      else throw std::invalid_argument(std::string("DDMI_BEVPROJ must be fused, lowres or concat, got ") + e);
    }
    if (const char* e = getenv("DDMI_DECODER_MK")) decoder_mk = atoi(e) != 0;
    if (const char* e = getenv("DDMI_TFDEC_MK")) tfdec_mk = atoi(e) != 0;
    if (const char* e = getenv("DDMI_TF_GROUPS")) tf_groups_env = atoi(e);
    if (const char* e = getenv("DDMI_GPT_ATTN_X3")) gpt_attn_x3 = atoi(e) != 0;
    if (const char* e = getenv("DDMI_FUSE_POOL")) fuse_pool = atoi(e) != 0;
    if (const char* e = getenv("DDMI_MK_STAMPS")) mk_stamps = atoi(e) != 0;
    if (const char* e = getenv("DDMI_MK_GROUPS")) {
      mk_groups_env = atoi(e);
      if (mk_groups_env != 1 && mk_groups_env != 2 && mk_groups_env != 4)
        throw std::invalid_argument("DDMI_MK_GROUPS must be 1, 2 or 4");
    }
    if (const char* e = getenv("DDMI_MAX_CHUNK")) {
      max_chunk = atoi(e);
      if (max_chunk < 1 || max_chunk > 256) throw std::invalid_argument("DDMI_MAX_CHUNK must be in [1, 256]");
    }
    DD_HIP_CHECK(hipMalloc(&num_flags, sizeof(unsigned)));
    DD_HIP_CHECK(hipMemsetAsync(num_flags, 0, sizeof(unsigned), st_own));
    DD_HIP_CHECK(hipStreamSynchronize(st_own));
    if (const char* g = getenv("DDMI_GEMM")) {
      if (!strcmp(g, "fp32")) gemm_mode = DD_GEMM_FP32;
      else if (!strcmp(g, "f16x3")) gemm_mode = DD_GEMM_F16X3;
      else if (!strcmp(g, "bf16")) gemm_mode = DD_GEMM_BF16;
      else throw std::invalid_argument(std::string("DDMI_GEMM must be fp32, f16x3 or bf16, got ") + g);
    }
    DD_HIP_CHECK(hipEventCreateWithFlags(&ev_in, hipEventDisableTiming));
    DD_HIP_CHECK(hipEventCreateWithFlags(&ev_out, hipEventDisableTiming));
    DD_HIP_CHECK(hipEventRecord(ev_out, st_own));  // recorded once, so every later wait on it is well defined
    // diffusers DDIMScheduler(beta_schedule="scaled_linear") schedule, bit-exact to the float32
    // arithmetic PyTorch-CPU performs for it (transfuser_model_v2.py:447-451):
    //   betas = torch.linspace(sqrt(1e-4), sqrt(0.02), 1000, float32) ** 2
    //     (ATen linspace: step = (end - start) / 999 in float; value = fma(step, i, start) for
    //      i < 500, fma(-step, 999 - i, end) otherwise)
    //   alphas_cumprod = torch.cumprod(1 - betas)  (CPU cumprod accumulates in double).
    // The truncated add_noise multiplies noise by sqrt(1 - alphas_cumprod[8]) ~ 0.03: one ulp of
    // alphas_cumprod[8] moves every noisy anchor by ~3e-5 m, so this table must be exact.
    {
      const float start = 0.01f, end = (float)std::sqrt(0.02);
      const float step = (end - start) / 999.0f;
      double acc = 1.0;
      for (int i = 0; i < 1000; ++i) {
        const float lin = i < 500 ? std::fma(step, (float)i, start) : std::fma(-step, (float)(999 - i), end);
        const float beta = lin * lin;
        acc *= (double)(1.0f - beta);
        ac[i] = (float)acc;
      }
    }
    DD_HIP_CHECK(hipMalloc(&ac_dev, sizeof(ac)));
    DD_HIP_CHECK(hipMemcpy(ac_dev, ac, sizeof(ac), hipMemcpyHostToDevice));
    DD_HIP_CHECK(hipMalloc(&train_loss_dev, 4 * sizeof(float)));
  }

  ~Model() {
    DD_TRACE("destroy model %p st_main=%p st_side=%p programs=%zu", (void*)this, (void*)st_main, (void*)st_side,
             programs.size());
    if (ev_out) (void)hipEventSynchronize(ev_out);  // the last forward, also when it ran on a caller's stream
    if (st_main) (void)hipStreamSynchronize(st_main);
    if (st_side) (void)hipStreamSynchronize(st_side);
    drop_graphs();
    if (ev_in) (void)hipEventDestroy(ev_in);
    if (ev_out) (void)hipEventDestroy(ev_out);
    for (auto& e : fj_ev) (void)hipEventDestroy(e);
    if (st_own) release_stream(device, st_own, 0);
    if (st_side) release_stream(device, st_side);
    if (num_flags) (void)hipFree(num_flags);
    if (in_tab) (void)hipFree(in_tab);
    if (tf_mk_layers) (void)hipFree(tf_mk_layers);
    if (ac_dev) (void)hipFree(ac_dev);
    if (train_part) (void)hipFree(train_part);
    if (train_loss_dev) (void)hipFree(train_loss_dev);
    for (auto& kv : bufs) (void)hipFree(kv.second.first);
    for (auto& e : ev_pool) (void)hipEventDestroy(e);
    for (auto& p : pending) {
      (void)hipEventDestroy(p.a);
      (void)hipEventDestroy(p.b);
    }
  }

  // ------------------------------------------------------------------ construction
  void build_trunk(const BlobIndex& bx, const std::string& p, int arch, int in_ch, TrunkW& t) {
    bool bott;
    trunk_channels(arch, t.ch, bott);
    t.stem = prep_conv(bx, ar, p + ".conv1.weight", 64, in_ch, 7, 2, 3, p + ".bn1", "");
    const int nblk[4] = {3, 4, 6, 3};
    const int planes[4] = {64, 128, 256, 512};
    int inpl = 64;
    t.stages.resize(4);
    for (int s = 0; s < 4; ++s) {
      const int stride = s == 0 ? 1 : 2;
      for (int b = 0; b < nblk[s]; ++b) {
        const std::string q = p + ".layer" + std::to_string(s + 1) + "." + std::to_string(b);
        const int st_b = b == 0 ? stride : 1;
        Block blk;
        blk.bottleneck = bott;
        const int outc = bott ? planes[s] * 4 : planes[s];
        if (!bott) {
          blk.c1 = prep_conv(bx, ar, q + ".conv1.weight", planes[s], inpl, 3, st_b, 1, q + ".bn1", "");
          blk.c2 = prep_conv(bx, ar, q + ".conv2.weight", planes[s], planes[s], 3, 1, 1, q + ".bn2", "");
        } else {
          blk.c1 = prep_conv(bx, ar, q + ".conv1.weight", planes[s], inpl, 1, 1, 0, q + ".bn1", "");
          blk.c2 = prep_conv(bx, ar, q + ".conv2.weight", planes[s], planes[s], 3, st_b, 1, q + ".bn2", "");
          blk.c3 = prep_conv(bx, ar, q + ".conv3.weight", outc, planes[s], 1, 1, 0, q + ".bn3", "");
        }
        if (b == 0 && (st_b != 1 || inpl != outc)) {
          blk.has_ds = true;
          blk.ds = prep_conv(bx, ar, q + ".downsample.0.weight", outc, inpl, 1, st_b, 0, q + ".downsample.1", "");
        }
        inpl = outc;
        t.stages[s].push_back(blk);
      }
    }
  }

  Lin prep_qkv(const BlobIndex& bx, const std::string& p, int C) {
    // GPT SelfAttention query/key/value (transfuser_backbone.py:375-377) packed as one [3C][C] GEMM (q|k|v).
    std::vector<float> w((size_t)3 * C * C), b((size_t)3 * C);
    const char* names[3] = {".query", ".key", ".value"};
    for (int i = 0; i < 3; ++i) {
      const HostTensor& tw = bx.get(p + names[i] + ".weight", {C, C});
      const HostTensor& tb = bx.get(p + names[i] + ".bias", {C});
      std::memcpy(w.data() + (size_t)i * C * C, tw.data, sizeof(float) * C * C);
      std::memcpy(b.data() + (size_t)i * C, tb.data, sizeof(float) * C);
    }
    Lin l;
    l.w = ar.add(w);
    l.x3 = prep_split(ar, w.data(), 3 * C, C);
    l.b = ar.add(b);
    l.nout = 3 * C;
    l.nin = C;
    return l;
  }

  void build(const BlobIndex& bx) {
    if (cfg.lidar_channels < 1 || cfg.lidar_channels > 4) throw std::invalid_argument("lidar_channels must be 1..4");
    build_trunk(bx, "_backbone.image_encoder", cfg.image_arch, 3, img);
    build_trunk(bx, "_backbone.lidar_encoder", cfg.lidar_arch, cfg.lidar_channels, lid);
    const int T = 8 * 32 + 8 * 8;
    for (int i = 0; i < 4; ++i) {
      const int C = img.ch[1 + i];
      const std::string p = "_backbone.transformers." + std::to_string(i);
      GptW& g = gpt[i];
      g.C = C;
      g.pos = ar.add(bx.get(p + ".pos_emb", {1, T, C}).data, (size_t)T * C);
      for (int b = 0; b < 2; ++b) {
        const std::string q = p + ".blocks." + std::to_string(b);
        GptBlockW w;
        w.ln1 = prep_ln(bx, ar, q + ".ln1", C);
        w.ln2 = prep_ln(bx, ar, q + ".ln2", C);
        w.qkv = prep_qkv(bx, q + ".attn", C);
        w.proj = prep_linear(bx, ar, q + ".attn.proj", C, C);
        w.mlp0 = prep_linear(bx, ar, q + ".mlp.0", 4 * C, C);
        w.mlp2 = prep_linear(bx, ar, q + ".mlp.2", C, 4 * C);
        g.blocks.push_back(w);
      }
      g.lnf = prep_ln(bx, ar, p + ".ln_f", C);
      l2i[i] = prep_conv(bx, ar, "_backbone.lidar_channel_to_img." + std::to_string(i) + ".weight", C, lid.ch[1 + i], 1,
                         1, 0, "", "_backbone.lidar_channel_to_img." + std::to_string(i) + ".bias");
      i2l[i] = prep_conv(bx, ar, "_backbone.img_channel_to_lidar." + std::to_string(i) + ".weight", lid.ch[1 + i], C, 1,
                         1, 0, "", "_backbone.img_channel_to_lidar." + std::to_string(i) + ".bias");
    }
    const int bc = 64;
    up5 = prep_conv(bx, ar, "_backbone.up_conv5.weight", bc, bc, 3, 1, 1, "", "_backbone.up_conv5.bias");
    up4 = prep_conv(bx, ar, "_backbone.up_conv4.weight", bc, bc, 3, 1, 1, "", "_backbone.up_conv4.bias");
    c5 = prep_conv(bx, ar, "_backbone.c5_conv.weight", bc, lid.ch[4], 1, 1, 0, "", "_backbone.c5_conv.bias");
    const int d = 256;
    kv_emb = ar.add(bx.get("_keyval_embedding.weight", {65, d}).data, (size_t)65 * d);
    q_emb = ar.add(bx.get("_query_embedding.weight", {31, d}).data, (size_t)31 * d);
    bev_down = prep_conv(bx, ar, "_bev_downscale.weight", d, 512, 1, 1, 0, "", "_bev_downscale.bias");
    status = prep_linear(bx, ar, "_status_encoding", d, 8);
    sem0 = prep_conv(bx, ar, "_bev_semantic_head.0.weight", bc, bc, 3, 1, 1, "", "_bev_semantic_head.0.bias");
    sem2 = prep_conv(bx, ar, "_bev_semantic_head.2.weight", 7, bc, 1, 1, 0, "", "_bev_semantic_head.2.bias");
    for (int i = 0; i < 3; ++i) {
      const std::string p = "_tf_decoder.layers." + std::to_string(i);
      TfLayerW w;
      w.sa_in = prep_linear_rows(bx, ar, p + ".self_attn.in_proj_weight", p + ".self_attn.in_proj_bias", 3 * d, d, 0, 3 * d);
      w.sa_out = prep_linear(bx, ar, p + ".self_attn.out_proj", d, d);
      w.ca_q = prep_linear_rows(bx, ar, p + ".multihead_attn.in_proj_weight", p + ".multihead_attn.in_proj_bias", 3 * d,
                                d, 0, d);
      w.ca_kv = prep_linear_rows(bx, ar, p + ".multihead_attn.in_proj_weight", p + ".multihead_attn.in_proj_bias",
                                 3 * d, d, d, 2 * d);
      w.ca_out = prep_linear(bx, ar, p + ".multihead_attn.out_proj", d, d);
      w.l1 = prep_linear(bx, ar, p + ".linear1", 1024, d);
      w.l2 = prep_linear(bx, ar, p + ".linear2", d, 1024);
      w.n1 = prep_ln(bx, ar, p + ".norm1", d);
      w.n2 = prep_ln(bx, ar, p + ".norm2", d);
      w.n3 = prep_ln(bx, ar, p + ".norm3", d);
      tf.push_back(w);
    }
    ag0 = prep_linear(bx, ar, "_agent_head._mlp_states.0", 1024, d);
    ag2 = prep_linear(bx, ar, "_agent_head._mlp_states.2", 5, 1024);
    agl = prep_linear(bx, ar, "_agent_head._mlp_label.0", 1, d);
    const int Q = cfg.num_modes, P = cfg.num_poses;
    const std::string th = "_trajectory_head";
    anchor = ar.add(bx.get(th + ".plan_anchor", {Q, P, 2}).data, (size_t)Q * P * 2);
    pa0 = prep_linear(bx, ar, th + ".plan_anchor_encoder.0", d, 512);
    pa2 = prep_ln(bx, ar, th + ".plan_anchor_encoder.2", d);
    pa3 = prep_linear(bx, ar, th + ".plan_anchor_encoder.3", d, d);
    tm1 = prep_linear(bx, ar, th + ".time_mlp.1", 4 * d, d);
    tm3 = prep_linear(bx, ar, th + ".time_mlp.3", d, 4 * d);
    for (int l = 0; l < 2; ++l) {
      const std::string q = th + ".diff_decoder.layers." + std::to_string(l);
      DiffLayerW w;
      w.attw = prep_linear(bx, ar, q + ".cross_bev_attention.attention_weights", P, d);
      w.outp = prep_linear(bx, ar, q + ".cross_bev_attention.output_proj", d, d);
      w.vproj = prep_conv(bx, ar, q + ".cross_bev_attention.value_proj.0.weight", 256, 256, 3, 1, 1, "",
                          q + ".cross_bev_attention.value_proj.0.bias");
      const std::string ca = q + ".cross_agent_attention", ce = q + ".cross_ego_attention";
      w.ag_q = prep_linear_rows(bx, ar, ca + ".in_proj_weight", ca + ".in_proj_bias", 3 * d, d, 0, d);
      w.ag_kv = prep_linear_rows(bx, ar, ca + ".in_proj_weight", ca + ".in_proj_bias", 3 * d, d, d, 2 * d);
      w.ag_out = prep_linear(bx, ar, ca + ".out_proj", d, d);
      w.eg_v = prep_linear_rows(bx, ar, ce + ".in_proj_weight", ce + ".in_proj_bias", 3 * d, d, 2 * d, d);
      w.eg_out = prep_linear(bx, ar, ce + ".out_proj", d, d);
      w.ffn0 = prep_linear(bx, ar, q + ".ffn.0", 1024, d);
      w.ffn2 = prep_linear(bx, ar, q + ".ffn.2", d, 1024);
      w.n1 = prep_ln(bx, ar, q + ".norm1", d);
      w.n2 = prep_ln(bx, ar, q + ".norm2", d);
      w.n3 = prep_ln(bx, ar, q + ".norm3", d);
      w.film = prep_linear(bx, ar, q + ".time_modulation.scale_shift_mlp.1", 2 * d, 256);
      const std::string t = q + ".task_decoder";
      w.c0 = prep_linear(bx, ar, t + ".plan_cls_branch.0", d, d);
      w.c2 = prep_ln(bx, ar, t + ".plan_cls_branch.2", d);
      w.c3 = prep_linear(bx, ar, t + ".plan_cls_branch.3", d, d);
      w.c5 = prep_ln(bx, ar, t + ".plan_cls_branch.5", d);
      w.c6 = prep_linear(bx, ar, t + ".plan_cls_branch.6", 1, d);
      w.r0 = prep_linear(bx, ar, t + ".plan_reg_branch.0", d, d);
      w.r2 = prep_linear(bx, ar, t + ".plan_reg_branch.2", d, d);
      w.r4 = prep_linear(bx, ar, t + ".plan_reg_branch.4", P * 3, d);
      dl.push_back(w);
    }
    bevproj = prep_linear(bx, ar, "bev_proj.0", d, 320);
    bevproj_ln = prep_ln(bx, ar, "bev_proj.2", d);
    if (bevproj_supported(d, 64, cfg.lidar_h / 4, cfg.lidar_w / 4, 8, 8)) {
      Lin p3 = bevproj;  // the p3 columns 256..319 as a [256][64] Linear for the image
      std::vector<float> w((size_t)d * 64);
      for (int r = 0; r < d; ++r)
        for (int k = 0; k < 64; ++k) w[(size_t)r * 64 + k] = ar.host(bevproj.w)[(size_t)r * 320 + 256 + k];
      p3.w = ar.add(w);
      p3.nin = 64;
      m_bevp3 = pack_mk(p3);
    }
    // tf-decoder megakernel images (tfdec_mk.hip)
    tf_mk_ready = tfdec_mk_supported(31, 65, d, 8, 1024, (int)tf.size()) && dl.size() == 2;
    if (tf_mk_ready) {
      for (int i = 0; i < 3; ++i) {
        m_tf[i].sa_in = pack_mk(tf[i].sa_in);
        m_tf[i].sa_out = pack_mk(tf[i].sa_out);
        m_tf[i].ca_q = pack_mk(tf[i].ca_q);
        m_tf[i].ca_out = pack_mk(tf[i].ca_out);
        m_tf[i].l1 = pack_mk(tf[i].l1);
        m_tf[i].l2 = pack_mk(tf[i].l2);
      }
      for (int l = 0; l < 2; ++l) {
        m_agkv[l] = pack_mk(dl[l].ag_kv);
        m_egv[l] = pack_mk(dl[l].eg_v);
        m_egout[l] = pack_mk(dl[l].eg_out);
      }
      std::vector<float> w, bsum;
      for (int i = 0; i < 3; ++i) {
        const Lin& c = tf[i].ca_kv;
        w.insert(w.end(), ar.host(c.w), ar.host(c.w) + (size_t)c.nout * c.nin);
        bsum.insert(bsum.end(), ar.host(c.b), ar.host(c.b) + c.nout);
      }
      tf_cakv.nout = 3 * 2 * d;
      tf_cakv.nin = d;
      tf_cakv.w = ar.add(w);
      tf_cakv.x3 = prep_split(ar, w.data(), tf_cakv.nout, d);
      tf_cakv.b = ar.add(bsum);
    }
    // decoder megakernel images (the reference configuration only)
    mk_ready = decoder_mk_supported(Q, P, d, 30, cfg.lidar_h / 4, cfg.lidar_w / 4, 1024);
    if (mk_ready) {
      mk_w_begin = ar.add_zero(0);
      for (DiffLayerW& w : dl) {
        w.m_outp = pack_mk(w.outp);
        w.m_ag_q = pack_mk(w.ag_q);
        w.m_ag_out = pack_mk(w.ag_out);
        w.m_ffn0 = pack_mk(w.ffn0);
        w.m_ffn2 = pack_mk(w.ffn2);
        w.m_c0 = pack_mk(w.c0);
        w.m_c3 = pack_mk(w.c3);
        w.m_r0 = pack_mk(w.r0);
        w.m_r2 = pack_mk(w.r2);
      }
      m_pa0 = pack_mk(pa0);
      m_pa3 = pack_mk(pa3);
      std::vector<float> t(16);
      for (int j = 0; j < 16; ++j) t[j] = (float)std::pow(10000.0, (double)j / 16.0);  // as decoder.hip
      dim_t_off = ar.add(t);
      mk_w_end = ar.add_zero(0);
    }
  }

  // f16x3 image of a Linear in MFMA-fragment order (decoder_mk.h MkLin): the split of prep_split (same
  // per-output power-of-two scale, hi = f16(w s), lo = f16(w s - hi)), block (nt, ks) = 64 lanes x (8 hi,
  // 8 lo) halfs, lane = col % 32 + 32 ((k % 16) / 8)
  MkLinOff pack_mk(const Lin& L) {
    const std::vector<float> w(ar.host(L.w), ar.host(L.w) + (size_t)L.nout * L.nin);
    std::vector<_Float16> pk;
    std::vector<float> sinv;
    pack_mk_weights(w.data(), L.nout, L.nin, pk, sinv);
    MkLinOff m;
    m.w = ar.add(reinterpret_cast<const float*>(pk.data()), pk.size() / 2);
    m.s = ar.add(sinv);
    m.b = L.b;
    m.nks = L.nin / 16;
    return m;
  }
  MkLin mk(const MkLinOff& o) const {
    MkLin m;
    m.w = reinterpret_cast<const uint4*>(W(o.w));
    m.s = W(o.s);
    m.b = W(o.b);
    m.nks = o.nks;
    return m;
  }
  MkLayer mk_layer(int l) const {
    const DiffLayerW& w = dl[l];
    MkLayer L;
    L.outp = mk(w.m_outp);
    L.ag_q = mk(w.m_ag_q);
    L.ag_out = mk(w.m_ag_out);
    L.ffn0 = mk(w.m_ffn0);
    L.ffn2 = mk(w.m_ffn2);
    L.c0 = mk(w.m_c0);
    L.c3 = mk(w.m_c3);
    L.r0 = mk(w.m_r0);
    L.r2 = mk(w.m_r2);
    L.attw_w = W(w.attw.w);
    L.attw_b = W(w.attw.b);
    L.c6_w = W(w.c6.w);
    L.c6_b = W(w.c6.b);
    L.r4_w = W(w.r4.w);
    L.r4_b = W(w.r4.b);
    L.n1g = W(w.n1.g);
    L.n1b = W(w.n1.b);
    L.n2g = W(w.n2.g);
    L.n2b = W(w.n2.b);
    L.n3g = W(w.n3.g);
    L.n3b = W(w.n3.b);
    L.c2g = W(w.c2.g);
    L.c2b = W(w.c2.b);
    L.c5g = W(w.c5.g);
    L.c5b = W(w.c5.b);
    return L;
  }

  // value_proj (3x3 conv 256 -> 256 + ReLU, blocks.py:68-76,114) of layer l evaluated only at the map
  // pixels the (step, layer)'s taps read: conv_x3 over the deduplicated row list `rows`
  // counts (nullable): the scenes' live-row counts - the launch then runs the scenes' rows compacted (full
  // 128-row tiles; without counts one tile run per scene). Timed under its own class "value_proj";
  // its FLOPs count every row slot (2 x slots x 256 x 2304; bench.py derives the live-row rate from the counts).
  // busy_cus: CUs a kernel on the other branch holds meanwhile (the tf-decoder megakernel: one per scene)
  void gathered_value(int l, const int* rows, const int* counts, float* vrows, const float* cross, int B, int HB,
                      int WB, int MR, int busy_cus = 0) {
    const int d = 256;
    ConvArgs a = conv_args(dl[l].vproj, cross, (int64_t)HB * WB * d, (int64_t)WB * d, d, B, HB, WB, vrows,
                           (int64_t)MR * d, d, 0, true, nullptr, 0, 0, 0);
    a.Nimg = 1;
    a.Ho = MR;
    a.Wo = 1;
    a.rowmap = rows;
    a.rowmap_nimg = B;
    if (counts) {
      a.rowcount = counts;
      a.rowcap = MR / B;
    }
    const double fl = 2.0 * MR * (double)d * 9 * dl[l].vproj.cin_real;
    const Conv& vc = dl[l].vproj;
    if (value_splitk && counts && vproj_supported(vc.cin, vc.cout, HB, WB) && a.wh && a.prec == 0) {
      // value_proj.hip: compacted rows in 256-row tiles, two 128-channel halves each
      VprojArgs v;
      v.map = cross;
      v.wh = a.wh;
      v.wl = a.wl;
      v.wsinv = a.wsinv;
      v.ldh = (int)a.ldh;
      v.bias = a.bias;
      v.rows = rows;
      v.counts = counts;
      v.B = B;
      v.cap = MR / B;
      v.out = vrows;
      v.flags = num_flags;
      const int max_wgs = std::max(64, num_cus() - busy_cus);
      v.union_stage = vproj_union ? 1 : 0;
      v.umax = vproj_umax;
      if (v.union_stage) {
        const size_t t8 = (vproj_tiles(B, MR / B) + 7) / 8 * 8;
        v.fb = reinterpret_cast<unsigned*>(buf_zeroed("vproj_fb", 2 * t8));
        // K split over channel groups while the (tile, half) units leave CUs idle: ~330 live rows per scene
        // (B = 64: 166 units, no split; B = 1: 4 units x 8 splits). At most 8: the last split to arrive reads the
        // others' partials (S x 128 KB per unit), which at 16 costs more than the K loop it saves
        const int units = 2 * (int)((B * 330 + 255) / 256);
        int us = 1;
        while (us < 8 && units * us * 2 <= max_wgs) us *= 2;
        if (vproj_usplit_env > 0) us = vproj_usplit_env;
        v.usplit = us;
        if (us > 1) {
          v.ucnt = reinterpret_cast<unsigned*>(buf_zeroed("vproj_ucnt", 2 * t8));
          v.part = buf("vproj_upart", (size_t)us * MR * d);
        }
      }
      launch("value_proj", fl, [&] { launch_vproj(v, st); });
      return;
    }
    struct ClassScope {
      const char*& c;
      ClassScope(const char*& cc, const char* v) : c(cc) { c = v; }
      ~ClassScope() { c = nullptr; }
    } cls(force_class, "value_proj");
    launch("conv_x3", fl, [&] { launch_conv_gemm(a, st); }, &a);
  }

  // TrajectoryHead.forward_test (:578-641) as 1 + 2 x steps x 2 launches: the DDIM start + first taps, then
  // per (step, layer) the gathered value_proj conv and the decoder megakernel (decoder_mk.hip)
  void traj_head_mk(int B, int steps, const float* cross, float* const akv[2], float* const egos[2],
                    bool& tf_pending, const float* noise) {
    const int d = 256, Q = cfg.num_modes, P = cfg.num_poses, R = B * Q;
    const int HB = cfg.lidar_h / 4, WB = cfg.lidar_w / 4, MR = R * P * 4;
    const bool vanilla = schedule == DD_SCHED_VANILLA;
    const std::vector<int> roll = denoise_timesteps(steps);
    const int ratio = vanilla ? 1000 / steps : 1;
    auto sfx = [](int s, int l) { return "_s" + std::to_string(s) + "l" + std::to_string(l); };
    auto rows_of = [&](int s, int l) { return reinterpret_cast<int*>(buf("value_taps" + sfx(s, l), (size_t)MR)); };
    auto slots_of = [&](int s, int l) { return reinterpret_cast<int*>(buf("value_slots" + sfx(s, l), (size_t)MR)); };
    auto counts_of = [&](int s, int l) { return reinterpret_cast<int*>(buf("value_cnt" + sfx(s, l), (size_t)B)); };
    float* imgx = buf("ddim_img", (size_t)R * P * 2);
    float* tfe = buf("traj_feature", (size_t)R * d);
    float* pts = buf("pts", (size_t)R * P * 2);
    float* pts2 = buf("pts_next", (size_t)R * P * 2);
    float* traj = buf("trajectory", (size_t)B * P * 3);
    int* idx = reinterpret_cast<int*>(buf("mode_idx", B));
    {
      // truncated: add_noise(norm_odo(anchor), noise, t = trunc_timestep) (:593-597);
      // vanilla (C5 ablation): x_T = noise (sa = 0, s1a = 1 keep it bit-exact)
      const float a8 = ac[cfg.trunc_timestep];
      MkInitArgs ia;
      ia.anchor = W(anchor);
      ia.noise = noise;
      ia.imgx = imgx;
      ia.rows = rows_of(0, 0);
      ia.slots = slots_of(0, 0);
      ia.counts = counts_of(0, 0);
      ia.sa = vanilla ? 0.0f : std::sqrt(a8);
      ia.s1a = vanilla ? 1.0f : std::sqrt(1.0f - a8);
      if (train) {  // forward_train: per-scene timesteps (train_time_film)
        ia.sa_b = bufs.at("train_sa").first;
        ia.s1a_b = bufs.at("train_s1a").first;
      }
      ia.B = B;
      launch("decoder", 0, [&] { launch_decoder_mk_init(ia, st); });
      // the packed decoder weights (~8.6 MB) into the MALL before the first layer streams them from HBM
      launch("misc", 0, [&] {
        launch_mk_prefetch(W(mk_w_begin), (mk_w_end - mk_w_begin) * sizeof(float), st);
      });
    }
    const MkLayer layers[2] = {mk_layer(0), mk_layer(1)};
    MkAnchor anc;
    anc.pa0 = mk(m_pa0);
    anc.pa3 = mk(m_pa3);
    anc.pa2g = W(pa2.g);
    anc.pa2b = W(pa2.b);
    float* reg_last = nullptr;
    float* cls_last = nullptr;
    for (int si = 0; si < steps; ++si) {
      for (int l = 0; l < 2; ++l) {
        const std::string sf = sfx(si, l);
        float* vrows = buf("value_rows" + sf, (size_t)MR * d);
        gathered_value(l, rows_of(si, l), counts_of(si, l), vrows, cross, B, HB, WB, MR, tf_pending ? B : 0);
        if (tf_pending) {
          join();  // tf decoder: agent K / V and ego rows of both layers
          tf_pending = false;
        }
        MkArgs m;
        m.L = layers[l];
        m.A = anc;
        m.layer = l;
        m.B = B;
        m.imgx = imgx;
        m.tfe = tfe;
        m.pts = l == 0 ? pts : pts2;
        m.pts_next = l == 0 ? pts2 : nullptr;
        m.vrows = vrows;
        m.slots = slots_of(si, l);
        m.akv = akv[l];
        m.ego = egos[l];
        if (train) {
          m.film = bufs.at("train_film_l" + std::to_string(l)).first;
          m.film_stride = 2 * d;
        } else {
          m.film = buf("film_s" + std::to_string(si) + "l" + std::to_string(l), 2 * d);
        }
        m.gs_out = buf("gs" + sf, (size_t)R * d);
        m.reg_out = buf("reg" + sf, (size_t)R * P * 3);
        m.cls_out = buf("cls" + sf, R);
        if (l == 0) {
          m.next_rows = rows_of(si, 1);
          m.next_slots = slots_of(si, 1);
          m.next_counts = counts_of(si, 1);
        } else if (si + 1 < steps) {
          m.next_rows = rows_of(si + 1, 0);
          m.next_slots = slots_of(si + 1, 0);
          m.next_counts = counts_of(si + 1, 0);
          const int k = roll[si];
          const float a_t = ac[k], a_p = (k - ratio >= 0) ? ac[k - ratio] : 1.0f;
          m.ddim = 1;
          m.sa_t = std::sqrt(a_t);
          m.sb_t = std::sqrt(1.0f - a_t);
          m.sa_p = std::sqrt(a_p);
          m.sdir = std::sqrt(1.0f - a_p);
        } else {
          m.traj = traj;
          m.mode_idx = idx;
        }
        m.flags = num_flags;
        m.dim_t = W(dim_t_off);
        // query groups: 4 workgroups of 5 queries per scene at small batches (stamps: one per scene). Every group
        // streams all of the layer's weight images, so the groups cost L2 bandwidth: at B = 64 four groups (256
        // workgroups) took 0.50 against 0.40 ms per forward, at B = 1 they save 10 %. Up to 64 workgroups per launch.
        m.groups = mk_stamps ? 1 : (mk_groups_env ? mk_groups_env : (B * 4 <= 64 ? 4 : (B * 2 <= 64 ? 2 : 1)));
        if (m.groups > 1) {
          m.scene_cnt = reinterpret_cast<unsigned*>(buf_zeroed("mk_scene_cnt", (size_t)B));
          m.next_pts = buf("mk_next_pts", (size_t)R * P * 2);
          m.cls_x = buf("mk_cls_x", (size_t)B * 32);
        }
        if (mk_stamps) m.stamps = reinterpret_cast<unsigned long long*>(buf("mk_stamps" + sf, (size_t)B * 80));
        // algorithmic FLOPs of the launch: the 256-wide Linears (+ the anchor encoder at layer 0) and the
        // fp32 heads, 2 x rows x sum(K x N)
        double kn = 7.0 * d * d + 2.0 * d * 1024 + (double)d * (P + 1 + 3 * P);
        if (l == 0) kn += 512.0 * d + (double)d * d;
        launch("decoder", 2.0 * R * kn, [&] { launch_decoder_mk(m, st); });
        reg_last = m.reg_out;
        cls_last = m.cls_out;
      }
    }
    join();  // the heads branch on the side stream
    alias("poses_reg", reg_last);
    alias("poses_cls", cls_last);
    train_loss_partials(B);
  }

  // ------------------------------------------------------------------ runtime helpers
  const float* W(size_t off) const { return ar.ptr(off); }

  int num_cus() {
    if (!cu_count) {
      int dev = 0;
      DD_HIP_CHECK(hipGetDevice(&dev));
      DD_HIP_CHECK(hipDeviceGetAttribute(&cu_count, hipDeviceAttributeMultiprocessorCount, dev));
    }
    return cu_count;
  }
  int cu_count = 0;

  // a workspace buffer whose words start zeroed when it is (re)allocated (allocation only happens in eager,
  // uncaptured forwards; kernels that use such words leave them zeroed). The memset is ordered on the handle's
  // stream: that stream is non-blocking, so a plain hipMemset (legacy stream) could land after the first kernels.
  float* buf_zeroed(const std::string& name, size_t n) {
    const uint64_t g = generation;
    float* p = buf(name, n);
    if (generation != g) DD_HIP_CHECK(hipMemsetAsync(p, 0, std::max<size_t>(n, 4) * sizeof(float), st));
    return p;
  }

  float* buf(const std::string& name, size_t n) {
    auto it = bufs.find(name);
    if (it != bufs.end() && it->second.second >= n) return it->second.first;
    if (it != bufs.end()) {
      DD_HIP_CHECK(hipFree(it->second.first));
      bufs.erase(it);
    }
    float* p = nullptr;
    DD_HIP_CHECK(hipMalloc(&p, std::max<size_t>(n, 4) * sizeof(float)));
    bufs[name] = {p, n};
    ++generation;
    return p;
  }

  // ---- two-stream fork / join. Independent branches of the forward (the LiDAR trunk stage beside
  // the image one, the tf decoder beside the FPN / bev_proj / value_proj chain, the optional heads
  // beside the trajectory head) are issued on the side stream between fork() and join(); under
  // stream capture this becomes a graph with parallel branches, so a branch's small launches fill
  // CUs the other leaves idle. side(f) runs f with every launch going to the side stream.
  hipEvent_t fj_event() {
    if (fj_next == fj_ev.size()) {
      hipEvent_t e;
      DD_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      fj_ev.push_back(e);
    }
    return fj_ev[fj_next++];
  }
  // profiled runs stay on one stream: per-launch event timing needs launches that do not overlap
  bool sides() const { return use_side && !profiling; }

  // Segmented capture (capture_program): every launch goes to st_cap under stream capture; fork / join / side close
  // the open segment (a single-stream graph of the launches since the last boundary, tagged with its logical stream),
  // append the event operations and open the next segment.
  bool seg_cap = false;
  int seg_s = 0;
  hipStream_t st_cap = nullptr;
  Program* seg_prog = nullptr;
  void seg_begin(int s) {
    seg_s = s;
    DD_HIP_CHECK(hipStreamBeginCapture(st_cap, hipStreamCaptureModeThreadLocal));
  }
  void seg_end() {
    hipGraph_t g = nullptr;
    DD_HIP_CHECK(hipStreamEndCapture(st_cap, &g));
    size_t n = 0, roots = 0;
    hipError_t e = hipGraphGetNodes(g, nullptr, &n);
    if (e == hipSuccess) e = hipGraphGetRootNodes(g, nullptr, &roots);
    if (e == hipSuccess && n > 0) {
      if (roots > 1) ++seg_prog->branched;
      std::vector<hipGraphNode_t> nodes(n);
      e = hipGraphGetNodes(g, nodes.data(), &n);
      for (size_t i = 0; e == hipSuccess && i < n; ++i) {
        hipGraphNodeType ty;
        e = hipGraphNodeGetType(nodes[i], &ty);
        if (e == hipSuccess) ++(ty == hipGraphNodeTypeKernel ? seg_prog->kernel_nodes : seg_prog->other_nodes);
      }
    }
    if (e == hipSuccess && n > 0) {
      hipGraphExec_t ex = nullptr;
      e = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
      if (e == hipSuccess) {
        seg_prog->ops.push_back({0, seg_s, ex, -1});
        ++seg_prog->segments;
      }
    }
    (void)hipGraphDestroy(g);
    DD_HIP_CHECK(e);
  }
  void seg_event(int from, int to) {
    const int e = (int)fj_next;
    (void)fj_event();
    seg_prog->ops.push_back({1, from, nullptr, e});
    seg_prog->ops.push_back({2, to, nullptr, e});
  }
  void fork() {
    if (!sides()) return;
    if (seg_cap) {
      seg_end();
      seg_event(0, 1);
      seg_begin(0);
      return;
    }
    hipEvent_t e = fj_event();
    DD_HIP_CHECK(hipEventRecord(e, st_main));
    DD_HIP_CHECK(hipStreamWaitEvent(st_side, e, 0));
  }
  void join() {
    if (!sides()) return;
    if (seg_cap) {
      seg_end();
      seg_event(1, 0);
      seg_begin(0);
      return;
    }
    hipEvent_t e = fj_event();
    DD_HIP_CHECK(hipEventRecord(e, st_side));
    DD_HIP_CHECK(hipStreamWaitEvent(st_main, e, 0));
  }
  bool in_side = false;  // inside side(f): per-stream scratch (conv_x3's K-split partials) takes the side's copy
  template <class F>
  void side(F&& f) {
    struct SideFlag {
      bool& b;
      explicit SideFlag(bool& x) : b(x) { b = true; }
      ~SideFlag() { b = false; }
    } flag(in_side);
    if (seg_cap) {  // launches stay on st_cap; the segment is tagged with the side stream
      seg_end();
      seg_begin(1);
      f();
      seg_end();
      seg_begin(0);
      return;
    }
    st = sides() ? st_side : st_main;
    try {
      f();
    } catch (...) {
      st = st_main;
      throw;
    }
    st = st_main;
  }

  // Capture the forward into p: one single-stream graph, or (two streams) the segmented program above.
  void capture_program(int B, int steps, bool heads, Program& p) {
    seg_prog = &p;
    st_cap = st;
    seg_cap = sides();
    try {
      seg_begin(0);
      forward_body(B, steps, heads);
      seg_end();
    } catch (...) {
      hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
      if (hipStreamIsCapturing(st_cap, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) {
        hipGraph_t dummy = nullptr;
        if (hipStreamEndCapture(st_cap, &dummy) == hipSuccess && dummy) (void)hipGraphDestroy(dummy);
      }
      (void)hipGetLastError();
      seg_cap = false;
      seg_prog = nullptr;
      destroy_program(p);
      throw;
    }
    seg_cap = false;
    seg_prog = nullptr;
  }
  void run_program(const Program& p) {
    const hipStream_t ss[2] = {st_main, st_side};
    for (const SegOp& op : p.ops) {
      if (op.kind == 0)
        DD_HIP_CHECK(hipGraphLaunch(op.ex, ss[op.s]));
      else if (op.kind == 1)
        DD_HIP_CHECK(hipEventRecord(fj_ev[op.ev], ss[op.s]));
      else
        DD_HIP_CHECK(hipStreamWaitEvent(ss[op.s], fj_ev[op.ev], 0));
    }
  }

  template <class F>
  void launch(const char* name, double flops, F&& f, const ConvArgs* shape = nullptr, double bytes = -1.0) {
    if (!profiling) {
      f();
      return;
    }
    hipEvent_t a, b;
    if (ev_pool.size() >= 2) {
      a = ev_pool.back();
      ev_pool.pop_back();
      b = ev_pool.back();
      ev_pool.pop_back();
    } else {
      DD_HIP_CHECK(hipEventCreate(&a));
      DD_HIP_CHECK(hipEventCreate(&b));
    }
    DD_HIP_CHECK(hipEventRecord(a, st));
    f();
    DD_HIP_CHECK(hipEventRecord(b, st));
    // conv / GEMM launches are attributed to the kernel the dispatcher actually chose (or a forced class)
    if (force_class) name = force_class;
    else if (shape) name = last_conv_kernel();
    std::string detail;
    if (shape) {
      const ConvArgs& c = *shape;
      detail = "M=" + std::to_string((int64_t)c.Nimg * c.Ho * c.Wo) + " N=" + std::to_string(c.Cout) +
               " K=" + std::to_string(c.KH * c.KW * c.Cin) + " k=" + std::to_string(c.KH) + " s=" +
               std::to_string(c.stride) + " z=" + std::to_string(c.batch) + " HW=" + std::to_string(c.H) + "x" +
               std::to_string(c.W);
    }
    pending.push_back({name, flops, bytes >= 0.0 ? bytes : (shape ? conv_algo_bytes(*shape) : 0.0), a, b, detail});
  }

  void collect() {
    const char* log_path = getenv("DDMI_LAUNCH_LOG");
    FILE* log = log_path ? fopen(log_path, "a") : nullptr;
    for (auto& p : pending) {
      DD_HIP_CHECK(hipEventSynchronize(p.b));
      float ms = 0;
      DD_HIP_CHECK(hipEventElapsedTime(&ms, p.a, p.b));
      KStat& s = stats[p.name];
      s.ms += ms;
      s.n += 1;
      s.flops += p.flops;
      s.bytes += p.bytes;
      if (log) fprintf(log, "%s\t%s\t%.6g\t%.6f\t%.6g\n", p.name.c_str(), p.detail.c_str(), p.flops, ms, p.bytes);
      ev_pool.push_back(p.a);
      ev_pool.push_back(p.b);
    }
    pending.clear();
    if (log) fclose(log);
  }

  // route a conv / linear to the f16x3 split-MFMA kernel when that mode is on
  void use_split(ConvArgs& a, const SplitW& x) {
    if (gemm_mode == DD_GEMM_FP32 || x.hi == kNone) return;
    a.prec = gemm_mode == DD_GEMM_BF16 ? 1 : 0;
    a.wh = reinterpret_cast<const uint16_t*>(W(a.prec ? x.b16 : x.hi));
    a.wl = reinterpret_cast<const uint16_t*>(W(x.lo));
    a.wsinv = W(x.sinv);
    a.ldh = x.ldh;
    a.flags = num_flags;
  }

  // GPT token pooling fused into the next conv's epilogue (conv_x6; see ConvArgs::pool_out): set before
  // the conv, consumed by it; pool_done tells whether that conv wrote the tokens (otherwise the caller runs
  // launch_avgpool, e.g. in the fp32 mode or when the conv routes elsewhere)
  struct PoolSpec {
    float* out = nullptr;
    int64_t sn = 0, sh = 0, sw = 0;
    const float* add = nullptr;
    int64_t add_sh = 0, add_sw = 0;
    int oh = 0, ow = 0;  // pooled grid
  };
  PoolSpec pool_next;
  int pool_next_p = 0;
  bool pool_done = false;

  // conv on strided NHWC views
  ConvArgs conv_args(const Conv& c, const float* in, int64_t isn, int64_t ish, int64_t isw, int N, int H, int Wd,
                     float* out, int64_t osn, int64_t osh, int64_t osw, bool relu, const float* res, int64_t rsn,
                     int64_t rsh, int64_t rsw) {
    ConvArgs a;
    a.in = in;
    a.in_sn = isn;
    a.in_sh = ish;
    a.in_sw = isw;
    a.H = H;
    a.W = Wd;
    a.Cin = c.cin;
    a.wgt = W(c.w);
    a.ldb = (int64_t)c.k * c.k * c.cin;
    a.bias = W(c.b);
    a.res = res;
    a.res_sn = rsn;
    a.res_sh = rsh;
    a.res_sw = rsw;
    a.out = out;
    a.out_sn = osn;
    a.out_sh = osh;
    a.out_sw = osw;
    a.Nimg = N;
    a.Ho = (H + 2 * c.pad - c.k) / c.stride + 1;
    a.Wo = (Wd + 2 * c.pad - c.k) / c.stride + 1;
    a.Cout = c.cout;
    a.KH = a.KW = c.k;
    a.stride = c.stride;
    a.pad = c.pad;
    a.relu = relu;
    use_split(a, c.x3);
    if (pool_next_p > 0) {
      a.pool_out = pool_next.out;
      a.pool_p = pool_next_p;
      a.pool_sn = pool_next.sn;
      a.pool_sh = pool_next.sh;
      a.pool_sw = pool_next.sw;
      a.pool_add = pool_next.add;
      a.pool_add_sh = pool_next.add_sh;
      a.pool_add_sw = pool_next.add_sw;
      pool_next_p = 0;
    }
    return a;
  }
  void conv(const Conv& c, const float* in, int64_t isn, int64_t ish, int64_t isw, int N, int H, int Wd, float* out,
            int64_t osn, int64_t osh, int64_t osw, bool relu, const float* res = nullptr, int64_t rsn = 0,
            int64_t rsh = 0, int64_t rsw = 0) {
    ConvArgs a = conv_args(c, in, isn, ish, isw, N, H, Wd, out, osn, osh, osw, relu, res, rsn, rsh, rsw);
    const double fl = 2.0 * N * a.Ho * a.Wo * (double)c.cout * c.k * c.k * c.cin_real;
    // small outputs (batch-1-sized maps): K-split scratch for conv_x3, one per stream of the forward
    const int64_t mo = (int64_t)N * a.Ho * a.Wo * c.cout;
    if (a.wh && a.prec == 0 && mo <= (int64_t(1) << 20)) {
      a.split_cap = 8 * mo;
      a.split_part = buf(in_side ? "x3_split_side" : "x3_split_main", (size_t)a.split_cap);
    }
    launch(a.wh ? "conv_x3" : "conv_gemm", fl, [&] { launch_conv_gemm(a, st); }, &a);
    pool_done = a.pool_out && last_conv_pooled();
  }
  // timm stem conv1 / bn1 / act1 + maxpool 3x3/2: one fused kernel (stem_pool.hip) in f16x3 mode,
  // otherwise the conv into `stem` and the pool from it
  // in_idx / in_c: with the NCHW stem (use_nchw_stem) the kernel reads the caller's NCHW input of in_c channels
  // through the device input table entry in_idx instead of the NHWC4 copy (which is then never made)
  void stem_and_pool(const Conv& c, const float* in4, int N, int H, int Wd, float* stem, float* pool, int hp, int wp,
                     int in_idx, int in_c) {
    const int hs = (H + 2 * c.pad - c.k) / c.stride + 1, ws = (Wd + 2 * c.pad - c.k) / c.stride + 1;
    ConvArgs a = conv_args(c, in4, (int64_t)H * Wd * c.cin, (int64_t)Wd * c.cin, c.cin, N, H, Wd, stem,
                           (int64_t)hs * ws * c.cout, (int64_t)ws * c.cout, c.cout, true, nullptr, 0, 0, 0);
    bool done = false;
    const double fl = 2.0 * N * hs * ws * (double)c.cout * c.k * c.k * c.cin_real;
    const bool nchw = use_nchw_stem();
    launch("stem_pool", fl, [&] {
      done = launch_stem_pool(a, pool, hp, wp, st, nchw ? in_tab + in_idx : nullptr, nchw ? in_c : 0);
    });
    if (done) return;
    if (nchw) throw std::runtime_error("stem: the NCHW-input fused stem refused this shape (DDMI_STEM_NCHW=0 avoids it)");
    conv_c(c, in4, N, H, Wd, stem, true);
    launch("pool", 0, [&] { launch_maxpool3x3s2(stem, pool, N, hs, ws, c.cout, hp, wp, st); });
  }
  // contiguous NHWC conv; returns output spatial size
  void conv_c(const Conv& c, const float* in, int N, int H, int Wd, float* out, bool relu, const float* res = nullptr) {
    const int Ho = (H + 2 * c.pad - c.k) / c.stride + 1, Wo = (Wd + 2 * c.pad - c.k) / c.stride + 1;
    conv(c, in, (int64_t)H * Wd * c.cin, (int64_t)Wd * c.cin, c.cin, N, H, Wd, out, (int64_t)Ho * Wo * c.cout,
         (int64_t)Wo * c.cout, c.cout, relu, res, (int64_t)Ho * Wo * c.cout, (int64_t)Wo * c.cout, c.cout);
  }

  // C[M][N] = A[M][K] W^T (+bias) (+res) (relu); rows grouped: row m -> (m / G, m % G) with
  // A offset (m/G)*a_gs + (m%G)*a_rs (dense when G == M).
  void gemm(const Lin& L, const float* A, int64_t lda, int M, float* C, int64_t ldc, bool relu = false,
            const float* res = nullptr, int64_t ldr = 0) {
    gemm_g(L, A, (int64_t)M * lda, lda, 1, M, C, (int64_t)M * ldc, ldc, relu, res, (int64_t)M * ldr, ldr);
  }
  void gemm_g(const Lin& L, const float* A, int64_t a_gs, int64_t a_rs, int G, int R, float* C, int64_t c_gs,
              int64_t c_rs, bool relu = false, const float* res = nullptr, int64_t r_gs = 0, int64_t r_rs = 0) {
    ConvArgs a;
    a.in = A;
    a.in_sn = a_gs;
    a.in_sh = a_rs;
    a.in_sw = 0;
    a.H = R;
    a.W = 1;
    a.Cin = L.nin;
    a.wgt = W(L.w);
    a.ldb = L.nin;
    a.bias = W(L.b);
    a.res = res;
    a.res_sn = r_gs;
    a.res_sh = r_rs;
    a.out = C;
    a.out_sn = c_gs;
    a.out_sh = c_rs;
    a.out_sw = 0;
    a.Nimg = G;
    a.Ho = R;
    a.Wo = 1;
    a.Cout = L.nout;
    a.relu = relu;
    use_split(a, L.x3);
    const double fl = 2.0 * G * R * (double)L.nout * L.nin;
    launch(a.wh ? "conv_x3" : "conv_gemm", fl, [&] { launch_conv_gemm(a, st); }, &a);
  }

  // C = A W^T + bias + res, and (when the GEMM can fuse it: conv_x3's quad epilogue with one N tile per row, Cout 64
  // or 128) Y = LayerNorm(C) in the same pass, bit-identical to ln(); returns whether Y was written (otherwise the
  // caller runs ln()). DDMI_LN_FOLD=0: never fused.
  bool gemm_ln(const Lin& L, const float* A, int64_t lda, int M, float* C, int64_t ldc, const float* res, int64_t ldr,
               const LNp& p, float* Y) {
    ConvArgs a;
    a.in = A;
    a.in_sn = (int64_t)M * lda;
    a.in_sh = lda;
    a.in_sw = 0;
    a.H = M;
    a.W = 1;
    a.Cin = L.nin;
    a.wgt = W(L.w);
    a.ldb = L.nin;
    a.bias = W(L.b);
    a.res = res;
    a.res_sn = (int64_t)M * ldr;
    a.res_sh = ldr;
    a.out = C;
    a.out_sn = (int64_t)M * ldc;
    a.out_sh = ldc;
    a.out_sw = 0;
    a.Nimg = 1;
    a.Ho = M;
    a.Wo = 1;
    a.Cout = L.nout;
    use_split(a, L.x3);
    if (ln_fold && p.c == L.nout) {
      a.ln_out = Y;
      a.ln_g = W(p.g);
      a.ln_b = W(p.b);
    }
    const double fl = 2.0 * M * (double)L.nout * L.nin;
    bool fused = false;
    launch(a.wh ? "conv_x3" : "conv_gemm", fl, [&] {
      launch_conv_gemm(a, st);
      fused = a.ln_out && last_conv_ln();
    }, &a);
    return fused;
  }

  // C = A[:, 0:kn] W[:, k0:k0+kn]^T (+bias when with_bias) (+res) (relu): a K-slice of a Linear (the weight
  // rows keep their full stride; 16-B aligned slices only)
  void gemm_slice(const Lin& L, int k0, int kn, bool with_bias, const float* A, int64_t a_gs, int64_t a_rs, int G,
                  int R, float* C, int64_t c_gs, int64_t c_rs, bool relu, const float* res, int64_t r_gs,
                  int64_t r_rs) {
    if (k0 % 8 || kn % 8 || k0 + kn > L.nin) throw std::runtime_error("gemm_slice: bad K slice");
    ConvArgs a;
    a.in = A;
    a.in_sn = a_gs;
    a.in_sh = a_rs;
    a.in_sw = 0;
    a.H = R;
    a.W = 1;
    a.Cin = kn;
    a.wgt = W(L.w) + k0;
    a.ldb = L.nin;
    a.bias = with_bias ? W(L.b) : nullptr;
    a.res = res;
    a.res_sn = r_gs;
    a.res_sh = r_rs;
    a.out = C;
    a.out_sn = c_gs;
    a.out_sh = c_rs;
    a.out_sw = 0;
    a.Nimg = G;
    a.Ho = R;
    a.Wo = 1;
    a.Cout = L.nout;
    a.relu = relu;
    use_split(a, L.x3);
    if (a.wh) {
      a.wh += k0;
      if (L.x3.lo != kNone) a.wl += k0;
    }
    const double fl = 2.0 * G * R * (double)L.nout * kn;
    launch(a.wh ? "conv_x3" : "conv_gemm", fl, [&] { launch_conv_gemm(a, st); }, &a);
  }

  void ln(const LNp& p, const float* x, int64_t ldx, float* y, int64_t ldy, int rows, const float* res = nullptr,
          int64_t ldres = 0, int res_div = 1, const float* fs = nullptr, const float* fb = nullptr, int film_div = 0,
          int64_t film_ld = 0) {
    launch("layernorm", 0, [&] {
      launch_layernorm(x, ldx, res, ldres, res_div, W(p.g), W(p.b), fs, fb, y, ldy, rows, p.c, st, film_div, film_ld);
    });
  }

  // ------------------------------------------------------------------ backbone
  // one ResNet stage; x (B,H,W,Cin) contiguous -> returns output buffer, updates H/W
  // `pool`: token pooling of the stage output to fuse into the final conv (pooled = whether it was)
  float* run_stage(const TrunkW& t, int s, const float* x, int B, int& H, int& Wd, const std::string& tag,
                   const PoolSpec* pool = nullptr, bool* pooled = nullptr) {
    if (pooled) *pooled = false;
    const std::vector<Block>& blocks = t.stages[s];
    const int stride = s == 0 ? 1 : 2;
    const int Ho = (H + 2 - 3) / stride + 1, Wo = (Wd + 2 - 3) / stride + 1;
    const int outc = t.ch[1 + s];
    const size_t n_out = (size_t)B * Ho * Wo * outc;
    const int mid = blocks[0].bottleneck ? outc / 4 : outc;
    float* bufA = buf(tag + "_s" + std::to_string(s) + "_a", n_out);
    float* bufB = buf(tag + "_s" + std::to_string(s) + "_b", n_out);
    float* tmp1 = buf(tag + "_s" + std::to_string(s) + "_t1", (size_t)B * std::max(H * Wd, Ho * Wo) * mid);
    float* tmp2 = buf(tag + "_s" + std::to_string(s) + "_t2", (size_t)B * Ho * Wo * mid);
    float* dsb = buf(tag + "_s" + std::to_string(s) + "_ds", n_out);
    // (layer 1 in MALL-sized chunks of scenes and fused BasicBlocks were measured slower and removed in round 6)
    bool all_pooled = true;
    const float* cur = x;
    int ch = H, cw = Wd;
    {
      const int nb = B;
      float* outs[2] = {bufA, bufB};
      for (size_t b = 0; b < blocks.size(); ++b) {
        const Block& blk = blocks[b];
        float* y = outs[b & 1];
        const float* sc = cur;
        const int bs = b == 0 ? stride : 1;
        const int oh = (ch + 2 - 3) / bs + 1, ow = (cw + 2 - 3) / bs + 1;
        if (blk.has_ds) {
          conv_c(blk.ds, cur, nb, ch, cw, dsb, false);
          sc = dsb;
        }
        const bool last = b + 1 == blocks.size();
        auto request_pool = [&]() {  // square windows that tile the output exactly
          if (!last || !pool || oh % pool->oh || ow % pool->ow || oh / pool->oh != ow / pool->ow) return;
          pool_next = *pool;
          pool_next_p = oh / pool->oh;
        };
        if (!blk.bottleneck) {
          conv_c(blk.c1, cur, nb, ch, cw, tmp2, true);
          request_pool();
          conv_c(blk.c2, tmp2, nb, oh, ow, y, true, sc);
        } else {
          conv_c(blk.c1, cur, nb, ch, cw, tmp1, true);
          conv_c(blk.c2, tmp1, nb, ch, cw, tmp2, true);
          request_pool();
          conv_c(blk.c3, tmp2, nb, oh, ow, y, true, sc);
        }
        if (last && pool) all_pooled = all_pooled && pool_done;
        pool_next_p = 0;
        cur = y;
        ch = oh;
        cw = ow;
      }
    }
    if (pool && pooled) *pooled = all_pooled;
    H = ch;
    Wd = cw;
    // the stage output: the last block's buffer, from the first scene
    return ((blocks.size() - 1) & 1) ? bufB : bufA;
  }

  // GPT fusion at scale i (transfuser_backbone.py:241-362); img (B,Hi,Wi,C), lid (B,Hl,Wl,Cl) in place.
  // the GPT token buffers of scale i (also the fused-pool targets of the stage's final convs)
  PoolSpec img_pool_spec(int i, int B) {
    const int C = gpt[i].C, T = 320;
    PoolSpec p;
    p.out = buf("gpt_x", (size_t)B * T * C);
    p.sn = (int64_t)T * C;
    p.sh = (int64_t)32 * C;
    p.sw = C;
    p.add = W(gpt[i].pos);
    p.add_sh = (int64_t)32 * C;
    p.add_sw = C;
    p.oh = 8;
    p.ow = 32;
    return p;
  }
  PoolSpec lid_pool_spec(int i, int B) {
    const int Cl = lid.ch[1 + i];
    PoolSpec p;
    p.out = buf("gpt_lpool", (size_t)B * 64 * Cl);
    p.sn = (int64_t)64 * Cl;
    p.sh = (int64_t)8 * Cl;
    p.sw = Cl;
    p.oh = 8;
    p.ow = 8;
    return p;
  }
  void fuse(int i, float* imgf, int B, int Hi, int Wi, float* lidf, int Hl, int Wl, bool img_pooled = false,
            bool lid_pooled = false) {
    const GptW& g = gpt[i];
    const int C = g.C, Cl = lid.ch[1 + i];
    const int T = 320, nimg = 256;
    const int hs = C / 4;
    float* X = buf("gpt_x", (size_t)B * T * C);
    float* Hb = buf("gpt_h", (size_t)B * T * C);
    float* QKV = buf("gpt_qkv", (size_t)B * T * 3 * C);
    float* Y = buf("gpt_y", (size_t)B * T * C);
    float* MLP = buf("gpt_mlp", (size_t)B * T * 4 * C);
    float* LP = buf("gpt_lpool", (size_t)B * 64 * Cl);
    float* LO = buf("gpt_lout", (size_t)B * 64 * Cl);
    // tokens: pooled image (8x32) + pos_emb, then lidar_channel_to_img(pooled lidar 8x8) + pos_emb
    View4 xo{X, (int64_t)T * C, (int64_t)32 * C, C, 1};
    if (!img_pooled) launch("pool", 0, [&] { launch_avgpool(imgf, B, Hi, Wi, C, 8, 32, xo, W(g.pos), st); });
    View4 lpo{LP, (int64_t)64 * Cl, (int64_t)8 * Cl, Cl, 1};
    if (!lid_pooled) launch("pool", 0, [&] { launch_avgpool(lidf, B, Hl, Wl, Cl, 8, 8, lpo, nullptr, st); });
    conv(l2i[i], LP, (int64_t)64 * Cl, (int64_t)8 * Cl, Cl, B, 8, 8, X + (size_t)nimg * C, (int64_t)T * C,
         (int64_t)8 * C, C, false, W(g.pos) + (size_t)nimg * C, 0, (int64_t)8 * C, C);
    const int M = B * T;
    // Hb = ln1(x) before each block's qkv, ln2(x) before its MLP, ln_f(x) at the end. Where the GEMM producing x
    // (proj, MLP-down) spans the row in one tile (C <= 128), its epilogue writes the LayerNorm too (gemm_ln)
    bool hb_ready = false;  // Hb already holds ln1 of the next block (or ln_f after the last)
    for (size_t bi = 0; bi < g.blocks.size(); ++bi) {
      const GptBlockW& w = g.blocks[bi];
      if (!hb_ready) ln(w.ln1, X, C, Hb, C, M);
      gemm(w.qkv, Hb, C, M, QKV, 3 * C);
      // softmax(Q K^T / sqrt(hs)) V per (scene, head), one fused launch (attention.hip): fp32 MFMA in the
      // fp32 mode, f16x3 MFMA in the f16x3 mode (two-way split scores) and the bf16 mode (three-way)
      const int aprec = (gemm_mode == DD_GEMM_FP32 || !gpt_attn_x3 || C / 4 > 128 || T % 32 || T > 1024)
                            ? 0
                            : (gemm_mode == DD_GEMM_BF16 ? 2 : 1);
      launch("attn", 4.0 * B * T * T * (double)C, [&] { launch_gpt_attention(QKV, B, T, C, 4, Y, aprec, st); });
      const LNp& nx = bi + 1 < g.blocks.size() ? g.blocks[bi + 1].ln1 : g.lnf;
      // C <= 128 in f16x3 at small batches: proj + ln2 + MLP + the next LayerNorm as one launch (gpt_tail.hip,
      // bit-identical): 3 launches -> 1 per block (C1 2.623 -> 2.600 ms); at B = 64 the fused launch's longer
      // dependent chain measured 0.3 % slower than the three kernels (profiles/round5_ab.md)
      const bool tail_on = gpt_tail_env >= 0 ? gpt_tail_env != 0 : B <= 16;
      if (tail_on && ln_fold && gemm_mode == DD_GEMM_F16X3 && gpt_tail_supported(C) && w.ln2.c == C && nx.c == C &&
          w.proj.x3.hi != kNone && w.mlp0.x3.hi != kNone && w.mlp2.x3.hi != kNone) {
        auto tw = [&](const Lin& L) {
          GptTailW t;
          t.wh = reinterpret_cast<const uint16_t*>(W(L.x3.hi));
          t.wl = reinterpret_cast<const uint16_t*>(W(L.x3.lo));
          t.sinv = W(L.x3.sinv);
          t.bias = W(L.b);
          t.ldh = L.x3.ldh;
          return t;
        };
        GptTailArgs t;
        t.y = Y;
        t.x = X;
        t.hb = Hb;
        t.M = M;
        t.C = C;
        t.proj = tw(w.proj);
        t.up = tw(w.mlp0);
        t.down = tw(w.mlp2);
        t.ln2_g = W(w.ln2.g);
        t.ln2_b = W(w.ln2.b);
        t.lnn_g = W(nx.g);
        t.lnn_b = W(nx.b);
        t.flags = num_flags;
        launch("gpt_tail", 2.0 * M * 9.0 * C * C, [&] { launch_gpt_tail(t, st); });
        hb_ready = true;
        continue;
      }
      if (!gemm_ln(w.proj, Y, C, M, X, C, X, C, w.ln2, Hb))  // x = x + proj(y); Hb = ln2(x)
        ln(w.ln2, X, C, Hb, C, M);
      gemm(w.mlp0, Hb, C, M, MLP, 4 * C, true);
      hb_ready = gemm_ln(w.mlp2, MLP, 4 * C, M, X, C, X, C, nx, Hb);  // x = x + mlp(ln2 x); Hb = next LN(x)
    }
    if (!hb_ready) ln(g.lnf, X, C, Hb, C, M);  // Hb = ln_f(x): image tokens rows 0..255, lidar 256..319 per scene
    conv(i2l[i], Hb + (size_t)nimg * C, (int64_t)T * C, (int64_t)8 * C, C, B, 8, 8, LO, (int64_t)64 * Cl,
         (int64_t)8 * Cl, Cl, false);
    // the image branch after the last fusion is never read (the BEV path takes the LiDAR features:
    // transformer_decoder_join, transfuser_backbone.py:204-205), so its upsample-add is skipped at i == 3
    if (i + 1 < 4) {
      View4 gi{Hb, (int64_t)T * C, (int64_t)32 * C, C, 1};
      View4 io{imgf, (int64_t)Hi * Wi * C, (int64_t)Wi * C, C, 1};
      launch("bilinear", 0, [&] { launch_bilinear(gi, B, 8, 32, C, io, Hi, Wi, 8.0f / Hi, 32.0f / Wi, 1, st); });
    }
    View4 gl{LO, (int64_t)64 * Cl, (int64_t)8 * Cl, Cl, 1};
    View4 lo{lidf, (int64_t)Hl * Wl * Cl, (int64_t)Wl * Cl, Cl, 1};
    launch("bilinear", 0, [&] { launch_bilinear(gl, B, 8, 8, Cl, lo, Hl, Wl, 8.0f / Hl, 8.0f / Wl, 1, st); });
  }

  // ------------------------------------------------------------------ forward
  // The bf16 mode (configs C2-bf16 / C4) is a BACKBONE mode: the trunks and the GPT fusion (60 of the 65
  // GFLOP/scene at ResNet-34, 160 of 162 at ResNet-50) take one bf16 product per MAC; everything after them -
  // FPN, BEV tokens, tf decoder, bev_proj, the optional heads and the trajectory head with its time MLP - runs
  // in f16x3 (on the megakernels), so the decoder adds fp32-class rounding only to the backbone's bf16 error.
  int head_mode() const { return gemm_mode == DD_GEMM_BF16 ? DD_GEMM_F16X3 : gemm_mode; }
  // the fused stems (f16x3 / bf16) read the caller's NCHW camera / LiDAR tensors directly (DDMI_STEM_NCHW=0: the
  // NHWC4 transpose pass first, as the fp32 mode always does)
  bool use_nchw_stem() const { return stem_nchw && gemm_mode != DD_GEMM_FP32 && cfg.lidar_channels <= 3; }
  struct ModeScope {
    Model* m;
    int saved;
    ModeScope(Model* mm, int mode) : m(mm), saved(mm->gemm_mode) { m->gemm_mode = mode; }
    ~ModeScope() { m->gemm_mode = saved; }
  };

  struct Outs {
    float* traj = nullptr;
    float* modes = nullptr;
    float* cls = nullptr;
    float* sem = nullptr;
    float* ag_states = nullptr;
    float* ag_labels = nullptr;
    // forward_train: every layer's poses_reg / poses_cls and LossComputer partials ([B][2] per layer)
    float* reg_l[2] = {nullptr, nullptr};
    float* cls_l[2] = {nullptr, nullptr};
    float* part_l[2] = {nullptr, nullptr};
  };

  // denoise timesteps. truncated: roll_timesteps = round(arange(steps) * step_span / steps)[::-1]
  // (:585-588; numpy round-half-even), DDIM prev = t - 1 (set_timesteps(1000), :584);
  // vanilla: diffusers "leading" set_timesteps(steps): t_i = (steps-1-i) * (1000 / steps), prev = t - ratio.
  std::vector<int> denoise_timesteps(int steps) const {
    const bool vanilla = schedule == DD_SCHED_VANILLA;
    std::vector<int> roll(steps);
    const int ratio = vanilla ? 1000 / steps : 1;
    for (int s = 0; s < steps; ++s)
      roll[steps - 1 - s] = vanilla ? s * ratio
                                    : (int)std::nearbyint((double)s * ((double)cfg.step_span / (double)steps));
    return roll;
  }
  // time_mlp (SinusoidalPosEmb -> Linear -> Mish -> Linear, :463-468) -> Mish -> FiLM scale / shift
  // of both decoder layers (:259-294), for every denoise step. A function of the weights and the
  // (fixed) denoise timesteps only, so it is computed once per (steps, schedule, arithmetic mode) into
  // persistent buffers (fixed-size, never reallocated) outside the captured forward; the forward reads
  // the cached table (the reference recomputes it per call, :580-641 - same values).
  std::string film_key;
  void ensure_film(int steps) {
    const std::string k = std::to_string(steps) + "/" + std::to_string(schedule) + "/" + std::to_string(gemm_mode);
    if (k == film_key) return;
    film_key.clear();
    time_film(steps);
    film_key = k;
  }
  void time_film(int steps) {
    ModeScope head_scope(this, head_mode());
    const int d = 256;
    const std::vector<int> roll = denoise_timesteps(steps);
    float* te0 = buf("temb0", d);
    float* te1 = buf("temb1", 4 * d);
    float* te2 = buf("temb2", d);
    float* mte = buf("temb_mish", d);
    for (int si = 0; si < steps; ++si) {
      const int k = roll[si];
      launch("misc", 0, [&] { launch_timestep_embed((float)k, te0, d, st); });
      gemm(tm1, te0, d, 1, te1, 4 * d);
      launch("misc", 0, [&] { launch_activation(te1, te1, 4 * d, 0, st); });
      gemm(tm3, te1, 4 * d, 1, te2, d);
      launch("misc", 0, [&] { launch_activation(te2, mte, d, 0, st); });
      for (int l = 0; l < 2; ++l)
        gemm(dl[l].film, mte, d, 1, buf("film_s" + std::to_string(si) + "l" + std::to_string(l), 2 * d), 2 * d);
    }
  }

  // training head: time_mlp(SinusoidalPosEmb(t_b)) -> Mish -> FiLM scale / shift of both layers for every scene
  // (forward_train :549-551, ModulationLayer :259-294), and the per-scene add_noise coefficients
  void train_time_film(int B) {
    const int d = 256;
    const int* t = reinterpret_cast<const int*>(bufs.at("in_tsteps").first);
    float* te0 = buf("train_temb0", (size_t)B * d);
    float* te1 = buf("train_temb1", (size_t)B * 4 * d);
    float* te2 = buf("train_temb2", (size_t)B * d);
    float* mte = buf("train_temb_mish", (size_t)B * d);
    launch("misc", 0, [&] { launch_timestep_embed_rows(t, te0, B, d, st); });
    gemm(tm1, te0, d, B, te1, 4 * d);
    launch("misc", 0, [&] { launch_activation(te1, te1, (int64_t)B * 4 * d, 0, st); });
    gemm(tm3, te1, 4 * d, B, te2, d);
    launch("misc", 0, [&] { launch_activation(te2, mte, (int64_t)B * d, 0, st); });
    for (int l = 0; l < 2; ++l) gemm(dl[l].film, mte, d, B, buf("train_film_l" + std::to_string(l), (size_t)B * 2 * d), 2 * d);
    float* sa = buf("train_sa", B);
    float* s1a = buf("train_s1a", B);
    launch("misc", 0, [&] { launch_train_coeffs(t, ac_dev, sa, s1a, B, 1000, st); });
  }

  // training head with targets: LossComputer's per-scene partials of both layers into "train_part_l*"
  void train_loss_partials(int B) {
    if (!train || !train_target) return;
    const int Q = cfg.num_modes, P = cfg.num_poses;
    for (int l = 0; l < 2; ++l) {
      const std::string sf = "_s0l" + std::to_string(l);
      float* part = buf("train_part_l" + std::to_string(l), (size_t)2 * B);
      launch("misc", 0, [&] {
        launch_traj_loss_scene(bufs.at("reg" + sf).first, bufs.at("cls" + sf).first, bufs.at("in_target").first,
                               W(anchor), part, B, Q, P, st);
      });
    }
  }

  void forward_body(int B, int steps, bool heads) {
    const int d = 256, Q = cfg.num_modes, P = cfg.num_poses;
    const int HC = cfg.cam_h, WC = cfg.cam_w, HL = cfg.lidar_h, WL = cfg.lidar_w;
    const bool nchw = use_nchw_stem();
    float* cam4 = nchw ? nullptr : bufs.at("in_cam4").first;
    float* lid4 = nchw ? nullptr : bufs.at("in_lid4").first;
    const float* stat = bufs["in_status"].first;
    const float* noise = bufs["in_noise"].first;

    // ---- stems + maxpool (timm conv1/bn1/act1/maxpool); the LiDAR trunk runs on the side stream
    fj_next = 0;
    int hi = (HC + 6 - 7) / 2 + 1, wi = (WC + 6 - 7) / 2 + 1;
    float* stem_i = buf("img_stem", (size_t)B * hi * wi * 64);
    int hl = (HL + 6 - 7) / 2 + 1, wl = (WL + 6 - 7) / 2 + 1;
    float* stem_l = buf("lid_stem", (size_t)B * hl * wl * 64);
    const int hi2 = (hi + 2 - 3) / 2 + 1, wi2 = (wi + 2 - 3) / 2 + 1;
    float* pool_i = buf("img_pool", (size_t)B * hi2 * wi2 * 64);
    const int hl2 = (hl + 2 - 3) / 2 + 1, wl2 = (wl + 2 - 3) / 2 + 1;
    float* pool_l = buf("lid_pool", (size_t)B * hl2 * wl2 * 64);
    fork();
    side([&] { stem_and_pool(lid.stem, lid4, B, HL, WL, stem_l, pool_l, hl2, wl2, 1, cfg.lidar_channels); });
    stem_and_pool(img.stem, cam4, B, HC, WC, stem_i, pool_i, hi2, wi2, 0, 3);

    // ---- 4 scales: trunk stages (image on the main stream, LiDAR beside it) + GPT fusion
    float* xi = pool_i;
    float* xl = pool_l;
    int Hi = hi2, Wi = wi2, Hl = hl2, Wl = wl2;
    for (int s = 0; s < 4; ++s) {
      if (s > 0) fork();
      // the stages' final convs also write the GPT tokens (fused pooling) where conv_x6 runs them
      const PoolSpec ip = img_pool_spec(s, B), lp = lid_pool_spec(s, B);
      bool ipooled = false, lpooled = false;
      side([&] { xl = run_stage(lid, s, xl, B, Hl, Wl, "lid", fuse_pool ? &lp : nullptr, &lpooled); });
      xi = run_stage(img, s, xi, B, Hi, Wi, "img", fuse_pool ? &ip : nullptr, &ipooled);
      join();
      fuse(s, xi, B, Hi, Wi, xl, Hl, Wl, ipooled, lpooled);
    }
    alias("img_l4", xi);  // before the (skipped, dead) last fusion add
    alias("bev_feature", xl);  // (B, 8, 8, 512) NHWC; transformer_decoder_join -> fused = lidar (:204-205)
    // everything past the backbone runs in the head arithmetic (bf16 mode: f16x3; see head_mode)
    ModeScope head_scope(this, head_mode());
    if (train) train_time_film(B);

    // ---- BEV tokens + status -> keyval (B, 65, 256) (+= _keyval_embedding)
    float* KV = buf("keyval", (size_t)B * 65 * d);
    conv(bev_down, xl, (int64_t)Hl * Wl * 512, (int64_t)Wl * 512, 512, B, Hl, Wl, KV, (int64_t)65 * d, (int64_t)Wl * d,
         d, false, W(kv_emb), 0, (int64_t)Wl * d, d);
    gemm_g(status, stat, 8, 8, B, 1, KV + (size_t)64 * d, (int64_t)65 * d, d, false, W(kv_emb) + (size_t)64 * d, 0, d);

    // ---- _tf_decoder: 3 post-norm layers over 31 queries, memory = keyval (:141-142), on the side
    // stream beside the FPN / bev_proj / value_proj chain below
    const int NQ = 31;
    float* q = buf("query_out", (size_t)B * NQ * d);
    float* egos[2];
    float* akv[2];
    fork();
    side([&] {
      if (tfdec_mk && tf_mk_layers && gemm_mode == DD_GEMM_F16X3) {
        // the memory's cross-attention K | V of all 3 layers in one GEMM, then one megakernel launch
        float* kvx = buf("tf_kvx", (size_t)B * 65 * 6 * d);
        gemm(tf_cakv, KV, d, B * 65, kvx, 6 * d);
        TfMkArgs t;
        t.layers = tf_mk_layers;
        for (int l = 0; l < 2; ++l) {
          t.ag_kv[l] = mk(m_agkv[l]);
          t.eg_v[l] = mk(m_egv[l]);
          t.eg_out[l] = mk(m_egout[l]);
          egos[l] = buf("ego_out" + std::to_string(l), (size_t)B * d);
          akv[l] = buf("agent_kv" + std::to_string(l), (size_t)B * 30 * 2 * d);
          t.akv[l] = akv[l];
          t.ego[l] = egos[l];
        }
        t.qemb = W(q_emb);
        t.kvx = kvx;
        t.query_out = q;
        t.B = B;
        t.flags = num_flags;
        // four workgroups per scene (heads / FFN chunks split, three L2 exchanges per layer) while B x 4 fits a
        // quarter of the chip: batch 1 2.745 -> 2.62 ms, but at B = 64 the 256 mostly-waiting workgroups crowd out
        // the main stream's work beside them (3 in flight -1.5 %, profiles/round5_ab.md). DDMI_TF_GROUPS=1 / 4
        // forces a form; the stamps diagnostics take the one-workgroup kernel
        t.groups = (mk_stamps || tf_groups_env == 1) ? 1 : ((tf_groups_env == 4 || B * 4 <= 64) ? 4 : 1);
        if (t.groups == 4) {
          t.xbuf_floats = tfdec_mk_xbuf_floats(B);
          t.xbuf = buf("tf_xbuf", t.xbuf_floats);
          t.sync_cnt_n = (size_t)2 * B;
          t.sync_cnt = reinterpret_cast<unsigned*>(buf_zeroed("tf_sync_cnt", t.sync_cnt_n));
        }
        if (mk_stamps) t.stamps = reinterpret_cast<unsigned long long*>(buf("tf_stamps", (size_t)B * 80));
        // 2 x rows x sum(K x N): per layer q|k|v, 2 out_proj, cross q, FFN (+ the attention products), hoists
        const double kn = 3.0 * (3584.0 * d) + 4.0 * d * d + 4.0 * d * d;
        const double att = 3.0 * 8 * (31.0 * 31 + 31.0 * 65) * 32 * 2;
        launch("tfdec", 2.0 * B * (NQ * kn + att), [&] { launch_tfdec_mk(t, st); });
        return;
      }
      launch("misc", 0, [&] { launch_broadcast_rows(W(q_emb), NQ, q, B * NQ, d, st); });
      float* qkv = buf("tf_qkv", (size_t)B * NQ * 3 * d);
      float* att = buf("tf_att", (size_t)B * NQ * d);
      float* tmp = buf("tf_tmp", (size_t)B * NQ * d);
      float* kvp = buf("tf_kvp", (size_t)B * 65 * 2 * d);
      float* ff = buf("tf_ff", (size_t)B * NQ * 1024);
      const int MQ = B * NQ;
      for (const TfLayerW& w : tf) {
        gemm(w.sa_in, q, d, MQ, qkv, 3 * d);
        launch("mha", 0, [&] {
          launch_mha_small(qkv, 3 * d, qkv + d, qkv + 2 * d, 3 * d, att, d, B, NQ, NQ, 8, 32, (int64_t)NQ * 3 * d,
                           (int64_t)NQ * 3 * d, (int64_t)NQ * d, st);
        });
        gemm(w.sa_out, att, d, MQ, tmp, d, false, q, d);
        ln(w.n1, tmp, d, q, d, MQ);
        gemm(w.ca_q, q, d, MQ, qkv, d);
        gemm(w.ca_kv, KV, d, B * 65, kvp, 2 * d);
        launch("mha", 0, [&] {
          launch_mha_small(qkv, d, kvp, kvp + d, 2 * d, att, d, B, NQ, 65, 8, 32, (int64_t)NQ * d, (int64_t)65 * 2 * d,
                           (int64_t)NQ * d, st);
        });
        gemm(w.ca_out, att, d, MQ, tmp, d, false, q, d);
        ln(w.n2, tmp, d, q, d, MQ);
        gemm(w.l1, q, d, MQ, ff, 1024, true);
        gemm(w.l2, ff, 1024, MQ, tmp, d, false, q, d);
        ln(w.n3, tmp, d, q, d, MQ);
      }
      // per decoder layer, step-invariant (exact hoists): ego cross-attention over ONE key =
      // out_proj(v_proj(ego)); agent K / V projections
      for (int l = 0; l < 2; ++l) {
        const DiffLayerW& w = dl[l];
        float* e1 = buf("ego_v" + std::to_string(l), (size_t)B * d);
        gemm_g(w.eg_v, q, (int64_t)NQ * d, d, B, 1, e1, d, d);
        egos[l] = buf("ego_out" + std::to_string(l), (size_t)B * d);
        gemm(w.eg_out, e1, d, B, egos[l], d);
        akv[l] = buf("agent_kv" + std::to_string(l), (size_t)B * 30 * 2 * d);
        gemm_g(w.ag_kv, q + d, (int64_t)NQ * d, d, B, 30, akv[l], (int64_t)30 * 2 * d, 2 * d);
      }
    });

    // ---- FPN top_down (transfuser_backbone.py:153-159); p3 lands in channels 256..319 of the
    // concat buffer that feeds bev_proj (transfuser_model_v2.py:123-140).
    const int bc = 64, HB = HL / 4, WB = WL / 4;  // 64 x 64
    float* p5 = buf("p5", (size_t)B * Hl * Wl * bc);
    conv_c(c5, xl, B, Hl, Wl, p5, true);
    float* up2 = buf("p5_up", (size_t)B * Hl * 2 * Wl * 2 * bc);
    {
      View4 a{p5, (int64_t)Hl * Wl * bc, (int64_t)Wl * bc, bc, 1};
      View4 o{up2, (int64_t)4 * Hl * Wl * bc, (int64_t)2 * Wl * bc, bc, 1};
      launch("bilinear", 0, [&] { launch_bilinear(a, B, Hl, Wl, bc, o, 2 * Hl, 2 * Wl, 0.5f, 0.5f, 0, st); });
    }
    float* p4 = buf("p4", (size_t)B * 4 * Hl * Wl * bc);
    conv_c(up5, up2, B, 2 * Hl, 2 * Wl, p4, true);
    float* up3 = buf("p4_up", (size_t)B * HB * WB * bc);
    {
      View4 a{p4, (int64_t)4 * Hl * Wl * bc, (int64_t)2 * Wl * bc, bc, 1};
      View4 o{up3, (int64_t)HB * WB * bc, (int64_t)WB * bc, bc, 1};
      launch("bilinear", 0, [&] {
        launch_bilinear(a, B, 2 * Hl, 2 * Wl, bc, o, HB, WB, (float)(2 * Hl) / HB, (float)(2 * Wl) / WB, 0, st);
      });
    }
    const int CC = 320;
    float* cross_in = buf("cross_in", (size_t)B * HB * WB * CC);
    conv(up4, up3, (int64_t)HB * WB * bc, (int64_t)WB * bc, bc, B, HB, WB, cross_in + 256, (int64_t)HB * WB * CC,
         (int64_t)WB * CC, CC, true);

    const int MB = B * HB * WB;
    float* cross = buf("cross_bev", (size_t)MB * d);
    const int bp_mode = (bevproj_mode == 2 && (gemm_mode == DD_GEMM_FP32 || m_bevp3.w == kNone)) ? 1 : bevproj_mode;
    if (bp_mode >= 1) {
      // bev_proj(cat(bilinear(keyval 8x8), p3)) = bilinear(W[:, :256] keyval) + W[:, 256:] p3 + b: bilinear
      // interpolation is linear with weights summing to 1, so the keyval half of the 320 -> 256 projection runs
      // on the 8 x 8 tokens and is upsampled into cross_bev, which the p3 half (K = 64) then adds to in place
      float* kvp = buf("kv_proj", (size_t)B * 64 * d);
      gemm_slice(bevproj, 0, d, false, KV, (int64_t)65 * d, d, B, 64, kvp, (int64_t)64 * d, d, false, nullptr, 0, 0);
      if (bp_mode == 2) {
        // one pass: p3 in, cross_bev out (bevproj.hip)
        BevProjArgs a;
        a.p3 = cross_in + 256;
        a.p3_ld = CC;
        a.kvp = kvp;
        a.w = reinterpret_cast<const uint4*>(W(m_bevp3.w));
        a.s = W(m_bevp3.s);
        a.bias = W(bevproj.b);
        a.g = W(bevproj_ln.g);
        a.beta = W(bevproj_ln.b);
        a.out = cross;
        a.B = B;
        a.H = HB;
        a.W = WB;
        a.Hk = 8;
        a.Wk = 8;
        a.flags = num_flags;
        launch("bevproj", 2.0 * MB * 64 * d * 3, [&] { launch_bevproj(a, st); });
      } else {
        View4 a{kvp, (int64_t)64 * d, (int64_t)8 * d, d, 1};
        View4 o{cross, (int64_t)HB * WB * d, (int64_t)WB * d, d, 1};
        launch("bilinear", 0, [&] { launch_bilinear(a, B, 8, 8, d, o, HB, WB, 8.0f / HB, 8.0f / WB, 0, st); });
        gemm_slice(bevproj, d, CC - d, true, cross_in + d, (int64_t)MB * CC, CC, 1, MB, cross, (int64_t)MB * d, d,
                   true, cross, (int64_t)MB * d, d);
        ln(bevproj_ln, cross, d, cross, d, MB);
      }
    } else {
      // concat_cross_bev: keyval[:, :64] as (B,8,8,256) -> bilinear 64x64 -> channels 0..255
      View4 a{KV, (int64_t)65 * d, (int64_t)8 * d, d, 1};
      View4 o{cross_in, (int64_t)HB * WB * CC, (int64_t)WB * CC, CC, 1};
      launch("bilinear", 0, [&] { launch_bilinear(a, B, 8, 8, d, o, HB, WB, 8.0f / HB, 8.0f / WB, 0, st); });
      gemm(bevproj, cross_in, CC, MB, cross, d, true);
      ln(bevproj_ln, cross, d, cross, d, MB);
    }

    // value_proj for both decoder layers (main stream, beside the tf decoder), then join. (Layer 1's
    // on a third stream beside the first trajectory-head layer was measured: the graph put it on
    // the hardware queue of layer 0's and the head behind it - no overlap.)
    const int R = B * Q;  // trajectory query rows
    // In f16x3 mode the conv is instead evaluated per (step, layer) at the B x Q x P x 4 bilinear taps
    // grid_sample reads (gathered rows, below): 40960 rows per call at B = 64 instead of 262144 per layer.
    const bool gathered = gemm_mode == DD_GEMM_F16X3 && dl[0].vproj.x3.hi != kNone &&
                          dl[1].vproj.x3.hi != kNone;
    float* vals[2] = {nullptr, nullptr};
    for (int l = 0; l < 2 && !gathered; ++l) {
      vals[l] = buf("value_l" + std::to_string(l), (size_t)MB * d);
      conv_c(dl[l].vproj, cross, B, HB, WB, vals[l], true);
    }
    // the tf decoder branch is joined only where the trajectory head first reads its output (the
    // agent cross-attention of step 0 / layer 0): the trajectory embedding, anchor encoder, BEV
    // sampling (and its gathered value rows) of that layer run beside the tf decoder's tail (joining
    // before the trajectory head measured 1.4 % slower)
    bool tf_pending = true;
    const float* agents = q + d;   // rows 1..30

    // ---- optional heads (off the waypoint path), on the side stream beside the trajectory head
    fork();
    side([&] {
      if (heads) {
        float* s1 = buf("sem_h", (size_t)B * HB * WB * bc);
        conv(sem0, cross_in + 256, (int64_t)HB * WB * CC, (int64_t)WB * CC, CC, B, HB, WB, s1, (int64_t)HB * WB * bc,
             (int64_t)WB * bc, bc, true);
        float* s2 = buf("sem_logits", (size_t)B * HB * WB * 8);
        conv(sem2, s1, (int64_t)HB * WB * bc, (int64_t)WB * bc, bc, B, HB, WB, s2, (int64_t)HB * WB * 7, (int64_t)WB * 7, 7,
             false);
        const int SH = HL / 2, SW = WL;
        float* sem = buf("bev_semantic_map", (size_t)B * 7 * SH * SW);
        View4 a{s2, (int64_t)HB * WB * 7, (int64_t)WB * 7, 7, 1};
        View4 o{sem, (int64_t)7 * SH * SW, SW, 1, (int64_t)SH * SW};
        launch("bilinear", 0, [&] {
          launch_bilinear(a, B, HB, WB, 7, o, SH, SW, (float)HB / SH, (float)WB / SW, 0, st);
        });
        float* a1 = buf("agent_h", (size_t)B * 30 * 1024);
        gemm_g(ag0, agents, (int64_t)NQ * d, d, B, 30, a1, (int64_t)30 * 1024, 1024, true);
        float* ast = buf("agent_states", (size_t)B * 30 * 5);
        gemm(ag2, a1, 1024, B * 30, ast, 5);
        launch("misc", 0, [&] { launch_agent_post(ast, B * 30, st); });
        float* alb = buf("agent_labels", (size_t)B * 30);
        gemm_g(agl, agents, (int64_t)NQ * d, d, B, 30, alb, 30, 1);
      }
    });

    // ---- trajectory head (TrajectoryHead.forward_test, :578-641)
    if (decoder_mk && mk_ready && gathered) {
      traj_head_mk(B, steps, cross, akv, egos, tf_pending, noise);
      return;
    }
    float* imgx = buf("ddim_img", (size_t)R * P * 2);
    const bool vanilla = schedule == DD_SCHED_VANILLA;
    {
      // truncated: add_noise(norm_odo(anchor), noise, t = trunc_timestep) (:593-597);
      // vanilla (C5 ablation): x_T = noise (sa = 0, s1a = 1 keep it bit-exact)
      const float a8 = ac[cfg.trunc_timestep];
      const float sa = vanilla ? 0.0f : std::sqrt(a8), s1a = vanilla ? 1.0f : std::sqrt(1.0f - a8);
      if (train)  // forward_train: per-scene timesteps (train_time_film)
        launch("misc", 0, [&] {
          launch_train_noisy(W(anchor), noise, bufs.at("train_sa").first, bufs.at("train_s1a").first, imgx, B, Q * P,
                             st);
        });
      else
        launch("misc", 0, [&] { launch_ddim_init(W(anchor), noise, imgx, B, Q * P, sa, s1a, st); });
    }
    float* pts = buf("pts", (size_t)R * P * 2);
    float* pts2 = buf("pts_next", (size_t)R * P * 2);
    float* emb = buf("traj_emb", (size_t)R * P * 64);
    float* tf1 = buf("traj_tf1", (size_t)R * d);
    float* tfe = buf("traj_feature", (size_t)R * d);
    float* te0 = buf("temb0", d);
    float* te1 = buf("temb1", 4 * d);
    float* te2 = buf("temb2", d);
    float* logit = buf("bev_logits", (size_t)R * 8);
    float* gs = buf("gs", (size_t)R * d);
    float* x1 = buf("dx1", (size_t)R * d);
    float* x3 = buf("dx3", (size_t)R * d);
    float* qa = buf("dqa", (size_t)R * d);
    float* hf = buf("dffn", (size_t)R * 1024);
    float* c1 = buf("dc1", (size_t)R * d);
    float* c2 = buf("dc2", (size_t)R * d);
    float* r1 = buf("dr1", (size_t)R * d);
    float* r2 = buf("dr2", (size_t)R * d);
    float* rr = buf("dr", (size_t)R * P * 3);
    const std::vector<int> roll = denoise_timesteps(steps);
    const int ratio = vanilla ? 1000 / steps : 1;
    float* reg_last = nullptr;
    float* cls_last = nullptr;
    for (int si = 0; si < steps; ++si) {
      const int k = roll[si];
      // FiLM scale / shift of both layers: the cached table of ensure_film()
      float* film_ss[2];
      for (int l = 0; l < 2; ++l)
        film_ss[l] = buf("film_s" + std::to_string(si) + "l" + std::to_string(l), 2 * d);
      launch("misc", 0, [&] { launch_traj_embed(imgx, pts, emb, R, P, st); });
      // gathered value_proj of layer 0 (its points are known now) on the side stream, beside the
      // trajectory-feature GEMMs; layer 1's follows layer 0's reg branch on the main stream
      float* vrows_l[2] = {nullptr, nullptr};
      const int* vslots_l[2] = {nullptr, nullptr};
      auto gather_value = [&](int l, const float* pts_l) {
        const std::string sfx = "_s" + std::to_string(si) + "l" + std::to_string(l);
        const int MR = R * P * 4;
        int* rows = reinterpret_cast<int*>(buf("value_taps" + sfx, (size_t)MR));
        int* slots = reinterpret_cast<int*>(buf("value_slots" + sfx, (size_t)MR));
        float* vrows = buf("value_rows" + sfx, (size_t)MR * d);
        bool dd = false;
        if (slots)
          launch("misc", 0, [&] {
            dd = launch_bev_tap_dedup(pts_l, rows, slots, B, Q, P, HB, WB, 1.0f / 32.0f, 1.0f / 32.0f, st);
          });
        if (!dd) {
          slots = nullptr;
          launch("misc", 0, [&] { launch_bev_tap_rows(pts_l, rows, B, Q, P, HB, WB, 1.0f / 32.0f, 1.0f / 32.0f, st); });
        }
        vslots_l[l] = slots;
        ConvArgs a = conv_args(dl[l].vproj, cross, (int64_t)HB * WB * d, (int64_t)WB * d, d, B, HB, WB, vrows,
                               (int64_t)MR * d, d, 0, true, nullptr, 0, 0, 0);
        a.Nimg = 1;
        a.Ho = MR;
        a.Wo = 1;
        a.rowmap = rows;
        a.rowmap_nimg = B;
        const double fl = 2.0 * MR * (double)d * 9 * dl[l].vproj.cin_real;
        launch("conv_x3", fl, [&] { launch_conv_gemm(a, st); }, &a);
        vrows_l[l] = vrows;
      };
      if (gathered) {
        if (si == 0) {
          gather_value(0, pts);  // the side stream still carries the tf decoder
        } else {
          fork();
          side([&] { gather_value(0, pts); });
        }
      }
      gemm(pa0, emb, 512, R, tf1, d, true);
      ln(pa2, tf1, d, tf1, d, R);
      gemm(pa3, tf1, d, R, tfe, d);
      const float* cur = pts;
      for (int l = 0; l < 2; ++l) {
        const DiffLayerW& w = dl[l];
        const std::string sfx = "_s" + std::to_string(si) + "l" + std::to_string(l);
        float* ss = film_ss[l];
        // per-(step, layer) buffer: the cls branch of this layer reads it beside the next layer
        float* x2 = buf("dx2" + sfx, (size_t)R * d);
        // GridSampleCrossBEVAttention
        gemm(w.attw, tfe, d, R, logit, P);
        float* gso = buf("gs" + sfx, (size_t)R * d);
        if (gathered) {
          if (l == 0) {
            if (si > 0) join();  // layer 0's gathered value rows
          } else {
            gather_value(l, cur);
          }
          float* vrows = vrows_l[l];
          launch("bev_sample", 0, [&] {
            launch_bev_sample_attn_gathered(logit, cur, vrows, vslots_l[l], gso, B, Q, P, HB, WB, d, 1.0f / 32.0f,
                                            1.0f / 32.0f, st);
          });
        } else {
          launch("bev_sample", 0, [&] {
            launch_bev_sample_attn(logit, cur, vals[l], gso, B, Q, P, HB, WB, d, 1.0f / 32.0f, 1.0f / 32.0f, st);
          });
        }
        gemm(w.outp, gso, d, R, x1, d, false, tfe, d);
        // cross_agent_attention + norm1
        gemm(w.ag_q, x1, d, R, qa, d);
        if (tf_pending) {
          join();  // tf decoder: agent K / V and ego rows of both layers
          tf_pending = false;
        }
        launch("mha", 0, [&] {
          launch_mha_small(qa, d, akv[l], akv[l] + d, 2 * d, gs, d, B, Q, 30, 8, 32, (int64_t)Q * d,
                           (int64_t)30 * 2 * d, (int64_t)Q * d, st);
        });
        gemm(w.ag_out, gs, d, R, x2, d, false, x1, d);
        ln(w.n1, x2, d, x2, d, R);
        // cross_ego_attention (hoisted, exact) + norm2
        ln(w.n2, x2, d, x3, d, R, egos[l], d, Q);
        // ffn -> norm3 -> FiLM time modulation
        gemm(w.ffn0, x3, d, R, hf, 1024, true);
        gemm(w.ffn2, hf, 1024, R, x2, d);
        if (train) {  // one FiLM vector per scene (its Q rows)
          const float* fl = bufs.at("train_film_l" + std::to_string(l)).first;
          ln(w.n3, x2, d, x2, d, R, nullptr, 0, 1, fl, fl + d, Q, 2 * d);
        } else {
          ln(w.n3, x2, d, x2, d, R, nullptr, 0, 1, ss, ss + d);
        }
        // task decoder: cls branch on the side stream beside the reg branch (and the next layer)
        float* cls = buf("cls" + sfx, R);
        fork();
        side([&] {
          gemm(w.c0, x2, d, R, c1, d, true);
          ln(w.c2, c1, d, c1, d, R);
          gemm(w.c3, c1, d, R, c2, d, true);
          ln(w.c5, c2, d, c2, d, R);
          gemm(w.c6, c2, d, R, cls, 1);
        });
        float* reg = buf("reg" + sfx, (size_t)R * P * 3);
        float* nxt = (l == 0) ? pts2 : nullptr;
        gemm(w.r0, x2, d, R, r1, d, true);
        gemm(w.r2, r1, d, R, r2, d, true);
        gemm(w.r4, r2, d, R, rr, P * 3);
        launch("misc", 0, [&] { launch_reg_finalize(rr, cur, reg, nxt, R, P, st); });
        cur = pts2;
        reg_last = reg;
        cls_last = cls;
      }
      if (si + 1 < steps) {
        const float a_t = ac[k];
        const float a_p = (k - ratio >= 0) ? ac[k - ratio] : 1.0f;
        launch("misc", 0, [&] { launch_ddim_step(reg_last, imgx, R, P, a_t, a_p, st); });
      }
    }
    float* traj = buf("trajectory", (size_t)B * P * 3);
    int* idx = reinterpret_cast<int*>(buf("mode_idx", B));
    join();  // the cls branches (and the heads branch before them on the side stream)
    launch("misc", 0, [&] { launch_select_mode(cls_last, reg_last, traj, idx, B, Q, P, st); });
    alias("poses_reg", reg_last);
    alias("poses_cls", cls_last);
    train_loss_partials(B);
  }

  std::map<std::string, float*> aliases;
  void alias(const std::string& name, float* p) { aliases[name] = p; }

  // noise == NULL: draw it on the device for scenes [scene0, scene0 + B) of the handle's stream
  void stage_inputs(const float* camera, const float* lidar, const float* status, const float* noise, int B,
                    uint64_t scene0) {
    float* st_in = buf("in_status", (size_t)B * 8);
    const size_t per = (size_t)cfg.num_modes * cfg.num_poses * 2;
    float* nz = buf("in_noise", (size_t)B * per);
    if (use_nchw_stem()) {
      // the stems read the caller's NCHW tensors in place: only their addresses go to the device table (the
      // captured graph reads them from there); the caller's buffers outlive the forward (stream order)
      launch("misc", 0, [&] { launch_set_ptrs(in_tab, camera, lidar, st); });
    } else {
      float* cam4 = buf("in_cam4", (size_t)B * cfg.cam_h * cfg.cam_w * 4);
      float* lid4 = buf("in_lid4", (size_t)B * cfg.lidar_h * cfg.lidar_w * 4);
      launch("misc", 0, [&] { launch_nchw_to_nhwc(camera, cam4, B, 3, cfg.cam_h, cfg.cam_w, 4, st); });
      launch("misc", 0, [&] { launch_nchw_to_nhwc(lidar, lid4, B, cfg.lidar_channels, cfg.lidar_h, cfg.lidar_w, 4, st); });
    }
    DD_HIP_CHECK(hipMemcpyAsync(st_in, status, sizeof(float) * B * 8, hipMemcpyDeviceToDevice, st));
    if (train) {
      float* tb = buf("in_tsteps", (size_t)B);
      DD_HIP_CHECK(hipMemcpyAsync(tb, train_t, sizeof(int) * B, hipMemcpyDeviceToDevice, st));
      if (train_target) {
        float* tg = buf("in_target", (size_t)B * cfg.num_poses * 3);
        DD_HIP_CHECK(hipMemcpyAsync(tg, train_target, sizeof(float) * B * cfg.num_poses * 3, hipMemcpyDeviceToDevice, st));
      }
    }
    if (noise)
      DD_HIP_CHECK(hipMemcpyAsync(nz, noise, sizeof(float) * B * per, hipMemcpyDeviceToDevice, st));
    else
      launch("misc", 0, [&] { launch_normal_philox(nz, (int64_t)(B * per), rng_seed, scene0 * per, st); });
  }

  void copy_out(float* dst, const std::string& name, size_t n) {
    if (!dst) return;
    float* src = nullptr;
    auto a = aliases.find(name);
    if (a != aliases.end())
      src = a->second;
    else
      src = bufs.at(name).first;
    DD_HIP_CHECK(hipMemcpyAsync(dst, src, n * sizeof(float), hipMemcpyDeviceToDevice, st));
  }

  // The forward of B scenes. More than max_chunk scenes run as ceil(B / max_chunk) equal chunks (the last one
  // may be shorter) through the same per-chunk path, in order on the handle's stream; every kernel of the path
  // is per scene, so a chunked forward equals the forward of its chunks scene for scene.
  void forward(const float* camera, const float* lidar, const float* status, const float* noise, int B, int steps,
               const Outs& o, hipStream_t caller) {
    if (B <= 0) throw std::invalid_argument("batch must be positive");
    if (steps <= 0 || steps > (schedule == DD_SCHED_VANILLA ? 1000 : cfg.step_span))
      throw std::invalid_argument("steps must be in [1, step_span] (truncated) or [1, 1000] (vanilla)");
    if (!camera || !lidar || !status || !o.traj) throw std::invalid_argument("null input/output pointer");
    if (!noise && (cfg.num_modes * cfg.num_poses) % 2)
      throw std::invalid_argument("device noise draw needs num_modes * num_poses even");
    const int Q = cfg.num_modes, P = cfg.num_poses;
    const int nch = (B + max_chunk - 1) / max_chunk, chunk = (B + nch - 1) / nch;
    for (int b0 = 0; b0 < B; b0 += chunk) {
      const int n = std::min(chunk, B - b0);
      auto off = [&](const float* p, size_t per) { return p ? p + (size_t)b0 * per : nullptr; };
      auto offw = [&](float* p, size_t per) { return p ? p + (size_t)b0 * per : nullptr; };
      Outs oc;
      oc.traj = offw(o.traj, (size_t)P * 3);
      oc.modes = offw(o.modes, (size_t)Q * P * 3);
      oc.cls = offw(o.cls, (size_t)Q);
      oc.sem = offw(o.sem, (size_t)7 * (cfg.lidar_h / 2) * cfg.lidar_w);
      oc.ag_states = offw(o.ag_states, (size_t)30 * 5);
      oc.ag_labels = offw(o.ag_labels, (size_t)30);
      forward_chunk(off(camera, (size_t)3 * cfg.cam_h * cfg.cam_w),
                    off(lidar, (size_t)cfg.lidar_channels * cfg.lidar_h * cfg.lidar_w), off(status, 8),
                    off(noise, (size_t)Q * P * 2), n, steps, oc, caller, rng_next + (uint64_t)b0);
    }
    if (!noise) rng_next += (uint64_t)B;
  }

  // The training-mode trajectory head (forward_train, transfuser_model_v2.py:520-576) over the eval-mode network, as
  // a loss evaluator: per-scene timesteps / noise in, every layer's poses out, and with targets the LossComputer losses
  // (multimodal_loss.py:119-168) of both layers and their sum (loss[3]), reduced over the whole batch after its chunks.
  void forward_train(const float* camera, const float* lidar, const float* status, const float* noise,
                     const int* timesteps, const float* target, int B, const Outs& o, float* loss, float cls_w,
                     float reg_w, hipStream_t caller) {
    if (B <= 0) throw std::invalid_argument("batch must be positive");
    if (!camera || !lidar || !status || !noise || !timesteps || !o.traj)
      throw std::invalid_argument("dd_forward_train: null input / output pointer (noise and timesteps are required)");
    if (loss && !target) throw std::invalid_argument("dd_forward_train: loss requested without targets");
    const int Q = cfg.num_modes, P = cfg.num_poses;
    if (target && train_part_n < (size_t)B) {
      DD_HIP_CHECK(hipDeviceSynchronize());  // an earlier call's reduction may still read the old buffer
      if (train_part) DD_HIP_CHECK(hipFree(train_part));
      train_part = nullptr;
      DD_HIP_CHECK(hipMalloc(&train_part, sizeof(float) * 4 * (size_t)B));
      train_part_n = (size_t)B;
    }
    struct Reset {
      Model& m;
      ~Reset() {
        m.train = false;
        m.train_t = nullptr;
        m.train_target = nullptr;
      }
    } reset{*this};
    train = true;
    const int nch = (B + max_chunk - 1) / max_chunk, chunk = (B + nch - 1) / nch;
    for (int b0 = 0; b0 < B; b0 += chunk) {
      const int n = std::min(chunk, B - b0);
      auto off = [&](const float* p, size_t per) { return p ? p + (size_t)b0 * per : nullptr; };
      auto offw = [&](float* p, size_t per) { return p ? p + (size_t)b0 * per : nullptr; };
      Outs oc;
      oc.traj = offw(o.traj, (size_t)P * 3);
      oc.sem = offw(o.sem, (size_t)7 * (cfg.lidar_h / 2) * cfg.lidar_w);
      oc.ag_states = offw(o.ag_states, (size_t)30 * 5);
      oc.ag_labels = offw(o.ag_labels, (size_t)30);
      for (int l = 0; l < 2; ++l) {
        oc.reg_l[l] = o.reg_l[l] ? o.reg_l[l] + (size_t)b0 * Q * P * 3 : nullptr;
        oc.cls_l[l] = o.cls_l[l] ? o.cls_l[l] + (size_t)b0 * Q : nullptr;
        oc.part_l[l] = target ? train_part + (size_t)l * 2 * B + (size_t)b0 * 2 : nullptr;
      }
      train_t = timesteps + b0;
      train_target = target ? target + (size_t)b0 * P * 3 : nullptr;
      forward_chunk(off(camera, (size_t)3 * cfg.cam_h * cfg.cam_w),
                    off(lidar, (size_t)cfg.lidar_channels * cfg.lidar_h * cfg.lidar_w), off(status, 8),
                    off(noise, (size_t)Q * P * 2), n, 1, oc, caller, 0);
    }
    if (target) {
      // the batch means of both layers and their sum, on the caller's stream (every chunk handed back to it)
      launch_traj_loss_reduce(train_part, train_loss_dev, B, Q, P, cls_w, reg_w, caller);
      launch_traj_loss_reduce(train_part + 2 * (size_t)B, train_loss_dev + 1, B, Q, P, cls_w, reg_w, caller);
      launch_add2(train_loss_dev, caller);
      if (loss) DD_HIP_CHECK(hipMemcpyAsync(loss, train_loss_dev, 3 * sizeof(float), hipMemcpyDeviceToDevice, caller));
      // the reduction read the handle-wide partials: the handle's next forward waits for it (OnStream)
      DD_HIP_CHECK(hipEventRecord(ev_out, caller));
    }
  }

  // Single-stream forwards (dd_set_streams(h, 1)) called on a non-default stream run on the CALLER's stream
  // itself: no hand-off through the handle's own stream, so N handles driven from N caller streams (N batches
  // in flight) occupy N hardware queues, not 2N (the device has 4 per process by default; streams beyond them
  // share queues and serialise). Restores the handle's stream on exit. Either way the forward is ordered after the
  // handle's previous one (ev_out; it may have run - or reduced losses - on another caller's stream), since both
  // use the same workspace.
  struct OnStream {
    Model& m;
    bool direct;
    OnStream(Model& mm, hipStream_t caller) : m(mm), direct(!mm.use_side && caller != nullptr && !mm.profiling) {
      if (direct) {
        m.st_main = caller;
        m.st = caller;
        DD_HIP_CHECK(hipStreamWaitEvent(caller, m.ev_out, 0));
      } else {
        // order the handle's stream after the caller's stream, run everything there, then hand back
        DD_HIP_CHECK(hipEventRecord(m.ev_in, caller));
        DD_HIP_CHECK(hipStreamWaitEvent(m.st, m.ev_in, 0));
        DD_HIP_CHECK(hipStreamWaitEvent(m.st, m.ev_out, 0));
      }
    }
    ~OnStream() {
      if (direct) m.st = m.st_main = m.st_own;
    }
  };

  void forward_chunk(const float* camera, const float* lidar, const float* status, const float* noise, int B,
                     int steps, const Outs& o, hipStream_t caller, uint64_t scene0) {
    DD_HIP_CHECK(hipSetDevice(device));
    DD_TRACE("forward_chunk B=%d steps=%d caller=%p use_side=%d", B, steps, (void*)caller, (int)use_side);
    OnStream on(*this, caller);
    const bool heads = o.sem || o.ag_states || o.ag_labels;
    const uint64_t gen0 = generation;
    stage_inputs(camera, lidar, status, noise, B, scene0);
    DD_TRACE("staged");
    ensure_film(steps);
    DD_TRACE("film");
    if (generation != gen0) known_shapes.clear();
    const std::string key = std::to_string(B) + "/" + std::to_string(steps) + "/" + std::to_string(heads) + "/g" +
                            std::to_string(gemm_mode) + "/s" + std::to_string(schedule) +
                            (train ? (train_target ? "/train1" : "/train0") : "");
    if (use_graph && !profiling && known_shapes.count(key)) {
      if (graph_gen != generation || programs.size() > 8) {
        // an earlier replay may still run (on the caller's stream in direct mode): ev_out marks the last forward
        DD_HIP_CHECK(hipEventSynchronize(ev_out));
        drop_graphs();
        graph_gen = generation;
      }
      auto it = programs.find(key);
      DD_TRACE("graph key %s cached=%d", key.c_str(), (int)(it != programs.end()));
      if (it == programs.end()) {
        Program p;
        capture_program(B, steps, heads, p);
        DD_TRACE("captured %d segments (model %p)", p.segments, (void*)this);
        it = programs.emplace(key, std::move(p)).first;
      }
      run_program(it->second);
      DD_TRACE("launched");
    } else {
      // eager run (the first call for a shape allocates every buffer; later calls are captured)
      const uint64_t gen1 = generation;
      DD_TRACE("eager");
      forward_body(B, steps, heads);
      DD_TRACE("eager done");
      if (generation != gen1) known_shapes.clear();
      known_shapes.insert(key);
    }
    const int Q = cfg.num_modes, P = cfg.num_poses;
    DD_TRACE("copy out");
    copy_out(o.traj, "trajectory", (size_t)B * P * 3);
    copy_out(o.modes, "poses_reg", (size_t)B * Q * P * 3);
    copy_out(o.cls, "poses_cls", (size_t)B * Q);
    if (heads) {
      copy_out(o.sem, "bev_semantic_map", (size_t)B * 7 * (cfg.lidar_h / 2) * cfg.lidar_w);
      copy_out(o.ag_states, "agent_states", (size_t)B * 30 * 5);
      copy_out(o.ag_labels, "agent_labels", (size_t)B * 30);
    }
    if (train) {
      for (int l = 0; l < 2; ++l) {
        const std::string sf = "_s0l" + std::to_string(l);
        copy_out(o.reg_l[l], "reg" + sf, (size_t)B * Q * P * 3);
        copy_out(o.cls_l[l], "cls" + sf, (size_t)B * Q);
        if (train_target) copy_out(o.part_l[l], "train_part_l" + std::to_string(l), (size_t)B * 2);
      }
    }
    // ev_out marks the end of this forward on whichever stream it ran (dd_numerics_flags / dd_tap wait for it)
    DD_HIP_CHECK(hipEventRecord(ev_out, st));
    if (!on.direct) DD_HIP_CHECK(hipStreamWaitEvent(caller, ev_out, 0));
    if (profiling) collect();
  }
};

}  // namespace ddmi

// ====================================================================== C ABI
using ddmi::Model;

struct dd_handle {
  std::unique_ptr<Model> m;
  std::mutex mu;
};

static thread_local std::string g_last_error;

#ifdef DDMI_SEGV_TRACE
// diagnostic build only (DDMI_BUILD_VARIANT=dbg): a host backtrace on SIGSEGV (addr2line -e the library)
#include <execinfo.h>
#include <csignal>
#include <unistd.h>
static void ddmi_segv(int sig) {
  void* fr[64];
  const int n = backtrace(fr, 64);
  const char msg[] = "[ddmi] SIGSEGV backtrace:\n";
  (void)!write(2, msg, sizeof(msg) - 1);
  backtrace_symbols_fd(fr, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}
__attribute__((constructor)) static void ddmi_segv_install() { signal(SIGSEGV, ddmi_segv); }
#endif

template <class F>
static int guarded(F&& f) {
  try {
    f();
    g_last_error.clear();
    return DD_OK;
  } catch (const std::invalid_argument& e) {
    g_last_error = e.what();
    return DD_ERR_INVALID;
  } catch (const std::out_of_range& e) {
    g_last_error = std::string("out of range: ") + e.what();
    return DD_ERR_INVALID;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return DD_ERR_RUNTIME;
  } catch (...) {
    g_last_error = "unknown error";
    return DD_ERR_RUNTIME;
  }
}

extern "C" {

void dd_default_config(dd_config* c) {
  if (!c) return;
  c->abi_version = DD_ABI_VERSION;
  c->image_arch = 34;
  c->lidar_arch = 34;
  c->cam_h = 256;
  c->cam_w = 1024;
  c->lidar_h = 256;
  c->lidar_w = 256;
  c->lidar_channels = 1;
  c->num_modes = 20;
  c->num_poses = 8;
  c->trunc_timestep = 8;
  c->step_span = 20;
}

const char* dd_last_error(void) { return g_last_error.c_str(); }

int dd_create(const dd_config* cfg, const void* blob, size_t bytes, int device, dd_handle** out) {
  return guarded([&] {
    if (!cfg || !blob || !out) throw std::invalid_argument("dd_create: null argument");
    if (cfg->abi_version != DD_ABI_VERSION) throw std::invalid_argument("dd_create: ABI version mismatch");
    if (cfg->cam_h != 256 || cfg->cam_w != 1024 || cfg->lidar_h != 256 || cfg->lidar_w != 256)
      throw std::invalid_argument("dd_create: only the reference resolutions (256x1024 camera, 256x256 LiDAR) are supported");
    if (cfg->num_modes > 128 || cfg->num_poses > 16) throw std::invalid_argument("dd_create: too many modes/poses");
    auto h = std::make_unique<dd_handle>();
    h->m = std::make_unique<Model>(*cfg, blob, bytes, device);
    *out = h.release();
  });
}

int dd_forward_ex(dd_handle* h, const float* camera, const float* lidar, const float* status, const float* noise,
                  int B, int steps, const dd_outputs* outs, void* stream) {
  return guarded([&] {
    if (!h || !outs) throw std::invalid_argument("dd_forward_ex: null handle/outputs");
    std::lock_guard<std::mutex> lk(h->mu);
#ifdef DDMI_SEGV_TRACE
    signal(SIGSEGV, ddmi_segv);  // the HSA runtime may have replaced it since the library loaded
#endif
    Model::Outs o;
    o.traj = outs->trajectory;
    o.modes = outs->poses_reg;
    o.cls = outs->poses_cls;
    o.sem = outs->bev_semantic_map;
    o.ag_states = outs->agent_states;
    o.ag_labels = outs->agent_labels;
    h->m->forward(camera, lidar, status, noise, B, steps, o, static_cast<hipStream_t>(stream));
  });
}

int dd_forward_train(dd_handle* h, const float* camera, const float* lidar, const float* status, const float* noise,
                     const int* timesteps, const float* target_traj, int B, float cls_weight, float reg_weight,
                     const dd_train_outputs* outs, void* stream) {
  return guarded([&] {
    if (!h || !outs) throw std::invalid_argument("dd_forward_train: null handle/outputs");
    std::lock_guard<std::mutex> lk(h->mu);
    Model::Outs o;
    o.traj = outs->trajectory;
    o.sem = outs->bev_semantic_map;
    o.ag_states = outs->agent_states;
    o.ag_labels = outs->agent_labels;
    for (int l = 0; l < 2; ++l) {
      o.reg_l[l] = outs->poses_reg[l];
      o.cls_l[l] = outs->poses_cls[l];
    }
    h->m->forward_train(camera, lidar, status, noise, timesteps, target_traj, B, o, outs->loss, cls_weight, reg_weight,
                        static_cast<hipStream_t>(stream));
  });
}

int dd_forward(dd_handle* h, const float* camera, const float* lidar, const float* status, const float* noise, int B,
               int steps, float* out_traj, float* out_modes, float* out_cls, void* stream) {
  dd_outputs o;
  std::memset(&o, 0, sizeof(o));
  o.trajectory = out_traj;
  o.poses_reg = out_modes;
  o.poses_cls = out_cls;
  return dd_forward_ex(h, camera, lidar, status, noise, B, steps, &o, stream);
}

int dd_destroy(dd_handle* h) {
  return guarded([&] { delete h; });
}

int dd_set_profiling(dd_handle* h, int enable) {
  return guarded([&] {
    if (!h) throw std::invalid_argument("null handle");
    std::lock_guard<std::mutex> lk(h->mu);
    h->m->profiling = enable != 0;
  });
}

int dd_set_streams(dd_handle* h, int n) {
  return guarded([&] {
    if (!h) throw std::invalid_argument("null handle");
    if (n != 1 && n != 2) throw std::invalid_argument("dd_set_streams: n must be 1 or 2");
    std::lock_guard<std::mutex> lk(h->mu);  // a forward on another thread may be replaying a cached exec
    Model& m = *h->m;
    DD_HIP_CHECK(hipSetDevice(m.device));
    if (m.use_side == (n == 2)) return;
    DD_HIP_CHECK(hipStreamSynchronize(m.st));
    DD_HIP_CHECK(hipEventSynchronize(m.ev_out));  // a graph replayed on a caller's stream may still run
    m.drop_graphs();  // captured with the other topology
    m.use_side = n == 2;
  });
}

int dd_graph_info(dd_handle* h, int* programs, int* segments, int* multi_stream_execs) {
  return guarded([&] {
    if (!h) throw std::invalid_argument("null handle");
    std::lock_guard<std::mutex> lk(h->mu);
    int np = 0, ns = 0, nb = 0;
    for (auto& kv : h->m->programs) {
      ++np;
      ns += kv.second.segments;
      nb += kv.second.branched;
    }
    if (programs) *programs = np;
    if (segments) *segments = ns;
    if (multi_stream_execs) *multi_stream_execs = nb;
  });
}

int dd_graph_nodes(dd_handle* h, int* kernel_nodes, int* other_nodes) {
  return guarded([&] {
    if (!h) throw std::invalid_argument("null handle");
    std::lock_guard<std::mutex> lk(h->mu);
    int nk = 0, no = 0;
    for (auto& kv : h->m->programs) {
      nk += kv.second.kernel_nodes;
      no += kv.second.other_nodes;
    }
    if (kernel_nodes) *kernel_nodes = nk;
    if (other_nodes) *other_nodes = no;
  });
}

int dd_get_streams(dd_handle* h, int* n) {
  return guarded([&] {
    if (!h || !n) throw std::invalid_argument("null argument");
    std::lock_guard<std::mutex> lk(h->mu);
    *n = h->m->use_side ? 2 : 1;
  });
}

int dd_set_graph(dd_handle* h, int enable) {
  return guarded([&] {
    if (!h) throw std::invalid_argument("null handle");
    std::lock_guard<std::mutex> lk(h->mu);
    h->m->use_graph = enable != 0;
  });
}

int dd_set_gemm_mode(dd_handle* h, int mode) {
  return guarded([&] {
    if (!h) throw std::invalid_argument("null handle");
    if (mode != DD_GEMM_FP32 && mode != DD_GEMM_F16X3 && mode != DD_GEMM_BF16)
      throw std::invalid_argument("unknown gemm mode");
    std::lock_guard<std::mutex> lk(h->mu);
    h->m->gemm_mode = mode;
  });
}

int dd_set_schedule(dd_handle* h, int schedule) {
  return guarded([&] {
    if (!h) throw std::invalid_argument("null handle");
    if (schedule != DD_SCHED_TRUNCATED && schedule != DD_SCHED_VANILLA)
      throw std::invalid_argument("unknown schedule");
    std::lock_guard<std::mutex> lk(h->mu);
    h->m->schedule = schedule;
  });
}

int dd_get_gemm_mode(dd_handle* h, int* mode) {
  return guarded([&] {
    if (!h || !mode) throw std::invalid_argument("null argument");
    *mode = h->m->gemm_mode;
  });
}

int dd_numerics_flags(dd_handle* h, unsigned* flags, int clear) {
  return guarded([&] {
    if (!h || !flags) throw std::invalid_argument("null argument");
    std::lock_guard<std::mutex> lk(h->mu);
    Model& m = *h->m;
    DD_HIP_CHECK(hipSetDevice(m.device));
    DD_HIP_CHECK(hipStreamSynchronize(m.st));
    DD_HIP_CHECK(hipEventSynchronize(m.ev_out));  // a single-stream forward may have run on the caller's stream
    DD_HIP_CHECK(hipMemcpy(flags, m.num_flags, sizeof(unsigned), hipMemcpyDeviceToHost));
    if (clear) {
      // a megakernel's inter-workgroup wait failed or found a dirty counter: every forward has completed (the
      // synchronisations above), so the counters are re-zeroed here, ordered before any later forward
      if (*flags & (DD_NUM_SYNC_TIMEOUT_BIT | DD_NUM_SYNC_STATE_BIT))
        for (const char* name : {"tf_sync_cnt", "mk_scene_cnt"}) {
          auto it = m.bufs.find(name);
          if (it != m.bufs.end())
            DD_HIP_CHECK(hipMemsetAsync(it->second.first, 0, std::max<size_t>(it->second.second, 4) * sizeof(float),
                                        m.st_own));
        }
      DD_HIP_CHECK(hipMemsetAsync(m.num_flags, 0, sizeof(unsigned), m.st_own));
      DD_HIP_CHECK(hipStreamSynchronize(m.st_own));  // cleared before any later forward's kernels run
    }
  });
}

int dd_reset_stats(dd_handle* h) {
  return guarded([&] {
    if (!h) throw std::invalid_argument("null handle");
    std::lock_guard<std::mutex> lk(h->mu);
    h->m->collect();
    h->m->stats.clear();
  });
}

int dd_kernel_stats(dd_handle* h, const char* kernel, double* total_ms, long long* launches, double* flops) {
  return guarded([&] {
    if (!h || !kernel) throw std::invalid_argument("null argument");
    std::lock_guard<std::mutex> lk(h->mu);
    h->m->collect();
    auto it = h->m->stats.find(kernel);
    ddmi::KStat s;
    if (it != h->m->stats.end()) s = it->second;
    if (total_ms) *total_ms = s.ms;
    if (launches) *launches = s.n;
    if (flops) *flops = s.flops;
  });
}

int dd_kernel_bytes(dd_handle* h, const char* kernel, double* bytes) {
  return guarded([&] {
    if (!h || !kernel || !bytes) throw std::invalid_argument("null argument");
    std::lock_guard<std::mutex> lk(h->mu);
    h->m->collect();
    auto it = h->m->stats.find(kernel);
    *bytes = it != h->m->stats.end() ? it->second.bytes : 0.0;
  });
}

int dd_set_seed(dd_handle* h, unsigned long long seed) { return dd_set_seed_at(h, seed, 0); }

int dd_set_seed_at(dd_handle* h, unsigned long long seed, unsigned long long first_scene) {
  return guarded([&] {
    if (!h) throw std::invalid_argument("null handle");
    std::lock_guard<std::mutex> lk(h->mu);
    h->m->rng_seed = seed;
    h->m->rng_next = first_scene;
  });
}

int dd_tap(dd_handle* h, const char* name, float* dst, size_t count, size_t* actual, void* stream) {
  return guarded([&] {
    if (!h || !name) throw std::invalid_argument("null argument");
    std::lock_guard<std::mutex> lk(h->mu);
    Model& m = *h->m;
    float* src = nullptr;
    size_t n = 0;
    auto a = m.aliases.find(name);
    if (a != m.aliases.end()) {
      src = a->second;
      for (auto& kv : m.bufs)
        if (kv.second.first == src) n = kv.second.second;
    } else {
      auto it = m.bufs.find(name);
      if (it == m.bufs.end()) throw std::invalid_argument(std::string("unknown tap ") + name);
      src = it->second.first;
      n = it->second.second;
    }
    if (actual) *actual = n;
    if (dst && count) {
      DD_HIP_CHECK(hipEventSynchronize(m.ev_out));  // the last forward, on whichever stream it ran
      DD_HIP_CHECK(hipMemcpyAsync(dst, src, std::min(n, count) * sizeof(float), hipMemcpyDeviceToDevice,
                                  static_cast<hipStream_t>(stream)));
      DD_HIP_CHECK(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
    }
  });
}

}  // extern "C"
