// Sequential-VAE training-step engine: parameter layout, activation arena, and the
// forward / backward schedule of the executed training subgraph
// (sequential_vae.py:877-1212, 1537-1842; abstract_network.py:8-71).
//
// The chain is unrolled exactly as construct_network does (:934-975); the backward is
// written out by hand in reverse order (there is no autodiff here).  The T recognition
// ladders depend only on x, so they run as ONE batched launch per layer (blockIdx.z =
// step) with their parameters laid out at a constant per-step stride.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <string>
#include <vector>

#include "kernels.h"
#include "knobs.h"
#include "svae_hip.h"

namespace {

enum Init { INIT_ZERO = 0, INIT_NORMAL = 1, INIT_GLOROT = 2 };
enum Region { R_PHI = 0, R_THETA = 1, R_FROZEN = 2 };

struct PDesc {
  std::string name;
  std::vector<int> shape;
  int init;
  bool dead, zero_grad;
  int region, step;
  long long size, offset;
};

struct ConvL {
  int w = -1, beta = -1;  // desc indices (resolved to offsets later)
  long long ow = 0, obeta = 0;
  int cin = 0, cout = 0, stride = 1, hin = 0, hout = 0;
  bool tr = false;
};
struct FcL {
  int w = -1, beta = -1;
  long long ow = 0, obeta = 0;
  int nin = 0, nout = 0;
};
struct HeadL {
  int wm = -1, bm = -1, ws = -1, bs = -1;
  long long owm = 0, obm = 0, ows = 0, obs = 0;
  int nin = 0, d = 0, off = 0, src_level = 0;
};
struct InfStep {
  ConvL a[8], b[8];
  HeadL head[8];
};
struct EncStep {
  ConvL a[8], b[8];
  ConvL c;
  FcL fc;
};
struct GenStep {
  FcL split[8];
  FcL top;
  ConvL s2[8], s1[8];  // indexed by level
  int wout = -1, bout = -1, wratio = -1, bratio = -1;
  long long owout = 0, obout = 0, owratio = 0, obratio = 0;
  // stddevs_prediction (:1866-1875): conv2d_bn_lrelu layers + 1x1 conv
  ConvL sd[8];
  int wsd = -1, bsd = -1;
  long long owsd = 0, obsd = 0;
};

struct Geo {
  int B, H, W, C, L, T;
  int F[10], D[8], S[10];
  int Dz;
  bool interm;
  float c_first, prior, clipv, lo, hi, minh, maxh;
  bool bf16;
  // dtype = 2 (bf16x6): the fp32-accurate mode on bf16 MFMA.  bf16 is set too (shadows, the bf16
  // kernel families); split = operands as bf16 planes (opload.h split8): 3 planes / 6 products in the
  // gather-GEMMs (forward, input gradients), 2 planes / 3 products in the weight-GEMMs; fp32 storage
  // everywhere; shapes without a split kernel run the fp32 kernels
  bool split;
  // external generator (c_pixelvae, generator_pixelcnn sequential_vae.py:535, :1943-1971): steps
  // t >= Te run the caller's generator (the PixelCNN++ head); the engine runs their recognition
  // (z_t, KL_t) only and takes d loss / d x_hat_{Te-1} and d loss / d z_t back (svae_set_external_grads)
  int Te;
  bool share_theta, share_phi;
  bool plc, plc_reg;          // predict_latent_code (+ _with_regularization)
  unsigned long long unreg;   // steps without a KL term
  // chain variants
  bool uniform;               // use_uniform_prior
  bool noisy, pgn, imp;       // add_noise_to_chain, predict_generator_noise, improvement loss
  float nstd[64];             // noise_stddevs
  float sd_max, lp_coef;      // predict_generator_stddev_max, latent_pred_loss_coeff
  int sd_nl, sd_F[9];         // stddev network: layers and channels (sd_F[0] = C)
  // weight of step t's KL term relative to reg * c_first (compute_and_accumulate_loss :1154-1172)
  float kl_on(int t) const {
    if ((unreg >> t) & 1ULL) return 0.f;
    return (!plc || plc_reg || t == 0) ? 1.f : 0.f;
  }
};

bool make_geo(const svae_config* c, Geo& g, std::string& err) {
  if (!c) { err = "null config"; return false; }
  g.B = c->batch; g.H = c->height; g.W = c->width; g.C = c->channels;
  g.L = c->levels; g.T = c->mc_steps;
  if (g.L < 2 || g.L > 7) { err = "levels must be in [2,7]"; return false; }
  if (g.T < 1 || g.T > 64) { err = "mc_steps must be in [1,64]"; return false; }
  if (g.H != g.W) { err = "square images only (sequential_vae.py:1701)"; return false; }
  if (g.C < 1 || g.C > 3) { err = "channels must be 1..3"; return false; }
  if (g.B < 2) { err = "batch >= 2 required (training BatchNorm over the batch)"; return false; }
  if (g.B > 256) { err = "batch <= 256 per context (split-latent backward keeps 64 rows per wave in registers)"; return false; }
  for (int i = 0; i < g.L + 2; ++i) {
    g.F[i] = c->filter_sizes[i];
    if (g.F[i] <= 0) { err = "filter_sizes must be positive"; return false; }
  }
  if (g.F[0] != g.C) { err = "filter_sizes[0] must equal channels"; return false; }
  g.Dz = 0;
  for (int i = 0; i < g.L; ++i) {
    g.D[i] = c->latent_dims[i];
    if (g.D[i] <= 0 || g.D[i] > 32) { err = "latent_dims must be in [1,32]"; return false; }
    g.Dz += g.D[i];
  }
  for (int i = 0; i <= g.L; ++i) {
    g.S[i] = g.H >> i;
    if ((g.S[i] << i) != g.H || g.S[i] < 1) { err = "image size must be divisible by 2^levels"; return false; }
  }
  for (int i = 1; i <= g.L; ++i)
    if (g.F[i] % 4) { err = "filter_sizes[1..L] must be multiples of 4"; return false; }
  if (g.F[g.L + 1] % 4) { err = "filter_sizes[L+1] must be a multiple of 4"; return false; }
  g.interm = c->intermediate_reconstruction != 0;
  g.c_first = c->first_step_loss_coeff;
  g.prior = c->latent_prior_stddev;
  g.clipv = c->latent_mean_clip;
  g.lo = c->range_lo; g.hi = c->range_hi;
  g.minh = c->min_highway; g.maxh = c->max_highway;
  if (c->dtype < 0 || c->dtype > 2) { err = "dtype must be 0 (fp32), 1 (bf16 MFMA) or 2 (bf16x6 split)"; return false; }
  g.bf16 = c->dtype == 1 || c->dtype == 2;
  g.split = c->dtype == 2;
  g.share_theta = c->share_theta != 0;
  g.share_phi = c->share_phi != 0;
  g.Te = g.T;
  if (c->external_generator_from != 0) {
    if (c->external_generator_from < 1 || c->external_generator_from >= g.T) {
      err = "external_generator_from must be in [1, mc_steps)";
      return false;
    }
    if (c->predict_latent_code || c->add_noise_to_chain || c->add_improvement_maximization_loss) {
      err = "external_generator_from: no Latent InfoMax / chain noise / improvement loss";
      return false;
    }
    g.Te = c->external_generator_from;
  }
  g.plc = c->predict_latent_code != 0;
  g.plc_reg = c->predict_latent_code_with_regularization != 0;
  g.unreg = (unsigned long long)c->unregularized_steps_mask[0] | ((unsigned long long)c->unregularized_steps_mask[1] << 32);
  g.uniform = c->use_uniform_prior != 0;
  g.noisy = c->add_noise_to_chain != 0;
  g.pgn = c->predict_generator_noise != 0;
  g.imp = c->add_improvement_maximization_loss != 0;
  g.sd_max = c->predict_generator_stddev_max;
  g.lp_coef = c->latent_pred_loss_coeff;
  for (int t = 0; t < 64; ++t) g.nstd[t] = g.noisy ? c->noise_stddevs[t] : 0.f;
  g.sd_nl = 0;
  g.sd_F[0] = g.C;
  if (g.pgn) {
    // stddevs = 0 without chain noise (:1664-1671) and the NLL would take log(0)
    if (!g.noisy) { err = "predict_generator_noise needs add_noise_to_chain"; return false; }
    g.sd_nl = c->stddev_layers;
    if (g.sd_nl < 1 || g.sd_nl > 8) { err = "stddev_layers must be in [1,8]"; return false; }
    for (int i = 0; i < g.sd_nl; ++i) {
      g.sd_F[i + 1] = c->stddev_filter_sizes[i];
      if (g.sd_F[i + 1] < 1 || g.sd_F[i + 1] > 8) { err = "stddev_filter_sizes must be in [1,8]"; return false; }
    }
    if (!(g.sd_max > 0.f)) { err = "predict_generator_stddev_max must be > 0"; return false; }
    if (g.H % 4) { err = "predict_generator_noise needs an image size divisible by 4"; return false; }
  }
  return true;
}

// tf.contrib.layers default scope naming (Conv, Conv_1, ..., BatchNorm_3, fully_connected_2)
struct Scope {
  std::string prefix;
  std::vector<PDesc>* out;
  int region, step;
  int n_conv = 0, n_convt = 0, n_bn = 0, n_fc = 0;
  static std::string nm(const char* k, int i) { return i == 0 ? std::string(k) : std::string(k) + "_" + std::to_string(i); }
  int add(const std::string& layer, const char* suffix, std::vector<int> shape, int init, bool dead, bool zg) {
    PDesc d;
    d.name = prefix + "/" + layer + "/" + suffix;
    d.shape = shape;
    d.init = init;
    d.dead = dead;
    d.zero_grad = zg || dead;
    d.region = (dead || zg) ? R_FROZEN : region;
    d.step = step;
    d.size = 1;
    for (int s : shape) d.size *= s;
    d.offset = -1;
    out->push_back(d);
    return (int)out->size() - 1;
  }
  ConvL conv_bn(int cin, int cout, int stride, int hin, bool tr, bool dead = false) {
    ConvL c;
    std::string ln = tr ? nm("Conv2d_transpose", n_convt++) : nm("Conv", n_conv++);
    if (tr) c.w = add(ln, "weights", {4, 4, cout, cin}, INIT_NORMAL, dead, false);
    else c.w = add(ln, "weights", {4, 4, cin, cout}, INIT_NORMAL, dead, false);
    add(ln, "biases", {cout}, INIT_ZERO, dead, true);
    c.beta = add(nm("BatchNorm", n_bn++), "beta", {cout}, INIT_ZERO, dead, false);
    c.cin = cin; c.cout = cout; c.stride = stride; c.hin = hin; c.tr = tr;
    c.hout = tr ? hin * stride : hin / stride;
    return c;
  }
  FcL fc_bn(int nin, int nout, bool dead = false) {
    FcL f;
    std::string ln = nm("fully_connected", n_fc++);
    f.w = add(ln, "weights", {nin, nout}, INIT_NORMAL, dead, false);
    add(ln, "biases", {nout}, INIT_ZERO, dead, true);
    f.beta = add(nm("BatchNorm", n_bn++), "beta", {nout}, INIT_ZERO, dead, false);
    f.nin = nin; f.nout = nout;
    return f;
  }
  void fc(int nin, int nout, int& w, int& b) {
    std::string ln = nm("fully_connected", n_fc++);
    w = add(ln, "weights", {nin, nout}, INIT_GLOROT, false, false);
    b = add(ln, "biases", {nout}, INIT_ZERO, false, false);
  }
  void conv_plain(int k, int cin, int cout, int& w, int& b) {  // conv2d without BN (default xavier init)
    std::string ln = nm("Conv", n_conv++);
    w = add(ln, "weights", {k, k, cin, cout}, INIT_GLOROT, false, false);
    b = add(ln, "biases", {cout}, INIT_ZERO, false, false);
  }
  void convt_plain(int cin, int cout, int& w, int& b) {
    std::string ln = nm("Conv2d_transpose", n_convt++);
    w = add(ln, "weights", {4, 4, cout, cin}, INIT_GLOROT, false, false);
    b = add(ln, "biases", {cout}, INIT_ZERO, false, false);
  }
};

struct Model {
  Geo g;
  std::vector<PDesc> descs;
  std::vector<InfStep> inf;
  std::vector<EncStep> enc;
  std::vector<GenStep> gen;
  long long n_total = 0, n_live = 0, phi_stride = 0;
  // gradient buckets in backward completion order: theta of step t = [step_lo[t], step_hi[t]),
  // all recognition weights = [0, phi_hi) (parallel.step_buckets restates these)
  std::vector<long long> step_lo, step_hi;
  long long phi_hi = 0;

  // Public table (what svae_param_layout reports and the caller's buffers hold).  Without
  // weight sharing it is descs itself.  With sharing the engine still runs on a private
  // "virtual" copy in the inhomogeneous layout above (descs, offsets): every step's scope gets
  // its own copy of the shared tensor (broadcast from the public buffer before the forward),
  // and each public gradient is the fixed-order sum of its copies' gradients after the
  // backward -- exactly TF's gradient of a variable used by several steps.
  std::vector<PDesc> pub;
  std::vector<int> vpub;  // descs index -> pub index
  long long p_total = 0, p_live = 0;
  long long p_phi_end = 0;  // public recognition variables occupy [0, p_phi_end)
  bool shared = false;

  long long off(int idx) const { return idx < 0 ? -1 : descs[idx].offset; }

  // TF scope of a virtual tensor under variable sharing (sequential_vae.py:1573-1577,1683-1687,1757-1761)
  std::string public_name(const std::string& n) const {
    auto swap = [&](const char* pre, const char* to, int min_step, std::string& out) {
      const size_t lp = strlen(pre);
      if (n.compare(0, lp, pre) != 0) return false;
      const size_t sl = n.find('/', lp);
      if (sl == std::string::npos || atoi(n.c_str() + lp) < min_step) return false;
      out = std::string(to) + n.substr(sl);
      return true;
    };
    std::string o;
    if (g.share_phi && swap("phi/inference_step_", "phi/inference_network", g.plc ? 1 : 0, o)) return o;
    if (g.share_theta && swap("theta/generative_encoder_step_", "theta/generative_encoder_network", 0, o)) return o;
    if (g.share_theta && swap("theta/generative_step_", "theta/generative_network", 1, o)) return o;
    return n;
  }

  void build_public() {
    shared = g.share_theta || g.share_phi;
    std::vector<int> order(descs.size());
    for (size_t i = 0; i < descs.size(); ++i) order[i] = (int)i;
    std::sort(order.begin(), order.end(), [&](int a, int b) { return descs[a].offset < descs[b].offset; });
    std::map<std::string, int> by_name;
    vpub.assign(descs.size(), -1);
    pub.clear();
    for (int i : order) {
      const std::string pn = public_name(descs[i].name);
      auto it = by_name.find(pn);
      if (it == by_name.end()) {
        PDesc d = descs[i];
        d.name = pn;
        by_name[pn] = (int)pub.size();
        vpub[i] = (int)pub.size();
        pub.push_back(d);
      } else {
        vpub[i] = it->second;
      }
    }
    // first-appearance order keeps the live tensors ahead of the frozen tail
    long long o = 0;
    bool frozen_seen = false;
    p_live = -1;
    for (auto& d : pub) {
      const bool fz = d.region == R_FROZEN;
      if (fz && !frozen_seen) { frozen_seen = true; p_live = o; }
      o = (o + 63) / 64 * 64;
      d.offset = o;
      o += d.size;
      o = (o + 63) / 64 * 64;
    }
    p_total = o;
    if (p_live < 0) p_live = o;
    p_phi_end = 0;
    for (auto& d : pub)
      if (d.region == R_PHI) p_phi_end = std::max(p_phi_end, d.offset + d.size);
    p_phi_end = (p_phi_end + 63) / 64 * 64;
  }

  void build() {
    const int L = g.L;
    const int* F = g.F;
    const int* S = g.S;
    inf.assign(g.T, InfStep());
    enc.assign(g.T, EncStep());
    gen.assign(g.T, GenStep());
    for (int t = 0; t < g.T; ++t) {
      // phi/inference_step_t  (sequential_vae.py:1579-1609)
      Scope sc{"phi/inference_step_" + std::to_string(t), &descs, R_PHI, t};
      InfStep& I = inf[t];
      int cin = F[0];
      int off = 0;
      for (int lvl = 0; lvl < L - 1; ++lvl) {
        I.a[lvl] = sc.conv_bn(cin, F[lvl + 1], 2, S[lvl], false);
        I.b[lvl] = sc.conv_bn(F[lvl + 1], F[lvl + 1], 1, S[lvl + 1], false);
        HeadL& h = I.head[lvl];
        h.nin = S[lvl + 1] * S[lvl + 1] * F[lvl + 1];
        h.d = g.D[lvl];
        h.off = off;
        h.src_level = lvl;
        off += h.d;
        sc.fc(h.nin, h.d, h.wm, h.bm);
        sc.fc(h.nin, h.d, h.ws, h.bs);
        cin = F[lvl + 1];
      }
      sc.conv_bn(F[L - 1], F[L - 1], 2, S[L - 1], false, /*dead=*/true);   // :1602 (dead)
      sc.fc_bn(S[L] * S[L] * F[L - 1], F[L], /*dead=*/true);              // :1605 (dead)
      HeadL& h = I.head[L - 1];                                            // :1607-1609 read `ladder`
      h.nin = S[L - 1] * S[L - 1] * F[L - 1];
      h.d = g.D[L - 1];
      h.off = off;
      h.src_level = L - 2;
      sc.fc(h.nin, h.d, h.wm, h.bm);
      sc.fc(h.nin, h.d, h.ws, h.bs);
      // theta/generative_encoder_step_t  (:1764-1775); steps t >= Te have no encoder / generator here
      if (t >= g.Te) continue;
      if (t >= 1) {
        Scope se{"theta/generative_encoder_step_" + std::to_string(t), &descs, R_THETA, t};
        EncStep& E = enc[t];
        cin = F[0];
        for (int lvl = 0; lvl < L - 1; ++lvl) {
          E.a[lvl] = se.conv_bn(cin, F[lvl + 1], 2, S[lvl], false);
          E.b[lvl] = se.conv_bn(F[lvl + 1], F[lvl + 1], 1, S[lvl + 1], false);
          cin = F[lvl + 1];
        }
        E.c = se.conv_bn(F[L - 1], F[L - 1], 2, S[L - 1], false);
        E.fc = se.fc_bn(S[L] * S[L] * F[L - 1], F[L]);
      }
      // theta/generative_step_t  (:1689-1727, split_latent :1796-1806)
      Scope sg{"theta/generative_step_" + std::to_string(t), &descs, R_THETA, t};
      GenStep& G = gen[t];
      for (int i = 0; i < L - 1; ++i) G.split[i] = sg.fc_bn(g.D[i], S[i + 1] * S[i + 1] * F[i + 1]);
      G.split[L - 1] = sg.fc_bn(g.D[L - 1], F[L + 1]);
      G.top = sg.fc_bn(F[L + 1] + (t >= 1 ? F[L] : 0), S[L] * S[L] * F[L]);
      cin = F[L];
      for (int lvl = L - 2; lvl >= 0; --lvl) {
        G.s2[lvl] = sg.conv_bn(cin, F[lvl + 1], 2, S[lvl + 2], true);
        G.s1[lvl] = sg.conv_bn(2 * F[lvl + 1], F[lvl + 1], 1, S[lvl + 1], true);
        cin = F[lvl + 1];
      }
      sg.convt_plain(F[1], g.C, G.wout, G.bout);
      if (t >= 1) sg.convt_plain(F[1], 1, G.wratio, G.bratio);
      // stddevs_prediction, created after the output / ratio conv-T (:1734-1735, :1866-1870)
      for (int l = 0; l < g.sd_nl; ++l) G.sd[l] = sg.conv_bn(g.sd_F[l], g.sd_F[l + 1], 1, g.H, false);
      if (g.sd_nl) sg.conv_plain(1, g.sd_F[g.sd_nl], 1, G.wsd, G.bsd);
    }
    // offsets: live phi blocks (uniform per-step stride), live theta blocks, frozen tail.
    // Every tensor starts on a 64-float (256 B) boundary: the GEMM kernels stage weights
    // with 16-byte vector loads, and rows of NHWC tiles stay line-aligned.
    auto align = [](long long v) { return (v + 63) / 64 * 64; };
    long long o = 0;
    step_lo.assign(g.T, 0);
    step_hi.assign(g.T, 0);
    for (int r = 0; r < 3; ++r) {
      for (int t = 0; t < g.T; ++t) {
        long long start = o;
        for (auto& d : descs)
          if (d.region == r && d.step == t) {
            o = align(o);
            d.offset = o;
            o += d.size;
          }
        o = align(o);
        if (r == R_PHI && t == 0) phi_stride = o - start;
        if (r == R_THETA) { step_lo[t] = start; step_hi[t] = o; }
      }
      if (r == R_PHI) phi_hi = o;
      if (r == R_THETA) n_live = o;
    }
    n_total = o;
    build_public();
    auto rc = [&](ConvL& c) { c.ow = off(c.w); c.obeta = off(c.beta); };
    auto rf = [&](FcL& f) { f.ow = off(f.w); f.obeta = off(f.beta); };
    for (int t = 0; t < g.T; ++t) {
      for (int l = 0; l < L - 1; ++l) { rc(inf[t].a[l]); rc(inf[t].b[l]); rc(enc[t].a[l]); rc(enc[t].b[l]); rc(gen[t].s2[l]); rc(gen[t].s1[l]); }
      for (int l = 0; l < L; ++l) {
        HeadL& h = inf[t].head[l];
        h.owm = off(h.wm); h.obm = off(h.bm); h.ows = off(h.ws); h.obs = off(h.bs);
        rf(gen[t].split[l]);
      }
      rc(enc[t].c); rf(enc[t].fc); rf(gen[t].top);
      GenStep& G = gen[t];
      G.owout = off(G.wout); G.obout = off(G.bout); G.owratio = off(G.wratio); G.obratio = off(G.bratio);
      for (int l = 0; l < g.sd_nl; ++l) rc(G.sd[l]);
      G.owsd = off(G.wsd); G.obsd = off(G.bsd);
    }
  }
};

const char* g_err_noctx = "";
thread_local std::string g_tls_err;

}  // namespace

// the context-free ops of other translation units (pcnn.hip) report through svae_last_error(NULL)
void svae_tls_error(const std::string& msg) { g_tls_err = msg; }

// ============================================================================
// engine context
// ============================================================================
struct Defer;
struct View {
  float* p = nullptr;
  int ld = 0;
  long long gs = 0;
  int bf = 0;  // stored as bf16 (element ld / gs unchanged): only bf16 GEMMs read it (opload.h)
  const Defer* dfr = nullptr;  // the tensor's BN apply was deferred to the side stream (SVAE_FOLD)
};

struct BNS {  // per-layer BN statistics (mean / invstd), groups x C
  float* mean = nullptr;
  float* invstd = nullptr;
};

// Launch probe: times every launch of one bf16 GEMM instance with an event pair on the
// launch stream and accumulates its algorithmic FLOPs (bench.py's roofline line).
struct Probe {
  int kid = KID_NONE;
  std::vector<hipEvent_t> ev;  // pairs
  int used = 0;                // pairs recorded
  long long launches = 0;
  double flops = 0;
};

struct svae_ctx {
  Probe probe;
  // ---- backward: weight gradients on a side stream (overlap the BN / dgrad chain) ----
  static constexpr int NR = 6;  // "ready" events (re-recorded in turn: each is waited on right after its record)
  bool side = false;
  hipStream_t st2 = nullptr;
  // SVAE_SIDE2=1: a second weight-gradient stream; the conv weight-GEMMs alternate between st2 and st2b
  // (own split slab each).  A wgrad launch holds ~64 CUs, so two run side by side where one left
  // the rest of the machine to latency-bound main-stream kernels.  Every ordering point that
  // follows "the side stream" first merges st2b into st2 (side_merge).
  hipStream_t st2b = nullptr;
  float* slab2b = nullptr;
  hipEvent_t ev_merge = nullptr;
  unsigned side_rr = 0;
  bool side_pin = false;  // the closure being handed over uses shared scratch: st2 only
  hipStream_t st3 = nullptr;  // split-latent FCs (fwd up front, bwd per level): no weight-GEMM queue ahead
  hipEvent_t ev_dz = nullptr, ev_j3 = nullptr;
  // recognition backward overlapped with the chain backward: groups of rec_group steps on st4 as soon
  // as their dz_t are final (0 = one batched launch per layer after the chain)
  hipStream_t st4 = nullptr;
  hipEvent_t ev_j4 = nullptr;
  float* slab4 = nullptr;
  int rec_group = 0;
  // forward recognition split (SVAE_REC_SPLIT=1): step 0's ladder on the main stream, the batched
  // ladders of steps 1..T-1 on st4 (own split slab), overlapping the chain's step 0
  int rec_split = 0;
  hipEvent_t ev_rs = nullptr, ev_rs2 = nullptr;
  float* slab2 = nullptr;
  // BN-backward outputs read by the side stream's weight GEMMs: every one of a backward pass gets
  // its own region of these arenas (bump-allocated, reset per pass), so the main stream never
  // waits for the side stream to release a buffer -- the previous pass's side-stream work is
  // joined into the caller's stream at its end (svae_backward).  A cross-stream wait costs the
  // main stream a 5-7 us dispatch gap even when already satisfied (profiles/r02_v4_streams.txt).
  float* dpre_arena = nullptr;
  float* idpre_arena = nullptr;
  long long dpre_cap = 0, dpre_off = 0, idpre_cap = 0, idpre_off = 0;
  hipEvent_t ev_ready[NR] = {}, ev_iready[NR] = {};
  hipEvent_t ev_drain = nullptr;  // arena overflow: the side stream drained before reuse
  hipEvent_t ev_da_ready = nullptr, ev_da_free = nullptr, ev_start = nullptr, ev_join = nullptr;
  int ring_pos = 0, iring_pos = 0;
  // batched hand-over to the side stream (SVAE_SIDE_BATCH = k > 1): weight-gradient work is queued
  // and enqueued on st2 behind ONE main-stream event per k layers (and at every split-latent
  // hand-over, which shares that event with st3).  Each event record on the main stream is a
  // marker packet that drains the queue before the next dispatch (a 4-10 us gap per record).
  std::vector<std::function<int()>> side_q;
  int side_batch = 1;
  bool side2 = false;  // SVAE_SIDE2 (read at svae_create, before the arena plan)
  bool fc_fuse = true;  // E.fc BN-backward sums fused into the top FC's input gradient (SVAE_BWFUSE_FC)
  // SVAE_FOLD=1: the forward BN apply of a layer whose only main-stream consumer is a wave-split halo
  // gather runs on st2 (for the backward's weight gradients), and the gather stages act(bn_y(pre))
  // itself (FwdArgs::ain): the apply leaves the critical path.  Bitwise the same tensors.
  bool fold = false;
  static constexpr int NFOLD = 32;
  hipEvent_t ev_fold[NFOLD] = {};
  int fold_pos = 0;
  bool fold_used = false;
  hipEvent_t ev_fold_join = nullptr;
  static constexpr int NF = 4;
  hipEvent_t ev_flush[NF] = {};
  int flush_pos = 0;
  // backward step hook (data-parallel bucketed all-reduce): called on the host after the
  // backward of chain step t is enqueued, with the side stream ordered after all of that step's
  // work on both streams; t = -1 after the whole backward (streams joined)
  // split-latent FCs on the side stream: forward for all steps up front (they depend only on z),
  // backward per level off the critical path, reading ring copies of dcat / dtop
  // their inputs (dcat, dtop) and the output layer's da: per-pass regions as for dpre
  float* dcat_arena = nullptr;
  float* dtop_arena = nullptr;
  float* da_base = nullptr;  // [T][B*H*W][C+1]: step t's da (the output weight gradient reads it on st2)
  long long dcat_cap = 0, dcat_off = 0, dtop_cap = 0, dtop_off = 0;
  hipEvent_t ev_drain3 = nullptr;
  hipEvent_t ev_aux = nullptr, ev_aux2 = nullptr;
  hipEvent_t ev_sfc[64] = {};
  svae_step_hook hook = nullptr;
  void* hook_user = nullptr;
  hipEvent_t ev_hook = nullptr;     // (system-scope release: a collective's peers read the bucket)
  hipEvent_t ev_hook_dev = nullptr; // the same hand-over without a hook (fused Adam only): device scope
  float* cs_part = nullptr;  // output-bias column-sum partials (side stream)
  bool generative = false;   // svae_generate: chain on caller / prior latents, no recognition
  float* zero_img = nullptr; // [B,H,W,C] zeros: reconstruction target of the generative chain
  int wg_path = 2;  // bf16 weight-GEMM: 0 tap-merged kernel only, 2 halo kernel where it qualifies
  Model m;
  std::string err;
  int device = 0;
  float* P = nullptr;   // params the engine reads (the caller's, or the virtual copy under sharing)
  float* Gr = nullptr;  // grads the engine writes (likewise)
  // weight sharing (Model::shared): the caller's public buffers and the virtual copies
  float* Ppub = nullptr;
  float* Gpub = nullptr;
  float* Pv = nullptr;
  float* Gv = nullptr;
  long long* share_seg = nullptr;   // [nseg][3] virtual offset, public offset, size (broadcast)
  long long* share_tab = nullptr;   // [ntab][4] public offset, size, first copy, copies (gather-sum)
  long long* share_cp = nullptr;    // virtual offsets of the copies
  int share_nseg = 0, share_ntab = 0;
  float* adam_m = nullptr;
  float* adam_v = nullptr;
  char* arena = nullptr;
  size_t arena_bytes = 0, arena_used = 0;
  hipStream_t st = 0;
  unsigned long long rng_offset = 0;
  float reg = 1.f;

  // ---------- inference (batched over T, group stride = one step's slab) ----------
  float *inf_pre_a[8], *inf_act_a[8], *inf_pre_b[8], *inf_act_b[8];
  long long inf_gs[8];  // elements per step at level lvl
  BNS inf_bn_a[8], inf_bn_b[8];
  float *head_part, *mu, *sig, *z, *eps_buf, *kl_img, *kl_coef;
  int head_nsplit;
  // ---------- chain (per step) ----------
  struct StepBufs {
    float *enc_pre_a[8], *enc_act_a[8], *enc_pre_b[8], *enc_act_b[8];
    BNS enc_bn_a[8], enc_bn_b[8];
    float *enc_c_pre, *enc_c_act, *encfc_pre;
    BNS enc_bn_c, enc_bn_fc;
    float* split_mean[8];
    float* split_inv[8];
    float *top_cat, *top_pre, *top_act;
    int ktop;
    BNS top_bn;
    float *s2_pre[8], *cat[8], *s1_pre[8], *s1_act[8];
    BNS s2_bn[8], s1_bn[8];
    float *wpack, *a_out, *xhat, *rec_part, *rec_img, *stats;
    void* wpack_h;  // bf16 copy of wpack (NK [tap][C+1][F1]) for the bf16 output conv-T
    // chain variants: training_samples[t] (when noise perturbs it), predicted stddevs and the
    // stddev network's saved tensors
    bool has_sample;
    float *sample, *sd;
    float *sd_pre[8], *sd_act[8], *sd_mean[8], *sd_inv[8];
  };
  std::vector<StepBufs> sb;
  int out_nblk = 0;
  // ---------- backward scratch ----------
  float *dx[2], *da, *dcur, *dnext, *dpre, *dcat, *dtop, *denc_c, *denc_fc;
  float* denc[8];
  float *sfc_part, *dz, *dhead;
  float *idb, *ida, *idpre;  // inference bwd: [T] x max level slab
  float* slab;
  // chain variants: chain noise, stddev-network backward scratch, improvement loss
  const float* noise_in = nullptr;   // caller's N(0,1) [T,B,H,W,C] (svae_set_chain_noise)
  const float* noise_used = nullptr;
  float* noise_buf = nullptr;
  float *sd_d[2] = {}, *sd_dpre = nullptr, *sd_wpart = nullptr, *sd_sums = nullptr, *dmle = nullptr;
  double* sd_part = nullptr;
  float *dseed = nullptr, *imp_img = nullptr, *kl_zero = nullptr;
  bool imp_pass = false;             // svae_backward_imp: seeds from the improvement loss only
  // external generator steps (Geo::Te < T): the caller's d loss / d x_hat_{Te-1} [B,H,W,C] and
  // d loss / d z [T,B,Dz] (rows t >= Te) for the next backward (svae_set_external_grads, one-shot)
  const float* ext_dx = nullptr;
  const float* ext_dz = nullptr;
  // bf16 mode: BN-backward outputs (dpre) stored as bf16 -- their only consumers, the dgrad and
  // wgrad GEMMs, round them identically while staging (opload.h)
  int dbf = 0;
  int abf = 0;  // bf16 mode: the post-activation tensors read only by bf16 GEMMs are stored as bf16
  // bf16 mode: every conv layer's pre-BN output is stored as bf16 by its GEMM epilogue (the BN statistics
  // of the stored values); the BN apply / backward passes and the fused backward-BN epilogues widen it
  int pbf = 0;
  // bf16 mode: the decoder concat buffers [s2 output | split latent] are stored as bf16 -- read only by the
  // s1 gather and weight-GEMM (which round them the same way) and, for the s2 BN backward, by act' (the
  // sign of y, which bf16 rounding keeps): bitwise the fp32-stored step (SVAE_CAT_F32=1)
  int cbf = 0;
  // conv BN statistics finalised by the producing halo_kw launch's last block (common.h BnFin): the apply
  // passes read mean / invstd (bit 0, forward) or a, b (bit 1, the fused backward sums) instead of every
  // block finalising its channels (SVAE_BN_LAF; bitwise, but off: 9.5 % / 16 % slower, profiles/r04_laf_ab.txt)
  int laf = 0;
  // BN statistics finalised by one small launch per layer and pass (SVAE_BN_FIN) instead of by every apply
  // block from the accumulator shards
  int bnfin = 0;
  float* Gimp_pub = nullptr;         // caller's improvement-loss gradient (svae_bind_imp)
  float* Gimp_v = nullptr;           // its virtual copy under weight sharing
  // BN statistics: fixed-point column accumulators (common.h stat_put), one region per BN
  // instance of a pass, handed out in launch order and zeroed once per pass (acc_reset)
  u64* bnacc = nullptr;
  long long bnacc_cap = 0, bnacc_used = 0, bnacc_hw = -1;
  void *wN = nullptr, *wT = nullptr;   // bf16 weight shadows (dtype=1; dtype=2: nsp planes of wplane elements each)
  int nsp = 1;                         // shadow planes (3 in the split mode)
  long long wplane = 0;
  void *tiles_d = nullptr, *offs_d = nullptr;
  int ntiles = 0;
  std::vector<long long> tile_off;  // tiles sorted by tensor offset: each tile's tensor offset
  long long fresh = 0;  // live elements whose bf16 shadows an Adam update refreshed since the last forward
  // split mode: the fp16 weight planes' exponent per 64-float block (common.h h16_pair), the GEMM weight
  // tensors {offset, elements, R, Cc} it is derived over, and the Adam overflow flag (wexp_fixup)
  int* wtab = nullptr;
  long long* winfo_d = nullptr;
  int nwinfo = 0;
  int* wovf = nullptr;
  // svae_backward_adam: clip + Adam of each step's bucket inside the backward (side stream)
  bool fa_on = false;
  float fa_lr = 0.f, fa_clip = 0.f;
  long long fa_step = 0;
  long long slab_cap;
  const float* x_in = nullptr;
  const float* tgt_in = nullptr;
  const float* eps_in = nullptr;
  const float* eps_used = nullptr;
  float* reg_host = nullptr;  // [T] kl coefficients staged on the host (set_small copies them by value)
  int dbg_stop_step = -1, dbg_stop_lvl = -1, dbg_stop_lvl2 = -1;
  float* dbg_last = nullptr;
  bool counting = false;

  float* alloc(long long n) {
    size_t bytes = ((size_t)n * sizeof(float) + 255) & ~(size_t)255;
    if (counting) {
      arena_used += bytes;
      return (float*)(uintptr_t)256;
    }
    if (arena_used + bytes > arena_bytes) return nullptr;
    float* p = (float*)(arena + arena_used);
    arena_used += bytes;
    return p;
  }
};

static int fail(svae_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  else g_tls_err = msg;
  return code;
}

#define HIPCHK(ctx, x)                                                                       \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) return fail(ctx, SVAE_EHIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

// BN accumulator regions: acc_reset zeroes what the previous passes used (all of it the
// first time) with one memset; acc_take hands out the next region of n words
static int acc_reset(svae_ctx* c) {
  const long long n = c->bnacc_hw < 0 ? c->bnacc_cap : c->bnacc_hw;
  if (n > 0) HIPCHK(c, hipMemsetAsync(c->bnacc, 0, (size_t)n * sizeof(u64), c->st));
  c->bnacc_used = 0;
  c->bnacc_hw = 0;
  return 0;
}
static u64* acc_take(svae_ctx* c, long long n) {
  if (c->bnacc_used + n > c->bnacc_cap) return nullptr;
  u64* p = c->bnacc + c->bnacc_used;
  c->bnacc_used += (n + 31) / 32 * 32;
  if (c->bnacc_used > c->bnacc_hw) c->bnacc_hw = c->bnacc_used;
  return p;
}

// the accumulators of one BN instance: groups x 4C words per shard, shards by row-block count
struct AccR {
  u64* p = nullptr;
  long long gs = 0, sh = 0;
  int nsh = 1;
};
static AccR acc_bn(svae_ctx* c, int groups, int C, long long rowblocks) {
  AccR r;
  r.nsh = bn_acc_shards(rowblocks, c->m.g.split ? 32 : 16);
  r.gs = 4LL * C;
  r.sh = ((long long)groups * r.gs + 31) / 32 * 32;
  r.p = acc_take(c, r.sh * r.nsh);
  return r;
}
// a BN(+act) apply deferred to the side stream: what a consumer needs to stage it from pre
struct Defer {
  const float* pre = nullptr;
  int ld = 0;
  long long gs = 0;
  AccR acc;
  long long rows = 0;
  const float* beta = nullptr;
  long long beta_gs = 0;
  BNS bn;
  long long bn_gs = 0;
  int act = 0;
  bool fin = false;              // mean / invstd finalised by the producer's last block (BnFin)
  hipEvent_t applied = nullptr;  // on st2, after the apply
};

static void set_stats(FwdArgs& a, const AccR& r) {
  a.stats = r.p;
  a.s_gs = r.gs;
  a.s_sh = r.sh;
  a.s_nsh = r.nsh;
}

// ---------------------------------------------------------------------------
// layer helpers
// ---------------------------------------------------------------------------
namespace {

FwdArgs fwd_args_conv(const ConvL& L, int B, const float* W, long long w_gs) {
  FwdArgs a{};
  a.B = W;
  a.b_gs = w_gs;
  a.b_tap = (long long)L.cin * L.cout;
  a.g.nimg = B;
  a.g.Hi = a.g.Wi = L.hin;
  a.g.Ho = a.g.Wo = L.hout;
  a.g.stride = L.stride;
  a.g.pad = 1;
  a.g.ksz = 4;
  a.N = L.cout;
  a.Cin = L.cin;
  if (!L.tr) {  // conv2d: W [tap][ci][co] = KN
    a.g.mode = GM_CONV;
    a.b_nk = 0;
    a.ldb = L.cout;
    a.rows = B * L.hout * L.hout;
    a.nclass = 1;
  } else {  // conv2d_transpose: W [tap][co][ci] = NK
    a.g.mode = GM_CONVT;
    a.b_nk = 1;
    a.ldb = L.cin;
    if (L.stride == 2) {
      a.rows = B * (L.hout / 2) * (L.hout / 2);
      a.nclass = 4;
    } else {
      a.rows = B * L.hout * L.hout;
      a.nclass = 1;
    }
  }
  return a;
}

int nrb_of(const FwdArgs& a) {
  int bm = igemm_fwd_bm(a);
  return a.nclass * ((a.rows + bm - 1) / bm);
}

}  // namespace

// bf16 shadow views of a weight tensor: N = TF layout, T = per-tap transpose
static const void* shadowN(svae_ctx* c, long long off) { return (const void*)((const __bf16*)c->wN + off); }
static const void* shadowT(svae_ctx* c, long long off) { return (const void*)((const __bf16*)c->wT + off); }

// launches the gather-GEMM; returns the number of BN-stat row blocks it wrote
// event pair for the next probed launch (nullptr when the pool is exhausted)
static hipEvent_t* probe_pair(svae_ctx* c, int kid, double flops) {
  Probe& p = c->probe;
  if (p.kid == KID_NONE || kid != p.kid) return nullptr;
  p.launches++;
  if (2 * (size_t)p.used + 1 >= p.ev.size()) return nullptr;
  p.flops += flops;  // FLOPs of timed launches only
  hipEvent_t* e = &p.ev[2 * p.used++];
  hipEventRecord(e[0], c->st);
  return e;
}

// ---- side-stream weight gradients ----
// Next BN-backward output slot: the main stream first waits until the side stream has finished
// the weight gradient that read the slot's previous contents.
struct Slot {
  float* p;
  hipEvent_t ready, freed;
};
// next region of `n` elements of a per-pass arena; on overflow (a geometry the plan did not
// size) the main stream waits for the side stream to drain and the arena starts over
static int side_flush(svae_ctx* c, hipStream_t also = nullptr);
static int side_run_queued(svae_ctx* c);
// st2 after everything enqueued so far on st2b (no-op without the second side stream)
static void side_merge(svae_ctx* c) {
  if (!c->st2b) return;
  hipEventRecord(c->ev_merge, c->st2b);
  hipStreamWaitEvent(c->st2, c->ev_merge, 0);
}
static float* arena_next(svae_ctx* c, float* base, long long cap, long long& off, long long n,
                         bool st3_reads = false) {
  n = (n + 63) / 64 * 64;
  if (off + n > cap) {
    side_flush(c);
    if (!st3_reads) side_merge(c);
    hipEvent_t ev = st3_reads ? c->ev_drain3 : c->ev_drain;
    hipEventRecord(ev, st3_reads ? c->st3 : c->st2);
    hipStreamWaitEvent(c->st, ev, 0);
    off = 0;
  }
  float* p = base + off;
  off += n;
  return p;
}
static Slot dpre_next(svae_ctx* c, long long n) {
  if (!c->side) return Slot{c->dpre, nullptr, nullptr};
  const int i = c->ring_pos;
  c->ring_pos = (i + 1) % svae_ctx::NR;
  return Slot{arena_next(c, c->dpre_arena, c->dpre_cap, c->dpre_off, n), c->ev_ready[i], nullptr};
}
static Slot idpre_next(svae_ctx* c, long long n) {
  if (!c->side) return Slot{c->idpre, nullptr, nullptr};
  const int i = c->iring_pos;
  c->iring_pos = (i + 1) % svae_ctx::NR;
  return Slot{arena_next(c, c->idpre_arena, c->idpre_cap, c->idpre_off, n), c->ev_iready[i], nullptr};
}
// run fn (weight-gradient launches) on the side stream after everything enqueued so far on the
// main stream; the side stream uses its own split slab
// enqueue the queued side-stream work behind one main-stream event; `also` (st3) waits on the
// same event.  Returns the first error of the queued work.
static int side_flush(svae_ctx* c, hipStream_t also) {
  if (!c->side) return 0;
  if (c->side_q.empty() && !also) return 0;
  hipEvent_t ev = c->ev_flush[c->flush_pos];
  c->flush_pos = (c->flush_pos + 1) % svae_ctx::NF;
  hipEventRecord(ev, c->st);
  if (also) hipStreamWaitEvent(also, ev, 0);
  if (c->side_q.empty()) return 0;
  hipStreamWaitEvent(c->st2, ev, 0);
  return side_run_queued(c);
}
// enqueue the queued work on st2, which the caller has already ordered after the main stream
static int side_run_queued(svae_ctx* c) {
  if (c->side_q.empty()) return 0;
  hipStream_t s0 = c->st;
  float* sl0 = c->slab;
  c->st = c->st2;
  c->slab = c->slab2;
  int r = 0;
  for (auto& f : c->side_q) {
    const int e = f();
    if (e && !r) r = e;
  }
  c->side_q.clear();
  c->st = s0;
  c->slab = sl0;
  return r;
}
// queued form of on_side for closures that capture by value (SVAE_SIDE_BATCH > 1); otherwise at once.
// Contract of the queued form:
//  - a closure's inputs are produced on the stream that is c->st when it is queued; the queue
//    must be flushed (side_flush records its event on c->st) before c->st changes, so the
//    event orders st2 after the producing stream (the st4 recognition groups flush before
//    restoring the main stream);
//  - there is no per-slot "freed" event: every dpre / dcat / dtop / da region lives in a per-pass
//    arena and is never reused within a pass, so no slot waits for its reader;
//  - c->st / c->slab are read when the closure RUNS (side_run_queued swaps in st2 / slab2).
template <class Fn>
static int on_side_q(svae_ctx* c, hipEvent_t ready, Fn&& fn) {
  if (!c->side || !ready || c->side_batch <= 1) {
    if (c->side && ready) {
      const bool b = c->st2b && !c->side_pin && (c->side_rr++ & 1);
      hipStream_t sx = b ? c->st2b : c->st2;
      hipEventRecord(ready, c->st);
      hipStreamWaitEvent(sx, ready, 0);
      hipStream_t s0 = c->st;
      float* sl0 = c->slab;
      c->st = sx;
      c->slab = b ? c->slab2b : c->slab2;
      const int r = fn();
      c->st = s0;
      c->slab = sl0;
      return r;
    }
    return fn();
  }
  c->side_q.emplace_back(std::forward<Fn>(fn));
  return (int)c->side_q.size() >= c->side_batch ? side_flush(c) : 0;
}
template <class Fn>
static int on_side(svae_ctx* c, hipEvent_t ready, hipEvent_t freed, Fn&& fn) {
  if (!c->side || !ready) return fn();
  if (int r = side_flush(c)) return r;  // queued work first (stream order on st2)
  hipEventRecord(ready, c->st);
  hipStreamWaitEvent(c->st2, ready, 0);
  hipStream_t s0 = c->st;
  float* sl0 = c->slab;
  c->st = c->st2;
  c->slab = c->slab2;
  const int r = fn();
  c->st = s0;
  c->slab = sl0;
  if (freed) hipEventRecord(freed, c->st2);
  return r;
}

// SVAE_TRACE_GEMM=1: every main-stream gather-GEMM timed alone (the stream is drained around
// it) and printed with its shape -- a per-layer breakdown for tuning, not for measurement runs
static bool trace_gemm() {
  static const bool v = svae_knob("SVAE_TRACE_GEMM", 0) == 1;
  return v;
}
static int gemm(svae_ctx* c, FwdArgs a, int groups) {
  if (c->m.g.split && a.Bh) {
    a.nsp = 3;
    if (!a.b_plane) {  // (the packed output weights carry their own plane stride and no fp16 planes)
      a.b_plane = c->wplane;
      a.h16 = 1;  // a weight shadow: the fp16 planes H16_PLANE.. follow the bf16 ones
      // ... at its tensor's exponent: the table entry of the weight's offset in the shadow, per group
      const __bf16* b = (const __bf16*)a.Bh;
      const __bf16* bn = (const __bf16*)c->wN;
      const __bf16* bt = (const __bf16*)c->wT;
      long long off = -1;
      if (b >= bn && b < bn + c->wplane) off = b - bn;
      else if (b >= bt && b < bt + c->wplane) off = b - bt;
      if (off < 0 || (off & 63) || (a.b_gs & 63) || !c->wtab) return fail(c, SVAE_EBADARG, "weight outside the shadows");
      a.wexp = c->wtab + (off >> 6);
      a.wexp_gs = a.b_gs >> 6;
    }
    a.part = c->slab;
    a.part_cap = c->slab_cap;
    if (!igemm_split_ok(a, groups)) {  // no split kernel for this shape: the fp32 kernels
      a.Bh = nullptr;
      a.nsp = 0;
      a.ldb = a.b_nk ? a.Cin : a.N;  // the fp32 weight's own layout (TF [tap][k][n] or [tap][n][k])
      a.bw = BwStat{};                // (conv_dgrad fused the BN partials only where a split kernel runs)
      a.ksplit = 1;
      igemm_fwd(a, groups, c->st);
      return 0;
    }
  }
  if (c->m.g.bf16 && a.Bh && trace_gemm()) {
    a.part = c->slab;
    a.part_cap = c->slab_cap;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipDeviceSynchronize();
    hipEventRecord(e0, c->st);
    const int r = igemm_bf16(a, groups, c->st);
    hipEventRecord(e1, c->st);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    const int ntap = a.g.mode == GM_DENSE ? 1 : (a.g.mode == GM_CONVT && a.g.stride == 2 ? 4 : 16);
    const double fl = 2.0 * a.rows * a.nclass * a.N * (double)ntap * a.Cin * groups;
    fprintf(stderr, "GEMM mode %d s %d hi %d ho %d cin %d n %d rows %d cls %d grp %d abf %d bw %d st %d  %8.2f us %7.1f TF/s\n",
            a.g.mode, a.g.stride, a.g.Hi, a.g.Ho, a.Cin, a.N, a.rows, a.nclass, groups, a.a_bf16, a.bw.pre != nullptr,
            a.stats != nullptr, ms * 1e3, fl / (ms * 1e9));
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return r;
  }
  if (c->m.g.bf16 && a.Bh) {
    a.part = c->slab;
    a.part_cap = c->slab_cap;
    if (c->probe.kid != KID_NONE) {  // algorithmic FLOPs: 2 * rows * N * taps * Cin per class
      const int ntap = a.g.mode == GM_DENSE ? 1 : (a.g.mode == GM_CONVT && a.g.stride == 2 ? 4 : 16);
      const double fl = 2.0 * a.rows * a.nclass * a.N * (double)ntap * a.Cin * groups;
      hipEvent_t* e = probe_pair(c, igemm_bf16_kid(a), fl);
      if (e) return igemm_bf16(a, groups, c->st, e[1]);
    }
    return igemm_bf16(a, groups, c->st);
  }
  a.ksplit = 1;
  igemm_fwd(a, groups, c->st);
  return 0;
}
// stats row-blocks the GEMM will use (accumulator sharding)
static int gemm_nrb(svae_ctx* c, FwdArgs a, int groups) {
  if (c->m.g.split && a.Bh) {
    a.nsp = 3;
    a.part = c->slab;
    a.part_cap = c->slab_cap;
    if (!igemm_split_ok(a, groups)) {
      a.Bh = nullptr;
      return nrb_of(a);
    }
  }
  if (c->m.g.bf16 && a.Bh) {
    a.part = c->slab;
    a.part_cap = c->slab_cap;
    return igemm_bf16_plan(a, groups, nullptr);
  }
  return nrb_of(a);
}
static void wgemm(svae_ctx* c, const WgArgs& w, int groups) {
  if (!c->m.g.bf16) {
    wgrad(w, groups, c->st);
    return;
  }
  static const bool split_wg = svae_knob("SVAE_SPLIT_WG", 1) != 0;  // 0: the fp32 weight-GEMM in split mode
  if (c->m.g.split && !split_wg) {
    wgrad(w, groups, c->st);
    return;
  }
  if (c->m.g.split) {  // the tap-merged bf16 kernel on w.nsp operand planes (wgrad_bf16_kernel NSP)
    WgArgs ws = w;
    if (ws.nsp < 2) ws.nsp = 2;
    wgrad_bf16(ws, groups, c->st);
    return;
  }
  if (c->probe.kid != KID_NONE) {  // algorithmic FLOPs: 2 * taps * M * N * row pixels
    const double fl = 2.0 * w.ntap * (double)w.M * w.N * w.rows * groups;
    hipEvent_t* e = probe_pair(c, wgrad_bf16_kid(w), fl);
    if (e) {
      wgrad_bf16(w, groups, c->st, e[1]);
      return;
    }
  }
  wgrad_bf16(w, groups, c->st);
}

// SVAE_DBG_SKIP (timing probe, WRONG RESULTS): bit 0 skips the forward BN apply of the layers whose
// output only bf16 GEMMs read, bit 1 the backward BN apply of the conv layers without a shortcut --
// the step time without the passes a consumer-side fold would remove (an upper bound of its gain);
// bit 2 every conv weight gradient (side stream), bit 3 the per-bucket Adam of the chain steps; bit 4 makes
// the conv layers' forward BN apply read last step's mean / invstd instead of finalising the statistics
// accumulators per block (the gain a producer-side finalise could bring).  Compiled only into a
// -DSVAE_DEBUG_PROBES build: the shipping library ignores the variable (tests/test_knobs.py)
#ifdef SVAE_DEBUG_PROBES
static int dbg_skip() {
  static const int v = [] {
    const char* e = getenv("SVAE_DBG_SKIP");
    return e ? atoi(e) : 0;
  }();
  return v;
}
#else
static inline int dbg_skip() { return 0; }
#endif

// the consumer-side BN gather is available for this launch (the wave-split halo gather takes it)
static bool ain_ok(svae_ctx* c, const FwdArgs& t, int groups) {
  // (the split mode's gathers scale their staged window by its running maximum, taken before a
  // consumer-side BN could be applied: the knob-only fold runs in the bf16 mode alone)
  if (!c->m.g.bf16 || !t.Bh || c->m.g.split) return false;
  return halo_kw_plan(t, groups) > 0;
}

// Forward conv/convT + BN + act.  in: [B,hin,hin,cin] (ld), out view gets act(BN(pre)+res).
// in.dfr: the input's BN apply was deferred (its gather stages act(bn_y(pre)), or waits for the apply
// where it cannot); dfr_out: defer this layer's apply to st2 when SVAE_FOLD is on (no residual)
static int conv_bn_act_fwd(svae_ctx* c, const ConvL& L, int groups, long long w_gs, View in, float* pre,
                           long long pre_gs, BNS bn, long long bn_gs, View res, int act, View out,
                           Defer* dfr_out = nullptr) {
  const int B = c->m.g.B;
  FwdArgs a = fwd_args_conv(L, B, c->P + L.ow, w_gs);
  a.A = in.p;
  a.a_gs = in.gs;
  a.lda = in.ld;
  a.a_bf16 = in.bf;
  a.C = pre;
  a.c_gs = pre_gs;
  a.ldc = L.cout;
  if (c->m.g.bf16) {  // NK bf16: conv -> T copy [tap][co][ci], conv-T -> N copy [tap][co][ci]
    a.Bh = L.tr ? shadowN(c, L.ow) : shadowT(c, L.ow);
    a.ldb = L.cin;
  }
  if (in.dfr) {
    const Defer& d = *in.dfr;
    FwdArgs t = a;
    t.A = d.pre;
    t.a_gs = d.gs;
    t.lda = d.ld;
    t.a_bf16 = c->pbf;  // the pre-BN tensor's storage
    t.ain = AinBN{d.acc.p, d.acc.gs, d.acc.sh, d.acc.nsh, d.rows, d.beta, d.beta_gs, d.bn.mean, d.bn.invstd, d.bn_gs,
                  d.act, 1e-3f, d.fin ? 1 : 0};
    if (ain_ok(c, t, groups)) a = t;
    else hipStreamWaitEvent(c->st, d.applied, 0);  // stage the applied tensor
  }
  const AccR acc = acc_bn(c, groups, L.cout, gemm_nrb(c, a, groups));
  if (!acc.p) return fail(c, SVAE_EBADARG, "BN accumulator arena too small");
  set_stats(a, acc);
  if (c->pbf) {  // every conv BN layer: its readers in the backward take the same flag (c->pbf)
    if (!igemm_c_bf16_ok(a, groups)) return fail(c, SVAE_EBADARG, "bf16 pre-BN output: no kernel for this launch");
    a.c_bf16 = 1;
  }
  const long long rows = (long long)B * L.hout * L.hout;
  bool fin = false;  // mean / invstd finalised by the producer's last block
  if ((c->laf & 1) && c->m.g.bf16 && a.Bh) {
    FwdArgs u = a;
    if (c->m.g.split) {
      u.nsp = 3;
      u.b_plane = c->wplane;
      u.h16 = 1;
    }
    if (igemm_fin_ok(u, groups)) {
      u64* cnt = acc_take(c, groups);
      if (!cnt) return fail(c, SVAE_EBADARG, "BN accumulator arena too small");
      a.fin = BnFin{cnt, 0, acc.p, acc.gs, acc.sh, acc.nsh, L.cout, rows, 1e-3f, bn.mean, bn.invstd, bn_gs, 0, nullptr, 0};
      fin = true;
    }
  }
  gemm(c, a, groups);
  if ((dbg_skip() & 1) && out.bf && !res.p) return 0;  // TIMING PROBE ONLY (wrong results): no apply pass
  if (dfr_out && c->fold && c->side && !res.p) {  // the apply on st2, off the critical path
    hipEvent_t ready = c->ev_fold[c->fold_pos];
    hipEvent_t applied = c->ev_fold[c->fold_pos + 1];
    c->fold_pos = (c->fold_pos + 2) % svae_ctx::NFOLD;
    hipEventRecord(ready, c->st);
    hipStreamWaitEvent(c->st2, ready, 0);
    bn_apply(pre, L.cout, pre_gs, rows, L.cout, fin ? nullptr : acc.p, acc.gs, acc.sh, acc.nsh, 1e-3f, bn.mean, bn.invstd,
             bn_gs, c->P + L.obeta, w_gs, nullptr, 0, 0, act, out.p, out.ld, out.gs, groups, c->st2, out.bf, c->pbf);
    hipEventRecord(applied, c->st2);
    c->fold_used = true;
    Defer& d = *dfr_out;
    d.pre = pre;
    d.ld = L.cout;
    d.gs = pre_gs;
    d.acc = acc;
    d.rows = rows;
    d.beta = c->P + L.obeta;
    d.beta_gs = w_gs;
    d.bn = bn;
    d.bn_gs = bn_gs;
    d.act = act;
    d.fin = fin;
    d.applied = applied;
    return 0;
  }
  if (dfr_out) *dfr_out = Defer{};
  if (c->bnfin && !fin && !(dbg_skip() & 16)) {  // the statistics finalised once, read by every apply block
    bn_finalize(acc.p, acc.gs, acc.sh, acc.nsh, rows, L.cout, 1e-3f, bn.mean, bn.invstd, bn_gs, nullptr, nullptr, 0,
                groups, c->st);
    fin = true;
  }
  bn_apply(pre, L.cout, pre_gs, rows, L.cout, (fin || (dbg_skip() & 16)) ? nullptr : acc.p, acc.gs, acc.sh, acc.nsh, 1e-3f, bn.mean,
           bn.invstd, bn_gs, c->P + L.obeta, w_gs, res.p, res.ld, res.gs, act, out.p, out.ld, out.gs, groups, c->st, out.bf,
           c->pbf);
  return 0;
}

static void choose_split(long long rows, int taps, int tiles, int groups, long long per_split_elems, long long cap,
                         int& nsplit, int& chunk, int target = 1024, long long min_rows = 512) {
  long long blocks = (long long)taps * tiles * groups;
  long long want = (target + blocks - 1) / blocks;
  long long maxs = std::max<long long>(1, rows / min_rows);
  long long ns = std::min(want, maxs);
  long long capn = cap / std::max<long long>(1, per_split_elems * groups);
  ns = std::max<long long>(1, std::min(ns, capn));
  long long ch = (rows + ns - 1) / ns;
  ch = (ch + 31) / 32 * 32;
  nsplit = (int)((rows + ch - 1) / ch);
  chunk = (int)ch;
}

// dpre of layer L is stored as bf16 (bf16 mode) unless its input gradient takes the fp32 small-N
// gather (image-channel conv whose Cout is not a multiple of 32: tiny test geometries)
static int dpre_bf(const svae_ctx* c, const ConvL& L) {
  if (!c->dbf) return 0;
  return (L.cin % 4 != 0 && !(L.cout % 32 == 0 && !L.tr)) ? 0 : 1;
}

// weight gradient of a conv/convT layer: dpre = grad wrt pre-BN output, in = layer input
static int conv_wgrad(svae_ctx* c, const ConvL& L, int groups, long long w_gs, View in, const float* dpre,
                      long long dpre_gs, float* dW) {
  const int B = c->m.g.B;
  if (dbg_skip() & 4) return 0;  // TIMING PROBE ONLY (wrong results): no conv weight gradients
  WgArgs w{};
  w.g.ksz = 4;
  w.g.pad = 1;
  w.g.stride = L.stride;
  w.g.mode = GM_CONV;
  w.g.nimg = B;
  w.ntap = 16;
  if (!L.tr) {
    // dW[tap][ci][co] = sum_{p out} x[src(p,tap)][ci] * dpre[p][co]
    w.G = in.p; w.g_gs = in.gs; w.ldg = in.ld; w.g_bf16 = in.bf;
    w.D = dpre; w.d_gs = dpre_gs; w.ldd = L.cout;
    w.d_bf16 = dpre_bf(c, L);
    w.M = L.cin; w.N = L.cout;
    w.g.Hi = w.g.Wi = L.hin;
    w.g.Ho = w.g.Wo = L.hout;
    w.rows = B * L.hout * L.hout;
  } else {
    // dW[tap][co][ci] = sum_{p in} dpre[src(p,tap)][co] * x[p][ci]
    w.G = dpre; w.g_gs = dpre_gs; w.ldg = L.cout;
    w.g_bf16 = dpre_bf(c, L);
    w.D = in.p; w.d_gs = in.gs; w.ldd = in.ld; w.d_bf16 = in.bf;
    w.M = L.cout; w.N = L.cin;
    w.g.Hi = w.g.Wi = L.hout;
    w.g.Ho = w.g.Wo = L.hin;
    w.rows = B * L.hin * L.hin;
  }
  w.nsp = c->m.g.split ? 2 : 1;
  if (c->m.g.bf16 && c->wg_path == 2 && wgrad_halo2_ok(w)) {  // stride 1 / 2: compile-time-geometry kernel
    hipEvent_t* ev = nullptr;
    if (c->probe.kid != KID_NONE)
      ev = probe_pair(c, w.g.stride == 1 ? KID_WHALO2_S1 : KID_WHALO2_S2, 2.0 * 16 * (double)w.M * w.N * w.rows * groups);
    // the T-batched recognition layers (groups > 1) run after the chain backward, beside the recognition
    // input gradients and then alone: twice the default split target (SVAE_WH2_GTARGET, 0 = the default)
    static const int gtarget = svae_knob("SVAE_WH2_GTARGET", 256);
    if (wgrad_halo2(w, groups, c->slab, c->slab_cap, dW, w_gs, c->st, ev ? ev[1] : nullptr, groups > 1 ? gtarget : 0))
      return 0;
  }
  const bool bfk = c->m.g.bf16 && !c->m.g.split;  // plain-bf16 weight-GEMM kernels
  if (bfk && c->wg_path != 0 && wgrad_halo_enabled()) {
    WHaloPlanOut pl;
    if (wgrad_halo_plan(w, groups, &pl)) {
      // pixel chunks split over blocks: ~1024 blocks in flight, slab within capacity
      const long long per = 16LL * w.M * w.N;
      // ~wh_target blocks, but >= wh_minch chunks per block: every split writes (and the reduce
      // reads) a full 16*M*N partial, so short splits cost more partial traffic than they save
      static const int wh_target = svae_knob("SVAE_WH_TARGET", 256);
      static const int wh_minch = svae_knob("SVAE_WH_MINCH", 8);
      long long ns = (wh_target + (long long)pl.tiles * groups - 1) / ((long long)pl.tiles * groups);
      ns = std::min<long long>(ns, std::max<long long>(1, pl.h.nchunk / wh_minch));
      ns = std::min<long long>(ns, std::max<long long>(1, c->slab_cap / (per * groups)));
      w.nsplit = (int)std::max<long long>(1, ns);
      if (w.nsplit == 1) {
        w.part = dW;
        w.p_gs = w_gs;
      } else {
        w.part = c->slab;
        w.p_gs = (long long)w.nsplit * per;
      }
      hipEvent_t* ev = nullptr;
      if (c->probe.kid != KID_NONE)
        ev = probe_pair(c, w.g.stride == 1 ? KID_WHALO_32_S1 : KID_WHALO_32_S2,
                        2.0 * 16 * (double)w.M * w.N * w.rows * groups);
      wgrad_halo(pl, w, groups, c->st, ev ? ev[1] : nullptr);
      if (w.nsplit > 1)
        wgrad_reduce(c->slab, w.p_gs, w.nsplit, 16, w.M, w.N, dW, w_gs, w.M, nullptr, 0, 0, groups, c->st);
      return 0;
    }
  }
  // image-space stride-2 conv with Cin <= 3: im2col in LDS, MFMA over pixel chunks
  if ((bfk || c->m.g.split) && wgrad_smallc(w, groups, c->slab, c->slab_cap, dW, w_gs, c->st)) return 0;
  if (bfk || c->m.g.split)  // tap-merged tiles; longer splits (less slab traffic)
    choose_split(w.rows, 1, wgrad_bf16_tiles(w), groups, 16LL * w.M * w.N, c->slab_cap, w.nsplit, w.chunk, 2048,
                 256);
  else
    choose_split(w.rows, 16, ((w.M + 63) / 64) * ((w.N + 63) / 64), groups, 16LL * w.M * w.N, c->slab_cap,
                 w.nsplit, w.chunk);
  if (w.nsplit == 1) {  // single split: the [tap][m][n] partial IS the TF weight layout
    w.part = dW;
    w.p_gs = w_gs;
    wgemm(c, w, groups);
    return 0;
  }
  w.part = c->slab;
  w.p_gs = (long long)w.nsplit * 16 * w.M * w.N;
  if (w.p_gs * groups > c->slab_cap) return fail(c, SVAE_EBADARG, "wgrad slab too small");
  wgemm(c, w, groups);
  wgrad_reduce(c->slab, w.p_gs, w.nsplit, 16, w.M, w.N, dW, w_gs, w.M, nullptr, 0, 0, groups, c->st);
  return 0;
}

// input gradient of a conv/convT layer: din (+)= dgrad(dpre)
// Fused backward-BN reduction: the input-gradient GEMM that is the LAST writer of a layer's dy
// also emits that layer's (sum dz, sum dz*xhat) partials (BwStat epilogue, bf16 kernels), and
// bn_act_bwd then skips bn_bwd_reduce (one full read of dy and pre less per layer).
struct BwFuse {
  BwStat bw{};
  AccR acc;  // accumulators the fused epilogue adds into
  bool used = false;
  float* dbeta = nullptr;   // the layer's beta gradient
  long long dbeta_gs = 0;
  float* ab = nullptr;      // a, b finalised by the producing launch's last block ([group][2C]; BnFin mode 1)
};
static BwFuse bw_fuse(svae_ctx* c, const float* pre, int ldp, long long pre_gs, const float* y, int ldy, long long y_gs,
                      BNS bn, long long bn_gs, long long beta_off, long long w_gs, int act, int C, int pre_bf16) {
  BwFuse f;
  f.bw.pre = pre; f.bw.ldp = ldp; f.bw.pre_gs = pre_gs;
  f.bw.y = y; f.bw.ldy = ldy; f.bw.y_gs = y_gs;
  f.bw.mean = bn.mean; f.bw.invstd = bn.invstd; f.bw.ms_gs = bn_gs;
  f.bw.beta = c->P + beta_off; f.bw.beta_gs = w_gs;
  f.bw.act = act; f.bw.C = C;
  f.bw.pre_bf16 = pre_bf16;
  f.dbeta = c->Gr ? c->Gr + beta_off : nullptr;
  f.dbeta_gs = w_gs;
  return f;
}

static bool nofuse_out() {  // SVAE_NO_BWFUSE_OUT=1: s1[0]'s BN-backward sums in their own pass (A/B)
  static const bool v = svae_knob("SVAE_NO_BWFUSE_OUT", 0) == 1;
  return v;
}
static int conv_dgrad(svae_ctx* c, const ConvL& L, int groups, long long w_gs, const float* dpre, long long dpre_gs,
                      View din, int accumulate, BwFuse* fu = nullptr) {
  if (fu) fu->used = false;
  const int B = c->m.g.B;
  const float* W = c->P + L.ow;
  if (L.cin % 4 != 0 && c->m.g.bf16 && L.cout % 32 == 0 && !L.tr) {
    // layer-0 conv input gradient (N = image channels): bf16 small-N conv-T gather (CONVT mode from
    // dpre); split mode: the same kernel on the three planes (convt_smalln_kernel<3>)
    FwdArgs a{};
    a.A = dpre; a.a_gs = dpre_gs; a.lda = L.cout; a.a_bf16 = dpre_bf(c, L);
    a.B = W;  // (fp32 fallback of a split-mode shape without a split kernel)
    a.Bh = shadowN(c, L.ow); a.b_nk = 1; a.ldb = L.cout; a.b_tap = (long long)L.cin * L.cout; a.b_gs = w_gs;
    a.C = din.p; a.c_gs = din.gs; a.ldc = din.ld;
    a.N = L.cin; a.Cin = L.cout;
    a.g = ConvGeom{GM_CONVT, B, L.hout, L.hout, L.hin, L.hin, L.stride, 1, 4};
    a.rows = L.stride == 2 ? B * (L.hin / 2) * (L.hin / 2) : B * L.hin * L.hin;
    a.nclass = L.stride == 2 ? 4 : 1;
    a.accumulate = accumulate;
    gemm(c, a, groups);
    return 0;
  }
  if (L.cin % 4 != 0) {
    // layer-0 conv (Cin = image channels): small-N gather (CONVT mode from dpre)
    if (groups != 1) return fail(c, SVAE_EBADARG, "small-N dgrad is not batched");
    ConvGeom g{GM_CONVT, B, L.hout, L.hout, L.hin, L.hin, L.stride, 1, 4};
    gconv_smalln(dpre, L.cout, L.cout, W, L.cin, nullptr, 0, (long long)L.cin * L.cout, 0, nullptr, nullptr, g,
                 (long long)B * L.hin * L.hin, din.p, din.ld, accumulate, c->st);
    return 0;
  }
  FwdArgs a{};
  a.A = dpre; a.a_gs = dpre_gs; a.lda = L.cout; a.a_bf16 = dpre_bf(c, L);
  a.B = W; a.b_gs = w_gs; a.b_tap = (long long)L.cin * L.cout;
  a.C = din.p; a.c_gs = din.gs; a.ldc = din.ld;
  a.N = L.cin; a.Cin = L.cout;
  a.g.nimg = B; a.g.Hi = a.g.Wi = L.hout; a.g.Ho = a.g.Wo = L.hin;
  a.g.stride = L.stride; a.g.pad = 1; a.g.ksz = 4;
  a.accumulate = accumulate;
  if (!L.tr) {  // conv dgrad = CONVT gather, weights read [tap][ci][co] as NK
    a.g.mode = GM_CONVT;
    a.b_nk = 1;
    a.ldb = L.cout;
    if (L.stride == 2) { a.rows = B * (L.hin / 2) * (L.hin / 2); a.nclass = 4; }
    else { a.rows = B * L.hin * L.hin; a.nclass = 1; }
  } else {  // conv-T dgrad = CONV gather, weights [tap][co][ci] as KN
    a.g.mode = GM_CONV;
    a.b_nk = 0;
    a.ldb = L.cin;
    a.rows = B * L.hin * L.hin;
    a.nclass = 1;
  }
  if (c->m.g.bf16 && c->wN) {  // NK bf16 [tap][ci][co]: conv -> N copy, conv-T -> T copy
    a.Bh = L.tr ? shadowT(c, L.ow) : shadowN(c, L.ow);
    a.ldb = L.cout;
    static const int nofuse = svae_knob("SVAE_NO_BWFUSE", 0) == 1;
    FwdArgs sa = a;  // split mode: the fused partials need the split kernel (the fp32 one has none)
    sa.nsp = 3;
    const bool fuse_ok = !c->m.g.split || igemm_split_ok(sa, groups);
    if (fu && fu->bw.pre && fu->bw.C % 4 == 0 && !nofuse && fuse_ok) {
      a.bw = fu->bw;
      const AccR acc = acc_bn(c, groups, fu->bw.C, gemm_nrb(c, a, groups));
      if (!acc.p) return fail(c, SVAE_EBADARG, "BN accumulator arena too small");
      set_stats(a, acc);
      fu->acc = acc;
      fu->used = true;
      fu->ab = nullptr;
      FwdArgs u = a;
      if (c->m.g.split) {
        u.nsp = 3;
        u.b_plane = c->wplane;
        u.h16 = 1;
      }
      if ((c->laf & 2) && fu->dbeta && igemm_fin_ok(u, groups)) {  // a, b, dbeta by the last block
        const int C = fu->bw.C;
        u64* cnt = acc_take(c, groups);
        float* ab = (float*)acc_take(c, (long long)groups * C);  // [group][2C] floats
        if (!cnt || !ab) return fail(c, SVAE_EBADARG, "BN accumulator arena too small");
        a.fin = BnFin{cnt, 0, acc.p, acc.gs, acc.sh, acc.nsh, C, (long long)B * L.hin * L.hin, 1e-3f, ab, ab + C,
                      2LL * C, 1, fu->dbeta, fu->dbeta_gs};
        fu->ab = ab;
      }
    }
  }
  gemm(c, a, groups);
  return 0;
}

// BN(+act) backward: dy (grad wrt post-act out y) -> dpre; dbeta into grads; optional dres
static int bn_act_bwd(svae_ctx* c, int groups, long long rows, int C, View dy, View y, const float* pre, long long pre_gs,
                      int ldp, BNS bn, long long bn_gs, long long beta_off, long long w_gs, int act, float* dpre,
                      long long dpre_gs, View dres, int res_acc, const BwFuse* fu = nullptr, int dpre_bf16 = 0,
                      int pre_bf16 = 0) {
  const bool pre_reduced = fu && fu->used;  // sums already added by the fused dgrad epilogue
  const AccR acc = pre_reduced ? fu->acc : acc_bn(c, groups, C, bn_bwd_rowblocks(rows));
  if (!acc.p) return fail(c, SVAE_EBADARG, "BN accumulator arena too small");
  // without a shortcut add, act'(y) follows from the recomputed BN output: y is not read
  const float* yp = (dres.p || !c->P) ? y.p : nullptr;  // (per-op entry: no beta, reads y)
  const float* beta = c->P + beta_off;
  if (!pre_reduced)
    bn_bwd_reduce(dy.p, dy.ld, dy.gs, yp, y.ld, y.gs, pre, ldp, pre_gs, rows, C, bn.mean, bn.invstd, bn_gs, beta, w_gs,
                  act, acc.p, acc.gs, acc.sh, acc.nsh, groups, c->st, pre_bf16, yp ? y.bf : 0);
  if ((dbg_skip() & 2) && !dres.p && rows > c->m.g.B) return 0;  // TIMING PROBE ONLY (wrong results)
  const float* ab = pre_reduced ? fu->ab : nullptr;
  if (c->bnfin && !ab) {  // a, b and dbeta finalised once, read by every apply block
    float* t = (float*)acc_take(c, (long long)groups * C);  // [group][2C] floats
    if (!t) return fail(c, SVAE_EBADARG, "BN accumulator arena too small");
    bn_finalize(acc.p, acc.gs, acc.sh, acc.nsh, rows, C, 1e-3f, nullptr, nullptr, 0, t, c->Gr + beta_off, w_gs, groups,
                c->st);
    ab = t;
  }
  bn_bwd_apply(dy.p, dy.ld, dy.gs, yp, y.ld, y.gs, pre, ldp, pre_gs, rows, C, bn.mean, bn.invstd, bn_gs, beta, w_gs,
               acc.p, acc.gs, acc.sh, acc.nsh, c->Gr + beta_off, w_gs, act, dpre, C, dpre_gs, dres.p, dres.ld, dres.gs, res_acc, groups,
               c->st, dpre_bf16, pre_bf16, ab, yp ? y.bf : 0);
  return 0;
}

// dense (FC) forward + BN + lrelu; in [B][nin] (ld), out view
static int fc_bn_fwd(svae_ctx* c, const FcL& f, View in, float* pre, BNS bn, View out) {
  const int B = c->m.g.B;
  FwdArgs a{};
  a.A = in.p; a.lda = in.ld; a.a_bf16 = in.bf;
  a.B = c->P + f.ow; a.b_nk = 0; a.ldb = f.nout; a.b_tap = 0;
  a.C = pre; a.ldc = f.nout;
  a.N = f.nout; a.Cin = f.nin;
  a.g.mode = GM_DENSE; a.g.nimg = B; a.g.ksz = 1; a.g.stride = 1;
  a.rows = B; a.nclass = 1;
  if (c->m.g.bf16) {
    a.Bh = shadowT(c, f.ow);  // [out][in]
    a.ldb = f.nin;
  }
  const AccR acc = acc_bn(c, 1, f.nout, gemm_nrb(c, a, 1));
  if (!acc.p) return fail(c, SVAE_EBADARG, "BN accumulator arena too small");
  set_stats(a, acc);
  gemm(c, a, 1);
  bn_apply(pre, f.nout, 0, B, f.nout, acc.p, acc.gs, acc.sh, acc.nsh, 1e-3f, bn.mean, bn.invstd, 0, c->P + f.obeta, 0, nullptr, 0, 0,
           ACT_LRELU, out.p, out.ld, 0, 1, c->st, out.bf);
  return 0;
}

// dense backward: dy wrt post-act (view), y, pre -> grads; din (=) if non-null
// fu_self: this layer's BN-backward sums were added by the producer of dy (pre-reduced);
// fu_din: the BN layer whose dy is din, its sums fused into this layer's input-gradient GEMM when
// that runs the split-K dense kernel (splitk_reduce carries the BwStat terms)
static int fc_bn_bwd(svae_ctx* c, const FcL& f, View in, View dy, View y, const float* pre, BNS bn, View din,
                     BwFuse* fu_self = nullptr, BwFuse* fu_din = nullptr) {
  const int B = c->m.g.B;
  const Slot sl = dpre_next(c, (long long)B * f.nout);
  int r = bn_act_bwd(c, 1, B, f.nout, dy, y, pre, 0, f.nout, bn, 0, f.obeta, 0, ACT_LRELU, sl.p, 0, View{}, 0, fu_self,
                     c->dbf);
  if (r) return r;
  WgArgs w{};
  w.G = in.p; w.ldg = in.ld; w.g_bf16 = in.bf;
  w.D = sl.p; w.ldd = f.nout; w.d_bf16 = c->dbf;
  w.M = f.nin; w.N = f.nout;
  w.g.mode = GM_DENSE; w.g.nimg = B; w.g.ksz = 1; w.g.stride = 1;
  w.ntap = 1;
  w.rows = B;
  w.nsplit = 1;
  w.chunk = (B + 31) / 32 * 32;
  w.part = c->Gr + f.ow;  // single split over the batch rows: write dW [nin][nout] directly
  w.nsp = c->m.g.split ? 3 : 1;  // split mode: six plane products (K = the batch: short sums)
  if ((r = on_side_q(c, sl.ready, [=] {
         wgemm(c, w, 1);
         return 0;
       })))
    return r;
  if (din.p) {
    FwdArgs a{};
    a.A = sl.p; a.lda = f.nout; a.a_bf16 = c->dbf;
    a.B = c->P + f.ow; a.b_nk = 1; a.ldb = f.nout; a.b_tap = 0;
    a.C = din.p; a.ldc = din.ld;
    a.N = f.nin; a.Cin = f.nout;
    a.g.mode = GM_DENSE; a.g.nimg = B; a.g.ksz = 1; a.g.stride = 1;
    a.rows = B; a.nclass = 1;
    if (c->m.g.bf16) a.Bh = shadowN(c, f.ow);  // [in][out] as NK (n = in, k = out)
    if (fu_din) fu_din->used = false;
    // E.fc's BN-backward sums in the top FC's input gradient: +0.3 % (profiles/r03_fc_ab.txt);
    // SVAE_BWFUSE_FC=0 at svae_create restores the separate pass
    if (fu_din && fu_din->bw.pre && c->m.g.bf16 && !c->m.g.split && fu_din->bw.C % 4 == 0 && fu_din->bw.C <= a.N &&
        c->fc_fuse) {
      FwdArgs t = a;
      t.part = c->slab;
      t.part_cap = c->slab_cap;
      t.bw = fu_din->bw;
      if (dense_kw_ok(t, 1) && dense_kw_ks(t) > 1) {
        const AccR acc = acc_bn(c, 1, fu_din->bw.C, dense_kw_nrb(t));
        if (!acc.p) return fail(c, SVAE_EBADARG, "BN accumulator arena too small");
        a.bw = fu_din->bw;
        set_stats(a, acc);
        fu_din->acc = acc;
        fu_din->used = true;
      }
    }
    gemm(c, a, 1);
  }
  return 0;
}

// host hook after chain step t's backward: the side stream is ordered after all of the step's
// work on both streams, so a collective issued on it sees that step's complete gradients
static void adam_range(svae_ctx* c, long long lo, long long hi, float lr, long long step, float clip, hipStream_t s);

static int step_hook(svae_ctx* c, int t) {
  if ((!c->hook && !c->fa_on) || c->m.shared) return 0;  // shared tensors are complete only after every step
  if (c->side) {
    // the system-scope release only where a collective reads the bucket (8 per step otherwise: each writes the
    // L2s back on the main stream for no reader outside this device)
    hipEvent_t ev = c->hook ? c->ev_hook : c->ev_hook_dev;
    hipEventRecord(ev, c->st);
    hipStreamWaitEvent(c->st2, ev, 0);
    if (int r = side_run_queued(c)) return r;  // the step's queued weight gradients, before its bucket
    side_merge(c);
    hipEventRecord(c->ev_j3, c->st3);  // the step's split-latent gradients
    hipStreamWaitEvent(c->st2, c->ev_j3, 0);
  }
  if (c->hook) c->hook(c->hook_user, t);
  // the bucket's update follows whatever exchange the hook ordered on the side stream; the
  // backward of steps < t reads neither theta_t nor its shadows
  if (c->fa_on && !(dbg_skip() & 8)) adam_range(c, c->m.step_lo[t], c->m.step_hi[t], c->fa_lr, c->fa_step, c->fa_clip, c->st2);
  return 0;
}

// `off` elements into a tensor stored as fp32 or (bf) bf16, as a float* view base.  A group stride
// of a bf16 tensor counts bf16 elements (the producing kernels index it so), so step t0's group of
// the T-batched recognition activations starts t0 * gs bf16 elements in; float* arithmetic would
// put it twice as far, which only the same call's own reads agree with (found by a split forward /
// batched backward mismatch, tools/gpu/r03_recdiag.py)
static float* elem_off(float* base, long long off, int bf) {
  return bf ? (float*)((__bf16*)base + off) : base + off;
}

// Recognition ladders of steps [t0, t0+n) (inference_ladder :1579-1630, heads :1592-1609) on
// input `in` (group stride in.gs), then mu / sigma / z / KL (:1022-1024, :1156-1158).
static int inference_fwd(svae_ctx* c, int t0, int n, View in0) {
  Model& M = c->m;
  const Geo& g = M.g;
  const int B = g.B, L = g.L;
  const int* F = g.F;
  const long long wg = M.phi_stride;
  hipStream_t st = c->st;
  const InfStep& I = M.inf[t0];
  const long long hps = (long long)c->head_nsplit * B * 2 * g.Dz;
  int r;
  HIPCHK(c, hipMemsetAsync(c->head_part + t0 * hps, 0, (size_t)n * hps * sizeof(float), st));
  auto bns = [&](const BNS& b, int C) { return BNS{b.mean + (long long)t0 * C, b.invstd + (long long)t0 * C}; };
  for (int lvl = 0; lvl < L - 1; ++lvl) {
    const long long gs = c->inf_gs[lvl];
    const int Fl = F[lvl + 1];
    View in = lvl == 0 ? in0 : View{c->inf_act_b[lvl - 1] + t0 * c->inf_gs[lvl - 1], F[lvl], c->inf_gs[lvl - 1]};
    float* act_a = elem_off(c->inf_act_a[lvl], t0 * gs, c->abf);  // bf16 storage: step t0's group in bf16 elements
    Defer da;  // conv a's apply deferred to st2 (SVAE_FOLD): conv b's gather stages it from pre
    r = conv_bn_act_fwd(c, I.a[lvl], n, wg, in, elem_off(c->inf_pre_a[lvl], t0 * gs, c->pbf), gs, bns(c->inf_bn_a[lvl], Fl), Fl, View{},
                        ACT_LRELU, View{act_a, Fl, gs, c->abf}, &da);
    if (r) return r;
    r = conv_bn_act_fwd(c, I.b[lvl], n, wg, View{act_a, Fl, gs, c->abf, da.pre ? &da : nullptr},
                        elem_off(c->inf_pre_b[lvl], t0 * gs, c->pbf), gs,
                        bns(c->inf_bn_b[lvl], Fl), Fl, View{}, ACT_LRELU, View{c->inf_act_b[lvl] + t0 * gs, Fl, gs});
    if (r) return r;
    for (int hl = 0; hl < L; ++hl) {
      const HeadL& h = I.head[hl];
      if (h.src_level != lvl) continue;
      heads_fwd(c->inf_act_b[lvl] + t0 * gs, gs, B, h.nin, c->P + h.owm, c->P + h.ows, wg, h.d, c->head_part + t0 * hps,
                hps, 2 * g.Dz, h.off, n, st);
    }
  }
  LatentLvls lv{};
  lv.L = L;
  for (int l = 0; l < L; ++l) {
    const HeadL& h = I.head[l];
    lv.bm[l] = c->P + h.obm;
    lv.bs[l] = c->P + h.obs;
    lv.off[l] = h.off;
    lv.dim[l] = h.d;
  }
  const long long ms = (long long)B * g.Dz;
  latent_fwd(c->head_part + t0 * hps, hps, c->head_nsplit, B, g.Dz, lv, wg, g.clipv, g.prior, g.uniform, c->eps_used + t0 * ms, ms,
             c->mu + t0 * ms, c->sig + t0 * ms, c->z + t0 * ms, ms, c->kl_img + (long long)t0 * B, B, n, st);
  return 0;
}

// split_latent of step t (:1796-1806): ladder_i straight into the step's concat buffers
// The output / ratio conv-T operands of every step, PACK_MAXT steps per launch (misc.hip
// pack_out_kernel): [tap][C+1][F1] weights (ratio row zero at t = 0), 4 bias floats, bf16 copy.
static bool pack_step_mode() {
  static const bool v = svae_knob("SVAE_PACK_STEP", 0) == 1;
  return v;
}

static void pack_out_all(svae_ctx* c, hipStream_t st) {
  if (pack_step_mode()) return;
  const Model& M = c->m;
  const Geo& g = M.g;
  for (int t0 = 0; t0 < g.Te; t0 += PACK_MAXT) {
    const int nt = std::min(PACK_MAXT, g.Te - t0);
    PackOutArgs a{};
    a.P = c->P;
    a.C = g.C;
    a.F1 = g.F[1];
    a.nsp = g.split ? 3 : 1;
    for (int i = 0; i < nt; ++i) {
      const int t = t0 + i;
      const GenStep& G = M.gen[t];
      a.owout[i] = G.owout;
      a.obout[i] = G.obout;
      a.owratio[i] = t >= 1 ? G.owratio : -1;
      a.obratio[i] = t >= 1 ? G.obratio : -1;
      a.wpack[i] = c->sb[t].wpack;
      a.wpack_h[i] = g.bf16 ? (__bf16*)c->sb[t].wpack_h : nullptr;
    }
    pack_out(a, nt, st);
  }
}

// split_latent of every step, one launch per level over all steps (splitfc_fwd_steps, grid.y = step), top
// level first: ev_top after it (the top FC of step 0 waits only on that), ev_all after the rest
static void split_latent_fwd_all(svae_ctx* c, hipStream_t stream, hipEvent_t ev_top, hipEvent_t ev_all) {
  const Model& M = c->m;
  const Geo& g = M.g;
  const int B = g.B, L = g.L;
  const int* F = g.F;
  const int* S = g.S;
  int zoff[8] = {};
  for (int i = 1; i < L; ++i) zoff[i] = zoff[i - 1] + g.D[i - 1];
  for (int pass = 0; pass < 2; ++pass) {
    for (int i = pass == 0 ? L - 1 : 0; i < (pass == 0 ? L : L - 1); ++i) {
      for (int t0 = 0; t0 < g.Te; t0 += SFC_MAXT) {
        const int nt = std::min(SFC_MAXT, g.Te - t0);
        SfcSteps a{};
        for (int k = 0; k < nt; ++k) {
          const int t = t0 + k;
          svae_ctx::StepBufs& s = c->sb[t];
          const FcL& f = M.gen[t].split[i];
          a.W[k] = c->P + f.ow;
          a.beta[k] = c->P + f.obeta;
          a.mean[k] = s.split_mean[i];
          a.invstd[k] = s.split_inv[i];
          if (i < L - 1) {
            a.out[k] = elem_off(s.cat[i], F[i + 1], c->cbf);
            a.o_n[k] = (long long)S[i + 1] * S[i + 1] * 2 * F[i + 1];
          } else {
            a.out[k] = s.top_cat + (t >= 1 ? F[L] : 0);
            a.o_n[k] = s.ktop;
          }
        }
        const int J = M.gen[t0].split[i].nout;
        const float* z0 = c->z + (long long)t0 * B * g.Dz;
        if (i < L - 1)
          splitfc_fwd_steps(z0, (long long)B * g.Dz, g.Dz, zoff[i], B, g.D[i], J, F[i + 1], 2 * F[i + 1], c->cbf, a, nt,
                            stream);
        else
          splitfc_fwd_steps(z0, (long long)B * g.Dz, g.Dz, zoff[i], B, g.D[i], J, J, 0, 0, a, nt, stream);
      }
    }
    hipEventRecord(pass == 0 ? ev_top : ev_all, stream);
  }
}

static void split_latent_fwd(svae_ctx* c, int t, hipStream_t stream) {
  const Model& M = c->m;
  const Geo& g = M.g;
  const int B = g.B, L = g.L;
  const int* F = g.F;
  const int* S = g.S;
  svae_ctx::StepBufs& s = c->sb[t];
  const GenStep& G = M.gen[t];
  const float* zt = c->z + (long long)t * B * g.Dz;
  int zoff = 0;
  for (int i = 0; i < L; ++i) {
    const FcL& f = G.split[i];
    if (i < L - 1) {
      splitfc_fwd(zt, g.Dz, zoff, B, g.D[i], c->P + f.ow, c->P + f.obeta, f.nout, s.split_mean[i], s.split_inv[i],
                  elem_off(s.cat[i], F[i + 1], c->cbf), (long long)S[i + 1] * S[i + 1] * 2 * F[i + 1], F[i + 1],
                  2 * F[i + 1], stream, c->cbf);
    } else {
      const int coff = t >= 1 ? F[L] : 0;
      splitfc_fwd(zt, g.Dz, zoff, B, g.D[i], c->P + f.ow, c->P + f.obeta, f.nout, s.split_mean[i], s.split_inv[i],
                  s.top_cat + coff, s.ktop, f.nout, 0, stream);
    }
    zoff += g.D[i];
  }
}

// training_samples[t] (:963, :1090): what step t+1 (encoder, highway, Latent InfoMax recognition)
// consumes -- the MLE unless chain noise perturbs it
static const float* chain_x(const svae_ctx* c, int t) {
  const svae_ctx::StepBufs& s = c->sb[t];
  return s.has_sample ? s.sample : s.xhat;
}

// stddevs_prediction of step t (:1866-1875) on conv_output = sigmoid(output conv-T pre-activation),
// then sample = mle + reg * sd * noise and the NLL per-image partials (:1090, :1149-1150)
static void sd_forward(svae_ctx* c, int t) {
  const Geo& g = c->m.g;
  const GenStep& G = c->m.gen[t];
  svae_ctx::StepBufs& s = c->sb[t];
  hipStream_t st = c->st;
  const long long P = (long long)g.B * g.H * g.W;
  const int nblk = sd_pixel_blocks(P);
  const float* in = s.a_out;
  int ldi = g.C + 1, sig = 1;
  for (int l = 0; l < g.sd_nl; ++l) {
    const int Ci = g.sd_F[l], Co = g.sd_F[l + 1];
    sd_conv_fwd(in, ldi, sig, Ci, c->P + G.sd[l].ow, Co, g.H, g.W, P, s.sd_pre[l], c->sd_part, st);
    sd_stat_fin(c->sd_part, nblk, Co, P, 1e-3f, 0, s.sd_mean[l], s.sd_inv[l], nullptr, nullptr, st);
    sd_bn_apply(s.sd_pre[l], Co, P, s.sd_mean[l], s.sd_inv[l], c->P + G.sd[l].obeta, s.sd_act[l], st);
    in = s.sd_act[l];
    ldi = Co;
    sig = 0;
  }
  sd_head_fwd(in, g.sd_F[g.sd_nl], c->P + G.owsd, c->P + G.obsd, g.sd_max, s.xhat, c->tgt_in,
              c->noise_used + (long long)t * P * g.C, c->reg, g.B, g.C, g.H * g.W, s.sd, s.sample, s.rec_part,
              c->out_nblk, st);
}

// backward of sd_forward's head: dmle (-> c->dmle) = dsample + NLL term; the stddev network's
// gradients; its input gradient accumulates into da (the output conv-T pre-activation)
static void sd_backward(svae_ctx* c, int t, const float* dsample, float nll_coef) {
  const Geo& g = c->m.g;
  const GenStep& G = c->m.gen[t];
  svae_ctx::StepBufs& s = c->sb[t];
  hipStream_t st = c->st;
  const long long P = (long long)g.B * g.H * g.W;
  const int nblk = sd_pixel_blocks(P);
  const int nl = g.sd_nl;
  sd_head_bwd(s.sd_act[nl - 1], g.sd_F[nl], c->P + G.owsd, c->P + G.obsd, g.sd_max, s.xhat, c->tgt_in,
              c->noise_used + (long long)t * P * g.C, c->reg, nll_coef, dsample, g.C, P, c->dmle, c->sd_d[0],
              c->sd_wpart, c->Gr + G.owsd, c->Gr + G.obsd, st);
  int cur = 0;
  for (int l = nl - 1; l >= 0; --l) {
    const int Ci = g.sd_F[l], Co = g.sd_F[l + 1];
    const ConvL& L = G.sd[l];
    const float* dact = c->sd_d[cur];
    sd_bn_bwd_reduce(dact, s.sd_pre[l], Co, P, s.sd_mean[l], s.sd_inv[l], c->P + L.obeta, c->sd_part, st);
    sd_stat_fin(c->sd_part, nblk, Co, P, 0.f, 1, nullptr, nullptr, c->sd_sums, c->Gr + L.obeta, st);
    sd_bn_bwd_apply(dact, s.sd_pre[l], Co, P, s.sd_mean[l], s.sd_inv[l], c->P + L.obeta, c->sd_sums, c->sd_dpre, st);
    if (l > 0) {
      sd_conv_wgrad(s.sd_act[l - 1], Ci, 0, Ci, c->sd_dpre, Co, g.B, g.H, g.W, c->sd_wpart, c->Gr + L.ow, st);
      sd_conv_dgrad(c->sd_dpre, Co, c->P + L.ow, Ci, g.H, g.W, P, c->sd_d[cur ^ 1], Ci, nullptr, 0, 0, st);
      cur ^= 1;
    } else {  // layer 0's input gradient waits in sd_dpre for sd_backward_input
      sd_conv_wgrad(s.a_out, g.C + 1, 1, Ci, c->sd_dpre, Co, g.B, g.H, g.W, c->sd_wpart, c->Gr + L.ow, st);
    }
  }
}

// d conv_output of the stddev network, times sigmoid', added into da after output_bwd wrote it
static void sd_backward_input(svae_ctx* c, int t) {
  const Geo& g = c->m.g;
  const long long P = (long long)g.B * g.H * g.W;
  sd_conv_dgrad(c->sd_dpre, g.sd_F[1], c->P + c->m.gen[t].sd[0].ow, g.C, g.H, g.W, P, c->da, g.C + 1, c->sb[t].a_out,
                g.C + 1, 1, c->st);
}

// ============================================================================
// forward
// ============================================================================
static int engine_forward(svae_ctx* c) {
  Model& M = c->m;
  const Geo& g = M.g;
  const int B = g.B, L = g.L, T = g.T;
  const int* F = g.F;
  const int* S = g.S;
  const long long wg = M.phi_stride;
  hipStream_t st = c->st;
  int r;

  if ((r = acc_reset(c))) return r;
  if (M.shared) share_broadcast(c->Ppub, c->Pv, c->share_seg, c->share_nseg, st);
  // the shadows are current when the last Adam updates covered the whole live region
  if (g.bf16 && !(c->fresh == M.n_live && !M.shared)) {
    // split mode: every tensor's fp16-plane exponent from its max |w| first (clears the overflow flag)
    if (g.split) wexp_refresh(c->P, c->winfo_d, c->nwinfo, c->wtab, c->wovf, st);
    shadow_weights(c->P, c->wN, c->wT, M.n_live, c->tiles_d, c->ntiles, c->offs_d, c->nsp, c->wplane, st, c->wtab);
  } else if (g.split) {
    // the planes the Adam updates wrote: re-made at fresh exponents if a weight outgrew its tensor's
    // (one block that returns at once unless the flag is up)
    wexp_fixup(c->P, c->winfo_d, c->nwinfo, c->wtab, c->wovf, c->wN, c->wT, c->wplane, st);
  }
  c->fresh = 0;
  if (g.noisy) {  // chain noise N(0,1) [T,B,H,W,C] (tf.random_normal(image_batch_shape), :1090)
    const long long n = (long long)T * B * g.H * g.W * g.C;
    if (c->noise_in) {
      c->noise_used = c->noise_in;
    } else {
      philox_normal(c->noise_buf, n, 0xC4A1C4A1ULL, c->rng_offset, st);
      c->rng_offset += (n + 3) / 4;
      c->noise_used = c->noise_buf;
    }
  }
  if (c->generative) {
    // generative mode (sequential_vae.py:947-952, :1025 latent_generative = self.latents[t]):
    // z_t comes from the caller (or N(0,1)), the recognition networks do not run
    const long long n = (long long)T * B * g.Dz;
    if (c->eps_in) {
      HIPCHK(c, hipMemcpyAsync(c->z, c->eps_in, n * sizeof(float), hipMemcpyDeviceToDevice, st));
    } else {
      philox_normal(c->z, n, 0x6E6E6E6EULL, c->rng_offset, st);
      c->rng_offset += (n + 3) / 4;
    }
    HIPCHK(c, hipMemsetAsync(c->kl_img, 0, (size_t)T * B * sizeof(float), st));
  } else {
  // eps for every step up front (device Philox unless injected)
  const float* eps = c->eps_in;
  if (!eps) {
    philox_normal(c->eps_buf, (long long)T * B * g.Dz, 0x5EED5EEDULL, c->rng_offset, st);
    c->rng_offset += ((long long)T * B * g.Dz + 3) / 4;
    eps = c->eps_buf;
  }
  c->eps_used = eps;
  // recognition: q(z_t | x) for every step at once (groups = T), or, in Latent InfoMax mode,
  // q(z_0 | x) here and q(z_t | x_{t-1}) inside the chain (create_recognition_network :1013-1027)
  if (c->rec_split && c->st4 && !g.plc && T > 1) {
    if ((r = inference_fwd(c, 0, 1, View{(float*)c->x_in, g.C, 0}))) return r;
    hipEventRecord(c->ev_rs, st);
    hipStreamWaitEvent(c->st4, c->ev_rs, 0);
    hipStream_t s0 = c->st;
    float* sl0 = c->slab;
    c->st = c->st4;
    c->slab = c->slab4;
    r = inference_fwd(c, 1, T - 1, View{(float*)c->x_in, g.C, 0});
    c->st = s0;
    c->slab = sl0;
    if (r) return r;
    hipEventRecord(c->ev_rs2, c->st4);
  } else if ((r = inference_fwd(c, 0, g.plc ? 1 : T, View{(float*)c->x_in, g.C, 0}))) {
    return r;
  }
  }  // !generative
  const bool rsplit = c->rec_split && c->st4 && !g.plc && T > 1 && !c->generative;
  // split_latent of every step on the side stream (z is known for all steps unless Latent
  // InfoMax draws z_t inside the chain); step t's decoder waits on ev_sfc[t]
  static const int sfc_mode = svae_knob("SVAE_SFC", 1);  // 0 = split-latent forward on the main stream per step
  const bool sfc_side = sfc_mode != 0 && c->side && !g.plc && T <= 64;
  // output / ratio operands packed before the split-latent hand-over to st3 (+0.5 % per step in a
  // same-box A/B, profiles/r03_ab3.txt); SVAE_PACK_FIRST=0 packs after it (round 2's order)
  static const bool pack_first = svae_knob("SVAE_PACK_FIRST", 1) != 0;
  if (pack_first) pack_out_all(c, st);
  // every step's split-latent forward batched per level (SVAE_SFC_STEPS=0: one launch per level and step, the
  // round-5 schedule); not with the knob-only recognition split, whose z_t of steps >= 1 arrive later
  static const bool sfc_steps = svae_knob("SVAE_SFC_STEPS", 1) != 0;
  const bool sfc_all = sfc_side && sfc_steps && !rsplit;
  if (sfc_side) {
    hipEventRecord(c->ev_aux, st);
    hipStreamWaitEvent(c->st3, c->ev_aux, 0);
    if (sfc_all) {
      split_latent_fwd_all(c, c->st3, c->ev_sfc[0], c->ev_sfc[1]);
    } else {
      for (int t = 0; t < g.Te; ++t) {
        if (t == 1 && rsplit) hipStreamWaitEvent(c->st3, c->ev_rs2, 0);  // z_t of steps >= 1 (st4)
        split_latent_fwd(c, t, c->st3);
        hipEventRecord(c->ev_sfc[t], c->st3);
      }
    }
  }

  if (!pack_first) pack_out_all(c, st);

  // ---------------- the chain ----------------
  for (int t = 0; t < T; ++t) {
    svae_ctx::StepBufs& s = c->sb[t];
    if (t == 1 && rsplit) hipStreamWaitEvent(st, c->ev_rs2, 0);  // recognition of steps >= 1 (st4)
    if (t >= g.Te) {  // external generator step: only its KL statistics here (recon 0: the caller's)
      HIPCHK(c, hipMemsetAsync(s.rec_part, 0, (size_t)B * c->out_nblk * sizeof(float), st));
      loss_reduce(s.rec_part, c->out_nblk, c->kl_img + (long long)t * B, B, g.H * g.W * g.C, s.stats, s.rec_img, st);
      continue;
    }
    const GenStep& G = M.gen[t];
    const float* xprev = t >= 1 ? chain_x(c, t - 1) : nullptr;
    if (g.plc && t >= 1 && !c->generative)  // Latent InfoMax: z_t from the previous sample (:1014-1015)
      if ((r = inference_fwd(c, t, 1, View{(float*)xprev, g.C, 0}))) return r;
    // g_theta encoder of x_{t-1}  (compute_encodings :1764-1777)
    if (t >= 1) {
      const EncStep& E = M.enc[t];
      View in{(float*)xprev, g.C, 0};
      for (int lvl = 0; lvl < L - 1; ++lvl) {
        const int Fl = F[lvl + 1];
        Defer da;  // conv a's apply deferred to st2 (SVAE_FOLD): conv b's gather stages it from pre
        r = conv_bn_act_fwd(c, E.a[lvl], 1, 0, in, s.enc_pre_a[lvl], 0, s.enc_bn_a[lvl], 0, View{}, ACT_LRELU,
                            View{s.enc_act_a[lvl], Fl, 0, c->abf}, &da);
        if (r) return r;
        r = conv_bn_act_fwd(c, E.b[lvl], 1, 0, View{s.enc_act_a[lvl], Fl, 0, c->abf, da.pre ? &da : nullptr}, s.enc_pre_b[lvl], 0, s.enc_bn_b[lvl], 0,
                            View{}, ACT_LRELU, View{s.enc_act_b[lvl], Fl, 0});
        if (r) return r;
        in = View{s.enc_act_b[lvl], Fl, 0};
      }
      r = conv_bn_act_fwd(c, E.c, 1, 0, in, s.enc_c_pre, 0, s.enc_bn_c, 0, View{}, ACT_LRELU,
                          View{s.enc_c_act, F[L - 1], 0, c->abf});
      if (r) return r;
      r = fc_bn_fwd(c, E.fc, View{s.enc_c_act, S[L] * S[L] * F[L - 1], 0, c->abf}, s.encfc_pre, s.enc_bn_fc,
                    View{s.top_cat, s.ktop, 0});
      if (r) return r;
    }
    // split_latent (:1796-1806): ladder_i straight into the concat buffers
    if (sfc_all) {
      if (t == 0) hipStreamWaitEvent(st, c->ev_sfc[0], 0);  // the top level of every step
    } else if (sfc_side) {
      hipStreamWaitEvent(st, c->ev_sfc[t], 0);
    } else {
      split_latent_fwd(c, t, st);
    }
    // generator_ladder decoder (:1695-1721)
    r = fc_bn_fwd(c, G.top, View{s.top_cat, s.ktop, 0}, s.top_pre, s.top_bn, View{s.top_act, S[L] * S[L] * F[L], 0, c->abf});
    if (r) return r;
    View cur{s.top_act, F[L], 0, c->abf};
    Defer ds1;  // s1[lvl >= 1]'s apply deferred to st2 (SVAE_FOLD): s2[lvl-1]'s conv-T gather stages it
    for (int lvl = L - 2; lvl >= 0; --lvl) {
      const int Fl = F[lvl + 1];
      View res = t >= 1 ? View{s.enc_act_b[lvl], Fl, 0} : View{};
      r = conv_bn_act_fwd(c, G.s2[lvl], 1, 0, cur, s.s2_pre[lvl], 0, s.s2_bn[lvl], 0, res, ACT_RELU,
                          View{s.cat[lvl], 2 * Fl, 0, c->cbf});
      if (r) return r;
      if (sfc_all && t == 0 && lvl == L - 2) hipStreamWaitEvent(st, c->ev_sfc[1], 0);  // the other levels, every step
      r = conv_bn_act_fwd(c, G.s1[lvl], 1, 0, View{s.cat[lvl], 2 * Fl, 0, c->cbf}, s.s1_pre[lvl], 0, s.s1_bn[lvl], 0, View{},
                          ACT_RELU, View{s.s1_act[lvl], Fl, 0, c->abf}, lvl >= 1 ? &ds1 : nullptr);
      if (r) return r;
      cur = View{s.s1_act[lvl], Fl, 0, c->abf, (lvl >= 1 && ds1.pre) ? &ds1 : nullptr};
    }
    // output + ratio conv-T (:1720, :1727) as one 4-channel small-N gather
    {
      const int C1 = g.C + 1;
      const int F1 = F[1];
      // pack [tap][C+1][F1] (ratio row zero at t=0) for the fused output conv-T and its dgrad
      // (wpack / wpack_h / bias packed for every step by pack_out_all at the start of the forward;
      // SVAE_PACK_STEP=1: the former per-step copies, kept for bitwise A/B checks)
      float* bpack = s.wpack + 16 * C1 * F1;
      if (pack_step_mode()) {
        HIPCHK(c, hipMemsetAsync(s.wpack, 0, (size_t)(16 * C1 * F1 + 4) * sizeof(float), st));
        HIPCHK(c, hipMemcpyAsync(bpack, c->P + G.obout, g.C * sizeof(float), hipMemcpyDeviceToDevice, st));
        if (t >= 1) HIPCHK(c, hipMemcpyAsync(bpack + g.C, c->P + G.obratio, sizeof(float), hipMemcpyDeviceToDevice, st));
        HIPCHK(c, hipMemcpy2DAsync(s.wpack, (size_t)C1 * F1 * sizeof(float), c->P + G.owout,
                                   (size_t)g.C * F1 * sizeof(float), (size_t)g.C * F1 * sizeof(float), 16,
                                   hipMemcpyDeviceToDevice, st));
        if (t >= 1)
          HIPCHK(c, hipMemcpy2DAsync(s.wpack + g.C * F1, (size_t)C1 * F1 * sizeof(float), c->P + G.owratio,
                                     (size_t)F1 * sizeof(float), (size_t)F1 * sizeof(float), 16,
                                     hipMemcpyDeviceToDevice, st));
        if (g.bf16)
          shadow_weights(s.wpack, s.wpack_h, nullptr, 16LL * C1 * F1, nullptr, 0, nullptr, g.split ? 3 : 1,
                         g.split ? 16LL * C1 * F1 : 0, st);
      }
      ConvGeom og{GM_CONVT, B, S[1], S[1], g.H, g.W, 2, 1, 4};
      if (g.bf16) {  // small-N conv-T gather (split mode: on the three planes of the packed weights), bias in the epilogue
        FwdArgs a{};
        a.A = cur.p; a.lda = F1; a.a_bf16 = cur.bf;
        a.B = s.wpack;  // (fp32 fallback)
        a.Bh = s.wpack_h; a.b_nk = 1; a.ldb = F1; a.b_tap = (long long)C1 * F1;
        a.b_plane = g.split ? 16LL * C1 * F1 : 0;
        a.C = s.a_out; a.ldc = C1;
        a.N = C1; a.Cin = F1;
        a.g = og;
        a.rows = B * (g.H / 2) * (g.W / 2); a.nclass = 4;
        a.bias = bpack;
        gemm(c, a, 1);
      } else {
        gconv_smalln(cur.p, F1, F1, s.wpack, C1, nullptr, 0, (long long)C1 * F1, 0, bpack, nullptr, og,
                     (long long)B * g.H * g.W, s.a_out, C1, 0, st);
      }
      output_fwd(s.a_out, B, g.H * g.W, g.C, xprev, c->tgt_in, g.lo, g.hi, g.minh, g.maxh, s.xhat, s.rec_part,
                 c->out_nblk, st);
      const long long nimg = (long long)B * g.H * g.W * g.C;
      if (g.pgn)  // predicted stddevs: noisy sample and the NLL partials (replace the MSE partials)
        sd_forward(c, t);
      else if (s.has_sample)  // fixed noise_stddevs[t]
        chain_noise(s.xhat, c->noise_used + t * nimg, c->reg * g.nstd[t], nimg, s.sample, st);
      loss_reduce(s.rec_part, c->out_nblk, c->kl_img + (long long)t * B, B, g.H * g.W * g.C, s.stats, s.rec_img, st);
      if (g.imp && t >= 1)  // ||mle_t - mle_{t-1}||^2 per image (:1190-1191)
        sqdiff_img(s.xhat, c->sb[t - 1].xhat, B, (long long)g.H * g.W * g.C, c->imp_img + (long long)t * B, st);
    }
  }
  if (c->fold_used) {  // the deferred applies (st2) before anything after the forward
    hipEventRecord(c->ev_fold_join, c->st2);
    hipStreamWaitEvent(st, c->ev_fold_join, 0);
    c->fold_used = false;
  }
  return 0;
}

// ============================================================================
// backward  (d self.loss / d theta, phi; sequential_vae.py:1273)
// ============================================================================
// Backward of the recognition ladders of steps [t0, t0+n) (reverse of inference_fwd): dz_t ->
// latent / heads / ladder weight gradients; dx0 != nullptr adds d loss / d in0 (one step).
static int inference_bwd(svae_ctx* c, int t0, int n, View in0, float* dx0) {
  Model& M = c->m;
  const Geo& g = M.g;
  const int B = g.B, L = g.L;
  const int* F = g.F;
  const int* S = g.S;
  const long long wg = M.phi_stride;
  hipStream_t st = c->st;
  int r;
  const long long ms = (long long)B * g.Dz;
  if (c->side) hipStreamWaitEvent(st, c->ev_dz, 0);  // dz_t: split-latent backward (st3)
  // the improvement-loss pass carries no KL term
  latent_bwd(c->mu + t0 * ms, c->sig + t0 * ms, c->eps_used + t0 * ms, c->dz + t0 * ms, ms, ms, B, g.Dz,
             (c->imp_pass ? c->kl_zero : c->kl_coef) + t0, 1, g.prior, g.uniform, g.clipv, c->dhead,
             (long long)B * 2 * g.Dz, n, st);
  const InfStep& I0 = M.inf[t0];
  auto bns = [&](const BNS& b, int C) { return BNS{b.mean + (long long)t0 * C, b.invstd + (long long)t0 * C}; };
  auto act_a = [&](int l) { return elem_off(c->inf_act_a[l], t0 * c->inf_gs[l], c->abf); };
  auto act_b = [&](int l) { return c->inf_act_b[l] + t0 * c->inf_gs[l]; };
  auto pre_a = [&](int l) { return elem_off(c->inf_pre_a[l], t0 * c->inf_gs[l], c->pbf); };
  auto pre_b = [&](int l) { return elem_off(c->inf_pre_b[l], t0 * c->inf_gs[l], c->pbf); };
  // heads of ladder level l -> idb (first write), l's own conv-a input gradient (level l+1) after them
  auto heads_of = [&](int l) {
    bool first = true;
    for (int hl = 0; hl < L; ++hl) {
      const HeadL& h = I0.head[hl];
      if (h.src_level != l) continue;
      const long long gl = c->inf_gs[l];
      heads_bwd(act_b(l), gl, c->idb, gl, B, h.nin, c->P + h.owm, c->P + h.ows, wg, h.d, c->dhead,
                (long long)B * 2 * g.Dz, 2 * g.Dz, h.off, c->Gr + h.owm, c->Gr + h.ows, c->Gr + h.obm, c->Gr + h.obs,
                first ? 0 : 1, n, st);
      first = false;
    }
    return !first;  // wrote idb
  };
  BwFuse fu_ib;  // level lvl's conv-b BN partials from level lvl+1's conv-a input-gradient epilogue
  for (int lvl = L - 2; lvl >= 0; --lvl) {
    const int Fl = F[lvl + 1];
    const long long gs = c->inf_gs[lvl];
    const long long rows = (long long)B * S[lvl + 1] * S[lvl + 1];
    if (lvl == L - 2) heads_of(lvl);
    Slot sb = idpre_next(c, n * gs);
    r = bn_act_bwd(c, n, rows, Fl, View{c->idb, Fl, gs}, View{act_b(lvl), Fl, gs}, pre_b(lvl), gs, Fl,
                   bns(c->inf_bn_b[lvl], Fl), Fl, I0.b[lvl].obeta, wg, ACT_LRELU, sb.p, gs, View{}, 0, &fu_ib,
                   dpre_bf(c, I0.b[lvl]), c->pbf);
    if (r) return r;
    {
      const ConvL Lw = I0.b[lvl];
      const View in_{act_a(lvl), Fl, gs, c->abf};
      const float* dp = sb.p;
      float* dW = c->Gr + Lw.ow;
      r = on_side_q(c, sb.ready, [=] { return conv_wgrad(c, Lw, n, wg, in_, dp, gs, dW); });
    }
    if (r) return r;
    BwFuse fu_ia = bw_fuse(c, pre_a(lvl), Fl, gs, nullptr, 0, 0, bns(c->inf_bn_a[lvl], Fl), Fl, I0.a[lvl].obeta, wg,
                           ACT_LRELU, Fl, c->pbf);
    r = conv_dgrad(c, I0.b[lvl], n, wg, sb.p, gs, View{c->ida, Fl, gs}, 0, &fu_ia);
    if (r) return r;
    Slot sa = idpre_next(c, n * gs);
    r = bn_act_bwd(c, n, rows, Fl, View{c->ida, Fl, gs}, View{act_a(lvl), Fl, gs}, pre_a(lvl), gs, Fl,
                   bns(c->inf_bn_a[lvl], Fl), Fl, I0.a[lvl].obeta, wg, ACT_LRELU, sa.p, gs, View{}, 0, &fu_ia,
                   dpre_bf(c, I0.a[lvl]), c->pbf);
    if (r) return r;
    View in = lvl == 0 ? in0 : View{act_b(lvl - 1), F[lvl], c->inf_gs[lvl - 1]};
    {
      const ConvL Lw = I0.a[lvl];
      const float* dp = sa.p;
      float* dW = c->Gr + Lw.ow;
      // the backward's last weight gradient (the image conv of every step's ladder) on the main stream,
      // which has nothing left to run: it overlaps the side stream's backlog instead of queueing behind it
      // (SVAE_TAIL_MAIN=0: the side stream, round 5)
      static const bool tail_main = svae_knob("SVAE_TAIL_MAIN", 1) != 0;
      if (lvl == 0 && !dx0 && tail_main && c->side)
        r = conv_wgrad(c, Lw, n, wg, in, dp, gs, dW);
      else
        r = on_side_q(c, sa.ready, [=] { return conv_wgrad(c, Lw, n, wg, in, dp, gs, dW); });
    }
    if (r) return r;
    if (lvl > 0) {
      const bool wrote = heads_of(lvl - 1);
      fu_ib = bw_fuse(c, pre_b(lvl - 1), F[lvl], c->inf_gs[lvl - 1], nullptr, 0, 0, bns(c->inf_bn_b[lvl - 1], F[lvl]), F[lvl],
                      I0.b[lvl - 1].obeta, wg, ACT_LRELU, F[lvl], c->pbf);
      r = conv_dgrad(c, I0.a[lvl], n, wg, sa.p, gs, View{c->idb, F[lvl], c->inf_gs[lvl - 1]}, wrote ? 1 : 0, &fu_ib);
      if (r) return r;
    } else if (dx0) {  // Latent InfoMax: d loss / d x_{t-1} through q(z_t | x_{t-1})
      r = conv_dgrad(c, I0.a[0], n, wg, sa.p, gs, View{dx0, g.C, 0}, 1);
      if (r) return r;
    }
  }
  return 0;
}

static int engine_backward_pass(svae_ctx* c);
// the pass, then whatever side-stream work is still queued (early debug returns, errors)
static int engine_backward(svae_ctx* c) {
  const int r = engine_backward_pass(c);
  const int r2 = side_flush(c);
  c->side_q.clear();
  return r ? r : r2;
}
static int engine_backward_pass(svae_ctx* c) {
  Model& M = c->m;
  const Geo& g = M.g;
  const int B = g.B, L = g.L, T = g.T;
  const int* F = g.F;
  const int* S = g.S;
  const int C1 = g.C + 1;
  const long long P0 = (long long)B * g.H * g.W;
  const long long wg = M.phi_stride;
  hipStream_t st = c->st;
  int r;

  if ((r = acc_reset(c))) return r;
  HIPCHK(c, hipMemsetAsync(c->dz, 0, (size_t)T * B * g.Dz * sizeof(float), st));
  if (g.Te < T && c->ext_dz) {  // d loss / d z_t of the external generator's steps (t >= Te)
    const long long off = (long long)g.Te * B * g.Dz;
    HIPCHK(c, hipMemcpyAsync(c->dz + off, c->ext_dz + off, (size_t)((long long)T * B * g.Dz - off) * sizeof(float),
                             hipMemcpyDeviceToDevice, st));
  }
  const bool rec_ov = c->side && c->st4 && c->rec_group > 0 && !g.plc && g.Te == T;
  if (rec_ov) {  // st4 starts after the forward and the accumulator / dz zeroing
    hipEventRecord(c->ev_start, st);
    hipStreamWaitEvent(c->st4, c->ev_start, 0);
  }
  if (c->side) {  // the side stream starts after the forward (and anything before it)
    hipEventRecord(c->ev_start, st);
    hipStreamWaitEvent(c->st2, c->ev_start, 0);
    if (c->st2b) hipStreamWaitEvent(c->st2b, c->ev_start, 0);
    // re-arm the slot-free events on the main stream: the previous backward's side-stream work
    // was joined into it, so "free" holds now, and every later wait depends only on work of this
    // pass (required when the step is captured into a graph)
    // the previous pass's readers were joined into this stream: every per-pass region is free
    c->dpre_off = c->idpre_off = c->dcat_off = c->dtop_off = 0;
  }
  for (int t = g.Te - 1; t >= 0; --t) {
    if (t < g.Te - 1) {
      if (g.plc) {  // q(z_{t+1} | x_t): its weights' gradients and its share of d loss / d x_t
        r = inference_bwd(c, t + 1, 1, View{(float*)chain_x(c, t), g.C, 0}, c->dx[t & 1]);
        if (r) return r;
      }
      if ((r = step_hook(c, t + 1))) return r;  // step t+1's gradients are complete
    }
    if (t < c->dbg_stop_step) return 0;  // debug: stop after step dbg_stop_step
    svae_ctx::StepBufs& s = c->sb[t];
    const GenStep& G = M.gen[t];
    const float* xprev = t >= 1 ? chain_x(c, t - 1) : nullptr;
    // d loss / d training_samples[t]: from step t+1's backward, or for the last internal step from
    // the external generator (svae_set_external_grads)
    const float* dxin = t < g.Te - 1 ? c->dx[t & 1] : (g.Te < T ? c->ext_dx : nullptr);
    float* dxout = t >= 1 ? c->dx[(t - 1) & 1] : nullptr;
    const float cf = t == 0 ? g.c_first : 1.f;
    float rec_coef = (g.interm || t == T - 1) ? 16.f * cf / (float)(P0 * g.C) : 0.f;
    const float imp_coef = -c->reg * g.lp_coef / (float)B;
    if (c->imp_pass) {  // improvement loss: its d / d mle_t seeds the chain instead of the ELBO's
      rec_coef = 0.f;
      if (!g.pgn) {  // d sample / d mle = 1: the seed joins the chain gradient
        imp_seed(dxin, t >= 1 ? c->sb[t - 1].xhat : nullptr, s.xhat, t < T - 1 ? c->sb[t + 1].xhat : nullptr,
                 imp_coef, P0 * g.C, c->dseed, st);
        dxin = c->dseed;
      }
    }
    float* dzt = c->dz + (long long)t * B * g.Dz;
    BwFuse fu_s1;  // s1[lvl]'s BN partials: from the output layer's (lvl 0) / s2[lvl-1]'s input-gradient epilogue

    // ---- output + highway (:1720-1729)
    c->da = c->da_base + (long long)t * P0 * C1;  // own region per step: no wait for the previous reader
    if (g.pgn) {  // NLL + sample = mle + reg*sd*noise: d mle and the stddev network, then the output layer
      sd_backward(c, t, dxin, rec_coef);  // rec_coef = 16 cf / (B H W C), the NLL's element weight
      if (c->imp_pass)  // the improvement seed is on the MLE, not on the noisy sample: no stddev term
        imp_seed(c->dmle, t >= 1 ? c->sb[t - 1].xhat : nullptr, s.xhat, t < T - 1 ? c->sb[t + 1].xhat : nullptr,
                 imp_coef, P0 * g.C, c->dmle, st);
      output_bwd(s.a_out, B, g.H * g.W, g.C, xprev, s.xhat, c->tgt_in, g.lo, g.hi, g.minh, g.maxh, 0.f, c->dmle, c->da,
                 dxout, st);
      // the stddev network's input gradient (d conv_output) joins da after output_bwd wrote it
      sd_backward_input(c, t);
    } else {
      output_bwd(s.a_out, B, g.H * g.W, g.C, xprev, s.xhat, c->tgt_in, g.lo, g.hi, g.minh, g.maxh, rec_coef, dxin,
                 c->da, dxout, st);
    }
    {
      // packed [C | ratio] columns; at t=0 the ratio column of da is zero (output_bwd) and its
      // gradient row is dropped by the reduce -> always the 4-wide vector gather
      const int M_out = C1;
      WgArgs w{};
      w.G = c->da; w.ldg = C1;
      w.D = s.s1_act[0]; w.ldd = F[1]; w.d_bf16 = c->abf;
      w.M = M_out; w.N = F[1];
      w.g = ConvGeom{GM_CONV, B, g.H, g.W, S[1], S[1], 2, 1, 4};
      w.ntap = 16;
      w.rows = B * S[1] * S[1];
      const bool bfk = g.bf16 && !g.split;  // (split mode: the fp32 weight-GEMM)
      if (bfk)
        choose_split(w.rows, 1, wgrad_bf16_tiles(w), 1, 16LL * M_out * F[1], c->slab_cap, w.nsplit, w.chunk, 2048,
                     256);
      else
        choose_split(w.rows, 16, (F[1] + 127) / 128, 1, 16LL * M_out * F[1], c->slab_cap, w.nsplit, w.chunk);
      w.nsp = g.split ? 2 : 1;
      float* da = c->da;
      const int F1 = F[1], Cc = g.C;
      float* gout = c->Gr + G.owout;
      float* gratio = t >= 1 ? c->Gr + G.owratio : nullptr;
      float* gbout = c->Gr + G.obout;
      float* gbratio = t >= 1 ? c->Gr + G.obratio : nullptr;
      c->side_pin = true;  // (colsum_small's cs_part scratch is shared by every step's closure)
      if ((r = on_side_q(c, c->ev_da_ready, [=]() mutable {
        w.part = c->slab;
        const int ns = (bfk || g.split) ? wgrad_smallc_part(w, 1, c->slab, c->slab_cap, c->st) : 0;
        if (ns) w.nsplit = ns;  // LDS im2col kernel (wgrad_smallc.hip)
        else wgemm(c, w, 1);
        wgrad_reduce(c->slab, 0, w.nsplit, 16, M_out, F1, gout, 0, Cc, gratio, 0, 0, 1, c->st);
        // output / ratio bias gradients (own scratch)
        colsum_small(da, C1, P0, M_out, c->cs_part, gbout, Cc, gbratio, c->st);
        return 0;
      }))) return r;
      c->side_pin = false;
      // d cur = conv-T dgrad (CONV gather over da with the packed [tap][C+1][F1] weights as KN)
      FwdArgs a{};
      a.A = c->da; a.lda = C1;
      a.B = s.wpack; a.b_nk = 0; a.ldb = F[1]; a.b_tap = (long long)C1 * F[1];
      a.C = c->dcur; a.ldc = F[1];
      a.N = F[1]; a.Cin = C1;
      a.g = ConvGeom{GM_CONV, B, g.H, g.W, S[1], S[1], 2, 1, 4};
      a.rows = B * S[1] * S[1]; a.nclass = 1;
      // s1[0]'s BN-backward partials in this input gradient's epilogue (small-channel kernel only)
      fu_s1 = BwFuse{};
      if (!nofuse_out()) {
        BwFuse f = bw_fuse(c, s.s1_pre[0], F[1], 0, nullptr, 0, 0, s.s1_bn[0], 0, G.s1[0].obeta, 0, ACT_RELU, F[1], c->pbf);
        FwdArgs t = a;
        t.bw = f.bw;
        t.stats = (u64*)1;  // (eligibility only)
        if (f.bw.C % 4 == 0 && smallc_ok(t, false)) {
          const AccR acc = acc_bn(c, 1, F[1], smallc_nrb(t));
          if (!acc.p) return fail(c, SVAE_EBADARG, "BN accumulator arena too small");
          a.bw = f.bw;
          set_stats(a, acc);
          f.acc = acc;
          f.used = true;
          fu_s1 = f;
        }
      }
      igemm_fwd(a, 1, st);
    }
    // ---- decoder levels, bottom-up (reverse of :1710-1717)
    float* dcur = c->dcur;
    float* dnext = c->dnext;
    for (int lvl = 0; lvl <= L - 2; ++lvl) {
      const int Fl = F[lvl + 1];
      const long long rows = (long long)B * S[lvl + 1] * S[lvl + 1];
      const ConvL& l1 = G.s1[lvl];
      const ConvL& l2 = G.s2[lvl];
      // s1: relu(BN(convT_s1(cat)))
      Slot sl = dpre_next(c, rows * Fl);
      r = bn_act_bwd(c, 1, rows, Fl, View{dcur, Fl, 0}, View{s.s1_act[lvl], Fl, 0}, s.s1_pre[lvl], 0, Fl, s.s1_bn[lvl],
                     0, l1.obeta, 0, ACT_RELU, sl.p, 0, View{}, 0, &fu_s1, dpre_bf(c, l1), c->pbf);
      if (r) return r;
      if (t == c->dbg_stop_step && lvl == c->dbg_stop_lvl2) { c->dbg_last = dcur; return 0; }
      {
        const ConvL Lw = l1;
        const View in_{s.cat[lvl], 2 * Fl, 0, c->cbf};
        const float* dp = sl.p;
        float* dW = c->Gr + Lw.ow;
        r = on_side_q(c, sl.ready, [=] { return conv_wgrad(c, Lw, 1, 0, in_, dp, 0, dW); });
      }
      if (r) return r;
      // s2[lvl]'s BN partials over the d-half of dcat (shortcut at t >= 1: act' from the stored y)
      BwFuse fu_s2 = bw_fuse(c, s.s2_pre[lvl], Fl, 0, t >= 1 ? s.cat[lvl] : nullptr, 2 * Fl, 0, s.s2_bn[lvl], 0,
                             l2.obeta, 0, ACT_RELU, Fl, c->pbf);
      fu_s2.bw.y_bf16 = t >= 1 ? c->cbf : 0;
      // dcat: its own region per pass when the split-latent backward reads it on the side stream
      float* dcat = c->side ? arena_next(c, c->dcat_arena, c->dcat_cap, c->dcat_off, rows * 2 * Fl, true) : c->dcat;
      r = conv_dgrad(c, l1, 1, 0, sl.p, 0, View{dcat, 2 * Fl, 0}, 0, &fu_s2);
      if (r) return r;
      // latent half of the concat -> split_latent level lvl (side stream: off the critical path)
      {
        const FcL& f = G.split[lvl];
        int zoff = 0;
        for (int i = 0; i < lvl; ++i) zoff += g.D[i];
        hipStream_t ss = st;
        if (c->side) {
          if ((r = side_flush(c, c->st3))) return r;  // one event for st3 and the queued st2 work
          ss = c->st3;
        }
        splitfc_bwd(c->z + (long long)t * B * g.Dz, g.Dz, zoff, B, g.D[lvl], c->P + f.ow, c->P + f.obeta, f.nout,
                    s.split_mean[lvl], s.split_inv[lvl], dcat + Fl, (long long)S[lvl + 1] * S[lvl + 1] * 2 * Fl, Fl,
                    2 * Fl, c->Gr + f.ow, c->Gr + f.obeta, c->sfc_part, ss);
        splitfc_dz_reduce(c->sfc_part, splitfc_blocks(f.nout), B, g.D[lvl], dzt, g.Dz, zoff, ss);
      }
      // s2: relu(BN(convT_s2(cur)) + enc_{lvl+1})
      View dres = t >= 1 ? View{c->denc[lvl], Fl, 0} : View{};
      sl = dpre_next(c, rows * Fl);
      r = bn_act_bwd(c, 1, rows, Fl, View{dcat, 2 * Fl, 0}, View{s.cat[lvl], 2 * Fl, 0, c->cbf}, s.s2_pre[lvl], 0, Fl,
                     s.s2_bn[lvl], 0, l2.obeta, 0, ACT_RELU, sl.p, 0, dres, 0, &fu_s2, dpre_bf(c, l2), c->pbf);
      if (r) return r;
      View in = lvl == L - 2 ? View{s.top_act, F[L], 0, c->abf} : View{s.s1_act[lvl + 1], F[lvl + 2], 0, c->abf};
      {
        const ConvL Lw = l2;
        const float* dp = sl.p;
        float* dW = c->Gr + Lw.ow;
        r = on_side_q(c, sl.ready, [=] { return conv_wgrad(c, Lw, 1, 0, in, dp, 0, dW); });
      }
      if (r) return r;
      if (lvl < L - 2) {  // next: s1[lvl+1] (no shortcut)
        fu_s1 = bw_fuse(c, s.s1_pre[lvl + 1], F[lvl + 2], 0, nullptr, 0, 0, s.s1_bn[lvl + 1], 0, G.s1[lvl + 1].obeta, 0,
                        ACT_RELU, F[lvl + 2], c->pbf);
        r = conv_dgrad(c, l2, 1, 0, sl.p, 0, View{dnext, in.ld, 0}, 0, &fu_s1);
      } else {
        r = conv_dgrad(c, l2, 1, 0, sl.p, 0, View{dnext, in.ld, 0}, 0);
      }
      if (r) return r;
      std::swap(dcur, dnext);
      if (t == c->dbg_stop_step && lvl == c->dbg_stop_lvl) return 0;
    }
    // ---- top fc_bn_lrelu (:1704)
    const int ntop = S[L] * S[L] * F[L];
    // own region per pass when the side stream's split-latent backward reads it
    float* dtop = c->side ? arena_next(c, c->dtop_arena, c->dtop_cap, c->dtop_off, (long long)B * s.ktop, true)
                          : c->dtop;
    // E.fc's BN-backward sums (t >= 1: columns [0, nout) of dtop) from the top FC's input gradient
    BwFuse fu_efc;
    if (t >= 1) {
      const FcL& ef = M.enc[t].fc;
      fu_efc = bw_fuse(c, s.encfc_pre, ef.nout, 0, nullptr, 0, 0, s.enc_bn_fc, 0, ef.obeta, 0, ACT_LRELU, ef.nout, 0);
    }
    r = fc_bn_bwd(c, G.top, View{s.top_cat, s.ktop, 0}, View{dcur, ntop, 0}, View{s.top_act, ntop, 0}, s.top_pre,
                  s.top_bn, View{dtop, s.ktop, 0}, nullptr, t >= 1 ? &fu_efc : nullptr);
    if (r) return r;
    {
      const FcL& f = G.split[L - 1];
      const int coff = t >= 1 ? F[L] : 0;
      hipStream_t ss = st;
      if (c->side) {
        if ((r = side_flush(c, c->st3))) return r;
        ss = c->st3;
      }
      splitfc_bwd(c->z + (long long)t * B * g.Dz, g.Dz, g.Dz - g.D[L - 1], B, g.D[L - 1], c->P + f.ow, c->P + f.obeta,
                  f.nout, s.split_mean[L - 1], s.split_inv[L - 1], dtop + coff, s.ktop, f.nout, 0, c->Gr + f.ow,
                  c->Gr + f.obeta, c->sfc_part, ss);
      splitfc_dz_reduce(c->sfc_part, splitfc_blocks(f.nout), B, g.D[L - 1], dzt, g.Dz, g.Dz - g.D[L - 1], ss);
      if (c->side) hipEventRecord(c->ev_dz, c->st3);  // dz_t complete (the top level is the step's last split FC)
    }
    // ---- g_theta encoder of x_{t-1} (reverse of :1764-1775)
    if (t >= 1) {
      const EncStep& E = M.enc[t];
      const int nc = S[L] * S[L] * F[L - 1];
      r = fc_bn_bwd(c, E.fc, View{s.enc_c_act, nc, 0, c->abf}, View{dtop, s.ktop, 0}, View{s.top_cat, s.ktop, 0},
                    s.encfc_pre, s.enc_bn_fc, View{c->denc_c, nc, 0}, fu_efc.used ? &fu_efc : nullptr);
      if (r) return r;
      const long long rc = (long long)B * S[L] * S[L];
      Slot sl = dpre_next(c, rc * F[L - 1]);
      r = bn_act_bwd(c, 1, rc, F[L - 1], View{c->denc_c, F[L - 1], 0}, View{s.enc_c_act, F[L - 1], 0}, s.enc_c_pre, 0,
                     F[L - 1], s.enc_bn_c, 0, E.c.obeta, 0, ACT_LRELU, sl.p, 0, View{}, 0, nullptr,
                     dpre_bf(c, E.c), c->pbf);
      if (r) return r;
      {
        const ConvL Lw = E.c;
        const View in_{s.enc_act_b[L - 2], F[L - 1], 0};
        const float* dp = sl.p;
        float* dW = c->Gr + Lw.ow;
        r = on_side_q(c, sl.ready, [=] { return conv_wgrad(c, Lw, 1, 0, in_, dp, 0, dW); });
      }
      if (r) return r;
      // E.c's input gradient accumulates last into denc[L-2] (after the decoder shortcut term)
      BwFuse fu_eb = bw_fuse(c, s.enc_pre_b[L - 2], F[L - 1], 0, nullptr, 0, 0, s.enc_bn_b[L - 2], 0, E.b[L - 2].obeta,
                             0, ACT_LRELU, F[L - 1], c->pbf);
      r = conv_dgrad(c, E.c, 1, 0, sl.p, 0, View{c->denc[L - 2], F[L - 1], 0}, 1, &fu_eb);
      if (r) return r;
      for (int lvl = L - 2; lvl >= 0; --lvl) {
        const int Fl = F[lvl + 1];
        const long long rows = (long long)B * S[lvl + 1] * S[lvl + 1];
        Slot sb = dpre_next(c, rows * Fl);
        r = bn_act_bwd(c, 1, rows, Fl, View{c->denc[lvl], Fl, 0}, View{s.enc_act_b[lvl], Fl, 0}, s.enc_pre_b[lvl], 0,
                       Fl, s.enc_bn_b[lvl], 0, E.b[lvl].obeta, 0, ACT_LRELU, sb.p, 0, View{}, 0, &fu_eb,
                       dpre_bf(c, E.b[lvl]), c->pbf);
        if (r) return r;
        {
          const ConvL Lw = E.b[lvl];
          const View in_{s.enc_act_a[lvl], Fl, 0, c->abf};
          const float* dp = sb.p;
          float* dW = c->Gr + Lw.ow;
          r = on_side_q(c, sb.ready, [=] { return conv_wgrad(c, Lw, 1, 0, in_, dp, 0, dW); });
        }
        if (r) return r;
        BwFuse fu_ea = bw_fuse(c, s.enc_pre_a[lvl], Fl, 0, nullptr, 0, 0, s.enc_bn_a[lvl], 0, E.a[lvl].obeta, 0,
                               ACT_LRELU, Fl, c->pbf);
        r = conv_dgrad(c, E.b[lvl], 1, 0, sb.p, 0, View{c->dcur, Fl, 0}, 0, &fu_ea);
        if (r) return r;
        Slot sa = dpre_next(c, rows * Fl);
        r = bn_act_bwd(c, 1, rows, Fl, View{c->dcur, Fl, 0}, View{s.enc_act_a[lvl], Fl, 0}, s.enc_pre_a[lvl], 0, Fl,
                       s.enc_bn_a[lvl], 0, E.a[lvl].obeta, 0, ACT_LRELU, sa.p, 0, View{}, 0, &fu_ea,
                       dpre_bf(c, E.a[lvl]), c->pbf);
        if (r) return r;
        View in = lvl == 0 ? View{(float*)xprev, g.C, 0} : View{s.enc_act_b[lvl - 1], F[lvl], 0};
        {
          const ConvL Lw = E.a[lvl];
          const float* dp = sa.p;
          float* dW = c->Gr + Lw.ow;
          r = on_side_q(c, sa.ready, [=] { return conv_wgrad(c, Lw, 1, 0, in, dp, 0, dW); });
        }
        if (r) return r;
        View din = lvl == 0 ? View{dxout, g.C, 0} : View{c->denc[lvl - 1], F[lvl], 0};
        if (lvl > 0) {  // accumulates last into denc[lvl-1]: E.b[lvl-1]'s BN partials
          fu_eb = bw_fuse(c, s.enc_pre_b[lvl - 1], F[lvl], 0, nullptr, 0, 0, s.enc_bn_b[lvl - 1], 0, E.b[lvl - 1].obeta,
                          0, ACT_LRELU, F[lvl], c->pbf);
          r = conv_dgrad(c, E.a[lvl], 1, 0, sa.p, 0, din, 1, &fu_eb);
        } else {
          r = conv_dgrad(c, E.a[lvl], 1, 0, sa.p, 0, din, 1);
        }
        if (r) return r;
      }
    }
    // recognition backward of steps [t, t + rec_group) on st4, overlapping the chain backward of the
    // earlier steps: q(z_t | x) needs only dz_t (inference_bwd waits on ev_dz), its weight gradients
    // go to the side stream like every other; own split slab
    if (rec_ov && t % c->rec_group == 0) {
      if ((r = side_flush(c))) return r;
      hipStream_t s0 = c->st;
      float* sl0 = c->slab;
      c->st = c->st4;
      c->slab = c->slab4;
      r = inference_bwd(c, t, std::min(c->rec_group, T - t), View{(float*)c->x_in, g.C, 0}, nullptr);
      // the group's queued weight-gradient closures read st4's dpre: flush them behind an event
      // recorded on st4 (side_flush records on c->st), before the main stream is restored
      const int rf = side_flush(c);
      if (!r) r = rf;
      c->st = s0;
      c->slab = sl0;
      if (r) return r;
    }
  }

  if ((r = step_hook(c, 0))) return r;

  // ---------------- recognition ladders: all steps batched, or step 0 (Latent InfoMax) ----------------
  if (rec_ov) {  // joined: every recognition group was enqueued on st4 during the chain backward
    hipEventRecord(c->ev_j4, c->st4);
    hipStreamWaitEvent(st, c->ev_j4, 0);
  } else if ((r = inference_bwd(c, 0, g.plc ? 1 : T, View{(float*)c->x_in, g.C, 0}, nullptr))) {
    return r;
  }
  if ((r = side_flush(c))) return r;
  if (M.shared) {  // public gradient = fixed-order sum of the step copies (side stream joined first)
    if (c->side) {
      side_merge(c);
    hipEventRecord(c->ev_join, c->st2);
      hipStreamWaitEvent(st, c->ev_join, 0);
      hipEventRecord(c->ev_j3, c->st3);
      hipStreamWaitEvent(st, c->ev_j3, 0);
    }
    share_gather(c->Gv, c->Gpub, c->share_tab, c->share_cp, c->share_ntab, st);
  }
  return 0;
}

// ============================================================================
// arena planning (counting pass, then carving pass)
// ============================================================================
static bool plan(svae_ctx* c) {
  const Geo& g = c->m.g;
  const int B = g.B, L = g.L, T = g.T;
  const int* F = g.F;
  const int* S = g.S;
  const int C1 = g.C + 1;
  auto A = [&](long long n) { return c->alloc(n); };
  auto bn = [&](int groups, int C) {
    BNS b;
    b.mean = A((long long)groups * C);
    b.invstd = A((long long)groups * C);
    return b;
  };
  long long max_inf = 0, maxact = 0, maxJ = 0;
  int maxK = 0;
  for (int lvl = 0; lvl < L - 1; ++lvl) {
    long long gs = (long long)B * S[lvl + 1] * S[lvl + 1] * F[lvl + 1];
    gs = (gs + 63) / 64 * 64;
    c->inf_gs[lvl] = gs;
    max_inf = std::max(max_inf, gs);
    c->inf_pre_a[lvl] = A(T * gs);
    c->inf_act_a[lvl] = A(T * gs);
    c->inf_pre_b[lvl] = A(T * gs);
    c->inf_act_b[lvl] = A(T * gs);
    c->inf_bn_a[lvl] = bn(T, F[lvl + 1]);
    c->inf_bn_b[lvl] = bn(T, F[lvl + 1]);
    maxact = std::max(maxact, 2 * gs);
  }
  int maxnin = 0;
  for (int l = 0; l < L; ++l) maxnin = std::max(maxnin, c->m.inf[0].head[l].nin);
  c->head_nsplit = heads_splits(maxnin);  // latent_fwd_kernel sums the head partials 32 splits at a time
  c->head_part = A((long long)T * c->head_nsplit * B * 2 * g.Dz);
  c->mu = A((long long)T * B * g.Dz);
  c->sig = A((long long)T * B * g.Dz);
  c->z = A((long long)T * B * g.Dz);
  c->eps_buf = A((long long)T * B * g.Dz);
  c->kl_img = A((long long)T * B);
  c->kl_coef = A(64);
  c->out_nblk = output_blocks_per_img(g.H * g.W);
  c->sb.assign(T, svae_ctx::StepBufs());
  for (int t = 0; t < T; ++t) {
    svae_ctx::StepBufs& s = c->sb[t];
    memset(&s, 0, sizeof(s));
    if (t >= 1) {
      for (int lvl = 0; lvl < L - 1; ++lvl) {
        long long n = (long long)B * S[lvl + 1] * S[lvl + 1] * F[lvl + 1];
        s.enc_pre_a[lvl] = A(n); s.enc_act_a[lvl] = A(n); s.enc_pre_b[lvl] = A(n); s.enc_act_b[lvl] = A(n);
        s.enc_bn_a[lvl] = bn(1, F[lvl + 1]); s.enc_bn_b[lvl] = bn(1, F[lvl + 1]);
      }
      long long nc = (long long)B * S[L] * S[L] * F[L - 1];
      s.enc_c_pre = A(nc); s.enc_c_act = A(nc); s.enc_bn_c = bn(1, F[L - 1]);
      s.encfc_pre = A((long long)B * F[L]); s.enc_bn_fc = bn(1, F[L]);
    }
    for (int i = 0; i < L; ++i) {
      int J = c->m.gen[t].split[i].nout;
      maxJ = std::max<long long>(maxJ, J);
      maxK = std::max(maxK, g.D[i]);
      s.split_mean[i] = A(J);
      s.split_inv[i] = A(J);
    }
    s.ktop = F[L + 1] + (t >= 1 ? F[L] : 0);
    s.top_cat = A((long long)B * s.ktop);
    long long ntop = (long long)B * S[L] * S[L] * F[L];
    s.top_pre = A(ntop); s.top_act = A(ntop); s.top_bn = bn(1, S[L] * S[L] * F[L]);
    maxact = std::max(maxact, ntop);
    for (int lvl = 0; lvl < L - 1; ++lvl) {
      long long n = (long long)B * S[lvl + 1] * S[lvl + 1] * F[lvl + 1];
      s.s2_pre[lvl] = A(n); s.cat[lvl] = A(2 * n); s.s1_pre[lvl] = A(n); s.s1_act[lvl] = A(n);
      s.s2_bn[lvl] = bn(1, F[lvl + 1]); s.s1_bn[lvl] = bn(1, F[lvl + 1]);
      maxact = std::max(maxact, 2 * n);
    }
    s.wpack = A(16LL * C1 * F[1] + 4);
    s.wpack_h = A((g.split ? 24LL : 8LL) * C1 * F[1] + 4);  // bf16 [tap][C+1][F1] (split mode: 3 planes)
    s.a_out = A((long long)B * g.H * g.W * C1);
    s.xhat = A((long long)B * g.H * g.W * g.C);
    s.rec_part = A((long long)B * c->out_nblk);
    s.rec_img = A(B);
    s.stats = A(2);
    const long long npx = (long long)B * g.H * g.W;
    // training_samples[t] differs from the MLE under predicted noise, or a fixed stddev != 0
    s.has_sample = g.pgn || (g.noisy && g.nstd[t] != 0.f);
    if (s.has_sample) s.sample = A(npx * g.C);
    if (g.pgn) {
      s.sd = A(npx);
      for (int l = 0; l < g.sd_nl; ++l) {
        const int Co = g.sd_F[l + 1];
        s.sd_pre[l] = A(npx * Co);
        s.sd_act[l] = A(npx * Co);
        s.sd_mean[l] = A(Co);
        s.sd_inv[l] = A(Co);
      }
    }
  }
  {
    const long long npx = (long long)B * g.H * g.W;
    if (g.noisy) c->noise_buf = A((long long)T * npx * g.C);
    if (g.pgn) {
      for (int i = 0; i < 2; ++i) c->sd_d[i] = A(npx * 8);
      c->sd_dpre = A(npx * 8);
      c->sd_part = (double*)A(2LL * sd_pixel_blocks(npx) * 2 * 8);
      c->sd_wpart = A(std::max<long long>((long long)sd_wgrad_blocks(B, g.H) * 16 * 64, 9LL * sd_pixel_blocks(npx)));
      c->sd_sums = A(16);
      c->dmle = A(npx * g.C);
    }
    if (g.imp) {
      c->dseed = A(npx * g.C);
      c->imp_img = A((long long)T * B);
    }
    c->kl_zero = A(64);
  }
  const long long P0 = (long long)B * g.H * g.W;
  c->dx[0] = A(P0 * g.C);
  c->dx[1] = A(P0 * g.C);
  c->da_base = A((long long)T * P0 * C1);
  c->da = c->da_base;
  c->dcur = A(maxact);
  c->dnext = A(maxact);
  c->dpre = A(maxact);
  {  // one region per BN-backward output of a pass (dpre_next / idpre_next sizes, 64-element aligned)
    const Model& M = c->m;
    auto cl = [&](const ConvL& l) { return ((long long)B * l.hout * l.hout * l.cout + 63) / 64 * 64; };
    auto fl = [&](const FcL& f) { return ((long long)B * f.nout + 63) / 64 * 64; };
    long long n = 0;
    for (int t = 0; t < T; ++t) {
      const GenStep& G = M.gen[t];
      for (int lvl = 0; lvl < L - 1; ++lvl) n += cl(G.s1[lvl]) + cl(G.s2[lvl]);
      n += fl(G.top);
      if (t >= 1) {
        const EncStep& E = M.enc[t];
        n += fl(E.fc) + cl(E.c);
        for (int lvl = 0; lvl < L - 1; ++lvl) n += cl(E.a[lvl]) + cl(E.b[lvl]);
      }
    }
    c->dpre_cap = n;
    c->dpre_arena = A(n);
    long long ni = 0;
    for (int lvl = 0; lvl < L - 1; ++lvl) ni += 2 * (((long long)T * c->inf_gs[lvl] + 63) / 64 * 64 + 64 * T);
    c->idpre_cap = ni;
    c->idpre_arena = A(ni);
  }
  c->dcat = A(maxact);
  c->dtop = A((long long)B * (F[L] + F[L + 1]));
  {  // per-pass regions of dcat (every decoder level of every step) and dtop (every step)
    long long n = 0;
    for (int lvl = 0; lvl < L - 1; ++lvl) n += ((long long)B * S[lvl + 1] * S[lvl + 1] * 2 * F[lvl + 1] + 63) / 64 * 64;
    c->dcat_cap = T * n;
    c->dcat_arena = A(c->dcat_cap);
    c->dtop_cap = T * (((long long)B * (F[L] + F[L + 1]) + 63) / 64 * 64);
    c->dtop_arena = A(c->dtop_cap);
  }
  c->denc_c = A((long long)B * S[L] * S[L] * F[L - 1]);
  for (int lvl = 0; lvl < L - 1; ++lvl) c->denc[lvl] = A((long long)B * S[lvl + 1] * S[lvl + 1] * F[lvl + 1]);
  c->sfc_part = A((long long)splitfc_blocks((int)maxJ) * B * maxK);
  c->dz = A((long long)T * B * g.Dz);
  c->dhead = A((long long)T * B * 2 * g.Dz);
  c->idb = A((long long)T * max_inf);
  c->ida = A((long long)T * max_inf);
  c->idpre = A((long long)T * max_inf);

  c->bnacc_cap = 8LL << 20;  // words (64 MB); a CelebA pass takes a few M
  c->bnacc = (u64*)A(2 * c->bnacc_cap);
  c->slab_cap = 64LL << 20;
  c->slab = A(c->slab_cap);
  c->slab2 = A(c->slab_cap);
  if (c->side2) c->slab2b = A(c->slab_cap);
  if (c->rec_group > 0 || c->rec_split) c->slab4 = A(c->slab_cap);
  c->cs_part = A(64 * 1024);
  c->zero_img = A((long long)B * g.H * g.W * g.C);
  return true;
}

// ============================================================================
// C ABI
// ============================================================================
extern "C" {

#ifndef SVAE_SRC_HASH
#define SVAE_SRC_HASH "unknown"
#endif
// build.py's hash of the sources this library was compiled from (the literal stays in the binary)
static const char kSrcHash[] = "SVAE_SRC_HASH=" SVAE_SRC_HASH;
const char* svae_build_hash(void) { return kSrcHash + 14; }

int svae_param_count(const svae_config* cfg, int64_t* n_total, int64_t* n_live, int32_t* n_tensors) {
  Model m;
  std::string err;
  if (!make_geo(cfg, m.g, err)) return fail(nullptr, SVAE_EBADCONFIG, err);
  m.build();
  if (n_total) *n_total = m.p_total;
  if (n_live) *n_live = m.p_live;
  if (n_tensors) *n_tensors = (int32_t)m.pub.size();
  return 0;
}

int svae_param_layout(const svae_config* cfg, svae_param_desc* out, int32_t cap) {
  Model m;
  std::string err;
  if (!make_geo(cfg, m.g, err)) return fail(nullptr, SVAE_EBADCONFIG, err);
  m.build();
  if (!out || cap < (int32_t)m.pub.size()) return fail(nullptr, SVAE_EBADARG, "layout capacity too small");
  for (size_t i = 0; i < m.pub.size(); ++i) {
    const PDesc& d = m.pub[i];
    svae_param_desc& o = out[i];
    memset(&o, 0, sizeof(o));
    strncpy(o.name, d.name.c_str(), sizeof(o.name) - 1);
    o.ndim = (int32_t)d.shape.size();
    for (size_t k = 0; k < d.shape.size() && k < 4; ++k) o.shape[k] = d.shape[k];
    o.offset = d.offset;
    o.init = d.init;
    o.flags = (d.dead ? 1 : 0) | (d.zero_grad ? 2 : 0);
  }
  return 0;
}

int svae_create(const svae_config* cfg, int device, svae_ctx** out) {
  if (!out) return fail(nullptr, SVAE_EBADARG, "null out");
  *out = nullptr;
  svae_ctx* c = new svae_ctx();
  std::string err;
  if (!make_geo(cfg, c->m.g, err)) {
    delete c;
    return fail(nullptr, SVAE_EBADCONFIG, err);
  }
  c->m.build();
  c->device = device;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) {
    delete c;
    return fail(nullptr, SVAE_EHIP, std::string("hipSetDevice: ") + hipGetErrorString(e));
  }
  {
    // measured-slower alternatives, reachable only in a -DSVAE_KNOBS build, read per context
    c->fold = svae_knob("SVAE_FOLD", 0) == 1;          // forward BN applies of gather-only tensors on st2
    c->side2 = svae_knob("SVAE_SIDE2", 0) == 1;        // a second weight-gradient stream
    c->rec_group = svae_knob("SVAE_REC_GROUP", 0);     // recognition-backward group size (0 = batched after the chain)
    if (c->rec_group < 0 || c->m.g.plc) c->rec_group = 0;
    c->rec_split = (svae_knob("SVAE_REC_SPLIT", 0) == 1 && !c->m.g.plc && c->m.g.T > 1) ? 1 : 0;  // forward recognition of steps >= 1 on st4
  }
  {
    // operand storage in bf16 mode; the fp32 alternatives are bitwise A/B checks (knob builds)
    c->dbf = (c->m.g.bf16 && !c->m.g.split && svae_knob("SVAE_DPRE_F32", 0) != 1) ? 1 : 0;  // BN-backward outputs
    c->abf = (c->m.g.bf16 && !c->m.g.split && svae_knob("SVAE_ACT_F32", 0) != 1) ? 1 : 0;   // GEMM-only activations
    c->cbf = (c->abf && svae_knob("SVAE_CAT_F32", 0) != 1) ? 1 : 0;                        // decoder concat buffers
    c->laf = svae_knob("SVAE_BN_LAF", 0);  // last-arriver BN finalisation (experimental: off)
    c->bnfin = svae_knob("SVAE_BN_FIN", 0);
    c->pbf = (c->m.g.bf16 && !c->m.g.split && svae_knob("SVAE_PRE_F32", 0) != 1) ? 1 : 0;   // conv pre-BN outputs
  }
  c->counting = true;
  c->arena_used = 0;
  plan(c);
  if (c->m.g.Dz > 256) {  // latent_fwd_kernel: whole images per 256-thread block (unreachable: make_geo caps Dz)
    delete c;
    return fail(nullptr, SVAE_EBADCONFIG, "latent over 256 dimensions");
  }
  c->arena_bytes = c->arena_used;
  c->counting = false;
  c->arena_used = 0;
  e = hipMalloc((void**)&c->arena, c->arena_bytes);
  if (e != hipSuccess) {
    delete c;
    return fail(nullptr, SVAE_ENOMEM, std::string("hipMalloc arena: ") + hipGetErrorString(e));
  }
  plan(c);
  const long long nl = c->m.n_live;
  e = hipMalloc((void**)&c->adam_m, (size_t)nl * sizeof(float) * 2);
  if (e != hipSuccess) {
    hipFree(c->arena);
    delete c;
    return fail(nullptr, SVAE_ENOMEM, std::string("hipMalloc adam: ") + hipGetErrorString(e));
  }
  c->adam_v = c->adam_m + nl;
  hipMemset(c->adam_m, 0, (size_t)nl * sizeof(float) * 2);
  if (c->m.shared) {
    const Model& M = c->m;
    std::vector<long long> seg, tab, cp;
    std::vector<std::vector<long long>> copies(M.pub.size());
    std::vector<int> order(M.descs.size());
    for (size_t i = 0; i < M.descs.size(); ++i) order[i] = (int)i;
    std::sort(order.begin(), order.end(), [&](int a, int b) { return M.descs[a].offset < M.descs[b].offset; });
    for (int i : order) {  // step order within a public tensor = virtual layout order (fixed)
      const PDesc& d = M.descs[i];
      const PDesc& p = M.pub[M.vpub[i]];
      seg.insert(seg.end(), {d.offset, p.offset, d.size});
      if (!d.zero_grad) copies[M.vpub[i]].push_back(d.offset);
    }
    for (size_t j = 0; j < M.pub.size(); ++j) {
      if (copies[j].empty()) continue;
      tab.insert(tab.end(), {M.pub[j].offset, M.pub[j].size, (long long)cp.size(), (long long)copies[j].size()});
      cp.insert(cp.end(), copies[j].begin(), copies[j].end());
    }
    c->share_nseg = (int)(seg.size() / 3);
    c->share_ntab = (int)(tab.size() / 4);
    size_t bytes = (seg.size() + tab.size() + cp.size()) * sizeof(long long);
    e = hipMalloc((void**)&c->Pv, (size_t)M.n_total * sizeof(float) * 2);
    if (e == hipSuccess) e = hipMalloc((void**)&c->share_seg, bytes);
    if (e != hipSuccess) {
      svae_destroy(c);
      return fail(nullptr, SVAE_ENOMEM, std::string("hipMalloc shared copies: ") + hipGetErrorString(e));
    }
    c->Gv = c->Pv + M.n_total;
    c->share_tab = c->share_seg + seg.size();
    c->share_cp = c->share_tab + tab.size();
    hipMemset(c->Pv, 0, (size_t)M.n_total * sizeof(float) * 2);
    hipMemcpy(c->share_seg, seg.data(), seg.size() * sizeof(long long), hipMemcpyHostToDevice);
    hipMemcpy(c->share_tab, tab.data(), tab.size() * sizeof(long long), hipMemcpyHostToDevice);
    hipMemcpy(c->share_cp, cp.data(), cp.size() * sizeof(long long), hipMemcpyHostToDevice);
  }
  if (c->m.g.bf16) {
    // bf16 shadows of the live region + the per-tap transpose tile table of every GEMM weight
    // split mode: three planes (hi / mid / lo, opload.h split8) of wplane elements each
    c->nsp = c->m.g.split ? 3 : 1;
    c->wplane = ((long long)nl + 127) / 128 * 128;
    // (split mode: + the two scaled fp16 planes H16_PLANE, H16_PLANE + 1 that the wave-split gathers read)
    const size_t sbytes = (size_t)(c->nsp == 3 ? H16_PLANE + 2 : c->nsp) * c->wplane * 2;
    e = hipMalloc(&c->wN, sbytes);
    if (e == hipSuccess) e = hipMalloc(&c->wT, sbytes);
    if (e != hipSuccess) {
      svae_destroy(c);
      return fail(nullptr, SVAE_ENOMEM, std::string("hipMalloc shadows: ") + hipGetErrorString(e));
    }
    hipMemset(c->wT, 0, sbytes);
    std::vector<long long> offs;
    std::vector<int> tiles;
    struct TT { long long off; int taps, R, Cc; };
    std::vector<TT> tt;
    auto add = [&](long long off, int taps, int R, int Cc) { tt.push_back(TT{off, taps, R, Cc}); };
    auto conv = [&](const ConvL& L) {
      if (L.w < 0) return;
      if (L.tr) add(L.ow, 16, L.cout, L.cin);   // [tap][co][ci]
      else add(L.ow, 16, L.cin, L.cout);        // [tap][ci][co]
    };
    const Geo& g = c->m.g;
    for (int t = 0; t < g.T; ++t) {
      for (int l = 0; l < g.L - 1; ++l) {
        conv(c->m.inf[t].a[l]); conv(c->m.inf[t].b[l]);
        if (t >= g.Te) continue;
        conv(c->m.gen[t].s2[l]); conv(c->m.gen[t].s1[l]);
        if (t >= 1) { conv(c->m.enc[t].a[l]); conv(c->m.enc[t].b[l]); }
      }
      if (t >= g.Te) continue;
      if (t >= 1) { conv(c->m.enc[t].c); add(c->m.enc[t].fc.ow, 1, c->m.enc[t].fc.nin, c->m.enc[t].fc.nout); }
      add(c->m.gen[t].top.ow, 1, c->m.gen[t].top.nin, c->m.gen[t].top.nout);
    }
    // tiles in tensor-offset order, so the tiles of a parameter range are contiguous (adam_range)
    std::sort(tt.begin(), tt.end(), [](const TT& a, const TT& b) { return a.off < b.off; });
    for (const TT& x : tt) {
      int id = (int)(offs.size() / 3);
      offs.push_back(x.off); offs.push_back(x.R); offs.push_back(x.Cc);
      for (int t = 0; t < x.taps; ++t)
        for (int r = 0; r < x.R; r += 32)
          for (int q = 0; q < x.Cc; q += 32) {
            tiles.push_back(id); tiles.push_back(t); tiles.push_back(r); tiles.push_back(q);
            c->tile_off.push_back(x.off);
          }
    }
    c->ntiles = (int)(tiles.size() / 4);
    e = hipMalloc(&c->tiles_d, tiles.size() * sizeof(int));
    if (e == hipSuccess) e = hipMalloc(&c->offs_d, offs.size() * sizeof(long long));
    if (e != hipSuccess) {
      svae_destroy(c);
      return fail(nullptr, SVAE_ENOMEM, std::string("hipMalloc tiles: ") + hipGetErrorString(e));
    }
    hipMemcpy(c->tiles_d, tiles.data(), tiles.size() * sizeof(int), hipMemcpyHostToDevice);
    hipMemcpy(c->offs_d, offs.data(), offs.size() * sizeof(long long), hipMemcpyHostToDevice);
    if (c->m.g.split) {  // the fp16 weight planes' exponent table (H16_WS until the first shadow refresh)
      std::vector<long long> info;
      for (const TT& x : tt) {
        info.push_back(x.off); info.push_back((long long)x.taps * x.R * x.Cc); info.push_back(x.R); info.push_back(x.Cc);
      }
      c->nwinfo = (int)tt.size();
      const long long nb = c->wplane / 64 + 1;
      e = hipMalloc(&c->wtab, nb * sizeof(int));
      if (e == hipSuccess) e = hipMalloc(&c->winfo_d, std::max<size_t>(1, info.size()) * sizeof(long long));
      if (e == hipSuccess) e = hipMalloc(&c->wovf, sizeof(int));
      if (e != hipSuccess) {
        svae_destroy(c);
        return fail(nullptr, SVAE_ENOMEM, std::string("hipMalloc exponent table: ") + hipGetErrorString(e));
      }
      // exponent H16_WS until the first shadow refresh; the bf16-planes flag on the tensors a small-N conv-T
      // may read (a side under 32 channels: the image-channel convs, whose input gradients run on
      // convt_smalln's 3 bf16 planes); every other split-mode GEMM reads the fp16 pair only (halo_x3,
      // halo_kw and dense_kw take the shadows with FwdArgs::h16 set)
      std::vector<int> w0((size_t)nb, H16_WS & 0xffff);
      for (const TT& x : tt)
        if (x.taps == 16 && (x.R < 32 || x.Cc < 32))
          for (long long b = x.off >> 6; b < (x.off + (long long)x.taps * x.R * x.Cc + 63) >> 6; ++b) w0[b] |= WTAB_BF16;
      hipMemcpy(c->wtab, w0.data(), nb * sizeof(int), hipMemcpyHostToDevice);
      if (!info.empty()) hipMemcpy(c->winfo_d, info.data(), info.size() * sizeof(long long), hipMemcpyHostToDevice);
      hipMemset(c->wovf, 0, sizeof(int));
    }
  }
  hipHostMalloc((void**)&c->reg_host, 64 * sizeof(float), hipHostMallocDefault);
  {
    if (svae_knob("SVAE_NO_SIDE", 0) != 1) {
      // SVAE_SIDE_CUMASK=k (A/B): the weight-gradient stream runs on all CUs but every k-th, so the
      // main stream's latency-bound kernels always find free CUs.  A CU-masked stream is a blocking
      // stream (it synchronises with the NULL stream), so this is only meaningful when the caller's
      // stream is not the NULL stream (bench.py SVAE_BENCH_STREAM=1)
      const int cmk = svae_knob("SVAE_SIDE_CUMASK", 0);
      bool ok;
      if (cmk >= 2) {
        int ncu = 0;
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device);
        std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
        for (int i = 0; i < ncu; ++i)
          if (i % cmk != cmk - 1) mask[i / 32] |= 1u << (i % 32);
        ok = hipExtStreamCreateWithCUMask(&c->st2, (uint32_t)mask.size(), mask.data()) == hipSuccess;
      } else {
        ok = hipStreamCreateWithFlags(&c->st2, hipStreamNonBlocking) == hipSuccess;
      }
      ok = ok && hipStreamCreateWithFlags(&c->st3, hipStreamNonBlocking) == hipSuccess;
      if (c->side2) ok = ok && hipStreamCreateWithFlags(&c->st2b, hipStreamNonBlocking) == hipSuccess;
      if (c->rec_group > 0 || c->rec_split)
        ok = ok && hipStreamCreateWithFlags(&c->st4, hipStreamNonBlocking) == hipSuccess;
      // cross-stream ordering on this device only: no system-scope fence (a system-scope release
      // writes the L2s back for host / peer visibility, a GPU-side bubble at every record); the
      // gradient-hook event, which orders a collective's peer traffic, keeps it
      // (SVAE_EV_SYSFENCE=1: every event with the system fence)
      static const bool sysf = svae_knob("SVAE_EV_SYSFENCE", 0) == 1;
      const unsigned evf = hipEventDisableTiming | (sysf ? 0u : (unsigned)hipEventDisableSystemFence);
      auto mk = [&](hipEvent_t* ev) { ok = ok && hipEventCreateWithFlags(ev, evf) == hipSuccess; };
      for (int i = 0; i < svae_ctx::NR; ++i) { mk(&c->ev_ready[i]); mk(&c->ev_iready[i]); }
      mk(&c->ev_drain);
      mk(&c->ev_da_ready); mk(&c->ev_da_free); mk(&c->ev_start); mk(&c->ev_join);
      ok = ok && hipEventCreateWithFlags(&c->ev_hook, hipEventDisableTiming) == hipSuccess;
      mk(&c->ev_hook_dev);
      mk(&c->ev_aux); mk(&c->ev_aux2); mk(&c->ev_dz); mk(&c->ev_j3); mk(&c->ev_j4);
      mk(&c->ev_drain3);
      for (int i = 0; i < 64; ++i) mk(&c->ev_sfc[i]);
      for (int i = 0; i < svae_ctx::NF; ++i) mk(&c->ev_flush[i]);
      mk(&c->ev_rs);
      mk(&c->ev_rs2);
      if (c->side2) mk(&c->ev_merge);
      for (int i = 0; i < svae_ctx::NFOLD; ++i) mk(&c->ev_fold[i]);
      mk(&c->ev_fold_join);
      {  // SVAE_SIDE_BATCH (read per context): weight-gradient layers per side-stream hand-over
        c->side_batch = std::max(1, svae_knob("SVAE_SIDE_BATCH", 1));
      }
      c->side = ok;
    }
  }
  {
    c->fc_fuse = svae_knob("SVAE_BWFUSE_FC", 1) != 0;  // read per context (A/B and the bitwise test)
  }
  for (int i = 0; i < 64; ++i) c->reg_host[i] = 0.f;
  *out = c;
  return 0;
}

int svae_destroy(svae_ctx* c) {
  if (!c) return 0;
  for (hipStream_t sx : {c->st2b, c->st2, c->st3, c->st4})
    if (sx) {
      hipStreamSynchronize(sx);
      hipStreamDestroy(sx);
    }
  for (hipEvent_t ev : {c->ev_da_ready, c->ev_da_free, c->ev_start, c->ev_join, c->ev_hook, c->ev_hook_dev, c->ev_aux, c->ev_aux2, c->ev_dz, c->ev_j3, c->ev_j4,
                        c->ev_drain3})
    if (ev) hipEventDestroy(ev);
  for (hipEvent_t ev : c->ev_sfc)
    if (ev) hipEventDestroy(ev);
  for (hipEvent_t ev : c->ev_flush)
    if (ev) hipEventDestroy(ev);
  for (hipEvent_t ev : {c->ev_rs, c->ev_rs2, c->ev_merge, c->ev_fold_join})
    if (ev) hipEventDestroy(ev);
  for (hipEvent_t ev : c->ev_fold)
    if (ev) hipEventDestroy(ev);
  for (int i = 0; i < svae_ctx::NR; ++i) {
    if (c->ev_ready[i]) hipEventDestroy(c->ev_ready[i]);
    if (c->ev_iready[i]) hipEventDestroy(c->ev_iready[i]);
  }
  if (c->ev_drain) hipEventDestroy(c->ev_drain);
  for (hipEvent_t ev : c->probe.ev) hipEventDestroy(ev);
  if (c->arena) hipFree(c->arena);
  if (c->adam_m) hipFree(c->adam_m);
  if (c->reg_host) hipHostFree(c->reg_host);
  if (c->wN) hipFree(c->wN);
  if (c->wT) hipFree(c->wT);
  if (c->tiles_d) hipFree(c->tiles_d);
  if (c->offs_d) hipFree(c->offs_d);
  if (c->wtab) hipFree(c->wtab);
  if (c->winfo_d) hipFree(c->winfo_d);
  if (c->wovf) hipFree(c->wovf);
  if (c->Pv) hipFree(c->Pv);
  if (c->Gimp_v) hipFree(c->Gimp_v);
  if (c->share_seg) hipFree(c->share_seg);
  delete c;
  return 0;
}

int svae_probe_begin(svae_ctx* c, int kid, int max_launches) {
  if (!c || kid < 0 || kid >= KID_COUNT || max_launches < 0) return fail(c, SVAE_EBADARG, "bad probe request");
  Probe& p = c->probe;
  const size_t need = 2 * (size_t)max_launches + 2;
  while (p.ev.size() < need) {
    hipEvent_t ev;
    hipError_t er = hipEventCreate(&ev);
    if (er != hipSuccess) return fail(c, SVAE_EHIP, std::string("hipEventCreate: ") + hipGetErrorString(er));
    p.ev.push_back(ev);
  }
  p.kid = kid;
  p.used = 0;
  p.launches = 0;
  p.flops = 0;
  return 0;
}

int svae_probe_end(svae_ctx* c, int64_t* launches, int64_t* timed, double* flops, double* total_ms) {
  if (!c) return fail(c, SVAE_EBADARG, "null ctx");
  Probe& p = c->probe;
  double ms = 0;
  for (int i = 0; i < p.used; ++i) {
    hipError_t er = hipEventSynchronize(p.ev[2 * i + 1]);
    float t = 0.f;
    if (er == hipSuccess) er = hipEventElapsedTime(&t, p.ev[2 * i], p.ev[2 * i + 1]);
    if (er != hipSuccess) return fail(c, SVAE_EHIP, std::string("probe events: ") + hipGetErrorString(er));
    ms += t;
  }
  if (launches) *launches = p.launches;
  if (timed) *timed = p.used;
  if (flops) *flops = p.flops;
  if (total_ms) *total_ms = ms;
  p.kid = KID_NONE;
  return 0;
}

const char* svae_kernel_name(int kid) { return kernel_name(kid); }

const char* svae_last_error(const svae_ctx* c) { return c ? c->err.c_str() : g_tls_err.c_str(); }

int64_t svae_workspace_bytes(const svae_ctx* c) { return c ? (int64_t)c->arena_bytes : 0; }

int svae_bind(svae_ctx* c, float* params, float* grads) {
  if (!c || !params || !grads) return fail(c, SVAE_EBADARG, "null buffer");
  c->Ppub = params;
  c->Gpub = grads;
  c->fresh = 0;  // caller-written parameters: the next forward rebuilds the bf16 shadows
  HIPCHK(c, hipMemset(grads, 0, (size_t)c->m.p_total * sizeof(float)));
  if (c->m.shared) {
    c->P = c->Pv;
    c->Gr = c->Gv;
    HIPCHK(c, hipMemset(c->Gv, 0, (size_t)c->m.n_total * sizeof(float)));
  } else {
    c->P = params;
    c->Gr = grads;
  }
  return 0;
}

int svae_forward(svae_ctx* c, const float* x, const float* target, const float* eps, float reg_coeff, void* stream) {
  if (!c || !x || !target) return fail(c, SVAE_EBADARG, "null input");
  if (!c->P) return fail(c, SVAE_EBADARG, "parameters not bound (svae_bind)");
  c->st = (hipStream_t)stream;
  c->x_in = x;
  c->tgt_in = target;
  c->eps_in = eps;
  c->reg = reg_coeff;
  const Geo& g = c->m.g;
  // per-step KL coefficients, passed by value to a one-block kernel: captured at enqueue time,
  // so a host running steps ahead of the GPU cannot change an earlier step's values
  for (int t = 0; t < g.T; ++t) c->reg_host[t] = reg_coeff * (t == 0 ? g.c_first : 1.f) * g.kl_on(t) / (float)g.B;
  set_small(c->kl_coef, c->reg_host, g.T, c->st);
  int r = engine_forward(c);
  c->noise_in = nullptr;  // one-shot (svae_set_chain_noise); the backward reads noise_used
  if (r) return r;
  HIPCHK(c, hipGetLastError());
  return 0;
}

int svae_generate(svae_ctx* c, const float* z, void* stream) {
  if (!c || !c->P) return fail(c, SVAE_EBADARG, "svae_bind must run first");
  const Geo& g = c->m.g;
  c->st = (hipStream_t)stream;
  HIPCHK(c, hipMemsetAsync(c->zero_img, 0, (size_t)g.B * g.H * g.W * g.C * sizeof(float), c->st));
  c->generative = true;
  c->x_in = nullptr;  // no training forward state: svae_backward is refused until svae_forward
  c->tgt_in = c->zero_img;
  c->eps_in = z;
  c->reg = 1.f;  // the generative chain's noise uses reg_coeff's default (placeholder_with_default 1.0, :917)
  const int r = engine_forward(c);
  c->generative = false;
  // injected chain noise is one-shot: the next call draws its own (tf.random_normal, :1090-1091)
  c->noise_in = nullptr;
  if (r) return r;
  HIPCHK(c, hipGetLastError());
  return 0;
}

int svae_set_external_grads(svae_ctx* c, const float* dxhat, const float* dz) {
  if (!c) return fail(c, SVAE_EBADARG, "null ctx");
  if (c->m.g.Te == c->m.g.T && (dxhat || dz)) return fail(c, SVAE_EBADARG, "external_generator_from is off");
  c->ext_dx = dxhat;
  c->ext_dz = dz;
  return 0;
}

int svae_backward(svae_ctx* c, void* stream) {
  if (!c || !c->x_in) return fail(c, SVAE_EBADARG, "svae_forward must run first");
  c->st = (hipStream_t)stream;
  int r = engine_backward(c);
  c->ext_dx = c->ext_dz = nullptr;  // one-shot
  if (c->side) {  // join: the side stream's weight gradients are ordered before later caller work
    side_merge(c);
    hipEventRecord(c->ev_join, c->st2);
    hipStreamWaitEvent(c->st, c->ev_join, 0);
    hipEventRecord(c->ev_j3, c->st3);
    hipStreamWaitEvent(c->st, c->ev_j3, 0);
  }
  if (!r && c->hook) c->hook(c->hook_user, -1);
  if (r) return r;
  HIPCHK(c, hipGetLastError());
  return 0;
}

int svae_set_chain_noise(svae_ctx* c, const float* noise) {
  if (!c) return fail(c, SVAE_EBADARG, "null ctx");
  if (noise && !c->m.g.noisy) return fail(c, SVAE_EBADARG, "add_noise_to_chain is off");
  c->noise_in = noise;
  return 0;
}

int svae_imp_range(svae_ctx* c, int64_t* phi_end) {
  if (!c || !phi_end) return fail(c, SVAE_EBADARG, "null");
  *phi_end = c->m.p_phi_end;
  return 0;
}

int svae_bind_imp(svae_ctx* c, float* grads_imp) {
  if (!c || !grads_imp) return fail(c, SVAE_EBADARG, "null buffer");
  if (!c->m.g.imp) return fail(c, SVAE_EBADARG, "add_improvement_maximization_loss is off");
  HIPCHK(c, hipMemset(grads_imp, 0, (size_t)c->m.p_total * sizeof(float)));
  if (c->m.shared && !c->Gimp_v) {
    hipError_t e = hipMalloc((void**)&c->Gimp_v, (size_t)c->m.n_total * sizeof(float));
    if (e != hipSuccess) return fail(c, SVAE_ENOMEM, std::string("hipMalloc imp copies: ") + hipGetErrorString(e));
  }
  if (c->Gimp_v) HIPCHK(c, hipMemset(c->Gimp_v, 0, (size_t)c->m.n_total * sizeof(float)));
  c->Gimp_pub = grads_imp;
  return 0;
}

// d improvement_maximization_loss / d every variable (:1302-1303): the chain backward again, seeded
// by the improvement loss alone, into the svae_bind_imp buffer (no hook, no fused update)
int svae_backward_imp(svae_ctx* c, void* stream) {
  if (!c || !c->x_in) return fail(c, SVAE_EBADARG, "svae_forward must run first");
  if (!c->m.g.imp || !c->Gimp_pub) return fail(c, SVAE_EBADARG, "svae_bind_imp must run first");
  if (c->m.g.T < 2) return fail(c, SVAE_EBADARG, "the improvement loss needs mc_steps >= 2");
  c->st = (hipStream_t)stream;
  HIPCHK(c, hipMemsetAsync(c->kl_zero, 0, 64 * sizeof(float), c->st));
  float *gr = c->Gr, *gv = c->Gv, *gp = c->Gpub;
  svae_step_hook hk = c->hook;
  const bool fa = c->fa_on;
  c->hook = nullptr;
  c->fa_on = false;
  c->imp_pass = true;
  c->Gpub = c->Gimp_pub;
  c->Gv = c->Gimp_v;
  c->Gr = c->m.shared ? c->Gimp_v : c->Gimp_pub;
  int r = engine_backward(c);
  if (c->side) {
    side_merge(c);
    hipEventRecord(c->ev_join, c->st2);
    hipStreamWaitEvent(c->st, c->ev_join, 0);
    hipEventRecord(c->ev_j3, c->st3);
    hipStreamWaitEvent(c->st, c->ev_j3, 0);
  }
  c->imp_pass = false;
  c->Gr = gr;
  c->Gv = gv;
  c->Gpub = gp;
  c->hook = hk;
  c->fa_on = fa;
  if (r) return r;
  HIPCHK(c, hipGetLastError());
  return 0;
}

int svae_set_backward_hook(svae_ctx* c, svae_step_hook hook, void* user) {
  if (!c) return fail(c, SVAE_EBADARG, "null ctx");
  c->hook = hook;
  c->hook_user = user;
  return 0;
}

void* svae_hook_stream(svae_ctx* c) { return c ? (void*)(c->side ? c->st2 : c->st) : nullptr; }

// clip + TF Adam (sequential_vae.py:1267,1274-1276) on the public live sub-range [lo, hi); in bf16
// mode without sharing also the bf16 shadows of the tensors that start in it (N layout fused into
// the update, per-tap transposes of its tiles), counted in c->fresh for the next forward
static void adam_range(svae_ctx* c, long long lo, long long hi, float lr, long long step, float clip, hipStream_t s) {
  const double b1 = 0.9, b2 = 0.999;
  const double lr_t = lr * std::sqrt(1.0 - std::pow(b2, (double)step)) / (1.0 - std::pow(b1, (double)step));
  const bool sh = c->m.g.bf16 && !c->m.shared && c->wN;
  adam_step(c->Ppub + lo, c->Gpub + lo, c->adam_m + lo, c->adam_v + lo, sh ? (void*)((__bf16*)c->wN + lo) : nullptr,
            hi - lo, (float)lr_t, (float)b1, (float)b2, 1e-8f, clip, c->nsp, c->wplane, s, c->wtab, lo, c->wovf);
  if (sh) {
    const long long tb = std::lower_bound(c->tile_off.begin(), c->tile_off.end(), lo) - c->tile_off.begin();
    const long long te = std::lower_bound(c->tile_off.begin(), c->tile_off.end(), hi) - c->tile_off.begin();
    shadow_t_tiles(c->Ppub, c->wT, (const int*)c->tiles_d + 4 * tb, (int)(te - tb), c->offs_d, c->nsp, c->wplane, s,
                   c->wtab);
    c->fresh += hi - lo;
  }
}

int svae_adam(svae_ctx* c, float lr, int64_t step, float clip, void* stream) {
  if (!c || !c->P || step < 1) return fail(c, SVAE_EBADARG, "bad adam args");
  adam_range(c, 0, c->m.p_live, lr, step, clip, (hipStream_t)stream);
  HIPCHK(c, hipGetLastError());
  return 0;
}

int svae_adam_range(svae_ctx* c, int64_t lo, int64_t hi, float lr, int64_t step, float clip, void* stream) {
  if (!c || !c->P || step < 1 || lo < 0 || hi > c->m.p_live || lo >= hi || (lo & 3))
    return fail(c, SVAE_EBADARG, "bad adam range");
  adam_range(c, lo, hi, lr, step, clip, (hipStream_t)stream);
  HIPCHK(c, hipGetLastError());
  return 0;
}

int svae_backward_adam(svae_ctx* c, float lr, int64_t step, float clip, void* stream) {
  if (!c || !c->P || step < 1) return fail(c, SVAE_EBADARG, "bad adam args");
  const bool fuse = c->side && !c->m.shared;
  c->fa_on = fuse;
  c->fa_lr = lr;
  c->fa_step = step;
  c->fa_clip = clip;
  const int r = svae_backward(c, stream);
  c->fa_on = false;
  if (r) return r;
  if (!fuse) return svae_adam(c, lr, step, clip, stream);
  adam_range(c, 0, c->m.phi_hi, lr, step, clip, (hipStream_t)stream);  // recognition bucket, after hook(-1)
  HIPCHK(c, hipGetLastError());
  return 0;
}

// the improvement loss's own apply_gradients over the recognition variables (:1304-1306), with the
// ELBO update's Adam moments (one AdamOptimizer)
int svae_adam_imp(svae_ctx* c, float lr, int64_t step, float clip, void* stream) {
  if (!c || !c->P || step < 1 || !c->Gimp_pub) return fail(c, SVAE_EBADARG, "bad adam_imp args");
  float* gp = c->Gpub;
  const long long f0 = c->fresh;  // re-refreshes shadows the ELBO update already counted
  c->Gpub = c->Gimp_pub;
  adam_range(c, 0, c->m.p_phi_end, lr, step, clip, (hipStream_t)stream);
  c->Gpub = gp;
  c->fresh = f0;
  HIPCHK(c, hipGetLastError());
  return 0;
}

int svae_adam_state(svae_ctx* c, int dir, float* m, float* v, int64_t n, void* stream) {
  if (!c || !m || !v || n != c->m.p_live || (dir != 0 && dir != 1)) return fail(c, SVAE_EBADARG, "bad adam_state args");
  const size_t b = (size_t)n * sizeof(float);
  hipStream_t s = (hipStream_t)stream;
  if (dir == 0) {
    HIPCHK(c, hipMemcpyAsync(m, c->adam_m, b, hipMemcpyDeviceToDevice, s));
    HIPCHK(c, hipMemcpyAsync(v, c->adam_v, b, hipMemcpyDeviceToDevice, s));
  } else {
    HIPCHK(c, hipMemcpyAsync(c->adam_m, m, b, hipMemcpyDeviceToDevice, s));
    HIPCHK(c, hipMemcpyAsync(c->adam_v, v, b, hipMemcpyDeviceToDevice, s));
  }
  return 0;
}

int svae_copy_out(svae_ctx* c, int which, int step, float* dst, int64_t n, void* stream) {
  if (!c || !dst) return fail(c, SVAE_EBADARG, "null");
  const Geo& g = c->m.g;
  if (which < 100 && (step < 0 || step >= g.T)) return fail(c, SVAE_EBADARG, "step out of range");
  const float* src = nullptr;
  long long cnt = 0;
  bool src_bf16 = false;  // bf16-stored activation (abf): widened to fp32 on the way out
  const long long ml = (long long)g.B * g.Dz;
  switch (which) {
    case SVAE_BUF_XHAT: src = c->sb[step].xhat; cnt = (long long)g.B * g.H * g.W * g.C; break;
    case SVAE_BUF_MU: src = c->mu + step * ml; cnt = ml; break;
    case SVAE_BUF_SIGMA: src = c->sig + step * ml; cnt = ml; break;
    case SVAE_BUF_Z: src = c->z + step * ml; cnt = ml; break;
    case SVAE_BUF_STEP_STATS: src = c->sb[step].stats; cnt = 2; break;
    case SVAE_BUF_REC_IMG: src = c->sb[step].rec_img; cnt = g.B; break;
    case SVAE_BUF_KL_IMG: src = c->kl_img + (long long)step * g.B; cnt = g.B; break;
    case SVAE_BUF_DZ: src = c->dz + step * ml; cnt = ml; break;
    case SVAE_BUF_SAMPLE: src = chain_x(c, step); cnt = (long long)g.B * g.H * g.W * g.C; break;
    case SVAE_BUF_STDDEV:
      if (!g.pgn) return fail(c, SVAE_EBADARG, "predict_generator_noise is off");
      src = c->sb[step].sd; cnt = (long long)g.B * g.H * g.W;
      break;
    case SVAE_BUF_IMP_IMG:
      if (!g.imp || step < 1) return fail(c, SVAE_EBADARG, "improvement loss off, or step 0");
      src = c->imp_img + (long long)step * g.B; cnt = g.B;
      break;
    case 100: src = c->dx[step & 1]; cnt = (long long)g.B * g.H * g.W * g.C; break;  // debug: dx carry
    case 101: c->dbg_stop_step = step; return 0;                                    // debug: stop step
    case 102: c->dbg_stop_lvl = step; return 0;                                     // debug: stop level
    case 103: src = c->dcur; cnt = n; break;                                        // debug: raw scratch
    case 104: src = c->dnext; cnt = n; break;
    case 105: src = c->sb[c->dbg_stop_step].s1_pre[step]; cnt = n; src_bf16 = c->pbf; break;  // debug: saved tensors
    case 109: src = c->dpre; cnt = n; break;
    case 110: src = c->dbg_last; cnt = n; break;
    case 111: c->dbg_stop_lvl2 = step; return 0;
    case 113: src = c->inf_pre_a[step]; cnt = n; src_bf16 = c->pbf; break;  // debug: inference level `step`, all T groups
    case 114: src = c->inf_act_a[step]; cnt = n; src_bf16 = c->abf; break;
    case 115: src = c->inf_pre_b[step]; cnt = n; src_bf16 = c->pbf; break;
    case 116: src = c->inf_act_b[step]; cnt = n; break;
    case 106: src = c->sb[c->dbg_stop_step].s1_act[step]; cnt = n; src_bf16 = c->abf; break;
    case 107: src = c->sb[c->dbg_stop_step].s1_bn[step].mean; cnt = n; break;
    case 108: src = c->sb[c->dbg_stop_step].s1_bn[step].invstd; cnt = n; break;
    default: return fail(c, SVAE_EBADARG, "unknown buffer");
  }
  if (n < cnt) return fail(c, SVAE_EBADARG, "destination too small");
  if (src_bf16) {
    bf16_to_f32(src, dst, cnt, (hipStream_t)stream);
    HIPCHK(c, hipGetLastError());
    return 0;
  }
  HIPCHK(c, hipMemcpyAsync(dst, src, cnt * sizeof(float), hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return 0;
}

}  // extern "C"

// ============================================================================
// per-op entry points (kernel-level parity tests; same launch paths as the engine)
// ============================================================================
extern "C" {

int svae_op_conv(const float* x, int n, int h, int cin, const float* w, int cout, int stride, int transpose, float* y,
                 void* stream) {
  if (!x || !w || !y || (stride != 1 && stride != 2) || cout % 4) return fail(nullptr, SVAE_EBADARG, "bad op args");
  ConvL L;
  L.cin = cin; L.cout = cout; L.stride = stride; L.hin = h; L.tr = transpose != 0;
  L.hout = L.tr ? h * stride : h / stride;
  FwdArgs a = fwd_args_conv(L, n, w, 0);
  a.A = x; a.lda = cin;
  a.C = y; a.ldc = cout;
  igemm_fwd(a, 1, (hipStream_t)stream);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(nullptr, SVAE_EHIP, hipGetErrorString(e));
}

int svae_op_gather_bf16(const float* x, int n, int h, int cin, const void* w_nk, int cout, int stride, int transpose,
                        int path, float* y, void* scratch, int64_t scratch_bytes, void* stream) {
  const int split = (path >> 4) & 1;  // bit 4: split-bf16 planes (dtype bf16x6): w_nk holds 3 planes
  const int path_in = path;
  path &= 15;
  if (!x || !w_nk || !y || (stride != 1 && stride != 2) || path < 0 || path > 2)
    return fail(nullptr, SVAE_EBADARG, "bad op args");
  ConvL L;
  L.cin = cin; L.cout = cout; L.stride = stride; L.hin = h; L.tr = transpose != 0;
  L.hout = L.tr ? h * stride : h / stride;
  FwdArgs a = fwd_args_conv(L, n, nullptr, 0);
  a.A = x; a.lda = cin;
  a.Bh = w_nk; a.ldb = cin; a.b_tap = (long long)cin * cout;
  a.C = y; a.ldc = cout;
  a.part = (float*)scratch;
  a.part_cap = scratch ? scratch_bytes / (int64_t)sizeof(float) : 0;
  if (split) {
    a.nsp = 3;
    a.b_plane = 16LL * cin * cout;
    a.h16 = (path_in >> 5) & 1;  // bit 5: w_nk also holds the scaled fp16 planes (5 planes in all)
  }
  if (igemm_bf16_path(a, 1, path, (hipStream_t)stream) < 0)
    return fail(nullptr, SVAE_EBADARG, "shape does not qualify for the halo-tile kernel");
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(nullptr, SVAE_EHIP, hipGetErrorString(e));
}

int svae_op_wgrad_bf16(const float* x, int n, int h, int cin, const float* dy, int cout, int stride, int transpose,
                       int path, float* dw, void* scratch, int64_t scratch_bytes, void* stream) {
  const int xbf = (path >> 4) & 1, dybf = (path >> 5) & 1;  // operand storage bits (bf16 tensors)
  path &= 15;
  if (!x || !dy || !dw || !scratch || (path != 0 && path != 2 && path != 3))
    return fail(nullptr, SVAE_EBADARG, "bad op args");
  static svae_ctx dummy;
  dummy.m.g.B = n;
  dummy.m.g.bf16 = 1;
  dummy.dbf = dybf;
  dummy.wg_path = path;
  dummy.st = (hipStream_t)stream;
  dummy.slab = (float*)scratch;
  dummy.slab_cap = scratch_bytes / (int64_t)sizeof(float);
  ConvL L;
  L.cin = cin; L.cout = cout; L.stride = stride; L.hin = h; L.tr = transpose != 0;
  L.hout = L.tr ? h * stride : h / stride;
  const int r = conv_wgrad(&dummy, L, 1, 0, View{(float*)x, cin, 0, xbf}, dy, 0, dw);
  dummy.m.g.bf16 = 0;
  dummy.dbf = 0;
  if (r) return fail(nullptr, r, dummy.err);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(nullptr, SVAE_EHIP, hipGetErrorString(e));
}

int svae_op_conv_dgrad(const float* dy, int n, int h, int cin, const float* w, int cout, int stride, int transpose,
                       float* dx, void* stream) {
  if (!dy || !w || !dx) return fail(nullptr, SVAE_EBADARG, "bad op args");
  static svae_ctx dummy;
  dummy.m.g.B = n;
  dummy.P = (float*)w;
  dummy.st = (hipStream_t)stream;
  ConvL L;
  L.cin = cin; L.cout = cout; L.stride = stride; L.hin = h; L.tr = transpose != 0;
  L.hout = L.tr ? h * stride : h / stride;
  L.ow = 0;
  int r = conv_dgrad(&dummy, L, 1, 0, dy, 0, View{dx, cin, 0}, 0);
  if (r) return fail(nullptr, r, dummy.err);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(nullptr, SVAE_EHIP, hipGetErrorString(e));
}

int svae_op_conv_wgrad(const float* x, int n, int h, int cin, const float* dy, int cout, int stride, int transpose,
                       float* dw, void* scratch, int64_t scratch_bytes, void* stream) {
  if (!x || !dy || !dw || !scratch) return fail(nullptr, SVAE_EBADARG, "bad op args");
  static svae_ctx dummy;
  dummy.m.g.B = n;
  dummy.st = (hipStream_t)stream;
  dummy.slab = (float*)scratch;
  dummy.slab_cap = scratch_bytes / (int64_t)sizeof(float);
  ConvL L;
  L.cin = cin; L.cout = cout; L.stride = stride; L.hin = h; L.tr = transpose != 0;
  L.hout = L.tr ? h * stride : h / stride;
  int r = conv_wgrad(&dummy, L, 1, 0, View{(float*)x, cin, 0}, dy, 0, dw);
  if (r) return fail(nullptr, r, dummy.err);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(nullptr, SVAE_EHIP, hipGetErrorString(e));
}

int svae_op_bn_act(const float* x, int64_t rows, int c, const float* beta, int act, float* y, float* mean,
                   float* invstd, void* scratch, int64_t scratch_bytes, void* stream) {
  if (!x || !beta || !y || !mean || !invstd || !scratch || c % 4) return fail(nullptr, SVAE_EBADARG, "bad op args");
  hipStream_t s = (hipStream_t)stream;
  const int nsh = bn_acc_shards(bn_bwd_rowblocks(rows));
  if ((int64_t)nsh * 4 * c * 8 + 2 * c * 4 > scratch_bytes) return fail(nullptr, SVAE_EBADARG, "scratch too small");
  u64* acc = (u64*)scratch;
  float* zi = (float*)(acc + (long long)nsh * 4 * c);  // zeros (mean) / ones (invstd): raw-moment reduction
  if (hipMemsetAsync(acc, 0, (size_t)nsh * 4 * c * sizeof(u64), s) != hipSuccess)
    return fail(nullptr, SVAE_EHIP, "hipMemsetAsync");
  fill_f32(zi, c, 0.f, s);
  fill_f32(zi + c, c, 1.f, s);
  // sum(x), sum(x^2) via the backward reducer with act=none, mean=0, invstd=1
  bn_bwd_reduce(x, c, 0, x, c, 0, x, c, 0, rows, c, zi, zi + c, 0, nullptr, 0, ACT_NONE, acc, 0, 4LL * c, nsh, 1, s);
  bn_apply(x, c, 0, rows, c, acc, 0, 4LL * c, nsh, 1e-3f, mean, invstd, 0, beta, 0, nullptr, 0, 0, act, y, c, 0, 1, s);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(nullptr, SVAE_EHIP, hipGetErrorString(e));
}

int svae_op_bn_act_bwd(const float* dy, const float* y, const float* x, int64_t rows, int c, const float* mean,
                       const float* invstd, int act, float* dx, float* dbeta, void* scratch, int64_t scratch_bytes,
                       void* stream) {
  if (!dy || !y || !x || !dx || !dbeta || !scratch || c % 4) return fail(nullptr, SVAE_EBADARG, "bad op args");
  static svae_ctx dummy;
  dummy.st = (hipStream_t)stream;
  dummy.bnacc = (u64*)scratch;
  dummy.bnacc_cap = scratch_bytes / (int64_t)sizeof(u64);
  dummy.bnacc_hw = 4LL * c * bn_acc_shards(bn_bwd_rowblocks(rows));  // zero just the region this op takes
  if (dummy.bnacc_hw > dummy.bnacc_cap) return fail(nullptr, SVAE_EBADARG, "scratch too small");
  if (acc_reset(&dummy)) return fail(nullptr, SVAE_EHIP, dummy.err);
  dummy.Gr = dbeta;
  BNS bn{(float*)mean, (float*)invstd};
  int r = bn_act_bwd(&dummy, 1, rows, c, View{(float*)dy, c, 0}, View{(float*)y, c, 0}, x, 0, c, bn, 0, 0, 0, act, dx,
                     0, View{}, 0);
  if (r) return fail(nullptr, r, dummy.err);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(nullptr, SVAE_EHIP, hipGetErrorString(e));
}

int svae_op_fc(const float* x, int b, int k, const float* w, int nout, float* y, void* stream) {
  if (!x || !w || !y || nout % 4 || k % 4) return fail(nullptr, SVAE_EBADARG, "bad op args");
  FwdArgs a{};
  a.A = x; a.lda = k;
  a.B = w; a.b_nk = 0; a.ldb = nout; a.b_tap = 0;
  a.C = y; a.ldc = nout;
  a.N = nout; a.Cin = k;
  a.g.mode = GM_DENSE; a.g.nimg = b; a.g.ksz = 1; a.g.stride = 1;
  a.rows = b; a.nclass = 1;
  igemm_fwd(a, 1, (hipStream_t)stream);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(nullptr, SVAE_EHIP, hipGetErrorString(e));
}

}  // extern "C"
