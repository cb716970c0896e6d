// Host-side fuzz of the C-ABI (include/rgan.h) under AddressSanitizer + UBSan, CPU only.
//
// Built by tests/test_host_asan.py from the product's own csrc/*.hip with -fsanitize=address,
// undefined on the host half only (hipcc -Xarch_host; the device half is compiled normally and
// never launched).  What runs is every host-side planner / validator the entry points
// reach before a launch: descriptor checks (desc_ok), the GEMM planners (plan_fwd / dgrad /
// wgrad, choose_tiling, set_fast, the narrow / dense / 3x3 planners), workspace / pack / BN
// segment sizing, and the RGAN_EINVAL paths of the compute entry points.  No call here may
// reach a kernel launch: the compute entry points only ever get malformed arguments, and each
// must answer RGAN_EINVAL (a launch attempt on this GPU-less host would return a HIP error
// instead, which the harness reports as "reached a launch").
//
// Exit 0 and one "abi_fuzz ok" line, or a sanitizer report / a list of failures.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstdint>
#include <vector>
#include <string>

#include "rgan.h"

static int g_fail = 0;
static long long g_calls = 0;

static void expect_einval(int rc, const char* what) {
  ++g_calls;
  if (rc != RGAN_EINVAL) {
    std::fprintf(stderr, "FAIL %s: rc %d (want RGAN_EINVAL %d)\n", what, rc, RGAN_EINVAL);
    ++g_fail;
  }
}

// deterministic generator (splitmix64)
struct Rng {
  uint64_t s;
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  int pick(const std::vector<int>& v) { return v[next() % v.size()]; }
  long long pickl(const std::vector<long long>& v) { return v[next() % v.size()]; }
};

static const std::vector<int> kInts = {-2147483647 - 1, -65536, -7, -1, 0, 1, 2, 3, 4, 5, 7, 8, 16, 31, 32, 33,
                                       64, 128, 129, 1024, 4096, 65535, 65536, 1 << 20, 1 << 28, 2147483647};
static const std::vector<int> kSmall = {-1, 0, 1, 2, 3, 4, 8, 16, 32, 64, 128, 256};

static void nhwc_strides(RganConv& d) {
  d.xs[0] = (long long)d.hin * d.win * d.cin; d.xs[1] = 1; d.xs[2] = (long long)d.win * d.cin; d.xs[3] = d.cin;
  d.ys[0] = (long long)d.hout * d.wout * d.cout; d.ys[1] = 1; d.ys[2] = (long long)d.wout * d.cout; d.ys[3] = d.cout;
}

// a consistent descriptor of a random family the planners special-case
static RganConv valid_desc(Rng& r) {
  RganConv d{};
  d.batch = 1 + (int)(r.next() % 64);
  const int fam = (int)(r.next() % 7);
  auto ch = [&]() { return r.pick({1, 2, 3, 4, 8, 16, 32, 48, 64, 96, 128, 256, 512, 1024}); };
  switch (fam) {
    case 0:  // k4 s2 p1 conv (D's layers)
    case 1:  // k4 s2 p1 ConvT (G's layers)
      d.kh = d.kw = 4; d.stride = 2; d.pad = 1; d.transposed = fam;
      d.cin = ch(); d.cout = ch();
      d.hin = d.win = r.pick({1, 2, 4, 8, 16, 32});
      if (fam == 0) { d.hin *= 2; d.win *= 2; d.hout = d.hin / 2; d.wout = d.win / 2; }
      else { d.hout = 2 * d.hin; d.wout = 2 * d.win; }
      break;
    case 2:  // G's 1x1 -> 4x4 first layer
      d.kh = d.kw = 4; d.stride = 1; d.pad = 0; d.transposed = 1;
      d.cin = ch(); d.cout = ch(); d.hin = d.win = 1; d.hout = d.wout = 4;
      break;
    case 3:  // D's dense head
      d.kh = d.kw = 4; d.stride = 1; d.pad = 0; d.transposed = 0;
      d.cin = ch(); d.cout = 1; d.hin = d.win = 4; d.hout = d.wout = 1;
      break;
    case 4:  // arch 1's 3x3 stride-1 layers
      d.kh = d.kw = 3; d.stride = 1; d.pad = 1; d.transposed = 0;
      d.cin = ch(); d.cout = ch(); d.hin = d.win = r.pick({4, 8, 16, 32}); d.hout = d.hin; d.wout = d.win;
      break;
    case 5:  // NN_conv's folded / odd shapes
      d.kh = d.kw = 3; d.stride = 1; d.pad = 1; d.transposed = 1;
      d.cin = ch(); d.cout = ch(); d.hin = d.win = r.pick({2, 4, 8}); d.hout = d.hin; d.wout = d.win;
      break;
    default:  // generic strided conv
      d.kh = r.pick({1, 2, 3, 5}); d.kw = d.kh; d.stride = r.pick({1, 2, 3}); d.pad = r.pick({0, 1, 2});
      d.transposed = 0; d.cin = ch(); d.cout = ch();
      d.hin = d.win = r.pick({5, 7, 9, 16});
      d.hout = (d.hin + 2 * d.pad - d.kh) / d.stride + 1; d.wout = (d.win + 2 * d.pad - d.kw) / d.stride + 1;
      if (d.hout < 1) { d.hin = d.win = d.kh + 4; d.hout = d.wout = (d.hin + 2 * d.pad - d.kh) / d.stride + 1; }
      break;
  }
  nhwc_strides(d);
  if (r.next() % 4 == 0) {  // NCHW
    d.xs[0] = (long long)d.cin * d.hin * d.win; d.xs[1] = (long long)d.hin * d.win; d.xs[2] = d.win; d.xs[3] = 1;
    d.ys[0] = (long long)d.cout * d.hout * d.wout; d.ys[1] = (long long)d.hout * d.wout; d.ys[2] = d.wout; d.ys[3] = 1;
  }
  return d;
}

// one field of a valid descriptor replaced by an extreme value
static RganConv mangle(Rng& r, RganConv d) {
  int* f[] = {&d.batch, &d.cin, &d.hin, &d.win, &d.cout, &d.hout, &d.wout, &d.kh, &d.kw, &d.stride, &d.pad,
              &d.transposed};
  const int n = 1 + (int)(r.next() % 3);
  for (int i = 0; i < n; ++i) {
    const uint64_t k = r.next() % 14;
    if (k < 12) *f[k] = r.pick(kInts);
    else (k == 12 ? d.xs : d.ys)[r.next() % 4] = r.pickl({-1, 0, 3, 1LL << 40, -(1LL << 40), 0x7fffffffffffffffLL});
  }
  return d;
}

static void query_all(const RganConv* d) {
  int ph = 0;
  for (int which = -1; which <= 3; ++which) {
    (void)rgan_conv_workspace(d, which, 0);
    (void)rgan_conv_workspace(d, which, 1);
    (void)rgan_conv_pack_floats(d, which);
    for (int mode = 0; mode <= 3; ++mode)
      for (int nseg = -1; nseg <= 2; ++nseg) (void)rgan_conv_post_segments(d, which, mode, nseg, &ph);
    g_calls += 4 + 16;
  }
  for (int segs = -1; segs <= 3; ++segs) (void)rgan_conv_bn_segments(d, segs);
  (void)rgan_conv_post_segments(d, 1, 2, 1, nullptr);
  g_calls += 6;
}

// every compute entry point with malformed arguments: RGAN_EINVAL, no launch
static void malformed_compute(Rng& r, const RganConv& good) {
  alignas(16) static float buf[64];
  float* p = buf;
  const RganConv* d = &good;
  RganConv bad = good;
  bad.hout += 1;  // inconsistent geometry
  int fused = 0;
  RganPost post{};
  char ws[256];
  // conv family: null operands, bad descriptors, bad which / post
  expect_einval(rgan_conv_fwd(d, nullptr, p, nullptr, nullptr, nullptr, p, 0, 0.f, ws, sizeof ws, nullptr), "conv_fwd x=0");
  expect_einval(rgan_conv_fwd(d, p, nullptr, nullptr, nullptr, nullptr, p, 0, 0.f, ws, sizeof ws, nullptr), "conv_fwd w=0");
  expect_einval(rgan_conv_fwd(&bad, p, p, nullptr, nullptr, nullptr, p, 0, 0.f, ws, sizeof ws, nullptr), "conv_fwd bad desc");
  expect_einval(rgan_conv_fwd(nullptr, p, p, nullptr, nullptr, nullptr, p, 0, 0.f, ws, sizeof ws, nullptr), "conv_fwd d=0");
  expect_einval(rgan_conv_fwd_bn(d, p, p, nullptr, nullptr, nullptr, p, ws, sizeof ws, nullptr, 0, 0, &fused, nullptr), "conv_fwd_bn segs=0");
  expect_einval(rgan_conv_fwd_bn(d, p, p, nullptr, nullptr, nullptr, p, ws, sizeof ws, nullptr, 0, 1, nullptr, nullptr), "conv_fwd_bn fused=0");
  expect_einval(rgan_conv_fwd_bn(&bad, p, p, nullptr, nullptr, nullptr, p, ws, sizeof ws, nullptr, 0, 1, &fused, nullptr), "conv_fwd_bn bad desc");
  expect_einval(rgan_conv_dgrad(d, nullptr, p, nullptr, nullptr, p, ws, sizeof ws, nullptr), "conv_dgrad dy=0");
  expect_einval(rgan_conv_dgrad(&bad, p, p, nullptr, nullptr, p, ws, sizeof ws, nullptr), "conv_dgrad bad desc");
  expect_einval(rgan_conv_wgrad(d, nullptr, p, p, nullptr, 0, ws, sizeof ws, nullptr), "conv_wgrad x=0");
  expect_einval(rgan_conv_wgrad(&bad, p, p, p, nullptr, 0, ws, sizeof ws, nullptr), "conv_wgrad bad desc");
  expect_einval(rgan_conv_wgrad_rows(d, p, p, p, p, -1, 0, ws, sizeof ws, nullptr), "conv_wgrad_rows row0<0");
  expect_einval(rgan_conv_wgrad_rows(d, p, p, p, p, 1LL << 40, 0, ws, sizeof ws, nullptr), "conv_wgrad_rows row0>=P");
  expect_einval(rgan_conv_wgrad_rows(d, nullptr, p, p, p, 0, 0, ws, sizeof ws, nullptr), "conv_wgrad_rows x=0");
  expect_einval(rgan_conv_post(d, 2, p, p, nullptr, nullptr, p, ws, sizeof ws, &post, &fused, nullptr), "conv_post which=2");
  post.mode = 3; post.x = p;
  expect_einval(rgan_conv_post(d, 1, p, p, nullptr, nullptr, p, ws, sizeof ws, &post, &fused, nullptr), "conv_post mode=3");
  post.mode = 2; post.nseg = 0;
  expect_einval(rgan_conv_post(d, 1, p, p, nullptr, nullptr, p, ws, sizeof ws, &post, &fused, nullptr), "conv_post nseg=0");
  post.mode = 1; post.x = nullptr;
  expect_einval(rgan_conv_post(d, 1, p, p, nullptr, nullptr, p, ws, sizeof ws, &post, &fused, nullptr), "conv_post x=0");
  expect_einval(rgan_conv_post(&bad, 1, p, p, nullptr, nullptr, p, ws, sizeof ws, nullptr, &fused, nullptr), "conv_post post=0");
  expect_einval(rgan_conv_pack(d, 2, p, p, nullptr), "conv_pack which=2");
  expect_einval(rgan_conv_pack(&bad, 0, p, p, nullptr), "conv_pack bad desc");
  expect_einval(rgan_conv_pack(d, 0, nullptr, p, nullptr), "conv_pack w=0");
  {
    const RganConv* ds[2] = {d, &bad};
    const int wh[2] = {0, 0};
    const float* ws_[2] = {p, p};
    float* pk[2] = {p, p};
    expect_einval(rgan_conv_pack_batch(-1, ds, wh, ws_, pk, nullptr), "conv_pack_batch n<0");
    expect_einval(rgan_conv_pack_batch(2, nullptr, wh, ws_, pk, nullptr), "conv_pack_batch d=0");
    const RganConv* ds2[1] = {&bad};
    expect_einval(rgan_conv_pack_batch(1, ds2, wh, ws_, pk, nullptr), "conv_pack_batch bad desc");
    const int wh2[1] = {5};
    expect_einval(rgan_conv_pack_batch(1, ds, wh2, ws_, pk, nullptr), "conv_pack_batch which=5");
  }
  // first layer (only instantiated B / Cin pass; the rest are refused)
  expect_einval(rgan_g1_fwd_bn(p, 33, 128, p, 64, nullptr, nullptr, 1e-5f, 0.1f, p, p, nullptr, 0, 0.f, p, p, p,
                               nullptr),
                "g1_fwd_bn B=33");
  expect_einval(rgan_g1_wgrad(p, 32, 7, p, 64, p, 0, nullptr), "g1_wgrad Cin=7");
  // BatchNorm / activation / sums
  const long long Pn = -5;
  const int Cn = r.pick({-3, 0});
  expect_einval(rgan_bn_stats(p, Pn, 8, 8, 1, 1e-5f, 0.1f, p, p, nullptr, p, ws, nullptr), "bn_stats P<0");
  expect_einval(rgan_bn_apply(nullptr, 16, 8, 8, 1, p, p, p, 0, 0.f, p, 8, 1, nullptr), "bn_apply y=0");
  expect_einval(rgan_bn_apply(p, 16, Cn, 8, 1, p, p, p, 0, 0.f, p, 8, 1, nullptr), "bn_apply C<=0");
  expect_einval(rgan_bn_apply_segments(p, 16, 8, 0, p, p, p, 0, 0.f, p, nullptr), "bn_apply_segments nseg=0");
  expect_einval(rgan_bn_moments(p, Pn, 8, 8, 1, (double*)p, ws, nullptr), "bn_moments P<0");
  expect_einval(rgan_bn_finalize(nullptr, 0, 8, 1e-5f, 0.1f, p, p, nullptr, p, nullptr), "bn_finalize nranks=0");
  expect_einval(rgan_bn_segment_stats(nullptr, 0, 0, 8, 64, 1e-5f, 0.1f, p, p, nullptr, p, nullptr, nullptr),
                "bn_segment_stats part=0");
  expect_einval(rgan_bn_segment_stats_n(nullptr, 0, 0, 0, 8, 64, 1e-5f, 0.1f, p, p, nullptr, p, nullptr), "bn_segment_stats_n nseg=0");
  expect_einval(rgan_bn_backward(p, 8, 1, p, Pn, 8, 8, 1, p, p, p, 0, 0.f, p, 8, 1, p, p, ws, nullptr),
                "bn_backward P<0");
  expect_einval(rgan_bn_backward_segments(p, p, 16, Cn, 1, p, p, p, 0, 0.f, p, p, p, ws, nullptr),
                "bn_backward_segments C<=0");
  expect_einval(rgan_bn_backward_parts(p, p, 16, 8, 0, p, p, p, nullptr, 0, 1, p, p, p, nullptr, nullptr),
                "bn_backward_parts nseg=0");
  expect_einval(rgan_bn_segment_apply((double*)p, 4, 0, 64, p, 256, 8, 1e-5f, 0.1f, p, p, nullptr, p, p, 0, 0.f, p,
                                      p, nullptr), "bn_segment_apply nseg=0");
  expect_einval(rgan_bn_segment_apply((double*)p, 4, 1, 64, p, 255, 8, 1e-5f, 0.1f, p, p, nullptr, p, p, 0, 0.f, p,
                                      p, nullptr), "bn_segment_apply P != S * seg_rows");
  expect_einval(rgan_bn_segment_apply((double*)p, 4, 1, 64, p, 256, 8, 1e-5f, 0.1f, p, p, nullptr, p, p, 99, 0.f,
                                      p, p, nullptr), "bn_segment_apply act=99");
  expect_einval(rgan_bn_backward_sums_apply(p, p, Pn, 8, p, p, p, 0, 0.f, nullptr, p, p, p, 0, (double*)p, ws,
                                            nullptr), "bn_backward_sums_apply P<0");
  expect_einval(rgan_bn_backward_sums_apply(p, p, 16, 8, p, p, p, 0, 0.f, nullptr, p, p, p, 0, nullptr, ws,
                                            nullptr), "bn_backward_sums_apply sums=0");
  expect_einval(rgan_act_backward(nullptr, p, 16, 1, 0.f, p, nullptr), "act_backward da=0");
  expect_einval(rgan_act_backward(p, p, -1, 1, 0.f, p, nullptr), "act_backward n<0");
  expect_einval(rgan_act_backward_ex(p, p, p, 16, 99, 0.f, p, nullptr), "act_backward_ex act=99");
  expect_einval(rgan_channel_sum(p, Pn, 8, 8, 1, p, 0, ws, nullptr), "channel_sum P<0");
  expect_einval(rgan_channel_sum(p, 16, 8, 8, 1, p, 0, nullptr, nullptr), "channel_sum partial=0");
  expect_einval(rgan_bn_affine_grads(nullptr, p, 8, p, p, 0, nullptr), "bn_affine_grads sums=0");
  // loss heads / GP / misc
  expect_einval(rgan_loss_head(9, 0, nullptr, nullptr, 8, nullptr, nullptr, nullptr, nullptr), "loss_head kind=9");
  expect_einval(rgan_loss_head(7, 0, p, p, 0, p, p, p, nullptr), "loss_head n=0");
  expect_einval(rgan_loss_head_pair(0, p, p, 8, p, p, p, nullptr), "loss_head_pair kind=0");
  expect_einval(rgan_loss_head_joint(7, nullptr, 8, p, p, nullptr), "loss_head_joint y=0");
  expect_einval(rgan_loss_head_dist(7, 0, 9, p, p, 8, 16, p, p, p, p, p, nullptr), "loss_head_dist phase=9");
  expect_einval(rgan_scale(p, p, -4, p, nullptr), "scale n<0");
  expect_einval(rgan_gp_interp(p, p, p, 0, 16, p, nullptr), "gp_interp batch=0");
  expect_einval(rgan_gp_penalty(nullptr, 4, 16, 10.f, 4, p, p, nullptr), "gp_penalty g=0");
  expect_einval(rgan_gp_penalty_backward(p, p, 4, -16, 10.f, 4, p, p, nullptr), "gp_penalty_backward per<0");
  expect_einval(rgan_spectral_power(nullptr, 8, 8, 8, 8, 8, 1e-12f, p, p, p, 1, ws, nullptr), "spectral_power W=0");
  expect_einval(rgan_spectral_power_batch(-1, nullptr, 1e-12f, ws, nullptr), "spectral_power_batch n<0");
  expect_einval(rgan_spectral_backward(p, p, 0, 8, 8, 8, 8, p, p, p, p, 0, ws, nullptr), "spectral_backward rows=0");
  expect_einval(rgan_adam(-1, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr), "adam n<0");
  expect_einval(rgan_adam(2, nullptr, nullptr, nullptr, nullptr, nullptr, (const double*)p, p, nullptr), "adam arrays=0");
  expect_einval(rgan_adam_packed(2, nullptr, nullptr, nullptr, nullptr, nullptr, (const double*)p, p, 0, nullptr, nullptr),
                "adam_packed arrays=0");
  expect_einval(rgan_adam_packed(0, nullptr, nullptr, nullptr, nullptr, nullptr, (const double*)p, p, 1, nullptr, nullptr),
                "adam_packed packs=0");
  {
    float* params[1] = {p};
    const float* grads[1] = {p};
    float* m[1] = {p};
    float* v[1] = {p};
    const long long numel[1] = {16};
    RganAdamPack pk{};
    pk.tensor = 3; pk.which = 0; pk.d = d; pk.packed = p;  // tensor index out of range
    expect_einval(rgan_adam_packed(1, params, grads, m, v, numel, (const double*)p, p, 1, &pk, nullptr),
                  "adam_packed tensor=3");
    pk.tensor = 0; pk.d = &bad;
    expect_einval(rgan_adam_packed(1, params, grads, m, v, numel, (const double*)p, p, 1, &pk, nullptr),
                  "adam_packed bad desc");
    const long long neg[1] = {-1};
    expect_einval(rgan_adam(1, params, grads, m, v, neg, (const double*)p, p, nullptr), "adam numel<0");
  }
  expect_einval(rgan_adam_step_inc(nullptr, nullptr), "adam_step_inc step=0");
  expect_einval(rgan_lr_decay(nullptr, 0.9, nullptr), "lr_decay hyper=0");
  expect_einval(rgan_gather_images(p, nullptr, 4, 16, p, nullptr), "gather_images idx=0");
  expect_einval(rgan_gather_images_u8(nullptr, nullptr, 4, 16, p, nullptr), "gather_images_u8 images=0");
  expect_einval(rgan_minmax(p, -1, p, ws, nullptr), "minmax n<0");
  expect_einval(rgan_images_to_u8(p, 0, 3, 8, 8, nullptr, 1.f, 0.f, nullptr, 0, 8, 2, (unsigned char*)ws, nullptr),
                "images_to_u8 B=0");
  {
    const long long st[4] = {192, 64, 8, 1};
    expect_einval(rgan_patches_k4s2(nullptr, 2, 3, 8, 8, st, p, nullptr), "patches img=0");
  }
  expect_einval(rgan_patch_weight(nullptr, 8, 3, 48, 16, p, nullptr), "patch_weight w=0");
  expect_einval(rgan_unpatch_grad(nullptr, 8, 3, 48, 1, p, 0, nullptr), "unpatch_grad g=0");
  expect_einval(rgan_nn_fold_weight(nullptr, 4, 4, p, nullptr), "nn_fold w=0");
  expect_einval(rgan_nn_unfold_grad(p, -4, 4, p, nullptr), "nn_unfold cout<0");
  expect_einval(rgan_rng_fill(p, 16, 7, 1, nullptr, nullptr), "rng_fill kind=7");
  expect_einval(rgan_rng_choice(nullptr, 8, 4, 1, nullptr, nullptr), "rng_choice out=0");
  expect_einval(rgan_rng_choice((long long*)p, 4, 8, 1, (unsigned long long*)p, nullptr), "rng_choice n>N");
  expect_einval(rgan_bn_dd_sums(nullptr, p, p, 16, 8, 8, 1, p, p, p, 0, 0.f, 1, nullptr, 16, (double*)p, ws, nullptr),
                "bn_dd_sums a=0");
  expect_einval(rgan_act_dd(nullptr, p, p, 16, 1, 0.f, p, p, nullptr), "act_dd a=0");
  (void)rgan_set_gemm_emulation(7);  // refused (-1), no state change
  ++g_calls;
}

int main(int argc, char** argv) {
  const long long iters = argc > 1 ? std::atoll(argv[1]) : 20000;
  Rng r{12345};
  // size queries on odd inputs
  for (long long P : {-1LL, 0LL, 1LL, 4095LL, 1LL << 31, 1LL << 40})
    for (int C : {-1, 0, 1, 3, 4096, 1 << 20}) {
      (void)rgan_bn_partial_bytes(P, C);
      (void)rgan_bn_dd_partial_bytes(P, C);
      (void)rgan_minmax_ws_bytes(P);
      g_calls += 3;
    }
  for (int rows : {-1, 0, 1, 4096, 1 << 30})
    for (int cols : {-1, 0, 1, 65536, 1 << 30}) { (void)rgan_spectral_ws_bytes(rows, cols); ++g_calls; }
  (void)rgan_spectral_batch_ws_bytes(-1, nullptr);
  (void)rgan_spectral_batch_ws_bytes(3, nullptr);
  {
    RganSnLayer l[2] = {};
    l[0].rows = -5; l[0].cols = 1 << 30;
    l[1].rows = 1 << 30; l[1].cols = 1 << 30;
    (void)rgan_spectral_batch_ws_bytes(2, l);
    expect_einval(rgan_spectral_power_batch(2, l, 1e-12f, nullptr, nullptr), "spectral_power_batch bad layers");
  }
  g_calls += 3;
  query_all(nullptr);
  // planners over valid descriptors of every family, then mangled ones
  for (long long it = 0; it < iters; ++it) {
    RganConv d = valid_desc(r);
    query_all(&d);
    if (it % 16 == 0) malformed_compute(r, d);
    RganConv m = mangle(r, d);
    query_all(&m);
  }
  if (g_fail) {
    std::fprintf(stderr, "abi_fuzz: %d failures over %lld calls\n", g_fail, g_calls);
    return 1;
  }
  std::printf("abi_fuzz ok: %lld calls\n", g_calls);
  return 0;
}
