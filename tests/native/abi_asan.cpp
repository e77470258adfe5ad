// Host AddressSanitizer check of the C ABI (include/admm_lstm.h) -- SURVEY.md section 5,
// "race detection / sanitizers": the library's host code (admm_host.hip: argument validation,
// create / bind / destroy, the step's launch sequence, the debug hooks) is built with
// -Xarch_host -fsanitize=address into libadmmlstm_asan.so (csrc/Makefile target `asan`); the GPU
// code is the product build's.  This driver exercises every entry point.
//
//   abi_asan args   -- argument / state validation only (no device needed; runs on CPU hosts)
//   abi_asan gpu    -- also full contexts on device 0: create, bind, init_state, several steps on
//                      the generic and the fast (persistent-sweep, split3, MFMA-trial) paths, stats,
//                      poll, profile, debug hooks, invalidate, forward, destroy
//
// Exit status 0 = every check passed and ASan reported nothing (ASan aborts on its first error).
#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include <sanitizer/lsan_interface.h>

#include "admm_lstm.h"

static int g_fail = 0;
#define CHECK(cond)                                                                   \
  do {                                                                                \
    if (!(cond)) {                                                                    \
      std::fprintf(stderr, "CHECK failed %s:%d: %s (last error: %s)\n", __FILE__,     \
                   __LINE__, #cond, admm_last_error());                               \
      ++g_fail;                                                                       \
    }                                                                                 \
  } while (0)

static AdmmParams google_params(int variant) {   // parameters.py 'GoogleStock'
  AdmmParams p{};
  const float rho[7] = {1.f, 1.f, 1.f, 1.f, 0.008f, 0.00045f, 0.0000562f};
  for (int i = 0; i < 7; ++i) p.rho[i] = rho[i];
  for (int q = 0; q < 4; ++q) p.beta_x[q] = p.beta_h[q] = 8e-7f;
  p.beta_y = 8e-7f;
  p.variant = variant;
  p.with_dual_y = 0;
  return p;
}

// argument and state validation: every call returns its error code and sets a message
static void check_args() {
  CHECK(admm_abi_version() == ADMM_LSTM_ABI_VERSION);
  CHECK(admm_build_info() != nullptr && std::strlen(admm_build_info()) > 0);
  AdmmDims d{64, 64, 4, 3, 32, 2};
  AdmmParams p = google_params(ADMM_VARIANT_ADMM);
  AdmmCtx* ctx = reinterpret_cast<AdmmCtx*>(0x1);
  CHECK(admm_create(&d, &p, 0, nullptr) == ADMM_EINVAL);
  CHECK(admm_create(nullptr, &p, 0, &ctx) == ADMM_EINVAL && ctx == nullptr);
  CHECK(std::strlen(admm_last_error()) > 0);
  CHECK(admm_create(&d, nullptr, 0, &ctx) == ADMM_EINVAL);
  AdmmDims bad = d;
  bad.batch = 0;
  CHECK(admm_create(&bad, &p, 0, &ctx) == ADMM_EINVAL);
  bad = d;
  bad.hidden_size = -4;
  CHECK(admm_create(&bad, &p, 0, &ctx) == ADMM_EINVAL);
  bad = d;
  bad.global_batch = 10;   // < batch
  CHECK(admm_create(&bad, &p, 0, &ctx) == ADMM_EINVAL);
  bad = d;
  bad.output_size = 1 << 20;
  CHECK(admm_create(&bad, &p, 0, &ctx) == ADMM_EINVAL);
  bad = d;
  bad.batch = bad.global_batch = 1ll << 26;
  bad.seq_len = 64;        // B T >= 2^31 rows
  CHECK(admm_create(&bad, &p, 0, &ctx) == ADMM_EINVAL);
  AdmmParams bp = p;
  bp.variant = 7;
  CHECK(admm_create(&d, &bp, 0, &ctx) == ADMM_EINVAL);
  bp = p;
  bp.rho[3] = NAN;
  CHECK(admm_create(&d, &bp, 0, &ctx) == ADMM_EINVAL);
  CHECK(std::strstr(admm_last_error(), "rho") != nullptr);
  // NULL contexts
  CHECK(admm_destroy(nullptr) == ADMM_OK);
  CHECK(admm_bind(nullptr, nullptr) == ADMM_EINVAL);
  CHECK(admm_init_state(nullptr, nullptr) == ADMM_EINVAL);
  CHECK(admm_step(nullptr, nullptr) == ADMM_EINVAL);
  CHECK(admm_set_with_dual_y(nullptr, 1) == ADMM_EINVAL);
  CHECK(admm_invalidate_cache(nullptr) == ADMM_EINVAL);
  CHECK(admm_ack_fault(nullptr) == ADMM_EINVAL);
  AdmmStats st;
  CHECK(admm_get_stats(nullptr, &st) != ADMM_OK);
  int32_t u = 0, nf = 0;
  CHECK(admm_poll_status(nullptr, &u, &nf) != ADMM_OK);
  CHECK(admm_poll_faults(nullptr, &u, &nf) == ADMM_EINVAL);     // ABI 2
  CHECK(admm_debug_fault(nullptr, 1) == ADMM_EINVAL);
  CHECK(admm_profile(nullptr, 1) != ADMM_OK);
  CHECK(admm_set_comm(nullptr, nullptr, 0, 0, 1) == ADMM_EINVAL);
  CHECK(admm_set_comm_host(nullptr, nullptr, nullptr, 0, 1) != ADMM_OK);
  char small[4];
  CHECK(admm_comm_unique_id(small, sizeof small) == ADMM_EINVAL);
  CHECK(admm_comm_unique_id(nullptr, 1024) == ADMM_EINVAL);
  CHECK(admm_debug_trace(nullptr, nullptr, nullptr) != ADMM_OK);
  CHECK(admm_debug_force(nullptr, nullptr, 0) != ADMM_OK);
  CHECK(admm_debug_trace_resid(nullptr, nullptr, nullptr) != ADMM_OK);
  CHECK(admm_debug_own(nullptr, nullptr, nullptr) != ADMM_OK);
  CHECK(admm_debug_workspace(nullptr, 0, nullptr, 0, nullptr) < 0);
  const float* w4[4] = {nullptr, nullptr, nullptr, nullptr};
  float* g6[6] = {};
  CHECK(admm_forward(nullptr, 0, 1, 1, 1, 1, w4, w4, nullptr, g6, nullptr, nullptr, nullptr, nullptr, nullptr) ==
        ADMM_EINVAL);
}

// deterministic host data (a small LCG), uploaded as the caller's tensors
struct Lcg {
  uint32_t s;
  float next() {
    s = s * 1664525u + 1013904223u;
    return (float)(s >> 8) * (1.f / 16777216.f);
  }
};

static float* upload(const std::vector<float>& h) {
  float* d = nullptr;
  if (hipMalloc(&d, h.size() * sizeof(float)) != hipSuccess) return nullptr;
  if (hipMemcpy(d, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess) return nullptr;
  return d;
}

static float* zeros(size_t n) {
  float* d = nullptr;
  if (hipMalloc(&d, n * sizeof(float)) != hipSuccess) return nullptr;
  if (hipMemset(d, 0, n * sizeof(float)) != hipSuccess) return nullptr;
  return d;
}

// one context through its whole life on device 0
static void run_context(int64_t B, int T, int D, int H, int O, int variant, int steps) {
  static const auto t_start = std::chrono::steady_clock::now();
  std::fprintf(stderr, "context B=%lld T=%d D=%d H=%d O=%d variant=%d (%.1f s)\n", (long long)B, T, D, H, O, variant,
               std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count());
  Lcg r{(uint32_t)(B * 131 + H)};
  std::vector<float> hx(B * T * D), hy(B * O);
  for (auto& v : hx) v = r.next();
  for (auto& v : hy) v = r.next();
  const float sc = 1.f / std::sqrt((float)H);
  AdmmBuffers b{};
  std::vector<float*> owned;
  auto keep = [&](float* p) { owned.push_back(p); return p; };
  b.x = keep(upload(hx));
  b.y = keep(upload(hy));
  for (int q = 0; q < 4; ++q) {
    std::vector<float> wx(D * H), wh(H * H);
    for (auto& v : wx) v = (2.f * r.next() - 1.f) * sc;
    for (auto& v : wh) v = (2.f * r.next() - 1.f) * sc;
    b.wx[q] = keep(upload(wx));
    b.wh[q] = keep(upload(wh));
  }
  std::vector<float> wy(H * O);
  for (auto& v : wy) v = (2.f * r.next() - 1.f) * sc;
  b.wy = keep(upload(wy));
  const size_t plane = (size_t)B * (T + 1) * H;
  for (int q = 0; q < 6; ++q) {
    b.gates[q] = keep(zeros(plane));
    b.duals[q] = keep(zeros(plane));
  }
  b.a = keep(zeros(B * O));
  b.dual_y = keep(zeros(B * O));
  for (float* p : owned) CHECK(p != nullptr);

  AdmmDims d{B, B, T, D, H, O};
  AdmmParams p = google_params(variant);
  AdmmCtx* ctx = nullptr;
  CHECK(admm_create(&d, &p, 0, &ctx) == ADMM_OK && ctx != nullptr);
  if (!ctx) return;
  // state errors before bind
  CHECK(admm_step(ctx, nullptr) == ADMM_ESTATE);
  CHECK(admm_init_state(ctx, nullptr) == ADMM_ESTATE);
  AdmmBuffers nb = b;
  nb.wh[2] = nullptr;
  CHECK(admm_bind(ctx, &nb) == ADMM_EINVAL);
  nb = b;
  nb.duals[5] = nullptr;
  CHECK(admm_bind(ctx, &nb) == ADMM_EINVAL);
  CHECK(admm_bind(ctx, &b) == ADMM_OK);
  CHECK(admm_init_state(ctx, nullptr) == ADMM_OK);
  CHECK(admm_set_with_dual_y(ctx, variant == ADMM_VARIANT_ADMM ? 1 : 0) == ADMM_OK);
  // the debug hooks with caller buffers, then off again
  float *gx = zeros((size_t)4 * D * H), *gh = zeros((size_t)4 * H * H);
  CHECK(admm_debug_trace(ctx, gx, gh) == ADMM_OK);
  float *rx = zeros((size_t)4 * B * T * H), *rh = zeros((size_t)4 * B * T * H);
  CHECK(admm_debug_trace_resid(ctx, rx, rh) == ADMM_OK);
  auto finite_dev = [&](const float* dptr, size_t n) {
    std::vector<float> h(n);
    if (hipMemcpy(h.data(), dptr, n * 4, hipMemcpyDeviceToHost) != hipSuccess) return false;
    for (float v : h)
      if (!std::isfinite(v)) return false;
    return true;
  };
  auto weights_finite = [&]() {
    bool ok = finite_dev(b.wy, (size_t)H * O) && finite_dev(b.a, (size_t)B * O);
    for (int q = 0; q < 4; ++q) ok = ok && finite_dev(b.wx[q], (size_t)D * H) && finite_dev(b.wh[q], (size_t)H * H);
    return ok;
  };
  for (int s = 0; s < steps; ++s) {
    if (s == 1) CHECK(admm_profile(ctx, (1u << ADMM_PROF_CLASSES) - 1) == ADMM_OK);
    CHECK(admm_step(ctx, nullptr) == ADMM_OK);
    AdmmStats ss{};
    CHECK(admm_get_stats(ctx, &ss) == ADMM_OK);
    std::fprintf(stderr, "  step %d k = %d %d %d %d %d %d %d %d theta_h %g\n", s + 1, ss.k[0], ss.k[1], ss.k[2], ss.k[3],
                 ss.k[4], ss.k[5], ss.k[6], ss.k[7], ss.theta_h);
    CHECK(weights_finite());
    if (s == 1) {
      double ms[ADMM_PROF_CLASSES];
      int32_t cnt[ADMM_PROF_CLASSES];
      CHECK(admm_profile_read(ctx, ms, cnt) == ADMM_OK);
      CHECK(admm_profile(ctx, 0) == ADMM_OK);
    }
    if (s == 2) CHECK(admm_invalidate_cache(ctx) == ADMM_OK);   // next step rebuilds the caches
  }
  CHECK(admm_debug_trace(ctx, nullptr, nullptr) == ADMM_OK);
  CHECK(admm_debug_trace_resid(ctx, nullptr, nullptr) == ADMM_OK);
  // replay: force the exponents the last step took (forcing arbitrary small ones can overflow
  // the weights), and one doubling more for the h_T search
  AdmmStats prev{};
  CHECK(admm_get_stats(ctx, &prev) == ADMM_OK);
  int32_t k8[8];
  for (int i = 0; i < 8; ++i) k8[i] = prev.k[i];
  CHECK(admm_debug_force(ctx, k8, 1) == ADMM_OK);
  CHECK(admm_step(ctx, nullptr) == ADMM_OK);
  CHECK(weights_finite());
  int32_t own[8];
  float th = 0.f;
  CHECK(admm_debug_own(ctx, own, &th) == ADMM_OK);
  CHECK(admm_debug_force(ctx, nullptr, 0) == ADMM_OK);
  AdmmStats st{};
  CHECK(admm_get_stats(ctx, &st) == ADMM_OK);
  CHECK(st.steps == steps + 1);
  for (int i = 0; i < 8; ++i) CHECK(st.k[i] == k8[i]);   // the forced exponents were applied
  CHECK(st.unresolved == 0 && st.nonfinite == 0);
  int32_t unres = -1, nonfin = -1;
  CHECK(admm_poll_status(ctx, &unres, &nonfin) == ADMM_OK);
  int32_t hf = -1, fb = -1;   // ABI 2: fault counts (no column split fault in a healthy run)
  CHECK(admm_poll_faults(ctx, &hf, &fb) == ADMM_OK && hf == 0);
  CHECK(admm_poll_faults(ctx, nullptr, &fb) == ADMM_EINVAL);
  CHECK(st.handoff_fail == 0 && st.graph_disabled == 0);
  CHECK(admm_debug_fault(ctx, 0) == ADMM_OK);
  CHECK(admm_ack_fault(ctx) == ADMM_OK);   // nothing to acknowledge: invalidates the caches only
  CHECK(admm_debug_fault(ctx, 7) == ADMM_EINVAL);
  // z cache copy-out: too small a destination is refused, the right size is accepted
  const int64_t zbytes = (int64_t)4 * B * T * H * 4;
  float* zc = zeros((size_t)4 * B * T * H);
  CHECK(admm_debug_workspace(ctx, 0, zc, zbytes - 4, nullptr) < 0);
  CHECK(admm_debug_workspace(ctx, 0, zc, zbytes, nullptr) >= 0);
  CHECK(admm_debug_workspace(ctx, 9, zc, zbytes, nullptr) < 0);
  // the forward pass without a context, into scratch
  float *hs = zeros((size_t)2 * B * H), *cs = zeros((size_t)2 * B * H), *oa = zeros((size_t)B * O);
  const float* wxc[4] = {b.wx[0], b.wx[1], b.wx[2], b.wx[3]};
  const float* whc[4] = {b.wh[0], b.wh[1], b.wh[2], b.wh[3]};
  CHECK(admm_forward(b.x, B, T, D, H, O, wxc, whc, b.wy, nullptr, hs, cs, nullptr, oa, nullptr) == ADMM_OK);
  CHECK(hipDeviceSynchronize() == hipSuccess);
  CHECK(finite_dev(oa, (size_t)B * O));
  CHECK(admm_destroy(ctx) == ADMM_OK);
  for (float* q : {gx, gh, rx, rh, zc, hs, cs, oa}) (void)hipFree(q);
  for (float* q : owned) (void)hipFree(q);
}

int main(int argc, char** argv) {
  const bool gpu = argc > 1 && std::strcmp(argv[1], "gpu") == 0;
  check_args();
  if (gpu) {
    int n = 0;
    CHECK(hipGetDeviceCount(&n) == hipSuccess && n > 0);
    if (n > 0) {
      run_context(64, 4, 3, 32, 2, ADMM_VARIANT_ADMM, 4);           // generic kernels, per-t sweep
      run_context(100, 3, 5, 64, 1, ADMM_VARIANT_NO_DUAL_Y, 4);     // fast path, ragged persistent sweep
      run_context(512, 3, 16, 256, 1, ADMM_VARIANT_ADMM, 4);        // the C3 kernels (split3, MFMA trials)
      run_context(96, 2, 1, 512, 1, ADMM_VARIANT_NO_DUAL_Y, 3);     // the C5 kernels (16-row sweep)
      run_context(70, 2, 4, 40, 300, ADMM_VARIANT_ADMM, 3);         // wide output layer
    }
  }
  // leak check now, then leave without running the ROCm runtime's static destructors: at exit they
  // call back into ASan's device-allocator hooks after ASan has torn them down (an ASan-internal
  // CHECK in sanitizer_allocator_device.h, not an error of this program)
  __lsan_do_leak_check();
  std::printf("abi_asan %s: %s (%d failed checks)\n", gpu ? "gpu" : "args", g_fail ? "FAIL" : "ok", g_fail);
  std::fflush(stdout);
  std::fflush(stderr);
  std::_Exit(g_fail ? 1 : 0);
}
