// Isolated timing of the library's kernels (admm_kernels.hip launchers) on random C3 data.
// build: see tools/kbench.sh ; run on the GPU box.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <random>
#include <vector>
#include <string>
#include <cmath>
#include <cstring>
#include <cstdint>
#include <algorithm>
#include "../admm-lstm_amd/admm_amd/csrc/admm_kernels.hpp"

using namespace admm;

static float* dev_random(size_t n, float lo, float hi, unsigned seed) {
  std::vector<float> h(n);
  std::mt19937 rng(seed);
  std::uniform_real_distribution<float> u(lo, hi);
  for (auto& v : h) v = u(rng);
  float* d;
  (void)hipMalloc(&d, n * 4);
  (void)hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice);
  return d;
}

#ifdef SR_TIMING
extern "C" void sr_timing_dump(int nblk);
#endif
#ifdef SR_CS_TIMING
extern "C" void cs_timing_dump(int T);
#endif
static void timeit(const char* name, double bytes, double flops, const std::function<void()>& f) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) f();
  (void)hipDeviceSynchronize();
  const int R = 10;
  (void)hipEventRecord(a);
  for (int i = 0; i < R; ++i) f();
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms; (void)hipEventElapsedTime(&ms, a, b);
  ms /= R;
  printf("%-22s %8.3f ms  %7.0f GB/s  %6.1f TF/s\n", name, ms, bytes / ms / 1e6, flops / ms / 1e9);
}

int main(int argc, char** argv) {
  Geom g{8192, 8192, 32, 16, 256, 1};
  if (argc > 3) g.T = atoi(argv[3]);
  if (argc > 4) g.D = atoi(argv[4]);
  if (argc > 5) g.H = atoi(argv[5]);
  g.set_T();
  if (argc > 1) g.B = g.Bg = atoll(argv[1]);
  const int64_t BT = g.BT(), n = BT * g.H, P = g.B * (int64_t)g.TP() * g.H;
  Hyper hp{};
  for (int i = 0; i < 7; ++i) hp.rho[i] = 1.f;
  hp.rho[4] = 0.008f; hp.rho[5] = 0.00045f; hp.rho[6] = 5.62e-5f;
  float* x = dev_random(BT * g.D, 0, 1, 1);
  float* zc = dev_random(4 * n, -2, 2, 2);
  float* tgt = dev_random(4 * n, 0, 1, 3);
  float* Q = dev_random(4 * n, -1e-4f, 1e-4f, 4);
  float* R = dev_random(4 * n, -1e-3f, 1e-3f, 5);
  Planes6 S, L;
  for (int q = 0; q < 6; ++q) { S.p[q] = dev_random(P, 0, 1, 10 + q); L.p[q] = dev_random(P, -1e-3f, 1e-3f, 20 + q); }
  float* W[8];
  for (int i = 0; i < 8; ++i) W[i] = dev_random(i < 4 ? g.D * g.H : g.H * g.H, -0.1f, 0.1f, 30 + i);
  Weights w;
  for (int q = 0; q < 4; ++q) { w.wx[q] = W[q]; w.wh[q] = W[4 + q]; }
  float* G = dev_random(4 * g.H * g.H, -1e-3f, 1e-3f, 40);
  float* dW = dev_random(4 * g.D * g.H, -1e-4f, 1e-4f, 41);
  float* slab; (void)hipMalloc(&slab, (size_t)256 * 4 * g.H * g.H * 4);
  double* part; (void)hipMalloc(&part, (size_t)4 * kTrialSlots * 4096 * 8);
  int* found; (void)hipMalloc(&found, 16); (void)hipMemset(found, 0, 16);
  hipStream_t s = 0;
  const double f4 = 4.0;
  const int nb = getenv("KB_NB") ? atoi(getenv("KB_NB")) : stream_blocks(g);   // trial grid override (A/B)
  auto run_s3 = [&] {
  if (split3_ok(g)) {
    // split-bf16 h-stage GEMMs: timing, and agreement with the f32-MFMA kernels above
    const int ns3 = atr3_splits(g);
    float* slab3; (void)hipMalloc(&slab3, (size_t)ns3 * 4 * g.H * g.H * 4);
    float* gimg; (void)hipMalloc(&gimg, split3_gimg_floats(g) * 4);
    float* Q3; (void)hipMalloc(&Q3, (size_t)4 * n * 4);
    timeit("atr3 (split bf16)", f4 * (2 * 4 * n + BT * g.H), 2.0 * BT * g.H * 4 * g.H,
           [&] { launch_atr3(g, S.p[5], zc, tgt, slab3, ns3, s); });
    timeit("qgemm3 (split bf16)", f4 * (4 * n + BT * g.H), 2.0 * BT * g.H * 4 * g.H,
           [&] { launch_qgemm3(g, S.p[5], G, gimg, Q3, s); });
    launch_atr_fused(g, hp, x, S.p[5], zc, tgt, dW, slab, atr_splits(g, 1), s);
    launch_qgemm(g, 1, x, S.p[5], G, Q, s);
    (void)hipDeviceSynchronize();
    const size_t gh = (size_t)4 * g.H * g.H;
    const int ns = atr_splits(g, 1);
    std::vector<float> a(ns * gh), b(ns3 * gh);
    (void)hipMemcpy(a.data(), slab, a.size() * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(b.data(), slab3, b.size() * 4, hipMemcpyDeviceToHost);
    double md = 0, mx = 0;
    for (size_t i = 0; i < gh; ++i) {
      double sa = 0, sb = 0;
      for (int k = 0; k < ns; ++k) sa += a[k * gh + i];
      for (int k = 0; k < ns3; ++k) sb += b[k * gh + i];
      md = std::max(md, std::fabs(sa - sb)); mx = std::max(mx, std::fabs(sa));
    }
    printf("atr3 vs atr_fused: max |diff| %.3e (max |G| %.3e, rel %.2e)\n", md, mx, md / mx);
    std::vector<float> qa(4 * n), qb(4 * n);
    (void)hipMemcpy(qa.data(), Q, qa.size() * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(qb.data(), Q3, qb.size() * 4, hipMemcpyDeviceToHost);
    md = 0; mx = 0;
    for (size_t i = 0; i < qa.size(); ++i) { md = std::max(md, (double)std::fabs(qa[i] - qb[i])); mx = std::max(mx, (double)std::fabs(qa[i])); }
    printf("qgemm3 vs qgemm: max |diff| %.3e (max |Q| %.3e, rel %.2e)\n", md, mx, md / mx);
  }
  };
  const std::string mode = argc > 2 ? argv[2] : "";
  if (mode == "s3") { run_s3(); return 0; }
  if (mode == "sel") {   // k_select of pass 0 (single process: it reduces the trial partials itself)
    DevStats* st; (void)hipMalloc(&st, sizeof(DevStats)); (void)hipMemset(st, 0, sizeof(DevStats));
    int* fl; (void)hipMalloc(&fl, 64); (void)hipMemset(fl, 0, 64);
    int* pick; (void)hipMalloc(&pick, 16);
    double* poly; (void)hipMalloc(&poly, 4 * kPolyN * 8);
    for (int side = 0; side < 2; ++side) {
      const int nred = side == 0 ? nb * (g.H / 128) : nb * (g.H / 256);
      (void)hipMemset(part, 0, (size_t)4 * kTrialSlots * nred * 8);
      SelectArgs sa{};
      sa.side = side; sa.pass = 0; sa.last_pass = kMaxPasses - 1;
      sa.part = part; sa.nred = nred; sa.poly = poly;
      sa.G = G;
      for (int q = 0; q < 4; ++q) sa.W[q] = W[side * 4 + q];
      sa.dW = side == 0 ? dW : nullptr;
      sa.found_in = fl; sa.found_out = fl + 4; sa.pick = pick; sa.stats = st;
      if (!getenv("KB_NOWT")) {   // as in the step: the selection also writes the sweep's weight image
        static float* wt = nullptr;
        if (!wt) (void)hipMalloc(&wt, sweep_wt_floats(g) * 4);
        sa.wt = wt; sa.wt_rows16 = sweep_wt_rows16(g); sa.wt_xc = sweep_wt_xc(g);
      }
      char nm[64]; snprintf(nm, sizeof nm, "select side %d (nred %d)", side, nred);
      for (int r = 0; r < 3; ++r) timeit(nm, 0, 0, [&] { launch_select(g, hp, sa, s); });
    }
    return 0;
  }
  if (mode == "trg") {   // gate imbalance: only gate 2 (g, tanh) in the per-candidate regime, as in the step
    const size_t ng = (size_t)g.D * g.H;
    std::vector<float> gh(4 * ng);
    (void)hipMemcpy(gh.data(), G, gh.size() * 4, hipMemcpyDeviceToHost);
    float* Gbig; (void)hipMalloc(&Gbig, gh.size() * 4);
    float* Gmix; (void)hipMalloc(&Gmix, gh.size() * 4);
    std::vector<float> gb(gh), gm(gh);
    for (auto& v : gb) v *= 100.f;                                    // |q| = |x G| ~ 0.5: per-candidate
    for (size_t i = 2 * ng; i < 3 * ng; ++i) gm[i] *= 100.f;          // gate 2 only
    (void)hipMemcpy(Gbig, gb.data(), gb.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(Gmix, gm.data(), gm.size() * 4, hipMemcpyHostToDevice);
    float* Qb = dev_random(4 * n, -1.f, 1.f, 7);
    float* Qmix = dev_random(4 * n, -1e-4f, 1e-4f, 4);
    (void)hipMemcpy(Qmix + 2 * n, Qb + 2 * n, n * 4, hipMemcpyDeviceToDevice);
    // the step's grids (KB_NB0 / KB_NB1: overrides for a scan)
    const int nb0 = getenv("KB_NB0") ? atoi(getenv("KB_NB0")) : trial_fast_blocks(g, 0);
    const int nb1 = getenv("KB_NB1") ? atoi(getenv("KB_NB1")) : trial_fast_blocks(g, 1);
    printf("trial grids: x %d, h %d workgroups per gate and column block\n", nb0, nb1);
    for (int r = 0; r < 3; ++r) {
      timeit("x trials, all poly", f4 * 2 * 4 * n, 0, [&] { launch_trial_fast(g, 0, 0, zc, tgt, nullptr, x, G, found, part, nb0, s); });
      timeit("x trials, g direct", f4 * 2 * 4 * n, 0, [&] { launch_trial_fast(g, 0, 0, zc, tgt, nullptr, x, Gmix, found, part, nb0, s); });
      timeit("x trials, all direct", f4 * 2 * 4 * n, 0, [&] { launch_trial_fast(g, 0, 0, zc, tgt, nullptr, x, Gbig, found, part, nb0, s); });
      timeit("h trials, all poly", f4 * 3 * 4 * n, 0, [&] { launch_trial_fast(g, 1, 0, zc, tgt, Q, x, dW, found, part, nb1, s, nullptr, 0); });
      timeit("h trials, g direct", f4 * 3 * 4 * n, 0, [&] { launch_trial_fast(g, 1, 0, zc, tgt, Qmix, x, dW, found, part, nb1, s, nullptr, 0); });
      timeit("h trials, all direct", f4 * 3 * 4 * n, 0, [&] { launch_trial_fast(g, 1, 0, zc, tgt, Qb, x, dW, found, part, nb1, s, nullptr, 0); });
    }
    return 0;
  }
  if (mode == "tr") {   // the two pass-0 trial kernels alone
    for (int r = 0; r < 3; ++r) {
      timeit("trial_fast side0", f4 * 2 * 4 * n, 0, [&] { launch_trial_fast(g, 0, 0, zc, tgt, nullptr, x, G, found, part, nb, s); });
      timeit("trial_fast side1", f4 * 3 * 4 * n, 0, [&] { launch_trial_fast(g, 1, 0, zc, tgt, Q, x, dW, found, part, nb, s); });
    }
    return 0;
  }
  if (mode == "q") {   // Q = Hprev G (k_qgemm_res at H = 256, else k_qgemm3<1>)
    float* gimg; (void)hipMalloc(&gimg, split3_gimg_floats(g) * 4);
    float* Q3; (void)hipMalloc(&Q3, (size_t)4 * n * 4);
    const double qb = f4 * BT * g.H + 2.0 * 4 * n, qf = 2.0 * 2 * BT * g.H * 4 * g.H;
    for (int r = 0; r < 3; ++r) timeit("qgemm3", qb, qf, [&] { launch_qgemm3(g, S.p[5], G, gimg, Q3, s); });
    return 0;
  }
  timeit("apply_dwx", 2 * f4 * 4 * n + f4 * BT * g.D, 0, [&] { launch_apply_dwx(g, x, dW, zc, s); });
  timeit("trial_fast side0", f4 * 2 * 4 * n, 0, [&] { launch_trial_fast(g, 0, 0, zc, tgt, nullptr, x, G, found, part, nb, s); });
  timeit("trial_fast side1", f4 * 3 * 4 * n, 0, [&] { launch_trial_fast(g, 1, 0, zc, tgt, Q, x, dW, found, part, nb, s); });
  {
    float* G0; (void)hipMalloc(&G0, 4 * g.H * g.H * 4); (void)hipMemset(G0, 0, 4 * g.H * g.H * 4);
    timeit("trial_fast side0 q=0", f4 * 2 * 4 * n, 0, [&] { launch_trial_fast(g, 0, 0, zc, tgt, nullptr, x, G0, found, part, nb, s); });
    float* Qb = dev_random(4 * n, -1.f, 1.f, 7);
    timeit("trial_fast side1 |q|<1", f4 * 3 * 4 * n, 0, [&] { launch_trial_fast(g, 1, 0, zc, tgt, Qb, x, dW, found, part, nb, s); });
    float* Qm = dev_random(4 * n, -0.01f, 0.01f, 8);
    timeit("trial_fast side1 |q|<.01", f4 * 3 * 4 * n, 0, [&] { launch_trial_fast(g, 1, 0, zc, tgt, Qm, x, dW, found, part, nb, s); });
    (void)hipFree(Qb); (void)hipFree(Qm); (void)hipFree(G0);
  }
  if (mode == "tr") return 0;
  timeit("trial generic", f4 * 3 * 4 * n, 0, [&] { launch_trial(g, 0, zc, tgt, Q, found, part, trial_blocks(g), s); });
  timeit("resid_gx", f4 * 4 * 4 * n, 0, [&] { launch_resid_gx(g, hp, x, S, L, zc, tgt, slab, resid_gx_blocks(g), false, s); });
  const int ns = atr_splits(g, 1);
  timeit("atr_fused", f4 * (2 * 4 * n + BT * g.H), 2.0 * BT * g.H * 4 * g.H,
         [&] { launch_atr_fused(g, hp, x, S.p[5], zc, tgt, dW, slab, ns, s); });
  timeit("atr (R materialised)", f4 * (4 * n + BT * g.H), 2.0 * BT * g.H * 4 * g.H,
         [&] { launch_atr(g, 1, x, S.p[5], R, slab, ns, s); });
  timeit("qgemm side1", f4 * (4 * n + BT * g.H), 2.0 * BT * g.H * 4 * g.H, [&] { launch_qgemm(g, 1, x, S.p[5], G, Q, s); });
  run_s3();
  SweepT sw{};
  sw.x = x; sw.S = S; sw.L = L; sw.zc = zc; sw.r0 = 0; sw.r1 = g.B;
  if (getenv("KB_GX")) {   // as in the step: the next x stage's targets, G_x partials and operand ranges
    sw.tgt = tgt;
    sw.gx_slab = slab;
    float* rg; (void)hipMalloc(&rg, 64); (void)hipMemset(rg, 0, 64);
    if (!getenv("KB_NORANGE")) sw.range = rg;
    if (getenv("KB_NOTGT")) { sw.tgt = nullptr; sw.gx_slab = nullptr; }
    if (getenv("KB_NOGXF")) sw.gx_slab = nullptr;   // tgt planes without the G_x fold
  }
  timeit("sweep_t (t=5)", f4 * g.B * (g.D + 27.0 * g.H), 2.0 * g.B * (g.D + g.H) * 4 * g.H,
         [&] { launch_sweep_t(g, 5, w, hp, sw, s); });
  {
    hipStream_t s2;
    hipEvent_t ef, ej;
    (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
    (void)hipEventCreateWithFlags(&ef, hipEventDisableTiming);
    (void)hipEventCreateWithFlags(&ej, hipEventDisableTiming);
    const double sb = f4 * g.T * g.B * (g.D + 27.0 * g.H), sf = 2.0 * g.T * g.B * (g.D + g.H) * 4 * g.H;
    timeit("sweep T steps, 1 stream", sb, sf, [&] {
      for (int t = 1; t <= g.T; ++t) launch_sweep_t(g, t, w, hp, sw, s);
    });
    if (sweep_rows_ok(g)) {
      float* wt; (void)hipMalloc(&wt, sweep_wt_floats(g) * 4);
      timeit("sweep_wt", 0, 0, [&] { launch_sweep_wt(g, w, wt, s); });
      timeit("sweep rows (1 launch)", sb, sf, [&] { launch_sweep_rows(g, wt, hp, sw, s); });
      if (sweep_rows_nc(g) > 1) {   // the column-split sweep (counters zeroed by sweep_wt each time)
        void* xc; (void)hipMalloc(&xc, sweep_xbuf_bytes(g));
        int* fl; (void)hipMalloc(&fl, 4); (void)hipMemset(fl, 0, 4);
        SweepT sc = sw;
        sc.xbuf = xc;
        sc.fail = fl;
        timeit("sweep column split", sb, sf, [&] { launch_sweep_wt(g, w, wt, s, xc); launch_sweep_rows(g, wt, hp, sc, s); });
        int f = 0; (void)hipMemcpy(&f, fl, 4, hipMemcpyDeviceToHost);
        printf("column split: nc %d, hand-off timeouts %d\n", sweep_rows_nc(g), f);
#ifdef SR_CS_TIMING
        cs_timing_dump(g.T);
#endif
      }
#ifdef SR_TIMING
      (void)hipDeviceSynchronize();
      sr_timing_dump((int)((g.B + 31) / 32));
#endif
    }
    timeit("sweep T steps, 2 streams", sb, sf, [&] {
      const int64_t mid = (g.B / 2 + 127) / 128 * 128;
      (void)hipEventRecord(ef, s);
      (void)hipStreamWaitEvent(s2, ef, 0);
      SweepT a1 = sw, a2 = sw;
      a1.r1 = mid; a2.r0 = mid;
      for (int t = 1; t <= g.T; ++t) {
        launch_sweep_t(g, t, w, hp, a1, s);
        launch_sweep_t(g, t, w, hp, a2, s2);
      }
      (void)hipEventRecord(ej, s2);
      (void)hipStreamWaitEvent(s, ej, 0);
    });
  }
  timeit("zgemm", f4 * (4 * n + BT * (g.D + g.H)), 2.0 * BT * (g.D + g.H) * 4 * g.H, [&] { launch_zgemm(g, w, x, S.p[5], zc, s); });
  return 0;
}
