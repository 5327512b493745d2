// GPU test program (not product): the device's supernodal factorisation
// and solve (solve_super.inc, compiled from the product source) on one
// workgroup, against the sparse KKT matrix -- the same random active set and
// values as tests/native/kkt_super_check.cpp (its CPU replay).  Reads the
// pattern and "seed fixed_frac inactive_frac delta" from stdin like that
// harness; prints JSON with the GPU solve's residual and its largest
// difference from the CPU replay's solution.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I mpi-sppy_amd/csrc \
//         tests/native/super_gpu_check.hip -o super_gpu_check
#include "phgpu.hip"

#include <cmath>
#include <cstdio>
#include <random>

namespace {
__global__ void __launch_bounds__(1024) super_check_kernel(const KsDev *sd, double *Lv, double *Dv, double *Uw, double *Vw,
                                                           double *rv, int N, double delta, unsigned long long *t0,
                                                           int solve) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  if (threadIdx.x == 0 && t0) *t0 = wall_clock64();
  super_factor(sd, Lv, Dv, Uw, lds, delta);
  if (solve) super_solve(sd, Lv, Dv, Vw, rv, lds, N);
}

template <class T>
T *up(const std::vector<T> &v) {
  T *d = nullptr;
  if (hipMalloc(&d, sizeof(T) * std::max<size_t>(1, v.size())) != hipSuccess) std::abort();
  if (!v.empty() && hipMemcpy(d, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice) != hipSuccess) std::abort();
  return d;
}
}  // namespace

int main() {
  int n, m, nnz;
  if (std::scanf("%d %d %d", &n, &m, &nnz) != 3) return 2;
  std::vector<int32_t> rp(m + 1), ci(nnz);
  for (auto &v : rp)
    if (std::scanf("%d", &v) != 1) return 2;
  for (auto &v : ci)
    if (std::scanf("%d", &v) != 1) return 2;
  unsigned seed = 1;
  double ffix = 0.2, finact = 0.3, delta = 1e-7;
  if (std::scanf("%u %lf %lf %lf", &seed, &ffix, &finact, &delta) != 4) return 2;
  KktSymbolic ks;
  if (!ks.analyze(n, m, rp.data(), ci.data(), false)) return 3;
  KktSuper sp;
  if (!sp.build(ks, rp.data(), ci.data())) {
    std::printf("{\"error\": \"%s\"}\n", sp.error);
    return 3;
  }
  const int N = sp.N;
  std::mt19937_64 rng(seed);
  std::uniform_real_distribution<double> U01(0.0, 1.0);
  std::vector<int> CC(n), RC(m);
  for (auto &c : CC) c = U01(rng) < ffix ? 1 : 0;
  for (auto &r : RC) r = U01(rng) < finact ? 0 : 1;
  std::vector<double> diag(N), aval(nnz);
  for (int j = 0; j < n; ++j) diag[j] = CC[j] ? 1.0 : (U01(rng) < 0.5 ? 0.0 : U01(rng)) + delta;
  for (int i = 0; i < m; ++i) diag[n + i] = RC[i] ? -delta : -1.0;
  for (int p = 0; p < nnz; ++p) aval[p] = 2.0 * U01(rng) - 1.0;
  std::vector<double> Lv(sp.panel_total, 0.0), Dv(N);
  for (int v = 0; v < N; ++v) Dv[sp.pos[v]] = diag[v];
  for (int i = 0; i < m; ++i)
    for (int p = rp[i]; p < rp[i + 1]; ++p)
      if (!CC[ci[p]] && RC[i]) Lv[sp.apos[p]] = -aval[p];
  std::vector<double> bv(N), rv(N);
  for (auto &x : bv) x = 2.0 * U01(rng) - 1.0;
  for (int v = 0; v < N; ++v) rv[sp.pos[v]] = bv[v];
  // device arrays (the packing of phgpu.hip super_setup)
  KsDev k{};
  k.on = 1;
  k.ns = sp.ns;
  k.nlev = sp.nlev;
  k.u_total = sp.u_total;
  k.v_total = sp.v_total;
  k.lds_base = (MAX_WAVES * 10 + 2 + 7) & ~7;
  k.pos = up(sp.pos);
  k.rec = (const int4 *)up(sp.rec);
  k.srow = up(sp.srow); k.rel = up(sp.rel); k.chl = up(sp.chl);
  k.lvi = up(sp.lvi); k.itg = up(sp.itg); k.itp = up(sp.itp); k.itsn = up(sp.itsn);
  k.lvr = up(sp.lvr); k.rdp = up(sp.rdp); k.rsn = up(sp.rsn); k.rlo = up(sp.rlo);
  k.lvb = up(sp.lvb); k.lbs = up(sp.lbs);
  unsigned long long *dprof = nullptr;
  if (hipMalloc(&dprof, sizeof(unsigned long long) * SUPER_PROF) != hipSuccess) return 4;
  (void)hipMemset(dprof, 0, sizeof(unsigned long long) * SUPER_PROF);
  unsigned long long *dt0 = nullptr;
  if (hipMalloc(&dt0, sizeof(unsigned long long)) != hipSuccess) return 4;
  double *dL = up(Lv), *dD = up(Dv), *dr = up(rv);
  double *dU = up(std::vector<double>(sp.u_total + 1, 0.0)), *dV = up(std::vector<double>(sp.v_total + 1, 0.0));
  const size_t lds = sizeof(double) * ((size_t)k.lds_base + SUPER_POOL);
  if (hipFuncSetAttribute((const void *)super_check_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) !=
      hipSuccess)
    return 4;
  KsDev *dk = nullptr;
  auto put_k = [&]() {
    if (!dk && hipMalloc(&dk, sizeof(KsDev)) != hipSuccess) std::abort();
    if (hipMemcpy(dk, &k, sizeof(KsDev), hipMemcpyHostToDevice) != hipSuccess) std::abort();
  };
  put_k();
  {  // the factor alone against the CPU replay (kkt_super_check.cpp's algorithm)
    hipLaunchKernelGGL(super_check_kernel, dim3(1), dim3(1024), lds, 0, dk, dL, dD, dU, dV, dr, N, delta,
                       (unsigned long long *)nullptr, 0);
    if (hipDeviceSynchronize() != hipSuccess) return 5;
    std::vector<double> gL(sp.panel_total), gD(N), gU(sp.u_total);
    if (hipMemcpy(gL.data(), dL, sizeof(double) * gL.size(), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(gD.data(), dD, sizeof(double) * N, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(gU.data(), dU, sizeof(double) * gU.size(), hipMemcpyDeviceToHost) != hipSuccess)
      return 6;
    std::vector<double> cL = Lv, cD = Dv, cU(sp.u_total, 0.0);
    std::vector<char> colv(N);
    for (int c = 0; c < N; ++c) colv[c] = cD[c] > 0.0;
    auto ucl = [](long r, long b) { return b * r - b * (b - 1) / 2; };
    int bad_t = -1;
    double bad_e = 0.0;
    const char *bad_what = "";
    for (int l = 0; l < sp.nlev && bad_t < 0; ++l)
      for (int qq = sp.lvp[l]; qq < sp.lvp[l + 1]; ++qq) {
        const int t = sp.lsn[qq];
        const int w = sp.sw[t], r = sp.sr[t], f = w + r, first = sp.sfirst[t];
        double *P = cL.data() + sp.poff[t];
        const int c0 = sp.chp[t], nch = sp.chp[t + 1] - c0;
        std::vector<int> tab((size_t)nch * f, -1);
        for (int q = 0; q < nch; ++q) {
          const int c = sp.chl[c0 + q];
          for (int o = sp.srp[c]; o < sp.srp[c + 1]; ++o) tab[(size_t)q * f + sp.rel[o]] = o - sp.srp[c];
        }
        auto child_sum = [&](int i, int kk) {
          double acc = 0.0;
          for (int q = 0; q < nch; ++q) {
            const int a = tab[(size_t)q * f + i], b = tab[(size_t)q * f + kk];
            if (a < 0 || b < 0) continue;
            const int c = sp.chl[c0 + q];
            acc += cU[sp.uoff[c] + ucl(sp.sr[c], b) + (a - b)];
          }
          return acc;
        };
        for (int kk = 0; kk < w; ++kk) {
          P[(size_t)kk * f + kk] = cD[first + kk] + child_sum(kk, kk);
          for (int i = kk + 1; i < f; ++i) P[(size_t)kk * f + i] += child_sum(i, kk);
        }
        for (int kk = 0; kk < w; ++kk) {
          double d = P[(size_t)kk * f + kk];
          d = colv[first + kk] ? std::fmax(d, delta) : std::fmin(d, -delta);
          cD[first + kk] = d;
          for (int i = kk + 1; i < f; ++i) P[(size_t)kk * f + i] /= d;
          for (int j = kk + 1; j < w; ++j) {
            const double ljd = P[(size_t)kk * f + j] * d;
            for (int i = j; i < f; ++i) P[(size_t)j * f + i] -= P[(size_t)kk * f + i] * ljd;
          }
        }
        double *Ut = cU.data() + sp.uoff[t];
        for (int b = 0; b < r; ++b)
          for (int a = b; a < r; ++a) {
            double acc = child_sum(w + a, w + b);
            for (int kk = 0; kk < w; ++kk)
              acc -= P[(size_t)kk * f + w + a] * cD[first + kk] * P[(size_t)kk * f + w + b];
            Ut[ucl(r, b) + (a - b)] = acc;
          }
        // compare this supernode
        auto rel_err = [](double x, double y) { return std::fabs(x - y) / std::fmax(1.0, std::fabs(y)); };
        for (int kk = 0; kk < w && bad_t < 0; ++kk) {
          if (rel_err(gD[first + kk], cD[first + kk]) > 1e-9) { bad_t = t; bad_e = rel_err(gD[first + kk], cD[first + kk]); bad_what = "D"; }
          for (int i = kk + 1; i < f && bad_t < 0; ++i)
            if (rel_err(gL[sp.poff[t] + (size_t)kk * f + i], P[(size_t)kk * f + i]) > 1e-9) {
              bad_t = t; bad_e = rel_err(gL[sp.poff[t] + (size_t)kk * f + i], P[(size_t)kk * f + i]); bad_what = "L";
            }
        }
        for (long e = 0; e < (long)r * (r + 1) / 2 && bad_t < 0; ++e)
          if (rel_err(gU[sp.uoff[t] + e], Ut[e]) > 1e-9) { bad_t = t; bad_e = rel_err(gU[sp.uoff[t] + e], Ut[e]); bad_what = "U"; }
        if (bad_t >= 0) {
          const bool sm = KktSuper::small_front(f, w);
          std::printf("{\"factor_mismatch\": {\"snode\": %d, \"level\": %d, \"what\": \"%s\", \"err\": %.3e, "
                      "\"w\": %d, \"r\": %d, \"nch\": %d, \"small\": %d}}\n", t, l, bad_what, bad_e, w, r, nch,
                      (int)sm);
          break;
        }
      }
    if (bad_t < 0) std::printf("{\"factor_match\": true}\n");
    if (hipMemcpy(dL, Lv.data(), sizeof(double) * Lv.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(dD, Dv.data(), sizeof(double) * N, hipMemcpyHostToDevice) != hipSuccess)
      return 6;
  }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  hipLaunchKernelGGL(super_check_kernel, dim3(1), dim3(1024), lds, 0, dk, dL, dD, dU, dV, dr, N, delta,
                     (unsigned long long *)nullptr, 1);
  (void)hipEventRecord(e1, 0);
  if (hipDeviceSynchronize() != hipSuccess) {
    std::printf("{\"error\": \"kernel failed\"}\n");
    return 5;
  }
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  // a second launch: the factor + solve time with warm caches
  if (hipMemcpy(dL, Lv.data(), sizeof(double) * Lv.size(), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(dD, Dv.data(), sizeof(double) * N, hipMemcpyHostToDevice) != hipSuccess)
    return 6;
  std::vector<double> out(N);
  if (hipMemcpy(out.data(), dr, sizeof(double) * N, hipMemcpyDeviceToHost) != hipSuccess) return 6;
  if (hipMemcpy(dr, rv.data(), sizeof(double) * N, hipMemcpyHostToDevice) != hipSuccess) return 6;
  (void)hipEventRecord(e0, 0);
  k.tprof = dprof;
  put_k();
  hipLaunchKernelGGL(super_check_kernel, dim3(1), dim3(1024), lds, 0, dk, dL, dD, dU, dV, dr, N, delta, dt0, 1);
  (void)hipEventRecord(e1, 0);
  if (hipDeviceSynchronize() != hipSuccess) return 5;
  std::vector<unsigned long long> tp(SUPER_PROF);
  unsigned long long t0h = 0;
  if (hipMemcpy(tp.data(), dprof, sizeof(unsigned long long) * SUPER_PROF, hipMemcpyDeviceToHost) != hipSuccess ||
      hipMemcpy(&t0h, dt0, sizeof(t0h), hipMemcpyDeviceToHost) != hipSuccess)
    return 6;
  float ms2 = 0.f;
  (void)hipEventElapsedTime(&ms2, e0, e1);
  std::vector<double> out2(N);
  if (hipMemcpy(out2.data(), dr, sizeof(double) * N, hipMemcpyDeviceToHost) != hipSuccess) return 6;
  double rerun = 0.0;
  for (int c = 0; c < N; ++c) rerun = std::fmax(rerun, std::fabs(out2[c] - out[c]));
  // residual against the sparse K (vertex order)
  std::vector<double> z(N), Kz(N, 0.0);
  for (int v = 0; v < N; ++v) z[v] = out[sp.pos[v]];
  for (int v = 0; v < N; ++v) Kz[v] = diag[v] * z[v];
  for (int i = 0; i < m; ++i)
    for (int p = rp[i]; p < rp[i + 1]; ++p) {
      const int j = ci[p];
      if (CC[j] || !RC[i]) continue;
      Kz[j] += -aval[p] * z[n + i];
      Kz[n + i] += -aval[p] * z[j];
    }
  double res = 0.0, zn = 0.0;
  int worst = -1;
  for (int v = 0; v < N; ++v) {
    const double e = std::fabs(Kz[v] - bv[v]);
    if (!(e <= res)) {
      res = e;
      worst = v;
    }
    zn = std::fmax(zn, std::fabs(z[v]));
  }
  // phase clocks (100 MHz wall clock): factor per level (small, big), solve per level
  std::printf("{\"factor_us\": [");
  unsigned long long prev = t0h;
  for (int l = 0; l < sp.nlev; ++l) {
    std::printf("%s[%.1f, %.1f]", l ? ", " : "", (tp[2 * l] - prev) / 100.0, (tp[2 * l + 1] - tp[2 * l]) / 100.0);
    prev = tp[2 * l + 1];
  }
  std::printf("], \"forward_us\": [");
  for (int l = 0; l < sp.nlev; ++l) {
    std::printf("%s%.1f", l ? ", " : "", (tp[128 + l] - prev) / 100.0);
    prev = tp[128 + l];
  }
  std::printf("], \"backward_us\": [");
  for (int l = sp.nlev - 1; l >= 0; --l) {
    std::printf("%s%.1f", l < sp.nlev - 1 ? ", " : "", (tp[192 + l] - prev) / 100.0);
    prev = tp[192 + l];
  }
  std::printf("], \"big_phase_us\": [");
  for (int q = 0; q < 7; ++q) std::printf("%s%.1f", q ? ", " : "", q < 6 ? tp[64 + q] / 100.0 : (double)tp[64 + q]);
  std::printf("]}\n");
  std::printf("{\"N\": %d, \"ns\": %d, \"nlev\": %d, \"residual\": %.3e, \"znorm\": %.3e, \"worst_vertex\": %d, "
              "\"worst_snode\": %d, \"rerun_diff\": %.3e, \"ms_first\": %.3f, \"ms\": %.3f}\n",
              N, sp.ns, sp.nlev, res, zn, worst, worst >= 0 ? sp.snode[sp.pos[worst]] : -1, rerun, ms, ms2);
  return 0;
}
