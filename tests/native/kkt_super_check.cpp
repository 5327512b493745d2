// Test harness (not product): the supernodal symbolic analysis of
// mpi-sppy_amd/csrc/kkt_super.h on a pattern read from stdin ("n m nnz",
// row_ptr, col_idx, then "seed fixed_frac inactive_frac delta"), and a CPU replay
// of the device's multifrontal factorisation and solve (the gather form of
// solve_big.inc's super_factor / super_solve: each front gathers its
// children's update matrices / vectors through the parents' front
// positions, level by level) on a random quasi-definite KKT matrix of an
// active set.  Prints JSON: the symbolic's sizes and checks, and the
// relative residual of K z = b against the sparse K.
#include "kkt_super.h"

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

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
  if (!ks.analyze(n, m, rp.data(), ci.data(), false)) {
    std::printf("{\"error\": \"%s\"}\n", ks.error ? ks.error : "?");
    return 1;
  }
  KktSuper sp;
  if (!sp.build(ks, rp.data(), ci.data())) {
    std::printf("{\"error\": \"%s\"}\n", sp.error ? sp.error : "?");
    return 1;
  }
  const int N = sp.N;
  // ---- the device plan covers every supernode once per level (factor:
  // small items + big rounds; solve: small items + the big list), the
  // rounds' LDS shares are disjoint and inside the pool, small panels fit
  // their lane group's 16 g doubles
  int plan_ok = 1;
  {
    std::vector<int> seen_f(sp.ns, 0), seen_s(sp.ns, 0);
    for (int l = 0; l < sp.nlev; ++l) {
      for (int it = sp.lvi[l]; it < sp.lvi[l + 1]; ++it) {
        const int g = sp.itg[it];
        if (sp.itp[it + 1] - sp.itp[it] > 64 / g) plan_ok = 0;
        for (int e = sp.itp[it]; e < sp.itp[it + 1]; ++e) {
          const int t = sp.itsn[e], f = sp.sw[t] + sp.sr[t];
          if (f > g || f * sp.sw[t] > 16 * g) plan_ok = 0;
          seen_f[t]++;
          seen_s[t]++;
        }
      }
      for (int rd = sp.lvr[l]; rd < sp.lvr[l + 1]; ++rd) {
        if (sp.rdp[rd + 1] - sp.rdp[rd] > 16) plan_ok = 0;
        std::vector<std::pair<int, int>> iv;
        for (int e = sp.rdp[rd]; e < sp.rdp[rd + 1]; ++e) {
          const int t = sp.rsn[e], need = (sp.sw[t] + sp.sr[t]) * sp.sw[t];
          if (sp.rlo[e] < 0 || sp.rlo[e] + need > KktSuper::kPool) plan_ok = 0;
          iv.push_back({sp.rlo[e], sp.rlo[e] + need});
          seen_f[t]++;
        }
        std::sort(iv.begin(), iv.end());
        for (size_t i = 1; i < iv.size(); ++i)
          if (iv[i].first < iv[i - 1].second) plan_ok = 0;
      }
      for (int e = sp.lvb[l]; e < sp.lvb[l + 1]; ++e) seen_s[sp.lbs[e]]++;
    }
    for (int t = 0; t < sp.ns; ++t)
      if (seen_f[t] != 1 || seen_s[t] != 1) plan_ok = 0;
  }
  // ---- a random active set and its KKT values (as big_kkt_factor forms them)
  std::mt19937_64 rng(seed);
  std::uniform_real_distribution<double> U01(0.0, 1.0);
  std::vector<int> CC(n), RC(m);
  for (auto &c : CC) c = U01(rng) < ffix ? 1 : 0;
  for (auto &r : RC) r = U01(rng) < finact ? 0 : 1;
  std::vector<double> diag(N), aval(nnz);  // by vertex
  for (int j = 0; j < n; ++j) diag[j] = CC[j] ? 1.0 : (U01(rng) < 0.5 ? 0.0 : U01(rng)) + delta;
  for (int i = 0; i < m; ++i) diag[n + i] = RC[i] ? -delta : -1.0;
  for (int p = 0; p < nnz; ++p) aval[p] = 2.0 * U01(rng) - 1.0;
  // ---- storage: panels (originals scattered), D, U, update vectors
  std::vector<double> Lv(sp.panel_total, 0.0), Dv(N), Uv(sp.u_total, 0.0), Vv(sp.v_total, 0.0);
  for (int v = 0; v < N; ++v) Dv[sp.pos[v]] = diag[v];
  for (int i = 0; i < m; ++i)
    for (int p = rp[i]; p < rp[i + 1]; ++p)
      if (!CC[ci[p]] && RC[i]) Lv[sp.apos[p]] = -aval[p];
  std::vector<char> colv(N);
  for (int c = 0; c < N; ++c) colv[c] = Dv[c] > 0.0;
  auto ucol = [](long r, long b) { return b * r - b * (b - 1) / 2; };
  // the gather table of front t: child position of every front row (or -1)
  std::vector<int> tab;
  auto build_tab = [&](int t, int f) {
    const int c0 = sp.chp[t], nch = sp.chp[t + 1] - c0;
    tab.assign((size_t)nch * f, -1);
    for (int q = 0; q < nch; ++q) {
      const int c = sp.chl[c0 + q];
      for (int o = sp.srp[c]; o < sp.srp[c + 1]; ++o) tab[(size_t)q * f + sp.rel[o]] = o - sp.srp[c];
    }
    return nch;
  };
  long held = 0;
  // ---- factorisation, level by level
  for (int l = 0; l < sp.nlev; ++l)
    for (int qq = sp.lvp[l]; qq < sp.lvp[l + 1]; ++qq) {
      const int t = sp.lsn[qq];
      const int w = sp.sw[t], r = sp.sr[t], f = w + r, first = sp.sfirst[t];
      const int nch = build_tab(t, f);
      double *P = Lv.data() + sp.poff[t];
      auto child_sum = [&](int i, int k) {  // sum of the children's U at front (i, k), i >= k
        double acc = 0.0;
        for (int q = 0; q < nch; ++q) {
          const int a = tab[(size_t)q * f + i], b = tab[(size_t)q * f + k];
          if (a < 0 || b < 0) continue;
          const int c = sp.chl[sp.chp[t] + q];
          acc += Uv[sp.uoff[c] + ucol(sp.sr[c], b) + (a - b)];
        }
        return acc;
      };
      for (int k = 0; k < w; ++k) {
        P[(size_t)k * f + k] = Dv[first + k] + child_sum(k, k);
        for (int i = k + 1; i < f; ++i) P[(size_t)k * f + i] += child_sum(i, k);
      }
      // dense LDL' of the panel (pivots held to their quasi-definite bounds)
      for (int k = 0; k < w; ++k) {
        double d = P[(size_t)k * f + k];
        const double d0 = d;
        d = colv[first + k] ? std::fmax(d, delta) : std::fmin(d, -delta);
        if (d != d0) ++held;
        Dv[first + k] = d;
        for (int i = k + 1; i < f; ++i) P[(size_t)k * f + i] /= d;
        for (int j = k + 1; j < w; ++j) {
          const double ljd = P[(size_t)k * f + j] * d;
          for (int i = j; i < f; ++i) P[(size_t)j * f + i] -= P[(size_t)k * f + i] * ljd;
        }
      }
      // the update matrix
      double *Ut = Uv.data() + sp.uoff[t];
      for (int b = 0; b < r; ++b)
        for (int a = b; a < r; ++a) {
          double acc = child_sum(w + a, w + b);
          for (int k = 0; k < w; ++k) acc -= P[(size_t)k * f + w + a] * Dv[first + k] * P[(size_t)k * f + w + b];
          Ut[ucol(r, b) + (a - b)] = acc;
        }
    }
  // ---- solve K z = b (b random, in vertex order)
  std::vector<double> bv(N), rv(N);
  for (auto &x : bv) x = 2.0 * U01(rng) - 1.0;
  for (int v = 0; v < N; ++v) rv[sp.pos[v]] = bv[v];
  for (int l = 0; l < sp.nlev; ++l)  // forward (update vectors)
    for (int qq = sp.lvp[l]; qq < sp.lvp[l + 1]; ++qq) {
      const int t = sp.lsn[qq];
      const int w = sp.sw[t], r = sp.sr[t], f = w + r, first = sp.sfirst[t];
      const int nch = build_tab(t, f);
      const double *P = Lv.data() + sp.poff[t];
      std::vector<double> z(f, 0.0);
      for (int i = 0; i < f; ++i) {
        double acc = i < w ? rv[first + i] : 0.0;
        for (int q = 0; q < nch; ++q) {
          const int a = tab[(size_t)q * f + i];
          if (a >= 0) acc += Vv[sp.voff[sp.chl[sp.chp[t] + q]] + a];
        }
        z[i] = acc;
      }
      for (int k = 0; k < w; ++k)
        for (int i = k + 1; i < f; ++i) z[i] -= P[(size_t)k * f + i] * z[k];
      for (int k = 0; k < w; ++k) rv[first + k] = z[k];
      for (int a = 0; a < r; ++a) Vv[sp.voff[t] + a] = z[w + a];
    }
  for (int c = 0; c < N; ++c) rv[c] /= Dv[c];
  for (int l = sp.nlev - 1; l >= 0; --l)  // backward
    for (int qq = sp.lvp[l]; qq < sp.lvp[l + 1]; ++qq) {
      const int t = sp.lsn[qq];
      const int w = sp.sw[t], r = sp.sr[t], f = w + r, first = sp.sfirst[t];
      const double *P = Lv.data() + sp.poff[t];
      for (int k = w - 1; k >= 0; --k) {
        double acc = rv[first + k];
        for (int i = k + 1; i < w; ++i) acc -= P[(size_t)k * f + i] * rv[first + i];
        for (int a = 0; a < r; ++a) acc -= P[(size_t)k * f + w + a] * rv[sp.srow[sp.srp[t] + a]];
        rv[first + k] = acc;
      }
    }
  // ---- residual against the sparse K (vertex order)
  std::vector<double> z(N), Kz(N, 0.0);
  for (int v = 0; v < N; ++v) z[v] = rv[sp.pos[v]];
  for (int v = 0; v < N; ++v) Kz[v] = diag[v] * z[v];
  double amax = 0.0;
  for (int i = 0; i < m; ++i)
    for (int p = rp[i]; p < rp[i + 1]; ++p) {
      const int j = ci[p];
      if (CC[j] || !RC[i]) continue;
      Kz[j] += -aval[p] * z[n + i];
      Kz[n + i] += -aval[p] * z[j];
      amax = std::fmax(amax, std::fabs(aval[p]));
    }
  double res = 0.0, bn = 0.0, zn = 0.0;
  for (int v = 0; v < N; ++v) {
    res = std::fmax(res, std::fabs(Kz[v] - bv[v]));
    bn = std::fmax(bn, std::fabs(bv[v]));
    zn = std::fmax(zn, std::fabs(z[v]));
  }
  int wide = 0;
  for (int t = 0; t < sp.ns; ++t) wide = std::max(wide, sp.sw[t]);
  std::printf(
      "{\"N\": %d, \"nnzL\": %d, \"ncontrib\": %ld, \"ns\": %d, \"nlev\": %d, \"panel_total\": %ld, "
      "\"u_total\": %ld, \"v_total\": %ld, \"flops\": %ld, \"max_f\": %d, \"max_w\": %d, \"max_nch\": %d, "
      "\"nbig\": %d, \"plan_ok\": %d, \"rounds\": %d, \"items\": %d, \"held\": %ld, \"residual\": %.3e, \"bnorm\": %.3e, \"znorm\": %.3e, \"amax\": %.3e}\n",
      N, ks.nnzL, ks.ncontrib, sp.ns, sp.nlev, sp.panel_total, sp.u_total, sp.v_total, sp.flops, sp.max_f, wide,
      sp.max_nch, sp.nbig, plan_ok, (int)sp.rdp.size() - 1, (int)sp.itg.size(), held, res, bn, zn, amax);
  return 0;
}
