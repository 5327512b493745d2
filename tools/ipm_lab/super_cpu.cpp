// Lab library (not product): the supernodal analysis of kkt_super.h and a
// CPU replay of solve_super.inc's factorisation / solve on a numeric
// quasi-definite KKT matrix K = [H -A'; -A -G] (vertex order: columns
// 0..n-1, rows n..n+m-1), for prototyping the interior-point solve in
// Python (tools/ipm_lab/ipm_lab.py) on the device's exact algorithm.
//   g++ -O2 -shared -fPIC -std=c++17 -I mpi-sppy_amd/csrc super_cpu.cpp -o libsuper_cpu.so
#include "kkt_super.h"

#include <cmath>
#include <cstring>
#include <vector>

namespace {
struct H {
  int n, m, nnz;
  std::vector<int32_t> rp, ci;
  KktSymbolic ks;
  KktSuper sp;
  std::vector<double> Lv, Dv, Uv, Vv;
  std::vector<char> colv;
  std::vector<int> tab;
  long held = 0;
};
inline long ucl(long r, long b) { return b * r - b * (b - 1) / 2; }
}  // namespace

extern "C" {
void *sc_create(int n, int m, const int32_t *rp, const int32_t *ci, long *info) {
  H *h = new H;
  h->n = n;
  h->m = m;
  h->nnz = rp[m];
  h->rp.assign(rp, rp + m + 1);
  h->ci.assign(ci, ci + h->nnz);
  if (!h->ks.analyze(n, m, rp, ci, false) || !h->sp.build(h->ks, rp, ci)) {
    delete h;
    return nullptr;
  }
  info[0] = h->sp.N;
  info[1] = h->sp.ns;
  info[2] = h->sp.nlev;
  info[3] = h->sp.panel_total;
  info[4] = h->sp.u_total;
  info[5] = h->sp.flops;
  info[6] = h->ks.nnzL;
  return h;
}

void sc_destroy(void *p) { delete (H *)p; }

// diag [N] (vertex order; columns > 0, rows < 0), aval [nnz] (A's values;
// K's off-diagonal entry is -A), colmask [n] (0: column dropped from the
// rows, its A entries omitted), rowmask [m] (0: row's entries omitted).
long sc_factor(void *p, const double *diag, const double *aval, const int32_t *colmask, const int32_t *rowmask,
               double delta) {
  H &h = *(H *)p;
  KktSuper &sp = h.sp;
  const int N = sp.N, n = h.n, m = h.m;
  h.Lv.assign(sp.panel_total, 0.0);
  h.Dv.assign(N, 0.0);
  h.Uv.assign(sp.u_total, 0.0);
  h.Vv.assign(sp.v_total, 0.0);
  for (int v = 0; v < N; ++v) h.Dv[sp.pos[v]] = diag[v];
  for (int i = 0; i < m; ++i)
    for (int q = h.rp[i]; q < h.rp[i + 1]; ++q)
      if (colmask[h.ci[q]] && rowmask[i]) h.Lv[sp.apos[q]] = -aval[q];
  h.colv.assign(N, 0);
  for (int c = 0; c < N; ++c) h.colv[c] = h.Dv[c] > 0.0;
  h.held = 0;
  for (int l = 0; l < sp.nlev; ++l)
    for (int qq = sp.lvp[l]; qq < sp.lvp[l + 1]; ++qq) {
      const int t = sp.lsn[qq];
      const int w = sp.sw[t], r = sp.sr[t], f = w + r, first = sp.sfirst[t];
      const int c0 = sp.chp[t], nch = sp.chp[t + 1] - c0;
      h.tab.assign((size_t)nch * f, -1);
      for (int q = 0; q < nch; ++q) {
        const int c = sp.chl[c0 + q];
        for (int o = sp.srp[c]; o < sp.srp[c + 1]; ++o) h.tab[(size_t)q * f + sp.rel[o]] = o - sp.srp[c];
      }
      double *P = h.Lv.data() + sp.poff[t];
      auto child_sum = [&](int i, int k) {
        double acc = 0.0;
        for (int q = 0; q < nch; ++q) {
          const int a = h.tab[(size_t)q * f + i], b = h.tab[(size_t)q * f + k];
          if (a < 0 || b < 0) continue;
          const int c = sp.chl[c0 + q];
          acc += h.Uv[sp.uoff[c] + ucl(sp.sr[c], b) + (a - b)];
        }
        return acc;
      };
      for (int k = 0; k < w; ++k) {
        P[(size_t)k * f + k] = h.Dv[first + k] + child_sum(k, k);
        for (int i = k + 1; i < f; ++i) P[(size_t)k * f + i] += child_sum(i, k);
      }
      for (int k = 0; k < w; ++k) {
        double d = P[(size_t)k * f + k];
        const double d0 = d;
        d = h.colv[first + k] ? std::fmax(d, delta) : std::fmin(d, -delta);
        if (d != d0) ++h.held;
        h.Dv[first + k] = d;
        for (int i = k + 1; i < f; ++i) P[(size_t)k * f + i] /= d;
        for (int j = k + 1; j < w; ++j) {
          const double ljd = P[(size_t)k * f + j] * d;
          for (int i = j; i < f; ++i) P[(size_t)j * f + i] -= P[(size_t)k * f + i] * ljd;
        }
      }
      double *Ut = h.Uv.data() + sp.uoff[t];
      for (int b = 0; b < r; ++b)
        for (int a = b; a < r; ++a) {
          double acc = child_sum(w + a, w + b);
          for (int k = 0; k < w; ++k) acc -= P[(size_t)k * f + w + a] * h.Dv[first + k] * P[(size_t)k * f + w + b];
          Ut[ucl(r, b) + (a - b)] = acc;
        }
    }
  return h.held;
}

// rhs [N] vertex order, overwritten by K^-1 rhs
void sc_solve(void *p, double *rhs) {
  H &h = *(H *)p;
  KktSuper &sp = h.sp;
  const int N = sp.N;
  std::vector<double> rv(N);
  for (int v = 0; v < N; ++v) rv[sp.pos[v]] = rhs[v];
  for (int l = 0; l < sp.nlev; ++l)
    for (int qq = sp.lvp[l]; qq < sp.lvp[l + 1]; ++qq) {
      const int t = sp.lsn[qq];
      const int w = sp.sw[t], r = sp.sr[t], f = w + r, first = sp.sfirst[t];
      const int c0 = sp.chp[t], nch = sp.chp[t + 1] - c0;
      std::vector<double> z(f, 0.0);
      for (int i = 0; i < w; ++i) z[i] = rv[first + i];
      for (int q = 0; q < nch; ++q) {
        const int c = sp.chl[c0 + q];
        for (int o = sp.srp[c]; o < sp.srp[c + 1]; ++o) z[sp.rel[o]] += h.Vv[sp.voff[c] + (o - sp.srp[c])];
      }
      const double *P = h.Lv.data() + sp.poff[t];
      for (int k = 0; k < w; ++k)
        for (int i = k + 1; i < f; ++i) z[i] -= P[(size_t)k * f + i] * z[k];
      for (int k = 0; k < w; ++k) rv[first + k] = z[k];
      for (int a = 0; a < r; ++a) h.Vv[sp.voff[t] + a] = z[w + a];
    }
  for (int c = 0; c < N; ++c) rv[c] /= h.Dv[c];
  for (int l = sp.nlev - 1; l >= 0; --l)
    for (int qq = sp.lvp[l]; qq < sp.lvp[l + 1]; ++qq) {
      const int t = sp.lsn[qq];
      const int w = sp.sw[t], r = sp.sr[t], f = w + r, first = sp.sfirst[t];
      const double *P = h.Lv.data() + sp.poff[t];
      for (int k = w - 1; k >= 0; --k) {
        double acc = rv[first + k];
        for (int i = k + 1; i < w; ++i) acc -= P[(size_t)k * f + i] * rv[first + i];
        for (int a = 0; a < r; ++a) acc -= P[(size_t)k * f + w + a] * rv[sp.srow[sp.srp[t] + a]];
        rv[first + k] = acc;
      }
    }
  for (int v = 0; v < N; ++v) rhs[v] = rv[sp.pos[v]];
}
}
