// kkt_symbolic.h -- host-side symbolic analysis of a scenario batch's KKT
// pattern, shared by every scenario of the batch (they share A's pattern).
//
// The active-set polish of mid-size scenarios (see phgpu.hip, solve_mid)
// factors the quasi-definite KKT matrix of an active set
//
//     [ H    -A' ]      H = diag(q_j + delta)  free column j, 1 fixed column
//     [ -A   -G  ]      G = diag(delta)        active row,    1 inactive row
//
// (entries of fixed columns / inactive rows zeroed) as L D L' with a
// fill-reducing order fixed per PATTERN: whatever the active set, the
// numeric matrix's nonzeros are a subset of the pattern's, and a
// quasi-definite matrix factors stably in any symmetric order, so the
// order, the elimination tree, L's pattern and the per-entry update lists
// are computed once here and every scenario's factorisation is a fixed,
// level-scheduled sequence of gathers on the device.
//
// Vertices: v < n is column v of A, v = n + i is row i.  Everything below
// is in permuted indices c = pos[v].
#pragma once

#include <algorithm>
#include <climits>
#include <cstdint>
#include <queue>
#include <utility>
#include <vector>

struct KktSymbolic {
  int n = 0, m = 0, N = 0, nnzL = 0, NL = 0;
  int chain0 = 0;  // levels chain0 .. NL-1 hold one column each (the top of the tree)
  long ncontrib = 0;
  const char *error = nullptr;  // why analyze() refused the pattern
  // the update lists' size a pattern may need at most (three int32 arrays)
  static constexpr long long kMaxContrib = 1LL << 28;
  std::vector<int32_t> pos;              // [N] vertex -> permuted index
  std::vector<int32_t> Lcp, Lri, Lcl;    // CSC of the strict lower triangle of L; column of entry
  std::vector<int32_t> Lrp, Lrc, Lrq;    // CSR view: row r -> columns k, CSC positions
  std::vector<int32_t> lvp, lvc;         // levels: [NL+1] ptr, permuted columns by level
  std::vector<int32_t> lep, lee;         // [NL+1] ptr, CSC positions of the level's entries
  std::vector<int32_t> ecp;              // [nnzL+1] update list ranges per L entry
  std::vector<int32_t> ec1, ec2, eck;    // updates of entry (r,c): L[ec1] * D[eck] * L[ec2]
  std::vector<int32_t> apos, arow;       // [nnz] CSR entry of A -> CSC position in L, its row

  // Minimum-degree order on the KKT graph (explicit elimination graph,
  // ties by vertex index: deterministic), then the symbolic factorisation.
  // lists = false: no update lists (ecp / ec1 / ec2 / eck stay empty; the
  // supernodal factorisation of kkt_super.h needs only the order and L's
  // pattern), ncontrib is still counted.
  bool analyze(int n_, int m_, const int32_t *row_ptr, const int32_t *col_idx, bool lists = true) {
    n = n_;
    m = m_;
    N = n + m;
    const int nnz = row_ptr[m];
    std::vector<std::vector<int32_t>> adj(N);
    for (int i = 0; i < m; ++i)
      for (int p = row_ptr[i]; p < row_ptr[i + 1]; ++p) {
        const int j = col_idx[p];
        adj[j].push_back(n + i);
        adj[n + i].push_back(j);
      }
    for (auto &a : adj) {
      std::sort(a.begin(), a.end());
      a.erase(std::unique(a.begin(), a.end()), a.end());
    }
    // ---- minimum degree
    std::vector<std::vector<int32_t>> g = adj;
    std::vector<char> alive(N, 1);
    std::vector<int32_t> order;
    order.reserve(N);
    using QE = std::pair<int, int>;
    std::priority_queue<QE, std::vector<QE>, std::greater<QE>> pq;
    for (int v = 0; v < N; ++v) pq.push({(int)g[v].size(), v});
    std::vector<int32_t> mark(N, -1), tmp;
    while (!pq.empty()) {
      const auto [d, v] = pq.top();
      pq.pop();
      if (!alive[v] || d != (int)g[v].size()) continue;
      alive[v] = 0;
      order.push_back(v);
      std::vector<int32_t> nb;
      for (int a : g[v])
        if (alive[a]) nb.push_back(a);
      for (int a : nb) {  // a's new neighbourhood: (adj(a) U nb) \ {a, v}
        tmp.clear();
        for (int b : g[a])
          if (b != v && alive[b]) {
            tmp.push_back(b);
            mark[b] = a;
          }
        for (int b : nb)
          if (b != a && mark[b] != a) {  // nb holds live vertices only
            tmp.push_back(b);
            mark[b] = a;
          }
        std::sort(tmp.begin(), tmp.end());
        g[a] = tmp;
        pq.push({(int)g[a].size(), a});
      }
      g[v].clear();
    }
    if ((int)order.size() != N) {
      error = "the minimum-degree order did not cover every vertex";
      return false;
    }
    // ---- symbolic factorisation: pattern(c) = {pos[a] > c} U children's
    // patterns; then once more in level order (leaves first, the columns
    // of a level contiguous): a topological order of the elimination tree
    // has the same fill, and the device then finds level l's columns at
    // lvp[l] .. lvp[l+1] and their CSC entries at Lcp[lvp[l]] .. without an
    // indirection (lvc and lee are the identity).
    std::vector<std::vector<int32_t>> pat;
    std::vector<int32_t> parent, level;
    auto symbolic = [&]() {
      pos.assign(N, 0);
      for (int c = 0; c < N; ++c) pos[order[c]] = c;
      pat.assign(N, {});
      parent.assign(N, -1);
      std::vector<std::vector<int32_t>> kids(N);
      std::fill(mark.begin(), mark.end(), -1);
      for (int c = 0; c < N; ++c) {
        auto &P = pat[c];
        const int v = order[c];
        for (int a : adj[v])
          if (pos[a] > c && mark[pos[a]] != c) {
            P.push_back(pos[a]);
            mark[pos[a]] = c;
          }
        for (int k : kids[c])
          for (int r : pat[k])
            if (r > c && mark[r] != c) {
              P.push_back(r);
              mark[r] = c;
            }
        std::sort(P.begin(), P.end());
        if (!P.empty()) {
          parent[c] = P[0];
          kids[P[0]].push_back(c);
        }
      }
      level.assign(N, 0);  // levels of the elimination tree (leaves 0)
      for (int c = 0; c < N; ++c)
        if (parent[c] >= 0) level[parent[c]] = std::max(level[parent[c]], level[c] + 1);
    };
    symbolic();
    {
      std::vector<int32_t> byl(N);
      for (int c = 0; c < N; ++c) byl[c] = c;
      std::stable_sort(byl.begin(), byl.end(), [&](int a, int b) { return level[a] < level[b]; });
      std::vector<int32_t> o2(N);
      for (int c = 0; c < N; ++c) o2[c] = order[byl[c]];
      order.swap(o2);
    }
    symbolic();
    {  // sizes in 64 bits first: a dense trailing block of a few thousand
       // vertices overflows int32 in the update lists
      long long nl = 0, nc = 0;
      for (int c = 0; c < N; ++c) {
        const long long sz = (long long)pat[c].size();
        nl += sz;
        nc += sz * (sz - 1) / 2;
      }
      if (nl > INT32_MAX) {
        error = "the KKT factor has more than 2^31 entries";
        return false;
      }
      ncontrib = (long)nc;
    }
    Lcp.assign(N + 1, 0);
    for (int c = 0; c < N; ++c) Lcp[c + 1] = Lcp[c] + (int)pat[c].size();
    nnzL = Lcp[N];
    Lri.resize(nnzL);
    for (int c = 0; c < N; ++c) std::copy(pat[c].begin(), pat[c].end(), Lri.begin() + Lcp[c]);
    Lcl.resize(nnzL);
    for (int c = 0; c < N; ++c)
      for (int p = Lcp[c]; p < Lcp[c + 1]; ++p) Lcl[p] = c;
    // CSR view
    Lrp.assign(N + 1, 0);
    for (int p = 0; p < nnzL; ++p) Lrp[Lri[p] + 1]++;
    for (int r = 0; r < N; ++r) Lrp[r + 1] += Lrp[r];
    Lrc.resize(nnzL);
    Lrq.resize(nnzL);
    {
      std::vector<int32_t> fill(Lrp.begin(), Lrp.end() - 1);
      for (int c = 0; c < N; ++c)
        for (int p = Lcp[c]; p < Lcp[c + 1]; ++p) {
          const int q = fill[Lri[p]]++;
          Lrc[q] = c;
          Lrq[q] = p;
        }
    }
    // ---- levels
    NL = 0;
    for (int c = 0; c < N; ++c) NL = std::max(NL, level[c] + 1);
    lvp.assign(NL + 1, 0);
    for (int c = 0; c < N; ++c) lvp[level[c] + 1]++;
    for (int l = 0; l < NL; ++l) lvp[l + 1] += lvp[l];
    lvc.resize(N);
    {
      std::vector<int32_t> fill(lvp.begin(), lvp.end() - 1);
      for (int c = 0; c < N; ++c) lvc[fill[level[c]]++] = c;
    }
    for (int c = 0; c < N; ++c)
      if (lvc[c] != c || (c > 0 && level[c] < level[c - 1])) {
        error = "the level-order renumbering failed";
        return false;
      }
    chain0 = NL;
    while (chain0 > 0 && lvp[chain0] - lvp[chain0 - 1] == 1) --chain0;
    lep.assign(NL + 1, 0);
    lee.clear();
    lee.reserve(nnzL);
    for (int l = 0; l < NL; ++l) {
      for (int q = lvp[l]; q < lvp[l + 1]; ++q)
        for (int p = Lcp[lvc[q]]; p < Lcp[lvc[q] + 1]; ++p) lee.push_back(p);
      lep[l + 1] = (int32_t)lee.size();
    }
    for (int e = 0; e < nnzL; ++e)
      if (lee[e] != e) {
        error = "the level-order renumbering failed";
        return false;
      }
    auto entry = [&](int r, int c) {
      const auto b = Lri.begin() + Lcp[c], e = Lri.begin() + Lcp[c + 1];
      return (int32_t)(std::lower_bound(b, e, r) - Lri.begin());
    };
    ecp.clear();
    ec1.clear();
    ec2.clear();
    eck.clear();
    if (lists && !build_lists()) return false;
    // ---- A's entries in L
    apos.resize(nnz);
    arow.resize(nnz);
    for (int i = 0; i < m; ++i)
      for (int p = row_ptr[i]; p < row_ptr[i + 1]; ++p) {
        const int pj = pos[col_idx[p]], pi = pos[n + i];
        apos[p] = pj > pi ? entry(pj, pi) : entry(pi, pj);
        arow[p] = i;
      }
    return true;
  }

  // The update lists of the per-entry factorisation (entry (r,c) -= L(r,k)
  // D(k) L(c,k) for k < c) from the analysed pattern: a pattern analysed
  // with lists = false gets them later without a second ordering (the big
  // path builds them only when its per-entry polish will run).
  bool build_lists() {
    if (ncontrib > kMaxContrib) {
      error = "the KKT factor's update lists exceed 2^28 entries";
      return false;
    }
    auto entry = [&](int r, int c) {
      const auto b = Lri.begin() + Lcp[c], e = Lri.begin() + Lcp[c + 1];
      return (int32_t)(std::lower_bound(b, e, r) - Lri.begin());
    };
    std::vector<int32_t> cnt(nnzL + 1, 0);
    for (int k = 0; k < N; ++k)
      for (int a = Lcp[k]; a < Lcp[k + 1]; ++a)
        for (int b = a + 1; b < Lcp[k + 1]; ++b) cnt[entry(Lri[b], Lri[a]) + 1]++;
    ecp.assign(nnzL + 1, 0);
    for (int e = 0; e < nnzL; ++e) ecp[e + 1] = ecp[e] + cnt[e + 1];
    ncontrib = ecp[nnzL];
    ec1.resize(ncontrib);
    ec2.resize(ncontrib);
    eck.resize(ncontrib);
    std::vector<int32_t> fill(ecp.begin(), ecp.end() - 1);
    for (int k = 0; k < N; ++k)
      for (int a = Lcp[k]; a < Lcp[k + 1]; ++a)
        for (int b = a + 1; b < Lcp[k + 1]; ++b) {
          const int e = entry(Lri[b], Lri[a]);
          const int q = fill[e]++;
          ec1[q] = b;  // L(r,k)
          ec2[q] = a;  // L(c,k)
          eck[q] = k;
        }
    return true;
  }
};
