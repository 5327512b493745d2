// kkt_super.h -- supernodal (multifrontal) symbolic analysis of a scenario
// batch's KKT pattern, for the big path's LDL' polish on patterns whose
// level-scheduled factorisation (kkt_symbolic.h: one gather per update
// contribution) is too slow -- the UC LP relaxation's KKT (N = 126,771,
// nnzL = 1.24M, 58M update contributions, 68 % of them into the last 256
// columns).  Built from KktSymbolic's fill-reducing order and L pattern.
//
// Supernodes: columns of the elimination tree merged bottom-up (relaxed
// amalgamation: a child supernode joins its parent while the merged dense
// panel stays within kWidthMax columns and adds at most kZeroFrac explicit
// zeros, or while it is narrower than kSmallWidth).  A supernode s owns the
// consecutive columns first .. first + w - 1 of the final numbering; its
// structure R_s (the rows below, sorted) is the pattern of its top column,
// and every member column's true pattern lies inside the later members and
// R_s (etree property), so its front F_s = members U R_s (f = w + r rows)
// is dense with explicit zeros.
//
// Storage per scenario (the device's polish workspace):
//  * panel of s: f x w doubles, column-major (entry (i, k) at poff + k f + i,
//    i >= k used; the diagonal block's D on the diagonal positions is not
//    used, D lives in Dv[first + k]);
//  * update matrix U_s (the Schur complement of the front onto R_s): r x r
//    lower triangle packed by columns (entry (a, b), a >= b, at
//    uoff + b r - b (b - 1) / 2 + (a - b));
//  * update vector of the forward solve: r doubles at voff.
// rel (aligned with R_s): the position of each structure row in the
// parent's front, so a parent gathers its children's U / update vectors.
//
// Work classes (solve_super.inc): every supernode is done by one wave.  A
// small front (f <= 64 rows, one per lane of a group of g = 8 .. 64 lanes,
// its panel within 16 g doubles) shares a wave with 64 / g - 1 others; a big
// one has a wave to itself and a share of the block's LDS pool, planned in
// rounds.  lvp / lsn list the supernodes by tree level, the small ones of a
// level first (lbig[l]: the first big one).
#pragma once

#include <algorithm>
#include <cstdint>
#include <numeric>
#include <vector>

#include "kkt_symbolic.h"

struct KktSuper {
  static constexpr int kWidthMax = 32;      // panel columns (the block's LDS panel is f x 32)
  static constexpr int kSmallWidth = 8;     // always merge below this width ...
  static constexpr int kSmallStruct = 16;   // ... when the structure is this short
  static constexpr double kZeroFrac = 0.25;  // explicit zeros a merge may add (of the merged panel)
  static constexpr int kWaveRows = 64;      // a small supernode: front rows <= one wave

  int N = 0, ns = 0, nlev = 0;
  long panel_total = 0, u_total = 0, v_total = 0, flops = 0;
  int max_f = 0, max_nch = 0, nbig = 0;
  const char *error = nullptr;
  std::vector<int32_t> pos;                    // [N] vertex -> final index
  std::vector<int32_t> sfirst, sw, sr;         // per supernode
  std::vector<int32_t> poff, uoff, voff;       // per supernode (doubles)
  std::vector<int32_t> srp, srow, rel;         // structure rows (CSR) and their parent-front positions
  std::vector<int32_t> chp, chl;               // children (CSR)
  std::vector<int32_t> lvp, lsn, lbig;         // levels: lsn[lvp[l] .. lvp[l+1]), big from lbig[l]
  std::vector<int32_t> apos;                   // [nnz] A entry -> panel offset of its KKT entry
  std::vector<int32_t> snode;                  // [N] final column -> supernode
  // the device's plan: kpre[t] (structure rows inside the parent's columns:
  // a prefix), small items by level (lvi; item: lane-group size itg, its
  // supernodes itsn[itp..]), big rounds by level (lvr; round: supernodes
  // rsn[rdp..] with their LDS offsets rlo), big supernodes by level (lvb /
  // lbs: the solve deals them to waves)
  std::vector<int32_t> kpre, lvi, itg, itp, itsn, lvr, rdp, rsn, rlo, lvb, lbs;
  // per supernode the device's record, three int4: {first, w, r, poff},
  // {uoff, voff, first child (chl), children}, {srp, kpre, level, 0}
  std::vector<int32_t> rec;

  static constexpr int kPool = 16 * 1024;  // doubles of the device's LDS pool (SUPER_POOL)
  // lane-group size of a small front (8 .. 64 lanes, one front row each)
  static int group_of(int f) {
    int g = 8;
    while (g < f) g *= 2;
    return g;
  }
  // small: one row per lane of a group and the panel within the group's
  // 16 g doubles of its wave's LDS slice
  static bool small_front(int f, int w) { return f <= kWaveRows && (long)f * w <= 16L * group_of(f); }

  // ks: the analysed pattern (ks.pos, ks.Lcp / Lri: the strict lower
  // triangle's pattern in ks's numbering, rows sorted).
  bool build(const KktSymbolic &ks, const int32_t *row_ptr, const int32_t *col_idx) {
    const int n = ks.n, m = ks.m;
    N = ks.N;
    std::vector<int32_t> cc(N), parent(N, -1);
    for (int c = 0; c < N; ++c) {
      cc[c] = ks.Lcp[c + 1] - ks.Lcp[c];
      if (cc[c]) parent[c] = ks.Lri[ks.Lcp[c]];
      if (parent[c] >= 0 && parent[c] <= c) {
        error = "the elimination tree is not topologically numbered";
        return false;
      }
    }
    // ---- relaxed amalgamation, bottom-up (a child's index is below its parent's)
    std::vector<std::vector<int32_t>> kids(N), members(N);
    for (int c = 0; c < N; ++c)
      if (parent[c] >= 0) kids[parent[c]].push_back(c);
    std::vector<long> w(N, 1), real(N);
    std::vector<int32_t> into(N, -1);  // merged into (a rep)
    for (int c = 0; c < N; ++c) real[c] = cc[c] + 1;
    auto panel = [](long ww, long rr) { return ww * (ww + 1) / 2 + ww * rr; };
    for (int c = 0; c < N; ++c) {
      std::vector<int32_t> cand = kids[c];
      std::vector<int32_t> keep;
      // cheapest merges first (explicit zeros added per merged panel entry)
      std::sort(cand.begin(), cand.end(), [&](int a, int b) {
        const double za = 1.0 - double(real[a] + real[c]) / double(panel(w[a] + w[c], cc[c]));
        const double zb = 1.0 - double(real[b] + real[c]) / double(panel(w[b] + w[c], cc[c]));
        return za < zb || (za == zb && a < b);
      });
      std::vector<int32_t> mem;
      for (int k : cand) {
        const long W = w[k] + w[c];
        const long P = panel(W, cc[c]);
        const long Z = P - (real[k] + real[c]);
        // (the small-width rule only at the bottom of the tree: a narrow
        // merge with a long structure row list would chain unrelated
        // siblings into the dense top of the tree)
        if (W <= kWidthMax && (Z <= kZeroFrac * P || (W <= kSmallWidth && cc[c] <= kSmallStruct))) {
          w[c] = W;
          real[c] += real[k];
          into[k] = c;
          mem.insert(mem.end(), members[k].begin(), members[k].end());
          members[k].clear();
          for (int g : kids[k]) keep.push_back(g);
        } else {
          keep.push_back(k);
        }
      }
      mem.push_back(c);
      members[c].swap(mem);
      std::sort(keep.begin(), keep.end());
      kids[c].swap(keep);
    }
    // ---- supernodes (reps) and their tree; postorder; the final numbering
    std::vector<int32_t> rep_of(N);
    for (int c = N - 1; c >= 0; --c) rep_of[c] = into[c] < 0 ? c : rep_of[into[c]];
    std::vector<int32_t> reps;
    for (int c = 0; c < N; ++c)
      if (into[c] < 0) reps.push_back(c);
    ns = (int)reps.size();
    std::vector<int32_t> sid(N, -1);
    for (int q = 0; q < ns; ++q) sid[reps[q]] = q;
    std::vector<int32_t> spar(ns, -1);
    std::vector<std::vector<int32_t>> skids(ns);
    for (int q = 0; q < ns; ++q) {
      const int top = reps[q];
      if (parent[top] >= 0) {
        spar[q] = sid[rep_of[parent[top]]];
        skids[spar[q]].push_back(q);
      }
    }
    std::vector<int32_t> post;
    post.reserve(ns);
    {
      std::vector<std::pair<int32_t, int32_t>> st;
      for (int q = 0; q < ns; ++q) {
        if (spar[q] >= 0) continue;
        st.push_back({q, 0});
        while (!st.empty()) {
          auto &t = st.back();
          if (t.second < (int)skids[t.first].size()) {
            const int ch = skids[t.first][t.second++];
            st.push_back({ch, 0});
          } else {
            post.push_back(t.first);
            st.pop_back();
          }
        }
      }
    }
    if ((int)post.size() != ns) {
      error = "the supernodal tree postorder missed a node";
      return false;
    }
    std::vector<int32_t> newidx(N, -1), order_of(ns);  // old column -> final; supernode q -> final id
    sfirst.assign(ns, 0);
    sw.assign(ns, 0);
    {
      int nxt = 0;
      for (int t = 0; t < ns; ++t) {
        const int q = post[t];
        order_of[q] = t;
        sfirst[t] = nxt;
        for (int c : members[reps[q]]) newidx[c] = nxt++;
        sw[t] = nxt - sfirst[t];
      }
      if (nxt != N) {
        error = "the supernodes do not cover every column";
        return false;
      }
    }
    pos.assign(N, 0);
    for (int v = 0; v < N; ++v) pos[v] = newidx[ks.pos[v]];
    snode.assign(N, 0);
    for (int t = 0; t < ns; ++t)
      for (int k = 0; k < sw[t]; ++k) snode[sfirst[t] + k] = t;
    // structures (final numbering, sorted), parents, children
    srp.assign(ns + 1, 0);
    std::vector<int32_t> sp(ns, -1);
    for (int t = 0; t < ns; ++t) {
      const int top = reps[post[t]];
      srp[t + 1] = srp[t] + cc[top];
      if (spar[post[t]] >= 0) sp[t] = order_of[spar[post[t]]];
    }
    srow.resize(srp[ns]);
    sr.assign(ns, 0);
    for (int t = 0; t < ns; ++t) {
      const int top = reps[post[t]];
      for (int p = ks.Lcp[top], o = srp[t]; p < ks.Lcp[top + 1]; ++p, ++o) srow[o] = newidx[ks.Lri[p]];
      std::sort(srow.begin() + srp[t], srow.begin() + srp[t + 1]);
      sr[t] = srp[t + 1] - srp[t];
      if (sr[t] && srow[srp[t]] < sfirst[t] + sw[t]) {
        error = "a supernode's structure overlaps its columns";
        return false;
      }
      if (sr[t] && sp[t] >= 0 && snode[srow[srp[t]]] != sp[t]) {
        error = "a supernode's first structure row is not in its parent";
        return false;
      }
    }
    // every member column's pattern within the later members and the structure
    for (int c = 0; c < N; ++c) {
      const int t = snode[newidx[c]];
      const int last = sfirst[t] + sw[t];
      for (int p = ks.Lcp[c]; p < ks.Lcp[c + 1]; ++p) {
        const int r = newidx[ks.Lri[p]];
        if (r < last) continue;
        if (!std::binary_search(srow.begin() + srp[t], srow.begin() + srp[t + 1], r)) {
          error = "a member column's pattern leaves its supernode's front";
          return false;
        }
      }
    }
    chp.assign(ns + 1, 0);
    for (int t = 0; t < ns; ++t)
      if (sp[t] >= 0) chp[sp[t] + 1]++;
    for (int t = 0; t < ns; ++t) chp[t + 1] += chp[t];
    chl.resize(chp[ns]);
    {
      std::vector<int32_t> fill(chp.begin(), chp.end() - 1);
      for (int t = 0; t < ns; ++t)
        if (sp[t] >= 0) chl[fill[sp[t]]++] = t;
    }
    // positions of the structure rows in the parent's front
    rel.assign(srow.size(), -1);
    for (int t = 0; t < ns; ++t) {
      const int p = sp[t];
      if (p < 0) {
        if (sr[t]) {
          error = "a root supernode has structure rows";
          return false;
        }
        continue;
      }
      for (int o = srp[t]; o < srp[t + 1]; ++o) {
        const int g = srow[o];
        int at = -1;
        if (g >= sfirst[p] && g < sfirst[p] + sw[p]) {
          at = g - sfirst[p];
        } else {
          const auto b = srow.begin() + srp[p], e = srow.begin() + srp[p + 1];
          const auto it = std::lower_bound(b, e, g);
          if (it != e && *it == g) at = sw[p] + (int)(it - b);
        }
        if (at < 0) {
          error = "a structure row is not in the parent's front";
          return false;
        }
        rel[o] = at;
      }
    }
    // levels (leaves 0); within a level the small supernodes first
    std::vector<int32_t> lev(ns, 0);
    for (int t = 0; t < ns; ++t)  // postorder: children before parents
      if (sp[t] >= 0) lev[sp[t]] = std::max(lev[sp[t]], lev[t] + 1);
    nlev = ns ? *std::max_element(lev.begin(), lev.end()) + 1 : 0;
    lvp.assign(nlev + 1, 0);
    for (int t = 0; t < ns; ++t) lvp[lev[t] + 1]++;
    for (int l = 0; l < nlev; ++l) lvp[l + 1] += lvp[l];
    lsn.resize(ns);
    lbig.assign(nlev, 0);
    {
      std::vector<int32_t> fill(lvp.begin(), lvp.end() - 1);
      for (int pass = 0; pass < 2; ++pass)
        for (int t = 0; t < ns; ++t) {
          const bool sm = small_front(sw[t] + sr[t], sw[t]);
          if (sm == (pass == 0)) lsn[fill[lev[t]]++] = t;
        }
      for (int l = 0; l < nlev; ++l) {
        int b = lvp[l];
        while (b < lvp[l + 1] && small_front(sw[lsn[b]] + sr[lsn[b]], sw[lsn[b]])) ++b;
        lbig[l] = b;
      }
    }
    // storage offsets (int32: the totals must stay below 2^31)
    poff.assign(ns, 0);
    uoff.assign(ns, 0);
    voff.assign(ns, 0);
    long P = 0, U = 0, V = 0;
    max_f = 0;
    max_nch = 0;
    nbig = 0;
    flops = 0;
    for (int t = 0; t < ns; ++t) {
      const long f = sw[t] + sr[t];
      poff[t] = (int32_t)P;
      uoff[t] = (int32_t)U;
      voff[t] = (int32_t)V;
      P += f * sw[t];
      U += (long)sr[t] * (sr[t] + 1) / 2;
      V += sr[t];
      max_f = std::max(max_f, (int)f);
      max_nch = std::max(max_nch, chp[t + 1] - chp[t]);
      if (!small_front((int)f, sw[t])) ++nbig;
      for (int k = 0; k < sw[t]; ++k) flops += (f - k - 1) * (f - k - 1);
      if (P >= INT32_MAX || U >= INT32_MAX) {
        error = "the supernodal factor storage exceeds 2^31 doubles";
        return false;
      }
    }
    panel_total = P;
    u_total = U;
    v_total = V;
    // ---- the device's work plan (solve_super.inc)
    kpre.assign(ns, 0);
    for (int t = 0; t < ns; ++t) {
      const int p = sp[t];
      int k = 0;
      if (p >= 0)
        while (k < sr[t] && rel[srp[t] + k] < sw[p]) ++k;
      kpre[t] = k;
    }
    lvi.assign(nlev + 1, 0);
    itg.clear();
    itp.assign(1, 0);
    itsn.clear();
    lvr.assign(nlev + 1, 0);
    rdp.assign(1, 0);
    rsn.clear();
    rlo.clear();
    lvb.assign(nlev + 1, 0);
    lbs.clear();
    for (int l = 0; l < nlev; ++l) {
      // small fronts by lane-group size g (8 .. 64): 64 / g per wave item
      for (int g = 8; g <= kWaveRows; g *= 2) {
        std::vector<int32_t> grp;
        for (int q = lvp[l]; q < lbig[l]; ++q) {
          const int t = lsn[q];
          if (group_of(sw[t] + sr[t]) == g) grp.push_back(t);
        }
        const int per = kWaveRows / g;
        for (size_t i = 0; i < grp.size(); i += per) {
          itg.push_back(g);
          for (size_t j = i; j < std::min(grp.size(), i + per); ++j) itsn.push_back(grp[j]);
          itp.push_back((int32_t)itsn.size());
        }
      }
      lvi[l + 1] = (int32_t)itg.size();
      // big fronts: rounds of at most 16 (one per wave), panels packed in the
      // pool (largest first, first fit)
      std::vector<int32_t> big(lsn.begin() + lbig[l], lsn.begin() + lvp[l + 1]);
      for (int t : big) {
        lbs.push_back(t);
        if (sw[t] + sr[t] > kPool / 16) {
          error = "a front exceeds the solve's per-wave LDS slice";
          return false;
        }
      }
      lvb[l + 1] = (int32_t)lbs.size();
      std::stable_sort(big.begin(), big.end(), [&](int a, int b) {
        return (long)(sw[a] + sr[a]) * sw[a] > (long)(sw[b] + sr[b]) * sw[b];
      });
      std::vector<std::pair<int, int>> rounds;  // (entries, used)
      std::vector<std::vector<std::pair<int32_t, int32_t>>> rent;
      for (int t : big) {
        const int need = (sw[t] + sr[t]) * sw[t];
        if (need > kPool) {
          error = "a supernode's panel exceeds the LDS pool";
          return false;
        }
        size_t k = 0;
        while (k < rounds.size() && (rounds[k].first >= 16 || rounds[k].second + need > kPool)) ++k;
        if (k == rounds.size()) {
          rounds.push_back({0, 0});
          rent.emplace_back();
        }
        rent[k].push_back({t, rounds[k].second});
        rounds[k].first += 1;
        rounds[k].second += (need + 1) & ~1;
      }
      for (auto &re : rent) {
        for (auto &pr : re) {
          rsn.push_back(pr.first);
          rlo.push_back(pr.second);
        }
        rdp.push_back((int32_t)rsn.size());
      }
      lvr[l + 1] = (int32_t)(rdp.size() - 1);
    }
    rec.assign((size_t)ns * 12, 0);
    for (int t = 0; t < ns; ++t) {
      int32_t *q = rec.data() + (size_t)t * 12;
      q[0] = sfirst[t];
      q[1] = sw[t];
      q[2] = sr[t];
      q[3] = poff[t];
      q[4] = uoff[t];
      q[5] = voff[t];
      q[6] = chp[t];
      q[7] = chp[t + 1] - chp[t];
      q[8] = srp[t];
      q[9] = kpre[t];
      q[10] = lev[t];
    }
    // A's entries: the panel offset of the lower KKT entry (max, min)
    const int nnz = row_ptr[m];
    apos.assign(nnz, 0);
    for (int i = 0; i < m; ++i)
      for (int p = row_ptr[i]; p < row_ptr[i + 1]; ++p) {
        const int a = pos[col_idx[p]], b = pos[n + i];
        const int R = std::max(a, b), C = std::min(a, b);
        const int t = snode[C];
        const int f = sw[t] + sr[t];
        int rp = -1;
        if (R < sfirst[t] + sw[t]) {
          rp = R - sfirst[t];
        } else {
          const auto bb = srow.begin() + srp[t], ee = srow.begin() + srp[t + 1];
          const auto it = std::lower_bound(bb, ee, R);
          if (it != ee && *it == R) rp = sw[t] + (int)(it - bb);
        }
        if (rp < 0) {
          error = "an entry of A lies outside its supernode's front";
          return false;
        }
        apos[p] = poff[t] + (C - sfirst[t]) * f + rp;
      }
    return true;
  }
};
