// Test harness (not product): runs KktSymbolic::analyze on a pattern read
// from stdin ("n m nnz", row_ptr, col_idx) and prints its arrays as JSON.
#include "kkt_symbolic.h"
#include <cstdio>
#include <vector>

static void arr(const char *name, const std::vector<int32_t> &v, bool last = false) {
  std::printf("\"%s\": [", name);
  for (size_t i = 0; i < v.size(); ++i) std::printf(i ? ",%d" : "%d", v[i]);
  std::printf("]%s\n", last ? "" : ",");
}

int main() {
  int n, m, nnz;
  if (std::scanf("%d %d %d", &n, &m, &nnz) != 3) return 2;
  std::vector<int32_t> rp(m + 1), ci(nnz);
  for (auto &v : rp) std::scanf("%d", &v);
  for (auto &v : ci) std::scanf("%d", &v);
  KktSymbolic k;
  if (!k.analyze(n, m, rp.data(), ci.data())) {
    std::printf("{\"error\": \"%s\"}\n", k.error ? k.error : "?");
    return 1;
  }
  std::printf("{\"N\": %d, \"nnzL\": %d, \"NL\": %d, \"chain0\": %d, \"ncontrib\": %ld,\n", k.N, k.nnzL, k.NL,
              k.chain0, k.ncontrib);
  arr("pos", k.pos); arr("Lcp", k.Lcp); arr("Lri", k.Lri); arr("Lcl", k.Lcl); arr("Lrp", k.Lrp);
  arr("Lrc", k.Lrc); arr("Lrq", k.Lrq); arr("lvp", k.lvp); arr("lvc", k.lvc); arr("lep", k.lep);
  arr("lee", k.lee); arr("ecp", k.ecp); arr("ec1", k.ec1); arr("ec2", k.ec2); arr("eck", k.eck);
  arr("apos", k.apos); arr("arow", k.arow, true);
  std::printf("}\n");
  return 0;
}
