// cr_graph_dump — prints the persistent CR task graph (cr_persist_graph) of a
// (p, n) system: one line per task "type I h a b : deps...". Host only (no GPU
// call); tests/test_cr_graph.py checks it against a data-hazard model.
#include <cstdio>
#include <cstdlib>

#include "../sqrtlm-slam_amd/csrc/sqlm_rcs_solve.hip"

int main(int argc, char **argv) {
  const int p = argc > 1 ? std::atoi(argv[1]) : 278, n = argc > 2 ? std::atoi(argv[2]) : 112;
  std::vector<sqlm::CRTask> T;
  std::vector<int> D;
  sqlm::cr_persist_graph(p, n, T, D);
  for (const auto &t : T) {
    std::printf("%d %d %d %d %d :", t.type, t.I, t.h, t.a, t.b);
    for (int k = 0; k < t.dep_cnt; ++k) std::printf(" %d", D[t.dep_off + k]);
    std::printf("\n");
  }
  return 0;
}
