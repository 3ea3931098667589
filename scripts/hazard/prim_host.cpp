// Host build of both Prim forms under UBSan/ASan: g++ -O2 -fsanitize=undefined,address
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
#include "prim_select.h"

int main() {
  std::mt19937_64 rng(1);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  long bad = 0, total = 0;
  for (int V : {2, 3, 5, 16, 33, 64}) {
    for (int rep = 0; rep < 2000; ++rep) {
      std::vector<double> ws(V), key(V);
      std::vector<unsigned char> from(V);
      for (int i = 0; i < V; ++i) ws[i] = (rep % 3 == 0) ? double(rng() % 4) : U(rng);  // ties too
      unsigned long long a1[64], a2[64];
      auto K = [&](int v) -> double& { return key[v]; };
      auto F = [&](int v) -> unsigned char& { return from[v]; };
      auto Wf = [&](int v) -> double { return ws[v]; };
      prim<true>(Wf, V, K, F, [&](int v) -> unsigned long long& { return a1[v]; });
      prim<false>(Wf, V, K, F, [&](int v) -> unsigned long long& { return a2[v]; });
      for (int i = 0; i < V; ++i) bad += a1[i] != a2[i];
      ++total;
    }
  }
  printf("host: %ld of %ld trees differ between the branchy and branch-free forms\n", bad, total);
  return bad != 0;
}
