// Prim selection step of masks.hip (k_pixel_masks, MST branch) in the two source forms:
// the branch-free one the product uses and the branchy one DESIGN.md's round-1 "codegen
// hazard" note describes.  Shared by the device harness (prim_hazard.hip) and a host
// build under -fsanitize=undefined (prim_host.cpp).  Root-cause study, not product code.
#pragma once
#ifndef HD
#define HD
#endif
#include <cstdint>

HD inline double qfun(double wi, double wj) { const double q = 0.5 * (wi + wj); return q > 1e-12 ? q : 1e-12; }
HD inline int imin(int a, int b) { return a < b ? a : b; }
HD inline int imax(int a, int b) { return a > b ? a : b; }
HD inline bool beats(double w, int a, int b, double w2, int c, int d, int V) {
  if (w != w2) return w > w2;
  return imin(a, b) * V + imax(a, b) < imin(c, d) * V + imax(c, d);
}

// maximum spanning tree of the complete graph with weights q(w_i, w_j), Prim from node 0
// under Kruskal's strict order; adjacency rows as bit masks.  KEY/FROM are caller storage
// (LDS columns on the device), accessed as key(v), from(v).
template <bool BRANCHY, typename WS, typename KEY, typename FROM, typename ADJ>
HD inline void prim(WS ws, int V, KEY key, FROM from, ADJ adj) {
  for (int i = 0; i < V; ++i) adj(i) = 0ull;
  unsigned long long in = 1ull;
  for (int v = 1; v < V; ++v) {
    key(v) = qfun(ws(0), ws(v));
    from(v) = 0;
  }
  for (int step = 1; step < V; ++step) {
    int bv, bf;
    if (BRANCHY) {
      bv = -1;
      bf = 0;
      double bk = 0.0;
      for (int v = 1; v < V; ++v) {
        if ((in >> v) & 1ull) continue;
        const double kv = key(v);
        const int fv = from(v);
        if (bv < 0 || beats(kv, fv, v, bk, bf, bv, V)) {
          bv = v;
          bf = fv;
          bk = kv;
        }
      }
    } else {
      bv = 0;
      bf = 0;
      int br = 0;
      double bk = -1.0;
      for (int v = 1; v < V; ++v) {
        if ((in >> v) & 1ull) continue;
        const double kv = key(v);
        const int fv = from(v);
        const int rv = imin(fv, v) * V + imax(fv, v);
        const bool better = (kv > bk) || (kv == bk && rv < br);
        bv = better ? v : bv;
        bf = better ? fv : bf;
        br = better ? rv : br;
        bk = better ? kv : bk;
      }
    }
    in |= 1ull << bv;
    adj(bf) |= 1ull << bv;
    adj(bv) |= 1ull << bf;
    const double wb = ws(bv);
    for (int u = 1; u < V; ++u) {
      if ((in >> u) & 1ull) continue;
      const double w = qfun(wb, ws(u));
      if (beats(w, bv, u, key(u), from(u), u, V)) {
        key(u) = w;
        from(u) = (unsigned char)bv;
      }
    }
  }
}
