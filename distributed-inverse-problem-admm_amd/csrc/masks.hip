// masks.hip -- per-pixel edge masks for masked precisions (setup path).
//
// Replaces the per-pixel networkx loop of
// /root/reference/block_3_graph_and_precisions.py:154-187 (_build_all_pixel_masks) and
// its helpers :62-151.  One thread per pixel; the node graph at a pixel has V <= 64
// nodes, so adjacency rows are 64-bit masks kept in LDS next to the pixel's W_i.
//
//   q_ij(p)  : block_3:26-39 (arithmetic / harmonic, floored at 1e-12).  q is symmetric
//              bit-for-bit, so the reference's q_sym = (q + q^T)/2 (:171-173) equals q.
//   MST      : nx.maximum_spanning_tree (Kruskal): edges sorted by weight descending with
//              a stable sort over G.edges() order, i.e. ties by lexicographic (i, j).  Under
//              that strict total order the maximum spanning tree is unique, so Prim's
//              algorithm with the same comparison yields the identical tree.
//   kNN      : per node the k_eff = min(k, V-1) largest q_ij (j != i), symmetrised
//              (:75-86); if the graph is disconnected, every edge of the MST above is added
//              (:97-107).  np.argpartition's choice among equal q is unspecified; here ties
//              go to the higher node index (numpy's usual outcome on tied rows).
//   chain    : edges between consecutive entries of a per-pixel permutation (:134-151),
//              drawn on the host by admm_chain_orders (numpy's PCG64 stream, replayed).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "../../include/admm_tomo.h"

namespace admm_internal {
int fail(int code, const std::string& msg);
}

namespace {

using admm_internal::fail;

#define MHIPCHK(expr)                                                                                     \
  do {                                                                                                    \
    hipError_t _e = (expr);                                                                               \
    if (_e != hipSuccess) return fail(ADMM_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));     \
  } while (0)

constexpr int kMaxV = ADMM_MASK_MAX_NODES;

__device__ __forceinline__ double qfun(double wi, double wj, int mode) {
  const double q = (mode == ADMM_Q_HARMONIC) ? (wi * wj) / (wi + wj) : 0.5 * (wi + wj);
  return fmax(q, 1e-12);
}

// edge (a, b) beats edge (c, d) in Kruskal's order: heavier, or equally heavy and
// earlier in lexicographic (min, max) order
__device__ __forceinline__ bool beats(double w, int a, int b, double w2, int c, int d, int V) {
  if (w != w2) return w > w2;
  const int r1 = min(a, b) * V + max(a, b), r2 = min(c, d) * V + max(c, d);
  return r1 < r2;
}

// MAXV >= V nodes, T pixels per block: LDS = 25 B x MAXV x T (100 KB for every instance)
template <int MAXV, int T>
__global__ __launch_bounds__(T) void k_pixel_masks(const double* __restrict__ W, int V, long long n, int strategy,
                                                   int k, int qmode, const int* __restrict__ orders,
                                                   unsigned char* __restrict__ keep) {
  __shared__ double ws[MAXV][T];
  __shared__ double key[MAXV][T];
  __shared__ unsigned long long adj[MAXV][T];
  __shared__ unsigned char from[MAXV][T];
  const int t = threadIdx.x;
  const long long p = (long long)blockIdx.x * T + t;
  if (p >= n) return;  // every thread touches only its own LDS column: no barriers
  for (int i = 0; i < V; ++i) {
    ws[i][t] = W[(size_t)i * n + p];
    adj[i][t] = 0ull;
  }
  const unsigned long long all = (V == 64) ? ~0ull : ((1ull << V) - 1ull);
  auto link = [&](int a, int b) {
    adj[a][t] |= 1ull << b;
    adj[b][t] |= 1ull << a;
  };
  if (strategy == ADMM_MASK_CHAIN) {
    const int* ord = orders + (size_t)p * V;
    for (int s = 0; s + 1 < V; ++s) link(ord[s], ord[s + 1]);
  } else {
    bool need_tree = (strategy == ADMM_MASK_MST);
    if (strategy == ADMM_MASK_KNN) {
      const int ke = min(k, V - 1);
      for (int i = 0; i < V; ++i) {
        const double wi = ws[i][t];
        unsigned long long chosen = 1ull << i;
        for (int r = 0; r < ke; ++r) {
          // every q >= 1e-12 beats bq = -1; >=: among equal q the higher index wins
          int bj = 0;
          double bq = -1.0;
          for (int j = 0; j < V; ++j) {
            if ((chosen >> j) & 1ull) continue;
            const double qj = qfun(wi, ws[j][t], qmode);
            const bool better = qj >= bq;
            bj = better ? j : bj;
            bq = better ? qj : bq;
          }
          chosen |= 1ull << bj;
          link(i, bj);
        }
      }
      // connectivity by breadth-first sweeps over the bitmask rows
      unsigned long long seen = 1ull, frontier = 1ull;
      while (frontier) {
        unsigned long long nf = 0ull;
        for (unsigned long long f = frontier; f; f &= f - 1ull) nf |= adj[__ffsll((long long)f) - 1][t];
        nf &= ~seen;
        seen |= nf;
        frontier = nf;
      }
      need_tree = (seen != all);
    }
    if (need_tree) {
      // Prim from node 0 under Kruskal's strict order
      unsigned long long in = 1ull;
      for (int v = 1; v < V; ++v) {
        key[v][t] = qfun(ws[0][t], ws[v][t], qmode);
        from[v][t] = 0;
      }
      for (int step = 1; step < V; ++step) {
        // best candidate as (key, edge rank); every q >= 1e-12, so bk = -1 loses to any key.
        // Branch-free on purpose: an `if (bv < 0 || beats(..)) { bv = v; bk = kv; .. }` form
        // of this loop came out of hipcc (ROCm 7.2, -O3) updating bk but not bv.
        int bv = 0, bf = 0, br = 0;
        double bk = -1.0;
        for (int v = 1; v < V; ++v) {
          if ((in >> v) & 1ull) continue;
          const double kv = key[v][t];
          const int fv = from[v][t];
          const int rv = min(fv, v) * V + max(fv, v);
          const bool better = (kv > bk) || (kv == bk && rv < br);
          bv = better ? v : bv;
          bf = better ? fv : bf;
          br = better ? rv : br;
          bk = better ? kv : bk;
        }
        in |= 1ull << bv;
        link(bf, bv);
        const double wb = ws[bv][t];
        for (int u = 1; u < V; ++u) {
          if ((in >> u) & 1ull) continue;
          const double w = qfun(wb, ws[u][t], qmode);
          if (beats(w, bv, u, key[u][t], from[u][t], u, V)) {
            key[u][t] = w;
            from[u][t] = (unsigned char)bv;
          }
        }
      }
    }
  }
  for (int i = 0; i < V; ++i) {
    const unsigned long long row = adj[i][t];
    for (int j = 0; j < V; ++j) keep[((size_t)i * V + j) * n + p] = (unsigned char)((row >> j) & 1ull);
  }
}

// ---------------------------------------------------------------------------
// numpy PCG64 (XSL-RR 128/64) and Generator.permutation, replayed on the host
// ---------------------------------------------------------------------------
using u128 = unsigned __int128;

struct Pcg64 {
  u128 state, inc;
  int has32;
  uint32_t u32;
  uint64_t next64() {
    const u128 mult = ((u128)2549297995355413924ull << 64) | (u128)4865540595714422341ull;
    state = state * mult + inc;
    const uint64_t x = (uint64_t)(state >> 64) ^ (uint64_t)state;
    const unsigned rot = (unsigned)(state >> 122);
    return (x >> rot) | (x << ((64u - rot) & 63u));
  }
  uint32_t next32() {  // numpy buffers the high half of a 64-bit draw
    if (has32) {
      has32 = 0;
      return u32;
    }
    const uint64_t v = next64();
    has32 = 1;
    u32 = (uint32_t)(v >> 32);
    return (uint32_t)(v & 0xffffffffu);
  }
  // numpy random_interval: masked rejection sampling on [0, max]
  uint64_t interval(uint64_t max) {
    if (max == 0) return 0;
    uint64_t mask = max;
    mask |= mask >> 1;
    mask |= mask >> 2;
    mask |= mask >> 4;
    mask |= mask >> 8;
    mask |= mask >> 16;
    mask |= mask >> 32;
    uint64_t v;
    if (max <= 0xffffffffull) {
      while ((v = (next32() & mask)) > max) {
      }
    } else {
      while ((v = (next64() & mask)) > max) {
      }
    }
    return v;
  }
};

}  // namespace

extern "C" {

int admm_pixel_masks(const double* W, int V, int64_t n, int strategy, int k, int q_mode, const int32_t* orders,
                     uint8_t* keep, void* stream) {
  if (!W || !keep) return fail(ADMM_E_INVALID, "null argument");
  if (V < 2 || V > kMaxV) return fail(ADMM_E_INVALID, "V must be in [2, 64]");
  if (n < 1) return fail(ADMM_E_INVALID, "n must be >= 1");
  if (strategy != ADMM_MASK_KNN && strategy != ADMM_MASK_MST && strategy != ADMM_MASK_CHAIN)
    return fail(ADMM_E_INVALID, "strategy must be one of ADMM_MASK_KNN / _MST / _CHAIN");
  if (q_mode != ADMM_Q_ARITHMETIC && q_mode != ADMM_Q_HARMONIC) return fail(ADMM_E_INVALID, "bad q_mode");
  if (strategy == ADMM_MASK_KNN && k < 0) return fail(ADMM_E_INVALID, "k must be >= 0");
  if (strategy == ADMM_MASK_CHAIN && !orders) return fail(ADMM_E_INVALID, "chain strategy needs orders");
  const int T = V <= 16 ? 256 : V <= 32 ? 128 : 64;
  const long long blocks = (n + T - 1) / T;
  if (blocks > 0x7fffffffll) return fail(ADMM_E_INVALID, "n too large");
  hipStream_t s = (hipStream_t)stream;
  const int* ord = (const int*)orders;
  unsigned char* kp = (unsigned char*)keep;
  if (V <= 16)
    hipLaunchKernelGGL((k_pixel_masks<16, 256>), dim3((unsigned)blocks), dim3(256), 0, s, W, V, (long long)n,
                       strategy, k, q_mode, ord, kp);
  else if (V <= 32)
    hipLaunchKernelGGL((k_pixel_masks<32, 128>), dim3((unsigned)blocks), dim3(128), 0, s, W, V, (long long)n,
                       strategy, k, q_mode, ord, kp);
  else
    hipLaunchKernelGGL((k_pixel_masks<64, 64>), dim3((unsigned)blocks), dim3(64), 0, s, W, V, (long long)n,
                       strategy, k, q_mode, ord, kp);
  MHIPCHK(hipGetLastError());
  return ADMM_OK;
}

int admm_chain_orders(const uint64_t pcg[4], int has_uint32, uint32_t uinteger, int V, int64_t n, int32_t* orders,
                      uint64_t pcg_out[6]) {
  if (!pcg || !orders) return fail(ADMM_E_INVALID, "null argument");
  if (V < 1 || n < 0) return fail(ADMM_E_INVALID, "bad V or n");
  Pcg64 g;
  g.state = ((u128)pcg[0] << 64) | (u128)pcg[1];
  g.inc = ((u128)pcg[2] << 64) | (u128)pcg[3];
  g.has32 = has_uint32 ? 1 : 0;
  g.u32 = uinteger;
  for (int64_t p = 0; p < n; ++p) {
    int32_t* a = orders + (size_t)p * V;
    for (int i = 0; i < V; ++i) a[i] = i;  // np.arange(V)
    for (int i = V - 1; i >= 1; --i) {     // Generator.shuffle: reversed(range(1, n))
      const int j = (int)g.interval((uint64_t)i);
      const int32_t tmp = a[i];
      a[i] = a[j];
      a[j] = tmp;
    }
  }
  if (pcg_out) {
    pcg_out[0] = (uint64_t)(g.state >> 64);
    pcg_out[1] = (uint64_t)g.state;
    pcg_out[2] = (uint64_t)(g.inc >> 64);
    pcg_out[3] = (uint64_t)g.inc;
    pcg_out[4] = (uint64_t)g.has32;
    pcg_out[5] = (uint64_t)g.u32;
  }
  return ADMM_OK;
}

}  // extern "C"
