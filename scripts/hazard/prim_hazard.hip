// Device harness: both Prim forms of prim_select.h inside a k_pixel_masks-shaped kernel
// (one thread per pixel, per-thread LDS columns, early return, no barriers), compared
// with the host result of the same code.  Root-cause study of DESIGN.md's round-1
// "codegen hazard" note.  Build: hipcc --offload-arch=gfx950 -O3 prim_hazard.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <random>
#include <vector>
#define HD __host__ __device__
#include "prim_select.h"

template <bool BRANCHY, int MAXV, int T>
__global__ __launch_bounds__(T) void k_prim(const double* __restrict__ W, int V, long long n,
                                            unsigned long long* __restrict__ out) {
  __shared__ double ws[MAXV][T];
  __shared__ double key[MAXV][T];
  __shared__ unsigned char from[MAXV][T];
  __shared__ unsigned long long adj[MAXV][T];
  const int t = threadIdx.x;
  const long long p = (long long)blockIdx.x * T + t;
  if (p >= n) return;
  for (int i = 0; i < V; ++i) ws[i][t] = W[(size_t)i * n + p];
  auto Wd = [&](int v) -> double { return ws[v][t]; };
  auto K = [&](int v) -> double& { return key[v][t]; };
  auto F = [&](int v) -> unsigned char& { return from[v][t]; };
  auto Ad = [&](int v) -> unsigned long long& { return adj[v][t]; };
  prim<BRANCHY>(Wd, V, K, F, Ad);
  for (int i = 0; i < V; ++i) out[(size_t)i * n + p] = adj[i][t];
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 2; } } while (0)

int main() {
  const long long n = 1 << 16;
  std::mt19937_64 rng(7);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  long bad_b = 0, bad_f = 0, trees = 0;
  for (int V : {3, 5, 16, 33, 64}) {
    std::vector<double> W((size_t)V * n);
    for (size_t i = 0; i < W.size(); ++i) W[i] = (i % 3 == 0) ? double(rng() % 4) : U(rng);
    double* dW;
    unsigned long long* dA;
    CK(hipMalloc(&dW, W.size() * 8));
    CK(hipMalloc(&dA, (size_t)V * n * 8));
    CK(hipMemcpy(dW, W.data(), W.size() * 8, hipMemcpyHostToDevice));
    std::vector<unsigned long long> Ab((size_t)V * n), Af((size_t)V * n);
    k_prim<true, 64, 32><<<n / 32, 32>>>(dW, V, n, dA);
    CK(hipGetLastError());
    CK(hipMemcpy(Ab.data(), dA, Ab.size() * 8, hipMemcpyDeviceToHost));
    k_prim<false, 64, 32><<<n / 32, 32>>>(dW, V, n, dA);
    CK(hipGetLastError());
    CK(hipMemcpy(Af.data(), dA, Af.size() * 8, hipMemcpyDeviceToHost));
    long vb = 0, vf = 0;
    for (long long p = 0; p < n; ++p) {
      double w[64], key[64];
      unsigned char from[64];
      unsigned long long ref[64];
      for (int i = 0; i < V; ++i) w[i] = W[(size_t)i * n + p];
      auto Kh = [&](int v) -> double& { return key[v]; };
      auto Fh = [&](int v) -> unsigned char& { return from[v]; };
      prim<false>([&](int v) -> double { return w[v]; }, V, Kh, Fh,
                  [&](int v) -> unsigned long long& { return ref[v]; });
      bool eb = false, ef = false;
      for (int i = 0; i < V; ++i) {
        eb |= Ab[(size_t)i * n + p] != ref[i];
        ef |= Af[(size_t)i * n + p] != ref[i];
      }
      vb += eb;
      vf += ef;
    }
    printf("V=%2d: branchy form wrong on %ld of %lld pixels, branch-free wrong on %ld\n", V, vb, n, vf);
    bad_b += vb;
    bad_f += vf;
    trees += n;
    CK(hipFree(dW));
    CK(hipFree(dA));
  }
  printf("total: branchy %ld, branch-free %ld of %ld\n", bad_b, bad_f, trees);
  return 0;
}
