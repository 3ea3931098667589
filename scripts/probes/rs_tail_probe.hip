// Probe: block_reduce_flat<NT, 16> (unpadded NA + NB tail) against the padded
// block_reduce_rs<NV, 16> on the same random inputs, 1024-thread blocks (the back
// projector's shape); prints the worst bit mismatch per value index.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o rs_tail_probe rs_tail_probe.hip
#include "../../distributed-inverse-problem-admm_amd/csrc/kernels.hpp"

#include <cstdio>
#include <cstdlib>
#include <cstring>

using namespace admm;

template <int NT, bool SPLIT>
__global__ __launch_bounds__(1024) void k_probe(const double* in, double* out) {
  constexpr int NS = SPLIT ? RsShape<NT>::NS : ((NT + 15) / 16) * 16;
  __shared__ double lds[16 * NS];
  __shared__ double tot[NS];
  double v[NT];
#pragma unroll
  for (int k = 0; k < NT; ++k) v[k] = in[((size_t)blockIdx.x * NT + k) * 1024 + threadIdx.x];
  if constexpr (SPLIT) {
    block_reduce_flat<NT, 16>(v, lds, tot);
  } else {
    constexpr int NV = ((NT + 15) / 16) * 16;
    double f[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) f[k] = k < NT ? v[k] : 0.0;
    block_reduce_rs<NV, 16>(f, lds, tot);
  }
  if ((int)threadIdx.x < NT) out[blockIdx.x * NT + threadIdx.x] = tot[threadIdx.x];
}

template <int NT>
int run() {
  const int B = 64;
  const size_t n = (size_t)B * NT * 1024;
  double* h = (double*)malloc(n * 8);
  srand(7);
  for (size_t i = 0; i < n; ++i) h[i] = (rand() / (double)RAND_MAX - 0.5) * (1 + (i % 97));
  double *d, *o1, *o2;
  hipMalloc(&d, n * 8);
  hipMalloc(&o1, B * NT * 8);
  hipMalloc(&o2, B * NT * 8);
  hipMemcpy(d, h, n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL((k_probe<NT, true>), dim3(B), dim3(1024), 0, 0, d, o1);
  hipLaunchKernelGGL((k_probe<NT, false>), dim3(B), dim3(1024), 0, 0, d, o2);
  double r1[B * NT], r2[B * NT];
  hipMemcpy(r1, o1, sizeof r1, hipMemcpyDeviceToHost);
  hipMemcpy(r2, o2, sizeof r2, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < B * NT; ++i) {
    // the exact sum of the block's 1024 inputs of value i % NT, for scale
    if (memcmp(&r1[i], &r2[i], 8) != 0) {
      if (bad < 8) printf("NT=%d block %d value %d: split %.17g padded %.17g\n", NT, i / NT, i % NT, r1[i], r2[i]);
      ++bad;
    }
  }
  printf("NT=%d (NA %d + NB %d): %d of %d totals differ\n", NT, RsShape<NT>::NA, RsShape<NT>::NB, bad, B * NT);
  hipFree(d);
  hipFree(o1);
  hipFree(o2);
  free(h);
  return bad;
}

int main() {
  int bad = run<20>() + run<40>() + run<18>() + run<17>();
  return bad ? 1 : 0;
}
