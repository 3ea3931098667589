// Probe: does buffer_load_dwordx4 ... lds (LDS-DMA through a raw buffer resource) write
// zeros to LDS for out-of-range lanes (negative voffset wrapped to 2^32-x, and offsets past
// num_records)?  Build: hipcc --offload-arch=gfx950 -O3 dma_oob.hip -o dma_oob
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __attribute__((address_space(3))) void lds_void;

__global__ void k(const float* src, float* out) {
  __shared__ float s[2 * 256];  // two 1-KiB pieces
  const int l = threadIdx.x;
  for (int i = l; i < 512; i += 64) s[i] = 7.0f;
  __syncthreads();
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, 1024, 0x00020000);
  // piece 0: lanes 0..15 negative offsets, the rest in range
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)&s[0], 16, (unsigned)(l * 16 - 256), 0, 0, 0);
  // piece 1: lanes whose offset is >= 1024 are past num_records
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)&s[256], 16, (unsigned)(l * 16 + 512), 0, 0, 0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int i = l; i < 512; i += 64) out[i] = s[i];
}

int main() {
  float h[1024], *d, *o, ho[512];
  for (int i = 0; i < 1024; ++i) h[i] = 1.0f + i;
  hipMalloc(&d, sizeof h);
  hipMalloc(&o, sizeof ho);
  hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
  k<<<1, 64>>>(d, o);
  if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 2; }
  hipMemcpy(ho, o, sizeof ho, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int lane = 0; lane < 64; ++lane)
    for (int c = 0; c < 4; ++c) {
      const int off0 = lane * 16 - 256, off1 = lane * 16 + 512;
      const float e0 = (off0 < 0) ? 0.0f : h[off0 / 4 + c];
      const float e1 = (off1 + 16 > 1024) ? 0.0f : h[off1 / 4 + c];
      if (ho[lane * 4 + c] != e0 || ho[256 + lane * 4 + c] != e1) {
        if (bad < 8) printf("lane %d c %d: got %g / %g want %g / %g\n", lane, c, ho[lane * 4 + c], ho[256 + lane * 4 + c], e0, e1);
        ++bad;
      }
    }
  printf("dma_oob: %s (%d mismatches)\n", bad ? "OOB lanes NOT zero-filled as expected" : "OOB lanes zero-filled", bad);
  return 0;
}
