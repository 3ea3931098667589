// kernels.hpp -- CDNA4 (gfx950) kernels of the decentralized-ADMM tomography hot path.
//
// Everything is batched over the graph nodes this GPU owns.  All nodes share one
// parallel-beam geometry (block_2_load_odl_data.py:51: every node spans [0, pi)
// with its own a angles), so one launch projects VB node images at once: the
// per-step geometry (interpolation position, weights, clamped offsets) is computed
// once and reused VB times.
//
// "Sample" buffers (projector inputs / outputs: p, p^T, Hp, x_s, sinograms) are
// node-interleaved:  element (node v, pixel-or-ray q) lives at
//     [(v / VB) * L + q] * VB + (v % VB)          (L = pixels or rays)
// so a tap loads the VB nodes' values of one pixel with 16-byte vector loads
// (buffer_load_dwordx4) instead of VB separate dword loads.  VB = 1 is the plain
// node-major layout (operator API).  Solver state (x, r, d, e, y, z, q) is float64
// node-major [V][n].
//
// Numerics (DESIGN.md "Numerics"):
//   * samples are T = float (C2-C4) or double (C5);
//   * interpolation positions are evaluated in float64 (a float32 position has
//     3e-5 absolute error at N = 512, which would perturb the operator ~1e-5);
//   * x, r, d, e, y, z are float64;
//   * every reduction is a fixed-order tree over fixed partial slots: bitwise
//     reproducible and independent of how the graph is sharded over GPUs.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace admm {

constexpr int kBlock = 256;
constexpr int kTile = 32;        // elementwise / transposing kernels: 32x32 pixel tiles, block 32 x 8
constexpr int kFwdRays = 64;     // forward-projector block: 64 rays x 8 step segments (512 threads)
constexpr int kFwdSegs = 8;
constexpr int kFwdBlock = kFwdRays * kFwdSegs;

// Per-angle forward-projector constants (host-computed in float64).
// Ray (t,k), step m:  l = A0 + k*A1 + m*dl  (interpolation coordinate).
struct FwdAngle {
  double A0, A1, dl;
  double L;   // path length per step h/|alpha|
  int caseA;  // 1: step over axis-1 index on the transposed image
  int pad;
};
// Per-angle back-projector constants: fractional bin k_f = B0 + i*Bi + j*Bj,
// weight(k) = max(0, 1 - |k-k_f|*slope) * L.
struct BackAngle {
  double B0, Bi, Bj;
  double slope, L;
};

// Compact per-angle record of the back projector's hot loop (one s_load_dwordx8):
// k_f = (i - c0) Bi + (j - c0) Bj + K with K = -det_min/hd - 1/2 the same for every
// angle; float32 weights w0 = max(0, L - f sL), w1 = max(0, (L - sL) + f sL), formed
// as one packed fma (f, f) * ws + wc with ws = (-sL, sL), wc = (L, L - sL).
typedef float float2v __attribute__((ext_vector_type(2)));
struct alignas(32) BackAngleC {
  double Bi, Bj;
  float2v ws, wc;
};

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return min(max(v, lo), hi); }

// Float back-projector taps take k_f + 2^20 (k_f in (0, 2^20): kbias makes it positive, N <= 4096
// keeps it small), so the sum lies in [2^20, 2^21): its high dword is 0x41300000 + floor(k_f) and
// its low dword is frac(k_f) x 2^32.  A tap then needs no v_fract_f64 / v_cvt_i32_f64 /
// v_cvt_f32_f64: the weights take one v_cvt_f32_u32 of the low dword (the host scales the angle
// records' ws by 2^-32) and the LDS address is one v_lshl_add of the high dword onto a window
// offset stored with -0x41300000 x sizeof(sample vector) folded in (mod 2^32).  Position
// resolution 2^-32 bin, the forward's 32.32 fixed point.
constexpr double kKfBias = 1048576.0;
constexpr unsigned kKfHi = 0x41300000u;
__device__ __forceinline__ void kf_split(double kfb, unsigned& hi, float& fu) {
  const uint64_t b = __builtin_bit_cast(uint64_t, kfb);
  hi = (unsigned)(b >> 32);
  fu = (float)(unsigned)b;  // frac(k_f) x 2^32
}
// hi x PB + koff in one v_lshl_add_u32 (written out: the compiler forms hi << 4 from the 64-bit
// value by a funnel shift, a mask and an add); PB = the window's sample-vector bytes
template <int PB>
__device__ __forceinline__ int kf_addr(unsigned hi, int koff) {
  static_assert(PB == 4 || PB == 8 || PB == 16 || PB == 32, "power-of-two sample vectors");
  constexpr int SH = PB == 4 ? 2 : PB == 8 ? 3 : PB == 16 ? 4 : 5;
  int off;
  asm("v_lshl_add_u32 %0, %1, %2, %3" : "=v"(off) : "v"(hi), "i"(SH), "v"(koff));
  return off;
}

// ---------------------------------------------------------------------------
// vector I/O of VB samples (VB*sizeof(T) contiguous bytes)
// ---------------------------------------------------------------------------
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}

template <typename T, int VB>
__device__ __forceinline__ void vload(__amdgpu_buffer_rsrc_t r, int voff, int soff, T (&o)[VB]) {
  constexpr int BYTES = VB * (int)sizeof(T);
  if constexpr (BYTES >= 16) {
    constexpr int PER = 16 / (int)sizeof(T);
#pragma unroll
    for (int q = 0; q < BYTES / 16; ++q) {
      auto v = __builtin_amdgcn_raw_buffer_load_b128(r, voff + 16 * q, soff, 0);
      T t[PER];
      __builtin_memcpy(t, &v, 16);
#pragma unroll
      for (int e = 0; e < PER; ++e) o[q * PER + e] = t[e];
    }
  } else if constexpr (BYTES == 8) {
    auto v = __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0);
    __builtin_memcpy(o, &v, 8);
  } else {
    auto v = __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0);
    __builtin_memcpy(o, &v, 4);
  }
}

template <typename T, int VB>
struct alignas((VB * sizeof(T)) >= 16 ? 16 : (VB * sizeof(T))) Pack {
  T v[VB];
};

template <typename T, int VB>
struct Planes {
  static constexpr int BYTES = VB * (int)sizeof(T);
  static constexpr int NPL = BYTES > 16 ? BYTES / 16 : 1;  // 16-byte planes
  static constexpr int PV = VB / NPL;                      // values per plane
};

template <typename T, int VB>
__device__ __forceinline__ void gload(const T* __restrict__ p, T (&o)[VB]) {
  const Pack<T, VB> k = *reinterpret_cast<const Pack<T, VB>*>(p);
#pragma unroll
  for (int u = 0; u < VB; ++u) o[u] = k.v[u];
}
template <typename T, int VB>
__device__ __forceinline__ void gstore(T* __restrict__ p, const T (&o)[VB]) {
  Pack<T, VB> k;
#pragma unroll
  for (int u = 0; u < VB; ++u) k.v[u] = o[u];
  *reinterpret_cast<Pack<T, VB>*>(p) = k;
}

// ---------------------------------------------------------------------------
// deterministic block reduction of NQ float64 values per thread (256 threads);
// result valid in thread 0.  Fixed shuffle tree + fixed LDS order.
// ---------------------------------------------------------------------------
// float64 lane exchange by DPP (two 32-bit moves); CTRL must describe an exact xor pairing
template <int CTRL>
__device__ __forceinline__ double dpp_d(double x) {
  const uint64_t b = __builtin_bit_cast(uint64_t, x);
  const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)b, CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(b >> 32), CTRL, 0xf, 0xf, false);
  return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
// x, y := the permlane swap of x and y (per 32-bit half): SWAP32 exchanges lanes 32-63 of x
// with lanes 0-31 of y, otherwise odd 16-lane rows of x with even rows of y
template <bool SWAP32>
__device__ __forceinline__ void permswap_d(double& x, double& y) {
  const uint64_t bx = __builtin_bit_cast(uint64_t, x), by = __builtin_bit_cast(uint64_t, y);
  uint32_t xl = (uint32_t)bx, xh = (uint32_t)(bx >> 32), yl = (uint32_t)by, yh = (uint32_t)(by >> 32);
  if constexpr (SWAP32) {
    const auto l = __builtin_amdgcn_permlane32_swap(xl, yl, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap(xh, yh, false, false);
    xl = l[0]; yl = l[1]; xh = h[0]; yh = h[1];
  } else {
    const auto l = __builtin_amdgcn_permlane16_swap(xl, yl, false, false);
    const auto h = __builtin_amdgcn_permlane16_swap(xh, yh, false, false);
    xl = l[0]; yl = l[1]; xh = h[0]; yh = h[1];
  }
  x = __builtin_bit_cast(double, ((uint64_t)xh << 32) | xl);
  y = __builtin_bit_cast(double, ((uint64_t)yh << 32) | yl);
}
// s + (s of lane ^ 32, 16, 8, 4, 2, 1): every lane ends with the wave total, the same sums in
// the same order as the __shfl_xor butterfly (a + b == b + a), without LDS round trips
__device__ __forceinline__ double wave_sum_d(double s) {
  const int lane = threadIdx.x & 63;
  double x = s, y = s;
  permswap_d<true>(x, y);  // x + y = s[i] + s[i ^ 32] in every lane
  s = x + y;
  x = s, y = s;
  permswap_d<false>(x, y);
  s = x + y;
  s += dpp_d<0x128>(s);  // row_ror:8 = xor 8
  const double up = dpp_d<0x104>(s), dn = dpp_d<0x114>(s);  // xor 4: row_shl:4 / row_shr:4
  s += (lane & 4) ? dn : up;
  s += dpp_d<0x4E>(s);  // quad_perm [2,3,0,1]
  s += dpp_d<0xB1>(s);  // quad_perm [1,0,3,2]
  return s;
}

template <int NQ>
__device__ __forceinline__ void block_reduce(double (&v)[NQ], double* lds /* >= 4*NQ */) {
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    v[q] = wave_sum_d(v[q]);
  }
  const int wid = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) lds[wid * NQ + q] = v[q];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) v[q] = ((lds[q] + lds[NQ + q]) + (lds[2 * NQ + q] + lds[3 * NQ + q]));
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// deterministic block reduction of NV (multiple of 16) float64 values per thread
// by a wave-level reduce-scatter butterfly: at offsets 32, 16, 8, 4 every lane
// keeps half of its values and adds its partner's copy of that half (NV/2 + NV/4
// + NV/8 + NV/16 exchanges instead of 6*NV), then a plain butterfly over offsets
// 2, 1 on the last NV/16.  Exchanges are gfx950 permlane32/16 swaps (offsets 32, 16)
// and DPP row moves (8, 4, 2, 1): every level an exact xor pairing, so the totals are
// the __shfl_xor butterfly's bit for bit (profiles/r2_reduce_dpp_bitwise.txt).  Lanes with (lane & 3) == 0 then hold the wave totals;
// the NW waves are combined in LDS in a fixed pairwise tree.  On return thread t < NV of the
// block can read total t from out_lds[t].  Fixed order -> bitwise reproducible.
// ---------------------------------------------------------------------------
// the wave part: on return the lanes with (lane & 3) == 0 hold NV / 16 wave totals each, of
// the values base .. base + NV/16 - 1 (base returned)
template <int NV>
__device__ __forceinline__ int wave_rs(double (&v)[NV]) {
  static_assert(NV % 16 == 0, "NV must be a multiple of 16");
  const int lane = threadIdx.x & 63;
  // at offsets 32 and 16: after the swap, lane i of x + y is (keep + partner's send), with no
  // LDS traffic and no selects
#pragma unroll
  for (int k = 0; k < NV / 2; ++k) {
    double x = v[k], y = v[NV / 2 + k];
    permswap_d<true>(x, y);
    v[k] = x + y;
  }
#pragma unroll
  for (int k = 0; k < NV / 4; ++k) {
    double x = v[k], y = v[NV / 4 + k];
    permswap_d<false>(x, y);
    v[k] = x + y;
  }
  const bool h8 = lane & 8, h4 = lane & 4;
#pragma unroll
  for (int k = 0; k < NV / 8; ++k) {  // xor 8 = row_ror:8 within a 16-lane row
    const double send = h8 ? v[k] : v[NV / 8 + k];
    const double keep = h8 ? v[NV / 8 + k] : v[k];
    v[k] = keep + dpp_d<0x128>(send);
  }
#pragma unroll
  for (int k = 0; k < NV / 16; ++k) {  // xor 4: row_shl:4 for lanes with bit 2 clear, row_shr:4 else
    const double send = h4 ? v[k] : v[NV / 16 + k];
    const double keep = h4 ? v[NV / 16 + k] : v[k];
    const double up = dpp_d<0x104>(send), dn = dpp_d<0x114>(send);
    v[k] = keep + (h4 ? dn : up);
  }
#pragma unroll
  for (int k = 0; k < NV / 16; ++k) {  // xor 2, xor 1: quad_perm [2,3,0,1], [1,0,3,2]
    double s = v[k];
    s += dpp_d<0x4E>(s);
    s += dpp_d<0xB1>(s);
    v[k] = s;
  }
  return ((lane >> 5) & 1) * (NV / 2) + ((lane >> 4) & 1) * (NV / 4) + ((lane >> 3) & 1) * (NV / 8) +
         ((lane >> 2) & 1) * (NV / 16);
}

// NB (1, 2, 4 or 8) values: halving exchanges while more than one value remains, then the plain
// butterfly over the remaining offsets (the same exact-xor pairing at every level, so each total
// is the full butterfly's bit for bit).  Every lane returns the total of value *idx; the lanes
// with (lane & (64 / NB - 1)) == 0 are one writer per value.
template <int NB>
__device__ __forceinline__ double wave_rs_tail(double (&t)[NB], int& idx) {
  static_assert(NB == 1 || NB == 2 || NB == 4 || NB == 8, "tail of 1, 2, 4 or 8 values");
  const int lane = threadIdx.x & 63;
  if constexpr (NB >= 2) {
#pragma unroll
    for (int k = 0; k < NB / 2; ++k) {
      double x = t[k], y = t[NB / 2 + k];
      permswap_d<true>(x, y);
      t[k] = x + y;
    }
  }
  if constexpr (NB >= 4) {
#pragma unroll
    for (int k = 0; k < NB / 4; ++k) {
      double x = t[k], y = t[NB / 4 + k];
      permswap_d<false>(x, y);
      t[k] = x + y;
    }
  }
  double s = t[0];
  if constexpr (NB >= 8) {
    const bool h8 = lane & 8;
    const double send = h8 ? t[0] : t[1], keep = h8 ? t[1] : t[0];
    s = keep + dpp_d<0x128>(send);
  }
  if constexpr (NB < 2) {
    double x = s, y = s;
    permswap_d<true>(x, y);
    s = x + y;
  }
  if constexpr (NB < 4) {
    double x = s, y = s;
    permswap_d<false>(x, y);
    s = x + y;
  }
  if constexpr (NB < 8) s += dpp_d<0x128>(s);
  const double up = dpp_d<0x104>(s), dn = dpp_d<0x114>(s);  // xor 4
  s += (lane & 4) ? dn : up;
  s += dpp_d<0x4E>(s);
  s += dpp_d<0xB1>(s);
  idx = (NB >= 2 ? ((lane >> 5) & 1) * (NB / 2) : 0) + (NB >= 4 ? ((lane >> 4) & 1) * (NB / 4) : 0) +
        (NB >= 8 ? ((lane >> 3) & 1) * (NB / 8) : 0);
  return s;
}

// the NW wave totals of value t (stride NS in lds) combined in a fixed pairwise tree
template <int NS, int NW>
__device__ __forceinline__ void block_combine(const double* lds, double* out_lds) {
  if ((int)threadIdx.x < NS) {
    const int t = threadIdx.x;
    double w[NW];
#pragma unroll
    for (int q = 0; q < NW; ++q) w[q] = lds[q * NS + t];
#pragma unroll
    for (int h = NW / 2; h >= 1; h >>= 1)
#pragma unroll
      for (int q = 0; q < h; ++q) w[q] = w[2 * q] + w[2 * q + 1];
    out_lds[t] = w[0];
  }
}

// ---------------------------------------------------------------------------
// deterministic block reduction of NV (multiple of 16) float64 values per thread
// by a wave-level reduce-scatter butterfly: at offsets 32, 16, 8, 4 every lane
// keeps half of its values and adds its partner's copy of that half (NV/2 + NV/4
// + NV/8 + NV/16 exchanges instead of 6*NV), then a plain butterfly over offsets
// 2, 1 on the last NV/16.  Exchanges are gfx950 permlane32/16 swaps (offsets 32, 16)
// and DPP row moves (8, 4, 2, 1): every level an exact xor pairing, so the totals are
// the __shfl_xor butterfly's bit for bit (profiles/r2_reduce_dpp_bitwise.txt).  Lanes with (lane & 3) == 0 then hold the wave totals;
// the NW waves are combined in LDS in a fixed pairwise tree.  On return thread t < NV of the
// block can read total t from out_lds[t].  Fixed order -> bitwise reproducible.
// ---------------------------------------------------------------------------
template <int NV, int NW = 4>
__device__ __forceinline__ void block_reduce_rs(double (&v)[NV], double* lds /* >= NW*NV */,
                                                double* out_lds /* >= NV */) {
  static_assert(NW == 4 || NW == 8 || NW == 16, "NW = 4, 8 or 16 waves");
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int base = wave_rs<NV>(v);
  if ((lane & 3) == 0) {
#pragma unroll
    for (int k = 0; k < NV / 16; ++k) lds[wid * NV + base + k] = v[k];
  }
  __syncthreads();
  block_combine<NV, NW>(lds, out_lds);
  __syncthreads();
}

// NA (multiple of 16) + NB (1, 2, 4 or 8) values without padding NA + NB up to a multiple of
// 16 (round 6: 20 = 16 + 4 CG dot partials of a 4-node back-projector lane block, 42 fewer
// VALU per thread than the padded 32): each value's total is the same butterfly, bit for bit,
// and the waves are combined in the same tree, so out_lds[t], t < NA + NB, is block_reduce_rs'
// result for the padded vector.
template <int NA, int NB, int NW>
__device__ __forceinline__ void block_reduce_rs_tail(double (&v)[NA], double (&tb)[NB], double* lds /* >= NW*(NA+NB) */,
                                                     double* out_lds /* >= NA+NB */) {
  static_assert(NW == 4 || NW == 8 || NW == 16, "NW = 4, 8 or 16 waves");
  constexpr int NS = NA + NB;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int base = wave_rs<NA>(v);
  int ti;
  const double ts = wave_rs_tail<NB>(tb, ti);
  if ((lane & 3) == 0) {
#pragma unroll
    for (int k = 0; k < NA / 16; ++k) lds[wid * NS + base + k] = v[k];
  }
  if ((lane & (64 / NB - 1)) == 0) lds[wid * NS + NA + ti] = ts;
  __syncthreads();
  block_combine<NS, NW>(lds, out_lds);
  __syncthreads();
}

// The block's NT = NQ x (lane-block nodes) dot partials per thread (pq flattened node-major)
// reduced to out_lds[0 .. NT): unpadded NA + NB when NT is 16k + 1, 2, 4 or 8 (k >= 1),
// otherwise padded to a multiple of 16 -- the same totals either way
#ifndef ADMM_RS_TAIL
#define ADMM_RS_TAIL 1  // 0: always the padded form (A/B builds)
#endif
template <int NT>
struct RsShape {
  static constexpr int NA = (NT / 16) * 16, NB = NT - NA;
  static constexpr bool SPLIT = ADMM_RS_TAIL && NA >= 16 && (NB == 1 || NB == 2 || NB == 4 || NB == 8);
  static constexpr int NS = SPLIT ? NT : ((NT + 15) / 16) * 16;  // LDS stride / out_lds size
};
template <int NT, int NW>
__device__ __forceinline__ void block_reduce_flat(const double (&vals)[NT], double* lds, double* out_lds) {
  using S = RsShape<NT>;
  if constexpr (S::SPLIT) {
    double fa[S::NA], fb[S::NB];
#pragma unroll
    for (int k = 0; k < S::NA; ++k) fa[k] = vals[k];
#pragma unroll
    for (int k = 0; k < S::NB; ++k) fb[k] = vals[S::NA + k];
    block_reduce_rs_tail<S::NA, S::NB, NW>(fa, fb, lds, out_lds);
  } else {
    constexpr int NV = ((NT + 15) / 16) * 16;
    double flat[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) flat[k] = k < NT ? vals[k] : 0.0;
    block_reduce_rs<NV, NW>(flat, lds, out_lds);
  }
}

// ===========================================================================
// Forward projector (Joseph, ray-driven):  sino[v][t][k] = sum_m L * interp(img_v, row m, l(m))
// Replaces the ODL RayTransform `Ai @ x` (block_2_load_odl_data.py:54, dense form :68-96;
// used at block_5_node_problem.py:21 and block_6_admm_loop_ver2.py:193).
//
// Block = 64 consecutive detector bins of one angle x 8 step segments (one wave each).
// Lanes are consecutive rays, so at every step a wave reads one contiguous row segment:
// case-B angles read img (row m = axis-0 index), case-A angles read the transposed
// copy imgT (row m = axis-1 index).  Each tap is one VB-vector load (VB nodes).
// The 8 segment partial sums are combined in LDS in fixed order.
// MODE 0: store A x (interleaved).
// MODE 1: store s = A x - b (interleaved; b node-major [V][m]) and partials of ||s||^2.
// ===========================================================================
template <typename T, int VB, int MODE>
__global__ __launch_bounds__(kFwdBlock) void k_fwd(const T* __restrict__ img, const T* __restrict__ imgT,
                                                T* __restrict__ sino, const T* __restrict__ bsino,
                                                double* __restrict__ part, const FwdAngle* __restrict__ ang,
                                                int N, int n_det, int n_ang, int V) {
  const int lane = threadIdx.x & 63;
  const int seg = threadIdx.x >> 6;
  const int k = blockIdx.x * kFwdRays + lane;
  const int t = blockIdx.y;
  const int chunk = blockIdx.z;
  const int v0 = chunk * VB;
  const int nv = min(VB, V - v0);
  const int npix = N * N;
  const int nch = (V + VB - 1) / VB;
  const FwdAngle a = ang[t];
  const T* src = a.caseA ? imgT : img;
  const __amdgpu_buffer_rsrc_t rs = make_rsrc(src, (uint32_t)((size_t)nch * npix * VB * sizeof(T)));
  const int soff = chunk * npix * VB * (int)sizeof(T);
  T acc[VB];
#pragma unroll
  for (int u = 0; u < VB; ++u) acc[u] = T(0);

  if (k < n_det) {
    const double l0 = fma((double)k, a.A1, a.A0);
    // steps whose interpolation coordinate lies in (-1, N); conservative, taps are predicated
    int mlo = 0, mhi = N - 1;
    if (fabs(a.dl) > 1e-12) {
      double ma = (-1.0 - l0) / a.dl, mb = ((double)N - l0) / a.dl;
      double lo = fmax(fmin(ma, mb), -1.0), hi = fmin(fmax(ma, mb), (double)N);
      mlo = max(0, (int)floor(lo));
      mhi = min(N - 1, (int)ceil(hi));
    } else if (!(l0 > -1.0 && l0 < (double)N)) {
      mlo = 1;
      mhi = 0;
    }
    const int segLen = (N + kFwdSegs - 1) / kFwdSegs;
    const int s0 = max(mlo, seg * segLen);
    const int s1 = min(mhi, seg * segLen + segLen - 1);
    // two steps per iteration: both steps' loads are in flight before the FMAs
    auto tap = [&](int m, T (&p0)[VB], T (&p1)[VB], T& w0, T& w1) {
      const double l = fma((double)m, a.dl, l0);
      const double fl = floor(l);
      const int i0 = (int)fl;
      w1 = (T)(l - fl);
      w0 = T(1) - w1;
      w0 = (i0 >= 0 && i0 <= N - 1) ? w0 : T(0);
      w1 = (i0 >= -1 && i0 <= N - 2) ? w1 : T(0);
      const int row = m * N;
      const int o0 = (row + clampi(i0, 0, N - 1)) * VB * (int)sizeof(T);
      const int o1 = (row + clampi(i0 + 1, 0, N - 1)) * VB * (int)sizeof(T);
      vload<T, VB>(rs, o0, soff, p0);
      vload<T, VB>(rs, o1, soff, p1);
    };
    int m = s0;
    for (; m + 1 <= s1; m += 2) {
      T a0[VB], a1[VB], b0[VB], b1[VB], wa0, wa1, wb0, wb1;
      tap(m, a0, a1, wa0, wa1);
      tap(m + 1, b0, b1, wb0, wb1);
#pragma unroll
      for (int u = 0; u < VB; ++u) {
        acc[u] = fma(wa0, a0[u], acc[u]);
        acc[u] = fma(wa1, a1[u], acc[u]);
        acc[u] = fma(wb0, b0[u], acc[u]);
        acc[u] = fma(wb1, b1[u], acc[u]);
      }
    }
    if (m <= s1) {
      T a0[VB], a1[VB], wa0, wa1;
      tap(m, a0, a1, wa0, wa1);
#pragma unroll
      for (int u = 0; u < VB; ++u) {
        acc[u] = fma(wa0, a0[u], acc[u]);
        acc[u] = fma(wa1, a1[u], acc[u]);
      }
    }
  }
  __shared__ T red[kFwdSegs][VB][kFwdRays];
#pragma unroll
  for (int u = 0; u < VB; ++u) red[seg][u][lane] = acc[u];
  __syncthreads();
  double sq[VB];
#pragma unroll
  for (int u = 0; u < VB; ++u) sq[u] = 0.0;
  if (seg == 0 && k < n_det) {
    const size_t ray = (size_t)t * n_det + k;
    T s[VB];
#pragma unroll
    for (int u = 0; u < VB; ++u) {
      s[u] = (((red[0][u][lane] + red[1][u][lane]) + (red[2][u][lane] + red[3][u][lane])) +
              ((red[4][u][lane] + red[5][u][lane]) + (red[6][u][lane] + red[7][u][lane]))) *
             (T)a.L;
      if (MODE == 1) {
        if (u < nv) {
          s[u] = s[u] - bsino[(size_t)(v0 + u) * n_ang * n_det + ray];
          sq[u] = (double)s[u] * (double)s[u];
        } else {
          s[u] = T(0);
        }
      }
    }
    gstore<T, VB>(sino + ((size_t)chunk * n_ang * n_det + ray) * VB, s);
  }
  if (MODE == 1 && seg == 0) {
    // only wave 0 holds residuals: one fixed-order wave reduction per node
#pragma unroll
    for (int u = 0; u < VB; ++u) {
      double v = sq[u];
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
      sq[u] = v;
    }
    if (lane == 0) {
      const int P = gridDim.x * gridDim.y;
      const int b = blockIdx.y * gridDim.x + blockIdx.x;
#pragma unroll
      for (int u = 0; u < VB; ++u)
        if (u < nv) part[(size_t)(v0 + u) * P + b] = sq[u];
    }
  }
}

// ===========================================================================
// Explicit-matrix forward (admm_ctx_create_matrix): sino = A x with A a CSR matrix
// (rows = sinogram entries in the reference's angle-major order, columns = C-order
// pixels), for operators given as matrices (the reference's A_dense_list,
// block_2_load_odl_data.py:68-96 / block_7_main.py:16-22) instead of a geometry.
// One thread per row over VB interleaved nodes; same outputs as k_fwd (MODE 0 / 1),
// ||s||^2 partials per 256-row block.
// ===========================================================================
template <typename T, int VB, int MODE>
__global__ __launch_bounds__(kBlock) void k_csr_fwd(const int* __restrict__ ptr, const int* __restrict__ idx,
                                                    const T* __restrict__ val, const T* __restrict__ img,
                                                    T* __restrict__ sino, const T* __restrict__ bsino,
                                                    double* __restrict__ part, int m, int npix, int V) {
  const int chunk = blockIdx.y, v0 = chunk * VB, nv = min(VB, V - v0);
  const int row = blockIdx.x * kBlock + threadIdx.x;
  const T* src = img + (size_t)chunk * npix * VB;
  double sq[VB];
#pragma unroll
  for (int u = 0; u < VB; ++u) sq[u] = 0.0;
  if (row < m) {
    T acc[VB], pv[VB];
#pragma unroll
    for (int u = 0; u < VB; ++u) acc[u] = T(0);
    for (int k = ptr[row]; k < ptr[row + 1]; ++k) {
      const T w = val[k];
      gload<T, VB>(src + (size_t)idx[k] * VB, pv);
#pragma unroll
      for (int u = 0; u < VB; ++u) acc[u] = fma(w, pv[u], acc[u]);
    }
    if (MODE == 1) {
#pragma unroll
      for (int u = 0; u < VB; ++u) {
        if (u < nv) {
          acc[u] = acc[u] - bsino[(size_t)(v0 + u) * m + row];
          sq[u] = (double)acc[u] * (double)acc[u];
        } else {
          acc[u] = T(0);
        }
      }
    }
    gstore<T, VB>(sino + ((size_t)chunk * m + row) * VB, acc);
  }
  if (MODE == 1) {
    __shared__ double lds[4 * VB];
    block_reduce<VB>(sq, lds);
    if (threadIdx.x == 0) {
#pragma unroll
      for (int u = 0; u < VB; ++u)
        if (u < nv) part[(size_t)(v0 + u) * gridDim.x + blockIdx.x] = sq[u];
    }
  }
}

// ===========================================================================
// Forward projector, angle-grouped (the hot-path version).
// Block = G <= kFgG consecutive angles of one case (one wave each) x up to 64 rays of
// each (its FgRange entry), over one of kFgSeg row segments.  Rows are processed in
// chunks (2 rows, LDS-DMA double buffer): for each row the block stages into LDS the
// window of image pixels (columns wlo .. wlo+kFgWin-1) that any of its rays can touch,
// zero-filled outside the image, then every ray takes its two taps per row from LDS.
// One staged pixel serves ~G x 1.4 x 2 taps, so L2 traffic drops ~G-fold and taps run
// at LDS rate.  The host plans groups and per-block ray ranges so every window fits
// (FgGroup / FgRange tables, three plans; admm_tomo.hip).  Segment partial sums go to
// part[seg][chunk][ray][VB] and k_fwd_combine adds them in fixed order.
//
// LDS bank conflicts.  Adjacent rays sit A1 in [1, 1.41] pixels apart, so a
// ds_read_b128 lane group of 16 rays spans up to ~23 pixels and, with one 16-B
// slot per pixel, wraps the 16 slots of the bank space (2-3-way conflicts).
// Each staged row is therefore split into its even and odd pixels (two
// half-windows, the odd one 64 B further so 8-lane staging writes stay
// conflict-free): a ray's taps {p, p+1} are one even and one odd pixel, the two
// reads of a row are "every lane's even tap" and "every lane's odd tap", and a
// 16-ray group needs <= 12 distinct slots of each.  Lanes are permuted so each
// hardware lane group ({0-3,12-15,20-27}, ...) holds 16 consecutive rays.
// ===========================================================================
#ifndef ADMM_FG_ROWS
#define ADMM_FG_ROWS 4
#endif
#ifndef ADMM_FG_SEG
#define ADMM_FG_SEG 8
#endif
#ifndef ADMM_FG_G
#define ADMM_FG_G 16
#endif
#ifndef ADMM_FG_WIN
#define ADMM_FG_WIN 256
#endif
constexpr int kFgRows = ADMM_FG_ROWS;  // rows staged per LDS chunk
constexpr int kFgG = ADMM_FG_G;        // max angles (waves) per block
constexpr int kFgThreads = 64 * kFgG;
constexpr int kFgWin = ADMM_FG_WIN;    // staged window width (pixels)
constexpr int kFgSeg = ADMM_FG_SEG;    // row segments (partial sums) per ray
#ifndef ADMM_FG_DMA_ROWS
#define ADMM_FG_DMA_ROWS 2  // rows per chunk of the LDS-DMA kernel (round 4: 4 rows 50.0 vs 51.2 us at C3, 28.2 vs 27.7 at 8 nodes)
#endif
constexpr int kFgHalf = kFgWin / 2;                // slots per parity
constexpr int kFgPieces = (kFgHalf + 63) / 64;     // 64-slot LDS-DMA pieces per parity half
constexpr int kFgOdd = 64 * kFgPieces + 4;         // odd half-window offset (+64 B bank shift)
constexpr int kFgRow = kFgOdd + 64 * kFgPieces;    // 16-B slots per staged row and plane

// ray (within a 64-ray chunk) of each lane: ds_read_b128 lane groups -> 16 consecutive rays
__device__ __forceinline__ int fg_ray_of_lane(int lane) {
  const int l = lane & 31;
  const int r = l < 4 ? l : l < 12 ? l + 12 : l < 16 ? l - 8 : l < 20 ? l + 8 : l < 28 ? l - 12 : l;
  return (lane & 32) + r;
}

// One angle group of the grouped forward projector: angles t0 .. t0+G-1 (one case).
struct FgGroup {
  int t0, G;
};
// The rays one block projects: angle t0+q of its group takes rays k0[q] .. k0[q]+nk[q]-1
// (0 <= nk <= 64, inside [0, n_det)).  Every plan is a table of these (one per (group,
// segment, chunk)); per (group, segment) the ranges of each angle partition its rays (less
// any ray a clipped plan drops because it misses the segment inside the image).  The
// 64-ray plans give angle q rays x*64 + delta_q + [0, 64), delta_q = 0 or the shift that
// makes every angle of the group cross the same pixels at the segment's centre row; the
// chunk-aligned plan starts every angle's chunk x at the same pixel of that row (a chunk
// spans 64 rays of the group's densest angle, so sparser angles use fewer lanes), which
// keeps the union window narrow far from the detector centre too.
struct FgRange {
  int k0[kFgG];
  int nk[kFgG];
};

// The float forward keeps its tap weights in the units of its 32.32 fixed-point positions
// (w1 = the fraction's low word as a float, w0 = 2^32 - w1: one VALU less per tap row than
// scaling each fraction by 2^-32), so its segment partials carry a factor 2^32 that the
// combines fold into L (kFgWScale).  Power-of-two scalings commute with rounding (no overflow
// or underflow at these magnitudes): every partial, sum and A x is bitwise what the unscaled
// weights gave.
template <typename T>
constexpr T kFgWOne = T(1);
template <>
constexpr float kFgWOne<float> = 4294967296.0f;
template <typename T>
constexpr T kFgWScale = T(1);
template <>
constexpr float kFgWScale<float> = 2.3283064365386963e-10f;

#ifndef ADMM_FG_WPE2
#define ADMM_FG_WPE2 8  // the same for two chunks per block (CPB = 2)
#endif
#ifndef ADMM_FG_WPE
#define ADMM_FG_WPE 8  // waves per SIMD the register budget must allow: <= 64 VGPRs, 2 blocks/CU
                       // (float64 samples otherwise take 67 and fall to one block per CU)
#endif
// MIRROR (the mirror-symmetric projection, admm_tomo.hip "mirror mode"): the geometry's angles
// are (t + 1/2) pi / a over [0, pi) with a symmetric detector, so angle a-1-t = pi - theta_t
// projects image I exactly as angle t projects flipud(I) (same detector order;
// tests/test_oracle.py::test_mirror_symmetry_of_the_joseph_operator).  A batch then projects
// VIRTUAL images over the first a/2 angles only: virtual lanes u < VB/2 are real node lanes at
// (i, j), lanes u >= VB/2 the same real nodes at (N-1-i, j).  The virtual image is never stored:
// staging reads the real node-interleaved buffers (VBR lanes per pixel) with the mirrored half
// taken from row N-1-m (case B, img) or column N-1-w (case A, img^T).  A narrow batch (4 float32
// nodes: VBR = 4) thereby projects 8-lane vectors -- the per-tap address / weight VALU is paid
// once per 8 lanes as in an 8-node batch -- and an 8-node batch runs two virtual chunks of
// half the angles (the same taps).  Virtual chunk c' = real chunk c' / S, lane block c' % S of
// VB/2 real lanes (S = 2 VBR / VB).
// CPB (round 6, mirror mode, float32): virtual chunks per block -- 2: one block projects the same
// rays of chunks 2p and 2p + 1 (ob.z carries the pair p), a tap row's position, weights and LDS
// slots formed once for both chunks' staged windows; the host uses it where the halved block
// table still fills every slot (fwd_cpb).  Per chunk the arithmetic is CPB = 1's, in the same
// order: bitwise the same partials.
template <typename T, int VB, bool MIRROR = false, int VBR = VB, int CPB = 1>
__global__ __launch_bounds__(kFgThreads) __attribute__((amdgpu_waves_per_eu(CPB == 1 ? ADMM_FG_WPE : ADMM_FG_WPE2))) void k_fwdg(const T* __restrict__ img, const T* __restrict__ imgT,
                                                 T* __restrict__ part, const FwdAngle* __restrict__ ang,
                                                 const FgGroup* __restrict__ groups, const FgRange* __restrict__ rng,
                                                 const int4* __restrict__ order, int N, int n_det, int n_ang, int V) {
  constexpr int NPL = Planes<T, VB>::NPL, PV = Planes<T, VB>::PV;
  constexpr int MH = VB / 2;                  // (MIRROR) real lanes per virtual chunk
  constexpr int MS = MIRROR ? VBR / MH : 1;   // (MIRROR) virtual chunks per real chunk
  static_assert(!MIRROR || (VB % 2 == 0 && VBR % MH == 0), "mirror: VB = 2 x (a divisor of VBR)");
  constexpr int PER = (kFgRows * kFgWin * NPL + kFgThreads - 1) / kFgThreads;  // staged packs per thread
  // g (the wave's angle slot) is wave-uniform: readfirstlane lets the compiler keep it, and
  // everything derived from it (group offsets, DMA piece indices, the idle test), in SGPRs
  // with scalar branches instead of VALU compares and EXEC masking
  const int lane = threadIdx.x & 63, g = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  // 1-D grid over a host-ordered block table (order[b] = {ray ranges, group, seg +
  // kFgSeg * node chunk}): heavy (large-G) blocks first, paired with light ones on a CU
  const int4 ob = order[blockIdx.x];
  const FgRange* rg = rng + ob.x;
  const FgGroup* gr = groups + ob.y;
  const int seg = ob.z % kFgSeg, chunk = (ob.z / kFgSeg) * CPB;  // (CPB: the pair's first chunk)
  const int G = gr->G, t0 = gr->t0;
  const int npix = N * N;
  const int gq = min(g, G - 1);
  // lanes past the angle's range repeat its last ray (taps inside the window, store masked)
  const int nkq = rg->nk[gq], rl = fg_ray_of_lane(lane);
  const int k = rg->k0[gq] + min(rl, nkq - 1);
  const int kcl = clampi(k, 0, n_det - 1);
  const int t = t0 + gq;
  const FwdAngle a = ang[t];
  const bool caseA = ang[t0].caseA != 0;
  // real buffer of this (virtual) chunk; MIRROR: real chunk chunk / MS, lane block mq
  const int mq = MIRROR ? chunk % MS : 0;
  const T* src = (caseA ? imgT : img) + (size_t)(MIRROR ? chunk / MS : chunk) * npix * VBR;
  const double l0 = fma((double)kcl, a.A1, a.A0);
  const int m_lo = seg * N / kFgSeg, m_hi = (seg + 1) * N / kFgSeg;
  const int nrows = m_hi - m_lo;

  // LDS-DMA staging (ADMM_FG_DMA): 16-byte sample planes land straight in LDS from a buffer
  // resource per staged row (out-of-image columns are out-of-range offsets: zero-filled by the
  // hardware, scripts/probes/dma_oob.hip), two chunk buffers, one barrier per chunk, and no
  // VGPRs or ds_write instructions spent on staging.  float64 x 8 nodes (4 planes) keeps the
  // register-staged single buffer (two would not fit two blocks per CU).
  constexpr bool kDma = sizeof(Pack<T, PV>) == 16 && NPL <= 2 && (!MIRROR || NPL == 2);
  // rows per staged chunk (2 in the LDS-DMA kernel: the next chunk's DMA is issued a
  // 2-row chunk of taps ahead; 4-row chunks, or a 3/4-buffer ring with counted vmcnt waits
  // keeping 2-3 chunks in flight, measured slower)
  static_assert(CPB == 1 || (kDma && MIRROR && MS == 1), "two chunks per block: LDS-DMA mirror kernel, one lane block per real chunk");
  constexpr int R = kDma ? ADMM_FG_DMA_ROWS : kFgRows;
  constexpr int PIECES = NPL * R * 2 * kFgPieces;  // 1-KiB LDS-DMA pieces per chunk
  // two NAMED chunk buffers (not one [2][...] array): the LDS-DMA into one and the tap reads of
  // the other then have distinct underlying objects, so the compiler's LDS-DMA alias tracking
  // does not put a vmcnt(0) -- a wait for the next chunk's DMA -- in front of the taps
  __shared__ Pack<T, PV> win[CPB][NPL][R][kFgRow];
  __shared__ Pack<T, PV> win1[kDma ? CPB : 1][kDma ? NPL : 1][kDma ? R : 1][kDma ? kFgRow : 1];
  // every row window of the segment (N <= 4096): origin and the width actually touched
  __shared__ __align__(16) int wlo_s[(4096 + kFgSeg - 1) / kFgSeg + 4];  // +4: int4 reads of the last chunk
  __shared__ int wnum_s[(4096 + kFgSeg - 1) / kFgSeg + 4];
  // Row windows in parallel: wave g < G bounds its own angle's rays on every row and
  // folds floor(l) into the row's min / max with LDS integer atomics (floor is monotone,
  // so min/max of floors == floor of min/max: the windows do not depend on the order).
  // The window origin is even: a tap's even/odd LDS half, and so the order of a ray's two
  // FMAs per row, then follows the absolute pixel parity -- identical for every group / ray
  // layout / block order, so results do not depend on the plan (or on the GPU count that
  // chooses it).  The one extra column fits the host's 2-pixel window margin.
  for (int r = threadIdx.x; r < nrows; r += kFgThreads) {
    wlo_s[r] = INT_MAX;
    wnum_s[r] = INT_MIN;  // floor(lmax) until the fix-up below
  }
  __syncthreads();
  if (g < G) {  // wave-uniform; a == ang[t0 + g] here
    const int ka = rg->k0[g], kb = rg->k0[g] + rg->nk[g] - 1;
    if (ka <= kb) {
      const double ca = fma((double)ka, a.A1, a.A0), cb = fma((double)kb, a.A1, a.A0);
      for (int r = lane; r < nrows; r += 64) {
        const double dm = (double)(m_lo + r);
        const double la = fma(dm, a.dl, ca), lb = fma(dm, a.dl, cb);
        atomicMin(&wlo_s[r], (int)floor(fmin(la, lb)));
        atomicMax(&wnum_s[r], (int)floor(fmax(la, lb)));
      }
    }
  }
  __syncthreads();
  for (int r = threadIdx.x; r < nrows; r += kFgThreads) {
    const int fmn = wlo_s[r], fmx = wnum_s[r];
    const bool any = fmn != INT_MAX;  // always true for host-planned chunks
    const int wlo = (fmn - 1) & ~1;   // even origin, as below
    wlo_s[r] = any ? wlo : 0;
    wnum_s[r] = any ? min(kFgWin, fmx - wlo + 2) : 0;
  }
  __syncthreads();

  // float samples: ray position l = l0 + m dl advanced per row in 32.32 fixed point
  // (|error| <= rows * 2^-33 pixel, below the float32 weights' own rounding)
  long long lfix = llrint(fma((double)m_lo, a.dl, l0) * 4294967296.0);
  const long long dlfix = llrint(a.dl * 4294967296.0);
  T acc[CPB][VB];
#pragma unroll
  for (int c = 0; c < CPB; ++c)
#pragma unroll
    for (int u = 0; u < VB; ++u) acc[c][u] = T(0);
  int wl_cur[R];  // the current chunk's window origins (scalars)
  // the chunk's window origins, read once into scalar registers (a per-row LDS read
  // would put a dependent LDS round trip in front of every row's tap reads)
  auto origins = [&](int m0, int (&wl)[R]) {
    if constexpr (R == 2) {  // one LDS round trip for both rows
      const int2 w2 = *reinterpret_cast<const int2*>(&wlo_s[m0 - m_lo]);
      wl[0] = w2.x;
      wl[1] = w2.y;
    } else if constexpr (R == 4) {
      const int4 w4 = *reinterpret_cast<const int4*>(&wlo_s[m0 - m_lo]);
      wl[0] = __builtin_amdgcn_readfirstlane(w4.x);
      wl[1] = __builtin_amdgcn_readfirstlane(w4.y);
      wl[2] = __builtin_amdgcn_readfirstlane(w4.z);
      wl[3] = __builtin_amdgcn_readfirstlane(w4.w);
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) wl[r] = wlo_s[m0 - m_lo + r];
    }
  };
  // the taps of one staged chunk: every row's two taps per ray from LDS
  auto taps = [&](const Pack<T, PV> (&wb)[CPB][NPL][R][kFgRow], int m0, int rows, const int (&wl)[R]) {
#pragma unroll
    for (int r = 0; r < R; ++r) {  // unrolled: the chunk's LDS reads can all be in flight
      if (r >= rows) break;
      int idx;
      T w1;
      if constexpr (std::is_same<T, float>::value) {
        idx = (int)(lfix >> 32) - wl[r];
        w1 = (float)(unsigned)lfix;  // fraction x 2^32 (kFgWScale<float>)
        lfix += dlfix;
      } else {
        const double l = fma((double)(m0 + r), a.dl, l0);
        const double fl = floor(l);
        idx = (int)fl - wl[r];
        w1 = (T)(l - fl);
      }
      const T w0 = kFgWOne<T> - w1;
      // taps idx (weight w0) and idx+1 (w1): one is even, one odd
      const bool odd = idx & 1;
      const int se = (idx + 1) >> 1, so = kFgOdd + (idx >> 1);
      const T we = odd ? w1 : w0, wo = odd ? w0 : w1;
#pragma unroll
      for (int c = 0; c < CPB; ++c)
#pragma unroll
        for (int q = 0; q < NPL; ++q) {
          const Pack<T, PV> s0 = wb[c][q][r][se];
          const Pack<T, PV> s1 = wb[c][q][r][so];
#pragma unroll
          for (int e = 0; e < PV; ++e) {
            acc[c][q * PV + e] = fma(we, s0.v[e], acc[c][q * PV + e]);
            acc[c][q * PV + e] = fma(wo, s1.v[e], acc[c][q * PV + e]);
          }
        }
    }
  };
  // Software-pipelined full chunk: every row's tap slots and weights first,
  // then row r+1's LDS reads issued before row r's FMAs, so one row's reads are always in
  // flight behind the other's arithmetic (the LDS-DMA staging freed the registers: the
  // register-staged kernel had no room for the second row's 16).  Same FMAs, same order.
  auto taps4 = [&](const Pack<T, PV> (&wb)[CPB][NPL][R][kFgRow], int m0) {
    int se[R], so[R];  // (float: byte offsets of the even / odd slot; else slot indices)
    T we[R], wo[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      int idx;
      T w1;
      if constexpr (std::is_same<T, float>::value) {
        idx = (int)(lfix >> 32) - wl_cur[r];
        w1 = (float)(unsigned)lfix;  // fraction x 2^32 (kFgWScale<float>)
        lfix += dlfix;
      } else {
        const double l = fma((double)(m0 + r), a.dl, l0);
        const double fl = floor(l);
        idx = (int)fl - wl_cur[r];
        w1 = (T)(l - fl);
      }
      const T w0 = kFgWOne<T> - w1;
      if constexpr (std::is_same<T, float>::value) {
        // parity mask (0 / -1) and two bitfield selects: 3 VALU instead of and + compare +
        // 2 conditional moves (same values, bit for bit)
        const int msk = __builtin_amdgcn_sbfe(idx, 0, 1);
        // slot byte offsets: odd (idx >> 1) x 16, even ceil(idx / 2) x 16 = odd - 16 msk (one
        // v_mad_i32_i24 on the mask instead of a shift-add and a mask of its own)
        so[r] = (idx >> 1) << 4;
        asm("v_mad_i32_i24 %0, %1, -16, %2" : "=v"(se[r]) : "v"(msk), "v"(so[r]));
        const int i0 = __float_as_int(w0), i1 = __float_as_int(w1);
        int ie, io;
        asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(ie) : "v"(msk), "v"(i1), "v"(i0));
        asm("v_bfi_b32 %0, %1, %2, %3" : "=v"(io) : "v"(msk), "v"(i0), "v"(i1));
        we[r] = __int_as_float(ie);
        wo[r] = __int_as_float(io);
      } else {
        se[r] = (idx + 1) >> 1;
        so[r] = kFgOdd + (idx >> 1);
        const bool odd = idx & 1;
        we[r] = odd ? w1 : w0;
        wo[r] = odd ? w0 : w1;
      }
    }
    // the even / odd tap samples of row r, plane q, chunk c
    auto slot = [&](int c, int q, int r, bool even) -> Pack<T, PV> {
      if constexpr (std::is_same<T, float>::value) {
        const char* row = reinterpret_cast<const char*>(&wb[c][q][r][0]);
        return *reinterpret_cast<const Pack<T, PV>*>(even ? row + se[r] : row + kFgOdd * (int)sizeof(Pack<T, PV>) + so[r]);
      } else {
        return wb[c][q][r][even ? se[r] : so[r]];
      }
    };
    // (row, chunk) steps in order; step s + 1's LDS reads issued before step s's FMAs
    Pack<T, PV> cur[2 * NPL], nxt[2 * NPL];
#pragma unroll
    for (int q = 0; q < NPL; ++q) {
      cur[2 * q] = slot(0, q, 0, true);
      cur[2 * q + 1] = slot(0, q, 0, false);
    }
#pragma unroll
    for (int st = 0; st < R * CPB; ++st) {
      const int r = st / CPB, c = st % CPB;
      if (st + 1 < R * CPB) {
        const int r1 = (st + 1) / CPB, c1 = (st + 1) % CPB;
#pragma unroll
        for (int q = 0; q < NPL; ++q) {
          nxt[2 * q] = slot(c1, q, r1, true);
          nxt[2 * q + 1] = slot(c1, q, r1, false);
        }
      }
#pragma unroll
      for (int q = 0; q < NPL; ++q)
#pragma unroll
        for (int e = 0; e < PV; ++e) {
          acc[c][q * PV + e] = fma(we[r], cur[2 * q].v[e], acc[c][q * PV + e]);
          acc[c][q * PV + e] = fma(wo[r], cur[2 * q + 1].v[e], acc[c][q * PV + e]);
        }
#pragma unroll
      for (int q = 0; q < 2 * NPL; ++q) cur[q] = nxt[q];
    }
  };
  // waves g >= G (groups smaller than kFgG) only stage and meet the barriers: their taps
  // would repeat angle G-1's and burn the LDS bandwidth the real taps are bound by
  // (and waves whose angle has no rays in this block)
  const bool idle = g >= G || nkq == 0;

  if constexpr (kDma) {
    // one 1-KiB piece per wave-instruction: 64 consecutive 16-B slots of one (plane, row,
    // parity half); a row's even half holds pixels wlo + 2s, its odd half wlo + 2s + 1
    const uint32_t rowbytes = (uint32_t)N * VBR * (uint32_t)sizeof(T);
    // This wave's pieces (NPW = PIECES / kFgG per chunk: one for 2-row chunks) are the same for
    // every chunk of the segment -- plane, row within the chunk, parity half, 64-slot piece and
    // LDS slot are set once here -- and a piece's staged row moves by a constant per chunk
    // (mirror plane 1, case B: rows N-1-m, a negative step).  The row address is kept as a
    // running scalar base instead of a per-chunk 64-bit row multiply and row select: the CU's one
    // scalar unit serves all 32 waves, and the mirror kernel's DMA block spent 30 scalar
    // instructions per chunk (the direct kernel's 18).  Same rows, columns and slots: bitwise the
    // same staging.
    constexpr int NPW = (PIECES + kFgG - 1) / kFgG;
    struct Piece {
      bool has, rev_col;
      int ph, ppar, pr, ppl, pslot, pcol, psgn;
      const char* prow;
      long long rstep;
    };
    Piece pc[NPW];
#pragma unroll
    for (int i = 0; i < NPW; ++i) {
      const int q = g + i * kFgG;
      Piece& P = pc[i];
      P.has = PIECES % kFgG == 0 || q < PIECES;  // (every wave has NPW at 16 / 32 pieces)
      P.ph = q % kFgPieces;
      P.ppar = (q / kFgPieces) & 1;
      const int prp = q / (2 * kFgPieces);
      P.pr = prp % R;
      P.ppl = prp / R;
      const bool prow_rev = MIRROR && P.ppl == 1 && !caseA;  // case B from row N-1-m
      P.rev_col = MIRROR && P.ppl == 1 && caseA;             // case A: column N-1-w of the same row
      P.pslot = (P.ppar ? kFgOdd : 0) + 64 * P.ph;
      const long long rstride = (long long)rowbytes;
      P.prow = reinterpret_cast<const char*>(src) +
               (prow_rev ? (long long)(N - 1 - (m_lo + P.pr)) : (long long)(m_lo + P.pr)) * rstride;
      P.rstep = (prow_rev ? -rstride : rstride) * R;
      // lane part of the staged column (the row's window origin is added per chunk); a mirrored
      // column N-1-(wo+c) is (N-1-c) - wo (a scalar multiply per chunk instead of a select)
      const int c = 128 * P.ph + P.ppar + 2 * lane;
      P.pcol = P.rev_col ? N - 1 - c : c;
      P.psgn = P.rev_col ? -1 : 1;
    }
    // dma(m0, b, full): chunk m0's pieces into buffer b; full (compile time): the chunk is known
    // to have all R rows.  Called once per chunk with m0 ascending by R from m_lo (the running
    // row addresses rely on it).
    auto dma = [&](int m0, int b, auto fullc) {
#pragma unroll
      for (int i = 0; i < NPW; ++i) {
        Piece& P = pc[i];
        const char* rowp = P.prow;
        P.prow += P.rstep;
        if (!P.has) continue;
        if (!decltype(fullc)::value && P.pr >= m_hi - m0) continue;  // row past the segment
        const int wo = __builtin_amdgcn_readfirstlane(wlo_s[m0 - m_lo + P.pr]);
        const int wn = __builtin_amdgcn_readfirstlane(wnum_s[m0 - m_lo + P.pr]);
        if (128 * P.ph + P.ppar >= wn) continue;  // piece wholly past the touched width
        // the row base is block-uniform: force it into SGPRs (a VGPR base makes hipcc wrap
        // the DMA in a waterfall loop over the distinct resource values)
        const uint64_t rb = (uint64_t)(uintptr_t)rowp;
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)rb);
        const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(rb >> 32));
        const __amdgpu_buffer_rsrc_t rs = make_rsrc((const void*)(uintptr_t)(((uint64_t)hi << 32) | lo), rowbytes);
        const int col = P.pcol + P.psgn * wo;
        // negative columns wrap to huge unsigned offsets: out of range, zero-filled (slots past
        // the row's touched width are fetched but never read by a tap: masking them cost more
        // VALU than the L2 fetch it saved)
        const unsigned voff = MIRROR ? (unsigned)((col * VBR + mq * MH) * (int)sizeof(T))
                                     : (unsigned)((col * VB + P.ppl * PV) * (int)sizeof(T));
#pragma unroll
        for (int c = 0; c < CPB; ++c) {
          // (chunk c of the pair: the next real chunk's image, npix x VBR samples further)
          const __amdgpu_buffer_rsrc_t rsc =
              c == 0 ? rs
                     : make_rsrc((const void*)(uintptr_t)((((uint64_t)hi << 32) | lo) + (uint64_t)c * npix * VBR * sizeof(T)),
                                 rowbytes);
          if (b == 0)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rsc, (__attribute__((address_space(3))) void*)&win[c][P.ppl][P.pr][P.pslot], 16, voff, 0, 0, 0);
          else
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rsc, (__attribute__((address_space(3))) void*)&win1[c][P.ppl][P.pr][P.pslot], 16, voff, 0, 0, 0);
        }
      }
    };
    dma(m_lo, 0, std::false_type{});
    __syncthreads();  // (its fence waits for this wave's LDS-DMA: vmcnt(0)) chunk 0 staged
    // one chunk: DMA of the next one into the other buffer, then this one's taps.  The
    // buffer index is a compile-time constant (the loop is unrolled by the two buffers), so
    // the LDS base of every tap read folds into the ds_read offset field instead of costing
    // two VALU adds per row (the kernel is VALU-issue bound)
    // FULL (compile time): the chunk has all R rows -- every chunk of the loop over chunk pairs;
    // only a segment's last chunk can be short.  Idle waves skip the origins and the taps
    // (wave-uniform branches; the row checks and selects they replace were scalar instructions
    // on every chunk of every wave)
    auto step = [&](auto cbc, auto fullc, int m0) __attribute__((always_inline)) {
      constexpr int cb = decltype(cbc)::value;
      constexpr bool full = decltype(fullc)::value;
      // the other buffer was last read by the previous chunk's taps (done: barrier below)
      // (in a full pair, chunk m0 + R of the first step is full too)
      if (m0 + R < m_hi) dma(m0 + R, cb ^ 1, std::integral_constant<bool, full && cb == 0>{});
      if (!idle) {
        origins(m0, wl_cur);
        if constexpr (full) {
          if constexpr (cb == 0)
            taps4(win, m0);
          else
            taps4(win1, m0);
        } else {
          const int rows = min(R, m_hi - m0);
          if constexpr (cb == 0) {
            if (rows == R)
              taps4(win, m0);
            else
              taps(win, m0, rows, wl_cur);
          } else {
            if (rows == R)
              taps4(win1, m0);
            else
              taps(win1, m0, rows, wl_cur);
          }
        }
      }
      __syncthreads();  // this chunk's readers done; next chunk's DMA landed (vmcnt(0) + barrier)
    };
    using C0 = std::integral_constant<int, 0>;
    using C1 = std::integral_constant<int, 1>;
    using Full = std::true_type;
    using Part = std::false_type;
    int m0 = m_lo;
    for (; m0 + 2 * R <= m_hi; m0 += 2 * R) {
      step(C0{}, Full{}, m0);
      step(C1{}, Full{}, m0 + R);
    }
    if (m0 < m_hi) {  // the segment's last one or two chunks (the last one may be short)
      step(C0{}, Part{}, m0);
      if (m0 + R < m_hi) step(C1{}, Part{}, m0 + R);
    }
  } else {
    // staging in two halves: issue global loads for chunk c+1 into registers
    // (prefetch), compute chunk c from LDS, then write the registers into LDS.
    Pack<T, PV> stage[PER];
    auto fetch = [&](int m0) {
      const int rows = min(R, m_hi - m0);
#pragma unroll
      for (int e = 0; e < PER; ++e) {
        const int q = threadIdx.x + e * kFgThreads;
        const int pl = q % NPL, rw = q / NPL;
        const int r = rw / kFgWin, w = rw - r * kFgWin;
        // only the row's touched width is fetched (the rest of the window is never read)
        // both reads unconditional (in bounds: +4 padding), so they issue together
        const int wn = wnum_s[m0 - m_lo + r], wo = wlo_s[m0 - m_lo + r];
        const int col = (r < rows && w < wn) ? wo + w : -1;
        if constexpr (MIRROR) {  // element-wise: a virtual plane may mix the two orientations
#pragma unroll
          for (int z = 0; z < PV; ++z) {
            const int u = pl * PV + z, o = u >= MH;
            const int srow = (o && !caseA) ? N - 1 - (m0 + r) : m0 + r;
            const int scol = (o && caseA) ? N - 1 - col : col;
            stage[e].v[z] = (q < R * kFgWin * NPL && col >= 0 && col < N)
                                ? src[((size_t)srow * N + scol) * VBR + mq * MH + (u - o * MH)]
                                : T(0);
          }
        } else if (q < R * kFgWin * NPL && col >= 0 && col < N) {
          stage[e] = *reinterpret_cast<const Pack<T, PV>*>(src + ((size_t)(m0 + r) * N + col) * VB + pl * PV);
        } else {
#pragma unroll
          for (int z = 0; z < PV; ++z) stage[e].v[z] = T(0);
        }
      }
    };
    auto commit = [&]() {
#pragma unroll
      for (int e = 0; e < PER; ++e) {
        const int q = threadIdx.x + e * kFgThreads;
        if (q < R * kFgWin * NPL) {
          const int pl = q % NPL, rw = q / NPL;
          const int r = rw / kFgWin, w = rw - r * kFgWin;
          win[0][pl][r][(w & 1) ? kFgOdd + (w >> 1) : (w >> 1)] = stage[e];
        }
      }
    };
    fetch(m_lo);
    for (int m0 = m_lo; m0 < m_hi; m0 += R) {
      int wl[R];
      origins(m0, wl);
      __syncthreads();  // previous chunk's readers are done
      commit();
      __syncthreads();
      // the next chunk's loads issue at raised wave priority (ahead of other waves' taps)
      __builtin_amdgcn_s_setprio(1);
      if (m0 + R < m_hi) fetch(m0 + R);
      __builtin_amdgcn_s_setprio(0);
      taps(win, m0, idle ? 0 : min(R, m_hi - m0), wl);
    }
  }
  if (g < G && rl < nkq) {
    const size_t m_rays = (size_t)n_ang * n_det;
#pragma unroll
    for (int c = 0; c < CPB; ++c)
      gstore<T, VB>(part + (((size_t)seg * ((V + VB - 1) / VB) + chunk + c) * m_rays + (size_t)t * n_det + k) * VB,
                    acc[c]);
  }
}

// Sum the kFgSeg segment partials in fixed order, scale by L(t):
// MODE 0: sino = A x.  MODE 1: s = A x - b (b node-major) + per-block partials of ||s||^2.
template <typename T, int VB, int MODE>
__global__ __launch_bounds__(kBlock) void k_fwd_combine(const T* __restrict__ part, T* __restrict__ sino,
                                                        const T* __restrict__ bsino, double* __restrict__ pout,
                                                        const FwdAngle* __restrict__ ang, int n_det, int n_ang,
                                                        int V) {
  const int chunk = blockIdx.y, v0 = chunk * VB, nv = min(VB, V - v0);
  const int nch = (V + VB - 1) / VB;
  const size_t m_rays = (size_t)n_ang * n_det;
  const size_t ray = (size_t)blockIdx.x * kBlock + threadIdx.x;
  double sq[VB];
#pragma unroll
  for (int u = 0; u < VB; ++u) sq[u] = 0.0;
  if (ray < m_rays) {
    const T L = (T)ang[ray / n_det].L * kFgWScale<T>;
    T acc[VB], pv[VB];
    gload<T, VB>(part + ((size_t)chunk * m_rays + ray) * VB, acc);
#pragma unroll
    for (int sg = 1; sg < kFgSeg; ++sg) {
      gload<T, VB>(part + (((size_t)sg * nch + chunk) * m_rays + ray) * VB, pv);
#pragma unroll
      for (int u = 0; u < VB; ++u) acc[u] += pv[u];
    }
#pragma unroll
    for (int u = 0; u < VB; ++u) {
      acc[u] *= L;
      if (MODE == 1) {
        if (u < nv) {
          acc[u] -= bsino[(size_t)(v0 + u) * m_rays + ray];
          sq[u] = (double)acc[u] * (double)acc[u];
        } else {
          acc[u] = T(0);
        }
      }
    }
    gstore<T, VB>(sino + ((size_t)chunk * m_rays + ray) * VB, acc);
  }
  if (MODE == 1) {
    __shared__ double lds[4 * VB];
    block_reduce<VB>(sq, lds);
    if (threadIdx.x == 0) {
#pragma unroll
      for (int u = 0; u < VB; ++u)
        if (u < nv) pout[(size_t)(v0 + u) * gridDim.x + blockIdx.x] = sq[u];
    }
  }
}

// The mirror-mode combine (k_fwdg<..., MIRROR>): virtual chunk c' of the half geometry's rays
// (a/2 angles) -> the REAL sinogram (VBR lanes, a angles) of real chunk c' / MS, lane block
// c' % MS: lanes u < VB/2 are angle t, lanes u >= VB/2 angle a-1-t (pi - theta_t) of the same
// real nodes.  MODE 1: s = A x - b against the real node-major b, and per real node one
// ||s||^2 partial per block holding both of its angles' residuals (summed in a fixed order).
template <typename T, int VB, int VBR, int MODE>
__global__ __launch_bounds__(kBlock) void k_fwd_combine_mirror(const T* __restrict__ part, T* __restrict__ sino,
                                                               const T* __restrict__ bsino,
                                                               double* __restrict__ pout,
                                                               const FwdAngle* __restrict__ ang, int n_det,
                                                               int n_ang_half, int V) {
  constexpr int MH = VB / 2, MS = VBR / MH;
  const int chunk = blockIdx.y, nch = gridDim.y;  // virtual chunks
  const int rc = chunk / MS, mq = chunk % MS;     // real chunk, lane block
  const int vr0 = rc * VBR + mq * MH;             // first real node of the lane block
  const size_t m_half = (size_t)n_ang_half * n_det, m_full = 2 * m_half;
  if constexpr (MODE == 0) {
    // two adjacent threads per virtual ray: lanes < VB/2 (-> angle t) and lanes >= VB/2 (-> angle
    // a-1-t), each summing its half over the segments in the same order as below (same bits),
    // twice the loads in flight of a thread-per-ray grid (grid.x doubled by the launcher)
    const size_t q = (size_t)blockIdx.x * kBlock + threadIdx.x;
    const size_t ray = q >> 1;
    const int h = (int)(q & 1);
    if (ray >= m_half) return;
    const int t = (int)(ray / n_det), k = (int)(ray % n_det);
    const T L = (T)ang[t].L * kFgWScale<T>;
    T acc[MH], pv[MH];
    gload<T, MH>(part + ((size_t)chunk * m_half + ray) * VB + h * MH, acc);
#pragma unroll
    for (int sg = 1; sg < kFgSeg; ++sg) {
      gload<T, MH>(part + (((size_t)sg * nch + chunk) * m_half + ray) * VB + h * MH, pv);
#pragma unroll
      for (int u = 0; u < MH; ++u) acc[u] += pv[u];
    }
#pragma unroll
    for (int u = 0; u < MH; ++u) acc[u] *= L;
    const size_t dst = h ? (size_t)(2 * n_ang_half - 1 - t) * n_det + k : ray;
    gstore<T, MH>(sino + (size_t)rc * m_full * VBR + mq * MH + dst * VBR, acc);
    return;
  }
  const size_t ray = (size_t)blockIdx.x * kBlock + threadIdx.x;
  double sq[MH];
#pragma unroll
  for (int u = 0; u < MH; ++u) sq[u] = 0.0;
  if (ray < m_half) {
    const int t = (int)(ray / n_det), k = (int)(ray % n_det);
    const size_t ray2 = (size_t)(2 * n_ang_half - 1 - t) * n_det + k;  // angle a-1-t
    const T L = (T)ang[t].L * kFgWScale<T>;
    T acc[VB], pv[VB];
    gload<T, VB>(part + ((size_t)chunk * m_half + ray) * VB, acc);
#pragma unroll
    for (int sg = 1; sg < kFgSeg; ++sg) {
      gload<T, VB>(part + (((size_t)sg * nch + chunk) * m_half + ray) * VB, pv);
#pragma unroll
      for (int u = 0; u < VB; ++u) acc[u] += pv[u];
    }
    T lo[MH], hi[MH];
#pragma unroll
    for (int u = 0; u < MH; ++u) {
      lo[u] = acc[u] * L;
      hi[u] = acc[MH + u] * L;
      if (MODE == 1) {
        if (vr0 + u < V) {
          lo[u] -= bsino[(size_t)(vr0 + u) * m_full + ray];
          hi[u] -= bsino[(size_t)(vr0 + u) * m_full + ray2];
          sq[u] = (double)lo[u] * (double)lo[u] + (double)hi[u] * (double)hi[u];
        } else {
          lo[u] = T(0);
          hi[u] = T(0);
        }
      }
    }
    T* base = sino + (size_t)rc * m_full * VBR + mq * MH;  // (MH-lane blocks: aligned vector stores)
    gstore<T, MH>(base + ray * VBR, lo);
    gstore<T, MH>(base + ray2 * VBR, hi);
  }
  if (MODE == 1) {
    __shared__ double lds[4 * MH];
    block_reduce<MH>(sq, lds);
    if (threadIdx.x == 0) {
#pragma unroll
      for (int u = 0; u < MH; ++u)
        if (vr0 + u < V) pout[(size_t)(vr0 + u) * gridDim.x + blockIdx.x] = sq[u];
    }
  }
}

// ===========================================================================
// Back projector (pixel-driven gather; exact transpose of the Joseph weights):
//   acc[v][i,j] = sum_t sum_{k in {k0,k0+1}} w_t(k) * sino[v][t][k]
// Replaces `Ai.T @ r` (block_6_admm_loop_ver2.py:145).  No atomics: each pixel
// gathers its <= 2 bins per angle.  The angle table is staged in LDS.
// Fused epilogues (MODE):
//   BACK_PLAIN : out = A^T s  (interleaved samples)                  (operator API)
//   BACK_ATB   : atb = A^T b (float64 node-major)                    (setup)
//   BACK_WSQ   : W = max(sum_r A[r,p]^2, 1e-12) (float64)            (make_precisions, block_3:20-23)
//   BACK_H     : Hp = A^T A p + rho D p + mu K^T K p; partials p.Hp, r.Hp, Hp.Hp, r.r, r.p (CG)
//   BACK_INIT  : r = A^T b + rho c + mu K^T(d-e) - H xs;  p = r                      (CG start)
//   BACK_DIAG  : g = A^T s + rho (D x - c) + lam K^T sub(Kx); partials |g|^2, TV(x),
//                sum_j rho/2 q_ij (x - v_ij)^2, |x - phantom|^2   (block_6_ver2.py:135-149),
//                |A^T s + rho (D x - c) + mu K^T e|^2 (split-Bregman stationarity residual)
// ===========================================================================
// Edge state a node's x-update reads (admm_batch): the duals and z, stored (z != null) or
// derived (z == null, ABI 7): z_ij = (x_prev[a] + x_prev[b]) / 2 from the endpoint images of
// the last consensus -- bitwise the z that consensus formed, since it computed (x_a + x_b) * 0.5
// from the very rows it then copied into x_prev.
struct EdgeIn {
  const double* z;   // [E][n] stored z, or null
  const double* y;   // [E][n] dual of the lower endpoint
  const double* yb;  // [E][n] dual of the higher endpoint (weighted fusion) or null
  const double* xp;  // [n_xext][n] x_prev (derived z)
  const int* ea;     // [E] x_ext rows of the endpoints
  const int* eb;
};

enum BackMode { BACK_PLAIN = 0, BACK_ATB = 1, BACK_WSQ = 2, BACK_H = 3, BACK_INIT = 4, BACK_DIAG = 5 };

template <typename T>
struct BackArgs {
  const T* sino;            // interleaved [C][m][VB]
  const BackAngle* ang;     // [n_ang]
  const BackAngleC* angc;   // [n_ang] compact records
  double K;                 // angle-independent part of k_f
  int kbias;                // integer added to every k_f so that k_f > 0 (host: from the geometry)
  int wexp;                 // float weights of angc are scaled by 2^-wexp so that they are <= 1
  int N, n_det, n_ang, V;
  // explicit-matrix contexts (admm_ctx_create_matrix): A^T as CSR, one row per pixel
  const int* csr_ptr;       // [n + 1]
  const int* csr_idx;       // [nnz] sinogram rows (rays)
  const T* csr_val;         // [nnz]
  // outputs
  T* out_t;                 // PLAIN: A^T s;  H: Hp;  INIT: p   (interleaved)
  double* out_d;            // ATB: atb;  WSQ: W;  INIT: r     (float64 node-major)
  double* part;             // [V][NQ][P]  (NQ = 5 for H, 4 for DIAG)
  // epilogue inputs
  const T* pin;             // H: p;  INIT: xs (interleaved)
  const double* r;          // H: r
  const double* dsum;       // [V][n]
  const T* dsum_s;          // H: D as interleaved samples [C][n][VB] (one VB-vector per pixel)
  const double* atb;        // INIT
  const double* cvec;       // INIT, DIAG: c = sum_j q v
  const double* dvar;       // INIT: d [V][2][n]
  const double* evar;       // INIT, DIAG: e [V][2][n]
  const double* x;          // DIAG: x rows of x_ext
  const double* phantom;    // DIAG (may be null)
  EdgeIn edges;             // DIAG: edge state (y, z or x_prev, y_b)
  const double* qv;         // DIAG: q slots
  const int* inc_off;       // DIAG
  const int* inc_edge;
  const int* inc_qslot;
  const int* inc_sign;
  double rho, lam, mu;
  int tv_kind;
};

// v_ij = z_ij - y_ij,i seen from the node at incidence sign s (+1 lower endpoint) for edge slot
// e at pixel pix: single-y form y_ij,max = -y when yb is null, else the stored higher-endpoint dual.
__device__ __forceinline__ double edge_v(const EdgeIn& E, int e, int s, int npix, int pix) {
  const size_t eo = (size_t)e * npix + pix;
  const double z = E.z ? E.z[eo]
                       : (E.xp[(size_t)E.ea[e] * npix + pix] + E.xp[(size_t)E.eb[e] * npix + pix]) * 0.5;
  if (E.yb == nullptr) return z - (double)s * E.y[eo];
  return z - (s > 0 ? E.y[eo] : E.yb[eo]);
}

// forward difference at (i,j) of a float64 image (zero at the last row / column)
__device__ __forceinline__ void grad_at(const double* __restrict__ x, int N, int i, int j, double& gx, double& gy) {
  const double c = x[i * N + j];
  gx = (i < N - 1) ? x[(i + 1) * N + j] - c : 0.0;
  gy = (j < N - 1) ? x[i * N + j + 1] - c : 0.0;
}

// TV subgradient direction at a gradient (block_4_tv_helpers.py:37-46, eps = 1e-12)
__device__ __forceinline__ void tv_sub(double gx, double gy, int kind, double& px, double& py) {
  if (kind == 0) {
    const double m = sqrt(gx * gx + gy * gy);
    if (m > 1e-12) {
      px = gx / m;
      py = gy / m;
    } else {
      px = 0.0;
      py = 0.0;
    }
  } else {
    px = fabs(gx) > 1e-12 ? copysign(1.0, gx) : 0.0;
    py = fabs(gy) > 1e-12 ? copysign(1.0, gy) : 0.0;
  }
}

// (K^T w)[i,j] for a two-component float64 field w = d - e stored [2][n]
__device__ __forceinline__ double kt_w_at(const double* __restrict__ d, const double* __restrict__ e, int N,
                                          int i, int j) {
  const int n = N * N;
  double s = 0.0;
  const int o = i * N + j;
  if (i >= 1) s += d[o - N] - e[o - N];
  if (i <= N - 2) s -= d[o] - e[o];
  if (j >= 1) s += d[n + o - 1] - e[n + o - 1];
  if (j <= N - 2) s -= d[n + o] - e[n + o];
  return s;
}

// Fused epilogue of one pixel: writes the mode's per-pixel outputs and stores the pixel's
// reduction terms into pq (ACC: adds them, the second pixel of a mirror pair; the caller
// zero-fills pq, so out-of-image pixels and dead lanes contribute 0).
// VS / lo (mirror mode): the VB lanes handled are lanes lo .. lo+VB-1 of VS-lane sample vectors.
template <typename T, int VB, int MODE, int NQ, int VS = VB, bool ACC = false>
__device__ __forceinline__ void back_epilogue(const BackArgs<T>& A, int i, int j, int chunk, int v0, int nv,
                                              const T (&acc)[VB], double (&pq)[VB][NQ], int lo = 0) {
  const int N = A.N;
  const int npix = N * N;
  const int pix = i * N + j;
  const size_t sbase = (size_t)chunk * npix * VS + lo;  // interleaved sample base of this chunk
  if constexpr (MODE == BACK_PLAIN) {
    gstore<T, VB>(A.out_t + sbase + (size_t)pix * VS, acc);
  } else if constexpr (MODE == BACK_ATB) {
#pragma unroll
    for (int u = 0; u < VB; ++u)
      if (u < nv) A.out_d[(size_t)(v0 + u) * npix + pix] = (double)acc[u];
  } else if constexpr (MODE == BACK_WSQ) {
    A.out_d[pix] = fmax((double)acc[0], 1e-12);
  } else if constexpr (MODE == BACK_H && std::is_same<T, float>::value) {
    // float32 samples: H p = acc + rho D p + mu K^T K p formed in float32 (p, D and the taps'
    // acc are float32 samples and Hp is stored as one, so float64 here only re-rounded the same
    // sum), lane pairs as packed instructions -- every lane the same IEEE single ops whether it
    // is packed or the odd tail, so a node's result does not depend on the batch width -- and
    // the five CG dots accumulated in float64 by explicit fma (p.Hp and Hp.Hp are exact float64
    // products of float32 values)
    using F2 = float2v;
    constexpr int NP = VB / 2;
    const T* pv = A.pin + sbase;
    T pc[VB], pn[VB], dv[VB], outv[VB];
    F2 kt2[NP > 0 ? NP : 1], pc2[NP > 0 ? NP : 1];
    float kt1 = 0.0f;  // (odd VB: the last lane)
    gload<T, VB>(pv + (size_t)pix * VS, pc);
#pragma unroll
    for (int h = 0; h < NP; ++h) {
      pc2[h] = F2{pc[2 * h], pc[2 * h + 1]};
      kt2[h] = F2{0.0f, 0.0f};
    }
    // K^T K p in the order of the float64 form: (pc - p_up) - (p_down - pc) + (pc - p_left) - (p_right - pc)
    auto nb = [&](size_t o, bool sub_pc_first) {
      gload<T, VB>(pv + o * VS, pn);
#pragma unroll
      for (int h = 0; h < NP; ++h) {
        const F2 q = F2{pn[2 * h], pn[2 * h + 1]};
        kt2[h] = sub_pc_first ? kt2[h] + (pc2[h] - q) : kt2[h] - (q - pc2[h]);
      }
      if constexpr (VB % 2) kt1 = sub_pc_first ? kt1 + (pc[VB - 1] - pn[VB - 1]) : kt1 - (pn[VB - 1] - pc[VB - 1]);
    };
    if (i >= 1) nb((size_t)(pix - N), true);
    if (i <= N - 2) nb((size_t)(pix + N), false);
    if (j >= 1) nb((size_t)(pix - 1), true);
    if (j <= N - 2) nb((size_t)(pix + 1), false);
    gload<T, VB>(A.dsum_s + sbase + (size_t)pix * VS, dv);
    const float rf = (float)A.rho, mf = (float)A.mu;
    const F2 rho2 = F2{rf, rf}, mu2 = F2{mf, mf};
#pragma unroll
    for (int h = 0; h < NP; ++h) {
      const F2 d2 = F2{dv[2 * h], dv[2 * h + 1]} * rho2;
      F2 hv = __builtin_elementwise_fma(d2, pc2[h], F2{acc[2 * h], acc[2 * h + 1]});
      hv = __builtin_elementwise_fma(mu2, kt2[h], hv);
      outv[2 * h] = hv.x;
      outv[2 * h + 1] = hv.y;
    }
    if constexpr (VB % 2) outv[VB - 1] = fmaf(mf, kt1, fmaf(dv[VB - 1] * rf, pc[VB - 1], acc[VB - 1]));
#pragma unroll
    for (int u = 0; u < VB; ++u) {
      if (u >= nv) outv[u] = T(0);
      if (u < nv) {
        const double hd = (double)outv[u], pcd = (double)pc[u];
        const double rv = A.r[(size_t)(v0 + u) * npix + pix];
        pq[u][0] = fma(pcd, hd, ACC ? pq[u][0] : 0.0);
        pq[u][1] = fma(rv, hd, ACC ? pq[u][1] : 0.0);
        pq[u][2] = fma(hd, hd, ACC ? pq[u][2] : 0.0);
        pq[u][3] = fma(rv, rv, ACC ? pq[u][3] : 0.0);
        pq[u][4] = fma(rv, pcd, ACC ? pq[u][4] : 0.0);
      }
    }
    gstore<T, VB>(A.out_t + sbase + (size_t)pix * VS, outv);
  } else if constexpr (MODE == BACK_H || MODE == BACK_INIT) {
    // H v = acc + rho D v + mu K^T K v  (v = p or xs, interleaved samples)
    const T* pv = A.pin + sbase;
    T pc[VB], pn[VB];
    double ktk[VB];
    gload<T, VB>(pv + (size_t)pix * VS, pc);
    if (i >= 1) {  // (the first term assigned: no 0 + x)
      gload<T, VB>(pv + (size_t)(pix - N) * VS, pn);
#pragma unroll
      for (int u = 0; u < VB; ++u) ktk[u] = (double)pc[u] - (double)pn[u];
    } else {
#pragma unroll
      for (int u = 0; u < VB; ++u) ktk[u] = 0.0;
    }
    if (i <= N - 2) {
      gload<T, VB>(pv + (size_t)(pix + N) * VS, pn);
#pragma unroll
      for (int u = 0; u < VB; ++u) ktk[u] -= (double)pn[u] - (double)pc[u];
    }
    if (j >= 1) {
      gload<T, VB>(pv + (size_t)(pix - 1) * VS, pn);
#pragma unroll
      for (int u = 0; u < VB; ++u) ktk[u] += (double)pc[u] - (double)pn[u];
    }
    if (j <= N - 2) {
      gload<T, VB>(pv + (size_t)(pix + 1) * VS, pn);
#pragma unroll
      for (int u = 0; u < VB; ++u) ktk[u] -= (double)pn[u] - (double)pc[u];
    }
    T outv[VB], dv[VB];
    // H: D read as one sample vector (float64 D rounded to T: a 2^-24-relative change of the
    // rho D p term, far below the float32 Hp it produces); INIT keeps float64 D
    if constexpr (MODE == BACK_H) gload<T, VB>(A.dsum_s + sbase + (size_t)pix * VS, dv);
#pragma unroll
    for (int u = 0; u < VB; ++u) {
      outv[u] = T(0);
      if (u < nv) {
        const size_t vo = (size_t)(v0 + u) * npix;
        const double pcd = (double)pc[u];
        const double dd = (MODE == BACK_H) ? (double)dv[u] : A.dsum[vo + pix];
        const double h = (double)acc[u] + A.rho * dd * pcd + A.mu * ktk[u];
        if constexpr (MODE == BACK_H) {
          const T hp = (T)h;
          outv[u] = hp;
          const double hd = (double)hp;
          const double rv = A.r[vo + pix];
          if constexpr (ACC) {  // the mirror pixel of a pair: onto the first pixel's terms
            pq[u][0] += pcd * hd;
            pq[u][1] += rv * hd;
            pq[u][2] += hd * hd;
            pq[u][3] += rv * rv;
            pq[u][4] += rv * pcd;
          } else {
            pq[u][0] = pcd * hd;
            pq[u][1] = rv * hd;
            pq[u][2] = hd * hd;
            pq[u][3] = rv * rv;
            pq[u][4] = rv * pcd;
          }
        } else {
          const double* dv = A.dvar + 2 * vo;
          const double* ev = A.evar + 2 * vo;
          const double rr = A.atb[vo + pix] + A.rho * A.cvec[vo + pix] + A.mu * kt_w_at(dv, ev, N, i, j) - h;
          A.out_d[vo + pix] = rr;
          outv[u] = (T)rr;
        }
      }
    }
    gstore<T, VB>(A.out_t + sbase + (size_t)pix * VS, outv);
  }  // BACK_DIAG: diag_epilogue_tile (block-cooperative)
}

// Back projector.  Block = 64 (j) x kBTI (i) pixel tile, one pixel per thread.
// Per chunk of kBAngC angles the block stages, for each angle, the window of
// kBWin detector bins its tile can touch (from the floor of the smallest corner
// k_f, minus 1) into LDS, zero-filled outside the detector, so each tap is an
// LDS read with no bin-range predicate; every staged bin serves ~7 taps.  A
// VB-vector of samples (32 B for 8 float nodes) is split into 16-byte planes so
// that lanes reading consecutive bins hit consecutive banks (no conflicts).
// Two angles are processed per iteration to keep 4 LDS reads in flight.
// Tile kBTJ x kBTI, one pixel per thread, each wave a 16 (j) x 4 (i) patch.  The window
// must hold the tile's projected extent, at most sqrt((kBTJ-1)^2 + (kBTI-1)^2) bins
// (|Bi|, |Bj| <= 1 because the detector is never finer than the pixel), plus 3 bins of
// floor / margin / second tap.  Bigger tiles stage one window for more pixels
// (L2 traffic per tap ~ window / pixels).
#ifndef ADMM_BK_TI
#define ADMM_BK_TI 32
#endif
#ifndef ADMM_BK_TJ
#define ADMM_BK_TJ 32
#endif
constexpr int kBTJ = ADMM_BK_TJ;
constexpr int kBTI = ADMM_BK_TI;
constexpr int kBkThreads = kBTJ * kBTI;
constexpr int kBkWaves = kBkThreads / 64;
constexpr int kBkPatchJ = kBTJ / 16;  // 16 x 4 wave patches per tile row
static_assert((kBTJ == 32 || kBTJ == 64) && kBTI % 4 == 0 && kBkThreads <= 1024 && kBkWaves >= 4,
              "unsupported back-projector tile");
constexpr int ce_isqrt_ceil(int v) {
  int r = 0;
  while (r * r < v) ++r;
  return r;
}
constexpr int kBWin = ((ce_isqrt_ceil((kBTJ - 1) * (kBTJ - 1) + (kBTI - 1) * (kBTI - 1)) + 3 + 7) / 8) * 8;
#ifndef ADMM_BK_ANGC
#define ADMM_BK_ANGC 32
#endif
constexpr int kBAngC = ADMM_BK_ANGC;  // angles per staged sinogram-window chunk

// DIAG epilogue for a whole kBTJ x kBTI tile (block-cooperative; replaces the per-pixel
// DIAG branch of back_epilogue, same formulas in the same order, so bitwise the same):
// per node, x over the tile plus one halo row/column on each side is staged in LDS and
// the TV subgradient of every point (tile + the halo row/column above/left) is computed
// ONCE into LDS -- the per-pixel form evaluated it at three points and re-read x nine
// times.  kDiagG nodes per pass (round 6: their x tiles load in one loop, one third of the
// barriers); `scratch`: kDiagScratch doubles of LDS.
#ifndef ADMM_DIAG_G
#define ADMM_DIAG_G 2
#endif
#ifndef ADMM_BK_DMA
#define ADMM_BK_DMA 1  // mirror back projector (H mode): window bins staged by LDS-DMA
#endif
#ifndef ADMM_BK_LB2
#define ADMM_BK_LB2 1  // ... and two lane blocks per block where the grid still fills the chip
#endif
constexpr int kDiagG = ADMM_DIAG_G;  // nodes per staging pass of the DIAG epilogue
constexpr int kDiagScratch = kDiagG * ((kBTI + 2) * (kBTJ + 2) + 2 * (kBTI + 1) * (kBTJ + 1));
template <typename T, int VB, int VS = VB>
__device__ __forceinline__ void diag_epilogue_tile(const BackArgs<T>& A, double* scratch, int ib, int jb, int i,
                                                   int j, bool inb, int chunk, int v0, int nv, const T (&acc)[VB],
                                                   double (&pq)[VB][5], int lo = 0) {
  constexpr int XC = kBTJ + 2, XR = kBTI + 2, SC = kBTJ + 1, SR = kBTI + 1;
  constexpr int G = kDiagG, XS = XR * XC, SS = SR * SC;
  // per node g of a pass: xt = scratch + g XS  [XR][XC]: rows ib-1 .. ib+kBTI, cols jb-1 .. jb+kBTJ;
  // sx, sy = scratch + G XS + 2 g SS (+ SS)  [SR][SC]: subgradient at rows ib-1 .., cols jb-1 ..
  const int N = A.N, npix = N * N;
  const int pix = i * N + j;
  const size_t sbase = (size_t)chunk * npix * VS + lo;
  if (inb && A.out_t) gstore<T, VB>(A.out_t + sbase + (size_t)pix * VS, acc);
  const int ti = i - ib + 1, tj = j - jb + 1;  // this pixel in the staged x tile
#pragma unroll
  for (int u0 = 0; u0 < VB; u0 += G) {  // constant bounds keep acc / pq in registers
    if (u0 >= nv) break;                // block-uniform: the barriers below stay uniform
    const int ng = min(G, nv - u0);
    __syncthreads();  // previous pass's (or the tap loop's) LDS readers are done
    // the pass's G x tiles in one loop: their global loads are in flight together
    for (int q = threadIdx.x; q < ng * XS; q += kBkThreads) {
      const int g = q / XS, e = q % XS;
      const int rr = e / XC, cc = e % XC;
      const int ii = ib - 1 + rr, jj = jb - 1 + cc;
      const double* xv = A.x + (size_t)(v0 + u0 + g) * npix;
      scratch[q] = (ii >= 0 && jj >= 0 && ii < N && jj < N) ? xv[ii * N + jj] : 0.0;
    }
    __syncthreads();
    for (int q = threadIdx.x; q < ng * SS; q += kBkThreads) {
      const int g = q / SS, e = q % SS;
      const int rr = e / SC, cc = e % SC;
      const int ii = ib - 1 + rr, jj = jb - 1 + cc;
      const double* xt = scratch + g * XS;
      double px = 0.0, py = 0.0;
      if (ii >= 0 && jj >= 0 && ii < N && jj < N) {
        const double c = xt[rr * XC + cc];
        const double gx = (ii < N - 1) ? xt[(rr + 1) * XC + cc] - c : 0.0;
        const double gy = (jj < N - 1) ? xt[rr * XC + cc + 1] - c : 0.0;
        tv_sub(gx, gy, A.tv_kind, px, py);
      }
      scratch[G * XS + 2 * g * SS + e] = px;
      scratch[G * XS + (2 * g + 1) * SS + e] = py;
    }
    __syncthreads();
    if (!inb) continue;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int u = u0 + g;
      if (u >= VB || g >= ng) break;
      const int v = v0 + u;
      const size_t vo = (size_t)v * npix;
      const double* xt = scratch + g * XS;
      const double* sx = scratch + G * XS + 2 * g * SS;
      const double* sy = sx + SS;
      const double xc = xt[ti * XC + tj];
      const double gx = (i < N - 1) ? xt[(ti + 1) * XC + tj] - xc : 0.0;
      const double gy = (j < N - 1) ? xt[ti * XC + tj + 1] - xc : 0.0;
      const double tvv = (A.tv_kind == 0) ? sqrt(gx * gx + gy * gy) : fabs(gx) + fabs(gy);
      // lam * K^T sub(Kx) at (i,j): subgradients at (i,j), (i-1,j), (i,j-1)
      double kts = 0.0;
      if (i <= N - 2) kts -= sx[ti * SC + tj];
      if (j <= N - 2) kts -= sy[ti * SC + tj];
      if (i >= 1) kts += sx[(ti - 1) * SC + tj];
      if (j >= 1) kts += sy[ti * SC + tj - 1];
      const double cc = A.cvec[vo + pix];
      const double sm = (double)acc[u] + A.rho * (A.dsum[vo + pix] * xc - cc);  // gradient of the quadratic
      const double gg = sm + A.lam * kts;
      // K^T e at (i, j) (e = final Bregman variable [2][n] of node v)
      const double* ev = A.evar + 2 * vo;
      double kte = 0.0;
      if (i >= 1) kte += ev[pix - N];
      if (i <= N - 2) kte -= ev[pix];
      if (j >= 1) kte += ev[npix + pix - 1];
      if (j <= N - 2) kte -= ev[npix + pix];
      const double rsb = sm + A.mu * kte;
      double quad = 0.0;
      for (int q = A.inc_off[v]; q < A.inc_off[v + 1]; ++q) {
        const double vij = edge_v(A.edges, A.inc_edge[q], A.inc_sign[q], npix, pix);
        const double dd = xc - vij;
        quad += A.qv[(size_t)A.inc_qslot[q] * npix + pix] * dd * dd;
      }
      pq[u][0] += gg * gg;
      pq[u][1] += tvv;
      pq[u][2] += 0.5 * A.rho * quad;
      if (A.phantom) {
        const double dp = xc - A.phantom[pix];
        pq[u][3] += dp * dp;
      }
      pq[u][4] += rsb * rsb;
    }
  }
}

#ifndef ADMM_BK_NARROW_WPE
#define ADMM_BK_NARROW_WPE 1  // 8: A/B candidate (64 VGPRs, spills 10 in H mode)
#endif
// Waves per SIMD the register budget must allow: float samples at VB <= 4 (narrow batches:
// C4's 4-node share per GPU at 8 GPUs) fit 64 VGPRs, so two 1024-thread blocks share a CU and
// one block's window staging / epilogue overlaps the other's taps (the wide kernels need more
// than 64 and run one block per CU).
template <typename T, int VB, int MODE>
constexpr int back_waves_per_eu() {
  return (std::is_same<T, float>::value && VB <= 4 && (MODE == BACK_H || MODE == BACK_INIT)) ? ADMM_BK_NARROW_WPE : 1;
}
template <typename T, int VB, int MODE, bool CSR = false>
__global__ __launch_bounds__(kBkThreads) __attribute__((amdgpu_waves_per_eu(back_waves_per_eu<T, VB, MODE>())))
void k_back(BackArgs<T> A) {
  constexpr int NQ = (MODE == BACK_H) ? 5 : (MODE == BACK_DIAG) ? 5 : 1;
  constexpr int NPL = Planes<T, VB>::NPL, PV = Planes<T, VB>::PV;
  const int N = A.N, n_det = A.n_det, n_ang = A.n_ang;
  const int m_rays = n_ang * n_det;
  const int jb = blockIdx.x * kBTJ, ib = blockIdx.y * kBTI;
  // each wave covers a 16 (j) x 4 (i) patch: a 16-lane ds_read_b128 group then spans
  // <= ~16 detector bins for any angle (64 x 1 rows spanned up to 27 -> bank conflicts)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int j = jb + 16 * (wv % kBkPatchJ) + (lane & 15);
  const int i = ib + 4 * (wv / kBkPatchJ) + (lane >> 4);
  const bool inb = (i < N) && (j < N);
  const int chunk = blockIdx.z;
  const int v0 = chunk * VB;
  const int nv = (MODE == BACK_WSQ) ? 1 : min(VB, A.V - v0);
  // geometry uses clamped coordinates so out-of-image threads stay inside the window;
  // the angle records are uniform -> scalar loads (shared table, scalar-cache resident)
  const double c0 = 0.5 * (N - 1);
  const double xi = (double)min(i, N - 1) - c0, yj = (double)min(j, N - 1) - c0;
  const int jhi = min(jb + kBTJ - 1, N - 1), ihi = min(ib + kBTI - 1, N - 1);
  // bin positions are biased by an integer (admm_ctx: smallest k_f of any pixel, negated, + 2),
  // so k_f > 0: floor is the truncating convert and the tap fraction one v_fract_f64; window
  // offsets and the staged bins take the same bias
  const int kbias = A.kbias;
  const double Kc = A.K + (double)kbias;
  const double Kcb = Kc + kKfBias;  // (float taps, kf_split)
  constexpr bool FB = std::is_same<T, float>::value;  // biased window offsets (kf_split)

  // angles per staged chunk: halved for 64-B sample vectors (8 float64 nodes) so the
  // window stays at 48 KB of LDS
  // (the DIAG epilogue's tile scratch needs LDS too: its windows stay within 96 KB)
  constexpr int ANGC_ = (NPL > 2) ? kBAngC / 2 : kBAngC;
  constexpr int ANGC_DIAG = (98304 / (NPL * kBWin * (int)sizeof(Pack<T, PV>))) & ~3;
  constexpr int ANGC = (MODE == BACK_DIAG && ANGC_ > ANGC_DIAG) ? ANGC_DIAG : ANGC_;
  static_assert(ANGC % 4 == 0, "angle chunks are read as int4 groups");
  __shared__ Pack<T, PV> win[NPL][(MODE == BACK_WSQ) ? 1 : ANGC][kBWin];
  __shared__ int4 kmin_s[2][ANGC / 4 + 1];  // per angle: window byte offset koff (see tap); + a spare slot
  T acc[VB];
#pragma unroll
  for (int u = 0; u < VB; ++u) acc[u] = T(0);
  const T* sino_c = A.sino + (size_t)chunk * m_rays * VB;
  int t0c = 0;  // first angle of the current chunk (float64 weight path)

  // window taps address LDS by byte offset: koff = (slot * kBWin - kmin) * sizeof(Pack) is formed
  // once per angle and chunk (kmin_chunk), so a tap's address is one v_lshl_add of k0
  constexpr int PB = (int)sizeof(Pack<T, PV>);
  auto tap = [&](const BackAngleC& g, int koff, T& w0, T& w1, Pack<T, PV> (&s0)[NPL], Pack<T, PV> (&s1)[NPL],
                 int tt) {
    int k0, off;
    if constexpr (std::is_same<T, float>::value) {
      // one v_pk_fma_f32 for both taps (bitwise the two scalar fmas: f * (-sL) == (-f) * sL)
      // wc to VGPRs by one v_mov_b64 (the compiler emits two v_mov_b32; VOP3P reads one SGPR
      // pair).  max(0, w) is the fma's clamp to [0, 1]: the host scales ws, wc by 2^-wexp so
      // that w <= L 2^-wexp <= 1 (wexp = 0 for N >= 3), undone exactly after the angle loop
      unsigned hi;
      float2v wc, fv, w;
      float fu;
      kf_split(fma(xi, g.Bi, fma(yj, g.Bj, Kcb)), hi, fu);  // (fu: frac x 2^32; ws carries 2^-32)
      fv.x = fu;  // op_sel_hi:[0,...] reads the low half for both lanes of the pair
      asm("v_mov_b64 %0, %1" : "=v"(wc) : "s"(g.wc));
      asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1] clamp" : "=v"(w) : "v"(fv), "s"(g.ws), "v"(wc));
      w0 = w.x;
      w1 = w.y;
      k0 = (int)(hi - kKfHi);
      off = kf_addr<PB>(hi, koff);  // (koff carries -kKfHi x PB)
    } else {
      const double kf = fma(xi, g.Bi, fma(yj, g.Bj, Kc));
      k0 = (int)kf;  // == floor(kf): kf > 0
      const T f = (T)__builtin_amdgcn_fract(kf);
      const BackAngle& gd = A.ang[t0c + tt];
      w0 = fmax(T(0), T(1) - f * (T)gd.slope) * (T)gd.L;
      w1 = fmax(T(0), T(1) - (T(1) - f) * (T)gd.slope) * (T)gd.L;
      off = k0 * PB + koff;
    }
    if constexpr (MODE == BACK_WSQ) {
      (void)off;
      w0 = (k0 >= kbias && k0 <= kbias + n_det - 1) ? w0 : T(0);
      w1 = (k0 >= kbias - 1 && k0 <= kbias + n_det - 2) ? w1 : T(0);
    } else {
#pragma unroll
      for (int q = 0; q < NPL; ++q) {
        const char* wb = reinterpret_cast<const char*>(&win[q][0][0]) + off;
        s0[q] = *reinterpret_cast<const Pack<T, PV>*>(wb);
        s1[q] = *reinterpret_cast<const Pack<T, PV>*>(wb + PB);
      }
    }
  };
  auto fmac = [&](T w0, T w1, const Pack<T, PV> (&s0)[NPL], const Pack<T, PV> (&s1)[NPL]) {
    if constexpr (MODE == BACK_WSQ) {
      acc[0] = fma(w0, w0, acc[0]);
      acc[0] = fma(w1, w1, acc[0]);
    } else {
#pragma unroll
      for (int q = 0; q < NPL; ++q)
#pragma unroll
        for (int e = 0; e < PV; ++e) {
          acc[q * PV + e] = fma(w0, s0[q].v[e], acc[q * PV + e]);
          acc[q * PV + e] = fma(w1, s1[q].v[e], acc[q * PV + e]);
        }
    }
  };

  // sinogram windows (MODE != WSQ).  PF: the next chunk's window is fetched into
  // registers before this chunk's taps and written to LDS after them (the single block per
  // CU otherwise waits for every chunk's loads with nothing to overlap; +12 VGPRs, still
  // 4 waves/SIMD); kmin is double-buffered.  Otherwise: compute kmin, stage, tap per chunk.
  // (float samples, H/INIT modes: the float64 and DIAG variants would spill)
  constexpr bool PF = (std::is_same<T, float>::value || NPL <= 2) && (MODE == BACK_H || MODE == BACK_INIT ||
                                                                     MODE == BACK_PLAIN || MODE == BACK_ATB);
  constexpr int SPER = (ANGC * kBWin * NPL + kBkThreads - 1) / kBkThreads;
  Pack<T, PV> wst[SPER];
  // a chunk's window offsets from its angle records; the record load (kmin_load) is split from
  // the offset computation (kmin_store) so the PF pipeline issues it a chunk ahead, under the
  // taps, instead of exposing its latency between the chunk-end barriers (one block per CU at
  // 512^2: nothing else on the CU would cover it)
  auto kmin_load = [&](int t0) {  // every thread loads (index clamped): no select, no zero-fill
    const BackAngleC& g = A.angc[min(t0 + (int)threadIdx.x, n_ang - 1)];
    return make_double2(g.Bi, g.Bj);
  };
  auto kmin_store = [&](int t0, int buf, double2 bij) {
    // the record is consumed by every thread (only the store is masked): its load is then
    // complete on every path, and the next chunk's load into the same registers needs no
    // vmcnt(0) -- which would also wait for the window prefetch issued before it
    auto kf = [&](int ii, int jj) { return fma((double)ii - c0, bij.x, fma((double)jj - c0, bij.y, Kc)); };
    const double kmn = fmin(fmin(kf(ib, jb), kf(ib, jhi)), fmin(kf(ihi, jb), kf(ihi, jhi)));
    int koff = ((int)threadIdx.x * kBWin - ((int)floor(kmn) - 1)) * PB;
    if constexpr (FB) koff = (int)((unsigned)koff - kKfHi * (unsigned)PB);  // (kf_split)
    // unmasked store (threads past the chunk's angles write slots no tap reads, or the spare
    // one): a masked store lets the compiler sink the whole computation under the mask
    reinterpret_cast<int*>(kmin_s[buf])[min((int)threadIdx.x, ANGC)] = koff;
    (void)t0;
  };
  auto kmin_chunk = [&](int t0, int buf) { kmin_store(t0, buf, kmin_load(t0)); };
  auto wfetch = [&](int t0, int buf) {
    const int nt = min(ANGC, n_ang - t0);
#pragma unroll
    for (int e = 0; e < SPER; ++e) {
      const int q = threadIdx.x + e * kBkThreads;
      const int pl = q % NPL, aw = q / NPL;
      const int a = aw / kBWin, w = aw - a * kBWin;
      int ko = (a < nt) ? reinterpret_cast<const int*>(kmin_s[buf])[a] : 0;
      if constexpr (FB) ko = (int)((unsigned)ko + kKfHi * (unsigned)PB);  // the unbiased offset
      const int k = (a < nt) ? a * kBWin - ko / PB + w - kbias : -1;
      if (a < nt && k >= 0 && k < n_det) {
        wst[e] = *reinterpret_cast<const Pack<T, PV>*>(sino_c + ((size_t)(t0 + a) * n_det + k) * VB + pl * PV);
      } else {
#pragma unroll
        for (int z = 0; z < PV; ++z) wst[e].v[z] = T(0);
      }
    }
  };
  auto wcommit = [&](int t0) {
    const int nt = min(ANGC, n_ang - t0);
#pragma unroll
    for (int e = 0; e < SPER; ++e) {
      const int q = threadIdx.x + e * kBkThreads;
      const int pl = q % NPL, aw = q / NPL;
      const int a = aw / kBWin, w = aw - a * kBWin;
      if (a < nt) win[pl][a][w] = wst[e];
    }
  };
  if constexpr (CSR) {
    // explicit matrix: this pixel's row of A^T (same tile / epilogue as the projector)
    if (inb) {
      const int pix = i * N + j;
      Pack<T, VB> sv;
      for (int k = A.csr_ptr[pix]; k < A.csr_ptr[pix + 1]; ++k) {
        const T w = A.csr_val[k];
        if constexpr (MODE == BACK_WSQ) {
          acc[0] = fma(w, w, acc[0]);
        } else {
          sv = *reinterpret_cast<const Pack<T, VB>*>(sino_c + (size_t)A.csr_idx[k] * VB);
#pragma unroll
          for (int u = 0; u < VB; ++u) acc[u] = fma(w, sv.v[u], acc[u]);
        }
      }
    }
  }
  if constexpr (PF && !CSR) {
    kmin_chunk(0, 0);
    __syncthreads();
    wfetch(0, 0);
    wcommit(0);
    if (ANGC < n_ang) kmin_chunk(ANGC, 1);
    __syncthreads();
  }
  for (int t0 = 0, ci = 0; !CSR && t0 < n_ang; t0 += ANGC, ++ci) {
    const int nt = min(ANGC, n_ang - t0);
    const int kb = (PF) ? (ci & 1) : 0;  // kmin buffer of this chunk
    double2 rec2;  // (PF) angle records of the chunk after next, loaded under this chunk's taps
    if constexpr (PF) {
      // (the record load first: a wait the compiler places before it then covers only older,
      // already consumed loads, not the window prefetch issued after it)
      rec2 = kmin_load(min(t0 + 2 * ANGC, n_ang - 1));
      if (t0 + ANGC < n_ang) wfetch(t0 + ANGC, kb ^ 1);  // in flight during this chunk's taps
    } else if constexpr (MODE != BACK_WSQ) {
      __syncthreads();
      kmin_chunk(t0, 0);
      __syncthreads();
      wfetch(t0, 0);
      wcommit(t0);
      __syncthreads();
    }
    // angles in groups of 4: the group's constants are scalar-loaded together (one
    // lgkmcnt(0) per group -- scalar and LDS loads share that counter), then its taps
    // run on LDS reads alone
    t0c = t0;
    int tt = 0;
    const BackAngleC* gq = A.angc + t0;  // (records at non-negative immediate offsets of one base)
    for (; tt + 4 <= nt; tt += 4, gq += 4) {
      BackAngleC g[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) g[u] = gq[u];
      int4 km = make_int4(0, 0, 0, 0);
      if constexpr (MODE != BACK_WSQ) km = kmin_s[kb][tt >> 2];
      const int kms[4] = {km.x, km.y, km.z, km.w};
#pragma unroll
      for (int u = 0; u < 4; u += 2) {
        T wa0, wa1, wb0, wb1;
        Pack<T, PV> sa0[NPL], sa1[NPL], sb0[NPL], sb1[NPL];
        tap(g[u], kms[u], wa0, wa1, sa0, sa1, tt + u);
        tap(g[u + 1], kms[u + 1], wb0, wb1, sb0, sb1, tt + u + 1);
        fmac(wa0, wa1, sa0, sa1);
        fmac(wb0, wb1, sb0, sb1);
      }
    }
    for (; tt < nt; ++tt) {
      const BackAngleC g = A.angc[t0 + tt];
      int km = 0;
      if constexpr (MODE != BACK_WSQ) km = reinterpret_cast<const int*>(kmin_s[kb])[tt];
      T wa0, wa1;
      Pack<T, PV> sa0[NPL], sa1[NPL];
      tap(g, km, wa0, wa1, sa0, sa1, tt);
      fmac(wa0, wa1, sa0, sa1);
    }
    if constexpr (PF) {
      if (t0 + ANGC < n_ang) {
        __syncthreads();  // this chunk's taps are done with win and kmin_s[kb]
        wcommit(t0 + ANGC);
        kmin_store(t0 + 2 * ANGC, kb, rec2);  // (garbage past the last chunk: never read)
        __syncthreads();
      }
    }
  }

  if constexpr (std::is_same<T, float>::value && !CSR) {
    if (A.wexp != 0) {  // undo the weight scaling (a power of two: exact)
      const int e = (MODE == BACK_WSQ) ? 2 * A.wexp : A.wexp;
#pragma unroll
      for (int u = 0; u < VB; ++u) acc[u] = ldexpf(acc[u], e);
    }
  }
  double pq[VB][NQ];
#pragma unroll
  for (int u = 0; u < VB; ++u)
#pragma unroll
    for (int q = 0; q < NQ; ++q) pq[u][q] = 0.0;
  if constexpr (MODE == BACK_DIAG) {
    __shared__ double diag_s[kDiagScratch];
    diag_epilogue_tile<T, VB>(A, diag_s, ib, jb, i, j, inb, chunk, v0, nv, acc, pq);
  } else if (inb) {
    back_epilogue<T, VB, MODE, NQ>(A, i, j, chunk, v0, nv, acc, pq);
  }

  if constexpr (MODE == BACK_H || MODE == BACK_DIAG) {
    constexpr int NT = VB * NQ, NS = RsShape<NT>::NS;
    __shared__ double lds[kBkWaves * NS];
    __shared__ double tot[NS];
    double flat[NT];
#pragma unroll
    for (int u = 0; u < VB; ++u)
#pragma unroll
      for (int q = 0; q < NQ; ++q) flat[u * NQ + q] = pq[u][q];
    block_reduce_flat<NT, kBkWaves>(flat, lds, tot);
    const int t = threadIdx.x;
    if (t < VB * NQ && t / NQ < nv) {
      const int P = gridDim.x * gridDim.y;
      const int b = blockIdx.y * gridDim.x + blockIdx.x;
      A.part[((size_t)v0 * NQ + t) * P + b] = tot[t];
    }
  }
}

// ===========================================================================
// Mirror-mode back projector (the adjoint of k_fwdg<..., MIRROR>; admm_tomo.hip mirror mode).
// A virtual lane block holds real nodes at (i, j) (lanes < VB/2) and at (N-1-i, j) (lanes >=
// VB/2) over the first a/2 angles; its window bins are the real sinogram's rays (t, k) and
// (a-1-t, k).  The real A^T s at (i, j) is the virtual result at (i, j), lanes < VB/2, plus the
// virtual result at (N-1-i, j), lanes >= VB/2 -- so each thread takes the pixel PAIR (i, j),
// (N-1-i, j) of an upper-half tile (i < ceil(N/2)) and both pixels' real sums form in its own
// registers: per (pixel, angle) one address / weight computation serves VB lanes (8 float32
// lanes even for a 4-node batch), and the fused epilogues (H, INIT, DIAG, ATB) run unchanged on
// the real lane block of both pixels (back_epilogue / diag_epilogue_tile with VS = VBR lanes per
// real vector).  Two LDS windows per angle (upper tile, mirror tile) at half the angles per
// chunk keep the LDS size and the staged bytes per tap of k_back.
// ===========================================================================
// the mirror back projector of (T, VB, MODE) stages its windows by LDS-DMA (H mode, 16-byte
// window packs) unless instantiated with DMAQ = false (the register-staged windows: A/B and the
// bitwise test, ADMM_BK_STAGING=reg at context creation)
template <typename T, int VB, int MODE>
constexpr bool back_mirror_dma() {
  return ADMM_BK_DMA && MODE == BACK_H && Planes<T, VB>::NPL == 2 && sizeof(Pack<T, Planes<T, VB>::PV>) == 16;
}
template <typename T, int VB, int VBR, int MODE, bool DMAQ>
__device__ __forceinline__ void back_mirror_body(const BackArgs<T>& A) {
  static_assert(MODE == BACK_H || MODE == BACK_INIT || MODE == BACK_DIAG || MODE == BACK_ATB, "batch modes");
  constexpr int MH = VB / 2, MS = VBR / MH;
  static_assert(VB % 2 == 0 && VBR % MH == 0, "mirror: VB = 2 x (a divisor of VBR)");
  constexpr int NQ = (MODE == BACK_H || MODE == BACK_DIAG) ? 5 : 1;
  constexpr int NPL = Planes<T, VB>::NPL, PV = Planes<T, VB>::PV;
  constexpr int PB = (int)sizeof(Pack<T, PV>);
  const int N = A.N, n_det = A.n_det, n_ang = A.n_ang;  // n_ang: the half geometry's a/2 angles
  const int Nh = (N + 1) / 2;
  const size_t m_full = (size_t)2 * n_ang * n_det;
  const int jb = blockIdx.x * kBTJ, ib = blockIdx.y * kBTI;  // upper tile: rows ib .. (< Nh)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int j = jb + 16 * (wv % kBkPatchJ) + (lane & 15);
  const int i = ib + 4 * (wv / kBkPatchJ) + (lane >> 4);
  const int i2 = N - 1 - i;                  // the mirror pixel's row
  const bool inb = (i < Nh) && (j < N);
  const bool inb2 = inb && (i2 != i);        // (odd N: the middle row pairs with itself)
  const int chunk = blockIdx.z, rc = chunk / MS, mq = chunk % MS;
  const int v0 = rc * VBR + mq * MH;         // first real node of this lane block
  const int nv = min(MH, A.V - v0);
  const double c0 = 0.5 * (N - 1);
  // clamped coordinates keep out-of-tile threads inside the windows; the mirror pixel's
  // x-coordinate is exactly -xi ((N-1-i) - c0 = c0 - i)
  const double xi = (double)min(i, Nh - 1) - c0, yj = (double)min(j, N - 1) - c0;
  const int jhi = min(jb + kBTJ - 1, N - 1), ihi = min(ib + kBTI - 1, Nh - 1);
  const int kbias = A.kbias;
  const double Kc = A.K + (double)kbias;
  const double Kcb = Kc + kKfBias;  // (float taps, kf_split)
  constexpr bool FB = std::is_same<T, float>::value;  // biased window offsets (kf_split)
  constexpr int ANGC_ = ((NPL > 2) ? kBAngC / 2 : kBAngC) / 2;
  constexpr int ANGC_DIAG = (98304 / (2 * NPL * kBWin * PB)) & ~3;
  constexpr int ANGC = (MODE == BACK_DIAG && ANGC_ > ANGC_DIAG) ? ANGC_DIAG : ANGC_;
  static_assert(ANGC % 4 == 0 && ANGC >= 4, "angle chunks are read as int4 groups");
  // DMA (round 6, BACK_H with 16-byte window packs): the window bins go straight from the
  // sinogram into LDS by LDS-DMA (buffer_load ... lds, no staging VGPRs, no LDS writes by the
  // waves) into two chunk buffers; the byte offset of a chunk's buffer is folded into its koff,
  // so the taps' LDS bases stay compile-time constants.  One barrier per chunk instead of two:
  // the next chunk's DMA is issued before this chunk's taps and the barrier after them waits for
  // it; the window offsets (kmin_s) and first bins (kst_s) rotate over three slots, written two
  // chunks ahead.
  constexpr bool DMA = DMAQ && back_mirror_dma<T, VB, MODE>();
  constexpr int NWB = DMA ? 4 : 2, NKS = DMA ? 3 : 2;
  constexpr int BUFB = 2 * NPL * ANGC * kBWin * PB;  // bytes of one chunk's windows
  __shared__ Pack<T, PV> win[NWB][NPL][ANGC][kBWin];  // [buffer x 2 + window (upper / mirror tile)]
  __shared__ int4 kmin_s[NKS][2][ANGC / 4 + 1];       // [slot][window]: byte offsets koff
  __shared__ int kst_s[DMA ? 3 : 1][2][DMA ? ANGC + 1 : 1];  // DMA: [slot][window] first bin - kbias
  T acc1[VB], acc2[VB];
#pragma unroll
  for (int u = 0; u < VB; ++u) acc1[u] = acc2[u] = T(0);
  const T* sino_c = A.sino + (size_t)rc * m_full * VBR + mq * MH;  // the real lane block
  int t0c = 0;

  // window offsets of a chunk: per angle and window the floor of the smallest corner k_f
  // (upper tile rows ib .. ihi, mirror tile rows N-1-ihi .. N-1-ib); the record load is split
  // from the store so the pipeline issues it a chunk ahead (as in k_back)
  auto kmin_load = [&](int t0) {
    const BackAngleC& g = A.angc[min(t0 + ((int)threadIdx.x % ANGC), n_ang - 1)];
    return make_double2(g.Bi, g.Bj);
  };
  auto kmin_store = [&](int buf, double2 bij, int bo = 0) {  // bo: DMA buffer byte offset
    const int w = (int)threadIdx.x / ANGC;  // threads 0 .. 2 ANGC - 1: (window, angle)
    const double xa = (double)ib - c0, xb = (double)ihi - c0;
    const double x0 = w ? -xb : xa, x1 = w ? -xa : xb;  // the window's row range (x-coordinates)
    auto kf = [&](double xx, int jj) { return fma(xx, bij.x, fma((double)jj - c0, bij.y, Kc)); };
    const double kmn = fmin(fmin(kf(x0, jb), kf(x0, jhi)), fmin(kf(x1, jb), kf(x1, jhi)));
    const int a = (int)threadIdx.x % ANGC;
    const int k0w = (int)floor(kmn) - 1;  // the window's first bin (+ kbias)
    int koff = (a * kBWin - k0w) * PB;
    if constexpr (FB) koff = (int)((unsigned)koff - kKfHi * (unsigned)PB);  // (kf_split)
    if constexpr (DMA) {
      koff = (int)((unsigned)koff + (unsigned)bo);
      kst_s[buf][min(w, 1)][w < 2 ? a : ANGC] = k0w - kbias;
    }
    reinterpret_cast<int*>(kmin_s[buf][min(w, 1)])[w < 2 ? a : ANGC] = koff;  // (spare slot)
  };
  auto kmin_chunk = [&](int t0, int buf) { kmin_store(buf, kmin_load(t0)); };
  auto kmin_chunk_b = [&](int t0, int buf, int bo) { kmin_store(buf, kmin_load(t0), bo); };
  constexpr int NE = 2 * ANGC * kBWin * NPL;  // staged packs per chunk
  constexpr int SPER = (NE + kBkThreads - 1) / kBkThreads;
  Pack<T, PV> wst[SPER];
  // (16-byte planes: the window bins as buffer loads at 32-bit offsets from one scalar base; a
  // bin outside the detector is an out-of-range offset, zero-filled by the hardware)
  constexpr bool WBUF = NPL == 2 && sizeof(Pack<T, PV>) == 16;
  const __amdgpu_buffer_rsrc_t rs_sino = [&] {
    const uint64_t b = (uint64_t)(uintptr_t)sino_c;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    return make_rsrc((const void*)(uintptr_t)(((uint64_t)hi << 32) | lo), (uint32_t)(m_full * VBR * sizeof(T)));
  }();
  auto wfetch = [&](int t0, int buf) {
    const int nt = min(ANGC, n_ang - t0);
#pragma unroll
    for (int e = 0; e < SPER; ++e) {
      const int q = threadIdx.x + e * kBkThreads;
      const int pl = q % NPL, rest = q / NPL, bin = rest % kBWin, aw = rest / kBWin;
      const int a = aw % ANGC, w = aw / ANGC;
      const bool live = q < NE && a < nt;
      int ko = live ? reinterpret_cast<const int*>(kmin_s[buf][w])[a] : 0;
      if constexpr (FB) ko = (int)((unsigned)ko + kKfHi * (unsigned)PB);  // the unbiased offset
      const int k = live ? a * kBWin - ko / PB + bin - kbias : -1;
      const int t = t0 + a;
      if constexpr (WBUF) {
        const int ray = (pl ? 2 * n_ang - 1 - t : t) * n_det + k;
        const int voff = (live && k >= 0 && k < n_det) ? ray * (VBR * (int)sizeof(T)) : -1;
        vload<T, PV>(rs_sino, voff, 0, wst[e].v);
        continue;
      }
      const size_t ray0 = (size_t)t * n_det + k, ray1 = (size_t)(2 * n_ang - 1 - t) * n_det + k;
      if (live && k >= 0 && k < n_det) {
        if constexpr (NPL == 2) {  // virtual plane pl = orientation pl: one 16-B real plane
          wst[e] = *reinterpret_cast<const Pack<T, PV>*>(sino_c + (pl ? ray1 : ray0) * VBR);
        } else {                   // one virtual plane holds both orientations: element gather
#pragma unroll
          for (int z = 0; z < PV; ++z) wst[e].v[z] = z < MH ? sino_c[ray0 * VBR + z] : sino_c[ray1 * VBR + z - MH];
        }
      } else {
#pragma unroll
        for (int z = 0; z < PV; ++z) wst[e].v[z] = T(0);
      }
    }
  };
  auto wcommit = [&](int t0) {
    const int nt = min(ANGC, n_ang - t0);
#pragma unroll
    for (int e = 0; e < SPER; ++e) {
      const int q = threadIdx.x + e * kBkThreads;
      const int pl = q % NPL, rest = q / NPL, bin = rest % kBWin, aw = rest / kBWin;
      const int a = aw % ANGC, w = aw / ANGC;
      if (q < NE && a < nt) win[w][pl][a][bin] = wst[e];
    }
  };
  // one angle's taps of one pixel from window W (k_back's tap; float: kf is biased, kf_split)
  auto tap1 = [&](auto wc_, const BackAngleC& g, double kf, int koff, int tt, T(&acc)[VB]) {
    constexpr int w = decltype(wc_)::value;
    {
      T w0, w1;
      int off;
      if constexpr (std::is_same<T, float>::value) {
        unsigned hi;
        float2v wc, fv, ww;
        float fu;
        kf_split(kf, hi, fu);
        fv.x = fu;
        asm("v_mov_b64 %0, %1" : "=v"(wc) : "s"(g.wc));
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1] clamp" : "=v"(ww) : "v"(fv), "s"(g.ws), "v"(wc));
        w0 = ww.x;
        w1 = ww.y;
        off = kf_addr<PB>(hi, koff);  // (koff carries -kKfHi x PB)
      } else {
        const int k0 = (int)kf;  // == floor(kf): kf > 0
        const T f = (T)__builtin_amdgcn_fract(kf);
        const BackAngle& gd = A.ang[t0c + tt];
        w0 = fmax(T(0), T(1) - f * (T)gd.slope) * (T)gd.L;
        w1 = fmax(T(0), T(1) - (T(1) - f) * (T)gd.slope) * (T)gd.L;
        off = k0 * PB + koff;
      }
#pragma unroll
      for (int q = 0; q < NPL; ++q) {
        const char* wb = reinterpret_cast<const char*>(&win[w][q][0][0]) + off;
        const Pack<T, PV> s0 = *reinterpret_cast<const Pack<T, PV>*>(wb);
        const Pack<T, PV> s1 = *reinterpret_cast<const Pack<T, PV>*>(wb + PB);
#pragma unroll
        for (int e = 0; e < PV; ++e) {
          acc[q * PV + e] = fma(w0, s0.v[e], acc[q * PV + e]);
          acc[q * PV + e] = fma(w1, s1.v[e], acc[q * PV + e]);
        }
      }
    }
  };
  // both pixels: kf at xi and at -xi (the mirror pixel), sharing the j term
  auto tap2 = [&](const BackAngleC& g, int koff1, int koff2, int tt) {
    const double inner = fma(yj, g.Bj, FB ? Kcb : Kc);
    tap1(std::integral_constant<int, 0>{}, g, fma(xi, g.Bi, inner), koff1, tt, acc1);
    tap1(std::integral_constant<int, 1>{}, g, fma(-xi, g.Bi, inner), koff2, tt, acc2);
  };
  // one chunk's taps, window offsets from kmin_s[kb]
  auto chunk_taps = [&](int t0, int nt, int kb) {
    t0c = t0;
    int tt = 0;
    // (records at non-negative immediate offsets of one base, read through the constant address
    // space: scalar loads even where the LDS-DMA intrinsic hides from the compiler that nothing
    // writes them -- as generic loads they became vector loads whose vmcnt waits also drained
    // the next chunk's DMA)
    using CRec = const __attribute__((address_space(4))) BackAngleC;
    auto rec = [](CRec* r) {  // field by field (no copy constructor binds an address_space(4) object)
      BackAngleC g;
      g.Bi = r->Bi;
      g.Bj = r->Bj;
      g.ws = r->ws;
      g.wc = r->wc;
      return g;
    };
    CRec* gq = (CRec*)(uintptr_t)(A.angc + t0);
    for (; tt + 4 <= nt; tt += 4, gq += 4) {
      BackAngleC g[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) g[u] = rec(gq + u);
      const int4 k1 = kmin_s[kb][0][tt >> 2], k2 = kmin_s[kb][1][tt >> 2];
      tap2(g[0], k1.x, k2.x, tt);
      tap2(g[1], k1.y, k2.y, tt + 1);
      tap2(g[2], k1.z, k2.z, tt + 2);
      tap2(g[3], k1.w, k2.w, tt + 3);
    }
    for (; tt < nt; ++tt) {
      const BackAngleC g = rec((CRec*)(uintptr_t)A.angc + t0 + tt);
      tap2(g, reinterpret_cast<const int*>(kmin_s[kb][0])[tt], reinterpret_cast<const int*>(kmin_s[kb][1])[tt], tt);
    }
  };
  if constexpr (DMA) {
    // this wave's NI 64-slot pieces of a chunk (slot = ((window x NPL + plane) x ANGC + angle)
    // x kBWin + bin, the windows' LDS order): fixed for the kernel, so their bin / angle /
    // plane / window are formed once
    constexpr int NI = NE / (64 * kBkWaves);
    static_assert(NE % (64 * kBkWaves) == 0, "whole 64-slot pieces per wave");
    const int wvu = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    int pbin[NI], pang[NI], pwin[NI];
    bool pmir[NI];
#pragma unroll
    for (int e = 0; e < NI; ++e) {
      const int q = (wvu * NI + e) * 64 + lane;
      pbin[e] = q % kBWin;
      const int rest = q / kBWin;
      pang[e] = rest % ANGC;
      pmir[e] = (rest / ANGC) % NPL;
      pwin[e] = rest / (ANGC * NPL);
    }
    auto dma = [&](int t0, int ks, int bo) {
      const int nt = min(ANGC, n_ang - t0);
#pragma unroll
      for (int e = 0; e < NI; ++e) {
        const int a = pang[e], t = t0 + a;
        const int k = kst_s[ks][pwin[e]][a] + pbin[e];
        const int ray = (pmir[e] ? 2 * n_ang - 1 - t : t) * n_det + k;
        // bins off the detector (and angles past a short last chunk) are out-of-range offsets:
        // the hardware writes zeros
        const unsigned voff = (a < nt && k >= 0 && k < n_det) ? (unsigned)ray * (unsigned)(VBR * sizeof(T)) : 0xFFFFFFFFu;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rs_sino,
            (__attribute__((address_space(3))) void*)(reinterpret_cast<char*>(&win[0][0][0][0]) + bo +
                                                       (wvu * NI + e) * 64 * PB),
            16, voff, 0, 0, 0);
      }
    };
    kmin_chunk_b(0, 0, 0);
    if (ANGC < n_ang) kmin_chunk_b(ANGC, 1, BUFB);
    __syncthreads();
    dma(0, 0, 0);
    __syncthreads();  // (its fence waits for this wave's LDS-DMA) chunk 0 staged
    for (int t0 = 0, ci = 0, ks = 0; t0 < n_ang; t0 += ANGC, ++ci, ks = ks == 2 ? 0 : ks + 1) {
      const int nt = min(ANGC, n_ang - t0);
      const double2 rec2 = kmin_load(min(t0 + 2 * ANGC, n_ang - 1));
      const int ks1 = ks == 2 ? 0 : ks + 1, ks2 = ks1 == 2 ? 0 : ks1 + 1;
      // the next chunk into the other buffer (last read by the previous chunk's taps, done at
      // the previous barrier), in flight during this chunk's taps
      if (t0 + ANGC < n_ang) dma(t0 + ANGC, ks1, (ci & 1) ? 0 : BUFB);
      chunk_taps(t0, nt, ks);
      if (t0 + ANGC < n_ang) {
        // chunk + 2's offsets into the slot chunk - 1 used (its taps and DMA are done); its
        // buffer is this chunk's (the same parity)
        if (t0 + 2 * ANGC < n_ang) kmin_store(ks2, rec2, (ci & 1) ? BUFB : 0);
        __syncthreads();  // next chunk's DMA landed (fence), this chunk's taps done, slot ks2 visible
      }
    }
  } else {
    // register-prefetched chunk pipeline (k_back's PF path)
    kmin_chunk(0, 0);
    __syncthreads();
    wfetch(0, 0);
    wcommit(0);
    if (ANGC < n_ang) kmin_chunk(ANGC, 1);
    __syncthreads();
    for (int t0 = 0, ci = 0; t0 < n_ang; t0 += ANGC, ++ci) {
      const int nt = min(ANGC, n_ang - t0);
      const int kb = ci & 1;
      const double2 rec2 = kmin_load(min(t0 + 2 * ANGC, n_ang - 1));
      if (t0 + ANGC < n_ang) wfetch(t0 + ANGC, kb ^ 1);  // in flight during this chunk's taps
      chunk_taps(t0, nt, kb);
      if (t0 + ANGC < n_ang) {
        __syncthreads();  // this chunk's taps are done with win and kmin_s[kb]
        wcommit(t0 + ANGC);
        kmin_store(kb, rec2);  // (garbage past the last chunk: never read)
        __syncthreads();
      }
    }
  }
  if constexpr (std::is_same<T, float>::value) {
    if (A.wexp != 0) {
#pragma unroll
      for (int u = 0; u < VB; ++u) {
        acc1[u] = ldexpf(acc1[u], A.wexp);
        acc2[u] = ldexpf(acc2[u], A.wexp);
      }
    }
  }
  // the real A^T s of both pixels: angles < a/2 from the pixel itself, angles >= a/2 from the
  // mirror pixel's mirrored lanes (fixed order: first half + second half)
  T r1[MH], r2[MH];
#pragma unroll
  for (int h = 0; h < MH; ++h) {
    r1[h] = acc1[h] + acc2[MH + h];
    r2[h] = acc2[h] + acc1[MH + h];
  }
  double pq[MH][NQ];
#pragma unroll
  for (int u = 0; u < MH; ++u)
#pragma unroll
    for (int q = 0; q < NQ; ++q) pq[u][q] = 0.0;
  if constexpr (MODE == BACK_DIAG) {
    __shared__ double diag_s[kDiagScratch];
    diag_epilogue_tile<T, MH, VBR>(A, diag_s, ib, jb, i, j, inb, rc, v0, nv, r1, pq, mq * MH);
    diag_epilogue_tile<T, MH, VBR>(A, diag_s, N - ib - kBTI, jb, i2, j, inb2, rc, v0, nv, r2, pq, mq * MH);
  } else {
    if (inb) back_epilogue<T, MH, MODE, NQ, VBR>(A, i, j, rc, v0, nv, r1, pq, mq * MH);
    if (inb2) back_epilogue<T, MH, MODE, NQ, VBR, true>(A, i2, j, rc, v0, nv, r2, pq, mq * MH);
  }
  if constexpr (MODE == BACK_H || MODE == BACK_DIAG) {
    constexpr int NT = MH * NQ, NS = RsShape<NT>::NS;
    __shared__ double lds[kBkWaves * NS];
    __shared__ double tot[NS];
    double flat[NT];
#pragma unroll
    for (int u = 0; u < MH; ++u)
#pragma unroll
      for (int q = 0; q < NQ; ++q) flat[u * NQ + q] = pq[u][q];
    block_reduce_flat<NT, kBkWaves>(flat, lds, tot);
    const int t = threadIdx.x;
    if (t < MH * NQ && t / NQ < nv) {
      const int P = gridDim.x * gridDim.y;
      const int b = blockIdx.y * gridDim.x + blockIdx.x;
      A.part[((size_t)v0 * NQ + t) * P + b] = tot[t];
    }
  }
}

// the kernels: windows by LDS-DMA where back_mirror_dma (the default), register-staged
// (k_back_mirror_reg, ADMM_BK_STAGING=reg at context creation; the same results bit for bit)
template <typename T, int VB, int VBR, int MODE>
__global__ __launch_bounds__(kBkThreads) void k_back_mirror(BackArgs<T> A) {
  back_mirror_body<T, VB, VBR, MODE, true>(A);
}
template <typename T, int VB, int VBR, int MODE>
__global__ __launch_bounds__(kBkThreads) void k_back_mirror_reg(BackArgs<T> A) {
  back_mirror_body<T, VB, VBR, MODE, false>(A);
}

// ===========================================================================
// Mirror back projector, H mode, two lane blocks per block (round 6, `ADMM_BK_LB2`): the same
// pixel tile of lane blocks 2z and 2z + 1 (8 real nodes).  A tap's position, weights and LDS
// address are formed once and applied to both lane blocks' windows (the per-tap overhead of
// k_back_mirror is paid per 8 nodes instead of 4), the windows arrive by LDS-DMA as in
// k_back_mirror's DMA path (half the angles per chunk: the two lane blocks' windows in two
// buffers fill the same 98 KB), and the grid is half as many blocks.  Per lane block the
// arithmetic is k_back_mirror's in the same order: bitwise the same Hp and dot partials.
// ===========================================================================
template <typename T, int VB, int VBR>
__global__ __launch_bounds__(kBkThreads) void k_back_mirror_2(BackArgs<T> A) {
  constexpr int MODE = BACK_H, NQ = 5, LB = 2;
  constexpr int MH = VB / 2, MS = VBR / MH;
  static_assert(VB % 2 == 0 && VBR % MH == 0, "mirror: VB = 2 x (a divisor of VBR)");
  constexpr int NPL = Planes<T, VB>::NPL, PV = Planes<T, VB>::PV;
  constexpr int PB = (int)sizeof(Pack<T, PV>);
  static_assert(std::is_same<T, float>::value && NPL == 2 && PB == 16, "float32 16-byte window packs");
  const int N = A.N, n_det = A.n_det, n_ang = A.n_ang;  // n_ang: the half geometry's a/2 angles
  const int Nh = (N + 1) / 2;
  const size_t m_full = (size_t)2 * n_ang * n_det;
  const int jb = blockIdx.x * kBTJ, ib = blockIdx.y * kBTI;  // upper tile: rows ib .. (< Nh)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int j = jb + 16 * (wv % kBkPatchJ) + (lane & 15);
  const int i = ib + 4 * (wv / kBkPatchJ) + (lane >> 4);
  const int i2 = N - 1 - i;                  // the mirror pixel's row
  const bool inb = (i < Nh) && (j < N);
  const bool inb2 = inb && (i2 != i);        // (odd N: the middle row pairs with itself)
  const double c0 = 0.5 * (N - 1);
  const double xi = (double)min(i, Nh - 1) - c0, yj = (double)min(j, N - 1) - c0;
  const int jhi = min(jb + kBTJ - 1, N - 1), ihi = min(ib + kBTI - 1, Nh - 1);
  const int kbias = A.kbias;
  const double Kc = A.K + (double)kbias;
  const double Kcb = Kc + kKfBias;  // (kf_split)
  constexpr int ANGC = kBAngC / 4;  // half of k_back_mirror's: two lane blocks' windows per buffer
  static_assert(ANGC % 4 == 0 && ANGC >= 4, "angle chunks are read as int4 groups");
  constexpr int WINB = 2 * NPL * ANGC * kBWin * PB;  // bytes of one lane block's windows per chunk
  constexpr int BUFB = LB * WINB;                    // bytes of one chunk buffer
  __shared__ Pack<T, PV> win[2 * LB * 2][NPL][ANGC][kBWin];  // [buffer][lane block][window]
  __shared__ int4 kmin_s[3][2][ANGC / 4 + 1];                // [slot][window]: byte offsets koff
  __shared__ int kst_s[3][2][ANGC + 1];                      // [slot][window]: first bin - kbias
  T acc1[LB][VB], acc2[LB][VB];
#pragma unroll
  for (int l = 0; l < LB; ++l)
#pragma unroll
    for (int u = 0; u < VB; ++u) acc1[l][u] = acc2[l][u] = T(0);

  auto kmin_load = [&](int t0) {
    const BackAngleC& g = A.angc[min(t0 + ((int)threadIdx.x % ANGC), n_ang - 1)];
    return make_double2(g.Bi, g.Bj);
  };
  auto kmin_store = [&](int ks, double2 bij, int bo) {  // bo: the chunk buffer's byte offset
    const int w = (int)threadIdx.x / ANGC;  // threads 0 .. 2 ANGC - 1: (window, angle)
    const double xa = (double)ib - c0, xb = (double)ihi - c0;
    const double x0 = w ? -xb : xa, x1 = w ? -xa : xb;  // the window's row range (x-coordinates)
    auto kf = [&](double xx, int jj) { return fma(xx, bij.x, fma((double)jj - c0, bij.y, Kc)); };
    const double kmn = fmin(fmin(kf(x0, jb), kf(x0, jhi)), fmin(kf(x1, jb), kf(x1, jhi)));
    const int a = (int)threadIdx.x % ANGC;
    const int k0w = (int)floor(kmn) - 1;  // the window's first bin (+ kbias)
    const int koff = (int)((unsigned)((a * kBWin - k0w) * PB) - kKfHi * (unsigned)PB + (unsigned)bo);
    kst_s[ks][min(w, 1)][w < 2 ? a : ANGC] = k0w - kbias;                      // (spare slot)
    reinterpret_cast<int*>(kmin_s[ks][min(w, 1)])[w < 2 ? a : ANGC] = koff;
  };
  constexpr int NE = LB * 2 * ANGC * kBWin * NPL;  // staged packs per chunk
  constexpr int NI = NE / (64 * kBkWaves);         // 64-slot pieces per wave
  static_assert(NE % (64 * kBkWaves) == 0 && (ANGC * kBWin) % 64 == 0, "whole pieces, one (lane block, window, plane) each");
  const int wvu = __builtin_amdgcn_readfirstlane(wv);
  auto dma = [&](int t0, int ks, int bo) {
    const int nt = min(ANGC, n_ang - t0);
#pragma unroll
    for (int e = 0; e < NI; ++e) {
      // slot q = (((lane block x 2 + window) x NPL + plane) x ANGC + angle) x kBWin + bin
      const int q0 = (wvu * NI + e) * 64;  // a piece lies in one (lane block, window, plane)
      const int q = q0 + lane;
      const int bin = q % kBWin, a = (q / kBWin) % ANGC;
      const int lwp = q0 / (ANGC * kBWin), pl = lwp % NPL, w = (lwp / NPL) % 2, l = lwp / (2 * NPL);
      const int z = (int)blockIdx.z * LB + l;
      const T* base = A.sino + (size_t)(z / MS) * m_full * VBR + (z % MS) * MH;  // lane block l
      const uint64_t b = (uint64_t)(uintptr_t)base;
      const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
      const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
      const __amdgpu_buffer_rsrc_t rs =
          make_rsrc((const void*)(uintptr_t)(((uint64_t)hi << 32) | lo), (uint32_t)(m_full * VBR * sizeof(T)));
      const int t = t0 + a;
      const int k = kst_s[ks][w][a] + bin;
      const int ray = (pl ? 2 * n_ang - 1 - t : t) * n_det + k;
      const unsigned voff = (a < nt && k >= 0 && k < n_det) ? (unsigned)ray * (unsigned)(VBR * sizeof(T)) : 0xFFFFFFFFu;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs, (__attribute__((address_space(3))) void*)(reinterpret_cast<char*>(&win[0][0][0][0]) + bo + q0 * PB), 16,
          voff, 0, 0, 0);
    }
  };
  // one angle's taps of one pixel from window W of both lane blocks: the weights and the LDS
  // address once (k_back_mirror's tap1), the two lane blocks' samples at the same offset
  auto tap1 = [&](auto wc_, const BackAngleC& g, double kf, int koff, T(&acc)[LB][VB]) {
    constexpr int w = decltype(wc_)::value;
    unsigned hi;
    float2v wc, fv, ww;
    float fu;
    kf_split(kf, hi, fu);
    fv.x = fu;
    asm("v_mov_b64 %0, %1" : "=v"(wc) : "s"(g.wc));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1] clamp" : "=v"(ww) : "v"(fv), "s"(g.ws), "v"(wc));
    const T w0 = ww.x, w1 = ww.y;
    const int off = kf_addr<PB>(hi, koff);  // (koff carries -kKfHi x PB and the buffer offset)
#pragma unroll
    for (int l = 0; l < LB; ++l)
#pragma unroll
      for (int q = 0; q < NPL; ++q) {
        const char* wb = reinterpret_cast<const char*>(&win[l * 2 + w][q][0][0]) + off;
        const Pack<T, PV> s0 = *reinterpret_cast<const Pack<T, PV>*>(wb);
        const Pack<T, PV> s1 = *reinterpret_cast<const Pack<T, PV>*>(wb + PB);
#pragma unroll
        for (int e = 0; e < PV; ++e) {
          acc[l][q * PV + e] = fma(w0, s0.v[e], acc[l][q * PV + e]);
          acc[l][q * PV + e] = fma(w1, s1.v[e], acc[l][q * PV + e]);
        }
      }
  };
  auto tap2 = [&](const BackAngleC& g, int koff1, int koff2) {
    const double inner = fma(yj, g.Bj, Kcb);
    tap1(std::integral_constant<int, 0>{}, g, fma(xi, g.Bi, inner), koff1, acc1);
    tap1(std::integral_constant<int, 1>{}, g, fma(-xi, g.Bi, inner), koff2, acc2);
  };
  using CRec = const __attribute__((address_space(4))) BackAngleC;
  auto rec = [](CRec* r) {  // field by field (no copy constructor binds an address_space(4) object)
    BackAngleC g;
    g.Bi = r->Bi;
    g.Bj = r->Bj;
    g.ws = r->ws;
    g.wc = r->wc;
    return g;
  };
  auto chunk_taps = [&](int t0, int nt, int ks) {
    int tt = 0;
    CRec* gq = (CRec*)(uintptr_t)(A.angc + t0);
    for (; tt + 4 <= nt; tt += 4, gq += 4) {
      BackAngleC g[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) g[u] = rec(gq + u);
      const int4 k1 = kmin_s[ks][0][tt >> 2], k2 = kmin_s[ks][1][tt >> 2];
      tap2(g[0], k1.x, k2.x);
      tap2(g[1], k1.y, k2.y);
      tap2(g[2], k1.z, k2.z);
      tap2(g[3], k1.w, k2.w);
    }
    for (; tt < nt; ++tt)
      tap2(rec(gq + (tt & 3)), reinterpret_cast<const int*>(kmin_s[ks][0])[tt],
           reinterpret_cast<const int*>(kmin_s[ks][1])[tt]);
  };
  kmin_store(0, kmin_load(0), 0);
  if (ANGC < n_ang) kmin_store(1, kmin_load(ANGC), BUFB);
  __syncthreads();
  dma(0, 0, 0);
  __syncthreads();  // (its fence waits for this wave's LDS-DMA) chunk 0 staged
  for (int t0 = 0, ci = 0, ks = 0; t0 < n_ang; t0 += ANGC, ++ci, ks = ks == 2 ? 0 : ks + 1) {
    const int nt = min(ANGC, n_ang - t0);
    const double2 rec2 = kmin_load(min(t0 + 2 * ANGC, n_ang - 1));
    const int ks1 = ks == 2 ? 0 : ks + 1, ks2 = ks1 == 2 ? 0 : ks1 + 1;
    if (t0 + ANGC < n_ang) dma(t0 + ANGC, ks1, (ci & 1) ? 0 : BUFB);
    chunk_taps(t0, nt, ks);
    if (t0 + ANGC < n_ang) {
      if (t0 + 2 * ANGC < n_ang) kmin_store(ks2, rec2, (ci & 1) ? BUFB : 0);
      __syncthreads();  // next chunk's DMA landed (fence), this chunk's taps done, slot ks2 visible
    }
  }
  // per lane block: k_back_mirror's epilogue (the real A^T s of both pixels, the fused H epilogue
  // and the block's 20 dot partials through the same reduction), one lane block at a time
  constexpr int NT = MH * NQ, NS = RsShape<NT>::NS;
  __shared__ double lds[kBkWaves * NS];
  __shared__ double tot[NS];
  const int P = gridDim.x * gridDim.y;
  const int b = blockIdx.y * gridDim.x + blockIdx.x;
#pragma unroll
  for (int l = 0; l < LB; ++l) {
    if (A.wexp != 0) {
#pragma unroll
      for (int u = 0; u < VB; ++u) {
        acc1[l][u] = ldexpf(acc1[l][u], A.wexp);
        acc2[l][u] = ldexpf(acc2[l][u], A.wexp);
      }
    }
    T r1[MH], r2[MH];
#pragma unroll
    for (int h = 0; h < MH; ++h) {
      r1[h] = acc1[l][h] + acc2[l][MH + h];
      r2[h] = acc2[l][h] + acc1[l][MH + h];
    }
    double pq[MH][NQ];
#pragma unroll
    for (int u = 0; u < MH; ++u)
#pragma unroll
      for (int q = 0; q < NQ; ++q) pq[u][q] = 0.0;
    const int z = (int)blockIdx.z * LB + l, rc = z / MS, mq = z % MS;
    const int v0 = rc * VBR + mq * MH, nv = min(MH, A.V - v0);
    if (inb) back_epilogue<T, MH, MODE, NQ, VBR>(A, i, j, rc, v0, nv, r1, pq, mq * MH);
    if (inb2) back_epilogue<T, MH, MODE, NQ, VBR, true>(A, i2, j, rc, v0, nv, r2, pq, mq * MH);
    double flat[NT];
#pragma unroll
    for (int u = 0; u < MH; ++u)
#pragma unroll
      for (int q = 0; q < NQ; ++q) flat[u * NQ + q] = pq[u][q];
    block_reduce_flat<NT, kBkWaves>(flat, lds, tot);
    const int t = threadIdx.x;
    if (t < NT && t / NQ < nv) A.part[((size_t)v0 * NQ + t) * P + b] = tot[t];
  }
}

// ===========================================================================
// Elementwise kernels, node-parallel: a block covers a 32 (j) x 32/VB (i) tile
// of VB nodes; its 256 threads are VB (node, fastest) x 32 (j) x 8/VB (row phase)
// and each handles one (pixel, node) in each of 4 rows.  Interleaved sample
// stores are contiguous across lanes and a launch has VB x more waves than a
// pixel-per-thread mapping.  Sample outputs are written row-major AND transposed
// (through a 4 KB LDS tile; every transposed row run is 32 samples = one 128-B
// line for float), because the forward projector reads the transposed copy for
// case-A angles.  blockIdx.z = chunk.
// ===========================================================================
template <int VB>
struct EwMap {
  static constexpr int TI = kTile / VB;  // tile rows
  static constexpr int RPI = 8 / VB;     // rows per iteration
  int u, jj, isub;
  __device__ EwMap() : u(threadIdx.x % VB), jj((threadIdx.x / VB) % kTile), isub(threadIdx.x / (kTile * VB)) {}
};

template <typename T, int VB>
struct TileT {
  T t[EwMap<VB>::TI][kTile + 1][VB];
};

// outT (interleaved, chunk base applied by caller): outT[j][i][u] = tile[i - i0][j - j0][u]
template <typename T, int VB>
__device__ __forceinline__ void tile_store_T(TileT<T, VB>& tl, T* __restrict__ outT, int N, int i0, int j0) {
  constexpr int TI = EwMap<VB>::TI;
  __syncthreads();
  const int u = threadIdx.x % VB, r = (threadIdx.x / VB) % TI, c0 = threadIdx.x / (VB * TI);
  for (int c = c0; c < kTile; c += kBlock / (VB * TI)) {
    const int jj = j0 + c, ii = i0 + r;
    if (jj < N && ii < N) outT[((size_t)jj * N + ii) * VB + u] = tl.t[r][c][u];
  }
}

// CG start from the previous x-update's diagnostics (batch flag ADMM_BATCH_KEEP_X: x_ext's
// local rows were last written by admm_node_update).  The previous DIAG left
// ats = A^T (A xs - b) for this very xs = (T) x, so A^T A xs = ats + A^T b needs no
// projection.  One kernel replaces gather + BACK_INIT + transpose:
//   c = sum_j q_ij (z_ij - y_ij,i)                         (k_gather's sum, same order)
//   r = A^T b + rho c + mu K^T (d - e) - (ats + A^T b + rho D xs + mu K^T K xs),  p = r
// (BACK_INIT's epilogue with its projected A^T A xs replaced; xs and its four neighbours
// are (T) x read straight from x), p also written transposed.  One thread per pixel, all
// VB nodes of the chunk; a block is kTile x kCgRows pixels (the CG update's grid).
template <typename T, int VB>
__global__ __launch_bounds__(kBlock) void k_start_reuse(
    const T* __restrict__ ats, const double* __restrict__ x, EdgeIn E, const double* __restrict__ q,
    const int* __restrict__ inc_off, const int* __restrict__ inc_edge, const int* __restrict__ inc_qslot,
    const int* __restrict__ inc_sign, const double* __restrict__ atb, double* __restrict__ cvec,
    const double* __restrict__ dsum, const double* __restrict__ dvar, const double* __restrict__ evar,
    double* __restrict__ r, T* __restrict__ p, T* __restrict__ pT, double rho, double mu, int N, int V) {
  constexpr int ROWS = kBlock / kTile;
  __shared__ T tl[ROWS][kTile + 1][VB];
  const int chunk = blockIdx.z, v0 = chunk * VB, nv = min(VB, V - v0);
  const int npix = N * N;
  const size_t sbase = (size_t)chunk * npix * VB;
  const int jj = threadIdx.x % kTile, ii = threadIdx.x / kTile;
  const int i0 = blockIdx.y * ROWS, j0 = blockIdx.x * kTile;
  const int i = i0 + ii, j = j0 + jj;
  if (i < N && j < N) {
    const int pix = i * N + j;
    T av[VB], outv[VB];
    gload<T, VB>(ats + sbase + (size_t)pix * VB, av);
#pragma unroll
    for (int u = 0; u < VB; ++u) {
      outv[u] = T(0);
      if (u < nv) {
        const int v = v0 + u;
        const size_t vo = (size_t)v * npix;
        const double* xv = x + vo;
        double cc = 0.0;
        for (int qq = inc_off[v]; qq < inc_off[v + 1]; ++qq) {
          const double vij = edge_v(E, inc_edge[qq], inc_sign[qq], npix, pix);
          cc += q[(size_t)inc_qslot[qq] * npix + pix] * vij;
        }
        cvec[vo + pix] = cc;
        // K^T K xs at (i, j) from (T) x, in BACK_INIT's order
        const double pcd = (double)(T)xv[pix];
        double ktk = 0.0;
        if (i >= 1) ktk += pcd - (double)(T)xv[pix - N];
        if (i <= N - 2) ktk -= (double)(T)xv[pix + N] - pcd;
        if (j >= 1) ktk += pcd - (double)(T)xv[pix - 1];
        if (j <= N - 2) ktk -= (double)(T)xv[pix + 1] - pcd;
        const double ab = atb[vo + pix];
        const double h = ((double)av[u] + ab) + rho * dsum[vo + pix] * pcd + mu * ktk;
        const double rr = ab + rho * cc + mu * kt_w_at(dvar + 2 * vo, evar + 2 * vo, N, i, j) - h;
        r[vo + pix] = rr;
        outv[u] = (T)rr;
      }
      tl[ii][jj][u] = outv[u];
    }
    gstore<T, VB>(p + sbase + (size_t)pix * VB, outv);
  }
  __syncthreads();
  // transposed copy: pT[j][i][u], runs of ROWS x VB samples per column
  const int u = threadIdx.x % VB, rr_ = (threadIdx.x / VB) % ROWS, c0 = threadIdx.x / (VB * ROWS);
  for (int c = c0; c < kTile; c += kBlock / (VB * ROWS)) {
    const int jc = j0 + c, ic = i0 + rr_;
    if (jc < N && ic < N) pT[sbase + ((size_t)jc * N + ic) * VB + u] = tl[rr_][c][u];
  }
}

// gather (prologue of the x-update, block_6_admm_loop_ver2.py:85-95,137-140):
//   c_v = sum_{e in inc(v)} q_e (z_e - sign * y_e);  xs = (T) x, xsT = xs^T
template <typename T, int VB>
__global__ __launch_bounds__(kBlock) void k_gather(const double* __restrict__ x, EdgeIn E,
                                                   const double* __restrict__ q,
                                                   const int* __restrict__ inc_off, const int* __restrict__ inc_edge,
                                                   const int* __restrict__ inc_qslot,
                                                   const int* __restrict__ inc_sign, double* __restrict__ c,
                                                   T* __restrict__ xs, T* __restrict__ xsT, int N, int V) {
  __shared__ TileT<T, VB> tl;
  const EwMap<VB> mp;
  const int chunk = blockIdx.z, v = chunk * VB + mp.u;
  const bool live = v < V;
  const int npix = N * N;
  const size_t sbase = (size_t)chunk * npix * VB;
  const int i0 = blockIdx.y * EwMap<VB>::TI, j0 = blockIdx.x * kTile;
  const int e0 = live ? inc_off[v] : 0, e1 = live ? inc_off[v + 1] : 0;
  for (int r = mp.isub; r < EwMap<VB>::TI; r += EwMap<VB>::RPI) {
    const int i = i0 + r, j = j0 + mp.jj;
    if (i < N && j < N) {
      const int pix = i * N + j;
      T sv = T(0);
      if (live) {
        double acc = 0.0;
        for (int qq = e0; qq < e1; ++qq) {
          const double vij = edge_v(E, inc_edge[qq], inc_sign[qq], npix, pix);
          acc += q[(size_t)inc_qslot[qq] * npix + pix] * vij;
        }
        c[(size_t)v * npix + pix] = acc;
        sv = (T)x[(size_t)v * npix + pix];
      }
      xs[sbase + (size_t)pix * VB + mp.u] = sv;
      tl.t[r][mp.jj][mp.u] = sv;
    }
  }
  tile_store_T<T, VB>(tl, xsT + sbase, N, i0, j0);
}

template <typename T, int VB>
__global__ __launch_bounds__(kBlock) void k_transpose(const T* __restrict__ in, T* __restrict__ outT, int N) {
  __shared__ TileT<T, VB> tl;
  const EwMap<VB> mp;
  const size_t sbase = (size_t)blockIdx.z * N * N * VB;
  const int i0 = blockIdx.y * EwMap<VB>::TI, j0 = blockIdx.x * kTile;
  for (int r = mp.isub; r < EwMap<VB>::TI; r += EwMap<VB>::RPI) {
    const int i = i0 + r, j = j0 + mp.jj;
    if (i < N && j < N) tl.t[r][mp.jj][mp.u] = in[sbase + ((size_t)i * N + j) * VB + mp.u];
  }
  tile_store_T<T, VB>(tl, outT + sbase, N, i0, j0);
}

// CG step from the five reductions of the preceding BACK_H launch (oracle/node_solver.py):
//   alpha = r.p / p.Hp (exact line search),  rr' = rr - 2 alpha rHp + alpha^2 HpHp,  beta = rr'/rr
//   x += alpha p;  r -= alpha Hp;  p = r + beta p  (p also written transposed)
// One thread per pixel, all VB nodes of the chunk: the interleaved p / Hp samples are
// one 32-B vector per lane and every node's float64 x / r is read in 32-pixel (256-B)
// runs (a node-per-lane mapping splits those into 64-B pieces across 8 arrays 2 MB apart).
constexpr int kCgRows = kBlock / kTile;  // 8 rows x 32 columns per block

// The CG x steps of a split-Bregman round are applied by the TV update that ends the round
// (k_tv_update FUSE): all K of them from a ring of the round's directions when K <=
// kMaxCgRing, else only the round's last one.
// WRITE_P = false: the last CG step of a split-Bregman round -- the TV update (or the next
// x-update's start) overwrites p and its transposed copy, so only x and r are written
// WRITE_X = false (direction ring): x is left alone -- the TV update applies the round's
// x += alpha_k p_k, k = 0..K-1, in the same order (so bitwise the same x) from the p ring;
// p_{k+1} then goes to its own slot pout (p_k stays readable for that).
template <typename T, int VB, bool WRITE_P = true, bool WRITE_X = true>
__global__ __launch_bounds__(kBlock) void k_cg_update(double* __restrict__ x, double* __restrict__ r,
                                                      const T* p, T* __restrict__ pT,
                                                      const T* __restrict__ Hp, const double* __restrict__ redH,
                                                      int N, int V, T* pout) {
  __shared__ T tl[kCgRows][kTile + 1][VB];
  __shared__ double ab_s[VB][2];
  const int chunk = blockIdx.z, v0 = chunk * VB;
  const int npix = N * N;
  const size_t sbase = (size_t)chunk * npix * VB;
  if ((int)threadIdx.x < VB) {
    const int v = v0 + threadIdx.x;
    double alpha = 0.0, beta = 0.0;
    if (v < V) {
      const double* S = redH + 5 * v;
      const double pHp = S[0], rHp = S[1], HH = S[2], rr = S[3], rp = S[4];
      alpha = (pHp != 0.0) ? rp / pHp : 0.0;
      double rrn = rr - 2.0 * alpha * rHp + alpha * alpha * HH;
      rrn = fmax(rrn, 0.0);
      beta = (rr != 0.0) ? rrn / rr : 0.0;
    }
    ab_s[threadIdx.x][0] = alpha;
    ab_s[threadIdx.x][1] = beta;
  }
  __syncthreads();
  const int jj = threadIdx.x % kTile, ii = threadIdx.x / kTile;
  const int i0 = blockIdx.y * kCgRows, j0 = blockIdx.x * kTile;
  const int i = i0 + ii, j = j0 + jj;
  if (i < N && j < N) {
    const int pix = i * N + j;
    T pv[VB], hv[VB], np[VB];
    gload<T, VB>(p + sbase + (size_t)pix * VB, pv);
    gload<T, VB>(Hp + sbase + (size_t)pix * VB, hv);
#pragma unroll
    for (int u = 0; u < VB; ++u) {
      np[u] = T(0);
      if (v0 + u < V) {
        const size_t o = (size_t)(v0 + u) * npix + pix;
        const double alpha = ab_s[u][0], beta = ab_s[u][1];
        const double pd = (double)pv[u];
        if constexpr (WRITE_X) x[o] = fma(alpha, pd, x[o]);  // (explicit fma: k_tv_update<FUSE> repeats it bitwise)
        const double rn = fma(-alpha, (double)hv[u], r[o]);
        r[o] = rn;
        np[u] = (T)(rn + beta * pd);
      }
      if constexpr (WRITE_P) tl[ii][jj][u] = np[u];
    }
    if constexpr (WRITE_P) gstore<T, VB>(pout + sbase + (size_t)pix * VB, np);
  }
  if constexpr (!WRITE_P) return;
  __syncthreads();
  // transposed copy: pT[j][i][u], runs of kCgRows x VB samples per column
  const int u = threadIdx.x % VB, rr_ = (threadIdx.x / VB) % kCgRows, c0 = threadIdx.x / (VB * kCgRows);
  for (int c = c0; c < kTile; c += kBlock / (VB * kCgRows)) {
    const int jc = j0 + c, ic = i0 + rr_;
    if (jc < N && ic < N) pT[sbase + ((size_t)jc * N + ic) * VB + u] = tl[rr_][c][u];
  }
}

// split-Bregman (d, e) update after a CG solve:
//   u = Kx + e, d' = shrink(u, lam/mu), e' = u - d'
// and, unless LAST, the residual shift r += mu K^T((d'-e') - (d-e)) and the CG
// restart p = r.  With LAST the sample copy xs = (T) x (+ transpose) is produced for
// the diagnostics epilogue instead.  d/e are ping-ponged (din -> dout) because the
// stencil reads neighbours' old values.
__device__ __forceinline__ void shrink2(double ux, double uy, double tau, int kind, double& dx, double& dy) {
  if (kind == 0) {
    const double s = sqrt(ux * ux + uy * uy);
    const double f = (s > tau) ? (s - tau) / s : 0.0;
    dx = f * ux;
    dy = f * uy;
  } else {
    dx = copysign(fmax(fabs(ux) - tau, 0.0), ux);
    dy = copysign(fmax(fabs(uy) - tau, 0.0), uy);
  }
}

// XCD-aware tile order (performance only): workgroups are dealt round-robin over the 8 XCDs,
// so consecutive ids land on different L2s.  Remap so that the ids sharing an XCD (orig % 8)
// get one contiguous run of tiles; a stencil's halo rows/columns are then fetched by the
// same L2.  Bijective for any nwg (guide: cdna_hip_programming.md, XCD swizzle).
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

// FUSE: the round's CG x steps are folded in (all K of them, the CG updates leaving x alone
// and keeping each direction p_k in a ring slot; K > kMaxCgRing: only the last one).
// x after those steps is formed once per pixel of the stencil region, from the old x and
// p_k with the same fmas in the same order, written once to xout (x ping-pongs: neighbour
// blocks still read the old x), and r gets the last step's update and the TV shift in one
// pass; the CG restart p = r goes to a slot no one reads here.  Bitwise the same iteration
// as the separate kernels (scripts/check_bitwise.py).
// The CG directions whose x steps the fused TV update applies (FUSE): p[k] with alpha_k
// from the reduction redH + k * 5V, k = 0 .. K-1 (K = 1: only the round's last step).
constexpr int kMaxCgRing = 8;
#ifndef ADMM_TV_ALIGN
#define ADMM_TV_ALIGN 1
#endif
template <typename T>
struct PRing {
  const T* p[kMaxCgRing];
  int K;
};
// UIN / UOUT: between the rounds of one x-update the split-Bregman state
// is kept as u = Kx + e_old alone (2 doubles per pixel instead of d and e, 4): the next
// round recomputes d = shrink(u) and e = u - d -- exactly the values the round that wrote
// u computed, so the iteration is bitwise the same -- and the traffic of a middle round
// drops by 4 of its ~34 bytes per node-pixel read+written.  UIN: din holds u (ein unused);
// UOUT: dout receives u (eout unused).  The x-update's first round reads d, e and its last
// writes them, so the state between x-updates (and every other kernel) is unchanged.
// Tile of the TV update: kTvTile columns x kTile / VB rows of VB nodes, kTvThreads threads
// (ADMM_TV_TW = 64: twice the columns per halo column pair, 512 threads -- fewer partial-line
// requests per pixel for the same rows; 32: the elementwise kernels' tile, 256 threads)
#ifndef ADMM_TV_TW
#define ADMM_TV_TW 64
#endif
constexpr int kTvTile = ADMM_TV_TW;
constexpr int kTvThreads = kTvTile == 64 ? 512 : 256;
static_assert(kTvTile == 32 || kTvTile == 64, "TV tile width 32 or 64");
template <int VB>
struct TvMap {
  static constexpr int TI = kTile / VB;                       // tile rows
  static constexpr int RPI = kTvThreads / (kTvTile * VB);     // rows per iteration
  int u, jj, isub;
  __device__ TvMap() : u(threadIdx.x % VB), jj((threadIdx.x / VB) % kTvTile), isub(threadIdx.x / (kTvTile * VB)) {}
};
template <typename T, int VB>
struct TvTile {
  T t[TvMap<VB>::TI][kTvTile + 1][VB];
};
// outT[j][i][u] = tile[i - i0][j - j0][u] (as tile_store_T, for the TV tile)
template <typename T, int VB>
__device__ __forceinline__ void tv_tile_store_T(TvTile<T, VB>& tl, T* __restrict__ outT, int N, int i0, int j0) {
  constexpr int TI = TvMap<VB>::TI;
  __syncthreads();
  const int u = threadIdx.x % VB, r = (threadIdx.x / VB) % TI, c0 = threadIdx.x / (VB * TI);
  for (int c = c0; c < kTvTile; c += kTvThreads / (VB * TI)) {
    const int jj = j0 + c, ii = i0 + r;
    if (jj < N && ii < N) outT[((size_t)jj * N + ii) * VB + u] = tl.t[r][c][u];
  }
}
template <typename T, int VB, bool LAST, bool FUSE = false, bool UIN = false, bool UOUT = false>
__global__ __launch_bounds__(kTvThreads) void k_tv_update(const double* __restrict__ x, const double* __restrict__ din,
                                                      const double* __restrict__ ein, double* __restrict__ dout,
                                                      double* __restrict__ eout, double* __restrict__ r,
                                                      T* __restrict__ p, T* __restrict__ pT, double tau,
                                                      double mu, int kind, int N, int V, double* __restrict__ xout,
                                                      PRing<T> pr, const T* __restrict__ Hp,
                                                      const double* __restrict__ redH) {
  static_assert(!(LAST && UOUT), "the last round writes d and e");
  __shared__ TvTile<T, VB> tl;
  const TvMap<VB> mp;
  const int chunk = blockIdx.z, v = chunk * VB + mp.u;
  const bool live = v < V;
  const int npix = N * N;
  const size_t sbase = (size_t)chunk * npix * VB;
  const int wg = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gridDim.y);
  const int i0 = (wg / gridDim.x) * TvMap<VB>::TI, j0 = (wg % gridDim.x) * kTvTile;
  // FUSE: x after the round's CG steps over the block's stencil region (rows i0-1 .. i0+TI,
  // columns j0-1 .. j0+kTvTile), formed once per pixel into LDS from the old x and the p ring
  // (32-B vector loads of each p), x = fma(alpha_k, p_k, x) for k = 0 .. K-1 as the CG
  // updates did it; the stencil then reads LDS only
  constexpr int PR = TvMap<VB>::TI + 2, PC = kTvTile + 2;
  __shared__ double al_s[FUSE ? kMaxCgRing : 1][VB];
  __shared__ double x_s[FUSE ? VB : 1][FUSE ? PR : 1][FUSE ? PC + 1 : 1];
  if constexpr (FUSE) {
    if ((int)threadIdx.x < VB * pr.K) {  // alpha_k per node (as k_cg_update)
      const int k = threadIdx.x / VB, u = threadIdx.x % VB, vv = chunk * VB + u;
      double alpha = 0.0;
      if (vv < V) {
        const double* S = redH + (size_t)k * 5 * V + 5 * vv;
        alpha = (S[0] != 0.0) ? S[4] / S[0] : 0.0;
      }
      al_s[k][u] = alpha;
    }
    __syncthreads();
    for (int q = threadIdx.x; q < PR * PC; q += kTvThreads) {
#if ADMM_TV_ALIGN
      // the tile's kTvTile columns first (rows of 256-B-aligned float64 runs per node), the two
      // halo columns after them: no lane group straddles a cache line
      int rr, cc;
      if (q < PR * kTvTile) {
        rr = q / kTvTile;
        cc = 1 + q % kTvTile;
      } else {
        const int h = q - PR * kTvTile;
        rr = h >> 1;
        cc = (h & 1) ? PC - 1 : 0;
      }
#else
      const int rr = q / PC, cc = q % PC;
#endif
      const int i = i0 - 1 + rr, j = j0 - 1 + cc;
      if (i < 0 || j < 0 || i >= N || j >= N) continue;
      const int o = i * N + j;
      double xn[VB];
#pragma unroll
      for (int u = 0; u < VB; ++u) {
        const int vq = chunk * VB + u;
        xn[u] = vq < V ? x[(size_t)vq * npix + o] : 0.0;
      }
      // direction k + 1 is loaded before step k's fmas (one load in flight; two: 60.4 us)
      T pa[VB], pb[VB];
      gload<T, VB>(pr.p[0] + sbase + (size_t)o * VB, pa);
      for (int k = 0; k < pr.K; ++k) {
        if (k + 1 < pr.K) gload<T, VB>(pr.p[k + 1] + sbase + (size_t)o * VB, pb);
#pragma unroll
        for (int u = 0; u < VB; ++u) xn[u] = fma(al_s[k][u], (double)pa[u], xn[u]);
#pragma unroll
        for (int u = 0; u < VB; ++u) pa[u] = pb[u];
      }
#pragma unroll
      for (int u = 0; u < VB; ++u) x_s[u][rr][cc] = xn[u];
    }
    __syncthreads();
  }
  // x of node u of the chunk at (i, j) after the round's CG steps
  auto xat = [&](int u, const double* xq, int i, int j) -> double {
    if constexpr (FUSE) return x_s[u][i - i0 + 1][j - j0 + 1];
    return xq[i * N + j];
  };
  auto gradx = [&](int u, const double* xq, int i, int j, double& gx, double& gy) {
    const double c = xat(u, xq, i, j);
    gx = (i < N - 1) ? xat(u, xq, i + 1, j) - c : 0.0;
    gy = (j < N - 1) ? xat(u, xq, i, j + 1) - c : 0.0;
  };
  const size_t vo = (size_t)(live ? v : 0) * npix;
  const double* xv = x + vo;
  const double* ev = ein + 2 * vo;
  if constexpr (!LAST) {
    // Phase 1: shrink once per point of the tile plus one halo row (i0-1) and column (j0-1),
    // keeping q = (d' - e') - (d - e) per component in LDS; tile points also store d', e'.
    // Phase 2: K^T q at each tile pixel from LDS (the same four terms, in the same order,
    // that the neighbour re-evaluation used), then r += mu K^T q, p = r.
    constexpr int TI = TvMap<VB>::TI, HC = kTvTile + 1, HR = TI + 1;
    // column-fastest: a wave reads runs of 33 consecutive pixels of one node
    __shared__ double qx_s[HR][VB][HC], qy_s[HR][VB][HC];
    for (int q = threadIdx.x; q < HR * HC * VB; q += kTvThreads) {
#if ADMM_TV_ALIGN
      // (as above: the kTvTile tile columns of every (row, node) first, the halo column after)
      int cc, u, rr;
      if (q < HR * VB * kTvTile) {
        cc = 1 + q % kTvTile;
        const int rest = q / kTvTile;
        u = rest % VB;
        rr = rest / VB;
      } else {
        const int h = q - HR * VB * kTvTile;
        cc = 0;
        u = h % VB;
        rr = h / VB;
      }
#else
      const int cc = q % HC, rest = q / HC;
      const int u = rest % VB, rr = rest / VB;  // halo-shifted (row 0 = i0-1, col 0 = j0-1)
#endif
      const int i = i0 + rr - 1, j = j0 + cc - 1;
      const int vq = chunk * VB + u;
      if (vq >= V || i < 0 || j < 0 || i >= N || j >= N) continue;
      const size_t vqo = (size_t)vq * npix;
      const double* xq = x + vqo;
      const int o = i * N + j;
      double d0, d1, e0, e1;  // this round's input d and e at (i, j)
      if constexpr (UIN) {
        const double u0 = din[2 * vqo + o], u1 = din[2 * vqo + npix + o];
        shrink2(u0, u1, tau, kind, d0, d1);
        e0 = u0 - d0;
        e1 = u1 - d1;
      } else {
        d0 = din[2 * vqo + o];
        d1 = din[2 * vqo + npix + o];
        e0 = ein[2 * vqo + o];
        e1 = ein[2 * vqo + npix + o];
      }
      double gx, gy, ndx, ndy;
      gradx(u, xq, i, j, gx, gy);
      const double ux = gx + e0, uy = gy + e1;
      shrink2(ux, uy, tau, kind, ndx, ndy);
      const double nex = ux - ndx, ney = uy - ndy;
      qx_s[rr][u][cc] = (ndx - nex) - (d0 - e0);
      qy_s[rr][u][cc] = (ndy - ney) - (d1 - e1);
      if (rr >= 1 && cc >= 1) {
        if constexpr (UOUT) {
          dout[2 * vqo + o] = ux;
          dout[2 * vqo + npix + o] = uy;
        } else {
          dout[2 * vqo + o] = ndx;
          dout[2 * vqo + npix + o] = ndy;
          eout[2 * vqo + o] = nex;
          eout[2 * vqo + npix + o] = ney;
        }
      }
    }
    __syncthreads();
    for (int rw = mp.isub; rw < TI; rw += TvMap<VB>::RPI) {
      const int i = i0 + rw, j = j0 + mp.jj;
      if (i >= N || j >= N) continue;
      const int o = i * N + j;
      T sv = T(0);
      if (live) {
        double kt = 0.0;
        if (i <= N - 2) kt -= qx_s[rw + 1][mp.u][mp.jj + 1];
        if (j <= N - 2) kt -= qy_s[rw + 1][mp.u][mp.jj + 1];
        if (i >= 1) kt += qx_s[rw][mp.u][mp.jj + 1];
        if (j >= 1) kt += qy_s[rw + 1][mp.u][mp.jj];
        double rv = r[vo + o];
        if constexpr (FUSE) {
          rv = fma(-al_s[pr.K - 1][mp.u], (double)Hp[sbase + (size_t)o * VB + mp.u], rv);
          xout[vo + o] = xat(mp.u, xv, i, j);
        }
        const double rn = fma(mu, kt, rv);
        r[vo + o] = rn;
        sv = (T)rn;
      }
      p[sbase + (size_t)o * VB + mp.u] = sv;
      tl.t[rw][mp.jj][mp.u] = sv;
    }
    tv_tile_store_T<T, VB>(tl, pT + sbase, N, i0, j0);
    return;
  }
  for (int rw = mp.isub; rw < TvMap<VB>::TI; rw += TvMap<VB>::RPI) {
    const int i = i0 + rw, j = j0 + mp.jj;
    if (i >= N || j >= N) continue;
    const int o = i * N + j;
    T sv = T(0);
    if (live) {
      double gx, gy, ux, uy, ndx, ndy, e0, e1;
      if constexpr (UIN) {
        const double u0 = din[2 * vo + o], u1 = din[2 * vo + npix + o];
        double d0, d1;
        shrink2(u0, u1, tau, kind, d0, d1);
        e0 = u0 - d0;
        e1 = u1 - d1;
      } else {
        e0 = ev[o];
        e1 = ev[npix + o];
      }
      gradx(mp.u, xv, i, j, gx, gy);
      ux = gx + e0;
      uy = gy + e1;
      shrink2(ux, uy, tau, kind, ndx, ndy);
      const double nex = ux - ndx, ney = uy - ndy;
      dout[2 * vo + o] = ndx;
      dout[2 * vo + npix + o] = ndy;
      eout[2 * vo + o] = nex;
      eout[2 * vo + npix + o] = ney;
      // (LAST only: the other rounds returned above) the diagnostics' sample copy of x
      const double xn = xat(mp.u, xv, i, j);
      if constexpr (FUSE) xout[vo + o] = xn;
      sv = (T)xn;
    }
    p[sbase + (size_t)o * VB + mp.u] = sv;
    tl.t[rw][mp.jj][mp.u] = sv;
  }
  tv_tile_store_T<T, VB>(tl, pT + sbase, N, i0, j0);
}

// node-major float64 [V][L] -> interleaved samples [C][L][VB] of type T  (grid.y = chunk)
template <typename T, int VB>
__global__ void k_pack_d(const double* __restrict__ in, T* __restrict__ out, int L, int V) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  const int chunk = blockIdx.y, v0 = chunk * VB;
  if (q >= L) return;
  T s[VB];
#pragma unroll
  for (int u = 0; u < VB; ++u) s[u] = (v0 + u < V) ? (T)in[(size_t)(v0 + u) * L + q] : T(0);
  gstore<T, VB>(out + ((size_t)chunk * L + q) * VB, s);
}

// node-major [V][L] samples -> interleaved [C][L][VB]  (grid.y = chunk)
template <typename T, int VB>
__global__ void k_pack(const T* __restrict__ in, T* __restrict__ out, int L, int V) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  const int chunk = blockIdx.y, v0 = chunk * VB;
  if (q >= L) return;
  T s[VB];
#pragma unroll
  for (int u = 0; u < VB; ++u) s[u] = (v0 + u < V) ? in[(size_t)(v0 + u) * L + q] : T(0);
  gstore<T, VB>(out + ((size_t)chunk * L + q) * VB, s);
}

// interleaved [C][L][VB] samples -> node-major [V][L]  (grid.y = chunk)
template <typename T, int VB>
__global__ void k_unpack(const T* __restrict__ in, T* __restrict__ out, int L, int V) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  const int chunk = blockIdx.y, v0 = chunk * VB;
  if (q >= L) return;
  T s[VB];
  gload<T, VB>(in + ((size_t)chunk * L + q) * VB, s);
#pragma unroll
  for (int u = 0; u < VB; ++u)
    if (v0 + u < V) out[(size_t)(v0 + u) * L + q] = s[u];
}

// ===========================================================================
// Consensus / dual / residual kernel, one edge per blockIdx.y
// (block_6_admm_loop_ver2.py:210-253):
//   a_a = x_a + y, a_b = x_b - y, z' = (a_a + a_b)/2, y' = y + x_a - z'
//   partials of |x_a - z'|^2, |x_b - z'|^2, |z' - z|^2
// ===========================================================================
// WEIGHTED: a_a = x_a + y, a_b = x_b + y_b, z' = (W_a a_a + W_b a_b)/(W_a + W_b),
//           y' = y + x_a - z', y_b' = y_b + x_b - z'   (_ver2:221-222 commented form, PDF eq.(2))
template <bool WEIGHTED>
__global__ __launch_bounds__(kBlock) void k_consensus(const double* __restrict__ xext, double* __restrict__ y,
                                                      double* __restrict__ yb, double* __restrict__ z,
                                                      const double* __restrict__ w,
                                                      const int* __restrict__ ea, const int* __restrict__ eb,
                                                      double* __restrict__ part, int npix, int e0 = 0) {
  __shared__ double lds[12];
  const int e = e0 + blockIdx.y;  // (e0: admm_consensus_range's first slot)
  const size_t eo = (size_t)e * npix;
  const size_t ra_off = (size_t)ea[e] * npix, rb_off = (size_t)eb[e] * npix;
  const double* xa = xext + ra_off;
  const double* xb = xext + rb_off;
  double acc[3] = {0.0, 0.0, 0.0};
  const int base = blockIdx.x * (kBlock * 4);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int pix = base + u * kBlock + threadIdx.x;
    if (pix < npix) {
      const double xav = xa[pix], xbv = xb[pix], yv = y[eo + pix], zo = z[eo + pix];
      double zn;
      if constexpr (WEIGHTED) {
        const double ybv = yb[eo + pix];
        const double wa = w[ra_off + pix], wb = w[rb_off + pix];
        const double aa = xav + yv, ab = xbv + ybv;
        zn = (wa * aa + wb * ab) / (wa + wb);
        yb[eo + pix] = ybv + xbv - zn;
      } else {
        const double aa = xav + yv, ab = xbv - yv;
        zn = (aa + ab) * 0.5;
      }
      y[eo + pix] = yv + xav - zn;
      z[eo + pix] = zn;
      const double ra = xav - zn, rb = xbv - zn, dz = zn - zo;
      acc[0] += ra * ra;
      acc[1] += rb * rb;
      acc[2] += dz * dz;
    }
  }
  block_reduce<3>(acc, lds);
  if (threadIdx.x == 0) {
    const int P = gridDim.x;
#pragma unroll
    for (int q = 0; q < 3; ++q) part[((size_t)e * 3 + q) * P + blockIdx.x] = acc[q];
  }
}

// Derived consensus (midpoint fusion, z never stored; admm_batch.x_prev, ABI 7):
//   z' = (x_a + x_b) * 0.5,  z = (xp_a + xp_b) * 0.5  (the previous consensus' z, bit for bit),
//   y' = y + x_a - z',  partials |x_a - z'|^2, |x_b - z'|^2, |z' - z|^2;  then x_prev = x_ext.
// Pixel-major: a block owns 64 pixels (one per lane) and stages every x_ext and x_prev row of
// them in LDS once; its 4 waves then take every 4th stored edge, so per edge only the dual y
// streams through HBM (16 B per pixel, against 48 B for the stored-z kernel's x_a, x_b, y, z
// reads and y, z writes), and the endpoint rows come from LDS however many edges share them
// (a dense graph's 476 edges per rank touch 64 rows).  Loads of KU edges' y are issued before
// their arithmetic.  Partials per (edge, 64-pixel block), wave-reduced in a fixed order.
// RMAX: LDS rows (x_ext rows <= RMAX); more rows take k_consensus_derived_direct.
constexpr int kConsPix = 64;
// (LDS: 2 x RMAX x 64 doubles = 128 KiB at RMAX = 128: gfx950's 160 KiB per workgroup; the
// build targets gfx950 only, admm_hip/build.py)
template <int RMAX>
__global__ __launch_bounds__(kBlock) void k_consensus_derived(const double* __restrict__ xext,
                                                              double* __restrict__ xprev, double* __restrict__ y,
                                                              const int* __restrict__ ea, const int* __restrict__ eb,
                                                              double* __restrict__ part, int npix, int R, int E) {
  __shared__ double xn[RMAX][kConsPix], xo[RMAX][kConsPix];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int p0 = blockIdx.x * kConsPix;
  const int pix = p0 + lane;
  const bool in = pix < npix;
  for (int q = threadIdx.x; q < R * kConsPix; q += kBlock) {
    const int r = q / kConsPix, l = q % kConsPix;
    const int px = p0 + l;
    double a = 0.0, b = 0.0;
    if (px < npix) {
      a = xext[(size_t)r * npix + px];
      b = xprev[(size_t)r * npix + px];
    }
    xn[r][l] = a;
    xo[r][l] = b;
  }
  __syncthreads();
  // the old rows are in LDS: x_prev takes this iteration's images now
  for (int q = threadIdx.x; q < R * kConsPix; q += kBlock) {
    const int r = q / kConsPix, l = q % kConsPix;
    if (p0 + l < npix) xprev[(size_t)r * npix + p0 + l] = xn[r][l];
  }
  const int P = gridDim.x;
  constexpr int KU = 4;  // edges per wave whose y loads are in flight together
  for (int e0 = w; e0 < E; e0 += 4 * KU) {
    double yv[KU];
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      const int e = e0 + 4 * u;
      yv[u] = (in && e < E) ? y[(size_t)e * npix + pix] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      const int e = e0 + 4 * u;
      if (e >= E) break;  // wave-uniform
      const int a = ea[e], b = eb[e];
      double s[3] = {0.0, 0.0, 0.0};
      if (in) {
        const double xa = xn[a][lane], xb = xn[b][lane];
        const double zn = (xa + xb) * 0.5;
        const double zo = (xo[a][lane] + xo[b][lane]) * 0.5;
        y[(size_t)e * npix + pix] = yv[u] + xa - zn;
        const double ra = xa - zn, rb = xb - zn, dz = zn - zo;
        s[0] = ra * ra;
        s[1] = rb * rb;
        s[2] = dz * dz;
      }
#pragma unroll
      for (int q = 0; q < 3; ++q) s[q] = wave_sum_d(s[q]);
      if (lane == 0) {
#pragma unroll
        for (int q = 0; q < 3; ++q) part[((size_t)e * 3 + q) * P + blockIdx.x] = s[q];
      }
    }
  }
}

// The same for batches with more x_ext rows than the LDS tile holds: endpoint rows read from
// HBM / L2 per edge (same arithmetic, same partial layout, bitwise the same results); x_prev
// is copied by a separate pass after it (k_copy_rows) because other blocks still read it.
__global__ __launch_bounds__(kBlock) void k_consensus_derived_direct(const double* __restrict__ xext,
                                                                     const double* __restrict__ xprev,
                                                                     double* __restrict__ y, const int* __restrict__ ea,
                                                                     const int* __restrict__ eb,
                                                                     double* __restrict__ part, int npix, int E) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int pix = blockIdx.x * kConsPix + lane;
  const bool in = pix < npix;
  const int P = gridDim.x;
  for (int e = w; e < E; e += 4) {
    const int a = ea[e], b = eb[e];
    double s[3] = {0.0, 0.0, 0.0};
    if (in) {
      const double xa = xext[(size_t)a * npix + pix], xb = xext[(size_t)b * npix + pix];
      const double zn = (xa + xb) * 0.5;
      const double zo = (xprev[(size_t)a * npix + pix] + xprev[(size_t)b * npix + pix]) * 0.5;
      const size_t eo = (size_t)e * npix + pix;
      y[eo] = y[eo] + xa - zn;
      const double ra = xa - zn, rb = xb - zn, dz = zn - zo;
      s[0] = ra * ra;
      s[1] = rb * rb;
      s[2] = dz * dz;
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) s[q] = wave_sum_d(s[q]);
    if (lane == 0) {
#pragma unroll
      for (int q = 0; q < 3; ++q) part[((size_t)e * 3 + q) * P + blockIdx.x] = s[q];
    }
  }
}

__global__ void k_copy_rows(const double* __restrict__ src, double* __restrict__ dst, size_t count) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

// rows of P partials -> one value each, fixed order (deterministic).
// out[(r / G) * ostride + ooff + (r % G)] = sum_p part[r * P + p]
__global__ __launch_bounds__(kBlock) void k_reduce_rows(const double* __restrict__ part, int P, double* __restrict__ out,
                                                        int G, int ostride, int ooff) {
  __shared__ double lds[4];
  const int r = blockIdx.x;
  double s = 0.0;
  for (int p = threadIdx.x; p < P; p += kBlock) s += part[(size_t)r * P + p];
  double a[1] = {s};
  block_reduce<1>(a, lds);
  if (threadIdx.x == 0) out[(size_t)(r / G) * ostride + ooff + (r % G)] = a[0];
}


// K x and K^T p for the operator API (float64 node-major)
__global__ void k_tv_grad(const double* __restrict__ x, double* __restrict__ gx, double* __restrict__ gy, int N) {
  const int v = blockIdx.z;
  const size_t vo = (size_t)v * N * N;
  const int j = blockIdx.x * 64 + (threadIdx.x & 63), i = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (i >= N || j >= N) return;
  double a, b;
  grad_at(x + vo, N, i, j, a, b);
  gx[vo + i * N + j] = a;
  gy[vo + i * N + j] = b;
}
__global__ void k_tv_div(const double* __restrict__ px, const double* __restrict__ py, double* __restrict__ out,
                         int N) {
  const int v = blockIdx.z;
  const size_t vo = (size_t)v * N * N;
  const int j = blockIdx.x * 64 + (threadIdx.x & 63), i = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (i >= N || j >= N) return;
  const int o = i * N + j;
  double s = 0.0;
  if (i >= 1) s += px[vo + o - N];
  if (i <= N - 2) s -= px[vo + o];
  if (j >= 1) s += py[vo + o - 1];
  if (j <= N - 2) s -= py[vo + o];
  out[vo + o] = s;
}

}  // namespace admm
