// admm_tomo.hip -- C-ABI implementation (include/admm_tomo.h) for MI355X (gfx950).
//
// Host side of the hot path: geometry tables, scratch, and the x-update /
// consensus sequences.  A bound batch's sequences are recorded once as
// hipGraphs and replayed every ADMM iteration (launch-bound at small N
// otherwise: ~170 kernels per x-update).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "../../include/admm_tomo.h"
#include "kernels.hpp"

using namespace admm;

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(expr)                                                                          \
  do {                                                                                        \
    hipError_t _e = (expr);                                                                   \
    if (_e != hipSuccess)                                                                     \
      return fail(ADMM_E_HIP, std::string(#expr) + ": " + hipGetErrorString(_e) + " @" +     \
                                  std::to_string(__LINE__));                                  \
  } while (0)

#define CHECK_LAUNCH() HIPCHK(hipGetLastError())

size_t dsize(int dtype) { return dtype == ADMM_DTYPE_F64 ? 8 : 4; }

// Makes `device` current for the scope of an entry point and restores the caller's device
// on every return path (the operator API is called freely from Python: applying an
// operator that lives on another GPU must not change torch.cuda.current_device()).
struct DeviceGuard {
  int prev = -1;
  hipError_t err = hipSuccess;
  explicit DeviceGuard(int device) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != device) err = hipSetDevice(device);
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};

#define DEVICE_SCOPE(dev)                                                                     \
  DeviceGuard _dg(dev);                                                                       \
  if (_dg.err != hipSuccess)                                                                  \
  return fail(ADMM_E_HIP, std::string("hipSetDevice: ") + hipGetErrorString(_dg.err))

struct Buf {
  void* p = nullptr;
  size_t bytes = 0;
};

int ensure(Buf& b, size_t bytes) {
  if (b.bytes >= bytes && b.p) return ADMM_OK;
  if (b.p) HIPCHK(hipFree(b.p));
  b.p = nullptr;
  b.bytes = 0;
  if (bytes == 0) return ADMM_OK;
  HIPCHK(hipMalloc(&b.p, bytes));
  // hipMemset is enqueued on the null stream, which does not order against non-blocking
  // streams (the capture stream, a caller's torch stream): finish the zero-fill before any
  // kernel can write the buffer (measured: the bind-time D packing on the capture stream
  // was overwritten by its own buffer's zero-fill)
  HIPCHK(hipMemset(b.p, 0, bytes));
  HIPCHK(hipDeviceSynchronize());
  b.bytes = bytes;
  return ADMM_OK;
}
}  // namespace

// error channel shared with the other translation units (masks.hip)
namespace admm_internal {
int fail(int code, const std::string& msg) { return ::fail(code, msg); }
}  // namespace admm_internal

struct admm_ctx {
  admm_geom g{};
  int dtype = ADMM_DTYPE_F32;
  int device = 0;
  int max_images = 0;
  int npix = 0, mrays = 0;
  FwdAngle* fang = nullptr;
  BackAngle* bang = nullptr;
  BackAngleC* bangc = nullptr;
  double Kb = 0.0;  // angle-independent part of the back projector's k_f
  int kbias = 0;    // integer bias making every pixel's k_f positive (k_back)
  int wexp = 0;     // k_back float weights scaled by 2^-wexp (<= 1 for the fma clamp)
  FgGroup* groups = nullptr;  // angle groups of the grouped forward projector (active plan)
  FgRange* rng = nullptr;     // its per-block ray ranges
  int n_groups = 0;           // 0: geometry does not fit the grouped kernel -> k_fwd
  // the group plans, chosen at bind time: 0: 64-ray chunks, 1: chunks aligned per (row
  // segment, angle) at the detector centre, 2: chunks aligned per (row segment, chunk);
  // 3-5: the same with every block's rays clipped to those crossing its segment inside the
  // image (groups re-planned on the narrower windows)
  static constexpr int kPlans = 6;
  FgGroup* plan_groups[kPlans] = {};
  FgRange* plan_rng[kPlans] = {};
  int plan_n[kPlans] = {}, plan_blocks[kPlans] = {};
  double plan_staged[kPlans] = {};      // touched row pixels staged per node chunk (host model)
  std::vector<int4> plan_blk[kPlans];  // per block: {ray-range index, group, segment, G}
  std::vector<char> plan_caseA[kPlans];  // per group: its angles read the transposed image
  bool mirror_half = false;  // the half geometry of a mirror-mode context (XCD mapping below)
  Buf fg_order;                       // int4 block table of the grouped forward projector
  int fg_nblk = 0, fg_order_nch = 0;
  int fg_cpb = 1;  // (mirror half geometry) virtual chunks per forward block of the bound table
  hipStream_t cap = nullptr;  // private capture stream

  // explicit-matrix context (admm_ctx_create_matrix): A and A^T as device CSR, values in
  // the sample dtype; the projector launches dispatch to k_csr_fwd / k_back<..., CSR>
  bool csr = false;
  long long nnz = 0;
  Buf f_ptr, f_idx, f_val, t_ptr, t_idx, t_val;

  // operator-API scratch (admm_project_fwd runs the hot grouped kernel on up to 8 images
  // per launch: node-major images packed into the interleaved sample layout)
  Buf op_img, op_imgT, op_sino, op_fpart;
  Buf op_order[kPlans];  // block tables of the forward plans for one node chunk
  int op_nblk[kPlans] = {};
  int op_fpart_key = -1;  // (plan, VB) whose partial slots op_fpart holds (others are zero)

  // batch
  bool bound = false;
  admm_batch b{};
  int vb = 1;  // node interleave width of the sample buffers
  // mirror mode (kernels.hpp k_fwdg MIRROR): the bound batch projects virtual images over the
  // first half of the angles with the half geometry's context `half` (tables and plans)
  bool mm = false;
  // ADMM_BK_STAGING at creation (A/B, tests): "reg" register-staged back windows, "dma1" LDS-DMA
  // windows with one lane block per block, "dma2" two lane blocks per block wherever the lane
  // blocks pair up; default: LDS-DMA, two lane blocks per block where the grid still fills the chip
  int bk_staging = 0;   // 0 default, 1 reg, 2 dma1, 3 dma2
  int n_cu = 0;         // compute units of the device
  admm_ctx* half = nullptr;
  Buf xs, xsT, p, pT, Hp, sino, bI, fpart, r, c, d2, e2;
  Buf dsumS;  // D = sum_j q_ij as interleaved samples (BACK_H epilogue)
  Buf x2, p2; // ping-pong partners of x (local rows) and p for the fused TV update
  Buf pring;  // CG direction slots 1 .. K-1 (direction ring; slot 0 = p, slot K = p2)
  Buf ats;    // A^T (A xs - b) of the last update's final x (ADMM_BATCH_KEEP_X)
  // admm_time_forward(in_solve): events around every CG-step forward tap launch of one
  // directly enqueued x-update (null outside that measurement)
  std::vector<hipEvent_t>* tf_ev = nullptr;
  size_t tf_next = 0;
  int tf_kind = 0;  // what the in-solve events bracket: 0 forward taps, 1 back projector (BACK_H)
  bool ats_valid = false;  // ats matches x_ext's local rows
  hipGraph_t g_update_reuse = nullptr;
  hipGraphExec_t x_update_reuse = nullptr;
  Buf partH, partS, partD, partE;
  Buf redH;
  int P_back = 0, P_tile = 0, P_fwd = 0, P_edge = 0;
  hipGraph_t g_update = nullptr, g_cons = nullptr;
  hipGraphExec_t x_update = nullptr, x_cons = nullptr;
};

namespace {

#define RET(expr)                   \
  do {                              \
    int _rc = (expr);               \
    if (_rc != ADMM_OK) return _rc; \
  } while (0)

constexpr int kXcds = 8;  // MI355X: 8 XCDs, workgroups dealt round-robin (id % 8)

// Node-interleave width of a batch of V nodes: 32-byte sample vectors at most for float64
// (8 float64 nodes = 64 B would need 4 sample planes per tap: the forward loses its
// LDS-DMA staging, the back projector spills at 128 VGPRs; C5s 65.0 vs 63.0 node-updates/s)
int vb_for(int V, int dtype) {
  const int vb = V >= 5 ? 8 : (V >= 3 ? 4 : (V == 2 ? 2 : 1));
  return dtype == ADMM_DTYPE_F64 ? std::min(vb, 4) : vb;
}

void select_fwd_plan(admm_ctx* C, int pl) {
  C->groups = C->plan_groups[pl];
  C->rng = C->plan_rng[pl];
  C->n_groups = C->plan_n[pl];
}

// Block table of the grouped forward projector for nch node chunks: every live
// (ray chunk, group, segment, node chunk), sorted by group size G (waves of work), heaviest
// first.  When every block is resident at once (<= 2 per CU) the second half is reversed so
// the blocks sharing a CU pair heavy with light (dispatch fills one slot per CU, then the
// second); otherwise heaviest-first is the longest-processing-time order.
int build_fwd_order_into(admm_ctx* C, int pl, int nch, int cus, Buf& buf, int* nblk) {
  struct Blk {
    int4 b;
    int w;
  };
  std::vector<Blk> v;
  for (int c = 0; c < nch; ++c)
    for (const int4& b : C->plan_blk[pl]) v.push_back({make_int4(b.x, b.y, b.z + kFgSeg * c, 0), b.w});
  const int n = (int)v.size();
  auto by_weight = [](std::vector<Blk>& l, int slots) {
    std::stable_sort(l.begin(), l.end(), [](const Blk& a, const Blk& b) { return a.w > b.w; });
    const int m = (int)l.size();
    if (m <= 2 * slots && m > slots) std::reverse(l.begin() + slots, l.end());
  };
  if (cus > 0 && cus % kXcds == 0) {
    // XCD-aware: workgroups are dealt round-robin over the 8 XCDs (id % 8), so launch
    // position p runs on XCD p % 8.  Row segment s goes to XCD s % 8: each XCD's L2 then
    // holds one band of image rows (and of the transposed copy) instead of re-fetching the
    // whole image from the Infinity Cache (LDS-DMA staging reads ~10x the image per launch).
    // Per XCD: heaviest first, the second round reversed (heavy + light per CU pair).
    // Mirror mode (the half geometry): a case-B block of segment s stages rows of band s
    // (virtual plane 0) and of band kFgSeg-1-s (plane 1, row N-1-m), a case-A block only
    // band s of the transposed image (plane 1 mirrors the column).  Segments s and
    // kFgSeg-1-s therefore share an XCD pair: one XCD takes their case-B blocks, the other
    // their case-A blocks, so each band of either image lives in one L2 (segment-per-XCD put
    // every img band in two L2s: FETCH_SIZE 2x, profiles/r4_mirror_xcd.txt).
    const char* mx = getenv("ADMM_FWD_MIRROR_XCD");  // "0": segment-per-XCD (A/B)
    const bool paired = C->mirror_half && !(mx && mx[0] == '0');
    auto xcd_of = [&](const int4& b) {
      const int sg = b.z % kFgSeg;
      if (!paired) return sg % kXcds;
      const int pair = std::min(sg, kFgSeg - 1 - sg);
      return (2 * pair + (C->plan_caseA[pl][b.y] ? 1 : 0)) % kXcds;
    };
    std::vector<std::vector<Blk>> L(kXcds);
    for (const Blk& b : v) L[xcd_of(b.b)].push_back(b);
    for (auto& l : L) by_weight(l, cus / kXcds);
    std::vector<size_t> pos(kXcds, 0);
    v.clear();
    for (int p = 0; p < n; ++p) {
      int x = p % kXcds;
      if (pos[x] >= L[x].size()) {  // this XCD's segment is used up: the fullest list lends
        size_t best = 0;
        for (int y = 0; y < kXcds; ++y)
          if (L[y].size() - pos[y] > best) best = L[y].size() - pos[y], x = y;
      }
      v.push_back(L[x][pos[x]++]);
    }
  } else if (cus > 0) {  // cus <= 0: launch order = table order (tuning comparison)
    by_weight(v, cus);
  }
  std::vector<int4> t(n);
  for (int i = 0; i < n; ++i) t[i] = v[i].b;
  const int rc = ensure(buf, (size_t)n * sizeof(int4));
  if (rc != ADMM_OK) return rc;
  HIPCHK(hipMemcpy(buf.p, t.data(), (size_t)n * sizeof(int4), hipMemcpyHostToDevice));
  *nblk = n;
  return ADMM_OK;
}

int build_fwd_order(admm_ctx* C, int pl, int nch, int cus) {
  RET(build_fwd_order_into(C, pl, nch, cus, C->fg_order, &C->fg_nblk));
  C->fg_order_nch = nch;
  return ADMM_OK;
}

// Forward plan for the bound batch, by rounds of resident blocks: a launch of B blocks on
// S = (blocks per CU) x CUs slots runs ceil(B / S) rounds, and a partial last round costs
// nearly a full one (C3 mirror mode: 1024 / 992 blocks = 2 rounds, 65 us; 1056-1296 = 3
// rounds, 74-84 us; profiles/r4_fwd_plan_rounds.txt).  Among the plans with the fewest
// rounds, the one staging the fewest row pixels (1024^2, 2048^2: the chunk-aligned plan with
// clipped rays, 107 / 870 us against 130 / 1020 for the best unclipped one) -- except in a
// single round, where the 64-ray plan's equal segment shares keep every XCD on its own row
// band (512^2, one chunk: 33 us against 35-37 for the clipped plans).
// ADMM_FWD_PLAN=0..5 forces a plan.
// MIRROR / VBR: the instantiation launch_fwdg_taps launches (mirror mode: k_fwdg<T, VBV, true,
// VBR>, whose piece state and second window buffer set its own registers and LDS), so the
// occupancy query prices the kernel that actually runs.
template <typename T, int VB, bool MIRROR = false, int VBR = VB, int CPB = 1>
int pick_fwd_plan(admm_ctx* C, int nch, int* pl_out, int* cus_out, long* slots_out = nullptr) {
  int per_cu = 0, cus = 0;
  HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_fwdg<T, VB, MIRROR, VBR, CPB>, kFgThreads, 0));
  HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, C->device));
  if (per_cu < 1) return fail(ADMM_E_HIP, "grouped forward projector cannot be resident");
  const long slots = (long)per_cu * std::max(1, cus);
  auto rounds = [&](int pl) { return ((long)C->plan_blocks[pl] * nch + slots - 1) / slots; };
  int pl = 0;
  for (int q = 1; q < admm_ctx::kPlans; ++q) {
    if (C->plan_n[q] == 0) continue;
    if (rounds(q) < rounds(pl) || (rounds(q) == rounds(pl) && C->plan_staged[q] < C->plan_staged[pl])) pl = q;
  }
  if (rounds(pl) == 1 && rounds(0) == 1) pl = 0;
  const char* f = getenv("ADMM_FWD_PLAN");
  if (f && f[0] >= '0' && f[0] < '0' + admm_ctx::kPlans && C->plan_n[f[0] - '0'] > 0) pl = f[0] - '0';
  *pl_out = pl;
  *cus_out = cus;
  if (slots_out) *slots_out = slots;
  return ADMM_OK;
}

// Two virtual chunks per forward block (k_fwdg CPB = 2: mirror mode, float32, one lane block per
// real chunk) where the halved block table still fills every resident slot -- C3 and larger on
// one GPU; the 8-node share of the scaling runs keeps one (its halved table would leave slots
// empty).  ADMM_FWD_CPB=1 / 2 forces one / two (A/B and the bitwise tests; 2 needs an even
// chunk count).
template <typename T, int VB, bool MIRROR, int VBR>
constexpr bool fwd_cpb2_ok() {
  return MIRROR && std::is_same<T, float>::value && VB / 2 == VBR && VB == 8;
}

template <typename T, int VB, bool MIRROR = false, int VBR = VB>
int choose_fwd_plan(admm_ctx* C, int V) {
  if (C->plan_n[0] == 0) return ADMM_OK;
  const int nch = (V + VB - 1) / VB;
  C->fg_cpb = 1;
  if constexpr (fwd_cpb2_ok<T, VB, MIRROR, VBR>()) {
    const char* f = getenv("ADMM_FWD_CPB");
    const int force = (f && f[0] >= '1' && f[0] <= '2') ? f[0] - '0' : 0;
    if (nch % 2 == 0 && force != 1) {
      int pl2 = 0, cus2 = 0;
      long slots2 = 0;
      RET((pick_fwd_plan<T, VB, MIRROR, VBR, 2>(C, nch / 2, &pl2, &cus2, &slots2)));
      if (force == 2 || (long)C->plan_blocks[pl2] * (nch / 2) >= slots2) {
        select_fwd_plan(C, pl2);
        RET(build_fwd_order(C, pl2, nch / 2, cus2));
        C->fg_order_nch = nch;
        C->fg_cpb = 2;
        return ADMM_OK;
      }
    }
  }
  int pl = 0, cus = 0;
  RET((pick_fwd_plan<T, VB, MIRROR, VBR>(C, nch, &pl, &cus)));
  select_fwd_plan(C, pl);
  return getenv("ADMM_FWD_NATURAL_ORDER") && getenv("ADMM_FWD_NATURAL_ORDER")[0] == '1'
             ? build_fwd_order(C, pl, nch, 0)
             : build_fwd_order(C, pl, nch, cus);
}

template <typename F>
int with_vb(int vb, F&& f) {
  switch (vb) {
    case 8: return f(std::integral_constant<int, 8>{});
    case 4: return f(std::integral_constant<int, 4>{});
    case 2: return f(std::integral_constant<int, 2>{});
    default: return f(std::integral_constant<int, 1>{});
  }
}

// Virtual node-interleave width of mirror mode for a real width VBR: twice VBR, at most one
// 32-byte vector (8 float32 / 4 float64 lanes)
template <typename T, int VBR>
constexpr int mirror_vb() {
  return 2 * VBR < 32 / (int)sizeof(T) ? 2 * VBR : 32 / (int)sizeof(T);
}
// Mirror mode applies to the geometry and sample type, never to the batch (so every node runs
// the same arithmetic whatever its batch's size: rank- and batch-invariant results): an even
// number of angles spanning [0, pi) (block_2_load_odl_data.py:51) and a detector symmetric
// about 0 (block_2:52, uniform_partition(-1, 1, N)).  On by default for float32 samples
// (C3: 62 vs 57 us per forward launch at 16 nodes, but a 4-node rank of C4 on 8 GPUs runs
// 9.4 instead of 11.5 ms per iteration: profiles/r4_mirror_ab.txt); float64 (C5: 2 real
// nodes per 16-byte vector) measured slower in both widths, so opt-in there.
// ADMM_FWD_MIRROR=0 / 1 forces it off / on.
bool mirror_eligible(const admm_ctx* C) {
  if (C->csr || C->g.n_angles < 2 || C->g.n_angles % 2 != 0) return false;
  const char* e = getenv("ADMM_FWD_MIRROR");
  const bool want = (e && e[0]) ? e[0] == '1' : C->dtype == ADMM_DTYPE_F32;
  if (!want) return false;
  const double pi = 3.14159265358979323846;
  return std::fabs(C->g.angle_min) <= 1e-15 && std::fabs(C->g.angle_max - pi) <= 1e-12 &&
         std::fabs(C->g.det_min + C->g.det_max) <= 1e-12 * std::fabs(C->g.det_max);
}

// The bound batch's forward plan and its segment-partial buffer, set together: the clipped
// plans (3-5) write only the (segment, ray) partials of rays crossing the segment inside the
// image and k_fwd_combine reads every slot, so whenever the plan (or the batch) changes, every
// slot is zeroed here -- the one place C->fpart's plan is chosen (the operator API's op_fpart
// keeps its own plan key, op_forward_chunk).
int bind_fwd_plan(admm_ctx* C, int V) {
  C->mm = C->n_groups > 0 && mirror_eligible(C);
  // mirror mode keeps the real sample vectors at 16 bytes (4 float32 / 2 float64 nodes): a
  // virtual chunk then stages every byte of the real vectors it reads -- with 32-byte real
  // vectors each virtual chunk read every other 16 bytes and its sibling chunk the rest
  // (C3: 76 vs 58 us per forward launch, profiles/r4_mirror_ab.txt)
  if (C->mm) C->vb = std::min(C->vb, 16 / (int)dsize(C->dtype));
  if (C->mm && !C->half) {
    // the half geometry: the first a/2 angles, bitwise the full geometry's (angle_max - angle_min
    // is halved exactly and so is the angle count: the same step (t + 1/2) pi / a)
    admm_geom hg = C->g;
    hg.n_angles = C->g.n_angles / 2;
    hg.angle_max = C->g.angle_min + 0.5 * (C->g.angle_max - C->g.angle_min);
    RET(admm_ctx_create(&C->half, &hg, C->dtype, 1, C->device));  // (tables and plans only)
    C->half->mirror_half = true;
    if (C->half->n_groups == 0) C->mm = false;  // (cannot happen: half the angles fit as well)
  }
  if (C->mm) {
    RET(with_vb(C->vb, [&](auto vbc) -> int {
      constexpr int VBR = decltype(vbc)::value;
      const int nchv = ((V + VBR - 1) / VBR) * (2 * VBR / (C->dtype == ADMM_DTYPE_F32 ? mirror_vb<float, VBR>()
                                                                                      : mirror_vb<double, VBR>()));
      if (C->dtype == ADMM_DTYPE_F32) {
        constexpr int VBV = mirror_vb<float, VBR>();
        return choose_fwd_plan<float, VBV, true, VBR>(C->half, nchv * VBV);
      }
      constexpr int VBV = mirror_vb<double, VBR>();
      return choose_fwd_plan<double, VBV, true, VBR>(C->half, nchv * VBV);
    }));
  } else {
    RET(with_vb(C->vb, [&](auto vbc) {
      constexpr int VB = decltype(vbc)::value;
      return C->dtype == ADMM_DTYPE_F32 ? choose_fwd_plan<float, VB>(C, V) : choose_fwd_plan<double, VB>(C, V);
    }));
  }
  if (C->n_groups > 0) {
    // (mirror: virtual chunks x half the rays x the virtual width -- the same element count)
    const size_t Vp = (size_t)((V + C->vb - 1) / C->vb) * C->vb;
    RET(ensure(C->fpart, (size_t)kFgSeg * Vp * C->mrays * dsize(C->dtype)));
    HIPCHK(hipMemset(C->fpart.p, 0, C->fpart.bytes));
    HIPCHK(hipDeviceSynchronize());
  }
  return ADMM_OK;
}

template <typename T, int VB, int MODE>
int launch_fwd(admm_ctx* C, const T* img, const T* imgT, T* sino, const T* b, double* part, int V, hipStream_t s) {
  if (C->csr) {  // explicit matrix: one thread per sinogram row
    dim3 cg((C->mrays + kBlock - 1) / kBlock, (V + VB - 1) / VB);
    hipLaunchKernelGGL((k_csr_fwd<T, VB, MODE>), cg, dim3(kBlock), 0, s, (const int*)C->f_ptr.p,
                       (const int*)C->f_idx.p, (const T*)C->f_val.p, img, sino, b, part, C->mrays, C->npix, V);
    CHECK_LAUNCH();
    return ADMM_OK;
  }
  dim3 grid((C->g.n_det + kFwdRays - 1) / kFwdRays, C->g.n_angles, (V + VB - 1) / VB);
  hipLaunchKernelGGL((k_fwd<T, VB, MODE>), grid, dim3(kFwdBlock), 0, s, img, imgT, sino, b, part, C->fang, C->g.N,
                     C->g.n_det, C->g.n_angles, V);
  CHECK_LAUNCH();
  return ADMM_OK;
}

// hot-path forward projection of the bound batch: grouped kernel + fixed-order combine
// the grouped forward projector's tap kernel (all sample taps; segment partials -> fpart)
template <typename T, int VB>
int launch_fwdg_taps_with(admm_ctx* C, const T* img, const T* imgT, T* fpart, const FgGroup* groups,
                          const FgRange* rng, const int4* order, int nblk, int V, hipStream_t s) {
  hipLaunchKernelGGL((k_fwdg<T, VB>), dim3(nblk), dim3(kFgThreads), 0, s, img, imgT, fpart, C->fang, groups, rng,
                     order, C->g.N, C->g.n_det, C->g.n_angles, V);
  CHECK_LAUNCH();
  return ADMM_OK;
}

template <typename T, int VB>
int launch_fwdg_taps(admm_ctx* C, const T* img, const T* imgT, int V, hipStream_t s) {
  if (C->mm) {  // mirror mode: virtual chunks of the half geometry (k_fwdg MIRROR)
    constexpr int VBV = mirror_vb<T, VB>(), MH = VBV / 2;
    const int nchv = ((V + VB - 1) / VB) * (VB / MH);
    const admm_ctx* H = C->half;
    if (nchv != H->fg_order_nch) return fail(ADMM_E_STATE, "mirror block table built for another batch size");
    if constexpr (fwd_cpb2_ok<T, VBV, true, VB>()) {
      if (H->fg_cpb == 2) {  // two virtual chunks per block (the table holds chunk pairs)
        hipLaunchKernelGGL((k_fwdg<T, VBV, true, VB, 2>), dim3(H->fg_nblk), dim3(kFgThreads), 0, s, img, imgT,
                           (T*)C->fpart.p, H->fang, H->groups, H->rng, (const int4*)H->fg_order.p, C->g.N,
                           C->g.n_det, H->g.n_angles, nchv * VBV);
        CHECK_LAUNCH();
        return ADMM_OK;
      }
    }
    hipLaunchKernelGGL((k_fwdg<T, VBV, true, VB>), dim3(H->fg_nblk), dim3(kFgThreads), 0, s, img, imgT,
                       (T*)C->fpart.p, H->fang, H->groups, H->rng, (const int4*)H->fg_order.p, C->g.N, C->g.n_det,
                       H->g.n_angles, nchv * VBV);
    CHECK_LAUNCH();
    return ADMM_OK;
  }
  const int nch = (V + VB - 1) / VB;
  if (nch != C->fg_order_nch) return fail(ADMM_E_STATE, "forward block table built for another batch size");
  return launch_fwdg_taps_with<T, VB>(C, img, imgT, (T*)C->fpart.p, C->groups, C->rng,
                                      (const int4*)C->fg_order.p, C->fg_nblk, V, s);
}

template <typename T, int VB, int MODE>
int launch_fwd_batch(admm_ctx* C, const T* img, const T* imgT, T* sino, const T* b, double* part, int V,
                     hipStream_t s, bool timed = false) {
  // timed (admm_time_forward in_solve): HIP events right before and after the tap kernel
  hipEvent_t* ev = nullptr;
  if (timed && C->tf_ev && C->tf_kind == 0 && C->tf_next + 2 <= C->tf_ev->size()) {
    ev = C->tf_ev->data() + C->tf_next;
    C->tf_next += 2;
    HIPCHK(hipEventRecord(ev[0], s));
  }
  if (C->n_groups == 0) {
    RET((launch_fwd<T, VB, MODE>(C, img, imgT, sino, b, part, V, s)));
    if (ev) HIPCHK(hipEventRecord(ev[1], s));
    return ADMM_OK;
  }
  const int nch = (V + VB - 1) / VB;
  RET((launch_fwdg_taps<T, VB>(C, img, imgT, V, s)));
  if (ev) HIPCHK(hipEventRecord(ev[1], s));
  if (C->mm) {  // virtual partials -> the real sinogram (both angles of every virtual ray)
    constexpr int VBV = mirror_vb<T, VB>(), MH = VBV / 2;
    const int mh = C->half->mrays;
    // MODE 0: two threads per virtual ray (k_fwd_combine_mirror); MODE 1: one (its block partials)
    const size_t mthreads = (size_t)mh * (MODE == 0 ? 2 : 1);
    dim3 mg((unsigned)((mthreads + kBlock - 1) / kBlock), nch * (VB / MH));
    hipLaunchKernelGGL((k_fwd_combine_mirror<T, VBV, VB, MODE>), mg, dim3(kBlock), 0, s, (const T*)C->fpart.p, sino,
                       b, part, C->half->fang, C->g.n_det, C->half->g.n_angles, V);
    CHECK_LAUNCH();
    return ADMM_OK;
  }
  dim3 cg((C->mrays + kBlock - 1) / kBlock, nch);
  hipLaunchKernelGGL((k_fwd_combine<T, VB, MODE>), cg, dim3(kBlock), 0, s, (const T*)C->fpart.p, sino, b, part,
                     C->fang, C->g.n_det, C->g.n_angles, V);
  CHECK_LAUNCH();
  return ADMM_OK;
}

template <typename T, int VB, int MODE>
int launch_back(admm_ctx* C, BackArgs<T> a, int V, hipStream_t s) {
  if constexpr (MODE == BACK_H || MODE == BACK_INIT || MODE == BACK_DIAG || MODE == BACK_ATB) {
    if (C->mm) {  // mirror mode: pixel pairs of the upper half, the half geometry's angles
      constexpr int VBV = mirror_vb<T, VB>(), MH = VBV / 2;
      const admm_ctx* H = C->half;
      a.ang = H->bang;
      a.angc = H->bangc;
      a.K = H->Kb;
      a.kbias = H->kbias;
      a.wexp = H->wexp;
      a.N = C->g.N;
      a.n_det = C->g.n_det;
      a.n_ang = H->g.n_angles;
      a.V = V;
      const int N = C->g.N, Nh = (N + 1) / 2;
      dim3 grid((N + kBTJ - 1) / kBTJ, (Nh + kBTI - 1) / kBTI, ((V + VB - 1) / VB) * (VB / MH));
      bool done = false;
      if constexpr (back_mirror_dma<T, VBV, MODE>()) {
        if (C->bk_staging == 1) {  // the register-staged windows (where DMA is the default)
          hipLaunchKernelGGL((k_back_mirror_reg<T, VBV, VB, MODE>), grid, dim3(kBkThreads), 0, s, a);
          done = true;
        } else if constexpr (std::is_same<T, float>::value && ADMM_BK_LB2) {
          // two lane blocks per block while half the blocks still give every CU one
          const bool fills = (long)grid.x * grid.y * grid.z >= 2L * C->n_cu;
          if (grid.z % 2 == 0 && (C->bk_staging == 3 || (C->bk_staging == 0 && fills))) {
            hipLaunchKernelGGL((k_back_mirror_2<T, VBV, VB>), dim3(grid.x, grid.y, grid.z / 2), dim3(kBkThreads), 0,
                               s, a);
            done = true;
          }
        }
      }
      if (!done) hipLaunchKernelGGL((k_back_mirror<T, VBV, VB, MODE>), grid, dim3(kBkThreads), 0, s, a);
      CHECK_LAUNCH();
      return ADMM_OK;
    }
  }
  a.ang = C->bang;
  a.angc = C->bangc;
  a.K = C->Kb;
  a.kbias = C->kbias;
  a.wexp = C->wexp;
  a.N = C->g.N;
  a.n_det = C->g.n_det;
  a.n_ang = C->g.n_angles;
  a.V = V;
  const int N = C->g.N;
  dim3 grid((N + kBTJ - 1) / kBTJ, (N + kBTI - 1) / kBTI, MODE == BACK_WSQ ? 1 : (V + VB - 1) / VB);
  if (C->csr) {
    a.csr_ptr = (const int*)C->t_ptr.p;
    a.csr_idx = (const int*)C->t_idx.p;
    a.csr_val = (const T*)C->t_val.p;
    hipLaunchKernelGGL((k_back<T, VB, MODE, true>), grid, dim3(kBkThreads), 0, s, a);
  } else {
    hipLaunchKernelGGL((k_back<T, VB, MODE>), grid, dim3(kBkThreads), 0, s, a);
  }
  CHECK_LAUNCH();
  return ADMM_OK;
}

int back_partitions(admm_ctx* C) {
  const int N = C->g.N;
  const int rows = C->mm ? (N + 1) / 2 : N;  // mirror mode: blocks over the upper half's pixel pairs
  return ((N + kBTJ - 1) / kBTJ) * ((rows + kBTI - 1) / kBTI);
}
dim3 tile_grid(admm_ctx* C, int nchunks, int vb) {
  const int N = C->g.N, ti = kTile / vb;
  return dim3((N + kTile - 1) / kTile, (N + ti - 1) / ti, nchunks);
}

int launch_reduce(const double* part, int rows, int P, double* out, int G, int ostride, int ooff, hipStream_t s) {
  hipLaunchKernelGGL(k_reduce_rows, dim3(rows), dim3(kBlock), 0, s, part, P, out, G, ostride, ooff);
  CHECK_LAUNCH();
  return ADMM_OK;
}

// the edge state the x-update reads (stored z, or z derived from x_prev: ABI 7)
EdgeIn edge_in(const admm_batch& B) {
  EdgeIn E{};
  E.z = B.z;
  E.y = B.y;
  E.yb = B.fusion == ADMM_FUSE_WEIGHTED ? B.y_b : nullptr;
  E.xp = B.x_prev;
  E.ea = B.edge_a;
  E.eb = B.edge_b;
  return E;
}

// --------------------------------------------------------------------------
// the x-update sequence for the bound batch (replaces block_6_admm_loop_ver2.py:81-197)
// --------------------------------------------------------------------------
template <typename T, int VB>
int enqueue_update(admm_ctx* C, hipStream_t s, bool reuse = false, int rounds = 0) {
  const admm_batch& B = C->b;
  const int V = B.V, N = C->g.N;
  const size_t npix = (size_t)N * N;
  const int nch = (V + VB - 1) / VB;
  T* xs = (T*)C->xs.p;
  T* xsT = (T*)C->xsT.p;
  T* p = (T*)C->p.p;
  T* pT = (T*)C->pT.p;
  T* Hp = (T*)C->Hp.p;
  T* sino = (T*)C->sino.p;
  double* r = (double*)C->r.p;
  double* c = (double*)C->c.p;
  double* redH = (double*)C->redH.p;
  const dim3 tg = tile_grid(C, nch, VB);
  const dim3 cgg((N + kTile - 1) / kTile, (N + kCgRows - 1) / kCgRows, nch);
  const dim3 tvg((N + kTvTile - 1) / kTvTile, (N + TvMap<VB>::TI - 1) / TvMap<VB>::TI, nch);  // k_tv_update
  const int Pb = C->P_back;

  // (D as interleaved samples for the CG operator, dsumS, is packed once at bind time)
  if (reuse) {
    // 1-4. one kernel from the previous update's A^T (A xs - b) (ADMM_BATCH_KEEP_X):
    //      c, r = A^T b + rho c + mu K^T(d - e) - H x, p = r (+ transpose)
    hipLaunchKernelGGL((k_start_reuse<T, VB>), cgg, dim3(kBlock), 0, s, (const T*)C->ats.p, B.x_ext, edge_in(B),
                       B.q, B.inc_off, B.inc_edge, B.inc_qslot, B.inc_sign, B.atb, c, B.dsum, B.d, B.e, r, p, pT,
                       B.rho, B.mu, N, V);
    CHECK_LAUNCH();
  } else {
  // 1. neighbour gather: c = sum_j q_ij (z_ij - y_ij,i); xs = (T) x (+ transpose)
  hipLaunchKernelGGL((k_gather<T, VB>), tg, dim3(kBlock), 0, s, B.x_ext, edge_in(B), B.q, B.inc_off, B.inc_edge,
                     B.inc_qslot, B.inc_sign, c, xs, xsT, N, V);
  CHECK_LAUNCH();
  // 2-4. r = A^T b + rho c + mu K^T(d - e) - H x,  p = r,  rr
  RET((launch_fwd_batch<T, VB, 0>(C, xs, xsT, sino, nullptr, nullptr, V, s)));
  {
    BackArgs<T> a{};
    a.sino = sino;
    a.out_t = p;
    a.out_d = r;
    a.pin = xs;
    a.dsum = B.dsum;
    a.atb = B.atb;
    a.cvec = c;
    a.dvar = B.d;
    a.evar = B.e;
    a.rho = B.rho;
    a.lam = B.lam;
    a.mu = B.mu;
    RET((launch_back<T, VB, BACK_INIT>(C, a, V, s)));
  }
  hipLaunchKernelGGL((k_transpose<T, VB>), tg, dim3(kBlock), 0, s, p, pT, N);
  CHECK_LAUNCH();
  }

  const double tau = B.lam / B.mu;
  double* dcur = B.d;
  double* ecur = B.e;
  double* dnxt = (double*)C->d2.p;
  double* enxt = (double*)C->e2.p;
  // Every x step of a round is applied by the TV update that ends it (F = 2: the CG updates
  // leave x alone and write each new direction to its own slot of a ring, p_0 .. p_K); with
  // more CG steps than ring slots only the round's last step is (F = 1).  The TV update reads
  // x and the directions over its tiles' halos while writing them, so x ping-pongs
  // (xcur -> xnxt) and the restart p = r goes to the ring's spare slot.
  const int K = B.cg_iters, Tt = rounds > 0 ? rounds : B.tv_iters;
  const int F = (K <= kMaxCgRing) ? 2 : 1;
  double* xcur = B.x_ext;
  double* xnxt = (double*)C->x2.p;
  std::vector<T*> slot(K + 1, p);
  if (F == 1) slot[1] = (T*)C->p2.p;
  if (F == 2) {
    slot[K] = (T*)C->p2.p;
    for (int k = 1; k < K; ++k) slot[k] = (T*)C->pring.p + (size_t)(k - 1) * nch * npix * VB;
  }
  const size_t rstride = (F == 2) ? (size_t)5 * V : 0;  // redH ring stride (one reduction per step)
  for (int t = 0; t < Tt; ++t) {
    for (int kk = 0; kk < K; ++kk) {
      T* pk = (F == 2) ? slot[kk] : slot[0];
      double* rk = redH + kk * rstride;
      RET((launch_fwd_batch<T, VB, 0>(C, pk, pT, sino, nullptr, nullptr, V, s, true)));
      BackArgs<T> a{};
      a.sino = sino;
      a.out_t = Hp;
      a.part = (double*)C->partH.p;
      a.pin = pk;
      a.r = r;
      a.dsum = B.dsum;
      a.dsum_s = (const T*)C->dsumS.p;
      a.rho = B.rho;
      a.lam = B.lam;
      a.mu = B.mu;
      // (admm_time_back: events right before and after each in-solve back projection)
      hipEvent_t* bev = nullptr;
      if (C->tf_ev && C->tf_kind == 1 && C->tf_next + 2 <= C->tf_ev->size()) {
        bev = C->tf_ev->data() + C->tf_next;
        C->tf_next += 2;
        HIPCHK(hipEventRecord(bev[0], s));
      }
      RET((launch_back<T, VB, BACK_H>(C, a, V, s)));
      if (bev) HIPCHK(hipEventRecord(bev[1], s));
      RET(launch_reduce((double*)C->partH.p, 5 * V, Pb, rk, 1, 1, 0, s));
      if (kk + 1 < K) {
        if (F == 2)
          hipLaunchKernelGGL((k_cg_update<T, VB, true, false>), cgg, dim3(kBlock), 0, s, xcur, r, (const T*)pk, pT,
                             Hp, rk, N, V, slot[kk + 1]);
        else
          hipLaunchKernelGGL((k_cg_update<T, VB, true, true>), cgg, dim3(kBlock), 0, s, xcur, r, (const T*)pk, pT,
                             Hp, rk, N, V, pk);
        CHECK_LAUNCH();
      }  // the round's last step: applied by the TV update
    }
    const bool last = (t + 1 == Tt);
    PRing<T> pr{};
    pr.K = (F == 2) ? K : 1;
    for (int k = 0; k < pr.K; ++k) pr.p[k] = slot[k];
    T* pout = last ? xs : (F == 2 ? slot[K] : (F == 1 ? slot[1] : slot[0]));
    T* poutT = last ? xsT : pT;
    // split-Bregman state in/out of this round: d, e (B.d / B.e or the scratch pair) or,
    // between the rounds of the update (Tt > 1), u = Kx + e in ua / ub
    const bool uin = t > 0 && Tt > 1;
    const bool uout = !last && Tt > 1;
    double* ua = (double*)C->d2.p;
    double* ub = (double*)C->e2.p;
    const double* din = uin ? ((t % 2) ? ua : ub) : dcur;
    const double* ein = ecur;  // (not read when uin)
    double* dout = uout ? ((t % 2) ? ub : ua) : (Tt > 1 ? B.d : dnxt);
    double* eout = uout ? nullptr : (Tt > 1 ? B.e : enxt);
#define TV_LAUNCH(LASTV, FUSEV, UINV, UOUTV)                                                                     \
  hipLaunchKernelGGL((k_tv_update<T, VB, LASTV, FUSEV, UINV, UOUTV>), tvg, dim3(kTvThreads), 0, s, xcur, din, ein, dout, \
                     eout, r, pout, poutT, tau, B.mu, B.tv_kind, N, V, xnxt, pr, Hp, redH)
    if (!last) {
      if (uin) TV_LAUNCH(false, true, true, true);
      else if (uout) TV_LAUNCH(false, true, false, true);
      else TV_LAUNCH(false, true, false, false);
    } else {
      if (uin) TV_LAUNCH(true, true, true, false);
      else TV_LAUNCH(true, true, false, false);
    }
#undef TV_LAUNCH
    CHECK_LAUNCH();
    if (Tt == 1) {  // one round: d, e went to the scratch pair
      std::swap(dcur, dnxt);
      std::swap(ecur, enxt);
    }
    std::swap(xcur, xnxt);
    if (!last) std::swap(slot[0], slot[F == 2 ? K : 1]);
  }
  if (xcur != B.x_ext)  // odd number of fused rounds: x ended in scratch
    HIPCHK(hipMemcpyAsync(B.x_ext, xcur, (size_t)V * npix * sizeof(double), hipMemcpyDeviceToDevice, s));
  if (dcur != B.d) {  // odd number of d / e rounds: state ended in scratch
    HIPCHK(hipMemcpyAsync(B.d, dcur, 2 * V * npix * sizeof(double), hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(B.e, ecur, 2 * V * npix * sizeof(double), hipMemcpyDeviceToDevice, s));
  }
  // diagnostics epilogue: s = A x - b, ||s||^2, g, TV, quad, image error
  RET((launch_fwd_batch<T, VB, 1>(C, xs, xsT, sino, (const T*)B.b, (double*)C->partS.p, V, s)));
  {
    BackArgs<T> a{};
    a.sino = sino;
    a.part = (double*)C->partD.p;
    a.dsum = B.dsum;
    a.cvec = c;
    a.x = B.x_ext;
    a.phantom = B.phantom;
    a.edges = edge_in(B);
    a.qv = B.q;
    a.inc_off = B.inc_off;
    a.inc_edge = B.inc_edge;
    a.inc_qslot = B.inc_qslot;
    a.inc_sign = B.inc_sign;
    a.rho = B.rho;
    a.lam = B.lam;
    a.mu = B.mu;
    a.tv_kind = B.tv_kind;
    a.evar = B.e;  // the final Bregman variable (copied back from scratch above for odd rounds)
    a.out_t = (B.flags & ADMM_BATCH_KEEP_X) ? (T*)C->ats.p : nullptr;
    RET((launch_back<T, VB, BACK_DIAG>(C, a, V, s)));
  }
  RET(launch_reduce((double*)C->partS.p, V, C->P_fwd, B.node_stats, 1, ADMM_NODE_STATS, ADMM_NODE_STAT_MSE_SINO, s));
  RET(launch_reduce((double*)C->partD.p, 5 * V, Pb, B.node_stats, 5, ADMM_NODE_STATS, ADMM_NODE_STAT_G2, s));
  return ADMM_OK;
}

template <typename T>
int enqueue_update_any(admm_ctx* C, hipStream_t s, bool reuse = false, int rounds = 0) {
  return with_vb(C->vb, [&](auto vbc) { return enqueue_update<T, decltype(vbc)::value>(C, s, reuse, rounds); });
}

// rows of the derived consensus' LDS tile (0: more x_ext rows than any tile: direct kernel)
int cons_rows(int n_xext) { return n_xext <= 16 ? 16 : n_xext <= 64 ? 64 : n_xext <= 128 ? 128 : 0; }

// stored-z midpoint consensus of edge slots [e0, e1) (k_consensus<false>: one edge per
// blockIdx.y, 1024 pixels per block; the endpoint rows are read from HBM / L2 per edge -- at C5's
// share, 476 edges over 64 rows, this streamed 48 B per pixel-edge in 14.1 ms against 17.4 ms for
// a pixel-major LDS-tile variant, profiles/AB_LOG.md round 5)
int enqueue_consensus_stored(admm_ctx* C, int e0, int e1, hipStream_t s) {
  const admm_batch& B = C->b;
  if (e1 <= e0) return ADMM_OK;
  const int npix = C->npix;
  dim3 grid((npix + kBlock * 4 - 1) / (kBlock * 4), e1 - e0);
  hipLaunchKernelGGL(k_consensus<false>, grid, dim3(kBlock), 0, s, B.x_ext, B.y, nullptr, B.z, nullptr, B.edge_a,
                     B.edge_b, (double*)C->partE.p, npix, e0);
  CHECK_LAUNCH();
  // rows 3 e0 .. 3 e1 - 1 of the partials -> edge_stats rows e0 .. e1 - 1
  RET(launch_reduce((double*)C->partE.p + (size_t)3 * e0 * C->P_edge, 3 * (e1 - e0), C->P_edge,
                    B.edge_stats + (size_t)3 * e0, 1, 1, 0, s));
  return ADMM_OK;
}

int enqueue_consensus(admm_ctx* C, hipStream_t s) {
  const admm_batch& B = C->b;
  if (B.n_edges == 0) return ADMM_OK;
  const int npix = C->npix;
  if (B.z == nullptr) {  // derived z (midpoint fusion, ABI 7)
    const dim3 g((npix + kConsPix - 1) / kConsPix);
    double* part = (double*)C->partE.p;
    switch (cons_rows(B.n_xext)) {
      case 16:
        hipLaunchKernelGGL(k_consensus_derived<16>, g, dim3(kBlock), 0, s, B.x_ext, B.x_prev, B.y, B.edge_a,
                           B.edge_b, part, npix, B.n_xext, B.n_edges);
        break;
      case 64:
        hipLaunchKernelGGL(k_consensus_derived<64>, g, dim3(kBlock), 0, s, B.x_ext, B.x_prev, B.y, B.edge_a,
                           B.edge_b, part, npix, B.n_xext, B.n_edges);
        break;
      case 128:
        hipLaunchKernelGGL(k_consensus_derived<128>, g, dim3(kBlock), 0, s, B.x_ext, B.x_prev, B.y, B.edge_a,
                           B.edge_b, part, npix, B.n_xext, B.n_edges);
        break;
      default: {
        hipLaunchKernelGGL(k_consensus_derived_direct, g, dim3(kBlock), 0, s, B.x_ext, B.x_prev, B.y, B.edge_a,
                           B.edge_b, part, npix, B.n_edges);
        CHECK_LAUNCH();
        const size_t cnt = (size_t)B.n_xext * npix;
        hipLaunchKernelGGL(k_copy_rows, dim3((unsigned)std::min<size_t>((cnt + kBlock - 1) / kBlock, 16384)),
                           dim3(kBlock), 0, s, (const double*)B.x_ext, B.x_prev, cnt);
      }
    }
    CHECK_LAUNCH();
    RET(launch_reduce(part, 3 * B.n_edges, C->P_edge, B.edge_stats, 1, 1, 0, s));
    return ADMM_OK;
  }
  if (B.fusion == ADMM_FUSE_MIDPOINT) return enqueue_consensus_stored(C, 0, B.n_edges, s);
  dim3 grid((npix + kBlock * 4 - 1) / (kBlock * 4), B.n_edges);
  hipLaunchKernelGGL(k_consensus<true>, grid, dim3(kBlock), 0, s, B.x_ext, B.y, B.y_b, B.z, B.w, B.edge_a,
                     B.edge_b, (double*)C->partE.p, npix);
  CHECK_LAUNCH();
  RET(launch_reduce((double*)C->partE.p, 3 * B.n_edges, C->P_edge, B.edge_stats, 1, 1, 0, s));
  return ADMM_OK;
}

int free_graphs(admm_ctx* C) {
  if (C->x_update) HIPCHK(hipGraphExecDestroy(C->x_update));
  if (C->g_update) HIPCHK(hipGraphDestroy(C->g_update));
  if (C->x_cons) HIPCHK(hipGraphExecDestroy(C->x_cons));
  if (C->g_cons) HIPCHK(hipGraphDestroy(C->g_cons));
  C->x_update = nullptr;
  C->g_update = nullptr;
  if (C->x_update_reuse) HIPCHK(hipGraphExecDestroy(C->x_update_reuse));
  if (C->g_update_reuse) HIPCHK(hipGraphDestroy(C->g_update_reuse));
  C->x_update_reuse = nullptr;
  C->g_update_reuse = nullptr;
  C->x_cons = nullptr;
  C->g_cons = nullptr;
  return ADMM_OK;
}

template <typename F>
int capture(admm_ctx* C, F&& fn, hipGraph_t* g, hipGraphExec_t* x) {
  HIPCHK(hipStreamBeginCapture(C->cap, hipStreamCaptureModeThreadLocal));
  int rc = fn(C->cap);
  hipGraph_t graph = nullptr;
  hipError_t e = hipStreamEndCapture(C->cap, &graph);
  if (rc != ADMM_OK) {
    if (graph) (void)hipGraphDestroy(graph);
    return rc;
  }
  if (e != hipSuccess) return fail(ADMM_E_HIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
  HIPCHK(hipGraphInstantiate(x, graph, nullptr, nullptr, 0));
  *g = graph;
  return ADMM_OK;
}

// Operator API forward projection (A @ x of node-major images).  When the geometry has
// angle-group plans this is the hot path's own kernel pair (k_fwdg + k_fwd_combine) on
// up to 8 images per launch: the images are packed into the interleaved sample layout
// (plus the transposed copy case-A angles read), projected, and the interleaved
// sinograms unpacked.  Otherwise (windows too wide for the grouped kernel) k_fwd.
template <typename T, int VB>
int op_forward_chunk(admm_ctx* C, const T* img, T* sino, int nc, hipStream_t s) {
  const int npix = C->npix, m = C->mrays;
  int pl = 0, cus = 0;
  RET((pick_fwd_plan<T, VB>(C, 1, &pl, &cus)));
  if (C->op_nblk[pl] == 0) RET(build_fwd_order_into(C, pl, 1, cus, C->op_order[pl], &C->op_nblk[pl]));
  if (C->op_fpart_key != pl * 16 + VB) {  // slots another plan / width wrote: back to 0
    HIPCHK(hipMemsetAsync(C->op_fpart.p, 0, C->op_fpart.bytes, s));
    C->op_fpart_key = pl * 16 + VB;
  }
  T* xs = (T*)C->op_img.p;
  T* xsT = (T*)C->op_imgT.p;
  T* sI = (T*)C->op_sino.p;
  hipLaunchKernelGGL((k_pack<T, VB>), dim3((npix + 255) / 256, 1), dim3(256), 0, s, img, xs, npix, nc);
  CHECK_LAUNCH();
  hipLaunchKernelGGL((k_transpose<T, VB>), tile_grid(C, 1, VB), dim3(kBlock), 0, s, (const T*)xs, xsT, C->g.N);
  CHECK_LAUNCH();
  RET((launch_fwdg_taps_with<T, VB>(C, xs, xsT, (T*)C->op_fpart.p, C->plan_groups[pl], C->plan_rng[pl],
                                    (const int4*)C->op_order[pl].p, C->op_nblk[pl], nc, s)));
  hipLaunchKernelGGL((k_fwd_combine<T, VB, 0>), dim3((m + kBlock - 1) / kBlock, 1), dim3(kBlock), 0, s,
                     (const T*)C->op_fpart.p, sI, (const T*)nullptr, (double*)nullptr, C->fang, C->g.n_det,
                     C->g.n_angles, nc);
  CHECK_LAUNCH();
  hipLaunchKernelGGL((k_unpack<T, VB>), dim3((m + 255) / 256, 1), dim3(256), 0, s, (const T*)sI, sino, m, nc);
  CHECK_LAUNCH();
  return ADMM_OK;
}

template <typename T>
int op_forward(admm_ctx* C, const T* img, T* sino, int nimg, hipStream_t s) {
  const size_t npix = C->npix, m = C->mrays, ds = sizeof(T);
  const int N = C->g.N;
  if (C->csr) return launch_fwd<T, 1, 0>(C, img, nullptr, sino, nullptr, nullptr, nimg, s);
  if (C->plan_n[0] == 0) {  // no angle-group plan for this geometry: ray-per-thread kernel
    RET(ensure(C->op_imgT, (size_t)nimg * npix * ds));
    hipLaunchKernelGGL((k_transpose<T, 1>), tile_grid(C, nimg, 1), dim3(kBlock), 0, s, img, (T*)C->op_imgT.p, N);
    CHECK_LAUNCH();
    return launch_fwd<T, 1, 0>(C, img, (const T*)C->op_imgT.p, sino, nullptr, nullptr, nimg, s);
  }
  const int step = vb_for(8, C->dtype);  // images per chunk: one sample vector (8 float32 / 4 float64)
  const int cmax = std::min(nimg, step);
  const int vbmax = vb_for(cmax, C->dtype);
  RET(ensure(C->op_img, vbmax * npix * ds));
  RET(ensure(C->op_imgT, vbmax * npix * ds));
  RET(ensure(C->op_sino, vbmax * m * ds));
  RET(ensure(C->op_fpart, (size_t)kFgSeg * vbmax * m * ds));
  for (int v0 = 0; v0 < nimg; v0 += step) {
    const int nc = std::min(step, nimg - v0);
    const T* in = img + (size_t)v0 * npix;
    T* out = sino + (size_t)v0 * m;
    RET(with_vb(vb_for(nc, C->dtype), [&](auto vbc) { return op_forward_chunk<T, decltype(vbc)::value>(C, in, out, nc, s); }));
  }
  return ADMM_OK;
}

}  // namespace

// ============================================================================
// C ABI
// ============================================================================
extern "C" {

int admm_abi_version(void) { return ADMM_ABI_VERSION; }
const char* admm_last_error(void) { return g_err.c_str(); }

int admm_ctx_create(admm_ctx** out, const admm_geom* geom, int dtype, int max_images, int device) {
  if (!out || !geom) return fail(ADMM_E_INVALID, "null argument");
  *out = nullptr;
  const admm_geom g = *geom;
  if (g.N < 2 || g.n_angles < 1 || g.n_det < 1) return fail(ADMM_E_INVALID, "bad geometry sizes");
  if (g.N > 4096) return fail(ADMM_E_INVALID, "N > 4096 is not supported");
  if (dtype != ADMM_DTYPE_F32 && dtype != ADMM_DTYPE_F64) return fail(ADMM_E_INVALID, "bad dtype");
  if (max_images < 1) return fail(ADMM_E_INVALID, "max_images < 1");
  const double h = 2.0 / g.N;
  const double hd = (g.det_max - g.det_min) / g.n_det;
  if (!(hd > 0)) return fail(ADMM_E_INVALID, "det_max <= det_min");
  if (hd < h * (1.0 - 1e-9))
    return fail(ADMM_E_INVALID, "detector spacing finer than the pixel size is not supported "
                                "(det_width_factor must be >= 1 with n_det = N)");
  const size_t npix = (size_t)g.N * g.N, m = (size_t)g.n_angles * g.n_det;
  if ((size_t)max_images * npix * 8 >= (1ull << 31) || (size_t)max_images * m * 8 >= (1ull << 31))
    return fail(ADMM_E_INVALID, "batch too large for 32-bit buffer offsets; split it across contexts");
  DEVICE_SCOPE(device);
  admm_ctx* C = new admm_ctx();
  C->g = g;
  C->dtype = dtype;
  C->device = device;
  {
    const char* st = getenv("ADMM_BK_STAGING");
    const std::string v = st ? st : "";
    C->bk_staging = v == "reg" ? 1 : v == "dma1" ? 2 : v == "dma2" ? 3 : 0;
  }
  HIPCHK(hipDeviceGetAttribute(&C->n_cu, hipDeviceAttributeMultiprocessorCount, device));
  C->max_images = max_images;
  C->npix = (int)npix;
  C->mrays = (int)m;

  // geometry tables, float64 (oracle/geometry.py)
  std::vector<FwdAngle> fa(g.n_angles);
  std::vector<BackAngle> ba(g.n_angles);
  std::vector<BackAngleC> bc(g.n_angles);
  C->Kb = -g.det_min / hd - 0.5;
  const double c0 = 0.5 * (g.N - 1);
  for (int t = 0; t < g.n_angles; ++t) {
    const double th = g.angle_min + (t + 0.5) * (g.angle_max - g.angle_min) / g.n_angles;
    const double cs = std::cos(th), sn = std::sin(th);
    const bool caseA = std::fabs(cs) >= std::fabs(sn);
    const double al = caseA ? cs : sn, be = caseA ? sn : cs;
    fa[t].A0 = c0 + (g.det_min / h + 0.5 * hd / h + c0 * be) / al;
    fa[t].A1 = (hd / h) / al;
    fa[t].dl = -be / al;
    fa[t].L = h / std::fabs(al);
    fa[t].caseA = caseA ? 1 : 0;
    ba[t].Bi = cs * h / hd;
    ba[t].Bj = sn * h / hd;
    ba[t].B0 = -c0 * (ba[t].Bi + ba[t].Bj) - g.det_min / hd - 0.5;
    ba[t].slope = (hd / h) / std::fabs(al);
    ba[t].L = h / std::fabs(al);
    bc[t].Bi = ba[t].Bi;
    bc[t].Bj = ba[t].Bj;
    const float sLf = (float)(ba[t].slope * ba[t].L);
    bc[t].ws = float2v{-sLf, sLf};
    bc[t].wc = float2v{(float)ba[t].L, (float)(ba[t].L - ba[t].slope * ba[t].L)};
    while (std::ldexp((double)bc[t].wc.x, -C->wexp) > 1.0) ++C->wexp;
    // smallest k_f of any pixel at this angle: Kb - c0 (|Bi| + |Bj|)
    const double kmn = C->Kb - c0 * (std::fabs(ba[t].Bi) + std::fabs(ba[t].Bj));
    C->kbias = std::max(C->kbias, (int)std::ceil(-kmn) + 2);
  }
  // the float taps' kf_split needs k_f + kbias in (0, 2^20) for every pixel and angle (the sum
  // with 2^20 must stay in [2^20, 2^21)); a detector far off the image could break that
  for (int t = 0; t < g.n_angles && dtype == ADMM_DTYPE_F32; ++t) {
    const double kmx = C->Kb + C->kbias + c0 * (std::fabs(ba[t].Bi) + std::fabs(ba[t].Bj)) + 2.0;
    if (kmx >= 1048576.0) {
      delete C;  // (nothing allocated on the device yet)
      return fail(ADMM_E_INVALID, "detector offset puts a bin position past 2^20 (kf_split)");
    }
  }
  // exact power-of-two scalings: 2^-wexp (N < 3: L = 2 / (N |cos|) can exceed 1) on ws and wc, and
  // 2^-32 on ws, whose float taps multiply frac(k_f) x 2^32 (kernels.hpp kf_split)
  for (int t = 0; t < g.n_angles; ++t) {
    bc[t].ws = float2v{std::ldexp(bc[t].ws.x, -C->wexp - 32), std::ldexp(bc[t].ws.y, -C->wexp - 32)};
    bc[t].wc = float2v{std::ldexp(bc[t].wc.x, -C->wexp), std::ldexp(bc[t].wc.y, -C->wexp)};
  }
  // angle groups for the grouped forward projector: consecutive angles of one case,
  // G <= kFgG, whose union row window of every block fits kFgWin (float64, same formulas as
  // the device; 2 pixels of margin).  Three plans, each a table of per-block ray ranges
  // (FgRange): plain 64-ray chunks; 64-ray chunks aligned per (row segment, angle) at the
  // detector centre (FgGroup.delta: narrower windows and larger groups, one more chunk per
  // segment); chunks aligned per (row segment, chunk) -- every angle's chunk x starts at the
  // same pixel of the segment's centre row, so windows stay narrow far from the detector
  // centre, where the rays' spacing 1/|cos| differs between the group's angles.
  // admm_batch_bind picks one (pick_fwd_plan).
  constexpr int kPlans = admm_ctx::kPlans;
  std::vector<FgGroup> groups_plan[kPlans];
  std::vector<FgRange> rng_plan[kPlans];
  std::vector<int4> blk_plan[kPlans];
  double staged_plan[kPlans] = {};
  bool fits = true;
  {
    const double cd = 0.5 * (g.n_det - 1);
    // touched row pixels of one block over its segment's rows, -1 if a row is too wide
    auto window_px = [&](int t0, int G, int mlo, int mhi, const FgRange& r) -> long {
      long px = 0;
      for (int m = mlo; m < mhi; ++m) {
        double lo = 1e300, hi = -1e300;
        for (int q = 0; q < G; ++q) {
          if (r.nk[q] == 0) continue;
          const FwdAngle& b = fa[t0 + q];
          for (int kk : {r.k0[q], r.k0[q] + r.nk[q] - 1}) {
            const double l = std::fma((double)m, b.dl, std::fma((double)kk, b.A1, b.A0));
            lo = std::min(lo, l);
            hi = std::max(hi, l);
          }
        }
        if (lo > hi) continue;
        const double w = std::floor(hi) - std::floor(lo) + 2;
        if (w > kFgWin - 2) return -1;
        px += (long)w;
      }
      return px;
    };
    // the blocks of group (t0, G) under plan pl: ray ranges rv, block entries bv
    // ({range index within rv, group index gi, segment, G}), staged pixels st
    auto plan_group = [&](int t0, int G, int pl, int gi, FgGroup& gr, std::vector<FgRange>& rv,
                          std::vector<int4>& bv, double& st) -> bool {
      for (int q = 0; q < G; ++q)
        if (fa[t0 + q].caseA != fa[t0].caseA) return false;
      const int scheme = pl % 3;
      const bool clipped = pl >= 3;
      gr = FgGroup{};
      gr.t0 = t0;
      gr.G = G;
      rv.clear();
      bv.clear();
      st = 0.0;
      for (int s = 0; s < kFgSeg; ++s) {
        const int mlo = s * g.N / kFgSeg, mhi = (s + 1) * g.N / kFgSeg;
        const double mc = 0.5 * (mlo + mhi - 1);
        // only rays that cross the segment's rows inside the image get lanes: a ray whose every
        // row position l lies outside [-2, N + 1] taps zero-filled columns only, so its partial
        // for this segment is exactly 0 and its slot keeps the zero it was filled with
        // (admm_batch_bind / op_forward_chunk zero the partials when the plan changes)
        const double dlo = std::min(mlo * 1.0, mhi - 1.0), dhi = std::max(mlo * 1.0, mhi - 1.0);
        auto clip = [&](FgRange& r) {
          for (int q = 0; q < G; ++q) {
            const FwdAngle& b = fa[t0 + q];
            const double e0 = std::min(dlo * b.dl, dhi * b.dl), e1 = std::max(dlo * b.dl, dhi * b.dl);
            const double ka = (-2.0 - b.A0 - e1) / b.A1, kb = (g.N + 1.0 - b.A0 - e0) / b.A1;
            const double klo = std::ceil(std::min(ka, kb)), khi = std::floor(std::max(ka, kb));
            const int lo = (int)std::max((double)r.k0[q], klo);
            const int hi = (int)std::min((double)(r.k0[q] + r.nk[q]), khi + 1.0);
            r.nk[q] = std::max(0, hi - lo);
            r.k0[q] = std::min(std::max(lo, 0), g.n_det - 1);
          }
        };
        auto emit = [&](FgRange r) -> bool {
          if (clipped) clip(r);
          bool any = false;
          for (int q = 0; q < G; ++q) any = any || r.nk[q] > 0;
          if (!any) return true;
          const long px = window_px(t0, G, mlo, mhi, r);
          if (px < 0) return false;
          st += (double)px;
          bv.push_back(make_int4((int)rv.size(), gi, s, G));
          rv.push_back(r);
          return true;
        };
        if (scheme < 2) {
          const FwdAngle& r0 = fa[t0];
          const double lref = r0.A0 + cd * r0.A1 + mc * r0.dl;  // reference ray at the centre row
          int delta[kFgG] = {};  // per-angle ray offset of the 64-ray chunks (scheme 1)
          int dmin = 0, dmax = 0;
          for (int q = 0; q < G; ++q) {
            const FwdAngle& b = fa[t0 + q];
            const int d = scheme == 1 ? (int)std::lround((lref - b.A0 - cd * b.A1 - mc * b.dl) / b.A1) : 0;
            delta[q] = d;
            dmin = std::min(dmin, d);
            dmax = std::max(dmax, d);
          }
          const int kcb = (int)std::floor(-dmax / 64.0);
          const int kce = (int)std::ceil((g.n_det - dmin) / 64.0);
          for (int kc = kcb; kc < kce; ++kc) {
            FgRange r{};
            for (int q = 0; q < G; ++q) {
              const int lo = std::max(kc * 64 + delta[q], 0);
              const int hi = std::min(kc * 64 + delta[q] + 64, g.n_det);
              r.k0[q] = lo;
              r.nk[q] = std::max(0, hi - lo);
            }
            if (!emit(r)) return false;
          }
        } else {
          // position of ray k at the centre row, along the direction of increasing k:
          // u_q(k) = sgn (A0 + mc dl) + k |A1|; chunk x holds the rays with u in
          // [U0 + x S, U0 + (x + 1) S), S = 64 min|A1| (<= 64 rays of every angle)
          const double sgn = fa[t0].A1 > 0 ? 1.0 : -1.0;
          double amin = 1e300, U0 = 1e300;
          double cq[kFgG], aq[kFgG];
          for (int q = 0; q < G; ++q) {
            const FwdAngle& b = fa[t0 + q];
            if ((b.A1 > 0) != (sgn > 0)) return false;
            aq[q] = std::fabs(b.A1);
            cq[q] = sgn * (b.A0 + mc * b.dl);
            amin = std::min(amin, aq[q]);
            U0 = std::min(U0, cq[q]);
          }
          const double S = 64.0 * amin * (1.0 - 1e-9);
          auto bnd = [&](int q, long x) {
            const double v = std::ceil((U0 + (double)x * S - cq[q]) / aq[q]);
            return (int)std::min(std::max(v, 0.0), (double)g.n_det);
          };
          for (long x = 0;; ++x) {
            if (x > 4L * g.n_det + 8) return false;  // (cannot happen: every chunk spans >= 64 pixels)
            FgRange r{};
            bool done = true;
            for (int q = 0; q < G; ++q) {
              const int lo = bnd(q, x), hi = bnd(q, x + 1);
              done = done && lo >= g.n_det;
              r.k0[q] = std::min(lo, g.n_det - 1);
              r.nk[q] = hi - lo;
              if (r.nk[q] > 64) return false;
            }
            if (done) break;
            if (!emit(r)) return false;
          }
        }
      }
      return true;
    };
    // greedy: the largest G <= kFgG consecutive same-case angles whose windows fit.
    // (Balanced splits of each same-case run were measured slower: they force wide windows
    // near 45 degrees, where greedy makes small narrow groups and stages fewer pixels.)
    for (int pl = 0; pl < kPlans && fits; ++pl) {
      for (int t0 = 0; t0 < g.n_angles;) {
        int G = std::min(kFgG, g.n_angles - t0);
        const int gi = (int)groups_plan[pl].size();
        FgGroup gr{};
        std::vector<FgRange> rv;
        std::vector<int4> bv;
        double st = 0.0;
        while (G > 1 && !plan_group(t0, G, pl, gi, gr, rv, bv, st)) --G;
        if (G == 1 && !plan_group(t0, 1, pl, gi, gr, rv, bv, st)) {
          if (pl < 2) fits = false;  // no grouped kernel for this geometry
          groups_plan[pl].clear();   // (plans 2-5 are optional)
          break;
        }
        const int base = (int)rng_plan[pl].size();
        for (int4 b : bv) blk_plan[pl].push_back(make_int4(b.x + base, b.y, b.z, b.w));
        rng_plan[pl].insert(rng_plan[pl].end(), rv.begin(), rv.end());
        groups_plan[pl].push_back(gr);
        staged_plan[pl] += st;
        t0 += G;
      }
    }
  }
  hipError_t e1 = hipMalloc(&C->fang, fa.size() * sizeof(FwdAngle));
  hipError_t e2 = hipMalloc(&C->bang, ba.size() * sizeof(BackAngle));
  if (e1 != hipSuccess || e2 != hipSuccess) {
    delete C;
    return fail(ADMM_E_HIP, "hipMalloc geometry tables");
  }
  HIPCHK(hipMemcpy(C->fang, fa.data(), fa.size() * sizeof(FwdAngle), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(C->bang, ba.data(), ba.size() * sizeof(BackAngle), hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&C->bangc, bc.size() * sizeof(BackAngleC)));
  HIPCHK(hipMemcpy(C->bangc, bc.data(), bc.size() * sizeof(BackAngleC), hipMemcpyHostToDevice));
  if (fits) {
    for (int pl = 0; pl < kPlans; ++pl) {
      const auto& gv = groups_plan[pl];
      const auto& rv = rng_plan[pl];
      if (gv.empty()) continue;
      HIPCHK(hipMalloc(&C->plan_groups[pl], gv.size() * sizeof(FgGroup)));
      HIPCHK(hipMemcpy(C->plan_groups[pl], gv.data(), gv.size() * sizeof(FgGroup), hipMemcpyHostToDevice));
      HIPCHK(hipMalloc(&C->plan_rng[pl], rv.size() * sizeof(FgRange)));
      HIPCHK(hipMemcpy(C->plan_rng[pl], rv.data(), rv.size() * sizeof(FgRange), hipMemcpyHostToDevice));
      C->plan_blk[pl] = blk_plan[pl];
      C->plan_caseA[pl].clear();
      for (const FgGroup& gr : gv) C->plan_caseA[pl].push_back(fa[gr.t0].caseA != 0);
      C->plan_n[pl] = (int)gv.size();
      C->plan_blocks[pl] = (int)blk_plan[pl].size();
      C->plan_staged[pl] = staged_plan[pl];
    }
    select_fwd_plan(C, 0);  // until a batch is bound
  }
  HIPCHK(hipStreamCreateWithFlags(&C->cap, hipStreamNonBlocking));
  *out = C;
  return ADMM_OK;
}

int admm_ctx_create_matrix(admm_ctx** out, int N, int m, long long nnz, const long long* indptr,
                           const int* indices, const double* values, int dtype, int max_images, int device) {
  if (!out || !indptr || (nnz > 0 && (!indices || !values))) return fail(ADMM_E_INVALID, "null argument");
  *out = nullptr;
  if (N < 2 || N > 4096 || m < 1) return fail(ADMM_E_INVALID, "bad matrix sizes");
  if (dtype != ADMM_DTYPE_F32 && dtype != ADMM_DTYPE_F64) return fail(ADMM_E_INVALID, "bad dtype");
  if (max_images < 1) return fail(ADMM_E_INVALID, "max_images < 1");
  const size_t npix = (size_t)N * N;
  if (nnz < 0 || nnz >= (1ll << 31)) return fail(ADMM_E_INVALID, "nnz must be < 2^31");
  if ((size_t)max_images * npix * 8 >= (1ull << 31) || (size_t)max_images * m * 8 >= (1ull << 31))
    return fail(ADMM_E_INVALID, "batch too large for 32-bit buffer offsets; split it across contexts");
  if (indptr[0] != 0 || indptr[m] != nnz) return fail(ADMM_E_INVALID, "indptr must run from 0 to nnz");
  for (int r = 0; r < m; ++r)
    if (indptr[r + 1] < indptr[r]) return fail(ADMM_E_INVALID, "indptr not non-decreasing");
  for (long long k = 0; k < nnz; ++k)
    if (indices[k] < 0 || (size_t)indices[k] >= npix) return fail(ADMM_E_INVALID, "column index out of range");
  // A^T by a counting sort over columns; within a column the rows stay ascending
  std::vector<int> tptr(npix + 1, 0), tidx((size_t)nnz);
  std::vector<double> tval((size_t)nnz);
  for (long long k = 0; k < nnz; ++k) ++tptr[(size_t)indices[k] + 1];
  for (size_t c = 0; c < npix; ++c) tptr[c + 1] += tptr[c];
  {
    std::vector<int> fill(tptr.begin(), tptr.end() - 1);
    for (int r = 0; r < m; ++r)
      for (long long k = indptr[r]; k < indptr[r + 1]; ++k) {
        const int q = fill[indices[k]]++;
        tidx[q] = r;
        tval[q] = values[k];
      }
  }
  std::vector<int> fptr(m + 1);
  for (int r = 0; r <= m; ++r) fptr[r] = (int)indptr[r];
  DEVICE_SCOPE(device);
  admm_ctx* C = new admm_ctx();
  // a one-"angle" geometry (n_det = m, L = 1): every m-sized buffer, the fixed-order
  // reductions and the combine/residual kernels keep their shapes
  C->g = admm_geom{};
  C->g.N = N;
  C->g.n_angles = 1;
  C->g.n_det = m;
  C->dtype = dtype;
  C->device = device;
  C->max_images = max_images;
  C->npix = (int)npix;
  C->mrays = m;
  C->csr = true;
  C->nnz = nnz;
  FwdAngle fa{};
  fa.L = 1.0;
  BackAngle ba{};
  BackAngleC bc{};
  int rc = ADMM_OK;
  auto up = [&](Buf& b, const void* src, size_t bytes) {
    if (rc != ADMM_OK) return;
    rc = ensure(b, std::max<size_t>(bytes, 16));
    if (rc == ADMM_OK && bytes > 0 && hipMemcpy(b.p, src, bytes, hipMemcpyHostToDevice) != hipSuccess)
      rc = fail(ADMM_E_HIP, "hipMemcpy (matrix upload)");
  };
  auto upv = [&](Buf& b, const std::vector<double>& v) {
    if (dtype == ADMM_DTYPE_F64) return up(b, v.data(), v.size() * 8);
    std::vector<float> f(v.begin(), v.end());
    up(b, f.data(), f.size() * 4);
  };
  up(C->f_ptr, fptr.data(), fptr.size() * 4);
  up(C->f_idx, indices, (size_t)nnz * 4);
  upv(C->f_val, std::vector<double>(values, values + nnz));
  up(C->t_ptr, tptr.data(), tptr.size() * 4);
  up(C->t_idx, tidx.data(), tidx.size() * 4);
  upv(C->t_val, tval);
  if (rc == ADMM_OK && (hipMalloc(&C->fang, sizeof(FwdAngle)) != hipSuccess ||
                        hipMalloc(&C->bang, sizeof(BackAngle)) != hipSuccess ||
                        hipMalloc(&C->bangc, sizeof(BackAngleC)) != hipSuccess))
    rc = fail(ADMM_E_HIP, "hipMalloc tables");
  if (rc == ADMM_OK && (hipMemcpy(C->fang, &fa, sizeof(fa), hipMemcpyHostToDevice) != hipSuccess ||
                        hipMemcpy(C->bang, &ba, sizeof(ba), hipMemcpyHostToDevice) != hipSuccess ||
                        hipMemcpy(C->bangc, &bc, sizeof(bc), hipMemcpyHostToDevice) != hipSuccess))
    rc = fail(ADMM_E_HIP, "hipMemcpy tables");
  if (rc == ADMM_OK && hipStreamCreateWithFlags(&C->cap, hipStreamNonBlocking) != hipSuccess)
    rc = fail(ADMM_E_HIP, "hipStreamCreate");
  if (rc != ADMM_OK) {
    const std::string msg = g_err;
    admm_ctx_destroy(C);
    return fail(rc, msg);
  }
  *out = C;
  return ADMM_OK;
}

int admm_ctx_destroy(admm_ctx* C) {
  if (!C) return ADMM_OK;
  DeviceGuard _dg(C->device);
  (void)hipDeviceSynchronize();
  free_graphs(C);
  if (C->half) (void)admm_ctx_destroy(C->half);
  C->half = nullptr;
  Buf* bufs[] = {&C->op_img, &C->op_imgT, &C->op_sino, &C->op_fpart, &C->xs, &C->xsT, &C->p, &C->pT, &C->Hp, &C->sino, &C->bI, &C->fpart, &C->r, &C->c,
                 &C->d2, &C->e2, &C->partH, &C->partS, &C->partD, &C->partE, &C->redH, &C->fg_order, &C->dsumS, &C->ats,
                 &C->f_ptr, &C->f_idx, &C->f_val, &C->t_ptr, &C->t_idx, &C->t_val, &C->x2, &C->p2, &C->pring};
  for (Buf* b : bufs)
    if (b->p) (void)hipFree(b->p);
  for (Buf& b : C->op_order)
    if (b.p) (void)hipFree(b.p);
  if (C->fang) (void)hipFree(C->fang);
  if (C->bang) (void)hipFree(C->bang);
  if (C->bangc) (void)hipFree(C->bangc);
  for (FgGroup* pg : C->plan_groups)
    if (pg) (void)hipFree(pg);
  for (FgRange* pr : C->plan_rng)
    if (pr) (void)hipFree(pr);
  if (C->cap) (void)hipStreamDestroy(C->cap);
  delete C;
  return ADMM_OK;
}

int admm_project_fwd(admm_ctx* C, const void* img, void* sino, int nimg, void* stream) {
  if (!C || !img || !sino) return fail(ADMM_E_INVALID, "null argument");
  if (nimg < 1 || nimg > C->max_images) return fail(ADMM_E_INVALID, "nimg out of range");
  hipStream_t s = (hipStream_t)stream;
  DEVICE_SCOPE(C->device);
  return C->dtype == ADMM_DTYPE_F32 ? op_forward<float>(C, (const float*)img, (float*)sino, nimg, s)
                                    : op_forward<double>(C, (const double*)img, (double*)sino, nimg, s);
}

int admm_project_adj(admm_ctx* C, const void* sino, void* img, int nimg, void* stream) {
  if (!C || !img || !sino) return fail(ADMM_E_INVALID, "null argument");
  if (nimg < 1 || nimg > C->max_images) return fail(ADMM_E_INVALID, "nimg out of range");
  DEVICE_SCOPE(C->device);
  hipStream_t s = (hipStream_t)stream;
  if (C->dtype == ADMM_DTYPE_F32) {
    BackArgs<float> a{};
    a.sino = (const float*)sino;
    a.out_t = (float*)img;
    return launch_back<float, 1, BACK_PLAIN>(C, a, nimg, s);
  }
  BackArgs<double> a{};
  a.sino = (const double*)sino;
  a.out_t = (double*)img;
  return launch_back<double, 1, BACK_PLAIN>(C, a, nimg, s);
}

int admm_column_norms_sq(admm_ctx* C, double* W, void* stream) {
  if (!C || !W) return fail(ADMM_E_INVALID, "null argument");
  DEVICE_SCOPE(C->device);
  hipStream_t s = (hipStream_t)stream;
  if (C->dtype == ADMM_DTYPE_F32) {
    BackArgs<float> a{};
    a.out_d = W;
    return launch_back<float, 1, BACK_WSQ>(C, a, 1, s);
  }
  BackArgs<double> a{};
  a.out_d = W;
  return launch_back<double, 1, BACK_WSQ>(C, a, 1, s);
}

int admm_tv_grad(admm_ctx* C, const double* x, double* gx, double* gy, int nimg, void* stream) {
  if (!C || !x || !gx || !gy || nimg < 1) return fail(ADMM_E_INVALID, "bad argument");
  DEVICE_SCOPE(C->device);
  const int N = C->g.N;
  hipLaunchKernelGGL(k_tv_grad, dim3((N + 63) / 64, (N + 3) / 4, nimg), dim3(kBlock), 0, (hipStream_t)stream, x,
                     gx, gy, N);
  CHECK_LAUNCH();
  return ADMM_OK;
}

int admm_tv_div(admm_ctx* C, const double* px, const double* py, double* out, int nimg, void* stream) {
  if (!C || !px || !py || !out || nimg < 1) return fail(ADMM_E_INVALID, "bad argument");
  DEVICE_SCOPE(C->device);
  const int N = C->g.N;
  hipLaunchKernelGGL(k_tv_div, dim3((N + 63) / 64, (N + 3) / 4, nimg), dim3(kBlock), 0, (hipStream_t)stream, px,
                     py, out, N);
  CHECK_LAUNCH();
  return ADMM_OK;
}

int admm_batch_bind(admm_ctx* C, const admm_batch* batch) {
  if (!C || !batch) return fail(ADMM_E_INVALID, "null argument");
  const admm_batch& B = *batch;
  if (B.V < 1) return fail(ADMM_E_INVALID, "batch V < 1");
  if (B.n_xext < B.V) return fail(ADMM_E_INVALID, "n_xext < V");
  if (B.tv_iters < 1 || B.cg_iters < 1) return fail(ADMM_E_INVALID, "tv_iters and cg_iters must be >= 1");
  if (B.tv_kind != ADMM_TV_ISO && B.tv_kind != ADMM_TV_ANISO) return fail(ADMM_E_INVALID, "bad tv_kind");
  if (!(B.mu > 0)) return fail(ADMM_E_INVALID, "mu must be > 0");
  if (!B.x_ext || !B.d || !B.e || !B.atb || !B.dsum || !B.b || !B.inc_off || !B.node_stats)
    return fail(ADMM_E_INVALID, "null batch pointer");
  if (B.n_edges > 0 && (!B.y || !B.q || !B.edge_a || !B.edge_b || !B.inc_edge || !B.inc_qslot ||
                        !B.inc_sign || !B.edge_stats))
    return fail(ADMM_E_INVALID, "null edge pointer");
  if (B.n_edges > 0 && !B.z) {
    if (!B.x_prev) return fail(ADMM_E_INVALID, "z == NULL needs x_prev (derived consensus)");
    if (B.fusion != ADMM_FUSE_MIDPOINT) return fail(ADMM_E_INVALID, "derived z needs midpoint fusion");
  }
  if (B.fusion != ADMM_FUSE_MIDPOINT && B.fusion != ADMM_FUSE_WEIGHTED) return fail(ADMM_E_INVALID, "bad fusion");
  if (B.flags & ~ADMM_BATCH_KEEP_X) return fail(ADMM_E_INVALID, "unknown batch flags");
  if (B.fusion == ADMM_FUSE_WEIGHTED && B.n_edges > 0 && (!B.y_b || !B.w))
    return fail(ADMM_E_INVALID, "weighted fusion needs y_b and w");
  if (B.n_edges > 65535) return fail(ADMM_E_INVALID, "more than 65535 edge slots on one device");
  const size_t npix = C->npix, m = C->mrays;
  if ((size_t)B.V * npix * 8 >= (1ull << 31) || (size_t)B.V * m * 8 >= (1ull << 31))
    return fail(ADMM_E_INVALID, "batch too large for 32-bit buffer offsets");
  DEVICE_SCOPE(C->device);
  HIPCHK(hipDeviceSynchronize());
  RET(free_graphs(C));
  C->b = B;
  const int V = B.V;
  C->vb = vb_for(V, C->dtype);
  RET(bind_fwd_plan(C, V));
  const size_t Vp = (size_t)((V + C->vb - 1) / C->vb) * C->vb;  // padded to whole chunks
  const size_t ds = dsize(C->dtype);
  RET(ensure(C->xs, Vp * npix * ds));
  RET(ensure(C->xsT, Vp * npix * ds));
  RET(ensure(C->p, Vp * npix * ds));
  RET(ensure(C->pT, Vp * npix * ds));
  RET(ensure(C->Hp, Vp * npix * ds));
  RET(ensure(C->dsumS, Vp * npix * ds));
  RET(ensure(C->x2, (size_t)V * npix * 8));
  RET(ensure(C->p2, Vp * npix * ds));
  if (B.cg_iters > 1 && B.cg_iters <= kMaxCgRing)
    RET(ensure(C->pring, (size_t)(B.cg_iters - 1) * Vp * npix * ds));
  if (B.flags & ADMM_BATCH_KEEP_X) RET(ensure(C->ats, Vp * npix * ds));
  C->ats_valid = false;
  RET(ensure(C->sino, Vp * m * ds));
  RET(ensure(C->bI, Vp * m * ds));
  RET(ensure(C->r, V * npix * 8));
  RET(ensure(C->c, V * npix * 8));
  RET(ensure(C->d2, 2 * V * npix * 8));
  RET(ensure(C->e2, 2 * V * npix * 8));
  C->P_back = back_partitions(C);
  const int N = C->g.N;
  C->P_tile = ((N + kTile - 1) / kTile) * ((N + kTile - 1) / kTile);
  if ((size_t)Vp * npix * ds >= (1ull << 31) || (size_t)Vp * m * ds >= (1ull << 31))
    return fail(ADMM_E_INVALID, "batch too large for 32-bit buffer offsets");
  C->P_fwd = C->mm ? (int)((C->half->mrays + kBlock - 1) / kBlock)
           : (C->n_groups > 0 || C->csr) ? (int)((m + kBlock - 1) / kBlock)
                                         : ((C->g.n_det + kFwdRays - 1) / kFwdRays) * C->g.n_angles;
  // partials per (edge, 1024 pixels) for the stored-z kernels, per (edge, 64-pixel block) for the
  // derived-z ones
  C->P_edge = B.z ? (int)((npix + kBlock * 4 - 1) / (kBlock * 4)) : (int)((npix + kConsPix - 1) / kConsPix);
  RET(ensure(C->partH, (size_t)5 * V * C->P_back * 8));
  RET(ensure(C->partS, (size_t)V * C->P_fwd * 8));
  RET(ensure(C->partD, (size_t)5 * V * C->P_back * 8));
  RET(ensure(C->partE, (size_t)3 * std::max(1, B.n_edges) * C->P_edge * 8));
  RET(ensure(C->redH, (size_t)5 * V * 8 * std::max(1, std::min(B.cg_iters, kMaxCgRing))));
  C->bound = true;
  // D = sum_j q_ij as interleaved samples of the sample dtype (the BACK_H epilogue's rho D p
  // term): setup data, packed once here rather than in every x-update
  RET(with_vb(C->vb, [&](auto vbc) {
    constexpr int VB = decltype(vbc)::value;
    const int nch = (V + VB - 1) / VB;
    if (C->dtype == ADMM_DTYPE_F32)
      hipLaunchKernelGGL((k_pack_d<float, VB>), dim3((unsigned)((npix + 255) / 256), nch), dim3(256), 0, C->cap,
                         B.dsum, (float*)C->dsumS.p, (int)npix, V);
    else
      hipLaunchKernelGGL((k_pack_d<double, VB>), dim3((unsigned)((npix + 255) / 256), nch), dim3(256), 0, C->cap,
                         B.dsum, (double*)C->dsumS.p, (int)npix, V);
    CHECK_LAUNCH();
    return ADMM_OK;
  }));
  HIPCHK(hipStreamSynchronize(C->cap));
  // the x-update and consensus sequences, recorded once and replayed every iteration
  auto fu = [&](hipStream_t s) {
    return C->dtype == ADMM_DTYPE_F32 ? enqueue_update_any<float>(C, s) : enqueue_update_any<double>(C, s);
  };
  RET(capture(C, fu, &C->g_update, &C->x_update));
  if (B.flags & ADMM_BATCH_KEEP_X) {
    auto fr = [&](hipStream_t s) {
      return C->dtype == ADMM_DTYPE_F32 ? enqueue_update_any<float>(C, s, true)
                                        : enqueue_update_any<double>(C, s, true);
    };
    RET(capture(C, fr, &C->g_update_reuse, &C->x_update_reuse));
  }
  if (B.n_edges > 0) {
    auto fc = [&](hipStream_t s) { return enqueue_consensus(C, s); };
    RET(capture(C, fc, &C->g_cons, &C->x_cons));
  }
  HIPCHK(hipDeviceSynchronize());
  return ADMM_OK;
}

extern "C++" {
template <typename T>
int batch_atb(admm_ctx* C, double* atb_out, hipStream_t s) {
  const int V = C->b.V;
  return with_vb(C->vb, [&](auto vbc) {
    constexpr int VB = decltype(vbc)::value;
    const int nch = (V + VB - 1) / VB;
    hipLaunchKernelGGL((k_pack<T, VB>), dim3((C->mrays + 255) / 256, nch), dim3(256), 0, s, (const T*)C->b.b,
                       (T*)C->bI.p, C->mrays, V);
    CHECK_LAUNCH();
    BackArgs<T> a{};
    a.sino = (const T*)C->bI.p;
    a.out_d = atb_out;
    return launch_back<T, VB, BACK_ATB>(C, a, V, s);
  });
}
}  // extern "C++"

int admm_batch_atb(admm_ctx* C, double* atb_out, void* stream) {
  if (!C || !C->bound) return fail(ADMM_E_STATE, "no batch bound");
  if (!atb_out) return fail(ADMM_E_INVALID, "null atb_out");
  DEVICE_SCOPE(C->device);
  hipStream_t s = (hipStream_t)stream;
  return C->dtype == ADMM_DTYPE_F32 ? batch_atb<float>(C, atb_out, s) : batch_atb<double>(C, atb_out, s);
}

int admm_node_update(admm_ctx* C, void* stream) {
  if (!C || !C->bound) return fail(ADMM_E_STATE, "no batch bound");
  DEVICE_SCOPE(C->device);
  hipStream_t s = (hipStream_t)stream;
  const bool keep = (C->b.flags & ADMM_BATCH_KEEP_X) != 0;
  const bool reuse = keep && C->ats_valid;
  int rc = ADMM_OK;
  if (C->x_update) {
    HIPCHK(hipGraphLaunch(reuse ? C->x_update_reuse : C->x_update, s));
  } else {
    rc = C->dtype == ADMM_DTYPE_F32 ? enqueue_update_any<float>(C, s, reuse)
                                    : enqueue_update_any<double>(C, s, reuse);
  }
  if (rc == ADMM_OK && keep) C->ats_valid = true;  // this update's DIAG left A^T s of its x
  return rc;
}

int admm_node_update_rounds(admm_ctx* C, int tv_iters, void* stream) {
  if (!C || !C->bound) return fail(ADMM_E_STATE, "no batch bound");
  if (tv_iters < 1) return fail(ADMM_E_INVALID, "tv_iters must be >= 1");
  if (tv_iters == C->b.tv_iters) return admm_node_update(C, stream);
  DEVICE_SCOPE(C->device);
  hipStream_t s = (hipStream_t)stream;
  const bool keep = (C->b.flags & ADMM_BATCH_KEEP_X) != 0;
  const bool reuse = keep && C->ats_valid;
  // a round count other than the bound one: enqueued directly (no recorded graph)
  const int rc = C->dtype == ADMM_DTYPE_F32 ? enqueue_update_any<float>(C, s, reuse, tv_iters)
                                            : enqueue_update_any<double>(C, s, reuse, tv_iters);
  if (rc == ADMM_OK && keep) C->ats_valid = true;
  return rc;
}

int admm_consensus(admm_ctx* C, void* stream) {
  if (!C || !C->bound) return fail(ADMM_E_STATE, "no batch bound");
  DEVICE_SCOPE(C->device);
  hipStream_t s = (hipStream_t)stream;
  if (C->x_cons) {
    HIPCHK(hipGraphLaunch(C->x_cons, s));
    return ADMM_OK;
  }
  return enqueue_consensus(C, s);
}

extern "C++" {
// One x-update enqueued directly (the graph's launch sequence, no graph) with timing-only
// events around every in-solve launch of `kind` (0: the forward tap kernel of each CG step,
// right after the CG / TV update that wrote p and p^T; 1: the back projector of each CG step,
// right after its forward combine), exactly as in every replay; ms = their average duration.
template <typename T>
int time_in_solve(admm_ctx* C, int kind, hipStream_t s, float* ms) {
  return with_vb(C->vb, [&](auto vbc) -> int {
    constexpr int VB = decltype(vbc)::value;
    const int n = C->b.tv_iters * C->b.cg_iters;
    std::vector<hipEvent_t> ev(2 * n);
    // no system-scope fence (cache writeback / invalidation) at each record, which would
    // perturb the launches they bracket
    for (auto& e : ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    C->tf_ev = &ev;
    C->tf_next = 0;
    C->tf_kind = kind;
    const bool keep = (C->b.flags & ADMM_BATCH_KEEP_X) != 0;
    int rc = enqueue_update<T, VB>(C, s, keep && C->ats_valid);
    const size_t used = C->tf_next;
    C->tf_ev = nullptr;
    C->tf_kind = 0;
    if (rc == ADMM_OK && keep) C->ats_valid = true;
    if (rc == ADMM_OK && used == 0) rc = fail(ADMM_E_STATE, "no launch was timed");
    if (rc == ADMM_OK) {
      HIPCHK(hipEventSynchronize(ev[used - 1]));
      float tot = 0.f;
      for (size_t i = 0; i < used; i += 2) {
        float t = 0.f;
        HIPCHK(hipEventElapsedTime(&t, ev[i], ev[i + 1]));
        tot += t;
      }
      *ms = tot / (float)(used / 2);
    }
    for (auto& e : ev) (void)hipEventDestroy(e);
    return rc;
  });
}

template <typename T>
int time_fwd(admm_ctx* C, int reps, int in_solve, hipStream_t s, float* ms) {
  if (in_solve) return time_in_solve<T>(C, 0, s, ms);
  return with_vb(C->vb, [&](auto vbc) -> int {
    constexpr int VB = decltype(vbc)::value;
    // the forward tap kernel alone, back to back: k_fwdg (every sample tap) when grouped, else k_fwd
    auto one = [&]() -> int {
      if (C->n_groups > 0) return launch_fwdg_taps<T, VB>(C, (T*)C->xs.p, (T*)C->xsT.p, C->b.V, s);
      return launch_fwd<T, VB, 0>(C, (T*)C->xs.p, (T*)C->xsT.p, (T*)C->sino.p, nullptr, nullptr, C->b.V, s);
    };
    RET(one());
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreateWithFlags(&e0, hipEventDisableSystemFence));
    HIPCHK(hipEventCreateWithFlags(&e1, hipEventDisableSystemFence));
    HIPCHK(hipEventRecord(e0, s));
    int rc = ADMM_OK;
    for (int i = 0; i < reps && rc == ADMM_OK; ++i) rc = one();
    HIPCHK(hipEventRecord(e1, s));
    HIPCHK(hipEventSynchronize(e1));
    HIPCHK(hipEventElapsedTime(ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return rc;
  });
}
}  // extern "C++"

int admm_time_forward(admm_ctx* C, int reps, int in_solve, void* stream, double* ms_out) {
  if (!C || !C->bound) return fail(ADMM_E_STATE, "no batch bound");
  if (reps < 1 || !ms_out) return fail(ADMM_E_INVALID, "bad argument");
  DEVICE_SCOPE(C->device);
  hipStream_t s = (hipStream_t)stream;
  float ms = 0.f;
  RET(C->dtype == ADMM_DTYPE_F32 ? time_fwd<float>(C, reps, in_solve, s, &ms)
                                  : time_fwd<double>(C, reps, in_solve, s, &ms));
  *ms_out = in_solve ? (double)ms : (double)ms / reps;
  return ADMM_OK;
}

int admm_consensus_range(admm_ctx* C, int e0, int e1, int rows, void* stream) {
  if (!C || !C->bound) return fail(ADMM_E_STATE, "no batch bound");
  const admm_batch& B = C->b;
  if (B.z == nullptr || B.fusion != ADMM_FUSE_MIDPOINT)
    return fail(ADMM_E_STATE, "admm_consensus_range needs stored z and midpoint fusion");
  if (e0 < 0 || e1 < e0 || e1 > B.n_edges) return fail(ADMM_E_INVALID, "edge range out of bounds");
  if (rows < 1 || rows > B.n_xext) return fail(ADMM_E_INVALID, "rows out of range");
  DEVICE_SCOPE(C->device);
  return enqueue_consensus_stored(C, e0, e1, (hipStream_t)stream);
}

int admm_time_back(admm_ctx* C, void* stream, double* ms_out) {
  if (!C || !C->bound) return fail(ADMM_E_STATE, "no batch bound");
  if (!ms_out) return fail(ADMM_E_INVALID, "bad argument");
  DEVICE_SCOPE(C->device);
  hipStream_t s = (hipStream_t)stream;
  float ms = 0.f;
  RET(C->dtype == ADMM_DTYPE_F32 ? time_in_solve<float>(C, 1, s, &ms) : time_in_solve<double>(C, 1, s, &ms));
  *ms_out = (double)ms;
  return ADMM_OK;
}

int admm_batch_info(admm_ctx* C, int* vb, int* mirror) {
  if (!C || !vb || !mirror) return fail(ADMM_E_INVALID, "bad argument");
  if (!C->bound) return fail(ADMM_E_STATE, "no batch bound");
  *vb = C->vb;
  *mirror = C->mm ? 1 : 0;
  return ADMM_OK;
}

int admm_fwd_plan_info(admm_ctx* C, int plan, int* groups, int* blocks, double* staged, int* active) {
  if (!C || plan < 0 || plan >= admm_ctx::kPlans || !groups || !blocks || !staged || !active)
    return fail(ADMM_E_INVALID, "bad argument");
  if (C->mm && C->half) C = C->half;  // mirror mode: the half geometry's plans are the bound ones
  *groups = C->plan_n[plan];
  *blocks = C->plan_blocks[plan];
  *staged = C->plan_staged[plan];
  *active = (C->plan_n[plan] > 0 && C->groups == C->plan_groups[plan]) ? 1 : 0;
  return ADMM_OK;
}

}  // extern "C"
