// qldpc_hip.hip — host runtime + C ABI (include/qldpc_hip.h) of the MI355X engine.
//
// Graph/decoder/MC handles own their device buffers; launches take a caller
// stream.  Three kernel engines are built:
//   engine 3 (default) — bp_reg.h: engine 2's LDS image with each thread's
//                        variables (edge addresses, priors, own messages)
//                        resident in VGPRs, compile-time VPL <= 8, column
//                        degree <= 4 and an image addressable with 16 bits;
//   engine 2           — bp_slot.h: small workgroups with streamed variables,
//                        row-major v2c slots, check-centric gather, NS decodes
//                        in flight per workgroup (any graph that fits LDS);
//   engine 1           — bp_kernels.h: per-check LDS state updated by
//                        returning LDS atomics (kept for A/B measurements,
//                        selected with QLDPC_ENGINE=1).
// Variants (fp32/fp64 × variables per thread × max column degree × slots) are
// selected per graph at create time.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/qldpc_hip.h"
#include "variants.h"
#include "runtime.h"

using namespace qldpc;
using namespace qldpc_rt;

thread_local std::string qldpc_rt::g_err;

namespace {

const int kVplSet[] = {1, 2, 3, 4, 5, 6, 7, 8, 10, 12};
constexpr int kLdsMax = 160 * 1024;
constexpr int kChunkMax = 1024;

int env_int(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return (e && *e) ? std::atoi(e) : dflt;
}

}  // namespace

// --------------------------------------------------------------- dispatch
namespace {

Variant get_variant(int precision, int vpl, int dmax) {
  if (precision == 32) return dmax == 4 ? get_variant_f32_d4(vpl) : get_variant_f32_d8(vpl);
  return dmax == 4 ? get_variant_f64_d4(vpl) : get_variant_f64_d8(vpl);
}

SVariant get_svariant(int precision, int dmax, int ns) {
  if (precision == 32) return dmax == 4 ? get_svariant_f32_d4(ns) : get_svariant_f32_d8(ns);
  return dmax == 4 ? get_svariant_f64_d4(ns) : get_svariant_f64_d8(ns);
}

SVariant get_rvariant(int engine, int precision, int vpl, int d3k, int dmax) {
  if (engine == 4) return precision == 32 ? get_r4variant_f32(vpl) : get_r4variant_f64(vpl);
  if (precision == 32 && dmax == 5) return get_rvariant_f32_d5(vpl, d3k);
  if (precision == 32 && dmax == 6) return get_rvariant_f32_d6(vpl, d3k);
  return precision == 32 ? get_rvariant_f32(vpl, d3k) : get_rvariant_f64(vpl);
}

// fp64 engine-3 kernels built for <= 256-thread workgroups (engine id 103:
// 256-VGPR budget, own v2c in VGPRs, compile-time D3K); QLDPC_F64W=0 disables.
bool use_f64w(int engine, int precision, int dmax, int tb, int vpl, int ea_shift, int nch) {
  // column degree 5 (kern_r_f64_d5.hip): VPL 4-5 only
  // (column degree 5 also with rows of 9-10 = 5 chunks: the lifted-product [h | I] graphs, round 6)
  return engine == 3 && precision == 64 && (dmax == 4 || (dmax == 5 && (vpl <= 5 || (vpl == 6 && nch == 5)))) &&
         ea_shift == 0 && tb <= 256 && vpl >= 4 && vpl <= 8 && (nch == 3 || nch == 4 || (dmax == 5 && nch == 5)) &&
         env_int("QLDPC_F64W", 1) != 0;
}

// fp32 engine-3 kernels with the compile-time 2-chunk check phase (rows of <= 8 edges);
// QLDPC_F32W=0 falls back to the runtime-width check loop.
bool use_f32w(int engine, int precision, int dmax, int tb, int vpl, int ea_shift, int nch) {
  (void)tb;
  return engine == 3 && precision == 32 && dmax == 4 && ea_shift == 0 && vpl >= 5 && vpl <= 8 && nch == 2 &&
         env_int("QLDPC_F32W", 1) != 0;
}

#if QLDPC_STAMPS
// diagnostic build: phase-cycle sums of the fused MC kernels (bp_reg.h, QLDPC_STAMPS)
unsigned long long* debug_stamps_buffer() {
  static unsigned long long* buf = nullptr;
  if (!buf && hipMalloc(&buf, 10 * sizeof(unsigned long long)) == hipSuccess) (void)hipMemset(buf, 0, 80);
  return buf;
}
#endif

// fp64 engine-3 kernels for 257-512-thread workgroups (engine id 303, VPL 3-4); opt-in QLDPC_F64X=1
bool use_f64x(int engine, int precision, int dmax, int tb, int vpl, int ea_shift) {
  return engine == 3 && precision == 64 && dmax == 4 && ea_shift == 0 && tb > 256 && tb <= 512 && vpl >= 3 &&
         vpl <= 4 && QLDPC_EXPERIMENTAL && env_int("QLDPC_F64X", 0) != 0;
}

// Slot-family kernels of an engine (2, 3 or 4).
SVariant slot_variant(int engine, int precision, int dmax, int ns, int vpl, int d3k, int ea_shift = 0, int tb = 1024,
                      int nch = 0, int tail = 0, int m2s = 0, int fb = 0, int d2k = 0, int pk = 0) {
  // fp32 space-time family with byte F words (rows of 2 chunks + a tail slot, 512 threads, 2 per CU)
  if (fb) {
    const bool ok = engine == 3 && precision == 32 && dmax == 4 && ea_shift == 2 && nch == 2 && tail && tb == 512;
    return ok ? get_rvariant_f32_stfb(vpl, d3k, d2k) : SVariant{nullptr, nullptr, nullptr, nullptr};
  }
  // fp64 m2-in-slot family (rows of 3 chunks + a tail slot, <= 256 threads, 3 workgroups per CU)
  if (m2s) {
    // the fp64 space-time graphs: rows of 4 chunks + a tail slot, dword-scaled addresses, 1024
    // threads (engine id 111313, round 6)
    if (m2s == 1 && engine == 3 && precision == 64 && dmax == 4 && ea_shift == 2 && nch == 4 && tail && tb >= 512)
      return get_rvariant_f64_m2st(vpl, d3k, d2k);
    // rows of 8 (4 chunks, no tail array), column degree 5, 256 threads (128 / 192 for small graphs): engine id 10103
    if (m2s == 1 && engine == 3 && precision == 64 && dmax == 5 && ea_shift == 0 && nch == 4 && !tail && tb <= 256)
      return pk ? get_rvariant_f64_m2s8pk(vpl, d3k) : get_rvariant_f64_m2s8(vpl, d3k);
    const bool ok = engine == 3 && precision == 64 && dmax == 4 && ea_shift == 0 && nch == 3 && tail && tb <= 256;
    if (m2s == 3)  // variable-major V slots: no tail array, 256 threads
      return (engine == 3 && precision == 64 && dmax == 4 && ea_shift == 0 && tb == 256) ? get_rvariant_f64_m2v(vpl, d3k)
                                                                                          : SVariant{nullptr, nullptr, nullptr, nullptr};
    if (!ok) return SVariant{nullptr, nullptr, nullptr, nullptr};
    return m2s == 2 ? get_rvariant_f64_c2s(vpl, d3k) : get_rvariant_f64_m2s(vpl, d3k);
  }
  // fp64 tail layout (rows of 4 chunks + a tail slot, dword-scaled addresses, 1024 threads)
  if (tail) {
    const bool ok = engine == 3 && dmax == 4 && ea_shift == 2 && nch == (precision == 64 ? 4 : 2) &&
                    (tb > 512 || (precision == 64 && tb == 512));
    if (!ok) return SVariant{nullptr, nullptr, nullptr, nullptr};
    return precision == 64 ? get_rvariant_f64_st(vpl, d3k, d2k) : get_rvariant_f32_st(vpl, d3k);
  }
  if (use_f64w(engine, precision, dmax, tb, vpl, ea_shift, nch))
    return dmax == 5 ? get_rvariant_f64_w_d5(vpl, d3k, nch) : get_rvariant_f64_w(vpl, d3k, nch);
  if (use_f64x(engine, precision, dmax, tb, vpl, ea_shift)) return get_rvariant_f64_x(vpl, d3k);
  if (use_f32w(engine, precision, dmax, tb, vpl, ea_shift, nch)) return get_rvariant_f32_w(vpl, d3k);
  if (engine == 4 && precision == 64 && tb <= 256 && vpl >= 4) return get_r4variant_f64_w(vpl);
  if (engine == 3 && ea_shift == 2)
    return (precision == 32 && dmax == 4) ? get_rvariant_f32_big(vpl, d3k) : SVariant{nullptr, nullptr, nullptr, nullptr};
  return engine >= 3 ? get_rvariant(engine, precision, vpl, d3k, dmax) : get_svariant(precision, dmax, ns);
}

int round_up(int x, int a) { return (x + a - 1) / a * a; }

// ---- engine 1 geometry: threads per shot TB (multiple of 64, <= 512)
// Largest vars-per-thread whose kernels compile without register spills (gfx950,
// -Rpass-analysis=kernel-resource-usage).
int max_spill_free_vpl(int precision, int dmax) {
  if (precision == 32) return dmax == 4 ? 10 : 5;
  return dmax == 4 ? 6 : 3;
}

int choose_geometry(int n, int m, int requested_vpl, int vmax, int& TB, int& VPL) {
  if (requested_vpl > 0) {
    bool ok = false;
    for (int v : kVplSet) ok |= (v == requested_vpl);
    if (!ok) return set_err(QLDPC_EINVAL, "vars_per_thread must be one of 1-8,10,12");
    VPL = requested_vpl;
    TB = round_up((n + VPL - 1) / VPL, 64);
    if (TB > kMaxThreads) return set_err(QLDPC_EINVAL, "vars_per_thread too small for this graph (>512 threads)");
  } else {
    double best = 1e30;
    for (int v : kVplSet) {
      const int tb = round_up((n + v - 1) / v, 64);
      if (tb > kMaxThreads || v > vmax) continue;
      const double waste = (double)(tb * v - n) / (double)(tb * v);
      const double score = waste + (v < 4 ? 0.25 : 0.0) + 0.01 * v;
      if (score < best) {
        best = score;
        TB = tb;
        VPL = v;
      }
    }
    if (best >= 1e30) return set_err(QLDPC_ENOTSUP, "graph too large for the register-resident kernel");
  }
  if ((m + TB - 1) / TB > 32) return set_err(QLDPC_ENOTSUP, "too many checks per thread (m > 32*threads)");
  return 0;
}

size_t lds_for(int precision, int mmax) {
  const size_t pair = precision == 32 ? 8 : 16;
  return pair * 2 * (size_t)mmax + 4 * 2 * (size_t)mmax + 64;
}

// ---- engine 2 geometry: threads per shot TB (multiple of 64, 64..1024) and a
// runtime count of variables per thread VPL = ceil(n / TB) <= 32.  Default TB
// 256; QLDPC_TB or vars_per_thread override it.
int choose_sgeometry(int n, int m, int requested_vpl, int& TB, int& VPL) {
  const int forced_tb = env_int("QLDPC_TB", 0);
  if (requested_vpl > 0) {
    VPL = requested_vpl;
    TB = round_up((n + VPL - 1) / VPL, 64);
  } else if (forced_tb > 0) {
    TB = round_up(forced_tb, 64);
    VPL = (n + TB - 1) / TB;
  } else {
    // 256 threads (4 waves) per shot measured best on n225..n1600 (DESIGN.md
    // §Kernels): four workgroups per CU, short check-phase tails.
    TB = std::min(256, round_up(n, 64));
    VPL = (n + TB - 1) / TB;
    if (VPL > kMaxVplS) {
      TB = std::min(kMaxThreadsS, round_up((n + kMaxVplS - 1) / kMaxVplS, 64));
      VPL = (n + TB - 1) / TB;
    }
  }
  if (TB > kMaxThreadsS || TB < 64) return set_err(QLDPC_EINVAL, "threads per shot out of range (64..1024)");
  if (VPL > kMaxVplS) return set_err(QLDPC_ENOTSUP, "more than 32 variables per thread (n > 32768)");
  if ((m + TB - 1) / TB > 32) return set_err(QLDPC_ENOTSUP, "too many checks per thread (m > 32*threads)");
  return 0;
}

// ---- engine 3 geometry: compile-time VPL <= 8.  Default: the smallest
// power-of-two TB (64..1024) with VPL = ceil(n / TB) <= 7 -- measured best or
// within 4 % of the best on n126..n1600 (profiles/r01/geometry_sweep_e3.txt:
// n1600 256x7, n625 128x5, n225 64x4, GBC A4 256x4, GBC A1 64x2; fewer,
// longer threads win through the software-pipelined variable loop and shorter
// check-phase tails).  QLDPC_TB or vars_per_thread override it.  Returns
// nonzero if engine 3 cannot take the graph (the caller falls back to engine 2).
constexpr int kMaxVplR = 8;
constexpr int kPrefVplR = 7;
int choose_rgeometry(int n, int m, int requested_vpl, int& TB, int& VPL, int pref = kPrefVplR, int vmax = kMaxVplR) {
  const int forced_tb = env_int("QLDPC_TB", 0);
  if (requested_vpl > 0) {
    VPL = requested_vpl;
    TB = round_up((n + VPL - 1) / VPL, 64);
  } else if (forced_tb > 0) {
    TB = round_up(forced_tb, 64);
    VPL = (n + TB - 1) / TB;
  } else {
    TB = 64;
    while (TB < kMaxThreadsS && ((n + TB - 1) / TB > pref || (m + TB - 1) / TB > 32)) TB *= 2;
    VPL = (n + TB - 1) / TB;
  }
  if (TB > kMaxThreadsS || TB < 64 || VPL < 1 || VPL > vmax || (m + TB - 1) / TB > 32) return 1;
  return 0;
}

// Engines 3 and 4 address their image with 16-bit byte offsets.
// Engines 3 and 4 address their image with 16-bit byte offsets; engine 3 with
// dword-scaled offsets (kernel id 13, ea_shift 2) reaches 256 KiB.
bool r_fits(int eng, int vslots, int mmax, int tsize, int ea_shift = 0, int tail = 0, int m2s = 0, int fb = 0) {
  const RLayout L = r_layout(eng, vslots, mmax, tsize, tail, m2s, fb);
  return L.lred <= (65536u << ea_shift) && r_lds_bytes((int)L.total, kChunkMax) <= (size_t)kLdsMax;
}

// Slots per workgroup: QLDPC_NS, else 1 (independent workgroups interleave
// better than lock-stepped slots).
int choose_ns(int img) {
  const int forced = env_int("QLDPC_NS", 1);
  const int ns = (forced == 2 || forced == 4) ? forced : 1;
  return slot_lds_bytes(ns, img, kChunkMax) <= (size_t)kLdsMax ? ns : 1;
}

int device_cus(int dev, int& cus) {
  hipDeviceProp_t prop;
  QLDPC_HIP(hipGetDeviceProperties(&prop, dev));
  cus = prop.multiProcessorCount;
  return 0;
}

}  // namespace

// ================================================================== C ABI
extern "C" {

#if QLDPC_STAMPS
// diagnostic builds only (not in include/qldpc_hip.h): read and clear the phase-cycle sums
int qldpc_debug_stamps(unsigned long long* out) {
  unsigned long long* b = debug_stamps_buffer();
  if (!b || hipDeviceSynchronize() != hipSuccess || hipMemcpy(out, b, 80, hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return hipMemset(b, 0, 80) == hipSuccess ? 0 : -1;
}
#endif

int qldpc_abi_version(void) { return QLDPC_ABI_VERSION; }

const char* qldpc_last_error(void) { return qldpc_rt::g_err.c_str(); }

int qldpc_build_flags(void) { return QLDPC_EXPERIMENTAL ? QLDPC_BUILD_EXPERIMENTAL : 0; }

int qldpc_device_count(int* out) {
  if (!out) return set_err(QLDPC_EINVAL, "out is NULL");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) {
    *out = 0;
    return set_err(QLDPC_EHIP, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
  }
  *out = c;
  return 0;
}

int qldpc_graph_create(int device, int32_t m, int32_t n, const int32_t* row_ptr, const int32_t* col_idx,
                       qldpc_graph** out) {
  if (!out || !row_ptr || (m > 0 && !col_idx)) return set_err(QLDPC_EINVAL, "NULL argument");
  if (m < 0 || n <= 0) return set_err(QLDPC_EINVAL, "bad shape");
  if (m >= 0xFFFF) return set_err(QLDPC_ENOTSUP, "more than 65534 checks");
  if (row_ptr[0] != 0) return set_err(QLDPC_EINVAL, "row_ptr[0] != 0");
  auto* g = new qldpc_graph();
  g->device = device;
  g->m = m;
  g->n = n;
  g->nnz = row_ptr[m];
  g->row_ptr.assign(row_ptr, row_ptr + m + 1);
  g->col_idx.assign(col_idx, col_idx + g->nnz);
  g->col_rows.assign(n, {});
  for (int i = 0; i < m; ++i) {
    if (row_ptr[i + 1] < row_ptr[i]) {
      delete g;
      return set_err(QLDPC_EINVAL, "row_ptr not monotone");
    }
    g->max_row = std::max(g->max_row, row_ptr[i + 1] - row_ptr[i]);
    for (int e = row_ptr[i]; e < row_ptr[i + 1]; ++e) {
      const int c = col_idx[e];
      if (c < 0 || c >= n || (e > row_ptr[i] && col_idx[e - 1] >= c)) {
        delete g;
        return set_err(QLDPC_EINVAL, "col_idx out of range or not strictly ascending within a row");
      }
      g->col_rows[c].push_back(i);
    }
  }
  for (int j = 0; j < n; ++j) g->max_col = std::max<int>(g->max_col, (int)g->col_rows[j].size());
  *out = g;
  return 0;
}

int qldpc_graph_destroy(qldpc_graph* g) {
  delete g;
  return 0;
}

int qldpc_graph_info(const qldpc_graph* g, int32_t* m, int32_t* n, int32_t* nnz, int32_t* max_row_deg,
                     int32_t* max_col_deg) {
  if (!g) return set_err(QLDPC_EINVAL, "NULL graph");
  if (m) *m = g->m;
  if (n) *n = g->n;
  if (nnz) *nnz = g->nnz;
  if (max_row_deg) *max_row_deg = g->max_row;
  if (max_col_deg) *max_col_deg = g->max_col;
  return 0;
}

static int upload_llr(qldpc_bp* bp) {
  const int TB = bp->TB, VPL = bp->VPL, n = bp->g->n;
  if (bp->engine == 6) {  // HBM engine: log((1-p)/p) per variable, variable order
    std::vector<double> l64(n);
    for (int j = 0; j < n; ++j) l64[j] = std::log((1.0 - bp->probs[j]) / bp->probs[j]);  // glibc log, as Cython
    if (bp->precision == 32) {
      std::vector<float> l32(l64.begin(), l64.end());
      QLDPC_HIP(hipMemcpy(bp->llr.p, l32.data(), (size_t)n * 4, hipMemcpyHostToDevice));
    } else {
      QLDPC_HIP(hipMemcpy(bp->llr.p, l64.data(), (size_t)n * 8, hipMemcpyHostToDevice));
    }
    return 0;
  }
  if (bp->engine == 5) {  // product-sum priors: ratio p / (1 - p), computed in double (oracle ws_priors)
    std::vector<double> r64(n);
    for (int j = 0; j < n; ++j) r64[j] = bp->probs[j] / (1.0 - bp->probs[j]);
    if (bp->precision == 32) {
      std::vector<float> r32(r64.begin(), r64.end());
      QLDPC_HIP(hipMemcpy(bp->llr.p, r32.data(), (size_t)n * 4, hipMemcpyHostToDevice));
    } else {
      QLDPC_HIP(hipMemcpy(bp->llr.p, r64.data(), (size_t)n * 8, hipMemcpyHostToDevice));
    }
    return 0;
  }
  const size_t cnt = (size_t)VPL * TB;
  std::vector<double> l64(cnt, 1.0);
  for (int k = 0; k < VPL; ++k)
    for (int t = 0; t < TB; ++t) {
      const int j = bp->slot_var.empty() ? (k * TB + t < n ? k * TB + t : -1) : bp->slot_var[(size_t)k * TB + t];
      if (j >= 0) l64[(size_t)k * TB + t] = std::log((1.0 - bp->probs[j]) / bp->probs[j]);  // glibc log, as Cython
    }
  if (bp->precision == 32) {
    std::vector<float> l32(cnt);
    for (size_t i = 0; i < cnt; ++i) l32[i] = (float)l64[i];
    QLDPC_HIP(hipMemcpy(bp->llr.p, l32.data(), cnt * sizeof(float), hipMemcpyHostToDevice));
  } else {
    QLDPC_HIP(hipMemcpy(bp->llr.p, l64.data(), cnt * sizeof(double), hipMemcpyHostToDevice));
  }
  return 0;
}

// Engine-2/3 edge table: for slot (k, t) holding variable j = slot_var[k*TB+t]
// and its d-th check i (rows ascending), the word ((i + 1) | slot<<16) where
// slot is the position of edge (i, j) in row i of the row-major V image (after
// the 16-byte sink), with the 16-byte chunks of row i XOR-swizzled so that
// consecutive rows read by consecutive lanes hit distinct LDS banks.  Missing
// edges are the word 0 (dummies, bp_slot.h).
//
// Where an edge sits inside its row is free (the check phase takes an
// order-independent min / second min / parity), so with `vbase_dw` >= 0 (engine
// 3, fp32: dword offset of V in the image) the positions are chosen greedily,
// per v2c store instruction of the variable phase (slot (k, t), 32-lane half
// wave), to spread its 32 stores over the 32 banks: at most 2 per bank, which
// ds_write_b32 absorbs for free (MI355X_MICROARCH.md §LDS).  vbase_dw < 0
// keeps the ascending-column order (engine 4 relies on it).
//
// `lab` (engine 3, may be empty = identity) relabels the checks: check i keeps
// its CS entry at lab[i] + 1 and its row at position lab[i] of V (see
// label_checks below).  The F words and the check phase follow the labels; the
// decode path maps syndromes through the inverse permutation (bp->rperm).
// Slot plan of the fp64 space-time m2s family (engine id 111313, kern_r_f64_m2st.hip): the slot map
// (variable of every physical position k * tb + t, -1 = padding), its D2K / D3K, the private dummy
// count, the narrow-wave masks and the waves live in the last variable slot.  Round 6: the degree
// classes 1 / 2 / 3 / 4 in column order fill the LOGICAL positions slot-major; per variable slot k <
// kNwSlots of compile-time width w_k (2 below D2K, 3 below D3K, else DM) the leading logical waves whose
// variables all have degree <= w_k - 1 compute that slot one edge slot narrower (a wave-uniform branch,
// SSector::nw bit 16 k + physical wave): config 5 executes 15,360 edge slots per iteration for 15,288
// edges instead of 16,640, with 68 private dummies instead of 1,348.  Then (balance) the logical waves
// are placed on physical waves so that the four SIMDs (wave w on SIMD w mod 4) carry equal edge slots
// per iteration: config 5's logical waves execute 13-17 edge slots per thread (the five holding the
// sixth variable slot 17), 62 / 59 / 59 / 60 per SIMD in wave order, 60 on every SIMD placed (longest
// first onto the least loaded SIMD).  !narrow: the classes <= 2 / 3 / 4, no narrow waves.
struct StPlan {
  std::vector<int32_t> slots;
  int d2 = 0, d3 = 0, nd = 0;
  uint32_t nw = 0, live_last = 0;
};
static StPlan st_plan(const qldpc_graph* g, int tb, int vpl, int DM, bool narrow, bool balance) {
  StPlan P;
  auto cls = [&](int d) { return narrow ? std::min(std::max(d, 1), 4) - 1 : (d <= 2 ? 0 : d <= 3 ? 1 : 2); };
  std::vector<int32_t> order;
  order.reserve(g->n);
  for (int c = 0; c < (narrow ? 4 : 3); ++c)
    for (int j = 0; j < g->n; ++j)
      if (cls((int)g->col_rows[j].size()) == c) order.push_back(j);
  std::vector<int> deg((size_t)vpl * tb, -1);
  for (int p = 0; p < g->n && p < vpl * tb; ++p) deg[p] = (int)g->col_rows[order[p]].size();
  auto whole = [&](int lim) {  // leading variable slots whose variables all have degree <= lim
    int kk = 0;
    for (; kk < vpl; ++kk) {
      bool ok = true;
      for (int t = 0; t < tb && ok; ++t) ok = deg[(size_t)kk * tb + t] <= lim;
      if (!ok) break;
    }
    return kk;
  };
  P.d2 = whole(2);
  P.d3 = whole(3);
  const int nwv = (tb + 63) / 64;
  std::vector<int> W(vpl, 0), units(nwv, 0);
  for (int k = 0; k < vpl; ++k) {
    const int w = k < P.d2 ? 2 : k < P.d3 ? 3 : DM;
    if (narrow && k < kNwSlots && nwv <= 16)
      for (; W[k] < nwv; ++W[k]) {
        bool ok = true;
        for (int t = W[k] * 64; t < W[k] * 64 + 64 && t < tb && ok; ++t) ok = deg[(size_t)k * tb + t] <= w - 1;
        if (!ok) break;
      }
    for (int v = 0; v < nwv; ++v) {
      bool live = k < vpl - 1;
      for (int t = v * 64; t < v * 64 + 64 && t < tb && !live; ++t) live = deg[(size_t)k * tb + t] >= 0;
      if (live) units[v] += w - (v < W[k] ? 1 : 0);
    }
    for (int t = 0; t < tb; ++t) {
      const int d = deg[(size_t)k * tb + t];
      if (d >= 0) P.nd += w - ((t >> 6) < W[k] ? 1 : 0) - d;
    }
  }
  // logical wave -> physical wave (identity, or balanced over the 4 SIMDs: longest first, least loaded)
  std::vector<int> phys(nwv);
  for (int v = 0; v < nwv; ++v) phys[v] = v;
  if (balance && nwv % 4 == 0 && nwv <= 16) {
    std::vector<int> byu(nwv);
    for (int v = 0; v < nwv; ++v) byu[v] = v;
    std::stable_sort(byu.begin(), byu.end(), [&](int a, int b) { return units[a] > units[b]; });
    int load[4] = {0, 0, 0, 0}, cnt[4] = {0, 0, 0, 0};
    for (int v : byu) {
      int best = -1;
      for (int q = 0; q < 4; ++q)
        if (cnt[q] < nwv / 4 && (best < 0 || load[q] < load[best])) best = q;
      phys[v] = best + 4 * cnt[best]++;
      load[best] += units[v];
    }
  }
  P.slots.assign((size_t)vpl * tb, -1);
  for (int p = 0; p < g->n && p < vpl * tb; ++p) {
    const int k = p / tb, t = p % tb;
    P.slots[(size_t)k * tb + phys[t >> 6] * 64 + (t & 63)] = order[p];
  }
  for (int v = 0; v < nwv && v < 32; ++v) {
    bool live = false;
    for (int t = v * 64; t < v * 64 + 64 && t < tb && !live; ++t) live = deg[(size_t)(vpl - 1) * tb + t] >= 0;
    if (live) P.live_last |= 1u << phys[v];
    for (int k = 0; k < kNwSlots && k < vpl; ++k)
      if (v < W[k]) P.nw |= 1u << (16 * k + phys[v]);
  }
  return P;
}

static void build_slot_edges(const qldpc_graph* g, int TB, int VPL, int DM, int tsize, int nch,
                             const std::vector<int32_t>& slot_var, std::vector<uint32_t>& out, int vbase_dw = -1,
                             const std::vector<int>& lab = {}, int tail = 0, int m2s = 0, int d3k = 0,
                             int dummy0 = -1, int* ndummy = nullptr, int anneal = 0, int anneal_iters = -1,
                             int tail_base = -1, int d2k = 0, uint32_t nw = 0) {
  const int nv = 16 / tsize;  // messages per 16-byte chunk
  const int rw = nch * nv;
  const int rwt = rw + (tail ? 1 : 0);  // tail layouts: logical slot rw = the row's tail slot
  // first tail slot: right after V (bp_reg.h r_layout), i.e. after the private dummy slots when the
  // layout has them (tail_base, the space-time m2s family)
  const int tail0 = tail_base >= 0 ? tail_base : (1 + g->m * nch) * nv;
  const int swz_mask = (nch == 2) ? 1 : (nch == 4) ? 3 : 0;
  const int swz_shift = (nch == 2) ? 3 : 2;
  auto L = [&](int i) { return lab.empty() ? i : lab[i]; };
  auto phys = [&](int i, int ls) {
    const int r = L(i);
    if (ls == rw) return tail0 + r;
    return nv + r * rw + ((ls / nv) ^ ((r >> swz_shift) & swz_mask)) * nv + ls % nv;
  };
  // logical slot of every edge (CSR order); default = ascending column position
  std::vector<int> lslot(g->nnz);
  for (int i = 0; i < g->m; ++i)
    for (int e = g->row_ptr[i]; e < g->row_ptr[i + 1]; ++e) lslot[e] = e - g->row_ptr[i];
  auto edge_of = [&](int i, int j) {
    const int32_t* b = g->col_idx.data() + g->row_ptr[i];
    const int32_t* e = g->col_idx.data() + g->row_ptr[i + 1];
    return (int)(std::lower_bound(b, e, (int32_t)j) - g->col_idx.data());
  };
  // v2c store instructions: ds_write_b32 (float) = 2 groups of 32 lanes over 32
  // banks; ds_write_b64 (double) = 4 groups of 16 contiguous lanes, an 8-byte
  // slot s on bank pair s mod 16 (MI355X_MICROARCH.md §LDS)
  const int sg = tsize == 4 ? 32 : 16, nb = tsize == 4 ? 32 : 16;
  const int vbase_u = vbase_dw < 0 ? 0 : (tsize == 4 ? vbase_dw : vbase_dw / 2);
  if (vbase_dw >= 0 && rwt <= 32 && m2s) {
    // m2s (fp64): the variable phase also READS each edge's V slot (ds_read_b64: 2 groups of 32
    // lanes, 8-byte slot s on bank pair s mod 32), besides storing it (ds_write_b64: 4 groups of 16
    // contiguous lanes, bank pair s mod 16).  Place per 32-lane group: distinct s mod 32 over the
    // group first, distinct s mod 16 within each 16-lane half second.
    std::vector<uint32_t> used(g->m, 0u);
    const bool greedy = env_int("QLDPC_M2S_GREEDY", 1) != 0;
    for (int k = 0; k < VPL && greedy; ++k)
      for (int d = 0; d < DM; ++d)
        for (int h0 = 0; h0 < TB; h0 += 32) {
          int c32[32] = {0}, c16[2][16] = {{0}};
          for (int t = h0; t < h0 + 32 && t < TB; ++t) {
            const int j = slot_var[(size_t)k * TB + t];
            if (j < 0 || d >= (int)g->col_rows[j].size()) continue;
            const int i = g->col_rows[j][d];
            const int hf = (t - h0) >> 4;
            int best = -1, bc = 1 << 30;
            for (int ls = 0; ls < rwt; ++ls) {
              if ((used[i] >> ls) & 1u) continue;
              const int sl = vbase_u + phys(i, ls);
              const int c = 4 * c32[sl % 32] + c16[hf][sl % 16];
              if (c < bc) {
                bc = c;
                best = ls;
              }
            }
            used[i] |= 1u << best;
            const int sl = vbase_u + phys(i, best);
            c32[sl % 32]++;
            c16[hf][sl % 16]++;
            lslot[edge_of(i, j)] = best;
          }
        }
  } else if (vbase_dw >= 0 && rwt <= 32) {
    std::vector<uint32_t> used(g->m, 0u);
    for (int k = 0; k < VPL; ++k)
      for (int d = 0; d < DM; ++d)
        for (int h0 = 0; h0 < TB; h0 += sg) {
          int cnt[32] = {0};
          for (int t = h0; t < h0 + sg && t < TB; ++t) {
            const int j = slot_var[(size_t)k * TB + t];
            if (j < 0 || d >= (int)g->col_rows[j].size()) continue;
            const int i = g->col_rows[j][d];
            int best = -1, bc = 1 << 30;
            for (int ls = 0; ls < rwt; ++ls) {
              if ((used[i] >> ls) & 1u) continue;
              const int c = cnt[(vbase_u + phys(i, ls)) % nb];
              if (c < bc) {
                bc = c;
                best = ls;
              }
            }
            used[i] |= 1u << best;
            cnt[(vbase_u + phys(i, best)) % nb]++;
            lslot[edge_of(i, j)] = best;
          }
        }
  }
  // Annealed placement (round 4, fp64 engine-3 families; `anneal` 1: the variable phase reads and
  // stores each edge's V slot (m2s, the 1024-thread tail family), 2: stores only (own v2c in VGPRs)).
  if (anneal && vbase_dw >= 0 && rwt <= 32) {
    // Then a seeded annealed local search over the rows' slot permutations (swap the positions of
    // two edges of one row, or move one into a free position) on the EXACT cost of the lane-group
    // bank model (qldpc_bp_lds_model): per 32-lane read group the maximum number of addresses on one
    // bank pair (slot mod 32), per 16-lane store group the same over slot mod 16; objective = reads
    // + ws * stores, temperature T0 falling linearly to 0 (round 4; tools/dev/place_opt3.cpp is the
    // offline study: 20 M moves take the n1600 hz model from 362 / 715 to 327 / 442 cycles).
    // default 4000 moves per edge, capped at 2^25 moves (~6 s on one host core; n1600: 21.5 M moves,
    // ~3.9 s; measured +3.1 %: 1.221 M vs 1.184 M shots/s, bank-conflict share 0.338 -> 0.276,
    // profiles/r04/passd/); QLDPC_M2S_ANNEAL=<moves> or DeviceBP(anneal_iters=...) overrides it (0 =
    // the greedy placement only, for short runs).  The result is memoised per process for the same
    // graph, lane map and layout (decoders for other error rates of one code reuse it); the memo keeps
    // at most kAnnealMemo placements (a sweep over many codes does not grow it without bound)
    const int iters_env = anneal_iters >= 0 ? anneal_iters : env_int("QLDPC_M2S_ANNEAL", -1);
    const int iters = iters_env >= 0 ? iters_env : (int)std::min<long long>(4000LL * g->nnz, 1LL << 25);
    constexpr size_t kAnnealMemo = 16;
    static std::mutex memo_mu;
    static std::map<uint64_t, std::vector<int>> memo;
    uint64_t key = 0xcbf29ce484222325ull;
    auto mix = [&](uint64_t v) { key = (key ^ v) * 0x100000001b3ull; };
    bool hit = false;
    if (iters > 0) {
      for (int v : {g->m, g->n, TB, VPL, DM, nch, tail, vbase_u, iters, anneal, env_int("QLDPC_M2S_ANNEAL_T", 50),
                    env_int("QLDPC_M2S_ANNEAL_WS", 1000)})
        mix((uint64_t)(uint32_t)v);
      for (int32_t v : slot_var) mix((uint64_t)(uint32_t)v);
      for (int32_t v : g->col_idx) mix((uint64_t)(uint32_t)v);
      for (int v : lslot) mix((uint64_t)(uint32_t)v);  // the greedy start
      std::lock_guard<std::mutex> lk(memo_mu);
      auto it = memo.find(key);
      if (it != memo.end() && it->second.size() == lslot.size()) {
        lslot = it->second;
        hit = true;
      }
    }
    if (iters > 0 && !hit) {
      const double T0 = env_int("QLDPC_M2S_ANNEAL_T", 50) * 1e-3, ws = env_int("QLDPC_M2S_ANNEAL_WS", 1000) * 1e-3;
      const double wr = anneal == 1 ? 1.0 : 0.0;  // 2: the family keeps its own v2c in VGPRs (no V reads)
      const int nrg = VPL * DM * ((TB + 31) / 32), nwg = VPL * DM * ((TB + 15) / 16);
      std::vector<int> erg(g->nnz, -1), ewg(g->nnz, -1);
      for (int k = 0; k < VPL; ++k)
        for (int t = 0; t < TB; ++t) {
          const int j = slot_var[(size_t)k * TB + t];
          if (j < 0) continue;
          const auto& rows = g->col_rows[j];
          for (int d = 0; d < (int)rows.size() && d < DM; ++d) {
            const int e = edge_of(rows[d], j);
            erg[e] = (k * DM + d) * ((TB + 31) / 32) + t / 32;
            ewg[e] = (k * DM + d) * ((TB + 15) / 16) + t / 16;
          }
        }
      // per group: addresses per bank and a histogram of those counts (max in O(1) amortised)
      struct BankG {
        uint8_t cnt[32] = {0};
        int hist[64] = {0};
        int mx = 0;
        void add(int b) { hist[cnt[b]]--; hist[++cnt[b]]++; mx = std::max(mx, (int)cnt[b]); }
        void sub(int b) { hist[cnt[b]]--; hist[--cnt[b]]++; while (mx > 0 && hist[mx] == 0) --mx; }
        int cost() const { return mx > 1 ? mx : 1; }
      };
      std::vector<BankG> RG(nrg), WG(nwg);
      std::vector<int> at((size_t)g->m * rwt, -1);  // position -> edge per row (-1 = free)
      auto put = [&](int e, int i, int sg) {
        const int sl = vbase_u + phys(i, lslot[e]);
        if (sg > 0) { RG[erg[e]].add(sl % 32); WG[ewg[e]].add(sl % 16); }
        else { RG[erg[e]].sub(sl % 32); WG[ewg[e]].sub(sl % 16); }
      };
      for (int i = 0; i < g->m; ++i)
        for (int e = g->row_ptr[i]; e < g->row_ptr[i + 1]; ++e) {
          at[(size_t)i * rwt + lslot[e]] = e;
          if (erg[e] >= 0) put(e, i, +1);
        }
      uint64_t rs = 0x2545F4914F6CDD1Dull;
      auto rnd = [&]() { rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17; return rs; };
      auto cost2 = [&](int ea, int eb) {  // cost of the (deduplicated) groups of two edges
        double c = 0;
        int r0 = -1, w0 = -1;
        for (int e : {ea, eb}) {
          if (e < 0) continue;
          if (erg[e] != r0) c += wr * RG[erg[e]].cost();
          if (ewg[e] != w0) c += ws * WG[ewg[e]].cost();
          r0 = erg[e];
          w0 = ewg[e];
        }
        return c;
      };
      for (int it = 0; it < iters; ++it) {
        const int i = (int)(rnd() % (uint64_t)g->m);
        const int a = (int)(rnd() % (uint64_t)rwt), b = (int)(rnd() % (uint64_t)rwt);
        if (a == b) continue;
        const int ea = at[(size_t)i * rwt + a], eb = at[(size_t)i * rwt + b];
        if ((ea < 0 || erg[ea] < 0) && (eb < 0 || erg[eb] < 0)) continue;
        if ((ea >= 0 && erg[ea] < 0) || (eb >= 0 && erg[eb] < 0)) continue;
        const double before = cost2(ea, eb);
        auto swap_ab = [&]() {
          if (ea >= 0) put(ea, i, -1);
          if (eb >= 0) put(eb, i, -1);
          if (ea >= 0) lslot[ea] = lslot[ea] == a ? b : a;
          if (eb >= 0) lslot[eb] = lslot[eb] == a ? b : a;
          if (ea >= 0) put(ea, i, +1);
          if (eb >= 0) put(eb, i, +1);
        };
        swap_ab();
        const double dlt = cost2(ea, eb) - before;
        const double T = T0 * (1.0 - (double)it / iters);
        const bool take = dlt <= 0 || (T > 0 && (double)(rnd() % 1000000) / 1e6 < std::exp(-dlt / T));
        if (take) {
          at[(size_t)i * rwt + a] = eb;
          at[(size_t)i * rwt + b] = ea;
        } else {
          swap_ab();
        }
      }
      std::lock_guard<std::mutex> lk(memo_mu);
      if (memo.size() >= kAnnealMemo) memo.clear();
      memo[key] = lslot;
    }
  }
  out.assign((size_t)VPL * DM * TB, kNoEdgeS);
  for (int k = 0; k < VPL; ++k)
    for (int t = 0; t < TB; ++t) {
      const int j = slot_var[(size_t)k * TB + t];
      if (j < 0) continue;
      const auto& rows = g->col_rows[j];
      for (int d = 0; d < (int)rows.size(); ++d) {
        const int i = rows[d];
        const int slot = phys(i, lslot[edge_of(i, j)]);
        out[((size_t)k * DM + d) * TB + t] = (uint32_t)(L(i) + 1) | ((uint32_t)slot << 16);
      }
    }
  // m2s rows of 8 / space-time rows: the missing edges of real variables (slots k >= d3k hold DM
  // edge slots, d2k <= k < d3k three, k < d2k two; one fewer in the narrow waves of `nw`) get private
  // V slots from dummy0 on, lane-consecutive per (k, d) (conflict-free reads and stores), and the
  // dummy CS entry 0
  int nd = 0;
  if (dummy0 >= 0)
    for (int k = 0; k < VPL; ++k)
      for (int d = 0; d < DM; ++d)
        for (int t = 0; t < TB; ++t) {
          const int j = slot_var[(size_t)k * TB + t];
          const int w = (k < d2k ? 2 : k < d3k ? 3 : DM) - (k < kNwSlots && ((nw >> (16 * k + (t >> 6))) & 1u) ? 1 : 0);
          if (j >= 0 && d >= (int)g->col_rows[j].size() && d < w)
            out[((size_t)k * DM + d) * TB + t] = (uint32_t)(dummy0 + nd++) << 16;
        }
  if (ndummy) *ndummy = nd;
}

// Static LDS model of one engine-3 fp64 variable phase (per workgroup and iteration): LDS-array
// cycles and the extra (bank-conflict) cycles of the CS gathers, the V-slot reads (one-word m2s
// families) and the v2c stores, from the final edge table.  Lane groups and bank mapping of
// MI355X_MICROARCH.md §LDS: ds_read_b64 2 x 32 lanes, bank pair (a / 8) mod 32; ds_read_b128 the
// 4 lane sets of 16 (kB128 below), bank quad (a / 16) mod 16; ds_write_b64 4 x 16 contiguous
// lanes, bank pair (a / 8) mod 16.  Identical addresses broadcast.  A group costs max over its
// banks of the distinct addresses there (1 = conflict-free).  Compared against SQ_LDS_BANK_CONFLICT
// / SQ_LDS_IDX_ACTIVE (tools/lds_model.py).
static void lds_model_var_phase(const std::vector<uint32_t>& edges, int TB, int VPL, int DM, int d3k, uint32_t vbase,
                                bool m2s, int64_t* out) {
  static const int kB128[4][16] = {{0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
                                   {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
                                   {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
                                   {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};
  for (int q = 0; q < 6; ++q) out[q] = 0;
  auto group_cost = [](const std::vector<std::pair<uint32_t, uint32_t>>& ab) {  // (bank, address)
    std::vector<std::pair<uint32_t, uint32_t>> v(ab);
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
    int mx = 0;
    for (size_t i = 0; i < v.size();) {
      size_t j = i;
      while (j < v.size() && v[j].first == v[i].first) ++j;
      mx = std::max(mx, (int)(j - i));
      i = j;
    }
    return std::max(mx, 1);
  };
  for (int k = 0; k < VPL; ++k)
    for (int d = 0; d < DM; ++d) {
      if (k < d3k && d >= 3) continue;  // compile-time degree-3 slots issue no 4th edge
      for (int w = 0; w * 64 < TB; ++w) {
        auto lane_word = [&](int l) {
          const int t = w * 64 + l;
          return t < TB ? edges[((size_t)k * DM + d) * TB + t] : 0u;
        };
        // CS gathers
        if (m2s) {
          for (int h = 0; h < 2; ++h) {
            std::vector<std::pair<uint32_t, uint32_t>> ab;
            for (int l = h * 32; l < h * 32 + 32; ++l) {
              const uint32_t a = (lane_word(l) & 0xFFFFu) * 8u;
              ab.emplace_back((a / 8u) % 32u, a);
            }
            const int c = group_cost(ab);
            out[0] += c;
            out[1] += c - 1;
          }
        } else {
          for (int h = 0; h < 4; ++h) {
            std::vector<std::pair<uint32_t, uint32_t>> ab;
            for (int q = 0; q < 16; ++q) {
              const uint32_t a = (lane_word(kB128[h][q]) & 0xFFFFu) * 16u;
              ab.emplace_back((a / 16u) % 16u, a);
            }
            const int c = group_cost(ab);
            out[0] += c;
            out[1] += c - 1;
          }
        }
        // V-slot reads (m2s) and v2c stores
        for (int h = 0; h < 2 && m2s; ++h) {
          std::vector<std::pair<uint32_t, uint32_t>> ab;
          for (int l = h * 32; l < h * 32 + 32; ++l) {
            const uint32_t a = vbase + (lane_word(l) >> 16) * 8u;
            ab.emplace_back((a / 8u) % 32u, a);
          }
          const int c = group_cost(ab);
          out[2] += c;
          out[3] += c - 1;
        }
        for (int h = 0; h < 4; ++h) {
          std::vector<std::pair<uint32_t, uint32_t>> ab;
          for (int l = h * 16; l < h * 16 + 16; ++l) {
            const uint32_t a = vbase + (lane_word(l) >> 16) * 8u;
            ab.emplace_back((a / 8u) % 16u, a);
          }
          const int c = group_cost(ab);
          out[4] += c;
          out[5] += c - 1;
        }
      }
    }
}

// Engine-3 check labelling against LDS bank conflicts.  The variable phase
// gathers CS[lab[i] + 1] for the d-th check of each lane's variable: one
// ds_read_b64 (float: 8-byte entries, 2 groups of 32 lanes, bank pair = entry
// mod 32) or ds_read_b128 (double: 16-byte entries, the 4 lane groups of 16 of
// MI355X_MICROARCH.md §LDS, bank quad = entry mod 16) per (slot k, edge d).
// Distinct checks of one lane group that share a colour (entry mod NC) cost an
// extra LDS cycle each (one check gathered by several lanes broadcasts).  The
// labels are a permutation; a seeded local search swaps the labels of two
// checks whenever that does not increase Σ_groups Σ_colours count² (= the group
// size exactly when every group is conflict free).  For double it also balances
// each 16-lane v2c store group over the two row-label parities (ds_write_b64:
// a row of 8 slots covers half of the 16 bank pairs), so build_slot_edges's
// in-row placement can make the stores conflict free too.  Pure host work, done
// once per decoder; the arithmetic is untouched (labels only move storage).
static std::vector<int> label_checks(const qldpc_graph* g, const std::vector<int32_t>& slot_var, int TB, int VPL,
                                     int DM, int tsize, int* cost_before = nullptr, int* cost_after = nullptr,
                                     int m2s = 0) {
  const int m = g->m;
  std::vector<int> lab(m);
  for (int i = 0; i < m; ++i) lab[i] = i;
  if (m < 2) return lab;
  // CS entries of 8 bytes (fp32 pairs; fp64 m2s words): ds_read_b64 gathers, 2 groups of 32 lanes,
  // bank pair = entry mod 32.  16-byte fp64 pairs: ds_read_b128, bank quad = entry mod 16.
  const bool cs8 = tsize == 4 || m2s;
  const int NC = cs8 ? 32 : 16;
  static const int kB128[4][16] = {{0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
                                   {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
                                   {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
                                   {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};
  // groups (gather groups first, then double's store groups), as check lists
  std::vector<int> gs{0}, gm;
  std::vector<char> gstore;
  auto add_group = [&](int k, int d, int w, const int* lanes, int nl, bool store) {
    const size_t start = gm.size();
    for (int q = 0; q < nl; ++q) {
      const int t = w * 64 + lanes[q];
      if (t >= TB) continue;
      const int j = slot_var[(size_t)k * TB + t];
      if (j < 0 || d >= (int)g->col_rows[j].size()) continue;
      const int i = g->col_rows[j][d];
      if (std::find(gm.begin() + start, gm.end(), i) == gm.end()) gm.push_back(i);
    }
    if (gm.size() - start >= 2) {
      gs.push_back((int)gm.size());
      gstore.push_back(store ? 1 : 0);
    } else {
      gm.resize(start);
    }
  };
  int lanes32[2][32], lanes16[4][16];
  for (int q = 0; q < 64; ++q) {
    lanes32[q / 32][q % 32] = q;
    lanes16[q / 16][q % 16] = q;
  }
  for (int k = 0; k < VPL; ++k)
    for (int d = 0; d < DM; ++d)
      for (int w = 0; w * 64 < TB; ++w) {
        if (cs8) {
          for (int h = 0; h < 2; ++h) add_group(k, d, w, lanes32[h], 32, false);
        } else {
          for (int h = 0; h < 4; ++h) add_group(k, d, w, kB128[h], 16, false);
        }
        if (tsize == 8)
          for (int h = 0; h < 4; ++h) add_group(k, d, w, lanes16[h], 16, true);
      }
  const int ng = (int)gstore.size();
  if (ng == 0) return lab;
  std::vector<std::vector<int>> of(m);  // groups of each check
  for (int q = 0; q < ng; ++q)
    for (int e = gs[q]; e < gs[q + 1]; ++e) of[gm[e]].push_back(q);
  // colour of a label in a group: gathers (label + 1) mod NC, stores the row parity
  auto col = [&](int q, int l) { return gstore[q] ? (l & 1) : (l + 1) % NC; };
  const int W = 32;
  // weights of the two kinds of groups in the objective (double: the stores
  // conflict far more than the gathers of structured codes)
  const int wg = env_int("QLDPC_LABEL_WG", tsize == 4 ? 1 : 1), ws = env_int("QLDPC_LABEL_WS", 4);
  std::vector<int> gw(ng);
  for (int q = 0; q < ng; ++q) gw[q] = gstore[q] ? ws : wg;
  std::vector<int> cnt((size_t)ng * W, 0);
  long long cost = 0;
  for (int q = 0; q < ng; ++q)
    for (int e = gs[q]; e < gs[q + 1]; ++e) {
      int& c = cnt[(size_t)q * W + col(q, lab[gm[e]])];
      cost += (long long)gw[q] * (2 * c + 1);
      ++c;
    }
  auto conflicts = [&]() {  // extra gather cycles: Σ (max count - 1) over gather groups
    int tot = 0;
    for (int q = 0; q < ng; ++q) {
      if (gstore[q]) continue;
      int mx = 0;
      for (int c = 0; c < W; ++c) mx = std::max(mx, cnt[(size_t)q * W + c]);
      tot += mx - 1;
    }
    return tot;
  };
  if (cost_before) *cost_before = conflicts();
  uint64_t rs = 0x9E3779B97F4A7C15ull ^ (uint64_t)m * 0x100000001B3ull;
  auto rnd = [&]() {
    rs ^= rs << 13;
    rs ^= rs >> 7;
    rs ^= rs << 17;
    return rs;
  };
  const long long iters = std::min<long long>(4000000LL, (long long)m * env_int("QLDPC_LABEL_IT", 600));
  for (long long it = 0; it < iters; ++it) {
    const int a = (int)(rnd() % (uint64_t)m), b = (int)(rnd() % (uint64_t)m);
    if (a == b) continue;
    const int la = lab[a], lb = lab[b];
    // delta of Σ count² when a takes label lb and b takes la
    long long delta = 0;
    auto move = [&](int q, int from, int to) {
      const int cf = col(q, from), ct = col(q, to);
      if (cf == ct) return;
      int& x = cnt[(size_t)q * W + cf];
      int& y = cnt[(size_t)q * W + ct];
      delta += (long long)gw[q] * ((2 * y + 1) - (2 * x - 1));
      --x;
      ++y;
    };
    for (int q : of[a]) move(q, la, lb);
    for (int q : of[b]) move(q, lb, la);
    if (delta <= 0 && (delta < 0 || (rnd() & 3) == 0)) {
      lab[a] = lb;
      lab[b] = la;
      cost += delta;
    } else {  // undo (reverse order)
      for (int q : of[b]) {
        const int cf = col(q, lb), ct = col(q, la);
        if (cf == ct) continue;
        ++cnt[(size_t)q * W + cf];
        --cnt[(size_t)q * W + ct];
      }
      for (int q : of[a]) {
        const int cf = col(q, la), ct = col(q, lb);
        if (cf == ct) continue;
        ++cnt[(size_t)q * W + cf];
        --cnt[(size_t)q * W + ct];
      }
    }
  }
  if (cost_after) *cost_after = conflicts();
  return lab;
}

// Engine 5 (product-sum): the row-ordered / column-ordered products need the
// plain CSR and CSC (edge ids in row-major order, rows ascending per column).
static int create_ps(qldpc_graph* g, const double* channel_probs, int32_t max_iter, int32_t precision,
                     qldpc_bp** out) {
  auto* bp = new qldpc_bp();
  bp->g = g;
  bp->engine = 5;
  bp->method = QLDPC_PRODUCT_SUM;
  bp->precision = precision;
  bp->max_iter = max_iter > 0 ? max_iter : g->n;
  bp->alpha = 0;
  bp->TB = 256;
  bp->VPL = (g->n + 255) / 256;
  bp->probs.assign(channel_probs, channel_probs + g->n);
  auto fail = [&](int code) {
    for (DevBuf* d : {&bp->llr, &bp->ps_rp, &bp->ps_ci, &bp->ps_cp, &bp->ps_ce, &bp->ps_ws}) d->release();
    delete bp;
    return code;
  };
  const int E = g->nnz;
  std::vector<int32_t> cp(g->n + 1, 0), ce;
  ce.reserve(E);
  for (int j = 0; j < g->n; ++j) {
    for (int i : g->col_rows[j]) {
      const int* b = g->col_idx.data() + g->row_ptr[i];
      const int* e = g->col_idx.data() + g->row_ptr[i + 1];
      ce.push_back((int32_t)(std::lower_bound(b, e, j) - g->col_idx.data()));
    }
    cp[j + 1] = (int32_t)ce.size();
  }
  int rc;
  if ((rc = bp->ps_rp.alloc((size_t)(g->m + 1) * 4)) || (rc = bp->ps_ci.alloc((size_t)std::max(1, E) * 4)) ||
      (rc = bp->ps_cp.alloc((size_t)(g->n + 1) * 4)) || (rc = bp->ps_ce.alloc((size_t)std::max(1, E) * 4)) ||
      (rc = bp->llr.alloc((size_t)g->n * (precision == 32 ? 4 : 8))))
    return fail(rc);
  if (hipMemcpy(bp->ps_rp.p, g->row_ptr.data(), (size_t)(g->m + 1) * 4, hipMemcpyHostToDevice) != hipSuccess ||
      (E && hipMemcpy(bp->ps_ci.p, g->col_idx.data(), (size_t)E * 4, hipMemcpyHostToDevice) != hipSuccess) ||
      hipMemcpy(bp->ps_cp.p, cp.data(), cp.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
      (E && hipMemcpy(bp->ps_ce.p, ce.data(), (size_t)E * 4, hipMemcpyHostToDevice) != hipSuccess))
    return fail(set_err(QLDPC_EHIP, "upload product-sum graph"));
  if ((rc = upload_llr(bp))) return fail(rc);
  // messages in LDS when 2E values fit in 96 KiB (>= 1 workgroup per CU with room), else in HBM
  const bool lds_msgs = ps_lds_bytes(precision, g->m, g->n, E, true) <= 96 * 1024;
  bp->lds_bytes = (int)ps_lds_bytes(precision, g->m, g->n, E, lds_msgs);
  if (bp->lds_bytes > kLdsMax) return fail(set_err(QLDPC_ENOTSUP, "graph too large for the product-sum engine"));
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, ps_kernel(precision), bp->TB, bp->lds_bytes) != hipSuccess)
    nb = 1;
  bp->blocks_per_cu = std::max(1, nb);
  if ((rc = device_cus(g->device, bp->cus))) return fail(rc);
  bp->ps_grid = (long long)bp->blocks_per_cu * bp->cus;
  if (!lds_msgs && (rc = bp->ps_ws.alloc((size_t)bp->ps_grid * 2 * E * (precision == 32 ? 4 : 8)))) return fail(rc);
  *out = bp;
  return 0;
}

static int create_min_sum(qldpc_graph* g, const double* channel_probs, int32_t max_iter, int32_t bp_method,
                          double ms_scaling_factor, int32_t precision, int32_t vars_per_thread,
                          int32_t min_col_slots, int forced_engine, qldpc_bp** out);

// The one-iteration first-min step kernel of a max_iter = 1 min-sum decoder (decode_batch routes
// its decodes there), built when the decoder is created and whenever its priors change, so that
// decode_batch only launches kernels (no synchronous uploads or occupancy queries between
// stream-ordered launches).  Graphs past the kernel's LDS envelope keep the engine.
static void bp1_prepare(qldpc_bp* bp) {
  if (bp->bp1) {
    qldpc_firstmin_destroy(bp->bp1);
    bp->bp1 = nullptr;
  }
  bp->bp1_off = !(bp->max_iter == 1 && bp->method == 1) || env_int("QLDPC_BP1", 1) == 0;
  if (bp->bp1_off) return;
  const std::string keep = qldpc_rt::g_err;  // an ENOTSUP here is not the caller's error
  if (qldpc_firstmin_create(bp->g, bp->probs.data(), 0, bp->alpha, bp->precision, &bp->bp1) != 0) {
    bp->bp1 = nullptr;
    bp->bp1_off = true;
    qldpc_rt::g_err = keep;
  }
}

int qldpc_bp_create(qldpc_graph* g, const double* channel_probs, int32_t max_iter, int32_t bp_method,
                    double ms_scaling_factor, int32_t precision, int32_t vars_per_thread, int32_t min_col_slots,
                    qldpc_bp** out) {
  return create_min_sum(g, channel_probs, max_iter, bp_method, ms_scaling_factor, precision, vars_per_thread,
                        min_col_slots, 0, out);
}

// Engine 6: HBM-resident messages, one decode per lane (any graph; chosen automatically when
// no LDS engine holds the per-decode image).
int qldpc_bp_create_hbm(qldpc_graph* g, const double* channel_probs, int32_t max_iter, double ms_scaling_factor,
                        int32_t precision, qldpc_bp** out) {
  return create_min_sum(g, channel_probs, max_iter, QLDPC_MIN_SUM, ms_scaling_factor, precision, 0, 0, 6, out);
}

// Engine 1 is the one whose decode kernel can hand back the final posteriors.
int qldpc_bp_create_soft(qldpc_graph* g, const double* channel_probs, int32_t max_iter, double ms_scaling_factor,
                         int32_t precision, qldpc_bp** out) {
  return create_min_sum(g, channel_probs, max_iter, QLDPC_MIN_SUM, ms_scaling_factor, precision, 0, 0, 1, out);
}

static int create_min_sum(qldpc_graph* g, const double* channel_probs, int32_t max_iter, int32_t bp_method,
                          double ms_scaling_factor, int32_t precision, int32_t vars_per_thread,
                          int32_t min_col_slots, int forced_engine, qldpc_bp** out) {
  if (!g || !channel_probs || !out) return set_err(QLDPC_EINVAL, "NULL argument");
  if (precision != 32 && precision != 64) return set_err(QLDPC_EINVAL, "precision must be 32 or 64");
  if (bp_method != QLDPC_MIN_SUM && bp_method != QLDPC_PRODUCT_SUM)
    return set_err(QLDPC_EINVAL, "bp_method must be 0 (product_sum) or 1 (minimum_sum)");
  QLDPC_HIP(hipSetDevice(g->device));
  if (bp_method == QLDPC_PRODUCT_SUM) return create_ps(g, channel_probs, max_iter, precision, out);
  const int want_engine = forced_engine ? forced_engine : env_int("QLDPC_ENGINE", 3);
  if (want_engine == 4 && !QLDPC_EXPERIMENTAL)
    return set_err(QLDPC_ENOTSUP, "engine 4 is built only with -DQLDPC_EXPERIMENTAL=1 (tools/build_variant.py)");
  auto* bp = new qldpc_bp();
  bp->g = g;
  bp->engine = ((want_engine >= 1 && want_engine <= 4) || want_engine == 6) ? want_engine : 3;
  // column degree > 8: beyond the LDS engines' edge slots -> engine 6 (row and column degree <= 12); soft BP stays engine 1
  if ((g->max_col > 8 || min_col_slots > 8) && bp->engine != 6) {
    if (bp->engine == 1) {
      delete bp;
      return set_err(QLDPC_ENOTSUP, "column degree > 8");
    }
    bp->engine = 6;
  }
  bp->max_iter = max_iter > 0 ? max_iter : g->n;
  bp->method = bp_method;
  bp->alpha = ms_scaling_factor;
  bp->precision = precision;
  const int colmax = std::max(g->max_col, (int)min_col_slots);
  bp->DMAX = colmax <= 4 ? 4 : 8;
  // engine 3 also takes fp32 graphs with column degree 5-6 (lifted-product codes), exact slot count
  if (bp->engine == 3 && precision == 32 && colmax > 4 && colmax <= 6 && env_int("QLDPC_E3_D56", 1) != 0)
    bp->DMAX = colmax;
  // fp64: column degree 5 on the <= 256-thread family (checked with the geometry below)
  if (bp->engine == 3 && precision == 64 && colmax == 5 && env_int("QLDPC_E3_D56", 1) != 0) bp->DMAX = 5;
  bp->probs.assign(channel_probs, channel_probs + g->n);
  auto fail = [&](int code) {
    for (DevBuf* d : {&bp->vchk, &bp->llr, &bp->rdeg, &bp->rowtab, &bp->perm, &bp->rperm, &bp->work, &bp->h_rp, &bp->h_rcol,
                      &bp->h_rcpos, &bp->h_cp, &bp->h_crpos, &bp->h_ws})
      d->release();
    delete bp;
    return code;
  };
  // engine 6: messages in HBM, one decode per lane (bp_hbm.hip) -- requested, or below when the
  // per-decode LDS image of every LDS engine exceeds the 160 KiB of a CU
  auto setup_hbm = [&]() {
    bp->engine = 6;
    bp->ea_shift = 0;
    bp->slot_var.clear();
    int rc6 = hbm_prepare(bp);
    if (rc6) return fail(rc6);
    bp->llr.release();
    if ((rc6 = bp->llr.alloc((size_t)g->n * (precision == 32 ? 4 : 8))) || (rc6 = upload_llr(bp))) return fail(rc6);
    int nb6 = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb6, hbm_kernel(precision), bp->TB, 0) != hipSuccess) nb6 = 1;
    bp->blocks_per_cu = std::max(1, nb6);
    if ((rc6 = device_cus(g->device, bp->cus))) return fail(rc6);
    bp1_prepare(bp);
    *out = bp;
    return 0;
  };
  if (bp->engine == 6) return setup_hbm();
  const int tsize = precision == 32 ? 4 : 8;
  int DM = bp->DMAX;
  std::vector<uint32_t> vchk;
  const void* kern = nullptr;
  int rc;
  if (bp->engine == 1) {
    rc = choose_geometry(g->n, g->m, vars_per_thread, max_spill_free_vpl(precision, DM), bp->TB, bp->VPL);
    if (rc) return fail(rc);
    const int TB = bp->TB, VPL = bp->VPL, D2 = DM / 2;
    vchk.assign((size_t)VPL * D2 * TB, 0xFFFFFFFFu);
    for (int k = 0; k < VPL; ++k)
      for (int t = 0; t < TB; ++t) {
        const int j = k * TB + t;
        if (j >= g->n) continue;
        const auto& rows = g->col_rows[j];
        for (int d = 0; d < DM; ++d) {
          const uint32_t v = d < (int)rows.size() ? (uint32_t)rows[d] : 0xFFFFu;
          uint32_t& w = vchk[((size_t)k * D2 + d / 2) * TB + t];
          w = (d & 1) ? ((w & 0xFFFFu) | (v << 16)) : ((w & 0xFFFF0000u) | v);
        }
      }
    bp->lds_bytes = (int)lds_for(precision, g->m);
    kern = get_variant(precision, bp->VPL, DM).dec_k;
  } else {
    if (bp->engine == 4 && g->max_row > 8) bp->engine = 3;  // engine 4 rows are 8 slots wide
    bp->nch = bp->engine == 4 ? 8 * tsize / 16 : (std::max(1, g->max_row) * tsize + 15) / 16;
    const int vslots = (1 + g->m * bp->nch) * (16 / tsize);
    if (vslots >= 0xFFFF) {  // no LDS image addresses this many slots: HBM-resident messages (engine 6)
      if (env_int("QLDPC_HBM_FALLBACK", 1) == 0)
        return fail(set_err(QLDPC_ENOTSUP, "V image exceeds 65535 message slots (QLDPC_HBM_FALLBACK=0)"));
      return setup_hbm();
    }
    // degree-5/6 variables hold 2.5x the registers of degree-4 ones: fewer per thread
    const int pref = DM == 4 ? kPrefVplR : 4;
    int vmax = DM == 4 ? kMaxVplR : 5;
    // images of 64-256 KiB (space-time graphs): engine 3 with dword-scaled addresses (fp32, 4 slots)
    if (bp->engine == 3 && precision == 32 && DM == 4 && !r_fits(3, vslots, g->m, tsize) &&
        r_fits(3, vslots, g->m, tsize, 2) && env_int("QLDPC_E3_BIG", 1) != 0)
      bp->ea_shift = 2;
    // rows one message wider than whole chunks (space-time graphs: rows of 9 = 4 fp64 / 2 fp32
    // chunks + 1): chunk rows + a tail slot per row, dword-scaled addresses, 1024-thread
    // workgroups.  fp64: the image fits LDS at all (162.7 KB instead of 176 KB); fp32: the check
    // phase reads 36 instead of 48 bytes per row through the compile-time-width loop.  fp64 images
    // past the 16-bit layout's 64 KiB take it too (round 6: e.g. hgp_34_n1600 over two rounds, 1536 x
    // 4736, 117 KB, which ran on engine 2 before: fp64 engine 3 has no dword-scaled plain layout), and
    // so do fp64 rows of 8 (the tail slot stays empty: GenBicycleA3 / A4 over 2-5 rounds) and graphs
    // whose geometry is 512 threads (hgp_34_n625 over three rounds, 900 x 2775: two decodes per CU)
    const bool f64t = precision == 64 && env_int("QLDPC_E3_TAIL64", 1) != 0;
    if (bp->engine == 3 && DM == 4 && (g->max_row == 9 || (f64t && g->max_row == 8)) && env_int("QLDPC_E3_TAIL", 1) != 0 &&
        (precision == 32 || !r_fits(3, vslots, g->m, tsize, f64t ? 0 : 2))) {
      const int nch_t = 8 * tsize / 16;
      const int vst = (1 + g->m * nch_t) * (16 / tsize);
      int tb = 0, vpl = 0;
      // fp32: byte F words shrink the image below half a CU (config 5: 85.1 -> 79.6 KB), so two
      // 512-thread decodes share a CU (bp_reg.h eng_fb; QLDPC_E3_FB=0 keeps one 1024-thread decode)
      const int vpl_fb = (g->n + 511) / 512;
      if (precision == 32 && vars_per_thread <= 0 && env_int("QLDPC_TB", 0) <= 0 && env_int("QLDPC_E3_FB", 1) != 0 &&
          vpl_fb >= 9 && vpl_fb <= 12 && (g->m + 511) / 512 <= 32 && r_fits(3, vst, g->m, tsize, 2, 1, 0, 1) &&
          2 * r_lds_bytes((int)r_layout(3, vst, g->m, tsize, 1, 0, 1).total, kChunkMax) <= (size_t)kLdsMax) {
        bp->tail = 1;
        bp->fb = 1;
        bp->nch = nch_t;
        bp->ea_shift = 2;
        bp->TB = 512;
        bp->VPL = vpl_fb;
      } else if (r_fits(3, vst, g->m, tsize, 2, 1) && !choose_rgeometry(g->n, g->m, vars_per_thread, tb, vpl) &&
                 (tb > 512 || (f64t && tb == 512)) && vpl >= 4 && vpl <= 8) {
        bp->tail = 1;
        bp->nch = nch_t;
        bp->ea_shift = 2;
      }
    }
    // fp64 "m2 in slot" family (bp_reg.h eng_m2s, kern_r_f64_m2s.hip): one-word check state, m2 in
    // the argmin edge's V slot, rows of up to 7 edges as 3 chunks + a tail slot, <= 256 threads.
    // The headline hgp_34_n1600 image drops from 65.0 KB to 52.3 KB: 3 workgroups per CU instead
    // of 2.  The kernel keeps no dummy edges for real variables, so every column degree must be
    // 3 or 4 with the degree-3 variables filling whole variable slots (host degree sort).
    if (bp->engine == 3 && precision == 64 && DM == 4 && !bp->tail && g->max_row >= 1 && g->max_row <= 7 &&
        env_int("QLDPC_M2S", 1) != 0 && env_int("QLDPC_DEGSORT", 1) != 0) {
      int tb = 0, vpl = 0, n3 = 0, nother = 0;
      for (int j = 0; j < g->n; ++j) {
        const int d = (int)g->col_rows[j].size();
        n3 += d == 3;
        nother += d != 3 && d != 4;
      }
      bool uni = true;  // QLDPC_M2S_UNIL kernels hold one prior for every variable
      for (int j = 1; j < g->n && QLDPC_M2S_UNIL; ++j) uni = uni && channel_probs[j] == channel_probs[0];
      if (!nother && uni && !choose_rgeometry(g->n, g->m, vars_per_thread, tb, vpl) && tb <= 256 && vpl >= 4 &&
          vpl <= 8 && (n3 % tb == 0 || n3 == g->n) && r_fits(3, (1 + g->m * 3) * 2, g->m, 8, 0, 1, 1)) {
        bp->tail = 1;
        bp->m2s = 1;
        bp->nch = 3;
        bp->ea_shift = 0;
        // "c2v in slot" (bp_reg.h eng_c2s, kern_r_f64_c2s.hip, opt-in QLDPC_C2S=1): the check phase
        // writes the c2v of every edge into the row's slots, so no row may have a padding slot:
        // every row exactly 7 edges (the headline HGP graphs).  No CS array (n1600 52.3 -> 46.2 KB)
        // and 25 % fewer VALU, but its check phase stores 7 words per row where m2s stores 2, and
        // LDS stores cost 3x the cycles of reads per byte: 1.141 M vs 1.189 M shots/s
        // (profiles/r03/c2s/), so m2s stays the default
        bool full = true;
        for (int i = 0; i < g->m && full; ++i) full = g->row_ptr[i + 1] - g->row_ptr[i] == 7;
        if (full && QLDPC_EXPERIMENTAL && env_int("QLDPC_C2S", 0) != 0 && r_fits(3, (1 + g->m * 3) * 2, g->m, 8, 0, 1, 2)) bp->m2s = 2;
        // variable-major V slots (bp_reg.h eng_m2v, kern_r_f64_m2v.hip): edge (k, d) of lane t at
        // slot (ecnt(k) + d) * 256 + t, the last variable slot at ecnt * 256 + d * NL + t, then one
        // sentinel slot; the check phase's rows come from a register table (m <= 4 * 256)
        const int d3 = n3 == g->n ? vpl : n3 / 256;
        const int nlast = g->n - (vpl - 1) * 256, NL = (nlast + 63) & ~63;
        const int ecl = 3 * std::min(vpl - 1, d3) + 4 * std::max(0, vpl - 1 - d3);
        const int vm = ecl * 256 + (vpl - 1 < d3 ? 3 : 4) * NL + 1;
        if (bp->m2s == 1 && tb == 256 && g->m <= 4 * 256 && vm * 8 < 65536 && QLDPC_EXPERIMENTAL && env_int("QLDPC_M2V", 0) != 0 &&
            r_fits(3, vm, g->m, 8, 0, 0, 1)) {
          bp->m2s = 3;
          bp->tail = 0;
          bp->vslots_m2v = vm;
          bp->m2v_vlast = ecl * 256;
          bp->m2v_nl = NL;
        }
      }
    }
    // fp64 space-time graphs on the tail layout (rows of 8 / 9 as 4 chunks + a tail slot, 1024 threads,
    // one decode per CU): the one-word check state too (round 6, kern_r_f64_m2st.hip, engine id
    // 111313).  The two-word tail family re-reads each edge's own previous v2c from LDS (its 128-VGPR
    // budget had no room for it) and gathers 16-byte check states: 24 B of variable-phase reads per
    // edge.  Here the own v2c lives in VGPRs (118 with the uniform prior in SGPRs, no scratch) and an
    // edge reads the 8-byte CS and its own slot: 16 B.  Real variables never touch a shared dummy:
    // the measurement variables in 3-edge slots and the degree-3 ones in 4-edge slots get private
    // dummy V slots (config 5: 1,348, 10.8 KB), placed before the tail array.  Uniform priors only.
    if (bp->engine == 3 && precision == 64 && DM == 4 && bp->tail && !bp->fb && !bp->m2s && bp->nch == 4 &&
        env_int("QLDPC_M2ST", 1) != 0 && env_int("QLDPC_DEGSORT", 1) != 0 && env_int("QLDPC_D2K", 1) != 0) {
      int tb = 0, vpl = 0;
      bool uni = true;
      for (int j = 1; j < g->n && QLDPC_M2S_UNIL; ++j) uni = uni && channel_probs[j] == channel_probs[0];
      if (uni && !choose_rgeometry(g->n, g->m, vars_per_thread, tb, vpl) && tb >= 512) {
        // the slot map the build below makes (st_plan), its D2K / D3K and the private dummies of
        // build_slot_edges
        const StPlan P = st_plan(g, tb, vpl, DM, env_int("QLDPC_NW", 1) != 0, env_int("QLDPC_NW_BAL", 1) != 0);
        const int d2 = P.d2, d3 = P.d3, nd = P.nd;
        int dmax = 0;
        for (int j = 0; j < g->n; ++j) dmax = std::max(dmax, (int)g->col_rows[j].size());
        const int vs = (1 + g->m * 4) * 2 + nd;
        if (dmax <= DM && d2 >= 1 && vs < 0x3FFFF && get_rvariant_f64_m2st(vpl, d3, d2).dec_k &&
            r_fits(3, vs, g->m, 8, 2, 1, 1)) {
          bp->m2s = 1;
          bp->vslots_dummy = nd;
          bp->nw = P.nw;
          bp->live_last = P.live_last;
#if QLDPC_DIAG_NOLAST
          // diagnostic builds only (results invalid): no wave runs the last variable slot, to time the
          // cost of the waves that hold it
          bp->live_last = 0;
#endif
        }
      }
    }
    int m2s8_vpt = 0;  // (the rows-of-8 family's 128-thread geometry for small graphs, below)
    // fp64 column degree 5 graphs that come out at 512 threads x <= 3 variables (LP_Matg8_L21 / L30's
    // [h | I], 315 x 1029 / 450 x 1470): the two-word degree-5 family at 256 threads x 5 / 6 variables
    // instead of engine 2 (round 6; QLDPC_D5_256=0 keeps the old geometry)
    if (bp->engine == 3 && precision == 64 && DM == 5 && vars_per_thread <= 0 && env_int("QLDPC_TB", 0) <= 0 &&
        env_int("QLDPC_D5_256", 1) != 0 && g->max_row > 8 && g->max_row <= 10) {
      int tb = 0, vpl = 0;
      if (!choose_rgeometry(g->n, g->m, 0, tb, vpl, pref, vmax) && tb > 256)
        for (int v = 5; v <= 6 && vars_per_thread <= 0; ++v) {
          int tb5 = 0, vpl5 = 0;
          if (!choose_rgeometry(g->n, g->m, v, tb5, vpl5, pref, 6) && tb5 <= 256) {
            vars_per_thread = v;
            vmax = std::max(vmax, v);
          }
        }
    }
    // the same family for rows of 8 and column degree 5 (kern_r_f64_m2s8.hip, engine id 10103): the
    // lifted-product codes (LP_Matg8_L30: 750 degree-3 and 270 degree-5 columns, rows of 8).  Rows of
    // 4 chunks, no tail array.  Slots k >= D3K hold 5 edge slots; a real variable with fewer edges
    // there (a degree-3 variable in the slot shared with the degree-5 class) gets a PRIVATE dummy V
    // slot per missing edge, past the rows, and the dummy CS entry 0 (+0, parity 0): no other lane
    // writes that slot, so the variable phase always reads its own previous v2c back and takes
    // c2v = +-0, which leaves every sum bit-exact (w-domain sums are never -0).  The two-word family
    // runs these graphs at 2 workgroups per CU (256 VGPRs); the one-word state fits 3.
    if (bp->engine == 3 && precision == 64 && DM == 5 && !bp->tail && !bp->m2s && g->max_row >= 1 && g->max_row <= 8 &&
        env_int("QLDPC_M2S", 1) != 0 && env_int("QLDPC_M2S8", 1) != 0 && env_int("QLDPC_DEGSORT", 1) != 0) {
      int tb = 0, vpl = 0, n3 = 0;
      for (int j = 0; j < g->n; ++j) n3 += g->col_rows[j].size() <= 3;
      bool uni = true;
      for (int j = 1; j < g->n && QLDPC_M2S_UNIL; ++j) uni = uni && channel_probs[j] == channel_probs[0];
      bool ok = uni && !choose_rgeometry(g->n, g->m, vars_per_thread, tb, vpl, pref, vmax);
      // smaller graphs (LP_Matg8_L16 / L21, the Threshold notebook's codes: 544 / 714 columns) come out
      // at 256 threads x 3 variables, below the family's 4-6: run them at the most variables per thread
      // (<= 5 for degree 5) whose workgroup is smaller, 128 x 5 / 192 x 5 (round 6; they ran on engine 2
      // before).  The geometry call below then takes this VPL.
      if (ok && tb == 256 && vpl < 4 && vars_per_thread <= 0 && env_int("QLDPC_TB", 0) <= 0 &&
          env_int("QLDPC_M2S8_SMALL", 1) != 0)
        for (int v = std::min(6, vmax); v >= 4 && !m2s8_vpt; --v) {
          int tb2 = 0, vpl2 = 0;
          if (!choose_rgeometry(g->n, g->m, v, tb2, vpl2, pref, vmax) && tb2 < 256 && vpl2 == v) {
            tb = tb2;
            vpl = vpl2;
            m2s8_vpt = v;
          }
        }
      if (ok && (tb == 256 || (tb < 256 && m2s8_vpt > 0)) && vpl >= 4 && vpl <= 6) {
        // the slot map below: degree <= 3 first, so slots k < n3 / tb (whole) hold degree <= 3 only
        const int d3 = n3 == g->n ? vpl : n3 / tb;
        int nd = 0;
        for (int p = 0, c = 0; c < 2; ++c)
          for (int j = 0; j < g->n; ++j) {
            const int d = (int)g->col_rows[j].size();
            if ((d <= 3 ? 0 : 1) != c) continue;
            nd += ((p / tb) < d3 ? 3 : DM) - d;
            ++p;
          }
        const int vs = (1 + g->m * 4) * 2 + nd;
        if (vs < 0xFFFF && r_fits(3, vs, g->m, 8, 0, 0, 1)) {
          bp->m2s = 1;
          bp->nch = 4;
          bp->ea_shift = 0;
          bp->vslots_dummy = nd;
          if (m2s8_vpt > 0) vars_per_thread = m2s8_vpt;
          // packed absolute addresses, 4 workgroups per CU: LP L30 fp64 4.08 M vs 3.67 M shots/s
          // (0.622 vs 0.561 of the LDS roofline, profiles/r04/passd/); QLDPC_M2S8_PK=0 keeps 10103
          bp->m2s_pk = env_int("QLDPC_M2S8_PK", 1) != 0 && vpl <= 5 &&
                       4 * r_lds_bytes((int)r_layout(3, vs, g->m, 8, 0, 1).total, kChunkMax) <= (size_t)kLdsMax;
        }
      }
    }
    const int vslots_e3 = bp->vslots_m2v ? bp->vslots_m2v : (1 + g->m * bp->nch) * (16 / tsize) + bp->vslots_dummy;
    if (bp->engine >= 3 && ((DM != 4 && !(bp->engine == 3 && (DM == 5 || DM == 6))) ||
                            (!bp->fb && choose_rgeometry(g->n, g->m, vars_per_thread, bp->TB, bp->VPL, pref, vmax)) ||
                            !r_fits(bp->engine, vslots_e3, g->m, tsize, bp->ea_shift, bp->tail, bp->m2s, bp->fb) ||
                            (precision == 64 && DM == 5 && !bp->m2s &&
                             !use_f64w(bp->engine, precision, DM, bp->TB, bp->VPL, bp->ea_shift, bp->nch)))) {
      bp->ea_shift = 0;
      bp->tail = 0;
      bp->m2s = 0;
      bp->vslots_dummy = 0;
      bp->m2s_pk = 0;
      bp->fb = 0;
      bp->engine = 2;  // graph outside the register engines' envelope
      bp->nch = (std::max(1, g->max_row) * tsize + 15) / 16;
      if (DM == 5 || DM == 6) bp->DMAX = DM = 8;  // engine 2 kernels come in 4 and 8 slots
    }
    const int vslots2 = bp->vslots_m2v ? bp->vslots_m2v : (1 + g->m * bp->nch) * (16 / tsize) + bp->vslots_dummy;
    if (bp->engine >= 3) {
      bp->NS = 1;
      bp->lds_bytes =
          (int)r_lds_bytes((int)r_layout(bp->engine, vslots2, g->m, tsize, bp->tail, bp->m2s, bp->fb).total, kChunkMax);
    } else {
      rc = choose_sgeometry(g->n, g->m, vars_per_thread, bp->TB, bp->VPL);
      if (rc) return fail(rc);
      const int img = (int)slot_img_bytes(vslots2, g->m, tsize);
      bp->NS = choose_ns(img);
      bp->lds_bytes = (int)slot_lds_bytes(bp->NS, img, kChunkMax);
      // big images leave room for few workgroups per CU: widen the workgroup so
      // the CU still holds >= 16 waves (ST n1225 fp32: 1 x 1024 threads, 2x the
      // samples/s of 1 x 256, bench.py --workload phenl)
      const int bpc = std::max(1, kLdsMax / std::max(1, bp->lds_bytes));
      if (vars_per_thread <= 0 && env_int("QLDPC_TB", 0) <= 0 && bpc * bp->TB / 64 < 16) {
        const int tb = std::min(kMaxThreadsS, round_up((16 + bpc - 1) / bpc * 64, 64));
        if (tb > bp->TB) {
          bp->TB = tb;
          bp->VPL = (g->n + tb - 1) / tb;
        }
      }
    }
    if (bp->lds_bytes > kLdsMax) {  // no LDS engine holds this decode: HBM-resident messages
      if (env_int("QLDPC_HBM_FALLBACK", 1) == 0)
        return fail(set_err(QLDPC_ENOTSUP, "per-shot LDS image exceeds 160 KiB (QLDPC_HBM_FALLBACK=0)"));
      return setup_hbm();
    }
    // slot -> variable map: identity, or (engine 3) degree <= 3 variables first
    const int TB = bp->TB, VPL = bp->VPL;
    std::vector<int32_t> order;
    order.reserve(g->n);
    const bool sort3 = bp->engine == 3 && DM >= 4 && env_int("QLDPC_DEGSORT", 1) != 0;
    // byte-F kernels also keep degree <= 2 variables (the space-time measurement columns) in
    // compile-time 2-edge slots: those go first
    const bool sort2 = sort3 && (bp->fb || (bp->tail && precision == 64 && (!bp->m2s || bp->nch == 4))) &&
                       env_int("QLDPC_D2K", 1) != 0;
    auto cls = [&](int j) {
      const int d = (int)g->col_rows[j].size();
      return sort2 ? (d <= 2 ? 0 : d <= 3 ? 1 : 2) : (d <= 3 ? 0 : 1);
    };
    // (the fp64 space-time m2s family: st_plan's order, degree classes 1 / 2 / 3 / 4 with narrow waves)
    const bool stm2s = bp->engine == 3 && precision == 64 && bp->tail && bp->m2s == 1 && bp->nch == 4;
    if (stm2s) {
      bp->slot_var = st_plan(g, bp->TB, bp->VPL, DM, env_int("QLDPC_NW", 1) != 0, env_int("QLDPC_NW_BAL", 1) != 0).slots;
    } else {
      for (int pass = 0; pass < (sort2 ? 3 : sort3 ? 2 : 1); ++pass)
        for (int j = 0; j < g->n; ++j)
          if (!sort3 || cls(j) == pass) order.push_back(j);
      bp->slot_var.assign((size_t)VPL * TB, -1);
      for (int j = 0; j < g->n; ++j) bp->slot_var[j] = order[j];
    }
    bp->npos = g->n;
    bp->d3k = 0;
    if (sort3)
      for (int k = 0; k < VPL; ++k) {
        bool ok = true;
        for (int t = 0; t < TB && ok; ++t) {
          const int j = bp->slot_var[(size_t)k * TB + t];
          ok = j < 0 || (int)g->col_rows[j].size() <= 3;
        }
        if (!ok) break;
        bp->d3k = k + 1;
      }
    bp->d2k = 0;
    if (sort2)
      for (int k = 0; k < VPL; ++k) {
        bool ok = true;
        for (int t = 0; t < TB && ok; ++t) {
          const int j = bp->slot_var[(size_t)k * TB + t];
          ok = j < 0 || (int)g->col_rows[j].size() <= 2;
        }
        if (!ok) break;
        bp->d2k = k + 1;
      }
    const int vbase_dw = (bp->engine == 3 && env_int("QLDPC_BANKOPT", 1) != 0)
                             ? (int)(r_layout(3, vslots2, g->m, tsize, bp->tail, bp->m2s).v / 4)
                             : -1;
    // fp64 engine-3 kernels are built with D3K = 0 only, except the <= 256-thread family
    if (precision != 32 && !use_f64w(bp->engine, precision, DM, bp->TB, bp->VPL, bp->ea_shift, bp->nch) &&
        !use_f64x(bp->engine, precision, DM, bp->TB, bp->VPL, bp->ea_shift) && !bp->tail && !bp->m2s)
      bp->d3k = 0;
    std::vector<int> lab;
    if (bp->m2s == 3 && env_int("QLDPC_M2V_PERM", 0) != 0) {  // (opt-in: measured 1.6 % slower)
      // m2v: a variable's V slots sit in its lane's bank pair (slot mod 32 = lane mod 32), so which
      // lane a variable occupies inside its slot k sets the banks of the check phase's gathers.  A
      // seeded local search swaps two variables of one slot k (same degree class) whenever that
      // does not raise Σ_{row group of 32, bank} load² (the check gathers; a group whose bank loads
      // are all <= 7 admits conflict-free gather orders) + Σ_{32-lane group, edge, bank} count² of
      // the variable phase's CS gathers (bank pair = (check + 1) mod 32).  Storage only.
      const int TBm = bp->TB, VPLm = bp->VPL, M = g->m;
      const int ng = (M + 31) / 32;
      std::vector<int> L((size_t)ng * 32, 0);                       // check groups x banks
      std::vector<int> C((size_t)VPLm * DM * (TBm / 32) * 32, 0);   // CS gather groups x banks
      auto cidx = [&](int k, int d, int h, int b) { return (((size_t)k * DM + d) * (TBm / 32) + h) * 32 + b; };
      auto add = [&](int j, int pos, int sg) {
        const int k = pos / TBm, t = pos % TBm, b = t % 32, h = t / 32;
        const auto& rows = g->col_rows[j];
        for (int d = 0; d < (int)rows.size(); ++d) {
          L[(size_t)(rows[d] / 32) * 32 + b] += sg;
          C[cidx(k, d, h, (rows[d] + 1) % 32)] += sg;
        }
      };
      auto sq = [&](int j, int pos) {  // Σ of the counts this variable's entries see (for the delta)
        const int k = pos / TBm, t = pos % TBm, b = t % 32, h = t / 32;
        long long v = 0;
        const auto& rows = g->col_rows[j];
        for (int d = 0; d < (int)rows.size(); ++d) v += 2 * L[(size_t)(rows[d] / 32) * 32 + b] + C[cidx(k, d, h, (rows[d] + 1) % 32)];
        return v;
      };
      for (int pos = 0; pos < VPLm * TBm; ++pos)
        if (bp->slot_var[pos] >= 0) add(bp->slot_var[pos], pos, +1);
      uint64_t rs = 0xD1B54A32D192ED03ull;
      auto rnd = [&]() { rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17; return rs; };
      const int iters = env_int("QLDPC_M2V_PERM_IT", 400000);
      for (int it = 0; it < iters; ++it) {
        const int k = (int)(rnd() % (uint64_t)VPLm);
        const int pa = k * TBm + (int)(rnd() % (uint64_t)TBm), pb = k * TBm + (int)(rnd() % (uint64_t)TBm);
        const int ja = bp->slot_var[pa], jb = bp->slot_var[pb];
        if (ja < 0 || jb < 0 || pa == pb || (pa % 32) == (pb % 32) && (pa / 32) == (pb / 32)) continue;
        if (g->col_rows[ja].size() != g->col_rows[jb].size()) continue;
        // cost change: remove both, measure, add swapped, measure (counts are small integers)
        add(ja, pa, -1);
        add(jb, pb, -1);
        const long long before = sq(ja, pa) + sq(jb, pb);
        const long long after = sq(ja, pb) + sq(jb, pa);
        if (after <= before) {
          bp->slot_var[pa] = jb;
          bp->slot_var[pb] = ja;
          add(jb, pa, +1);
          add(ja, pb, +1);
        } else {
          add(ja, pa, +1);
          add(jb, pb, +1);
        }
      }
    }
    // fp64 two-word families (measured +3 % with the bank-aware fp64 v2c placement); fp32 gathers of
    // the structured codes are already near conflict-free, and the m2s family runs 2.5 % faster on
    // the identity labels (1.188 M vs 1.159 M shots/s, profiles/r03/m2s_ab/ab_label.txt): off there
    // (QLDPC_LABEL=1 forces it on)
    if (bp->engine == 3 && env_int("QLDPC_LABEL", precision == 64 && !bp->m2s ? 1 : 0) != 0) {
      lab = label_checks(g, bp->slot_var, bp->TB, bp->VPL, DM, tsize, &bp->gather_conf[0], &bp->gather_conf[1], bp->m2s);
      std::vector<int32_t> inv(g->m);
      for (int i = 0; i < g->m; ++i) inv[lab[i]] = i;
      if ((rc = bp->rperm.alloc((size_t)std::max(1, g->m) * 4))) return fail(rc);
      if (g->m && hipMemcpy(bp->rperm.p, inv.data(), (size_t)g->m * 4, hipMemcpyHostToDevice) != hipSuccess)
        return fail(set_err(QLDPC_EHIP, "upload check labels"));
    }
    int ndummy = 0;
    build_slot_edges(g, bp->TB, bp->VPL, DM, tsize, bp->nch, bp->slot_var, vchk, vbase_dw, lab, bp->tail,
                     bp->m2s == 1 && env_int("QLDPC_M2S_PLACE", 1) != 0, bp->d3k,
                     bp->vslots_dummy ? (1 + g->m * bp->nch) * (16 / tsize) : -1, &ndummy,
                     (bp->engine == 3 && precision == 64 && bp->m2s != 3)
                         ? ((bp->m2s || bp->tail) ? 1 : env_int("QLDPC_ANNEAL_2W", 1) != 0 ? 2 : 0)
                         : 0,
                     -1,
                     (bp->tail && bp->vslots_dummy) ? (int)(r_layout(3, vslots2, g->m, tsize, 1, bp->m2s).t - r_layout(3, vslots2, g->m, tsize, 1, bp->m2s).v) / tsize : -1,
                     bp->d2k, bp->nw);
    if (ndummy != bp->vslots_dummy) return fail(set_err(QLDPC_EINVAL, "m2s private dummy slot count mismatch"));
    if (bp->engine == 3 && precision == 64 && bp->m2s != 3 && bp->ea_shift == 0)
      lds_model_var_phase(vchk, bp->TB, bp->VPL, DM, bp->d3k,
                          (uint32_t)r_layout(3, vslots2, g->m, tsize, bp->tail, bp->m2s).v, bp->m2s == 1,
                          bp->lds_model);
    if (bp->m2s == 3) {
      // m2v row table (bp_reg.h M2vRows): row i = q * TB + t -> uint4 (q * TB + t): the byte offsets
      // from the V base of its edges' variable-major slots, two 16-bit offsets per word, the unused
      // entries at the sentinel slot
      const int TBm = bp->TB, VPLm = bp->VPL, d3 = std::min(bp->d3k, VPLm);
      auto ecnt = [&](int k) { return 3 * std::min(k, d3) + 4 * std::max(0, k - d3); };
      if (ecnt(VPLm - 1) * TBm != bp->m2v_vlast) return fail(set_err(QLDPC_ENOTSUP, "m2v layout mismatch"));
      const uint32_t sent = (uint32_t)(bp->vslots_m2v - 1) * 8u;
      std::vector<std::vector<uint32_t>> roff(g->m);
      for (int k = 0; k < VPLm; ++k)
        for (int t = 0; t < TBm; ++t) {
          const int j = bp->slot_var[(size_t)k * TBm + t];
          if (j < 0) continue;
          const auto& rows = g->col_rows[j];
          for (int d = 0; d < (int)rows.size(); ++d) {
            const int vs = k < VPLm - 1 ? (ecnt(k) + d) * TBm + t : bp->m2v_vlast + d * bp->m2v_nl + t;
            roff[rows[d]].push_back((uint32_t)vs * 8u);
          }
        }
      for (int i = 0; i < g->m; ++i) {
        if (roff[i].size() > 7) return fail(set_err(QLDPC_ENOTSUP, "m2v row wider than 7"));
        while (roff[i].size() < 8) roff[i].push_back(sent);
      }
      // The check phase gathers entry e of its rows with one ds_read_b64 per e: 32-lane groups,
      // bank pair = slot mod 32 (MI355X_MICROARCH.md §LDS).  The order of a row's entries is
      // free: per group of 32 rows, a seeded local search swaps two entries of a row whenever that
      // does not raise Σ_e Σ_bank count² (the sentinel broadcasts: not counted).  Host work only.
      if (env_int("QLDPC_M2V_ORDER", 1) != 0) {
        uint64_t rs = 0x9E3779B97F4A7C15ull;
        auto rnd = [&]() { rs ^= rs << 13; rs ^= rs >> 7; rs ^= rs << 17; return rs; };
        for (int q = 0; q < 4; ++q)
          for (int g0 = 0; g0 < TBm; g0 += 32) {
            std::vector<int> rr;
            for (int l = 0; l < 32; ++l)
              if (q * TBm + g0 + l < g->m) rr.push_back(q * TBm + g0 + l);
            if (rr.size() < 2) continue;
            int cnt[7][32] = {{0}};
            auto bk = [&](uint32_t o) { return (int)((o / 8u) % 32u); };
            for (int i : rr)
              for (int e = 0; e < 7; ++e)
                if (roff[i][e] != sent) cnt[e][bk(roff[i][e])]++;
            for (int it = 0; it < 4000; ++it) {
              const int i = rr[rnd() % rr.size()], a = (int)(rnd() % 7), b = (int)(rnd() % 7);
              const uint32_t oa = roff[i][a], ob = roff[i][b];
              if (a == b || oa == ob) continue;
              auto term = [&](int e, uint32_t o, int dlt) {  // change of count^2 when o enters (+1) / leaves (-1) e
                if (o == sent) return 0;
                const int c = cnt[e][bk(o)];
                return dlt > 0 ? 2 * c + 1 : -(2 * c - 1);
              };
              int d = term(a, oa, -1);
              if (oa != sent) cnt[a][bk(oa)]--;
              d += term(b, ob, -1);
              if (ob != sent) cnt[b][bk(ob)]--;
              d += term(a, ob, +1);
              if (ob != sent) cnt[a][bk(ob)]++;
              d += term(b, oa, +1);
              if (oa != sent) cnt[b][bk(oa)]++;
              if (d <= 0) {
                roff[i][a] = ob;
                roff[i][b] = oa;
              } else {  // undo
                if (ob != sent) cnt[a][bk(ob)]--;
                if (oa != sent) cnt[b][bk(oa)]--;
                if (oa != sent) cnt[a][bk(oa)]++;
                if (ob != sent) cnt[b][bk(ob)]++;
              }
            }
          }
      }
      std::vector<uint32_t> tab((size_t)4 * TBm * 4, 0);
      for (int q = 0; q < 4; ++q)
        for (int t = 0; t < TBm; ++t) {
          const int i = q * TBm + t;
          uint32_t o[8];
          for (int e = 0; e < 8; ++e) o[e] = i < g->m ? roff[i][e] : sent;
          for (int w = 0; w < 4; ++w) tab[((size_t)q * TBm + t) * 4 + w] = o[2 * w] | (o[2 * w + 1] << 16);
        }
      if ((rc = bp->rowtab.alloc(tab.size() * 4))) return fail(rc);
      if (hipMemcpy(bp->rowtab.p, tab.data(), tab.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
        return fail(set_err(QLDPC_EHIP, "upload m2v row table"));
    }
    kern = slot_variant(bp->engine, precision, DM, bp->NS, bp->VPL, bp->d3k, bp->ea_shift, bp->TB, bp->nch, bp->tail,
                        bp->m2s, bp->fb, bp->d2k, bp->m2s_pk).dec_k;
    if (bp->engine >= 3) {
      // row degrees by check label: engine 4 keeps them in F, engine 3 their parity (bp_reg.h, w domain)
      std::vector<uint8_t> deg(std::max(1, g->m));
      for (int i = 0; i < g->m; ++i) deg[lab.empty() ? i : lab[i]] = (uint8_t)(g->row_ptr[i + 1] - g->row_ptr[i]);
      if ((rc = bp->rdeg.alloc(deg.size()))) return fail(rc);
      if (hipMemcpy(bp->rdeg.p, deg.data(), deg.size(), hipMemcpyHostToDevice) != hipSuccess)
        return fail(set_err(QLDPC_EHIP, "upload row degrees"));
    }
  }
  if (!kern && (bp->engine == 3 || bp->engine == 4) && env_int("QLDPC_HBM_FALLBACK", 1) != 0) {
    // no kernel compiled for this engine-3/4 geometry (e.g. fp32 images past 64 KiB at 8 variables per
    // thread, GenBicycleA4 over five rounds): the HBM-resident engine serves any graph
    bp->tail = bp->m2s = bp->fb = bp->m2s_pk = bp->vslots_dummy = bp->d3k = bp->d2k = 0;
    bp->nw = bp->live_last = 0;
    bp->rperm.release();
    bp->rowtab.release();
    bp->rdeg.release();
    return setup_hbm();
  }
  if (!kern) return fail(set_err(QLDPC_ENOTSUP, "no kernel variant"));
  if ((rc = bp->vchk.alloc(vchk.size() * 4)) || (rc = bp->llr.alloc((size_t)bp->VPL * bp->TB * tsize))) return fail(rc);
  if (hipMemcpy(bp->vchk.p, vchk.data(), vchk.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
    return fail(set_err(QLDPC_EHIP, "upload edge table"));
  if ((rc = upload_llr(bp))) return fail(rc);
  if (!bp->slot_var.empty()) {
    if ((rc = bp->perm.alloc(bp->slot_var.size() * 4))) return fail(rc);
    if (hipMemcpy(bp->perm.p, bp->slot_var.data(), bp->slot_var.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
      return fail(set_err(QLDPC_EHIP, "upload slot map"));
  }
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, bp->TB, bp->lds_bytes) != hipSuccess) nb = 1;
  bp->blocks_per_cu = std::max(1, nb);
  if ((rc = device_cus(g->device, bp->cus))) return fail(rc);
  bp1_prepare(bp);
  *out = bp;
  return 0;
}

int qldpc_bp_destroy(qldpc_bp* bp) {
  if (!bp) return 0;
  if (bp->bp1) qldpc_firstmin_destroy(bp->bp1);
  for (DevBuf* d : {&bp->vchk, &bp->llr, &bp->rdeg, &bp->rowtab, &bp->perm, &bp->rperm, &bp->work, &bp->ps_rp, &bp->ps_ci, &bp->ps_cp,
                    &bp->ps_ce, &bp->ps_ws, &bp->h_rp, &bp->h_rcol, &bp->h_rcpos, &bp->h_cp, &bp->h_crpos, &bp->h_ws})
    d->release();
  delete bp;
  return 0;
}

int qldpc_bp_set_channel_probs(qldpc_bp* bp, const double* channel_probs) {
  if (!bp || !channel_probs) return set_err(QLDPC_EINVAL, "NULL argument");
  if (bp->m2s && QLDPC_M2S_UNIL)
    for (int j = 1; j < bp->g->n; ++j)
      if (channel_probs[j] != channel_probs[0])
        return set_err(QLDPC_ENOTSUP, "this decoder's kernels hold one uniform prior: create a new decoder for "
                                      "non-uniform channel_probs");
  bp->probs.assign(channel_probs, channel_probs + bp->g->n);
  const int rc = upload_llr(bp);
  if (rc) return rc;
  bp1_prepare(bp);  // rebuilt from the new priors
  return 0;
}

int qldpc_bp_degree3_slots(const qldpc_bp* bp, int32_t* d3k) {
  if (!bp || !d3k) return set_err(QLDPC_EINVAL, "NULL argument");
  *d3k = bp->engine == 3 ? bp->d3k : 0;
  return 0;
}

int qldpc_bp_lds_model(const qldpc_bp* bp, int64_t* out6) {
  if (!bp || !out6) return set_err(QLDPC_EINVAL, "NULL argument");
  for (int q = 0; q < 6; ++q) out6[q] = bp->lds_model[q];
  return 0;
}

int qldpc_m2s_place_model(const qldpc_graph* g, int32_t anneal_iters, int64_t* out6) {
  if (!g || !out6) return set_err(QLDPC_EINVAL, "NULL argument");
  // the decoder build of the fp64 m2s family (qldpc_bp_create), host side only: geometry, degree
  // sort, greedy + annealed V-slot placement, then the static LDS model of its variable phase
  int n3 = 0;
  for (int j = 0; j < g->n; ++j) {
    const int d = (int)g->col_rows[j].size();
    if (d != 3 && d != 4) return set_err(QLDPC_ENOTSUP, "m2s placement model: column degrees 3 / 4 only");
    n3 += d == 3;
  }
  int TB = 0, VPL = 0;
  if (g->max_row < 1 || g->max_row > 7 || choose_rgeometry(g->n, g->m, 0, TB, VPL) || TB > 256 || VPL < 4 || VPL > 8 ||
      !(n3 % TB == 0 || n3 == g->n))
    return set_err(QLDPC_ENOTSUP, "graph outside the m2s envelope (rows <= 7, <= 256 threads x 4-8 slots)");
  std::vector<int32_t> slot_var((size_t)VPL * TB, -1);
  int p = 0;
  for (int c = 0; c < 2; ++c)
    for (int j = 0; j < g->n; ++j)
      if (((int)g->col_rows[j].size() <= 3 ? 0 : 1) == c) slot_var[p++] = j;
  int d3k = 0;
  for (int k = 0; k < VPL; ++k) {
    bool ok = true;
    for (int t = 0; t < TB && ok; ++t) {
      const int j = slot_var[(size_t)k * TB + t];
      ok = j < 0 || (int)g->col_rows[j].size() <= 3;
    }
    if (!ok) break;
    d3k = k + 1;
  }
  const int vslots = (1 + g->m * 3) * 2;
  const uint32_t vbase = (uint32_t)r_layout(3, vslots, g->m, 8, 1, 1).v;
  std::vector<uint32_t> edges;
  build_slot_edges(g, TB, VPL, 4, 8, 3, slot_var, edges, (int)(vbase / 4), {}, 1, 1, d3k, -1, nullptr, 1,
                   anneal_iters);
  lds_model_var_phase(edges, TB, VPL, 4, d3k, vbase, true, out6);
  return 0;
}

int qldpc_bp_bank_stats(const qldpc_bp* bp, int32_t* before, int32_t* after) {
  if (!bp) return set_err(QLDPC_EINVAL, "NULL decoder");
  if (before) *before = bp->gather_conf[0];
  if (after) *after = bp->gather_conf[1];
  return 0;
}

int qldpc_bp_kernel_id(const qldpc_bp* bp, int32_t* kernel_id, int32_t* row_chunks) {
  if (!bp) return set_err(QLDPC_EINVAL, "NULL decoder");
  int id = bp->engine;
  if (bp->engine == 3) {
    if (bp->m2s)
      id = bp->m2s == 2 ? 31103 : bp->m2s == 3 ? 40103 : (bp->tail && bp->nch == 4) ? 11313 + 100000 * std::min(bp->d2k, 1)
           : bp->tail ? 11103 : bp->m2s_pk ? 10203 : 10103;
    else if (bp->fb)
      id = 21013 + ((bp->d3k >= 8 && bp->d2k > 0) ? 100000 * std::min(bp->d2k, 4) : 0);  // + D2K digit
    else if (bp->tail)
      id = 1013 + ((bp->precision == 64 && bp->VPL == 6 && bp->d2k >= 1 && bp->d3k >= 1) ? 100000 : 0);
    else if (use_f64w(bp->engine, bp->precision, bp->DMAX, bp->TB, bp->VPL, bp->ea_shift, bp->nch))
      id = 103;
    else if (use_f64x(bp->engine, bp->precision, bp->DMAX, bp->TB, bp->VPL, bp->ea_shift))
      id = 303;
    else if (bp->ea_shift == 2)
      id = 13;
  }
  if (kernel_id) *kernel_id = id;
  if (row_chunks) *row_chunks = bp->nch;
  return 0;
}

int qldpc_bp_engine(const qldpc_bp* bp, int32_t* engine) {
  if (!bp || !engine) return set_err(QLDPC_EINVAL, "NULL argument");
  *engine = bp->engine;
  return 0;
}

int qldpc_bp_geometry(const qldpc_bp* bp, int32_t* threads, int32_t* vpl, int32_t* lds_bytes,
                      int32_t* blocks_per_cu) {
  if (!bp) return set_err(QLDPC_EINVAL, "NULL decoder");
  if (threads) *threads = bp->TB;
  if (vpl) *vpl = bp->VPL;
  if (lds_bytes) *lds_bytes = bp->lds_bytes;
  if (blocks_per_cu) *blocks_per_cu = bp->blocks_per_cu;
  return 0;
}

static SectorDev sector_of(const qldpc_bp* bp, const unsigned long long* lmask, int kw) {
  SectorDev s;
  s.vchk = static_cast<const uint32_t*>(bp->vchk.p);
  s.llr = bp->llr.p;
  s.lmask = lmask;
  s.m = bp->g->m;
  s.n = bp->g->n;
  s.kw = kw;
  s.max_iter = bp->max_iter;
  s.alpha = bp->alpha;
  return s;
}

static SSector ssector_of(const qldpc_bp* bp, const unsigned long long* lmask, int kw) {
  SSector s;
  s.edges = static_cast<const uint32_t*>(bp->vchk.p);
  s.llr = bp->llr.p;
  s.lmask = lmask;
  s.rdeg = static_cast<const uint8_t*>(bp->rdeg.p);
  s.perm = static_cast<const int32_t*>(bp->perm.p);
  s.rperm = static_cast<const int32_t*>(bp->rperm.p);
  s.d3k = bp->d3k;
  s.m = bp->g->m;
  s.n = bp->g->n;
  s.kw = kw;
  s.max_iter = bp->max_iter;
  s.nch = bp->nch;
  s.vpl = bp->VPL;
  s.alpha = bp->alpha;
  s.rows = static_cast<const uint32_t*>(bp->rowtab.p);
  s.vlast = bp->m2v_vlast;
  s.vnl = bp->m2v_nl;
  s.npos = bp->npos > 0 ? bp->npos : bp->g->n;
  s.nw = bp->nw;
  s.live_last = bp->live_last;
  return s;
}

// Shots (or syndromes) per chunk of a slot kernel: enough chunks to give every
// resident workgroup work, at most kChunkMax (the LDS fail bitmaps' size).
static int chunk_for(long long count, long long grid, int ns) {
  long long c = (count + grid - 1) / grid;
  c = std::max<long long>(c, ns);
  c = std::min<long long>(c, kChunkMax);
  return (int)c;
}

static int decode_batch(qldpc_bp* bp, const uint8_t* d_synd, uint8_t* d_corr, int32_t* d_iters, uint8_t* d_conv,
                        double* d_post, int64_t B, void* stream);

int qldpc_bp_decode_batch(qldpc_bp* bp, const uint8_t* d_synd, uint8_t* d_corr, int32_t* d_iters, uint8_t* d_conv,
                          int64_t B, void* stream) {
  return decode_batch(bp, d_synd, d_corr, d_iters, d_conv, nullptr, B, stream);
}

int qldpc_bp_decode_batch_soft(qldpc_bp* bp, const uint8_t* d_synd, uint8_t* d_corr, int32_t* d_iters,
                               uint8_t* d_conv, double* d_post, int64_t B, void* stream) {
  if (!bp || (B > 0 && !d_post)) return set_err(QLDPC_EINVAL, "NULL argument");
  // engine 1 (min-sum, qldpc_bp_create_soft) or engine 5 (product-sum: any qldpc_bp_create decoder with
  // bp_method 0 writes ldpc's log_prob_ratios on request)
  if (bp->engine != 1 && bp->engine != 5)
    return set_err(QLDPC_ENOTSUP, "soft output needs a decoder from qldpc_bp_create_soft (min-sum) or a product-sum decoder");
  return decode_batch(bp, d_synd, d_corr, d_iters, d_conv, d_post, B, stream);
}

static int decode_batch(qldpc_bp* bp, const uint8_t* d_synd, uint8_t* d_corr, int32_t* d_iters, uint8_t* d_conv,
                        double* d_post, int64_t B, void* stream) {
  if (!bp || (B > 0 && (!d_synd || !d_corr))) return set_err(QLDPC_EINVAL, "NULL argument");
  if (B == 0) return 0;
  QLDPC_HIP(hipSetDevice(bp->g->device));
  // max_iter = 1 min-sum (the circuit loop's h1 rounds: max_iter = int(18 / 10)): a one-iteration BP
  // from fresh state is the first-min step kernel (per-edge magnitudes fixed by the priors, bit-exact
  // with every engine); QLDPC_BP1=0 keeps the engine
  // (built with the decoder and on every qldpc_bp_set_channel_probs, bp1_prepare: no uploads here)
  if (!d_post && bp->bp1) return qldpc_rt::bp1_decode(bp->bp1, d_synd, d_corr, d_iters, d_conv, B, (hipStream_t)stream);
  if (bp->engine == 5) return ps_decode_launch(bp, d_synd, d_corr, d_iters, d_conv, B, (hipStream_t)stream, d_post);
  if (bp->engine == 6) return hbm_decode_launch(bp, d_synd, d_corr, d_iters, d_conv, B, (hipStream_t)stream);
  const long long cap = (long long)bp->blocks_per_cu * bp->cus;
  if (bp->engine == 1) {
    DecArgs a;
    a.sec = sector_of(bp, nullptr, 0);
    a.synd = d_synd;
    a.corr = d_corr;
    a.iters = d_iters;
    a.conv = d_conv;
    a.post = d_post;
    a.B = B;
    const int grid = (int)std::max<long long>(1, std::min<long long>(B, cap));
    Variant v = get_variant(bp->precision, bp->VPL, bp->DMAX);
    QLDPC_HIP(v.dec(dim3(grid), dim3(bp->TB), bp->lds_bytes, (hipStream_t)stream, a));
  } else {
    const int tsize = bp->precision == 32 ? 4 : 8;
    SDecArgs a;
    a.sec = ssector_of(bp, nullptr, 0);
    a.synd = d_synd;
    a.corr = d_corr;
    a.iters = d_iters;
    a.conv = d_conv;
    a.B = B;
    a.mmax = bp->g->m;
    a.vslots = bp->vslots_m2v ? bp->vslots_m2v : (1 + bp->g->m * bp->nch) * (16 / tsize) + bp->vslots_dummy;
    a.img_bytes = (int)slot_img_bytes(a.vslots, a.mmax, tsize);
    a.chunk = chunk_for(B, cap, bp->NS);
    a.work = nullptr;
#if QLDPC_STAMPS
    a.stamps = debug_stamps_buffer();
#else
    a.stamps = nullptr;
#endif
    if (bp->engine >= 3 && env_int("QLDPC_DYN", 1) != 0) {  // chunk queue, ~64 chunks per workgroup
      if (!bp->work.p && bp->work.alloc(16)) return QLDPC_ENOMEM;
      // at most kMaxQueuePops pops of the one queue counter per launch: small graphs run many
      // workgroups per CU and decode a syndrome in microseconds, and 65,536 one-syndrome pops of one
      // address serialised at ~12 ns each (0.8 ms per launch whatever max_iter; round 5 probe,
      // tools/dev/probe_small_dec.py)
      constexpr long long kMaxQueuePops = 8192;
      a.chunk = (int)std::max<long long>(1, std::min<long long>(kChunkMax, B / (cap * std::max(1, env_int("QLDPC_DYN_PER", 64)))));
      a.chunk = (int)std::min<long long>(kChunkMax, std::max<long long>(a.chunk, (B + kMaxQueuePops - 1) / kMaxQueuePops));
      QLDPC_HIP(hipMemsetAsync(bp->work.p, 0, 4, (hipStream_t)stream));
      a.work = static_cast<unsigned int*>(bp->work.p);
    }
    const long long nchunks = (B + a.chunk - 1) / a.chunk;
    const int grid = (int)std::max<long long>(1, std::min<long long>(nchunks, cap));
    SVariant v = slot_variant(bp->engine, bp->precision, bp->DMAX, bp->NS, bp->VPL, bp->d3k, bp->ea_shift, bp->TB, bp->nch,
                              bp->tail, bp->m2s, bp->fb, bp->d2k, bp->m2s_pk);
    QLDPC_HIP(v.dec(dim3(grid), dim3(bp->TB), bp->lds_bytes, (hipStream_t)stream, a));
  }
  return 0;
}

static int build_lmask(const qldpc_graph* L, int n, DevBuf& buf, int& kw) {
  if (!L) {
    kw = 0;
    return 0;
  }
  if (L->n != n) return set_err(QLDPC_EINVAL, "logical operator width != code length");
  kw = (L->m + 63) / 64;
  if (kw > 4) return set_err(QLDPC_ENOTSUP, "more than 256 logical operators");
  if (kw == 0) kw = 1;
  std::vector<unsigned long long> mask((size_t)n * kw, 0ull);
  for (int r = 0; r < L->m; ++r)
    for (int e = L->row_ptr[r]; e < L->row_ptr[r + 1]; ++e)
      mask[(size_t)L->col_idx[e] * kw + r / 64] |= 1ull << (r % 64);
  int rc = buf.alloc(mask.size() * 8);
  if (rc) return rc;
  QLDPC_HIP(hipMemcpy(buf.p, mask.data(), mask.size() * 8, hipMemcpyHostToDevice));
  return 0;
}

int qldpc_mc_create(qldpc_bp* dec_x, const qldpc_graph* logical_x, qldpc_bp* dec_z, const qldpc_graph* logical_z,
                    qldpc_mc** out) {
  if (!out || (!dec_x && !dec_z)) return set_err(QLDPC_EINVAL, "need at least one sector decoder");
  qldpc_bp* d0 = dec_x ? dec_x : dec_z;
  const bool staged = (dec_x && dec_x->engine >= 5) || (dec_z && dec_z->engine >= 5) ||
                      // (the space-time tail families, two-word or one-word: decode_batch kernels only)
                      (dec_x && dec_x->tail && (!dec_x->m2s || dec_x->nch == 4)) ||
                      (dec_z && dec_z->tail && (!dec_z->m2s || dec_z->nch == 4)) ||
                      // the fused kernel runs one layout family for both sectors
                      (dec_x && dec_z &&
                       (dec_x->m2s != dec_z->m2s || dec_x->tail != dec_z->tail || dec_x->fb != dec_z->fb ||
                        dec_x->m2s_pk != dec_z->m2s_pk)) ||
                      // one-slot families (m2s / c2s / m2v) keep no dummy edge on a real variable:
                      // the kernel's compile-time D3K must be each sector's own (a degree-3
                      // variable past it would run the 4-edge path and read the shared dummy slot)
                      (dec_x && dec_z && dec_x->m2s && dec_x->d3k != dec_z->d3k) ||
                      env_int("QLDPC_MC_STAGED", 0) == 1;
  if (staged) {  // staged pipeline around decode_batch (staged.hip): any decoder pair
    if (dec_x && dec_z && (dec_x->g->n != dec_z->g->n || dec_x->g->device != dec_z->g->device))
      return set_err(QLDPC_EINVAL, "sector decoders differ in code length or device");
    QLDPC_HIP(hipSetDevice(d0->g->device));
    auto* mc = new qldpc_mc();
    mc->dec[0] = dec_x;
    mc->dec[1] = dec_z;
    mc->engine = d0->engine;
    mc->precision = d0->precision;
    mc->TB = d0->TB;
    mc->VPL = d0->VPL;
    int rc = mc->counters.alloc(sizeof(qldpc_counters));
    if (!rc) rc = staged_mc_prepare(mc, logical_x, logical_z);
    if (rc) {
      staged_mc_release(mc);
      mc->counters.release();
      delete mc;
      return rc;
    }
    *out = mc;
    return 0;
  }
  if (dec_x && dec_z) {
    if (dec_x->g->n != dec_z->g->n) return set_err(QLDPC_EINVAL, "sector code lengths differ");
    if (dec_x->TB != dec_z->TB || dec_x->VPL != dec_z->VPL || dec_x->DMAX != dec_z->DMAX ||
        dec_x->precision != dec_z->precision || dec_x->engine != dec_z->engine)
      return set_err(QLDPC_EINVAL, "sector decoders need identical geometry/precision (same vars_per_thread)");
    if (dec_x->g->device != dec_z->g->device) return set_err(QLDPC_EINVAL, "sector decoders on different devices");
    if (dec_x->m2s != dec_z->m2s || dec_x->tail != dec_z->tail || dec_x->fb != dec_z->fb)
      return set_err(QLDPC_EINVAL, "sector decoders use different LDS layouts (QLDPC_M2S)");
  }
  QLDPC_HIP(hipSetDevice(d0->g->device));
  auto* mc = new qldpc_mc();
  auto fail = [&](int code) {
    mc->lmask[0].release();
    mc->lmask[1].release();
    mc->counters.release();
    mc->work.release();
    delete mc;
    return code;
  };
  mc->dec[0] = dec_x;
  mc->dec[1] = dec_z;
  int rc = 0;
  if (dec_x && (rc = build_lmask(logical_x, dec_x->g->n, mc->lmask[0], mc->kw[0]))) return fail(rc);
  if (dec_z && (rc = build_lmask(logical_z, dec_z->g->n, mc->lmask[1], mc->kw[1]))) return fail(rc);
  mc->engine = d0->engine;
  mc->TB = d0->TB;
  mc->VPL = d0->VPL;
  mc->DMAX = d0->DMAX;
  mc->ea_shift = std::max(dec_x ? dec_x->ea_shift : 0, dec_z ? dec_z->ea_shift : 0);
  if (dec_x && dec_z && dec_x->ea_shift != dec_z->ea_shift)
    return fail(set_err(QLDPC_EINVAL, "sector decoders use different LDS address scales"));
  // one kernel serves both sectors: only slots that hold degree <= 3 variables in both skip slot 4
  mc->d3k = std::min(dec_x ? dec_x->d3k : 1 << 20, dec_z ? dec_z->d3k : 1 << 20);
  mc->precision = d0->precision;
  // compile-time row width (fp64 <= 256-thread family): one kernel serves both sectors
  mc->nch = d0->nch;
  if (dec_x && dec_z && dec_x->nch != dec_z->nch) mc->nch = 0;
  mc->mmax = std::max(dec_x ? dec_x->g->m : 0, dec_z ? dec_z->g->m : 0);
  mc->tail = d0->tail;
  mc->m2s = d0->m2s;
  mc->m2s_pk = d0->m2s_pk;
  mc->fb = d0->fb;
  const void* kern;
  if (mc->engine == 1) {
    mc->lds_bytes = (int)lds_for(mc->precision, mc->mmax);
    kern = get_variant(mc->precision, mc->VPL, mc->DMAX).mc_k;
  } else {
    const int tsize = mc->precision == 32 ? 4 : 8;
    for (qldpc_bp* d : {dec_x, dec_z})
      if (d)
        mc->vslots = std::max(mc->vslots,
                              d->vslots_m2v ? d->vslots_m2v : (1 + d->g->m * d->nch) * (16 / tsize) + d->vslots_dummy);
    mc->img_bytes = (int)slot_img_bytes(mc->vslots, mc->mmax, tsize);
    if (mc->engine >= 3) {
      if (!r_fits(mc->engine, mc->vslots, mc->mmax, tsize, mc->ea_shift, mc->tail, mc->m2s, mc->fb))
        return fail(set_err(QLDPC_ENOTSUP, "sector images exceed the register engines' 64 KiB addressing (QLDPC_ENGINE=2)"));
      mc->NS = 1;
      mc->lds_bytes =
          (int)r_lds_bytes((int)r_layout(mc->engine, mc->vslots, mc->mmax, tsize, mc->tail, mc->m2s, mc->fb).total, kChunkMax);
    } else {
      mc->NS = choose_ns(mc->img_bytes);
      mc->lds_bytes = (int)slot_lds_bytes(mc->NS, mc->img_bytes, kChunkMax);
    }
    kern = slot_variant(mc->engine, mc->precision, mc->DMAX, mc->NS, mc->VPL, mc->d3k, mc->ea_shift, mc->TB, mc->nch,
                        mc->tail, mc->m2s, mc->fb, 0, mc->m2s_pk).mc_k;
  }
  if (mc->lds_bytes > kLdsMax) return fail(set_err(QLDPC_ENOTSUP, "per-shot LDS image exceeds 160 KiB"));
  if (!kern) return fail(set_err(QLDPC_ENOTSUP, "no kernel variant"));
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, mc->TB, mc->lds_bytes) != hipSuccess) nb = 1;
  mc->blocks_per_cu = std::max(1, nb);
  mc->cus = d0->cus;
  if ((rc = mc->counters.alloc(sizeof(qldpc_counters))) || (rc = mc->work.alloc(16))) return fail(rc);
  *out = mc;
  return 0;
}

int qldpc_mc_set_osd(qldpc_mc* mc, qldpc_osd_gpu* osd_x, qldpc_osd_gpu* osd_z) {
  if (!mc) return set_err(QLDPC_EINVAL, "NULL mc");
  qldpc_osd_gpu* o[2] = {osd_x, osd_z};
  for (int q = 0; q < 2; ++q) {
    if (!o[q]) continue;
    if (mc->staged || mc->engine != 3)
      return set_err(QLDPC_ENOTSUP, "BP+OSD shot loop needs the fused engine-3 MC kernel");
    if (!mc->dec[q] || !osd_gpu_matches(o[q], mc->dec[q]->g))
      return set_err(QLDPC_EINVAL, q == 0 ? "X-sector OSD handle was built on a different graph than dec_x"
                                          : "Z-sector OSD handle was built on a different graph than dec_z");
  }
  mc->osd[0] = osd_x;
  mc->osd[1] = osd_z;
  mc->c_cap = 0;  // the next launch (re)allocates the capture buffers of every enabled sector
  return 0;
}

int qldpc_mc_destroy(qldpc_mc* mc) {
  if (!mc) return 0;
  for (int q = 0; q < 2; ++q)
    for (DevBuf* d : {&mc->c_post[q], &mc->c_synd[q], &mc->c_err[q], &mc->c_shot[q], &mc->c_outw[q]}) d->release();
  mc->c_n.release();
  mc->c_fail.release();
  mc->lmask[0].release();
  mc->lmask[1].release();
  mc->counters.release();
  mc->work.release();
  mc->cls_cache.release();
  staged_mc_release(mc);
  delete mc;
  return 0;
}

static unsigned long long ceil_2p53(double t) {
  if (!(t > 0.0)) return 0ull;
  if (t >= 1.0) return 1ull << 53;
  return (unsigned long long)std::ceil(std::ldexp(t, 53));
}

int qldpc_mc_launch(qldpc_mc* mc, double px, double py, double pz, uint64_t seed, uint64_t shot_begin,
                    int64_t shot_count, int32_t logical_mode, const double* d_uniforms, void* d_counters,
                    uint8_t* d_fail, uint8_t* d_err, uint8_t* d_corr, int32_t* d_iters, int32_t grid_blocks,
                    void* stream) {
  if (!mc || !d_counters) return set_err(QLDPC_EINVAL, "NULL argument");
  if (logical_mode < 0 || logical_mode > 2) return set_err(QLDPC_EINVAL, "logical_mode must be 0 (X), 1 (Z), 2 (Total)");
  if (!(px >= 0 && py >= 0 && pz >= 0)) return set_err(QLDPC_EINVAL, "negative Pauli probability");
  if (shot_count <= 0) return 0;
  const bool need[2] = {logical_mode != 1, logical_mode != 0};
  for (int q = 0; q < 2; ++q) {
    if (!need[q]) continue;
    if (!mc->dec[q]) return set_err(QLDPC_EINVAL, q == 0 ? "logical_mode needs the X sector (hz decoder)"
                                                          : "logical_mode needs the Z sector (hx decoder)");
    if (!mc->staged && !mc->lmask[q].p) return set_err(QLDPC_EINVAL, "sector has no logical operators");
  }
  if (mc->staged) {
    QLDPC_HIP(hipSetDevice((mc->dec[0] ? mc->dec[0] : mc->dec[1])->g->device));
    return staged_mc_launch(mc, px, py, pz, seed, shot_begin, shot_count, logical_mode, d_uniforms, d_counters, d_fail,
                            d_err, d_corr, d_iters, (hipStream_t)stream);
  }
  QLDPC_HIP(hipSetDevice((mc->dec[0] ? mc->dec[0] : mc->dec[1])->g->device));
  const bool bposd = mc->engine != 1 && ((need[0] && mc->osd[0]) || (need[1] && mc->osd[1]));
  if (bposd) {
    // capture slots per sector, bounded by a memory budget (QLDPC_OSD_CAPTURE_MB per sector,
    // default 2048); a launch larger than that runs as pieces of at most c_cap shots, each
    // shot claims at most one slot per sector, so no candidate can ever be dropped
    long long slot_bytes = 0;
    for (int q = 0; q < 2; ++q)
      if (need[q] && mc->osd[q]) {
        const long long n = mc->dec[q]->g->n, m = mc->dec[q]->g->m;
        slot_bytes = std::max(slot_bytes, n * 8 + m + n + 8 + n);
      }
    const long long budget = (long long)std::max(1, env_int("QLDPC_OSD_CAPTURE_MB", 2048)) << 20;
    const long long slots = std::max<long long>(1024, budget / slot_bytes);
    if (shot_count > slots) {
      const long long n = (mc->dec[0] ? mc->dec[0] : mc->dec[1])->g->n;
      for (long long off = 0; off < shot_count; off += slots) {
        const long long c = std::min(slots, shot_count - off);
        int rc = qldpc_mc_launch(mc, px, py, pz, seed, shot_begin + (uint64_t)off, c, logical_mode,
                                 d_uniforms ? d_uniforms + off * n : nullptr, d_counters, d_fail ? d_fail + off : nullptr,
                                 d_err ? d_err + off * n : nullptr, d_corr ? d_corr + off * 2 * n : nullptr,
                                 d_iters ? d_iters + off * 2 : nullptr, grid_blocks, stream);
        if (rc) return rc;
      }
      return 0;
    }
  }
  const long long cap = (long long)mc->blocks_per_cu * mc->cus;
  // thresholds of the 3-way split, in the evaluation order of src/Simulators.py:102-108
  const double t1 = pz, t2 = pz + px, t3 = (pz + px) + py;
  if (mc->engine == 1) {
    McArgs a;
    std::memset(&a, 0, sizeof(a));
    for (int q = 0; q < 2; ++q) {
      if (!need[q]) continue;
      a.sec[a.nsec] = sector_of(mc->dec[q], static_cast<const unsigned long long*>(mc->lmask[q].p), mc->kw[q]);
      a.sec_id[a.nsec++] = q;
    }
    a.logical_mode = logical_mode;
    a.mmax = mc->mmax;
    a.t1 = t1; a.t2 = t2; a.t3 = t3;
    a.K1 = ceil_2p53(t1); a.K2 = ceil_2p53(t2); a.K3 = ceil_2p53(t3);
    a.seed = seed; a.shot_begin = shot_begin; a.shot_count = shot_count;
    a.uniforms = d_uniforms;
    a.counters = static_cast<unsigned long long*>(d_counters);
    a.fail = d_fail; a.err = d_err; a.corr = d_corr; a.iters = d_iters;
    long long grid = grid_blocks > 0 ? grid_blocks : cap;
    grid = std::max<long long>(1, std::min<long long>(grid, shot_count));
    Variant v = get_variant(mc->precision, mc->VPL, mc->DMAX);
    QLDPC_HIP(v.mc(dim3((unsigned)grid), dim3(mc->TB), mc->lds_bytes, (hipStream_t)stream, a));
  } else {
    SMcArgs a;
    std::memset(&a, 0, sizeof(a));
    int ids[2] = {0, 0};
    for (int q = 0; q < 2; ++q) {
      if (!need[q]) continue;
      a.sec[a.nsec] = ssector_of(mc->dec[q], static_cast<const unsigned long long*>(mc->lmask[q].p), mc->kw[q]);
      ids[a.nsec++] = q;
    }
    a.sec_id0 = ids[0];
    a.sec_id1 = ids[1];
    a.logical_mode = logical_mode;
    a.mmax = mc->mmax;
    a.vslots = mc->vslots;
    a.img_bytes = mc->img_bytes;
    const long long want = grid_blocks > 0 ? grid_blocks : cap;
    a.chunk = chunk_for(shot_count, want, mc->NS);
    // engine 3: chunks from a queue, ~64 per workgroup (no tail behind the slowest static share)
    if (mc->engine >= 3 && mc->work.p && env_int("QLDPC_DYN", 1) != 0) {
      const int per = std::max(1, env_int("QLDPC_DYN_PER", 64));  // measured plateau 64-128 (n1600)
      a.chunk = (int)std::max<long long>(1, std::min<long long>(kChunkMax, shot_count / (want * per)));
      QLDPC_HIP(hipMemsetAsync(mc->work.p, 0, 4, (hipStream_t)stream));
      a.work = static_cast<unsigned int*>(mc->work.p);
    }
    a.t1 = t1; a.t2 = t2; a.t3 = t3;
    a.K1 = ceil_2p53(t1); a.K2 = ceil_2p53(t2); a.K3 = ceil_2p53(t3);
    a.seed = seed; a.shot_begin = shot_begin; a.shot_count = shot_count;
    a.uniforms = d_uniforms;
    a.counters = static_cast<unsigned long long*>(d_counters);
    a.fail = d_fail; a.err = d_err; a.corr = d_corr; a.iters = d_iters;
#if QLDPC_STAMPS
    a.stamps = debug_stamps_buffer();
#endif
    const long long nchunks = (shot_count + a.chunk - 1) / a.chunk;
    if (nchunks > 0x7fffffffLL) return set_err(QLDPC_EINVAL, "too many shots for one launch (chunk count >= 2^31)");
    const long long grid = std::max<long long>(1, std::min<long long>(nchunks, want));
    // both sectors drawing Philox errors: the first sector's pass caches each shot's classes for the
    // second (SMcArgs::cls_cache; [grid][chunk][TB] u16, one Philox draw per (shot, variable) instead of
    // two; QLDPC_CLS_CACHE=0 draws in both passes)
    a.cls_cache = nullptr;
    const size_t cc_need = (size_t)grid * (size_t)a.chunk * (size_t)mc->TB * 2;
    // (bounded: 256 MiB covers every bundled code at the bench's launch sizes; huge launches of small
    // codes, e.g. 10^9 shots of GenBicycleA1 at 1024-shot chunks, would need ~0.7 GB: they draw twice)
    if (a.nsec == 2 && !d_uniforms && mc->VPL <= 8 && env_int("QLDPC_CLS_CACHE", 1) != 0 && cc_need <= (256u << 20)) {
      const size_t need = cc_need;
      if (mc->cls_cache.bytes < need) {
        mc->cls_cache.release();
        int rc = mc->cls_cache.alloc(need);
        if (rc) return rc;
      }
      a.cls_cache = static_cast<uint16_t*>(mc->cls_cache.p);
    }
    // BP+OSD: capture buffers with one slot per shot of this launch (<= the budgeted slots)
    hipStream_t st = (hipStream_t)stream;
    if (bposd) {
      if (mc->c_cap < shot_count) {
        for (int q = 0; q < 2; ++q) {
          for (DevBuf* d : {&mc->c_post[q], &mc->c_synd[q], &mc->c_err[q], &mc->c_shot[q], &mc->c_outw[q]}) d->release();
          if (!mc->dec[q] || !mc->osd[q]) continue;
          const int n = mc->dec[q]->g->n, m = mc->dec[q]->g->m;
          int rc;
          if ((rc = mc->c_post[q].alloc((size_t)shot_count * n * 8)) || (rc = mc->c_synd[q].alloc((size_t)shot_count * m)) ||
              (rc = mc->c_err[q].alloc((size_t)shot_count * n)) || (rc = mc->c_shot[q].alloc((size_t)shot_count * 8)) ||
              (rc = mc->c_outw[q].alloc((size_t)shot_count * n)))
            return rc;
        }
        mc->c_fail.release();
        int rc;
        if ((rc = mc->c_fail.alloc((size_t)shot_count)) || (!mc->c_n.p && (rc = mc->c_n.alloc(16)))) return rc;
        mc->c_cap = shot_count;
      }
      QLDPC_HIP(hipMemsetAsync(mc->c_n.p, 0, 16, st));
      a.c_n = static_cast<unsigned int*>(mc->c_n.p);
      a.c_cap = shot_count;
      for (int q = 0; q < 2; ++q) {
        const bool on = need[q] && mc->osd[q];
        a.c_post[q] = on ? static_cast<double*>(mc->c_post[q].p) : nullptr;
        a.c_synd[q] = on ? static_cast<uint8_t*>(mc->c_synd[q].p) : nullptr;
        a.c_err[q] = on ? static_cast<uint8_t*>(mc->c_err[q].p) : nullptr;
        a.c_shot[q] = on ? static_cast<long long*>(mc->c_shot[q].p) : nullptr;
      }
      if (!a.fail) a.fail = static_cast<uint8_t*>(mc->c_fail.p);  // per-shot verdicts the OSD stage revises
    }
    SVariant v = slot_variant(mc->engine, mc->precision, mc->DMAX, mc->NS, mc->VPL, mc->d3k, mc->ea_shift, mc->TB, mc->nch,
                              mc->tail, mc->m2s, mc->fb, 0, mc->m2s_pk);
    QLDPC_HIP(v.mc(dim3((unsigned)grid), dim3(mc->TB), mc->lds_bytes, st, a));
    if (bposd) {
      unsigned int nc[4] = {0, 0, 0, 0};
      QLDPC_HIP(hipMemcpyAsync(nc, mc->c_n.p, 16, hipMemcpyDeviceToHost, st));
      QLDPC_HIP(hipStreamSynchronize(st));
      for (int q = 0; q < 2; ++q) {
        if (!(need[q] && mc->osd[q]) || nc[q] == 0) continue;
        if ((long long)nc[q] > a.c_cap)  // cannot happen (one slot per shot and sector): never drop silently
          return set_err(QLDPC_EINVAL, "BP+OSD capture overflow: more candidates than capture slots");
        const long long ncand = nc[q];
        int rc = osd_gpu_bposd_stage(mc->osd[q], static_cast<const uint8_t*>(mc->c_synd[q].p),
                                     static_cast<const double*>(mc->c_post[q].p), static_cast<const uint8_t*>(mc->c_err[q].p),
                                     static_cast<const long long*>(mc->c_shot[q].p), static_cast<uint8_t*>(mc->c_outw[q].p),
                                     ncand, static_cast<const unsigned long long*>(mc->lmask[q].p), mc->kw[q], q,
                                     logical_mode, a.fail, static_cast<unsigned long long*>(d_counters), st);
        if (rc) return rc;
      }
    }
  }
  return 0;
}

int qldpc_mc_run(qldpc_mc* mc, double px, double py, double pz, uint64_t seed, uint64_t shot_begin,
                 int64_t shot_count, int32_t logical_mode, qldpc_counters* out, void* stream) {
  if (!mc || !out) return set_err(QLDPC_EINVAL, "NULL argument");
  hipStream_t s = (hipStream_t)stream;
  QLDPC_HIP(hipMemsetAsync(mc->counters.p, 0, sizeof(qldpc_counters), s));
  int rc = qldpc_mc_launch(mc, px, py, pz, seed, shot_begin, shot_count, logical_mode, nullptr, mc->counters.p,
                           nullptr, nullptr, nullptr, nullptr, 0, stream);
  if (rc) return rc;
  qldpc_counters c;
  QLDPC_HIP(hipMemcpyAsync(&c, mc->counters.p, sizeof(c), hipMemcpyDeviceToHost, s));
  QLDPC_HIP(hipStreamSynchronize(s));
  out->shots += c.shots;
  out->failures += c.failures;
  for (int q = 0; q < 2; ++q) {
    out->sector_decodes[q] += c.sector_decodes[q];
    out->sector_iters[q] += c.sector_iters[q];
    out->sector_nonconv[q] += c.sector_nonconv[q];
    out->sector_fail[q] += c.sector_fail[q];
    for (int b = 0; b < QLDPC_HIST_BINS; ++b) out->iter_hist[q][b] += c.iter_hist[q][b];
  }
  return 0;
}

}  // extern "C"
