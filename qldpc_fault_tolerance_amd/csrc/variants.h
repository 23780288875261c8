// variants.h — launchable kernel variants (fp32/fp64 × vars-per-thread × max column degree).
// Each kern_*.hip translation unit instantiates one (T, DMAX) family so the
// build compiles them in parallel.
//   v1 (bp_kernels.h): per-check LDS state updated by returning LDS atomics;
//   v4 (bp_slot.h):    row-major v2c slots, check-centric gather, streamed
//                      variables, NS shots in flight per workgroup;
//   v5 (bp_reg.h):     v4's LDS image with register-resident variables and
//                      a compile-time VPL (default when the graph fits).
#pragma once
#include "bp_reg.h"

// measured-and-not-kept kernel families (c2s, m2v, fp64 x 512 threads, engine 4): out of the
// product build unless -DQLDPC_EXPERIMENTAL=1
#ifndef QLDPC_EXPERIMENTAL
#define QLDPC_EXPERIMENTAL 0
#endif

namespace qldpc {

using DecLaunch = hipError_t (*)(dim3, dim3, size_t, hipStream_t, const DecArgs&);
using McLaunch = hipError_t (*)(dim3, dim3, size_t, hipStream_t, const McArgs&);
using SDecLaunch = hipError_t (*)(dim3, dim3, size_t, hipStream_t, const SDecArgs&);
using SMcLaunch = hipError_t (*)(dim3, dim3, size_t, hipStream_t, const SMcArgs&);

struct Variant {
  DecLaunch dec;
  McLaunch mc;
  const void* dec_k;
  const void* mc_k;
};

struct SVariant {
  SDecLaunch dec;
  SMcLaunch mc;
  const void* dec_k;
  const void* mc_k;
};

Variant get_variant_f32_d4(int vpl);
Variant get_variant_f32_d8(int vpl);
Variant get_variant_f64_d4(int vpl);
Variant get_variant_f64_d8(int vpl);
SVariant get_rvariant_f32(int vpl, int d3k);  // kern_r_f32_{a,b,c}.hip by VPL range
SVariant get_rvariant_f32_a(int vpl, int d3k);
SVariant get_rvariant_f32_b(int vpl, int d3k);
SVariant get_rvariant_f32_c(int vpl, int d3k);
SVariant get_rvariant_f32_big(int vpl, int d3k);  // kern_r_f32_big.hip: images of 64-256 KiB
SVariant get_rvariant_f32_d5(int vpl, int d3k);  // kern_r_f32_d56.hip: column degree 5
SVariant get_rvariant_f32_d6(int vpl, int d3k);  //                      column degree 6
SVariant get_rvariant_f64(int vpl);
SVariant get_rvariant_f32_w(int vpl, int d3k);  // kern_r_f32_w.hip: compile-time 2-chunk rows
SVariant get_rvariant_f64_w(int vpl, int d3k, int nch);  // kern_r_f64_w{3,4}.hip: <= 256 threads, own v2c in VGPRs, D3K
SVariant get_rvariant_f64_w3(int vpl, int d3k);
SVariant get_rvariant_f64_w_d5(int vpl, int d3k, int nch);  // kern_r_f64_d5.hip: column degree 5
SVariant get_rvariant_f64_x(int vpl, int d3k);  // kern_r_f64_x.hip: 257-512 threads, 128 VGPRs (opt-in)
SVariant get_rvariant_f64_w4(int vpl, int d3k);
SVariant get_rvariant_f64_st(int vpl, int d3k, int d2k = 0);  // kern_r_f64_st*.hip: tail layout, 1024 threads (engine id 1013)
SVariant get_rvariant_f64_st_hi(int vpl, int d3k);
SVariant get_rvariant_f32_st(int vpl, int d3k);  // kern_r_f32_st.hip: tail layout in float (engine id 1013)
SVariant get_rvariant_f64_m2st(int vpl, int d3k, int d2k);  // kern_r_f64_m2st.hip: m2s on the fp64 space-time tail layout, 1024 threads (engine id 111313)
SVariant get_rvariant_f64_m2s(int vpl, int d3k);  // kern_r_f64_m2s.hip: m2 in the argmin slot, rows of 3 chunks + tail (engine id 11103)
SVariant get_rvariant_f64_m2s8(int vpl, int d3k);  // kern_r_f64_m2s8.hip: m2s, rows of 4 chunks (8 edges), column degree 5 (engine id 10103)
SVariant get_rvariant_f64_m2s8pk(int vpl, int d3k);  // the same with packed absolute edge addresses, 4 per CU (engine id 10203)
SVariant get_rvariant_f64_m2v(int vpl, int d3k);  // kern_r_f64_m2v.hip: m2s with variable-major V slots (engine id 40103)
SVariant get_rvariant_f64_c2s(int vpl, int d3k);  // kern_r_f64_c2s.hip: c2v written by the check phase into the slots (engine id 31103)
SVariant get_rvariant_f32_stfb(int vpl, int d3k, int d2k);  // kern_r_f32_stfb.hip: fp32 tail layout, byte F, 512 threads (engine id 21013 + 100000 * D2K)
SVariant get_r4variant_f32(int vpl);
SVariant get_r4variant_f64(int vpl);
SVariant get_r4variant_f64_w(int vpl);  // <= 256 threads
SVariant get_svariant_f32_d4(int ns);
SVariant get_svariant_f32_d8(int ns);
SVariant get_svariant_f64_d4(int ns);
SVariant get_svariant_f64_d8(int ns);

#ifdef QLDPC_VARIANT_TU
template <typename T, int VPL, int DMAX>
hipError_t launch_dec(dim3 g, dim3 b, size_t lds, hipStream_t s, const DecArgs& a) {
  hipLaunchKernelGGL((bp_decode_kernel<T, VPL, DMAX>), g, b, lds, s, a);
  return hipGetLastError();
}
template <typename T, int VPL, int DMAX>
hipError_t launch_mc(dim3 g, dim3 b, size_t lds, hipStream_t s, const McArgs& a) {
  hipLaunchKernelGGL((mc_kernel<T, VPL, DMAX>), g, b, lds, s, a);
  return hipGetLastError();
}
template <typename T, int VPL, int DMAX>
Variant make_variant() {
  return Variant{&launch_dec<T, VPL, DMAX>, &launch_mc<T, VPL, DMAX>,
                 reinterpret_cast<const void*>(&bp_decode_kernel<T, VPL, DMAX>),
                 reinterpret_cast<const void*>(&mc_kernel<T, VPL, DMAX>)};
}
template <typename T, int DMAX>
Variant pick_vpl(int vpl) {
  switch (vpl) {
    case 1: return make_variant<T, 1, DMAX>();
    case 2: return make_variant<T, 2, DMAX>();
    case 3: return make_variant<T, 3, DMAX>();
    case 4: return make_variant<T, 4, DMAX>();
    case 5: return make_variant<T, 5, DMAX>();
    case 6: return make_variant<T, 6, DMAX>();
    case 7: return make_variant<T, 7, DMAX>();
    case 8: return make_variant<T, 8, DMAX>();
    case 10: return make_variant<T, 10, DMAX>();
    case 12: return make_variant<T, 12, DMAX>();
    default: return Variant{nullptr, nullptr, nullptr, nullptr};
  }
}

template <typename T, int DMAX, int NS>
hipError_t slaunch_dec(dim3 g, dim3 b, size_t lds, hipStream_t s, const SDecArgs& a) {
  hipLaunchKernelGGL((sdec_kernel<T, DMAX, NS>), g, b, lds, s, a);
  return hipGetLastError();
}
template <typename T, int DMAX, int NS>
hipError_t slaunch_mc(dim3 g, dim3 b, size_t lds, hipStream_t s, const SMcArgs& a) {
  hipLaunchKernelGGL((smc_kernel<T, DMAX, NS>), g, b, lds, s, a);
  return hipGetLastError();
}
template <typename T, int DMAX, int NS>
SVariant make_svariant() {
  return SVariant{&slaunch_dec<T, DMAX, NS>, &slaunch_mc<T, DMAX, NS>,
                  reinterpret_cast<const void*>(&sdec_kernel<T, DMAX, NS>),
                  reinterpret_cast<const void*>(&smc_kernel<T, DMAX, NS>)};
}
template <typename T, int DMAX>
SVariant pick_sns(int ns) {
  switch (ns) {
    case 1: return make_svariant<T, DMAX, 1>();
    case 2: return make_svariant<T, DMAX, 2>();
    case 4: return make_svariant<T, DMAX, 4>();
    default: return SVariant{nullptr, nullptr, nullptr, nullptr};
  }
}

template <typename T, int VPL, int ENG, int D3K, int DM = 4, int LB = kMaxThreadsS, int NCH = 0>
hipError_t rlaunch_dec(dim3 g, dim3 b, size_t lds, hipStream_t s, const SDecArgs& a) {
  hipLaunchKernelGGL((rdec_kernel<T, DM, VPL, ENG, D3K, LB, NCH>), g, b, lds, s, a);
  return hipGetLastError();
}
template <typename T, int VPL, int ENG, int D3K, int DM = 4, int LB = kMaxThreadsS, int NCH = 0>
hipError_t rlaunch_mc(dim3 g, dim3 b, size_t lds, hipStream_t s, const SMcArgs& a) {
  hipLaunchKernelGGL((rmc_kernel<T, DM, VPL, ENG, D3K, LB, NCH>), g, b, lds, s, a);
  return hipGetLastError();
}
template <typename T, int VPL, int ENG, int D3K, int DM = 4, int LB = kMaxThreadsS, int NCH = 0>
SVariant make_rvariant() {
  return SVariant{&rlaunch_dec<T, VPL, ENG, D3K, DM, LB, NCH>, &rlaunch_mc<T, VPL, ENG, D3K, DM, LB, NCH>,
                  reinterpret_cast<const void*>(&rdec_kernel<T, DM, VPL, ENG, D3K, LB, NCH>),
                  reinterpret_cast<const void*>(&rmc_kernel<T, DM, VPL, ENG, D3K, LB, NCH>)};
}
// D3K = 0 only (fp64 and engine 4)
template <typename T, int ENG>
SVariant pick_rvpl(int vpl) {
  switch (vpl) {
    case 1: return make_rvariant<T, 1, ENG, 0>();
    case 2: return make_rvariant<T, 2, ENG, 0>();
    case 3: return make_rvariant<T, 3, ENG, 0>();
    case 4: return make_rvariant<T, 4, ENG, 0>();
    case 5: return make_rvariant<T, 5, ENG, 0>();
    case 6: return make_rvariant<T, 6, ENG, 0>();
    case 7: return make_rvariant<T, 7, ENG, 0>();
    case 8: return make_rvariant<T, 8, ENG, 0>();
    default: return SVariant{nullptr, nullptr, nullptr, nullptr};
  }
}
// every D3K in 0..VPL for one VPL (DM = edge slots per variable: 4, or 5/6 for degree-5/6 columns)
template <typename T, int VPL, int ENG, int DM = 4, int LB = kMaxThreadsS, int NCH = 0>
SVariant pick_rd3k(int d3k) {
  switch (d3k < 0 ? 0 : d3k > VPL ? VPL : d3k) {
    case 0: return make_rvariant<T, VPL, ENG, 0, DM, LB, NCH>();
    case 1: return make_rvariant<T, VPL, ENG, (1 <= VPL ? 1 : 0), DM, LB, NCH>();
    case 2: return make_rvariant<T, VPL, ENG, (2 <= VPL ? 2 : 0), DM, LB, NCH>();
    case 3: return make_rvariant<T, VPL, ENG, (3 <= VPL ? 3 : 0), DM, LB, NCH>();
    case 4: return make_rvariant<T, VPL, ENG, (4 <= VPL ? 4 : 0), DM, LB, NCH>();
    case 5: return make_rvariant<T, VPL, ENG, (5 <= VPL ? 5 : 0), DM, LB, NCH>();
    case 6: return make_rvariant<T, VPL, ENG, (6 <= VPL ? 6 : 0), DM, LB, NCH>();
    case 7: return make_rvariant<T, VPL, ENG, (7 <= VPL ? 7 : 0), DM, LB, NCH>();
    default: return make_rvariant<T, VPL, ENG, (8 <= VPL ? 8 : 0), DM, LB, NCH>();
  }
}
#endif

}  // namespace qldpc
