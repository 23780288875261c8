// bp_reg.h — engine 3: register-resident variables (gfx950).
//
// Same flooding min-sum as engine 2 (bp_slot.h: compressed check state
// {m1 | parity<<sign, m2}, row-major v2c slots, canonical messages, dummies for
// missing edges) with the per-variable state moved out of the memory system:
//   * each thread's VPL (compile-time) variables keep, in VGPRs for the whole
//     pass, their DMAX edge words pre-converted to absolute LDS byte addresses
//     (CS address | V address << 16), their prior, and (float) their own
//     previous v2c messages — the variable phase issues one random LDS read per
//     edge (the CS gather) and one write (the new v2c), no global traffic;
//   * the CS gathers of variable k+1 are issued before variable k's arithmetic
//     (software pipeline), so LDS latency hides under VALU work;
//   * padding variables (j >= n) have only dummy edges and prior +1, so no
//     per-variable bounds test remains in the hot loop;
//   * redundant ops of ldpc's backward pass (`0 + c`, `f + 0`) are dropped: they
//     change at most the sign of a zero, which the canonical encoding (sign :=
//     v <= 0) erases, so the stored messages and decisions stay bit-identical.
// The LDS image puts CS first so that its byte address is the edge word's low
// half: [CS (m+1) pairs][V: 16-byte sink + m rows][F (m+1)][lred 8][flags 2].
// One decode in flight per workgroup; several workgroups share a CU.
//
// Engine 4 (same file, ENG = 4) moves the c2v arithmetic into the check phase:
// the check thread, which holds its whole row in registers, computes every
// edge's c2v (m2 if the edge holds m1 else m1, times ±alpha) and writes them
// back into the row's slots; the variable phase then reads its c2v with one
// 4-byte LDS read per edge and overwrites the slot with the new v2c.  No CS
// array and no own-message registers remain, the random LDS reads halve in
// width, and the image shrinks by 8 bytes per check.  Padding slots of a row
// (logical position >= row degree) are rewritten with the sentinel, so the
// next min pass ignores them.  Missing edges read a constant zero chunk and
// write a sink.  Image: [V: zero chunk + m rows][F (m+1): bit0 (H x)_i, bit1
// syndrome, bits 16.. row degree][sink 16][lred 8][flags 2].
#pragma once

#ifndef QLDPC_TID_LAUNDER
#define QLDPC_TID_LAUNDER 1
#endif
// Diagnostic build only (tools/build_variant.py ... QLDPC_STAMPS=1): s_memtime stamps at the
// phase boundaries of the fused MC pass, summed per wave into SMcArgs::stamps.  Never on in
// the shipped library; its run times are not quoted (the stamps' waits forbid overlaps).
#ifndef QLDPC_STAMPS
#define QLDPC_STAMPS 0
#endif
#ifndef QLDPC_FLIP_BRANCHFREE
#define QLDPC_FLIP_BRANCHFREE 0
#endif
// A/B build: the F-word xors of flipped variables after the whole variable loop (one divergent
// region) instead of after each variable
#ifndef QLDPC_FLIPLATE
#define QLDPC_FLIPLATE 0
#endif
// A/B build: the m2s check phase derives tid from an SGPR wave base + mbcnt
#ifndef QLDPC_M2S_MBCNT
#define QLDPC_M2S_MBCNT 0
#endif
// c2s family: variables whose c2v reads are issued ahead of the current one's arithmetic
#ifndef QLDPC_C2S_PF
#define QLDPC_C2S_PF 2
#endif
// fp32 c2v in 4 VALU per edge (r_var_one); the check phases then store m2 | parity
#ifndef QLDPC_F32_C2V4
#define QLDPC_F32_C2V4 1
#endif
// fp64 c2v in 5 VALU per edge (r_var_one, two-word families); the check phases store m2 | parity
#ifndef QLDPC_F64_C2V5
#define QLDPC_F64_C2V5 1
#endif
// dword-scaled packed edge words (space-time families) hold absolute dword indices (SDWA unpack)
#ifndef QLDPC_ABS_SH2
#define QLDPC_ABS_SH2 1
#endif
// c2s check phase: the row's c2v as one 16-byte store per chunk (else 4-byte stores the
// compiler pairs)
#ifndef QLDPC_C2S_W128
#define QLDPC_C2S_W128 1
#endif
// m2s family: one uniform prior in SGPRs instead of one per variable slot in VGPRs
#ifndef QLDPC_M2S_UNIL
#define QLDPC_M2S_UNIL 1
#endif
// m2s on dword-scaled words (space-time family 111313): the V slot address unpacked for the
// gather is carried to the store (one SDWA per edge and iteration fewer; the backend otherwise
// unpacks it again at the store)
#ifndef QLDPC_M2S_KEEPVA
#define QLDPC_M2S_KEEPVA 1
#endif
// m2s check phase: explicit row / tail / F / CS pointers stepped per row
#ifndef QLDPC_M2S_RPTR
#define QLDPC_M2S_RPTR 1
#endif
// two-word check phase (r_check_c): absolute LDS addresses for the rows, tails and CS stores
#ifndef QLDPC_RC_RPTR
#define QLDPC_RC_RPTR 1
#endif
// m2s check phase of the space-time family: rows in pairs, the second row's first QLDPC_M2S_ROWPAIR
// chunks loaded before the first row is reduced (A/B build; 4 = the whole row spills).  Measured slower:
// config 5 kernel 94.5 ms with one row at a time against 96.1-96.6 ms with 1-3 chunks ahead
// (profiles/r06/config5/rowpair/), so 0 (one row at a time) is the product
#ifndef QLDPC_M2S_ROWPAIR
#define QLDPC_M2S_ROWPAIR 0
#endif
// m2s families: each variable slot's previous decisions as a wave lane mask (SGPRs): the flip test
// is a scalar xor of two masks instead of a bit extract and compare per variable and iteration
// (not the dword-scaled 1024-thread space-time family: measured 1-2% slower with it, r06g)
#ifndef QLDPC_M2S_XMASK
#define QLDPC_M2S_XMASK 1
#endif
#include "bp_slot.h"

namespace qldpc {

// Engine ids of this file: 3, 4, and 13 = engine 3 with dword-scaled edge
// addresses (images of 64-256 KiB: the space-time graphs); + 100 = engine 3
// keeping its own previous v2c in VGPRs in double precision too (the fp64
// kernels built for <= 256-thread workgroups, whose register budget is 256).
constexpr int eng_base(int E) { return E % 10; }
constexpr int eng_sh(int E) { return (E / 10) % 10 ? 2 : 0; }
constexpr bool eng_kv64(int E) { return (E / 100) % 10 != 0; }
// + 1000 = rows of NCH chunks plus one "tail" slot per row in a separate array (rows one
// message wider than the chunks: the fp64 space-time graphs, 8 + 1 slots), engine 3 only
constexpr int eng_tail(int E) { return (E / 1000) % 10; }
// + 10000 = "m2 in slot" (fp64 <= 256-thread family with tail rows, engine id 11103): the check
// state is ONE word per check, CS = {m1 | parity << 63}, and the check phase stores m2 | parity in
// the V slot of the row's argmin edge.  A variable edge gathers CS and its own V slot: a slot that
// no longer holds the edge's own previous v2c (kept in VGPRs) is the argmin, and its value is m2.
// The image shrinks by 8 bytes per check; with rows of 7 as 3 chunks + a tail slot the n1600 fp64
// image is 52.3 KB, so 3 workgroups share a CU (168-VGPR budget).
constexpr bool eng_m2s(int E) { return (E / 10000) % 10 == 1 || (E / 10000) % 10 == 4; }
// + 40000 = m2s with variable-major v2c slots ("m2v", engine id 40103): edge (k, d) of lane t owns
// V slot (ecnt(k) + d) * LB + t (the last variable slot: ecnt * LB + d * NL + t), so the variable
// phase reads and writes its slots lane-linearly (conflict-free, one base VGPR and immediate
// offsets), and the check phase gathers its row's 7 slots from a per-thread register table
constexpr bool eng_m2v(int E) { return (E / 10000) % 10 == 4; }
// m2s + tail + dword-scaled packed addresses + 300 (own v2c in VGPRs, neither split nor byte-packed)
// = engine id 11313 (+ 100000 * D2K): the fp64 space-time family (rows of 4 chunks + a tail slot,
// 1024-thread workgroups, 128-VGPR budget, kern_r_f64_m2st.hip), round 6
// edge slots of variable slots 0..k-1 (degree-3 slots k < D3K keep 3)
template <int D3K>
__host__ __device__ constexpr int m2v_ecnt(int k) { return 3 * (k < D3K ? k : D3K) + 4 * (k > D3K ? k - D3K : 0); }
// rows per thread the m2v check phase keeps in its register table (host-enforced m <= 4 * TB)
constexpr int kM2vRows = 4;
// + 20000 = byte F ("fb": the per-check flags F as one byte per check instead of a word, flips
// xored into the containing word at the byte's shift): the fp32 space-time tail family for 512-thread
// workgroups (engine id 21013), whose 79.6 KB image lets 2 decodes share a CU
constexpr bool eng_fb(int E) { return (E / 10000) % 10 == 2; }
// + 30000 = "c2v in slot" (fp64 <= 256-thread family with tail rows, engine id 31103): the check
// phase writes each edge's c2v into the edge's own V slot (alpha * m1 with the edge's sign for
// every edge, then one ds_xor_b64 turns the argmin edge's word into alpha * m2 with its sign), so
// the variable phase reads one word per edge and keeps neither a check-state array nor its own
// previous v2c; the F word addresses of the edges are held in VGPRs instead of the CS addresses.
// Every row must hold exactly 2 * NCH + 1 edges (no padding slot is overwritten).
constexpr bool eng_c2s(int E) { return (E / 10000) % 10 == 3; }
// + 100000 * D2K (byte-F family): slots k < D2K hold variables of column degree <= 2 (the
// space-time graphs' measurement variables, host-sorted first): no third edge slot kept
constexpr int eng_d2k(int E) { return (E / 100000) % 10; }
// narrow waves (round 6): in the fp64 space-time m2s family the waves 0..W_k-1 of variable slot
// k < kNwSlots (a wave mask per slot in SSector::nw, host-planned by qldpc_hip.hip st_plan) hold variables of one
// degree fewer than the slot's compile-time width and compute that slot with one edge slot fewer (no
// c2v, sum, v2c store or flip xor for it; one wave-uniform branch per such slot): no private dummy
// edges for the measurement columns of config 5.  The gathers stay full width (the missing edge reads
// CS[0] / the shared V dummy, unused): branches around them too split the variable phase into basic
// blocks the scheduler cannot overlap (+2.7 % instead of the edge count's 7.7 %, twice the SALU, 3x
// the branches; one variable phase compiled per narrow mask instead spills, profiles/r06/config5/)
constexpr bool eng_nw(int E) { return eng_m2s(E) && !eng_m2v(E) && eng_tail(E) && eng_sh(E) == 2; }
constexpr int kNwSlots = 2;
// edge slot t of variable slot k is compile-time absent (m2s / c2s / byte-F kernels)
template <int ENG, int D3K>
__device__ constexpr bool no_edge(int k, int t) {
  return (eng_m2s(ENG) || eng_c2s(ENG) || eng_fb(ENG)) && ((k < D3K && t >= 3) || (k < eng_d2k(ENG) && t >= 2));
}
// the one-word / no-word check-state families share the register layout and the shot setup
constexpr bool eng_m2x(int E) { return eng_m2s(E) || eng_c2s(E); }
// launch bounds: LB threads per workgroup at most; 256-thread fp64 kernels are
// built for 2 workgroups per CU (2 waves per SIMD: up to 256 VGPRs, no spills)
template <typename T, int ENG>
constexpr int lb_waves(int LB) {
  // engine 4 fp64 images (no CS array) fit 3 workgroups per CU: <= 168 VGPRs
  // (the fp64 512-thread family: 2 workgroups of 8 waves per CU, 128 VGPRs)
  // (the one-word family with packed addresses, engine id 10203: 4 workgroups per CU, 128 VGPRs)
  return LB <= 256 ? (sizeof(T) == 8 ? (eng_m2s(ENG) && (ENG / 100) % 10 == 2 ? 4
                                        : (eng_base(ENG) == 4 || eng_m2x(ENG)) ? 3 : 2) : 4)
                   : (LB <= 512 && (eng_kv64(ENG) || eng_fb(ENG))) ? 4 : 1;
}
__device__ inline unsigned long long qstamp() {
#if QLDPC_STAMPS
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
#else
  return 0;
#endif
}
template <int ENG>
__device__ inline uint32_t ea_cs(uint32_t ea) { return (ea & 0xFFFFu) << eng_sh(ENG); }
template <int ENG>
__device__ inline uint32_t ea_v(uint32_t ea) { return (ea >> 16) << eng_sh(ENG); }

struct RLayout {
  uint32_t v, t, f, sink, lred, total;  // byte offsets (engine 3: CS at 0; engine 4: V at 0)
};

// [CS][V][tail: one slot per row label (tail layouts only)][F][sink][lred]
// (m2s = 1: CS entries of one message word instead of two; m2s = 2, c2s: no CS array)
__host__ __device__ inline RLayout r_layout(int eng, int vslots, int mmax, int tsize, int tail = 0, int m2s = 0,
                                            int fb = 0) {
  RLayout L;
  L.v = eng == 4 ? 0u : (uint32_t)a16((size_t)(mmax + 1) * (m2s == 2 ? 0 : m2s ? 1 : 2) * tsize);
  L.t = L.v + (uint32_t)a16((size_t)vslots * tsize);
  L.f = L.t + (tail ? (uint32_t)a16((size_t)mmax * tsize) : 0u);
  L.sink = L.f + (uint32_t)a16((size_t)(mmax + 1) * (fb ? 1 : 4));
  L.lred = L.sink + (eng == 4 ? 16u : 0u);
  L.total = L.lred + 48;
  return L;
}
// Block LDS: image + 2 sector fail bitmaps of `chunk` shots + counters.
__host__ __device__ inline size_t r_lds_bytes(int img, int chunk) {
  return (size_t)img + 2 * a16((size_t)((chunk + 31) / 32) * 4) + 8 * 12;
}

// Engine-3 check-state entry CS[i+1] of check i ({m1 | parity<<sign, m2}; CS[0]
// = the missing-edge dummy).  A pre-scaled 16-byte float variant {m1|par,
// alpha*m2, alpha*m1} saves two VALU ops per edge but measured 15 % slower
// (ds_read_b128 gathers, +VGPRs): the gather bandwidth, not VALU, binds.
template <typename T>
struct CSEntry {
  using type = Pair<T>;
};

template <typename T>
__device__ inline T& lds_at(unsigned char* smem, uint32_t off) {
  return *reinterpret_cast<T*>(smem + off);
}
// LDS access by absolute address (no add of the dynamic-LDS base per access)
template <typename X>
using LdsPtr = __attribute__((address_space(3))) X*;
__device__ inline uint32_t lds_base(unsigned char* smem) {
  return (uint32_t)(uintptr_t)(LdsPtr<unsigned char>)smem;
}
// load / store of an LDS word at `a`: absolute address (ABS) or offset from smem
// (through a same-size clang vector: the message structs have no address-space copy)
template <int B>
struct LdsWord;
template <>
struct LdsWord<4> {
  typedef uint32_t type;
};
template <>
struct LdsWord<8> {
  typedef uint32_t type __attribute__((ext_vector_type(2)));
};
template <>
struct LdsWord<16> {
  typedef uint32_t type __attribute__((ext_vector_type(4)));
};
template <typename X, bool ABS>
__device__ inline X lds_ld(unsigned char* smem, uint32_t a) {
  if constexpr (ABS) {
    using W = typename LdsWord<sizeof(X)>::type;
    const W w = *(LdsPtr<const W>)(uintptr_t)a;
    X x;
    __builtin_memcpy(&x, &w, sizeof(X));
    return x;
  } else {
    return lds_at<X>(smem, a);
  }
}
template <typename X, bool ABS>
__device__ inline void lds_st(unsigned char* smem, uint32_t a, X v) {
  if constexpr (ABS) {
    using W = typename LdsWord<sizeof(X)>::type;
    W w;
    __builtin_memcpy(&w, &v, sizeof(X));
    *(LdsPtr<W>)(uintptr_t)a = w;
  } else {
    lds_at<X>(smem, a) = v;
  }
}
// LDS atomic xor (no return) at an absolute address
__device__ inline void lds_xor_abs(uint32_t a, uint32_t v) {
  __hip_atomic_fetch_xor((LdsPtr<uint32_t>)(uintptr_t)a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// canonical bits: |v| with the sign bit := (v <= 0).  Only +0 differs from the
// raw bits (-0 and negatives already carry the sign bit; NaN never occurs).
// Branch- and VCC-free form: b | ((b - 1) & ~b & sign) sets the sign bit only
// for b == 0 (one add and one three-input bit op; no compare hazard nops).
template <typename T>
__device__ inline typename FT<T>::U canon2(T v) {
  using U = typename FT<T>::U;
  const U b = FT<T>::bits(v);
  if constexpr (sizeof(T) == 8) {
    // hi | (hi(b - 1) & sign): `& ~b` is implied (a set sign bit is kept anyway);
    // one 64-bit add and one v_and_or
    const U bm = b - (U)1;
    uint32_t hi;
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(hi) : "v"((uint32_t)(bm >> 32)), "v"(0x80000000u), "v"((uint32_t)(b >> 32)));
    return ((U)hi << 32) | (uint32_t)b;
  } else {
    return b | ((b - (U)1) & ~b & FT<T>::kSign);
  }
}

// Engine 3 keeps its messages NEGATED ("w domain"): w = -v for every prior, v2c and c2v,
// except that a zero prior is +0.  Then every w is either exactly -v (v != 0) or +0 (v
// == 0: an exact cancellation rounds to +0, and a sum is -0 only when all its leaves are
// -0, which a +0-or-nonzero prior rules out), so the sign bit of w is exactly NOT the
// canonical sign (v <= 0) the min-sum parity needs: the v2c leave-one-out sums are stored
// as they come out of the adds (no canon2 per edge), the decision is w >= 0, and the
// check phase flips its parity by the row degree (F bit 2, folded into the syndrome bit it
// keeps per row), which turns the xor of the w signs back into the xor of the canonical
// ones.  -w is the c2v product with the same sign rule, so the c2v arithmetic is unchanged.
template <typename T>
__device__ inline T w_prior(T l) {
  using U = typename FT<T>::U;
  const U b = FT<T>::bits(-l);
  return FT<T>::val(b == FT<T>::kSign ? (U)0 : b);  // -(+0) = -0 -> +0
}

// XOR of a 32-bit value over the 64 lanes of a wave (all lanes active), without the LDS
// crossbar: quad butterflies and row rotations in DPP give each lane its 16-lane row's xor,
// then the four row values are read into SGPRs.  The result is wave-uniform.
__device__ inline uint32_t wave_xor_u32(uint32_t v) {
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xF, 0xF, false);  // row_ror:4
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) ^ (uint32_t)__builtin_amdgcn_readlane((int)v, 16) ^
         (uint32_t)__builtin_amdgcn_readlane((int)v, 32) ^ (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
}

// x is +0 or -0 (v_cmp_class_*: class bits 5 = -0, 6 = +0)
__device__ inline bool is_zero(float x) { return __builtin_amdgcn_classf(x, 0x60); }
__device__ inline bool is_zero(double x) { return __builtin_amdgcn_class(x, 0x60); }

// median of three (the backend selects v_med3_u32 for this pattern)
__device__ inline uint32_t med3u(uint32_t a, uint32_t b, uint32_t c) {
  const uint32_t lo = a < b ? a : b, hi = a < b ? b : a;
  const uint32_t h2 = hi < c ? hi : c;
  return lo > h2 ? lo : h2;
}

// Register state of one thread in one sector pass.  Edge words: engine 3 =
// CS address | V slot address << 16; engine 4 = read address | write address
// << 16 (equal for real edges; zero chunk / sink for missing ones).
template <typename T, int DMAX, int VPL, int ENG = 3>
struct RState {
  using U = typename FT<T>::U;
  static constexpr bool kKeepV =
      eng_base(ENG) == 3 && (sizeof(T) == 4 || eng_kv64(ENG)) && !eng_c2s(ENG);  // own v2c in VGPRs
  // the fp64 <= 256-thread family (256-VGPR budget) keeps the two addresses of an edge
  // unpacked and absolute (ea = CS address, ev = V slot address): no unpack / base add
  // per access, 2 VALU per edge and iteration fewer
  static constexpr bool kSplit = (ENG / 100) % 10 == 1 && sizeof(T) == 8;  // engine id 103 (not 303)
  // + 200 instead of + 100 on the one-word family (engine id 10203): the edge's CS and V slot byte
  // addresses packed absolute into one VGPR (images < 64 KiB), unpacked by one VALU each per access:
  // 16 fewer VGPRs for 16 edges per thread (LP L30: 4 workgroups per CU instead of 3)
  static constexpr bool kPk = (ENG / 100) % 10 == 2 && sizeof(T) == 8 && eng_m2s(ENG) && !eng_m2v(ENG);
  // absolute LDS addresses: split words, or (dword-scaled packed words: the space-time families
  // 13 / 1013 / 21013) absolute dword indices, unpacked by one SDWA shift per access and used
  // without a base add
  static constexpr bool kAbs = kSplit || kPk || (eng_sh(ENG) == 2 && QLDPC_ABS_SH2);
  // m2s with QLDPC_M2S_UNIL: one prior for every variable (uniform channel_probs, host-checked),
  // loaded by a scalar load: 2 SGPRs instead of 2 * VPL VGPRs
  static constexpr bool kUniL = eng_m2x(ENG) && QLDPC_M2S_UNIL;
  static constexpr bool kM2v = eng_m2v(ENG);
  uint32_t ea[VPL][DMAX];
  uint32_t ev[kSplit && !kM2v ? VPL : 1][kSplit && !kM2v ? DMAX : 1];
  T L[kUniL ? 1 : VPL];
  U ov[kKeepV ? VPL : 1][kKeepV ? DMAX : 1];
  // m2v: lane base of the V slots and the last variable slot's per-edge addresses
  uint32_t vlane;
  uint32_t vl[kM2v ? DMAX : 1];
};
// m2v row table of one thread: row q (check tid + q * TB) = 7 16-bit slot offsets from the V base,
// two per word; loaded from global memory before the barrier that precedes each check phase
// (registers live across that barrier only)
struct M2vRows {
  uint4 w[kM2vRows];
};
__device__ inline void m2v_rows_load(const SSector& S, int tid, int TB, int m, M2vRows& r) {
#pragma unroll
  for (int q = 0; q < kM2vRows; ++q)
    if (q * TB < m) r.w[q] = reinterpret_cast<const uint4*>(S.rows)[(size_t)q * TB + tid];
}
// m2v: absolute V slot address of edge (k, t) (immediate offsets from the lane base)
template <typename T, int DMAX, int VPL, int ENG, int D3K, int LB>
__device__ inline uint32_t m2v_va(const RState<T, DMAX, VPL, ENG>& R, int k, int t) {
  if (k < VPL - 1) return R.vlane + (uint32_t)((m2v_ecnt<D3K>(k) + t) * LB * 8);
  return R.vl[RState<T, DMAX, VPL, ENG>::kM2v ? t : 0];
}
// 4 * (16-bit half h of w) in one VALU (SDWA word select feeding the shift)
template <int H, int SH>
__device__ inline uint32_t sdwa_shl(uint32_t w) {
  uint32_t r;
  if constexpr (H == 0)
    asm("v_lshlrev_b32_sdwa %0, %2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0"
        : "=v"(r) : "v"(w), "i"(SH));
  else
    asm("v_lshlrev_b32_sdwa %0, %2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1"
        : "=v"(r) : "v"(w), "i"(SH));
  return r;
}
// CS / V slot address of edge (k, t): absolute when split or kAbs, else offsets from smem
template <typename T, int DMAX, int VPL, int ENG>
__device__ inline uint32_t r_csa(const RState<T, DMAX, VPL, ENG>& R, int k, int t) {
  if constexpr (RState<T, DMAX, VPL, ENG>::kSplit)
    return R.ea[k][t];
  else if constexpr (RState<T, DMAX, VPL, ENG>::kPk)
    return R.ea[k][t] & 0xFFFFu;
  else if constexpr (RState<T, DMAX, VPL, ENG>::kAbs)
    return sdwa_shl<0, 2>(R.ea[k][t]);
  else
    return ea_cs<ENG>(R.ea[k][t]);
}
template <typename T, int DMAX, int VPL, int ENG>
__device__ inline uint32_t r_va(const RState<T, DMAX, VPL, ENG>& R, int k, int t) {
  if constexpr (RState<T, DMAX, VPL, ENG>::kSplit)
    return R.ev[k][t];
  else if constexpr (RState<T, DMAX, VPL, ENG>::kPk)
    return R.ea[k][t] >> 16;
  else if constexpr (RState<T, DMAX, VPL, ENG>::kAbs)
    return sdwa_shl<1, 2>(R.ea[k][t]);
  else
    return ea_v<ENG>(R.ea[k][t]);
}

template <typename T, int DMAX, int VPL, int ENG>
__device__ inline void r_load(const SSector& S, RState<T, DMAX, VPL, ENG>& R, const RLayout& Ly, int tid, int TB,
                              uint32_t sbase) {
  const T* llr = static_cast<const T*>(S.llr);
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
#pragma unroll
    for (int t = 0; t < DMAX; ++t) {
      const uint32_t e = S.edges[(k * DMAX + t) * TB + tid];
      const uint32_t va = Ly.v + eslot(e) * (uint32_t)sizeof(T);
      if (eng_base(ENG) == 4) {
        R.ea[k][t] = e == kNoEdgeS ? (Ly.v | (Ly.sink << 16)) : (va | (va << 16));
      } else if constexpr (RState<T, DMAX, VPL, ENG>::kSplit) {
        // c2s: the absolute address of the edge's F word (entry = check label + 1)
        R.ea[k][t] = eng_c2s(ENG) ? sbase + Ly.f + 4u * echk(e) : sbase + echk(e) * (uint32_t)((eng_m2s(ENG) ? 1 : 2) * sizeof(T));
        if constexpr (!RState<T, DMAX, VPL, ENG>::kM2v) R.ev[k][t] = sbase + va;
      } else if constexpr (RState<T, DMAX, VPL, ENG>::kPk) {  // absolute byte addresses, packed
        R.ea[k][t] = (sbase + echk(e) * (uint32_t)sizeof(T)) | ((sbase + va) << 16);
      } else if constexpr (RState<T, DMAX, VPL, ENG>::kAbs) {  // absolute dword indices
        // (m2s: one-word CS entries)
        R.ea[k][t] = ((sbase + echk(e) * (uint32_t)((eng_m2s(ENG) ? 1 : 2) * sizeof(T))) >> 2) | (((sbase + va) >> 2) << 16);
      } else {
        R.ea[k][t] = ((echk(e) * (uint32_t)(2 * sizeof(T))) >> eng_sh(ENG)) | ((va >> eng_sh(ENG)) << 16);
      }
    }
    if constexpr (!RState<T, DMAX, VPL, ENG>::kUniL) {
      const T l = (S.perm[k * TB + tid] >= 0) ? llr[k * TB + tid] : (T)1;
      R.L[k] = eng_base(ENG) == 3 ? w_prior<T>(l) : l;  // engine 3: w domain
    }
  }
  // uniform prior (slot 0 of lane 0 holds a real variable); padding lanes take it too (their
  // results are never read)
  if constexpr (RState<T, DMAX, VPL, ENG>::kUniL) R.L[0] = w_prior<T>(llr[0]);
  if constexpr (RState<T, DMAX, VPL, ENG>::kM2v) {
    // lane base (LDS addresses are < 64 KiB: the mask makes the sign bit known, so the per-edge
    // offsets fold into the DS instructions' offset fields); the last variable slot strides S.vnl
    R.vlane = (sbase + Ly.v + 8u * (uint32_t)tid) & 0xFFFFu;
    const uint32_t last = (uint32_t)S.vlast * 8u;  // byte offset of the last slot's first edge
#pragma unroll
    for (int t = 0; t < DMAX; ++t) R.vl[t] = R.vlane + last + (uint32_t)t * (uint32_t)S.vnl * 8u;
  }
}
template <typename T, int DMAX, int VPL, int ENG>
__device__ inline T r_prior(const RState<T, DMAX, VPL, ENG>& R, int k) {
  return R.L[RState<T, DMAX, VPL, ENG>::kUniL ? 0 : k];
}

// F word of an edge.  Engine 3: from the CS address.  Engine 4: from the row
// of the read address (rows start 16 bytes into V, row stride 1 << rsh); the
// zero chunk maps to row -1, i.e. the F[0] sink.
struct FMap {
  uint32_t fbase;   // engine 3: Ly.f; engine 4: Ly.f + 4
  uint32_t rstart;  // engine 4: Ly.v + 16
  int rsh;          // engine 4: log2(row stride)
};
template <typename T, int ENG>
__device__ inline uint32_t f_addr(uint32_t ea, const FMap& M) {
  if (eng_base(ENG) == 4) return M.fbase + 4u * (uint32_t)((int)((ea & 0xFFFFu) - M.rstart) >> M.rsh);
  return (ea_cs<ENG>(ea) >> (sizeof(T) == 4 ? 1 : 2)) + M.fbase;
}
// F entry access (engine 3): entry e (= check label + 1) at byte Ly.f + 4e, or Ly.f + e in byte-F
// kernels, whose xors go to the containing word at the byte's shift (order-free, so still atomic
// and commutative) and whose plain stores are byte stores (one owner per byte)
template <int ENG>
__device__ inline uint32_t f_off(const RLayout& Ly, int e) {
  return Ly.f + (eng_fb(ENG) ? (uint32_t)e : 4u * (uint32_t)e);
}
template <int ENG>
__device__ inline uint32_t f_ld(unsigned char* smem, uint32_t off) {
  if constexpr (eng_fb(ENG)) return lds_at<uint8_t>(smem, off);
  return lds_at<uint32_t>(smem, off);
}
template <int ENG>
__device__ inline void f_st(unsigned char* smem, uint32_t off, uint32_t v) {
  if constexpr (eng_fb(ENG))
    lds_at<uint8_t>(smem, off) = (uint8_t)v;
  else
    lds_at<uint32_t>(smem, off) = v;
}
template <int ENG>
__device__ inline void f_xor(unsigned char* smem, uint32_t off, uint32_t v) {
  if constexpr (eng_fb(ENG))
    atomicXor(&lds_at<uint32_t>(smem, off & ~3u), v << (8u * (off & 3u)));
  else
    atomicXor(&lds_at<uint32_t>(smem, off), v);
}

// F word offset of edge (k, t) (engine 3); split addresses are absolute: fbase is then
// Ly.f - (LDS base >> 2)
template <typename T, int DMAX, int VPL, int ENG>
__device__ inline uint32_t r_fa(const RState<T, DMAX, VPL, ENG>& R, int k, int t, uint32_t fbase) {
  // CS entry (i + 1) of 2 words (fp32: 8 B, fp64: 16 B) or, m2s, one fp64 word (8 B) -> F word i + 1
  // (byte-F kernels: fp32 CS entries of 8 B -> F byte i + 1)
  if constexpr (RState<T, DMAX, VPL, ENG>::kPk) return ((R.ea[k][t] & 0xFFFFu) >> 1) + fbase;
  if constexpr (RState<T, DMAX, VPL, ENG>::kAbs && !RState<T, DMAX, VPL, ENG>::kSplit) {
    // absolute dword index w = csa / 4 in the low half: csa >> 3 = w >> 1, csa >> 1 = 2 w, csa >> 2 = w
    const uint32_t w = R.ea[k][t];
    if constexpr (eng_fb(ENG)) return __builtin_amdgcn_ubfe(w, 1, 15) + fbase;
    // fp32 two-word and fp64 one-word (m2s) CS entries are 8 bytes: F word = 2 x the dword index
    if constexpr (sizeof(T) == 4 || eng_m2s(ENG)) return sdwa_shl<0, 1>(w) + fbase;
    return (w & 0xFFFFu) + fbase;
  }
  if constexpr (eng_fb(ENG)) return (r_csa(R, k, t) >> 3) + fbase;
  return (r_csa(R, k, t) >> ((sizeof(T) == 4 || eng_m2s(ENG)) ? 1 : 2)) + fbase;
}

// Opaque redefinition of the edge words (no instruction): without it the
// compiler hoists their derived CS / V / F addresses out of the iteration and
// shot loops, tripling the VGPRs per edge and spilling.
// m2s and byte-F kernels (D3K > 0 passed) keep no edge words for the unused 4th edge of degree-3 slots.
template <typename T, int DMAX, int VPL, int ENG, int D3K = 0>
__device__ inline void r_launder(RState<T, DMAX, VPL, ENG>& R) {
#pragma unroll
  for (int k = 0; k < VPL; ++k)
#pragma unroll
    for (int t = 0; t < DMAX; ++t) {
      if (no_edge<ENG, D3K>(k, t)) continue;
      asm volatile("" : "+v"(R.ea[k][t]));
      if constexpr (RState<T, DMAX, VPL, ENG>::kSplit && !RState<T, DMAX, VPL, ENG>::kM2v)
        asm volatile("" : "+v"(R.ev[k][t]));
    }
}

// Variable phase (one flooding iteration's column pass).  Returns decision bits.
// F bit0 holds (H x)_i for the current decisions: only variables whose decision
// flipped since the previous iteration (xprev) xor their checks.  Slots k < D3K
// (compile time) hold variables of column degree <= 3 (host-sorted), so their
// 4th edge slot is skipped entirely (no gather, no arithmetic, no store).
template <typename T, int DMAX, int VPL, int ND, int ENG>
__device__ inline void r_gather(unsigned char* smem, const RState<T, DMAX, VPL, ENG>& R, int k,
                                typename CSEntry<T>::type (&pn)[DMAX],
                                typename FT<T>::U (&on)[DMAX]) {
  constexpr bool KV = RState<T, DMAX, VPL, ENG>::kKeepV;
  constexpr bool SP = RState<T, DMAX, VPL, ENG>::kAbs;
#pragma unroll
  for (int t = 0; t < ND; ++t) {
    pn[t] = lds_ld<typename CSEntry<T>::type, SP>(smem, r_csa(R, k, t));
    if (!KV) on[t] = FT<T>::bits(lds_ld<T, SP>(smem, r_va(R, k, t)));
  }
}

template <typename T, int DMAX, int VPL, int ND, int ENG>
__device__ inline bool r_var_one(unsigned char* smem, RState<T, DMAX, VPL, ENG>& R, int k,
                                 const typename CSEntry<T>::type (&pr)[DMAX],
                                 const typename FT<T>::U (&o)[DMAX], uint32_t fdelta, T alpha, bool xprev,
                                 double* post, const int32_t* perm) {
  using U = typename FT<T>::U;
  constexpr U kS = FT<T>::kSign;
  constexpr bool KV = RState<T, DMAX, VPL, ENG>::kKeepV;
  T c[ND];
#pragma unroll
  for (int t = 0; t < ND; ++t) {
    const U a = pr[t].a;
    const U d = a ^ o[t];
    // min over the other edges: m2 if this edge holds m1 (|own| == m1), else m1;
    // sign = parity of the others and the syndrome = sign bit of d
    // (m2 carries no sign bit, so masking after the select is the same value;
    // masking `a` before it trips an instruction-selection crash in this LLVM).
    // |d| == 0 is tested with v_cmp_class (+-0 only): one instruction instead of
    // mask + compare (bit patterns of any class, denormals and NaNs included).
    U sel;
    if constexpr (sizeof(T) == 4 && QLDPC_F32_C2V4) {
      // 4 VALU: |own| == |m1| by v_cmp_eq_f32 on the absolute values (the magnitude-bits test of
      // the class form: denormals compare exactly, no flush; NaN never occurs), select m1 | parity
      // or m2 | parity (the check phase stores both with the parity), and the own sign rides on
      // alpha: (alpha ^ own sign) * sel has sign parity ^ own and magnitude |sel| * alpha
      // (sign-symmetric rounding), the value of the class form bit for bit, zeros included
      (void)d;
      asm("v_cmp_eq_f32 vcc, |%1|, |%2|\n\ts_nop 1\n\tv_cndmask_b32 %0, %3, %4, vcc"
          : "=v"(sel)
          : "v"(a), "v"(o[t]), "v"(a), "v"(pr[t].b)
          : "vcc");
      uint32_t as;
      asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x6c"
          : "=v"(as)
          : "v"((uint32_t)o[t]), "v"(FT<T>::bits(alpha)), "v"(0x80000000u));
      c[t] = FT<T>::val(sel) * FT<T>::val(as);
    } else if constexpr (sizeof(T) == 4) {
      // v_cmp_class (+-0) feeding v_cndmask; LLVM would rewrite the class test as
      // mask + integer compare.  s_nop 1: the VALU-writes-VCC -> VALU-reads-VCC
      // hazard the compiler itself pads on gfx950.
      asm("v_cmp_class_f32 vcc, %1, %2\n\ts_nop 1\n\tv_cndmask_b32 %0, %3, %4, vcc"
          : "=v"(sel)
          : "v"(d), "v"(0x60u), "v"(a), "v"(pr[t].b)
          : "vcc");
      sel &= ~kS;
      c[t] = FT<T>::val(FT<T>::bits(FT<T>::val(sel) * alpha) ^ (d & kS));
    } else if constexpr (QLDPC_F64_C2V5) {
      // double in 5 VALU (the class form takes 7: the 64-bit xor is 2): |own| == |m1| by
      // v_cmp_eq_f64 on absolute values, two cndmasks select m1 | parity or m2 | parity, and the
      // own sign rides on alpha's high word: (alpha ^ own sign) * sel, the same bits
      (void)d;
      uint32_t slo, shi;
      asm("v_cmp_eq_f64 vcc, |%2|, |%3|\n\ts_nop 1\n\tv_cndmask_b32 %0, %4, %5, vcc\n\tv_cndmask_b32 %1, %6, %7, vcc"
          : "=&v"(slo), "=&v"(shi)
          : "v"(FT<T>::val(a)), "v"(FT<T>::val(o[t])), "v"((uint32_t)a), "v"((uint32_t)pr[t].b),
            "v"((uint32_t)(a >> 32)), "v"((uint32_t)(pr[t].b >> 32))
          : "vcc");
      const U ab = FT<T>::bits(alpha);
      uint32_t ahs;
      asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x6c"
          : "=v"(ahs)
          : "v"((uint32_t)(o[t] >> 32)), "v"((uint32_t)(ab >> 32)), "v"(0x80000000u));
      c[t] = FT<T>::val(((U)shi << 32) | slo) * FT<T>::val(((U)ahs << 32) | (uint32_t)ab);
    } else {
      // double: the same class test on the 64-bit pair and two cndmasks; |sel| folds
      // into v_mul_f64's source modifier; sign = hi(product) ^ (hi(d) & sign bit) in
      // one v_bitop3 (truth table 0x6c = S1 ^ (S0 & S2))
      uint32_t slo, shi;
      asm("v_cmp_class_f64 vcc, %2, %3\n\ts_nop 1\n\tv_cndmask_b32 %0, %4, %5, vcc\n\tv_cndmask_b32 %1, %6, %7, vcc"
          : "=&v"(slo), "=&v"(shi)
          : "v"(FT<T>::val(d)), "v"(0x60u), "v"((uint32_t)a), "v"((uint32_t)pr[t].b), "v"((uint32_t)(a >> 32)),
            "v"((uint32_t)(pr[t].b >> 32))
          : "vcc");
      sel = ((U)shi << 32) | slo;
      const U pb = FT<T>::bits(__builtin_fabs(FT<T>::val(sel)) * alpha);
      uint32_t hi;
      asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x6c"
          : "=v"(hi)
          : "v"((uint32_t)(d >> 32)), "v"((uint32_t)(pb >> 32)), "v"(0x80000000u));
      c[t] = FT<T>::val(((U)hi << 32) | (uint32_t)pb);
    }
  }
  // ldpc column pass: forward partial sums from the prior, then backward
  T f[ND];
  T acc = R.L[k];
#pragma unroll
  for (int t = 0; t < ND; ++t) {
    f[t] = acc;
    acc = acc + c[t];
  }
  const bool x = acc >= (T)0;  // w domain: v <= 0
  if (post) {  // BP+OSD capture (last iteration): ldpc's log_prob_ratios, the OSD sort key
    const int j = *perm;
    if (j >= 0) post[j] = -(double)acc;  // (a zero's sign may differ: the OSD sort ties +-0)
  }
  T b = c[ND - 1];
  U nv[ND];
  nv[ND - 1] = FT<T>::bits(f[ND - 1]);  // w domain: stored as computed (no canon2)
#pragma unroll
  for (int t = ND - 2; t >= 0; --t) {
    nv[t] = FT<T>::bits(f[t] + b);
    if (t > 0) b = b + c[t];
  }
#pragma unroll
  for (int t = 0; t < ND; ++t) {
    lds_st<U, RState<T, DMAX, VPL, ENG>::kAbs>(smem, r_va(R, k, t), nv[t]);
    if (KV) R.ov[KV ? k : 0][KV ? t : 0] = nv[t];
  }
#if QLDPC_FLIPLATE
  (void)xprev;  // flips applied by r_var after the loop
#elif QLDPC_FLIP_BRANCHFREE
  // diagnostic variant: every edge xors (x != xprev) into its check's F word, no branch
#pragma unroll
  for (int t = 0; t < ND; ++t) f_xor<ENG>(smem, r_fa(R, k, t, fdelta), (uint32_t)(x != xprev));
#else
  if (x != xprev) {
#pragma unroll
    for (int t = 0; t < ND; ++t) f_xor<ENG>(smem, r_fa(R, k, t, fdelta), 1u);
  }
#endif
  return x;
}

// Rows loaded ahead of the reduced one in the compile-time-width check phase (A/B builds:
// QLDPC_PFC=0/1/2).  n1600: 0 (each row loaded where it is reduced) is 4 % faster than 1 in
// fp64 (928k -> 968k shots/s) and fp32 (1.79M -> 1.86M); 2 is 5 % / 10 % slower than 1.
#ifndef QLDPC_PFC
#define QLDPC_PFC 0
#endif
// Wave priority (s_setprio) in the variable phase / the check phase.  Variable phase at 2 (the
// other workgroups of the CU are mostly in their check phases or barriers then): n1600 fp32
// 1.88M -> 1.98M shots/s, fp64 +0.4 %; the check phase raised instead: -1 % / -2 %.
#ifndef QLDPC_PRIO_V
#define QLDPC_PRIO_V 2
#endif
#ifndef QLDPC_PRIO_C
#define QLDPC_PRIO_C 0
#endif
// How many variables ahead the CS gathers are issued: 2 in the fp64 <= 256-thread family
// (engine id 103, 256-VGPR budget: +4 VGPRs, n1600 fp64 909k -> 927k shots/s), 1 elsewhere
// (fp32 measured unchanged).  QLDPC_PF=1 / 2 overrides it in an A/B build.
#ifndef QLDPC_PF
#define QLDPC_PF 0
#endif
template <typename T, int DMAX, int VPL, int D3K, int ENG>
__device__ inline void r_gather_k(unsigned char* smem, const RState<T, DMAX, VPL, ENG>& R, int k,
                                  typename CSEntry<T>::type (&pn)[DMAX], typename FT<T>::U (&on)[DMAX]) {
  constexpr int N3 = DMAX > 3 ? 3 : DMAX;
  if (k < eng_d2k(ENG))
    r_gather<T, DMAX, VPL, 2, ENG>(smem, R, k, pn, on);
  else if (k < D3K)
    r_gather<T, DMAX, VPL, N3, ENG>(smem, R, k, pn, on);
  else
    r_gather<T, DMAX, VPL, DMAX, ENG>(smem, R, k, pn, on);
}

template <typename T, int DMAX, int VPL, int D3K, int ENG>
__device__ inline uint32_t r_var(unsigned char* smem, RState<T, DMAX, VPL, ENG>& R, uint32_t fdelta, T alpha,
                                 uint32_t xprev, bool last_live, double* post = nullptr, const int32_t* perm = nullptr,
                                 int TB = 0) {
  using U = typename FT<T>::U;
  constexpr bool KV = RState<T, DMAX, VPL, ENG>::kKeepV;
  constexpr int N3 = DMAX > 3 ? 3 : DMAX;  // low-degree slots use 3 edge slots
  constexpr int PF0 = QLDPC_PF >= 1 ? QLDPC_PF : (RState<T, DMAX, VPL, ENG>::kSplit ? 2 : 1);
  constexpr int PF = PF0 < VPL ? PF0 : VPL;
  r_launder<T, DMAX, VPL, ENG, D3K>(R);
  uint32_t xbits = 0;
  // gather ring: variable k's CS entries (and, without kKeepV, own v2c) live in slot k % PF
  typename CSEntry<T>::type pb[PF][DMAX];
  U ob[PF][DMAX];
#pragma unroll
  for (int k = 0; k < PF; ++k) r_gather_k<T, DMAX, VPL, D3K, ENG>(smem, R, k, pb[k], ob[k]);
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    typename CSEntry<T>::type pr[DMAX];
    U o[DMAX];
#pragma unroll
    for (int t = 0; t < DMAX; ++t) {
      pr[t] = pb[k % PF][t];
      o[t] = KV ? R.ov[KV ? k : 0][KV ? t : 0] : ob[k % PF][t];
    }
    // variable k + PF's gathers go out before this one's arithmetic
    if (k + PF < VPL) r_gather_k<T, DMAX, VPL, D3K, ENG>(smem, R, k + PF, pb[k % PF], ob[k % PF]);
    if (k == VPL - 1 && !last_live) break;  // every lane of this wave holds padding
    const bool xp = ((xprev >> k) & 1u) != 0;
    const int32_t* pk = perm ? perm + k * TB : nullptr;
    const bool x = k < eng_d2k(ENG) ? r_var_one<T, DMAX, VPL, 2, ENG>(smem, R, k, pr, o, fdelta, alpha, xp, post, pk)
                   : k < D3K        ? r_var_one<T, DMAX, VPL, N3, ENG>(smem, R, k, pr, o, fdelta, alpha, xp, post, pk)
                                    : r_var_one<T, DMAX, VPL, DMAX, ENG>(smem, R, k, pr, o, fdelta, alpha, xp, post, pk);
    xbits |= (x ? 1u : 0u) << k;
  }
#if QLDPC_FLIPLATE
  const uint32_t fl = xbits ^ xprev;
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    if ((fl >> k) & 1u) {
      const int nd = k < eng_d2k(ENG) ? 2 : k < D3K ? N3 : DMAX;
#pragma unroll
      for (int t = 0; t < DMAX; ++t)
        if (t < nd) f_xor<ENG>(smem, r_fa(R, k, t, fdelta), 1u);
    }
  }
#endif
  return xbits;
}

// Check phase: FIRST records the syndrome bits (F bit1) into sbits; otherwise
// tests (H x)_i == s_i (F bit0).  Clears F and rebuilds CS from the rows.
template <typename T, bool FIRST>
__device__ inline int r_check(unsigned char* smem, const RLayout& Ly, int m, int nch, int tid, int TB,
                              uint32_t& sbits, T alpha_next) {
  using U = typename FT<T>::U;
  using VT = typename V16<T>::type;
  constexpr int NV = V16<T>::N;
  constexpr U kS = FT<T>::kSign;
  int mism = 0;
  int q = 0;
  // chunk rotation against ds_read_b128 bank conflicts (as r_check_c; power-of-two widths)
  const int rmask = (nch & (nch - 1)) == 0 ? nch - 1 : 0;
  const int rot = rmask ? (tid / (nch < 16 ? 16 / nch : 1)) & rmask : 0;
  for (int i = tid; i < m; i += TB, ++q) {
    const VT* row = reinterpret_cast<const VT*>(smem + Ly.v + 16 + (uint32_t)i * (uint32_t)nch * 16u);
    uint32_t& F = lds_at<uint32_t>(smem, Ly.f + 4u * (uint32_t)(i + 1));
    const uint32_t f = F;
    uint32_t s;
    if (FIRST) {
      // w domain: the kept bit is syndrome ^ row-degree parity (F bit 2), and F bit 0 =
      // (H x) ^ that parity starts at the parity, so mism below compares like for like
      s = ((f >> 1) ^ (f >> 2)) & 1u;
      sbits |= s << q;
      F = (f & 4u) | ((f >> 2) & 1u);  // H x starts at 0; the variable phases keep it current
    } else {
      s = (sbits >> q) & 1u;
      mism |= (int)((f ^ s) & 1u);
    }
    U m1 = FT<T>::kSent, m2 = FT<T>::kSent;
    U px = s ? kS : (U)0;
    if constexpr (sizeof(U) == 4) {
      // float min / median with |x| source modifiers: on non-negative, non-NaN
      // floats the float order is the bit order and v_med3_f32 returns one of its
      // inputs unchanged, so this is the integer min / second min of |v2c| bits
      // with the masking folded into the instructions
      float f1 = FT<T>::val(m1), f2 = FT<T>::val(m2);
      for (int c = 0; c < nch; ++c) {
        const VT v = row[(c + rot) & (rmask | (rmask ? 0 : 0x7fffffff))];
#pragma unroll
        for (int k = 0; k < NV; ++k) {
          const float x = V16<T>::get(v, k);
          f2 = __builtin_amdgcn_fmed3f(f1, f2, __builtin_fabsf(x));  // f1 <= f2: the new second minimum
          // v_min_f32 with the |x| modifier (as a builtin, LLVM would add a canonicalize)
          asm("v_min_f32 %0, %1, |%2|" : "=v"(f1) : "v"(f1), "v"(x));
        }
        // parity of the chunk's sign bits: two three-input xors (v_bitop3 0x96 = a^b^c)
        uint32_t p01, p23;
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(p01) : "v"((uint32_t)px), "v"(FT<T>::bits(v.x)), "v"(FT<T>::bits(v.y)));
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(p23) : "v"(p01), "v"(FT<T>::bits(v.z)), "v"(FT<T>::bits(v.w)));
        px = p23;
      }
      m1 = FT<T>::bits(f1);
      m2 = FT<T>::bits(f2);
    } else {
      for (int c = 0; c < nch; ++c) {
        const VT v = row[(c + rot) & (rmask | (rmask ? 0 : 0x7fffffff))];
#pragma unroll
        for (int k = 0; k < NV; ++k) {
          const U xb = FT<T>::bits(V16<T>::get(v, k));
          const U a = xb & ~kS;
          const U hi = m1 > a ? m1 : a;
          m2 = m2 < hi ? m2 : hi;
          m1 = m1 < a ? m1 : a;
          px ^= xb;
        }
      }
    }
    (void)alpha_next;
    typename CSEntry<T>::type st;
    st.a = m1 | (px & kS);
    st.b = m2 | ((sizeof(T) == 4 ? QLDPC_F32_C2V4 : QLDPC_F64_C2V5) ? (px & kS) : (U)0);  // m2 | parity too
    lds_at<typename CSEntry<T>::type>(smem, (uint32_t)(i + 1) * (uint32_t)(2 * sizeof(T))) = st;
  }
  return mism;
}

// Check phase with a compile-time row width of NCH 16-byte chunks (same
// contract as r_check).  The next row's chunks and F word are loaded before the
// current row is reduced, so each thread keeps one row of LDS reads in flight.
// Double rows reduce on v_max_f64 / v_min_f64 with |x| source modifiers: on
// non-negative, non-NaN doubles the float order is the bit order and the
// results are inputs unchanged, i.e. the integer min / second min of |v2c| bits
// (three instructions per edge instead of three 64-bit compares + six selects).
template <typename T, bool FIRST, int NCH, int TAIL = 0, int PFC = 1, int ENG = 3>
__device__ inline int r_check_c(unsigned char* smem, const RLayout& Ly, int m, int tid, int TB, uint32_t& sbits) {
  using U = typename FT<T>::U;
  using VT = typename V16<T>::type;
  constexpr int NV = V16<T>::N;
  constexpr U kS = FT<T>::kSign;
  int mism = 0;
  int q = 0;
  const uint32_t rstride = (uint32_t)NCH * 16u;
  // Bank rotation: the 16 lanes of a ds_read_b128 lane group read rows whose 16-byte chunk c
  // would fall on only 256 / rstride bank groups (rows of 2^k chunks: a 16 / (256 / rstride)-
  // way conflict).  Each lane reads its row's chunks rotated by (lane / rows-per-256-B):
  // conflict-free, and the row's min / second min / parity do not depend on the order.
  constexpr int kRows256 = 256 / (16 * NCH) > 0 ? 256 / (16 * NCH) : 1;
#ifndef QLDPC_ROT
#define QLDPC_ROT 1
#endif
  // fp32 2-chunk rows: 2-way only, not worth its VGPRs
#ifndef QLDPC_ROT32
#define QLDPC_ROT32 1
#endif
  // fp32 2-chunk rows: +1.2 % on n1600 (4 workgroups per CU), -1.5 % on the tail family (one)
  constexpr bool kRot =
      QLDPC_ROT && (((NCH == 4 || NCH == 8) && sizeof(T) == 8) || (QLDPC_ROT32 && NCH == 2 && sizeof(T) == 4 && !TAIL));
  const uint32_t rot = kRot ? ((uint32_t)(tid / kRows256) & (uint32_t)(NCH - 1)) : 0u;
  uint32_t coff[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) coff[c] = kRot ? (((uint32_t)c + rot) & (uint32_t)(NCH - 1)) * 16u : (uint32_t)c * 16u;
  // rows are loaded PFC (1 or 2) rows ahead of the one being reduced
  // (QLDPC_RC_RPTR: absolute LDS row / tail / CS addresses, as the m2s check phase's pointers; fp64
  // only: the two-word tail family +1.5 %, the fp32 families -0.6 %, profiles/r06/rc_rptr/)
  constexpr bool RP = QLDPC_RC_RPTR != 0 && sizeof(T) == 8;
  const uint32_t sbase = RP ? lds_base(smem) : 0u;
  auto load = [&](int r, VT (&v)[NCH], T& tv, uint32_t& fv) {
    if (r < m) {
      if constexpr (RP) {
        const uint32_t row = sbase + Ly.v + 16u + (uint32_t)r * rstride;
#pragma unroll
        for (int c = 0; c < NCH; ++c) v[c] = lds_ld<VT, true>(nullptr, row + coff[c]);
        if (TAIL) tv = lds_ld<T, true>(nullptr, sbase + Ly.t + (uint32_t)r * (uint32_t)sizeof(T));
      } else {
        const unsigned char* row = smem + Ly.v + 16 + (uint32_t)r * rstride;
#pragma unroll
        for (int c = 0; c < NCH; ++c) v[c] = *reinterpret_cast<const VT*>(row + coff[c]);
        if (TAIL) tv = lds_at<T>(smem, Ly.t + (uint32_t)r * (uint32_t)sizeof(T));
      }
      fv = f_ld<ENG>(smem, f_off<ENG>(Ly, r + 1));
    }
  };
  VT cur[NCH], mid[NCH];
  T tcur = (T)0, tmid = (T)0;  // TAIL: the row's slot in the tail array (sentinel when the row has no 9th edge)
  uint32_t fcur = 0, fmid = 0;
  int i = tid;
  if (PFC >= 1) load(i, cur, tcur, fcur);
  if (PFC == 2) load(i + TB, mid, tmid, fmid);
  for (; i < m; i += TB, ++q) {
    VT nxt[NCH];
    T tnxt = (T)0;
    uint32_t fnxt = 0;
    if (PFC == 0)
      load(i, cur, tcur, fcur);
    else
      load(i + PFC * TB, nxt, tnxt, fnxt);
    uint32_t s;
    if (FIRST) {
      s = ((fcur >> 1) ^ (fcur >> 2)) & 1u;  // as r_check: syndrome ^ row-degree parity
      sbits |= s << q;
      f_st<ENG>(smem, f_off<ENG>(Ly, i + 1), (fcur & 4u) | ((fcur >> 2) & 1u));
    } else {
      s = (sbits >> q) & 1u;
      mism |= (int)((fcur ^ s) & 1u);
    }
    typename CSEntry<T>::type st;
    if constexpr (sizeof(U) == 8) {
      double f1 = FT<T>::val(FT<T>::kSent), f2 = f1;
      uint32_t px = s ? 0x80000000u : 0u;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
#pragma unroll
        for (int k = 0; k < NV; ++k) {
          const double x = V16<T>::get(cur[c], k);
          double t;
          asm("v_max_f64 %0, %1, |%2|" : "=v"(t) : "v"(f1), "v"(x));
          asm("v_min_f64 %0, %1, %2" : "=v"(f2) : "v"(f2), "v"(t));
          asm("v_min_f64 %0, %1, |%2|" : "=v"(f1) : "v"(f1), "v"(x));
        }
        uint32_t p;
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96"
            : "=v"(p)
            : "v"(px), "v"((uint32_t)(FT<T>::bits(cur[c].x) >> 32)), "v"((uint32_t)(FT<T>::bits(cur[c].y) >> 32)));
        px = p;
      }
      if (TAIL) {
        const double x = (double)tcur;
        double t;
        asm("v_max_f64 %0, %1, |%2|" : "=v"(t) : "v"(f1), "v"(x));
        asm("v_min_f64 %0, %1, %2" : "=v"(f2) : "v"(f2), "v"(t));
        asm("v_min_f64 %0, %1, |%2|" : "=v"(f1) : "v"(f1), "v"(x));
        px ^= (uint32_t)(FT<T>::bits(tcur) >> 32);
      }
      st.a = FT<T>::bits(f1) | ((U)(px & 0x80000000u) << 32);
      st.b = FT<T>::bits(f2) | (QLDPC_F64_C2V5 ? ((U)(px & 0x80000000u) << 32) : (U)0);  // m2 | parity
    } else {
      float f1 = FT<T>::val(FT<T>::kSent), f2 = f1;
      uint32_t px = s ? kS : 0u;
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
#pragma unroll
        for (int k = 0; k < NV; ++k) {
          const float x = V16<T>::get(cur[c], k);
          f2 = __builtin_amdgcn_fmed3f(f1, f2, __builtin_fabsf(x));
          asm("v_min_f32 %0, %1, |%2|" : "=v"(f1) : "v"(f1), "v"(x));
        }
        uint32_t p01, p23;
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(p01) : "v"(px), "v"(FT<T>::bits(cur[c].x)), "v"(FT<T>::bits(cur[c].y)));
        asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(p23) : "v"(p01), "v"(FT<T>::bits(cur[c].z)), "v"(FT<T>::bits(cur[c].w)));
        px = p23;
      }
      if (TAIL) {
        const float x = (float)tcur;
        f2 = __builtin_amdgcn_fmed3f(f1, f2, __builtin_fabsf(x));
        asm("v_min_f32 %0, %1, |%2|" : "=v"(f1) : "v"(f1), "v"(x));
        px ^= (uint32_t)FT<T>::bits(tcur);
      }
      st.a = FT<T>::bits(f1) | (px & kS);
      st.b = FT<T>::bits(f2) | (QLDPC_F32_C2V4 ? (px & kS) : 0u);  // m2 | parity (r_var_one's 4-VALU c2v)
    }
    if constexpr (RP) {
      lds_st<typename CSEntry<T>::type, true>(nullptr, sbase + (uint32_t)(i + 1) * (uint32_t)(2 * sizeof(T)), st);
    } else {
      lds_at<typename CSEntry<T>::type>(smem, (uint32_t)(i + 1) * (uint32_t)(2 * sizeof(T))) = st;
    }
    if (PFC == 2) {
#pragma unroll
      for (int c = 0; c < NCH; ++c) {
        cur[c] = mid[c];
        mid[c] = nxt[c];
      }
      tcur = tmid;
      tmid = tnxt;
      fcur = fmid;
      fmid = fnxt;
    } else if (PFC == 1) {
#pragma unroll
      for (int c = 0; c < NCH; ++c) cur[c] = nxt[c];
      tcur = tnxt;
      fcur = fnxt;
    }
  }
  return mism;
}

// ------------------------------------------------------------------ m2-in-slot family
// (engine id + 10000, fp64, split absolute addresses, own v2c in VGPRs).  Per edge the variable
// phase gathers CS = m1 | parity (ds_read_b64) and the edge's own V slot (ds_read_b64); the
// check phase left m2 | parity in the slot of the row's argmin edge, so "slot != own previous
// v2c" marks the argmin and c2v = alpha * m2, else alpha * m1.  Same values as ldpc's "m2 if
// |own| == m1 else m1": with a tie m1 == m2; a slot equal to the own word by chance has
// m2 == m1 and the own sign == parity, i.e. the same c2v either way.
constexpr bool m_xmask(int eng) { return QLDPC_M2S_XMASK && eng_sh(eng) != 2; }

// the V slot address a gather computed is kept for the store (m_keepva): the sdwa unpack is an asm
// statement, which the backend cannot rematerialize once the value passes through an opaque copy
template <typename T, int DMAX, int VPL, int ENG>
constexpr bool m_keepva() {
  return QLDPC_M2S_KEEPVA && eng_m2s(ENG) && !eng_m2v(ENG) && !eng_c2s(ENG) && eng_sh(ENG) == 2 &&
         RState<T, DMAX, VPL, ENG>::kAbs && !RState<T, DMAX, VPL, ENG>::kSplit && !RState<T, DMAX, VPL, ENG>::kPk;
}

template <typename T, int DMAX, int VPL, int ND, int ENG, int D3K = 0, int LB = 256>
__device__ inline void m_gather(const RState<T, DMAX, VPL, ENG>& R, int k, typename FT<T>::U (&an)[DMAX],
                                typename FT<T>::U (&vn)[DMAX], uint32_t (&va)[DMAX]) {
  using U = typename FT<T>::U;
#pragma unroll
  for (int t = 0; t < ND; ++t) {
    if constexpr (!eng_c2s(ENG)) an[t] = lds_ld<U, true>(nullptr, r_csa(R, k, t));  // (c2s: ea = F word)
    if constexpr (eng_m2v(ENG)) {
      vn[t] = lds_ld<U, true>(nullptr, m2v_va<T, DMAX, VPL, ENG, D3K, LB>(R, k, t));
    } else if constexpr (m_keepva<T, DMAX, VPL, ENG>()) {
      uint32_t a = r_va(R, k, t);
      asm volatile("" : "+v"(a));
      va[t] = a;
      vn[t] = lds_ld<U, true>(nullptr, a);
    } else {
      vn[t] = lds_ld<U, true>(nullptr, r_va(R, k, t));
    }
  }
}

template <typename T, int DMAX, int VPL, int ND, int ENG, int D3K = 0, int LB = 256>
__device__ inline bool m_var_one(unsigned char* smem, RState<T, DMAX, VPL, ENG>& R, int k,
                                 const typename FT<T>::U (&an)[DMAX],
                                 const typename FT<T>::U (&vn)[DMAX], const uint32_t (&va)[DMAX], uint32_t fdelta,
                                 T alpha, bool xprev, uint64_t& xmk, double* post, const int32_t* perm) {
  using U = typename FT<T>::U;
  constexpr bool KV1 = RState<T, DMAX, VPL, ENG>::kKeepV;
  static_assert(sizeof(T) == 8 && RState<T, DMAX, VPL, ENG>::kAbs && (RState<T, DMAX, VPL, ENG>::kKeepV || eng_c2s(ENG)),
                "m2s / c2s: fp64 absolute-address families only");
  T c[ND];
#pragma unroll
  for (int t = 0; t < ND; ++t) {
    if constexpr (eng_c2s(ENG)) {  // the slot holds this edge's c2v (c2s_check)
      c[t] = FT<T>::val(vn[t]);
      continue;
    }
    const U o = R.ov[KV1 ? k : 0][KV1 ? t : 0];
    // argmin edge <=> its slot no longer holds our own previous v2c: m2 | parity, else m1 | parity
    const U sel = vn[t] != o ? vn[t] : an[t];
    // sign(sel) = parity; sel * alpha is exactly +-(|sel| * alpha) (IEEE rounding is sign-symmetric),
    // then the own sign: c2v sign = parity ^ own sign (one v_bitop3, truth table S1 ^ (S0 & S2))
    const U pb = FT<T>::bits(FT<T>::val(sel) * alpha);
    uint32_t hi;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x6c"
        : "=v"(hi)
        : "v"((uint32_t)(o >> 32)), "v"((uint32_t)(pb >> 32)), "v"(0x80000000u));
    c[t] = FT<T>::val(((U)hi << 32) | (uint32_t)pb);
  }
  // ldpc column pass (as r_var_one)
  T f[ND];
  T acc = r_prior(R, k);
#pragma unroll
  for (int t = 0; t < ND; ++t) {
    f[t] = acc;
    acc = acc + c[t];
  }
  const bool x = acc >= (T)0;  // w domain: v <= 0
  if (post) {
    const int j = *perm;
    if (j >= 0) post[j] = -(double)acc;
  }
  T b = c[ND - 1];
  U nv[ND];
  nv[ND - 1] = FT<T>::bits(f[ND - 1]);
#pragma unroll
  for (int t = ND - 2; t >= 0; --t) {
    nv[t] = FT<T>::bits(f[t] + b);
    if (t > 0) b = b + c[t];
  }
#pragma unroll
  for (int t = 0; t < ND; ++t) {
    if constexpr (eng_m2v(ENG))
      lds_st<U, true>(nullptr, m2v_va<T, DMAX, VPL, ENG, D3K, LB>(R, k, t), nv[t]);
    else if constexpr (m_keepva<T, DMAX, VPL, ENG>())
      lds_st<U, true>(nullptr, va[t], nv[t]);
    else
      lds_st<U, true>(nullptr, r_va(R, k, t), nv[t]);
    if constexpr (KV1) R.ov[k][t] = nv[t];
  }
  bool flip;
  if constexpr (m_xmask(ENG)) {  // (every lane active here: the variable phase is not divergent)
    const uint64_t bx = __ballot(x);
    flip = __builtin_amdgcn_inverse_ballot_w64(bx ^ xmk);
    xmk = bx;
  } else {
    flip = x != xprev;
  }
  if (flip) {
#pragma unroll
    for (int t = 0; t < ND; ++t) {
      if constexpr (eng_c2s(ENG))
        lds_xor_abs(R.ea[k][t], 1u);
      else
        atomicXor(&lds_at<uint32_t>(smem, r_fa(R, k, t, fdelta)), 1u);
    }
  }
  return x;
}

template <typename T, int DMAX, int VPL, int D3K, int ENG, int LB = 256>
__device__ inline uint32_t m_var(unsigned char* smem, RState<T, DMAX, VPL, ENG>& R, uint32_t fdelta, T alpha, uint32_t xprev,
                                 uint64_t (&xm)[VPL], bool last_live, double* post = nullptr, const int32_t* perm = nullptr,
                                 int TB = 0, uint32_t nwm = 0) {
  using U = typename FT<T>::U;
  constexpr int N3 = DMAX > 3 ? 3 : DMAX;
  // gathers one variable ahead: two ahead needs 32 more VGPRs than the 168 of 3 workgroups per
  // CU and spills (n1600: 849k vs 1.13M shots/s, profiles/r03/m2s_ab/)
  // c2s keeps no own v2c (48 VGPRs fewer): QLDPC_C2S_PF variables ahead
  constexpr int PF0 = eng_c2s(ENG) ? QLDPC_C2S_PF : QLDPC_PF >= 1 ? QLDPC_PF : 1;
  constexpr int PF = PF0 < VPL ? PF0 : VPL;
  r_launder<T, DMAX, VPL, ENG, D3K>(R);
  uint32_t xbits = 0;
  U ab[PF][DMAX], vb[PF][DMAX];
  uint32_t vab[PF][DMAX];
  auto gk = [&](int k, U (&an)[DMAX], U (&vn)[DMAX], uint32_t (&va)[DMAX]) {
    if (k < eng_d2k(ENG))  // (the space-time family's measurement variables: two edge slots)
      m_gather<T, DMAX, VPL, 2, ENG, D3K, LB>(R, k, an, vn, va);
    else if (k < D3K)
      m_gather<T, DMAX, VPL, N3, ENG, D3K, LB>(R, k, an, vn, va);
    else
      m_gather<T, DMAX, VPL, DMAX, ENG, D3K, LB>(R, k, an, vn, va);
  };
#pragma unroll
  for (int k = 0; k < PF; ++k) gk(k, ab[k], vb[k], vab[k]);
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    U an[DMAX], vn[DMAX];
    uint32_t va[DMAX];
#pragma unroll
    for (int t = 0; t < DMAX; ++t) {
      an[t] = ab[k % PF][t];
      vn[t] = vb[k % PF][t];
      va[t] = vab[k % PF][t];
    }
    if (k + PF < VPL) gk(k + PF, ab[k % PF], vb[k % PF], vab[k % PF]);
    if (k == VPL - 1 && !last_live) break;
    const bool xp = ((xprev >> k) & 1u) != 0;
    const int32_t* pk = perm ? perm + k * TB : nullptr;
    bool x;
    // (narrow waves: bit k of the wave-uniform nwm = this wave computes slot k one edge slot narrower)
    if (eng_nw(ENG) && k < kNwSlots && ((nwm >> k) & 1u))
      x = k < eng_d2k(ENG) ? m_var_one<T, DMAX, VPL, 1, ENG, D3K, LB>(smem, R, k, an, vn, va, fdelta, alpha, xp, xm[k], post, pk)
          : k < D3K        ? m_var_one<T, DMAX, VPL, (N3 > 1 ? N3 - 1 : 1), ENG, D3K, LB>(smem, R, k, an, vn, va, fdelta, alpha, xp, xm[k], post, pk)
                           : m_var_one<T, DMAX, VPL, (DMAX > 1 ? DMAX - 1 : 1), ENG, D3K, LB>(smem, R, k, an, vn, va, fdelta, alpha, xp, xm[k], post, pk);
    else
      x = k < eng_d2k(ENG) ? m_var_one<T, DMAX, VPL, 2, ENG, D3K, LB>(smem, R, k, an, vn, va, fdelta, alpha, xp, xm[k], post, pk)
          : k < D3K        ? m_var_one<T, DMAX, VPL, N3, ENG, D3K, LB>(smem, R, k, an, vn, va, fdelta, alpha, xp, xm[k], post, pk)
                           : m_var_one<T, DMAX, VPL, DMAX, ENG, D3K, LB>(smem, R, k, an, vn, va, fdelta, alpha, xp, xm[k], post, pk);
    if constexpr (!m_xmask(ENG)) xbits |= (x ? 1u : 0u) << k;
  }
  return xbits;
}

// m2s check phase (rows of NCH chunks + a tail slot when TAIL; fp64): min / second min / parity
// as r_check_c plus the row's argmin slot (first strict minimum); CS[i+1] = m1 | parity and
// V[argmin] = m2 | parity.  Any edge holding m1 would do as the argmin: with a tie m2 == m1.
template <typename T, bool FIRST, int NCH, int TAIL>
__device__ inline int m_check(unsigned char* smem, const RLayout& Ly, int m, int wbase, int wtid, int TB, uint32_t& sbits) {
  using U = typename FT<T>::U;
  using VT = typename V16<T>::type;
  constexpr int NV = V16<T>::N;
  static_assert(sizeof(T) == 8, "m2s: fp64 only");
  int mism = 0;
  int q = 0;
#if QLDPC_M2S_MBCNT
  // tid from the wave's base (an SGPR) and the lane's mbcnt: no VGPR holds tid across the
  // variable phase (A/B build: the register allocator then spills elsewhere)
  const int tid = wbase + (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
#else
  // opaque tid: the row / F / tail offsets are recomputed per pass instead of being hoisted out
  // of the iteration loop (where they outlive the variable phase and spill)
  int tid = wtid;
  asm volatile("" : "+v"(tid));
  (void)wbase;
#endif
  const uint32_t rstride = (uint32_t)NCH * 16u;
  // chunk rotation for power-of-two rows (as r_check_c); rows of 3 chunks are conflict-free
  constexpr int kRows256 = 256 / (16 * NCH) > 0 ? 256 / (16 * NCH) : 1;
  constexpr bool kRot = QLDPC_ROT && (NCH == 4 || NCH == 8);
  const uint32_t rot = kRot ? ((uint32_t)(tid / kRows256) & (uint32_t)(NCH - 1)) : 0u;
  uint32_t coff[NCH];
#pragma unroll
  for (int c = 0; c < NCH; ++c) coff[c] = kRot ? (((uint32_t)c + rot) & (uint32_t)(NCH - 1)) * 16u : (uint32_t)c * 16u;
  // explicit absolute row pointers (QLDPC_M2S_RPTR): one row base stepped per row (opaque, so the
  // backend neither splits it into one induction variable per chunk nor re-adds the region offset
  // per row) plus the tail, F and CS pointers; the argmin is selected as an offset from the row base
  constexpr bool AP = QLDPC_M2S_RPTR;
  const uint32_t sb = AP ? lds_base(smem) : 0u;
  uint32_t rb = sb + Ly.v + 16u + (uint32_t)tid * rstride;
  uint32_t tp = sb + Ly.t + (uint32_t)tid * (uint32_t)sizeof(T);
  uint32_t fp = sb + Ly.f + 4u * (uint32_t)(tid + 1);
  uint32_t cp = sb + (uint32_t)(tid + 1) * (uint32_t)sizeof(T);
  // one row: its loads, then its reduction and stores (kept apart so that rows can be loaded in pairs)
  struct RowIn {
    VT cur[NCH];
    T tcur;
    uint32_t fcur, roff, toff, fo, co;
  };
  // (c0..c1: the chunks to load; the tail and F word with the last chunk)
  auto load_row = [&](RowIn& r, int i, uint32_t rb_, uint32_t tp_, uint32_t fp_, uint32_t cp_, int c0 = 0, int c1 = NCH) {
    r.roff = AP ? rb_ : Ly.v + 16u + (uint32_t)i * rstride;
    r.toff = AP ? tp_ : Ly.t + (uint32_t)i * (uint32_t)sizeof(T);
    r.fo = AP ? fp_ : Ly.f + 4u * (uint32_t)(i + 1);
    r.co = AP ? cp_ : (uint32_t)(i + 1) * (uint32_t)sizeof(T);
#pragma unroll
    for (int c = 0; c < NCH; ++c)
      if (c >= c0 && c < c1) r.cur[c] = lds_ld<VT, AP>(smem, r.roff + coff[c]);
    if (c1 == NCH) {
      r.tcur = (T)0;
      if (TAIL) r.tcur = lds_ld<T, AP>(smem, r.toff);
      r.fcur = lds_ld<uint32_t, AP>(smem, r.fo);
    }
  };
  auto reduce_row = [&](const RowIn& r, int qq) {
    uint32_t s;
    if (FIRST) {
      s = ((r.fcur >> 1) ^ (r.fcur >> 2)) & 1u;
      sbits |= s << qq;
      lds_st<uint32_t, AP>(smem, r.fo, (r.fcur & 4u) | ((r.fcur >> 2) & 1u));
    } else {
      s = (sbits >> qq) & 1u;
      mism |= (int)((r.fcur ^ s) & 1u);
    }
    double f1 = FT<T>::val(FT<T>::kSent), f2 = f1;
    uint32_t px = s ? 0x80000000u : 0u;
    uint32_t aoff = coff[0];  // argmin slot (offset from the row base); any slot when no edge is below the sentinel
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const double x = V16<T>::get(r.cur[c], k);
        aoff = __builtin_fabs(x) < f1 ? coff[c] + 8u * (uint32_t)k : aoff;
        double t;
        asm("v_max_f64 %0, %1, |%2|" : "=v"(t) : "v"(f1), "v"(x));
        asm("v_min_f64 %0, %1, %2" : "=v"(f2) : "v"(f2), "v"(t));
        asm("v_min_f64 %0, %1, |%2|" : "=v"(f1) : "v"(f1), "v"(x));
      }
      uint32_t p;
      asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96"
          : "=v"(p)
          : "v"(px), "v"((uint32_t)(FT<T>::bits(r.cur[c].x) >> 32)), "v"((uint32_t)(FT<T>::bits(r.cur[c].y) >> 32)));
      px = p;
    }
    uint32_t amin = r.roff + aoff;
    if (TAIL) {
      const double x = (double)r.tcur;
      amin = __builtin_fabs(x) < f1 ? r.toff : amin;
      double t;
      asm("v_max_f64 %0, %1, |%2|" : "=v"(t) : "v"(f1), "v"(x));
      asm("v_min_f64 %0, %1, %2" : "=v"(f2) : "v"(f2), "v"(t));
      asm("v_min_f64 %0, %1, |%2|" : "=v"(f1) : "v"(f1), "v"(x));
      px ^= (uint32_t)(FT<T>::bits(r.tcur) >> 32);
    }
    const U par = (U)(px & 0x80000000u) << 32;
    lds_st<U, AP>(smem, r.co, FT<T>::bits(f1) | par);
    lds_st<U, AP>(smem, amin, FT<T>::bits(f2) | par);
  };
  const uint32_t drb = (uint32_t)TB * rstride, dtp = (uint32_t)TB * (uint32_t)sizeof(T), dfp = 4u * (uint32_t)TB,
                 dcp = (uint32_t)TB * (uint32_t)sizeof(T);
  // QLDPC_M2S_ROWPAIR (the space-time family: one decode per CU, 1-2 rows per thread): both rows' loads
  // are issued before the first row is reduced (their addresses never alias: distinct rows, tails, F
  // words and CS entries), so the second row's LDS latency hides under the first row's arithmetic
  if constexpr (QLDPC_M2S_ROWPAIR > 0 && TAIL && NCH == 4) {
    for (int i = tid; i < m; i += 2 * TB, q += 2) {
      if constexpr (AP) asm volatile("" : "+v"(rb));
      RowIn a, b;
      load_row(a, i, rb, tp, fp, cp);
      const bool hb = i + TB < m;
      // the second row's first QLDPC_M2S_ROWPAIR chunks ahead, the rest after the first row (VGPRs)
      constexpr int PC = QLDPC_M2S_ROWPAIR < NCH ? QLDPC_M2S_ROWPAIR : NCH;
      if (hb) load_row(b, i + TB, rb + drb, tp + dtp, fp + dfp, cp + dcp, 0, PC);
      reduce_row(a, q);
      if (hb) {
        if constexpr (PC < NCH) load_row(b, i + TB, rb + drb, tp + dtp, fp + dfp, cp + dcp, PC, NCH);
        reduce_row(b, q + 1);
      }
      rb += 2 * drb;
      tp += 2 * dtp;
      fp += 2 * dfp;
      cp += 2 * dcp;
    }
  } else {
    for (int i = tid; i < m; i += TB, ++q) {
      if constexpr (AP) asm volatile("" : "+v"(rb));
      RowIn a;
      load_row(a, i, rb, tp, fp, cp);
      reduce_row(a, q);
      rb += drb;
      tp += dtp;
      fp += dfp;
      cp += dcp;
    }
  }
  return mism;
}

// m2v check phase (fp64): row q of this thread (check i = tid + q * TB) gathers its 7 V slots
// through the register table (scattered ds_read_b64), then min / second min / parity / argmin as
// m_check: CS[i+1] = m1 | parity, V[argmin] = m2 | parity.  Rows of fewer edges point their unused
// entries at a slot that holds the sentinel forever (never the argmin: no edge is below it).
template <typename T, bool FIRST>
__device__ inline int m2v_check(unsigned char* smem, const RLayout& Ly, int m, int tid, int TB, uint32_t& sbits,
                                const M2vRows& RW, uint32_t vbase) {
  using U = typename FT<T>::U;
  static_assert(sizeof(T) == 8, "m2v: fp64 only");
  int mism = 0;
#pragma unroll
  for (int q = 0; q < kM2vRows; ++q) {
    const int i = tid + q * TB;
    if (i >= m) break;
    const uint32_t wd[4] = {RW.w[q].x, RW.w[q].y, RW.w[q].z, RW.w[q].w};
    uint32_t a[7];
#pragma unroll
    for (int e = 0; e < 7; ++e) a[e] = vbase + ((e & 1) ? (wd[e >> 1] >> 16) : (wd[e >> 1] & 0xFFFFu));
    double x[7];
#pragma unroll
    for (int e = 0; e < 7; ++e) x[e] = FT<T>::val(lds_ld<U, true>(nullptr, a[e]));
    const uint32_t fo = Ly.f + 4u * (uint32_t)(i + 1);
    const uint32_t fcur = lds_at<uint32_t>(smem, fo);
    uint32_t s;
    if (FIRST) {
      s = ((fcur >> 1) ^ (fcur >> 2)) & 1u;
      sbits |= s << q;
      lds_at<uint32_t>(smem, fo) = (fcur & 4u) | ((fcur >> 2) & 1u);
    } else {
      s = (sbits >> q) & 1u;
      mism |= (int)((fcur ^ s) & 1u);
    }
    double f1 = FT<T>::val(FT<T>::kSent), f2 = f1;
    uint32_t px = s ? 0x80000000u : 0u;
    uint32_t amin = a[0];
#pragma unroll
    for (int e = 0; e < 7; ++e) {
      amin = __builtin_fabs(x[e]) < f1 ? a[e] : amin;
      double t;
      asm("v_max_f64 %0, %1, |%2|" : "=v"(t) : "v"(f1), "v"(x[e]));
      asm("v_min_f64 %0, %1, %2" : "=v"(f2) : "v"(f2), "v"(t));
      asm("v_min_f64 %0, %1, |%2|" : "=v"(f1) : "v"(f1), "v"(x[e]));
    }
#pragma unroll
    for (int e = 0; e + 1 < 7; e += 2) {
      uint32_t p;
      asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96"
          : "=v"(p)
          : "v"(px), "v"((uint32_t)(FT<T>::bits(x[e]) >> 32)), "v"((uint32_t)(FT<T>::bits(x[e + 1]) >> 32)));
      px = p;
    }
    px ^= (uint32_t)(FT<T>::bits(x[6]) >> 32);
    const U par = (U)(px & 0x80000000u) << 32;
    lds_at<U>(smem, (uint32_t)(i + 1) * (uint32_t)sizeof(T)) = FT<T>::bits(f1) | par;
    lds_st<U, true>(nullptr, amin, FT<T>::bits(f2) | par);
  }
  return mism;
}

// c2s check phase (rows of exactly 2 * NCH + TAIL edges; fp64): min / second min / parity / argmin
// as m_check, then the c2v of the NEXT variable phase into the row's own slots: every edge gets
// alpha * m1 with sign parity ^ own sign, written as {lo(a1), hi(a1) ^ parity ^ (own hi & sign)}
// (one v_bitop3 per edge, the low word shared), and one ds_xor_b64 of bits(a1) ^ bits(a2) turns the
// argmin's word into alpha * m2 with the same sign.  alpha * m with the sign applied afterwards is
// bit-identical to ldpc's (+-m) * alpha (IEEE rounding is sign-symmetric); with a tie m1 == m2 and
// the xor is zero.
template <typename T, bool FIRST, int NCH, int TAIL>
__device__ inline int c2s_check(unsigned char* smem, const RLayout& Ly, int m, int wtid, int TB, uint32_t& sbits,
                                T alpha) {
  using U = typename FT<T>::U;
  using VT = typename V16<T>::type;
  constexpr int NV = V16<T>::N;
  static_assert(sizeof(T) == 8, "c2s: fp64 only");
  int mism = 0;
  int q = 0;
  int tid = wtid;  // opaque: the row offsets are re-derived per pass (as m_check)
  asm volatile("" : "+v"(tid));
  const uint32_t rstride = (uint32_t)NCH * 16u;
  for (int i = tid; i < m; i += TB, ++q) {
    const uint32_t roff = Ly.v + 16u + (uint32_t)i * rstride;
    VT cur[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) cur[c] = *reinterpret_cast<const VT*>(smem + roff + 16u * (uint32_t)c);
    const uint32_t toff = Ly.t + (uint32_t)i * (uint32_t)sizeof(T);
    T tcur = (T)0;
    if (TAIL) tcur = lds_at<T>(smem, toff);
    const uint32_t fcur = lds_at<uint32_t>(smem, Ly.f + 4u * (uint32_t)(i + 1));
    uint32_t s;
    if (FIRST) {
      s = ((fcur >> 1) ^ (fcur >> 2)) & 1u;
      sbits |= s << q;
      lds_at<uint32_t>(smem, Ly.f + 4u * (uint32_t)(i + 1)) = (fcur & 4u) | ((fcur >> 2) & 1u);
    } else {
      s = (sbits >> q) & 1u;
      mism |= (int)((fcur ^ s) & 1u);
    }
    double f1 = FT<T>::val(FT<T>::kSent), f2 = f1;
    uint32_t px = s ? 0x80000000u : 0u;
    uint32_t amin = roff;  // argmin slot (byte offset)
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const double x = V16<T>::get(cur[c], k);
        amin = __builtin_fabs(x) < f1 ? roff + 16u * (uint32_t)c + 8u * (uint32_t)k : amin;
        double t;
        asm("v_max_f64 %0, %1, |%2|" : "=v"(t) : "v"(f1), "v"(x));
        asm("v_min_f64 %0, %1, %2" : "=v"(f2) : "v"(f2), "v"(t));
        asm("v_min_f64 %0, %1, |%2|" : "=v"(f1) : "v"(f1), "v"(x));
      }
      uint32_t p;
      asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96"
          : "=v"(p)
          : "v"(px), "v"((uint32_t)(FT<T>::bits(cur[c].x) >> 32)), "v"((uint32_t)(FT<T>::bits(cur[c].y) >> 32)));
      px = p;
    }
    if (TAIL) {
      const double x = (double)tcur;
      amin = __builtin_fabs(x) < f1 ? toff : amin;
      double t;
      asm("v_max_f64 %0, %1, |%2|" : "=v"(t) : "v"(f1), "v"(x));
      asm("v_min_f64 %0, %1, %2" : "=v"(f2) : "v"(f2), "v"(t));
      asm("v_min_f64 %0, %1, |%2|" : "=v"(f1) : "v"(f1), "v"(x));
      px ^= (uint32_t)(FT<T>::bits(tcur) >> 32);
    }
    const U a1 = FT<T>::bits(f1 * alpha);
    const U a2 = FT<T>::bits(f2 * alpha);
    const uint32_t lo = (uint32_t)a1;
    const uint32_t ah = (uint32_t)(a1 >> 32) ^ (px & 0x80000000u);
    auto hiw = [&](double x) {
      uint32_t hi;
      asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x6c"
          : "=v"(hi)
          : "v"((uint32_t)(FT<T>::bits(x) >> 32)), "v"(ah), "v"(0x80000000u));
      return hi;
    };
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const uint32_t off = roff + 16u * (uint32_t)c;
      if (QLDPC_C2S_W128) {  // one 16-byte store per chunk (conflict-free at the 48-byte row stride)
        typename LdsWord<16>::type w;
        w.x = lo;
        w.y = hiw(cur[c].x);
        w.z = lo;
        w.w = hiw(cur[c].y);
        *reinterpret_cast<typename LdsWord<16>::type*>(smem + off) = w;
      } else {
        lds_at<uint32_t>(smem, off) = lo;
        lds_at<uint32_t>(smem, off + 4u) = hiw(cur[c].x);
        lds_at<uint32_t>(smem, off + 8u) = lo;
        lds_at<uint32_t>(smem, off + 12u) = hiw(cur[c].y);
      }
    }
    if (TAIL) {
      lds_at<uint32_t>(smem, toff) = lo;
      lds_at<uint32_t>(smem, toff + 4u) = hiw((double)tcur);
    }
    atomicXor(reinterpret_cast<unsigned long long*>(&lds_at<U>(smem, amin)), (unsigned long long)(a1 ^ a2));
  }
  return mism;
}

// Engine-4 variable phase: c2v from the slots, ldpc's column pass, v2c back.
// Variable VPL-1 is skipped by waves whose lanes are all padding.
template <typename T, int DMAX, int VPL>
__device__ inline uint32_t c_var(unsigned char* smem, RState<T, DMAX, VPL, 4>& R, const FMap& M, bool last_live) {
  using U = typename FT<T>::U;
  r_launder(R);
  uint32_t xbits = 0;
  T cn[DMAX];
#pragma unroll
  for (int t = 0; t < DMAX; ++t) cn[t] = lds_at<T>(smem, R.ea[0][t] & 0xFFFFu);
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    T c[DMAX];
#pragma unroll
    for (int t = 0; t < DMAX; ++t) c[t] = cn[t];
    if (k + 1 < VPL) {  // next variable's reads go out before this one's arithmetic
#pragma unroll
      for (int t = 0; t < DMAX; ++t) cn[t] = lds_at<T>(smem, R.ea[k + 1][t] & 0xFFFFu);
    }
    if (k == VPL - 1 && !last_live) break;
    T f[DMAX];
    T acc = R.L[k];
#pragma unroll
    for (int t = 0; t < DMAX; ++t) {
      f[t] = acc;
      acc = acc + c[t];
    }
    const bool x = acc <= (T)0;
    xbits |= (x ? 1u : 0u) << k;
    T b = c[DMAX - 1];
    U nv[DMAX];
    nv[DMAX - 1] = canon2<T>(f[DMAX - 1]);
#pragma unroll
    for (int t = DMAX - 2; t >= 0; --t) {
      nv[t] = canon2<T>(f[t] + b);
      if (t > 0) b = b + c[t];
    }
#pragma unroll
    for (int t = 0; t < DMAX; ++t) lds_at<U>(smem, R.ea[k][t] >> 16) = nv[t];
    if (x) {
#pragma unroll
      for (int t = 0; t < DMAX; ++t) atomicXor(&lds_at<uint32_t>(smem, f_addr<T, 4>(R.ea[k][t], M)), 1u);
    }
  }
  return xbits;
}

// Engine-4 check phase over rows with NCH 16-byte chunks: syndrome / (H x)
// test as r_check, then every slot of the row receives its c2v for the next
// variable phase (computed with `alpha`); padding slots get the sentinel.
template <typename T, bool FIRST, int NCH>
__device__ inline int c_check(unsigned char* smem, const RLayout& Ly, int m, int tid, int TB, uint32_t& sbits,
                              T alpha) {
  using U = typename FT<T>::U;
  using VT = typename V16<T>::type;
  constexpr int NV = V16<T>::N;
  constexpr U kS = FT<T>::kSign;
  int mism = 0;
  int q = 0;
  for (int i = tid; i < m; i += TB, ++q) {
    VT* row = reinterpret_cast<VT*>(smem + Ly.v + 16 + (uint32_t)i * (uint32_t)(NCH * 16));
    uint32_t& F = lds_at<uint32_t>(smem, Ly.f + 4u * (uint32_t)(i + 1));
    const uint32_t f = F;
    uint32_t s;
    if (FIRST) {
      s = (f >> 1) & 1u;
      sbits |= s << q;
    } else {
      s = (sbits >> q) & 1u;
      mism |= (int)((f ^ s) & 1u);
    }
    F = f & 0xFFFF0000u;  // keep the row degree
    const int deg = (int)(f >> 16);
    U xb[NCH * NV];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const VT v = row[c];
#pragma unroll
      for (int k = 0; k < NV; ++k) xb[c * NV + k] = FT<T>::bits(V16<T>::get(v, k));
    }
    U m1 = FT<T>::kSent, m2 = FT<T>::kSent;
    U px = s ? kS : (U)0;
#pragma unroll
    for (int e = 0; e < NCH * NV; ++e) {
      const U a = xb[e] & ~kS;
      if constexpr (sizeof(U) == 4) {
        m2 = med3u(m1, m2, a);
      } else {
        const U hi = m1 > a ? m1 : a;
        m2 = m2 < hi ? m2 : hi;
      }
      m1 = m1 < a ? m1 : a;
      px ^= xb[e];
    }
    // chunk swizzle of build_slot_edges (qldpc_hip.hip): physical chunk c holds logical chunk c ^ swz
    const int swz = NCH == 2 ? ((i >> 3) & 1) : NCH == 4 ? ((i >> 2) & 3) : 0;
    const T sm1 = FT<T>::val(m1) * alpha, sm2 = FT<T>::val(m2) * alpha;
    const U b1 = FT<T>::bits(sm1), b2 = FT<T>::bits(sm2);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int lim = deg - (c ^ swz) * NV;  // slots k < lim of this chunk are real edges
      U o[NV];
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const U x = xb[c * NV + k];
        const U sel = ((x & ~kS) == m1) ? b2 : b1;  // |c2v| = alpha * (min over the other edges)
        const U cv = sel ^ ((px ^ x) & kS);         // sign = parity of the others and the syndrome
        o[k] = k < lim ? cv : FT<T>::kSent;
      }
      VT w;
      if constexpr (NV == 4) {
        w = make_float4(FT<T>::val(o[0]), FT<T>::val(o[1]), FT<T>::val(o[2]), FT<T>::val(o[3]));
      } else {
        w = make_double2(FT<T>::val(o[0]), FT<T>::val(o[1]));
      }
      row[c] = w;
    }
  }
  return mism;
}

template <typename T, int ENG>
__device__ inline void r_fill(const SSector& S, unsigned char* smem, const RLayout& Ly, int vslots, int mmax, int tid,
                              int TB) {
  using VT = typename V16<T>::type;
  VT* V4 = reinterpret_cast<VT*>(smem + Ly.v);
  const VT s = V16<T>::splat(FT<T>::val(FT<T>::kSent));
  // engine 4: the first chunk is the zero chunk missing edges read
  (void)vslots;
  const int nchunks = (int)((Ly.f - Ly.v) / 16u);  // V rows and (tail layouts) the tail slots
  for (int i = tid; i < nchunks; i += TB) V4[i] = (eng_base(ENG) == 4 && i == 0) ? V16<T>::splat((T)0) : s;
  // engine 4: row degree in the high half; engine 3: row-degree parity in bit 2 (w domain)
  for (int i = tid; i <= mmax; i += TB)
    f_st<ENG>(smem, f_off<ENG>(Ly, i),
              (i >= 1 && i <= S.m) ? (eng_base(ENG) == 4 ? ((uint32_t)S.rdeg[i - 1] << 16) : (((uint32_t)S.rdeg[i - 1] & 1u) << 2))
                                   : 0u);
  uint32_t* lred = reinterpret_cast<uint32_t*>(smem + Ly.lred);
  if (tid < 10) lred[tid] = 0;  // lred[0..7], flags[0..1]
  if (eng_base(ENG) == 3 && tid == 0) {
    // missing-edge dummy: c2v = ±0 (an opaque zero: a hoisted zero pair outlives the loops)
    uint32_t zz = 0;
    asm volatile("" : "+v"(zz));
    Pair<T> z;
    z.a = (typename FT<T>::U)zz;
    z.b = (typename FT<T>::U)zz;
    lds_at<Pair<T>>(smem, 0) = z;
  }
}

// Engine 4 lays every row out as 8 slots (row degree <= 8): 2 chunks in fp32,
// 4 in fp64 (one compile-time row width keeps the check phase's VGPRs low).
template <typename T>
constexpr int kRowChunks4 = 8 * (int)sizeof(T) / 16;
template <typename T, bool FIRST>
__device__ inline int c_check_any(unsigned char* smem, const RLayout& Ly, int m, int nch, int tid, int TB,
                                  uint32_t& sbits, T alpha) {
  (void)nch;  // == kRowChunks4<T> (host-enforced)
  return c_check<T, FIRST, kRowChunks4<T>>(smem, Ly, m, tid, TB, sbits, alpha);
}

// One sector pass over `cn` shots (chunk-relative), one decode in flight.
template <typename T, int DMAX, int VPL, bool MC, int ENG, int D3K, int NCH = 0>
__device__ void r_pass(const SSector& S, int q, long long c0, int cn, unsigned char* smem, const RLayout& Ly,
                       int vslots, int mmax, uint32_t* failmap, unsigned long long* cnt, const SMcArgs* A,
                       const SDecArgs* D, int tid, int TB) {
  using U = typename FT<T>::U;
  constexpr bool KV = RState<T, DMAX, VPL, ENG>::kKeepV;
  const int m = S.m, n = S.n, nch = S.nch;
  // Re-derive tid-based table addresses in every pass: without the opaque copy the
  // compiler hoists ~20 64-bit addresses out of the chunk loop and spills them.
  int tidp = tid;
#if QLDPC_TID_LAUNDER
  asm volatile("" : "+v"(tidp));
#endif
  RState<T, DMAX, VPL, ENG> R;
  constexpr bool SP = RState<T, DMAX, VPL, ENG>::kSplit;
  const int wbase = (int)__builtin_amdgcn_readfirstlane((uint32_t)tid) & ~63;  // (m2s check phase)
  const uint32_t sbase = lds_base(smem);
  r_load<T, DMAX, VPL, ENG>(S, R, Ly, tidp, TB, sbase);
  r_fill<T, ENG>(S, smem, Ly, vslots, mmax, tidp, TB);
  FMap M;
  M.fbase = eng_base(ENG) == 4 ? Ly.f + 4u : Ly.f;
  M.rstart = Ly.v + 16u;
  M.rsh = 4 + __builtin_ctz((unsigned)nch);
  // absolute CS addresses (split or kAbs; 16-byte aligned base): fbase absorbs the base
  constexpr bool AB = RState<T, DMAX, VPL, ENG>::kAbs;
  if (AB) M.fbase = Ly.f - (sbase >> (eng_fb(ENG) ? 3 : (sizeof(T) == 4 || eng_m2s(ENG)) ? 1 : 2));
  const uint32_t fdelta = eng_base(ENG) == 4 ? Ly.f : M.fbase;
  // waves whose lanes all hold padding variables skip the last variable (engine 4)
  // (the fp64 space-time m2s family places its waves over the SIMDs: a mask, not a prefix)
  const bool last_live = eng_nw(ENG) ? ((S.live_last >> ((uint32_t)wbase >> 6)) & 1u) != 0
                                     : uni((VPL - 1) * TB + (tid & ~63) < S.npos ? 1 : 0) != 0;
  // narrow-wave mask of this wave (eng_nw: bit k = slot k one edge slot narrower), scalar
  uint32_t nwm = 0;
  if constexpr (eng_nw(ENG)) {
    const uint32_t wv = (uint32_t)wbase >> 6;
#pragma unroll
    for (int k = 0; k < kNwSlots && k < VPL; ++k) nwm |= ((S.nw >> (16 * k + wv)) & 1u) << k;
    nwm = __builtin_amdgcn_readfirstlane(nwm);
  }
  uint32_t* lred = reinterpret_cast<uint32_t*>(smem + Ly.lred);
  uint32_t* flags = lred + 8;
  const bool adaptive = S.alpha == 0.0;
  const T alpha_fixed = (T)S.alpha;
  __syncthreads();

  int pshot = -1, pit = 0, pconv = 0;
  // QLDPC_STAMPS: [0] variable phase, [1] its barrier, [2] check phase, [3] flags + barrier,
  // [4] shot setup (priors, sampling), [5] epilogue, [6] iterations, [7] shots,
  // [8] setup barrier + previous decode's bookkeeping, [9] first check pass + barrier
  unsigned long long st_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long st_a = qstamp();
  for (int sh = 0; sh <= cn; ++sh) {
    const bool have = sh < cn;
    uint32_t eb = 0, sb = 0;
    r_launder<T, DMAX, VPL, ENG, D3K>(R);
    int tidl = tid;  // opaque copy: keeps per-variable addresses from being hoisted (VGPRs)
    asm volatile("" : "+v"(tidl));
    // ---------------------------------------------------------- priors / sampling
    if (have) {
#pragma unroll
      for (int k = 0; k < VPL; ++k) {
        const U cl = FT<T>::bits(r_prior(R, k));  // w domain: the prior as is
#pragma unroll
        for (int t = 0; t < DMAX; ++t) {
          if (no_edge<ENG, D3K>(k, t)) continue;  // (no dummy edge kept)
          if constexpr (eng_m2v(ENG)) {  // (m2v: 256-thread workgroups, host-enforced)
            // lanes past the last variable slot's S.vnl own no slots there (their lane-linear
            // addresses would run into the next edge's slots and past the V region)
            if (k == VPL - 1 && tidl >= S.vnl) continue;
            lds_st<U, true>(smem, m2v_va<T, DMAX, VPL, ENG, D3K, 256>(R, k, t), cl);
          }
          else
            lds_st<U, AB>(smem, r_va(R, k, t), cl);
          if (KV) R.ov[KV ? k : 0][KV ? t : 0] = cl;
        }
      }
      if (MC) {
        // sample this shot's Pauli error (src/Simulators.py:99-113); stage s = H e in F bit1
        const long long sl = c0 + sh;
        const unsigned long long gshot = A->shot_begin + (unsigned long long)sl;
        // the slot map first, in one batch: inside the loop its loads would queue behind the
        // err stores (u8, may alias) and wait out one memory latency per variable
        int jv[VPL];
#pragma unroll
        for (int k = 0; k < VPL; ++k) jv[k] = S.perm[k * TB + tidl];
        // the per-shot class cache (SMcArgs::cls_cache, both sectors with Philox draws): the first
        // sector's pass stores this thread's classes, the second reads them back (same thread, same
        // address: program order) instead of drawing again
        uint16_t* cc = nullptr;
        bool cc_read = false;
        uint32_t cw = 0;
        if (A->cls_cache && !A->uniforms && VPL <= 8) {
          cc = A->cls_cache + ((long long)blockIdx.x * A->chunk + sh) * TB + tidl;
          cc_read = q == A->sec_id1;
          if (cc_read) cw = *cc;
        }
#pragma unroll
        for (int k = 0; k < VPL; ++k) {
          const int j = jv[k];
          if (j >= 0) {
            uint32_t cls;
            if (A->uniforms) {
              const double u = A->uniforms[sl * (long long)n + j];
              cls = (u < A->t1) ? 2u : (A->t1 <= u && u < A->t2) ? 1u : (A->t2 <= u && u < A->t3) ? 3u : 0u;
            } else if (cc_read) {
              cls = (cw >> (2 * k)) & 3u;
            } else {
              const unsigned long long kk = philox_k53(A->seed, gshot, (uint32_t)j);
              cls = (kk < A->K1) ? 2u : (kk < A->K2) ? 1u : (kk < A->K3) ? 3u : 0u;
              cw |= cls << (2 * k);
            }
            const uint32_t e = (q == 0) ? (cls & 1u) : (cls >> 1);
            eb |= e << k;
            if (A->err && q == A->sec_id0) A->err[sl * (long long)n + j] = (uint8_t)cls;
            if (e) {
#pragma unroll
              for (int t = 0; t < DMAX; ++t) {
                if (no_edge<ENG, D3K>(k, t)) continue;
                if constexpr (eng_base(ENG) == 4)
                  atomicXor(&lds_at<uint32_t>(smem, f_addr<T, ENG>(R.ea[k][t], M)), 2u);
                else if constexpr (eng_c2s(ENG))
                  lds_xor_abs(R.ea[k][t], 2u);
                else
                  f_xor<ENG>(smem, r_fa(R, k, t, M.fbase), 2u);
              }
            }
          }
        }
        if (cc && !cc_read) *cc = (uint16_t)cw;
      } else {
        const uint8_t* srow = D->synd + (c0 + sh) * (long long)m;
        for (int i = tidl; i < m; i += TB) {  // i = check label (engine 3: S.rperm maps it to the check)
          const uint32_t fo = f_off<ENG>(Ly, i + 1);
          const uint32_t F = f_ld<ENG>(smem, fo);
          const int oi = S.rperm ? S.rperm[i] : i;
          f_st<ENG>(smem, fo, (eng_base(ENG) == 4 ? (F & 0xFFFF0000u) : (F & 4u)) | ((uint32_t)(srow[oi] & 1u) << 1));
        }
      }
    }
    if (QLDPC_STAMPS) {
      const unsigned long long t = qstamp();
      st_acc[4] += t - st_a;
      st_a = t;
    }
    M2vRows rwv;  // m2v: this thread's rows, loaded ahead of each check phase's barrier
    if constexpr (eng_m2v(ENG))
      if (have) m2v_rows_load(S, tid, TB, m, rwv);
    __syncthreads();
    // ---------------------------------------------------------- finish the previous decode
    if (pshot >= 0) {
      uint32_t lf = 0;
      if (MC) {
#pragma unroll
        for (int w = 0; w < 8; ++w) lf |= lred[w];
      }
      const int f = (!pconv || lf) ? 1 : 0;
      if (tid == 0) {
        const long long sl = c0 + pshot;
        if (MC) {
          if (f) failmap[pshot >> 5] |= 1u << (pshot & 31);
          cnt[kCntDec + q] += 1;
          cnt[kCntIters + q] += (unsigned long long)pit;
          cnt[kCntNonconv + q] += pconv ? 0 : 1;
          cnt[kCntSecFail + q] += (unsigned long long)f;
          atomicAdd(&A->counters[kCntHist + q * kHistBins + (pit < kHistBins ? pit : kHistBins - 1)], 1ull);
          if (A->iters) A->iters[sl * 2 + q] = pit;
        } else {
          if (D->iters) D->iters[sl] = pit;
          if (D->conv) D->conv[sl] = pconv ? 1 : 0;
        }
      }
    }
    if (!have) break;
    if (QLDPC_STAMPS) {
      const unsigned long long t = qstamp();
      st_acc[8] += t - st_a;
      st_a = t;
    }
    // ---------------------------------------------------------- first check pass (CS / c2v from priors)
    if constexpr (eng_base(ENG) == 4)
      c_check_any<T, true>(smem, Ly, m, nch, tid, TB, sb, adaptive ? (T)0.5 : alpha_fixed);
    else if constexpr (eng_c2s(ENG))
      c2s_check<T, true, NCH, eng_tail(ENG)>(smem, Ly, m, tid, TB, sb, adaptive ? (T)0.5 : alpha_fixed);
    else if constexpr (eng_m2v(ENG))
      m2v_check<T, true>(smem, Ly, m, tid, TB, sb, rwv, sbase + Ly.v);
    else if constexpr (eng_m2s(ENG))
      m_check<T, true, NCH, eng_tail(ENG)>(smem, Ly, m, wbase, tid, TB, sb);
    else if constexpr (NCH > 0)
      r_check_c<T, true, NCH, eng_tail(ENG), QLDPC_PFC, ENG>(smem, Ly, m, tid, TB, sb);
    else
      r_check<T, true>(smem, Ly, m, nch, tid, TB, sb, adaptive ? (T)0.5 : alpha_fixed);
    __syncthreads();
    if (tid < 10) lred[tid] = 0;  // lred read above (before the barrier); flags[0..1] start clear
    if (QLDPC_STAMPS) {
      const unsigned long long t = qstamp();
      st_acc[9] += t - st_a;
      st_acc[7] += 1;
      st_a = t;
    }
    // ---------------------------------------------------------- iterations
    int it = 1;
    bool conv = false;
    uint32_t xb = 0;
    uint64_t xm[VPL];  // (m2s families, QLDPC_M2S_XMASK: decisions as wave lane masks)
#pragma unroll
    for (int k = 0; k < VPL; ++k) xm[k] = 0;
    long long cslot = -1;  // BP+OSD capture slot of this decode (claimed at its last iteration)
    while (true) {
      int mism;
      double* cpost = nullptr;
      if constexpr (MC && eng_base(ENG) == 3) {
        if (A->c_n && A->c_post[q] && it >= S.max_iter) {  // uniform: the last iteration may end unconverged
          // (lred word 11: no static LDS in these kernels, so the dynamic image starts at address 0
          // and its offsets fold into the LDS instructions)
          uint32_t* s_cslot = lred + 11;
          if (tid == 0) *s_cslot = atomicAdd(&A->c_n[q], 1u);
          __syncthreads();
          cslot = (long long)*s_cslot;
          if (cslot < A->c_cap) cpost = A->c_post[q] + cslot * (long long)n;
        }
      }
      if constexpr (eng_base(ENG) == 4) {
        xb = c_var<T, DMAX, VPL>(smem, R, M, last_live);
        __syncthreads();
        // c2v for iteration it + 1 (wasted if this one converged)
        const T alpha = adaptive ? (T)(1.0 - ldexp(1.0, -(it + 1))) : alpha_fixed;
        mism = c_check_any<T, false>(smem, Ly, m, nch, tid, TB, sb, alpha);
      } else {
        const T alpha = adaptive ? (T)(1.0 - ldexp(1.0, -it)) : alpha_fixed;
        // (the 1024-thread tail family runs one workgroup per CU: nothing to take priority over)
        constexpr int kPV = (eng_tail(ENG) && !eng_m2x(ENG) && !eng_fb(ENG)) ? 0 : QLDPC_PRIO_V;
        if (kPV) __builtin_amdgcn_s_setprio(kPV);
        if constexpr (eng_m2x(ENG))
          xb = m_var<T, DMAX, VPL, D3K, ENG>(smem, R, fdelta, alpha, xb, xm, last_live, cpost, S.perm + tidl, TB, nwm);
        else
          xb = r_var<T, DMAX, VPL, D3K, ENG>(smem, R, fdelta, alpha, xb, last_live, cpost, S.perm + tidl, TB);
        if (kPV) __builtin_amdgcn_s_setprio(0);
        if constexpr (eng_m2v(ENG)) m2v_rows_load(S, tid, TB, m, rwv);
        unsigned long long t1 = 0;
        if (QLDPC_STAMPS) {
          t1 = qstamp();
          st_acc[0] += t1 - st_a;
        }
        __syncthreads();
        if (QLDPC_STAMPS) {
          st_a = qstamp();
          st_acc[1] += st_a - t1;
        }
        // check state for iteration it + 1 (float: pre-scaled by its alpha)
        const T alpha_next = adaptive ? (T)(1.0 - ldexp(1.0, -(it + 1))) : alpha_fixed;
        if (QLDPC_PRIO_C) __builtin_amdgcn_s_setprio(QLDPC_PRIO_C);
        if constexpr (eng_c2s(ENG))
          mism = c2s_check<T, false, NCH, eng_tail(ENG)>(smem, Ly, m, tid, TB, sb, alpha_next);
        else if constexpr (eng_m2v(ENG))
          mism = m2v_check<T, false>(smem, Ly, m, tid, TB, sb, rwv, sbase + Ly.v);
        else if constexpr (eng_m2s(ENG))
          mism = m_check<T, false, NCH, eng_tail(ENG)>(smem, Ly, m, wbase, tid, TB, sb);
        else if constexpr (NCH > 0)
          mism = r_check_c<T, false, NCH, eng_tail(ENG), QLDPC_PFC, ENG>(smem, Ly, m, tid, TB, sb);
        else
          mism = r_check<T, false>(smem, Ly, m, nch, tid, TB, sb, alpha_next);
        if (QLDPC_PRIO_C) __builtin_amdgcn_s_setprio(0);
        if (QLDPC_STAMPS) {
          const unsigned long long t = qstamp();
          st_acc[2] += t - st_a;
          st_a = t;
        }
      }
      if (__any(mism) && (tid & 63) == 0) flags[it & 1] = 1u;
      __syncthreads();
      if (QLDPC_STAMPS) {
        const unsigned long long t = qstamp();
        st_acc[3] += t - st_a;
        st_acc[6] += 1;
        st_a = t;
      }
      const int any = uni((int)flags[it & 1]);
      if (tid == 0) flags[(it & 1) ^ 1] = 0;  // read by everyone before this barrier
      conv = any == 0;
      if (conv || it >= S.max_iter) break;
      ++it;
    }
    if constexpr (eng_m2x(ENG) && eng_base(ENG) != 4 && m_xmask(ENG)) {
      xb = 0;
#pragma unroll
      for (int k = 0; k < VPL; ++k) xb |= (__builtin_amdgcn_inverse_ballot_w64(xm[k]) ? 1u : 0u) << k;
    }
    const long long sl = c0 + sh;
    if (MC && cslot >= 0 && cslot < A->c_cap) {
      // BP+OSD candidate: syndrome (original check order), sampled error, shot
      if (!conv) {
        uint8_t* cs = A->c_synd[q] + cslot * (long long)m;
        int qq = 0;
        for (int i = tidl; i < m; i += TB, ++qq)  // sb holds syndrome ^ row-degree parity (F bit 2)
          cs[S.rperm ? S.rperm[i] : i] =
              (uint8_t)(((sb >> qq) ^ (f_ld<ENG>(smem, f_off<ENG>(Ly, i + 1)) >> 2)) & 1u);
        uint8_t* ce = A->c_err[q] + cslot * (long long)n;
#pragma unroll
        for (int k = 0; k < VPL; ++k) {
          const int j = S.perm[k * TB + tidl];
          if (j >= 0) ce[j] = (uint8_t)((eb >> k) & 1u);
        }
      }
      if (tid == 0) A->c_shot[q][cslot] = conv ? -1 : sl;
    }
    if (MC) {
      // residual r = e ^ x and its logical syndrome L r (src/Simulators.py:135-160): the
      // wave's rows of L r are gathered in batches (slot map, then masks), xor-reduced
      // across the wave, and lane 0 folds them into lred (one LDS atomic per word and wave)
      const uint32_t r = eb ^ xb;
      if (__any(r != 0)) {
        int jv[VPL];
#pragma unroll
        for (int k = 0; k < VPL; ++k) jv[k] = ((r >> k) & 1u) ? S.perm[k * TB + tidl] : -1;
        const int kw = S.kw;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          if (w >= kw) break;  // uniform
          unsigned long long lm[VPL];
#pragma unroll
          for (int k = 0; k < VPL; ++k) lm[k] = jv[k] >= 0 ? S.lmask[(long long)jv[k] * kw + w] : 0ull;
          unsigned long long a = 0;
#pragma unroll
          for (int k = 0; k < VPL; ++k) a ^= lm[k];
          const uint32_t lo = wave_xor_u32((uint32_t)a), hi = wave_xor_u32((uint32_t)(a >> 32));
          if ((tid & 63) == 0) {
            if (lo) atomicXor(&lred[2 * w], lo);
            if (hi) atomicXor(&lred[2 * w + 1], hi);
          }
        }
      }
      if (A->corr) {
#pragma unroll
        for (int k = 0; k < VPL; ++k) {
          const int j = S.perm[k * TB + tidl];
          if (j >= 0) A->corr[(sl * 2 + q) * (long long)n + j] = (uint8_t)((xb >> k) & 1u);
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < VPL; ++k) {
        const int j = S.perm[k * TB + tidl];
        if (j >= 0) D->corr[sl * (long long)n + j] = (uint8_t)((xb >> k) & 1u);
      }
    }
    pshot = sh;
    pit = conv ? it : S.max_iter;
    pconv = conv ? 1 : 0;
    if (QLDPC_STAMPS) {
      const unsigned long long t = qstamp();
      st_acc[5] += t - st_a;
      st_a = t;
    }
  }
  if (QLDPC_STAMPS && (tid & 63) == 0) {
    unsigned long long* stp = MC ? A->stamps : D->stamps;
    if (stp) {
#pragma unroll
      for (int k = 0; k < 10; ++k) atomicAdd(&stp[k], st_acc[k]);
    }
  }
  __syncthreads();  // image reused by the next pass
}

template <typename T, int DMAX, int VPL, int ENG, int D3K, int LB = kMaxThreadsS, int NCH = 0>
__global__ __launch_bounds__(LB, (lb_waves<T, ENG>(LB))) void rmc_kernel(SMcArgs A) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, TB = blockDim.x;
  const int CH = A.chunk;
  const int fw = (CH + 31) / 32;
  const RLayout Ly = r_layout(eng_base(ENG), A.vslots, A.mmax, (int)sizeof(T), eng_tail(ENG), eng_m2s(ENG) ? 1 : eng_c2s(ENG) ? 2 : 0, eng_fb(ENG));
  uint32_t* fm0 = reinterpret_cast<uint32_t*>(smem + Ly.total);
  uint32_t* fm1 = fm0 + ((fw + 3) & ~3);
  unsigned long long* cnt = reinterpret_cast<unsigned long long*>(fm1 + ((fw + 3) & ~3));
  if (tid < kCntHist) cnt[tid] = 0;
  // chunk indices are 32-bit (host-checked) and c0 a 32x32-bit product: no 64-bit copy of the
  // chunk size stays live across the loops (it was spilled)
  const int nchunks = (int)((A.shot_count + CH - 1) / CH);
  // chunks come from a queue (A.work): a workgroup that drew short decodes takes more
  // chunks, so the launch does not wait on the unluckiest static share
  // the chunk queue's next index in lred word 10 (r_pass clears words 0-9 only; no static LDS)
  int* s_next = reinterpret_cast<int*>(smem + Ly.lred + 40);
  int ch = blockIdx.x;
  if (A.work) {
    if (tid == 0) *s_next = (int)atomicAdd(A.work, 1u);
    __syncthreads();
    ch = *s_next;
  }
  for (; ch < nchunks;) {
    const long long c0 = (long long)((unsigned long long)(unsigned)ch * (unsigned)CH);
    const unsigned long long rem = (unsigned long long)(A.shot_count - c0);  // > 0
    const int cn = (rem >> 31) ? CH : ((int)rem < CH ? (int)rem : CH);  // no 64-bit compare (VALU on gfx9)
    for (int i = tid; i < fw; i += TB) {
      fm0[i] = 0;
      fm1[i] = 0;
    }
    __syncthreads();
    for (int qi = 0; qi < A.nsec; ++qi) {
      const SSector S = pick_ssector(A, qi);
      const int q = qi == 0 ? A.sec_id0 : A.sec_id1;
      r_pass<T, DMAX, VPL, true, ENG, D3K, NCH>(S, q, c0, cn, smem, Ly, A.vslots, A.mmax, q == 0 ? fm0 : fm1, cnt, &A, nullptr,
                                 tid, TB);
    }
    // combine the sectors per shot (eval_logical_type, src/Simulators.py:162-168)
    unsigned long long nf = 0;
    for (int j = tid; j < cn; j += TB) {
      const uint32_t fx = (fm0[j >> 5] >> (j & 31)) & 1u, fz = (fm1[j >> 5] >> (j & 31)) & 1u;
      const uint32_t f = A.logical_mode == 0 ? fx : A.logical_mode == 1 ? fz : (fx | fz);
      nf += f;
      if (A.fail) A.fail[c0 + j] = (uint8_t)(fx | (fz << 1));
    }
    if (nf) atomicAdd(&cnt[kCntFail], nf);
    if (tid == 0) {
      cnt[kCntShots] += (unsigned long long)cn;
      if (A.work) *s_next = (int)atomicAdd(A.work, 1u);
    }
    __syncthreads();
    ch = A.work ? *s_next : ch + (int)gridDim.x;
  }
  __syncthreads();
  if (tid < kCntHist && cnt[tid]) atomicAdd(&A.counters[tid], cnt[tid]);
}

template <typename T, int DMAX, int VPL, int ENG, int D3K, int LB = kMaxThreadsS, int NCH = 0>
__global__ __launch_bounds__(LB, (lb_waves<T, ENG>(LB))) void rdec_kernel(SDecArgs D) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, TB = blockDim.x;
  const int CH = D.chunk;
  const RLayout Ly = r_layout(eng_base(ENG), D.vslots, D.mmax, (int)sizeof(T), eng_tail(ENG), eng_m2s(ENG) ? 1 : eng_c2s(ENG) ? 2 : 0, eng_fb(ENG));
  const long long nchunks = (D.B + CH - 1) / CH;
  // the chunk queue's next index in lred words 10-11 (r_pass clears words 0-9 only; no static LDS)
  long long* s_next = reinterpret_cast<long long*>(smem + Ly.lred + 40);
  long long ch = blockIdx.x;
  if (D.work) {
    if (tid == 0) *s_next = (long long)atomicAdd(D.work, 1u);
    __syncthreads();
    ch = *s_next;
  }
  while (ch < nchunks) {
    const long long c0 = ch * CH;
    const int cn = (int)(D.B - c0 < CH ? D.B - c0 : CH);
    r_pass<T, DMAX, VPL, false, ENG, D3K, NCH>(D.sec, 0, c0, cn, smem, Ly, D.vslots, D.mmax, nullptr, nullptr, nullptr, &D, tid,
                                TB);
    if (D.work) {  // r_pass ends with a barrier: every thread has read s_next
      if (tid == 0) *s_next = (long long)atomicAdd(D.work, 1u);
      __syncthreads();
      ch = *s_next;
    } else {
      ch += gridDim.x;
    }
  }
}

}  // namespace qldpc
