// bp_slot.h — CDNA4 (gfx950) BP engine: small workgroups, NS decodes in flight each.
//
// A workgroup of TB threads (default 256-320) owns NS "slots"; a slot holds one
// decode's LDS image
//   V [1+m·RW] v2c messages in row-major slot order (row = check, its edges in
//              ascending column order, 16-byte chunks XOR-swizzled so a wave's
//              row reads are bank-conflict free), padding = min-sum sentinel,
//              the first 16 bytes a write sink for missing edges;
//   CS[1+m]    compressed check state {m1 | parity<<sign, m2}, CS[0] = {0,0};
//   F [1+m]    bit0 = (H x)_i accumulator, bit1 = syndrome staging, F[0] sink;
//   lred[8]    logical syndrome of the finished residual; flags[2] block-OR.
// A thread owns variables j = k·TB + tid (k < VPL, a RUNTIME count) and checks
// i = q·TB + tid.  The variable phase streams each variable's edge words and
// prior from global memory (L1-resident: one sector's table is n·DMAX·4 bytes,
// prefetched one variable ahead), gathers CS and its own previous v2c from LDS,
// applies ldpc's arithmetic and scatters the new v2c; registers no longer grow
// with VPL, so several workgroups (independent barrier domains) share a CU and
// one's LDS phase overlaps another's VALU phase.
// All slots of a workgroup advance in lock-step phases separated by ONE barrier
// each, but every slot has its own shot and iteration counter: a converged (or
// max_iter) decode is finalised and its slot refilled at the next round.
// Messages are stored "canonical": magnitude bits with the sign bit replaced by
// ldpc's (v2c <= 0) predicate, so the check phase reads the parity from sign bits
// and the variable phase recovers its own previous v2c from its slot.
// Arithmetic is ldpc's, operation for operation (DESIGN.md §Kernels,
// oracle/qldpc_oracle.c), hence bit-exact.
#pragma once
#include "bp_kernels.h"

namespace qldpc {

constexpr int kMaxThreadsS = 1024;
constexpr int kMaxVplS = 32;  // variables per thread (bit masks are 32-bit)
// Edge word: (check + 1) in bits 0-15 | V slot in bits 16-31.  A missing edge
// (column degree < DMAX) is the word 0: it gathers CS[0] = {0, 0} (its c2v is
// ±0, which leaves every ldpc sum unchanged), writes its v2c into the V sink
// and xors into F[0].  No branch on edge validity remains in the hot loops.
constexpr uint32_t kNoEdgeS = 0u;
__device__ inline uint32_t echk(uint32_t e) { return e & 0xFFFFu; }
__device__ inline uint32_t eslot(uint32_t e) { return e >> 16; }

struct SSector {
  const uint32_t* edges;            // [VPL][DMAX][TB]
  const void* llr;                  // T [VPL][TB]
  const unsigned long long* lmask;  // [n][kw] logical-row masks per column (MC only)
  const uint8_t* rdeg;              // [m] row degrees by check label (engines 3, 4)
  const int32_t* perm;              // [VPL][TB] variable of each slot, -1 = padding (engines 3/4)
  const int32_t* rperm;             // [m] original check of each check label (engine 3), NULL = identity
  int m, n, kw, max_iter, nch, vpl; // nch = 16-byte chunks per row; vpl = variables per thread
  int d3k;                          // engine 3: slots k < d3k hold variables of degree <= 3 only
  double alpha;                     // 0 => 1 - 2^-iter
  // m2v (variable-major V slots): the check phase's row table [kM2vRows][4][TB] (two 16-bit slot
  // byte offsets from the V base per word), the last variable slot's first V slot and per-edge stride
  const uint32_t* rows;
  int vlast, vnl;
  int npos;                         // 1 + the last slot position holding a variable (= n unless the
                                    // slot map pads a degree class to whole variable slots)
  uint32_t nw;                      // narrow waves (the fp64 space-time m2s family): bit 16 k + w = wave w
                                    // computes variable slot k (< kNwSlots) one edge slot narrower
  uint32_t live_last;               // (the same family) bit w = wave w holds variables in the last slot
};

struct SMcArgs {
  SSector sec[2];
  int nsec, sec_id0, sec_id1, logical_mode;
  int mmax, vslots, img_bytes, chunk;
  unsigned long long K1, K2, K3;
  double t1, t2, t3;
  unsigned long long seed, shot_begin;
  long long shot_count;
  const double* uniforms;
  unsigned long long* counters;
  uint8_t* fail;
  uint8_t* err;
  uint8_t* corr;
  int* iters;
  unsigned int* work;  // engine 3: chunk queue head (zeroed per launch), NULL = static chunk striding
  // BP+OSD capture (engine 3, qldpc_mc_set_osd): every decode that reaches max_iter claims a slot
  // of its sector q and leaves its last-iteration posteriors, syndrome, sampled error and shot
  // index there; c_n == NULL disables it
  unsigned int* c_n;      // [2] slots claimed per sector (zeroed per launch)
  double* c_post[2];      // [cap][n]
  uint8_t* c_synd[2];     // [cap][m]
  uint8_t* c_err[2];      // [cap][n]
  long long* c_shot[2];   // [cap] launch-relative shot, -1 = converged at max_iter (no OSD)
  long long c_cap;
  unsigned long long* stamps;  // diagnostic builds (QLDPC_STAMPS): per-segment cycle sums, else NULL
  // both sectors: the first sector's pass leaves each shot's sampled 3-way classes (2 bits per variable
  // slot, [grid][chunk][TB]) for the second's, which then skips its Philox draws; NULL = both draw
  uint16_t* cls_cache;
};

struct SDecArgs {
  SSector sec;
  const uint8_t* synd;
  uint8_t* corr;
  int* iters;
  uint8_t* conv;
  long long B;
  int mmax, vslots, img_bytes, chunk;
  unsigned int* work;  // engine 3: chunk queue head (zeroed per launch), NULL = static chunk striding
  unsigned long long* stamps;  // diagnostic builds (QLDPC_STAMPS): per-segment cycle sums, else NULL
};

template <typename T> struct V16;
template <> struct V16<float> {
  using type = float4;
  static constexpr int N = 4;
  __device__ static inline float get(const float4& v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; }
  __device__ static inline float4 splat(float s) { return make_float4(s, s, s, s); }
};
template <> struct V16<double> {
  using type = double2;
  static constexpr int N = 2;
  __device__ static inline double get(const double2& v, int k) { return k == 0 ? v.x : v.y; }
  __device__ static inline double2 splat(double s) { return make_double2(s, s); }
};

__host__ __device__ inline size_t a16(size_t x) { return (x + 15) & ~(size_t)15; }

// Bytes of one slot image (host and device agree on this layout).  vslots
// counts the V sink (16 bytes) plus m rows; CS and F have m + 1 entries.
__host__ __device__ inline size_t slot_img_bytes(int vslots, int mmax, int tsize) {
  return a16((size_t)vslots * tsize) + a16((size_t)(mmax + 1) * 2 * tsize) + a16((size_t)(mmax + 1) * 4) + 48;
}
// Block LDS: NS images + 2 sector fail bitmaps of `chunk` shots + 10 u64 counters.
__host__ __device__ inline size_t slot_lds_bytes(int ns, int img, int chunk) {
  return (size_t)ns * img + 2 * a16((size_t)((chunk + 31) / 32) * 4) + 8 * 12;
}

template <typename T>
struct Img {
  T* V;
  Pair<T>* CS;
  uint32_t* F;
  uint32_t* lred;
  uint32_t* flags;
};

template <typename T>
__device__ inline Img<T> slot_img(unsigned char* smem, int q, int img_bytes, int vslots, int mmax) {
  unsigned char* b = smem + (size_t)q * img_bytes;
  Img<T> I;
  I.V = reinterpret_cast<T*>(b);
  size_t off = a16((size_t)vslots * sizeof(T));
  I.CS = reinterpret_cast<Pair<T>*>(b + off);
  off += a16((size_t)(mmax + 1) * 2 * sizeof(T));
  I.F = reinterpret_cast<uint32_t*>(b + off);
  off += a16((size_t)(mmax + 1) * 4);
  I.lred = reinterpret_cast<uint32_t*>(b + off);
  I.flags = I.lred + 8;
  return I;
}

// canonical message bits: |v| with sign bit := (v <= 0)  (ldpc's sign test)
template <typename T>
__device__ inline typename FT<T>::U canon(T v) {
  using U = typename FT<T>::U;
  return (FT<T>::bits(v) & ~FT<T>::kSign) | ((v <= (T)0) ? FT<T>::kSign : (U)0);
}

template <int DMAX>
__device__ inline void load_edges(const SSector& S, int k, int tid, int TB, uint32_t (&e)[DMAX]) {
#pragma unroll
  for (int t = 0; t < DMAX; ++t) e[t] = S.edges[(k * DMAX + t) * TB + tid];
}

// v2c = prior on every edge (ldpc's first check update reads the channel LLRs).
template <typename T, int DMAX>
__device__ inline void s_priors(const SSector& S, T* V, int tid, int TB) {
  const T* llr = static_cast<const T*>(S.llr);
  for (int k = 0; k < S.vpl; ++k) {
    uint32_t e[DMAX];
    load_edges<DMAX>(S, k, tid, TB, e);
    const T c = FT<T>::val(canon<T>(llr[k * TB + tid]));
#pragma unroll
    for (int t = 0; t < DMAX; ++t) V[eslot(e[t])] = c;
  }
}

// Variable phase of one flooding iteration for one slot.  Returns decision bits.
template <typename T, int DMAX>
__device__ inline uint32_t s_var(const SSector& S, const Img<T>& I, T alpha, int tid, int TB) {
  using U = typename FT<T>::U;
  constexpr U kS = FT<T>::kSign;
  const T* llr = static_cast<const T*>(S.llr);
  const int n = S.n, vpl = S.vpl;
  uint32_t xbits = 0;
  uint32_t en[DMAX];
  load_edges<DMAX>(S, 0, tid, TB, en);
  T Ln = llr[tid];
  for (int k = 0; k < vpl; ++k) {
    uint32_t e[DMAX];
#pragma unroll
    for (int t = 0; t < DMAX; ++t) e[t] = en[t];
    const T L = Ln;
    if (k + 1 < vpl) {  // next variable's edge words / prior stream in under this one's work
      load_edges<DMAX>(S, k + 1, tid, TB, en);
      Ln = llr[(k + 1) * TB + tid];
    }
    Pair<T> pr[DMAX];
    U ov[DMAX];
#pragma unroll
    for (int t = 0; t < DMAX; ++t) {
      pr[t] = I.CS[echk(e[t])];
      ov[t] = FT<T>::bits(I.V[eslot(e[t])]);
    }
    T c[DMAX];
#pragma unroll
    for (int t = 0; t < DMAX; ++t) {
      const U a = pr[t].a;
      const U m1 = a & ~kS;
      // min over the OTHER edges of the check: m2 if this edge holds m1, else m1
      const U sel = ((ov[t] & ~kS) == m1) ? pr[t].b : m1;
      // c2v = sel * (±alpha): x*(-a) == -(x*a) exactly, so flip the product's sign bit
      c[t] = FT<T>::val(FT<T>::bits(FT<T>::val(sel) * alpha) ^ ((a ^ ov[t]) & kS));
    }
    // ldpc column pass (rows ascending): forward partial sums from the prior
    T f[DMAX];
    T acc = L;
#pragma unroll
    for (int t = 0; t < DMAX; ++t) {
      f[t] = acc;
      acc = acc + c[t];
    }
    const uint32_t x = (acc <= (T)0 && k * TB + tid < n) ? 1u : 0u;
    xbits |= x << k;
    T b = (T)0;
#pragma unroll
    for (int t = DMAX - 1; t >= 0; --t) {
      const T v = f[t] + b;
      b = b + c[t];
      I.V[eslot(e[t])] = FT<T>::val(canon<T>(v));
      if (x) atomicXor(&I.F[echk(e[t])], 1u);
    }
  }
  return xbits;
}

// Check phase for one slot.  FIRST: syndrome bits from F bit1 into sbits; else
// test (H x)_i == s_i from F bit0.  Always clears F and rebuilds CS from V.
template <typename T, bool FIRST>
__device__ inline int s_check(const Img<T>& I, int m, int nch, int tid, int TB, uint32_t& sbits) {
  using U = typename FT<T>::U;
  using VT = typename V16<T>::type;
  constexpr int NV = V16<T>::N;
  constexpr U kS = FT<T>::kSign;
  int mism = 0;
  int q = 0;
  for (int i = tid; i < m; i += TB, ++q) {
    const VT* row = reinterpret_cast<const VT*>(I.V + NV + (size_t)i * nch * NV);
    const uint32_t f = I.F[i + 1];
    uint32_t s;
    if (FIRST) {
      s = (f >> 1) & 1u;
      sbits |= s << q;
    } else {
      s = (sbits >> q) & 1u;
      mism |= (int)((f ^ s) & 1u);
    }
    I.F[i + 1] = 0;
    U m1 = FT<T>::kSent, m2 = FT<T>::kSent;
    U px = s ? kS : (U)0;
    for (int c = 0; c < nch; ++c) {
      const VT v = row[c];
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const U xb = FT<T>::bits(V16<T>::get(v, k));
        const U a = xb & ~kS;
        const U hi = m1 > a ? m1 : a;
        m2 = m2 < hi ? m2 : hi;
        m1 = m1 < a ? m1 : a;
        px ^= xb;  // canonical sign bit = (v2c <= 0)
      }
    }
    Pair<T> st;
    st.a = m1 | (px & kS);
    st.b = m2;
    I.CS[i + 1] = st;
  }
  return mism;
}

template <typename T>
__device__ inline void s_fill(const Img<T>& I, int vslots, int mmax, int tid, int TB) {
  using VT = typename V16<T>::type;
  VT* V4 = reinterpret_cast<VT*>(I.V);
  const VT s = V16<T>::splat(FT<T>::val(FT<T>::kSent));
  for (int i = tid; i < vslots / V16<T>::N; i += TB) V4[i] = s;
  for (int i = tid; i <= mmax; i += TB) I.F[i] = 0;
  if (tid < 10) I.lred[tid] = 0;  // lred[0..7], flags[0..1]
  if (tid == 0) {
    Pair<T> z;
    z.a = 0;
    z.b = 0;
    I.CS[0] = z;  // missing-edge dummy: c2v = ±0
  }
}

__device__ inline int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }

// ---------------------------------------------------------------------------
// One sector pass over `cn` shots (chunk-relative 0..cn-1) with NS slots.
// MC: shots are sampled (Philox / external u) and checked against the logicals;
// DEC: syndromes come from D->synd and corrections/iters/conv are written.
template <typename T, int DMAX, int NS, bool MC>
__device__ void s_pass(const SSector& S, int q, long long c0, int cn, unsigned char* smem, int img_bytes, int vslots,
                       int mmax, uint32_t* failmap, unsigned long long* cnt, const SMcArgs* A, const SDecArgs* D,
                       int tid, int TB) {
  const int m = S.m, n = S.n, nch = S.nch, vpl = S.vpl;
  for (int s = 0; s < NS; ++s) s_fill<T>(slot_img<T>(smem, s, img_bytes, vslots, mmax), vslots, mmax, tid, TB);
  __syncthreads();

  uint32_t xb[NS], eb[NS], sb[NS];
  int shot[NS], it[NS], pshot[NS], pit[NS], pconv[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    shot[s] = -1;
    pshot[s] = -1;
    it[s] = 0;
    pit[s] = 0;
    pconv[s] = 0;
    xb[s] = eb[s] = sb[s] = 0;
  }
  const bool adaptive = S.alpha == 0.0;
  const T alpha_fixed = (T)S.alpha;
  int next = 0;
  while (true) {
    bool live = false;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (shot[s] < 0 && next < cn) {
        shot[s] = next++;
        it[s] = 0;
      }
      live |= shot[s] >= 0 || pshot[s] >= 0;
    }
    if (!live) break;
    // ------------------------------------------------------------ phase V
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (shot[s] < 0) continue;
      const Img<T> I = slot_img<T>(smem, s, img_bytes, vslots, mmax);
      if (it[s] == 0) {
        s_priors<T, DMAX>(S, I.V, tid, TB);
        sb[s] = 0;
        if (MC) {
          // sample this shot's Pauli error (src/Simulators.py:99-113); stage s = H e in F bit1
          const long long sl = c0 + shot[s];
          const unsigned long long gshot = A->shot_begin + (unsigned long long)sl;
          uint32_t ebits = 0;
          for (int k = 0; k < vpl; ++k) {
            const int j = k * TB + tid;
            if (j < n) {
              uint32_t cls;
              if (A->uniforms) {
                const double u = A->uniforms[sl * (long long)n + j];
                cls = (u < A->t1) ? 2u : (A->t1 <= u && u < A->t2) ? 1u : (A->t2 <= u && u < A->t3) ? 3u : 0u;
              } else {
                const unsigned long long kk = philox_k53(A->seed, gshot, (uint32_t)j);
                cls = (kk < A->K1) ? 2u : (kk < A->K2) ? 1u : (kk < A->K3) ? 3u : 0u;
              }
              const uint32_t e = (q == 0) ? (cls & 1u) : (cls >> 1);
              ebits |= e << k;
              if (A->err && q == A->sec_id0) A->err[sl * (long long)n + j] = (uint8_t)cls;
              if (e) {
                uint32_t ed[DMAX];
                load_edges<DMAX>(S, k, tid, TB, ed);
#pragma unroll
                for (int t = 0; t < DMAX; ++t) atomicXor(&I.F[echk(ed[t])], 2u);
              }
            }
          }
          eb[s] = ebits;
        } else {
          const uint8_t* srow = D->synd + (c0 + shot[s]) * (long long)m;
          for (int i = tid; i < m; i += TB) I.F[i + 1] = (uint32_t)(srow[i] & 1u) << 1;
        }
      } else {
        const T alpha = adaptive ? (T)(1.0 - ldexp(1.0, -it[s])) : alpha_fixed;
        xb[s] = s_var<T, DMAX>(S, I, alpha, tid, TB);
      }
    }
    __syncthreads();
    // ------------------------------------------------------------ phase C
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const Img<T> I = slot_img<T>(smem, s, img_bytes, vslots, mmax);
      if (pshot[s] >= 0) {
        // finish the slot's previous decode (its logical xors preceded the barrier)
        uint32_t lf = 0;
        if (MC) {
#pragma unroll
          for (int w = 0; w < 8; ++w) lf |= I.lred[w];
        }
        const int f = (!pconv[s] || lf) ? 1 : 0;
        if (tid == 0) {
          const long long sl = c0 + pshot[s];
          if (MC) {
            if (f) failmap[pshot[s] >> 5] |= 1u << (pshot[s] & 31);
            cnt[kCntDec + q] += 1;
            cnt[kCntIters + q] += (unsigned long long)pit[s];
            cnt[kCntNonconv + q] += pconv[s] ? 0 : 1;
            cnt[kCntSecFail + q] += (unsigned long long)f;
            atomicAdd(&A->counters[kCntHist + q * kHistBins + (pit[s] < kHistBins ? pit[s] : kHistBins - 1)], 1ull);
            if (A->iters) A->iters[sl * 2 + q] = pit[s];
          } else {
            if (D->iters) D->iters[sl] = pit[s];
            if (D->conv) D->conv[sl] = pconv[s] ? 1 : 0;
          }
        }
      }
      if (shot[s] < 0) continue;
      if (it[s] == 0) {
        s_check<T, true>(I, m, nch, tid, TB, sb[s]);
      } else {
        const int mism = s_check<T, false>(I, m, nch, tid, TB, sb[s]);
        if (__any(mism) && (tid & 63) == 0) I.flags[it[s] & 1] = 1u;
      }
    }
    __syncthreads();
    // ------------------------------------------------------------ post
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const Img<T> I = slot_img<T>(smem, s, img_bytes, vslots, mmax);
      if (pshot[s] >= 0) {
        if (MC && tid < 8) I.lred[tid] = 0;  // every thread read it in phase C
        pshot[s] = -1;
      }
      if (shot[s] < 0) continue;
      if (it[s] == 0) {
        if (tid == 0) {
          I.flags[0] = 0;
          I.flags[1] = 0;
        }
        it[s] = 1;
        continue;
      }
      const int any = uni((int)I.flags[it[s] & 1]);
      if (tid == 0) I.flags[(it[s] & 1) ^ 1] = 0;  // next iteration's word (read before this barrier)
      const bool conv = any == 0;
      if (conv || it[s] >= S.max_iter) {
        const long long sl = c0 + shot[s];
        if (MC) {
          // residual r = e ^ x and its logical syndrome L r (src/Simulators.py:135-160)
          const uint32_t r = eb[s] ^ xb[s];
          if (r) {
            unsigned long long acc[4] = {0, 0, 0, 0};
            for (int k = 0; k < vpl; ++k) {
              if ((r >> k) & 1u) {
                const int j = k * TB + tid;
#pragma unroll
                for (int w = 0; w < 4; ++w)
                  if (w < S.kw) acc[w] ^= S.lmask[(long long)j * S.kw + w];
              }
            }
#pragma unroll
            for (int w = 0; w < 4; ++w) {
              if ((uint32_t)acc[w]) atomicXor(&I.lred[2 * w], (uint32_t)acc[w]);
              if ((uint32_t)(acc[w] >> 32)) atomicXor(&I.lred[2 * w + 1], (uint32_t)(acc[w] >> 32));
            }
          }
          if (A->corr) {
            for (int k = 0; k < vpl; ++k) {
              const int j = k * TB + tid;
              if (j < n) A->corr[(sl * 2 + q) * (long long)n + j] = (uint8_t)((xb[s] >> k) & 1u);
            }
          }
        } else {
          for (int k = 0; k < vpl; ++k) {
            const int j = k * TB + tid;
            if (j < n) D->corr[sl * (long long)n + j] = (uint8_t)((xb[s] >> k) & 1u);
          }
        }
        pshot[s] = shot[s];
        pit[s] = conv ? it[s] : S.max_iter;
        pconv[s] = conv ? 1 : 0;
        shot[s] = -1;
      } else {
        it[s] += 1;
      }
    }
  }
  __syncthreads();  // images reused by the next pass
}

__device__ inline SSector pick_ssector(const SMcArgs& A, int qi) {
  SSector S;
  const bool b = qi != 0;
  S.edges = b ? A.sec[1].edges : A.sec[0].edges;
  S.llr = b ? A.sec[1].llr : A.sec[0].llr;
  S.lmask = b ? A.sec[1].lmask : A.sec[0].lmask;
  S.rdeg = b ? A.sec[1].rdeg : A.sec[0].rdeg;
  S.perm = b ? A.sec[1].perm : A.sec[0].perm;
  S.rperm = b ? A.sec[1].rperm : A.sec[0].rperm;
  S.d3k = b ? A.sec[1].d3k : A.sec[0].d3k;
  S.m = b ? A.sec[1].m : A.sec[0].m;
  S.n = b ? A.sec[1].n : A.sec[0].n;
  S.kw = b ? A.sec[1].kw : A.sec[0].kw;
  S.max_iter = b ? A.sec[1].max_iter : A.sec[0].max_iter;
  S.nch = b ? A.sec[1].nch : A.sec[0].nch;
  S.vpl = b ? A.sec[1].vpl : A.sec[0].vpl;
  S.alpha = b ? A.sec[1].alpha : A.sec[0].alpha;
  S.rows = b ? A.sec[1].rows : A.sec[0].rows;
  S.vlast = b ? A.sec[1].vlast : A.sec[0].vlast;
  S.vnl = b ? A.sec[1].vnl : A.sec[0].vnl;
  S.npos = b ? A.sec[1].npos : A.sec[0].npos;
  return S;
}

template <typename T, int DMAX, int NS>
__global__ __launch_bounds__(kMaxThreadsS) void smc_kernel(SMcArgs A) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, TB = blockDim.x;
  const int CH = A.chunk;
  const int fw = (CH + 31) / 32;
  uint32_t* fm0 = reinterpret_cast<uint32_t*>(smem + (size_t)NS * A.img_bytes);
  uint32_t* fm1 = fm0 + ((fw + 3) & ~3);
  unsigned long long* cnt = reinterpret_cast<unsigned long long*>(fm1 + ((fw + 3) & ~3));
  if (tid < kCntHist) cnt[tid] = 0;
  const long long nchunks = (A.shot_count + CH - 1) / CH;
  for (long long ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    const long long c0 = ch * CH;
    const int cn = (int)(A.shot_count - c0 < CH ? A.shot_count - c0 : CH);
    for (int i = tid; i < fw; i += TB) {
      fm0[i] = 0;
      fm1[i] = 0;
    }
    __syncthreads();
    for (int qi = 0; qi < A.nsec; ++qi) {
      const SSector S = pick_ssector(A, qi);
      const int q = qi == 0 ? A.sec_id0 : A.sec_id1;
      s_pass<T, DMAX, NS, true>(S, q, c0, cn, smem, A.img_bytes, A.vslots, A.mmax, q == 0 ? fm0 : fm1, cnt, &A,
                                nullptr, tid, TB);
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
    if (tid == 0) cnt[kCntShots] += (unsigned long long)cn;
    __syncthreads();
  }
  __syncthreads();
  if (tid < kCntHist && cnt[tid]) atomicAdd(&A.counters[tid], cnt[tid]);
}

template <typename T, int DMAX, int NS>
__global__ __launch_bounds__(kMaxThreadsS) void sdec_kernel(SDecArgs D) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, TB = blockDim.x;
  const int CH = D.chunk;
  const long long nchunks = (D.B + CH - 1) / CH;
  for (long long ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    const long long c0 = ch * CH;
    const int cn = (int)(D.B - c0 < CH ? D.B - c0 : CH);
    s_pass<T, DMAX, NS, false>(D.sec, 0, c0, cn, smem, D.img_bytes, D.vslots, D.mmax, nullptr, nullptr, nullptr, &D,
                               tid, TB);
  }
}

}  // namespace qldpc
