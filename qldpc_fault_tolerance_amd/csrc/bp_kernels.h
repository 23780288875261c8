// bp_kernels.h — CDNA4 (gfx950) kernels of the Monte Carlo BP decoding engine.
//
// One workgroup decodes one shot at a time and walks its shots persistently
// (grid = resident blocks).  Threads own variables (strided: j = k*TB + tid,
// k < VPL) for the variable-node update and checks (i = q*TB + tid) for the
// per-iteration check bookkeeping.
//
// Min-sum state is kept per CHECK in LDS, not per edge:
//   pair[i] = {m1, m2}  smallest / second smallest |v2c| over the check's
//                       edges (as order-preserving unsigned bits), m1's sign
//                       bit = syndrome ^ parity of (v2c <= 0) over the row;
//   flag[i]             bit0 parity accumulator, bit1 (H x)_i ^ s_i.
// This reproduces ldpc's forward/backward min-sum exactly (min over "all but
// me" = m2 if my |v2c| == m1 else m1; sign = parity ^ my sign), in any
// arithmetic order, so the flooding check update becomes three LDS atomics per
// edge (two unsigned mins + one xor) issued by the variable owners:
// old = min(m1, v); min(m2, max(old, v)) keeps the two smallest of the multiset.
// The variable update keeps ldpc's exact summation order
// (v2c_e = (((L + c_0) + c_1) ... + c_{e-1}) + ((0 + c_last) + ... + c_{e+1}),
// Λ = ((L + c_0) + ...) + c_{d-1}) in registers, so float64 results are
// bit-identical to the reference arithmetic (oracle/qldpc_oracle.c) and
// float32 results bit-identical to the oracle's float32 mode.
// Each thread keeps its edges' previous |v2c| and sign in registers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qldpc {

constexpr int kMaxThreads = 512;
constexpr uint32_t kNoEdge = 0xFFFFu;
constexpr uint32_t kStreamData = 0x51D50001u;

template <typename T> struct FT;
template <> struct FT<float> {
  using U = uint32_t;
  static constexpr U kSign = 0x80000000u;
  static constexpr U kSent = 0x7F7FFFFFu;  // FLT_MAX (ldpc's 1e308 is not a float)
  __device__ static inline U bits(float x) { return __float_as_uint(x); }
  __device__ static inline float val(U u) { return __uint_as_float(u); }
};
template <> struct FT<double> {
  using U = unsigned long long;
  static constexpr U kSign = 0x8000000000000000ull;
  static constexpr U kSent = 0x7FE1CCF385EBC8A0ull;  // 1e308, ldpc's min-sum sentinel
  __device__ static inline U bits(double x) { return (U)__double_as_longlong(x); }
  __device__ static inline double val(U u) { return __longlong_as_double((long long)u); }
};

__device__ inline float qabs(float x) { return fabsf(x); }
__device__ inline double qabs(double x) { return fabs(x); }

// Philox4x32-10 (Salmon et al., SC'11); identical to oracle_philox4x32_10.
__device__ inline void philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                     uint32_t k1, uint32_t& o0, uint32_t& o1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  o0 = c0; o1 = c1;
}

// 53-bit integer k of CPython's random(): u = k / 2^53.
__device__ inline unsigned long long philox_k53(unsigned long long seed, unsigned long long shot, uint32_t qubit) {
  uint32_t w0, w1;
  philox4x32_10(qubit, (uint32_t)shot, (uint32_t)(shot >> 32), kStreamData, (uint32_t)seed,
                (uint32_t)(seed >> 32), w0, w1);
  return ((unsigned long long)(w0 >> 5) << 26) | (unsigned long long)(w1 >> 6);
}

struct SectorDev {
  const uint32_t* vchk;            // [VPL][DMAX/2][TB] packed u16 check ids (0xFFFF = no edge)
  const void* llr;                 // T [VPL][TB] channel log-likelihood ratios
  const unsigned long long* lmask; // [n][kw] logical-row masks of each column (MC only)
  int m, n, kw, max_iter;
  double alpha;                    // 0 => 1 - 2^-iter
};

struct McArgs {
  SectorDev sec[2];
  int nsec;
  int sec_id[2];           // 0 = X errors (hz, lz), 1 = Z errors (hx, lx)
  int logical_mode;        // 0 X, 1 Z, 2 Total
  int mmax;
  unsigned long long K1, K2, K3;  // ceil(t * 2^53) thresholds of the 3-way split
  double t1, t2, t3;              // the same thresholds as doubles (external u)
  unsigned long long seed, shot_begin;
  long long shot_count;
  const double* uniforms;  // [S][n] or null
  unsigned long long* counters;  // qldpc_counters as u64 words
  uint8_t* fail;
  uint8_t* err;
  uint8_t* corr;
  int* iters;
};

struct DecArgs {
  SectorDev sec;
  const uint8_t* synd;
  uint8_t* corr;
  int* iters;
  uint8_t* conv;
  double* post;  // [B][n] final posterior log-probability ratios (BP+OSD input) or null
  long long B;
};

// counters layout (u64 words), mirrors qldpc_counters
constexpr int kCntShots = 0, kCntFail = 1, kCntDec = 2, kCntIters = 4, kCntNonconv = 6, kCntSecFail = 8,
              kCntHist = 10, kHistBins = 1025;

template <typename T>
struct alignas(2 * sizeof(typename FT<T>::U)) Pair {
  typename FT<T>::U a, b;
};

// ---------------------------------------------------------------------------
// Per-thread register image of the variables it owns in one sector.
template <typename T, int VPL, int DMAX>
struct VarRegs {
  using U = typename FT<T>::U;
  uint32_t cpk[VPL][DMAX / 2];  // packed check ids
  T L[VPL];
  U mag[VPL][DMAX];             // previous |v2c| bits
  unsigned long long sgn;       // previous (v2c <= 0), bit k*DMAX+t

  __device__ inline uint32_t chk(int k, int t) const {
    return (cpk[k][t >> 1] >> ((t & 1) * 16)) & 0xFFFFu;
  }

  __device__ inline void load(const SectorDev& S, int tid, int TB) {
    const T* llr = static_cast<const T*>(S.llr);
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
      L[k] = llr[k * TB + tid];
#pragma unroll
      for (int t2 = 0; t2 < DMAX / 2; ++t2) cpk[k][t2] = S.vchk[(k * (DMAX / 2) + t2) * TB + tid];
    }
  }
};

// Insert |v| into check i's (m1, m2) and xor the flag word.
template <typename T>
__device__ inline void check_insert(Pair<T>* P, uint32_t* F, uint32_t i, typename FT<T>::U v, uint32_t fx) {
  using U = typename FT<T>::U;
  const U old = atomicMin(&P[i].a, v);
  atomicMin(&P[i].b, old > v ? old : v);
  if (fx) atomicXor(&F[i], fx);
}

// ---------------------------------------------------------------------------
// Set up the first check state from v2c = L (iteration-1 check input) and the
// syndrome.  Entry: F0[i] = s_i*3 (decode) or 0 (MC, e_xor carries e_j*3).
template <typename T, int VPL, int DMAX>
__device__ inline void insert_priors(VarRegs<T, VPL, DMAX>& R, Pair<T>* P0, uint32_t* F0, uint32_t ebits, int tid,
                                     int TB, int n) {
  using U = typename FT<T>::U;
  R.sgn = 0;
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    const T Lk = R.L[k];
    const U mg = FT<T>::bits(qabs(Lk));
    const uint32_t neg = (Lk <= (T)0) ? 1u : 0u;
    const uint32_t e3 = ((ebits >> k) & 1u) * 3u;
#pragma unroll
    for (int t = 0; t < DMAX; ++t) {
      const uint32_t i = R.chk(k, t);
      R.mag[k][t] = mg;
      if (i != kNoEdge) {
        R.sgn |= (unsigned long long)neg << (k * DMAX + t);
        check_insert<T>(P0, F0, i, mg, e3 ^ neg);
      }
    }
  }
}

// One flooding iteration's variable-node half: read check state `Pc`, update
// v2c / posterior / decision, and insert into the next check state `Pn`/`Fn`.
template <typename T, int VPL, int DMAX>
__device__ inline uint32_t variable_phase(VarRegs<T, VPL, DMAX>& R, const Pair<T>* Pc, Pair<T>* Pn,
                                          uint32_t* Fn, T alpha, int tid, int TB, int n, T (&lam)[VPL]) {
  using U = typename FT<T>::U;
  uint32_t xbits = 0;
  unsigned long long nsgn = 0;
#pragma unroll
  for (int k = 0; k < VPL; ++k) {
    T c[DMAX];
#pragma unroll
    for (int t = 0; t < DMAX; ++t) {
      const uint32_t i = R.chk(k, t);
      c[t] = (T)0;
      if (i != kNoEdge) {
        const Pair<T> pr = Pc[i];
        const U m1 = pr.a & ~FT<T>::kSign;
        const bool par = (pr.a & FT<T>::kSign) != 0;
        const bool own = (R.sgn >> (k * DMAX + t)) & 1ull;
        const U sel = (R.mag[k][t] == m1) ? pr.b : m1;
        c[t] = FT<T>::val(sel) * ((par != own) ? -alpha : alpha);
      }
    }
    // forward partial sums (ldpc column pass, rows ascending)
    T f[DMAX];
    T acc = R.L[k];
#pragma unroll
    for (int t = 0; t < DMAX; ++t) {
      f[t] = acc;
      if (R.chk(k, t) != kNoEdge) acc = acc + c[t];
    }
    lam[k] = acc;
    const uint32_t x = (acc <= (T)0) ? 1u : 0u;
    if (k * TB + tid < n) xbits |= x << k;
    // backward sums and insertion into the next check state
    T b = (T)0;
#pragma unroll
    for (int t = DMAX - 1; t >= 0; --t) {
      const uint32_t i = R.chk(k, t);
      if (i != kNoEdge) {
        const T v = f[t] + b;
        b = b + c[t];
        const U mg = FT<T>::bits(qabs(v));
        const uint32_t neg = (v <= (T)0) ? 1u : 0u;
        R.mag[k][t] = mg;
        nsgn |= (unsigned long long)neg << (k * DMAX + t);
        check_insert<T>(Pn, Fn, i, mg, neg | (x << 1));
      }
    }
  }
  R.sgn = nsgn;
  return xbits;
}

// Full BP decode of one sector for the block.  Entry: F0 set as for
// insert_priors, P0/P1 = SENT, F1 arbitrary.  Returns decision bits of the
// thread's variables (and their last-iteration posteriors in `lam`);
// iters/conv set for all threads.
template <typename T, int VPL, int DMAX>
__device__ inline uint32_t bp_decode_block(VarRegs<T, VPL, DMAX>& R, const SectorDev& S, Pair<T>* P, uint32_t* F,
                                           int mmax, uint32_t ebits, int tid, int TB, int& iters, bool& conv,
                                           T (&lam)[VPL]) {
  using U = typename FT<T>::U;
  const int m = S.m, n = S.n;
  Pair<T>* P0 = P;
  Pair<T>* P1 = P + mmax;
  uint32_t* F0 = F;
  uint32_t* F1 = F + mmax;

  insert_priors<T, VPL, DMAX>(R, P0, F0, ebits, tid, TB, n);
  __syncthreads();
  uint32_t sbits = 0;
  {
    int q = 0;
    for (int i = tid; i < m; i += TB, ++q) {
      const uint32_t f = F0[i];
      const uint32_t sb = (f >> 1) & 1u;
      sbits |= sb << q;
      F1[i] = sb * 3u;
      if (f & 1u) P0[i].a |= FT<T>::kSign;
    }
  }
  __syncthreads();

  int cur = 0;
  uint32_t xbits = 0;
  conv = false;
  int it = 1;
  for (; it <= S.max_iter; ++it) {
    const T alpha = (S.alpha == 0.0) ? (T)(1.0 - ldexp(1.0, -it)) : (T)S.alpha;
    Pair<T>* Pc = cur ? P1 : P0;
    Pair<T>* Pn = cur ? P0 : P1;
    uint32_t* Fc = cur ? F1 : F0;
    uint32_t* Fn = cur ? F0 : F1;
    xbits = variable_phase<T, VPL, DMAX>(R, Pc, Pn, Fn, alpha, tid, TB, n, lam);
    __syncthreads();
    int mism = 0;
    int q = 0;
    for (int i = tid; i < m; i += TB, ++q) {
      const uint32_t f = Fn[i];
      mism |= (int)((f >> 1) & 1u);
      if (f & 1u) Pn[i].a |= FT<T>::kSign;
      Pc[i].a = FT<T>::kSent;
      Pc[i].b = FT<T>::kSent;
      Fc[i] = ((sbits >> q) & 1u) * 3u;
    }
    const int any = __syncthreads_or(mism);
    cur ^= 1;
    if (!any) {
      conv = true;
      break;
    }
  }
  iters = conv ? it : S.max_iter;
  return xbits;
}

// Reset both check-state buffers and F0 := f0 (per check i), for the block.
template <typename T>
__device__ inline void reset_checks(Pair<T>* P, uint32_t* F, int mmax, int m, int tid, int TB,
                                    const uint8_t* synd_row) {
  for (int i = tid; i < m; i += TB) {
    P[i].a = FT<T>::kSent;
    P[i].b = FT<T>::kSent;
    P[mmax + i].a = FT<T>::kSent;
    P[mmax + i].b = FT<T>::kSent;
    F[i] = synd_row ? (uint32_t)(synd_row[i] & 1u) * 3u : 0u;
  }
}

// ---------------------------------------------------------------------------
template <typename T, int VPL, int DMAX>
__global__ __launch_bounds__(kMaxThreads) void bp_decode_kernel(DecArgs A) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, TB = blockDim.x;
  const int m = A.sec.m, n = A.sec.n;
  Pair<T>* P = reinterpret_cast<Pair<T>*>(smem);
  uint32_t* F = reinterpret_cast<uint32_t*>(smem + sizeof(Pair<T>) * 2 * (size_t)m);
  VarRegs<T, VPL, DMAX> R;
  R.load(A.sec, tid, TB);
  for (long long b = blockIdx.x; b < A.B; b += gridDim.x) {
    reset_checks<T>(P, F, m, m, tid, TB, A.synd + b * (long long)m);
    __syncthreads();
    int iters;
    bool conv;
    T lam[VPL];
    const uint32_t x = bp_decode_block<T, VPL, DMAX>(R, A.sec, P, F, m, 0u, tid, TB, iters, conv, lam);
#pragma unroll
    for (int k = 0; k < VPL; ++k) {
      const int j = k * TB + tid;
      if (j < n) {
        A.corr[b * (long long)n + j] = (uint8_t)((x >> k) & 1u);
        if (A.post) A.post[b * (long long)n + j] = (double)lam[k];
      }
    }
    if (tid == 0) {
      if (A.iters) A.iters[b] = iters;
      if (A.conv) A.conv[b] = conv ? 1 : 0;
    }
  }
}

template <typename T, int VPL, int DMAX>
__global__ __launch_bounds__(kMaxThreads) void mc_kernel(McArgs A) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, TB = blockDim.x;
  const int mmax = A.mmax;
  Pair<T>* P = reinterpret_cast<Pair<T>*>(smem);
  uint32_t* F = reinterpret_cast<uint32_t*>(smem + sizeof(Pair<T>) * 2 * (size_t)mmax);
  uint32_t* lred = F + 2 * mmax;  // 8 words: logical syndrome of the residual

  // per-sector counters as named scalars (a runtime-indexed array would live in scratch)
  unsigned long long c_shots = 0, c_fail = 0, c_dec0 = 0, c_dec1 = 0, c_it0 = 0, c_it1 = 0, c_nc0 = 0,
                     c_nc1 = 0, c_sf0 = 0, c_sf1 = 0;
  VarRegs<T, VPL, DMAX> R;

  for (long long s = blockIdx.x; s < A.shot_count; s += gridDim.x) {
    const unsigned long long gshot = A.shot_begin + (unsigned long long)s;
    int secfail0 = 0, secfail1 = 0;
    for (int qi = 0; qi < A.nsec; ++qi) {
      const SectorDev& S = A.sec[qi];
      const int q = A.sec_id[qi];
      const int n = S.n;
      R.load(S, tid, TB);
      // --- sample the Pauli error of this shot (src/Simulators.py:99-113)
      uint32_t ebits = 0;
#pragma unroll
      for (int k = 0; k < VPL; ++k) {
        const int j = k * TB + tid;
        if (j < n) {
          uint32_t cls;
          if (A.uniforms) {
            const double u = A.uniforms[s * (long long)n + j];
            cls = (u < A.t1) ? 2u : (A.t1 <= u && u < A.t2) ? 1u : (A.t2 <= u && u < A.t3) ? 3u : 0u;
          } else {
            const unsigned long long kk = philox_k53(A.seed, gshot, (uint32_t)j);
            cls = (kk < A.K1) ? 2u : (kk < A.K2) ? 1u : (kk < A.K3) ? 3u : 0u;
          }
          const uint32_t e = (q == 0) ? (cls & 1u) : (cls >> 1);
          ebits |= e << k;
          if (A.err && qi == 0) A.err[s * (long long)n + j] = (uint8_t)cls;
        }
      }
      reset_checks<T>(P, F, mmax, S.m, tid, TB, nullptr);
      if (tid < 8) lred[tid] = 0;
      __syncthreads();
      int iters;
      bool conv;
      T lam[VPL];
      const uint32_t x = bp_decode_block<T, VPL, DMAX>(R, S, P, F, mmax, ebits, tid, TB, iters, conv, lam);
      // --- residual r = e ^ x and its logical syndrome L r (src/Simulators.py:135-160)
      const uint32_t r = ebits ^ x;
      if (r) {
        unsigned long long acc[4] = {0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < VPL; ++k) {
          if ((r >> k) & 1u) {
            const int j = k * TB + tid;
#pragma unroll
            for (int w = 0; w < 4; ++w)
              if (w < S.kw) acc[w] ^= S.lmask[(long long)j * S.kw + w];
          }
        }
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          if ((uint32_t)acc[w]) atomicXor(&lred[2 * w], (uint32_t)acc[w]);
          if ((uint32_t)(acc[w] >> 32)) atomicXor(&lred[2 * w + 1], (uint32_t)(acc[w] >> 32));
        }
      }
      if (A.corr) {
#pragma unroll
        for (int k = 0; k < VPL; ++k) {
          const int j = k * TB + tid;
          if (j < n) A.corr[(s * 2 + q) * (long long)n + j] = (uint8_t)((x >> k) & 1u);
        }
      }
      __syncthreads();
      uint32_t lf = 0;
#pragma unroll
      for (int w = 0; w < 8; ++w) lf |= lred[w];
      const int f = (!conv || lf) ? 1 : 0;
      if (q == 0) secfail0 = f; else secfail1 = f;
      if (tid == 0) {
        if (q == 0) {
          c_dec0 += 1; c_it0 += (unsigned long long)iters; c_nc0 += conv ? 0 : 1; c_sf0 += (unsigned long long)f;
        } else {
          c_dec1 += 1; c_it1 += (unsigned long long)iters; c_nc1 += conv ? 0 : 1; c_sf1 += (unsigned long long)f;
        }
        atomicAdd(&A.counters[kCntHist + q * kHistBins + (iters < kHistBins ? iters : kHistBins - 1)], 1ull);
        if (A.iters) A.iters[s * 2 + q] = iters;
      }
      __syncthreads();  // lred / check state reused by the next sector or shot
    }
    if (tid == 0) {
      const int f = A.logical_mode == 0 ? secfail0 : A.logical_mode == 1 ? secfail1 : (secfail0 | secfail1);
      c_shots += 1;
      c_fail += (unsigned long long)f;
      if (A.fail) A.fail[s] = (uint8_t)(secfail0 | (secfail1 << 1));
    }
  }
  if (tid == 0) {
    atomicAdd(&A.counters[kCntShots], c_shots);
    atomicAdd(&A.counters[kCntFail], c_fail);
    atomicAdd(&A.counters[kCntDec + 0], c_dec0);
    atomicAdd(&A.counters[kCntDec + 1], c_dec1);
    atomicAdd(&A.counters[kCntIters + 0], c_it0);
    atomicAdd(&A.counters[kCntIters + 1], c_it1);
    atomicAdd(&A.counters[kCntNonconv + 0], c_nc0);
    atomicAdd(&A.counters[kCntNonconv + 1], c_nc1);
    atomicAdd(&A.counters[kCntSecFail + 0], c_sf0);
    atomicAdd(&A.counters[kCntSecFail + 1], c_sf1);
  }
}

}  // namespace qldpc
