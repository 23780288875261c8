// bp_hbm.hip — engine 6: min-sum BP with HBM-resident messages, one decode per lane.
//
// For Tanner graphs whose per-decode LDS image exceeds the 160 KiB of a CU (the
// fp64 space-time graph of config 5: 1764 x 5439, E = 15,288, ~176 KB) and on
// request (QLDPC_ENGINE=6 / qldpc_bp_create_hbm) for any graph.  Each lane of a
// wave decodes its own syndrome; the 64 lanes of a wave walk the graph in
// lock step, so every graph index is wave-uniform (scalar loads of the edge
// tables) and every message access is one coalesced 512-byte (fp64) / 256-byte
// (fp32) segment of an [edge][lane] array in HBM:
//   V [E][64]   v2c, canonical bits (sign := v2c <= 0), row-major edge order
//   C [E][64]   c2v, column-major edge order (rows ascending per column)
//   X [n][64]   decisions (u8); syndromes are read straight from the [B][m] input
//               (graphs of n + m <= 2048: the decisions are instead one ballot word per variable
//               in the wave's LDS, xs [n] u64, and the syndromes one ballot word per check,
//               sw [m] u64, filled once per shot when a lane takes it: no decision traffic to
//               HBM, and no per-iteration re-read of scattered syndrome lines)
// One flooding iteration = a check sweep (rows: read V, min / second min /
// parity, write every edge's c2v = (-1)^sgn alpha min_{others}|v2c| into C at
// its column-major position; the H x == s test of the previous iteration's
// decisions rides along) and a variable sweep (columns: read C, ldpc's forward
// / backward sums in row order, write canonical v2c back into V, the decision
// into X).  Per edge and iteration that is one read and one write of each of V
// and C: 32 B (fp64) / 16 B (fp32) of HBM traffic, exactly SURVEY.md §8d's
// algorithmic bytes, plus 1 B of decision per edge.  No barrier, no LDS: waves
// are independent; a lane whose decode ends takes the next syndrome from a device
// queue at the next sweep boundary, so lanes of different iteration counts never
// wait for each other.  The next row's / column's messages are loaded while the
// current one is reduced (two rows or columns of loads in flight per lane).
//
// Arithmetic is ldpc 0.1.x's minimum_sum operation for operation (oracle
// bp_ms_*): the check phase's {min over the others, parity} is order
// independent, the variable phase keeps ldpc's summation order, both with
// -ffp-contract=off, so fp64 results are bit-identical to the oracle and fp32 to
// its float mode.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "bp_kernels.h"
#include "runtime.h"

namespace {

using namespace qldpc;

constexpr int kHRow = 12;  // max row degree (compile-time register block)
constexpr int kHCol = 12;  // max column degree
constexpr int kHThreads = 256;

struct HArgs {
  const int32_t* rp;     // [m+1] CSR row pointers (row-major edge ids)
  const int32_t* rcol;   // [m][kHRow] variable of each row edge
  const int32_t* rcpos;  // [m][kHRow] column-major position of each row edge
  const int32_t* cp;     // [n+1] CSC column pointers (column-major edge ids)
  const int32_t* crpos;  // [n][kHCol] row-major position of each column edge (rows ascending)
  const void* llr;       // T [n] log((1-p)/p)
  void* ws;              // per wave: V, C (T [E][64]) then X [n][64] (u8)
  unsigned long long ws_wave_bytes;
  const uint8_t* synd;   // [B][m]
  uint8_t* corr;         // [B][n]
  int32_t* iters;        // [B] or NULL
  uint8_t* conv;         // [B] or NULL
  unsigned int* work;    // chunk-queue head (zeroed per launch)
  long long B;
  int m, n, E, max_iter;
  double alpha;          // 0 => 1 - 2^-iter
};

template <typename T>
__device__ inline typename FT<T>::U hcanon(T v) {
  using U = typename FT<T>::U;
  const U b = FT<T>::bits(v);
  return b | ((b - (U)1) & ~b & FT<T>::kSign);  // sign bit := v <= 0 (only +0 changes)
}

// Row / column records of the uniform edge tables, prefetched one ahead of use.
template <typename T>
struct HRow {
  typename FT<T>::U v[kHRow];
  uint32_t x[kHRow];  // decision byte, or (LDS ballot words) the 32-lane half word holding it
  int e0, d;
};

// The edge tables come in as separate __restrict__ kernel arguments: never written by the
// kernel, so the backend may read them with scalar loads (uniform addresses) instead of one
// vector load per lane.
template <typename T, bool XL>
__global__ void __launch_bounds__(kHThreads, 2) hdec_kernel(HArgs A, const int32_t* __restrict__ rp,
                                                         const int32_t* __restrict__ rcol,
                                                         const int32_t* __restrict__ rcpos,
                                                         const int32_t* __restrict__ cp,
                                                         const int32_t* __restrict__ crpos,
                                                         const void* __restrict__ llr) {
  using U = typename FT<T>::U;
  constexpr U kS = FT<T>::kSign;
  const int lane = threadIdx.x & 63;
  const long long wave = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  unsigned char* wb = static_cast<unsigned char*>(A.ws) + (size_t)wave * A.ws_wave_bytes;
  U* __restrict__ V = reinterpret_cast<U*>(wb) + lane;
  U* __restrict__ C = reinterpret_cast<U*>(wb) + (size_t)A.E * 64 + lane;
  uint8_t* __restrict__ X = reinterpret_cast<uint8_t*>(reinterpret_cast<U*>(wb) + (size_t)2 * A.E * 64) + lane;
  // xlds: bit `lane` of xs[j] = this lane's decision on variable j (one u64 per variable and wave,
  // written by the variable sweep's ballot, read back as a broadcast LDS word)
  extern __shared__ unsigned long long hx_lds[];
  unsigned long long* xs = hx_lds + (size_t)(threadIdx.x >> 6) * (size_t)A.n;
  // per-lane 32-bit view: word 2j + (lane >> 5), bit lane & 31 (32-bit loads keep the prefetched
  // rows at one VGPR per edge)
  const uint32_t* xs32 = reinterpret_cast<const uint32_t*>(xs) + (lane >> 5);
  unsigned long long* sw = hx_lds + (size_t)(blockDim.x >> 6) * (size_t)A.n + (size_t)(threadIdx.x >> 6) * (size_t)A.m;
  const uint32_t* sw32 = reinterpret_cast<const uint32_t*>(sw) + (lane >> 5);
  const uint32_t xsh = XL ? (uint32_t)(lane & 31) : 0u;
  constexpr bool xl = XL;
  const T* __restrict__ L = static_cast<const T*>(llr);
  const int m = A.m, n = A.n;
  const bool adaptive = A.alpha == 0.0;
  // per-lane decode state: lanes refill from the shot queue as soon as their decode ends, so
  // a wave never idles behind its slowest lane (iteration counts differ per lane)
  long long shot = -1;   // this lane's syndrome, -1 = none
  int it = 0;            // iterations completed by this lane's decode
  bool idle = false;     // queue drained for this lane
  while (true) {
    // ---------------------------------------- refill lanes without a decode
    const bool need = shot < 0 && !idle;
    const unsigned long long nb = __ballot(need);
    if (nb) {
      const int cnt = __popcll(nb);
      int base = 0;
      if (lane == __ffsll((long long)nb) - 1) base = (int)atomicAdd(A.work, (unsigned)cnt);
      base = __builtin_amdgcn_readfirstlane(__shfl(base, __ffsll((long long)nb) - 1));
      if (need) {
        const long long s = (long long)base + __popcll(nb & ((1ull << lane) - 1ull));
        if (s < A.B) {
          shot = s;
          it = 0;
        } else {
          idle = true;
        }
      }
    }
    const bool active = shot >= 0;
    if (!__any(active)) break;
    if constexpr (XL) {
      // syndrome bits of the lanes that just took a shot into the wave's ballot words (once per
      // shot; 32 byte loads in flight per lane)
      const bool fresh = need && active;
      const unsigned long long fb = __ballot(fresh);
      if (fb) {
        const uint8_t* sr = A.synd + (fresh ? shot : 0) * (long long)m;
        for (int i0 = 0; i0 < m; i0 += 32) {
          uint32_t b[32];
#pragma unroll
          for (int u = 0; u < 32; ++u) b[u] = (fresh && i0 + u < m) ? (uint32_t)(sr[i0 + u] & 1u) : 0u;
#pragma unroll
          for (int u = 0; u < 32; ++u) {
            if (i0 + u < m) {
              const unsigned long long w = __ballot(b[u] != 0);
              if (lane == 0) sw[i0 + u] = (sw[i0 + u] & ~fb) | w;
            }
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      }
    }
    const uint8_t* srow = A.synd + (active ? shot : 0) * (long long)m;
    const bool first = it == 0;
    // ---------------------------------------- check sweep (+ the H x == s test of iteration it)
    const T alpha = adaptive ? (T)(1.0 - ldexp(1.0, -(it + 1))) : (T)A.alpha;
    uint32_t mism = 0;
    auto load_row = [&](int i, HRow<T>& r) {
      // the row record (uniform) is read in uniform control flow: scalar loads
      r.e0 = rp[i];
      r.d = rp[i + 1] - r.e0;
      const int32_t* rc = rcol + (size_t)i * kHRow;
      int jv[kHRow];
#pragma unroll
      for (int k = 0; k < kHRow; ++k) jv[k] = rc[k];  // padded records: index 0 beyond the degree
#pragma unroll
      for (int k = 0; k < kHRow; ++k) {
        if (k < r.d) {
          const T lj = L[jv[k]];
          if (active) {
            if (first) {
              r.v[k] = hcanon<T>(lj);  // ldpc's first check update reads the channel LLRs
              r.x[k] = 0;
            } else {
              r.v[k] = V[(size_t)(r.e0 + k) * 64];
              r.x[k] = xl ? xs32[2 * jv[k]] : (uint32_t)X[(size_t)jv[k] * 64];
            }
          }
        }
      }
    };
    // two rows of loads in flight ahead of the row being reduced
    HRow<T> cur, nx1;
    load_row(0, cur);
    if (1 < m) load_row(1, nx1);
    for (int i = 0; i < m; ++i) {
      HRow<T> nx2;
      if (i + 2 < m) load_row(i + 2, nx2);
      const int d = cur.d;
      const int32_t* rqp = rcpos + (size_t)i * kHRow;
      int rq[kHRow];
#pragma unroll
      for (int k = 0; k < kHRow; ++k) rq[k] = rqp[k];
      const uint32_t s = !active ? 0u : XL ? (sw32[2 * i] >> xsh) & 1u : (srow[i] & 1u);
      uint32_t hx = 0;
      U m1 = FT<T>::kSent, m2 = FT<T>::kSent, px = s ? kS : (U)0;
#pragma unroll
      for (int k = 0; k < kHRow; ++k) {
        if (k < d) {
          hx ^= cur.x[k];
          const U a = cur.v[k] & ~kS;
          const U hi = m1 > a ? m1 : a;
          m2 = m2 < hi ? m2 : hi;
          m1 = m1 < a ? m1 : a;
          px ^= cur.v[k];
        }
      }
      mism |= ((hx >> xsh) ^ s) & 1u;
      const U b1 = FT<T>::bits(FT<T>::val(m1) * alpha), b2 = FT<T>::bits(FT<T>::val(m2) * alpha);
#pragma unroll
      for (int k = 0; k < kHRow; ++k) {
        if (k < d && active) {
          // min over the others (m2 if this edge holds m1), sign = syndrome ^ parity of the others
          const U mag = (cur.v[k] & ~kS) == m1 ? b2 : b1;
          C[(size_t)rq[k] * 64] = mag ^ ((px ^ cur.v[k]) & kS);
        }
      }
      cur = nx1;
      nx1 = nx2;
    }
    // ---------------------------------------- end of this lane's decode?
    bool fin = false;
    int conv = 0;
    if (active && !first) {
      if (!mism) {
        fin = true;
        conv = 1;
      } else if (it >= A.max_iter) {
        fin = true;
      }
    }
    if (__any(fin)) {
      if (fin) {
        for (int j = 0; j < n; ++j)
          A.corr[shot * (long long)n + j] = xl ? (uint8_t)((xs32[2 * j] >> xsh) & 1u) : X[(size_t)j * 64];
        if (A.iters) A.iters[shot] = conv ? it : A.max_iter;
        if (A.conv) A.conv[shot] = (uint8_t)conv;
        shot = -1;
      }
    }
    const bool run = shot >= 0;  // lanes continuing into iteration it + 1
    if (!__any(run)) continue;
    // ---------------------------------------- variable sweep (ldpc's column order)
    // two columns of c2v loads in flight ahead of the column being summed
    T c1[kHCol], c2[kHCol];
    int d1 = cp[1] - cp[0], d2 = n > 1 ? cp[2] - cp[1] : 0;
#pragma unroll
    for (int t = 0; t < kHCol; ++t) {
      if (t < d1 && run) c1[t] = FT<T>::val(C[(size_t)(cp[0] + t) * 64]);
      if (t < d2 && run) c2[t] = FT<T>::val(C[(size_t)(cp[1] + t) * 64]);
    }
    for (int j = 0; j < n; ++j) {
      T c[kHCol];
      const int d = d1;
#pragma unroll
      for (int t = 0; t < kHCol; ++t) {
        c[t] = c1[t];
        c1[t] = c2[t];
      }
      d1 = d2;
      if (j + 2 < n) {  // the column after next: its c2v in flight under two columns of sums
        const int k0n = cp[j + 2];
        d2 = cp[j + 3] - k0n;
#pragma unroll
        for (int t = 0; t < kHCol; ++t)
          if (t < d2 && run) c2[t] = FT<T>::val(C[(size_t)(k0n + t) * 64]);
      }
      const int32_t* crp = crpos + (size_t)j * kHCol;
      int cr[kHCol];
#pragma unroll
      for (int t = 0; t < kHCol; ++t) cr[t] = crp[t];
      T f[kHCol];
      T acc = L[j];
#pragma unroll
      for (int t = 0; t < kHCol; ++t) {
        if (t < d) {
          f[t] = acc;
          acc = acc + c[t];
        }
      }
      if (xl) {
        const unsigned long long w = __ballot(run && acc <= (T)0);
        if (lane == 0) xs[j] = w;
      }
      if (run) {
        if (!xl) X[(size_t)j * 64] = acc <= (T)0 ? 1 : 0;
        // backward sums: v2c_t = f_t + ((c_last + ...) + c_{t+1}); the redundant `0 + c`
        // and `f + 0` of ldpc's loop change at most the sign of a zero (erased by hcanon)
        T b = (T)0;
#pragma unroll
        for (int t = kHCol - 1; t >= 0; --t) {
          if (t < d) {
            const T vv = (t == d - 1) ? f[t] : f[t] + b;
            b = (t == d - 1) ? c[t] : b + c[t];
            V[(size_t)cr[t] * 64] = hcanon<T>(vv);
          }
        }
      }
    }
    if (run) ++it;
    // the ballot words written by lane 0 are read by every lane of the wave in the next check
    // sweep: LDS operations of a wave complete in order; this keeps the compiler from moving
    // those reads above the writes
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
}

}  // namespace

namespace qldpc_rt {

// Host tables of engine 6 (fixed-stride row / column records, uniform loads).
int hbm_prepare(qldpc_bp* bp) {
  const qldpc_graph* g = bp->g;
  const int m = g->m, n = g->n, E = g->nnz;
  if (g->max_row > kHRow || g->max_col > kHCol)
    return set_err(QLDPC_ENOTSUP, "HBM engine: row or column degree above 12");
  std::vector<int32_t> rcol((size_t)std::max(1, m) * kHRow, 0), rcpos((size_t)std::max(1, m) * kHRow, 0);
  std::vector<int32_t> cp(n + 1, 0), crpos((size_t)n * kHCol, 0);
  // column-major numbering: columns ascending, rows ascending within a column (ldpc's order)
  std::vector<int32_t> cpos_of(std::max(1, E));
  for (int j = 0; j < n; ++j) cp[j + 1] = cp[j] + (int)g->col_rows[j].size();
  std::vector<int> fill(n, 0);
  for (int i = 0; i < m; ++i)
    for (int e = g->row_ptr[i]; e < g->row_ptr[i + 1]; ++e) {
      const int j = g->col_idx[e];
      const int t = fill[j]++;  // rows visited ascending: t-th row of column j
      cpos_of[e] = cp[j] + t;
      crpos[(size_t)j * kHCol + t] = e;
      rcol[(size_t)i * kHRow + (e - g->row_ptr[i])] = j;
      rcpos[(size_t)i * kHRow + (e - g->row_ptr[i])] = cp[j] + t;
    }
  int rc;
  if ((rc = bp->h_rp.alloc((size_t)(m + 1) * 4)) || (rc = bp->h_rcol.alloc(rcol.size() * 4)) ||
      (rc = bp->h_rcpos.alloc(rcpos.size() * 4)) || (rc = bp->h_cp.alloc(cp.size() * 4)) ||
      (rc = bp->h_crpos.alloc(std::max<size_t>(1, crpos.size()) * 4)) || (rc = bp->work.alloc(16)))
    return rc;
  if (hipMemcpy(bp->h_rp.p, g->row_ptr.data(), (size_t)(m + 1) * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(bp->h_rcol.p, rcol.data(), rcol.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(bp->h_rcpos.p, rcpos.data(), rcpos.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(bp->h_cp.p, cp.data(), cp.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
      (!crpos.empty() && hipMemcpy(bp->h_crpos.p, crpos.data(), crpos.size() * 4, hipMemcpyHostToDevice) != hipSuccess))
    return set_err(QLDPC_EHIP, "upload HBM-engine tables");
  bp->TB = kHThreads;
  bp->VPL = 1;
  bp->lds_bytes = 0;
  return 0;
}

// decisions and syndromes in LDS when 4 waves x (n + m) x 8 B leave room for 2 workgroups per CU
bool hbm_xlds(const qldpc_bp* bp) {
  const char* e = std::getenv("QLDPC_HBM_XLDS");
  return bp->g->n + bp->g->m <= 2048 && !(e && *e && std::atoi(e) == 0);
}

size_t hbm_wave_bytes(const qldpc_bp* bp) {
  const size_t tsize = bp->precision == 32 ? 4 : 8;
  const size_t b = (size_t)2 * bp->g->nnz * 64 * tsize + (hbm_xlds(bp) ? 0 : (size_t)bp->g->n * 64);
  return (b + 255) & ~(size_t)255;
}

const void* hbm_kernel(int precision) {
  return precision == 32 ? reinterpret_cast<const void*>(&hdec_kernel<float, false>)
                         : reinterpret_cast<const void*>(&hdec_kernel<double, false>);
}

int hbm_decode_launch(qldpc_bp* bp, const uint8_t* synd, uint8_t* corr, int32_t* iters, uint8_t* conv, int64_t B,
                      hipStream_t stream) {
  // resident waves: enough to keep HBM busy, bounded by the batch and by a
  // workspace budget (QLDPC_HBM_WS_GB, default 16 GiB of the 288 GB)
  const size_t wb = hbm_wave_bytes(bp);
  const char* e = std::getenv("QLDPC_HBM_WS_GB");
  const double gb = (e && *e) ? std::atof(e) : 16.0;
  const char* ew = std::getenv("QLDPC_HBM_WAVES");  // resident waves per CU (default 8)
  const long long wpc = (ew && *ew) ? std::max(1, std::atoi(ew)) : 8;
  long long waves = std::min<long long>((long long)bp->cus * wpc, (B + 63) / 64);
  waves = std::min<long long>(waves, std::max<long long>(1, (long long)(gb * (1ull << 30) / (double)wb)));
  const int wpb = kHThreads / 64;
  const long long blocks = (waves + wpb - 1) / wpb;
  const size_t need = (size_t)blocks * wpb * wb;
  if (bp->h_ws.bytes < need) {
    bp->h_ws.release();
    int rc = bp->h_ws.alloc(need);
    if (rc) return rc;
  }
  HArgs a;
  a.rp = static_cast<const int32_t*>(bp->h_rp.p);
  a.rcol = static_cast<const int32_t*>(bp->h_rcol.p);
  a.rcpos = static_cast<const int32_t*>(bp->h_rcpos.p);
  a.cp = static_cast<const int32_t*>(bp->h_cp.p);
  a.crpos = static_cast<const int32_t*>(bp->h_crpos.p);
  a.llr = bp->llr.p;
  a.ws = bp->h_ws.p;
  a.ws_wave_bytes = wb;
  a.synd = synd;
  a.corr = corr;
  a.iters = iters;
  a.conv = conv;
  a.work = static_cast<unsigned int*>(bp->work.p);
  a.B = B;
  a.m = bp->g->m;
  a.n = bp->g->n;
  a.E = bp->g->nnz;
  a.max_iter = bp->max_iter;
  a.alpha = bp->alpha;
  const bool xl = hbm_xlds(bp);
  const size_t shm = xl ? (size_t)wpb * (bp->g->n + bp->g->m) * 8 : 0;
  QLDPC_HIP(hipMemsetAsync(bp->work.p, 0, 4, stream));
  auto launch = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kHThreads), shm, stream, a, a.rp, a.rcol, a.rcpos, a.cp,
                       a.crpos, a.llr);
  };
  if (bp->precision == 32)
    xl ? launch(hdec_kernel<float, true>) : launch(hdec_kernel<float, false>);
  else
    xl ? launch(hdec_kernel<double, true>) : launch(hdec_kernel<double, false>);
  QLDPC_HIP(hipGetLastError());
  return 0;
}

}  // namespace qldpc_rt
