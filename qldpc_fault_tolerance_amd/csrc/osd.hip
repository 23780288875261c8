// osd.hip — ordered-statistics post-processing (BP+OSD) of non-converged BP
// decodes: the `bposd_decoder(..., osd_method, osd_order)` the reference's
// BPOSD_Decoder wraps (src/Decoders.py:26-41; osd_method="osd_e", osd_order=10
// in every notebook).  Host code: the GPU BP decode (engine 1,
// qldpc_bp_decode_batch_soft) hands over the final posteriors, and this stage
// runs GF(2) elimination per non-converged syndrome on host threads.
//
// Algorithm (ldpc 0.1 OSD, restated; oracle/oracle.py osd_decode follows the
// same spec literally with an LU solve per candidate):
//   1. columns sorted by posterior log-probability ratio, ascending (stable);
//   2. LU-style elimination choosing, for pivot i = 0..rank-1, the first column
//      in the current order independent of the earlier pivots and SWAPPING it
//      into position i (Neal's mod2sparse_decomp with the "first" strategy) — the
//      non-pivot columns Ht = cols[rank:] inherit that swap order;
//   3. OSD-0: x_S = H_S^-1 s on the pivots, 0 elsewhere;
//   4. OSD-E: every t in {0,1}^w on Ht[0:w] (w = min(order, n-rank)), natural
//      binary order; OSD-CS: weight-1 t over all of Ht, then weight-2 t inside
//      Ht[0:w]; candidate x_S = H_S^-1 (s + H_T t); keep the first candidate of
//      strictly smaller soft weight sum_{j: x_j=1} log(1/p_j) (ascending j).
// Linear algebra: pivot columns are found by xor-basis insertion on m-bit
// column vectors, each basis vector carrying its combination of pivots, so
// H_S^-1 g is one basis reduction; candidates use linearity,
// x(s + sum t_j h_j) = x(s) + sum t_j x(h_j), i.e. one rank-bit xor each.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <numeric>
#include <thread>
#include <type_traits>
#include <utility>
#include <vector>

#include "runtime.h"

// measured-and-not-kept elimination variants (panel modes PNL 1-5, two rows per thread, the column
// window, two syndromes per workgroup): out of the product build unless -DQLDPC_EXPERIMENTAL=1
#ifndef QLDPC_EXPERIMENTAL
#define QLDPC_EXPERIMENTAL 0
#endif


using qldpc_rt::set_err;

struct qldpc_osd {
  int m = 0, n = 0, method = 1, order = 0, rank = 0;
  std::vector<std::vector<int32_t>> col_rows;
  std::vector<double> w;  // log(1/p_j)
  bool uniform = true;
};

namespace {

using u64 = unsigned long long;

inline int ctz64(u64 x) { return __builtin_ctzll(x); }

// Column vectors over rows, xor basis keyed by the lowest set row bit.
struct Basis {
  int W = 0, RW = 0;
  std::vector<int32_t> key;  // row bit -> basis slot or -1
  std::vector<u64> vec;      // [slot][W]
  std::vector<u64> comb;     // [slot][RW] pivots combined into the slot
  int count = 0;

  void init(int m, int rank) {
    W = (m + 63) / 64;
    RW = std::max(1, (rank + 63) / 64);
    key.assign(m, -1);
    vec.assign((size_t)std::max(rank, 1) * W, 0);
    comb.assign((size_t)std::max(rank, 1) * RW, 0);
    count = 0;
  }
  // Reduce v (W words) in place, accumulating the used combination into c (RW words).
  // Returns the lowest set bit left, or -1 if v reduced to zero.
  int reduce(u64* v, u64* c) const {
    for (;;) {
      int b = -1;
      for (int q = 0; q < W; ++q)
        if (v[q]) {
          b = q * 64 + ctz64(v[q]);
          break;
        }
      if (b < 0) return -1;
      const int s = key[b];
      if (s < 0) return b;
      const u64* bv = &vec[(size_t)s * W];
      const u64* bc = &comb[(size_t)s * RW];
      for (int q = b / 64; q < W; ++q) v[q] ^= bv[q];
      for (int q = 0; q < RW; ++q) c[q] ^= bc[q];
    }
  }
};

void load_col(const qldpc_osd& O, int j, u64* v, int W) {
  std::fill(v, v + W, 0ull);
  for (int r : O.col_rows[j]) v[r >> 6] ^= 1ull << (r & 63);
}

int gf2_rank(const qldpc_osd& O) {
  Basis B;
  B.init(O.m, std::min(O.m, O.n));
  std::vector<u64> v(B.W), c(B.RW);
  int rank = 0;
  for (int j = 0; j < O.n && rank < O.m; ++j) {
    load_col(O, j, v.data(), B.W);
    std::fill(c.begin(), c.end(), 0ull);
    const int b = B.reduce(v.data(), c.data());
    if (b >= 0) {
      B.key[b] = rank;
      std::copy(v.begin(), v.end(), &B.vec[(size_t)rank * B.W]);
      ++rank;
    }
  }
  return rank;
}

struct Work {
  Basis B;
  std::vector<int32_t> cols, pivpos, ht;
  std::vector<u64> v, c, xs, xh, X;
  std::vector<uint8_t> cand;
};

double soft_weight(const qldpc_osd& O, const uint8_t* x) {
  double s = 0.0;
  for (int j = 0; j < O.n; ++j)
    if (x[j]) s += O.w[j];
  return s;
}

// Decode one non-converged syndrome; writes OSD-0 and OSD-w corrections.
void osd_one(const qldpc_osd& O, Work& K, const uint8_t* synd, const double* post, uint8_t* out0, uint8_t* outw) {
  const int m = O.m, n = O.n, rank = O.rank;
  K.cols.resize(n);
  std::iota(K.cols.begin(), K.cols.end(), 0);
  std::stable_sort(K.cols.begin(), K.cols.end(), [&](int a, int b) { return post[a] < post[b]; });
  Basis& B = K.B;
  B.init(m, rank);
  const int W = B.W, RW = B.RW;
  K.v.resize(W);
  K.c.resize(RW);
  // 1. greedy pivots in sorted order (positions recorded for the swap replay)
  K.pivpos.clear();
  for (int pos = 0; pos < n && (int)K.pivpos.size() < rank; ++pos) {
    load_col(O, K.cols[pos], K.v.data(), W);
    std::fill(K.c.begin(), K.c.end(), 0ull);
    const int b = B.reduce(K.v.data(), K.c.data());
    if (b < 0) continue;
    const int s = B.count++;
    B.key[b] = s;
    K.c[s >> 6] ^= 1ull << (s & 63);
    std::copy(K.v.begin(), K.v.end(), &B.vec[(size_t)s * W]);
    std::copy(K.c.begin(), K.c.end(), &B.comb[(size_t)s * RW]);
    K.pivpos.push_back(pos);
  }
  const int r = (int)K.pivpos.size();
  // 2. Neal's swap: pivot i moves to position i, the column there to its place
  for (int i = 0; i < r; ++i) std::swap(K.cols[i], K.cols[K.pivpos[i]]);
  const int k = n - r;
  K.ht.assign(K.cols.begin() + r, K.cols.end());
  // 3. OSD-0
  K.xs.assign(RW, 0ull);
  std::fill(K.v.begin(), K.v.end(), 0ull);
  for (int i = 0; i < m; ++i)
    if (synd[i] & 1u) K.v[i >> 6] ^= 1ull << (i & 63);
  B.reduce(K.v.data(), K.xs.data());
  auto expand = [&](const u64* x, uint8_t* dst) {
    std::fill(dst, dst + n, (uint8_t)0);
    for (int i = 0; i < r; ++i)
      if ((x[i >> 6] >> (i & 63)) & 1ull) dst[K.cols[i]] = 1;
  };
  expand(K.xs.data(), out0);
  if (O.method == 0 || O.order == 0 || k == 0) {
    std::copy(out0, out0 + n, outw);
    return;
  }
  const int w = std::min(O.order, k);
  const int nh = O.method == 2 ? k : w;  // columns whose x(h_j) is needed
  K.xh.assign((size_t)nh * RW, 0ull);
  for (int j = 0; j < nh; ++j) {
    load_col(O, K.ht[j], K.v.data(), W);
    B.reduce(K.v.data(), &K.xh[(size_t)j * RW]);
  }
  K.cand.resize(n);
  // weight of OSD-0; candidates must be strictly lighter
  long long best_cnt = 0;
  double best_w = 0.0;
  if (O.uniform) {
    for (int q = 0; q < RW; ++q) best_cnt += __builtin_popcountll(K.xs[q]);
  } else {
    best_w = soft_weight(O, out0);
  }
  std::copy(out0, out0 + n, outw);
  // candidate: x = xs ^ (xor of xh over t's bits); t bits are Ht positions
  auto consider = [&](const u64* x, const int* tj, int nt) {
    if (O.uniform) {
      long long cnt = nt;
      for (int q = 0; q < RW; ++q) cnt += __builtin_popcountll(x[q]);
      if (cnt >= best_cnt) return;
      best_cnt = cnt;
      expand(x, outw);
      for (int a = 0; a < nt; ++a) outw[K.ht[tj[a]]] = 1;
    } else {
      expand(x, K.cand.data());
      for (int a = 0; a < nt; ++a) K.cand[K.ht[tj[a]]] = 1;
      const double sw = soft_weight(O, K.cand.data());
      if (sw >= best_w) return;
      best_w = sw;
      std::copy(K.cand.begin(), K.cand.end(), outw);
    }
  };
  std::vector<u64> tmp(RW);
  if (O.method == 1) {  // osd_e: all 2^w inputs, natural order (l = 0 is OSD-0 itself)
    const long long L = 1ll << w;
    K.X.assign((size_t)L * RW, 0ull);
    std::copy(K.xs.begin(), K.xs.end(), K.X.begin());
    int tj[64];
    for (long long l = 1; l < L; ++l) {
      const u64* prev = &K.X[(size_t)(l & (l - 1)) * RW];
      const u64* h = &K.xh[(size_t)ctz64((u64)l) * RW];
      u64* cur = &K.X[(size_t)l * RW];
      for (int q = 0; q < RW; ++q) cur[q] = prev[q] ^ h[q];
      int nt = 0;
      for (u64 b = (u64)l; b; b &= b - 1) tj[nt++] = ctz64(b);
      consider(cur, tj, nt);
    }
  } else {  // osd_cs: weight-1 over all of Ht, then weight-2 pairs inside Ht[0:w]
    for (int j = 0; j < k; ++j) {
      for (int q = 0; q < RW; ++q) tmp[q] = K.xs[q] ^ K.xh[(size_t)j * RW + q];
      consider(tmp.data(), &j, 1);
    }
    for (int i = 0; i < w; ++i)
      for (int j = i + 1; j < w; ++j) {
        for (int q = 0; q < RW; ++q) tmp[q] = K.xs[q] ^ K.xh[(size_t)i * RW + q] ^ K.xh[(size_t)j * RW + q];
        const int tj[2] = {i, j};
        consider(tmp.data(), tj, 2);
      }
  }
}

}  // namespace

extern "C" {

int qldpc_osd_create(int32_t m, int32_t n, const int32_t* row_ptr, const int32_t* col_idx,
                     const double* channel_probs, int32_t osd_method, int32_t osd_order, qldpc_osd** out) {
  if (!row_ptr || !col_idx || !channel_probs || !out) return set_err(QLDPC_EINVAL, "NULL argument");
  if (m < 0 || n <= 0) return set_err(QLDPC_EINVAL, "bad matrix shape");
  if (osd_method < 0 || osd_method > 2) return set_err(QLDPC_EINVAL, "osd_method must be 0 (osd_0), 1 (osd_e) or 2 (osd_cs)");
  if (osd_order < 0 || (osd_method == 1 && osd_order > 20))
    return set_err(QLDPC_EINVAL, "osd_order must be >= 0 (and <= 20 for osd_e)");
  auto* O = new qldpc_osd();
  O->m = m;
  O->n = n;
  O->method = osd_method;
  O->order = osd_order;
  O->col_rows.assign(n, {});
  for (int i = 0; i < m; ++i)
    for (int e = row_ptr[i]; e < row_ptr[i + 1]; ++e) {
      const int j = col_idx[e];
      if (j < 0 || j >= n) {
        delete O;
        return set_err(QLDPC_EINVAL, "column index out of range");
      }
      O->col_rows[j].push_back(i);
    }
  O->w.resize(n);
  for (int j = 0; j < n; ++j) {
    if (!(channel_probs[j] > 0.0 && channel_probs[j] < 1.0)) {
      delete O;
      return set_err(QLDPC_EINVAL, "channel_probs must lie in (0, 1)");
    }
    O->w[j] = std::log(1.0 / channel_probs[j]);
    if (O->w[j] != O->w[0]) O->uniform = false;
  }
  O->rank = gf2_rank(*O);
  *out = O;
  return 0;
}

int qldpc_osd_destroy(qldpc_osd* osd) {
  delete osd;
  return 0;
}

int qldpc_osd_rank(const qldpc_osd* osd, int32_t* rank) {
  if (!osd || !rank) return set_err(QLDPC_EINVAL, "NULL argument");
  *rank = osd->rank;
  return 0;
}

int qldpc_osd_decode_batch(const qldpc_osd* osd, const uint8_t* synd, const double* post, const uint8_t* conv,
                           const uint8_t* bp_corr, uint8_t* out_osd0, uint8_t* out_osdw, int64_t B,
                           int32_t threads) {
  if (!osd || (B > 0 && (!synd || !post || !out_osdw))) return set_err(QLDPC_EINVAL, "NULL argument");
  if (conv && !bp_corr) return set_err(QLDPC_EINVAL, "conv needs bp_corr");
  if (B <= 0) return 0;
  const int m = osd->m, n = osd->n;
  std::vector<int64_t> todo;
  for (int64_t b = 0; b < B; ++b) {
    if (conv && conv[b]) {
      std::copy(bp_corr + b * n, bp_corr + (b + 1) * n, out_osdw + b * n);
      if (out_osd0) std::copy(bp_corr + b * n, bp_corr + (b + 1) * n, out_osd0 + b * n);
    } else {
      todo.push_back(b);
    }
  }
  int T = threads;
  if (T <= 0) {  // the process's CPU share when the launcher states it (OMP_NUM_THREADS), else all cores
    const char* e = std::getenv("OMP_NUM_THREADS");
    T = e ? std::atoi(e) : 0;
    if (T <= 0) T = (int)std::max(1u, std::thread::hardware_concurrency());
  }
  T = (int)std::min<int64_t>(T, (int64_t)todo.size());
  if (T <= 0) return 0;
  auto run = [&](int t) {
    Work K;
    std::vector<uint8_t> o0(n);
    for (size_t a = t; a < todo.size(); a += T) {
      const int64_t b = todo[a];
      osd_one(*osd, K, synd + b * m, post + b * n, out_osd0 ? out_osd0 + b * n : o0.data(), out_osdw + b * n);
    }
  };
  if (T == 1) {
    run(0);
  } else {
    std::vector<std::thread> pool;
    for (int t = 0; t < T; ++t) pool.emplace_back(run, t);
    for (auto& th : pool) th.join();
  }
  return 0;
}

}  // extern "C"

// ===========================================================================
// GPU OSD: one workgroup per syndrome, persistent over the batch (uniform priors: popcount
// weights; non-uniform: soft weights summed in column order, candidate step 6').  Same algorithm and outputs as the host stage above, laid out for the
// GPU: the columns are bitonic-sorted in LDS by (posterior, index) — a stable
// ascending order — and H is loaded with its columns permuted into that order,
// word-major (word q of row i at q*m + i) in a per-workgroup HBM slice, so a
// pivot search tests one coalesced word per row and a row update xors
// coalesced words.  Full Gauss-Jordan over the positions in order finds the
// same greedy pivots (the x of an independent pivot set is unique, whatever
// pivot rows are chosen); the OSD inputs are then bit-vectors over the pivot
// index, and every candidate's weight (popcount, the order relation of the
// uniform soft weight) is reduced to the lexicographic minimum of
// (weight, candidate index) = the first strictly lightest in ldpc's order.
namespace {

constexpr int kOsdThreads = 256;      // HBM-slice image: memory-latency bound, 3 workgroups per CU
constexpr int kOsdThreadsLds = 1024;  // LDS-resident image: one workgroup per CU, 16 waves on its rows

#ifndef QLDPC_STAMPS
#define QLDPC_STAMPS 0
#endif
// diagnostic builds (QLDPC_STAMPS): per-step cycle sums of osd_gpu_kernel, wave 0 of each
// workgroup: [0] sort, [1] H load, [2] Gauss-Jordan, [3] swaps + bit-vectors, [4] candidates,
// [5] outputs, [6] syndromes, [7] positions visited, [8] of [2]: pivot searches + their barrier,
// [9] of [2] (register rows): pivot-row publication + its barrier
__device__ unsigned long long g_osd_stamps[16];
__device__ inline unsigned long long osd_stamp() {
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
constexpr int kOsdMaxN = 8192;
// column-window launch: the mark a syndrome whose elimination overran the window leaves in its
// outw[0] for the full-width redo launch (outputs are 0 / 1 bytes otherwise)
constexpr uint8_t kOsdRedo = 0xFF;
// column window: positions past rank + nh the window words cover (dependent positions allowed
// before the rank is reached)
constexpr int kOsdWinSlack = 64;
// forward elimination (PNL 5): bytes of the compaction staging area (64 rows in, 64 out)
__host__ __device__ inline size_t osd_fwd_stg_bytes(int wr) { return 2 * ((size_t)wr * 64 * 8 + 64 * 4); }
// forward elimination: U words of pivot row k over pivot block B >= k / 64, packed upper-triangular
// by blocks (block b's 64 rows hold RW - b words each)
__host__ __device__ inline int osd_ul_at(int k, int B, int RW) {
  const int b = k >> 6;
  return 64 * (b * RW - (b * (b - 1)) / 2 + (B - b)) + (k & 63);
}
__host__ __device__ inline int osd_ul_words(int RW) { return 64 * (RW * (RW + 1) / 2); }
// register-row mode: pivot-row words read per batch ahead of their xors
#ifndef QLDPC_OSD_XB
#define QLDPC_OSD_XB 8
#endif
constexpr int kOsdXB = QLDPC_OSD_XB;
// register-row mode: the lean per-pivot loop (one stamped LDS max per wave instead of a
// triple-buffered atomicMin, a DPP row-broadcast wave minimum, pivots recorded in LDS); 0 = the
// round-3 loop (A/B builds)
#ifndef QLDPC_OSD_LEAN
#define QLDPC_OSD_LEAN 1
#endif
// A/B build: one barrier per pivot in register-row mode (the candidate row published before the
// search barrier, per-wave slots of two step parities)
#ifndef QLDPC_OSD_1B
#define QLDPC_OSD_1B 0
#endif
// register-row mode: Four-Russians groups of kOsdG pivots (QLDPC_OSD_M4R): within a group only
// the pivot word is updated per pivot (plus a mask of the group pivots' start rows each row has
// absorbed); at the group's end every row xors in ONE table entry (the xor of its mask's start
// rows) per remaining word.  MEASURED AND NOT KEPT (A/B builds only): bit-exact (57 GPU tests),
// n1600 BP+OSD 595 k (G = 4) / 596 k (G = 6) vs 614 k with the lean loop, n225 10.6 M vs 12.3 M
// (profiles/r04/passr/): the group ends' two extra barriers and table build cost more than the
// row xors they save
#ifndef QLDPC_OSD_M4R
#define QLDPC_OSD_M4R 0
#endif
#ifndef QLDPC_OSD_G
#define QLDPC_OSD_G 4
#endif
constexpr bool kOsdM4R = QLDPC_OSD_M4R && !QLDPC_OSD_1B;
// A/B build: OSD steps 4-5 from the register rows (see the RR branch's end); 0 = the HBM path
#ifndef QLDPC_OSD_XREG
#define QLDPC_OSD_XREG 0
#endif
// diagnostic A/B build: the lean loop's row xors done three times (same rows): the step's
// sensitivity to its row-update VALU work
#ifndef QLDPC_OSD_XOR3
#define QLDPC_OSD_XOR3 0
#endif
// blocked mode (PNL 3): byte offset of the Four-Russians tables in the panel area (after the
// half-words and masks [m] u32, pk [32], pidx [m]) and the area's size with them ([8][16][WR + 1] u64)
__host__ __device__ inline size_t osd_blk_tab_off(int m) { return ((size_t)12 * m + 128 + 15) & ~(size_t)15; }
inline size_t osd_blk_bytes(int m, int wr) { return osd_blk_tab_off(m) + (size_t)8 * 16 * (wr + 1) * 8; }

constexpr int kOsdG = QLDPC_OSD_G;
// rows of (WR + 1) words in the register-row pivot area: the pivot row (1), the one-barrier build's
// per-wave slots, or the Four-Russians table (2^G rows) and its per-pivot slots (4 rows)
constexpr int osd_prows(int lb) { return QLDPC_OSD_1B ? 2 * (lb / 64) : kOsdM4R ? (1 << kOsdG) + 4 : 1; }


// calls f(integral_constant<int, Q>) for Q = 0, 1, ... while it returns true (compile-time word index)
template <int... Q, class F>
__device__ __attribute__((always_inline)) inline void osd_for_words(std::integer_sequence<int, Q...>, F&& f) {
  (void)(f(std::integral_constant<int, Q>{}) && ...);
}

struct OsdGpuArgs {
  const int32_t* rp;
  const int32_t* ci;
  const uint8_t* synd;     // [B][m]
  const double* post;      // [B][n]
  const uint8_t* conv;     // [B] or null
  const long long* shot;   // [B] or null: fused-loop capture slots, < 0 = BP converged (skipped)
  const uint8_t* bp_corr;  // [B][n] or null
  const double* softw;     // [n] log(1 / p_j) for non-uniform priors, or null (uniform: popcount weights)
  uint8_t* out0;           // [B][n] or null
  uint8_t* outw;           // [B][n]
  u64* ws;                 // per workgroup: M [W][m] | X [(1 + nh)][RW]
  int32_t* iws;            // per workgroup: pivrow [rank] | pivpos [rank] | swp [n]
  long long B;
  int m, n, W, RW, rank, method, order, NP;
  int m_lds;  // 1: the matrix lives in LDS, aliasing the sort tables (copied out first), else in the HBM slice
  int bits_off;  // LDS byte offset of the used / syndrome bit-vectors
  int pbuf_off;  // register-row mode: LDS byte offset of the pivot-row broadcast buffer
  int pnl_off;   // panel mode: LDS byte offset of the panel area (words, masks, pivot rows, indices)
  int syn_lds;   // two-syndrome register-row kernel: LDS bytes per syndrome area
  int win;       // 1: column-window launch (rows hold the first WR words only; a syndrome whose
                 // elimination overruns them is marked for the redo launch), 2: the redo launch,
                 // 3: test hook (QLDPC_OSD_WIN_REDO=1): a window launch that also marks every odd b
  long long ws_words, iws_ints;
};

// dst[q*m] ^= src[q*m] for q < W: no aliasing between the two rows, so the loads can run ahead
// of the stores (in-place xors through one pointer would serialize word by word)
__device__ inline void row_xor(u64* __restrict__ dst, const u64* __restrict__ src, int W, int m) {
#pragma unroll 8
  for (int q = 0; q < W; ++q) dst[(size_t)q * m] ^= src[(size_t)q * m];
}

// minimum of a 32-bit value over the 64 lanes of a wave (all lanes active): DPP quad and row
// rotations give each lane its 16-lane row's minimum, four readlanes combine the rows
__device__ inline uint32_t wave_min_u32(uint32_t v) {
  auto mn = [](uint32_t a, uint32_t b) { return a < b ? a : b; };
  v = mn(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
  v = mn(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
  v = mn(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xF, 0xF, false));  // row_ror:4
  v = mn(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false));  // row_ror:8
  return mn(mn((uint32_t)__builtin_amdgcn_readlane((int)v, 0), (uint32_t)__builtin_amdgcn_readlane((int)v, 16)),
            mn((uint32_t)__builtin_amdgcn_readlane((int)v, 32), (uint32_t)__builtin_amdgcn_readlane((int)v, 48)));
}

// the same minimum in 6 DPP VALU + 1 readlane: rotations give every lane its 16-lane row's
// minimum, row_bcast:15 / row_bcast:31 fold rows 0-1 / 2-3 / all into lane 63 (the GFX9 DPP
// broadcasts; the s_nops are the DPP read-after-VALU-write wait states).  All lanes active.
__device__ inline uint32_t wave_min_u32_bc(uint32_t v) {
  asm volatile(
      "s_nop 1\n\t"
      "v_min_u32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_min_u32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_min_u32_dpp %0, %0, %0 row_ror:4 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_min_u32_dpp %0, %0, %0 row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_min_u32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_min_u32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
      "s_nop 1"
      : "+v"(v));
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// v_ffbl_b32: index of the lowest set bit, 0xFFFFFFFF for 0
__device__ inline uint32_t ffbl_u32(uint32_t x) {
  uint32_t r;
  asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}

// LDS max at byte address a by the calling lanes, completed before return (plain ds_max_u32: the
// compiler's atomic optimizer would wrap a builtin atomic in a first-lane election per call)
__device__ inline void lds_max_u32_sync(uint32_t a, uint32_t v) {
  asm volatile("ds_max_u32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : : "v"(a), "v"(v) : "memory");
}

__device__ inline u64 ord_key(double x) {
  if (x == 0.0) x = 0.0;  // -0 ties +0, as std::stable_sort's `<` has it
  const u64 u = (u64)__double_as_longlong(x);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}

// WR > 0: register-row mode (m <= LB, W <= WR): thread i keeps row i of the permuted H in WR
// u64 registers through the whole Gauss-Jordan; a pivot's owner publishes the pivot row's words
// q.. in an LDS buffer and the rows that have the pivot bit xor them in registers, so a row
// update costs no LDS writes (the word-major LDS / HBM image paid one 8-byte store per word and
// row).  The reduced rows go to the HBM slice afterwards for the candidate bit-vectors.
// PNL (register-row mode): panel elimination.  Pivots are searched a 64-column panel (one row word)
// at a time by ONE wave that holds every row's panel word and a 64-bit combination mask per row
// (which of the panel's pivot rows, in their panel-start state, the row has absorbed): no barrier
// per pivot.  Then the panel's pivot rows publish their remaining words once and every row xors in
// the rows its mask names (uniform loop, broadcast LDS reads).  Same pivots (the lexicographic
// minimum of (first set bit >= scan position, row) over unused rows, on up-to-date words) and the
// same reduced rows as the per-pivot elimination; three barriers per panel instead of two per pivot.
// WPE: minimum waves per SIMD the VGPR budget is pinned to (two workgroups per CU: the
// column-window kernels, 2 x 12 waves; the two-rows-per-thread blocked kernels, 2 x 6 waves).
template <int LB, int WR = 0, int RPT = 1, int PNL = 0, int WPE = 1>
__global__ void __launch_bounds__(LB) __attribute__((amdgpu_waves_per_eu(RPT == 2 ? 3 : WPE)))
osd_gpu_kernel(OsdGpuArgs A) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, TB = blockDim.x;
  const int m = A.m, n = A.n, W = A.W, RW = A.RW, NP = A.NP, rank = A.rank;
  u64* skey = reinterpret_cast<u64*>(smem);                    // [NP]
  int32_t* sidx = reinterpret_cast<int32_t*>(skey + NP);       // [NP] -> cols (sorted position -> column)
  int32_t* pos = sidx + NP;                                    // [n]  column -> sorted position
  uint32_t* used = reinterpret_cast<uint32_t*>(smem + A.bits_off);  // [ceil(m/32)]
  uint32_t* sb = used + (m + 31) / 32;                         // [ceil(m/32)] syndrome, reduced
  __shared__ int s_piv[3], s_npiv;  // s_piv triple-buffered by position: reset two columns ahead
  __shared__ uint32_t s_pivx;       // lean loop: (search step << 17) | (0x1FFFF - key), max over the waves
  __shared__ u64 s_best, s_bestw;
  u64* Mg = A.ws + (size_t)blockIdx.x * A.ws_words;
  u64* X = Mg + (size_t)W * m;  // X[0] = S0, X[1 + j] = x(h_j)
  // matrix: LDS when it fits (at offset 0, over the sort tables, which are copied to the
  // workgroup's HBM ints first), else the per-workgroup HBM slice
  // (compile-time per instantiation, so the accesses are ds_* or global_*, never flat)
  constexpr bool kRR = WR > 0;
  constexpr bool kMLds = !kRR && LB == kOsdThreadsLds;
  u64* M = kMLds ? reinterpret_cast<u64*>(smem) : Mg;  // register-row mode: Mg holds the reduced rows
  int32_t* pivrow = A.iws + (size_t)blockIdx.x * A.iws_ints;
  int32_t* pivpos = pivrow + rank;
  int32_t* swp = pivpos + rank;
  int32_t* gsidx = swp + n;   // [n] LDS mode: sorted position -> column
  int32_t* gpos = gsidx + n;  // [n] LDS mode: column -> sorted position
  const int32_t* sidxr = kMLds ? gsidx : sidx;
  const int k = n - rank;
  const int w = A.order < k ? A.order : k;
  const int nh = A.method == 2 ? k : w;

  unsigned long long st[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long t0 = osd_stamp(), t1;
#define OSD_ST(k)              \
  if (QLDPC_STAMPS) {          \
    t1 = osd_stamp();          \
    st[k] += t1 - t0;          \
    t0 = t1;                   \
  }
  for (long long b = blockIdx.x; b < A.B; b += gridDim.x) {
    uint8_t* ow = A.outw + b * (long long)n;
    uint8_t* o0 = A.out0 ? A.out0 + b * (long long)n : nullptr;
    if (A.win == 2 && ow[0] != kOsdRedo) continue;  // redo launch: only the window's overruns (uniform)
    if (A.shot && A.shot[b] < 0) continue;  // captured decode that converged at max_iter: no OSD
    if (A.conv && A.conv[b]) {  // BP converged: bposd_decoder returns the BP decoding
      for (int j = tid; j < n; j += TB) {
        const uint8_t v = A.bp_corr[b * (long long)n + j];
        ow[j] = v;
        if (o0) o0[j] = v;
      }
      continue;  // uniform over the workgroup
    }
    const double* post = A.post + b * (long long)n;
    const uint8_t* synd = A.synd + b * (long long)m;
    // 1. stable ascending sort of the columns by posterior (bitonic on (key, index))
    for (int q = tid; q < NP; q += TB) {
      skey[q] = q < n ? ord_key(post[q]) : ~0ull;
      sidx[q] = q < n ? q : 0x7FFFFFFF;
    }
    __syncthreads();
    for (int size = 2; size <= NP; size <<= 1)
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        for (int q = tid; q < NP / 2; q += TB) {
          const int lo = 2 * q - (q & (stride - 1));
          const int hi = lo + stride;
          const bool up = (lo & size) == 0;
          const u64 ka = skey[lo], kb = skey[hi];
          const int ia = sidx[lo], ib = sidx[hi];
          const bool gt = ka > kb || (ka == kb && ia > ib);
          if (gt == up) {
            skey[lo] = kb; skey[hi] = ka;
            sidx[lo] = ib; sidx[hi] = ia;
          }
        }
        __syncthreads();
      }
    OSD_ST(0)
    if (kMLds) {
      for (int q = tid; q < n; q += TB) {
        const int c = sidx[q];
        gsidx[q] = c;
        gpos[c] = q;
      }
    } else {
      for (int q = tid; q < n; q += TB) pos[sidx[q]] = q;
    }
    for (int q = tid; q < (m + 31) / 32; q += TB) {
      used[q] = 0;
      uint32_t v = 0;
      for (int t = 0; t < 32 && q * 32 + t < m; ++t) v |= (uint32_t)(synd[q * 32 + t] & 1u) << t;
      sb[q] = v;
    }
    if (tid == 0) {
      s_npiv = 0;
      s_piv[0] = s_piv[1] = s_piv[2] = 0x7FFFFFFF;
      s_pivx = 0u;
    }
    __syncthreads();
    bool xdone = false;  // uniform: S0 / x(h_j) built from the register rows (steps 4-5 done)
    if constexpr (kRR) {
      // 2-3 (register rows): rows tid + j*TB (j < RPT) of the permuted H, words by compile-time index
      u64 row[RPT][WR];
      uint32_t sbit[RPT];
      bool used_r[RPT];
#pragma unroll
      for (int j = 0; j < RPT; ++j) {
        const int i = tid + j * TB;
#pragma unroll
        for (int q = 0; q < WR; ++q) row[j][q] = 0;
        sbit[j] = 0;
        used_r[j] = i >= m;  // rows past m never become candidates
        if (i < m) {
          for (int e = A.rp[i]; e < A.rp[i + 1]; ++e) {
            const int p = pos[A.ci[e]];
            const int pq = p >> 6;
            const u64 bit = 1ull << (p & 63);
#pragma unroll
            for (int q = 0; q < WR; ++q) row[j][q] ^= (pq == q) ? bit : 0ull;
          }
          sbit[j] = synd[i] & 1u;
        }
      }
      u64* pbuf = reinterpret_cast<u64*>(smem + A.pbuf_off);  // [WR] pivot row, [WR] its syndrome bit
      OSD_ST(1)
      int npiv = 0;   // uniform
      if constexpr (PNL == 3) {
        // Blocked elimination (round 5; opt-in QLDPC_OSD_PNL=3, measured
        // slower than the lean loop): the
        // per-pivot loops below cost every wave two barriers and a pivot-row round trip per pivot
        // (~2,100 cycles per pivot at n1600, 0.62 of wave cycles parked, profiles/r04/passt/).  Here
        // the pivots of a 32-column panel (half a row word) are found by ONE search wave with no
        // barrier per pivot: it holds every row's panel half-word (rows s * 64 + lane, SM slots) and
        // a 32-bit combination mask per row (which of the panel's pivot rows, in their panel-start
        // state, the row has absorbed); a pivot step is a wave minimum over the unused rows' first
        // set bits (the lexicographic minimum of (column, row): the greedy scan's pivot and its lowest
        // row, as the loops below pick it), two readlanes and a masked xor per slot.  Then the panel's
        // pivot rows publish their panel-start words q.. (+ syndrome bit) as the single entries of
        // 4-pivot Four-Russians tables (16 combinations per group), the workgroup fills the tables,
        // and every row xors in ONE table entry per group for everything past the panel.  Exact: the
        // same pivots, pivot rows and reduced rows as the per-pivot elimination (an unused row is zero
        // before the scan position, so the pivot rows' earlier words are zero and the words < q never
        // change).  Four barriers per panel instead of two per pivot.
        constexpr int SM = (LB * RPT) / 64;  // row slots per lane of the search wave (rows s * 64 + lane)
        constexpr u64 kLo = 0xFFFFFFFFull, kHi = ~kLo;
        constexpr int TS = WR + 1;   // table entry stride: words of a start row + its syndrome bit
        uint32_t* pw = reinterpret_cast<uint32_t*>(smem + A.pnl_off);  // [m] panel half-words
        uint32_t* pmsk = pw + m;                                       // [m] combination masks
        int* pk = reinterpret_cast<int*>(pmsk + m);                    // [32] the panel's pivot rows
        int* pidx = pk + 32;                                           // [m] panel index of a pivot row
        u64* T = reinterpret_cast<u64*>(smem + A.pnl_off + osd_blk_tab_off(m));  // [8 groups][16][TS]
        int32_t* lkk = reinterpret_cast<int32_t*>(smem);  // pivots (position << 11) | row, over the dead sort keys
        __shared__ int s_P;
        uint32_t usedm = 0;  // search wave: bit s = row s * 64 + lane is used (rows >= m: always)
        if (tid < 64) {
#pragma unroll
          for (int s2 = 0; s2 < SM; ++s2)
            if (s2 * 64 + tid >= m) usedm |= 1u << s2;
        }
        // one compile-time word q per call (every row word stays in a VGPR; a runtime q would index
        // the row array and demote it to scratch)
        auto blk_word = [&](auto qc) __attribute__((always_inline)) -> bool {
          constexpr int q = decltype(qc)::value;
          if (q * 64 >= n || npiv >= rank) return false;  // uniform
          for (int h = 0; h < 2; ++h) {
            if (q * 64 + h * 32 >= n || npiv >= rank) break;  // uniform
            // 1. every row's panel half-word (every earlier panel applied)
            unsigned long long tb0 = QLDPC_STAMPS ? osd_stamp() : 0ull;
#pragma unroll
            for (int j = 0; j < RPT; ++j)
              if (tid + j * TB < m) pw[tid + j * TB] = (uint32_t)(row[j][q] >> (32 * h));
            __syncthreads();
            if (QLDPC_STAMPS) {  // [11]: step 1 + its barrier
              const unsigned long long t = osd_stamp();
              st[11] += t - tb0;
              tb0 = t;
            }
            // 2. the search wave: the panel's greedy pivots, its rows' final half-words and masks
            if (tid < 64) {
              // a lone wave is latency-bound: the pivot step keeps its dependent chains short (unused
              // masks as VGPRs, a min3 tree over the slots, a 4-level select tree for the pivot row's
              // half-word and mask, the pivot list in one VGPR written after the panel)
              uint32_t wv[SM], cm[SM];
              uint32_t ub = ~usedm;  // bit s: row s * 64 + lane is a candidate (unused, < m)
#pragma unroll
              for (int s2 = 0; s2 < SM; ++s2) {
                wv[s2] = s2 * 64 + tid < m ? pw[s2 * 64 + tid] : 0u;
                cm[s2] = 0u;
              }
              uint32_t pkv = 0;  // lane k: (position << 11) | row of the panel's pivot k
              int P = 0, np = npiv;
              while (np < rank) {  // uniform
                // key = (first set bit << 11) | row over the unused rows; none: >= 0xFFFFF800
                uint32_t kk[SM];
#pragma unroll
                for (int s2 = 0; s2 < SM; ++s2) {
                  const uint32_t um = (uint32_t)__builtin_amdgcn_sbfe((int)ub, s2, 1);
                  kk[s2] = (ffbl_u32(wv[s2] & um) << 11) | (uint32_t)(s2 * 64 + tid);
                }
                // min3 tree over the slots (compile-time shapes: SM <= 16 -> at most 3 levels)
                constexpr int N1 = (SM + 2) / 3, N2 = (N1 + 2) / 3, N3 = (N2 + 2) / 3;
                auto mn = [](uint32_t a, uint32_t b) { return a < b ? a : b; };
                uint32_t l1[N1], l2[N2];
#pragma unroll
                for (int i = 0; i < N1; ++i)
                  l1[i] = mn(kk[3 * i], mn(3 * i + 1 < SM ? kk[3 * i + 1 < SM ? 3 * i + 1 : 0] : ~0u,
                                           3 * i + 2 < SM ? kk[3 * i + 2 < SM ? 3 * i + 2 : 0] : ~0u));
#pragma unroll
                for (int i = 0; i < N2; ++i)
                  l2[i] = mn(l1[3 * i], mn(3 * i + 1 < N1 ? l1[3 * i + 1 < N1 ? 3 * i + 1 : 0] : ~0u,
                                           3 * i + 2 < N1 ? l1[3 * i + 2 < N1 ? 3 * i + 2 : 0] : ~0u));
                static_assert(N3 == 1, "search wave: at most 27 row slots");
                const uint32_t key = wave_min_u32_bc(mn(l2[0], mn(N2 > 1 ? l2[N2 > 1 ? 1 : 0] : ~0u,
                                                                  N2 > 2 ? l2[N2 > 2 ? 2 : 0] : ~0u)));
                if (key > 0x1FFFFu) break;  // no pivot left in this panel (uniform)
                const int fb = (int)(key >> 11), r = (int)(key & 2047u), sr = r >> 6, lr = r & 63;
                // the pivot row's half-word and mask: a select tree on sr's bits (levels of halving
                // arrays, short live ranges), then one readlane each
                constexpr int H1 = (SM + 1) / 2, H2 = (H1 + 1) / 2, H3 = (H2 + 1) / 2;
                uint32_t aw[H1], ac[H1];
                {
                  // bitwise selects (a select of two array loads would become a load at a selected
                  // index: a dynamically indexed array, demoted to scratch)
                  const uint32_t msk = (sr & 1) ? ~0u : 0u;  // uniform
#pragma unroll
                  for (int i = 0; i < H1; ++i) {
                    aw[i] = wv[2 * i] ^ ((wv[2 * i] ^ wv[2 * i + 1 < SM ? 2 * i + 1 : 2 * i]) & msk);
                    ac[i] = cm[2 * i] ^ ((cm[2 * i] ^ cm[2 * i + 1 < SM ? 2 * i + 1 : 2 * i]) & msk);
                  }
                }
                uint32_t bw[H2], bc[H2];
                {
                  const uint32_t msk = (sr & 2) ? ~0u : 0u;
#pragma unroll
                  for (int i = 0; i < H2; ++i) {
                    bw[i] = aw[2 * i] ^ ((aw[2 * i] ^ aw[2 * i + 1 < H1 ? 2 * i + 1 : 2 * i]) & msk);
                    bc[i] = ac[2 * i] ^ ((ac[2 * i] ^ ac[2 * i + 1 < H1 ? 2 * i + 1 : 2 * i]) & msk);
                  }
                }
                uint32_t cw[H3], cc[H3];
                {
                  const uint32_t msk = (sr & 4) ? ~0u : 0u;
#pragma unroll
                  for (int i = 0; i < H3; ++i) {
                    cw[i] = bw[2 * i] ^ ((bw[2 * i] ^ bw[2 * i + 1 < H2 ? 2 * i + 1 : 2 * i]) & msk);
                    cc[i] = bc[2 * i] ^ ((bc[2 * i] ^ bc[2 * i + 1 < H2 ? 2 * i + 1 : 2 * i]) & msk);
                  }
                }
                uint32_t dw = cw[0], dc = cc[0];
                if constexpr (H3 > 1) {
                  const uint32_t msk = (sr & 8) ? ~0u : 0u;
                  dw = cw[0] ^ ((cw[0] ^ cw[H3 > 1 ? 1 : 0]) & msk);
                  dc = cc[0] ^ ((cc[0] ^ cc[H3 > 1 ? 1 : 0]) & msk);
                }
                static_assert(SM <= 16, "search wave: at most 16 row slots");
                const uint32_t pwv = (uint32_t)__builtin_amdgcn_readlane((int)dw, lr);
                const uint32_t pmv = (uint32_t)__builtin_amdgcn_readlane((int)dc, lr);
                const uint32_t add = pmv | (1u << P);
                const bool me = tid == lr;
#pragma unroll
                for (int s2 = 0; s2 < SM; ++s2) {
                  const uint32_t sel = (uint32_t)__builtin_amdgcn_sbfe((int)wv[s2], fb, 1);  // -(bit fb)
                  const bool pr = me && s2 == sr;  // the pivot row keeps its word and mask
                  wv[s2] = pr ? pwv : wv[s2] ^ (pwv & sel);
                  cm[s2] = pr ? pmv : cm[s2] ^ (add & sel);
                }
                ub = me ? (ub & ~(1u << sr)) : ub;  // the pivot row leaves the candidates
                pkv = tid == P ? (uint32_t)(((q * 64 + h * 32 + fb) << 11) | r) : pkv;
                ++P;
                ++np;
              }
              if (tid < P) {
                lkk[npiv + tid] = (int32_t)pkv;
                pk[tid] = (int)(pkv & 2047u);
                pidx[pkv & 2047u] = tid;
              }
#pragma unroll
              for (int s2 = 0; s2 < SM; ++s2)
                if (s2 * 64 + tid < m) {
                  pw[s2 * 64 + tid] = wv[s2];
                  pmsk[s2 * 64 + tid] = cm[s2];
                }
              usedm = ~ub;
              if (tid == 0) {
                s_P = P;
                s_npiv = np;
              }
              if (QLDPC_STAMPS) {  // [8]: the search, [7]: its pivots
                const unsigned long long t = osd_stamp();
                st[8] += t - tb0;
                st[7] += (unsigned long long)P;
                tb0 = t;
              }
            }
            __syncthreads();
            const int P = s_P;
            npiv = s_npiv;
            // 3. the panel's pivot rows publish their panel-start rows (words q.., syndrome bit) as
            // the single entries of their group's table; every row takes its final half-word and mask
            uint32_t cmk[RPT], fw[RPT];
#pragma unroll
            for (int j = 0; j < RPT; ++j) {
              const int i = tid + j * TB;
              cmk[j] = 0;
              fw[j] = 0;
              if (i < m) {
                cmk[j] = pmsk[i];
                fw[j] = pw[i];
                const int kx = pidx[i];
                if (kx >= 0 && kx < P && pk[kx] == i) {  // (stale entries of earlier panels fail the check)
                  used_r[j] = true;
                  u64* d = T + (size_t)((kx >> 2) * 16 + (1 << (kx & 3))) * TS;
#pragma unroll
                  for (int q2 = q; q2 < WR; ++q2) d[q2] = row[j][q2];
                  d[WR] = sbit[j];
                }
              }
            }
            __syncthreads();
            // 4. every group's entries of >= 2 pivots: the xor of its single entries
            const int ng = (P + 3) >> 2;
            constexpr int nw = WR + 1 - q;  // words q..WR-1 and the syndrome entry
            for (int t = tid; t < ng * 16 * nw; t += TB) {
              const int gc = t / nw, c = gc & 15;
              const int wd = q + t % nw;
              if (c & (c - 1)) {
                const u64* g0 = T + (size_t)(gc - c) * TS + wd;
                u64 v = 0;
#pragma unroll
                for (int i = 0; i < 4; ++i)
                  if ((c >> i) & 1) v ^= g0[(size_t)(1 << i) * TS];
                T[(size_t)gc * TS + wd] = v;
              }
            }
            __syncthreads();
            if (QLDPC_STAMPS) {  // [9]: the search barrier, the single entries and the table fill
              const unsigned long long t = osd_stamp();
              st[9] += t - tb0;
              tb0 = t;
            }
            // 5. every row: one table entry per group into everything past the panel (the high half
            // of word q when the panel is its low half, words q + 1.., the syndrome bit); the panel
            // half-word is the search's final value
#pragma unroll
            for (int j = 0; j < RPT; ++j) {
              if (tid + j * TB < m) {
                u64 accq = 0;
                for (int g = 0; g < ng; ++g) {  // uniform bound
                  const uint32_t c = (cmk[j] >> (4 * g)) & 15u;
                  if (c) {
                    const u64* src = T + (size_t)(g * 16 + (int)c) * TS;
                    accq ^= src[q];
#pragma unroll
                    for (int q2 = q + 1; q2 < WR; ++q2) row[j][q2] ^= src[q2];
                    sbit[j] ^= (uint32_t)src[WR];
                  }
                }
                row[j][q] = h ? ((row[j][q] & kLo) | ((u64)fw[j] << 32)) : (((row[j][q] ^ accq) & kHi) | (u64)fw[j]);
              }
            }
            if (QLDPC_STAMPS) st[10] += osd_stamp() - tb0;  // [10]: the row updates
            // (pw is rewritten by the next panel's step 1 after these reads; T behind its first two barriers)
          }
          return true;
        };
        osd_for_words(std::make_integer_sequence<int, WR>{}, blk_word);
        for (int i = tid; i < npiv; i += TB) {
          const int v = lkk[i];
          pivrow[i] = v & 2047;
          pivpos[i] = v >> 11;
        }
      } else if constexpr (PNL == 5) {
        // Forward elimination with compaction (round 5; QLDPC_OSD_PNL=5, osd_0 / osd_e).  A pivot
        // step costs every wave its search and its row xors (the step is VALU-bound: xoring the
        // pivot row three times instead of once made the lean loop's OSD 47 % slower,
        // profiles/r05/osd_notkept/xor3_*).  Gauss-Jordan xors the pivot row into EVERY row that has
        // the bit; plain forward elimination only into the unused rows, and every 64 pivots the
        // unused rows are packed into the leading waves (words q.. through an LDS staging area), so
        // the trailing waves drop out of the search and the xors: about half of both.  A pivot row
        // is final when chosen; the rows stay in registers (a compaction swaps the <= 64 rows used
        // since the last one out of the leading slots against the unused rows behind them, through
        // a 64-row LDS staging area) and go to the HBM slice once at the end, as row (pivot
        // index) -- a per-pivot global store would hold its wave at every barrier.  The rows' U
        // bits (bit p_k of pivot row i, k > i) are taken as the pivots come (a frozen row's bit
        // at the pivot position) and kept in LDS by blocks of 64 pivots (osd_ul_at).  The
        // Jordan half is done afterwards on the (1 + nh)-bit right-hand sides only (syndrome bit,
        // the nh non-pivot columns Ht): U x = b by blocks of 64 pivots (after step 4 below).  Same
        // pivots (lexicographic minimum of (first bit, ORIGINAL row)), same S0 / x(h_j).
        // MEASURED AND NOT KEPT (opt-in): bit-exact (11 GPU tests incl. non-uniform priors and the
        // circuit graphs), the elimination itself ~15 % shorter (1.21 M vs 1.41 M cycles per n1600
        // syndrome, stamps), but the compactions (46 k) and the back substitution (63 k) take most
        // of that back and the extra per-step bookkeeping the rest: n1600 BP+OSD-E(10) 581 k vs
        // 617 k shots/s (profiles/r05/osd_notkept/fwd_*).  What the halved VALU does not touch is
        // the step's latency chain (two barriers, four LDS round trips), ~1,100 of its ~1,800 cycles.
        static_assert(RPT == 1, "forward elimination: one row per thread");
        int32_t* lkk = reinterpret_cast<int32_t*>(smem);  // pivots: (sbit << 24) | (position << 11) | row
        u64* stgA = reinterpret_cast<u64*>(smem + A.pnl_off);  // [WR][64] words of the rows moving in
        u64* stgB = stgA + (size_t)WR * 64;                     // [WR][64] words of the rows moving out
        uint32_t* siA = reinterpret_cast<uint32_t*>(stgB + (size_t)WR * 64);  // [64] row | sbit << 11 | (pivot + 1) << 12
        uint32_t* siB = siA + 64;
        u64* Ul = reinterpret_cast<u64*>(smem + A.pnl_off + osd_fwd_stg_bytes(WR));  // U words, osd_ul_at
        __shared__ u64 s_bal[LB / 64];
        const uint32_t pivx_a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)(&s_pivx);
        uint32_t step = 0;  // uniform
        const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform
        int rid = tid < m ? tid : 2047;       // original row of the slot
        uint32_t um = used_r[0] ? 0u : ~0u;   // ~0 while the slot holds an unused row
        int pk = -1;                          // pivot index of the slot's row (-1: not a pivot row)
        u64 cu = 0;                           // the row's U bits over the pivots of block fl
        int fl = 0;                           // uniform: U blocks flushed
        int nact = ((m < TB ? m : TB) + 63) >> 6;  // uniform: waves that may hold unused rows
        int ncomp = 64;                       // uniform: next compaction at npiv == ncomp
        // one compile-time word q per call (a runtime q would index the row registers and put
        // them in scratch; the body is too large for the unroller); false = stop
        auto fwd_word = [&](auto qc) __attribute__((always_inline)) -> bool {
          constexpr int q = decltype(qc)::value;
          if (q * 64 >= n || npiv >= rank) return false;  // uniform
          const int bend = n - q * 64 < 64 ? n - q * 64 : 64;
          const u64 wmask = bend < 64 ? (1ull << bend) - 1ull : ~0ull;
          int b = 0;
          for (;;) {  // uniform
            if (npiv >= ncomp) {  // uniform: permute the slots, unused rows first (stable)
              const unsigned long long tc0 = QLDPC_STAMPS ? osd_stamp() : 0ull;
              ncomp += 64;
              if (pk >= 0) Ul[osd_ul_at(pk, fl, RW)] = cu;  // block fl of the U bits is complete
              cu = 0;
              ++fl;
              const bool u = um != 0u;
              const unsigned long long bal = __ballot(u);
              if ((tid & 63) == 0) s_bal[wv] = bal;
              __syncthreads();
              // lane l reads wave l's ballot (one LDS round trip); sums by readlane (SALU adds)
              const int ln = tid & 63;
              const unsigned long long bl = ln < (TB >> 6) ? s_bal[ln] : 0ull;
              const int cl = (int)__popcll(bl);
              int base = 0, tot = 0;  // unused rows in slots before this wave's / in all
#pragma unroll
              for (int w2 = 0; w2 < LB / 64; ++w2) {
                const int cw = __builtin_amdgcn_readlane(cl, w2);
                base += w2 < wv ? cw : 0;
                tot += cw;
              }
              const int tw = tot >> 6;
              const int ul = ln < tw ? cl : (ln == tw ? (int)__popcll(bl & ((1ull << (tot & 63)) - 1ull)) : 0);
              int Ut = 0;  // unused rows in slots < tot (uniform)
#pragma unroll
              for (int w2 = 0; w2 < LB / 64; ++w2) Ut += __builtin_amdgcn_readlane(ul, w2);
              const int Us = base + (int)__popcll(bal & ((1ull << (tid & 63)) - 1ull));
              // holes: used rows in slots < tot; movers: unused rows in slots >= tot (as many)
              const bool hole = !u && tid < tot, mover = u && tid >= tot;
              const int hi = hole ? tid - Us : Us - Ut;
              if (hole || mover) {
                u64* dp = hole ? stgB : stgA;
#pragma unroll
                for (int q2 = 0; q2 < WR; ++q2) dp[(size_t)q2 * 64 + hi] = row[0][q2];
                (hole ? siB : siA)[hi] = (uint32_t)rid | (sbit[0] << 11) | ((uint32_t)(pk + 1) << 12);
              }
              __syncthreads();  // (the staging is next written 64 pivots = 128 barriers later)
              if (hole || mover) {
                const u64* sp = hole ? stgA : stgB;
#pragma unroll
                for (int q2 = 0; q2 < WR; ++q2) row[0][q2] = sp[(size_t)q2 * 64 + hi];
                const uint32_t v = (hole ? siA : siB)[hi];
                rid = (int)(v & 2047u);
                sbit[0] = (v >> 11) & 1u;
                pk = (int)(v >> 12) - 1;
                um = hole ? ~0u : 0u;
              }
              nact = __builtin_amdgcn_readfirstlane((tot + 63) >> 6);
              if (QLDPC_STAMPS) st[15] += osd_stamp() - tc0;
            }
            ++step;
            if (QLDPC_STAMPS) st[7] += 1;
            if (wv < nact) {  // uniform per wave
              const u64 lowm = (~0ull << b) & wmask;
              const uint32_t ml = (uint32_t)row[0][q] & (uint32_t)lowm & um;
              const uint32_t mh = (uint32_t)(row[0][q] >> 32) & (uint32_t)(lowm >> 32) & um;
              const uint32_t fl = ffbl_u32(ml), fh = ffbl_u32(mh) | 32u;
              const uint32_t f = fl < fh ? fl : fh;
              const uint32_t key = wave_min_u32_bc((f << 11) | (uint32_t)rid);
              if ((tid & 63) == 0 && key <= 0x1FFFFu) lds_max_u32_sync(pivx_a, (step << 17) | (0x1FFFFu - key));
            }
            __syncthreads();
            const uint32_t vx = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_pivx);  // uniform
            if ((vx >> 17) != step) break;  // no pivot left in this word (uniform)
            const uint32_t kk = 0x1FFFFu - (vx & 0x1FFFFu);
            const int fb = (int)(kk >> 11), r = (int)(kk & 2047u);
            const bool hbit = ((row[0][q] >> fb) & 1ull) != 0;
            const bool upd = um != 0u && hbit && rid != r;
            if (pk >= 0 && hbit) cu |= 1ull << (npiv & 63);  // a frozen pivot row: U bit
            if (um != 0u && rid == r) {  // the pivot's owner: publish and record
              um = 0u;
              pk = npiv;
#pragma unroll
              for (int q2 = q; q2 < WR; ++q2) pbuf[q2] = row[0][q2];
              pbuf[WR] = sbit[0];
              lkk[npiv] = (int)((sbit[0] << 24) | ((uint32_t)(q * 64 + fb) << 11) | (uint32_t)r);
            }
            ++npiv;
            __syncthreads();
            if (upd) {  // pivot-row words through the rolling buffer, as the lean loop
              constexpr int XB = kOsdXB;
              u64 buf[XB];
#pragma unroll
              for (int u2 = 0; u2 < XB; ++u2)
                if (q + u2 < WR) buf[u2] = pbuf[q + u2];
              const uint32_t ps = (uint32_t)pbuf[WR];
#pragma unroll
              for (int q2 = q; q2 < WR; ++q2) {
                const u64 pv = buf[(q2 - q) % XB];
                if (q2 + XB < WR) buf[(q2 - q) % XB] = pbuf[q2 + XB];
                row[0][q2] ^= pv;
              }
              sbit[0] ^= ps;
            }
            b = fb + 1;
            if (b >= bend || npiv >= rank) break;  // uniform
          }
          return true;
        };
        osd_for_words(std::make_integer_sequence<int, WR>{}, fwd_word);
        if (pk >= 0 && npiv > fl * 64) Ul[osd_ul_at(pk, fl, RW)] = cu;  // the last block's U bits
        if (pk >= 0) {  // the pivot rows -> the HBM slice, row = pivot index
          u64* mrow = Mg + pk;
          asm volatile("" : "+v"(mrow));
#pragma unroll
          for (int q2 = 0; q2 < WR; ++q2)
            if (q2 < W) mrow[(size_t)q2 * m] = row[0][q2];
        }
        // the pivot list -> pivrow / pivpos (every lkk write precedes one of the loop's barriers)
        for (int i = tid; i < npiv; i += TB) {
          const int v = lkk[i];
          pivrow[i] = v & 2047;
          pivpos[i] = (v >> 11) & 0x1FFF;
        }
      } else if constexpr (PNL == 4) {
        // Lagged one-barrier loop (round 5; QLDPC_OSD_PNL=4).  The lean loop below walks two
        // barriers and four dependent LDS round trips per pivot (search max, barrier, winner read,
        // publication, barrier, pivot-row reads).  Here only the pivot WORD q is applied at once:
        // before the search barrier every wave's best candidate row also leaves its word q in a
        // per-wave slot, so after the barrier each row reads the winner and the winning wave's
        // slot and updates its word q -- the next search reads nothing else.  The pivot's other
        // words (and syndrome bit) are published by its owner after that barrier and applied one
        // step later, after the next barrier (the owner of the next pivot applies them before it
        // publishes its own row); at a word's end, and when the rank is reached, one extra barrier
        // flushes the pending row.  Same pivots and the same reduced rows as the lean loop; one
        // barrier per pivot.  Slots, winner words and pivot-row buffers are double-buffered by
        // step / pivot parity: a buffer is rewritten two barriers after it was read.
        // MEASURED AND NOT KEPT (opt-in): bit-exact (10 GPU tests incl. non-uniform priors and
        // circuit graphs), but n1600 BP+OSD-E(10) 578 k vs 616 k shots/s with the lean loop
        // (profiles/r05/osd_notkept/lag_*): the pending row xor and the slot round trip stay on
        // every wave's path between two barriers, so halving the barriers shortens nothing.
        static_assert(RPT == 1, "lagged loop: one row per thread");
        __shared__ uint32_t s_pv[2];        // per step parity: (step << 17) | (0x1FFFF - key), max over waves
        __shared__ u64 s_slot[2][LB / 64];  // per step parity and wave: word q of the wave's best row
        int32_t* lkk = reinterpret_cast<int32_t*>(smem);  // pivots over the dead sort keys, as the lean loop
        const uint32_t pv_a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)(&s_pv[0]);
        if (tid < 2) s_pv[tid] = 0u;
        __syncthreads();
        uint32_t step = 0;  // uniform
        uint32_t um = used_r[0] ? 0u : ~0u;
        const int wv = tid >> 6;
        bool pend = false;  // uniform: a pivot row waits in pbuf half pp
        int pp = 0;
        bool phb = false;   // this row takes the pending pivot row (it had the pivot bit, not its owner)
#pragma unroll
        for (int q = 0; q < WR; ++q) {
          if (q * 64 >= n || npiv >= rank) break;  // uniform
          const int bend = n - q * 64 < 64 ? n - q * 64 : 64;
          const u64 wmask = bend < 64 ? (1ull << bend) - 1ull : ~0ull;
          // the pending pivot row's words q+1.. and syndrome bit (published before the last barrier)
          auto apply_pending = [&]() __attribute__((always_inline)) {
            if (pend) {  // uniform
              const u64* pr = pbuf + (size_t)pp * (WR + 1);
              if (phb) {
                constexpr int XB = kOsdXB;
                u64 buf[XB];
#pragma unroll
                for (int u = 0; u < XB; ++u)
                  if (q + 1 + u < WR) buf[u] = pr[q + 1 + u];
                const uint32_t ps = (uint32_t)pr[WR];
#pragma unroll
                for (int q2 = q + 1; q2 < WR; ++q2) {
                  const u64 pv = buf[(q2 - q - 1) % XB];
                  if (q2 + XB < WR) buf[(q2 - q - 1) % XB] = pr[q2 + XB];
                  row[0][q2] ^= pv;
                }
                sbit[0] ^= ps;
              }
              pend = false;
            }
          };
          int b = 0;
          for (;;) {  // uniform
            ++step;
            asm volatile("" : "+s"(step));
            const int par = (int)(step & 1u);
            if (QLDPC_STAMPS) st[7] += 1;
            const u64 lowm = (~0ull << b) & wmask;
            const uint32_t ml = (uint32_t)row[0][q] & (uint32_t)lowm & um;
            const uint32_t mh = (uint32_t)(row[0][q] >> 32) & (uint32_t)(lowm >> 32) & um;
            const uint32_t fl = ffbl_u32(ml), fh = ffbl_u32(mh) | 32u;
            const uint32_t f = fl < fh ? fl : fh;
            const uint32_t key0 = (f << 11) | (uint32_t)tid;
            const uint32_t key = wave_min_u32_bc(key0);
            if (key <= 0x1FFFFu) {  // uniform per wave
              if (key0 == key) s_slot[par][wv] = row[0][q];
              if ((tid & 63) == 0) lds_max_u32_sync(pv_a + 4u * (uint32_t)par, (step << 17) | (0x1FFFFu - key));
            }
            __syncthreads();
            const uint32_t vx = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_pv[par]);  // uniform
            apply_pending();
            if ((vx >> 17) != step) break;  // no pivot left in this word (uniform; nothing pending)
            const uint32_t kk = 0x1FFFFu - (vx & 0x1FFFFu);
            const int fb = (int)(kk >> 11), r = (int)(kk & 2047u);
            const u64 pw = s_slot[par][r >> 6];
            const bool hb = ((row[0][q] >> fb) & 1ull) != 0;
            const bool own = tid == r;
            if (hb && !own) row[0][q] ^= pw;
            if (own) {
              used_r[0] = true;
              um = 0u;
              u64* pr = pbuf + (size_t)(npiv & 1) * (WR + 1);
#pragma unroll
              for (int q2 = q + 1; q2 < WR; ++q2) pr[q2] = row[0][q2];
              pr[WR] = sbit[0];
              lkk[npiv] = ((q * 64 + fb) << 11) | r;
            }
            pend = true;
            pp = npiv & 1;
            phb = hb && !own;
            ++npiv;
            b = fb + 1;
            if (b >= bend || npiv >= rank) {  // uniform: flush the pending row before the next word
              __syncthreads();
              apply_pending();
              break;
            }
          }
        }
        // the pivot list -> pivrow / pivpos (every lkk write precedes one of the loop's barriers)
        for (int i = tid; i < npiv; i += TB) {
          const int v = lkk[i];
          pivrow[i] = v & 2047;
          pivpos[i] = v >> 11;
        }
      } else if constexpr (PNL) {
        static_assert(RPT == 1, "panel mode: one row per thread");
        constexpr int SM = LB / 64;  // row slots per lane of the search wave (rows s * 64 + lane)
        constexpr u64 kLo = 0xFFFFFFFFull, kHi = ~kLo;
        uint32_t* pw = reinterpret_cast<uint32_t*>(smem + A.pnl_off);  // [m] panel half-word of every row
        uint32_t* pmask = pw + m;                                     // [m] combination masks
        u64* prow = reinterpret_cast<u64*>(smem + A.pnl_off + (((size_t)8 * m + 15) & ~(size_t)15));  // [32][WR+1]
        int* pk = reinterpret_cast<int*>(prow + 32 * (WR + 1));       // [32] pivot rows of the panel
        int* pidx = pk + 32;                                          // [m] panel index of a pivot row
        __shared__ int s_P;
        __shared__ uint32_t s_wslot[2][LB / 64][2];  // PNL == 2: per step parity and wave, (half-word, mask)
        int step3p = 0, sparp = 0;                   // PNL == 2: s_piv slot / s_wslot parity of the step
        uint32_t usedm = 0;  // search wave: bit s = row s * 64 + lane is used (rows >= m: always)
        if (tid < 64) {
#pragma unroll
          for (int s2 = 0; s2 < SM; ++s2)
            if (s2 * 64 + tid >= m) usedm |= 1u << s2;
        }
        // panels of 32 columns (half a row word): 32-bit panel words and masks keep the search
        // wave's state at 2 VGPRs per row slot.  Runtime panel index; row words are selected by
        // compile-time index under uniform predicates (never indexed dynamically: they stay in VGPRs).
        for (int qh = 0; qh < 2 * WR; ++qh) {
          const int q = qh >> 1, h = qh & 1;
          if (qh * 32 >= n || npiv >= rank) break;  // uniform
          const int bend = n - qh * 32 < 32 ? n - qh * 32 : 32;
          unsigned long long tp0 = QLDPC_STAMPS ? osd_stamp() : 0ull;
          if constexpr (PNL == 2) {
            // 1-2 (distributed panel, round 4): every thread keeps its own row's panel half-word and
            // combination mask in VGPRs and searches it: per pivot one wave minimum, one LDS atomic
            // and ONE barrier; each wave's best row publishes its (half-word, mask) in the wave's
            // slot of this step's parity before that barrier, so the winner's pair is readable
            // right after it (2 words, not the 25-word row of the per-pivot elimination)
            uint32_t wv = 0, cm = 0;
            if (tid < m) {
              u64 wq = 0;
#pragma unroll
              for (int q2 = 0; q2 < WR; ++q2)
                if (q2 == q) wq = row[0][q2];
              wv = (uint32_t)(h ? wq >> 32 : wq);
            }
            bool usd = used_r[0];  // (rows >= m: used from the start)
            const uint32_t wmask = bend < 32 ? (1u << bend) - 1u : ~0u;
            int P = 0, b = 0;
            while (b < bend && npiv < rank) {  // uniform
              const int slot = step3p;
              step3p = step3p == 2 ? 0 : step3p + 1;
              const int par = sparp;
              sparp ^= 1;
              const uint32_t lowm = (~0u << b) & wmask;
              const uint32_t mm = usd ? 0u : (wv & lowm);
              uint32_t key = mm ? ((uint32_t)(__ffs((int)mm) - 1) << 11) | (uint32_t)tid : 0x7FFFFFFFu;
              key = wave_min_u32(key);
              if (key != 0x7FFFFFFFu && (uint32_t)tid == (key & 2047u)) {
                s_wslot[par][tid >> 6][0] = wv;
                s_wslot[par][tid >> 6][1] = cm;
              }
              if ((tid & 63) == 0 && key != 0x7FFFFFFFu) atomicMin(&s_piv[slot], (int)key);
              __syncthreads();
              const int kk = s_piv[slot];
              if (tid == 0) s_piv[step3p == 2 ? 0 : step3p + 1] = 0x7FFFFFFF;  // re-arm two steps ahead
              if (kk == 0x7FFFFFFF) break;  // no pivot left in this panel (uniform)
              const int fb = kk >> 11, r = kk & 2047;
              const uint32_t pwv = s_wslot[par][r >> 6][0], pmv = s_wslot[par][r >> 6][1];
              if (tid == r) {
                usd = true;
                pivrow[npiv] = r;
                pivpos[npiv] = qh * 32 + fb;
                pk[P] = r;
                pidx[r] = P;
              }
              const bool hb = ((wv >> fb) & 1u) != 0 && tid != r;
              const uint32_t add = pmv | (1u << P);
              wv ^= hb ? pwv : 0u;
              cm ^= hb ? add : 0u;
              ++P;
              ++npiv;
              b = fb + 1;
            }
            used_r[0] = usd;
            if (tid < m) {
              pw[tid] = wv;
              pmask[tid] = cm;
            }
            if (tid == 0) {
              s_P = P;
              s_npiv = npiv;
            }
          } else {
          // 1. every row's panel half-word (up to date: all earlier panels applied)
          if (tid < m) {
            u64 wq = 0;
#pragma unroll
            for (int q2 = 0; q2 < WR; ++q2)
              if (q2 == q) wq = row[0][q2];
            pw[tid] = (uint32_t)(h ? wq >> 32 : wq);
          }
          __syncthreads();
          // 2. the search wave: greedy pivots of this panel, masks and final half-words of every row
          if (tid < 64) {
            uint32_t wv[SM], cm[SM];
#pragma unroll
            for (int s2 = 0; s2 < SM; ++s2) {
              wv[s2] = s2 * 64 + tid < m ? pw[s2 * 64 + tid] : 0u;
              cm[s2] = 0u;
            }
            const uint32_t wmask = bend < 32 ? (1u << bend) - 1u : ~0u;
            int P = 0, b = 0;
            while (b < bend && npiv < rank) {  // uniform
              const uint32_t lowm = (~0u << b) & wmask;
              uint32_t key = 0x7FFFFFFFu;  // (first set bit << 11) | row
#pragma unroll
              for (int s2 = 0; s2 < SM; ++s2) {
                const uint32_t mm = ((usedm >> s2) & 1u) ? 0u : (wv[s2] & lowm);
                const uint32_t kj = mm ? ((uint32_t)(__ffs((int)mm) - 1) << 11) | (uint32_t)(s2 * 64 + tid) : 0x7FFFFFFFu;
                key = kj < key ? kj : key;
              }
              key = wave_min_u32(key);
              if (key == 0x7FFFFFFFu) break;  // no pivot left in this panel (uniform)
              const int fb = (int)(key >> 11), r = (int)(key & 2047u), sr = r >> 6, lr = r & 63;
              uint32_t pwv = 0, pmv = 0;
#pragma unroll
              for (int s2 = 0; s2 < SM; ++s2)
                if (s2 == sr) {  // uniform
                  pwv = wv[s2];
                  pmv = cm[s2];
                }
              pwv = (uint32_t)__builtin_amdgcn_readlane((int)pwv, lr);
              pmv = (uint32_t)__builtin_amdgcn_readlane((int)pmv, lr);
              if (tid == lr) usedm |= 1u << sr;
              if (tid == 0) {
                pivrow[npiv] = r;
                pivpos[npiv] = qh * 32 + fb;
                pk[P] = r;
                pidx[r] = P;
              }
              const uint32_t add = pmv | (1u << P);
#pragma unroll
              for (int s2 = 0; s2 < SM; ++s2) {
                const bool hb = ((wv[s2] >> fb) & 1u) != 0 && s2 * 64 + tid != r;
                wv[s2] ^= hb ? pwv : 0u;
                cm[s2] ^= hb ? add : 0u;
              }
              ++P;
              ++npiv;
              b = fb + 1;
            }
#pragma unroll
            for (int s2 = 0; s2 < SM; ++s2)
              if (s2 * 64 + tid < m) {
                pw[s2 * 64 + tid] = wv[s2];
                pmask[s2 * 64 + tid] = cm[s2];
              }
            if (tid == 0) {
              s_P = P;
              s_npiv = npiv;
            }
          }
          }  // PNL == 1
          __syncthreads();
          const int P = s_P;
          npiv = s_npiv;
          if (QLDPC_STAMPS) {  // [8]: the panel's pivot search, [7]: its pivots
            const unsigned long long t = osd_stamp();
            st[8] += t - tp0;
            st[7] += (unsigned long long)P;
            tp0 = t;
          }
          // 3. the panel's pivot rows publish their panel-start words q.. and syndrome bit
          if (tid < m) {
            const int kx = pidx[tid];
            if (kx >= 0 && kx < P && pk[kx] == tid) {  // (stale entries of earlier panels fail the check)
              u64* dst = prow + kx * (WR + 1);
#pragma unroll
              for (int q2 = 0; q2 < WR; ++q2)
                if (q2 >= q) dst[q2] = row[0][q2];
              dst[WR] = sbit[0];
            }
          }
          __syncthreads();
          // 4. every row: the final panel half-word, then the named pivot rows into everything past
          // the panel (the high half of word q when the panel is its low half, words q+1..)
          if (tid < m) {
            const uint32_t msk = pmask[tid];
            u64 accq = 0;
            for (int kx = 0; kx < P; ++kx) {  // uniform loop: one broadcast read per word
              if constexpr (PNL == 2) {
                // branch-free: every word read (independent broadcast loads the compiler keeps in
                // flight together) and applied under predicates; the conditional form chained a
                // load-wait-xor per word behind uniform branches (the PNL = 1 measurement)
                const bool mine = ((msk >> kx) & 1u) != 0;
                if (!__any(mine)) continue;  // (no row of this wave names pivot kx)
                const u64* src = prow + kx * (WR + 1);
                constexpr int XB = kOsdXB;
                u64 buf[XB];
#pragma unroll
                for (int u = 0; u < XB; ++u)
                  if (u < WR) buf[u] = src[u];
                const uint32_t vs = (uint32_t)src[WR];
                const u64 lowq = (mine && h == 0) ? ~0ull : 0ull;
#pragma unroll
                for (int q2 = 0; q2 < WR; ++q2) {
                  const u64 pv = buf[q2 % XB];
                  if (q2 + XB < WR) buf[q2 % XB] = src[q2 + XB];
                  const u64 sel = (mine && q2 > q) ? ~0ull : 0ull;
                  row[0][q2] ^= pv & sel;
                  if (q2 == q) accq ^= pv & lowq;  // (q uniform: a select, no branch)
                }
                sbit[0] ^= mine ? vs : 0u;
              } else if ((msk >> kx) & 1u) {
                const u64* src = prow + kx * (WR + 1);
#pragma unroll
                for (int q2 = 0; q2 < WR; ++q2) {
                  if (q2 == q && h == 0) accq ^= src[q2];
                  if (q2 > q) row[0][q2] ^= src[q2];
                }
                sbit[0] ^= (uint32_t)src[WR];
              }
            }
            const u64 fw = (u64)pw[tid];
#pragma unroll
            for (int q2 = 0; q2 < WR; ++q2)
              if (q2 == q) row[0][q2] = h ? ((row[0][q2] & kLo) | (fw << 32)) : (((row[0][q2] ^ accq) & kHi) | fw);
          }
          if (QLDPC_STAMPS) st[9] += osd_stamp() - tp0;  // [9]: the panel's row updates
          // (the next panel rewrites pw[tid] / prow only behind its first two barriers)
        }
      } else if constexpr (kOsdM4R && RPT == 1) {
        // Four-Russians groups (round 4): the lean loop's search and winner (same pivots), but a
        // pivot updates only the pivot word q of the rows that have its bit (exact, the next
        // search reads nothing else) and their mask cm over the group's pivots: pivot k's row,
        // as it is when chosen, is its group-start row S_k xor the start rows its own mask names,
        // so absorbing it is cm ^= mask(k) ^ (1 << k).  At the group's end the pivot owners
        // publish their start rows (words q+1.., syndrome bit) as T[1 << k], the workgroup fills
        // T[c] = xor of the S_k, k in c, and every row xors T[cm] into its words q+1.. and its
        // syndrome bit: one LDS read and one xor per word for up to kOsdG pivots.
        int32_t* lkk = reinterpret_cast<int32_t*>(smem);
        const uint32_t pivx_a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)(&s_pivx);
        u64* T = pbuf;                                         // [2^G][WR + 1]
        u64* slot = pbuf + (size_t)(1 << kOsdG) * (WR + 1);   // [G][2]: pivot k's word q, its mask
        uint32_t step = 0;  // uniform
        uint32_t um = used_r[0] ? 0u : ~0u;
        uint32_t cm = 0;    // the group pivots' start rows this row has absorbed
        int gi = -1;        // this row's index among the group's pivots
#pragma unroll
        for (int q = 0; q < WR; ++q) {
          if (q * 64 >= n || npiv >= rank) break;  // uniform
          const int bend = n - q * 64 < 64 ? n - q * 64 : 64;
          const u64 wmask = bend < 64 ? (1ull << bend) - 1ull : ~0ull;
          int b = 0;
          bool more = true;  // uniform
          while (more) {
            int k = 0;  // pivots in this group (uniform)
            for (;;) {  // uniform
              ++step;
              asm volatile("" : "+s"(step));
              if (QLDPC_STAMPS) st[7] += 1;
              const u64 lowm = (~0ull << b) & wmask;
              const uint32_t ml = (uint32_t)row[0][q] & (uint32_t)lowm & um;
              const uint32_t mh = (uint32_t)(row[0][q] >> 32) & (uint32_t)(lowm >> 32) & um;
              const uint32_t fl = ffbl_u32(ml), fh = ffbl_u32(mh) | 32u;
              uint32_t key = ((fl < fh ? fl : fh) << 11) | (uint32_t)tid;
              key = wave_min_u32_bc(key);
              if ((tid & 63) == 0 && key <= 0x1FFFFu) lds_max_u32_sync(pivx_a, (step << 17) | (0x1FFFFu - key));
              __syncthreads();
              const uint32_t vx = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_pivx);  // uniform
              if ((vx >> 17) != step) {  // no pivot left in this word
                more = false;
                break;
              }
              const uint32_t kk = 0x1FFFFu - (vx & 0x1FFFFu);
              const int fb = (int)(kk >> 11), r = (int)(kk & 2047u);
              const bool hb = ((row[0][q] >> fb) & 1ull) != 0;
              if (tid == r) {
                used_r[0] = true;
                um = 0u;
                gi = k;
                slot[2 * k] = row[0][q];
                slot[2 * k + 1] = cm;
                lkk[npiv] = ((q * 64 + fb) << 11) | r;
              }
              ++npiv;
              __syncthreads();
              if (hb && tid != r) {
                row[0][q] ^= slot[2 * k];
                cm ^= (uint32_t)slot[2 * k + 1] ^ (1u << k);
              }
              ++k;
              b = fb + 1;
              if (b >= bend || npiv >= rank) {
                more = false;
                break;
              }
              if (k == kOsdG) break;
            }
            if (k > 0) {  // uniform: the group's end
              if (gi >= 0) {
                u64* d = T + (size_t)(1 << gi) * (WR + 1);
#pragma unroll
                for (int q2 = q + 1; q2 < WR; ++q2) d[q2] = row[0][q2];
                d[WR] = sbit[0];
              }
              __syncthreads();
              const int nw = WR - q;  // words q+1 .. WR-1 and the syndrome entry WR (constant once unrolled)
              for (int t = tid; t < (nw << kOsdG); t += TB) {
                const int c = t / nw, w = q + 1 + t % nw;
                if ((c >> k) == 0 && (c & (c - 1)) != 0) {  // combinations of >= 2 of the k pivots
                  u64 v = 0;
#pragma unroll
                  for (int i = 0; i < kOsdG; ++i)
                    if ((c >> i) & 1) v ^= T[(size_t)(1 << i) * (WR + 1) + w];
                  T[(size_t)c * (WR + 1) + w] = v;
                }
              }
              __syncthreads();
              if (cm) {
                const u64* src = T + (size_t)cm * (WR + 1);
#pragma unroll
                for (int q2 = q + 1; q2 < WR; ++q2) row[0][q2] ^= src[q2];
                sbit[0] ^= (uint32_t)src[WR];
              }
              cm = 0;
              gi = -1;
              // (T and the slots are rewritten only behind the next group's first barriers)
            }
          }
        }
        for (int i = tid; i < npiv; i += TB) {
          const int v = lkk[i];
          pivrow[i] = v & 2047;
          pivpos[i] = v >> 11;
        }
      } else if constexpr (QLDPC_OSD_LEAN && !QLDPC_OSD_1B) {
        // Lean per-pivot loop (round 4): same pivots as the loop below, fewer instructions per
        // wave and step (a pivot step is bound by every wave's own instruction stream: all waves
        // meet at its two barriers; profiles/r04/passo/).  The step's winner is the maximum of
        // (step << 17) | (0x1FFFF - key) over one ds_max per wave: a stale value from an earlier
        // step never matches the step, so the slot needs no re-arming.  Pivots go to an LDS list
        // over the (dead) sort keys: (position << 11) | row.
        int32_t* lkk = reinterpret_cast<int32_t*>(smem);
        const uint32_t pivx_a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)(&s_pivx);
        uint32_t step = 0;  // uniform
        uint32_t um[RPT];   // ~0 while row tid + j * TB is a candidate (unused, < m), else 0
#pragma unroll
        for (int j = 0; j < RPT; ++j) um[j] = used_r[j] ? 0u : ~0u;
#pragma unroll
        for (int q = 0; q < WR; ++q) {
          if (q * 64 >= n || npiv >= rank) break;  // uniform
          const int bend = n - q * 64 < 64 ? n - q * 64 : 64;
          const u64 wmask = bend < 64 ? (1ull << bend) - 1ull : ~0ull;
          int b = 0;
          for (;;) {  // uniform
            ++step;
            asm volatile("" : "+s"(step));  // opaque: no strength-reduced copies of step << 17 per word
            unsigned long long ts0 = 0;
            if (QLDPC_STAMPS) {
              ts0 = osd_stamp();
              st[7] += 1;
            }
            const u64 lowm = (~0ull << b) & wmask;
            // key = (first set bit >= b << 11) | row; a row without one gets first bit 0xFFFFFFFF
            // (v_ffbl of 0), i.e. a key >= 0xFFFFF800, above every real key (<= 0x1FFFF)
            uint32_t key = 0xFFFFFFFFu;
#pragma unroll
            for (int j = 0; j < RPT; ++j) {
              const uint32_t ml = (uint32_t)row[j][q] & (uint32_t)lowm & um[j];
              const uint32_t mh = (uint32_t)(row[j][q] >> 32) & (uint32_t)(lowm >> 32) & um[j];
              const uint32_t fl = ffbl_u32(ml), fh = ffbl_u32(mh) | 32u;
              const uint32_t f = fl < fh ? fl : fh;
              const uint32_t kj = (f << 11) | (uint32_t)(tid + j * TB);
              key = kj < key ? kj : key;
            }
            key = wave_min_u32_bc(key);
            if ((tid & 63) == 0 && key <= 0x1FFFFu) lds_max_u32_sync(pivx_a, (step << 17) | (0x1FFFFu - key));
            __syncthreads();
            if (QLDPC_STAMPS) {
              const unsigned long long t = osd_stamp();
              st[8] += t - ts0;
              ts0 = t;
            }
            const uint32_t vx = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_pivx);  // uniform
            if ((vx >> 17) != step) break;  // no pivot left in this word (uniform)
            const uint32_t kk = 0x1FFFFu - (vx & 0x1FFFFu);
            const int fb = (int)(kk >> 11), r = (int)(kk & 2047u);
            bool hb[RPT];
#pragma unroll
            for (int j = 0; j < RPT; ++j) {
              hb[j] = ((row[j][q] >> fb) & 1ull) != 0;
              if (tid + j * TB == r) {
                used_r[j] = true;
                um[j] = 0u;
#pragma unroll
                for (int q2 = q; q2 < WR; ++q2) pbuf[q2] = row[j][q2];
                pbuf[WR] = sbit[j];
                lkk[npiv] = ((q * 64 + fb) << 11) | r;
              }
            }
            ++npiv;
            __syncthreads();
            if (QLDPC_STAMPS) st[9] += osd_stamp() - ts0;
            bool upd[RPT], any = false;
#pragma unroll
            for (int j = 0; j < RPT; ++j) {
              upd[j] = hb[j] && tid + j * TB != r;
              any = any || upd[j];
            }
            if (any) {  // pivot-row words through the rolling buffer, as below
              constexpr int XB = kOsdXB;
              u64 buf[XB];
#pragma unroll
              for (int u = 0; u < XB; ++u)
                if (q + u < WR) buf[u] = pbuf[q + u];
              const uint32_t ps = (uint32_t)pbuf[WR];
#pragma unroll
              for (int q2 = q; q2 < WR; ++q2) {
                const u64 pv = buf[(q2 - q) % XB];
                if (q2 + XB < WR) buf[(q2 - q) % XB] = pbuf[q2 + XB];
#pragma unroll
                for (int j = 0; j < RPT; ++j) {
                  u64 t = upd[j] ? pv : 0ull;
                  row[j][q2] ^= t;
                  if (QLDPC_OSD_XOR3) {  // diagnostic: the same xor twice more (same result, 3x the work)
                    asm volatile("" : "+v"(t));
                    row[j][q2] ^= t;
                    asm volatile("" : "+v"(t));
                    row[j][q2] ^= t;
                  }
                }
              }
#pragma unroll
              for (int j = 0; j < RPT; ++j) sbit[j] ^= upd[j] ? ps : 0u;
            }
            b = fb + 1;
            if (b >= bend || npiv >= rank) break;  // uniform
          }
        }
        // the pivot list -> pivrow / pivpos (every lkk write precedes one of the loop's barriers)
        for (int i = tid; i < npiv; i += TB) {
          const int v = lkk[i];
          pivrow[i] = v & 2047;
          pivpos[i] = v >> 11;
        }
      } else {
      int step3 = 0;  // search step mod 3: s_piv slot of the step (triple-buffered as above)
      int spar = 0;   // search step mod 2
#pragma unroll
      for (int q = 0; q < WR; ++q) {
        if (q * 64 >= n || npiv >= rank) break;  // uniform
        const int bend = n - q * 64 < 64 ? n - q * 64 : 64;
        // Positions without a candidate row change nothing, so one search step finds the next
        // pivot of this word directly: the lexicographic minimum of (first set bit >= b, row)
        // over the unused rows = the first position with a candidate and its lowest row, as the
        // position-by-position greedy scan picks it (ldpc's pivot set), without a barrier per
        // dependent position.
        const u64 wmask = bend < 64 ? (1ull << bend) - 1ull : ~0ull;
        int b = 0;
        while (b < bend && npiv < rank) {  // uniform
          const int slot = step3;
          step3 = step3 == 2 ? 0 : step3 + 1;
          const int par = spar;  // QLDPC_OSD_1B: slot half of this step (alternates every step)
          spar ^= 1;
          (void)par;
          unsigned long long ts0 = 0;
          if (QLDPC_STAMPS) {
            ts0 = osd_stamp();
            st[7] += 1;
          }
          const u64 lowm = (~0ull << b) & wmask;
          uint32_t key = 0x7FFFFFFFu;  // (first set bit << 11) | row
#pragma unroll
          for (int j = 0; j < RPT; ++j) {
            const u64 mm = used_r[j] ? 0ull : (row[j][q] & lowm);
            const uint32_t kj = mm ? ((uint32_t)(__ffsll((long long)mm) - 1) << 11) | (uint32_t)(tid + j * TB) : 0x7FFFFFFFu;
            key = kj < key ? kj : key;
          }
          key = wave_min_u32(key);
#if QLDPC_OSD_1B
          // one barrier per pivot: the wave's winning row goes to the wave's slot of this step's
          // parity before the barrier (rewritten two steps later, behind the next barrier)
          u64* wsl = pbuf + (size_t)((par * (LB / 64) + (tid >> 6)) * (WR + 1));
          (void)wsl;
#endif
          if (QLDPC_OSD_1B && key != 0x7FFFFFFFu) {
#pragma unroll
            for (int j = 0; j < RPT; ++j)
              if ((uint32_t)(tid + j * TB) == (key & 2047u)) {
#if QLDPC_OSD_1B
#pragma unroll
                for (int q2 = q; q2 < WR; ++q2) wsl[q2] = row[j][q2];
                wsl[WR] = sbit[j];
#endif
              }
          }
          if ((tid & 63) == 0 && key != 0x7FFFFFFFu) atomicMin(&s_piv[slot], (int)key);
          __syncthreads();
          if (QLDPC_STAMPS) {
            const unsigned long long t = osd_stamp();
            st[8] += t - ts0;
            ts0 = t;
          }
          const int kk = s_piv[slot];
          if (tid == 0) s_piv[step3 == 2 ? 0 : step3 + 1] = 0x7FFFFFFF;  // re-arm the slot two steps ahead
          if (kk == 0x7FFFFFFF) break;  // no pivot left in this word (uniform)
          const int fb = kk >> 11, r = kk & 2047;
          const int p = q * 64 + fb;
          bool hb[RPT];
#pragma unroll
          for (int j = 0; j < RPT; ++j) {
            hb[j] = ((row[j][q] >> fb) & 1ull) != 0;
            if (tid + j * TB == r) {
              used_r[j] = true;
              if (!QLDPC_OSD_1B) {
#pragma unroll
                for (int q2 = q; q2 < WR; ++q2) pbuf[q2] = row[j][q2];
                pbuf[WR] = sbit[j];
              }
              pivrow[npiv] = r;
              pivpos[npiv] = p;
            }
          }
          ++npiv;
#if QLDPC_OSD_1B
          const u64* prow = pbuf + (size_t)(par * (LB / 64) + (r >> 6)) * (WR + 1);
#else
          __syncthreads();
          const u64* prow = pbuf;
#endif
          if (QLDPC_STAMPS) st[9] += osd_stamp() - ts0;
          bool upd[RPT], any = false;
#pragma unroll
          for (int j = 0; j < RPT; ++j) {
            upd[j] = hb[j] && tid + j * TB != r;
            any = any || upd[j];
          }
          if (any) {  // one broadcast read of each pivot word serves all of the thread's rows
            // pivot-row words read kOsdXB ahead of their xors (a rolling buffer): written as
            // read-xor pairs, the compiler chained them with a wait after each read (13 LDS round
            // trips per pivot on the 25-word rows, round 4 asm review)
            constexpr int XB = kOsdXB;
            u64 buf[XB];
#pragma unroll
            for (int u = 0; u < XB; ++u)
              if (q + u < WR) buf[u] = prow[q + u];
            const uint32_t ps = (uint32_t)prow[WR];
#pragma unroll
            for (int q2 = q; q2 < WR; ++q2) {
              const u64 pv = buf[(q2 - q) % XB];
              if (q2 + XB < WR) buf[(q2 - q) % XB] = prow[q2 + XB];
#pragma unroll
              for (int j = 0; j < RPT; ++j) row[j][q2] ^= upd[j] ? pv : 0ull;
            }
#pragma unroll
            for (int j = 0; j < RPT; ++j) sbit[j] ^= upd[j] ? ps : 0u;
          }
          b = fb + 1;
        }
      }
      }  // per-pivot elimination
      if ((A.win == 1 || A.win == 3) && (npiv < rank || (A.win == 3 && (b & 1)))) {
        // the pivots run past the column window (uniform): redo at full width
        if (tid == 0) ow[0] = kOsdRedo;
        __syncthreads();
        continue;
      }
      // Steps 4-5 from the registers (osd_e / osd_0, round 5): the reduced rows never leave them.
      // The swap trace runs on one wave with the staged pivot positions read 64 at a time (one LDS
      // round trip per 64 transpositions instead of one per transposition), the needed non-pivot
      // positions Ht[j] go to LDS, and every pivot row writes its bits of S0 / x(h_j) as bytes at
      // its pivot index (no atomics: one writer per index), packed by one ballot per word; the
      // reduced-row write-out to the HBM slice and step 5's two dependent global reads per bit are
      // gone.  MEASURED AND NOT KEPT (A/B build QLDPC_OSD_XREG=1): bit-exact (96 BP+OSD / circuit
      // GPU tests), but the n1600 OSD total is unchanged (1.672 M vs 1.675 M cycles per syndrome,
      // BP+OSD 605 k vs 614 k shots/s, profiles/r05/osd_notkept/xreg_*): the steps' time is not the
      // HBM round trips this removes.
      const int rW = (npiv + 63) / 64;
      if (QLDPC_OSD_XREG && PNL != 5 && nh <= 31 && (size_t)4 * (m + 32) + (size_t)(1 + nh) * npiv <= (size_t)NP * 8) {  // uniform
        if (tid == 0) s_npiv = npiv;
        int32_t* rowpiv = reinterpret_cast<int32_t*>(smem);  // [m] pivot index of each row, -1 (over the dead keys)
        int32_t* swl = rowpiv + m;                          // [32] Ht positions
        uint8_t* xb = reinterpret_cast<uint8_t*>(swl + 32);  // [1 + nh][npiv] bits of S0 / x(h_j) by pivot index
        int32_t* lpp = reinterpret_cast<int32_t*>(smem + A.pbuf_off + (size_t)(osd_prows(LB) + (PNL == 4 ? 1 : 0)) * (WR + 1) * 8);
        __syncthreads();  // pivrow / pivpos written, the (dead) pivot list read
        for (int i = tid; i < npiv; i += TB) lpp[i] = pivpos[i];
        for (int i = tid; i < m; i += TB) rowpiv[i] = -1;
        __syncthreads();
        for (int i = tid; i < npiv; i += TB) rowpiv[pivrow[i]] = i;
        if (tid < 64) {  // wave 0: lane j traces position npiv + j back through the transpositions
          int cur = npiv + tid;
          for (int c0 = ((npiv - 1) >> 6) << 6; c0 >= 0; c0 -= 64) {  // uniform
            const int il = c0 + tid;
            const int v = il < npiv ? lpp[il] : 0;
            const int top = npiv - 1 - c0 < 63 ? npiv - 1 - c0 : 63;
            for (int t = top; t >= 0; --t) {  // uniform
              const int pi = __builtin_amdgcn_readlane(v, t);
              const int i = c0 + t;
              cur = cur == i ? pi : (cur == pi ? i : cur);
            }
          }
          if (tid < nh && npiv + tid < n) {
            swp[npiv + tid] = cur;
            swl[tid] = cur;
          }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < RPT; ++j) {
          const int i = tid + j * TB;
          const int k = i < m ? rowpiv[i] : -1;
          if (k >= 0) {
            xb[k] = (uint8_t)(sbit[j] & 1u);
            for (int jj = 0; jj < nh; ++jj) {  // uniform
              const int hp = swl[jj];
              const int hq = hp >> 6;
              u64 wsel = 0;
              osd_for_words(std::make_integer_sequence<int, WR>{}, [&](auto Qc) __attribute__((always_inline)) {
                constexpr int Q = decltype(Qc)::value;
                if (Q == hq) wsel = row[j][Q];
                return true;
              });
              xb[(size_t)(1 + jj) * npiv + k] = (uint8_t)((wsel >> (hp & 63)) & 1ull);
            }
          }
        }
        __syncthreads();
        for (int t = tid >> 6; t < (1 + nh) * rW; t += TB >> 6) {  // uniform per wave: one ballot per word
          const int jj = t / rW, q = t % rW, i = q * 64 + (tid & 63);
          const unsigned long long v = __ballot(i < npiv && xb[(size_t)jj * npiv + i] != 0);
          if ((tid & 63) == 0) X[(size_t)jj * RW + q] = v;
        }
        xdone = true;
      }
      // reduced rows -> the HBM slice (word-major), syndrome bits -> sb (forward elimination: the
      // pivot rows are there already, in pivot order)
#pragma unroll
      for (int j = 0; j < RPT && PNL != 5 && !xdone; ++j) {
        const int i = tid + j * TB;
        if (i < m) {
          // opaque row pointer: the compiler otherwise hoists the WR word addresses out of the
          // syndrome loop, 2 * WR VGPRs live through the whole elimination (round 4 asm review)
          u64* mrow = Mg + i;
          asm volatile("" : "+v"(mrow));
#pragma unroll
          for (int q = 0; q < WR; ++q)
            if (q < W) mrow[(size_t)q * m] = row[j][q];
        }
        const unsigned long long sbal = __ballot(i < m && sbit[j]);
        if ((tid & 63) == 0) {
          const int w0 = ((tid & ~63) + j * TB) >> 5;
          if (w0 < (m + 31) / 32) sb[w0] = (uint32_t)sbal;
          if (w0 + 1 < (m + 31) / 32) sb[w0 + 1] = (uint32_t)(sbal >> 32);
        }
      }
      if (tid == 0) s_npiv = npiv;
      __syncthreads();
    } else {
    // 2. H with permuted columns, word-major; each thread owns whole rows (LDS mode: the
    // barrier above ended every read of the sort tables this overwrites)
    const int32_t* posr = kMLds ? gpos : pos;
    for (int i = tid; i < m; i += TB) {
      for (int q = 0; q < W; ++q) M[(size_t)q * m + i] = 0;
      for (int e = A.rp[i]; e < A.rp[i + 1]; ++e) {
        const int p = posr[A.ci[e]];
        M[(size_t)(p >> 6) * m + i] ^= 1ull << (p & 63);
      }
    }
    __syncthreads();
    OSD_ST(1)
    // 3. Gauss-Jordan over positions in order (greedy pivots = ldpc's pivot set).
    // Barriers: one per dependent position, two per pivot.  Slot p%3 of s_piv collects
    // column p's pivot row; thread 0 re-arms slot (p+2)%3 after this column's first
    // barrier (its last reader, column p-1, is past that barrier; its next writer,
    // column p+2, is behind column p+1's barrier).  used / pivrow / s_npiv change
    // between the two barriers of a pivot column, while nobody reads them.
    // Memory shape: M sits in an HBM (MALL/L2) slice, so every dependent round trip costs
    // ~1 us.  The search batch-loads column p's word of all the thread's rows at once and
    // keeps which of them have the bit (M does not change until the elimination); the
    // elimination loads the pivot row and the target row by blocks of kBW words, all loads of
    // a block ahead of its stores (in-place xors of one array would otherwise serialize).
    constexpr int kRowsPT = 2048 / LB;  // rows per thread kept in a mask (m <= 2048)
    const bool masked = m <= kRowsPT * TB;
    for (int p = 0; p < n; ++p) {
      if (s_npiv >= rank) break;
      unsigned long long ts0 = 0;
      if (QLDPC_STAMPS) {
        ts0 = osd_stamp();
        st[7] += 1;
      }
      const u64* Mp = M + (size_t)(p >> 6) * m;
      const u64 bit = 1ull << (p & 63);
      const int slot = p % 3;
      uint32_t hasb = 0;  // bit j: row tid + j*TB has column p set (masked mode)
      int cand = 0x7FFFFFFF;
      if (masked) {
        u64 wv[kRowsPT];
#pragma unroll
        for (int j = 0; j < kRowsPT; ++j) {
          const int i = tid + j * TB;
          wv[j] = i < m ? Mp[i] : 0ull;
        }
        // the wave's first candidate row by ballot (rows tid + j*TB are consecutive per wave for
        // each j): one LDS atomic per wave instead of one per candidate lane
        int wcand = 0x7FFFFFFF;
#pragma unroll
        for (int j = 0; j < kRowsPT; ++j) {
          const int i = tid + j * TB;
          const bool hb = (wv[j] & bit) != 0;
          if (hb) hasb |= 1u << j;
          const unsigned long long bal = __ballot(hb && !((used[i >> 5] >> (i & 31)) & 1u));
          if (wcand == 0x7FFFFFFF && bal) wcand = (tid & ~63) + j * TB + (__ffsll((long long)bal) - 1);
        }
        if ((tid & 63) == 0) cand = wcand;
      } else {
        for (int i = tid; i < m; i += TB)
          if (!((used[i >> 5] >> (i & 31)) & 1u) && (Mp[i] & bit)) {
            cand = i;
            break;
          }
      }
      if (cand != 0x7FFFFFFF) atomicMin(&s_piv[slot], cand);
      __syncthreads();
      if (QLDPC_STAMPS) st[8] += osd_stamp() - ts0;
      const int r = s_piv[slot];
      if (tid == 0) s_piv[(p + 2) % 3] = 0x7FFFFFFF;
      if (r == 0x7FFFFFFF) continue;  // dependent position (uniform)
      const uint32_t sr = (sb[r >> 5] >> (r & 31)) & 1u;
      if (tid == 0) {
        used[r >> 5] |= 1u << (r & 31);
        pivrow[s_npiv] = r;
        pivpos[s_npiv] = p;
        s_npiv = s_npiv + 1;
      }
      const u64* Mr = M + r;
      if (masked) {
        // syndrome bits of the updated rows: one ballot per row slot, two LDS xors per wave
#pragma unroll 1
        for (int j = 0; j < kRowsPT; ++j) {
          const int i = tid + j * TB;
          const bool upd = ((hasb >> j) & 1u) != 0 && i != r;
          if (upd) row_xor(M + i, Mr, W, m);
          if (sr) {
            const unsigned long long bal = __ballot(upd);
            const int i0 = (tid & ~63) + j * TB;  // 32-aligned: TB and the wave base are multiples of 64
            if ((tid & 63) == 0 && bal) {
              if ((uint32_t)bal) atomicXor(&sb[i0 >> 5], (uint32_t)bal);
              if ((uint32_t)(bal >> 32)) atomicXor(&sb[(i0 >> 5) + 1], (uint32_t)(bal >> 32));
            }
          }
        }
      } else {
        for (int i = tid; i < m; i += TB) {
          if (i == r || !(Mp[i] & bit)) continue;
          row_xor(M + i, Mr, W, m);
          if (sr) atomicXor(&sb[i >> 5], 1u << (i & 31));
        }
      }
      __syncthreads();
    }
    }
    const int r = s_npiv;
    OSD_ST(2)
    const int RWr = (r + 63) / 64;
    if (!xdone) {  // (register rows, osd_e / osd_0: done from the registers above)
    // 4. Neal's column swaps -> non-pivot order Ht.  Only the non-pivot positions swp[r + j],
    // j < nh, are used: each is the identity traced backwards through the transpositions
    // (i, pivpos[i]), i = r-1 .. 0 -- one thread per needed position, no serial replay.
    // (Register-row mode stages pivpos in LDS first: the trace reads it r times.)
    const int32_t* pp = pivpos;
    if constexpr (kRR) {
      int32_t* lpp = reinterpret_cast<int32_t*>(smem + A.pbuf_off + (size_t)(osd_prows(LB) + (PNL == 4 ? 1 : 0)) * (WR + 1) * 8);
      for (int i = tid; i < r; i += TB) lpp[i] = pivpos[i];
      __syncthreads();
      pp = lpp;
    }
    for (int x = r + tid; x < r + nh && x < n; x += TB) {
      int cur = x;
      for (int i = r - 1; i >= 0; --i) {
        const int pi = pp[i];
        cur = cur == i ? pi : (cur == pi ? i : cur);
      }
      swp[x] = cur;
    }
    __syncthreads();
    // 5. S0 and x(h_j) as bit-vectors over the pivot index: one wave per 64-bit word, lane c
    // forms bit c (pivot q*64 + c) and a ballot packs the word
    if constexpr (kRR && PNL == 5) {
      // 5'. (forward elimination) the Jordan half on the right-hand sides: thread k holds pivot row
      // k (final since it was chosen, HBM slice row k) and b_k = (syndrome bit, bits Ht[j] of the
      // row) as bits 0, 1 + j; U_kj = bit p_j of row k for pivots j > k (upper unitriangular in
      // pivot order, the pivots being found in ascending position; its words were taken during
      // the elimination).  Back substitution U x = b by blocks of 64 pivots from the last: the
      // block's wave solves it lane by lane (readlane of the finished lane's x, xor into the lanes
      // whose U bit names it), publishes x as 1 + nh ballot words, and every earlier row takes
      // parity(U_k,block & x) per right-hand side.
      const int32_t* lk = reinterpret_cast<const int32_t*>(smem);
      const u64* Ul = reinterpret_cast<const u64*>(smem + A.pnl_off + osd_fwd_stg_bytes(WR));
      u64* xv = const_cast<u64*>(Ul) + osd_ul_words(RW);      // [1 + nh][RWr] x as bit-vectors
      uint32_t bk = 0;
      {
        u64 rw[WR];
        const u64* mrow = Mg + tid;
        asm volatile("" : "+v"(mrow));
#pragma unroll
        for (int Q = 0; Q < WR; ++Q) rw[Q] = (tid < r && Q < W) ? mrow[(size_t)Q * m] : 0ull;
        if (tid < r) bk = ((uint32_t)lk[tid] >> 24) & 1u;
        for (int j = 0; j < nh; ++j) {  // uniform
          const int hp = swp[r + j];
          const int hq = hp >> 6;
          u64 wsel = 0;
          osd_for_words(std::make_integer_sequence<int, WR>{}, [&](auto Qc) __attribute__((always_inline)) {
            constexpr int Q = decltype(Qc)::value;
            if (Q == hq) wsel = rw[Q];
            return true;
          });
          bk |= (uint32_t)((wsel >> (hp & 63)) & 1ull) << (1 + j);
        }
      }
      unsigned long long tj0 = QLDPC_STAMPS ? osd_stamp() : 0ull;
      const int B0 = __builtin_amdgcn_readfirstlane(tid >> 6);  // this wave's pivot block (uniform)
      for (int B = RWr - 1; B >= 0; --B) {  // uniform
        if (B0 == B) {
          // U bits name later pivots only (bit t of lane l: t > l), lanes past r hold zeros
          const u64 uo = tid < r ? Ul[osd_ul_at(tid, B, RW)] : 0ull;
          const uint32_t ulo = (uint32_t)uo, uhi = (uint32_t)(uo >> 32);
#pragma unroll
          for (int t = 63; t > 0; --t) {  // lane t is final: x_t (constant lanes, no hazards)
            const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)bk, t);
            const uint32_t bit = ((t < 32 ? ulo : uhi) >> (t & 31)) & 1u;
            bk ^= x & (0u - bit);
          }
#pragma unroll
          for (int j = 0; j < 32; ++j) {
            if (j > nh) break;  // uniform
            const unsigned long long bal = __ballot(tid < r && ((bk >> j) & 1u));
            if ((tid & 63) == 0) xv[(size_t)j * RWr + B] = bal;
          }
        }
        __syncthreads();
        if (B0 < B) {  // uniform per wave; lanes past r: uB = 0
          const u64 uB = tid < r ? Ul[osd_ul_at(tid, B, RW)] : 0ull;
          uint32_t acc = 0;
#pragma unroll
          for (int j = 0; j < 32; ++j) {
            if (j > nh) break;  // uniform
            acc |= (uint32_t)(__popcll(uB & xv[(size_t)j * RWr + B]) & 1) << j;
          }
          bk ^= acc;
        }
      }
      if (QLDPC_STAMPS) st[13] += osd_stamp() - tj0;
      for (int t = tid; t < (1 + nh) * RWr; t += TB) X[(size_t)(t / RWr) * RW + t % RWr] = xv[t];
    } else
    for (int t = tid >> 6; t < (1 + nh) * RWr; t += TB >> 6) {  // uniform per wave
      const int j = t / RWr, q = t % RWr;
      const int c = tid & 63, i = q * 64 + c;
      bool bitv = false;
      if (i < r) {
        const int row = pivrow[i];
        if (j == 0) {
          bitv = ((sb[row >> 5] >> (row & 31)) & 1u) != 0;
        } else {
          const int hp = swp[r + j - 1];
          bitv = ((M[(size_t)(hp >> 6) * m + row] >> (hp & 63)) & 1ull) != 0;
        }
      }
      const unsigned long long v = __ballot(bitv);
      if (c == 0) X[(size_t)j * RW + q] = v;
    }
    }  // !xdone
    if (tid == 0) s_best = ~0ull;
    __syncthreads();
    OSD_ST(3)
    // 6. candidates: lexicographic min of (weight, index)
    long long L = 1;
    if (A.method == 1 && w > 0) L = 1ll << w;
    if (A.method == 2 && w >= 0) L = 1 + (long long)k + (long long)w * (w - 1) / 2;
    if (A.method == 0 || A.order == 0 || k == 0) L = 1;
    // candidate c -> its OSD input t: the bits of c (osd_e, natural binary order), or the weight-1
    // then weight-2 inputs (osd_cs); tj[] = Ht indices
    auto cand_input = [&](long long c, int* tj, unsigned long long& ebits) -> int {
      ebits = 0;
      if (A.method == 1) {
        ebits = (unsigned long long)c;
        return __popcll(ebits);
      }
      if (c >= 1 && c <= k) {
        tj[0] = (int)(c - 1);
        return 1;
      }
      if (c > k) {
        long long rem = c - 1 - k;
        int i = 0;
        while (rem >= w - 1 - i) {
          rem -= w - 1 - i;
          ++i;
        }
        tj[0] = i;
        tj[1] = i + 1 + (int)rem;
        return 2;
      }
      return 0;
    };
    if (A.softw) {
      // 6'. non-uniform priors (qldpc_osd_gpu_create with channel_probs that differ): the soft weight
      // sum_{j: x_j = 1} log(1 / p_j), added in ascending COLUMN order as the host stage's
      // soft_weight (and ldpc) adds it, so the candidates go to column space first: Xc[j] = X[j]
      // with pivot index i moved to its column, one ballot per 64 columns (colpiv: column -> pivot
      // index or -1); a candidate is then Xc[0] ^ (its Xc[1 + t]) | (its Ht columns), and its weight
      // one ascending walk over the set bits.  Winner: the lexicographic minimum of (weight, c), i.e.
      // the first strictly lightest candidate, as the uniform path.
      int32_t* colpiv = gpos + n;            // [n]
      u64* Xc = X + (size_t)(1 + nh) * RW;   // [(1 + nh)][W]
      for (int j = tid; j < n; j += TB) colpiv[j] = -1;
      __syncthreads();
      for (int i = tid; i < r; i += TB) colpiv[sidxr[pivpos[i]]] = i;
      __syncthreads();
      for (int t = tid >> 6; t < (1 + nh) * W; t += TB >> 6) {  // uniform per wave
        const int j = t / W, q = t % W;
        const int col = q * 64 + (tid & 63);
        bool bitv = false;
        if (col < n) {
          const int pi = colpiv[col];
          if (pi >= 0) bitv = ((X[(size_t)j * RW + (pi >> 6)] >> (pi & 63)) & 1ull) != 0;
        }
        const unsigned long long v = __ballot(bitv);
        if ((tid & 63) == 0) Xc[(size_t)j * W + q] = v;
      }
      if (tid == 0) s_bestw = ~0ull;
      __syncthreads();
      double bw = __builtin_huge_val();
      long long bc = -1;
      for (long long c = tid; c < L; c += TB) {
        int tj[2];
        unsigned long long ebits;
        const int nt = cand_input(c, tj, ebits);
        double sw = 0.0;
        for (int q = 0; q < W; ++q) {
          u64 v = Xc[q];
          if (A.method == 1) {
            for (unsigned long long e = ebits; e; e &= e - 1) {
              const int t = __ffsll((long long)e) - 1;
              v ^= Xc[(size_t)(1 + t) * W + q];
              const int hc = sidxr[swp[r + t]];
              if ((hc >> 6) == q) v |= 1ull << (hc & 63);
            }
          } else {
            for (int a = 0; a < nt; ++a) {
              v ^= Xc[(size_t)(1 + tj[a]) * W + q];
              const int hc = sidxr[swp[r + tj[a]]];
              if ((hc >> 6) == q) v |= 1ull << (hc & 63);
            }
          }
          for (; v; v &= v - 1) sw += A.softw[q * 64 + __ffsll((long long)v) - 1];
        }
        if (sw < bw) {  // c ascends per thread: the first of equal weights stays
          bw = sw;
          bc = c;
        }
      }
      // non-negative doubles order as their bit patterns
      const u64 wb = bc >= 0 ? (u64)__double_as_longlong(bw) : ~0ull;
      if (bc >= 0) atomicMin(&s_bestw, wb);
      __syncthreads();
      if (bc >= 0 && wb == s_bestw) atomicMin(&s_best, (u64)bc);
      __syncthreads();
    } else {
    u64 best = ~0ull;
    for (long long c = tid; c < L; c += TB) {
      int tj[2];
      unsigned long long ebits;
      const int nt = cand_input(c, tj, ebits);
      long long cnt = nt;
      for (int q = 0; q < RWr; ++q) {
        u64 v = X[q];
        if (A.method == 1) {
          for (unsigned long long e = ebits; e; e &= e - 1) v ^= X[(size_t)(1 + __ffsll((long long)e) - 1) * RW + q];
        } else {
          for (int a = 0; a < nt; ++a) v ^= X[(size_t)(1 + tj[a]) * RW + q];
        }
        cnt += __popcll(v);
      }
      const u64 key = ((u64)cnt << 40) | (u64)c;
      if (key < best) best = key;
    }
    if (best != ~0ull) atomicMin(&s_best, best);
    __syncthreads();
    }
    OSD_ST(4)
    // 7. outputs
    const long long cw = (long long)(s_best & ((1ull << 40) - 1));
    int tw[2];
    int ntw = 0;
    unsigned long long ewb = 0;
    if (A.method == 1) {
      ewb = (unsigned long long)cw;
    } else if (cw >= 1 && cw <= k) {
      tw[0] = (int)(cw - 1);
      ntw = 1;
    } else if (cw > k) {
      long long rem = cw - 1 - k;
      int i = 0;
      while (rem >= w - 1 - i) {
        rem -= w - 1 - i;
        ++i;
      }
      tw[0] = i;
      tw[1] = i + 1 + (int)rem;
      ntw = 2;
    }
    for (int j = tid; j < n; j += TB) {
      ow[j] = 0;
      if (o0) o0[j] = 0;
    }
    __syncthreads();
    for (int i = tid; i < r; i += TB) {
      const int q = i >> 6, c = i & 63;
      const u64 s0 = (X[q] >> c) & 1ull;
      u64 v = X[q];
      if (A.method == 1) {
        for (unsigned long long e = ewb; e; e &= e - 1) v ^= X[(size_t)(1 + __ffsll((long long)e) - 1) * RW + q];
      } else {
        for (int a = 0; a < ntw; ++a) v ^= X[(size_t)(1 + tw[a]) * RW + q];
      }
      const int col = sidxr[pivpos[i]];
      ow[col] = (uint8_t)((v >> c) & 1ull);
      if (o0) o0[col] = (uint8_t)s0;
    }
    if (tid == 0) {
      if (A.method == 1) {
        for (unsigned long long e = ewb; e; e &= e - 1) ow[sidxr[swp[r + __ffsll((long long)e) - 1]]] = 1;
      } else {
        for (int a = 0; a < ntw; ++a) ow[sidxr[swp[r + tw[a]]]] = 1;
      }
    }
    __syncthreads();
    OSD_ST(5)
    if (QLDPC_STAMPS) st[6] += 1;
  }
#undef OSD_ST
  if (QLDPC_STAMPS && tid == 0)
    for (int k2 = 0; k2 < 16; ++k2) atomicAdd(&g_osd_stamps[k2], st[k2]);
}

#if QLDPC_EXPERIMENTAL

// Two syndromes per workgroup (register-row mode, 768 threads, m <= 768; round 4, VERDICT r03 item
// 5).  The Gauss-Jordan of one syndrome is a chain of ~780 dependent steps (wave minimum, LDS
// atomic, barrier, pivot-row publication, barrier, row update) that leaves the CU mostly idle, and
// an OSD workgroup cannot share its CU with another (768 x 163 VGPRs).  Here every thread holds
// row tid of BOTH syndromes' permuted H (2 x WR words) and each step searches, publishes and
// updates both, so one chain of barriers serves two eliminations.  Per syndrome: its own LDS area
// (sort tables, bit-vectors, pivot-row buffer, staged pivots) at s * A.syn_lds, its own HBM slice
// (blockIdx.x * 2 + s), the same sort / swap trace / candidates / outputs as osd_gpu_kernel, one
// syndrome after the other.  A syndrome that finishes its word (no pivot left, or rank reached)
// idles through the other's remaining steps of that word.  Outputs identical to osd_gpu_kernel.
// MEASURED AND NOT KEPT (experimental builds only): bit-exact (52 BP+OSD / phenl / circuit GPU
// tests), but 2 x 25 row words left too few of the 168 VGPRs (105 spilled): n1600 BP+OSD 539 k
// vs 548 k shots/s with one syndrome per workgroup (profiles/r04/passf/).  Most of the pressure
// was hoisted write-out addresses; with those opaque (1 dword spilled, 57 GPU tests green) it is
// 537.5 k vs 539 k on one box (profiles/r04/passo/): two eliminations per chain of barriers cost
// what two chains cost, i.e. a pivot step is bound by its VALU issue (~3 waves per SIMD x ~90
// VALU x 4 cycles), not by the barrier latency.
template <int WR>
__global__ void __launch_bounds__(768) osd_rr2_kernel(OsdGpuArgs A) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, TB = blockDim.x;
  const int m = A.m, n = A.n, W = A.W, RW = A.RW, NP = A.NP, rank = A.rank;
  const int k = n - rank;
  const int w = A.order < k ? A.order : k;
  const int nh = A.method == 2 ? k : w;
  __shared__ int s_piv[2][3], s_npiv[2];
  __shared__ u64 s_best[2];
  constexpr int XB = kOsdXB;
  for (long long b0 = (long long)blockIdx.x * 2; b0 < A.B; b0 += 2ll * gridDim.x) {
    bool act[2];
    u64 row[2][WR];
    uint32_t sbit[2];
    bool used_r[2];
    // (per-syndrome phases as lambdas on a compile-time s: the row registers are never indexed by
    // a runtime value, which would put them in scratch)
    auto prologue = [&](auto sc) __attribute__((always_inline)) {
      constexpr int s = decltype(sc)::value;
      const long long b = b0 + s;
      act[s] = false;
#pragma unroll
      for (int q = 0; q < WR; ++q) row[s][q] = 0;
      sbit[s] = 0;
      used_r[s] = true;
      if (b >= A.B || (A.shot && A.shot[b] < 0)) return;
      uint8_t* ow = A.outw + b * (long long)n;
      uint8_t* o0 = A.out0 ? A.out0 + b * (long long)n : nullptr;
      if (A.conv && A.conv[b]) {  // BP converged: bposd_decoder returns the BP decoding
        for (int j = tid; j < n; j += TB) {
          const uint8_t v = A.bp_corr[b * (long long)n + j];
          ow[j] = v;
          if (o0) o0[j] = v;
        }
        return;
      }
      act[s] = true;
      unsigned char* L = smem + (size_t)s * A.syn_lds;
      u64* skey = reinterpret_cast<u64*>(L);
      int32_t* sidx = reinterpret_cast<int32_t*>(skey + NP);
      int32_t* pos = sidx + NP;
      uint32_t* used = reinterpret_cast<uint32_t*>(L + A.bits_off);
      uint32_t* sb = used + (m + 31) / 32;
      const double* post = A.post + b * (long long)n;
      const uint8_t* synd = A.synd + b * (long long)m;
      // 1. stable ascending sort of the columns by posterior (bitonic on (key, index))
      for (int q = tid; q < NP; q += TB) {
        skey[q] = q < n ? ord_key(post[q]) : ~0ull;
        sidx[q] = q < n ? q : 0x7FFFFFFF;
      }
      __syncthreads();
      for (int size = 2; size <= NP; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
          for (int q = tid; q < NP / 2; q += TB) {
            const int lo = 2 * q - (q & (stride - 1));
            const int hi = lo + stride;
            const bool up = (lo & size) == 0;
            const u64 ka = skey[lo], kb = skey[hi];
            const int ia = sidx[lo], ib = sidx[hi];
            const bool gt = ka > kb || (ka == kb && ia > ib);
            if (gt == up) {
              skey[lo] = kb; skey[hi] = ka;
              sidx[lo] = ib; sidx[hi] = ia;
            }
          }
          __syncthreads();
        }
      for (int q = tid; q < n; q += TB) pos[sidx[q]] = q;
      for (int q = tid; q < (m + 31) / 32; q += TB) {
        used[q] = 0;
        uint32_t v = 0;
        for (int t = 0; t < 32 && q * 32 + t < m; ++t) v |= (uint32_t)(synd[q * 32 + t] & 1u) << t;
        sb[q] = v;
      }
      if (tid == 0) {
        s_npiv[s] = 0;
        s_piv[s][0] = s_piv[s][1] = s_piv[s][2] = 0x7FFFFFFF;
      }
      __syncthreads();
      // 2. row tid of the permuted H
      const int i = tid;
      used_r[s] = i >= m;
      if (i < m) {
        for (int e = A.rp[i]; e < A.rp[i + 1]; ++e) {
          const int p = pos[A.ci[e]];
          const int pq = p >> 6;
          const u64 bit = 1ull << (p & 63);
#pragma unroll
          for (int q = 0; q < WR; ++q) row[s][q] ^= (pq == q) ? bit : 0ull;
        }
        sbit[s] = synd[i] & 1u;
      }
    };
    prologue(std::integral_constant<int, 0>{});
    prologue(std::integral_constant<int, 1>{});
    if (!act[0] && !act[1]) continue;  // uniform
    __syncthreads();
    // 3. joint Gauss-Jordan over positions in order (per syndrome as osd_gpu_kernel's search skip)
    int npiv[2] = {0, 0};
    int step3 = 0;
    // one word q per call, q compile-time (the unroller gives up on this loop nest: the row
    // registers would then be indexed at run time and live in scratch); false = stop
    auto word = [&](auto qc) __attribute__((always_inline)) -> bool {
      constexpr int q = decltype(qc)::value;
      if (q * 64 >= n) return false;  // uniform
      bool dn[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) dn[s] = !act[s] || npiv[s] >= rank;
      if (dn[0] && dn[1]) return false;  // uniform
      const int bend = n - q * 64 < 64 ? n - q * 64 : 64;
      const u64 wmask = bend < 64 ? (1ull << bend) - 1ull : ~0ull;
      int bs[2] = {0, 0};
      while (true) {  // uniform
        const int slot = step3;
        step3 = step3 == 2 ? 0 : step3 + 1;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          if (dn[s]) continue;  // uniform
          const u64 lowm = (~0ull << bs[s]) & wmask;
          const u64 mm = used_r[s] ? 0ull : (row[s][q] & lowm);
          uint32_t key = mm ? ((uint32_t)(__ffsll((long long)mm) - 1) << 11) | (uint32_t)tid : 0x7FFFFFFFu;
          key = wave_min_u32(key);
          if ((tid & 63) == 0 && key != 0x7FFFFFFFu) atomicMin(&s_piv[s][slot], (int)key);
        }
        __syncthreads();
        int kk[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) kk[s] = s_piv[s][slot];
        if (tid == 0) {
          const int nx = step3 == 2 ? 0 : step3 + 1;  // re-arm the slot two steps ahead
          s_piv[0][nx] = 0x7FFFFFFF;
          s_piv[1][nx] = 0x7FFFFFFF;
        }
#pragma unroll
        for (int s = 0; s < 2; ++s)
          if (kk[s] == 0x7FFFFFFF) dn[s] = true;  // no pivot left in this word (uniform)
        if (dn[0] && dn[1]) break;
        bool hb[2];
        int rr[2], fbs[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          hb[s] = false;
          rr[s] = -1;
          fbs[s] = 0;
          if (dn[s]) continue;
          const int fb = kk[s] >> 11, r = kk[s] & 2047;
          fbs[s] = fb;
          rr[s] = r;
          hb[s] = ((row[s][q] >> fb) & 1ull) != 0;
          if (tid == r) {
            used_r[s] = true;
            u64* pbuf = reinterpret_cast<u64*>(smem + (size_t)s * A.syn_lds + A.pbuf_off);
#pragma unroll
            for (int q2 = q; q2 < WR; ++q2) pbuf[q2] = row[s][q2];
            pbuf[WR] = sbit[s];
            int32_t* pivrow = A.iws + ((size_t)blockIdx.x * 2 + s) * A.iws_ints;
            pivrow[npiv[s]] = r;
            pivrow[rank + npiv[s]] = q * 64 + fb;  // pivpos
          }
          ++npiv[s];
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          if (dn[s]) continue;
          if (hb[s] && tid != rr[s]) {  // the pivot row's words q.., read XB ahead of their xors
            const u64* prow = reinterpret_cast<const u64*>(smem + (size_t)s * A.syn_lds + A.pbuf_off);
            u64 buf[XB];
#pragma unroll
            for (int u = 0; u < XB; ++u)
              if (q + u < WR) buf[u] = prow[q + u];
            const uint32_t ps = (uint32_t)prow[WR];
#pragma unroll
            for (int q2 = q; q2 < WR; ++q2) {
              const u64 pv = buf[(q2 - q) % XB];
              if (q2 + XB < WR) buf[(q2 - q) % XB] = prow[q2 + XB];
              row[s][q2] ^= pv;
            }
            sbit[s] ^= ps;
          }
          bs[s] = fbs[s] + 1;
          if (bs[s] >= bend || npiv[s] >= rank) dn[s] = true;
        }
        if (dn[0] && dn[1]) break;
      }
      return true;
    };
    osd_for_words(std::make_integer_sequence<int, WR>{}, word);
    // 4-7 per syndrome: reduced rows -> HBM slice, swaps, bit-vectors, candidates, outputs
    auto finish = [&](auto sc) __attribute__((always_inline)) {
      constexpr int s = decltype(sc)::value;
      if (!act[s]) return;  // uniform
      const long long b = b0 + s;
      unsigned char* L = smem + (size_t)s * A.syn_lds;
      const int32_t* sidx = reinterpret_cast<const int32_t*>(reinterpret_cast<u64*>(L) + NP);
      uint32_t* used = reinterpret_cast<uint32_t*>(L + A.bits_off);
      uint32_t* sb = used + (m + 31) / 32;
      int32_t* lpp = reinterpret_cast<int32_t*>(L + A.pbuf_off + (WR + 1) * 8);
      u64* Mg = A.ws + ((size_t)blockIdx.x * 2 + s) * A.ws_words;
      u64* X = Mg + (size_t)W * m;
      int32_t* pivrow = A.iws + ((size_t)blockIdx.x * 2 + s) * A.iws_ints;
      int32_t* pivpos = pivrow + rank;
      int32_t* swp = pivpos + rank;
      uint8_t* ow = A.outw + b * (long long)n;
      uint8_t* o0 = A.out0 ? A.out0 + b * (long long)n : nullptr;
      {
        const int i = tid;
        if (i < m) {
          // opaque row pointer: the compiler otherwise hoists the WR word addresses out of the
          // syndrome loop (2 * WR VGPRs live through the elimination: 105 VGPRs spilled -> 1 dword)
          u64* mrow = Mg + i;
          asm volatile("" : "+v"(mrow));
#pragma unroll
          for (int q = 0; q < WR; ++q)
            if (q < W) mrow[(size_t)q * m] = row[s][q];
        }
        const unsigned long long sbal = __ballot(i < m && sbit[s]);
        if ((tid & 63) == 0) {
          const int w0 = (tid & ~63) >> 5;
          if (w0 < (m + 31) / 32) sb[w0] = (uint32_t)sbal;
          if (w0 + 1 < (m + 31) / 32) sb[w0 + 1] = (uint32_t)(sbal >> 32);
        }
      }
      __syncthreads();  // pivrow / pivpos (global, written by the pivot owners) and sb visible
      const int r = npiv[s];
      for (int i = tid; i < r; i += TB) lpp[i] = pivpos[i];
      __syncthreads();
      for (int x = r + tid; x < r + nh && x < n; x += TB) {
        int cur = x;
        for (int i = r - 1; i >= 0; --i) {
          const int pi = lpp[i];
          cur = cur == i ? pi : (cur == pi ? i : cur);
        }
        swp[x] = cur;
      }
      __syncthreads();
      const int RWr = (r + 63) / 64;
      for (int t = tid >> 6; t < (1 + nh) * RWr; t += TB >> 6) {  // uniform per wave
        const int j = t / RWr, q = t % RWr;
        const int c = tid & 63, i = q * 64 + c;
        bool bitv = false;
        if (i < r) {
          const int rw = pivrow[i];
          if (j == 0) {
            bitv = ((sb[rw >> 5] >> (rw & 31)) & 1u) != 0;
          } else {
            const int hp = swp[r + j - 1];
            bitv = ((Mg[(size_t)(hp >> 6) * m + rw] >> (hp & 63)) & 1ull) != 0;
          }
        }
        const unsigned long long v = __ballot(bitv);
        if (c == 0) X[(size_t)j * RW + q] = v;
      }
      if (tid == 0) s_best[s] = ~0ull;
      __syncthreads();
      long long Lc = 1;
      if (A.method == 1 && w > 0) Lc = 1ll << w;
      if (A.method == 2 && w >= 0) Lc = 1 + (long long)k + (long long)w * (w - 1) / 2;
      if (A.method == 0 || A.order == 0 || k == 0) Lc = 1;
      u64 best = ~0ull;
      for (long long c = tid; c < Lc; c += TB) {
        int tj[2];
        int nt = 0;
        unsigned long long ebits = 0;
        if (A.method == 1) {
          ebits = (unsigned long long)c;
          nt = __popcll(ebits);
        } else if (c >= 1 && c <= k) {
          tj[0] = (int)(c - 1);
          nt = 1;
        } else if (c > k) {
          long long rem = c - 1 - k;
          int i = 0;
          while (rem >= w - 1 - i) {
            rem -= w - 1 - i;
            ++i;
          }
          tj[0] = i;
          tj[1] = i + 1 + (int)rem;
          nt = 2;
        }
        long long cnt = nt;
        for (int q = 0; q < RWr; ++q) {
          u64 v = X[q];
          if (A.method == 1) {
            for (unsigned long long e = ebits; e; e &= e - 1) v ^= X[(size_t)(1 + __ffsll((long long)e) - 1) * RW + q];
          } else {
            for (int a = 0; a < nt; ++a) v ^= X[(size_t)(1 + tj[a]) * RW + q];
          }
          cnt += __popcll(v);
        }
        const u64 key = ((u64)cnt << 40) | (u64)c;
        if (key < best) best = key;
      }
      if (best != ~0ull) atomicMin(&s_best[s], best);
      __syncthreads();
      const long long cw = (long long)(s_best[s] & ((1ull << 40) - 1));
      int tw[2];
      int ntw = 0;
      unsigned long long ewb = 0;
      if (A.method == 1) {
        ewb = (unsigned long long)cw;
      } else if (cw >= 1 && cw <= k) {
        tw[0] = (int)(cw - 1);
        ntw = 1;
      } else if (cw > k) {
        long long rem = cw - 1 - k;
        int i = 0;
        while (rem >= w - 1 - i) {
          rem -= w - 1 - i;
          ++i;
        }
        tw[0] = i;
        tw[1] = i + 1 + (int)rem;
        ntw = 2;
      }
      for (int j = tid; j < n; j += TB) {
        ow[j] = 0;
        if (o0) o0[j] = 0;
      }
      __syncthreads();
      for (int i = tid; i < r; i += TB) {
        const int q = i >> 6, c = i & 63;
        const u64 s0 = (X[q] >> c) & 1ull;
        u64 v = X[q];
        if (A.method == 1) {
          for (unsigned long long e = ewb; e; e &= e - 1) v ^= X[(size_t)(1 + __ffsll((long long)e) - 1) * RW + q];
        } else {
          for (int a = 0; a < ntw; ++a) v ^= X[(size_t)(1 + tw[a]) * RW + q];
        }
        const int col = sidx[pivpos[i]];
        ow[col] = (uint8_t)((v >> c) & 1ull);
        if (o0) o0[col] = (uint8_t)s0;
      }
      if (tid == 0) {
        if (A.method == 1) {
          for (unsigned long long e = ewb; e; e &= e - 1) ow[sidx[swp[r + __ffsll((long long)e) - 1]]] = 1;
        } else {
          for (int a = 0; a < ntw; ++a) ow[sidx[swp[r + tw[a]]]] = 1;
        }
      }
      __syncthreads();
    };
    finish(std::integral_constant<int, 0>{});
    finish(std::integral_constant<int, 1>{});
  }
}

#endif  // QLDPC_EXPERIMENTAL
}  // namespace

struct qldpc_osd_gpu {
  qldpc_osd host;  // shape, method, order, rank
  int device = 0, grid = 0, W = 0, RW = 0, NP = 0, nh = 0, m_lds = 0, bits_off = 0;
  int wr = 0, pbuf_off = 0;  // register-row mode: compile-time words per row (0 = off), LDS pivot buffer
  int rr_tb = 0;             // register-row mode: threads per workgroup = m rounded up to waves
  int pnl = 0, pnl_off = 0;  // register-row mode: panel elimination (QLDPC_OSD_PNL), its LDS area
  int nsy = 1, syn_lds = 0;  // register-row mode: syndromes per workgroup (osd_rr2_kernel), LDS per syndrome
  int win_wr = 0, win_grid = 0;  // column window (osd_win_kernel): row words held, workgroups
  size_t lds = 0;
  long long ws_words = 0, iws_ints = 0;
  qldpc_rt::DevBuf rp, ci, ws, iws, softw;  // softw: [n] log(1 / p_j) when the priors are not uniform
};

namespace {

// BP+OSD failure re-check of the fused shot loop's candidates (qldpc_mc_set_osd): per
// candidate, the residual r = e ^ x_osd against H (src/Simulators.py:139-160: a syndrome
// mismatch counts as a failure) and the logical operators (column masks, as the MC kernel uses);
// a sector verdict the OSD turned into a success clears that sector's bit of the shot's fail
// flags and takes the shot out of the sector / total failure counters.
__global__ void __launch_bounds__(256) osd_recheck_kernel(const int32_t* rp, const int32_t* ci, int m, int n,
                                                          const unsigned long long* lmask, int kw, const uint8_t* err,
                                                          const uint8_t* outw, const long long* shot, long long ncand,
                                                          int q, int logical_mode, uint8_t* fail,
                                                          unsigned long long* counters) {
  __shared__ uint32_t lsyn[8];
  __shared__ int hbad;
  const int tid = threadIdx.x;
  for (long long b = blockIdx.x; b < ncand; b += gridDim.x) {
    const long long s = shot[b];
    if (s < 0) continue;  // converged at max_iter: the BP verdict stands (uniform)
    if (tid < 8) lsyn[tid] = 0;
    if (tid == 0) hbad = 0;
    __syncthreads();
    const uint8_t* e = err + b * (long long)n;
    const uint8_t* x = outw + b * (long long)n;
    for (int j = tid; j < n; j += blockDim.x)
      if ((e[j] ^ x[j]) & 1u)
        for (int w = 0; w < kw; ++w) {
          const unsigned long long v = lmask[(long long)j * kw + w];
          if ((uint32_t)v) atomicXor(&lsyn[2 * w], (uint32_t)v);
          if ((uint32_t)(v >> 32)) atomicXor(&lsyn[2 * w + 1], (uint32_t)(v >> 32));
        }
    for (int i = tid; i < m; i += blockDim.x) {
      uint32_t par = 0;
      for (int k = rp[i]; k < rp[i + 1]; ++k) par ^= (uint32_t)(e[ci[k]] ^ x[ci[k]]);
      if (par & 1u) hbad = 1;
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t any = (uint32_t)hbad;
      for (int w = 0; w < 8; ++w) any |= lsyn[w];
      if (!any) {
        const uint32_t old = fail[s], nw = old & ~(1u << q);
        fail[s] = (uint8_t)nw;
        atomicAdd(&counters[8 + q], ~0ull);  // sector failures - 1
        auto tot = [&](uint32_t f) { return logical_mode == 0 ? (f & 1u) : logical_mode == 1 ? (f >> 1) & 1u : (f != 0); };
        if (tot(old) && !tot(nw)) atomicAdd(&counters[1], ~0ull);  // failures - 1
      }
    }
    __syncthreads();
  }
}

}  // namespace

namespace {
// register-row kernels: the compile-time row widths (words) built, smallest first
// Rows up to 16 words: 1024-thread workgroups (128 VGPRs); 20-25 words: 768 threads = 3 waves
// per SIMD, 168 VGPRs (m <= 768: hgp_34_n1600's 768 x 1600 exactly; wider rows spill).  One row
// per thread: 2 or 3 rows per thread in 384 / 256 threads (fewer waves reading each broadcast
// pivot word) measured 16 % / 26 % slower on n1600 (the per-pivot chain is latency-bound).
constexpr int kOsdWR[] = {2, 4, 8, 12, 16, 20, 25};
// rows per thread: 1, or 2 for the lean loop / blocked elimination of the 20-25-word rows with
// QLDPC_OSD_RPT=2 (384-thread workgroups, two syndromes per CU, VGPRs pinned to 3 waves per SIMD).
// MEASURED AND NOT KEPT (opt-in): bit-exact (GPU tests), but n1600 BP+OSD 521 k vs 588 k shots/s for
// the blocked elimination (46 VGPRs spilled) and 499 k vs 614 k for the lean loop (spills outside
// the pivot loop only): two half-size syndromes per CU cost more than one full-size
// (profiles/r05/osd_notkept/rpt2_*, lean_rpt2_*)
inline int osd_rpt(int wr, int pnl) {
#if QLDPC_EXPERIMENTAL
  const char* e = std::getenv("QLDPC_OSD_RPT");
  return ((pnl == 3 || pnl == 0) && wr >= 20 && e && std::atoi(e) == 2) ? 2 : 1;
#else
  (void)wr;
  (void)pnl;
  return 1;  // (two rows per thread: experimental builds only)
#endif
}
inline int osd_rr_threads(int wr, int pnl = 0) { return wr <= 16 ? 1024 : 768 / osd_rpt(wr, pnl); }
using OsdKern = void (*)(OsdGpuArgs);
template <int WR, int PNL>
OsdKern osd_rr_wide(int rpt) {
  if constexpr ((PNL == 3 || PNL == 0) && QLDPC_EXPERIMENTAL)  // two rows per thread, 384 threads, two syndromes per CU
    if (rpt == 2) return &osd_gpu_kernel<384, WR, 2, PNL>;
  (void)rpt;
  return &osd_gpu_kernel<768, WR, 1, PNL>;
}
template <int PNL>
OsdKern osd_rr_kernel_t(int wr) {
  switch (wr) {
    case 2: return &osd_gpu_kernel<1024, 2, 1, PNL>;
    case 4: return &osd_gpu_kernel<1024, 4, 1, PNL>;
    case 8: return &osd_gpu_kernel<1024, 8, 1, PNL>;
    case 12: return &osd_gpu_kernel<1024, 12, 1, PNL>;
    case 16: return &osd_gpu_kernel<1024, 16, 1, PNL>;
    case 20: return osd_rr_wide<20, PNL>(osd_rpt(wr, PNL));
    case 25: return osd_rr_wide<25, PNL>(osd_rpt(wr, PNL));
    default: return nullptr;
  }
}
// (the panel / blocked / lagged / forward-elimination modes PNL 1-5 were measured and not kept
// (DESIGN.md §4): compiled into experimental builds only, -DQLDPC_EXPERIMENTAL=1)
OsdKern osd_rr_kernel(int wr, int pnl) {
#if QLDPC_EXPERIMENTAL
  return pnl == 5 ? osd_rr_kernel_t<5>(wr) : pnl == 4 ? osd_rr_kernel_t<4>(wr) : pnl == 3 ? osd_rr_kernel_t<3>(wr) : pnl == 2 ? osd_rr_kernel_t<2>(wr) : pnl ? osd_rr_kernel_t<1>(wr)
                                                                                   : osd_rr_kernel_t<0>(wr);
#else
  return pnl ? nullptr : osd_rr_kernel_t<0>(wr);
#endif
}
// column-window kernels (register rows, m <= 768, no panel modes): the first WR row words only and
// a VGPR budget of 6 waves per SIMD, i.e. two 768-thread workgroups per CU
// (QLDPC_OSD_WPE=3: one workgroup per CU, no VGPR pinning -- A/B)
constexpr int kOsdWinWR[] = {8, 12, 14, 16};
template <int WPE>
OsdKern osd_win_kernel_t(int wr) {
  switch (wr) {
    case 8: return &osd_gpu_kernel<768, 8, 1, 0, WPE>;
    case 12: return &osd_gpu_kernel<768, 12, 1, 0, WPE>;
    case 14: return &osd_gpu_kernel<768, 14, 1, 0, WPE>;
    case 16: return &osd_gpu_kernel<768, 16, 1, 0, WPE>;
    default: return nullptr;
  }
}
OsdKern osd_win_kernel(int wr) {
#if QLDPC_EXPERIMENTAL  // (the column window: measured and not kept, experimental builds only)
  const char* e = std::getenv("QLDPC_OSD_WPE");
  return (e && std::atoi(e) == 3) ? osd_win_kernel_t<3>(wr) : osd_win_kernel_t<6>(wr);
#else
  (void)wr;
  return nullptr;
#endif
}
OsdKern osd_rr2_kernel_of(int wr) {
#if QLDPC_EXPERIMENTAL
  switch (wr) {
    case 20: return &osd_rr2_kernel<20>;
    case 25: return &osd_rr2_kernel<25>;
    default: return nullptr;
  }
#else
  (void)wr;
  return nullptr;
#endif
}
// LDS bytes of the panel area (osd_gpu_kernel PNL): half-words + masks [m] (u32), pivot rows [32][WR+1],
// pk [32], pidx [m]
inline size_t osd_pnl_bytes(int m, int wr) {
  return (((size_t)8 * m + 15) & ~(size_t)15) + (size_t)32 * (wr + 1) * 8 + 128 + (size_t)4 * m;
}
}  // namespace

namespace qldpc_rt {
// BP+OSD stage of the fused shot loop for one sector: GPU OSD on the ncand captured
// candidates, then the failure re-check (osd_recheck_kernel).
int osd_gpu_bposd_stage(qldpc_osd_gpu* osd, const uint8_t* synd, const double* post, const uint8_t* err,
                        const long long* shot, uint8_t* outw, long long ncand, const unsigned long long* lmask, int kw,
                        int q, int logical_mode, uint8_t* fail, unsigned long long* counters, hipStream_t stream) {
  if (ncand <= 0) return 0;
  int rc = osd_gpu_decode_slots(osd, synd, post, nullptr, shot, nullptr, nullptr, outw, ncand, stream);
  if (rc) return rc;
  const int grid = (int)std::min<long long>(ncand, 4096);
  hipLaunchKernelGGL(osd_recheck_kernel, dim3(grid), dim3(256), 0, stream, static_cast<const int32_t*>(osd->rp.p),
                     static_cast<const int32_t*>(osd->ci.p), osd->host.m, osd->host.n, lmask, kw, err, outw, shot,
                     ncand, q, logical_mode, fail, counters);
  QLDPC_HIP(hipGetLastError());
  return 0;
}

// true when the host OSD stage was built on exactly this graph (shape and edges)
bool osd_host_matches(const qldpc_osd* o, const qldpc_graph* g) {
  return o && g && o->m == g->m && o->n == g->n && o->col_rows == g->col_rows;
}

// true when the GPU OSD handle was built on exactly this graph (shape and edges)
bool osd_gpu_matches(const qldpc_osd_gpu* o, const qldpc_graph* g) {
  return o && g && o->host.m == g->m && o->host.n == g->n && o->host.col_rows == g->col_rows;
}
}  // namespace qldpc_rt

extern "C" {

int qldpc_osd_gpu_create(const qldpc_graph* g, const double* channel_probs, int32_t osd_method, int32_t osd_order,
                         qldpc_osd_gpu** out) {
  if (!g || !channel_probs || !out) return set_err(QLDPC_EINVAL, "NULL argument");
  qldpc_osd* O = nullptr;
  int rc = qldpc_osd_create(g->m, g->n, g->row_ptr.data(), g->col_idx.data(), channel_probs, osd_method, osd_order,
                            &O);
  if (rc) return rc;
  rc = qldpc_rt::osd_gpu_from_host(g, O, out);
  qldpc_osd_destroy(O);
  return rc;
}

}  // extern "C"

// The GPU OSD of a host OSD stage built on graph g (same method, order, rank and soft weights
// log(1 / p_j), copied: no re-derivation from probabilities).  qldpc_osd_gpu_create and the circuit
// loop (a host stage handed to qldpc_circ_set_final_osd runs on the GPU) both build through here.
int qldpc_rt::osd_gpu_from_host(const qldpc_graph* g, const qldpc_osd* O, qldpc_osd_gpu** out) {
  if (!g || !O || !out) return set_err(QLDPC_EINVAL, "NULL argument");
  if (!osd_host_matches(O, g)) return set_err(QLDPC_EINVAL, "host OSD stage was built on a different graph");
  const int osd_method = O->method, osd_order = O->order;
  int rc = 0;
  if (g->n > kOsdMaxN || (osd_method == 1 && osd_order > 24))
    return set_err(QLDPC_ENOTSUP, "GPU OSD: n > 8192 or osd_e order > 24");
  auto* G = new qldpc_osd_gpu();
  G->host = *O;
  G->device = g->device;
  const int m = g->m, n = g->n, rank = G->host.rank, k = n - rank;
  const int w = std::min(G->host.order, k);
  G->W = (n + 63) / 64;
  G->RW = std::max(1, (rank + 63) / 64);
  G->NP = 1;
  while (G->NP < n) G->NP <<= 1;
  G->nh = G->host.method == 2 ? k : w;
  // LDS: sort tables (skey, sidx, pos), then the used / syndrome bit-vectors.  The Gauss-Jordan
  // image goes to LDS too when it fits over the sort tables (those are copied to HBM ints before
  // the image is built): every pivot search / row update is then an LDS access instead of a
  // ~1 us HBM round trip.  QLDPC_OSD_LDS=0 keeps the image in the HBM slice.
  const size_t lsort = ((size_t)G->NP * 12 + (size_t)n * 4 + 15) & ~(size_t)15;
  const size_t mbytes = ((size_t)G->W * m * 8 + 15) & ~(size_t)15;
  const size_t lbits = (size_t)((m + 31) / 32) * 8 + 64;
  const char* lds_env = std::getenv("QLDPC_OSD_LDS");
  const bool want_lds = !lds_env || std::atoi(lds_env) != 0;
  // register-row mode (one row per thread of a 1024-thread workgroup, row words in VGPRs) when
  // m <= 1024 and n <= 2048; QLDPC_OSD_RR=0 keeps the LDS / HBM image
  const char* rr_env = std::getenv("QLDPC_OSD_RR");
  const char* pnl_env = std::getenv("QLDPC_OSD_PNL");
  const int want_pnl = (QLDPC_EXPERIMENTAL && pnl_env) ? std::atoi(pnl_env) : 0;  // (PNL 1-5: experimental builds)
  if (!rr_env || std::atoi(rr_env) != 0)
    for (int wr : kOsdWR)
      if (wr >= G->W) {
        const int rpt = osd_rpt(wr, want_pnl == 3 ? 3 : 0);
        if (m <= osd_rr_threads(wr, want_pnl == 3 ? 3 : 0) * rpt) {
          G->wr = wr;
          G->rr_tb = std::max(64, ((m + rpt - 1) / rpt + 63) / 64 * 64);  // RPT rows per thread, no idle waves
        }
        break;
      }
  G->m_lds = (!G->wr && want_lds && std::max(lsort, mbytes) + lbits <= (size_t)160 * 1024 - 256) ? 1 : 0;  // 256: static LDS
  G->bits_off = (int)(G->m_lds ? std::max(lsort, mbytes) : lsort);
  G->pbuf_off = (int)(((size_t)G->bits_off + lbits + 15) & ~(size_t)15);
  // register-row mode: pivot-row buffer (QLDPC_OSD_1B: a slot per wave and step parity), then
  // pivpos staged for the swap trace (rank ints)
  const size_t prows = (size_t)osd_prows(osd_rr_threads(std::max(2, G->wr)));
  G->lds = G->wr ? (size_t)G->pbuf_off + prows * (size_t)(G->wr + 1) * 8 + (size_t)std::max(1, rank) * 4
                 : (size_t)G->bits_off + lbits;
  // panel elimination (register-row mode), opt-in QLDPC_OSD_PNL=1: bit-exact, but the single search
  // wave's per-pivot chain (one wave alone issues a VALU op every 4 cycles) is longer than the two
  // barriers it saves: n1600 OSD-E(10) 6.66 vs 3.08 us per syndrome, BP+OSD 257k vs 490k shots/s
  // (profiles/r03/bposd_pnl/)
  if (G->wr && want_pnl != 0) {
    const int pv = want_pnl;
    G->pnl = pv == 5 ? 5 : pv == 4 ? 4 : pv == 3 ? 3 : pv == 2 ? 2 : 1;  // 2: the distributed panel search (one barrier per pivot); 3: blocked
    if (G->pnl == 5 && (G->host.method == 2 || G->nh > 31)) G->pnl = 0;  // forward elimination: <= 31 Ht columns
    G->pnl_off = (int)((G->lds + 15) & ~(size_t)15);
    if (G->pnl == 0) {
      G->pnl_off = 0;
    } else if (G->pnl == 5) {  // compaction staging, then (aliased) U words, x bit-vectors, word starts
      const size_t tb = (size_t)G->rr_tb, rw = (size_t)G->RW;
      (void)tb;
      G->lds = (size_t)G->pnl_off + osd_fwd_stg_bytes(G->wr) + (size_t)osd_ul_words((int)rw) * 8 +
               (size_t)(1 + G->nh) * rw * 8;
    } else if (G->pnl == 4)  // the lagged loop: a second pivot-row buffer (the pivpos staging moves behind it)
      G->lds += (size_t)(G->wr + 1) * 8;
    else
      G->lds = (size_t)G->pnl_off + (G->pnl == 3 ? osd_blk_bytes(m, G->wr) : osd_pnl_bytes(m, G->wr));
  }
  // two syndromes per workgroup (osd_rr2_kernel, the 768-thread register-row kernels): a second LDS
  // area and HBM slice per workgroup; QLDPC_OSD_NSY=1 keeps one
  const char* nsy_env = QLDPC_EXPERIMENTAL ? std::getenv("QLDPC_OSD_NSY") : nullptr;  // (osd_rr2_kernel: experimental builds)
  if (G->wr >= 20 && !G->pnl && !QLDPC_OSD_1B && G->host.uniform && (nsy_env ? std::atoi(nsy_env) : 1) == 2 && osd_rr2_kernel_of(G->wr)) {
    G->nsy = 2;
    G->syn_lds = (int)((G->lds + 15) & ~(size_t)15);
    G->lds = 2 * (size_t)G->syn_lds;
  }
  // column window (register rows, one syndrome per workgroup, the lean loop): the elimination
  // stops once rank pivots are found, and only the positions < rank + nh are read after it (the
  // pivots and the non-pivot columns Ht[0..nh)), so the rows need only the first words that
  // cover rank + nh + kOsdWinSlack positions; a syndrome whose pivots run past them (more than
  // ~kOsdWinSlack dependent positions before the rank) is redone at full width by a second
  // launch.  Opt-in: QLDPC_OSD_WIN=1 picks the width, =<words> forces one.  MEASURED AND NOT KEPT:
  // bit-exact (64 BP+OSD GPU tests), but on the reference codes the rank is reached only near
  // the END of the reliability order (hgp_34_n1600 at p = 0.04: last pivot at position 1419-1538
  // of 1600, tools/dev/osd_last_pivot.py), so nearly every syndrome overruns a 14-word window and
  // pays twice: 491 k BP+OSD shots/s vs 615 k at full width (profiles/r05/osd_notkept/window_*).
  const char* win_env = QLDPC_EXPERIMENTAL ? std::getenv("QLDPC_OSD_WIN") : nullptr;  // (experimental builds)
  const int win_force = win_env ? std::atoi(win_env) : 0;
  if (G->wr && !G->pnl && G->nsy == 1 && m <= 768 && win_force > 0 && QLDPC_OSD_LEAN && !kOsdM4R && !QLDPC_OSD_1B) {
    const long long need = (long long)rank + G->nh;
    for (int ww : kOsdWinWR) {
      const bool fits = win_force > 1 ? ww == win_force && (long long)ww * 64 >= need
                                      : (long long)ww * 64 >= need + kOsdWinSlack;
      if (fits) {
        if (ww < G->wr) G->win_wr = ww;
        break;
      }
    }
  }
  // non-uniform priors: the candidates' column-space vectors Xc [(1 + nh)][W] after X, and the
  // column -> pivot map [n] after the sort maps
  G->ws_words = (long long)G->W * m + (long long)(1 + G->nh) * G->RW +
                (G->host.uniform ? 0ll : (long long)(1 + G->nh) * G->W);
  G->iws_ints = 2ll * rank + 4ll * n;
  auto fail = [&](int code) {
    G->rp.release(); G->ci.release(); G->ws.release(); G->iws.release(); G->softw.release();
    delete G;
    return code;
  };
  if (hipSetDevice(g->device) != hipSuccess) return fail(set_err(QLDPC_EHIP, "hipSetDevice"));
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, g->device) != hipSuccess || cus <= 0)
    return fail(set_err(QLDPC_EHIP, "device CU count"));
  int nb = 0;
  const void* kf = G->nsy == 2 ? reinterpret_cast<const void*>(osd_rr2_kernel_of(G->wr))
                  : G->wr ? reinterpret_cast<const void*>(osd_rr_kernel(G->wr, G->pnl))
                  : G->m_lds ? reinterpret_cast<const void*>(&osd_gpu_kernel<kOsdThreadsLds>)
                             : reinterpret_cast<const void*>(&osd_gpu_kernel<kOsdThreads>);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kf,
                                                   G->wr ? G->rr_tb : G->m_lds ? kOsdThreadsLds : kOsdThreads,
                                                   G->lds) != hipSuccess || nb <= 0)
    nb = 1;
  G->grid = cus * nb;
  if (G->win_wr) {
    int nbw = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nbw, reinterpret_cast<const void*>(osd_win_kernel(G->win_wr)),
                                                     G->rr_tb, G->lds) != hipSuccess || nbw <= 0)
      nbw = 1;
    G->win_grid = cus * nbw;
  }
  const int slices = std::max(G->grid, G->win_grid);
  const size_t E = g->col_idx.size();
  if ((rc = G->rp.alloc((size_t)(m + 1) * 4)) || (rc = G->ci.alloc(std::max<size_t>(E, 1) * 4)) ||
      (rc = G->ws.alloc((size_t)slices * G->nsy * G->ws_words * 8)) ||
      (rc = G->iws.alloc((size_t)slices * G->nsy * G->iws_ints * 4)) ||
      (!G->host.uniform && (rc = G->softw.alloc((size_t)n * 8))))
    return fail(rc);
  if (!G->host.uniform && hipMemcpy(G->softw.p, G->host.w.data(), (size_t)n * 8, hipMemcpyHostToDevice) != hipSuccess)
    return fail(set_err(QLDPC_EHIP, "upload OSD soft weights"));
  if (hipMemcpy(G->rp.p, g->row_ptr.data(), (size_t)(m + 1) * 4, hipMemcpyHostToDevice) != hipSuccess ||
      (E && hipMemcpy(G->ci.p, g->col_idx.data(), E * 4, hipMemcpyHostToDevice) != hipSuccess))
    return fail(set_err(QLDPC_EHIP, "upload OSD graph"));
  *out = G;
  return 0;
}

extern "C" {

int qldpc_osd_gpu_geometry(const qldpc_osd_gpu* osd, int32_t* row_words, int32_t* window_words, int32_t* threads,
                           int32_t* workgroups) {
  if (!osd || !row_words || !window_words || !threads || !workgroups) return set_err(QLDPC_EINVAL, "NULL argument");
  *row_words = osd->wr;
  *window_words = osd->win_wr;
  *threads = osd->wr ? osd->rr_tb : osd->m_lds ? kOsdThreadsLds : kOsdThreads;
  *workgroups = osd->win_wr ? osd->win_grid : osd->grid;
  return 0;
}

int qldpc_osd_gpu_destroy(qldpc_osd_gpu* osd) {
  if (!osd) return 0;
  osd->rp.release(); osd->ci.release(); osd->ws.release(); osd->iws.release(); osd->softw.release();
  delete osd;
  return 0;
}

#if QLDPC_STAMPS
// diagnostic builds only: read and clear osd_gpu_kernel's step-cycle sums
int qldpc_debug_osd_stamps(unsigned long long* out) {
  unsigned long long z[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  if (hipDeviceSynchronize() != hipSuccess || hipMemcpyFromSymbol(out, HIP_SYMBOL(g_osd_stamps), 128) != hipSuccess)
    return -1;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_osd_stamps), z, 128) == hipSuccess ? 0 : -1;
}
#endif

}  // extern "C"

namespace qldpc_rt {
// qldpc_osd_gpu_decode with the fused loop's capture-slot shot indices (slots < 0 are skipped)
int osd_gpu_decode_slots(qldpc_osd_gpu* osd, const uint8_t* d_synd, const double* d_post, const uint8_t* d_conv,
                         const long long* d_shot, const uint8_t* d_bp_corr, uint8_t* d_out0, uint8_t* d_outw,
                         int64_t B, void* stream) {
  if (!osd || (B > 0 && (!d_synd || !d_post || !d_outw))) return set_err(QLDPC_EINVAL, "NULL argument");
  if (d_conv && !d_bp_corr) return set_err(QLDPC_EINVAL, "conv needs bp_corr");
  if (B <= 0) return 0;
  QLDPC_HIP(hipSetDevice(osd->device));
  OsdGpuArgs a;
  a.rp = static_cast<const int32_t*>(osd->rp.p);
  a.ci = static_cast<const int32_t*>(osd->ci.p);
  a.synd = d_synd; a.post = d_post; a.conv = d_conv; a.shot = d_shot; a.bp_corr = d_bp_corr; a.out0 = d_out0;
  a.softw = osd->host.uniform ? nullptr : static_cast<const double*>(osd->softw.p);
  a.outw = d_outw;
  a.ws = static_cast<u64*>(osd->ws.p);
  a.iws = static_cast<int32_t*>(osd->iws.p);
  a.B = B;
  a.m = osd->host.m; a.n = osd->host.n; a.W = osd->W; a.RW = osd->RW; a.rank = osd->host.rank;
  a.method = osd->host.method; a.order = osd->host.order; a.NP = osd->NP; a.m_lds = osd->m_lds; a.bits_off = osd->bits_off;
  a.pbuf_off = osd->pbuf_off;
  a.pnl_off = osd->pnl_off;
  a.syn_lds = osd->syn_lds;
  a.ws_words = osd->ws_words; a.iws_ints = osd->iws_ints;
  a.win = 0;
  const int grid = (int)std::min<long long>((B + osd->nsy - 1) / osd->nsy, osd->grid);
  if (osd->win_wr) {  // the column window, then the full-width redo of its overruns
    const char* tr = std::getenv("QLDPC_OSD_WIN_REDO");
    a.win = (tr && std::atoi(tr) == 1) ? 3 : 1;
    hipLaunchKernelGGL(osd_win_kernel(osd->win_wr), dim3((int)std::min<long long>(B, osd->win_grid)), dim3(osd->rr_tb),
                       osd->lds, (hipStream_t)stream, a);
    QLDPC_HIP(hipGetLastError());
    a.win = 2;
    hipLaunchKernelGGL(osd_rr_kernel(osd->wr, 0), dim3(grid), dim3(osd->rr_tb), osd->lds, (hipStream_t)stream, a);
  } else if (osd->nsy == 2)
    hipLaunchKernelGGL(osd_rr2_kernel_of(osd->wr), dim3(grid), dim3(osd->rr_tb), osd->lds, (hipStream_t)stream, a);
  else if (osd->wr)
    hipLaunchKernelGGL(osd_rr_kernel(osd->wr, osd->pnl), dim3(grid), dim3(osd->rr_tb), osd->lds, (hipStream_t)stream, a);
  else if (osd->m_lds)
    hipLaunchKernelGGL(osd_gpu_kernel<kOsdThreadsLds>, dim3(grid), dim3(kOsdThreadsLds), osd->lds, (hipStream_t)stream, a);
  else
    hipLaunchKernelGGL(osd_gpu_kernel<kOsdThreads>, dim3(grid), dim3(kOsdThreads), osd->lds, (hipStream_t)stream, a);
  QLDPC_HIP(hipGetLastError());
  return 0;
}
}  // namespace qldpc_rt

extern "C" {
int qldpc_osd_gpu_decode(qldpc_osd_gpu* osd, const uint8_t* d_synd, const double* d_post, const uint8_t* d_conv,
                         const uint8_t* d_bp_corr, uint8_t* d_out0, uint8_t* d_outw, int64_t B, void* stream) {
  return qldpc_rt::osd_gpu_decode_slots(osd, d_synd, d_post, d_conv, nullptr, d_bp_corr, d_out0, d_outw, B, stream);
}

}  // extern "C"
