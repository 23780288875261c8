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
#include <vector>

#include "runtime.h"

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
