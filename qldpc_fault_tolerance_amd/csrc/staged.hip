// staged.hip — bit-sliced staged pipelines around the batched BP engine:
//   (1) the phenomenological space-time shot loop (qldpc_phenl_*), and
//   (2) the staged data-error shot loop behind qldpc_mc_launch for decoders the
//       fused kernels do not serve (product-sum, engine 5) or when
//       QLDPC_MC_STAGED=1 asks for it (A/B against the fused min-sum kernels).
//
// (1) in detail:
// Replaces CodeSimulator_Phenon_SpaceTime._single_run / WordErrorRate
// (src/Simulators_SpaceTime.py:421-548) for a batch of samples at once.  One
// sample = (num_rounds - 1) noisy rounds of num_rep repetitions, each
// repetition adding a fresh depolarizing data error and fresh syndrome flips,
// the space-time BP decode of the round's detector history (ST_BP_Decoder_
// syndrome, src/Decoders_SpaceTime.py:200-223), then one perfect round decoded
// by the single-shot BP and the failure check of :500-529.
//
// Error state is BIT-SLICED: word w of row j holds qubit (or check) j of the 64
// samples 64w..64w+63, so
//   * sampling is one thread per (position, sample) whose wave ballots its 64
//     decisions into one word (ph_sample);
//   * H·e mod 2 is, per check row, an XOR of the row's column words: 64
//     syndromes per 8-byte load (ph_syndrome), likewise H·r and L·r (ph_check);
//   * detector histories and corrections cross to / from the BP engine's
//     per-sample byte layout in tiles that keep both sides coalesced
//     (ph_unpack, ph_fold).
// Uniforms: position p of repetition j of round r of sample s draws
// u = Philox4x32-10(key = seed, ctr = ((r·num_rep + j)·P + p, s_lo, s_hi,
// kStreamPhen)) with P = n + m_x + m_z, in the reference's draw order
// (n data qubits, then the hx-row syndrome flips of the Z sector, then the
// hz-row flips of the X sector, src/Simulators_SpaceTime.py:408-431); the final
// round draws at r = num_rounds - 1, j = 0.  An external [S][n_u] array of
// uniforms replays CPython's random() stream bit for bit.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "bp_kernels.h"
#include "runtime.h"

using namespace qldpc;
using namespace qldpc_rt;

namespace {

constexpr uint32_t kStreamPhen = 0x51D50002u;
constexpr int kTile = 256;  // threads per block of the layout kernels

__device__ inline unsigned long long phen_k53(unsigned long long seed, unsigned long long shot, uint32_t idx,
                                              uint32_t tag) {
  uint32_t w0, w1;
  philox4x32_10(idx, (uint32_t)shot, (uint32_t)(shot >> 32), tag, (uint32_t)seed, (uint32_t)(seed >> 32), w0, w1);
  return ((unsigned long long)(w0 >> 5) << 26) | (unsigned long long)(w1 >> 6);
}

struct SampleArgs {
  unsigned long long* cur[2];   // [n][W] X / Z error words (xor-updated)
  unsigned long long* serr[2];  // [m_q][W] syndrome-flip words (overwritten), NULL in the final round
  const double* uniforms;       // [S][nu] or NULL
  long long nu;                 // uniforms per sample
  long long c0;                 // first sample of this chunk (offset into uniforms / global shot index)
  unsigned long long seed, shot_begin;
  unsigned long long K1, K2, K3, Kq;  // ceil(t * 2^53) thresholds
  double t1, t2, t3, q;
  uint32_t base;                // (r·num_rep + j)·P
  uint32_t tag;                 // Philox counter word 3: kStreamPhen, or kStreamData for the staged MC
  int n, m0, m1, W;
  long long count;              // samples in this chunk
};

// grid: x = ceil(count / 256) sample tiles, y = position (n data, then m1, then m0; only n in the final round)
__global__ void __launch_bounds__(kTile) ph_sample(SampleArgs A) {
  const long long sl = (long long)blockIdx.x * kTile + threadIdx.x;
  const int p = blockIdx.y;
  const bool valid = sl < A.count;
  const long long gs = A.c0 + sl;
  bool bx = false, bz = false;
  if (valid) {
    const uint32_t idx = A.base + (uint32_t)p;
    if (A.uniforms) {
      const double u = A.uniforms[gs * A.nu + idx];
      if (p < A.n) {  // src/Simulators_SpaceTime.py:408-422 three-way split
        const uint32_t cls = (u < A.t1) ? 2u : (A.t1 <= u && u < A.t2) ? 1u : (A.t2 <= u && u < A.t3) ? 3u : 0u;
        bx = cls & 1u;
        bz = cls >> 1;
      } else {
        bx = u < A.q;  // :425-431
      }
    } else {
      const unsigned long long k = phen_k53(A.seed, A.shot_begin + (unsigned long long)gs, idx, A.tag);
      if (p < A.n) {
        const uint32_t cls = (k < A.K1) ? 2u : (k < A.K2) ? 1u : (k < A.K3) ? 3u : 0u;
        bx = cls & 1u;
        bz = cls >> 1;
      } else {
        bx = k < A.Kq;
      }
    }
  }
  const unsigned long long wx = __ballot(bx), wz = __ballot(bz);
  const long long w = sl >> 6;
  if (__lane_id() != 0 || w >= A.W) return;  // a wave past the last sample word writes nothing
  if (p < A.n) {
    if (A.cur[0]) A.cur[0][(long long)p * A.W + w] ^= wx;
    if (A.cur[1]) A.cur[1][(long long)p * A.W + w] ^= wz;
  } else if (p < A.n + A.m1) {  // syndrome flips on the hx rows: Z sector
    if (A.serr[1]) A.serr[1][(long long)(p - A.n) * A.W + w] = wx;
  } else {  // syndrome flips on the hz rows: X sector
    if (A.serr[0]) A.serr[0][(long long)(p - A.n - A.m1) * A.W + w] = wx;
  }
}

// s_i = (H cur)_i ^ serr_i for 64 samples per thread; detector row j·m + i.
// diff: detector = s ^ previous repetition's s (Z sector; the X sector keeps
// raw syndromes, quirk Q3, src/Simulators_SpaceTime.py:472-476).
// grid: x = ceil(W / 256), y = row i
__global__ void __launch_bounds__(kTile) ph_syndrome(const int32_t* __restrict__ rp, const int32_t* __restrict__ ci,
                                                   const unsigned long long* __restrict__ cur,
                                                   const unsigned long long* __restrict__ serr,
                                                   unsigned long long* __restrict__ sprev,
                                                   unsigned long long* __restrict__ D, int W, int row0, int diff) {
  const int w = blockIdx.x * kTile + threadIdx.x;
  if (w >= W) return;
  const int i = blockIdx.y;
  unsigned long long s = serr ? serr[(long long)i * W + w] : 0ull;
  for (int e = rp[i]; e < rp[i + 1]; ++e) s ^= cur[(long long)ci[e] * W + w];
  unsigned long long d = s;
  if (diff > 0) d ^= sprev[(long long)i * W + w];
  if (diff >= 0 && sprev) sprev[(long long)i * W + w] = s;
  D[(long long)(row0 + i) * W + w] = d;
}

// Bit-sliced D [R][W] -> bytes out[s][R] (and optionally trace[s][toff + r]).
// grid: x = ceil(R / 256) row tiles, y = word w.  Per sample the 256 threads
// write 256 consecutive bytes.
__global__ void __launch_bounds__(kTile) ph_unpack(const unsigned long long* __restrict__ D, uint8_t* __restrict__ out,
                                                 uint8_t* __restrict__ trace, long long tstride, long long toff,
                                                 long long c0, int R, int W, long long count) {
  const int r = blockIdx.x * kTile + threadIdx.x;
  const int w = blockIdx.y;
  if (r >= R) return;
  const unsigned long long d = D[(long long)r * W + w];
  const int nb = (int)std::min<long long>(64, count - (long long)w * 64);
  for (int b = 0; b < nb; ++b) {
    const long long s = (long long)w * 64 + b;
    const uint8_t v = (uint8_t)((d >> b) & 1ull);
    out[s * R + r] = v;
    if (trace) trace[(c0 + s) * tstride + toff + r] = v;
  }
}

// cur[j] ^= (Σ_i corr[s][i·stride_rep + j]) mod 2, bit-sliced over s:
// the fold of src/Decoders_SpaceTime.py:218-223 applied as :478-481 (reps = 1,
// stride = n: the final round's residual, :493-495).
// grid: x = ceil(n / 256), y = word w
__global__ void __launch_bounds__(kTile) ph_fold(const uint8_t* __restrict__ corr, unsigned long long* __restrict__ cur,
                                               int n, int W, int reps, int stride_rep, int row_len, long long count) {
  const int j = blockIdx.x * kTile + threadIdx.x;
  const int w = blockIdx.y;
  if (j >= n) return;
  const int nb = (int)std::min<long long>(64, count - (long long)w * 64);
  unsigned long long acc = 0;
  for (int b = 0; b < nb; ++b) {
    const uint8_t* c = corr + ((long long)w * 64 + b) * row_len + j;
    uint32_t x = 0;
    for (int i = 0; i < reps; ++i) x ^= c[(long long)i * stride_rep];
    acc |= (unsigned long long)(x & 1u) << b;
  }
  cur[(long long)j * W + w] ^= acc;
}

// failure words: OR over the rows of [H; L] of (row · r) for 64 samples per thread.
// grid: x = ceil(W / 256), y = row
__global__ void __launch_bounds__(kTile) ph_check(const int32_t* __restrict__ rp, const int32_t* __restrict__ ci,
                                                const unsigned long long* __restrict__ r,
                                                unsigned long long* __restrict__ failw, int W) {
  const int w = blockIdx.x * kTile + threadIdx.x;
  if (w >= W) return;
  const int i = blockIdx.y;
  unsigned long long s = 0;
  for (int e = rp[i]; e < rp[i + 1]; ++e) s ^= r[(long long)ci[e] * W + w];
  if (s) atomicOr(&failw[w], s);
}

// per word: failures by eval_logical_type, per-sample flags, counters.
__global__ void __launch_bounds__(kTile) ph_tally(const unsigned long long* __restrict__ fx,
                                                const unsigned long long* __restrict__ fz,
                                                unsigned long long* __restrict__ cnt, uint8_t* __restrict__ fail_out,
                                                long long c0, int W, long long count, int mode) {
  const int w = blockIdx.x * kTile + threadIdx.x;
  if (w >= W) return;
  const int nb = (int)std::min<long long>(64, count - (long long)w * 64);
  const unsigned long long valid = nb >= 64 ? ~0ull : ((1ull << nb) - 1ull);
  const unsigned long long a = fx ? (fx[w] & valid) : 0ull, b = fz ? (fz[w] & valid) : 0ull;
  const unsigned long long f = mode == 0 ? a : mode == 1 ? b : (a | b);
  atomicAdd(&cnt[kCntShots], (unsigned long long)nb);
  if (f) atomicAdd(&cnt[kCntFail], (unsigned long long)__popcll(f));
  if (a) atomicAdd(&cnt[kCntSecFail + 0], (unsigned long long)__popcll(a));
  if (b) atomicAdd(&cnt[kCntSecFail + 1], (unsigned long long)__popcll(b));
  if (fail_out)
    for (int k = 0; k < nb; ++k)
      fail_out[c0 + (long long)w * 64 + k] = (uint8_t)(((a >> k) & 1ull) | (((b >> k) & 1ull) << 1));
}

// decode statistics of one batched BP call into sector q's counters
__global__ void __launch_bounds__(kTile) ph_iters(const int32_t* __restrict__ iters, const uint8_t* __restrict__ conv,
                                                unsigned long long* __restrict__ cnt, int q, long long count) {
  __shared__ unsigned long long sit, snc;
  if (threadIdx.x == 0) sit = snc = 0;
  __syncthreads();
  const long long s = (long long)blockIdx.x * kTile + threadIdx.x;
  if (s < count) {
    const int it = iters[s];
    atomicAdd(&sit, (unsigned long long)it);
    if (!conv[s]) atomicAdd(&snc, 1ull);
    atomicAdd(&cnt[kCntHist + q * kHistBins + std::min(it, kHistBins - 1)], 1ull);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const long long nb = std::min<long long>(kTile, count - (long long)blockIdx.x * kTile);
    atomicAdd(&cnt[kCntDec + q], (unsigned long long)nb);
    atomicAdd(&cnt[kCntIters + q], sit);
    atomicAdd(&cnt[kCntNonconv + q], snc);
  }
}

// per-sample Pauli classes err[s][j] = x | z << 1 from the bit-sliced error words
// grid: x = ceil(n / 256), y = word w
__global__ void __launch_bounds__(kTile) ph_err_out(const unsigned long long* __restrict__ ex,
                                                  const unsigned long long* __restrict__ ez, uint8_t* __restrict__ err,
                                                  long long c0, int n, int W, long long count) {
  const int j = blockIdx.x * kTile + threadIdx.x;
  const int w = blockIdx.y;
  if (j >= n) return;
  const unsigned long long a = ex[(long long)j * W + w], b = ez[(long long)j * W + w];
  const int nb = (int)std::min<long long>(64, count - (long long)w * 64);
  for (int t = 0; t < nb; ++t)
    err[(c0 + (long long)w * 64 + t) * n + j] = (uint8_t)(((a >> t) & 1ull) | (((b >> t) & 1ull) << 1));
}

unsigned long long ceil53(double t) {
  if (!(t > 0.0)) return 0ull;
  if (t >= 1.0) return 1ull << 53;
  return (unsigned long long)std::ceil(std::ldexp(t, 53));
}

// Space-time check matrix of h (src/Decoders_SpaceTime.py:179-194), CSR with
// ascending columns: row block i = [h | I] on column block i, [0 | I] on block i-1.
void st_csr(const qldpc_graph* h, int reps, std::vector<int32_t>& rp, std::vector<int32_t>& ci) {
  const int m = h->m, n = h->n, w = n + m;
  rp.assign(1, 0);
  ci.clear();
  for (int i = 0; i < reps; ++i)
    for (int r = 0; r < m; ++r) {
      if (i > 0) ci.push_back((i - 1) * w + n + r);
      for (int e = h->row_ptr[r]; e < h->row_ptr[r + 1]; ++e) ci.push_back(i * w + h->col_idx[e]);
      ci.push_back(i * w + n + r);
      rp.push_back((int32_t)ci.size());
    }
}

}  // namespace

struct qldpc_phenl {
  qldpc_bp* st[2] = {nullptr, nullptr};  // [0] X sector: ST graph of hz; [1] Z sector: ST graph of hx
  qldpc_bp* d2[2] = {nullptr, nullptr};  // final-round decoders on hz / hx
  int device = 0, n = 0, m[2] = {0, 0}, k[2] = {0, 0}, reps = 1;
  long long max_batch = 0;
  int Wmax = 0;
  DevBuf hl_rp[2], hl_ci[2];  // [H; L] stacked CSR per sector
  DevBuf cur[2], serr[2], sprev, D[2], det[2], corr[2], iters, conv, failw[2];
  // BP+OSD final round (qldpc_phenl_set_final_osd): soft BP posteriors and BP decisions
  qldpc_osd_gpu* osd2[2] = {nullptr, nullptr};
  DevBuf post, bpcorr;
  // FirstMinBPDecoder noisy rounds (qldpc_phenl_set_round_firstmin): replace the ST BP decodes
  qldpc_firstmin* fm1[2] = {nullptr, nullptr};
};

extern "C" {

int qldpc_phenl_create(qldpc_bp* st_x, qldpc_bp* st_z, qldpc_bp* dec2_x, qldpc_bp* dec2_z,
                       const qldpc_graph* logical_x, const qldpc_graph* logical_z, int32_t num_rep, int64_t max_batch,
                       qldpc_phenl** out) {
  if (!out) return set_err(QLDPC_EINVAL, "out is NULL");
  if (num_rep < 1) return set_err(QLDPC_EINVAL, "num_rep must be >= 1");
  qldpc_bp* st[2] = {st_x, st_z};
  qldpc_bp* d2[2] = {dec2_x, dec2_z};
  const qldpc_graph* L[2] = {logical_x, logical_z};
  int n = -1, dev = -1;
  for (int q = 0; q < 2; ++q) {
    // both sectors always: the uniform stream interleaves the flips of both check sets
    if (!st[q] || !d2[q] || !L[q])
      return set_err(QLDPC_EINVAL, "both sectors need their ST decoder, final decoder and logicals");
    const qldpc_graph* h = d2[q]->g;
    if (n >= 0 && h->n != n) return set_err(QLDPC_EINVAL, "sector code lengths differ");
    if (dev >= 0 && h->device != dev) return set_err(QLDPC_EINVAL, "sectors on different devices");
    n = h->n;
    dev = h->device;
    if (L[q]->n != n) return set_err(QLDPC_EINVAL, "logical operator width != code length");
    // the ST decoder must run on exactly GetSpaceTimeCheckMat(h, num_rep)
    std::vector<int32_t> rp, ci;
    st_csr(h, num_rep, rp, ci);
    const qldpc_graph* g = st[q]->g;
    if (g->m != num_rep * h->m || g->n != num_rep * (n + h->m) || g->row_ptr != rp || g->col_idx != ci)
      return set_err(QLDPC_EINVAL, "ST decoder graph is not GetSpaceTimeCheckMat(h, num_rep) of the final decoder's h");
    if (g->device != dev || L[q]->device != dev) return set_err(QLDPC_EINVAL, "sectors on different devices");
  }
  if (max_batch <= 0) max_batch = 1 << 16;
  max_batch = std::max<long long>(64, (max_batch + 63) / 64 * 64);
  QLDPC_HIP(hipSetDevice(dev));
  auto* P = new qldpc_phenl();
  P->device = dev;
  P->n = n;
  P->reps = num_rep;
  P->max_batch = max_batch;
  P->Wmax = (int)(max_batch / 64);
  const size_t W = (size_t)P->Wmax;
  auto fail = [&](int rc) {
    for (int q = 0; q < 2; ++q) {
      P->hl_rp[q].release(); P->hl_ci[q].release(); P->cur[q].release(); P->serr[q].release();
      P->D[q].release(); P->det[q].release(); P->corr[q].release(); P->failw[q].release();
    }
    P->sprev.release(); P->iters.release(); P->conv.release();
    delete P;
    return rc;
  };
  int rc = 0;
  size_t mm = 0;
  for (int q = 0; q < 2; ++q) {
    P->st[q] = st[q];
    P->d2[q] = d2[q];
    const qldpc_graph* h = d2[q]->g;
    P->m[q] = h->m;
    P->k[q] = L[q]->m;
    mm = std::max(mm, (size_t)h->m);
    std::vector<int32_t> rp(h->row_ptr), ci(h->col_idx);
    for (int r = 0; r < L[q]->m; ++r) {
      for (int e = L[q]->row_ptr[r]; e < L[q]->row_ptr[r + 1]; ++e) ci.push_back(L[q]->col_idx[e]);
      rp.push_back((int32_t)ci.size());
    }
    const size_t R = (size_t)num_rep * h->m, C = (size_t)num_rep * (n + h->m);
    if ((rc = P->hl_rp[q].alloc(rp.size() * 4)) || (rc = P->hl_ci[q].alloc(std::max<size_t>(4, ci.size() * 4))) ||
        (rc = P->cur[q].alloc((size_t)n * W * 8)) || (rc = P->serr[q].alloc((size_t)h->m * W * 8)) ||
        (rc = P->D[q].alloc(R * W * 8)) || (rc = P->det[q].alloc(R * (size_t)max_batch)) ||
        (rc = P->corr[q].alloc(C * (size_t)max_batch)) || (rc = P->failw[q].alloc(W * 8)))
      return fail(rc);
    if (hipMemcpy(P->hl_rp[q].p, rp.data(), rp.size() * 4, hipMemcpyHostToDevice) != hipSuccess ||
        (!ci.empty() && hipMemcpy(P->hl_ci[q].p, ci.data(), ci.size() * 4, hipMemcpyHostToDevice) != hipSuccess))
      return fail(set_err(QLDPC_EHIP, "hipMemcpy of the check graphs failed"));
  }
  if ((rc = P->sprev.alloc(mm * W * 8)) || (rc = P->iters.alloc((size_t)max_batch * 4)) ||
      (rc = P->conv.alloc((size_t)max_batch)))
    return fail(rc);
  *out = P;
  return 0;
}

int qldpc_phenl_set_final_osd(qldpc_phenl* P, qldpc_osd_gpu* osd_x, qldpc_osd_gpu* osd_z) {
  if (!P) return set_err(QLDPC_EINVAL, "NULL phenl");
  qldpc_osd_gpu* o[2] = {osd_x, osd_z};
  for (int q = 0; q < 2; ++q) {
    if (!o[q]) continue;
    int32_t eng = 0;
    qldpc_bp_engine(P->d2[q], &eng);
    if (eng != 1) return set_err(QLDPC_ENOTSUP, "BP+OSD final round needs dec2 from qldpc_bp_create_soft");
    // the OSD stage reads dec2's syndromes (row stride m) and eliminates its H: same graph only
    if (!osd_gpu_matches(o[q], P->d2[q]->g))
      return set_err(QLDPC_EINVAL, q == 0 ? "X-sector OSD handle was built on a different graph than dec2_x"
                                          : "Z-sector OSD handle was built on a different graph than dec2_z");
  }
  if ((osd_x || osd_z) && !P->post.p) {
    QLDPC_HIP(hipSetDevice(P->device));
    int rc;
    if ((rc = P->post.alloc((size_t)P->max_batch * P->n * 8)) || (rc = P->bpcorr.alloc((size_t)P->max_batch * P->n)))
      return rc;
  }
  P->osd2[0] = osd_x;
  P->osd2[1] = osd_z;
  return 0;
}

int qldpc_phenl_set_round_firstmin(qldpc_phenl* P, qldpc_firstmin* fm_x, qldpc_firstmin* fm_z) {
  if (!P) return set_err(QLDPC_EINVAL, "NULL phenl");
  qldpc_firstmin* f[2] = {fm_x, fm_z};
  for (int q = 0; q < 2; ++q)
    if (f[q] && !qldpc_rt::firstmin_matches(f[q], P->st[q]->g))
      return set_err(QLDPC_EINVAL, q == 0 ? "X-sector first-min decoder was built on a different graph than st_x"
                                          : "Z-sector first-min decoder was built on a different graph than st_z");
  P->fm1[0] = fm_x;
  P->fm1[1] = fm_z;
  return 0;
}

int qldpc_phenl_destroy(qldpc_phenl* P) {
  if (!P) return 0;
  for (int q = 0; q < 2; ++q) {
    P->hl_rp[q].release(); P->hl_ci[q].release(); P->cur[q].release(); P->serr[q].release();
    P->D[q].release(); P->det[q].release(); P->corr[q].release(); P->failw[q].release();
  }
  P->sprev.release(); P->iters.release(); P->conv.release();
  P->post.release(); P->bpcorr.release();
  delete P;
  return 0;
}

int qldpc_phenl_trace_len(const qldpc_phenl* P, int32_t num_rounds, int64_t* out) {
  if (!P || !out || num_rounds < 1) return set_err(QLDPC_EINVAL, "bad argument");
  const long long m0 = P->m[0], m1 = P->m[1];
  *out = (long long)(num_rounds - 1) * P->reps * (m1 + m0) + m1 + m0;
  return 0;
}

int qldpc_phenl_launch(qldpc_phenl* P, double px, double py, double pz, double q, uint64_t seed, uint64_t shot_begin,
                       int64_t shot_count, int32_t num_rounds, int32_t logical_mode, const double* d_uniforms,
                       void* d_counters, uint8_t* d_fail, uint8_t* d_trace, void* stream) {
  if (!P || !d_counters) return set_err(QLDPC_EINVAL, "NULL argument");
  if (logical_mode < 0 || logical_mode > 2) return set_err(QLDPC_EINVAL, "logical_mode must be 0 (X), 1 (Z), 2 (Total)");
  if (num_rounds < 1) return set_err(QLDPC_EINVAL, "num_rounds must be >= 1");
  if (!(px >= 0 && py >= 0 && pz >= 0 && q >= 0)) return set_err(QLDPC_EINVAL, "negative probability");
  // sectors the returned outcome cannot depend on are skipped (their draws are still indexed)
  const bool need[2] = {logical_mode != 1, logical_mode != 0};
  if (shot_count <= 0) return 0;
  QLDPC_HIP(hipSetDevice(P->device));
  hipStream_t st = (hipStream_t)stream;
  auto* cnt = static_cast<unsigned long long*>(d_counters);
  const int n = P->n;
  const int m0 = P->m[0], m1 = P->m[1];  // hz rows (X sector), hx rows (Z sector)
  const int Pw = n + m1 + m0;  // uniforms per repetition
  const long long nu = ((long long)(num_rounds - 1) * P->reps + 1) * Pw;
  if (nu > 0xFFFFFFFFll) return set_err(QLDPC_EINVAL, "too many uniforms per sample (> 2^32)");
  const long long tlen = (long long)(num_rounds - 1) * P->reps * (m1 + m0) + m1 + m0;
  const double t1 = pz, t2 = pz + px, t3 = (pz + px) + py;
  SampleArgs A;
  std::memset(&A, 0, sizeof(A));
  A.uniforms = d_uniforms;
  A.tag = kStreamPhen;
  A.nu = nu;
  A.seed = seed;
  A.shot_begin = shot_begin;
  A.t1 = t1; A.t2 = t2; A.t3 = t3; A.q = q;
  A.K1 = ceil53(t1); A.K2 = ceil53(t2); A.K3 = ceil53(t3); A.Kq = ceil53(q);
  A.n = n; A.m0 = m0; A.m1 = m1;
  for (long long c0 = 0; c0 < shot_count; c0 += P->max_batch) {
    const long long B = std::min<long long>(P->max_batch, shot_count - c0);
    const int W = (int)((B + 63) / 64);
    A.c0 = c0;
    A.count = B;
    A.W = W;
    const dim3 wgrid((W + kTile - 1) / kTile);
    for (int s = 0; s < 2; ++s) {
      A.cur[s] = need[s] ? static_cast<unsigned long long*>(P->cur[s].p) : nullptr;
      if (need[s]) {
        QLDPC_HIP(hipMemsetAsync(P->cur[s].p, 0, (size_t)n * W * 8, st));
        QLDPC_HIP(hipMemsetAsync(P->failw[s].p, 0, (size_t)W * 8, st));
      }
    }
    long long toff = 0;
    // ---- noisy rounds (src/Simulators_SpaceTime.py:442-481)
    for (int r = 0; r + 1 < num_rounds; ++r) {
      for (int j = 0; j < P->reps; ++j) {
        A.base = (uint32_t)((long long)(r * P->reps + j) * Pw);
        for (int s = 0; s < 2; ++s) A.serr[s] = need[s] ? static_cast<unsigned long long*>(P->serr[s].p) : nullptr;
        hipLaunchKernelGGL(ph_sample, dim3((unsigned)((B + kTile - 1) / kTile), (unsigned)Pw), dim3(kTile), 0, st, A);
        QLDPC_HIP(hipGetLastError());
        for (int s = 0; s < 2; ++s) {
          if (!need[s]) continue;
          const int diff = s == 1 ? (j > 0 ? 1 : 0) : -1;  // Z sector: consecutive-syndrome detectors
          hipLaunchKernelGGL(ph_syndrome, dim3(wgrid.x, (unsigned)P->m[s]), dim3(kTile), 0, st,
                             static_cast<const int32_t*>(P->hl_rp[s].p), static_cast<const int32_t*>(P->hl_ci[s].p),
                             static_cast<const unsigned long long*>(P->cur[s].p),
                             static_cast<const unsigned long long*>(P->serr[s].p),
                             diff >= 0 ? static_cast<unsigned long long*>(P->sprev.p) : nullptr,
                             static_cast<unsigned long long*>(P->D[s].p), W, j * P->m[s], diff);
          QLDPC_HIP(hipGetLastError());
        }
      }
      // space-time decode + fold, Z sector first (the reference's order; the trace keeps it)
      for (int s : {1, 0}) {
        const int R = P->reps * (s == 1 ? m1 : m0);
        if (need[s]) {
          hipLaunchKernelGGL(ph_unpack, dim3((unsigned)((R + kTile - 1) / kTile), (unsigned)W), dim3(kTile), 0, st,
                             static_cast<const unsigned long long*>(P->D[s].p), static_cast<uint8_t*>(P->det[s].p),
                             d_trace, tlen, toff, c0, R, W, B);
          QLDPC_HIP(hipGetLastError());
          int rc;
          if (P->fm1[s]) {  // FirstMinBPDecoder: accepted steps as "iterations", never non-converged
            rc = qldpc_firstmin_decode(P->fm1[s], static_cast<const uint8_t*>(P->det[s].p),
                                       static_cast<uint8_t*>(P->corr[s].p), static_cast<int32_t*>(P->iters.p), B, stream);
            if (rc) return rc;
            QLDPC_HIP(hipMemsetAsync(P->conv.p, 1, (size_t)B, st));
          } else {
            rc = qldpc_bp_decode_batch(P->st[s], static_cast<const uint8_t*>(P->det[s].p),
                                       static_cast<uint8_t*>(P->corr[s].p), static_cast<int32_t*>(P->iters.p),
                                       static_cast<uint8_t*>(P->conv.p), B, stream);
            if (rc) return rc;
          }
          hipLaunchKernelGGL(ph_iters, dim3((unsigned)((B + kTile - 1) / kTile)), dim3(kTile), 0, st,
                             static_cast<const int32_t*>(P->iters.p), static_cast<const uint8_t*>(P->conv.p), cnt, s, B);
          QLDPC_HIP(hipGetLastError());
          const int w = n + P->m[s];
          hipLaunchKernelGGL(ph_fold, dim3((unsigned)((n + kTile - 1) / kTile), (unsigned)W), dim3(kTile), 0, st,
                             static_cast<const uint8_t*>(P->corr[s].p), static_cast<unsigned long long*>(P->cur[s].p),
                             n, W, P->reps, w, P->reps * w, B);
          QLDPC_HIP(hipGetLastError());
        }
        toff += R;
      }
    }
    // ---- final perfect round with dec2 (:483-529)
    A.base = (uint32_t)((long long)(num_rounds - 1) * P->reps * Pw);
    A.serr[0] = A.serr[1] = nullptr;
    hipLaunchKernelGGL(ph_sample, dim3((unsigned)((B + kTile - 1) / kTile), (unsigned)n), dim3(kTile), 0, st, A);
    QLDPC_HIP(hipGetLastError());
    for (int s : {1, 0}) {
      const int R = s == 1 ? m1 : m0;
      if (need[s]) {
        hipLaunchKernelGGL(ph_syndrome, dim3(wgrid.x, (unsigned)P->m[s]), dim3(kTile), 0, st,
                           static_cast<const int32_t*>(P->hl_rp[s].p), static_cast<const int32_t*>(P->hl_ci[s].p),
                           static_cast<const unsigned long long*>(P->cur[s].p), nullptr, nullptr,
                           static_cast<unsigned long long*>(P->D[s].p), W, 0, -1);
        QLDPC_HIP(hipGetLastError());
        hipLaunchKernelGGL(ph_unpack, dim3((unsigned)((R + kTile - 1) / kTile), (unsigned)W), dim3(kTile), 0, st,
                           static_cast<const unsigned long long*>(P->D[s].p), static_cast<uint8_t*>(P->det[s].p),
                           d_trace, tlen, toff, c0, R, W, B);
        QLDPC_HIP(hipGetLastError());
        int rc;
        if (P->osd2[s]) {  // bposd_decoder as decoder2: BP, then OSD where BP did not converge
          rc = qldpc_bp_decode_batch_soft(P->d2[s], static_cast<const uint8_t*>(P->det[s].p),
                                          static_cast<uint8_t*>(P->bpcorr.p), static_cast<int32_t*>(P->iters.p),
                                          static_cast<uint8_t*>(P->conv.p), static_cast<double*>(P->post.p), B, stream);
          if (!rc)
            rc = qldpc_osd_gpu_decode(P->osd2[s], static_cast<const uint8_t*>(P->det[s].p),
                                      static_cast<const double*>(P->post.p), static_cast<const uint8_t*>(P->conv.p),
                                      static_cast<const uint8_t*>(P->bpcorr.p), nullptr,
                                      static_cast<uint8_t*>(P->corr[s].p), B, stream);
        } else {
          rc = qldpc_bp_decode_batch(P->d2[s], static_cast<const uint8_t*>(P->det[s].p),
                                     static_cast<uint8_t*>(P->corr[s].p), static_cast<int32_t*>(P->iters.p),
                                     static_cast<uint8_t*>(P->conv.p), B, stream);
        }
        if (rc) return rc;
        hipLaunchKernelGGL(ph_iters, dim3((unsigned)((B + kTile - 1) / kTile)), dim3(kTile), 0, st,
                           static_cast<const int32_t*>(P->iters.p), static_cast<const uint8_t*>(P->conv.p), cnt, s, B);
        QLDPC_HIP(hipGetLastError());
        // residual r = cur ^ decoded (in place), then failure words over [H; L]
        hipLaunchKernelGGL(ph_fold, dim3((unsigned)((n + kTile - 1) / kTile), (unsigned)W), dim3(kTile), 0, st,
                           static_cast<const uint8_t*>(P->corr[s].p), static_cast<unsigned long long*>(P->cur[s].p), n,
                           W, 1, n, n, B);
        QLDPC_HIP(hipGetLastError());
        hipLaunchKernelGGL(ph_check, dim3(wgrid.x, (unsigned)(P->m[s] + P->k[s])), dim3(kTile), 0, st,
                           static_cast<const int32_t*>(P->hl_rp[s].p), static_cast<const int32_t*>(P->hl_ci[s].p),
                           static_cast<const unsigned long long*>(P->cur[s].p),
                           static_cast<unsigned long long*>(P->failw[s].p), W);
        QLDPC_HIP(hipGetLastError());
      }
      toff += R;
    }
    hipLaunchKernelGGL(ph_tally, wgrid, dim3(kTile), 0, st,
                       need[0] ? static_cast<const unsigned long long*>(P->failw[0].p) : nullptr,
                       need[1] ? static_cast<const unsigned long long*>(P->failw[1].p) : nullptr, cnt, d_fail, c0, W,
                       B, logical_mode);
    QLDPC_HIP(hipGetLastError());
  }
  return 0;
}

}  // extern "C"

// ===================================================== (2) staged data-error MC
// CodeSimulator_DataError._single_run (src/Simulators.py:117-168) as a
// pipeline: Philox sampling of both Pauli components with the fused kernels'
// stream (kStreamData, ctr = (qubit, shot)) -> per needed sector: bit-sliced
// H e, unpack, qldpc_bp_decode_batch, residual fold, [H; L] check -> tally.
namespace qldpc_rt {

constexpr long long kStagedBatch = 1 << 16;

void staged_mc_release(qldpc_mc* mc) {
  for (int q = 0; q < 2; ++q) {
    mc->s_rp[q].release(); mc->s_ci[q].release(); mc->s_cur[q].release(); mc->s_failw[q].release();
  }
  for (DevBuf* d : {&mc->s_D, &mc->s_det, &mc->s_corr, &mc->s_iters, &mc->s_conv}) d->release();
}

int staged_mc_prepare(qldpc_mc* mc, const qldpc_graph* logical_x, const qldpc_graph* logical_z) {
  const qldpc_graph* L[2] = {logical_x, logical_z};
  const qldpc_bp* d0 = mc->dec[0] ? mc->dec[0] : mc->dec[1];
  const int n = d0->g->n;
  // the HBM engine decodes one syndrome per lane: a batch of many syndromes per resident lane
  // keeps its lanes refilled instead of waiting on the batch's slowest decode
  const bool hbm = (mc->dec[0] && mc->dec[0]->engine == 6) || (mc->dec[1] && mc->dec[1]->engine == 6);
  const char* eb = std::getenv("QLDPC_STAGED_BATCH");
  // HBM engine: 4M shots per batch (~32 decodes per resident lane and sector: the batch's tail, where
  // lanes run out of syndromes and their partial-wave accesses still move whole lines, drops from 1/2
  // of the traffic at 262k shots to a few %; LP L30 fp64 0.28 -> 0.45 of HBM, profiles/r03/e6/),
  // bounded to ~8 GB of per-shot buffers
  const long long hbm_b = std::max<long long>(kStagedBatch, std::min<long long>(kStagedBatch * 64,
                                                                                 (8ll << 30) / std::max(1, n + d0->g->m)));
  long long B = (eb && *eb) ? std::max(64LL, std::atoll(eb) / 64 * 64) : (hbm ? hbm_b / 64 * 64 : kStagedBatch);
  const size_t W = (size_t)(B / 64);
  int mm = 1, rc;
  for (int q = 0; q < 2; ++q) {
    if ((rc = mc->s_cur[q].alloc((size_t)n * W * 8)) || (rc = mc->s_failw[q].alloc(W * 8))) return rc;
    if (!mc->dec[q]) continue;
    const qldpc_graph* h = mc->dec[q]->g;
    if (!L[q]) return set_err(QLDPC_EINVAL, "sector has no logical operators");
    std::vector<int32_t> rp(h->row_ptr), ci(h->col_idx);
    for (int r = 0; r < L[q]->m; ++r) {
      for (int e = L[q]->row_ptr[r]; e < L[q]->row_ptr[r + 1]; ++e) ci.push_back(L[q]->col_idx[e]);
      rp.push_back((int32_t)ci.size());
    }
    mc->sm[q] = h->m;
    mc->sk[q] = L[q]->m;
    mm = std::max(mm, h->m);
    if ((rc = mc->s_rp[q].alloc(rp.size() * 4)) || (rc = mc->s_ci[q].alloc(std::max<size_t>(4, ci.size() * 4))))
      return rc;
    QLDPC_HIP(hipMemcpy(mc->s_rp[q].p, rp.data(), rp.size() * 4, hipMemcpyHostToDevice));
    if (!ci.empty()) QLDPC_HIP(hipMemcpy(mc->s_ci[q].p, ci.data(), ci.size() * 4, hipMemcpyHostToDevice));
  }
  if ((rc = mc->s_D.alloc((size_t)mm * W * 8)) || (rc = mc->s_det.alloc((size_t)mm * B)) ||
      (rc = mc->s_corr.alloc((size_t)n * B)) || (rc = mc->s_iters.alloc((size_t)B * 4)) ||
      (rc = mc->s_conv.alloc((size_t)B)))
    return rc;
  mc->sbatch = B;
  mc->staged = true;
  return 0;
}

int staged_mc_launch(qldpc_mc* mc, double px, double py, double pz, uint64_t seed, uint64_t shot_begin,
                     int64_t shot_count, int32_t logical_mode, const double* d_uniforms, void* d_counters,
                     uint8_t* d_fail, uint8_t* d_err, uint8_t* d_corr, int32_t* d_iters, hipStream_t st) {
  const bool need[2] = {logical_mode != 1, logical_mode != 0};
  const qldpc_bp* d0 = mc->dec[0] ? mc->dec[0] : mc->dec[1];
  const int n = d0->g->n;
  auto* cnt = static_cast<unsigned long long*>(d_counters);
  const double t1 = pz, t2 = pz + px, t3 = (pz + px) + py;
  SampleArgs A;
  std::memset(&A, 0, sizeof(A));
  A.uniforms = d_uniforms;
  A.tag = kStreamData;
  A.nu = n;
  A.seed = seed;
  A.shot_begin = shot_begin;
  A.t1 = t1; A.t2 = t2; A.t3 = t3;
  A.K1 = ceil53(t1); A.K2 = ceil53(t2); A.K3 = ceil53(t3);
  A.n = n;
  A.base = 0;
  for (long long c0 = 0; c0 < shot_count; c0 += mc->sbatch) {
    const long long B = std::min<long long>(mc->sbatch, shot_count - c0);
    const int W = (int)((B + 63) / 64);
    A.c0 = c0;
    A.count = B;
    A.W = W;
    const dim3 wgrid((W + kTile - 1) / kTile);
    for (int q = 0; q < 2; ++q) {
      A.cur[q] = static_cast<unsigned long long*>(mc->s_cur[q].p);
      QLDPC_HIP(hipMemsetAsync(mc->s_cur[q].p, 0, (size_t)n * W * 8, st));
      QLDPC_HIP(hipMemsetAsync(mc->s_failw[q].p, 0, (size_t)W * 8, st));
    }
    hipLaunchKernelGGL(ph_sample, dim3((unsigned)((B + kTile - 1) / kTile), (unsigned)n), dim3(kTile), 0, st, A);
    QLDPC_HIP(hipGetLastError());
    if (d_err) {
      hipLaunchKernelGGL(ph_err_out, dim3((unsigned)((n + kTile - 1) / kTile), (unsigned)W), dim3(kTile), 0, st,
                         static_cast<const unsigned long long*>(mc->s_cur[0].p),
                         static_cast<const unsigned long long*>(mc->s_cur[1].p), d_err, c0, n, W, B);
      QLDPC_HIP(hipGetLastError());
    }
    for (int q = 0; q < 2; ++q) {
      if (!need[q]) continue;
      const int m = mc->sm[q];
      auto* cur = static_cast<unsigned long long*>(mc->s_cur[q].p);
      hipLaunchKernelGGL(ph_syndrome, dim3(wgrid.x, (unsigned)m), dim3(kTile), 0, st,
                         static_cast<const int32_t*>(mc->s_rp[q].p), static_cast<const int32_t*>(mc->s_ci[q].p), cur,
                         nullptr, nullptr, static_cast<unsigned long long*>(mc->s_D.p), W, 0, -1);
      QLDPC_HIP(hipGetLastError());
      hipLaunchKernelGGL(ph_unpack, dim3((unsigned)((m + kTile - 1) / kTile), (unsigned)W), dim3(kTile), 0, st,
                         static_cast<const unsigned long long*>(mc->s_D.p), static_cast<uint8_t*>(mc->s_det.p),
                         nullptr, 0, 0, c0, m, W, B);
      QLDPC_HIP(hipGetLastError());
      int rc = qldpc_bp_decode_batch(mc->dec[q], static_cast<const uint8_t*>(mc->s_det.p),
                                     static_cast<uint8_t*>(mc->s_corr.p), static_cast<int32_t*>(mc->s_iters.p),
                                     static_cast<uint8_t*>(mc->s_conv.p), B, st);
      if (rc) return rc;
      hipLaunchKernelGGL(ph_iters, dim3((unsigned)((B + kTile - 1) / kTile)), dim3(kTile), 0, st,
                         static_cast<const int32_t*>(mc->s_iters.p), static_cast<const uint8_t*>(mc->s_conv.p), cnt, q,
                         B);
      QLDPC_HIP(hipGetLastError());
      if (d_corr)
        QLDPC_HIP(hipMemcpy2DAsync(d_corr + (c0 * 2 + q) * n, (size_t)2 * n, mc->s_corr.p, (size_t)n, (size_t)n,
                                   (size_t)B, hipMemcpyDeviceToDevice, st));
      if (d_iters)
        QLDPC_HIP(hipMemcpy2DAsync(d_iters + c0 * 2 + q, 8, mc->s_iters.p, 4, 4, (size_t)B, hipMemcpyDeviceToDevice,
                                   st));
      hipLaunchKernelGGL(ph_fold, dim3((unsigned)((n + kTile - 1) / kTile), (unsigned)W), dim3(kTile), 0, st,
                         static_cast<const uint8_t*>(mc->s_corr.p), cur, n, W, 1, n, n, B);
      QLDPC_HIP(hipGetLastError());
      hipLaunchKernelGGL(ph_check, dim3(wgrid.x, (unsigned)(m + mc->sk[q])), dim3(kTile), 0, st,
                         static_cast<const int32_t*>(mc->s_rp[q].p), static_cast<const int32_t*>(mc->s_ci[q].p), cur,
                         static_cast<unsigned long long*>(mc->s_failw[q].p), W);
      QLDPC_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(ph_tally, wgrid, dim3(kTile), 0, st,
                       need[0] ? static_cast<const unsigned long long*>(mc->s_failw[0].p) : nullptr,
                       need[1] ? static_cast<const unsigned long long*>(mc->s_failw[1].p) : nullptr, cnt, d_fail, c0,
                       W, B, logical_mode);
    QLDPC_HIP(hipGetLastError());
  }
  return 0;
}

}  // namespace qldpc_rt
