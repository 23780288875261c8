// circuit.hip — the circuit-level space-time shot loop:
// CodeSimulator_Circuit_SpaceTime._single_run / WordErrorRate (src/Simulators_SpaceTime.py:968-1049)
// for a batch of samples at once, on the detector error model (DEM) of the full syndrome circuit
// and the fault hypergraphs h1 / h2 of one round (qldpc_fault_tolerance_amd/circuit.py builds both).
//
// One sample:
//   (1) every DEM mechanism j fires independently: Philox4x32-10 uniform of (seed, global sample,
//       j) in the circuit stream < p_j (53-bit compare, as the data-error stream);
//   (2) detectors / observables = XOR of the fired mechanisms' rows;
//   (3) for each of the num_rounds rounds: the round's num_rep·m detector rows, the first m XORed
//       with the accumulated space correction, decoded by decoder1 on h1; the correction's space
//       effect (h1_space_cor · c) and logical effect (L1 · c) accumulate (:983-993);
//   (4) the final m detector rows XOR the accumulated space correction, decoded by decoder2 on h2
//       (BP, or BP + OSD on the GPU: the DEM's non-uniform priors weigh the OSD candidates by
//       sum log(1 / p_j), osd.hip step 6'; no host round trip — a host OSD stage past the GPU
//       kernel's envelope decodes on the host, circ_host_osd);
//   (5) failure = (final syndrome + h2 · c2 != 0) or (observables + Σ L · c != 0) (:996-1004).
// State is BIT-SLICED between the stages (word w of row r = row r of samples 64w..64w+63), so the
// mechanism scatter of (1)-(2) is one wave ballot + one 64-bit atomic xor per (mechanism row, 64
// samples), and (3)-(5)'s GF(2) products are word XORs; decoder I/O crosses to bytes per sample.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "bp_kernels.h"
#include "runtime.h"

using namespace qldpc;
using namespace qldpc_rt;

namespace {

constexpr uint32_t kStreamCirc = 0x51D50003u;
constexpr int kTileC = 256;
using u64 = unsigned long long;

__device__ inline u64 circ_k53(u64 seed, u64 shot, uint32_t j) {
  uint32_t w0, w1;
  philox4x32_10(j, (uint32_t)shot, (uint32_t)(shot >> 32), kStreamCirc, (uint32_t)seed, (uint32_t)(seed >> 32), w0, w1);
  return ((u64)(w0 >> 5) << 26) | (u64)(w1 >> 6);
}

// (1)+(2): grid x = sample tiles of 256, y = mechanisms (strided).  Lane 0 of each wave xors the
// wave's 64-sample word into every row the mechanism touches (detectors, then observables at D+k).
__global__ void __launch_bounds__(kTileC) cs_sample(const int32_t* __restrict__ mp, const int32_t* __restrict__ mr,
                                                   const u64* __restrict__ k53, int M, u64 seed, u64 shot0, long long count,
                                                   int W, u64* __restrict__ DO) {
  const long long s = (long long)blockIdx.x * kTileC + threadIdx.x;
  const int w = (int)(s >> 6);
  for (int j = blockIdx.y; j < M; j += gridDim.y) {
    const bool fire = s < count && circ_k53(seed, shot0 + (u64)s, (uint32_t)j) < k53[j];
    const u64 word = __ballot(fire);
    if (__lane_id() == 0 && word && w < W)
      for (int e = mp[j]; e < mp[j + 1]; ++e) atomicXor(&DO[(long long)mr[e] * W + w], word);
  }
}

// Geometric-skip DEM sampling (round 6; the default sampler).  The keyed sampler
// above draws one Philox number per (sample, mechanism): B x M draws per batch, almost all of them
// misses at circuit-level rates (p_j ~ 1e-3).  Here the samples of mechanism j are generated per
// GLOBAL 64-sample word gw (samples 64 gw .. 64 gw + 63) as a run of geometric gaps: from position
// pos, the number of non-firing samples before the next firing is G = #{k in 1..64-pos : u < T_k},
// u the 53-bit Philox integer of (seed, j, gw, draw index c), T_k = ceil(2^53 (1 - p_j)^k) (host
// table, (1 - p)^k by repeated IEEE multiplication), so P(G >= k) = (1 - p_j)^k exactly as the
// keyed comparison u < ceil(2^53 p) prices one sample; the word costs 1 + (#firings) draws, ~1.06 at
// p = 1e-3 instead of 64.  The words are keyed by the global word index, so any batching or sharding
// (shot0 not a multiple of 64: a batch word spans two global words) draws the same samples.
// oracle/circuit_oracle.py sample_mechanisms restates it.
constexpr uint32_t kStreamSkip = 0x51D50004u;
__device__ inline u64 skip_word(u64 seed, uint32_t j, u64 gw, const u64* __restrict__ t) {
  u64 bits = 0;
  int pos = 0;
  for (uint32_t c = 0; c <= 64u; ++c) {  // at most 64 firings: the loop always ends
    uint32_t w0, w1;
    philox4x32_10(j, (uint32_t)gw, ((uint32_t)(gw >> 32) << 8) | c, kStreamSkip, (uint32_t)seed, (uint32_t)(seed >> 32),
                  w0, w1);
    const u64 u = ((u64)(w0 >> 5) << 26) | (u64)(w1 >> 6);
    // G = the largest k in [0, 64 - pos] with k == 0 or T_k > u (T non-increasing): binary search
    int lo = 0, hi = 64 - pos;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (t[mid - 1] > u) lo = mid; else hi = mid - 1;
    }
    pos += lo;
    if (pos >= 64) break;
    bits |= 1ull << pos;
    ++pos;
  }
  return bits;
}
// grid x = batch words (tiles of 256), y = mechanisms (strided); one thread per (mechanism, word):
// its batch word from the one or two global words it spans, then one 64-bit atomic xor per touched
// row when the word is nonzero
__global__ void __launch_bounds__(kTileC) cs_sample_skip(const int32_t* __restrict__ mp, const int32_t* __restrict__ mr,
                                                        const u64* __restrict__ T, int M, u64 seed, u64 shot0,
                                                        long long count, int W, u64* __restrict__ DO) {
  const int w = blockIdx.x * kTileC + threadIdx.x;
  if (w >= W) return;
  const int a = (int)(shot0 & 63u);
  const u64 gw = (shot0 >> 6) + (u64)w;
  const long long nb = count - (long long)w * 64;
  const u64 valid = nb >= 64 ? ~0ull : ((1ull << nb) - 1ull);
  for (int j = blockIdx.y; j < M; j += gridDim.y) {
    const u64* t = T + (size_t)j * 64;
    u64 word = skip_word(seed, (uint32_t)j, gw, t) >> a;
    if (a) word |= skip_word(seed, (uint32_t)j, gw + 1, t) << (64 - a);
    word &= valid;
    if (word)
      for (int e = mp[j]; e < mp[j + 1]; ++e) atomicXor(&DO[(long long)mr[e] * W + w], word);
  }
}

// bit-sliced rows [row0, row0 + R) (the first nx XORed with X) -> bytes out[s][R].
// grid x = row tiles, y = word w
__global__ void __launch_bounds__(kTileC) cs_unpack(const u64* __restrict__ DO, const u64* __restrict__ X, int row0,
                                                   int R, int nx, uint8_t* __restrict__ out, int W, long long count) {
  const int r = blockIdx.x * kTileC + threadIdx.x;
  const int w = blockIdx.y;
  if (r >= R) return;
  u64 d = DO[(long long)(row0 + r) * W + w];
  if (r < nx) d ^= X[(long long)r * W + w];
  const int nb = (int)std::min<long long>(64, count - (long long)w * 64);
  for (int b = 0; b < nb; ++b) out[((long long)w * 64 + b) * R + r] = (uint8_t)((d >> b) & 1ull);
}

// acc[r][w] ^= bit-sliced parities of the CSR rows r of A (cols over the decoder's n) on the byte
// corrections corr[s][n]: one thread per SAMPLE (its corr row is contiguous, a wave's 64 rows one
// ~64 n-byte span), every row's parity a ballot = the word of its 64 samples, written by lane 0
// (each (r, w) belongs to one wave: no atomics).  grid x = sample tiles
__global__ void __launch_bounds__(kTileC) cs_apply(const int32_t* __restrict__ rp, const int32_t* __restrict__ ci,
                                                  int rows, const uint8_t* __restrict__ corr, int n,
                                                  u64* __restrict__ acc, int W, long long count) {
  const long long s = (long long)blockIdx.x * kTileC + threadIdx.x;
  const int w = (int)(s >> 6);
  if (((long long)w << 6) >= count) return;  // whole wave past the batch (uniform per wave)
  const uint8_t* c = corr + (s < count ? s : 0) * (long long)n;
  for (int r = 0; r < rows; ++r) {
    uint32_t x = 0;
    if (s < count)
      for (int e = rp[r]; e < rp[r + 1]; ++e) x ^= c[ci[e]];
    const u64 bits = __ballot((x & 1u) != 0);
    if (__lane_id() == 0 && bits) acc[(long long)r * W + w] ^= bits;
  }
}

// (5): rows 0..m-1 of [h2; L2]: final syndrome (detector rows fin0.., XOR the accumulated space
// correction) + h2 · c2; rows m..m+K-1: observables (rows obs0..) + the accumulated L1 · c + L2 · c2.
// Any nonzero residual bit fails its sample.  One thread per sample as cs_apply; lane 0 ORs the
// residual words and writes the wave's failure word.  grid x = sample tiles
__global__ void __launch_bounds__(kTileC) cs_final(const int32_t* __restrict__ rp, const int32_t* __restrict__ ci,
                                                  const uint8_t* __restrict__ corr, int n, const u64* __restrict__ DO,
                                                  int fin0, int obs0, const u64* __restrict__ acc, int m, int K,
                                                  u64* __restrict__ failw, int W, long long count) {
  const long long s = (long long)blockIdx.x * kTileC + threadIdx.x;
  const int w = (int)(s >> 6);
  if (((long long)w << 6) >= count) return;  // (uniform per wave)
  const int nb = (int)std::min<long long>(64, count - (long long)w * 64);
  const u64 valid = nb >= 64 ? ~0ull : ((1ull << nb) - 1ull);
  const uint8_t* c = corr + (s < count ? s : 0) * (long long)n;
  u64 fw = 0;
  for (int r = 0; r < m + K; ++r) {
    uint32_t x = 0;
    if (s < count)
      for (int e = rp[r]; e < rp[r + 1]; ++e) x ^= c[ci[e]];
    const u64 bits = __ballot((x & 1u) != 0);
    const u64 base = DO[(long long)(r < m ? fin0 + r : obs0 + (r - m)) * W + w] ^ acc[(long long)r * W + w];
    fw |= (base ^ bits) & valid;
  }
  if (__lane_id() == 0) failw[w] = fw;
}

__global__ void __launch_bounds__(kTileC) cs_tally(const u64* __restrict__ failw, u64* __restrict__ cnt,
                                                  uint8_t* __restrict__ fail_out, long long c0, int W, long long count) {
  const int w = blockIdx.x * kTileC + threadIdx.x;
  if (w >= W) return;
  const int nb = (int)std::min<long long>(64, count - (long long)w * 64);
  const u64 f = failw[w];
  atomicAdd(&cnt[kCntShots], (u64)nb);
  if (f) {
    atomicAdd(&cnt[kCntFail], (u64)__popcll(f));
    atomicAdd(&cnt[kCntSecFail + 1], (u64)__popcll(f));
  }
  if (fail_out)
    for (int k = 0; k < nb; ++k) fail_out[c0 + (long long)w * 64 + k] = (uint8_t)((f >> k) & 1ull);
}

// decode statistics of one batched decode into counter sector q (0 = decoder1 rounds, 1 = decoder2):
// the iteration histogram in LDS first (every sample of a batch usually lands in the same few bins,
// so per-sample global atomics serialised on one address), then one global add per non-empty bin
__global__ void __launch_bounds__(kTileC) cs_iters(const int32_t* __restrict__ iters, const uint8_t* __restrict__ conv,
                                                  u64* __restrict__ cnt, int q, long long count) {
  __shared__ uint32_t hist[kHistBins];
  __shared__ u64 sit, snc;
  for (int b = threadIdx.x; b < kHistBins; b += kTileC) hist[b] = 0;
  if (threadIdx.x == 0) sit = snc = 0;
  __syncthreads();
  u64 it_sum = 0, nc = 0;
  for (long long s = (long long)blockIdx.x * kTileC + threadIdx.x; s < count; s += (long long)gridDim.x * kTileC) {
    const int it = iters[s];
    it_sum += (u64)it;
    nc += conv[s] ? 0u : 1u;
    atomicAdd(&hist[std::min(it, kHistBins - 1)], 1u);
  }
  // wave sums, one LDS add per wave
  for (int off = 32; off > 0; off >>= 1) {
    it_sum += __shfl_down(it_sum, off);
    nc += __shfl_down(nc, off);
  }
  if (__lane_id() == 0) {
    atomicAdd(&sit, it_sum);
    atomicAdd(&snc, nc);
  }
  __syncthreads();
  for (int b = threadIdx.x; b < kHistBins; b += kTileC)
    if (hist[b]) atomicAdd(&cnt[kCntHist + q * kHistBins + b], (u64)hist[b]);
  if (threadIdx.x == 0) {
    const long long first = (long long)blockIdx.x * kTileC;
    long long tot = 0;  // samples this block visited
    for (long long s0 = first; s0 < count; s0 += (long long)gridDim.x * kTileC) tot += std::min<long long>(kTileC, count - s0);
    atomicAdd(&cnt[kCntDec + q], (u64)tot);
    atomicAdd(&cnt[kCntIters + q], sit);
    atomicAdd(&cnt[kCntNonconv + q], snc);
  }
}

// cs_iters: enough blocks to spread the samples, few enough that each block's LDS histogram flush
// (one global add per non-empty bin) stays cheap
unsigned iters_grid(long long B) { return (unsigned)std::max<long long>(1, std::min<long long>(256, (B + kTileC - 1) / kTileC)); }

u64 ceil53c(double t) {
  if (!(t > 0.0)) return 0ull;
  if (t >= 1.0) return 1ull << 53;
  return (u64)std::ceil(std::ldexp(t, 53));
}

}  // namespace

struct qldpc_circ {
  int device = 0;
  qldpc_bp* dec1 = nullptr;
  qldpc_bp* dec2 = nullptr;
  qldpc_osd_gpu* osd_gpu = nullptr;
  qldpc_osd_gpu* osd_owned = nullptr;  // the GPU OSD built from a host stage (qldpc_circ_set_final_osd)
  // a host stage past the GPU kernel's envelope (n > 8192, osd_e order > 24, priors of 0 or 1): the
  // final layer's soft BP output goes to the host, through qldpc_osd_decode_batch, and back
  const qldpc_osd* osd_host = nullptr;
  std::vector<uint8_t> h_synd, h_conv, h_bpc, h_out;
  std::vector<double> h_post;
  int D = 0, K = 0, M = 0, m = 0, n1 = 0, n2 = 0, rounds = 0, reps = 0;
  long long max_batch = 0;
  DevBuf mp, mr, k53, a_rp, a_ci, f_rp, f_ci;  // mechanism rows, thresholds, [Hs; L1], [h2; L2]
  DevBuf skipT;                                // [M][64] geometric-skip thresholds ceil(2^53 (1 - p_j)^k)
  int sampler = 1;                             // 1 = geometric skip (default), 0 = keyed per (sample, mechanism)
  DevBuf DO, acc, failw, synd1, corr1, synd2, corr2, bpcorr2, post2, iters, conv;
};

namespace {

int upload_i32(DevBuf& b, const std::vector<int32_t>& v) {
  int rc = b.alloc(std::max<size_t>(4, v.size() * 4));
  if (rc) return rc;
  if (!v.empty() && hipMemcpy(b.p, v.data(), v.size() * 4, hipMemcpyHostToDevice) != hipSuccess)
    return set_err(QLDPC_EHIP, "hipMemcpy of a circuit table failed");
  return 0;
}

// rows of A then rows of B (same column count) as one CSR
void stack_csr(const qldpc_graph* A, const qldpc_graph* B, std::vector<int32_t>& rp, std::vector<int32_t>& ci) {
  rp.assign(1, 0);
  ci.clear();
  for (const qldpc_graph* g : {A, B}) {
    if (!g) continue;
    for (int r = 0; r < g->m; ++r) {
      for (int e = g->row_ptr[r]; e < g->row_ptr[r + 1]; ++e) ci.push_back(g->col_idx[e]);
      rp.push_back((int32_t)ci.size());
    }
  }
}

// the final layer's OSD through a host stage: D2H of the layer's syndromes, posteriors, BP
// corrections and convergence flags, qldpc_osd_decode_batch, H2D of the osdw corrections
int circ_host_osd(qldpc_circ* c, long long B, hipStream_t st) {
  const size_t m = (size_t)c->m, n2 = (size_t)c->n2;
  c->h_synd.resize((size_t)B * m);
  c->h_post.resize((size_t)B * n2);
  c->h_bpc.resize((size_t)B * n2);
  c->h_conv.resize((size_t)B);
  c->h_out.resize((size_t)B * n2);
  QLDPC_HIP(hipMemcpyAsync(c->h_synd.data(), c->synd2.p, (size_t)B * m, hipMemcpyDeviceToHost, st));
  QLDPC_HIP(hipMemcpyAsync(c->h_post.data(), c->post2.p, (size_t)B * n2 * 8, hipMemcpyDeviceToHost, st));
  QLDPC_HIP(hipMemcpyAsync(c->h_bpc.data(), c->bpcorr2.p, (size_t)B * n2, hipMemcpyDeviceToHost, st));
  QLDPC_HIP(hipMemcpyAsync(c->h_conv.data(), c->conv.p, (size_t)B, hipMemcpyDeviceToHost, st));
  QLDPC_HIP(hipStreamSynchronize(st));
  const int rc = qldpc_osd_decode_batch(c->osd_host, c->h_synd.data(), c->h_post.data(), c->h_conv.data(),
                                        c->h_bpc.data(), nullptr, c->h_out.data(), B, 0);
  if (rc) return rc;
  QLDPC_HIP(hipMemcpyAsync(c->corr2.p, c->h_out.data(), (size_t)B * n2, hipMemcpyHostToDevice, st));
  // the host buffer is reused by the next batch: wait for the copy to land
  QLDPC_HIP(hipStreamSynchronize(st));
  return 0;
}

// (1)-(2) of one batch: the geometric-skip sampler (default) or the keyed one (qldpc_circ_set_sampler)
int circ_sample_launch(qldpc_circ* c, uint64_t seed, u64 shot0, long long B, int W, u64* DO, hipStream_t st) {
  const unsigned gy = (unsigned)std::min(c->M, 65535);
  if (c->sampler == 1)
    hipLaunchKernelGGL(cs_sample_skip, dim3((unsigned)((W + kTileC - 1) / kTileC), gy), dim3(kTileC), 0, st,
                       static_cast<const int32_t*>(c->mp.p), static_cast<const int32_t*>(c->mr.p),
                       static_cast<const u64*>(c->skipT.p), c->M, (u64)seed, shot0, B, W, DO);
  else
    hipLaunchKernelGGL(cs_sample, dim3((unsigned)((B + kTileC - 1) / kTileC), gy), dim3(kTileC), 0, st,
                       static_cast<const int32_t*>(c->mp.p), static_cast<const int32_t*>(c->mr.p),
                       static_cast<const u64*>(c->k53.p), c->M, (u64)seed, shot0, B, W, DO);
  QLDPC_HIP(hipGetLastError());
  return 0;
}

void circ_release(qldpc_circ* c) {
  if (c->osd_owned) qldpc_osd_gpu_destroy(c->osd_owned);
  c->osd_owned = nullptr;
  for (DevBuf* b : {&c->mp, &c->mr, &c->k53, &c->skipT, &c->a_rp, &c->a_ci, &c->f_rp, &c->f_ci, &c->DO, &c->acc, &c->failw,
                    &c->synd1, &c->corr1, &c->synd2, &c->corr2, &c->bpcorr2, &c->post2, &c->iters, &c->conv})
    b->release();
}

}  // namespace

extern "C" {

int qldpc_circ_create(const qldpc_graph* dem, const qldpc_graph* dem_obs, const double* probs, qldpc_bp* dec1,
                      const qldpc_graph* h1_space_cor, const qldpc_graph* L1, qldpc_bp* dec2, const qldpc_graph* L2,
                      int32_t num_rounds, int32_t num_rep, int64_t max_batch, qldpc_circ** out) {
  if (!out || !dem || !dem_obs || !probs) return set_err(QLDPC_EINVAL, "NULL argument");
  // no decoders at all: a sampler-only handle (qldpc_circ_sample) for decoders outside the engine
  const bool sampler_only = !dec1 && !dec2;
  if (!sampler_only && (!dec1 || !h1_space_cor || !L1 || !dec2 || !L2)) return set_err(QLDPC_EINVAL, "NULL argument");
  if (num_rounds < 0 || num_rep < 1) return set_err(QLDPC_EINVAL, "num_rounds must be >= 0 and num_rep >= 1");
  const int M = dem->n, D = dem->m, K = dem_obs->m;
  if (dem_obs->n != M) return set_err(QLDPC_EINVAL, "DEM detector and observable matrices differ in mechanism count");
  const int m = sampler_only ? 0 : dec2->g->m, n1 = sampler_only ? 0 : dec1->g->n, n2 = sampler_only ? 0 : dec2->g->n;
  if (!sampler_only) {
    if (dec1->g->m != num_rep * m) return set_err(QLDPC_EINVAL, "decoder1's h1 must have num_rep * m rows");
    if (D != (num_rounds * num_rep + 1) * m)
      return set_err(QLDPC_EINVAL, "DEM detectors != (num_rounds * num_rep + 1) * m (num_cycles syndrome layers)");
    if (h1_space_cor->m != m || h1_space_cor->n != n1 || L1->n != n1 || L1->m != K || L2->n != n2 || L2->m != K)
      return set_err(QLDPC_EINVAL, "h1_space_cor / L1 / L2 shapes do not match the decoders and the DEM");
    if (dec2->g->device != dec1->g->device) return set_err(QLDPC_EINVAL, "decoders on different devices");
  }
  for (int j = 0; j < M; ++j)
    if (!(probs[j] >= 0.0 && probs[j] <= 1.0)) return set_err(QLDPC_EINVAL, "mechanism probability outside [0, 1]");
  const int dev = sampler_only ? dem->device : dec1->g->device;
  QLDPC_HIP(hipSetDevice(dev));
  auto* c = new qldpc_circ();
  c->device = dev;
  c->dec1 = dec1;
  c->dec2 = dec2;
  c->D = D;
  c->K = K;
  c->M = M;
  c->m = m;
  c->n1 = n1;
  c->n2 = n2;
  c->rounds = num_rounds;
  c->reps = num_rep;
  if (max_batch <= 0) max_batch = 1 << 16;
  c->max_batch = std::max<long long>(64, (max_batch + 63) / 64 * 64);
  auto fail = [&](int rc) {
    circ_release(c);
    delete c;
    return rc;
  };
  // mechanism -> rows (detectors 0..D-1, observables D..D+K-1), ascending
  std::vector<std::vector<int32_t>> rows(M);
  for (int r = 0; r < D; ++r)
    for (int e = dem->row_ptr[r]; e < dem->row_ptr[r + 1]; ++e) rows[dem->col_idx[e]].push_back(r);
  for (int k = 0; k < K; ++k)
    for (int e = dem_obs->row_ptr[k]; e < dem_obs->row_ptr[k + 1]; ++e) rows[dem_obs->col_idx[e]].push_back(D + k);
  std::vector<int32_t> mp(1, 0), mr;
  for (int j = 0; j < M; ++j) {
    mr.insert(mr.end(), rows[j].begin(), rows[j].end());
    mp.push_back((int32_t)mr.size());
  }
  std::vector<u64> k53(std::max(1, M));
  for (int j = 0; j < M; ++j) k53[j] = ceil53c(probs[j]);
  std::vector<u64> skipT((size_t)std::max(1, M) * 64);
  for (int j = 0; j < M; ++j) {
    const double q = 1.0 - probs[j];
    double t = 1.0;
    for (int k = 0; k < 64; ++k) {
      t *= q;  // (1 - p)^(k + 1), the same IEEE products as the oracle's
      skipT[(size_t)j * 64 + k] = ceil53c(t);
    }
  }
  std::vector<int32_t> arp, aci, frp, fci;
  if (!sampler_only) {
    stack_csr(h1_space_cor, L1, arp, aci);
    stack_csr(dec2->g, L2, frp, fci);
  }
  int rc;
  if ((rc = upload_i32(c->mp, mp)) || (rc = upload_i32(c->mr, mr)) || (rc = upload_i32(c->a_rp, arp)) ||
      (rc = upload_i32(c->a_ci, aci)) || (rc = upload_i32(c->f_rp, frp)) || (rc = upload_i32(c->f_ci, fci)) ||
      (rc = c->k53.alloc(k53.size() * 8)) || (rc = c->skipT.alloc(skipT.size() * 8)))
    return fail(rc);
  if (hipMemcpy(c->k53.p, k53.data(), k53.size() * 8, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(c->skipT.p, skipT.data(), skipT.size() * 8, hipMemcpyHostToDevice) != hipSuccess)
    return fail(set_err(QLDPC_EHIP, "hipMemcpy of the mechanism thresholds failed"));
  const size_t B = (size_t)c->max_batch, W = B / 64;
  if ((rc = c->DO.alloc((size_t)(D + K) * W * 8)) || (rc = c->acc.alloc((size_t)(m + K) * W * 8)) ||
      (rc = c->failw.alloc(W * 8)) || (rc = c->synd1.alloc((size_t)num_rep * m * B)) ||
      (rc = c->corr1.alloc((size_t)n1 * B)) || (rc = c->synd2.alloc((size_t)m * B)) ||
      (rc = c->corr2.alloc((size_t)n2 * B)) || (rc = c->iters.alloc(B * 4)) || (rc = c->conv.alloc(B)))
    return fail(rc);
  *out = c;
  return 0;
}

int qldpc_circ_set_final_osd(qldpc_circ* c, qldpc_osd_gpu* osd_gpu, const qldpc_osd* osd_host) {
  if (!c) return set_err(QLDPC_EINVAL, "NULL circuit handle");
  if (!c->dec2) return set_err(QLDPC_EINVAL, "sampler-only circuit handle has no decoder2");
  if (osd_gpu && osd_host) return set_err(QLDPC_EINVAL, "give the GPU OSD or the host OSD stage, not both");
  if (osd_gpu || osd_host) {
    int32_t eng = 0;
    qldpc_bp_engine(c->dec2, &eng);
    if (eng != 1) return set_err(QLDPC_ENOTSUP, "BP+OSD decoder2 needs qldpc_bp_create_soft");
    if (osd_gpu && !osd_gpu_matches(osd_gpu, c->dec2->g))
      return set_err(QLDPC_EINVAL, "GPU OSD handle was built on a different graph than decoder2");
    if (osd_host && !osd_host_matches(osd_host, c->dec2->g))
      return set_err(QLDPC_EINVAL, "host OSD stage was built on a different graph than decoder2");
    QLDPC_HIP(hipSetDevice(c->device));
    int rc;
    if (!c->post2.p && ((rc = c->post2.alloc((size_t)c->max_batch * c->n2 * 8)) ||
                        (rc = c->bpcorr2.alloc((size_t)c->max_batch * c->n2))))
      return rc;
  }
  // a host stage runs on the GPU too (its method, order, rank and soft weights): the launch never
  // leaves the device.  Past the GPU kernel's envelope it stays a host stage (one D2H / H2D round
  // trip per batch of the final layer).
  qldpc_osd_gpu* own = nullptr;
  const qldpc_osd* keep_host = nullptr;
  if (osd_host) {
    // (QLDPC_CIRC_HOST_OSD=1 keeps any host stage on the host: the test hook of that branch, whose
    // natural trigger, n > 8192 mechanisms in h2, is too large a circuit for a unit test)
    const char* ho = std::getenv("QLDPC_CIRC_HOST_OSD");
    const int rc = (ho && std::atoi(ho) == 1) ? QLDPC_ENOTSUP : osd_gpu_from_host(c->dec2->g, osd_host, &own);
    if (rc == QLDPC_ENOTSUP) {
      own = nullptr;
      keep_host = osd_host;
    } else if (rc) {
      return rc;
    }
  }
  if (c->osd_owned) qldpc_osd_gpu_destroy(c->osd_owned);
  c->osd_owned = own;
  c->osd_gpu = osd_gpu ? osd_gpu : own;
  c->osd_host = keep_host;
  return 0;
}

int qldpc_circ_set_sampler(qldpc_circ* c, int32_t sampler) {
  if (!c) return set_err(QLDPC_EINVAL, "NULL circuit handle");
  if (sampler != 0 && sampler != 1) return set_err(QLDPC_EINVAL, "sampler must be 0 (keyed) or 1 (geometric skip)");
  c->sampler = sampler;
  return 0;
}

int qldpc_circ_destroy(qldpc_circ* c) {
  if (!c) return 0;
  (void)hipSetDevice(c->device);
  circ_release(c);
  delete c;
  return 0;
}

int qldpc_circ_info(const qldpc_circ* c, int32_t* detectors, int32_t* observables, int32_t* mechanisms) {
  if (!c) return set_err(QLDPC_EINVAL, "NULL circuit handle");
  if (detectors) *detectors = c->D;
  if (observables) *observables = c->K;
  if (mechanisms) *mechanisms = c->M;
  return 0;
}

// The sampling step alone (stim's compile_detector_sampler().sample(shots, append_observables=True),
// src/Simulators_SpaceTime.py:940, :1029): d_out [S][D + K] detector then observable bits, the
// same draws as qldpc_circ_launch's samples.
int qldpc_circ_sample(qldpc_circ* c, uint64_t seed, uint64_t shot_begin, int64_t shot_count, uint8_t* d_out,
                      void* stream) {
  if (!c || !d_out) return set_err(QLDPC_EINVAL, "NULL argument");
  if (shot_count <= 0) return 0;
  QLDPC_HIP(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  auto* DO = static_cast<u64*>(c->DO.p);
  const int DK = c->D + c->K;
  for (long long c0 = 0; c0 < shot_count; c0 += c->max_batch) {
    const long long B = std::min<long long>(c->max_batch, shot_count - c0);
    const int W = (int)((B + 63) / 64);
    QLDPC_HIP(hipMemsetAsync(DO, 0, (size_t)DK * W * 8, st));
    if (c->M > 0) {
      const int rc = circ_sample_launch(c, seed, (u64)(shot_begin + c0), B, W, DO, st);
      if (rc) return rc;
    }
    hipLaunchKernelGGL(cs_unpack, dim3((unsigned)((DK + kTileC - 1) / kTileC), (unsigned)W), dim3(kTileC), 0, st, DO,
                       static_cast<const u64*>(c->acc.p), 0, DK, 0, d_out + c0 * (long long)DK, W, B);
    QLDPC_HIP(hipGetLastError());
  }
  return 0;
}

int qldpc_circ_launch(qldpc_circ* c, uint64_t seed, uint64_t shot_begin, int64_t shot_count, void* d_counters,
                      uint8_t* d_fail, uint8_t* d_detobs, void* stream) {
  if (!c || !d_counters) return set_err(QLDPC_EINVAL, "NULL argument");
  if (!c->dec1) return set_err(QLDPC_EINVAL, "sampler-only circuit handle: qldpc_circ_launch needs the decoders");
  if (shot_count <= 0) return 0;
  QLDPC_HIP(hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  auto* cnt = static_cast<u64*>(d_counters);
  auto* DO = static_cast<u64*>(c->DO.p);
  auto* acc = static_cast<u64*>(c->acc.p);
  const int m = c->m, K = c->K, D = c->D, R1 = c->reps * m;
  for (long long c0 = 0; c0 < shot_count; c0 += c->max_batch) {
    const long long B = std::min<long long>(c->max_batch, shot_count - c0);
    const int W = (int)((B + 63) / 64);
    QLDPC_HIP(hipMemsetAsync(DO, 0, (size_t)(D + K) * W * 8, st));
    QLDPC_HIP(hipMemsetAsync(acc, 0, (size_t)(m + K) * W * 8, st));
    QLDPC_HIP(hipMemsetAsync(c->failw.p, 0, (size_t)W * 8, st));
    // (1)-(2) sample the mechanisms, scatter into the detector / observable words
    if (c->M > 0) {
      const int rc = circ_sample_launch(c, seed, (u64)(shot_begin + c0), B, W, DO, st);
      if (rc) return rc;
    }
    if (d_detobs) {
      hipLaunchKernelGGL(cs_unpack, dim3((unsigned)((D + K + kTileC - 1) / kTileC), (unsigned)W), dim3(kTileC), 0, st,
                         DO, acc, 0, D + K, 0, d_detobs + c0 * (long long)(D + K), W, B);
      QLDPC_HIP(hipGetLastError());
    }
    // (3) the noisy rounds: decoder1 on h1, space / logical corrections accumulated
    for (int r = 0; r < c->rounds; ++r) {
      hipLaunchKernelGGL(cs_unpack, dim3((unsigned)((R1 + kTileC - 1) / kTileC), (unsigned)W), dim3(kTileC), 0, st,
                         DO, acc, r * R1, R1, m, static_cast<uint8_t*>(c->synd1.p), W, B);
      QLDPC_HIP(hipGetLastError());
      int rc = qldpc_bp_decode_batch(c->dec1, static_cast<const uint8_t*>(c->synd1.p), static_cast<uint8_t*>(c->corr1.p),
                                     static_cast<int32_t*>(c->iters.p), static_cast<uint8_t*>(c->conv.p), B, stream);
      if (rc) return rc;
      hipLaunchKernelGGL(cs_iters, dim3(iters_grid(B)), dim3(kTileC), 0, st,
                         static_cast<const int32_t*>(c->iters.p), static_cast<const uint8_t*>(c->conv.p), cnt, 0, B);
      QLDPC_HIP(hipGetLastError());
      hipLaunchKernelGGL(cs_apply, dim3((unsigned)((B + kTileC - 1) / kTileC)), dim3(kTileC), 0, st,
                         static_cast<const int32_t*>(c->a_rp.p), static_cast<const int32_t*>(c->a_ci.p), m + K,
                         static_cast<const uint8_t*>(c->corr1.p), c->n1, acc, W, B);
      QLDPC_HIP(hipGetLastError());
    }
    // (4) the final layer: decoder2 on h2
    const int fin0 = c->rounds * R1;
    hipLaunchKernelGGL(cs_unpack, dim3((unsigned)((m + kTileC - 1) / kTileC), (unsigned)W), dim3(kTileC), 0, st, DO,
                       acc, fin0, m, m, static_cast<uint8_t*>(c->synd2.p), W, B);
    QLDPC_HIP(hipGetLastError());
    int rc;
    auto* synd2 = static_cast<const uint8_t*>(c->synd2.p);
    auto* corr2 = static_cast<uint8_t*>(c->corr2.p);
    if (c->osd_gpu) {  // bposd_decoder: BP, then OSD where BP did not converge (GPU OSD, any priors)
      rc = qldpc_bp_decode_batch_soft(c->dec2, synd2, static_cast<uint8_t*>(c->bpcorr2.p),
                                      static_cast<int32_t*>(c->iters.p), static_cast<uint8_t*>(c->conv.p),
                                      static_cast<double*>(c->post2.p), B, stream);
      if (!rc)
        rc = qldpc_osd_gpu_decode(c->osd_gpu, synd2, static_cast<const double*>(c->post2.p),
                                  static_cast<const uint8_t*>(c->conv.p), static_cast<const uint8_t*>(c->bpcorr2.p),
                                  nullptr, corr2, B, stream);
    } else if (c->osd_host) {  // host OSD stage: soft BP on the device, OSD on the host, corr2 back
      rc = qldpc_bp_decode_batch_soft(c->dec2, synd2, static_cast<uint8_t*>(c->bpcorr2.p),
                                      static_cast<int32_t*>(c->iters.p), static_cast<uint8_t*>(c->conv.p),
                                      static_cast<double*>(c->post2.p), B, stream);
      if (!rc) rc = circ_host_osd(c, B, st);
    } else {
      rc = qldpc_bp_decode_batch(c->dec2, synd2, corr2, static_cast<int32_t*>(c->iters.p),
                                 static_cast<uint8_t*>(c->conv.p), B, stream);
    }
    if (rc) return rc;
    hipLaunchKernelGGL(cs_iters, dim3(iters_grid(B)), dim3(kTileC), 0, st,
                       static_cast<const int32_t*>(c->iters.p), static_cast<const uint8_t*>(c->conv.p), cnt, 1, B);
    QLDPC_HIP(hipGetLastError());
    // (5) residual syndrome / logicals -> failures
    hipLaunchKernelGGL(cs_final, dim3((unsigned)((B + kTileC - 1) / kTileC)), dim3(kTileC), 0, st,
                       static_cast<const int32_t*>(c->f_rp.p), static_cast<const int32_t*>(c->f_ci.p), corr2, c->n2, DO,
                       fin0, D, acc, m, K, static_cast<u64*>(c->failw.p), W, B);
    QLDPC_HIP(hipGetLastError());
    hipLaunchKernelGGL(cs_tally, dim3((unsigned)((W + kTileC - 1) / kTileC)), dim3(kTileC), 0, st,
                       static_cast<const u64*>(c->failw.p), cnt, d_fail, c0, W, B);
    QLDPC_HIP(hipGetLastError());
  }
  return 0;
}

}  // extern "C"
