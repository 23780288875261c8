// firstmin.hip — FirstMinBPDecoder (src/Decoders.py:49-74) on the device.
//
// The reference repeats a ONE-iteration min-sum BP (ldpc bp_decoder, max_iter = 1) on the running
// syndrome while the residual syndrome weight does not grow:
//
//   new = BP1(cur); ns = H new + cur;  while |ns| <= |cur| and k < max_iter: cur = ns, x ^= new, k++, ...
//
// A one-iteration min-sum from fresh state only ever sees the channel priors as bit-to-check
// messages, so its check-to-bit magnitudes (alpha x the minimum |prior| over the row's other edges)
// and their prior-sign parities are fixed per edge; only the syndrome signs change from step to
// step.  The host computes them once, in the oracle's precision and operation order
// (oracle/qldpc_oracle.c bp_ms: SENTINEL minimum, c2b = min * (+-alpha)); a step is then, per
// variable, prior + the signed magnitudes of its edges in column order (the same adds as ldpc's
// variable pass) and the decision post <= 0, then H d + cur and its weight.  One workgroup per
// syndrome (persistent), the running syndrome / decision / correction in LDS, the whole loop on the
// device: no host round trip per first-min step (round 4 ran one engine launch per step and
// compared the weights on the host).  Once the running syndrome is zero and BP1(0) decides nothing
// (positive priors), every remaining step would accept an empty correction: the loop stops there
// with the step count the reference reaches (max_iter).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <vector>

#include "runtime.h"

using qldpc_rt::set_err;

struct qldpc_firstmin {
  int device = 0, m = 0, n = 0, E = 0, max_iter = 0, precision = 64, grid = 0;
  size_t lds = 0;
  qldpc_rt::DevBuf rp, ci;      // CSR: H d
  qldpc_rt::DevBuf cp, crow;    // CSC in column order (rows ascending): col_ptr [n + 1], row [E]
  qldpc_rt::DevBuf csb, cmag;   // per CSC entry: prior-sign parity of the row's other edges (u8), |c2b| (T)
  qldpc_rt::DevBuf prior;       // [n] T
  std::vector<int32_t> row_ptr, col_idx;  // the graph it was built on (qldpc_phenl_set_round_firstmin checks it)
  qldpc_rt::DevBuf colm;  // m <= 64: [n] u64 row mask of each column (the one-iteration thread-per-syndrome kernel)
};

bool qldpc_rt::firstmin_matches(const qldpc_firstmin* fm, const qldpc_graph* g) {
  return fm && g && fm->device == g->device && fm->m == g->m && fm->n == g->n && fm->row_ptr == g->row_ptr &&
         fm->col_idx == g->col_idx;
}

namespace {

constexpr int kFmThreads = 256;

struct FmArgs {
  const int32_t* rp;
  const int32_t* ci;
  const int32_t* cp;
  const int32_t* crow;
  const uint8_t* csb;
  const void* cmag;
  const void* prior;
  const uint8_t* synd;  // [B][m]
  uint8_t* corr;        // [B][n]
  int32_t* steps;       // [B] or null (BP1: iterations)
  uint8_t* conv;        // BP1: [B] or null
  long long B;
  int m, n, max_iter;
};

// BP1: one step only -- the one-iteration BP's decision, iterations 1, converged iff H d == s
template <typename T, bool BP1 = false>
__global__ void __launch_bounds__(kFmThreads) firstmin_kernel(FmArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  const int tid = threadIdx.x, TB = blockDim.x, m = a.m, n = a.n;
  uint8_t* cur = sm;       // [m] running syndrome
  uint8_t* nsy = cur + m;  // [m] H new + cur
  uint8_t* dec = nsy + m;  // [n] this step's BP decision
  uint8_t* cor = dec + n;  // [n] accepted correction
  __shared__ int s_w, s_any;
  const T* mag = static_cast<const T*>(a.cmag);
  const T* prior = static_cast<const T*>(a.prior);
  // one first-min step on cur: dec = BP1(cur), nsy = H dec + cur; returns |nsy| (uniform)
  auto step = [&]() -> int {
    if (tid == 0) {
      s_w = 0;
      s_any = 0;
    }
    __syncthreads();
    bool any = false;
    for (int j = tid; j < n; j += TB) {
      T post = prior[j];
      for (int k = a.cp[j]; k < a.cp[j + 1]; ++k) {
        const T c = mag[k];
        post += ((cur[a.crow[k]] ^ a.csb[k]) & 1u) ? -c : c;
      }
      dec[j] = post <= (T)0 ? 1 : 0;
      any = any || post <= (T)0;
    }
    if (any) s_any = 1;
    __syncthreads();
    int w = 0;
    for (int i = tid; i < m; i += TB) {
      uint8_t x = cur[i];
      for (int e = a.rp[i]; e < a.rp[i + 1]; ++e) x ^= dec[a.ci[e]];
      nsy[i] = x;
      w += x;
    }
    if (w) atomicAdd(&s_w, w);
    __syncthreads();
    const int r = s_w;
    __syncthreads();  // s_w is rewritten by the next step
    return r;
  };
  for (long long b = blockIdx.x; b < a.B; b += gridDim.x) {
    const uint8_t* sy = a.synd + b * (long long)m;
    if (tid == 0) s_w = 0;
    __syncthreads();
    int w = 0;
    for (int i = tid; i < m; i += TB) {
      const uint8_t x = sy[i] & 1u;
      cur[i] = x;
      w += x;
    }
    for (int j = tid; j < n; j += TB) cor[j] = 0;
    if (w) atomicAdd(&s_w, w);
    __syncthreads();
    int wc = s_w;  // |cur| (uniform)
    __syncthreads();
    int k = 0;
    int wn = step();
    if (BP1) {
      uint8_t* out = a.corr + b * (long long)n;
      for (int j = tid; j < n; j += TB) out[j] = dec[j];
      if (tid == 0) {
        if (a.steps) a.steps[b] = 1;
        if (a.conv) a.conv[b] = wn == 0 ? 1 : 0;
      }
      __syncthreads();
      continue;
    }
    while (wn <= wc && k < a.max_iter) {  // uniform
      if (wc == 0 && !s_any) {  // cur = 0 and BP1(0) = 0: every remaining step accepts nothing
        k = a.max_iter;
        break;
      }
      for (int i = tid; i < m; i += TB) cur[i] = nsy[i];
      for (int j = tid; j < n; j += TB) cor[j] ^= dec[j];
      ++k;
      wc = wn;
      __syncthreads();
      wn = step();
    }
    uint8_t* out = a.corr + b * (long long)n;
    for (int j = tid; j < n; j += TB) out[j] = cor[j];
    if (tid == 0 && a.steps) a.steps[b] = k;
    __syncthreads();  // LDS reused by the next syndrome
  }
}

// One-iteration BP for graphs of <= 64 checks (the circuit loop's h1: 27 x 153): one THREAD per
// syndrome, the syndrome and its residual as 64-bit masks in registers, the tables walked in the
// same (uniform) order by every lane (scalar / broadcast loads).  The workgroup-per-syndrome kernel
// above spends its time in barriers on such graphs (0.20 ms per 65,536 syndromes against the
// engine's 0.18).  Same adds in the same order: identical decisions.
// One WAVE per syndrome (4 per 256-thread workgroup), no workgroup barrier: a wave's LDS accesses
// are processed in order, so the running syndrome / decision arrays only need the compiler fence
// between a wave's writes and its other lanes' reads; the weights are wave sums.  Same steps, same
// arithmetic as firstmin_kernel.
__device__ inline int wave_sum_i32(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
#define FM_WAVE_FENCE() __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront")

template <typename T>
__global__ void __launch_bounds__(256) firstmin_wave_kernel(FmArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, m = a.m, n = a.n;
  const size_t per = ((size_t)2 * m + (size_t)2 * n + 15) & ~(size_t)15;
  uint8_t* cur = sm + (size_t)wv * per;
  uint8_t* nsy = cur + m;
  uint8_t* dec = nsy + m;
  uint8_t* cor = dec + n;
  const T* mag = static_cast<const T*>(a.cmag);
  const T* prior = static_cast<const T*>(a.prior);
  auto step = [&]() -> int {
    for (int j = lane; j < n; j += 64) {
      T post = prior[j];
      for (int k = a.cp[j]; k < a.cp[j + 1]; ++k) {
        const T c = mag[k];
        post += ((cur[a.crow[k]] ^ a.csb[k]) & 1u) ? -c : c;
      }
      dec[j] = post <= (T)0 ? 1 : 0;
    }
    FM_WAVE_FENCE();
    int w = 0;
    for (int i = lane; i < m; i += 64) {
      uint8_t x = cur[i];
      for (int e = a.rp[i]; e < a.rp[i + 1]; ++e) x ^= dec[a.ci[e]];
      nsy[i] = x;
      w += x;
    }
    FM_WAVE_FENCE();
    return wave_sum_i32(w);
  };
  const long long nw = (long long)gridDim.x * 4;
  for (long long b = (long long)blockIdx.x * 4 + wv; b < a.B; b += nw) {  // uniform per wave
    const uint8_t* sy = a.synd + b * (long long)m;
    int w = 0;
    for (int i = lane; i < m; i += 64) {
      const uint8_t x = sy[i] & 1u;
      cur[i] = x;
      w += x;
    }
    for (int j = lane; j < n; j += 64) cor[j] = 0;
    FM_WAVE_FENCE();
    int wc = wave_sum_i32(w);
    int k = 0;
    int wn = step();
    while (wn <= wc && k < a.max_iter) {  // uniform per wave
      if (wc == 0) {  // cur = 0: does BP1(0) decide anything?
        int any = 0;
        for (int j = lane; j < n; j += 64) any |= dec[j];
        if (!__any(any)) {
          k = a.max_iter;
          break;
        }
      }
      for (int i = lane; i < m; i += 64) cur[i] = nsy[i];
      for (int j = lane; j < n; j += 64) cor[j] ^= dec[j];
      ++k;
      wc = wn;
      FM_WAVE_FENCE();
      wn = step();
    }
    uint8_t* out = a.corr + b * (long long)n;
    for (int j = lane; j < n; j += 64) out[j] = cor[j];
    if (lane == 0 && a.steps) a.steps[b] = k;
    FM_WAVE_FENCE();
  }
}

// STG: the workgroup's 256 syndromes and decisions staged through LDS (coalesced global reads and
// writes of its contiguous [256][m] / [256][n] blocks) when 256 (m + n) bytes fit
template <typename T, bool STG>
__global__ void __launch_bounds__(256) bp1_small_kernel(FmArgs a, const unsigned long long* __restrict__ colm) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  const int m = a.m, n = a.n, tid = threadIdx.x;
  const long long b0 = (long long)blockIdx.x * 256, b = b0 + tid;
  const int nb = (int)(a.B - b0 < 256 ? a.B - b0 : 256);
  uint8_t* ssy = sm;                        // [256][m]
  uint8_t* sdc = sm + (size_t)256 * m;      // [256][n]
  if (STG) {
    for (int t = tid; t < nb * m; t += 256) ssy[t] = a.synd[b0 * m + t];
    __syncthreads();
  }
  const T* mag = static_cast<const T*>(a.cmag);
  const T* prior = static_cast<const T*>(a.prior);
  if (b < a.B) {
    const uint8_t* sy = STG ? ssy + (size_t)tid * m : a.synd + b * (long long)m;
    unsigned long long cur = 0;
    for (int i = 0; i < m; ++i) cur |= (unsigned long long)(sy[i] & 1u) << i;
    unsigned long long ns = cur;
    uint8_t* out = STG ? sdc + (size_t)tid * n : a.corr + b * (long long)n;
    for (int j = 0; j < n; ++j) {
      T post = prior[j];
      for (int k = a.cp[j]; k < a.cp[j + 1]; ++k) {
        const T c = mag[k];
        post += (((cur >> a.crow[k]) ^ a.csb[k]) & 1ull) ? -c : c;
      }
      const bool d = post <= (T)0;
      out[j] = d ? 1 : 0;
      ns ^= d ? colm[j] : 0ull;
    }
    if (a.steps) a.steps[b] = 1;
    if (a.conv) a.conv[b] = ns == 0 ? 1 : 0;
  }
  if (STG) {
    __syncthreads();
    for (int t = tid; t < nb * n; t += 256) a.corr[b0 * n + t] = sdc[t];
  }
}

// per-edge one-iteration check-to-bit magnitudes and prior-sign parities in precision T, as the
// oracle's bp_ms computes them in its first iteration (b2c = prior)
template <typename T>
void firstmin_tables(const qldpc_graph* g, const std::vector<double>& pr, double alpha_in, T sentinel,
                     std::vector<T>& prior, std::vector<T>& emag, std::vector<uint8_t>& esb) {
  const int m = g->m, n = g->n;
  prior.resize(n);
  for (int j = 0; j < n; ++j) prior[j] = (T)pr[j];
  const T alpha = (alpha_in == 0.0) ? (T)(1.0 - std::ldexp(1.0, -1)) : (T)alpha_in;
  emag.assign(g->col_idx.size(), (T)0);
  esb.assign(g->col_idx.size(), 0);
  for (int i = 0; i < m; ++i) {
    const int e0 = g->row_ptr[i], e1 = g->row_ptr[i + 1];
    for (int e = e0; e < e1; ++e) {
      T mn = sentinel;
      int s = 0;
      for (int f = e0; f < e1; ++f) {
        if (f == e) continue;
        const T b2c = prior[g->col_idx[f]];
        const T aa = std::fabs(b2c);
        if (aa < mn) mn = aa;
        if (b2c <= (T)0) s += 1;
      }
      emag[e] = mn * alpha;
      esb[e] = (uint8_t)(s & 1);
    }
  }
}

}  // namespace

extern "C" {

int qldpc_firstmin_create(const qldpc_graph* g, const double* channel_probs, int32_t max_iter,
                          double ms_scaling_factor, int32_t precision, qldpc_firstmin** out) {
  if (!g || !channel_probs || !out) return set_err(QLDPC_EINVAL, "NULL argument");
  if (precision != 32 && precision != 64) return set_err(QLDPC_EINVAL, "precision must be 32 or 64");
  const int m = g->m, n = g->n, E = (int)g->col_idx.size();
  const size_t lds = (size_t)2 * m + (size_t)2 * n;
  if (lds > 64 * 1024) return set_err(QLDPC_ENOTSUP, "first-min decoder: 2 (m + n) bytes of LDS > 64 KiB");
  std::vector<double> pr(n);
  for (int j = 0; j < n; ++j) {
    const double p = channel_probs[j];
    if (!(p > 0.0 && p < 1.0)) return set_err(QLDPC_EINVAL, "channel_probs must lie in (0, 1)");
    pr[j] = std::log((1.0 - p) / p);  // ldpc's channel LLR, double libm (as the oracle)
  }
  // CSC in column order: rows ascending (ldpc's column lists), each entry's CSR edge
  std::vector<int32_t> cp(n + 1, 0), crow(E), cedge(E);
  for (int e = 0; e < E; ++e) cp[g->col_idx[e] + 1] += 1;
  for (int j = 0; j < n; ++j) cp[j + 1] += cp[j];
  {
    std::vector<int32_t> fill(cp.begin(), cp.end() - 1);
    for (int i = 0; i < m; ++i)
      for (int e = g->row_ptr[i]; e < g->row_ptr[i + 1]; ++e) {
        const int j = g->col_idx[e];
        crow[fill[j]] = i;
        cedge[fill[j]++] = e;
      }
  }
  auto* F = new qldpc_firstmin();
  F->device = g->device;
  F->m = m;
  F->n = n;
  F->E = E;
  F->max_iter = max_iter > 0 ? max_iter : 0;
  F->precision = precision;
  F->lds = lds;
  F->row_ptr = g->row_ptr;
  F->col_idx = g->col_idx;
  std::vector<unsigned long long> colm;
  if (m <= 64) {
    colm.assign(std::max(n, 1), 0ull);
    for (int i = 0; i < m; ++i)
      for (int e = g->row_ptr[i]; e < g->row_ptr[i + 1]; ++e) colm[g->col_idx[e]] ^= 1ull << i;
  }
  auto fail = [&](int code) {
    F->rp.release(); F->ci.release(); F->cp.release(); F->crow.release(); F->csb.release(); F->cmag.release();
    F->prior.release(); F->colm.release();
    delete F;
    return code;
  };
  if (hipSetDevice(g->device) != hipSuccess) return fail(set_err(QLDPC_EHIP, "hipSetDevice"));
  std::vector<uint8_t> esb, csb(E);
  const size_t ts = precision == 64 ? 8 : 4;
  std::vector<unsigned char> cmag((size_t)E * ts), prior((size_t)n * ts);
  if (precision == 64) {
    std::vector<double> p, em;
    firstmin_tables<double>(g, pr, ms_scaling_factor, 1e308, p, em, esb);
    for (int k = 0; k < E; ++k) reinterpret_cast<double*>(cmag.data())[k] = em[cedge[k]];
    std::copy(p.begin(), p.end(), reinterpret_cast<double*>(prior.data()));
  } else {
    std::vector<float> p, em;
    firstmin_tables<float>(g, pr, ms_scaling_factor, FLT_MAX, p, em, esb);
    for (int k = 0; k < E; ++k) reinterpret_cast<float*>(cmag.data())[k] = em[cedge[k]];
    std::copy(p.begin(), p.end(), reinterpret_cast<float*>(prior.data()));
  }
  for (int k = 0; k < E; ++k) csb[k] = esb[cedge[k]];
  int rc;
  if ((rc = F->rp.alloc((size_t)(m + 1) * 4)) || (rc = F->ci.alloc(std::max(E, 1) * (size_t)4)) ||
      (rc = F->cp.alloc((size_t)(n + 1) * 4)) || (rc = F->crow.alloc(std::max(E, 1) * (size_t)4)) ||
      (rc = F->csb.alloc(std::max(E, 1))) || (rc = F->cmag.alloc(std::max(E, 1) * ts)) ||
      (rc = F->prior.alloc(std::max(n, 1) * ts)) || (m <= 64 && (rc = F->colm.alloc(colm.size() * 8))))
    return fail(rc);
  if (m <= 64 && hipMemcpy(F->colm.p, colm.data(), colm.size() * 8, hipMemcpyHostToDevice) != hipSuccess)
    return fail(set_err(QLDPC_EHIP, "upload first-min column masks"));
  if (hipMemcpy(F->rp.p, g->row_ptr.data(), (size_t)(m + 1) * 4, hipMemcpyHostToDevice) != hipSuccess ||
      (E && hipMemcpy(F->ci.p, g->col_idx.data(), (size_t)E * 4, hipMemcpyHostToDevice) != hipSuccess) ||
      hipMemcpy(F->cp.p, cp.data(), (size_t)(n + 1) * 4, hipMemcpyHostToDevice) != hipSuccess ||
      (E && hipMemcpy(F->crow.p, crow.data(), (size_t)E * 4, hipMemcpyHostToDevice) != hipSuccess) ||
      (E && hipMemcpy(F->csb.p, csb.data(), (size_t)E, hipMemcpyHostToDevice) != hipSuccess) ||
      (E && hipMemcpy(F->cmag.p, cmag.data(), (size_t)E * ts, hipMemcpyHostToDevice) != hipSuccess) ||
      (n && hipMemcpy(F->prior.p, prior.data(), (size_t)n * ts, hipMemcpyHostToDevice) != hipSuccess))
    return fail(set_err(QLDPC_EHIP, "upload first-min tables"));
  int cus = 0, nb = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, g->device) != hipSuccess || cus <= 0)
    return fail(set_err(QLDPC_EHIP, "device CU count"));
  const void* kf = precision == 64 ? reinterpret_cast<const void*>(&firstmin_kernel<double>)
                                   : reinterpret_cast<const void*>(&firstmin_kernel<float>);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kf, kFmThreads, lds) != hipSuccess || nb <= 0) nb = 1;
  F->grid = cus * nb;
  *out = F;
  return 0;
}

}  // extern "C"

int qldpc_rt::bp1_decode(qldpc_firstmin* fm, const uint8_t* d_synd, uint8_t* d_corr, int32_t* d_iters, uint8_t* d_conv,
                         int64_t B, hipStream_t stream) {
  if (!fm || (B > 0 && (!d_synd || !d_corr))) return set_err(QLDPC_EINVAL, "NULL argument");
  if (B <= 0) return 0;
  FmArgs a;
  a.rp = static_cast<const int32_t*>(fm->rp.p);
  a.ci = static_cast<const int32_t*>(fm->ci.p);
  a.cp = static_cast<const int32_t*>(fm->cp.p);
  a.crow = static_cast<const int32_t*>(fm->crow.p);
  a.csb = static_cast<const uint8_t*>(fm->csb.p);
  a.cmag = fm->cmag.p;
  a.prior = fm->prior.p;
  a.synd = d_synd;
  a.corr = d_corr;
  a.steps = d_iters;
  a.conv = d_conv;
  a.B = B;
  a.m = fm->m;
  a.n = fm->n;
  a.max_iter = 0;
  if (fm->colm.p) {  // <= 64 checks: one thread per syndrome
    const unsigned g1 = (unsigned)((B + 255) / 256);
    const auto* cm = static_cast<const unsigned long long*>(fm->colm.p);
    const size_t sl = (size_t)256 * (fm->m + fm->n);
    const bool stg = sl <= 64 * 1024;
    if (fm->precision == 64) {
      if (stg) hipLaunchKernelGGL((bp1_small_kernel<double, true>), dim3(g1), dim3(256), sl, stream, a, cm);
      else hipLaunchKernelGGL((bp1_small_kernel<double, false>), dim3(g1), dim3(256), 0, stream, a, cm);
    } else {
      if (stg) hipLaunchKernelGGL((bp1_small_kernel<float, true>), dim3(g1), dim3(256), sl, stream, a, cm);
      else hipLaunchKernelGGL((bp1_small_kernel<float, false>), dim3(g1), dim3(256), 0, stream, a, cm);
    }
    QLDPC_HIP(hipGetLastError());
    return 0;
  }
  const int grid = (int)std::min<long long>(B, fm->grid);
  if (fm->precision == 64)
    hipLaunchKernelGGL((firstmin_kernel<double, true>), dim3(grid), dim3(kFmThreads), fm->lds, stream, a);
  else
    hipLaunchKernelGGL((firstmin_kernel<float, true>), dim3(grid), dim3(kFmThreads), fm->lds, stream, a);
  QLDPC_HIP(hipGetLastError());
  return 0;
}

extern "C" {

int qldpc_firstmin_destroy(qldpc_firstmin* fm) {
  if (!fm) return 0;
  fm->rp.release(); fm->ci.release(); fm->cp.release(); fm->crow.release(); fm->csb.release(); fm->cmag.release();
  fm->prior.release(); fm->colm.release();
  delete fm;
  return 0;
}

int qldpc_firstmin_decode(qldpc_firstmin* fm, const uint8_t* d_synd, uint8_t* d_corr, int32_t* d_steps, int64_t B,
                          void* stream) {
  if (!fm || (B > 0 && (!d_synd || !d_corr))) return set_err(QLDPC_EINVAL, "NULL argument");
  if (B <= 0) return 0;
  QLDPC_HIP(hipSetDevice(fm->device));
  FmArgs a;
  a.rp = static_cast<const int32_t*>(fm->rp.p);
  a.ci = static_cast<const int32_t*>(fm->ci.p);
  a.cp = static_cast<const int32_t*>(fm->cp.p);
  a.crow = static_cast<const int32_t*>(fm->crow.p);
  a.csb = static_cast<const uint8_t*>(fm->csb.p);
  a.cmag = fm->cmag.p;
  a.prior = fm->prior.p;
  a.synd = d_synd;
  a.corr = d_corr;
  a.steps = d_steps;
  a.conv = nullptr;
  a.B = B;
  a.m = fm->m;
  a.n = fm->n;
  a.max_iter = fm->max_iter;
  // one wave per syndrome when four syndromes' arrays fit 64 KiB (QLDPC_FM_WAVE=0: one workgroup each)
  const size_t per = ((size_t)2 * fm->m + (size_t)2 * fm->n + 15) & ~(size_t)15;
  const char* we = std::getenv("QLDPC_FM_WAVE");
  if (4 * per <= 64 * 1024 && !(we && std::atoi(we) == 0)) {
    const int gw = (int)std::min<long long>((B + 3) / 4, (long long)fm->grid * 4);
    if (fm->precision == 64)
      hipLaunchKernelGGL(firstmin_wave_kernel<double>, dim3(gw), dim3(256), 4 * per, (hipStream_t)stream, a);
    else
      hipLaunchKernelGGL(firstmin_wave_kernel<float>, dim3(gw), dim3(256), 4 * per, (hipStream_t)stream, a);
    QLDPC_HIP(hipGetLastError());
    return 0;
  }
  const int grid = (int)std::min<long long>(B, fm->grid);
  if (fm->precision == 64)
    hipLaunchKernelGGL(firstmin_kernel<double>, dim3(grid), dim3(kFmThreads), fm->lds, (hipStream_t)stream, a);
  else
    hipLaunchKernelGGL(firstmin_kernel<float>, dim3(grid), dim3(kFmThreads), fm->lds, (hipStream_t)stream, a);
  QLDPC_HIP(hipGetLastError());
  return 0;
}

}  // extern "C"
