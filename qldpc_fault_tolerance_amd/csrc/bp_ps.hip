// bp_ps.hip — engine 5: product-sum BP (ldpc bp_method="product_sum").
//
// Restates ldpc 0.1.x `bp_decode_prob_ratios` (the reference selects it with
// bp_method="product_sum", src/Decoders.py:80-84; oracle: bp_ps_* in
// oracle/qldpc_oracle.c): messages are probability ratios, the check update is
// an ordered forward / backward product of (2/(1+b2c) - 1) terms per row, the
// variable update an ordered product with NaN -> 1 guards per column, the
// decision is ratio >= 1.  Those products are order dependent, so the engine
// keeps ldpc's order exactly: one thread walks a whole row (check phase) or a
// whole column (variable phase, rows ascending) — the result is bit-identical
// to the oracle in fp64 and in fp32.
//
// One decode per workgroup at a time, workgroups persistent over the batch.
// Messages (b2c, c2b: 2·E values, row-major edge order) live in LDS when they
// fit, else in a per-workgroup slice of an HBM workspace (flat addressing
// serves both); decisions and the syndrome are always LDS bytes.  Convergence
// (H x == s) is tested every iteration by the check threads with one shared
// flag, double-buffered so one barrier per test suffices.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "runtime.h"

namespace {

constexpr int kPsThreads = 256;

struct PsArgs {
  const int32_t* rp;    // CSR row pointers [m+1]
  const int32_t* ci;    // CSR columns (ascending) [E]
  const int32_t* cp;    // CSC column pointers [n+1]
  const int32_t* ce;    // CSC: edge ids (row-major numbering), rows ascending [E]
  const void* ratio;    // T [n]: p / (1 - p)
  void* ws;             // HBM message workspace (T [grid][2E]) or NULL (messages in LDS)
  const uint8_t* synd;  // [B][m]
  uint8_t* corr;        // [B][n]
  int32_t* iters;       // [B] or NULL
  uint8_t* conv;        // [B] or NULL
  double* post;         // [B][n] or NULL: ldpc's log_prob_ratios = log(1 / ratio) of the last iteration
  long long B;
  int m, n, E, max_iter;
};

template <typename T>
__global__ void __launch_bounds__(kPsThreads) ps_decode_kernel(PsArgs A) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, TB = blockDim.x;
  const int m = A.m, n = A.n, E = A.E;
  T* b2c;
  unsigned char* tail;
  if (A.ws) {
    b2c = static_cast<T*>(A.ws) + (size_t)blockIdx.x * 2 * E;
    tail = smem;
  } else {
    b2c = reinterpret_cast<T*>(smem);
    tail = smem + (size_t)2 * E * sizeof(T);
  }
  T* c2b = b2c + E;
  int* flag = reinterpret_cast<int*>(tail);  // [2]
  uint8_t* dec = tail + 8;
  uint8_t* syn = dec + n;
  const T* ratio = static_cast<const T*>(A.ratio);
  const T one = (T)1, two = (T)2;
  for (long long b = blockIdx.x; b < A.B; b += gridDim.x) {
    for (int i = tid; i < m; i += TB) syn[i] = A.synd[b * m + i] & 1;
    for (int j = tid; j < n; j += TB) {
      const T r = ratio[j];
      for (int k = A.cp[j]; k < A.cp[j + 1]; ++k) b2c[A.ce[k]] = r;
    }
    if (tid == 0) flag[0] = flag[1] = 0;
    __syncthreads();
    int it = 1;
    bool converged = false;
    for (; it <= A.max_iter; ++it) {
      // check update, ldpc row order: forward products then backward products
      for (int i = tid; i < m; i += TB) {
        const int e0 = A.rp[i], e1 = A.rp[i + 1];
        T temp = syn[i] ? -one : one;
        for (int e = e0; e < e1; ++e) {
          c2b[e] = temp;
          temp *= two / (one + b2c[e]) - one;
        }
        temp = one;
        for (int e = e1 - 1; e >= e0; --e) {
          const T c = c2b[e] * temp;
          c2b[e] = (one - c) / (one + c);
          temp *= two / (one + b2c[e]) - one;
        }
      }
      __syncthreads();
      // variable update, rows ascending: prefix products from the prior ratio, then suffix products
      for (int j = tid; j < n; j += TB) {
        const int k0 = A.cp[j], k1 = A.cp[j + 1];
        T temp = ratio[j];
        for (int k = k0; k < k1; ++k) {
          const int e = A.ce[k];
          b2c[e] = temp;
          temp *= c2b[e];
          if (__builtin_isnan(temp)) temp = one;
        }
        dec[j] = temp >= one ? 1 : 0;
        // soft output (BP+OSD with bp_method="product_sum"): ldpc sets log_prob_ratios[j] = log(1 / temp)
        // every iteration, so the last one's stays; evaluated in double with the device's log (libm's
        // log on the host: the two agree to the last bit except for rare 1-ulp differences)
        if (A.post) A.post[b * n + j] = (double)(T)log(1.0 / (double)temp);
        temp = one;
        for (int k = k1 - 1; k >= k0; --k) {
          const int e = A.ce[k];
          b2c[e] *= temp;
          temp *= c2b[e];
          if (__builtin_isnan(temp)) temp = one;
        }
      }
      __syncthreads();
      // H x == s ?
      int* f = &flag[it & 1];
      for (int i = tid; i < m; i += TB) {
        uint32_t par = syn[i];
        for (int e = A.rp[i]; e < A.rp[i + 1]; ++e) par ^= dec[A.ci[e]];
        if (par) *f = 1;
      }
      if (tid == 0) flag[(it + 1) & 1] = 0;
      __syncthreads();
      if (*f == 0) {
        converged = true;
        break;
      }
    }
    for (int j = tid; j < n; j += TB) A.corr[b * n + j] = dec[j];
    if (tid == 0) {
      if (A.iters) A.iters[b] = converged ? it : A.max_iter;
      if (A.conv) A.conv[b] = converged ? 1 : 0;
    }
    __syncthreads();
  }
}

}  // namespace

namespace qldpc_rt {

size_t ps_lds_bytes(int precision, int m, int n, int E, bool lds_messages) {
  const size_t tail = 8 + (size_t)n + (size_t)m;
  return (lds_messages ? (size_t)2 * E * (precision == 32 ? 4 : 8) : 0) + ((tail + 15) / 16) * 16;
}

const void* ps_kernel(int precision) {
  return precision == 32 ? reinterpret_cast<const void*>(&ps_decode_kernel<float>)
                         : reinterpret_cast<const void*>(&ps_decode_kernel<double>);
}

int ps_decode_launch(const qldpc_bp* bp, const uint8_t* synd, uint8_t* corr, int32_t* iters, uint8_t* conv, int64_t B,
                     hipStream_t stream, double* post) {
  const qldpc_graph* g = bp->g;
  PsArgs a;
  a.rp = static_cast<const int32_t*>(bp->ps_rp.p);
  a.ci = static_cast<const int32_t*>(bp->ps_ci.p);
  a.cp = static_cast<const int32_t*>(bp->ps_cp.p);
  a.ce = static_cast<const int32_t*>(bp->ps_ce.p);
  a.ratio = bp->llr.p;
  a.ws = bp->ps_ws.p;
  a.synd = synd;
  a.corr = corr;
  a.iters = iters;
  a.conv = conv;
  a.post = post;
  a.B = B;
  a.m = g->m;
  a.n = g->n;
  a.E = g->nnz;
  a.max_iter = bp->max_iter;
  const long long cap = bp->ps_grid;
  const int grid = (int)std::max<long long>(1, std::min<long long>(B, cap));
  if (bp->precision == 32)
    hipLaunchKernelGGL(ps_decode_kernel<float>, dim3(grid), dim3(kPsThreads), bp->lds_bytes, stream, a);
  else
    hipLaunchKernelGGL(ps_decode_kernel<double>, dim3(grid), dim3(kPsThreads), bp->lds_bytes, stream, a);
  QLDPC_HIP(hipGetLastError());
  return 0;
}

}  // namespace qldpc_rt
