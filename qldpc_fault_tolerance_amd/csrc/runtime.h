// runtime.h — host-side internals shared by the engine's translation units:
// the thread-local error message behind qldpc_last_error(), device buffers,
// and the opaque handle types of include/qldpc_hip.h.
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "../../include/qldpc_hip.h"

namespace qldpc_rt {

extern thread_local std::string g_err;

inline int set_err(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define QLDPC_HIP(x)                                                                        \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) return qldpc_rt::set_err(QLDPC_EHIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  int alloc(size_t b) {
    bytes = b;
    if (b == 0) return 0;
    if (hipMalloc(&p, b) != hipSuccess) {
      p = nullptr;
      return set_err(QLDPC_ENOMEM, "hipMalloc failed");
    }
    return 0;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
};

}  // namespace qldpc_rt

struct qldpc_graph {
  int device = 0;
  int m = 0, n = 0, nnz = 0, max_row = 0, max_col = 0;
  std::vector<int32_t> row_ptr, col_idx;
  std::vector<std::vector<int32_t>> col_rows;  // rows of each column, ascending
};

struct qldpc_bp {
  qldpc_graph* g = nullptr;
  int engine = 2;
  int max_iter = 0, method = 1, precision = 64;
  double alpha = 0.625;
  int TB = 64, VPL = 1, DMAX = 4, NS = 1;
  int nch = 0;  // engine 2: 16-byte chunks per check row
  int lds_bytes = 0, blocks_per_cu = 0, cus = 0;
  std::vector<double> probs;
  qldpc_rt::DevBuf vchk, llr;  // engine 1: packed u16 check ids; engines 2-4: edge words (check | slot<<16)
  qldpc_rt::DevBuf rdeg;       // engine 4: u8 row degrees
};

struct qldpc_mc {
  qldpc_bp* dec[2] = {nullptr, nullptr};
  int kw[2] = {0, 0};
  qldpc_rt::DevBuf lmask[2];
  qldpc_rt::DevBuf counters;
  int engine = 2, TB = 0, VPL = 0, DMAX = 0, NS = 1, precision = 64, lds_bytes = 0, blocks_per_cu = 0, cus = 0;
  int mmax = 0, vslots = 0, img_bytes = 0;
};

