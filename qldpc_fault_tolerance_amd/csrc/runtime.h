// runtime.h — host-side internals shared by the engine's translation units:
// the thread-local error message behind qldpc_last_error(), device buffers,
// and the opaque handle types of include/qldpc_hip.h.
#pragma once
#include <hip/hip_runtime.h>

// measured-and-not-kept kernel families (c2s, m2v, fp64 x 512 threads, engine 4): out of the
// product build unless -DQLDPC_EXPERIMENTAL=1
#ifndef QLDPC_EXPERIMENTAL
#define QLDPC_EXPERIMENTAL 0
#endif

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
  // max_iter = 1 min-sum decodes (qldpc_bp_decode_batch): the first-min step kernel's one-iteration
  // BP (firstmin.hip), built on first use from these priors; dropped when they change
  qldpc_firstmin* bp1 = nullptr;
  bool bp1_off = false;
  qldpc_rt::DevBuf vchk, llr;  // engine 1: packed u16 check ids; engines 2-4: edge words (check | slot<<16)
  qldpc_rt::DevBuf rdeg;       // engines 3/4: u8 row degrees (by check label)
  qldpc_rt::DevBuf rowtab;     // m2v: the check phase's row table [kM2vRows][TB] x 4 u32
  int vslots_m2v = 0;          // m2v: V slots of the variable-major layout (0 = row-major formula)
  int m2v_vlast = 0, m2v_nl = 0;  // m2v: first V slot of the last variable slot, its per-edge stride
  int m2s_pk = 0;        // m2s rows of 8 with packed absolute edge addresses (engine id 10203)
  int vslots_dummy = 0;  // m2s rows of 8 (engine id 10103): private V slots of real variables' missing edges
  uint32_t nw = 0;       // narrow waves of the fp64 space-time m2s family (SSector::nw)
  uint32_t live_last = 0;  // its waves live in the last variable slot (SSector::live_last)
  int npos = 0;       // 1 + the last slot position holding a variable (SSector::npos)
  qldpc_rt::DevBuf work;       // engine 3 decode_batch: chunk-queue head
  // engines 3/4: variable of each (k, t) slot (-1 = padding).  Engine 3 sorts
  // degree <= 3 variables first so that slots k < d3k skip the 4th edge slot.
  std::vector<int32_t> slot_var;
  qldpc_rt::DevBuf perm;
  qldpc_rt::DevBuf rperm;  // engine 3: original check of each check label (label_checks)
  int gather_conf[2] = {0, 0};  // engine 3: extra gather cycles per pass before / after labelling
  // engine-3 fp64 variable phase, static LDS model per workgroup-iteration (qldpc_bp_lds_model):
  // CS gather cycles / extra, V-slot read cycles / extra, v2c store group-cycles / extra
  int64_t lds_model[6] = {0, 0, 0, 0, 0, 0};
  int d3k = 0;
  int d2k = 0;  // byte-F family: compile-time degree-2 slot count (slots of the measurement variables)
  int ea_shift = 0;  // engine 3: 2 = dword-scaled LDS addresses in the edge words (images > 64 KiB)
  int tail = 0;      // engine 3: 1 = rows of nch chunks + one tail slot per row (bp_reg.h eng_tail)
  int m2s = 0;       // engine 3: 1 = one-word check state, m2 in the argmin slot (bp_reg.h eng_m2s);
                     // 3 = the same with variable-major V slots (eng_m2v);
                     // 2 = c2v written into the slots by the check phase (eng_c2s)
  int fb = 0;        // engine 3: 1 = byte F words (fp32 space-time family, 512 threads; bp_reg.h eng_fb)
  // engine 5 (product-sum, bp_ps.hip): CSR / CSC on the device, optional HBM message workspace
  qldpc_rt::DevBuf ps_rp, ps_ci, ps_cp, ps_ce, ps_ws;
  long long ps_grid = 0;
  // engine 6 (HBM-resident messages, bp_hbm.hip): uniform edge tables and the message workspace
  qldpc_rt::DevBuf h_rp, h_rcol, h_rcpos, h_cp, h_crpos, h_ws;
};

struct qldpc_mc {
  qldpc_bp* dec[2] = {nullptr, nullptr};
  int kw[2] = {0, 0};
  qldpc_rt::DevBuf lmask[2];
  qldpc_rt::DevBuf counters;
  qldpc_rt::DevBuf work;  // engine 3: chunk-queue head
  qldpc_rt::DevBuf cls_cache;  // engine 3, both sectors: sampled classes of the first sector's pass (SMcArgs)
  int engine = 2, TB = 0, VPL = 0, DMAX = 0, NS = 1, precision = 64, lds_bytes = 0, blocks_per_cu = 0, cus = 0;
  int mmax = 0, vslots = 0, img_bytes = 0;
  int d3k = 0;  // engine 3: compile-time degree-3 slot count of the kernel (min over sectors)
  int nch = 0;  // 16-byte chunks per check row when both sectors agree (else 0)
  int ea_shift = 0;
  int tail = 0, m2s = 0, fb = 0, m2s_pk = 0;  // engine 3 layout flags shared by both sectors
  // staged pipeline (staged.hip): product-sum decoders, or QLDPC_MC_STAGED=1
  bool staged = false;
  long long sbatch = 0;
  // BP+OSD (qldpc_mc_set_osd): GPU OSD per sector on the decodes that reached max_iter.
  // c_cap capture slots per sector (bounded by QLDPC_OSD_CAPTURE_MB); a launch is split into
  // pieces of at most c_cap shots, so a slot can never be lost (one slot per shot and sector)
  qldpc_osd_gpu* osd[2] = {nullptr, nullptr};
  long long c_cap = 0;
  qldpc_rt::DevBuf c_post[2], c_synd[2], c_err[2], c_shot[2], c_outw[2], c_n, c_fail;
  int sm[2] = {0, 0}, sk[2] = {0, 0};
  qldpc_rt::DevBuf s_rp[2], s_ci[2], s_cur[2], s_failw[2], s_D, s_det, s_corr, s_iters, s_conv;
};


namespace qldpc_rt {

// engine 5 (bp_ps.hip)
size_t ps_lds_bytes(int precision, int m, int n, int E, bool lds_messages);
const void* ps_kernel(int precision);
int ps_decode_launch(const qldpc_bp* bp, const uint8_t* synd, uint8_t* corr, int32_t* iters, uint8_t* conv, int64_t B,
                     hipStream_t stream,
                     double* post = nullptr);

// GPU OSD handle built on this graph? (osd.hip; qldpc_phenl_set_final_osd checks it)
bool osd_gpu_matches(const qldpc_osd_gpu* o, const qldpc_graph* g);
// host OSD stage built on this graph? (osd.hip; qldpc_circ_set_final_osd checks it)
bool osd_host_matches(const qldpc_osd* o, const qldpc_graph* g);
// GPU OSD handle from a host OSD stage on graph g: same method / order / rank / soft weights (osd.hip)
int osd_gpu_from_host(const qldpc_graph* g, const qldpc_osd* host, qldpc_osd_gpu** out);
// true when the first-min decoder was built on exactly this graph (shape and edges) and device
bool firstmin_matches(const qldpc_firstmin* fm, const qldpc_graph* g);
// one-iteration min-sum BP through a first-min handle (built with max_iter 0): corrections, iterations
// (1) and convergence (H d == s), the qldpc_bp_decode_batch contract at max_iter = 1
int bp1_decode(qldpc_firstmin* fm, const uint8_t* d_synd, uint8_t* d_corr, int32_t* d_iters, uint8_t* d_conv,
               int64_t B, hipStream_t stream);
// BP+OSD stage of the fused shot loop, one sector (osd.hip)
int osd_gpu_bposd_stage(qldpc_osd_gpu* osd, const uint8_t* synd, const double* post, const uint8_t* err,
                        const long long* shot, uint8_t* outw, long long ncand, const unsigned long long* lmask, int kw,
                        int q, int logical_mode, uint8_t* fail, unsigned long long* counters, hipStream_t stream);
// qldpc_osd_gpu_decode that skips the capture slots whose shot index is < 0 (osd.hip)
int osd_gpu_decode_slots(qldpc_osd_gpu* osd, const uint8_t* d_synd, const double* d_post, const uint8_t* d_conv,
                         const long long* d_shot, const uint8_t* d_bp_corr, uint8_t* d_out0, uint8_t* d_outw,
                         int64_t B, void* stream);

// engine 6 (bp_hbm.hip)
int hbm_prepare(qldpc_bp* bp);
const void* hbm_kernel(int precision);
int hbm_decode_launch(qldpc_bp* bp, const uint8_t* synd, uint8_t* corr, int32_t* iters, uint8_t* conv, int64_t B,
                      hipStream_t stream);

// staged data-error shot loop (staged.hip): bit-sliced sampling / syndromes /
// checks around qldpc_bp_decode_batch, for decoders the fused kernels do not serve
int staged_mc_prepare(qldpc_mc* mc, const qldpc_graph* logical_x, const qldpc_graph* logical_z);
void staged_mc_release(qldpc_mc* mc);
int staged_mc_launch(qldpc_mc* mc, double px, double py, double pz, uint64_t seed, uint64_t shot_begin,
                     int64_t shot_count, int32_t logical_mode, const double* d_uniforms, void* d_counters,
                     uint8_t* d_fail, uint8_t* d_err, uint8_t* d_corr, int32_t* d_iters, hipStream_t stream);

}  // namespace qldpc_rt
